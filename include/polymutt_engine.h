/*
 * polymutt_engine.h -- C ABI of the MI355X-native polyMutt per-site family-likelihood engine.
 *
 * The reference (genome-vendor/polymutt v0.13) has no plugin/FFI boundary; its hot path is the C++
 * class surface FamilyLikelihoodSeq (-> NucFamGenotypeLikelihood -> ScalarMinimizer) driven once per
 * site by the OpenMP site loop of src/main.cpp:325-594.  This header is the drop-in replacement for
 * that loop body: the host driver (polymutt_amd/host, or any FFI caller) packs a batch of sites into a
 * dense block and one call evaluates, per site, everything main.cpp:327-589 computes:
 *
 *   CalcReadStats + depth/PS/MQ filters ........ src/NucFamGenotypeLikelihood.cpp:520-546, main.cpp:343-348
 *   MonomorphismLogLikelihood(_denovo) ......... NucFamGenotypeLikelihood.cpp:502-517, FamilyLikelihoodSeq.cpp:68-72
 *   PolymorphismLogLikelihood x3 (+x3) ......... FamilyLikelihoodSeq.cpp:91-104 -> OptimizeFrequency
 *                                                 NucFamGenotypeLikelihood.cpp:432-444 -> Brent core/MathGold.cpp:81-177
 *   CalcVarPosterior(4 | 7) .................... NucFamGenotypeLikelihood.cpp:1693-1749
 *   allele switch / counters / de-novo LR ...... main.cpp:539-574
 *   CalcPostProb (genotype posteriors, GQ, DS) . FamilyLikelihoodSeq.cpp:74-89, NucFamGenotypeLikelihood.cpp:590-868
 *   CalculateAB ................................ NucFamGenotypeLikelihood.cpp:1006-1039
 *
 * VCF text formatting (OutputVCF, NucFamGenotypeLikelihood.cpp:1751-1915) stays on the host.
 *
 * Conventions: plain C types, caller-owned buffers, no global state except the thread-local last-error
 * string.  Every entry point returns 0 on success and a negative pm_status on failure; the message is
 * available from pm_last_error().  All computation is FP64 on the GPU; there is no CPU fallback -- a
 * missing/failed HIP device makes pm_engine_create fail loudly.
 */
#ifndef POLYMUTT_ENGINE_H
#define POLYMUTT_ENGINE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PM_ABI_VERSION 7   /* 7: pm_engine_stuck_site, partial batches on PM_EBRENT; 6: pm_engine_run_vcf; 5: submit / collect */
#define PM_NCFG 7           /* varllk slots: 0 mono, 1 ref/ts, 2 ref/tv1, 3 ref/tv2, 4 ts/tv1, 5 ts/tv2, 6 tv1/tv2 */

typedef enum { PM_OK = 0, PM_EINVAL = -1, PM_EHIP = -2, PM_ENOMEM = -3, PM_EBRENT = -4, PM_EPED = -5 } pm_status;

/* chromosome class of the current GLF section (main.cpp:312-315) */
typedef enum { PM_CHR_AUTO = 0, PM_CHR_X = 1, PM_CHR_Y = 2, PM_CHR_MT = 3 } pm_chrom;

/* How FamilyLikelihoodSeq::CalcAllFamLogLikelihood treats a family (FamilyLikelihoodSeq.cpp:228-234):
 * all-founder families -> product of single-person likelihoods (NucFamGenotypeLikelihood.cpp:943-949),
 * isNuclear() families -> closed form over 9 parental genotype pairs (:1041-1084),
 * everything else       -> Elston-Stewart peeling (FamilyLikelihoodES.cpp:1013-1057). */
typedef enum { PM_FAM_NUCLEAR = 0, PM_FAM_FOUNDERS = 1, PM_FAM_EXTENDED = 2 } pm_fam_kind;

/* One Elston-Stewart peeling step (ES_Peeling::from/to/peelingType, FamilyLikelihoodES.h:29-31).
 * Indices are family-local positions in Family::path (founders first). */
typedef struct {
  int32_t type;           /* 1 offspring->parents, 2 spouse->spouse, 3 parents->only offspring */
  int32_t from0, from1;   /* from1 = -1 unless type 3 (father, mother)            */
  int32_t to0, to1;       /* to1   = -1 unless type 1 (father, mother)            */
} pm_peel_step;

/* Flattened pedigree.  Persons are numbered in VCF column order: families in Pedigree order, members
 * in Family::path order (core/PedigreeFamily.cpp:11-85) -- i.e. exactly pedGLF->glf[i][j]. */
typedef struct {
  int32_t n_fam;
  int32_t n_person;
  const int32_t *fam_start;    /* [n_fam+1] first person of each family                         */
  const int32_t *fam_founders; /* [n_fam]  Family::founders                                      */
  const int32_t *fam_kind;     /* [n_fam]  pm_fam_kind                                           */
  const int8_t  *sex;          /* [n_person] 0 unknown, 1 male, 2 female (PedigreeGLF::sexes)    */
  const int8_t  *is_founder;   /* [n_person] Person::isFounder()                                 */
  const int32_t *father;       /* [n_person] person index of the father, -1 for founders          */
  const int32_t *mother;       /* [n_person] person index of the mother, -1 for founders          */
  const int32_t *peel_start;   /* [n_fam+1] offsets into steps (empty range for founders-only)    */
  const pm_peel_step *steps;   /* ES_Peeling::BuildPeelingOrder output for every family with
                                  offspring (FamilyLikelihoodSeq.cpp:14-35); nuclear families need
                                  theirs only in vcf_mode (chrX/Y/MT or a single family)          */
  int32_t n_founders;          /* PedigreeGLF::nFounders   (sum of Family::founders)             */
  int32_t male_founders;       /* PedigreeGLF::maleFounders                                      */
  int32_t female_founders;     /* PedigreeGLF::femaleFounders                                    */
} pm_pedigree;

/* Command-line parameters that reach the model (CmdLinePar, src/CmdLinePar.h; defaults main.cpp:59-85). */
typedef struct {
  double  theta;               /* --theta 1e-3 */
  double  poly_tstv;           /* --poly_tstv 2 */
  double  precision;           /* --prec 1e-4 (Brent tol) */
  double  posterior;           /* -c 0.5 */
  int32_t min_total_depth;     /* --minDepth */
  int32_t max_total_depth;     /* --maxDepth (0 = off) */
  double  min_ps;              /* --minPercSampleWithData */
  int32_t min_map_quality;     /* --minMapQuality */
  int32_t denovo;              /* --denovo */
  double  denovo_mut_rate;     /* --rate_denovo 1.5e-8 */
  double  denovo_tstv;         /* --tstv_denovo 2 */
  double  denovo_min_llr;      /* --minLLR_denovo 0.01 */
  int32_t force_call;          /* set by --pos */
  int32_t all_sites;           /* --all_sites */
  int32_t quick_call;          /* --quick_call */
  int32_t numerics;            /* pm_numerics: how the engine evaluates the Brent objective */
  int32_t vcf_mode;            /* --in_vcf: FamilyLikelihoodSeq_VCF semantics (PedVCF.cpp:43-164) -- one (ref, alt)
                                  Brent per site, ref[i] = refAllele | altAllele << 4, PL->lk table pow(10,-i/10),
                                  no filters; res.varllk[0] = mono, varllk[1] = poly (no priors), af = minimiser */
} pm_params;

/* Diagnostic environment variables read by pm_engine_create / pm_engine_run (tests and tools only; results
 * never depend on them beyond the documented bit-identical alternatives):
 *   PM_NO_PREFETCH=1  the lean kernels hoist from direct HBM loads instead of LDS-staged PL bytes (tests
 *                     compare the two paths bit for bit);
 *   PM_BRENT_TS=T,S   force the Brent lane plan to T threads x S slots when it holds the pedigree
 *                     (tools/brent_sweep.py geometry sweeps). */

/* Objective-evaluation numerics.  All three compute CalcAllFamLogLikelihood; they differ in rounding only.
 *   PM_NUM_PRODUCT: each family's likelihood exactly as the reference forms it (same operations, same order),
 *                   families combined as a normalised product, one log10 per evaluation;
 *   PM_NUM_EXACT:   one log10 per family, summed (the reference's form; ~2x slower);
 *   PM_NUM_POLY:    (default) nuclear families as a 4-FMA Horner quartic in min(f,1-f)/max(f,1-f) on the lean
 *                   autosomal kernel (>1 family); every other kernel flavour uses PRODUCT.  Objective values
 *                   differ from the reference by ~1e-14 relative, so on objectives flat to rounding noise Brent
 *                   may stop at another point of equal likelihood (never visible in the VCF). */
typedef enum { PM_NUM_PRODUCT = 0, PM_NUM_EXACT = 1, PM_NUM_POLY = 2 } pm_numerics;

/* Site status codes (which `continue` of main.cpp:300-594 was taken). */
typedef enum {
  PM_SITE_CALLED = 0,          /* evaluated; see emit */
  PM_SITE_MIN_DEPTH = 1, PM_SITE_MAX_DEPTH = 2, PM_SITE_MIN_PS = 3, PM_SITE_MIN_MAPQ = 4,
  PM_SITE_BAD_REF = 5,         /* refBase not in 1..4 (main.cpp:340) */
  PM_SITE_QUICK_SKIP = 7       /* rejected by the --quick_call pre-filter (main.cpp:432-433) */
} pm_site_status;

/* Genotype-label flavour of a person in an emitted record (the four labellers of
 * NucFamGenotypeLikelihood.cpp:1573-1608 plus the chrY-female "."). */
typedef enum { PM_LBL_VCF_DIPLOID = 0, PM_LBL_VCF_HAPLOID = 1, PM_LBL_ALLELES = 2, PM_LBL_GENO10 = 3, PM_LBL_DOT = 4 } pm_label_kind;

/* Per-site result (240 bytes, naturally aligned, no implicit padding). */
typedef struct {
  int32_t status;              /* pm_site_status */
  int32_t n_cfg;               /* 4 or 7 configurations evaluated */
  int32_t maxidx;              /* CalcVarPosterior argmax */
  int32_t emit;                /* 1: a VCF record is written; 2: OutputVCF_denovo called but record suppressed */
  int32_t total_depth;
  int32_t num_samp_with_data;
  double  avg_map_qual;
  double  perc_samp_with_data;
  double  var_post_prob;
  double  poly_qual;
  double  varllk[PM_NCFG];
  double  varfreq[PM_NCFG];    /* Brent minimiser per configuration (1.0 for mono) */
  double  af;                  /* GetMinimizer() printed as AF */
  double  ab;                  /* CalculateAB */
  double  denovo_lr;           /* DQ */
  int32_t evals[PM_NCFG];      /* objective evaluations per configuration */
  int32_t allele1, allele2;    /* famlk[0] alleles at output time (1..4) */
  int32_t is_mono;             /* famlk[0].isMono for the record (BA= tag) */
  int32_t denovo_mono;         /* OutputVCF_denovo prints ALT=allele1 */
  int32_t call_row;            /* row of pm_geno_call output for this site, -1 if none */
} pm_site_result;

/* Per-person genotype call of an emitted record (16 bytes). */
typedef struct {
  double  dosage;              /* DS */
  int16_t best;                /* bestGenoIdx (0..2, or 0..9 for de-novo kids) */
  int16_t gq;                  /* GQ */
  int8_t  label;               /* pm_label_kind */
  int8_t  _pad[3];
} pm_geno_call;

/* vcf_mode genotype row entry (FamilyLikelihoodSeq_VCF::OutputVCF prints GT/GQ only): the device rows of a
 * vcf_mode engine (pm_engine_run_device's d_calls) use this 4-byte layout; pm_engine_run expands them into
 * pm_geno_call rows with dosage 0. */
typedef struct {
  int8_t best;
  int8_t gq;
  int8_t label;                /* pm_label_kind */
  int8_t pad;
} pm_vcf_call;

/* Summary counters of one section (main.cpp:264-282, printed :596-619); summed over shards/GPUs. */
typedef struct {
  int64_t ref_base_counts[5];
  int64_t min_total_depth_filter, max_total_depth_filter, min_ps_filter, min_map_qual_filter;
  int64_t homo_ref, transitions, transversions, tstvs1, tstvs2, tvs1tvs2, nocall;
} pm_counters;

typedef struct pm_engine pm_engine;

/* Create an engine on HIP device `device` (one engine per GPU; engines are independent and thread-safe
 * with respect to each other).  max_batch bounds the sites per pm_engine_run call. */
int pm_engine_create(const pm_pedigree *ped, const pm_params *par, int device, int max_batch, pm_engine **out);
void pm_engine_destroy(pm_engine *eng);

/* The lane plan pm_engine_create chose for the Brent kernel: threads per item (one wave = 64) and
 * family slots per lane.  Diagnostics and tests only (no reference counterpart). */
int pm_engine_plan(pm_engine *eng, int32_t *threads, int32_t *slots);

/* famlk[0]'s stale state across sites: whether CalcPostProb has already run earlier in the run (any
 * earlier site reached OutputVCF).  The reference's likelihoodONEKid reads the object's member `sex`
 * (NucFamGenotypeLikelihood.cpp:1193, 1202-1264), which CalcPostProb leaves at the last person's sex; it
 * changes the first family's chrX/Y genotype posteriors.  The engine tracks it itself across
 * pm_engine_run calls; a driver that splits a run over several engines (site shards) sets it at each
 * shard's start.  0 at creation. */
int pm_engine_set_posterior_carry(pm_engine *eng, int32_t seen);

/* Start a GLF section: sets the chromosome class, recomputes the polymorphism prior
 * (GetPolyPrior, NucFamGenotypeLikelihood.cpp:295-304) and zeroes the section counters. */
int pm_engine_begin_section(pm_engine *eng, int32_t chrom);

/* Evaluate n sites.  Inputs are the dense per-site block, persons in pm_pedigree order:
 *   pl  [n][n_person][10]  phred genotype likelihoods AA,AC,AG,AT,CC,CG,CT,GG,GT,TT (0 when absent)
 *   dm  [n][n_person]      depth (bits 0-23) | mapQ << 24   (0 when absent; not read in vcf_mode -- the VCF path has no
 *                          depth -- where it may be NULL)
 *   ref [n]                refBase 1..4 (anything else -> PM_SITE_BAD_REF)
 * inputs_on_device != 0: pl/dm/ref are device pointers on this engine's GPU, else host pointers.
 * Outputs are host pointers: res[n]; calls[n_rows * n_person] receives one row per written record
 * (emit == 1; row index = res[i].call_row, rows numbered in site order, -1 for every other site: a
 * suppressed de novo record, emit == 2, prints nothing and gets no row); *n_rows is set to the row count.
 * Counters accumulate into the section totals.  Synchronous.
 * PM_EBRENT: some site's Brent maximisation hit ITMAX (ScalarMinimizer::Brent's numerror, core/MathGold.cpp:98,175,
 * where the reference's site loop ends the run).  res[] is still written for the whole batch, and the sites before the
 * first stuck one -- pm_engine_stuck_site -- are complete: their genotype rows are the first *n_rows rows (*n_rows
 * counts only their rows), as the reference had written their records (NucFamGenotypeLikelihood.cpp:1829, fflush per
 * record) before exiting at the stuck site.  The section counters then include the whole batch. */
int pm_engine_run(pm_engine *eng, int32_t n, const uint8_t *pl, const uint32_t *dm, const uint8_t *ref,
                  int32_t inputs_on_device, pm_site_result *res, pm_geno_call *calls, int32_t *n_rows);

/* vcf_mode engines only: pm_engine_run on host inputs (no depth plane) with the genotype rows returned in the
 * compact pm_vcf_call form the device writes -- best / GQ / label, all FamilyLikelihoodSeq_VCF::OutputVCF
 * (src/FamilyLikelihoodSeq_VCF.cpp:412-521) prints -- instead of widened into pm_geno_call rows: a quarter of
 * the bytes, copied straight into `calls` (one synchronous device-to-host copy; page-locked `calls` from
 * pm_host_alloc copy at full PCIe rate).  Replaces, for the --in_vcf path, the per-record
 * FamilyLikelihoodSeq_VCF::FillPenetrance -> CalcLikelihood -> OutputVCF calls of PedVCF::VarCallFromVCF
 * (src/PedVCF.cpp:103-160).  PM_EINVAL on an engine created without vcf_mode, or while a pm_engine_submit batch
 * has not been collected (that batch stays pending).  PM_EBRENT as for pm_engine_run. */
int pm_engine_run_vcf(pm_engine *eng, int32_t n, const uint8_t *pl, const uint8_t *ref, pm_site_result *res,
                      pm_vcf_call *calls, int32_t *n_rows);

/* pm_engine_run split in two, so a driver keeps several batches in flight (one per engine; each engine has its
 * own HIP stream): pm_engine_submit queues the batch's host-to-device copies (asynchronous when pl/dm/ref are
 * page-locked, pm_host_alloc), the pipeline and the copy-back of the per-site results on the engine's stream and
 * returns; pm_engine_collect waits for that batch and writes res[n], the genotype rows and *n_rows exactly as
 * pm_engine_run does.  One batch per engine between the two calls.  The input buffers must stay untouched until
 * the collect.  (The reference's site loop body, main.cpp:327-589, per batch; no reference counterpart for the
 * asynchrony itself.) */
int pm_engine_submit(pm_engine *eng, int32_t n, const uint8_t *pl, const uint32_t *dm, const uint8_t *ref);
int pm_engine_collect(pm_engine *eng, pm_site_result *res, pm_geno_call *calls, int32_t *n_rows);

/* After a batch returned PM_EBRENT (pm_engine_run, _run_vcf, _collect or _sync): *site = the batch index of the first
 * site whose Brent hit ITMAX, i.e. the number of leading sites whose results and rows are complete; -1 when the last
 * finished batch had none.  (core/MathGold.cpp:98,175: the reference exits at that site, its earlier records
 * written.)  The environment variable PM_TEST_ITMAX, read at pm_engine_create, lowers ITMAX (200) for tests. */
int pm_engine_stuck_site(pm_engine *eng, int32_t *site);

/* Page-locked host memory for pm_engine_submit's inputs and the result rows (H2D/D2H at full PCIe rate). */
int pm_host_alloc(uint64_t bytes, void **h_ptr);
int pm_host_free(void *h_ptr);

/* Device-resident variant for benchmarking / multi-GPU sharding: all pointers are device pointers,
 * results stay on the device (d_res[n], d_calls[n * n_person] indexed by site), launched on the
 * engine's stream; returns immediately.  pm_engine_sync waits.
 * d_pl is in the engine's GENOTYPE-PLANAR layout: [n][10][n_person] (site block of 10 planes, plane g
 * holding every person's phred for genotype g), so the engine's wavefronts read consecutive persons as
 * consecutive bytes.  pm_engine_synth writes this layout; pm_engine_to_planar converts person-major
 * GLF-record blocks (the layout of pm_engine_run). */
int pm_engine_run_device(pm_engine *eng, int32_t n, const uint8_t *d_pl, const uint32_t *d_dm, const uint8_t *d_ref,
                         pm_site_result *d_res, pm_geno_call *d_calls);
int pm_engine_sync(pm_engine *eng);

/* Person-major device block [n][n_person][10] -> genotype-planar [n][10][n_person] (distinct buffers),
 * on the engine's stream (asynchronous, like pm_engine_run_device). */
int pm_engine_to_planar(pm_engine *eng, int32_t n, const uint8_t *d_src, uint8_t *d_dst);

/* Section counters accumulated so far (device -> host copy). */
int pm_engine_counters(pm_engine *eng, pm_counters *out);

/* Deterministic synthetic GLF block generator on the device (SURVEY.md section 8(d) recipe):
 * families shaped by the engine's pedigree, 10% polymorphic sites, depth U{8..29}, error 1%.
 * Writes d_pl in the genotype-planar layout of pm_engine_run_device. */
int pm_engine_synth(pm_engine *eng, int32_t n, uint64_t seed, uint64_t site_offset,
                    uint8_t *d_pl, uint32_t *d_dm, uint8_t *d_ref);

/* Device allocation helpers (so FFI callers need no HIP runtime of their own). */
int pm_device_alloc(pm_engine *eng, uint64_t bytes, void **d_ptr);
int pm_device_free(pm_engine *eng, void *d_ptr);
int pm_copy_to_host(pm_engine *eng, void *h_dst, const void *d_src, uint64_t bytes);
int pm_copy_to_device(pm_engine *eng, void *d_dst, const void *h_src, uint64_t bytes);

/* Timing of the dominant (Brent) kernel over the last run: launches, summed kernel ms (HIP events on the
 * engine stream), total objective evaluations and family-evaluations (for roofline accounting). */
typedef struct {
  int64_t launches;      /* k_brent launches */
  double  kernel_ms;     /* summed k_brent time (HIP events on the engine stream) */
  int64_t evals;         /* objective evaluations computed by Brent items (OptimizeFrequency's f(a) and f(c),
                            which Brent never reads, are counted in pm_site_result.evals but not computed) */
  int64_t fam_evals;     /* evals x families */
  int64_t items;         /* (site, configuration) work items evaluated */
  int64_t sites;         /* sites processed */
  int64_t site_visits;   /* sum over k_brent launches of the distinct sites each launch touched (each visit
                            reads that site's PL block once: the launch's algorithmic HBM bytes) */
  int64_t hoist_wave_ns; /* with PM_PHASE_TIMING set at engine creation (else 0): k_brent wave time spent hoisting
                            the frequency-independent family terms, summed over the items' blocks (lane 0's clock) */
  int64_t eval_wave_ns;  /* ... and in the Brent loop (objective evaluations + updates) */
  int64_t timed_items;   /* items the two fields above cover */
  /* extended families in polynomial form (EP): the coefficient hoisting that precedes each Brent chunk, timed apart
     from the Brent launches (kernel_ms / launches above exclude it) */
  int64_t es_hoist_launches;
  double  es_hoist_ms;
  double  es_hoist_ops;  /* its FP64 operations (each mul, add or fma one), counted by the schedule compiler per family
                            shape and variant; 0 when the generic kernel ran (PM_NO_JIT) */
} pm_kernel_stats;
int pm_engine_kernel_stats(pm_engine *eng, pm_kernel_stats *out, int32_t reset);

const char *pm_last_error(void);
int pm_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* POLYMUTT_ENGINE_H */
