// engine.hip -- MI355X (gfx950) engine for polyMutt's per-site family likelihood.
//
// One call (pm_engine_run / pm_engine_run_device) replaces the body of the reference's site loop
// (src/main.cpp:327-589) for a whole batch of sites resident in HBM.  Pipeline per batch:
//
//   k_prep      block/site   CalcReadStats + filters + MonomorphismLogLikelihood (exact serial sum)
//                            -> enqueue Brent work items (site, configuration)
//   k_brent     block/item   OptimizeFrequency + Brent (core/MathGold.cpp:81-177) over the objective
//                            -CalcAllFamLogLikelihood(freq) (src/FamilyLikelihoodSeq.cpp:222-240):
//                            families spread over the block's lanes, the freq-independent part of every
//                            family term hoisted into registers once per item, FP64 throughout, one
//                            deterministic block reduction per objective evaluation
//   k_select    thread/site  CalcVarPosterior(4) (NucFamGenotypeLikelihood.cpp:1693-1749) -> 3 more items
//   k_brent                  the less-likely configurations (main.cpp:499-537)
//   k_finalize  thread/site  CalcVarPosterior(7), allele switch, counters, de-novo LR (main.cpp:539-574)
//   k_brent                  (--denovo) the non-de-novo re-optimisation of main.cpp:569-572
//   k_final_dn  thread/site  (--denovo) denovoLR
//   k_posterior block/site   CalcPostProb (genotype posteriors), GQ, DS, CalculateAB for emitted sites
//
// Design notes: the path is FP64-VALU/transcendental bound, not a GEMM, so no MFMA.
// Compiled with -ffp-contract=off so every multiply/add rounds exactly like the reference's SSE2 code;
// the only deviations from the reference's arithmetic are OCML log10/exp10 (<=1 ulp) and the order of
// the cross-family reduction inside the Brent objective (a fixed tree, deterministic for any batch).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include "../../include/polymutt_engine.h"
#include "synth_core.h"
#include "es_jit.h"

#define MALE 1
#define FEMALE 2
#ifndef PM_HOIST_CHUNK
#define PM_HOIST_CHUNK 4
#endif
#ifndef PM_POLY_WAVES
#define PM_POLY_WAVES 2
#endif

// ------------------------------------------------------------------------------------------------
// error reporting (thread-local, C ABI)
static thread_local std::string g_last_error;
extern "C" void pm_set_last_error(const char* msg) { g_last_error = msg ? msg : ""; }
extern "C" const char* pm_last_error(void) { return g_last_error.c_str(); }
extern "C" int pm_abi_version(void) { return PM_ABI_VERSION; }

#define HIP_TRY(expr)                                                                       \
  do {                                                                                      \
    hipError_t _e = (expr);                                                                 \
    if (_e != hipSuccess) {                                                                 \
      char _b[512];                                                                         \
      snprintf(_b, sizeof(_b), "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), __FILE__, __LINE__); \
      pm_set_last_error(_b);                                                                \
      return PM_EHIP;                                                                       \
    }                                                                                       \
  } while (0)

// ------------------------------------------------------------------------------------------------
// work-unit plan: families are dealt to the lanes of a Brent block; each lane owns up to S units
enum UnitType { U_NONE = 0, U_NUC = 1, U_FP = 2 /* founders-only chunk of <=3 persons */, U_EXT = 3 };
// unit = int4 {type, family, first person (global), count | FIRST<<8 | LAST<<9}
#define UF_FIRST 0x100
#define UF_LAST 0x200

// Brent item encoding: site << 3 | cfg.  cfg 0: de-novo monomorphism (single eval at 1.0);
// 1..6: the six allele configurations; 7: non-de-novo re-optimisation for the de-novo LR.
#define N_LISTS 3

struct DevArgs {
  // pedigree
  int n_fam, n_person, n_fam_gt1, single_nuclear;
  int max_nuc;             // largest nuclear family (persons)
  int chrom, denovo;
  const int* fam_start;
  const int* fam_kind;
  const int8_t* sex;
  const int32_t* fa_local;
  const int32_t* mo_local;
  const int4* units;       // [S][T]
  int T, S;
  // Elston-Stewart (extended families): per-lane family lists, packed schedules, workspace
  const int* fam_founders;
  const int8_t* is_founder;
  const int* peel_start;   // [n_fam+1] into steps
  const int2* steps;       // packed pm_peel_step + marriage-partial slot (see pack_steps)
  const int* ext_count;    // [T] ES families per lane
  const int* ext_fam;      // [max_ext][T]
  const double* T10;       // FamilyLikelihoodES::transmission        [10][10][10]
  const double* T10dn;     // FamilyLikelihoodES::transmission_denovo [10][10][10]
  double* ws;              // peeling workspace, lane-interleaved
  int ws_per_lane;         // doubles per lane (max over ES families of n*ns + couples*ns*ns)
  int ws_lds;              // ES workspace in dynamic LDS (lane-interleaved) instead of HBM
  // ES polynomial form (es_poly = 1, PM_NUM_POLY): per family, poly_lay[poly_start[f]..] = {couples, tmp offset,
  // degree D per chromosome class [4], per person off | cap << 24, per couple off | cap << 24}; poly_deg[4 s + class]
  // = the degrees a step combines (7 bits each); coefficients of the lane's q-th family at ws + poly_coef + q * poly_dcap
  int es_poly;
  const int* poly_start;
  const int* poly_lay;
  const int* poly_deg;
  int poly_coef, poly_dcap;
  // k_es_hoist -> k_brent hand-over (EP): the D + 1 coefficients (+ D at poly_dcap - 1) of every (item, ES family) of
  // the items [es_it0, es_it1) of a list at es_coef[(((it - es_it0) * max_ext + q) * poly_dcap + a) * T + lane]
  double* es_coef;
  int es_it0, es_it1, max_ext;
  int hoist_ws, hoist_tmp;   // k_es_hoist LDS per wave (doubles): the family's layout workspace, the step temporaries
  // posteriors of peeled families: one work item per (row, person) of es_pers[n_es_pers] = family << 8 | member
  const int* es_pers;
  int n_es_pers;
  const int* fam_perm;     // k_posterior: families ordered by (kind, size), so a wave's threads take one code path
  int unrelated;           // --quick_call MakeUnrelated(): every family is all-founder
  double theta_one;        // 1.0 (opaque to the compiler; timing experiments only)
  int vcf;                 // vcf_mode: one (ref, alt) Brent per site, FamilyLikelihoodSeq_VCF family rules
  int nuc_es;              // nuclear families are peeled (vcf_mode plan 1)
  int mono_dn;             // k_prep computes the de novo monomorphism item (cfg 0) itself (lean --denovo)
  int* row_blk;            // k_rows_count / k_rows: written records per 1024-site block
  int pf_npad;             // lean kernel: > 0 = the item's 3 genotype planes are prefetched into LDS (stride)
  int pf_dw;               // ... in 4-byte pieces (n_person % 16 != 0, n_person % 4 == 0)
  int dn_pf;               // lean --denovo kernel: PL windows staged through LDS by LDS-DMA (hoist_poly4_dn_pf)
  int quad_full;           // QUAD plan (hoist_quad): slot rows below this have no empty lane
  // tables
  const double* lktab;     // [256]
  const double* M;         // [100] genotype mutation matrix
  double Mk[100];          // the same, by value in the kernel arguments: uniform reads become scalar loads (QUAD hoisting)
  const pm_synth_tables* syn;
  // parameters
  double precision, posterior, theta;
  int min_total_depth, max_total_depth, min_map_quality;
  double min_ps, denovo_min_llr, log10_denovo_min_llr;
  int force_call, all_sites;
  double lp_mono, lp_ts, lp_tv, lp_other, np_ts, np_tv;   // log10 prior constants (host glibc)
  // batch
  int n;
  const uint8_t* pl;
  const uint32_t* dm;
  const uint8_t* ref;
  pm_site_result* res;
  pm_geno_call* calls;
  double* raw;             // [n][8] log-likelihood per configuration (without prior)
  double* minv;            // [n][8] Brent minimiser
  int* evals;              // [n][8]
  double* mono_plain;      // [n] MonomorphismLogLikelihood
  int* items[N_LISTS];
  int* counts;             // [0..2] list sizes, [3] rows, [4] first emitted site, [5] Brent stuck, [8]/[9] quick items/site visits
  unsigned long long* eval_total;
  unsigned long long* phase;   // PM_PHASE_TIMING: [0] hoisting, [1] evaluations, [2] items -- k_brent wave time (wall_clock64 ticks)
  int* row_site;           // [n] emitted row -> site
  unsigned long long* counters;   // pm_counters as 16 x u64
  int carry_postprob;      // famlk[0].CalcPostProb ran in an earlier batch
};

// ------------------------------------------------------------------------------------------------
// Genotype-planar site block (the engine's HBM layout): a site's 10 x n_person phred bytes are stored
// plane by plane, plane g holding every person's value for genotype g (AA, AC, ..., TT), so the lanes of a
// wave -- consecutive persons or families -- read consecutive bytes.  PLB(site block, n_person, person, g).
#define PLB(pl, np, p, g) (pl)[(size_t)(g) * (np) + (p)]

// small helpers (restating src/PedigreeGLF.h:14-53, core/glfHandler.h:102-106)
__device__ __forceinline__ int d_gi(int b1, int b2) {
  return b1 < b2 ? (b1 - 1) * (10 - b1) / 2 + (b2 - b1) : (b2 - 1) * (10 - b2) / 2 + (b1 - b2);
}
__device__ __forceinline__ int d_ts(int r) { return r == 1 ? 3 : r == 2 ? 4 : r == 3 ? 1 : 2; }
__device__ __forceinline__ int d_tv1(int r) { return (r == 1 || r == 3) ? 2 : 1; }
__device__ __forceinline__ int d_tv2(int r) { return (r == 1 || r == 3) ? 4 : 3; }
__device__ __forceinline__ double d_sign(double a, double b) { return b >= 0 ? fabs(a) : -fabs(a); }

__device__ __forceinline__ void cfg_alleles(int cfg, int r, int* a1, int* a2) {
  const int ts = d_ts(r), tv1 = d_tv1(r), tv2 = d_tv2(r);
  switch (cfg) {
    case 0: *a1 = r; *a2 = (r == 4) ? 3 : r + 1; break;   // main.cpp:458
    case 1: *a1 = r; *a2 = ts; break;
    case 2: *a1 = r; *a2 = tv1; break;
    case 3: *a1 = r; *a2 = tv2; break;
    case 4: *a1 = ts; *a2 = tv1; break;
    case 5: *a1 = ts; *a2 = tv2; break;
    default: *a1 = tv1; *a2 = tv2; break;
  }
}

// likelihoodONEKid, NucFamGenotypeLikelihood.cpp:1202-1264 (member `sex`, X/Y/MT branches)
__device__ __forceinline__ double d_one_kid(int k, int chrom, int sex, double l11, double l12, double l22) {
  const bool X = chrom == PM_CHR_X, Y = chrom == PM_CHR_Y, MT = chrom == PM_CHR_MT;
  switch (k) {
    case 0: return (Y && sex == FEMALE) ? 1.0 : l11;
    case 1: if (X) return sex == MALE ? 0.5 * (l11 + l22) : 0.5 * (l11 + l12);
            if (Y) return sex == MALE ? l11 : 1.0;
            if (MT) return 0.5 * (l11 + l22);
            return 0.5 * (l11 + l12);
    case 2: if (X) return sex == MALE ? l22 : l12;
            if (Y) return sex == MALE ? l11 : 1.0;
            if (MT) return l22;
            return l12;
    case 3: if (X || Y || MT) return 0.0; return 0.5 * (l11 + l12);
    case 4: if (X || Y || MT) return 0.0; return 0.25 * l11 + 0.5 * l12 + 0.25 * l22;
    case 5: if (X || Y || MT) return 0.0; return 0.5 * (l12 + l22);
    case 6: if (X) return sex == MALE ? l11 : l12;
            if (Y) return sex == MALE ? l22 : 1.0;
            if (MT) return l11;
            return l12;
    case 7: if (X) return sex == MALE ? 0.5 * (l11 + l22) : 0.5 * (l12 + l22);
            if (Y) return sex == MALE ? l22 : 1.0;
            if (MT) return 0.5 * (l11 + l22);
            return 0.5 * (l12 + l22);
    default: return (Y && sex == FEMALE) ? 1.0 : l22;
  }
}

// likelihoodONEKid_denovo (:1266-1296) from the three CalcDenovoMutLk dot products (:1553-1562)
__device__ __forceinline__ double d_one_kid_dn(int k, double D11, double D12, double D22) {
  switch (k) {
    case 0: return D11;
    case 1: case 3: return 0.5 * (D11 + D12);
    case 2: case 6: return D12;
    case 4: return 0.25 * D11 + 0.5 * D12 + 0.25 * D22;
    case 5: case 7: return 0.5 * (D12 + D22);
    default: return D22;
  }
}

// Prior modes of the nuclear closed form
enum PriorMode { PR_AUTO = 0, PR_X, PR_Y, PR_MT, PR_TRIO, PR_DN_SINGLE };

// SetParentPrior (:318-368), SetParentPrior_denovo (:370-381), SetParentPriorSingleTrio(_denovo) (:383-420)
__device__ __forceinline__ void d_parent_prior(int mode, double f, double* p) {
  if (mode == PR_DN_SINGLE) mode = (f != 1.0) ? PR_TRIO : PR_AUTO;
  const double g = 1 - f;
  switch (mode) {
    case PR_AUTO:
      p[0] = (f * f) * (f * f);
      p[1] = f * f * f * g * 2;
      p[2] = f * f * g * g;
      p[3] = f * g * 2 * f * f;
      p[4] = f * g * 2 * f * g * 2;
      p[5] = f * g * 2 * g * g;
      p[6] = g * g * f * f;
      p[7] = g * g * f * g * 2;
      p[8] = g * g * g * g;
      break;
    case PR_X:
      p[0] = (f * f) * f; p[1] = f * f * g * 2; p[2] = f * g * g; p[3] = 0; p[4] = 0; p[5] = 0;
      p[6] = g * f * f; p[7] = g * f * g * 2; p[8] = g * g * g;
      break;
    case PR_Y:
      p[0] = f; p[1] = f; p[2] = f; p[3] = 0; p[4] = 0; p[5] = 0; p[6] = g; p[7] = g; p[8] = g;
      break;
    case PR_MT:
      p[0] = f * f; p[1] = 0.0; p[2] = f * g; p[3] = 0; p[4] = 0; p[5] = 0; p[6] = g * f; p[7] = 0; p[8] = g * g;
      break;
    default:
      p[0] = 0.0; p[1] = 0.24; p[2] = 0.04; p[3] = 0.24; p[4] = 0.16; p[5] = 0.08; p[6] = 0.04; p[7] = 0.08; p[8] = 0.12;
      break;
  }
}

// ------------------------------------------------------------------------------------------------
// hoisting: the freq-independent part of one unit for one (site, allele pair, model)
struct ItemCtx {
  int a1, a2, g11, g12, g22;
  int denovo;      // objective uses the de-novo model
  int sex;         // member sex of the evaluating object
  int chrom;
};

// GEN: chrX/Y/MT branches; DN: the de novo kid terms (the lean polynomial kernel takes DN without GEN)
template <bool GEN, bool DN = GEN>
__device__ __forceinline__ void hoist_nuc(const DevArgs& A, const ItemCtx& I, const uint8_t* pl, const double* lk, const double* M,
                                          int p0, int n, double* cond) {
  const int np = A.n_person;
  double F11 = lk[PLB(pl, np, p0, I.g11)], F12 = lk[PLB(pl, np, p0, I.g12)], F22 = lk[PLB(pl, np, p0, I.g22)];
  double M11 = lk[PLB(pl, np, p0 + 1, I.g11)], M12 = lk[PLB(pl, np, p0 + 1, I.g12)], M22 = lk[PLB(pl, np, p0 + 1, I.g22)];
  if (GEN && !I.denovo) {   // CalcParentMarginal :1049-1051
    if (I.chrom == PM_CHR_X) F12 = 0.0;
    if (I.chrom == PM_CHR_Y) { M11 = M12 = M22 = 1.0; F12 = 0.0; }
    if (I.chrom == PM_CHR_MT) F12 = M12 = 0.0;
  }
  double kids[9];
#pragma unroll
  for (int k = 0; k < 9; k++) kids[k] = 1.0;
  for (int j = 2; j < n; j++) {
    const uint8_t* K = pl + p0 + j;   // person p0 + j of plane 0; plane g at K[g * np]
    if (!DN || !I.denovo) {
      const double l11 = lk[K[(size_t)I.g11 * np]], l12 = lk[K[(size_t)I.g12 * np]], l22 = lk[K[(size_t)I.g22 * np]];
#pragma unroll
      for (int k = 0; k < 9; k++) kids[k] *= d_one_kid(k, GEN ? I.chrom : (int)PM_CHR_AUTO, I.sex, l11, l12, l22);
    } else {
      double D11 = 0.0, D12 = 0.0, D22 = 0.0;
#pragma unroll
      for (int g = 0; g < 10; g++) {
        const double pg = lk[K[(size_t)g * np]];
        D11 += M[I.g11 * 10 + g] * pg;
        D12 += M[I.g12 * 10 + g] * pg;
        D22 += M[I.g22 * 10 + g] * pg;
      }
#pragma unroll
      for (int k = 0; k < 9; k++) kids[k] *= d_one_kid_dn(k, D11, D12, D22);
    }
  }
  const double lF[3] = {F11, F12, F22}, lM[3] = {M11, M12, M22};
#pragma unroll
  for (int a = 0; a < 3; a++)
#pragma unroll
    for (int b = 0; b < 3; b++) cond[3 * a + b] = kids[3 * a + b] * (lF[a] * lM[b]);
}

// founders-only chunk: per person (l11, l12, l22) + per-person flags (bit0 haploid, bit1 skip)
__device__ __forceinline__ int hoist_fp(const DevArgs& A, const ItemCtx& I, const uint8_t* pl, const double* lk, int p, int cnt,
                                        double* cond) {
  int fl = 0;
  for (int j = 0; j < 3; j++) {
    if (j >= cnt) { cond[3 * j] = cond[3 * j + 1] = cond[3 * j + 2] = 0.0; fl |= 2 << (2 * j); continue; }
    const int np = A.n_person;
    double l11 = lk[PLB(pl, np, p + j, I.g11)], l12 = lk[PLB(pl, np, p + j, I.g12)], l22 = lk[PLB(pl, np, p + j, I.g22)];
    const int sx = A.sex[p + j];
    int hap = 0, skip = 0;   // lkSinglePerson :987-1004
    if (I.chrom == PM_CHR_X && sx == MALE) { l12 = 0; hap = 1; }
    if (I.chrom == PM_CHR_Y) { if (sx == MALE) { l12 = 0; hap = 1; } else skip = 1; }
    if (I.chrom == PM_CHR_MT) { l12 = 0; hap = 1; }
    cond[3 * j] = l11; cond[3 * j + 1] = l12; cond[3 * j + 2] = l22;
    fl |= (hap | (skip << 1)) << (2 * j);
  }
  return fl;
}

// ------------------------------------------------------------------------------------------------
// Elston-Stewart peeling of one extended family (FamilyLikelihoodES.cpp), one lane per family.
// Restates CalcSingleFamLikelihood_BA / _denovo (FamilyLikelihoodSeq.cpp:256-279) with FillZeroPenetrance
// (:327-356) for the posteriors: SetFounderPriors(_BA) :643-687, InitializePartials(_BA) :1434-1465,
// peelOffspring2Parents :1105-1130/:1289-1310, peelSpouse2Spouse :1182-1230/:1312-1356,
// peelParents2Offspring :1260-1286/:1358-1395, CalculateLikelihood_BA :1013-1032.  Operation order is
// the reference's, so every family likelihood is bit-identical to it.  partials[n][ns] and the marriage
// partials [couples][ns][ns] live in a per-lane HBM workspace interleaved across lanes (coalesced, L2-hot).
//
// packed step: x = type | from0 << 8 | from1 << 16 | to0 << 24, y = to1 | slot << 8 | create << 16 | fa2mo << 17
// (255 = none); slot = marriage-partial index resolved on the host (created by the first type-1 step of a couple).
__constant__ double c_TBA[5][27];   // transmission_BA, _CHRX_2Female, _CHRX_2Male, _CHRY, _MITO (:812-924)

__device__ __forceinline__ double d_tba(int i, int j, int k, int chrom, int child_sex) {   // GetTransmissionProb_BA :1059-1075
  const int o = i * 9 + j * 3 + k;
  double t = c_TBA[0][o];
  if (chrom == PM_CHR_X) t = (child_sex == MALE) ? c_TBA[2][o] : c_TBA[1][o];
  if (chrom == PM_CHR_Y) t = (child_sex == MALE) ? c_TBA[3][o] : 1.0;
  if (chrom == PM_CHR_MT) t = c_TBA[4][o];
  return t;
}

template <int NS>
__device__ __forceinline__ double d_es_lk(const DevArgs& A, int f, const uint8_t* pl, const double* lk, int g11, int g12, int g22, int chrom,
                          double freq, int zp, int zg, double* ws, size_t st) {
  const int p0 = A.fam_start[f], n = A.fam_start[f + 1] - p0, nf = A.fam_founders[f];
  const bool X = chrom == PM_CHR_X, Y = chrom == PM_CHR_Y, MT = chrom == PM_CHR_MT;
  const int gidx[3] = {g11, g12, g22};
#define PP(i, j) ws[((size_t)(i) * NS + (j)) * st]
#define MPP(sl, x, y) ws[((size_t)n * NS + (size_t)(sl) * NS * NS + (x) * NS + (y)) * st]
  for (int i = 0; i < n; i++) {
    const int sx = A.sex[p0 + i];
    const bool fo = A.is_founder[p0 + i] != 0;
    const uint8_t* R = pl + p0 + i;   // plane g at R[g * n_person]
    const size_t np = (size_t)A.n_person;
    if (NS == 3) {
      double pr[3] = {0.0, 0.0, 0.0};
      if (i < nf) {
        pr[0] = freq * freq; pr[1] = 2 * freq * (1 - freq); pr[2] = (1 - freq) * (1 - freq);
        if (X) if (sx == MALE) { pr[0] = freq; pr[1] = 0; pr[2] = 1 - freq; }
        if (Y) { if (sx == MALE) { pr[0] = freq; pr[1] = 0; pr[2] = 1 - freq; } else { pr[0] = 1; pr[1] = 1; pr[2] = 1; } }
        if (MT) { pr[0] = freq; pr[1] = 0; pr[2] = 1 - freq; }
      }
#pragma unroll
      for (int j = 0; j < 3; j++) {
        const double pen = (zp == i && gidx[j] != zg) ? 0.0 : lk[R[gidx[j] * np]];
        PP(i, j) = (Y && sx == FEMALE) ? 1.0 : (fo ? pr[j] * pen : pen);
      }
    } else {
      double pr[10];
#pragma unroll
      for (int j = 0; j < 10; j++) pr[j] = 0.0;
      if (i < nf) {
        double q0 = freq * freq, q1 = 2 * freq * (1 - freq), q2 = (1 - freq) * (1 - freq);
        if (X) if (sx == MALE) { q0 = freq; q1 = 0; q2 = 1 - freq; }
        if (Y) { if (sx == MALE) { q0 = freq; q1 = 0; q2 = 1 - freq; } else { q0 = 1; q1 = 1; q2 = 1; } }
        if (MT) { q0 = freq; q1 = 0; q2 = 1 - freq; }
        // pr[gidx[0]] = q0; pr[gidx[1]] = q1; pr[gidx[2]] = q2 (static indexing keeps pr in registers)
#pragma unroll
        for (int j = 0; j < 10; j++) pr[j] = (j == g22) ? q2 : (j == g12) ? q1 : (j == g11) ? q0 : 0.0;
      }
#pragma unroll
      for (int j = 0; j < 10; j++) {
        const double pen = (zp == i && j != zg) ? 0.0 : lk[R[j * np]];
        PP(i, j) = fo ? pr[j] * pen : pen;
      }
    }
  }
  const int s0 = A.peel_start[f], s1 = A.peel_start[f + 1];
  for (int s = s0; s < s1; s++) {
    const int2 S = A.steps[s];
    const int type = S.x & 255, from0 = (S.x >> 8) & 255, from1 = (S.x >> 16) & 255, to0 = (S.x >> 24) & 255;
    const int to1 = S.y & 255, slot = (S.y >> 8) & 255, create = (S.y >> 16) & 1, fa2mo = (S.y >> 17) & 1;
    (void)to1;
    if (type == 1) {   // offspring -> parents
      const int off = from0;
      if (create)
        for (int x = 0; x < NS; x++)
          for (int y = 0; y < NS; y++) MPP(slot, x, y) = 1.0;
      const int csex = A.sex[p0 + off];
      double pk[NS];   // the offspring's partial, read once (the workspace may alias: keep it out of the loops)
#pragma unroll
      for (int k = 0; k < NS; k++) pk[k] = PP(off, k);
      for (int i = 0; i < NS; i++)
        for (int j = 0; j < NS; j++) {
          double sum = 0;
#pragma unroll
          for (int k = 0; k < NS; k++) {
            const double t = (NS == 3) ? d_tba(i, j, k, chrom, csex) : A.T10dn[(i * 10 + j) * 10 + k];
            sum += t * pk[k];
          }
          MPP(slot, i, j) *= sum;
        }
    } else if (type == 2) {   // spouse -> spouse
      const int sf = from0, stt = to0;
      double ps[NS];
#pragma unroll
      for (int j = 0; j < NS; j++) ps[j] = PP(sf, j);
      for (int i = 0; i < NS; i++) {
        double sum = 0.0;
        if (slot == 255) for (int j = 0; j < NS; j++) sum += ps[j];
        else if (fa2mo) for (int j = 0; j < NS; j++) sum += ps[j] * MPP(slot, j, i);
        else for (int j = 0; j < NS; j++) sum += ps[j] * MPP(slot, i, j);
        PP(stt, i) *= sum;
      }
    } else {   // parents -> only offspring
      const int fa = from0, mo = from1, off = to0;
      const int csex = A.sex[p0 + off];
      // loop order (i, j) outer, k inner with NS accumulators: each sum[k] still adds its (i, j) terms in the
      // reference's order, and every term keeps its association ((fa * m) * mo) * t -- identical results,
      // with each workspace value read once instead of NS times
      double pf[NS], pm[NS], sum[NS];
#pragma unroll
      for (int k = 0; k < NS; k++) { pf[k] = PP(fa, k); pm[k] = PP(mo, k); sum[k] = 0.0; }
      for (int i = 0; i < NS; i++)
        for (int j = 0; j < NS; j++) {
          const double w = (slot == 255) ? pf[i] * pm[j] : pf[i] * MPP(slot, i, j) * pm[j];
#pragma unroll
          for (int k = 0; k < NS; k++) {
            double t;
            if (NS == 3) t = d_tba(i, j, k, chrom, csex);
            else t = (slot == 255) ? A.T10dn[(i * 10 + j) * 10 + k] : A.T10[(i * 10 + j) * 10 + k];   // quirk :1391
            sum[k] += w * t;
          }
        }
#pragma unroll
      for (int k = 0; k < NS; k++) PP(off, k) *= sum[k];
    }
  }
  const int fin = (A.steps[s1 - 1].x >> 24) & 255;
  double L = 0.0;
  for (int i = 0; i < NS; i++) L += PP(fin, i);
  return L;
#undef PP
#undef MPP
}

// ------------------------------------------------------------------------------------------------
// ------------------------------------------------------------------------------------------------
// Elston-Stewart peeling in polynomial form (PM_NUM_POLY).  Every founder prior is a homogeneous polynomial in
// (f, g = 1 - f): f^2, 2fg, g^2 (degree 2); f, 0, g on chrX/Y males and chrMT (degree 1); constants for chrY
// females (degree 0).  The peel only multiplies and adds, so a family likelihood is
//     L(f) = sum_a c_a f^a g^(D - a),   c_a >= 0,   D = the founders' degrees summed,
// and every partial / marriage-partial entry along the way is such a polynomial of a degree the host tracks per
// step (poly_layout).  The same steps as d_es_lk (FamilyLikelihoodES.cpp :1013-1032, :1105-1395) run once per
// Brent item on coefficient vectors; each objective evaluation is then one Horner pass over D + 1 non-negative
// coefficients (no cancellation: relative error ~ (D + 2) ulp, the class of PM_NUM_POLY's nuclear quartics).
// The reference-order numeric peel stays in d_es_lk (PM_NUM_PRODUCT / PM_NUM_EXACT, and the posteriors).
// register tiles of the evaluation: a polynomial of degree <= PDM as PDM + 1 coefficients (zero above its degree)
#define PDM 8

// L(f) from the coefficients: g^D sum_a c_a t^a (t = f / g <= 1) or f^D sum_a c_a s^(D - a) (s = g / f < 1)
__device__ __forceinline__ double es_poly_eval(const double* c, size_t st, int D, double x) {
  const double g = 1 - x;
  double acc, base;
  if (x <= 0.5) {
    const double t = x / g;
    acc = c[(size_t)D * st];
    for (int a = D - 1; a >= 0; a--) acc = acc * t + c[(size_t)a * st];
    base = g;
  } else {
    const double sr = g / x;
    acc = c[0];
    for (int a = 1; a <= D; a++) acc = acc * sr + c[(size_t)a * st];
    base = x;
  }
  double p = 1.0;
  for (int a = 0; a < D; a++) p *= base;
  return acc * p;
}

// es_poly_eval on register-resident coefficients (c[a] = 0 above D <= PDM): the leading zeros leave the Horner
// sum's bits unchanged (0 * t + c = c)
#define PM_EPE 4   // extended families per lane whose coefficients stay in registers through an item's evaluations
__device__ __forceinline__ double es_poly_eval_r(const double* c, int D, double x) {
  const double g = 1 - x;
  double acc = 0.0, base;
  if (x <= 0.5) {
    const double t = x / g;
#pragma unroll
    for (int a = PDM; a >= 0; a--) acc = acc * t + c[a];
    base = g;
  } else {
    const double sr = g / x;
#pragma unroll
    for (int a = 0; a <= PDM; a++) acc = a <= D ? acc * sr + c[a] : acc;
    base = x;
  }
  double p = 1.0;
#pragma unroll
  for (int a = 0; a < PDM; a++) p = a < D ? p * base : p;
  return acc * p;
}

template <int T>
__device__ __forceinline__ double block_sum(double x, double* red, int& par) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);   // commutative butterfly: identical in all lanes
  if (T == 64) return x;
  constexpr int W = T / 64;
  if ((threadIdx.x & 63) == 0) red[par * 16 + (threadIdx.x >> 6)] = x;
  __syncthreads();
  double s = red[par * 16];
#pragma unroll
  for (int i = 1; i < W; i++) s += red[par * 16 + i];
  par ^= 1;
  return s;
}

template <int T>
__device__ __forceinline__ void block_sum3(double& x, double& y, double& z, double* red, int& par) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { x += __shfl_xor(x, o, 64); y += __shfl_xor(y, o, 64); z += __shfl_xor(z, o, 64); }
  if (T == 64) return;
  constexpr int W = T / 64;
  if ((threadIdx.x & 63) == 0) {
    red[par * 16 + (threadIdx.x >> 6)] = x;
    red[32 + par * 16 + (threadIdx.x >> 6)] = y;
    red[64 + par * 16 + (threadIdx.x >> 6)] = z;
  }
  __syncthreads();
  double sx = red[par * 16], sy = red[32 + par * 16], sz = red[64 + par * 16];
#pragma unroll
  for (int i = 1; i < W; i++) { sx += red[par * 16 + i]; sy += red[32 + par * 16 + i]; sz += red[64 + par * 16 + i]; }
  x = sx; y = sy; z = sz;
  par ^= 1;
}

// per-lane partial of CalcAllFamLogLikelihood(freq) over the lane's units
template <int S, bool GEN>
__device__ __forceinline__ double lane_loglik(double f, const int4* unit, const double (*cond)[9], const int* fl, int pmode,
                                              bool log_each = false) {
  double pp[9];
  d_parent_prior(pmode, f, pp);
  const double g = 1 - f;
  const double P0 = f * f, P1 = f * g * 2, P2 = g * g;   // lkSinglePerson priors
  double part = 0.0, prod = 1.0;
#pragma unroll
  for (int s = 0; s < S; s++) {
    const int ty = unit[s].x;
    if (ty == U_NUC) {
      double v = 0.0;   // lkSingleFam :950-955
#pragma unroll
      for (int k = 0; k < 9; k++) v += cond[s][k] * pp[k];
      part += log10(v);
    } else if (GEN && ty == U_FP) {
      if (unit[s].w & UF_FIRST) prod = 1.0;
#pragma unroll
      for (int j = 0; j < 3; j++) {
        const int b = (fl[s] >> (2 * j)) & 3;
        if (b & 2) continue;
        double sp = 0.0;
        if (b & 1) sp = sp + cond[s][3 * j] * f + cond[s][3 * j + 1] * 0 + cond[s][3 * j + 2] * g;
        else sp = sp + cond[s][3 * j] * P0 + cond[s][3 * j + 1] * P1 + cond[s][3 * j + 2] * P2;
        if (log_each) part += log10(sp);   // VCF path: sum of per-person log10
        else prod *= sp;
      }
      if (!log_each && (unit[s].w & UF_LAST)) part += log10(prod);
    }
  }
  return part;
}

// Product-mode objective: instead of summing log10 of every family likelihood (one log10 per family),
// each lane multiplies its families' likelihoods into a normalised (mantissa, exponent) pair, the block
// reduces the pairs by multiplication, and one log10 per evaluation turns the product into
// CalcAllFamLogLikelihood.  Sum-of-logs == log-of-product exactly in real arithmetic; the floating-point
// result is at least as accurate as the reference's serial sum (DESIGN.md "Numerics").
#define PM_LOG10_2_HI 0x1.3441350800000p-2
#define PM_LOG10_2_LO 0x1.f79fef311f12bp-34

template <int S, bool GEN>
__device__ __forceinline__ void lane_prod(double f, const int4* unit, const double (*cond)[9], const int* fl, int pmode, double& m,
                                          int& e) {
  double pp[9];
  d_parent_prior(pmode, f, pp);
  const double g = 1 - f;
  const double P0 = f * f, P1 = f * g * 2, P2 = g * g;
  // every slot's likelihood is normalised independently (no serial chain), then the mantissas
  // (each in [0.5, 1)) are multiplied as a tree and the exponents summed.
  double mv[S];
  int ev[S];
#pragma unroll
  for (int s = 0; s < S; s++) {
    const int ty = unit[s].x;
    double v = 1.0;
    if (ty == U_NUC) {
      v = 0.0;
#pragma unroll
      for (int k = 0; k < 9; k++) v += cond[s][k] * pp[k];
    } else if (GEN && ty == U_FP) {
#pragma unroll
      for (int j = 0; j < 3; j++) {
        const int b = (fl[s] >> (2 * j)) & 3;
        if (b & 2) continue;
        double sp = 0.0;
        if (b & 1) sp = sp + cond[s][3 * j] * f + cond[s][3 * j + 1] * 0 + cond[s][3 * j + 2] * g;
        else sp = sp + cond[s][3 * j] * P0 + cond[s][3 * j + 1] * P1 + cond[s][3 * j + 2] * P2;
        v *= sp;   // <= 3 persons: no underflow before normalisation
      }
    }
    mv[s] = frexp(v, &ev[s]);
  }
#pragma unroll
  for (int w = 1; w < S; w *= 2)
#pragma unroll
    for (int s = 0; s + w < S; s += 2 * w) {
      int x;
      mv[s] = frexp(mv[s] * mv[s + w], &x);
      ev[s] += ev[s + w] + x;
    }
  m = mv[0];
  e = ev[0];
}

// Lean product mode (autosomal HWE parent prior, nuclear families only): a family's likelihood
// Sum_k cond[k] * SetParentPrior(f)[k] is the quartic f^4 a0 + f^3 g a1 + f^2 g^2 a2 + f g^3 a3 + g^4 a4
// (a0 = c0, a1 = 2(c1+c3), a2 = c2+4c4+c6, a3 = 2(c5+c7), a4 = c8; SetParentPrior :323-331).  With
// M = max(f, g) and t = min(f, g)/M <= 1 it is M^4 h(t), h a 4-FMA Horner polynomial with non-negative
// coefficients (no cancellation: relative error <= ~8 ulp); M^(4 nFam) leaves the product as one log10.
// Empty lane slot: the "phantom family" (f + g)^4 = 1 -- coefficients (1, 4, 6, 4, 1) -- so lane_poly_r
// needs no per-slot mask.  In floating point g^4 h(r) = ((1 + r) g)^4 is 1 to within a few ulp.
__device__ __forceinline__ void phantom_poly(double* a) { a[0] = 1.0; a[1] = 4.0; a[2] = 6.0; a[3] = 4.0; a[4] = 1.0; }

__device__ __forceinline__ void fold_poly(const double* c, double* a) {
  a[0] = c[0];
  a[1] = 2 * (c[1] + c[3]);
  a[2] = c[2] + 4 * c[4] + c[6];
  a[3] = 2 * (c[5] + c[7]);
  a[4] = c[8];
}

// Lean kernels keep the lane plan in LDS, one int per (slot, lane): 0 = empty slot, else a nuclear family
// as first person | persons << 24 (k_brent fills it once per block; no global round trip per item).
__device__ __forceinline__ int unit_pack(const int4 u) { return u.x == U_NUC ? (u.z | (u.w << 24)) : 0; }
__device__ __forceinline__ int unit_nn(int u) { return (int)((unsigned)u >> 24); }
__device__ __forceinline__ int unit_first(int u) { return u & 0xFFFFFF; }
// The lane's S packed units, stored lane-major (s_u[lane * S + slot]) so they arrive in S/4 16-B LDS reads
// at the start of the hoisting, before any coefficient register is live.
template <int S>
__device__ __forceinline__ void load_units(const int* su, int* uu) {
  const int* p = su + threadIdx.x * S;
  if constexpr (S % 4 == 0) {
#pragma unroll
    for (int s = 0; s < S; s += 4) {
      const int4 v = *(const int4*)(p + s);
      uu[s] = v.x; uu[s + 1] = v.y; uu[s + 2] = v.z; uu[s + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int s = 0; s < S; s++) uu[s] = p[s];
  }
}


// One nuclear family's quartic coefficients from its PL bytes by[3q + {0,1,2}] = (g11, g12, g22) of person q
// (father, mother, kids), nn persons (0 = empty slot -> the phantom family).  Branch-free: lanes whose
// family has fewer persons multiply by exactly 1.0 and select, so no exec-masked regions (and no waits
// per region) are generated; the arithmetic and its order are hoist_nuc's.
__device__ __forceinline__ void fam_poly4(const uint32_t* by, int nn, const double* lk, double* a) {
  double kids[9];
#pragma unroll
  for (int k = 0; k < 9; k++) kids[k] = 1.0;
#pragma unroll
  for (int q = 2; q < 4; q++) {
    // a missing kid reads l = 1: every autosomal d_one_kid term is then exactly 1.0 (0.5 * (1 + 1),
    // 0.25 + 0.5 + 0.25), the factor the reference never multiplies in -- three selects instead of nine
    const bool kid = q < nn;
    const double l11 = kid ? lk[by[3 * q]] : 1.0, l12 = kid ? lk[by[3 * q + 1]] : 1.0, l22 = kid ? lk[by[3 * q + 2]] : 1.0;
#pragma unroll
    for (int k = 0; k < 9; k++) kids[k] *= d_one_kid(k, PM_CHR_AUTO, 0, l11, l12, l22);
  }
  // no parents (empty slot): lF = 0 makes every term +0 (all values finite and >= 0)
  const bool fam = nn >= 2;
  const double lF[3] = {fam ? lk[by[0]] : 0.0, fam ? lk[by[1]] : 0.0, fam ? lk[by[2]] : 0.0};
  const double lM[3] = {lk[by[3]], lk[by[4]], lk[by[5]]};
  double c9[9];
#pragma unroll
  for (int x = 0; x < 3; x++)
#pragma unroll
    for (int y = 0; y < 3; y++) c9[3 * x + y] = kids[3 * x + y] * (lF[x] * lM[y]);
  fold_poly(c9, a);
  if (nn == 0) {   // empty slot: the phantom family (f + g)^4 (selects, not a branch)
    a[0] = 1.0; a[1] = 4.0; a[2] = 6.0; a[3] = 4.0; a[4] = 1.0;
  }
}

// Chunked hoisting for the lean polynomial kernel when every nuclear family has <= 4 persons: the PL
// bytes of 4 slots (4 x 12 loads) are issued before any of them is used, so the HBM round trips of a
// chunk overlap instead of running slot after slot.  Arithmetic is hoist_nuc's, in the same order.
template <int S, int T>
__device__ __forceinline__ void hoist_poly4(const DevArgs& A, const int* su, const ItemCtx& I, const uint8_t* pl, const double* lk,
                                            double (*a)[5]) {
  constexpr int C = S < PM_HOIST_CHUNK ? S : PM_HOIST_CHUNK;
  const size_t np = (size_t)A.n_person;
  const uint8_t* P11 = pl + I.g11 * np;   // the three genotype planes of the item
  const uint8_t* P12 = pl + I.g12 * np;
  const uint8_t* P22 = pl + I.g22 * np;
  int uu[S];
  load_units<S>(su, uu);
#pragma unroll
  for (int c0 = 0; c0 < S; c0 += C) {
    uint32_t by[C][12];
    int nn[C];
#pragma unroll
    for (int j = 0; j < C; j++) {
      const int u = uu[c0 + j];
      nn[j] = unit_nn(u);
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int pp = unit_first(u) + (q < nn[j] ? q : 0);   // in range for every lane: no branch around the load
        by[j][3 * q + 0] = P11[pp];
        by[j][3 * q + 1] = P12[pp];
        by[j][3 * q + 2] = P22[pp];
      }
    }
#pragma unroll
    for (int j = 0; j < C; j++) fam_poly4(by[j], nn[j], lk, a[c0 + j]);
  }
}

// Item -> allele pair (cfg_alleles, the VCF path's (ref, alt), the cfg-7 re-optimisation's alleles).
__device__ __forceinline__ void item_alleles(const DevArgs& A, int site, int cfg, int r, int* a1, int* a2) {
  if (A.vcf) { *a1 = r & 15; *a2 = r >> 4; }
  else if (cfg == 7) { *a1 = A.res[site].allele1; *a2 = A.res[site].allele2; }
  else cfg_alleles(cfg, r, a1, a2);
}

// Lean-kernel plane prefetch: the three genotype planes (g11, g12, g22) of an item's site block are
// copied into this wave's LDS buffer with LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave-instruction,
// no VGPRs), issued right after the previous item's hoisting so the copy runs under that item's Brent
// evaluations.  16-B pieces need n_person % 16 == 0 (16-B aligned planes); with n_person % 4 == 0 (pf_dw) the
// copy goes in 4-B pieces (256 B per wave-instruction).  Lanes past a plane's end re-read its last piece (never
// used), so no access leaves the site block.  The waves of a multi-wave block split the pieces.
__device__ __forceinline__ void prefetch_planes(const DevArgs& A, const int* items, int it, int nItems, uint8_t* buf) {
  if (it >= nItems) return;
  const int item = items[it];
  const int site = item >> 3, cfg = item & 7;
  int a1, a2;
  item_alleles(A, site, cfg, A.ref[site], &a1, &a2);
  const int np = A.n_person, npad = A.pf_npad;
  const int gs[3] = {d_gi(a1, a1), d_gi(a1, a2), d_gi(a2, a2)};
  const uint8_t* base = A.pl + (size_t)site * np * 10;
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), W = blockDim.x >> 6;
  if (A.pf_dw) {
#pragma unroll
    for (int k = 0; k < 3; k++) {
      const uint8_t* plane = base + (size_t)gs[k] * np;
      for (int c = wv * 256; c < np; c += W * 256) {
        const int off = min(c + lane * 4, np - 4);
        __builtin_amdgcn_global_load_lds((const void*)(plane + off), (void*)(buf + k * npad + c), 4, 0, 0);
      }
    }
    return;
  }
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const uint8_t* plane = base + (size_t)gs[k] * np;
    for (int c = wv * 1024; c < npad; c += W * 1024) {
      const int off = min(c + lane * 16, np - 16);
      __builtin_amdgcn_global_load_lds((const void*)(plane + off), (void*)(buf + k * npad + c), 16, 0, 0);
    }
  }
}

// hoist_poly4 reading the item's planes from the LDS buffer of prefetch_planes (same arithmetic and order).
#ifndef PM_HOIST_CHUNK_LDS
#define PM_HOIST_CHUNK_LDS 2
#endif
template <int S, int T>
__device__ __forceinline__ void hoist_poly4_lds(const DevArgs& A, const int* su, const uint8_t* buf, const double* lk,
                                                double (*a)[5]) {
  const int npad = A.pf_npad;
  constexpr int C = S < PM_HOIST_CHUNK_LDS ? S : PM_HOIST_CHUNK_LDS;
  int uu[S];
  load_units<S>(su, uu);
#pragma unroll
  for (int s = 0; s < S; s++) {
    if (s % C == 0) __builtin_amdgcn_sched_barrier(0);   // chunks of C slots: bounded registers in flight
    const int u = uu[s];
    const int nn = unit_nn(u);
    uint32_t by[12];
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int pp = unit_first(u) + (q < nn ? q : 0);   // in range for every lane: no branch around the read
      by[3 * q + 0] = buf[pp];
      by[3 * q + 1] = buf[npad + pp];
      by[3 * q + 2] = buf[2 * npad + pp];
    }
    fam_poly4(by, nn, lk, a[s]);
  }
}

// De novo variant of hoist_poly4 (autosomal --denovo items, families of <= 4 persons): the kid terms are
// likelihoodONEKid_denovo's CalcDenovoMutLk dot products over all 10 genotype likelihoods (:1553-1562,
// :1266-1296), so each kid's whole 10-byte PL record is loaded.  Chunks of PM_HOIST_CHUNK_DN slots keep
// the in-flight bytes small next to the 5 x S hoisted coefficients.  Arithmetic is hoist_nuc's, same order.
#ifndef PM_HOIST_CHUNK_DN
#define PM_HOIST_CHUNK_DN 2
#endif
template <int S, int T>
__device__ __forceinline__ void hoist_poly4_dn(const DevArgs& A, const int* su, const ItemCtx& I, const uint8_t* pl, const double* lk,
                                               const double* M, double (*a)[5]) {
  constexpr int C = S < PM_HOIST_CHUNK_DN ? S : PM_HOIST_CHUNK_DN;
  const size_t np = (size_t)A.n_person;
  int uu[S];
  load_units<S>(su, uu);
#pragma unroll
  for (int c0 = 0; c0 < S; c0 += C) {
    uint32_t par[C][6], kid[C][2][10];
    int nn[C];
    // mutation-matrix rows: laundered per chunk so the compiler re-reads them from LDS instead of keeping
    // all 30 doubles live across the whole hoisting phase (which spills the 5 x S coefficients)
    int r11 = I.g11 * 10, r12 = I.g12 * 10, r22 = I.g22 * 10;
    asm volatile("" : "+v"(r11), "+v"(r12), "+v"(r22));   // (scalar loads from global memory instead: slower)
#pragma unroll
    for (int j = 0; j < C; j++) {
      const int u = uu[c0 + j];
      nn[j] = unit_nn(u);
#pragma unroll
      for (int q = 0; q < 2; q++) {
        const uint8_t* R = pl + unit_first(u) + (q < nn[j] ? q : 0);   // in range: no branch around the loads
        par[j][3 * q + 0] = R[I.g11 * np];
        par[j][3 * q + 1] = R[I.g12 * np];
        par[j][3 * q + 2] = R[I.g22 * np];
      }
#pragma unroll
      for (int q = 0; q < 2; q++) {
        const uint8_t* R = pl + unit_first(u) + (q + 2 < nn[j] ? q + 2 : 0);
#pragma unroll
        for (int g = 0; g < 10; g++) kid[j][q][g] = R[g * np];
      }
    }
#pragma unroll
    for (int j = 0; j < C; j++) {   // branch-free over the lanes' family sizes (see fam_poly4)
      double kids[9];
#pragma unroll
      for (int k = 0; k < 9; k++) kids[k] = 1.0;
#pragma unroll
      for (int q = 0; q < 2; q++) {
        double D11 = 0.0, D12 = 0.0, D22 = 0.0;
        if (I.denovo) {   // uniform per item
#pragma unroll
          for (int g = 0; g < 10; g++) {
            const double pg = lk[kid[j][q][g]];
            // fused multiply-add: <= 1 ulp from the reference's mul + add (POLY numerics)
            D11 = fma(M[r11 + g], pg, D11);
            D12 = fma(M[r12 + g], pg, D12);
            D22 = fma(M[r22 + g], pg, D22);
          }
        } else {   // cfg-7 items: likelihoodONEKid's autosomal terms are d_one_kid_dn's on (l11, l12, l22)
          uint32_t b11 = 0, b12 = 0, b22 = 0;   // register selects (a dynamic index would go to scratch)
#pragma unroll
          for (int g = 0; g < 10; g++) {
            b11 = g == I.g11 ? kid[j][q][g] : b11;
            b12 = g == I.g12 ? kid[j][q][g] : b12;
            b22 = g == I.g22 ? kid[j][q][g] : b22;
          }
          D11 = lk[b11]; D12 = lk[b12]; D22 = lk[b22];
        }
        const bool isKid = q + 2 < nn[j];   // a missing kid: D = 1, every term exactly 1.0 (fam_poly4)
        D11 = isKid ? D11 : 1.0; D12 = isKid ? D12 : 1.0; D22 = isKid ? D22 : 1.0;
#pragma unroll
        for (int k = 0; k < 9; k++) kids[k] *= d_one_kid_dn(k, D11, D12, D22);
      }
      const bool fam = nn[j] >= 2;
      const double lF[3] = {fam ? lk[par[j][0]] : 0.0, fam ? lk[par[j][1]] : 0.0, fam ? lk[par[j][2]] : 0.0};
      const double lM[3] = {lk[par[j][3]], lk[par[j][4]], lk[par[j][5]]};
      double c9[9];
#pragma unroll
      for (int x = 0; x < 3; x++)
#pragma unroll
        for (int y = 0; y < 3; y++) c9[3 * x + y] = kids[3 * x + y] * (lF[x] * lM[y]);
      fold_poly(c9, a[c0 + j]);
      if (nn[j] == 0) {   // empty slot: the phantom family (selects)
        a[c0 + j][0] = 1.0; a[c0 + j][1] = 4.0; a[c0 + j][2] = 6.0; a[c0 + j][3] = 4.0; a[c0 + j][4] = 1.0;
      }
    }
    __builtin_amdgcn_sched_barrier(0);   // keep the next chunk's loads from being hoisted above this one
  }
}

// hoist_poly4_dn with the PL bytes staged through LDS by LDS-DMA (A.dn_pf): the lean plan deals families
// round-robin, so the 64 families of one wave in one slot row are consecutive and their persons form one
// window of <= 256 bytes per genotype plane.  A chunk of DN_PF_C slots needs 10 planes x DN_PF_C windows
// (272 B each: the 16-B aligned start plus slack), fetched with global_load_lds_dwordx4 into this wave's
// half of a double buffer while the previous chunk is hoisted; every byte is then an LDS read.  Needs
// n_person % 16 == 0 (16-B aligned planes).  Arithmetic and order are hoist_poly4_dn's.
#ifndef DN_PF_C
#define DN_PF_C 1
#endif
#define DN_PF_WIN 272
typedef const __attribute__((address_space(3))) double* lds_cdp;   // an LDS pointer (32-bit, ds_* addressing)
#define DN_PF_BUF ((10 * DN_PF_C * DN_PF_WIN + 1023) / 1024 * 1024)   // per wave per chunk (C = 1: 2720 B as 3 x 1 KB)
__device__ __forceinline__ void dn_pf_issue(const DevArgs& A, const uint8_t* pl, const int* start_al, uint8_t* dst) {
  const int lane = threadIdx.x & 63, np = A.n_person;
#pragma unroll
  for (int i = 0; i < DN_PF_BUF / 1024; i++) {
    int P = i * 1024 + lane * 16;
    if (P >= 10 * DN_PF_C * DN_PF_WIN) P = 10 * DN_PF_C * DN_PF_WIN - 16;   // tail lanes: any valid source
    const int w = P / DN_PF_WIN, j = w / 10, g = w - 10 * j, off = P - w * DN_PF_WIN;
    const int src = min(start_al[j] + off, np - 16);
    __builtin_amdgcn_global_load_lds((const void*)(pl + (size_t)g * np + src), (void*)(dst + i * 1024), 16, 0, 0);
  }
}

template <int S, int T>
__device__ __forceinline__ void hoist_poly4_dn_pf(const DevArgs& A, const int* su, const ItemCtx& I, const uint8_t* pl,
                                                  const double* lk, const double* M, double (*a)[5],
                                                  uint8_t* wbuf) {
  static_assert(S % DN_PF_C == 0, "chunking");
  constexpr int C = DN_PF_C;
  const int wv = threadIdx.x >> 6;
  int uu[S];
  load_units<S>(su, uu);
  // window start per slot: the first person of this wave's lane-0 family (uniform), aligned down to 16 B
  int start_al[S];
#pragma unroll
  for (int s = 0; s < S; s++) start_al[s] = __builtin_amdgcn_readfirstlane(unit_first(su[(wv * 64) * S + s]) & ~15);
  __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): the previous item's reads of this wave's buffers are done
  __builtin_amdgcn_sched_barrier(0);
  dn_pf_issue(A, pl, start_al, wbuf);
#pragma unroll
  for (int c0 = 0; c0 < S; c0 += C) {
    uint8_t* cur = wbuf + ((c0 / C) & 1) * DN_PF_BUF;
    if (c0 + C < S) {
      __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): the reads of the buffer about to be refilled are done
      __builtin_amdgcn_sched_barrier(0);
      dn_pf_issue(A, pl, start_al + c0 + C, wbuf + (((c0 / C) + 1) & 1) * DN_PF_BUF);
      static_assert(DN_PF_BUF / 1024 <= 15, "vmcnt field");
      __builtin_amdgcn_s_waitcnt(0x0F70 | (DN_PF_BUF / 1024));   // vmcnt(#DMA of the next chunk): this chunk's have landed
    } else {
      __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
    }
    __builtin_amdgcn_sched_barrier(0);
    // the item's three mutation-matrix rows, as LDS addresses made opaque once per chunk: the 30 entries are
    // re-read per slot (holding them would take 60 VGPRs) with the entry offsets folded into ds_read2_b64
    lds_cdp M11 = (lds_cdp)(M + I.g11 * 10), M12 = (lds_cdp)(M + I.g12 * 10), M22 = (lds_cdp)(M + I.g22 * 10);
    asm volatile("" : "+v"(M11), "+v"(M12), "+v"(M22));
#pragma unroll
    for (int j = 0; j < C; j++) {
      const int u = uu[c0 + j];
      const int nn = unit_nn(u);
      const uint8_t* W = cur + j * 10 * DN_PF_WIN;   // plane g of this slot at W[g * DN_PF_WIN + person - start]
      const int rel = u ? unit_first(u) - start_al[c0 + j] : 0;
      // every PL byte of the slot first (one LDS round trip), then every table lookup (a second), then the
      // arithmetic: a byte -> lk[byte] -> fma chain per genotype costs two LDS latencies per term otherwise
      uint32_t par[6], kb[2][10];
#pragma unroll
      for (int q = 0; q < 2; q++) {
        const int pp = rel + (q < nn ? q : 0);
        par[3 * q + 0] = W[I.g11 * DN_PF_WIN + pp];
        par[3 * q + 1] = W[I.g12 * DN_PF_WIN + pp];
        par[3 * q + 2] = W[I.g22 * DN_PF_WIN + pp];
      }
      const int dnv = I.denovo;   // uniform per item
#pragma unroll
      for (int q = 0; q < 2; q++) {
        const int pk = rel + (q + 2 < nn ? q + 2 : 0);
        if (dnv) {
#pragma unroll
          for (int g = 0; g < 10; g++) kb[q][g] = W[g * DN_PF_WIN + pk];
        } else {   // cfg-7 items: likelihoodONEKid's autosomal terms need the item's three planes only
          kb[q][0] = W[I.g11 * DN_PF_WIN + pk]; kb[q][1] = W[I.g12 * DN_PF_WIN + pk]; kb[q][2] = W[I.g22 * DN_PF_WIN + pk];
#pragma unroll
          for (int g = 3; g < 10; g++) kb[q][g] = 0;
        }
      }
      __builtin_amdgcn_sched_barrier(0);   // (the scheduler would sink each byte read back into its chain)
      double kids[9];
#pragma unroll
      for (int k = 0; k < 9; k++) kids[k] = 1.0;
      double DK[2][3];   // (D11, D12, D22) per kid
      if (dnv) {
        double pg[2][10];   // both kids' twenty table lookups in flight together
#pragma unroll
        for (int q = 0; q < 2; q++)
#pragma unroll
          for (int g = 0; g < 10; g++) pg[q][g] = lk[kb[q][g]];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < 2; q++) DK[q][0] = DK[q][1] = DK[q][2] = 0.0;
#pragma unroll
        for (int g = 0; g < 10; g++) {   // each mutation-matrix entry read once for both kids (same per-kid order)
          const double m11 = M11[g], m12 = M12[g], m22 = M22[g];
#pragma unroll
          for (int q = 0; q < 2; q++) {
            DK[q][0] = fma(m11, pg[q][g], DK[q][0]);
            DK[q][1] = fma(m12, pg[q][g], DK[q][1]);
            DK[q][2] = fma(m22, pg[q][g], DK[q][2]);
          }
        }
      } else {
#pragma unroll
        for (int q = 0; q < 2; q++) { DK[q][0] = lk[kb[q][0]]; DK[q][1] = lk[kb[q][1]]; DK[q][2] = lk[kb[q][2]]; }
      }
#pragma unroll
      for (int q = 0; q < 2; q++) {
        // a missing kid gets D = 1: every d_one_kid_dn term is then exactly 1.0 (0.5 * (1 + 1), 0.25 + 0.5 + 0.25),
        // the factor the reference's loop never multiplies in -- three selects instead of nine
        const bool isKid = q + 2 < nn;
        const double D11 = isKid ? DK[q][0] : 1.0, D12 = isKid ? DK[q][1] : 1.0, D22 = isKid ? DK[q][2] : 1.0;
#pragma unroll
        for (int k = 0; k < 9; k++) kids[k] *= d_one_kid_dn(k, D11, D12, D22);
      }
      // no parents (empty or founder-only slot): lF = 0 makes every term +0 (all values finite, >= 0)
      const bool fam = nn >= 2;
      const double lF[3] = {fam ? lk[par[0]] : 0.0, fam ? lk[par[1]] : 0.0, fam ? lk[par[2]] : 0.0};
      const double lM[3] = {lk[par[3]], lk[par[4]], lk[par[5]]};
      double c9[9];
#pragma unroll
      for (int x = 0; x < 3; x++)
#pragma unroll
        for (int y = 0; y < 3; y++) c9[3 * x + y] = kids[3 * x + y] * (lF[x] * lM[y]);
      fold_poly(c9, a[c0 + j]);
      if (nn == 0) {
        a[c0 + j][0] = 1.0; a[c0 + j][1] = 4.0; a[c0 + j][2] = 6.0; a[c0 + j][3] = 4.0; a[c0 + j][4] = 1.0;
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// ---- QUAD plan (lean --denovo kernel; pm_engine::quad): families are 4-person nuclear families stored in order
// (family f = persons 4f..4f+3) and dealt round-robin, so slot row s of the wave holds families 64 s + lane and
// its persons are the 256-byte window [256 s, 256 s + 256) of every genotype plane, one aligned dword per lane
// (father, mother, kid 1, kid 2).  Each slot's ten windows arrive in LDS by three LDS-DMA instructions (lane l
// of instruction i copies 16 bytes of plane 4 i + l / 16: per-lane source offsets fixed for the kernel, the slot
// in the scalar base) into a ring of QB slot buffers, QD_AHEAD slots ahead of the hoisting; the next item's
// first QD_AHEAD slots are fetched while this item's Brent runs.  A slot is then 13 conflict-free ds_read_b32
// and 26 table lookups -- no per-byte address arithmetic, no per-family selects (only the partial last slot row
// needs the phantom family).
#define QB 3
#define QD_AHEAD 2
#define QSLOT 3072   // 10 planes x 256 B + the third DMA instruction's tail
#define QWAVE (QB * QSLOT)

// Per-lane source offset of DMA instruction i within a slot window (plane 4 i + lane / 16, 16 B per lane); lanes
// past plane 9 re-read plane 9 (their bytes land in the buffer's tail and are never read).
__device__ __forceinline__ uint32_t quad_voff(int i, int np) {
  const int lane = threadIdx.x & 63, g = min(4 * i + (lane >> 4), 9);
  return (uint32_t)(g * np + (lane & 15) * 16);
}

// DMA of slot row s of one site block into an LDS slot buffer.  Rows that reach past the plane end (the partial
// last row) clamp each lane's window start so that no read leaves the site block.  (Unsigned 32-bit lane offsets
// on a uniform base: the scalar-base + vector-offset form of the DMA instruction, no 64-bit address per lane.)
__device__ __forceinline__ void quad_dma(const uint8_t* site, int s, int np, const uint32_t* voff, uint8_t* dst) {
  if (256 * (s + 1) <= np) {
    const uint8_t* src = site + 256 * s;
    asm volatile("" : "+s"(src));   // an opaque scalar base: each lane adds only its 32-bit offset (saddr form)
#pragma unroll
    for (int i = 0; i < 3; i++) __builtin_amdgcn_global_load_lds((const void*)(src + voff[i]), (void*)(dst + i * 1024), 16, 0, 0);
  } else {
    int lane = threadIdx.x & 63;
    asm volatile("" : "+v"(lane));   // (no per-slot offsets hoisted out of the item loop)
    const int o = min(256 * s + (lane & 15) * 16, np - 16);
#pragma unroll
    for (int i = 0; i < 3; i++) {
      const int g = min(4 * i + (lane >> 4), 9);
      __builtin_amdgcn_global_load_lds((const void*)(site + (uint32_t)(g * np + o)), (void*)(dst + i * 1024), 16, 0, 0);
    }
  }
}

// One dword into LDS by LDS-DMA, every lane copying the same source (dst[0..63] all hold it).
__device__ __forceinline__ void quad_aux(const void* src, int* dst) {
  __builtin_amdgcn_global_load_lds(src, (void*)dst, 4, 0, 0);
}

// The first QD_AHEAD slots of an item (issued ahead: before the previous item's Brent loop).
__device__ __forceinline__ void quad_prefetch(const DevArgs& A, int item, const uint32_t* voff, uint8_t* ring) {
  const int site = item >> 3;
  int np = A.n_person;
  asm volatile("" : "+s"(np));   // (keeps the clamped-row offsets from being hoisted out of the item loop)
  const uint8_t* pl = A.pl + (size_t)site * np * 10;
#pragma unroll
  for (int s = 0; s < QD_AHEAD; s++) quad_dma(pl, s, np, voff, ring + s * QSLOT);
}

// One family's quartic from its kid terms (D[q] = (D11, D12, D22) of kid q: CalcDenovoMutLk's dot products for de
// novo items, (l11, l12, l22) otherwise) and parent likelihoods: the sums of hoist_nuc's c9 that share a kid factor
// (likelihoodONEKid(_denovo) gives k = 1, 3 / 2, 6 / 5, 7 equal terms, :1202-1296) are factored, and the powers of
// two of those terms (0.5, 0.25) are applied once at the end (exact scalings).  Equal to fold_poly(c9) in real
// arithmetic; non-negative throughout (POLY numerics).
__device__ __forceinline__ void quad_poly4(const double (*D)[3], const double* lF, const double* lM, double* a) {
  double At[2], Bt[2], Ct[2];
#pragma unroll
  for (int q = 0; q < 2; q++) {
    At[q] = D[q][0] + D[q][1];                     // 2 x likelihoodONEKid k = 1, 3
    Bt[q] = D[q][1] + D[q][2];                     // 2 x k = 5, 7
    Ct[q] = fma(2.0, D[q][1], D[q][0]) + D[q][2];  // 4 x k = 4
  }
  const double P0 = D[0][0] * D[1][0], P2 = D[0][1] * D[1][1], P8 = D[0][2] * D[1][2];
  const double PA = At[0] * At[1], PB = Bt[0] * Bt[1], PC = Ct[0] * Ct[1];
  const double s01 = fma(lF[0], lM[1], lF[1] * lM[0]);
  const double s02 = fma(lF[0], lM[2], lF[2] * lM[0]);
  const double s12 = fma(lF[1], lM[2], lF[2] * lM[1]);
  a[0] = P0 * (lF[0] * lM[0]);
  a[1] = (0.5 * PA) * s01;
  a[2] = fma(P2, s02, (0.25 * PC) * (lF[1] * lM[1]));
  a[3] = (0.5 * PB) * s12;
  a[4] = P8 * (lF[2] * lM[2]);
}

// QUAD hoisting of one item: slots 0 .. QD_AHEAD - 1 are already in the ring (quad_prefetch).  vmcnt counts in
// issue order (loads, stores and LDS-DMA together), so waiting until only the next slot's three DMA instructions
// may be outstanding means this slot's have landed.
template <int S, bool DNV>
__device__ __forceinline__ void hoist_quad_t(const DevArgs& A, const ItemCtx& I, const uint8_t* pl, const double* lk,
                                             const double* M, double (*a)[5], uint8_t* ring, const uint32_t* voff) {
  const int lane = threadIdx.x & 63;
  const uint32_t* rw = (const uint32_t*)ring + lane;   // the lane's dword of plane g, slot buffer b: rw[(b * QSLOT + g * 256) / 4]
  const int o11 = I.g11 * 64, o12 = I.g12 * 64, o22 = I.g22 * 64;
  // re-read per item (opaque), so the compiler does not keep S slot predicates live across the Brent loop
  int qfull = A.quad_full, nfam = A.n_fam, npo = A.n_person;
  asm volatile("" : "+s"(qfull), "+s"(nfam), "+s"(npo));
#pragma unroll
  for (int s = 0; s < S; s++) {
    if (s + 1 < S) __builtin_amdgcn_s_waitcnt(0x0F70 | 3);   // vmcnt(3): slot s has landed
    else __builtin_amdgcn_s_waitcnt(0x0F70);                   // vmcnt(0)
    __builtin_amdgcn_sched_barrier(0);
    const uint32_t* b = rw + (s % QB) * (QSLOT / 4);
    // byte j of a plane dword: person j of the family (0 father, 1 mother, 2 / 3 kids)
    uint32_t w[3];   // planes g11, g12, g22
    w[0] = b[o11]; w[1] = b[o12]; w[2] = b[o22];
    double lF[3], lM[3], D[2][3];
    if constexpr (DNV) {
      uint32_t wg[10];   // planes 0-9
#pragma unroll
      for (int g = 0; g < 10; g++) wg[g] = b[g * 64];
#pragma unroll
      for (int k = 0; k < 3; k++) { lF[k] = lk[w[k] & 0xFF]; lM[k] = lk[(w[k] >> 8) & 0xFF]; }
      double pg[2][10];   // both kids' 20 table lookups in flight together
#pragma unroll
      for (int g = 0; g < 10; g++) { pg[0][g] = lk[(wg[g] >> 16) & 0xFF]; pg[1][g] = lk[wg[g] >> 24]; }
      // the item's three mutation-matrix rows from the kernel arguments (scalar loads issued beside the lookups):
      // scalar FMA operands, no LDS read per slot
      double mr[3][10];
#pragma unroll
      for (int g = 0; g < 10; g++) { mr[0][g] = A.Mk[I.g11 * 10 + g]; mr[1][g] = A.Mk[I.g12 * 10 + g]; mr[2][g] = A.Mk[I.g22 * 10 + g]; }
      __builtin_amdgcn_sched_barrier(0);
      if (s + QD_AHEAD < S) quad_dma(pl, s + QD_AHEAD, npo, voff, ring + ((s + QD_AHEAD) % QB) * QSLOT);
#pragma unroll
      for (int q = 0; q < 2; q++) D[q][0] = D[q][1] = D[q][2] = 0.0;
#pragma unroll
      for (int g = 0; g < 10; g++) {   // CalcDenovoMutLk (:1553-1562), each matrix entry read once for both kids
        const double m11 = mr[0][g], m12 = mr[1][g], m22 = mr[2][g];
#pragma unroll
        for (int q = 0; q < 2; q++) {
          D[q][0] = fma(m11, pg[q][g], D[q][0]);
          D[q][1] = fma(m12, pg[q][g], D[q][1]);
          D[q][2] = fma(m22, pg[q][g], D[q][2]);
        }
      }
    } else {   // cfg-7 items: likelihoodONEKid's autosomal terms on the item's three planes
#pragma unroll
      for (int k = 0; k < 3; k++) { lF[k] = lk[w[k] & 0xFF]; lM[k] = lk[(w[k] >> 8) & 0xFF]; }
#pragma unroll
      for (int q = 0; q < 2; q++)
#pragma unroll
        for (int k = 0; k < 3; k++) D[q][k] = lk[(w[k] >> (16 + 8 * q)) & 0xFF];
      __builtin_amdgcn_sched_barrier(0);
      if (s + QD_AHEAD < S) quad_dma(pl, s + QD_AHEAD, npo, voff, ring + ((s + QD_AHEAD) % QB) * QSLOT);
    }
    quad_poly4(D, lF, lM, a[s]);
    if (s >= qfull) {   // the partial last slot row: empty lanes hold the phantom family (f + g)^4
      const bool empty = 64 * s + lane >= nfam;
      a[s][0] = empty ? 1.0 : a[s][0]; a[s][1] = empty ? 4.0 : a[s][1]; a[s][2] = empty ? 6.0 : a[s][2];
      a[s][3] = empty ? 4.0 : a[s][3]; a[s][4] = empty ? 1.0 : a[s][4];
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// de novo items and cfg-7 items (uniform per item) take separate straight-line slot loops
template <int S>
__device__ __forceinline__ void hoist_quad(const DevArgs& A, const ItemCtx& I, const uint8_t* pl, const double* lk,
                                           const double* M, double (*a)[5], uint8_t* ring, const uint32_t* voff) {
  if (I.denovo) hoist_quad_t<S, true>(A, I, pl, lk, M, a, ring, voff);
  else hoist_quad_t<S, false>(A, I, pl, lk, M, a, ring, voff);
}

// f = 1 (the generic-path de novo monomorphism item): L_fam(1) = a0, the f^4 coefficient; an empty slot's
// phantom family (f + g)^4 has a0 = 1, so no slot needs masking.  Four interleaved (mantissa, exponent)
// accumulators, renormalised after every factor.
template <int S>
__device__ __forceinline__ void lane_poly_top(const double (*a)[5], double& m, int& e) {
  constexpr int NA = S < 4 ? S : 4;
  double am[NA];
  int ae[NA];
#pragma unroll
  for (int j = 0; j < NA; j++) { am[j] = 1.0; ae[j] = 0; }
#pragma unroll
  for (int s = 0; s < S; s++) {
    int x;
    am[s % NA] = frexp(am[s % NA] * a[s][0], &x);
    ae[s % NA] += x;
  }
#pragma unroll
  for (int w = 1; w < NA; w *= 2)
#pragma unroll
    for (int j = 0; j + w < NA; j += 2 * w) {
      int x;
      am[j] = frexp(am[j] * am[j + w], &x);
      ae[j] += ae[j + w] + x;
    }
  m = am[0];
  e = ae[0];
}

// Hot form: L_fam(f) = g^4 h(r), h(r) = a0 r^4 + a1 r^3 + a2 r^2 + a3 r + a4 with r = f / g, g = 1 - f
// (non-negative coefficients: no cancellation, relative error <= ~8 ulp for any r).  g4 = g^4 is folded
// into every slot, so the objective needs no log10(g); empty slots hold the phantom family (f + g)^4.
template <int S>
__device__ __forceinline__ void lane_poly_r(double r, double g4, const double (*a)[5], double& m, int& e) {
  constexpr int NA = S < 4 ? S : 4;
  double am[NA];
  int ae[NA];
#pragma unroll
  for (int j = 0; j < NA; j++) { am[j] = 1.0; ae[j] = 0; }
#pragma unroll
  for (int s = 0; s < S; s++) {
    const double h = fma(r, fma(r, fma(r, fma(r, a[s][0], a[s][1]), a[s][2]), a[s][3]), a[s][4]) * g4;
    am[s % NA] = am[s % NA] * h;
    // renormalise after every second factor of an accumulator (and after the last): a nuclear family's
    // likelihood is >= ~1e-118 (PL <= 255 per person, HWE prior >= 1e-16), so two factors on a mantissa in
    // [0.5, 1) stay >= 1e-237, clear of underflow; the mantissa bits are those of step-wise renormalisation
    if ((s / NA) % 2 == 1 || s + NA >= S) {
      int x;
      am[s % NA] = frexp(am[s % NA], &x);
      ae[s % NA] += x;
    }
  }
#pragma unroll
  for (int w = 1; w < NA; w *= 2)
#pragma unroll
    for (int j = 0; j + w < NA; j += 2 * w) {   // 4 mantissas in [0.5, 1): product >= 1/16, renormalised in wave_prod
      am[j] = am[j] * am[j + w];
      ae[j] += ae[j + w];
    }
  m = am[0];
  e = ae[0];
}


// One step of the wave product reduction on the DPP crossbar (VALU latency, no LDS round trip): multiply
// by the (mantissa, exponent) of the lane selected by CTRL; rows outside ROWMASK keep their value (the
// DPP `old` operand is the identity 1.0 x 2^0).
template <int CTRL, int ROWMASK>
__device__ __forceinline__ void dpp_prod_step(double& m, int& e) {
  const int lo = __double2loint(m), hi = __double2hiint(m);
  int olo, ohi, oe;
  if constexpr (ROWMASK == 0xF) {   // every row written: no identity `old` operand (saves its two v_mov per step)
    olo = __builtin_amdgcn_mov_dpp(lo, CTRL, 0xF, 0xF, false);
    ohi = __builtin_amdgcn_mov_dpp(hi, CTRL, 0xF, 0xF, false);
    oe = __builtin_amdgcn_update_dpp(0, e, CTRL, ROWMASK, 0xF, false);   // (folds into one v_add_u32_dpp)
  } else {
    olo = __builtin_amdgcn_update_dpp(0, lo, CTRL, ROWMASK, 0xF, false);
    ohi = __builtin_amdgcn_update_dpp(0x3FF00000, hi, CTRL, ROWMASK, 0xF, false);
    oe = __builtin_amdgcn_update_dpp(0, e, CTRL, ROWMASK, 0xF, false);
  }
  m = m * __hiloint2double(ohi, olo);   // no renormalisation: 64 factors in [1/16, 1) stay >= 2^-256
  e += oe;
}

// Product of the 64 lanes' (m, e), in a fixed order: quad xor 1, quad xor 2, half-row mirror, row mirror
// (every lane of a row of 16 then holds the row product), row_bcast15 / row_bcast31 (lane 63 ends with
// ((R3 R2)(R1 R0))), broadcast from lane 63.  Deterministic for any batch, identical in every lane.
__device__ __forceinline__ void wave_prod(double& m, int& e) {
  dpp_prod_step<0xB1, 0xF>(m, e);    // quad_perm [1,0,3,2]
  dpp_prod_step<0x4E, 0xF>(m, e);    // quad_perm [2,3,0,1]
  dpp_prod_step<0x141, 0xF>(m, e);   // row_half_mirror
  dpp_prod_step<0x140, 0xF>(m, e);   // row_mirror
  dpp_prod_step<0x142, 0xA>(m, e);   // row_bcast:15 -> rows 1, 3
  dpp_prod_step<0x143, 0xC>(m, e);   // row_bcast:31 -> rows 2, 3
  const int lo = __builtin_amdgcn_readlane(__double2loint(m), 63), hi = __builtin_amdgcn_readlane(__double2hiint(m), 63);
  int ev;
  m = frexp(__hiloint2double(hi, lo), &ev);   // one normalisation (exact: the mantissa bits are those of the
  e = __builtin_amdgcn_readlane(e, 63) + ev;  // step-wise normalised product, scalings by 2^k being exact)
}

// log10(m * 2^e) for a normalised mantissa m in [0.5, 1) (or 0): m is moved to [sqrt(1/2), sqrt(2)) (exact),
// then log(m) = 2 atanh(t), t = (m - 1) / (m + 1), |t| <= 0.172, as 2t + t^3 P(t^2) with the 10-term
// atanh series (truncation < 3e-17 relative).  Absolute error <= ~7e-17 (OCML's double-double log10:
// ~3e-17), far below the ~1e-12 ulp of the objective it is added to; ~25 instructions instead of ~85.
#define PM_INV_LN10 0x1.bcb7b1526e50ep-2
__device__ __forceinline__ double sgpr_const(double c) {
  asm volatile("" : "+s"(c));
  return c;
}
// n / d for a finite n and a positive d in the normal range, from the hardware reciprocal: two Newton steps and one
// residual correction (within an ulp of the IEEE quotient; 8 dependent operations instead of the 11 of the IEEE
// division sequence, which matters on the serial per-evaluation path of Brent)
__device__ __forceinline__ double pos_div(double n, double d) {
  double y = __builtin_amdgcn_rcp(d);
  double e = fma(-d, y, 1.0);
  y = fma(y, e, y);
  e = fma(-d, y, 1.0);
  y = fma(y, e, y);
  const double q = n * y;
  return fma(fma(-d, q, n), y, q);
}

__device__ __forceinline__ double log10_mant(double m, int e) {
  if (m == 0.0) return -INFINITY;   // an underflowed family product: log10(0), as the reference
  if (m < 0.70710678118654752440) { m *= 2.0; e -= 1; }
  const double u = m - 1.0;                  // exact (Sterbenz)
  const double t = pos_div(u, m + 1.0);       // |t| <= 0.172
  const double t2 = t * t;
  // P(t2) = sum_k 2 / (2k + 3) t2^k, k = 0..9, by Estrin (all terms >= 0: no cancellation), depth 4 instead of 9;
  // the series coefficients as SGPR operands materialised at their use (otherwise the compiler keeps ten of
  // them in VGPRs across the Brent loop, next to the 5 x S hoisted coefficients)
  const double t4 = t2 * t2, t8 = t4 * t4, t16 = t8 * t8;
  const double q0 = fma(sgpr_const(2.0 / 5), t2, sgpr_const(2.0 / 3));
  const double q1 = fma(sgpr_const(2.0 / 9), t2, sgpr_const(2.0 / 7));
  const double q2 = fma(sgpr_const(2.0 / 13), t2, sgpr_const(2.0 / 11));
  const double q3 = fma(sgpr_const(2.0 / 17), t2, sgpr_const(2.0 / 15));
  const double q4 = fma(sgpr_const(2.0 / 21), t2, sgpr_const(2.0 / 19));
  const double r0 = fma(q1, t4, q0), r1 = fma(q3, t4, q2);
  const double p = fma(q4, t16, fma(r1, t8, r0));
  const double ln = fma(t * t2, p, 2.0 * t);
  const double de = (double)e;
  return ln * PM_INV_LN10 + (de * PM_LOG10_2_HI + de * PM_LOG10_2_LO);
}

template <int T>
__device__ __forceinline__ double block_logprod(double m, int e, double* red, int* rede, int& par) {
  wave_prod(m, e);
  if (T > 64) {
    constexpr int W = T / 64;
    if ((threadIdx.x & 63) == 0) { red[par * 16 + (threadIdx.x >> 6)] = m; rede[par * 16 + (threadIdx.x >> 6)] = e; }
    __syncthreads();
    m = red[par * 16]; e = rede[par * 16];
#pragma unroll
    for (int i = 1; i < W; i++) {
      int ev;
      m = frexp(m * red[par * 16 + i], &ev);
      e += rede[par * 16 + i] + ev;
    }
    par ^= 1;
  }
  return log10_mant(m, e);
}

// GEN=false: lean autosomal nuclear-only kernel; GEN=true: chrX/Y/MT, de novo, founder-only units;
// ES=true additionally peels the lane's extended families (instantiated only for pedigrees that have them).
// Occupancy target (waves per SIMD) of a Brent flavour: the lean polynomial kernel keeps 5 doubles per
// family, so even at S=16 two items fit on a SIMD if the hoisting phase is kept from spreading out.

// ------------------------------------------------------------------------------------------------
// k_es_hoist: the polynomial-form peel for one (Brent item, extended family) per wave, ahead of
// the item's k_brent (EP), which then reads the coefficients instead of peeling.  The family's schedule is
// wave-uniform (scalar control flow), its partials and marriage partials live in this wave's LDS slice, and each
// step runs as phases whose output elements -- a (state, coefficient) or (state pair, coefficient) each -- are
// spread over the lanes, with a wave-level barrier between phases (LDS ops of one wave complete in order).  Same
// steps and degrees as FamilyLikelihoodES.cpp :1105-1395 (plain `transmission` at :1391);
// every phase writes out of place (temporaries after the layout) and copies back.
// A wave's LDS: hoist_ws (the family layout of poly_layout) + hoist_tmp (the largest step's temporaries).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ double lds_tba(const double* tba, int i, int j, int k, int chrom, int child_sex) {   // d_tba on LDS
  const int o = i * 9 + j * 3 + k;
  double t = tba[o];
  if (chrom == PM_CHR_X) t = (child_sex == MALE) ? tba[2 * 27 + o] : tba[27 + o];
  if (chrom == PM_CHR_Y) t = (child_sex == MALE) ? tba[3 * 27 + o] : 1.0;
  if (chrom == PM_CHR_MT) t = tba[4 * 27 + o];
  return t;
}

template <int NS>
__device__ __forceinline__ void wave_poly_peel(const DevArgs& A, int f, const uint8_t* pl, const double* lk, const double* tba,
                                               const double* T10, const double* T10dn, int g11, int g12, int g22, int chrom,
                                               bool top, double* ws, int lane, double* out, int ostride) {
  const int p0 = A.fam_start[f], n = A.fam_start[f + 1] - p0, nf = A.fam_founders[f];
  const bool X = chrom == PM_CHR_X, Y = chrom == PM_CHR_Y, MT = chrom == PM_CHR_MT;
  const int* L = A.poly_lay + A.poly_start[f];
  const int D = top ? 0 : L[2 + chrom];
  const size_t np = (size_t)A.n_person;
  double* TB = ws + A.hoist_ws;   // step temporaries
#define WV(o) ws[(o)]
#define POFF(i) (L[6 + (i)] & 0xFFFFFF)
#define PCAP(i) (L[6 + (i)] >> 24)
#define MOFF(m) (L[6 + n + (m)] & 0xFFFFFF)
#define MCAP(m) (L[6 + n + (m)] >> 24)
  for (int x = lane; x < n * NS; x += 64) {   // InitializePartials(_BA) x SetFounderPriors(_BA)
    const int i = x / NS, j = x - i * NS;
    const int sx = A.sex[p0 + i];
    const bool fo = A.is_founder[p0 + i] != 0 && i < nf;
    const uint8_t* R = pl + p0 + i;
    const int o = POFF(i) + j * PCAP(i);
    const bool yf = Y && sx == FEMALE;
    const int dfull = !fo ? 0 : (Y && sx == FEMALE) ? 0 : ((X || Y) && sx == MALE) || MT ? 1 : 2;
    const int d = top ? 0 : dfull;
    for (int a = 0; a <= d; a++) WV(o + a) = 0.0;
    if (NS == 3) {
      const int gj = j == 0 ? g11 : j == 1 ? g12 : g22;
      const double pen = lk[R[gj * np]];
      if (yf) WV(o) = 1.0;                          // BA chrY females: partial 1.0 (:1449-1465)
      else if (!fo) WV(o) = pen;
      else if (top) { if (j == 0) WV(o) = pen; }    // the f^d term: f^2 or f
      else if (d == 2) WV(o + 2 - j) = j == 1 ? 2 * pen : pen;   // f^2, 2fg, g^2
      else if (j != 1) WV(o + (j == 0 ? 1 : 0)) = pen;          // f, 0, g
    } else {
      const double pen = lk[R[j * np]];
      const int q = j == g11 ? 0 : j == g12 ? 1 : j == g22 ? 2 : 3;
      if (!fo) WV(o) = pen;
      else if (q != 3) {
        if (top && dfull > 0) { if (q == 0) WV(o) = pen; }   // the f^d term
        else if (d == 2) WV(o + 2 - q) = q == 1 ? 2 * pen : pen;
        else if (d == 1) { if (q != 1) WV(o + (q == 0 ? 1 : 0)) = pen; }
        else WV(o) = pen;   // chrY female founder: q = 1, 1, 1
      }
    }
  }
  wave_sync();
  const int s0 = A.peel_start[f], s1 = A.peel_start[f + 1];
  for (int s = s0; s < s1; s++) {
    const int2 S = A.steps[s];
    const int type = S.x & 255, from0 = (S.x >> 8) & 255, from1 = (S.x >> 16) & 255, to0 = (S.x >> 24) & 255;
    const int slot = (S.y >> 8) & 255, create = (S.y >> 16) & 1, fa2mo = (S.y >> 17) & 1;
    const int dg = top ? 0 : A.poly_deg[4 * s + chrom];
    const int da = dg & 127, db = (dg >> 7) & 127, dc = (dg >> 14) & 127, de = (dg >> 21) & 127;
    if (type == 1) {   // offspring -> parents: M(i, j) *= sum_k T(i, j, k) P_off[k]   (da = deg P_off, db = deg M)
      const int off = from0, po = POFF(off), pc = PCAP(off), mo = MOFF(slot), mc = MCAP(slot);
      const int csex = A.sex[p0 + off];
      const int wa = da + 1;
      for (int x = lane; x < NS * NS * wa; x += 64) {   // S(e, a)
        const int e = x / wa, a = x - e * wa, i = e / NS, j = e - i * NS;
        double sum = 0;
#pragma unroll
        for (int k = 0; k < NS; k++) {
          const double t = (NS == 3) ? lds_tba(tba, i, j, k, chrom, csex) : T10dn[(i * 10 + j) * 10 + k];
          sum += t * WV(po + k * pc + a);
        }
        if (create) WV(mo + e * mc + a) = sum;
        else TB[x] = sum;
      }
      wave_sync();
      if (!create) {
        const int w = da + db + 1;
        double* TM = TB + NS * NS * wa;
        for (int x = lane; x < NS * NS * w; x += 64) {   // (M S)(e, a)
          const int e = x / w, a = x - e * w;
          double acc = 0;
          for (int c = max(0, a - da); c <= min(a, db); c++) acc += WV(mo + e * mc + c) * TB[e * wa + a - c];
          TM[x] = acc;
        }
        wave_sync();
        for (int x = lane; x < NS * NS * w; x += 64) {
          const int e = x / w, a = x - e * w;
          WV(mo + e * mc + a) = TM[x];
        }
        wave_sync();
      }
    } else if (type == 2) {   // spouse -> spouse: P_to[i] *= sum_j P_from[j] M(j, i)   (da from, db M, dc to)
      const int sf = from0, stt = to0, fo_ = POFF(sf), fc = PCAP(sf), to_ = POFF(stt), tc = PCAP(stt);
      const int mo = slot == 255 ? 0 : MOFF(slot), mc = slot == 255 ? 0 : MCAP(slot);
      const int ds = da + db, ws1 = ds + 1;
      for (int x = lane; x < NS * ws1; x += 64) {   // S(i, a)
        const int i = x / ws1, a = x - i * ws1;
        double sum = 0;
        for (int j = 0; j < NS; j++) {
          if (slot == 255) { if (a <= da) sum += WV(fo_ + j * fc + a); continue; }
          const int e0 = mo + (fa2mo ? j * NS + i : i * NS + j) * mc;
          for (int u = max(0, a - db); u <= min(a, da); u++) sum += WV(fo_ + j * fc + u) * WV(e0 + a - u);
        }
        TB[x] = sum;
      }
      wave_sync();
      const int w = dc + ds + 1;
      double* TM = TB + NS * ws1;
      for (int x = lane; x < NS * w; x += 64) {   // P_to S
        const int i = x / w, a = x - i * w;
        double acc = 0;
        for (int c = max(0, a - ds); c <= min(a, dc); c++) acc += WV(to_ + i * tc + c) * TB[i * ws1 + a - c];
        TM[x] = acc;
      }
      wave_sync();
      for (int x = lane; x < NS * w; x += 64) {
        const int i = x / w, a = x - i * w;
        WV(to_ + i * tc + a) = TM[x];
      }
      wave_sync();
    } else {   // parents -> only offspring: P_off[k] *= sum_ij P_fa[i] M(i, j) P_mo[j] T(i, j, k)   (da fa, db M, dc mo, de off)
      const int fa = from0, mo_ = from1, off = to0;
      const int fao = POFF(fa), fac = PCAP(fa), moo = POFF(mo_), moc = PCAP(mo_), oo = POFF(off), oc = PCAP(off);
      const int mo = slot == 255 ? 0 : MOFF(slot), mc = slot == 255 ? 0 : MCAP(slot);
      const int csex = A.sex[p0 + off];
      const int dw = da + db + dc, ww = dw + 1;
      for (int x = lane; x < NS * NS * ww; x += 64) {   // W(e, a) = P_fa[i] M(i, j) P_mo[j]
        const int e = x / ww, a = x - e * ww, i = e / NS, j = e - i * NS;
        double acc = 0;
        for (int u = 0; u <= da; u++)
          for (int v = 0; v <= db; v++) {
            const int r = a - u - v;
            if (r < 0 || r > dc) continue;
            const double m = slot == 255 ? 1.0 : WV(mo + e * mc + v);
            acc += WV(fao + i * fac + u) * m * WV(moo + j * moc + r);
          }
        TB[x] = acc;
      }
      wave_sync();
      double* TS = TB + NS * NS * ww;
      for (int x = lane; x < NS * ww; x += 64) {   // S(k, a) = sum_e T(i, j, k) W(e, a)
        const int k = x / ww, a = x - k * ww;
        double sum = 0;
        for (int e = 0; e < NS * NS; e++) {
          const int i = e / NS, j = e - i * NS;
          double t;
          if (NS == 3) t = lds_tba(tba, i, j, k, chrom, csex);
          else t = (slot == 255) ? T10dn[(i * 10 + j) * 10 + k] : T10[(i * 10 + j) * 10 + k];   // quirk :1391
          sum += t * TB[e * ww + a];
        }
        TS[x] = sum;
      }
      wave_sync();
      const int w = de + dw + 1;
      double* TM = TS + NS * ww;
      for (int x = lane; x < NS * w; x += 64) {   // P_off S
        const int k = x / w, a = x - k * w;
        double acc = 0;
        for (int c = max(0, a - dw); c <= min(a, de); c++) acc += WV(oo + k * oc + c) * TS[k * ww + a - c];
        TM[x] = acc;
      }
      wave_sync();
      for (int x = lane; x < NS * w; x += 64) {
        const int k = x / w, a = x - k * w;
        WV(oo + k * oc + a) = TM[x];
      }
      wave_sync();
    }
  }
  const int fin = (A.steps[s1 - 1].x >> 24) & 255, fo_ = POFF(fin), fc = PCAP(fin);
  for (int a = lane; a <= D; a += 64) {
    double sum = 0.0;
    for (int i = 0; i < NS; i++) sum += WV(fo_ + i * fc + a);
    out[(size_t)a * ostride] = sum;
  }
  if (lane == 0) out[(size_t)(A.poly_dcap - 1) * ostride] = (double)D;
  wave_sync();   // the next unit reuses the slice
#undef WV
#undef POFF
#undef PCAP
#undef MOFF
#undef MCAP
}

// grid: persistent, 4 waves per block (tables shared, one LDS slice per wave); units (item, ES family slot e = q T + lane
// of the lane plan) with the family fastest, so a block's waves share the item's site block in the caches.
template <bool DN>
__global__ void __launch_bounds__(256) k_es_hoist(DevArgs A, int list) {
  __shared__ double s_lk[256];
  __shared__ double s_tba[5 * 27];
  __shared__ double s_T10[DN ? 1000 : 1], s_T10dn[DN ? 1000 : 1];
  extern __shared__ double s_hw[];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) s_lk[i] = A.lktab[i];
  for (int i = threadIdx.x; i < 5 * 27; i += blockDim.x) s_tba[i] = (&c_TBA[0][0])[i];
  if constexpr (DN)
    for (int i = threadIdx.x; i < 1000; i += blockDim.x) { s_T10[i] = A.T10[i]; s_T10dn[i] = A.T10dn[i]; }
  __syncthreads();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  double* ws = s_hw + (size_t)wave * (A.hoist_ws + A.hoist_tmp);
  const int nItems = min(A.counts[list], A.es_it1);
  if (nItems <= A.es_it0) return;
  const int nslots = A.max_ext * A.T;
  const long long units = (long long)(nItems - A.es_it0) * nslots;
  const int waves = gridDim.x * (blockDim.x >> 6);
  for (long long u = (long long)blockIdx.x * (blockDim.x >> 6) + wave; u < units; u += waves) {
    const int it = A.es_it0 + (int)(u / nslots), e = (int)(u % nslots);
    const int f = __builtin_amdgcn_readfirstlane(A.ext_fam[e]);
    if (f < 0) continue;
    const int item = __builtin_amdgcn_readfirstlane(A.items[list][it]);
    const int site = item >> 3, cfg = item & 7;
    const int r = A.ref[site];
    int a1, a2;
    item_alleles(A, site, cfg, r, &a1, &a2);
    const int g11 = d_gi(a1, a1), g12 = d_gi(a1, a2), g22 = d_gi(a2, a2);
    const bool denovo = A.denovo && cfg != 7;
    const bool top = DN && cfg == 0 && !A.vcf;   // the de novo monomorphism item: one evaluation at f = 1
    const uint8_t* pl = A.pl + (size_t)site * A.n_person * 10;
    const int q = e / A.T, l = e - q * A.T;
    double* out = A.es_coef + ((size_t)(it - A.es_it0) * A.max_ext + q) * A.poly_dcap * A.T + l;
    if (DN && denovo) wave_poly_peel<10>(A, f, pl, s_lk, s_tba, s_T10, s_T10dn, g11, g12, g22, A.chrom, top, ws, lane, out, A.T);
    else wave_poly_peel<3>(A, f, pl, s_lk, s_tba, s_T10, s_T10dn, g11, g12, g22, A.chrom, top, ws, lane, out, A.T);
  }
}

template <int T, int S, int NUM, bool GEN>
constexpr int brent_waves() { return (NUM == PM_NUM_POLY && !GEN && (T == 64 || T == 128) && S >= 8) ? PM_POLY_WAVES : 1; }

// DN: lean polynomial kernel for autosomal --denovo (instantiated separately so the common kernel carries
// no de novo hoisting code or register pressure).
// PF: lean kernel whose items' genotype planes are prefetched into LDS (prefetch_planes); no other hoisting path.
// EP: extended families in polynomial form (coefficients from k_es_hoist, es_poly_eval per evaluation); the
// reference-order peel (d_es_lk) is compiled out, and the block asks for 2 waves per SIMD.
// QD: lean --denovo kernel on a QUAD plan (hoist_quad: coalesced dword loads, prefetched across items).
template <int T, int S, int NUM, bool GEN, bool ES, bool DN = false, bool PF = false, bool EP = false, bool QD = false>
__global__ void __launch_bounds__(T, (EP ? 2 : brent_waves<T, S, NUM, GEN>())) k_brent(DevArgs A, int list) {
  constexpr bool PROD = NUM != PM_NUM_EXACT;
  constexpr bool POLYK = NUM == PM_NUM_POLY && !GEN;
  __shared__ double s_lk[256];
  __shared__ double s_M[(GEN || DN) ? 100 : 1];
  __shared__ double s_red[T > 64 ? 96 : 1];
  __shared__ int s_rede[T > 64 ? 32 : 1];
  __shared__ __attribute__((aligned(16))) int s_u[POLYK ? S * T : 4];   // packed lane plan (unit_pack, lane-major)
  for (int i = threadIdx.x; i < 256; i += T) s_lk[i] = A.lktab[i];
  if constexpr (GEN || DN)
    for (int i = threadIdx.x; i < 100; i += T) s_M[i] = A.M[i];
  if constexpr (POLYK)
#pragma unroll
    for (int s = 0; s < S; s++) s_u[threadIdx.x * S + s] = unit_pack(A.units[s * T + threadIdx.x]);
  __syncthreads();
  int4 unit[S];
  if constexpr (!POLYK) {
#pragma unroll
    for (int s = 0; s < S; s++) unit[s] = A.units[s * T + threadIdx.x];
  }
  const int nItems = A.counts[list];
  const int* items = A.items[list];
  int par = 0;
  // XCD-aware item order: blocks are dealt round-robin to the 8 XCDs (separate L2s), so consecutive
  // items -- the 2-4 configurations of one site, which read the same PL block -- go to blocks of one XCD.
  const int vb = (gridDim.x % 8 == 0) ? (blockIdx.x % 8) * (gridDim.x / 8) + blockIdx.x / 8 : blockIdx.x;
  // lean kernel, one or two waves per item: the item's genotype planes arrive in LDS by prefetch (pf_npad > 0)
  constexpr bool PFK = PF && NUM == PM_NUM_POLY && !GEN && !ES && !DN && (T == 64 || T == 128);
  // PF on the lean de novo kernel: the 64 x 16 instantiation with only the LDS-staged hoisting compiled (the
  // direct-load hoisting of 16 de novo slots spills; this one keeps 1024 families on one wave per item)
  constexpr bool DNPF_ONLY = PF && POLYK && DN && T == 64 && S == 16 && !QD;
  static_assert(!QD || (POLYK && DN && T == 64 && !ES), "QUAD plans run on the lean one-wave --denovo kernel");
  extern __shared__ uint8_t s_pf[];
  const bool pf = PFK && A.pf_npad > 0;
  if (pf) prefetch_planes(A, items, vb, nItems, s_pf);
  unsigned long long ev_acc = 0;   // evaluation count of this block's items: one atomic per block, at exit
  unsigned long long ph_h = 0, ph_e = 0, ph_n = 0, ph_t = 0;   // PM_PHASE_TIMING (A.phase): hoisting / evaluation split
  const int itEnd = min(nItems, A.es_it1);   // EP: this launch's chunk of the list [es_it0, es_it1)
  // QD: this wave's LDS slot ring and the per-lane DMA source offsets; the first item's first slots
  uint8_t* qring = s_pf + (QD ? __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) * QWAVE : 0);
  uint32_t qvoff[3];
  // QD: the next item's index and the dword holding its reference base arrive by LDS-DMA as well (every lane
  // copies the same dword: s_qaux[0..63] = the ref dword, s_qaux[64..127] = the item after it), so no load is
  // waited for at the top of an item.  Issue order per item: ref dword, slot 0, slot 1, next item index.
  __shared__ __attribute__((aligned(16))) int s_qaux[QD ? 128 : 1];
  int q_item = 0;
  if constexpr (QD) {
#pragma unroll
    for (int i = 0; i < 3; i++) qvoff[i] = quad_voff(i, A.n_person);
    if (A.es_it0 + vb < itEnd) {
      q_item = items[A.es_it0 + vb];
      quad_aux(A.ref + ((q_item >> 3) & ~3), s_qaux);
      quad_prefetch(A, q_item, qvoff, qring);
      if (A.es_it0 + vb + (int)gridDim.x < itEnd) quad_aux(items + A.es_it0 + vb + gridDim.x, s_qaux + 64);
    }
  }
  // QD: an item's results wait in LDS and are stored after the next item's hoisting, so that they are older
  // than that item's prefetch in vmcnt order
  __shared__ double s_pend[QD ? 2 : 1];
  __shared__ int s_pendi[QD ? 3 : 1];
  const int it_first = A.es_it0 + vb;
  for (int it = A.es_it0 + vb; it < itEnd; it += gridDim.x) {
    if (A.phase) ph_t = wall_clock64();
    const int item = QD ? q_item : items[it];
    const int site = item >> 3, cfg = item & 7;
    int r;
    if constexpr (QD) {
      __builtin_amdgcn_s_waitcnt(0x0F70 | 6);   // vmcnt(6): the ref dword has landed (slots 0, 1 and the next index may not)
      __builtin_amdgcn_sched_barrier(0);
      r = __builtin_amdgcn_readfirstlane(((const volatile __attribute__((address_space(3))) uint8_t*)s_qaux)[site & 3]);
    } else r = A.ref[site];
    ItemCtx I;
    item_alleles(A, site, cfg, r, &I.a1, &I.a2);
    I.g11 = d_gi(I.a1, I.a1); I.g12 = d_gi(I.a1, I.a2); I.g22 = d_gi(I.a2, I.a2);
    // the lean polynomial kernel also runs autosomal --denovo items (its hoisting has the de novo kid terms)
    I.denovo = (GEN || (POLYK && DN)) ? (A.denovo && cfg != 7) : 0;
    I.sex = 0;   // famlk[1..6]'s member sex stays 0; famlk[0]'s stale one only reaches the posteriors (de novo cfg-7 items: 0)
    I.chrom = GEN ? A.chrom : PM_CHR_AUTO;
    int pmode;
    if (I.denovo) pmode = A.n_fam_gt1 ? PR_AUTO : PR_DN_SINGLE;
    else if (!A.n_fam_gt1) pmode = PR_TRIO;   // isMono is never set on the evaluating objects
    else if (!GEN) pmode = PR_AUTO;
    else pmode = A.chrom == PM_CHR_X ? PR_X : A.chrom == PM_CHR_Y ? PR_Y : A.chrom == PM_CHR_MT ? PR_MT : PR_AUTO;

    const uint8_t* pl = A.pl + (size_t)site * A.n_person * 10;
    // POLY (lean product kernel, always the autosomal HWE prior with > 1 family): 5 coefficients per family
    constexpr bool POLY = NUM == PM_NUM_POLY && !GEN;
    constexpr int NC = POLY ? 5 : 9;
    double cond[S][NC];
    int fl[S];
    bool hoisted = false;
    if constexpr (POLY) {
      if constexpr (PFK) {
        if (pf) {
          __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): this wave's pieces of the item's planes have landed
          if constexpr (T > 64) __syncthreads();   // ... and the other waves' pieces
          hoist_poly4_lds<S, T>(A, s_u, s_pf, s_lk, cond);
          __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): every read of the buffer is done ...
          if constexpr (T > 64) __syncthreads();   // ... by every wave of the block ...
          __builtin_amdgcn_sched_barrier(0);
          prefetch_planes(A, items, it + gridDim.x, nItems, s_pf);   // ... before the next item's planes overwrite it
          hoisted = true;
        }
      }
      if constexpr (QD) {
        hoist_quad<S>(A, I, pl, s_lk, s_M, cond, qring, qvoff);
        hoisted = true;
        const int itn = it + gridDim.x;   // the next item's first slots land during this item's Brent
        // (landed: the hoisting ended with vmcnt(0)); uniform, so the next site's addresses are scalar
        const int nitem = __builtin_amdgcn_readfirstlane(((const volatile __attribute__((address_space(3))) int*)s_qaux)[64]);
        if (threadIdx.x == 0 && it != it_first) {
          const int ps = s_pendi[0], pc = s_pendi[1];
          A.raw[(size_t)ps * 8 + pc] = s_pend[0];
          A.minv[ps * 8 + pc] = s_pend[1];
          A.evals[ps * 8 + pc] = s_pendi[2];
        }
        if (itn < itEnd) {
          __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): s_qaux has been read before the DMA refills it
          __builtin_amdgcn_sched_barrier(0);
          quad_aux(A.ref + ((nitem >> 3) & ~3), s_qaux);
          quad_prefetch(A, nitem, qvoff, qring);
          if (itn + (int)gridDim.x < itEnd) quad_aux(items + itn + gridDim.x, s_qaux + 64);
          q_item = nitem;
        }
      }
      if (!PFK && !QD && !hoisted && A.max_nuc <= 4) {
        if constexpr (DN) {   // de novo and cfg-7 items
          if constexpr (DNPF_ONLY) hoist_poly4_dn_pf<S, T>(A, s_u, I, pl, s_lk, s_M, cond, s_pf + (threadIdx.x >> 6) * 2 * DN_PF_BUF);
          else if constexpr (S % DN_PF_C == 0) {
            if (A.dn_pf) hoist_poly4_dn_pf<S, T>(A, s_u, I, pl, s_lk, s_M, cond, s_pf + (threadIdx.x >> 6) * 2 * DN_PF_BUF);
            else hoist_poly4_dn<S, T>(A, s_u, I, pl, s_lk, s_M, cond);
          } else hoist_poly4_dn<S, T>(A, s_u, I, pl, s_lk, s_M, cond);
        }
        else hoist_poly4<S, T>(A, s_u, I, pl, s_lk, cond);
        hoisted = true;
      }
    }
#pragma unroll
    for (int s = 0; s < S; s++) {
      fl[s] = 0;
      if (PFK || DNPF_ONLY || QD || hoisted) continue;
      if constexpr (POLY) {
        const int4 u = A.units[s * T + threadIdx.x];   // L1/L2-resident; not kept in registers
        double c9[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        if (u.x == U_NUC) hoist_nuc<false, DN>(A, I, pl, s_lk, s_M, u.z, u.w, c9);
        fold_poly(c9, cond[s]);
        if (u.x != U_NUC) phantom_poly(cond[s]);   // empty slot (lane_poly_r)
      } else if (unit[s].x == U_NUC) hoist_nuc<GEN>(A, I, pl, s_lk, s_M, unit[s].z, unit[s].w, cond[s]);
      else if (GEN && unit[s].x == U_FP) fl[s] = hoist_fp(A, I, pl, s_lk, unit[s].z, unit[s].w & 0xFF, cond[s]);
    }
    double* raw = A.raw + (size_t)site * 8;
    // ES workspace: lane-interleaved, in LDS when it fits the block's share (ws_lds), else in HBM (L2-resident)
    // (two pointers, so each inlined peel keeps a known address space: ds_* or global_* accesses, no flat)
    double* wsl = ES ? A.ws + (size_t)blockIdx.x * A.ws_per_lane * T + threadIdx.x : nullptr;
    double* wsl_lds = ES ? (double*)s_pf + threadIdx.x : nullptr;
    // EP: the first PM_EPE families' coefficients in registers for the item's evaluations (ed < 0: none or D > PDM)
    // (one-wave plans only: at 256 lanes the cache spills, and those plans hold one family per lane anyway)
    constexpr int EPE = (EP && T == 64) ? PM_EPE : 0;
    double ce[EPE ? EPE : 1][EPE ? PDM + 1 : 1];
    int ed[EPE ? EPE : 1];
    // EP: the lane's extended families' coefficients, peeled for this item by k_es_hoist
    const double* coef = (ES && EP) ? A.es_coef + (size_t)(it - A.es_it0) * A.max_ext * A.poly_dcap * T + threadIdx.x : nullptr;
    if constexpr (ES && EP) {
      const int cnt = A.ext_count ? A.ext_count[threadIdx.x] : 0;
#pragma unroll
      for (int q = 0; q < EPE; q++) {
        const double* co = coef + (size_t)q * A.poly_dcap * T;
        ed[q] = q < cnt ? (int)co[(size_t)(A.poly_dcap - 1) * T] : -1;
        if (ed[q] > PDM) ed[q] = -1;
#pragma unroll
        for (int a = 0; a <= PDM; a++) ce[q][a] = a <= ed[q] ? co[(size_t)a * T] : 0.0;
      }
    }
    if (A.phase) { const unsigned long long t = wall_clock64(); ph_h += t - ph_t; ph_t = t; }
    const bool single = !A.vcf && ((cfg == 0) || (A.single_nuclear && !A.unrelated));
    // One evaluation site for the objective: the three bracketing evaluations of OptimizeFrequency
    // (:432-444) and every Brent step (core/MathGold.cpp:81-177) run through the same loop body.
    const double tol = A.precision;
    double a = 0.0001, b = 0.9999, c = 0.5;
    double mn = 0, fmin = 0, w = 0, v = 0, fw = 0, fv = 0, delta = 0.0, d = 0.0;
    // OptimizeFrequency (NucFamGenotypeLikelihood.cpp:432-441) evaluates fa = f(a), fb = f(b), fc = f(c) and
    // calls Brent, which reads only fb (MathGold.cpp:85-93: a < c, so fa and fc are never swapped in or read).
    // f(a) and f(c) are therefore counted (pm_site_result.evals keeps the reference's count) but not computed.
    double x = single ? ((cfg == 0) ? 1.0 : 0.5) : b;   // MonomorphismLogLikelihood_denovo / single nuclear family at 0.5
    int phase = single ? 0 : 1, iter = 0, nev = single ? 0 : 1;   // nev: f(a) counted
    int skipped = single ? 0 : 2;
    bool ok = false;
    for (;;) {
      double tot;
      if constexpr (POLY) {
        // L_fam(f) = g^4 h(f / g) (g = 1 - f): one Horner direction, g^4 folded per slot, no per-slot
        // masking (empty slots hold the phantom family), one log10 per evaluation.  f = 1 (the generic-path
        // de novo monomorphism item) takes the reverse form M = f, t = g / f with masking.
        const double g = 1 - x;
        double m; int e;
        if (__builtin_amdgcn_readfirstlane((int)(g > 0.0))) {
          // (r from the hardware reciprocal + a Newton step instead of the division: measured no faster)
          lane_poly_r<S>(pos_div(x, g), (g * g) * (g * g), (const double(*)[5])cond, m, e);
          tot = block_logprod<T>(m, e, s_red, s_rede, par);
        } else {
          lane_poly_top<S>((const double(*)[5])cond, m, e);   // x = 1: L = a0 per family, log10(x^4) = 0
          tot = block_logprod<T>(m, e, s_red, s_rede, par);
        }
      } else if (PROD) {
        double m; int e;
        lane_prod<S, GEN>(x, unit, (const double(*)[9])cond, fl, pmode, m, e);
        if constexpr (ES && EP && EPE > 0) {   // register-resident coefficients first (independent Horner chains)
#pragma unroll
          for (int q = 0; q < EPE; q++)
            if (ed[q] >= 0) {
              int e1, e2;
              const double mv = frexp(es_poly_eval_r(ce[q], ed[q], x), &e1);
              m = frexp(m * mv, &e2);
              e += e1 + e2;
            }
        }
        if (ES && A.ext_count)   // extended families of this lane: Elston-Stewart peeling per evaluation
          for (int q = 0; q < A.ext_count[threadIdx.x]; q++) {
            const int f = A.ext_fam[q * T + threadIdx.x];
            double v;
            if constexpr (EP) {
              if constexpr (EPE > 0)
                if (q < EPE && ed[q] >= 0) continue;   // (evaluated from registers above)
              const double* co = coef + (size_t)q * A.poly_dcap * T;
              v = es_poly_eval(co, T, (int)co[(size_t)(A.poly_dcap - 1) * T], x);
            } else {
              v = I.denovo  ? d_es_lk<10>(A, f, pl, s_lk, I.g11, I.g12, I.g22, I.chrom, x, -1, -1, wsl, T)
                : A.ws_lds ? d_es_lk<3>(A, f, pl, s_lk, I.g11, I.g12, I.g22, I.chrom, x, -1, -1, wsl_lds, T)
                           : d_es_lk<3>(A, f, pl, s_lk, I.g11, I.g12, I.g22, I.chrom, x, -1, -1, wsl, T);
            }
            int e1, e2;
            const double mv = frexp(v, &e1);
            m = frexp(m * mv, &e2);
            e += e1 + e2;
          }
        tot = block_logprod<T>(m, e, s_red, s_rede, par);
      } else {
        double part = lane_loglik<S, GEN>(x, unit, (const double(*)[9])cond, fl, pmode, A.vcf != 0);
        if (ES && A.ext_count)
          for (int q = 0; q < A.ext_count[threadIdx.x]; q++) {
            const int f = A.ext_fam[q * T + threadIdx.x];
            part += log10(I.denovo  ? d_es_lk<10>(A, f, pl, s_lk, I.g11, I.g12, I.g22, I.chrom, x, -1, -1, wsl, T)
                          : A.ws_lds ? d_es_lk<3>(A, f, pl, s_lk, I.g11, I.g12, I.g22, I.chrom, x, -1, -1, wsl_lds, T)
                                     : d_es_lk<3>(A, f, pl, s_lk, I.g11, I.g12, I.g22, I.chrom, x, -1, -1, wsl, T));
          }
        tot = block_sum<T>(part, s_red, par);
      }
      nev++;
      if (single) { mn = 0.0; fmin = -tot; ok = true; break; }
      const double fx = -tot;
      if (phase == 1) {   // fb; then f(c), counted only (see above); Brent: min = b, fmin = fb (MathGold.cpp:91-93)
        fmin = fx; nev++;
        phase = 3; mn = b; w = b; v = b; fw = fmin; fv = fmin;
      } else {
        const double u = x, fu = fx;
        if (fu <= fmin) {
          if (u >= mn) a = mn; else c = mn;
          v = w; w = mn; mn = u;
          fv = fw; fw = fmin; fmin = fu;
        } else {
          if (u < mn) a = u; else c = u;
          if (fu <= fw || w == mn) { v = w; w = u; fv = fw; fw = fu; }
          else if (fu <= fv || v == mn || v == w) { v = u; fv = fu; }
        }
      }
      if (++iter > 200) break;   // ITMAX: numerror("ScalarMinimizer::Brent got stuck")
      const double middle = 0.5 * (a + c);
      const double tol1 = tol * fabs(mn) + 3.0e-10;
      const double tol2 = 2.0 * tol1;
      if (fabs(mn - middle) <= (tol2 - 0.5 * (c - a))) { ok = true; break; }
      if (fabs(delta) > tol1) {
        double rr = (mn - w) * (fmin - fv);
        double q = (mn - v) * (fmin - fw);
        double p = (mn - v) * q - (mn - w) * rr;
        q = 2.0 * (q - rr);
        if (q > 0.0) p = -p;
        q = fabs(q);
        const double temp = delta;
        delta = d;
        if (fabs(p) >= fabs(0.5 * q * temp) || p <= q * (a - mn) || p >= q * (c - mn)) {
          delta = mn >= middle ? a - mn : c - mn;
          d = 0.38196601 * delta;
        } else {
          d = p / q;
          const double u = mn + d;
          if (u - a < tol2 || c - u < tol2) d = d_sign(tol1, middle - mn);
        }
      } else {
        delta = mn >= middle ? a - mn : c - mn;
        d = 0.38196601 * delta;
      }
      x = fabs(d) >= tol1 ? mn + d : mn + d_sign(tol1, d);
    }
    if (threadIdx.x == 0) {
      if constexpr (QD) { s_pend[0] = -fmin; s_pend[1] = mn; s_pendi[0] = site; s_pendi[1] = cfg; s_pendi[2] = nev; }
      else {
        raw[cfg] = -fmin;
        A.minv[site * 8 + cfg] = mn;
        A.evals[site * 8 + cfg] = nev;
      }
      if (!single) ev_acc += nev - skipped;   // objective evaluations computed
      if (!ok) atomicExch(&A.counts[5], 1);
    }
    if (A.phase) { ph_e += wall_clock64() - ph_t; ph_n++; }
  }
  if (QD && threadIdx.x == 0 && it_first < itEnd) {
    const int ps = s_pendi[0], pc = s_pendi[1];
    A.raw[(size_t)ps * 8 + pc] = s_pend[0];
    A.minv[ps * 8 + pc] = s_pend[1];
    A.evals[ps * 8 + pc] = s_pendi[2];
  }
  if (threadIdx.x == 0 && ev_acc) atomicAdd(A.eval_total, ev_acc);
  if (A.phase && threadIdx.x == 0) { atomicAdd(&A.phase[0], ph_h); atomicAdd(&A.phase[1], ph_e); atomicAdd(&A.phase[2], ph_n); }
}

// ------------------------------------------------------------------------------------------------
// k_prep: one wave per site.  CalcReadStats (integer sums, order-free) and MonomorphismLogLikelihood
// (serial double sum, kept in the reference's person order) -- NucFamGenotypeLikelihood.cpp:502-546.
// k_prep per-lane loads: VEC consecutive persons per lane and iteration, fetched with vector loads (16 B
// of dm, VEC bytes of a genotype plane) so each wave keeps several KB in flight -- the loop is HBM-latency
// bound otherwise.  VEC = 16/8/4 needs n_person % VEC == 0 (all block offsets then stay 16-B aligned).
template <int VEC>
__device__ __forceinline__ void load_bytes(const uint8_t* p, uint8_t* out) {
  if constexpr (VEC == 16) { const uint4 v = *(const uint4*)p; memcpy(out, &v, 16); }
  else if constexpr (VEC == 8) { const uint2 v = *(const uint2*)p; memcpy(out, &v, 8); }
  else if constexpr (VEC == 4) { const uint32_t v = *(const uint32_t*)p; memcpy(out, &v, 4); }
  else out[0] = p[0];
}
template <int VEC>
__device__ __forceinline__ void load_dwords(const uint32_t* p, uint32_t* out) {
  if constexpr (VEC >= 4) {
#pragma unroll
    for (int q = 0; q < VEC / 4; q++) { const uint4 v = ((const uint4*)p)[q]; out[4 * q] = v.x; out[4 * q + 1] = v.y; out[4 * q + 2] = v.z; out[4 * q + 3] = v.w; }
  } else out[0] = p[0];
}

// k_prep: one wave per site.  CalcReadStats (integer sums, order-free) and MonomorphismLogLikelihood
// (NucFamGenotypeLikelihood.cpp:502-546).  SERIAL (PM_NUM_EXACT): the mono sum -PL/10 is accumulated in
// the reference's person order (VEC = 1, lanes ascending via ballot); otherwise it is -(Sum PL)/10 from
// the exact integer sum -- correctly rounded, within ~1e-14 relative of the serial sum.
template <int VEC, bool SERIAL>
__global__ void __launch_bounds__(256) k_prep(DevArgs A) {
  __shared__ unsigned long long s_c[9];
  __shared__ double s_lk[256];
  __shared__ double s_M[100];
  if (threadIdx.x < 9) s_c[threadIdx.x] = 0;
  if (A.mono_dn) {
    s_lk[threadIdx.x] = A.lktab[threadIdx.x];
    if (threadIdx.x < 100) s_M[threadIdx.x] = A.M[threadIdx.x];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int site = wave;
  bool valid = false;
  if (site < A.n) {
    const int rb = A.ref[site];
    const int r = A.vcf ? (rb & 15) : rb, alt = rb >> 4;
    const int np = A.n_person;
    const uint8_t* pl = A.pl + (size_t)site * np * 10;
    const uint32_t* dm = A.dm + (size_t)site * np;
    const bool okref = r >= 1 && r <= 4 && (!A.vcf || (alt >= 1 && alt <= 4 && alt != r));
    const int h = okref ? d_gi(r, r) : 0;
    long long dsum = 0, mqsum = 0, nsd = 0, plsum = 0;
    double mono = 0.0;
    // lean --denovo: MonomorphismLogLikelihood_denovo (the cfg-0 item: CalcAllFamLogLikelihood at f = 1).
    // SetParentPrior(1) = (1, 0, ..., 0), so each nuclear family contributes cond[0] = (Prod_kids
    // CalcDenovoMutLk(geno11)) * F11 * M11 (:1041-1132, :1553-1562): a product of per-person factors --
    // founders lk[geno11], kids their g11 dot product -- taken here as one normalised product per site.
    const bool mdn = A.mono_dn && okref;
    double dm_m = 1.0;
    int dm_e = 0;
    const uint8_t* plane_h = pl + (size_t)h * np;
    for (int base = 0; base < np; base += 64 * VEC) {
      const int p0 = base + lane * VEC;
      uint32_t x[VEC];
      uint8_t hr[VEC];
      if (p0 < np) {   // np % VEC == 0: a lane's VEC persons are all present or all absent
        if (!A.vcf) load_dwords<VEC>(dm + p0, x);
        else {   // the VCF path has no read depth or mapping quality (PedVCF / FamilyLikelihoodSeq_VCF): dm is not read
#pragma unroll
          for (int k = 0; k < VEC; k++) x[k] = 0;
        }
        load_bytes<VEC>(plane_h + p0, hr);
      } else {
#pragma unroll
        for (int k = 0; k < VEC; k++) { x[k] = 0; hr[k] = 0; }
      }
#pragma unroll
      for (int k = 0; k < VEC; k++) {
        const int d = (int)(x[k] & 0xFFFFFF);
        dsum += d; mqsum += (x[k] >> 24); nsd += d > 0;
        plsum += hr[k];
      }
      if constexpr (SERIAL) {   // VEC == 1: lanes in ascending person order
        unsigned long long m = __ballot(hr[0] != 0);   // zero terms add -0.0: no change to a sum starting at +0.0
        const double t = -(double)hr[0] / 10;
        while (m) {
          const int l = __ffsll((long long)m) - 1;
          m &= m - 1;
          mono += __shfl(t, l, 64);
        }
      }
      if (mdn && p0 < np) {
        uint8_t fo[VEC];
        load_bytes<VEC>((const uint8_t*)A.is_founder + p0, fo);
        uint8_t kb[10][VEC];
#pragma unroll
        for (int g = 0; g < 10; g++) load_bytes<VEC>(pl + (size_t)g * np + p0, kb[g]);
#pragma unroll
        for (int k = 0; k < VEC; k++) {
          double fct;
          if (fo[k]) fct = s_lk[hr[k]];
          else {
            fct = 0.0;
#pragma unroll
            for (int g = 0; g < 10; g++) fct += s_M[h * 10 + g] * s_lk[kb[g][k]];
          }
          int xe;
          dm_m = frexp(dm_m * fct, &xe);
          dm_e += xe;
        }
      }
    }
    if (mdn) {
      wave_prod(dm_m, dm_e);
      if (lane == 0) {
        A.raw[(size_t)site * 8] = log10_mant(dm_m, dm_e);
        A.minv[site * 8] = 0.0;
        A.evals[site * 8] = 1;
      }
    }
    if constexpr (!SERIAL) {
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) plsum += __shfl_xor(plsum, o, 64);
      mono = plsum ? -(double)plsum / 10 : 0.0;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { dsum += __shfl_xor(dsum, o, 64); mqsum += __shfl_xor(mqsum, o, 64); nsd += __shfl_xor(nsd, o, 64); }
    if (lane == 0) {
      pm_site_result O;
      memset(&O, 0, sizeof(O));
      O.maxidx = -2; O.call_row = -1; O.ab = 0.5; O.denovo_lr = -1;
      A.mono_plain[site] = mono;
      if (!okref) O.status = PM_SITE_BAD_REF;
      else {
        atomicAdd(&s_c[r], 1ull);
        const int td = (int)dsum, n = (int)nsd;
        double avgmq = 0., ps = 0.;
        if (n > 0) { avgmq = (double)mqsum / (double)n; ps = (double)n / (double)np; }
        O.total_depth = td; O.num_samp_with_data = n; O.avg_map_qual = avgmq; O.perc_samp_with_data = ps;
        int st = 0;   // filters, main.cpp:345-348 (the VCF path has none)
        if (A.vcf) st = 0;
        else if (td < A.min_total_depth) st = PM_SITE_MIN_DEPTH;
        else if (A.max_total_depth > 0 && td > A.max_total_depth) st = PM_SITE_MAX_DEPTH;
        else if (ps * 100 < A.min_ps) st = PM_SITE_MIN_PS;
        else if (avgmq < A.min_map_quality) st = PM_SITE_MIN_MAPQ;
        if (st) { O.status = st; atomicAdd(&s_c[4 + st], 1ull); }
        else { O.status = PM_SITE_CALLED; valid = true; }
      }
      A.res[site] = O;
      if (valid && A.vcf) {   // PedVCF.cpp:131: PolymorphismLogLikelihood(ref, alt), one Brent
        const int slot = atomicAdd(&A.counts[0], 1);
        A.items[0][slot] = (site << 3) | 1;
      } else if (valid && A.unrelated) {   // --quick_call pre-filter first (main.cpp:354-437)
        const int slot = atomicAdd(&A.counts[1], 3);
        for (int k = 0; k < 3; k++) A.items[1][slot + k] = (site << 3) | (k + 1);
      } else if (valid) {
        const int k0 = (A.denovo && !A.mono_dn) ? 0 : 1;   // cfg 0: de novo monomorphism (unless done above)
        const int nit = 4 - k0;
        const int slot = atomicAdd(&A.counts[0], nit);
        for (int k = 0; k < nit; k++) A.items[0][slot + k] = (site << 3) | (k + k0);
      }
    }
  }
  __syncthreads();
  if (threadIdx.x < 9 && s_c[threadIdx.x]) atomicAdd(&A.counters[threadIdx.x], s_c[threadIdx.x]);
}

// CalcVarPosterior (:1693-1749); returns maxidx, sets vpp/qual/alleles
__device__ int d_var_posterior(const double* v, int n, int r, double* vpp, double* qual, int* a1, int* a2) {
  int idx = 0; double mx = v[0];
  for (int i = 0; i < n; i++) if (mx < v[i]) { mx = v[i]; idx = i; }
  double sum = 0.0;
  for (int i = 0; i < n; i++) sum += exp10(v[i] - v[idx]);
  *vpp = 1 / sum;
  const int ts = d_ts(r), tv1 = d_tv1(r), tv2 = d_tv2(r);
  if (idx == 0) {
    int k = 1; double m = v[1];
    for (int i = 1; i < 4; i++) if (m < v[i]) { m = v[i]; k = i; }
    *a1 = r; *a2 = (k == 1) ? ts : (k == 2) ? tv1 : tv2;
  } else if (idx == 1) { *a1 = r; *a2 = ts; }
  else if (idx == 2) { *a1 = r; *a2 = tv1; }
  else if (idx == 3) { *a1 = r; *a2 = tv2; }
  else if (idx == 4) { *a1 = ts; *a2 = tv1; }
  else if (idx == 5) { *a1 = ts; *a2 = tv2; }
  else { *a1 = tv1; *a2 = tv2; }
  *qual = (*vpp > 0.9999999999) ? 100 : -10 * log10(1 - *vpp);
  return idx;
}

__device__ __forceinline__ void fill_varllk(const DevArgs& A, int site, int n, double* v) {
  const double* raw = A.raw + (size_t)site * 8;
  v[0] = A.lp_mono + (A.denovo ? raw[0] : A.mono_plain[site]);
  v[1] = A.lp_ts + raw[1];
  v[2] = A.lp_tv + raw[2];
  v[3] = A.lp_tv + raw[3];
  for (int k = 4; k < n; k++) v[k] = A.lp_other + raw[k];
}

__global__ void k_select(DevArgs A) {
  const int site = blockIdx.x * blockDim.x + threadIdx.x;
  if (site >= A.n) return;
  pm_site_result* R = A.res + site;
  if (R->status != PM_SITE_CALLED) return;
  double v[7], vpp, q; int a1, a2;
  fill_varllk(A, site, 4, v);
  d_var_posterior(v, 4, A.ref[site], &vpp, &q, &a1, &a2);
  if (vpp < 0.99) {
    const int slot = atomicAdd(&A.counts[1], 3);
    for (int k = 0; k < 3; k++) A.items[1][slot + k] = (site << 3) | (4 + k);
    R->n_cfg = 7;
  } else R->n_cfg = 4;
}

// --quick_call (main.cpp:354-437): the unrelated model's varllk -- MonomorphismLogLikelihood (plain, even
// under --denovo) and the all-founder Brent results of the quick pass.
__device__ __forceinline__ void fill_varllk_quick(const DevArgs& A, int site, int n, double* v) {
  const double* raw = A.raw + (size_t)site * 8;
  v[0] = A.lp_mono + A.mono_plain[site];
  v[1] = A.lp_ts + raw[1];
  v[2] = A.lp_tv + raw[2];
  v[3] = A.lp_tv + raw[3];
  for (int k = 4; k < n; k++) v[k] = A.lp_other + raw[k];
}

__global__ void k_quick_select(DevArgs A) {   // CalcVarPosterior(4) of the quick pass -> 3 more quick items
  const int site = blockIdx.x * blockDim.x + threadIdx.x;
  if (site >= A.n || A.res[site].status != PM_SITE_CALLED) return;
  double v[7], vpp, q; int a1, a2;
  fill_varllk_quick(A, site, 4, v);
  d_var_posterior(v, 4, A.ref[site], &vpp, &q, &a1, &a2);
  A.res[site].n_cfg = 4;
  if (vpp < 0.99) {
    const int slot = atomicAdd(&A.counts[2], 3);
    for (int k = 0; k < 3; k++) A.items[2][slot + k] = (site << 3) | (4 + k);
    A.res[site].n_cfg = 7;
  }
}

__global__ void k_quick_final(DevArgs A) {   // quick decision; survivors enter the pedigree model
  const int site = blockIdx.x * blockDim.x + threadIdx.x;
  if (site >= A.n) return;
  pm_site_result* R = A.res + site;
  if (R->status != PM_SITE_CALLED) return;
  double v[7], vpp, q; int a1, a2;
  const int n = R->n_cfg;
  fill_varllk_quick(A, site, n, v);
  const int maxidx = d_var_posterior(v, n, A.ref[site], &vpp, &q, &a1, &a2);
  R->n_cfg = 0;
  if (vpp < A.posterior || maxidx == 0) { R->status = PM_SITE_QUICK_SKIP; return; }
  const int nit = A.denovo ? 4 : 3;
  const int slot = atomicAdd(&A.counts[0], nit);
  for (int k = 0; k < nit; k++) A.items[0][slot + k] = (site << 3) | (A.denovo ? k : k + 1);
}

__global__ void k_quick_stats(DevArgs A) {   // the quick lists are recycled for the main stage: keep their sizes
  A.counts[8] = A.counts[1] + A.counts[2];
  A.counts[9] = A.counts[1] / 3 + A.counts[2] / 3;
}

// main.cpp:539-574 per site; counters aggregated per block
__global__ void __launch_bounds__(256) k_finalize(DevArgs A) {
  __shared__ unsigned long long s_c[16];
  if (threadIdx.x < 16) s_c[threadIdx.x] = 0;
  __syncthreads();
  const int site = blockIdx.x * blockDim.x + threadIdx.x;
  if (site < A.n && A.res[site].status == PM_SITE_CALLED) {
    pm_site_result* R = A.res + site;
    const int r = A.ref[site], ncfg = R->n_cfg;
    double v[7], vpp, q; int a1, a2;
    fill_varllk(A, site, ncfg, v);
    const int maxidx = d_var_posterior(v, ncfg, r, &vpp, &q, &a1, &a2);
    const double* raw = A.raw + (size_t)site * 8;
    R->maxidx = maxidx; R->var_post_prob = vpp; R->poly_qual = q;
    for (int k = 0; k < 7; k++) {
      R->varllk[k] = k < ncfg ? v[k] : 0.0;
      R->varfreq[k] = k == 0 ? 1.0 : (k < ncfg ? A.minv[site * 8 + k] : 0.0);
      R->evals[k] = k < ncfg ? A.evals[site * 8 + k] : 0;
    }
    if (!A.denovo) R->evals[0] = 0;
    R->allele1 = a1; R->allele2 = a2;
    bool emit = true;
    const bool fa = A.force_call || A.all_sites;
    if (vpp < A.posterior) { atomicAdd(&s_c[15], 1ull); if (!fa) emit = false; }
    double af = 0.0;
    if (emit) {
      const int cidx[7] = {9, 10, 11, 11, 12, 13, 14};   // homo_ref, transitions, transversions x2, tstvs1, tstvs2, tvs1tvs2
      atomicAdd(&s_c[cidx[maxidx]], 1ull);
      if (maxidx == 0) af = fa ? 1.0 : 0.0;
      else af = A.minv[site * 8 + maxidx];
      if (maxidx == 0 && !A.denovo && !fa) emit = false;
    }
    if (emit && A.denovo) {
      if (maxidx == 0) {
        af = 1.0;
        // noprior[0] = varllk[0] - log10(1-prior)  (main.cpp:460), lk_mono = MonomorphismLogLikelihood
        const double dlr = (v[0] - A.lp_mono) - A.mono_plain[site];
        R->denovo_lr = dlr;
        if (dlr <= A.log10_denovo_min_llr && !fa) emit = false;   // main.cpp:563 compares with log10(minLLR)
      }
    }
    R->af = af;
    if (emit) {
      // OutputVCF_denovo (:1868) suppresses the record when denovoLR < minLLR (no log10 there)
      R->emit = (A.denovo && maxidx == 0 && R->denovo_lr < A.denovo_min_llr) ? 2 : 1;
      R->is_mono = (!A.denovo && maxidx == 0) ? 1 : 0;
      R->denovo_mono = (A.denovo && maxidx == 0) ? 1 : 0;
      atomicMin(&A.counts[4], site);
      if (A.denovo && maxidx != 0) {
        const int slot = atomicAdd(&A.counts[2], 1);
        A.items[2][slot] = (site << 3) | 7;
      }
    }
  }
  __syncthreads();
  if (threadIdx.x < 16 && threadIdx.x >= 9 && s_c[threadIdx.x]) {
    // map to pm_counters layout: [9] homo_ref .. [14] tvs1tvs2, [15] nocall
    atomicAdd(&A.counters[threadIdx.x], s_c[threadIdx.x]);
  }
}

// vcf_mode: one record per called site (PedVCF.cpp:125-162); QUAL/AF/AC formatting is the host's.
__global__ void k_finalize_vcf(DevArgs A) {
  const int site = blockIdx.x * blockDim.x + threadIdx.x;
  if (site >= A.n) return;
  pm_site_result* R = A.res + site;
  if (R->status != PM_SITE_CALLED) return;
  const int rb = A.ref[site];
  R->n_cfg = 2; R->maxidx = 1;
  R->varllk[0] = A.mono_plain[site];              // MonomorphismLogLikelihood (:74-83)
  R->varllk[1] = A.raw[(size_t)site * 8 + 1];     // PolymorphismLogLikelihood (:85-91)
  R->varfreq[0] = 1.0; R->varfreq[1] = A.minv[site * 8 + 1];
  R->evals[1] = A.evals[site * 8 + 1];
  R->allele1 = rb & 15; R->allele2 = rb >> 4;
  R->af = A.minv[site * 8 + 1];                   // GetMinimizer(): CalcPostProb frequency, AF = 1 - min
  R->emit = 1;
}

// member `sex` of famlk[0] before site `site`'s CalcPostProb / re-optimisation (non-de-novo only
// changes it; stale-state quirk of NucFamGenotypeLikelihood::likelihoodONEKid)
__device__ __forceinline__ int d_member_sex_before(const DevArgs& A, int site) {
  if (A.denovo) return 0;
  const bool seen = A.carry_postprob || A.counts[4] < site;
  return seen ? A.sex[A.n_person - 1] : 0;
}


// --denovo: denovoLR = varllk_noprior[maxidx] - lk_poly (main.cpp:567-573); famlk[0].min is overwritten
// by that re-optimisation (the printed AF) whenever a Brent ran.
__global__ void k_final_dn(DevArgs A) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= A.counts[2]) return;
  const int site = A.items[2][i] >> 3;
  pm_site_result* R = A.res + site;
  const int mx = R->maxidx;
  const double* raw = A.raw + (size_t)site * 8;
  const double npc = (mx == 1) ? A.np_ts : (mx <= 3 ? A.np_tv : A.lp_other);
  const double noprior = R->varllk[mx] - npc;
  R->denovo_lr = noprior - raw[7];
  if (!A.single_nuclear) R->af = A.minv[site * 8 + 7];
  R->emit = (R->denovo_lr < A.denovo_min_llr) ? 2 : 1;
}

// ------------------------------------------------------------------------------------------------
// posteriors: one block per emitted site, families across lanes
__device__ __forceinline__ int d_best3(double p11, double p12, double p22) {
  int b = 0; double m = p11;
  if (p12 > m) { m = p12; b = 1; }
  if (p22 > m) { m = p22; b = 2; }
  return b;
}
__device__ __forceinline__ int8_t d_vcf_label(int chrom, int membersex) {
  if (chrom == PM_CHR_Y || chrom == PM_CHR_MT) return PM_LBL_VCF_HAPLOID;
  if (chrom == PM_CHR_X && membersex == MALE) return PM_LBL_VCF_HAPLOID;
  return PM_LBL_VCF_DIPLOID;
}
// GQ = (pb > 0.9999999999) ? 100 : int(-10 log10(1 - pb) + 0.5) (OutputVCF :1818-1820) without a log10: the
// host derives, with glibc's log10 in that very expression, the smallest q = 1 - pb giving GQ <= k for every
// k (c_gq_thr[k], decreasing in k), so GQ = #{k < 100 : q < thr[k]} (q >= 1e-10 keeps it <= 100).  A float
// log10 guess g is within 1 of that count (its error is < 1e-4 on -10 log10 q <= 100), so counting over the four
// thresholds [g-2, g+2) -- one round of independent LDS reads, no loop, no branch -- gives it exactly.
// Identical to the reference's glibc result for every double pb.
__constant__ double c_gq_thr[101];
// (thr: the block's LDS copy of c_gq_thr -- the lookups' index diverges, so they are not scalar loads)
__device__ __forceinline__ int d_gq(double pb, const double* thr) {
  const double q = 1. - pb;
  const int g = (int)(-10.0f * __log10f((float)q) + 0.5f);   // (q = 0: +inf saturates; the select below wins)
  const int base = min(max(g - 2, 0), 96);
  int k = base;
#pragma unroll
  for (int i = 0; i < 4; i++) k += q < thr[base + i] ? 1 : 0;
  return pb > 0.9999999999 ? 100 : k;
}
__device__ __forceinline__ void load_gq_thr(double* s_gq) {
  for (int i = threadIdx.x; i < 101; i += blockDim.x) s_gq[i] = c_gq_thr[i];
}

// one person's genotype row entry: pm_geno_call (16 B), or in vcf_mode the 4-B pm_vcf_call (best, GQ, label:
// FamilyLikelihoodSeq_VCF::OutputVCF prints no dosage), a quarter of the bytes of the row stream
// V: vcf_mode known at compile time (0 / 1), or -1 = read A.vcf
template <int V = -1>
__device__ __forceinline__ void d_emit_call(const DevArgs& A, const double* s_gq, size_t idx, const double* post, int best,
                                            int8_t label, double dosage) {
  const double pb = post[best];
  const int gq = d_gq(pb, s_gq);
  if (V < 0 ? A.vcf != 0 : V == 1) {
    pm_vcf_call c;
    c.best = (int8_t)best; c.gq = (int8_t)gq; c.label = label; c.pad = 0;
    ((pm_vcf_call*)A.calls)[idx] = c;
    return;
  }
  pm_geno_call c;
  c.dosage = dosage; c.best = (int16_t)best; c.gq = (int16_t)gq; c.label = label;
  c._pad[0] = c._pad[1] = c._pad[2] = 0;
  A.calls[idx] = c;
}

// vcf_mode row entry from post[best] alone (FamilyLikelihoodSeq_VCF::OutputVCF prints best and GQ, no dosage)
__device__ __forceinline__ void d_emit_vcf(const DevArgs& A, const double* s_gq, size_t idx, double pb, int best, int8_t label) {
  pm_vcf_call c;
  c.best = (int8_t)best; c.gq = (int8_t)d_gq(pb, s_gq); c.label = label; c.pad = 0;
  ((pm_vcf_call*)A.calls)[idx] = c;
}

// likelihoodKidGenotype, :1334-1443
__device__ void d_kid_geno(int chrom, const uint8_t* pl, int np, const double* lk, int p0, int n, const int8_t* sexv, int g11, int g12,
                           int g22, int kid, int k, double* out) {
  const bool X = chrom == PM_CHR_X, Y = chrom == PM_CHR_Y, MT = chrom == PM_CHR_MT;
  double G11 = 1.0, G12 = 1.0, G22 = 1.0, l = 0.0, q11 = 0, q12 = 0, q22 = 0;
  for (int i = 2; i < n; i++) {
    const double l11 = lk[PLB(pl, np, p0 + i, g11)], l12 = lk[PLB(pl, np, p0 + i, g12)], l22 = lk[PLB(pl, np, p0 + i, g22)];
    const int sex = sexv[p0 + i];
    switch (k) {
      case 0: l = l11; q11 = l11; q12 = q22 = 0; break;
      case 1:
        if (X) { l = sex == MALE ? 0.5 * (l11 + l22) : 0.5 * (l11 + l12);
                 if (sex == MALE) { q11 = 0.5 * l11; q12 = 0.0; q22 = 0.5 * l22; } else { q11 = 0.5 * l11; q12 = 0.5 * l12; q22 = 0; } }
        else if (Y) { l = sex == MALE ? l11 : 1.0; if (sex == MALE) { q11 = l11; q12 = q22 = 0.0; } else { q11 = q12 = q22 = 0.0; } }
        else if (MT) { l = 0.5 * (l11 + l22); q11 = 0.5 * l11; q22 = 0.5 * l22; q12 = 0.0; }
        else { l = 0.5 * (l11 + l12); q11 = l11 * 0.5; q12 = l12 * 0.5; q22 = 0; }
        break;
      case 2:
        if (X) { l = sex == MALE ? l22 : l12; if (sex == MALE) { q11 = q12 = 0; q22 = l22; } else { q11 = q22 = 0; q12 = l12; } }
        else if (Y) { l = sex == MALE ? l11 : 1.0; if (sex == MALE) { q11 = l11; q12 = q22 = 0; } else { q11 = q12 = q22 = 0.; } }
        else if (MT) { l = l22; q11 = q12 = 0; q22 = l22; }
        else { l = l12; q11 = 0; q12 = l12; q22 = 0; }
        break;
      case 3:
        if (X || Y || MT) { l = 0.0; q11 = q12 = q22 = 0.0; }
        else { l = 0.5 * (l11 + l12); q11 = l11 * 0.5; q12 = l12 * 0.5; q22 = 0; }
        break;
      case 4:
        if (X || Y || MT) { l = 0.0; q11 = q12 = q22 = 0.0; }
        else { l = 0.25 * l11 + 0.5 * l12 + 0.25 * l22; q11 = l11 * 0.25; q12 = l12 * 0.5; q22 = l22 * 0.25; }
        break;
      case 5:
        if (X || Y || MT) { l = 0.0; q11 = q12 = q22 = 0.0; }
        else { l = 0.5 * (l12 + l22); q11 = 0; q12 = l12 * 0.5; q22 = l22 * 0.5; }
        break;
      case 6:
        if (X) { l = sex == MALE ? l11 : l12; if (sex == MALE) { q11 = l11; q12 = q22 = 0.0; } else { q11 = q22 = 0.0; q12 = l12; } }
        else if (Y) { l = sex == MALE ? l22 : 1.0; if (sex == MALE) { q11 = q12 = 0.0; q22 = l22; } else { q11 = q12 = q22 = 0.0; } }
        else if (MT) { l = l11; q11 = l11; q12 = q22 = 0.0; }
        else { l = l12; q11 = 0; q12 = l12; q22 = 0; }
        break;
      case 7:
        if (X) { l = sex == MALE ? 0.5 * (l11 + l22) : 0.5 * (l12 + l22);
                 if (sex == MALE) { q11 = 0.5 * l11; q22 = 0.5 * l22; q12 = 0.0; } else { q11 = 0.0; q12 = 0.5 * l12; q22 = 0.5 * l22; } }
        else if (Y) { l = sex == MALE ? l22 : 1.0; if (sex == MALE) { q11 = q12 = 0.0; q22 = l22; } else { q11 = q12 = q22 = 0.0; } }
        else if (MT) { l = 0.5 * (l11 + l22); q11 = 0.5 * l11; q22 = 0.5 * l22; q12 = 0.0; }
        else { l = 0.5 * (l12 + l22); q11 = 0; q12 = l12 * 0.5; q22 = l22 * 0.5; }
        break;
      default:   // if/if/if-else chain of :1416-1422
        if (X) { l = l22; q11 = 0.0; q22 = l22; }
        if (Y) { l = sex == MALE ? l22 : 1.0; if (sex == MALE) { q11 = q12 = 0.0; q22 = l22; } else { q11 = q22 = q12 = 0.0; } }
        if (MT) { l = l22; q11 = q12 = 0.0; q22 = l22; }
        else { l = l22; q11 = 0; q12 = 0; q22 = l22; }
        break;
    }
    if (i != kid) { G11 *= l; G12 *= l; G22 *= l; }
    else { G11 *= q11; G12 *= q12; G22 *= q22; }
  }
  out[0] = G11; out[1] = G12; out[2] = G22;
}

// The 12 PL bytes of a nuclear family of <= 4 persons: (g11, g12, g22) of father, mother and the two kid slots
// (a trio's second kid slot repeats its kid; every read stays inside the family)
__device__ __forceinline__ void lean_fam_bytes(const uint8_t* pl, int np, int p0, int n, int g11, int g12, int g22, uint32_t* by) {
  const uint8_t *P11 = pl + (size_t)g11 * np, *P12 = pl + (size_t)g12 * np, *P22 = pl + (size_t)g22 * np;
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const int pq = p0 + (q < 2 ? q : 2 + (q < n ? q - 2 : 0));
    by[3 * q] = P11[pq]; by[3 * q + 1] = P12[pq]; by[3 * q + 2] = P22[pq];
  }
}

// LEAN nuclear family (autosome, <= 4 persons, not de novo) from its 12 PL bytes (lean_fam_bytes, loaded ahead by
// the caller): the arithmetic of hoist_nuc, CalcParentMarginal and KidJointGenoLikelihood below in the same
// operation order -- the same values bit for bit
// NF = the family's persons when the caller knows them for the whole wave (3: trio, 4: quad; 0 = runtime n): the
// kid loops and the one-kid / two-kid selects then resolve at compile time (same operations, same bits)
template <bool VCF, int NF = 0>
__device__ __forceinline__ void lean_nuc_post(const DevArgs& A, const double* s_lk, const double* s_gq, const uint32_t* by,
                                              size_t out, int p0, int n_rt, const double* pp) {
  const int n = NF ? NF : n_rt;
  double lF[3], lM[3], kl[2][3];
#pragma unroll
  for (int t = 0; t < 3; t++) {
    lF[t] = s_lk[by[t]]; lM[t] = s_lk[by[3 + t]]; kl[0][t] = s_lk[by[6 + t]]; kl[1][t] = s_lk[by[9 + t]];
  }
  double kids[9];
#pragma unroll
  for (int k = 0; k < 9; k++) kids[k] = 1.0;
#pragma unroll
  for (int i = 0; i < 2; i++) {   // hoist_nuc's kid loop, j = 2 .. n-1
    if (2 + i >= n) break;
#pragma unroll
    for (int k = 0; k < 9; k++) kids[k] *= d_one_kid(k, PM_CHR_AUTO, 0, kl[i][0], kl[i][1], kl[i][2]);
  }
  double m[9], wk[9];
#pragma unroll
  for (int a = 0; a < 3; a++)
#pragma unroll
    for (int b = 0; b < 3; b++) {
      const double pg = lF[a] * lM[b];
      m[3 * a + b] = (kids[3 * a + b] * pg) * pp[3 * a + b];   // cond[k] * pp[k]
      wk[3 * a + b] = pg * pp[3 * a + b];
    }
#pragma unroll
  for (int j = 0; j < 2; j++) {   // CalcPostProb parents
    double q11, q12, q22;
    if (j == 0) { q11 = m[0] + m[1] + m[2]; q12 = m[3] + m[4] + m[5]; q22 = m[6] + m[7] + m[8]; }
    else { q11 = m[0] + m[3] + m[6]; q12 = m[1] + m[4] + m[7]; q22 = m[2] + m[5] + m[8]; }
    const double sum = q11 + q12 + q22;
    if constexpr (VCF) {   // one quotient: post[best]
      const int best = d_best3(q11, q12, q22);
      const double qb = best == 0 ? q11 : best == 1 ? q12 : q22;
      d_emit_vcf(A, s_gq, out + p0 + j, sum != 0 ? qb / sum : 0.0, best, PM_LBL_VCF_DIPLOID);
      continue;
    }
    double post[3] = {0, 0, 0};
    if (sum != 0) { post[0] = q11 / sum; post[1] = q12 / sum; post[2] = q22 / sum; }
    d_emit_call<0>(A, s_gq, out + p0 + j, post, d_best3(q11, q12, q22), PM_LBL_VCF_DIPLOID, post[1] + post[2] * 2);
  }
#pragma unroll
  for (int j = 2; j < 4; j++) {   // KidJointGenoLikelihood :798-835, autosomal
    if (j >= n) break;
    // J[k][t] = prod over kids (in order, from 1.0) of q_j(k)[t] for kid j and l_i(k) for the other kid, then
    // g[t] = sum_k J[k][t] w[k].  The structurally zero q terms (e.g. q12 = q22 = 0 when both parents are 11) are
    // skipped: their products are +0 and adding +0 leaves every partial sum's bits unchanged (all terms finite, >= 0)
    const int me = j - 2, other = 1 - me;
    const bool two = n == 4;
    const double m11 = kl[me][0], m12 = kl[me][1], m22 = kl[me][2];
    const double o11 = kl[other][0], o12 = kl[other][1], o22 = kl[other][2];
    double g[3] = {0.0, 0.0, 0.0};
#pragma unroll
    for (int k = 0; k < 9; k++) {
      double lo, q11 = 0, q12 = 0, q22 = 0;   // the other kid's likelihood, this kid's genotype terms (d_kid_geno's switch)
      bool z11 = true, z12 = true, z22 = true;
      switch (k) {
        case 0: lo = o11; q11 = m11; z11 = false; break;
        case 1: case 3: lo = 0.5 * (o11 + o12); q11 = m11 * 0.5; q12 = m12 * 0.5; z11 = z12 = false; break;
        case 2: case 6: lo = o12; q12 = m12; z12 = false; break;
        case 4: lo = 0.25 * o11 + 0.5 * o12 + 0.25 * o22; q11 = m11 * 0.25; q12 = m12 * 0.5; q22 = m22 * 0.25; z11 = z12 = z22 = false; break;
        case 5: case 7: lo = 0.5 * (o12 + o22); q12 = m12 * 0.5; q22 = m22 * 0.5; z12 = z22 = false; break;
        default: lo = o22; q22 = m22; z22 = false; break;
      }
      const double w = wk[k];
      // kid order: (1.0 * f_kid2) * f_kid3 -- one product, whichever kid carries q
      if (!z11) g[0] = g[0] + (two ? q11 * lo : q11) * w;
      if (!z12) g[1] = g[1] + (two ? q12 * lo : q12) * w;
      if (!z22) g[2] = g[2] + (two ? q22 * lo : q22) * w;
    }
    const double sum = g[0] + g[1] + g[2];
    if constexpr (VCF) {
      // d_best3 over the quotients g[t] / sum (sum > 0, g >= 0: division is monotone) is the first t whose
      // quotient equals the largest one, post[b] with b = d_best3(g); an earlier quotient can only equal it
      // when its g is within a rounding of g[b], so the other divisions are done only then
      const int b = d_best3(g[0], g[1], g[2]);
      const double gb = b == 0 ? g[0] : b == 1 ? g[1] : g[2];
      double pb = 0.0;
      int best = b;
      if (sum != 0.0) {
        pb = gb / sum;
        const double near = gb * (1.0 - 1e-12);
        if (b >= 1 && g[0] >= near && g[0] / sum == pb) best = 0;
        else if (b == 2 && g[1] >= near && g[1] / sum == pb) best = 1;
      }
      d_emit_vcf(A, s_gq, out + p0 + j, pb, best, PM_LBL_VCF_DIPLOID);
      continue;
    }
    double post[3] = {0, 0, 0};
    if (sum != 0.0) { post[0] = g[0] / sum; post[1] = g[1] / sum; post[2] = g[2] / sum; }
    d_emit_call<0>(A, s_gq, out + p0 + j, post, d_best3(post[0], post[1], post[2]), PM_LBL_VCF_DIPLOID, post[1] + post[2] * 2);
  }
}

// (autosomal nuclear families of <= 4 persons without the de novo model and extended families: k_posterior_lean)
template <bool DN, bool ES>
__global__ void __launch_bounds__(256) k_posterior(DevArgs A) {
  __shared__ double s_lk[256];
  __shared__ double s_M[100];
  __shared__ double s_gq[101];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) s_lk[i] = A.lktab[i];
  for (int i = threadIdx.x; i < 100; i += blockDim.x) s_M[i] = A.M[i];
  load_gq_thr(s_gq);
  __syncthreads();
  const long long work = (long long)A.counts[3] * A.n_fam;
  const size_t gid_base = (size_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (size_t)gridDim.x * blockDim.x;
  for (long long gid = (long long)gid_base; gid < work; gid += (long long)stride) {
    // 32-bit division when the work index fits (a 64-bit divide is a long software sequence on the GPU)
    int row, f;
    if (work < 0xFFFFFFFFll) { const unsigned u = (unsigned)gid, nf = (unsigned)A.n_fam; row = (int)(u / nf); f = (int)(u - (unsigned)row * nf); }
    else { row = (int)(gid / A.n_fam); f = (int)(gid % A.n_fam); }
    f = A.fam_perm[f];
    const int site = A.row_site[row];
    const pm_site_result* R = A.res + site;
    const int np = A.n_person;
    const uint8_t* pl = A.pl + (size_t)site * np * 10;
    const size_t out = (size_t)row * np;   // genotype row index base
    const int a1 = R->allele1, a2 = R->allele2;
    const int g11 = d_gi(a1, a1), g12 = d_gi(a1, a2), g22 = d_gi(a2, a2);
    const int chrom = A.chrom;
    constexpr int dn = DN ? 1 : 0;
    // CalcPostProb freq (main.cpp:576-587)
    const double freq = (R->maxidx == 0) ? (dn ? 1.0 : 1 - A.theta) : R->af;
    const int is_mono = (R->maxidx == 0 && !dn) ? 1 : 0;
    const int sex_carry = d_member_sex_before(A, site);
    {
      const int p0 = A.fam_start[f], n = A.fam_start[f + 1] - p0, kind = A.fam_kind[f];
      // member sex when family f's CalcParentMarginal runs: last member of family f-1 (non-de-novo)
      const int msex = dn ? 0 : (f == 0 ? sex_carry : A.sex[p0 - 1]);
      if (kind == PM_FAM_FOUNDERS) {
        for (int j = 0; j < n; j++) {   // CalcPostProb_SinglePerson :754-795
          const int p = p0 + j, sx = A.sex[p];
          const double l11 = s_lk[PLB(pl, np, p, g11)], l12 = s_lk[PLB(pl, np, p, g12)], l22 = s_lk[PLB(pl, np, p, g22)];
          const double fq = freq, gq = 1 - freq;
          double pr0 = fq * fq, pr1 = fq * gq * 2, pr2 = gq * gq;
          if (chrom == PM_CHR_X) { if (sx == MALE) { pr0 = fq; pr1 = 0.; pr2 = 1 - fq; } else { pr0 = fq * fq; pr1 = 2 * fq * gq; pr2 = gq * gq; } }
          if (chrom == PM_CHR_Y) { if (sx == MALE) { pr0 = fq; pr1 = 0.; pr2 = 1 - fq; } else { pr0 = pr1 = pr2 = 1.0; } }
          if (chrom == PM_CHR_MT) { pr0 = fq; pr1 = 0; pr2 = 1 - fq; }
          const double m11 = l11 * pr0, m12 = l12 * pr1, m22 = l22 * pr2;
          const double sum = m11 + m12 + m22;
          double post[3] = {0, 0, 0};
          if (sum != 0) { post[0] = m11 / sum; post[1] = m12 / sum; post[2] = m22 / sum; }
          const bool yf = chrom == PM_CHR_Y && sx == FEMALE;
          if (yf) post[0] = post[1] = post[2] = 0.0;
          const int best = d_best3(m11, m12, m22);
          // label: own sex (non-de-novo sets member sex first); de novo leaves it stale (0)
          const int8_t lab = yf ? PM_LBL_DOT : d_vcf_label(chrom, dn ? 0 : sx);
          d_emit_call(A, s_gq, out + p, post, best, lab, post[1] + post[2] * 2);
        }
        continue;
      }
      if (ES && (kind == PM_FAM_EXTENDED || (A.nuc_es && kind == PM_FAM_NUCLEAR))) continue;   // k_posterior_es
      if (kind != PM_FAM_NUCLEAR) continue;
      // CalcParentMarginal(_denovo) at freq
      ItemCtx I;
      I.a1 = a1; I.a2 = a2; I.g11 = g11; I.g12 = g12; I.g22 = g22; I.denovo = dn; I.sex = msex; I.chrom = chrom;
      double cond[9], pp[9], pg[9];
      hoist_nuc<true>(A, I, pl, s_lk, s_M, p0, n, cond);
      int pmode;
      if (dn) pmode = A.n_fam_gt1 ? PR_AUTO : PR_DN_SINGLE;
      else if (!A.n_fam_gt1 && !is_mono) pmode = PR_TRIO;
      else pmode = chrom == PM_CHR_X ? PR_X : chrom == PM_CHR_Y ? PR_Y : chrom == PM_CHR_MT ? PR_MT : PR_AUTO;
      d_parent_prior(pmode, freq, pp);
      {
        double F11 = s_lk[PLB(pl, np, p0, g11)], F12 = s_lk[PLB(pl, np, p0, g12)], F22 = s_lk[PLB(pl, np, p0, g22)];
        double M11 = s_lk[PLB(pl, np, p0 + 1, g11)], M12 = s_lk[PLB(pl, np, p0 + 1, g12)], M22 = s_lk[PLB(pl, np, p0 + 1, g22)];
        if (!dn) {
          if (chrom == PM_CHR_X) F12 = 0.0;
          if (chrom == PM_CHR_Y) { M11 = M12 = M22 = 1.0; F12 = 0.0; }
          if (chrom == PM_CHR_MT) F12 = M12 = 0.0;
        }
        const double lF[3] = {F11, F12, F22}, lM[3] = {M11, M12, M22};
        for (int x = 0; x < 3; x++) for (int y = 0; y < 3; y++) pg[3 * x + y] = lF[x] * lM[y];
      }
      double m[9], wk[9];   // wk: the kid weights pg[k] * pp[k] of KidJointGenoLikelihood (cond, pg, pp die here)
      for (int k = 0; k < 9; k++) { m[k] = cond[k] * pp[k]; wk[k] = pg[k] * pp[k]; }
      for (int j = 0; j < n; j++) {
        const int p = p0 + j;
        const int sx = A.sex[p];
        if (j < 2) {
          double q11, q12, q22;
          if (j == 0) { q11 = m[0] + m[1] + m[2]; q12 = m[3] + m[4] + m[5]; q22 = m[6] + m[7] + m[8]; }
          else { q11 = m[0] + m[3] + m[6]; q12 = m[1] + m[4] + m[7]; q22 = m[2] + m[5] + m[8]; }
          const double sum = q11 + q12 + q22;
          double post[3] = {0, 0, 0};
          if (sum != 0) { post[0] = q11 / sum; post[1] = q12 / sum; post[2] = q22 / sum; }
          const int best = d_best3(q11, q12, q22);
          const int8_t lab = dn ? (int8_t)PM_LBL_ALLELES : ((chrom == PM_CHR_Y && sx == FEMALE) ? (int8_t)PM_LBL_DOT : d_vcf_label(chrom, sx));
          d_emit_call(A, s_gq, out + p, post, best, lab, post[1] + post[2] * 2);
        } else if (!dn && chrom == PM_CHR_AUTO && n <= 4) {   // KidJointGenoLikelihood :798-835, autosomal, <= 2 kids
          // d_kid_geno's autosomal branches with every kid's three likelihoods loaded once and k unrolled; the
          // products run over the kids in the same order from 1.0, so the values are d_kid_geno's bit for bit
          double kl[2][3];
#pragma unroll
          for (int i = 0; i < 2; i++) {
            const int pi = p0 + 2 + (2 + i < n ? i : 0);
            kl[i][0] = s_lk[PLB(pl, np, pi, g11)]; kl[i][1] = s_lk[PLB(pl, np, pi, g12)]; kl[i][2] = s_lk[PLB(pl, np, pi, g22)];
          }
          double g[3] = {0.0, 0.0, 0.0};
#pragma unroll
          for (int k = 0; k < 9; k++) {
            double G[3] = {1.0, 1.0, 1.0};
#pragma unroll
            for (int i = 0; i < 2; i++) {
              if (2 + i >= n) break;
              const double l11 = kl[i][0], l12 = kl[i][1], l22 = kl[i][2];
              double l, q11, q12, q22;
              switch (k) {
                case 0: l = l11; q11 = l11; q12 = q22 = 0; break;
                case 1: case 3: l = 0.5 * (l11 + l12); q11 = l11 * 0.5; q12 = l12 * 0.5; q22 = 0; break;
                case 2: case 6: l = l12; q11 = 0; q12 = l12; q22 = 0; break;
                case 4: l = 0.25 * l11 + 0.5 * l12 + 0.25 * l22; q11 = l11 * 0.25; q12 = l12 * 0.5; q22 = l22 * 0.25; break;
                case 5: case 7: l = 0.5 * (l12 + l22); q11 = 0; q12 = l12 * 0.5; q22 = l22 * 0.5; break;
                default: l = l22; q11 = 0; q12 = 0; q22 = l22; break;
              }
              if (2 + i != j) { G[0] *= l; G[1] *= l; G[2] *= l; }
              else { G[0] *= q11; G[1] *= q12; G[2] *= q22; }
            }
            const double w = wk[k];
#pragma unroll
            for (int t = 0; t < 3; t++) g[t] = (k == 0) ? G[t] * w : g[t] + G[t] * w;   // J[0] + J[1] + ... + J[8]
          }
          const double sum = g[0] + g[1] + g[2];
          double post[3] = {0, 0, 0};
          if (sum != 0.0) { post[0] = g[0] / sum; post[1] = g[1] / sum; post[2] = g[2] / sum; }
          d_emit_call(A, s_gq, out + p, post, d_best3(post[0], post[1], post[2]), d_vcf_label(chrom, sx), post[1] + post[2] * 2);
        } else if (!dn) {   // KidJointGenoLikelihood :798-835
          double J[9][3];
          for (int k = 0; k < 9; k++) {
            d_kid_geno(chrom, pl, np, s_lk, p0, n, A.sex, g11, g12, g22, j, k, J[k]);
            const double w = pg[k] * pp[k];
            J[k][0] *= w; J[k][1] *= w; J[k][2] *= w;
          }
          double g[3];
          for (int t = 0; t < 3; t++) g[t] = J[0][t] + J[1][t] + J[2][t] + J[3][t] + J[4][t] + J[5][t] + J[6][t] + J[7][t] + J[8][t];
          const double sum = g[0] + g[1] + g[2];
          double post[3] = {0, 0, 0};
          if (sum != 0.0) { post[0] = g[0] / sum; post[1] = g[1] / sum; post[2] = g[2] / sum; }
          const int best = d_best3(post[0], post[1], post[2]);
          const int8_t lab = (chrom == PM_CHR_Y && sx == FEMALE) ? (int8_t)PM_LBL_DOT : d_vcf_label(chrom, sx);
          d_emit_call(A, s_gq, out + p, post, best, lab, post[1] + post[2] * 2);
        } else {   // KidJointGenoLikelihood_denovo :838-868
          double gsum[10];
          for (int t = 0; t < 10; t++) gsum[t] = 0.0;
          for (int k = 0; k < 9; k++) {
            double Jk[10];
            for (int t = 0; t < 10; t++) Jk[t] = 1.0;
            for (int i = 2; i < n; i++) {
              const uint8_t* K = pl + p0 + i;   // plane g at K[g * np]
              if (i != j) {
                double D11 = 0.0, D12 = 0.0, D22 = 0.0;
                for (int gg = 0; gg < 10; gg++) {
                  const double pv = s_lk[K[(size_t)gg * np]];
                  D11 += s_M[g11 * 10 + gg] * pv; D12 += s_M[g12 * 10 + gg] * pv; D22 += s_M[g22 * 10 + gg] * pv;
                }
                const double l = d_one_kid_dn(k, D11, D12, D22);
                for (int t = 0; t < 10; t++) Jk[t] *= l;
              } else {   // GetJointGenoLk_denovo :1480-1551
                for (int t = 0; t < 10; t++) {
                  double mm;
                  switch (k) {
                    case 0: mm = s_M[g11 * 10 + t]; break;
                    case 1: case 3: mm = 0.5 * s_M[g11 * 10 + t] + 0.5 * s_M[g12 * 10 + t]; break;
                    case 2: case 6: mm = s_M[g12 * 10 + t]; break;
                    case 4: mm = 0.25 * s_M[g11 * 10 + t] + 0.5 * s_M[g12 * 10 + t] + 0.25 * s_M[g22 * 10 + t]; break;
                    case 5: case 7: mm = 0.5 * s_M[g12 * 10 + t] + 0.5 * s_M[g22 * 10 + t]; break;
                    default: mm = s_M[g22 * 10 + t]; break;
                  }
                  Jk[t] *= mm * s_lk[K[(size_t)t * np]];
                }
              }
            }
            const double w = pg[k] * pp[k];
            for (int t = 0; t < 10; t++) gsum[t] += Jk[t] * w;
          }
          double sum = 0.0;
          for (int t = 0; t < 10; t++) sum += gsum[t];
          double post[10];
          for (int t = 0; t < 10; t++) post[t] = (sum == 0.0) ? 0.0 : gsum[t] / sum;
          int best = 0; double mx = 0.0;
          for (int t = 0; t < 10; t++) if (mx < post[t]) { mx = post[t]; best = t; }
          d_emit_call(A, s_gq, out + p, post, best, PM_LBL_GENO10, 0.0);
        }
      }
    }
  }
}

// LEAN posteriors (autosome, no de novo model, nuclear families of <= 4 persons and founder families),
// row-blocked: a block takes one emitted row at a time and its threads stride over the row's families in
// fam_perm order (one family size per stretch of lanes).  The family table (fam_perm order, packed first person |
// persons << 24 | nuclear << 31) sits in LDS, so a family's PL addresses need no global round trip; the row's
// set-up (genotype indices, frequency, SetParentPrior :318-368) runs once per thread and row, and its successor's
// result fields are loaded while the row is computed.  VCF: vcf_mode rows (A.vcf).  Same arithmetic, in the same
// order, as k_posterior.
struct LeanRow {
  const uint8_t* pl;
  size_t out;
  int g11, g12, g22;
  double freq;
  int mono;
};
__device__ __forceinline__ void lean_row(const DevArgs& A, int row, LeanRow& r) {
  const int site = A.row_site[row];
  const pm_site_result* R = A.res + site;
  r.pl = A.pl + (size_t)site * A.n_person * 10;
  r.out = (size_t)row * A.n_person;
  const int a1 = R->allele1, a2 = R->allele2;
  r.g11 = d_gi(a1, a1); r.g12 = d_gi(a1, a2); r.g22 = d_gi(a2, a2);
  r.mono = R->maxidx == 0 ? 1 : 0;
  r.freq = r.mono ? 1 - A.theta : R->af;   // main.cpp:576-587
}
template <bool VCF>
__global__ void __launch_bounds__(256) k_posterior_lean(DevArgs A) {
  __shared__ double s_lk[256];
  __shared__ double s_gq[101];
  extern __shared__ uint32_t s_fam[];   // [n_fam]
  for (int i = threadIdx.x; i < 256; i += blockDim.x) s_lk[i] = A.lktab[i];
  load_gq_thr(s_gq);
  for (int fi = threadIdx.x; fi < A.n_fam; fi += blockDim.x) {
    const int f = A.fam_perm[fi];
    const int p0 = A.fam_start[f], n = A.fam_start[f + 1] - p0;
    s_fam[fi] = (uint32_t)p0 | (uint32_t)n << 24 | (A.fam_kind[f] == PM_FAM_NUCLEAR ? 1u << 31 : 0u);
  }
  __syncthreads();
  const int rows = A.counts[3], np = A.n_person, nf = A.n_fam;
  int row = blockIdx.x;
  if (row >= rows || (int)threadIdx.x >= nf) return;
  LeanRow cur, nxt;
  lean_row(A, row, cur);
  for (; row < rows; row += gridDim.x) {
    if (row + (int)gridDim.x < rows) lean_row(A, row + gridDim.x, nxt);
    double pp[9];
    d_parent_prior((!A.n_fam_gt1 && !cur.mono) ? PR_TRIO : PR_AUTO, cur.freq, pp);
    const double fq = cur.freq, gq = 1 - cur.freq;
    const double pr0 = fq * fq, pr1 = fq * gq * 2, pr2 = gq * gq;   // CalcPostProb_SinglePerson's HWE prior (:754-795)
    for (int fi = threadIdx.x; fi < nf; fi += blockDim.x) {
      const uint32_t d = s_fam[fi];
      const int p0 = d & 0xFFFFFF, n = (d >> 24) & 127;
      if (d >> 31) {
        uint32_t by[12];
        lean_fam_bytes(cur.pl, np, p0, n, cur.g11, cur.g12, cur.g22, by);
        // fam_perm groups families by size, so a wave's families almost always share one: specialised bodies
        const int n0 = __builtin_amdgcn_readfirstlane(n);
        const bool uni = __builtin_amdgcn_ballot_w64(n != n0) == 0;
        if (uni && n0 == 4) lean_nuc_post<VCF, 4>(A, s_lk, s_gq, by, cur.out, p0, n, pp);
        else if (uni && n0 == 3) lean_nuc_post<VCF, 3>(A, s_lk, s_gq, by, cur.out, p0, n, pp);
        else lean_nuc_post<VCF>(A, s_lk, s_gq, by, cur.out, p0, n, pp);
      } else {
        for (int j = 0; j < n; j++) {
          const int p = p0 + j;
          const double l11 = s_lk[PLB(cur.pl, np, p, cur.g11)], l12 = s_lk[PLB(cur.pl, np, p, cur.g12)], l22 = s_lk[PLB(cur.pl, np, p, cur.g22)];
          const double m11 = l11 * pr0, m12 = l12 * pr1, m22 = l22 * pr2;
          const double sum = m11 + m12 + m22;
          double post[3] = {0, 0, 0};
          if (sum != 0) { post[0] = m11 / sum; post[1] = m12 / sum; post[2] = m22 / sum; }
          d_emit_call<VCF ? 1 : 0>(A, s_gq, cur.out + p, post, d_best3(m11, m12, m22), PM_LBL_VCF_DIPLOID, post[1] + post[2] * 2);
        }
      }
    }
    cur = nxt;
  }
}

// CalculateAB (:1006-1039) for emitted autosomal non-de-novo sites: wave per row, per-person terms in
// parallel, the two sums reduced as lane partials + butterfly.  The reference sums in person order; the
// reordering changes AB by ~1e-16 relative (AB is printed with %.3f; parity tolerance 1e-9).
// CalcPostProb_SingleExtendedPed_BA (FamilyLikelihoodSeq.cpp:171-216) / _denovo (:140-169) for the peeled
// families: one thread per (row, person), three (or ten) FillZeroPenetrance peels (:327-356) of the person's
// family at the site's frequency, in the reference's operation order (d_es_lk).  Splitting the families'
// persons over threads gives ten times the parallelism of a thread per (row, family).
// LDSWS: each thread's peel workspace (ws_per_lane doubles) in LDS, interleaved across the block's threads, instead
// of the lane-interleaved HBM workspace: every partial / marriage-partial access of the 3 (10) peels per person
// is then an LDS round trip (~100 cycles) rather than an HBM one (the HBM workspace of the whole grid does not fit
// the caches: PMC showed 88% of wave cycles waiting).
template <bool DN, bool LDSWS = false>
__global__ void __launch_bounds__(256) k_posterior_es(DevArgs A) {
  __shared__ double s_lk[256];
  __shared__ double s_gq[101];
  extern __shared__ double s_wsp[];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) s_lk[i] = A.lktab[i];
  load_gq_thr(s_gq);
  __syncthreads();
  const long long work = (long long)A.counts[3] * A.n_es_pers;
  const size_t gid_base = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t stride = LDSWS ? (size_t)blockDim.x : (size_t)gridDim.x * blockDim.x;   // workspace stride
  double* wsl = LDSWS ? s_wsp + threadIdx.x : A.ws + gid_base;
  for (long long gid = (long long)gid_base; gid < work; gid += (long long)gridDim.x * blockDim.x) {
    const int row = (int)(gid / A.n_es_pers), e = A.es_pers[gid % A.n_es_pers];
    const int f = e >> 8, j = e & 255;
    const int site = A.row_site[row];
    const pm_site_result* R = A.res + site;
    const int np = A.n_person;
    const uint8_t* pl = A.pl + (size_t)site * np * 10;
    const size_t out = (size_t)row * np;   // genotype row index base
    const int a1 = R->allele1, a2 = R->allele2;
    const int g11 = d_gi(a1, a1), g12 = d_gi(a1, a2), g22 = d_gi(a2, a2);
    const int chrom = A.chrom;
    const double freq = (R->maxidx == 0) ? (DN ? 1.0 : 1 - A.theta) : R->af;   // main.cpp:576-587
    const int p = A.fam_start[f] + j, sx = A.sex[p];
    if (!DN) {
      if (chrom == PM_CHR_Y && sx == FEMALE) {
        const double z[3] = {0, 0, 0};
        d_emit_call(A, s_gq, out + p, z, 0, PM_LBL_DOT, 0.0);
        continue;
      }
      const double l11 = d_es_lk<3>(A, f, pl, s_lk, g11, g12, g22, chrom, freq, j, g11, wsl, stride);
      const double l12 = d_es_lk<3>(A, f, pl, s_lk, g11, g12, g22, chrom, freq, j, g12, wsl, stride);
      const double l22 = d_es_lk<3>(A, f, pl, s_lk, g11, g12, g22, chrom, freq, j, g22, wsl, stride);
      const double sum = l11 + l12 + l22;
      double post[3] = {0, 0, 0};
      if (sum != 0) { post[0] = l11 / sum; post[1] = l12 / sum; post[2] = l22 / sum; }
      d_emit_call(A, s_gq, out + p, post, d_best3(l11, l12, l22), d_vcf_label(chrom, sx), post[1] + post[2] * 2);
    } else {
      double lkv[10], sum = 0.0;
      for (int k = 0; k < 10; k++) lkv[k] = d_es_lk<10>(A, f, pl, s_lk, g11, g12, g22, chrom, freq, j, k, wsl, stride);
      for (int k = 0; k < 10; k++) sum += lkv[k];
      double post[10];
      for (int k = 0; k < 10; k++) post[k] = (sum == 0) ? 0 : lkv[k] / sum;
      int b = 0; double mx = 0.0;
      for (int k = 0; k < 10; k++) if (mx < lkv[k]) { mx = lkv[k]; b = k; }
      d_emit_call(A, s_gq, out + p, post, b, PM_LBL_GENO10, 0.0);
    }
  }
}

__global__ void __launch_bounds__(256) k_ab(DevArgs A) {
  __shared__ double s_lk[256];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) s_lk[i] = A.lktab[i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int rows = A.counts[3];
  for (int row = blockIdx.x * 4 + (threadIdx.x >> 6); row < rows; row += gridDim.x * 4) {
    const int site = A.row_site[row];
    const pm_site_result* R = A.res + site;
    const int np = A.n_person;
    const uint8_t* pl = A.pl + (size_t)site * np * 10;
    const uint32_t* dm = A.dm + (size_t)site * np;
    const int a1 = R->allele1, a2 = R->allele2;
    const int g11 = d_gi(a1, a1), g12 = d_gi(a1, a2), g22 = d_gi(a2, a2);
    const double fr = R->af;
    const double p11 = fr * fr, p12 = 2 * fr * (1 - fr), p22 = (1 - fr) * (1 - fr);
    double Asum = 0.0, Bsum = 0.0;
    for (int p = lane; p < np; p += 64) {
      const int depth = (int)(dm[p] & 0xFFFFFF);
      const int k11 = PLB(pl, np, p, g11), k12 = PLB(pl, np, p, g12), k22 = PLB(pl, np, p, g22);
      const double l11 = s_lk[k11], l12 = s_lk[k12], l22 = s_lk[k22];
      const double PHet = (p12 * l12) / (p11 * l11 + p12 * l12 + p22 * l22);
      if (PHet > 1e-05 && depth > 0) {
        int scale = k22 + k11 - 2 * k12 + 6 * depth;
        const int minimum = abs(k22 - k11);
        if (scale < 4) scale = 4;
        if (scale < minimum) scale = minimum;
        const int nRef = (int)(0.5 * depth * (1 + (k22 - k11) / (scale + 1e-30)));
        Asum += PHet * nRef;
        Bsum += PHet * depth;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { Asum += __shfl_xor(Asum, o, 64); Bsum += __shfl_xor(Bsum, o, 64); }
    if (lane == 0) A.res[site].ab = (0.05 + Asum) / (0.1 + Bsum);
  }
}

// Written records -> genotype rows, in site order, as a two-pass multi-block scan over 1024-site blocks
// (the single-block loop it replaces read the 240-B results at a 240-B stride, 64 sequential rounds per
// 65 536 sites).  Rows exist only for written records: an OutputVCF_denovo call that returns before the
// record (emit 2, NucFamGenotypeLikelihood.cpp:1868) has no observable genotype output.
__device__ __forceinline__ int block_excl_scan_1024(int e, int* s_w, int& total) {
  const unsigned long long bal = __ballot(e);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) s_w[wv] = __popcll(bal);
  __syncthreads();
  int off = 0, t = 0;
  for (int w = 0; w < (int)(blockDim.x >> 6); w++) { if (w < wv) off += s_w[w]; t += s_w[w]; }
  total = t;
  return off + __popcll(bal & ((1ull << lane) - 1ull));
}

__global__ void __launch_bounds__(1024) k_rows_count(DevArgs A) {
  __shared__ int s_w[16];
  const int site = blockIdx.x * 1024 + threadIdx.x;
  const int e = (site < A.n && A.res[site].emit == 1) ? 1 : 0;
  int total;
  (void)block_excl_scan_1024(e, s_w, total);
  if (threadIdx.x == 0) A.row_blk[blockIdx.x] = total;
}

__global__ void __launch_bounds__(1024) k_rows(DevArgs A) {
  __shared__ int s_w[16];
  __shared__ int s_base;
  if (threadIdx.x < 64) {   // rows of the blocks before this one
    int b = 0;
    for (int i = threadIdx.x; i < (int)blockIdx.x; i += 64) b += A.row_blk[i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) b += __shfl_xor(b, o, 64);
    if (threadIdx.x == 0) s_base = b;
  }
  const int site = blockIdx.x * 1024 + threadIdx.x;
  const int em = site < A.n ? A.res[site].emit : 0;
  const int e = em == 1 ? 1 : 0;
  if (em == 2) A.res[site].call_row = -1;
  int total;
  const int pre = block_excl_scan_1024(e, s_w, total);   // (its __syncthreads also publishes s_base)
  if (e) { const int row = s_base + pre; A.res[site].call_row = row; A.row_site[row] = site; }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) A.counts[3] = s_base + total;
}

// ------------------------------------------------------------------------------------------------
// synthetic generator: one thread per (site, family)
__global__ void k_synth(DevArgs A, int n, uint64_t seed, uint64_t off, uint8_t* pl, uint32_t* dm, uint8_t* ref) {
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (long long)n * A.n_fam) return;
  const int i = (int)(gid / A.n_fam), f = (int)(gid % A.n_fam);
  int r; double af;
  pm_syn_site(seed, off + (uint64_t)i, &r, &af);
  if (f == 0) ref[i] = (uint8_t)r;
  const int s = A.fam_start[f], cnt = A.fam_start[f + 1] - s;
  uint8_t hap[32];
  if (cnt > 32) return;
  // genotype-planar site block: person s + j, genotype k at pl[i * 10 * np + k * np + s + j]
  pm_syn_family(A.syn, seed, off + (uint64_t)i, r, af, cnt, A.fa_local + s, A.mo_local + s, (uint64_t)s,
                pl + (size_t)i * A.n_person * 10 + s, 1, (size_t)A.n_person, dm + (size_t)i * A.n_person + s, hap);
}

// person-major GLF records [site][person][10] -> genotype-planar site blocks [site][10][person]: thread per
// (site, person); consecutive threads write consecutive bytes of each plane
__global__ void k_to_planar(int n, int np, const uint8_t* __restrict__ src, uint8_t* __restrict__ dst) {
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (long long)n * np) return;
  const long long site = gid / np;
  const int p = (int)(gid - site * np);
  const uint8_t* r = src + (size_t)gid * 10;
  uint8_t* d = dst + (size_t)site * np * 10 + p;
#pragma unroll
  for (int g = 0; g < 10; g++) d[(size_t)g * np] = r[g];
}

// ================================================================================================
// host side
struct pm_engine {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  pm_params par;
  int n_fam = 0, n_person = 0, max_batch = 0;
  int chrom = PM_CHR_AUTO;
  int T = 64, S = 1;
  int grid_brent = 1024;
  bool has_fp = false;
  bool quad = false;       // QUAD lane plan (hoist_quad): every unit a 4-person nuclear family at a multiple-of-4 person
  int quad_full = 0;       // slot rows below this have no empty lane
  int last_n = 0;
  int n_cu = 256;
  bool carry_postprob = false;
  std::vector<int> fam_start_h;
  std::vector<int8_t> sex_h;
  int single_nuclear = 0, max_nuc = 0;
  int max_fam = 0;            // largest family (persons)
  double prior = 0;
  int n_founders = 0, male_founders = 0, female_founders = 0;
  // device buffers
  int *d_fam_start = nullptr, *d_fam_kind = nullptr, *d_fa = nullptr, *d_mo = nullptr;
  int8_t* d_sex = nullptr;
  int4* d_units = nullptr;
  double *d_lktab = nullptr, *d_M = nullptr;
  pm_synth_tables* d_syn = nullptr;
  uint8_t *d_pl = nullptr, *d_ref = nullptr;
  uint8_t* d_stage = nullptr;   // person-major staging block of pm_engine_run (transposed into d_pl)
  uint32_t* d_dm = nullptr;
  pm_site_result* d_res = nullptr;
  pm_geno_call* d_calls = nullptr;
  double *d_raw = nullptr, *d_minv = nullptr, *d_mono = nullptr;
  int* d_evals = nullptr;
  // extended families (Elston-Stewart)
  int n_ext = 0, max_ext = 0, ws_per_lane = 0, grid_post = 0;
  int *d_fam_founders = nullptr, *d_peel_start = nullptr, *d_ext_count = nullptr, *d_ext_fam = nullptr;
  int8_t* d_is_founder = nullptr;
  int2* d_steps = nullptr;
  double *d_T10 = nullptr, *d_T10dn = nullptr, *d_ws = nullptr, *d_tba = nullptr;
  // ES polynomial form (PM_NUM_POLY): per-family layouts and per-step degrees (poly_layout)
  bool es_poly = false;
  int poly_ws = 0, poly_coef = 0, poly_dcap = 0;
  int hoist_tmp = 0, hoist_waves = 4, es_chunk = 0;   // k_es_hoist: step temporaries per wave, waves per block, items per launch
  double* d_es_coef = nullptr;                        // [es_chunk][max_ext][poly_dcap][T] hoisted coefficients
  // the schedule compiler (es_jit.h): per plan (0, 1) and chromosome class, built on first use (0 untried, 1 ok, -1 failed)
  std::vector<int> ext_fam_h, ext_fam1_h, peel_start_h;
  std::vector<int2> steps_h;
  std::vector<int8_t> founder_h;
  std::vector<int> fam_founders_h;
  pmjit::Kernel jit[2][4];
  int jit_state[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
  int* d_jit_slots[2][4] = {{nullptr, nullptr, nullptr, nullptr}, {nullptr, nullptr, nullptr, nullptr}};   // e | sig | p0
  int *d_poly_start = nullptr, *d_poly_lay = nullptr, *d_poly_deg = nullptr;
  int *d_es_pers = nullptr, *d_es_pers1 = nullptr;   // (family << 8 | member) of peeled families: plan 0 / plan 1
  int* d_fam_perm = nullptr;   // families by (kind, size) for k_posterior
  int n_es_pers = 0, n_es_pers1 = 0;
  // vcf_mode on chrX/Y/MT or with a single family: nuclear families go through ES peeling as well
  // (FamilyLikelihoodSeq_VCF.cpp:97-103), so a second lane plan with them in the per-lane ES lists
  bool vcf = false, plan1_ok = false, use_plan1 = false;
  int T1 = 0, S1 = 0, grid1 = 0, n_ext1 = 0, max_ext1 = 0, has_fp1 = 0;
  int4* d_units1 = nullptr;
  int *d_ext_count1 = nullptr, *d_ext_fam1 = nullptr;
  // --quick_call: the MakeUnrelated() plan (every family an all-founder product) with its own geometry
  int Tq = 0, Sq = 0, grid_q = 0;
  int4* d_units_q = nullptr;
  int* d_items[N_LISTS] = {nullptr, nullptr, nullptr};
  int* d_counts = nullptr;
  unsigned long long* d_eval_total = nullptr;
  unsigned long long* d_phase = nullptr;   // PM_PHASE_TIMING set at engine creation: k_brent hoisting / evaluation wave time
  int wall_khz = 100000;                   // wall_clock64() rate (hipDeviceAttributeWallClockRate)
  int* d_row_site = nullptr;
  int* d_row_blk = nullptr;   // k_rows_count: written records per 1024-site block
  unsigned long long* d_counters = nullptr;
  double M_h[100];
  // stats
  pm_kernel_stats stats{};
  std::vector<std::pair<hipEvent_t, hipEvent_t>> brent_events;
};

static void geno_mut_matrix(double mu, double tstv, double* out) {   // src/MutationModel.cpp:15-90
  double A[4][4];
  for (int i = 0; i < 4; i++) for (int j = 0; j < 4; j++) A[i][j] = (i == j) ? 1 - mu : (1 - mu) / 3;
  if (tstv != 0.0) {
    A[0][2] = A[2][0] = A[1][3] = A[3][1] = mu / 3 * (3 - 3 / (1 + tstv));
    A[0][1] = A[0][3] = A[1][0] = A[1][2] = A[2][1] = A[2][3] = A[3][0] = A[3][2] = mu / 3 * (0.5 / (1 + tstv) * 3);
  }
  double R[16][16];
  int from = -1;
  for (int i = 0; i < 4; i++) for (int j = 0; j < 4; j++) {
    from++; int to = -1;
    for (int ii = 0; ii < 4; ii++) for (int jj = 0; jj < 4; jj++) { to++; R[from][to] = A[i][ii] * A[j][jj]; }
  }
  static const int h1[6] = {2, 3, 4, 7, 8, 12}, h2[6] = {5, 9, 13, 10, 14, 15};
  for (int i = 0; i < 6; i++) for (int j = 0; j < 16; j++) R[j][h1[i] - 1] += R[j][h2[i] - 1];
  static const int un[10] = {1, 2, 3, 4, 6, 7, 8, 11, 12, 16};
  for (int i = 0; i < 10; i++) for (int j = 0; j < 10; j++) out[i * 10 + j] = R[un[i] - 1][un[j] - 1];
}

template <typename X>
static int dalloc(X** p, size_t count) {
  if (count == 0) count = 1;
  hipError_t e = hipMalloc((void**)p, count * sizeof(X));
  if (e != hipSuccess) {
    char b[256]; snprintf(b, sizeof(b), "hipMalloc(%zu bytes) failed: %s", count * sizeof(X), hipGetErrorString(e));
    pm_set_last_error(b);
    return PM_ENOMEM;
  }
  return PM_OK;
}
#define DALLOC(p, n) do { int _r = dalloc(&(p), (n)); if (_r) { pm_engine_destroy(E); return _r; } } while (0)

static const struct { int T, S; } kVariants[] = {{64, 1}, {64, 2}, {64, 4}, {128, 4}, {128, 16}, {256, 1}, {256, 4}, {512, 2}, {512, 4},
                                                 {1024, 1}, {1024, 2}, {1024, 4}, {1024, 8}, {128, 8}, {64, 8}, {64, 16}};

// Deal families to lanes: family-major round robin; founders-only families are split into <=3-person chunks
// kept on one lane.  Returns false if the plan does not fit T x S.
// Extended families are not units: they go to per-lane lists (plan_ext).  unrelated = the --quick_call
// MakeUnrelated() view (FamilyLikelihoodSeq.cpp:54-59): every family is an all-founder product.
static bool plan_units(const pm_pedigree* ped, int T, int S, std::vector<int4>& units, bool unrelated = false,
                       bool nuc_es = false) {
  units.assign((size_t)T * S, make_int4(U_NONE, -1, 0, 0));
  std::vector<int> used(T, 0);
  int lane = 0;
  for (int f = 0; f < ped->n_fam; f++) {
    const int p0 = ped->fam_start[f], n = ped->fam_start[f + 1] - p0, kind = unrelated ? PM_FAM_FOUNDERS : ped->fam_kind[f];
    std::vector<int4> us;
    if (kind == PM_FAM_EXTENDED || (nuc_es && kind == PM_FAM_NUCLEAR)) continue;
    if (kind == PM_FAM_NUCLEAR) us.push_back(make_int4(U_NUC, f, p0, n));
    else if (kind == PM_FAM_FOUNDERS) {
      for (int j = 0; j < n; j += 3) {
        int c = std::min(3, n - j), fl = c;
        if (j == 0) fl |= UF_FIRST;
        if (j + 3 >= n) fl |= UF_LAST;
        us.push_back(make_int4(U_FP, f, p0 + j, fl));
      }
    }
    // choose the lane: next in round-robin order with enough room
    int tries = 0;
    while (used[lane] + (int)us.size() > S && tries < T) { lane = (lane + 1) % T; tries++; }
    if (tries >= T) return false;
    for (auto& u : us) units[(size_t)used[lane]++ * T + lane] = u;
    lane = (lane + 1) % T;
  }
  return true;
}

// pack_steps: es_jit.cpp (pmjit::pack_steps), shared with the schedule compiler.
using pmjit::pack_steps;

// Layout of one family's peel in polynomial form (k_es_hoist / wave_poly_peel): for every chromosome class the degree each
// step combines (founders: 2; 1 for chrX/Y males and chrMT; 0 for chrY females), per slot the coefficient
// capacity (largest degree + 1 over the classes), a temp region, and the likelihood's degree D.  Appends the
// family's layout ints to lay and its steps' degree words to deg; returns the workspace doubles, -1 if a degree
// exceeds the packing (the exact peel is used then).
static int poly_layout(const pm_pedigree* ped, int f, int ns, const int2* st, int nst, std::vector<int>& lay, std::vector<int>& deg) {
  const int p0 = ped->fam_start[f], n = ped->fam_start[f + 1] - p0, nf = ped->fam_founders[f];
  int nkeys = 0;
  for (int s = 0; s < nst; s++)
    if ((st[s].x & 255) == 1) nkeys = std::max(nkeys, ((st[s].y >> 8) & 255) + 1);
  std::vector<int> capP(n, 1), capM(nkeys, 1), Dc(4, 0);
  std::vector<int> dg((size_t)nst * 4, 0);
  int tmp = 1;
  for (int cls = 0; cls < 4; cls++) {
    const bool X = cls == PM_CHR_X, Y = cls == PM_CHR_Y, MT = cls == PM_CHR_MT;
    std::vector<int> dP(n), dM(nkeys, 0);
    for (int i = 0; i < n; i++) {
      const bool fo = ped->is_founder[p0 + i] && i < nf;
      const int sx = ped->sex[p0 + i];
      dP[i] = !fo ? 0 : (Y && sx == FEMALE) ? 0 : (((X || Y) && sx == MALE) || MT) ? 1 : 2;
      capP[i] = std::max(capP[i], dP[i] + 1);
    }
    for (int s = 0; s < nst; s++) {
      const int type = st[s].x & 255, from0 = (st[s].x >> 8) & 255, from1 = (st[s].x >> 16) & 255, to0 = (st[s].x >> 24) & 255;
      const int slot = (st[s].y >> 8) & 255, create = (st[s].y >> 16) & 1;
      int a = 0, b = 0, c = 0, e = 0;
      if (type == 1) {
        a = dP[from0]; b = create ? 0 : dM[slot];
        dM[slot] = a + b;
        capM[slot] = std::max(capM[slot], dM[slot] + 1);
        tmp = std::max(tmp, a + 1);
      } else if (type == 2) {
        a = dP[from0]; b = slot == 255 ? 0 : dM[slot]; c = dP[to0];
        dP[to0] = a + b + c;
        capP[to0] = std::max(capP[to0], dP[to0] + 1);
        tmp = std::max(tmp, a + b + 1);
      } else {
        a = dP[from0]; b = slot == 255 ? 0 : dM[slot]; c = dP[from1]; e = dP[to0];
        dP[to0] = a + b + c + e;
        capP[to0] = std::max(capP[to0], dP[to0] + 1);
        tmp = std::max(tmp, (ns + 1) * (a + b + c + 1));
      }
      if (std::max({a, b, c, e, a + b + c + e}) > 120) return -1;
      dg[(size_t)s * 4 + cls] = a | (b << 7) | (c << 14) | (e << 21);
    }
    Dc[cls] = dP[(st[nst - 1].x >> 24) & 255];
  }
  const size_t base = lay.size();
  lay.push_back(nkeys);
  lay.push_back(0);   // temp offset, below
  for (int c = 0; c < 4; c++) lay.push_back(Dc[c]);
  int off = 0;
  for (int i = 0; i < n; i++) { if (capP[i] > 127) return -1; lay.push_back(off | (capP[i] << 24)); off += ns * capP[i]; }
  for (int m = 0; m < nkeys; m++) { if (capM[m] > 127) return -1; lay.push_back(off | (capM[m] << 24)); off += ns * ns * capM[m]; }
  lay[base + 1] = off;
  off += tmp;
  if (off >= (1 << 24)) return -1;
  deg.insert(deg.end(), dg.begin(), dg.end());
  return off;
}

static int gi_h(int b1, int b2) { return b1 < b2 ? (b1 - 1) * (10 - b1) / 2 + (b2 - b1) : (b2 - 1) * (10 - b2) / 2 + (b1 - b2); }

// FamilyLikelihoodES::SetTransmissionMatrix (:752-785) and SetTransmissionMatrix_denovo (:787-810)
static void transmission_tables(const double* M, std::vector<double>& T10, std::vector<double>& T10dn) {
  T10.assign(1000, 0.0);
  T10dn.assign(1000, 0.0);
  for (int i = 1; i <= 4; i++)
    for (int j = i; j <= 4; j++) {
      const int x = gi_h(i, j);
      for (int k = 1; k <= 4; k++)
        for (int m = k; m <= 4; m++) {
          const int y = gi_h(k, m), g[4] = {gi_h(i, k), gi_h(i, m), gi_h(j, k), gi_h(j, m)};
          for (int t = 0; t < 4; t++) T10[(x * 10 + y) * 10 + g[t]] += 0.25;
        }
    }
  for (int i = 0; i < 10; i++)
    for (int j = 0; j < 10; j++)
      for (int k = 0; k < 10; k++) {
        double s = .0;
        for (int m = 0; m < 10; m++) s += T10[(i * 10 + j) * 10 + m] * M[m * 10 + k];
        T10dn[(i * 10 + j) * 10 + k] = s;
      }
}

// SetTransmissionMatrix_BA, _CHRX_2Female, _CHRX_2Male, _CHRY, _MITO (:812-924), [parent1][parent2][child]
static const double kTBA[5][27] = {
    {1, 0, 0, .5, .5, 0, 0, 1, 0, .5, .5, 0, .25, .5, .25, 0, .5, .5, 0, 1, 0, 0, .5, .5, 0, 0, 1},
    {1, 0, 0, .5, .5, 0, 0, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 0, 0, .5, .5, 0, 0, 1},
    {1, 0, 0, .5, 0, .5, 0, 0, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 0, 0, .5, 0, .5, 0, 0, 1},
    {1, 0, 0, 1, 0, 0, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 0, 0, 1, 0, 0, 1},
    {1, 0, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 0, 0, 0, 0, 1}};

extern "C" {

void pm_engine_destroy(pm_engine* E) {
  if (!E) return;
  hipSetDevice(E->device);
  void* bufs[] = {E->d_units1, E->d_ext_count1, E->d_ext_fam1, E->d_fam_founders, E->d_peel_start, E->d_ext_count, E->d_ext_fam, E->d_is_founder, E->d_steps, E->d_T10,
                  E->d_T10dn, E->d_ws, E->d_tba, E->d_units_q, E->d_poly_start, E->d_poly_lay, E->d_poly_deg, E->d_es_coef, E->d_es_pers, E->d_es_pers1, E->d_fam_perm,
                  E->d_fam_start, E->d_fam_kind, E->d_fa, E->d_mo, E->d_sex, E->d_units, E->d_lktab, E->d_M, E->d_syn,
                  E->d_pl, E->d_stage, E->d_ref, E->d_dm, E->d_res, E->d_calls, E->d_raw, E->d_minv, E->d_mono, E->d_evals,
                  E->d_items[0], E->d_items[1], E->d_items[2], E->d_counts, E->d_eval_total, E->d_row_site,
                  E->d_counters, E->d_row_blk};
  for (void* b : bufs) if (b) hipFree(b);
  for (auto& pl : E->d_jit_slots)
    for (int* b : pl) if (b) hipFree(b);
  for (auto& pr : E->brent_events) { hipEventDestroy(pr.first); hipEventDestroy(pr.second); }
  if (E->ev0) hipEventDestroy(E->ev0);
  if (E->ev1) hipEventDestroy(E->ev1);
  if (E->stream) hipStreamDestroy(E->stream);
  delete E;
}

int pm_engine_create(const pm_pedigree* ped, const pm_params* par, int device, int max_batch, pm_engine** out) {
  if (!ped || !par || !out || ped->n_fam <= 0 || ped->n_person <= 0 || max_batch <= 0) {
    pm_set_last_error("pm_engine_create: invalid arguments");
    return PM_EINVAL;
  }
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
    pm_set_last_error("pm_engine_create: no HIP device available (the engine has no CPU fallback)");
    return PM_EHIP;
  }
  if (device < 0 || device >= ndev) { pm_set_last_error("pm_engine_create: device index out of range"); return PM_EINVAL; }
  if (par->numerics < PM_NUM_PRODUCT || par->numerics > PM_NUM_POLY) {
    pm_set_last_error("pm_engine_create: unknown numerics mode");
    return PM_EINVAL;
  }
  pm_engine* E = new pm_engine;
  E->device = device;
  E->par = *par;
  E->vcf = par->vcf_mode != 0;
  if (E->vcf) { E->par.denovo = 0; E->par.quick_call = 0; }   // the VCF path has neither (PedVCF.cpp)
  par = &E->par;
  E->n_fam = ped->n_fam;
  E->n_person = ped->n_person;
  E->max_batch = max_batch;
  E->n_founders = ped->n_founders; E->male_founders = ped->male_founders; E->female_founders = ped->female_founders;
  // a lone nuclear family is evaluated once at 0.5 (FamilyLikelihoodSeq.cpp:91-104); the VCF path always runs Brent
  E->single_nuclear = (!E->vcf && ped->n_fam == 1 && ped->fam_kind[0] == PM_FAM_NUCLEAR) ? 1 : 0;
  for (int f = 0; f < ped->n_fam; f++) {
    if (ped->fam_kind[f] == PM_FAM_NUCLEAR) E->max_nuc = std::max(E->max_nuc, ped->fam_start[f + 1] - ped->fam_start[f]);
    E->max_fam = std::max(E->max_fam, ped->fam_start[f + 1] - ped->fam_start[f]);
  }
  for (int f = 0; f < ped->n_fam; f++) {
    if (ped->fam_kind[f] != PM_FAM_NUCLEAR) E->has_fp = true;
    if (ped->fam_kind[f] == PM_FAM_EXTENDED) E->n_ext++;
  }
  E->fam_start_h.assign(ped->fam_start, ped->fam_start + ped->n_fam + 1);
  E->sex_h.assign(ped->sex, ped->sex + ped->n_person);
  HIP_TRY(hipSetDevice(device));
  HIP_TRY(hipStreamCreateWithFlags(&E->stream, hipStreamNonBlocking));
  HIP_TRY(hipEventCreate(&E->ev0));
  HIP_TRY(hipEventCreate(&E->ev1));
  // plan
  std::vector<int4> units;
  bool planned = false;
  // optional override for geometry experiments: PM_BRENT_TS="T,S"
  if (const char* ov = getenv("PM_BRENT_TS")) {
    int t = 0, sl = 0;
    if (sscanf(ov, "%d,%d", &t, &sl) == 2)
      for (auto v : kVariants)
        if (v.T == t && v.S == sl && plan_units(ped, t, sl, units)) { E->T = t; E->S = sl; planned = true; }
  }
  // default: the first geometry (in preference order) that holds every family.  One wave per item
  // (T=64, no barrier) wins while its slots fit the register file without scratch: up to S=16 for the
  // lean autosomal kernel, S=8 for the generic one (de novo / founders-only units); beyond that the item
  // is spread over 2-8 waves (one barrier per evaluation).  Sections on chrX/Y/MT run the generic
  // kernel on the same plan.
  {
    const bool gen = (par->denovo && par->numerics != PM_NUM_POLY) || E->has_fp || ped->n_fam == 1;
    // (1025-2048 families: 2 waves x 16 slots, one two-wave exchange per evaluation, before 8 waves x 4)
    static const int2 lean[] = {{64, 1}, {64, 2}, {64, 4}, {64, 8}, {64, 16}, {128, 16}, {1024, 4}, {1024, 8}};
    static const int2 generic[] = {{64, 1}, {64, 2}, {64, 4}, {64, 8}, {256, 1}, {256, 4}, {512, 4}, {1024, 4}, {1024, 8}};
    // lean --denovo: the de novo hoisting state does not fit 16 slots per lane without spilling; 8 slots on
    // 2 waves per item is faster (measured: 6.6 vs 6.1 M sites/s, 1000 quads)
    static const int2 lean_dn[] = {{64, 1}, {64, 2}, {64, 4}, {64, 8}, {128, 8}, {512, 4}, {1024, 4}, {1024, 8}};
    const bool dn_lean = !gen && par->denovo;
    // ... unless the PL bytes can be staged through LDS (16-B aligned planes): then the 64 x 16 kernel with
    // LDS-staged hoisting only has no spills and beats 2 waves x 8 slots (11.9 vs 9.8 M sites/s, 1000 quads)
    static const int2 lean_dn_pf[] = {{64, 1}, {64, 2}, {64, 4}, {64, 8}, {64, 16}, {512, 4}, {1024, 4}, {1024, 8}};
    const bool dn_pf = dn_lean && par->numerics == PM_NUM_POLY && E->max_nuc <= 4 && ped->n_person % 16 == 0 &&
                       ped->n_person >= 16 && !getenv("PM_NO_PREFETCH");
    const int2* pref = gen ? generic : dn_lean ? (dn_pf ? lean_dn_pf : lean_dn) : lean;
    // extended families are the expensive terms: spread them one per lane up to 256 lanes
    // (polynomial form: up to PM_EPE families per lane, their coefficients in registers, one wave per item)
    const int per_lane = (par->numerics == PM_NUM_POLY && !par->denovo) ? PM_EPE : 1;   // (10-state hoisting: one per lane)
    int tmin = 1;
    while (tmin < std::min((E->n_ext + per_lane - 1) / per_lane, 256)) tmin *= 2;
    const int npref = gen ? 9 : 8;
    for (int i = 0; i < npref && !planned; i++)
      if (pref[i].x >= tmin && plan_units(ped, pref[i].x, pref[i].y, units)) { E->T = pref[i].x; E->S = pref[i].y; planned = true; }
  }
  if (!planned) { pm_engine_destroy(E); pm_set_last_error("pm_engine_create: pedigree too large for the lane plan"); return PM_EPED; }
  {   // QUAD plan: each nuclear family's four PL bytes of a genotype plane form one aligned dword
    bool q = E->n_person % 16 == 0 && !E->has_fp && E->T == 64;
    int full = E->S;
    for (int sl = 0; sl < E->S && q; sl++)
      for (int l = 0; l < E->T; l++) {
        const int4 u = units[(size_t)sl * E->T + l];
        if (u.x == U_NONE) { full = std::min(full, sl); continue; }
        if (u.x != U_NUC || u.w != 4 || u.z != 4 * (sl * E->T + l)) { q = false; break; }
      }
    E->quad = q && !getenv("PM_NO_QUAD");
    E->quad_full = full;
  }
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device));
  const int blocksPerCU = std::max(1, 1024 / E->T);   // ~16 waves per CU
  E->n_cu = prop.multiProcessorCount;
  E->grid_brent = prop.multiProcessorCount * blocksPerCU;
  // tables
  double lk[256];
  for (int i = 0; i <= 255; i++) lk[i] = pow(0.1, i * 0.1);   // core/BaseQualityHelper.cpp:13 (host glibc)
  if (E->vcf)   // FamilyLikelihoodSeq_VCF::PL2LK_table (src/FamilyLikelihoodSeq_VCF.cpp:21-22)
    for (int i = 0; i <= 255; i++) lk[i] = pow(10, -double(i) / 10.0);
  geno_mut_matrix(par->denovo_mut_rate, par->denovo_tstv, E->M_h);
  static pm_synth_tables syn;
  pm_synth_build_tables(&syn);
  std::vector<int32_t> fa(ped->n_person, -1), mo(ped->n_person, -1);
  if (ped->father && ped->mother)
    for (int f = 0; f < ped->n_fam; f++)
      for (int j = ped->fam_start[f]; j < ped->fam_start[f + 1]; j++) {
        fa[j] = ped->father[j] < 0 ? -1 : ped->father[j] - ped->fam_start[f];
        mo[j] = ped->mother[j] < 0 ? -1 : ped->mother[j] - ped->fam_start[f];
      }
  DALLOC(E->d_fam_start, ped->n_fam + 1);
  DALLOC(E->d_fam_kind, ped->n_fam);
  DALLOC(E->d_fa, ped->n_person);
  DALLOC(E->d_mo, ped->n_person);
  DALLOC(E->d_sex, ped->n_person);
  DALLOC(E->d_units, units.size());
  DALLOC(E->d_lktab, 256);
  DALLOC(E->d_M, 100);
  DALLOC(E->d_syn, 1);
  HIP_TRY(hipMemcpy(E->d_fam_start, ped->fam_start, sizeof(int) * (ped->n_fam + 1), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(E->d_fam_kind, ped->fam_kind, sizeof(int) * ped->n_fam, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(E->d_fa, fa.data(), sizeof(int) * ped->n_person, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(E->d_mo, mo.data(), sizeof(int) * ped->n_person, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(E->d_sex, ped->sex, ped->n_person, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(E->d_units, units.data(), sizeof(int4) * units.size(), hipMemcpyHostToDevice));
  {   // k_posterior's family order: by kind, then size (mixed trio / quad pedigrees: no divergent family-size paths)
    std::vector<int> perm(ped->n_fam);
    for (int f = 0; f < ped->n_fam; f++) perm[f] = f;
    std::stable_sort(perm.begin(), perm.end(), [&](int a, int b) {
      const int na = ped->fam_start[a + 1] - ped->fam_start[a], nb = ped->fam_start[b + 1] - ped->fam_start[b];
      return ped->fam_kind[a] != ped->fam_kind[b] ? ped->fam_kind[a] < ped->fam_kind[b] : na < nb;
    });
    DALLOC(E->d_fam_perm, ped->n_fam);
    HIP_TRY(hipMemcpy(E->d_fam_perm, perm.data(), sizeof(int) * ped->n_fam, hipMemcpyHostToDevice));
  }
  HIP_TRY(hipMemcpy(E->d_lktab, lk, sizeof(lk), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(E->d_M, E->M_h, sizeof(E->M_h), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(E->d_syn, &syn, sizeof(syn), hipMemcpyHostToDevice));
  // --- Elston-Stewart data: packed schedules, per-lane family lists, transmission tables, workspace
  {
    const int ns = par->denovo ? 10 : 3;
    std::vector<int> peel_start(ped->n_fam + 1, 0);
    std::vector<int2> steps;
    std::vector<int> founders(ped->fam_founders, ped->fam_founders + ped->n_fam);
    int wsmax = 0;
    E->plan1_ok = E->vcf;
    for (int f = 0; f < ped->n_fam; f++) {
      peel_start[f] = (int)steps.size();
      const int kind = ped->fam_kind[f];
      if (kind == PM_FAM_FOUNDERS || (kind == PM_FAM_NUCLEAR && !E->vcf)) continue;
      const size_t mark = steps.size();
      const int w = pack_steps(ped, f, ns, steps);
      if (w < 0 && kind == PM_FAM_EXTENDED) {
        pm_engine_destroy(E);
        pm_set_last_error("pm_engine_create: extended family without a usable peeling schedule (or > 255 members)");
        return PM_EPED;
      }
      if (w < 0) { steps.resize(mark); E->plan1_ok = false; continue; }   // nuclear without a schedule: no plan 1
      wsmax = std::max(wsmax, w);
    }
    peel_start[ped->n_fam] = (int)steps.size();
    E->ws_per_lane = wsmax;
    // polynomial-form layouts (PM_NUM_POLY): every family with a schedule.  Under --denovo the 10-state layout
    // also serves the BA (cfg-7) items: the degrees do not depend on the state count, the slots are larger.
    std::vector<int> poly_start(ped->n_fam + 1, 0), poly_lay, poly_deg((size_t)steps.size() * 4, 0);
    int poly_w = 0, poly_d = 0;
    E->es_poly = par->numerics == PM_NUM_POLY && !steps.empty();
    for (int f = 0; f < ped->n_fam && E->es_poly; f++) {
      poly_start[f] = (int)poly_lay.size();
      const int ns0 = peel_start[f], ns1 = peel_start[f + 1];
      if (ns1 == ns0) continue;
      std::vector<int> dg;
      const int w = poly_layout(ped, f, par->denovo ? 10 : 3, steps.data() + ns0, ns1 - ns0, poly_lay, dg);
      if (w < 0) { E->es_poly = false; break; }
      std::copy(dg.begin(), dg.end(), poly_deg.begin() + (size_t)ns0 * 4);
      poly_w = std::max(poly_w, w);
      for (int c = 0; c < 4; c++) poly_d = std::max(poly_d, poly_lay[poly_start[f] + 2 + c]);
    }
    poly_start[ped->n_fam] = (int)poly_lay.size();
    if (E->es_poly) {   // k_es_hoist temporaries: the largest step's out-of-place phases (wave_poly_peel)
      const int ns = par->denovo ? 10 : 3;
      for (size_t s = 0; s < steps.size(); s++)
        for (int cls = 0; cls < 4; cls++) {
          const int dg = poly_deg[s * 4 + cls], type = steps[s].x & 255;
          const int a = dg & 127, b = (dg >> 7) & 127, c = (dg >> 14) & 127, e = (dg >> 21) & 127;
          int need;
          if (type == 1) need = ns * ns * (a + 1) + ns * ns * (a + b + 1);
          else if (type == 2) need = ns * (a + b + 1) + ns * (a + b + c + 1);
          else need = ns * ns * (a + b + c + 1) + ns * (a + b + c + 1) + ns * (a + b + c + e + 1);
          E->hoist_tmp = std::max(E->hoist_tmp, need);
        }
      // 4 waves per block when their LDS slices fit, else fewer; none: the reference-order peel per evaluation
      const size_t stat = (256 + 5 * 27 + (par->denovo ? 2000 : 2)) * sizeof(double);
      const size_t per_wave = (size_t)(poly_w + E->hoist_tmp) * sizeof(double);
      E->hoist_waves = 0;
      for (int w = 4; w >= 1 && !E->hoist_waves; w--)
        if (stat + per_wave * w <= 150 * 1024) E->hoist_waves = w;
      if (!E->hoist_waves) E->es_poly = false;
    }
    const int T = E->T;
    E->max_ext = (E->n_ext + T - 1) / T;
    std::vector<int> ext_count(T, 0), ext_fam((size_t)std::max(1, E->max_ext) * T, -1);
    int q = 0;
    for (int f = 0; f < ped->n_fam; f++)
      if (ped->fam_kind[f] == PM_FAM_EXTENDED) { const int lane = q % T; ext_fam[(size_t)ext_count[lane]++ * T + lane] = f; q++; }
    {   // persons of the peeled families, for k_posterior_es: plan 0 (extended) and plan 1 (every family with offspring)
      std::vector<int> e0, e1;
      for (int f = 0; f < ped->n_fam; f++) {
        const int n = ped->fam_start[f + 1] - ped->fam_start[f];
        for (int j = 0; j < n && n <= 255; j++) {
          if (ped->fam_kind[f] == PM_FAM_EXTENDED) e0.push_back(f << 8 | j);
          if (ped->fam_kind[f] != PM_FAM_FOUNDERS) e1.push_back(f << 8 | j);
        }
      }
      E->n_es_pers = (int)e0.size();
      E->n_es_pers1 = (int)e1.size();
      DALLOC(E->d_es_pers, std::max<size_t>(1, e0.size()));
      DALLOC(E->d_es_pers1, std::max<size_t>(1, e1.size()));
      if (!e0.empty()) HIP_TRY(hipMemcpy(E->d_es_pers, e0.data(), sizeof(int) * e0.size(), hipMemcpyHostToDevice));
      if (!e1.empty()) HIP_TRY(hipMemcpy(E->d_es_pers1, e1.data(), sizeof(int) * e1.size(), hipMemcpyHostToDevice));
    }
    std::vector<double> T10, T10dn;
    transmission_tables(E->M_h, T10, T10dn);
    DALLOC(E->d_fam_founders, ped->n_fam);
    DALLOC(E->d_is_founder, ped->n_person);
    DALLOC(E->d_peel_start, ped->n_fam + 1);
    DALLOC(E->d_steps, std::max<size_t>(1, steps.size()));
    E->ext_fam_h = ext_fam;
    E->peel_start_h = peel_start;
    E->steps_h = steps;
    E->founder_h.assign(ped->is_founder, ped->is_founder + ped->n_person);
    E->fam_founders_h = founders;
    DALLOC(E->d_ext_count, T);
    DALLOC(E->d_ext_fam, ext_fam.size());
    DALLOC(E->d_T10, 1000);
    DALLOC(E->d_T10dn, 1000);
    HIP_TRY(hipMemcpy(E->d_fam_founders, founders.data(), sizeof(int) * ped->n_fam, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(E->d_is_founder, ped->is_founder, ped->n_person, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(E->d_peel_start, peel_start.data(), sizeof(int) * peel_start.size(), hipMemcpyHostToDevice));
    if (!steps.empty()) HIP_TRY(hipMemcpy(E->d_steps, steps.data(), sizeof(int2) * steps.size(), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(E->d_ext_count, ext_count.data(), sizeof(int) * T, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(E->d_ext_fam, ext_fam.data(), sizeof(int) * ext_fam.size(), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(E->d_T10, T10.data(), sizeof(double) * 1000, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(E->d_T10dn, T10dn.data(), sizeof(double) * 1000, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(c_TBA), kTBA, sizeof(kTBA)));
    DALLOC(E->d_tba, 5 * 27);
    HIP_TRY(hipMemcpy(E->d_tba, kTBA, sizeof(kTBA), hipMemcpyHostToDevice));
    {   // GQ thresholds (d_gq): smallest double q in (0, 1] with int(-10 log10(q) + 0.5) <= k, by bisection on the
        // bit patterns of positive doubles (ordered like their values), with the host's glibc log10
      double thr[101];
      auto gq_of = [](double q) { return (int)(-10. * log10(q) + 0.5); };
      for (int k = 0; k <= 100; k++) {
        uint64_t lo = 1, hi = 0x3FF0000000000000ull;   // gq_of(hi = 1.0) = 0 <= k; search the first bit pattern with gq <= k
        while (lo < hi) {
          const uint64_t mid = lo + (hi - lo) / 2;
          double q;
          memcpy(&q, &mid, 8);
          if (gq_of(q) <= k) hi = mid; else lo = mid + 1;
        }
        memcpy(&thr[k], &lo, 8);
      }
      HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(c_gq_thr), thr, sizeof(thr)));
    }
    // vcf_mode plan 1: nuclear families peeled too (chrX/Y/MT sections, or a single family)
    if (E->plan1_ok) {
      int n1 = 0;
      for (int f = 0; f < ped->n_fam; f++) {
        if (ped->fam_kind[f] != PM_FAM_FOUNDERS) n1++;
        else E->has_fp1 = 1;
      }
      int tmin = 1;
      while (tmin < std::min(std::max(n1, 1), 256)) tmin *= 2;
      static const int2 gp[] = {{64, 1}, {64, 2}, {64, 4}, {64, 8}, {256, 4}, {512, 4}, {1024, 4}, {1024, 8}};
      std::vector<int4> u1;
      for (auto g : gp)
        if (g.x >= tmin && plan_units(ped, g.x, g.y, u1, false, true)) { E->T1 = g.x; E->S1 = g.y; break; }
      if (!E->T1) E->plan1_ok = false;
      else {
        E->n_ext1 = n1;
        E->max_ext1 = (n1 + E->T1 - 1) / E->T1;
        std::vector<int> c1(E->T1, 0), e1((size_t)std::max(1, E->max_ext1) * E->T1, -1);
        int q1 = 0;
        for (int f = 0; f < ped->n_fam; f++)
          if (ped->fam_kind[f] != PM_FAM_FOUNDERS) { const int lane = q1 % E->T1; e1[(size_t)c1[lane]++ * E->T1 + lane] = f; q1++; }
        E->ext_fam1_h = e1;
        DALLOC(E->d_units1, u1.size());
        DALLOC(E->d_ext_count1, E->T1);
        DALLOC(E->d_ext_fam1, e1.size());
        HIP_TRY(hipMemcpy(E->d_units1, u1.data(), sizeof(int4) * u1.size(), hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(E->d_ext_count1, c1.data(), sizeof(int) * E->T1, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(E->d_ext_fam1, e1.data(), sizeof(int) * e1.size(), hipMemcpyHostToDevice));
        E->grid1 = E->n_cu * std::max(1, 1024 / E->T1);
      }
    }
    // polynomial form: per lane the peel workspace (reused family by family) and each ES family's D + 1
    // coefficients + D, kept for the item's evaluations
    if (E->es_poly) {
      E->poly_dcap = poly_d + 2;
      E->poly_coef = poly_w;
      E->poly_ws = poly_w + std::max({E->max_ext, E->max_ext1, 1}) * E->poly_dcap;
      DALLOC(E->d_poly_start, poly_start.size());
      DALLOC(E->d_poly_lay, std::max<size_t>(1, poly_lay.size()));
      DALLOC(E->d_poly_deg, std::max<size_t>(1, poly_deg.size()));
      HIP_TRY(hipMemcpy(E->d_poly_start, poly_start.data(), sizeof(int) * poly_start.size(), hipMemcpyHostToDevice));
      if (!poly_lay.empty()) HIP_TRY(hipMemcpy(E->d_poly_lay, poly_lay.data(), sizeof(int) * poly_lay.size(), hipMemcpyHostToDevice));
      if (!poly_deg.empty()) HIP_TRY(hipMemcpy(E->d_poly_deg, poly_deg.data(), sizeof(int) * poly_deg.size(), hipMemcpyHostToDevice));
      // hoisted coefficients of a chunk of items: <= 1 GiB, at most every item a batch can enqueue in one list (4 per site)
      const size_t per_item = (size_t)std::max({E->max_ext * E->T, E->max_ext1 * std::max(1, E->T1), 1}) * E->poly_dcap * sizeof(double);
      E->es_chunk = (int)std::max<size_t>(1, std::min<size_t>((size_t)4 * std::max(1, max_batch), ((size_t)1 << 30) / per_item));
      DALLOC(E->d_es_coef, (size_t)E->es_chunk * per_item / sizeof(double));
    }
    // workspace: the Brent grids and the posterior grid are capped so each needs <= 1 GiB
    E->grid_post = E->n_cu * 8;
    if (wsmax > 0) {
      const size_t cap = (size_t)1 << 30, per_lane = (size_t)wsmax * sizeof(double);
      const size_t per_lane_b = (size_t)wsmax * sizeof(double);   // Brent grids (EP kernels use no workspace: k_es_hoist)
      E->grid_brent = (int)std::max<size_t>(E->n_cu, std::min<size_t>(E->grid_brent, cap / (per_lane_b * T)));
      E->grid_brent -= E->grid_brent % 8;   // keep the XCD-aware item order exact
      if (E->T1) {
        E->grid1 = (int)std::max<size_t>(E->n_cu, std::min<size_t>(E->grid1, cap / (per_lane_b * E->T1)));
        E->grid1 -= E->grid1 % 8;
      }
      E->grid_post = (int)std::max<size_t>(E->n_cu, std::min<size_t>(E->grid_post, cap / (per_lane * 256)));
      const size_t words = std::max({(size_t)E->grid_brent * T * (per_lane_b / sizeof(double)),
                                     (size_t)E->grid1 * E->T1 * (per_lane_b / sizeof(double)), (size_t)E->grid_post * 256 * wsmax});
      DALLOC(E->d_ws, words);
    }
  }
  // --- --quick_call: the unrelated plan (all persons in <=3-person founder chunks)
  if (par->quick_call) {
    static const int2 gq[] = {{64, 1}, {64, 2}, {64, 4}, {64, 8}, {256, 4}, {512, 4}, {1024, 4}, {1024, 8}};
    std::vector<int4> uq;
    for (auto g : gq)
      if (plan_units(ped, g.x, g.y, uq, true)) { E->Tq = g.x; E->Sq = g.y; break; }
    if (!E->Tq) { pm_engine_destroy(E); pm_set_last_error("pm_engine_create: pedigree too large for the --quick_call lane plan"); return PM_EPED; }
    E->grid_q = E->n_cu * std::max(1, 1024 / E->Tq);
    DALLOC(E->d_units_q, uq.size());
    HIP_TRY(hipMemcpy(E->d_units_q, uq.data(), sizeof(int4) * uq.size(), hipMemcpyHostToDevice));
  }
  // batch buffers
  const size_t nb = (size_t)max_batch, np = (size_t)ped->n_person;
  DALLOC(E->d_pl, nb * np * 10);
  DALLOC(E->d_stage, nb * np * 10);
  DALLOC(E->d_dm, nb * np);
  DALLOC(E->d_ref, nb);
  DALLOC(E->d_res, nb);
  DALLOC(E->d_calls, nb * np);
  DALLOC(E->d_raw, nb * 8);
  DALLOC(E->d_minv, nb * 8);
  DALLOC(E->d_evals, nb * 8);
  DALLOC(E->d_mono, nb);
  for (int l = 0; l < N_LISTS; l++) DALLOC(E->d_items[l], nb * 4);
  DALLOC(E->d_counts, 16);
  DALLOC(E->d_eval_total, 1);
  DALLOC(E->d_row_site, nb);
  DALLOC(E->d_row_blk, nb / 1024 + 2);
  DALLOC(E->d_counters, 16);
  HIP_TRY(hipMemset(E->d_counters, 0, 16 * sizeof(unsigned long long)));
  HIP_TRY(hipMemset(E->d_eval_total, 0, sizeof(unsigned long long)));
  if (getenv("PM_PHASE_TIMING")) {
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) == hipSuccess && khz > 0) E->wall_khz = khz;
    DALLOC(E->d_phase, 3);
    HIP_TRY(hipMemset(E->d_phase, 0, 3 * sizeof(unsigned long long)));
  }
  int rc = pm_engine_begin_section(E, PM_CHR_AUTO);
  if (rc) { pm_engine_destroy(E); return rc; }
  *out = E;
  return PM_OK;
}

int pm_engine_plan(pm_engine* E, int32_t* threads, int32_t* slots) {
  if (!E || !threads || !slots) { pm_set_last_error("pm_engine_plan: invalid arguments"); return PM_EINVAL; }
  *threads = E->T;
  *slots = E->S;
  return PM_OK;
}

int pm_engine_set_posterior_carry(pm_engine* E, int32_t seen) {
  if (!E) { pm_set_last_error("pm_engine_set_posterior_carry: invalid arguments"); return PM_EINVAL; }
  E->carry_postprob = seen != 0;
  return PM_OK;
}

int pm_engine_begin_section(pm_engine* E, int32_t chrom) {
  if (!E || chrom < 0 || chrom > 3) { pm_set_last_error("pm_engine_begin_section: invalid arguments"); return PM_EINVAL; }
  E->chrom = chrom;
  E->use_plan1 = E->vcf && (chrom != PM_CHR_AUTO || E->n_fam == 1);
  if (E->use_plan1 && !E->plan1_ok) {
    pm_set_last_error("pm_engine_begin_section: vcf_mode on chrX/Y/MT (or with a single family) needs a peeling schedule "
                      "for every nuclear family (pm_pedigree.steps)");
    return PM_EPED;
  }
  // GetPolyPrior (NucFamGenotypeLikelihood.cpp:231-304)
  int n;
  if (chrom == PM_CHR_X) n = E->female_founders * 2 + E->male_founders;
  else if (chrom == PM_CHR_Y) n = E->male_founders;
  else if (chrom == PM_CHR_MT) n = E->n_founders;
  else n = 2 * E->n_founders;
  double p = 0;
  for (int i = 1; i <= n; i++) p += 1.0 / i;
  E->prior = p * E->par.theta;
  HIP_TRY(hipSetDevice(E->device));
  HIP_TRY(hipMemsetAsync(E->d_counters, 0, 16 * sizeof(unsigned long long), E->stream));
  HIP_TRY(hipStreamSynchronize(E->stream));
  return PM_OK;
}

// lean autosomal --denovo (POLY numerics, nuclear families only, no quick pre-filter): k_prep evaluates
// the cfg-0 de novo monomorphism item itself instead of enqueueing it for k_brent
static bool mono_dn_in_prep(const pm_engine* E) {
  return E->par.denovo && E->par.numerics == PM_NUM_POLY && !E->par.quick_call && !E->vcf && E->chrom == PM_CHR_AUTO &&
         !E->has_fp && E->n_ext == 0 && E->n_fam > 1;
}

static DevArgs make_args(pm_engine* E, int n, const uint8_t* pl, const uint32_t* dm, const uint8_t* ref, pm_site_result* res,
                         pm_geno_call* calls) {
  DevArgs A;
  memset(&A, 0, sizeof(A));
  A.n_fam = E->n_fam; A.n_person = E->n_person; A.n_fam_gt1 = E->n_fam > 1; A.single_nuclear = E->single_nuclear;
  A.max_nuc = E->max_nuc;
  A.chrom = E->chrom; A.denovo = E->par.denovo;
  A.fam_start = E->d_fam_start; A.fam_kind = E->d_fam_kind; A.sex = E->d_sex; A.fa_local = E->d_fa; A.mo_local = E->d_mo;
  A.units = E->d_units; A.T = E->T; A.S = E->S;
  A.fam_founders = E->d_fam_founders; A.is_founder = E->d_is_founder; A.peel_start = E->d_peel_start; A.steps = E->d_steps;
  A.ext_count = E->n_ext ? E->d_ext_count : nullptr; A.ext_fam = E->d_ext_fam;
  A.T10 = E->d_T10; A.T10dn = E->d_T10dn; A.ws = E->d_ws; A.ws_per_lane = E->ws_per_lane;
  A.es_poly = 0;   // set per Brent launch (launch_brent)
  A.poly_start = E->d_poly_start; A.poly_lay = E->d_poly_lay; A.poly_deg = E->d_poly_deg;
  A.poly_coef = E->poly_coef; A.poly_dcap = E->poly_dcap;
  A.es_coef = E->d_es_coef; A.es_it0 = 0; A.es_it1 = INT_MAX; A.max_ext = E->use_plan1 ? E->max_ext1 : E->max_ext;
  A.hoist_ws = E->poly_coef; A.hoist_tmp = E->hoist_tmp;
  A.es_pers = E->use_plan1 ? E->d_es_pers1 : E->d_es_pers;
  A.fam_perm = E->d_fam_perm;
  A.n_es_pers = E->use_plan1 ? E->n_es_pers1 : E->n_es_pers;
  A.theta_one = 1.0;
  A.unrelated = E->par.quick_call ? 1 : 0;   // k_prep: route sites through the quick pre-filter first
  A.vcf = E->vcf ? 1 : 0;
  if (E->use_plan1) {
    A.units = E->d_units1; A.T = E->T1; A.S = E->S1;
    A.ext_count = E->n_ext1 ? E->d_ext_count1 : nullptr; A.ext_fam = E->d_ext_fam1; A.nuc_es = 1;
  }
  A.lktab = E->d_lktab; A.M = E->d_M; A.syn = E->d_syn;
  memcpy(A.Mk, E->M_h, sizeof(A.Mk));
  A.precision = E->par.precision; A.posterior = E->par.posterior; A.theta = E->par.theta;
  A.min_total_depth = E->par.min_total_depth; A.max_total_depth = E->par.max_total_depth; A.min_map_quality = E->par.min_map_quality;
  A.min_ps = E->par.min_ps; A.denovo_min_llr = E->par.denovo_min_llr; A.log10_denovo_min_llr = log10(E->par.denovo_min_llr);
  A.force_call = E->par.force_call; A.all_sites = E->par.all_sites;
  const double pts = E->par.poly_tstv / (E->par.poly_tstv + 1), ptv = (1 - pts) / 2, prior = E->prior;
  A.lp_mono = log10(1 - prior);                  // main.cpp:450
  A.lp_ts = log10(prior * pts);                  // :469
  A.lp_tv = log10(prior * ptv);                  // :479, :489
  A.lp_other = log10(prior * 0.001);             // :509-529
  A.np_ts = log10(prior * 2. / 3.);              // :472
  A.np_tv = log10(prior * 1. / 6.);              // :482, :492
  A.n = n; A.pl = pl; A.dm = dm; A.ref = ref; A.res = res; A.calls = calls;
  A.raw = E->d_raw; A.minv = E->d_minv; A.evals = E->d_evals; A.mono_plain = E->d_mono;
  for (int l = 0; l < N_LISTS; l++) A.items[l] = E->d_items[l];
  A.counts = E->d_counts; A.eval_total = E->d_eval_total; A.phase = E->d_phase; A.row_site = E->d_row_site; A.row_blk = E->d_row_blk; A.counters = E->d_counters;
  A.carry_postprob = E->carry_postprob ? 1 : 0;
  A.mono_dn = mono_dn_in_prep(E) ? 1 : 0;
  return A;
}

typedef void (*BrentFn)(DevArgs, int);
// numerics: PM_NUM_PRODUCT / PM_NUM_EXACT for every flavour; PM_NUM_POLY only for the lean kernel
// (the generic and ES flavours fall back to PRODUCT numerics).
static BrentFn brent_kernel(int T, int S, int num, bool gen, bool es, bool dn = false, bool pf = false, bool ep = false) {
  const int n = (num == PM_NUM_POLY && gen) ? PM_NUM_PRODUCT : num;
  if (es && ep) {   // extended families in polynomial form (PM_NUM_POLY); DN: with the 10-state (--denovo) hoisting
#define PMKEP(t, s) \
  if (T == t && S == s) return dn ? k_brent<t, s, PM_NUM_PRODUCT, true, true, true, false, true> : k_brent<t, s, PM_NUM_PRODUCT, true, true, false, false, true>;
    PMKEP(64, 1) PMKEP(64, 2) PMKEP(64, 4) PMKEP(64, 8) PMKEP(256, 1) PMKEP(256, 4) PMKEP(512, 4) PMKEP(1024, 4) PMKEP(1024, 8)
#undef PMKEP
    return nullptr;
  }
  if (dn && !gen && !es && n == PM_NUM_POLY && pf && T == 64 && S == 16)   // lean --denovo, LDS-staged hoisting only
    return k_brent<64, 16, PM_NUM_POLY, false, false, true, true>;
  if (pf && !dn) {   // lean autosomal kernel with LDS plane prefetch
#define PMKP(s) if (T == 64 && S == s) return k_brent<64, s, PM_NUM_POLY, false, false, false, true>;
    PMKP(1) PMKP(2) PMKP(4) PMKP(8) PMKP(16)
#undef PMKP
    if (T == 128 && S == 16) return k_brent<128, 16, PM_NUM_POLY, false, false, false, true>;   // 1025-2048 families
    return nullptr;
  }
  if (dn && !gen && !es && n == PM_NUM_POLY) {   // lean autosomal --denovo
#define PMKD(t, s) if (T == t && S == s) return k_brent<t, s, PM_NUM_POLY, false, false, true>;
    PMKD(64, 1) PMKD(64, 2) PMKD(64, 4) PMKD(64, 8) PMKD(64, 16) PMKD(128, 8) PMKD(512, 4) PMKD(1024, 4) PMKD(1024, 8)
#undef PMKD
    return nullptr;
  }
#define PMK(t, s)                                                                                             \
  if (T == t && S == s) {                                                                                     \
    if (gen) return n == PM_NUM_EXACT ? k_brent<t, s, PM_NUM_EXACT, true, false> : k_brent<t, s, PM_NUM_PRODUCT, true, false>; \
    return n == PM_NUM_EXACT ? k_brent<t, s, PM_NUM_EXACT, false, false>                                      \
         : n == PM_NUM_POLY ? k_brent<t, s, PM_NUM_POLY, false, false> : k_brent<t, s, PM_NUM_PRODUCT, false, false>; \
  }
#define PMKE(t, s) \
  if (T == t && S == s) return n == PM_NUM_EXACT ? k_brent<t, s, PM_NUM_EXACT, true, true> : k_brent<t, s, PM_NUM_PRODUCT, true, true>;
  if (es) {
    PMKE(64, 1) PMKE(64, 2) PMKE(64, 4) PMKE(64, 8) PMKE(256, 1) PMKE(256, 4) PMKE(512, 4) PMKE(1024, 4) PMKE(1024, 8)
    return nullptr;
  }
  PMK(64, 1) PMK(64, 2) PMK(64, 4) PMK(128, 4) PMK(256, 4) PMK(512, 2) PMK(512, 4) PMK(1024, 1) PMK(1024, 2)
  PMK(1024, 4) PMK(1024, 8) PMK(128, 8) PMK(64, 8) PMK(64, 16) PMK(128, 16)
#undef PMK
#undef PMKE
  return nullptr;
}

// The schedule compiler's kernels for the current plan and chromosome class (es_jit.h), built on first use; nullptr
// when it is off (PM_NO_JIT) or failed to build (then the generic k_es_hoist / k_posterior_es run).
static const pmjit::Kernel* jit_kernel(pm_engine* E) {
  const int plan = E->use_plan1 ? 1 : 0, cls = E->chrom;
  if (!E->es_poly || getenv("PM_NO_JIT")) return nullptr;
  int& st = E->jit_state[plan][cls];
  if (st == 0) {
    st = -1;
    const std::vector<int>& ef = plan ? E->ext_fam1_h : E->ext_fam_h;
    std::vector<pmjit::Family> fams;
    for (size_t e = 0; e < ef.size(); e++) {
      const int f = ef[e];
      if (f < 0) continue;
      pmjit::Family F;
      F.e = (int)e;
      F.p0 = E->fam_start_h[f];
      F.n = E->fam_start_h[f + 1] - F.p0;
      F.nf = E->fam_founders_h[f];
      F.sex.assign(E->sex_h.begin() + F.p0, E->sex_h.begin() + F.p0 + F.n);
      F.founder.assign(E->founder_h.begin() + F.p0, E->founder_h.begin() + F.p0 + F.n);
      F.steps.assign(E->steps_h.begin() + E->peel_start_h[f], E->steps_h.begin() + E->peel_start_h[f + 1]);
      fams.push_back(F);
    }
    std::string err;
    pmjit::Kernel& K = E->jit[plan][cls];
    if (!fams.empty() && pmjit::build(E->device, cls, fams, kTBA, E->par.denovo != 0, &K, &err)) {
      const size_t ns = K.slot_e.size();
      std::vector<int> tab(3 * ns);
      for (size_t i = 0; i < ns; i++) { tab[i] = K.slot_e[i]; tab[ns + i] = K.slot_sig[i]; tab[2 * ns + i] = K.slot_p0[i]; }
      if (dalloc(&E->d_jit_slots[plan][cls], tab.size()) == PM_OK &&
          hipMemcpy(E->d_jit_slots[plan][cls], tab.data(), sizeof(int) * tab.size(), hipMemcpyHostToDevice) == hipSuccess)
        st = 1;
    } else if (!fams.empty())
      fprintf(stderr, "polymutt: peeling-schedule compiler unavailable (%s); using the generic hoisting kernel\n", err.c_str());
  }
  return st == 1 ? &E->jit[plan][cls] : nullptr;
}

static int launch_brent(pm_engine* E, const DevArgs& A0, int list, bool unrelated = false) {
  DevArgs A = A0;
  int T = E->T, S = E->S, grid = E->grid_brent;
  // lean kernel: autosome, no de novo model, nuclear families only (the common case)
  // (with POLY numerics the lean kernel also takes autosomal --denovo: its hoisting has the de novo kid terms)
  bool gen = E->chrom != PM_CHR_AUTO || (E->par.denovo && E->par.numerics != PM_NUM_POLY) || E->has_fp || E->n_fam == 1;
  int n_ext = E->n_ext;
  if (E->use_plan1) { T = E->T1; S = E->S1; grid = E->grid1; gen = true; n_ext = E->n_ext1; }
  if (unrelated) {   // MakeUnrelated(): all-founder products over the quick plan, no ES, no de novo model
    A.units = E->d_units_q; A.T = T = E->Tq; A.S = S = E->Sq; grid = E->grid_q;
    A.ext_count = nullptr; A.unrelated = 1; A.denovo = 0; gen = true;
  } else A.unrelated = 0;
  // lean non-de-novo kernel at one wave per item: LDS-DMA plane prefetch when the planes are 16-B aligned
  size_t shmem = 0;
  A.pf_npad = 0;
  A.pf_dw = 0;
  // (16-B pieces need 16-B aligned planes: n_person % 16 == 0 and a 16-B aligned block; 4-B pieces otherwise; the
  // 128 x 16 plan of 1025-2048 families shares one buffer between its two waves)
  const bool al16 = E->n_person % 16 == 0 && ((uintptr_t)A.pl & 15) == 0, al4 = E->n_person % 4 == 0 && ((uintptr_t)A.pl & 3) == 0;
  if (!gen && !unrelated && n_ext == 0 && !A.denovo && (T == 64 || (T == 128 && S == 16)) && E->par.numerics == PM_NUM_POLY &&
      E->max_nuc <= 4 && (al16 || al4) && E->n_person >= 16 && (E->n_person + 1023) / 1024 * 1024 * 3 <= 60 * 1024 &&
      !getenv("PM_NO_PREFETCH")) {
    A.pf_npad = (E->n_person + 1023) / 1024 * 1024;
    A.pf_dw = al16 ? 0 : 1;
    shmem = (size_t)3 * A.pf_npad;
  }
  // lean --denovo kernel: QUAD plans load each family's PL dwords directly (hoist_quad); other plans stage the PL
  // windows through LDS by LDS-DMA (double buffer per wave)
  A.dn_pf = 0;
  A.quad_full = E->quad_full;
  const bool quad = !gen && !unrelated && n_ext == 0 && A.denovo && E->par.numerics == PM_NUM_POLY && E->quad && T == 64 &&
                    (S == 8 || S == 16);
  if (quad) shmem = QWAVE;
  if (!quad && !gen && !unrelated && n_ext == 0 && A.denovo && E->par.numerics == PM_NUM_POLY && E->max_nuc <= 4 && S % DN_PF_C == 0 &&
      E->n_person % 16 == 0 && E->n_person >= 16 && !getenv("PM_NO_PREFETCH")) {
    A.dn_pf = 1;
    shmem = (size_t)(T / 64) * 2 * DN_PF_BUF;
  }
  const bool ep = !unrelated && n_ext > 0 && E->es_poly && E->par.numerics == PM_NUM_POLY;
  BrentFn fn = quad ? (S == 16 ? k_brent<64, 16, PM_NUM_POLY, false, false, true, false, false, true>
                              : k_brent<64, 8, PM_NUM_POLY, false, false, true, false, false, true>)
                   : brent_kernel(T, S, E->par.numerics, gen, !unrelated && n_ext > 0, A.denovo != 0, A.pf_npad > 0 || A.dn_pf, ep);
  if (!fn) { pm_set_last_error("launch_brent: no kernel variant for the lane plan"); return PM_EINVAL; }
  // multi-wave de novo plans (T = 512 / 1024: more than 1024 families) stage 2 buffers per wave: above the
  // default 64 KB dynamic-LDS limit the kernel must opt in, and the block (plus its static LDS: lane plan,
  // tables) must fit one CU's 160 KB; otherwise the same kernel hoists from direct loads
  if (A.dn_pf && !(T == 64 && S == 16)) {
    const size_t stat = (size_t)S * T * 4 + 256 * 8 + 100 * 8 + 96 * 8 + 32 * 4;
    bool ok = shmem + stat <= 160 * 1024;
    if (ok && shmem > 64 * 1024)
      ok = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shmem) == hipSuccess;
    if (!ok) { (void)hipGetLastError(); A.dn_pf = 0; shmem = 0; }
  }
  // Elston-Stewart workspace in LDS: every partial / marriage-partial access of the peel becomes an LDS round
  // trip instead of an L2 one.  Blocks per CU follow from the LDS budget (160 KB per CU).
  A.ws_lds = 0;
  if (ep) {   // polynomial-form peels: coefficients from k_es_hoist, no workspace in k_brent
    A.es_poly = 1;
  } else if (!unrelated && n_ext > 0 && !E->par.denovo) {   // BA peels (the 10-state one is too big)
    const size_t need = (size_t)E->ws_per_lane * T * sizeof(double);
    if (need > 0 && need <= 150 * 1024) {
      if (hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)need) == hipSuccess) {
        A.ws_lds = 1;
        shmem = need;
        grid = E->n_cu * std::max(1, std::min(1024 / T, (int)((160 * 1024) / (need + 8 * 1024))));
      } else (void)hipGetLastError();
    }
  }
  hipEvent_t a, b;
  HIP_TRY(hipEventCreate(&a));
  HIP_TRY(hipEventCreate(&b));
  HIP_TRY(hipEventRecord(a, E->stream));
  if (ep) {   // chunks of the list (the coefficient buffer holds es_chunk items): k_es_hoist, then the chunk's Brent items
    void (*hoist)(DevArgs, int) = A.denovo ? k_es_hoist<true> : k_es_hoist<false>;
    const size_t hlds = (size_t)E->hoist_waves * (E->poly_coef + E->hoist_tmp) * sizeof(double);
    if (hlds > 64 * 1024) HIP_TRY(hipFuncSetAttribute((const void*)hoist, hipFuncAttributeMaxDynamicSharedMemorySize, (int)hlds));
    const size_t stat = (256 + 5 * 27 + (A.denovo ? 2000 : 2)) * sizeof(double);
    const int hgrid = E->n_cu * std::max(1, std::min(8, (int)((160 * 1024) / (hlds + stat))));
    const int max_items = 4 * E->last_n;
    const pmjit::Kernel* K = jit_kernel(E);
    for (int it0 = 0; it0 < max_items; it0 += E->es_chunk) {
      A.es_it0 = it0;
      A.es_it1 = (int)std::min<long long>((long long)it0 + E->es_chunk, INT_MAX);
      if (K) {   // compiled schedule: one thread (--denovo: one wave) per (item, family)
        const int plan = E->use_plan1 ? 1 : 0, ns = (int)K->slot_e.size();
        const int* tab = E->d_jit_slots[plan][E->chrom];
        pmjit::Args J;
        J.items = A.items[list]; J.counts = A.counts; J.ref = A.ref; J.res = (const int*)A.res; J.pl = A.pl; J.lktab = A.lktab;
        J.coef = A.es_coef; J.slot_e = tab; J.slot_sig = tab + ns; J.slot_p0 = tab + 2 * ns;
        J.T10 = E->d_T10; J.T10dn = E->d_T10dn; J.tba = E->d_tba;
        J.list = list; J.it0 = A.es_it0; J.it1 = A.es_it1; J.nslots = ns; J.np = A.n_person; J.T = A.T; J.max_ext = A.max_ext;
        J.dcap = A.poly_dcap; J.vcf = A.vcf; J.res_words = sizeof(pm_site_result) / 4;
        J.res_a1 = offsetof(pm_site_result, allele1) / 4; J.res_a2 = offsetof(pm_site_result, allele2) / 4;
        J.denovo = A.denovo;
        void* params[] = {&J};
        if (K->wave)
          HIP_TRY(hipModuleLaunchKernel(K->fn, E->n_cu * std::max(1, 16 / K->wpb), 1, 1, 64 * K->wpb, 1, 1, 0, E->stream, params, nullptr));
        else HIP_TRY(hipModuleLaunchKernel(K->fn, E->n_cu * 8, 1, 1, 256, 1, 1, 0, E->stream, params, nullptr));
      } else hipLaunchKernelGGL(hoist, dim3(hgrid), dim3(64 * E->hoist_waves), hlds, E->stream, A, list);
      HIP_TRY(hipGetLastError());
      hipLaunchKernelGGL(fn, dim3(grid), dim3(T), shmem, E->stream, A, list);
      HIP_TRY(hipGetLastError());
    }
  } else {
    hipLaunchKernelGGL(fn, dim3(grid), dim3(T), shmem, E->stream, A, list);
  }
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipEventRecord(b, E->stream));
  E->brent_events.push_back({a, b});
  return PM_OK;
}

static int run_pipeline(pm_engine* E, int n, const uint8_t* pl, const uint32_t* dm, const uint8_t* ref, pm_site_result* res,
                        pm_geno_call* calls) {
  DevArgs A = make_args(E, n, pl, dm, ref, res, calls);
  E->last_n = n;
  HIP_TRY(hipMemsetAsync(E->d_counts, 0, 16 * sizeof(int), E->stream));
  {
    const int big = 0x7fffffff;   // counts[4] = first emitted site (atomicMin)
    HIP_TRY(hipMemcpyAsync(E->d_counts + 4, &big, sizeof(int), hipMemcpyHostToDevice, E->stream));
  }
  {   // persons per lane of k_prep: vector loads when n_person allows; the reference's serial mono order in EXACT
    const int np = E->n_person;
    int vmax = 8;   // measured best on 1000 quads (16 and 4 within 1%)
    void (*prep)(DevArgs) = E->par.numerics == PM_NUM_EXACT ? k_prep<1, true>
                          : (np % 16 == 0 && vmax >= 16) ? k_prep<16, false> : (np % 8 == 0 && vmax >= 8) ? k_prep<8, false>
                          : (np % 4 == 0 && vmax >= 4) ? k_prep<4, false> : k_prep<1, false>;
    hipLaunchKernelGGL(prep, dim3((n + 3) / 4), dim3(256), 0, E->stream, A);
  }
  HIP_TRY(hipGetLastError());
  int rc;
  const int tb = 256, gb = (n + tb - 1) / tb;
  if (E->par.quick_call) {   // main.cpp:354-437 on lists 1 and 2, survivors -> list 0
    if ((rc = launch_brent(E, A, 1, true))) return rc;
    hipLaunchKernelGGL(k_quick_select, dim3(gb), dim3(tb), 0, E->stream, A);
    HIP_TRY(hipGetLastError());
    if ((rc = launch_brent(E, A, 2, true))) return rc;
    hipLaunchKernelGGL(k_quick_final, dim3(gb), dim3(tb), 0, E->stream, A);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_quick_stats, dim3(1), dim3(1), 0, E->stream, A);
    HIP_TRY(hipMemsetAsync(E->d_counts + 1, 0, 2 * sizeof(int), E->stream));
  }
  if ((rc = launch_brent(E, A, 0))) return rc;
  if (E->vcf) {
    hipLaunchKernelGGL(k_finalize_vcf, dim3(gb), dim3(tb), 0, E->stream, A);
    HIP_TRY(hipGetLastError());
  } else {
    hipLaunchKernelGGL(k_select, dim3(gb), dim3(tb), 0, E->stream, A);
    HIP_TRY(hipGetLastError());
    if ((rc = launch_brent(E, A, 1))) return rc;
    hipLaunchKernelGGL(k_finalize, dim3(gb), dim3(tb), 0, E->stream, A);
    HIP_TRY(hipGetLastError());
  }
  if (E->par.denovo) {
    if ((rc = launch_brent(E, A, 2))) return rc;
    hipLaunchKernelGGL(k_final_dn, dim3(gb), dim3(tb), 0, E->stream, A);
    HIP_TRY(hipGetLastError());
  }
  {
    const int nb = std::max(1, (n + 1023) / 1024);
    hipLaunchKernelGGL(k_rows_count, dim3(nb), dim3(1024), 0, E->stream, A);
    hipLaunchKernelGGL(k_rows, dim3(nb), dim3(1024), 0, E->stream, A);
  }
  HIP_TRY(hipGetLastError());
  {
    const bool es = (E->use_plan1 ? E->n_ext1 : E->n_ext) > 0;
    // k_posterior_lean: its LDS family table packs first person (24 bits) and persons (7 bits), <= 48 KB
    const bool lean = !E->par.denovo && !es && E->chrom == PM_CHR_AUTO && E->max_nuc <= 4 && !E->use_plan1 &&
                      E->n_fam <= 12288 && E->max_fam <= 127 && E->n_person < (1 << 24);
    void (*post)(DevArgs) = E->par.denovo ? (es ? k_posterior<true, true> : k_posterior<true, false>)
                          : es ? k_posterior<false, true> : lean ? (E->vcf ? k_posterior_lean<true> : k_posterior_lean<false>)
                                                                 : k_posterior<false, false>;
    hipLaunchKernelGGL(post, dim3(E->grid_post), dim3(256), lean ? (size_t)E->n_fam * 4 : 0, E->stream, A);
    const pmjit::Kernel* K = es && A.n_es_pers > 0 ? jit_kernel(E) : nullptr;
    if (K && K->fn_post) {   // compiled schedule: one thread per (row, peeled family), all its persons' 3 peels in registers
      HIP_TRY(hipGetLastError());
      const int plan = E->use_plan1 ? 1 : 0, ns = (int)K->slot_e.size();
      const int* tab = E->d_jit_slots[plan][E->chrom];
      void* thr = nullptr;
      HIP_TRY(hipGetSymbolAddress(&thr, HIP_SYMBOL(c_gq_thr)));
      pmjit::PostArgs P;
      P.counts = A.counts; P.row_site = A.row_site; P.res = (const char*)A.res; P.pl = A.pl; P.lktab = A.lktab;
      P.gq_thr = (const double*)thr; P.calls = (void*)A.calls; P.fam_p0 = tab + 2 * ns; P.fam_sig = tab + ns;
      P.nfams = ns; P.np = A.n_person; P.vcf = A.vcf; P.res_bytes = sizeof(pm_site_result);
      P.off_a1 = offsetof(pm_site_result, allele1); P.off_a2 = offsetof(pm_site_result, allele2);
      P.off_maxidx = offsetof(pm_site_result, maxidx); P.off_af = offsetof(pm_site_result, af);
      P.theta = A.theta;
      void* params[] = {&P};
      HIP_TRY(hipModuleLaunchKernel(K->fn_post, E->n_cu * 8, 1, 1, 256, 1, 1, 0, E->stream, params, nullptr));
    } else if (es && A.n_es_pers > 0) {
      HIP_TRY(hipGetLastError());
      // LDS workspace when a 64-thread block's share fits: the block size is the largest of 256/128/64 whose
      // workspace stays within the 64 KB default dynamic-LDS limit
      const size_t per = (size_t)E->ws_per_lane * sizeof(double);
      int bt = 0;
      for (int t : {256, 128, 64})
        if (!bt && per * t <= 64 * 1024 && !getenv("PM_ES_POST_HBM")) bt = t;
      if (bt) {
        const int per_cu = std::max(1, (int)((160 * 1024) / (per * bt + 3 * 1024)));
        void (*pe)(DevArgs) = E->par.denovo ? k_posterior_es<true, true> : k_posterior_es<false, true>;
        hipLaunchKernelGGL(pe, dim3(E->n_cu * per_cu * 2), dim3(bt), per * bt, E->stream, A);
      } else
        hipLaunchKernelGGL(E->par.denovo ? k_posterior_es<true> : k_posterior_es<false>, dim3(E->grid_post), dim3(256), 0, E->stream, A);
    }
  }
  HIP_TRY(hipGetLastError());
  if (!E->par.denovo && E->chrom == PM_CHR_AUTO && !E->vcf) {
    hipLaunchKernelGGL(k_ab, dim3(E->n_cu * 8), dim3(256), 0, E->stream, A);
    HIP_TRY(hipGetLastError());
  }
  return PM_OK;
}

static int collect_stats(pm_engine* E) {
  for (auto& pr : E->brent_events) {
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, pr.first, pr.second));
    E->stats.kernel_ms += ms;
    E->stats.launches++;
    hipEventDestroy(pr.first); hipEventDestroy(pr.second);
  }
  E->brent_events.clear();
  return PM_OK;
}

int pm_engine_run_device(pm_engine* E, int32_t n, const uint8_t* d_pl, const uint32_t* d_dm, const uint8_t* d_ref, pm_site_result* d_res,
                         pm_geno_call* d_calls) {
  if (!E || n < 0 || n > E->max_batch) { pm_set_last_error("pm_engine_run_device: invalid arguments (n > max_batch?)"); return PM_EINVAL; }
  if (n == 0) return PM_OK;
  HIP_TRY(hipSetDevice(E->device));
  return run_pipeline(E, n, d_pl, d_dm, d_ref, d_res ? d_res : E->d_res, d_calls ? d_calls : E->d_calls);
}

int pm_engine_sync(pm_engine* E) {
  if (!E) return PM_EINVAL;
  HIP_TRY(hipSetDevice(E->device));
  HIP_TRY(hipStreamSynchronize(E->stream));
  int counts[16];
  HIP_TRY(hipMemcpy(counts, E->d_counts, sizeof(counts), hipMemcpyDeviceToHost));
  if (counts[4] != 0x7fffffff) E->carry_postprob = true;
  E->stats.items += (int64_t)counts[0] + counts[1] + counts[2] + counts[8];
  E->stats.site_visits += (int64_t)counts[0] / (E->vcf ? 1 : (E->par.denovo && !mono_dn_in_prep(E)) ? 4 : 3) + counts[1] / 3 +
                          counts[2] + counts[9];
  E->stats.sites += E->last_n;
  int rc = collect_stats(E);
  if (rc) return rc;
  if (counts[5]) { pm_set_last_error("ScalarMinimizer::Brent got stuck"); return PM_EBRENT; }
  return PM_OK;
}

int pm_engine_run(pm_engine* E, int32_t n, const uint8_t* pl, const uint32_t* dm, const uint8_t* ref, int32_t on_device,
                  pm_site_result* res, pm_geno_call* calls, int32_t* n_rows) {
  if (!E || n < 0 || n > E->max_batch || !res || !n_rows) { pm_set_last_error("pm_engine_run: invalid arguments"); return PM_EINVAL; }
  *n_rows = 0;
  if (n == 0) return PM_OK;
  HIP_TRY(hipSetDevice(E->device));
  const size_t np = E->n_person;
  const uint8_t* spl = pl;   // person-major GLF records (host or device)
  const uint32_t* ddm = dm;
  const uint8_t* dref = ref;
  if (!on_device) {
    HIP_TRY(hipMemcpyAsync(E->d_stage, pl, (size_t)n * np * 10, hipMemcpyHostToDevice, E->stream));
    HIP_TRY(hipMemcpyAsync(E->d_dm, dm, (size_t)n * np * 4, hipMemcpyHostToDevice, E->stream));
    HIP_TRY(hipMemcpyAsync(E->d_ref, ref, (size_t)n, hipMemcpyHostToDevice, E->stream));
    spl = E->d_stage; ddm = E->d_dm; dref = E->d_ref;
  }
  int rc = pm_engine_to_planar(E, n, spl, E->d_pl);   // the engine's genotype-planar layout
  if (rc) return rc;
  rc = run_pipeline(E, n, E->d_pl, ddm, dref, E->d_res, E->d_calls);
  if (rc) return rc;
  rc = pm_engine_sync(E);
  if (rc) return rc;
  HIP_TRY(hipMemcpy(res, E->d_res, sizeof(pm_site_result) * n, hipMemcpyDeviceToHost));
  int counts[16];
  HIP_TRY(hipMemcpy(counts, E->d_counts, sizeof(counts), hipMemcpyDeviceToHost));
  *n_rows = counts[3];
  if (calls && counts[3] > 0) {
    if (E->vcf) {   // 4-B rows on the device (pm_vcf_call), expanded into the caller's pm_geno_call rows
      const size_t nr = np * (size_t)counts[3];
      std::vector<pm_vcf_call> v(nr);
      HIP_TRY(hipMemcpy(v.data(), E->d_calls, sizeof(pm_vcf_call) * nr, hipMemcpyDeviceToHost));
      for (size_t i = 0; i < nr; i++) {
        pm_geno_call c;
        c.dosage = 0.0; c.best = v[i].best; c.gq = v[i].gq; c.label = v[i].label;
        c._pad[0] = c._pad[1] = c._pad[2] = 0;
        calls[i] = c;
      }
    } else HIP_TRY(hipMemcpy(calls, E->d_calls, sizeof(pm_geno_call) * np * counts[3], hipMemcpyDeviceToHost));
  }
  return PM_OK;
}

int pm_engine_to_planar(pm_engine* E, int32_t n, const uint8_t* d_src, uint8_t* d_dst) {
  if (!E || n < 0 || !d_src || !d_dst || d_src == d_dst) { pm_set_last_error("pm_engine_to_planar: invalid arguments"); return PM_EINVAL; }
  if (n == 0) return PM_OK;
  HIP_TRY(hipSetDevice(E->device));
  const long long total = (long long)n * E->n_person;
  const int tb = 256;
  hipLaunchKernelGGL(k_to_planar, dim3((unsigned)((total + tb - 1) / tb)), dim3(tb), 0, E->stream, n, E->n_person, d_src, d_dst);
  HIP_TRY(hipGetLastError());
  return PM_OK;
}

int pm_engine_counters(pm_engine* E, pm_counters* out) {
  if (!E || !out) return PM_EINVAL;
  HIP_TRY(hipSetDevice(E->device));
  unsigned long long c[16];
  HIP_TRY(hipStreamSynchronize(E->stream));
  HIP_TRY(hipMemcpy(c, E->d_counters, sizeof(c), hipMemcpyDeviceToHost));
  memset(out, 0, sizeof(*out));
  for (int k = 0; k < 5; k++) out->ref_base_counts[k] = (int64_t)c[k];
  out->min_total_depth_filter = (int64_t)c[5];
  out->max_total_depth_filter = (int64_t)c[6];
  out->min_ps_filter = (int64_t)c[7];
  out->min_map_qual_filter = (int64_t)c[8];
  out->homo_ref = (int64_t)c[9];
  out->transitions = (int64_t)c[10];
  out->transversions = (int64_t)c[11];
  out->tstvs1 = (int64_t)c[12];
  out->tstvs2 = (int64_t)c[13];
  out->tvs1tvs2 = (int64_t)c[14];
  out->nocall = (int64_t)c[15];
  return PM_OK;
}

int pm_engine_synth(pm_engine* E, int32_t n, uint64_t seed, uint64_t off, uint8_t* d_pl, uint32_t* d_dm, uint8_t* d_ref) {
  if (!E || n <= 0) return PM_EINVAL;
  HIP_TRY(hipSetDevice(E->device));
  DevArgs A = make_args(E, 0, nullptr, nullptr, nullptr, nullptr, nullptr);
  const long long total = (long long)n * E->n_fam;
  const int tb = 256;
  hipLaunchKernelGGL(k_synth, dim3((unsigned)((total + tb - 1) / tb)), dim3(tb), 0, E->stream, A, n, seed, off, d_pl, d_dm, d_ref);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(E->stream));
  return PM_OK;
}

int pm_device_alloc(pm_engine* E, uint64_t bytes, void** p) {
  if (!E || !p) return PM_EINVAL;
  HIP_TRY(hipSetDevice(E->device));
  HIP_TRY(hipMalloc(p, bytes ? bytes : 1));
  return PM_OK;
}
int pm_device_free(pm_engine* E, void* p) {
  if (!E) return PM_EINVAL;
  HIP_TRY(hipSetDevice(E->device));
  HIP_TRY(hipFree(p));
  return PM_OK;
}
int pm_copy_to_host(pm_engine* E, void* dst, const void* src, uint64_t bytes) {
  if (!E) return PM_EINVAL;
  HIP_TRY(hipSetDevice(E->device));
  HIP_TRY(hipStreamSynchronize(E->stream));
  HIP_TRY(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
  return PM_OK;
}

int pm_copy_to_device(pm_engine* E, void* dst, const void* src, uint64_t bytes) {
  if (!E) return PM_EINVAL;
  HIP_TRY(hipSetDevice(E->device));
  HIP_TRY(hipStreamSynchronize(E->stream));
  HIP_TRY(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
  return PM_OK;
}

int pm_engine_kernel_stats(pm_engine* E, pm_kernel_stats* out, int32_t reset) {
  if (!E || !out) return PM_EINVAL;
  HIP_TRY(hipSetDevice(E->device));
  unsigned long long ev = 0;
  HIP_TRY(hipStreamSynchronize(E->stream));
  int rc = collect_stats(E);
  if (rc) return rc;
  HIP_TRY(hipMemcpy(&ev, E->d_eval_total, sizeof(ev), hipMemcpyDeviceToHost));
  *out = E->stats;
  out->evals = (int64_t)ev;
  out->fam_evals = (int64_t)ev * E->n_fam;
  if (E->d_phase) {
    unsigned long long ph[3];
    HIP_TRY(hipMemcpy(ph, E->d_phase, sizeof(ph), hipMemcpyDeviceToHost));
    out->hoist_wave_ns = (int64_t)((double)ph[0] * 1e6 / E->wall_khz);   // wall_clock64 ticks at wall_khz
    out->eval_wave_ns = (int64_t)((double)ph[1] * 1e6 / E->wall_khz);
    out->timed_items = (int64_t)ph[2];
  }
  if (reset) {
    E->stats = pm_kernel_stats{};
    HIP_TRY(hipMemset(E->d_eval_total, 0, sizeof(ev)));
    if (E->d_phase) HIP_TRY(hipMemset(E->d_phase, 0, 3 * sizeof(unsigned long long)));
  }
  return PM_OK;
}

}  // extern "C"
