#pragma once
// engine_dev.h -- device side of the MI355X (gfx950) engine for polyMutt's per-site family likelihood.
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
#include "brent_core.h"   // pos_div, wave_prod, log10_mant_u, the Brent state machine (shared with the JIT kernels)

#define MALE 1
#define FEMALE 2
#ifndef PM_HOIST_CHUNK
#define PM_HOIST_CHUNK 4
#endif
#ifndef PM_QD_NC4
#define PM_QD_NC4 0   // QUAD plans: 4 normalised coefficients per family (hoist_quad_t; measured slower at 2 waves)
#endif
#ifndef PM_QD_WAVES
#define PM_QD_WAVES 2   // QUAD plans: waves per SIMD the k_brent instantiation is compiled for (launch bounds, grid)
#endif
#ifndef PM_G4_LATE
#define PM_G4_LATE 1   // lane_poly_r: the per-family g^4 factor applied once per lane as (g^4)^S
#endif
#ifndef PM_EPO_WAVES
#define PM_EPO_WAVES 3   // the ep_only EP kernels (NF = 1): 167 VGPRs fit 3 waves per SIMD
#endif
#ifndef PM_EP_WAVES
#define PM_EP_WAVES 2   // EP (polynomial-form extended families) k_brent: waves per SIMD of the launch bounds
#endif
#ifndef PM_QD_KIDSEQ
#define PM_QD_KIDSEQ 0   // QUAD de novo hoisting: the two kids' lookups one kid at a time
#endif
#ifndef PM_QD_MONO
#define PM_QD_MONO 1
#endif
#ifndef PM_POLY_WAVES
#define PM_POLY_WAVES 2
#endif

// ------------------------------------------------------------------------------------------------
// error reporting (thread-local, C ABI)
extern "C" void pm_set_last_error(const char* msg);   // (engine.hip)

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
  int mono_dn;             // lean --denovo: the de novo monomorphism item (cfg 0) is not enqueued; 1 = k_prep computes it,
                           // 2 = the site's cfg-1 QUAD item does (from its hoisted f^4 coefficients, no extra plane reads)
  int* row_blk;            // k_rows_count / k_rows: written records per 1024-site block
  int pf_npad;             // lean kernel: > 0 = the item's 3 genotype planes are prefetched into LDS (bytes copied per plane)
  int pf_stride;           // ... at this stride (pf_npad + 16: each plane's last 16 bytes are never written -- zeros: the
                           // persons of the virtual all-PL-0 family that fills a split plan's empty slots)
  int pf_dw;               // ... in 4-byte pieces (n_person % 16 != 0, n_person % 4 == 0)
  int dn_pf;               // lean --denovo kernel: PL windows staged through LDS by LDS-DMA (hoist_poly4_dn_pf)
  int quad_full;           // QUAD plan (hoist_quad): slot rows below this have no empty lane
  int ep_only;             // EP launches: the lane plan has no nuclear or founder units (every family is peeled)
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
  int* counts;             // [0..2] list sizes, [3] rows, [4] first emitted site, [5] Brent stuck, [6] first stuck site
                           // (atomicMin), [8]/[9] quick items/site visits
  int qd_group;            // QUAD kernel: items per site group of the list (a wave takes a site's items in turn)
  int itmax;               // Brent's ITMAX (MathGold.cpp:98: 200; PM_TEST_ITMAX lowers it for the failure-path tests)
  int* qd_ctr;             // QUAD kernel: the 8 per-XCD claim counters of the dynamic item order (zeroed per launch), or null
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
// SetTransmissionMatrix_BA, _CHRX_2Female, _CHRX_2Male, _CHRY, _MITO (:812-924), [parent1][parent2][child]
#define PM_TBA_VALUES                                                                                \
  {{1, 0, 0, .5, .5, 0, 0, 1, 0, .5, .5, 0, .25, .5, .25, 0, .5, .5, 0, 1, 0, 0, .5, .5, 0, 0, 1},  \
   {1, 0, 0, .5, .5, 0, 0, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 0, 0, .5, .5, 0, 0, 1},           \
   {1, 0, 0, .5, 0, .5, 0, 0, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 0, 0, .5, 0, .5, 0, 0, 1},           \
   {1, 0, 0, 1, 0, 0, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 0, 0, 1, 0, 0, 1},               \
   {1, 0, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 0, 0, 0, 0, 1}}
// (internal linkage and a static initialiser: every translation unit's code object carries its own copy, so the
// k_brent instantiations compiled in csrc/brent_inst.hip need no upload)
static __constant__ double c_TBA[5][27] = PM_TBA_VALUES;

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
// register tiles of the evaluation: a polynomial of degree <= PD as PD + 1 coefficients (zero above its degree).  PD is a
// template parameter of the EP k_brent instantiations: 8 (4 founders, ext10) or 12 (6 founders: config 4's 12-member
// three-generation pedigrees), picked per launch from the plan's largest degree in the section's class (launch_brent)
#define PM_PD_LO 8
#define PM_PD_HI 12

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

// es_poly_eval on register-resident coefficients (c[a] = 0 above D <= PD): the leading zeros leave the Horner
// sum's bits unchanged (0 * t + c = c)
#ifndef PM_EPE
#define PM_EPE 4   // extended families per lane whose coefficients stay in registers through an item's evaluations
#endif
template <int PD>
__device__ __forceinline__ double es_poly_eval_r(const double* c, int D, double x) {
  const double g = 1 - x;
  double acc = 0.0, base;
  if (x <= 0.5) {
    const double t = x / g;
#pragma unroll
    for (int a = PD; a >= 0; a--) acc = acc * t + c[a];
    base = g;
  } else {
    const double sr = g / x;
#pragma unroll
    for (int a = 0; a <= PD; a++) acc = a <= D ? acc * sr + c[a] : acc;
    base = x;
  }
  double p = 1.0;
#pragma unroll
  for (int a = 0; a < PD; a++) p = a < D ? p * base : p;
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
// NF = 3: the plan's every nuclear family is a trio (or the slot is empty): one kid, no second-kid loads or selects (an
// empty slot's kid terms multiply lF = 0 and are then replaced by the phantom family)
// PM_FAM_FACTORED (default): the quartic from quad_poly4's factored sums (the QUAD plan's form: equal to fold_poly(c9)
// in real arithmetic, about half the operations) instead of hoist_nuc's nine products
#ifndef PM_FAM_FACTORED
#define PM_FAM_FACTORED 1
#endif
__device__ __forceinline__ void quad_poly4(const double (*D)[3], const double* lF, const double* lM, double* a);
template <int NF = 0, bool VIRT = false>
__device__ __forceinline__ void fam_poly4(const uint32_t* by, int nn, const double* lk, double* a) {
  if constexpr (PM_FAM_FACTORED && VIRT) {   // every slot a real family or the virtual one (hoist_poly4_lds_rows)
    double D[2][3];
#pragma unroll
    for (int q = 0; q < 2; q++)
#pragma unroll
      for (int k = 0; k < 3; k++) D[q][k] = (NF == 3 && q == 1) ? 1.0 : lk[by[3 * (2 + q) + k]];
    const double lF[3] = {lk[by[0]], lk[by[1]], lk[by[2]]};
    const double lM[3] = {lk[by[3]], lk[by[4]], lk[by[5]]};
    quad_poly4(D, lF, lM, a);
    return;
  }
  if constexpr (PM_FAM_FACTORED) {
    // kid q's (l11, l12, l22); a missing kid is (1, 1, 1): its likelihoodONEKid terms are then exactly 1 (the factors
    // 2 and 4 of quad_poly4's sums are undone by its exact 0.5 / 0.25 scalings)
    double D[2][3];
#pragma unroll
    for (int q = 0; q < 2; q++) {
      const bool kid = NF == 3 ? q == 0 : NF == 4 ? true : 2 + q < nn;   // (NF = 4: quads or empty slots)
#pragma unroll
      for (int k = 0; k < 3; k++) D[q][k] = kid ? lk[by[3 * (2 + q) + k]] : 1.0;
    }
    const bool fam = nn >= 2;   // (no parents: lF = 0, every coefficient +0, then the phantom family)
    const double lF[3] = {fam ? lk[by[0]] : 0.0, fam ? lk[by[1]] : 0.0, fam ? lk[by[2]] : 0.0};
    const double lM[3] = {lk[by[3]], lk[by[4]], lk[by[5]]};
    quad_poly4(D, lF, lM, a);
    if (nn == 0) {
      a[0] = 1.0; a[1] = 4.0; a[2] = 6.0; a[3] = 4.0; a[4] = 1.0;
    }
    return;
  }
  double kids[9];
#pragma unroll
  for (int k = 0; k < 9; k++) kids[k] = 1.0;
#pragma unroll
  for (int q = 2; q < (NF == 3 ? 3 : 4); q++) {
    // a missing kid reads l = 1: every autosomal d_one_kid term is then exactly 1.0 (0.5 * (1 + 1),
    // 0.25 + 0.5 + 0.25), the factor the reference never multiplies in -- three selects instead of nine
    const bool kid = NF == 3 || q < nn;
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
  const int np = A.n_person, npad = A.pf_npad, stride = A.pf_stride;
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
        __builtin_amdgcn_global_load_lds((const void*)(plane + off), (void*)(buf + k * stride + c), 4, 0, 0);
      }
    }
    return;
  }
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const uint8_t* plane = base + (size_t)gs[k] * np;
    for (int c = wv * 1024; c < npad; c += W * 1024) {
      const int off = min(c + lane * 16, np - 16);
      __builtin_amdgcn_global_load_lds((const void*)(plane + off), (void*)(buf + k * stride + c), 16, 0, 0);
    }
  }
}

// hoist_poly4 reading the item's planes from the LDS buffer of prefetch_planes (same arithmetic and order).
#ifndef PM_HOIST_CHUNK_LDS
#define PM_HOIST_CHUNK_LDS 2
#endif
// NF = 34: a split plan (plan_split34): slot rows [0, S/2) hold quads (or nothing), rows [S/2, S) trios (or nothing), so
// each half is hoisted with its family size known -- the quads without the missing-kid selects, the trios without the
// second kid -- mixed trio / quad pedigrees (config 5's) get the trio plans' saving on half their slots
// (VIRT: the split plan's empty slots hold the virtual family -- persons at the planes' zero tail, every likelihood
// lk[0] = 1.0 -- whose quartic is exactly the phantom (1, 4, 6, 4, 1): no empty-slot selects at all)
template <int NF, int S, int C, int S0, int S1, bool VIRT = false>
__device__ __forceinline__ void hoist_poly4_lds_rows(const int* uu, const uint8_t* buf, int npad, const double* lk, double (*a)[5]) {
#pragma unroll
  for (int s = S0; s < S1; s++) {
    if (s % C == 0) __builtin_amdgcn_sched_barrier(0);   // chunks of C slots: bounded registers in flight
    const int u = uu[s];
    const int nn = unit_nn(u);
    uint32_t by[12];
#pragma unroll
    for (int q = 0; q < (NF == 3 ? 3 : 4); q++) {
      // in range for every lane: no branch around the read (NF = 4: an empty slot reads persons 0-3, then the phantom)
      const int pp = unit_first(u) + (NF == 4 ? q : q < nn ? q : 0);
      by[3 * q + 0] = buf[pp];
      by[3 * q + 1] = buf[npad + pp];
      by[3 * q + 2] = buf[2 * npad + pp];
    }
    fam_poly4<NF, VIRT>(by, nn, lk, a[s]);
  }
}
template <int S, int T, int NF = 0>
__device__ __forceinline__ void hoist_poly4_lds(const DevArgs& A, const int* su, const uint8_t* buf, const double* lk,
                                                double (*a)[5]) {
  const int npad = A.pf_stride;   // (the planes' stride in the buffer)
  constexpr int C = S < PM_HOIST_CHUNK_LDS ? S : PM_HOIST_CHUNK_LDS;
  int uu[S];
  load_units<S>(su, uu);
  if constexpr (NF == 34) {
    hoist_poly4_lds_rows<4, S, C, 0, S / 2, true>(uu, buf, npad, lk, a);
    hoist_poly4_lds_rows<3, S, C, S / 2, S, true>(uu, buf, npad, lk, a);
  } else hoist_poly4_lds_rows<NF, S, C, 0, S>(uu, buf, npad, lk, a);
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
#ifndef QB
#define QB 3          // slot buffers in the ring
#endif
#ifndef QD_AHEAD
#define QD_AHEAD 2    // slots in flight ahead of the hoisting (< QB)
#endif
static_assert(QD_AHEAD >= 1 && QD_AHEAD < QB && QD_AHEAD <= 6, "QUAD ring geometry");
// s_waitcnt immediate for vmcnt(n) alone (expcnt and lgkmcnt at their no-wait maxima; vmcnt's two high bits at 15:14)
#define PM_VMCNT(n) (0x0F70 | ((n) & 0xF) | (((n) >> 4) << 14))
template <int N> __device__ __forceinline__ void vm_wait() { __builtin_amdgcn_s_waitcnt(PM_VMCNT(N)); }
// wait until at most j slots' DMA (3 instructions each) are outstanding (j folds to a constant in unrolled loops)
__device__ __forceinline__ void vm_wait_slots(int j) {
  switch (j) {
    case 0: vm_wait<0>(); break;
    case 1: vm_wait<3>(); break;
    case 2: vm_wait<6>(); break;
    case 3: vm_wait<9>(); break;
    case 4: vm_wait<12>(); break;
    default: vm_wait<15>(); break;
  }
}
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
// NC = 4 (PM_QD_NC4): each family's quartic is stored normalised by its constant term a4 (> 0: every PL likelihood
// and mutation-matrix dot product is positive), b_k = a_k / a4 for k = 0..3, and the lane's product of the a4 is
// kept as one (mantissa, exponent) pair (m0, e0) that seeds the evaluation's product: 4 x S registers of
// coefficients instead of 5 x S, so the 16-slot kernel runs 3 waves per SIMD.  h(r) = a4 (b0 r^4 + .. + b3 r + 1):
// still non-negative throughout, the normalisation adds one rounding per coefficient.
template <int S, bool DNV, int NC>
__device__ __forceinline__ void hoist_quad_t(const DevArgs& A, const ItemCtx& I, const uint8_t* pl, const double* lk,
                                             const double* M, double (*a)[NC], uint8_t* ring, const uint32_t* voff, double& m0, int& e0) {
  if constexpr (NC == 4) { m0 = 1.0; e0 = 0; }
  const int lane = threadIdx.x & 63;
  const uint32_t* rw = (const uint32_t*)ring + lane;   // the lane's dword of plane g, slot buffer b: rw[(b * QSLOT + g * 256) / 4]
  const int o11 = I.g11 * 64, o12 = I.g12 * 64, o22 = I.g22 * 64;
  // re-read per item (opaque), so the compiler does not keep S slot predicates live across the Brent loop
  int qfull = A.quad_full, nfam = A.n_fam, npo = A.n_person;
  asm volatile("" : "+s"(qfull), "+s"(nfam), "+s"(npo));
#pragma unroll
  for (int s = 0; s < S; s++) {
    // slot s has landed: only the later slots' DMA (3 instructions each, at most QD_AHEAD - 1 of them) may be outstanding
    vm_wait_slots(QD_AHEAD - 1 < S - 1 - s ? QD_AHEAD - 1 : S - 1 - s);
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
      double pg[2][10];   // both kids' 20 table lookups in flight together (PM_QD_KIDSEQ: one kid at a time)
      if constexpr (!PM_QD_KIDSEQ)
#pragma unroll
        for (int g = 0; g < 10; g++) { pg[0][g] = lk[(wg[g] >> 16) & 0xFF]; pg[1][g] = lk[wg[g] >> 24]; }
      // the item's three mutation-matrix rows from the kernel arguments (scalar loads issued beside the lookups):
      // scalar FMA operands, no LDS read per slot
      double mr[3][10];
#pragma unroll
      for (int g = 0; g < 10; g++) { mr[0][g] = A.Mk[I.g11 * 10 + g]; mr[1][g] = A.Mk[I.g12 * 10 + g]; mr[2][g] = A.Mk[I.g22 * 10 + g]; }
      __builtin_amdgcn_sched_barrier(0);
      if (s + QD_AHEAD < S) quad_dma(pl, s + QD_AHEAD, npo, voff, ring + ((s + QD_AHEAD) % QB) * QSLOT);
      if constexpr (PM_QD_KIDSEQ) {
#pragma unroll
        for (int q = 0; q < 2; q++) {   // one kid at a time: 10 lookups in flight (register pressure at 3 waves / SIMD)
#pragma unroll
          for (int g = 0; g < 10; g++) pg[q][g] = lk[(wg[g] >> (16 + 8 * q)) & 0xFF];
          D[q][0] = D[q][1] = D[q][2] = 0.0;
#pragma unroll
          for (int g = 0; g < 10; g++) {   // CalcDenovoMutLk (:1553-1562)
            D[q][0] = fma(mr[0][g], pg[q][g], D[q][0]);
            D[q][1] = fma(mr[1][g], pg[q][g], D[q][1]);
            D[q][2] = fma(mr[2][g], pg[q][g], D[q][2]);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      } else {
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
    double q5x[5];
    double* q5 = NC == 5 ? a[s] : q5x;   // (NC = 5: the quartic straight into the slot's registers)
    quad_poly4(D, lF, lM, q5);
    if (s >= qfull) {   // the partial last slot row: empty lanes hold the phantom family (f + g)^4
      const bool empty = 64 * s + lane >= nfam;
      q5[0] = empty ? 1.0 : q5[0]; q5[1] = empty ? 4.0 : q5[1]; q5[2] = empty ? 6.0 : q5[2];
      q5[3] = empty ? 4.0 : q5[3]; q5[4] = empty ? 1.0 : q5[4];
    }
    if constexpr (NC == 4) {
      // 1 / a4 from the hardware reciprocal and two Newton steps (within an ulp), then the four quotients
      double y = __builtin_amdgcn_rcp(q5[4]);
      double ee = fma(-q5[4], y, 1.0);
      y = fma(y, ee, y);
      ee = fma(-q5[4], y, 1.0);
      y = fma(y, ee, y);
#pragma unroll
      for (int k = 0; k < 4; k++) a[s][k] = q5[k] * y;
      int x;
      m0 = frexp(m0 * q5[4], &x);   // a4 >= ~1e-120: one factor per renormalisation
      e0 += x;
      // pinned here: otherwise IR-level sinking moves every slot's arithmetic past the hoisting loop, where all the
      // slots' table lookups are then live at once (2 KB of spills)
      asm volatile("" : "+v"(a[s][0]), "+v"(a[s][1]), "+v"(a[s][2]), "+v"(a[s][3]), "+v"(m0), "+v"(e0));
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// de novo items and cfg-7 items (uniform per item) take separate straight-line slot loops
template <int S, int NC>
__device__ __forceinline__ void hoist_quad(const DevArgs& A, const ItemCtx& I, const uint8_t* pl, const double* lk,
                                           const double* M, double (*a)[NC], uint8_t* ring, const uint32_t* voff, double& m0, int& e0) {
  if (I.denovo) hoist_quad_t<S, true, NC>(A, I, pl, lk, M, a, ring, voff, m0, e0);
  else hoist_quad_t<S, false, NC>(A, I, pl, lk, M, a, ring, voff, m0, e0);
}

// f = 1 (the generic-path de novo monomorphism item): L_fam(1) = a0, the f^4 coefficient; an empty slot's
// phantom family (f + g)^4 has a0 = 1, so no slot needs masking.  Four interleaved (mantissa, exponent)
// accumulators, renormalised after every factor.
template <int S, int NC = 5>
__device__ __forceinline__ void lane_poly_top(const double (*a)[NC], double& m, int& e, double m0 = 1.0, int e0 = 0) {
  constexpr int NA = S < 4 ? S : 4;
  double am[NA];
  int ae[NA];
#pragma unroll
  for (int j = 0; j < NA; j++) { am[j] = 1.0; ae[j] = 0; }
  am[0] = m0; ae[0] = e0;   // (NC = 4: the lane's product of the a4, so that a0 = b0 a4)
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
// NC = 4: normalised coefficients (b0..b3, constant term 1) and the lane's product of the a4 as the seed (m0, e0):
// h = b0 r^4 + .. + b3 r + 1 >= 1, so two factors of g4 h stay within range as before.
template <int S, int NC = 5>
__device__ __forceinline__ void lane_poly_r(double r, double g4, const double (*a)[NC], double& m, int& e, double m0 = 1.0, int e0 = 0) {
  constexpr int NA = S < 4 ? S : 4;
  double am[NA];
  int ae[NA];
#pragma unroll
  for (int j = 0; j < NA; j++) { am[j] = 1.0; ae[j] = 0; }
  am[0] = m0; ae[0] = e0;
#pragma unroll
  for (int s = 0; s < S; s++) {
    // (PM_G4_LATE: the families' common factor g^4 applied once, as (g^4)^S after the product, instead of per family)
    const double h0 = NC == 4 ? fma(r, fma(r, fma(r, fma(r, a[s][0], a[s][1]), a[s][2]), a[s][3]), 1.0)
                              : fma(r, fma(r, fma(r, fma(r, a[s][0], a[s][1]), a[s][2]), a[s][3]), a[s][NC - 1]);
    const double h = PM_G4_LATE ? h0 : h0 * g4;
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
  if constexpr (PM_G4_LATE) {   // (g^4)^S by squaring (g >= 1e-4 on Brent's bracket: >= 1e-256), one renormalisation
    double p = 1.0, q = g4;
#pragma unroll
    for (int b = 1; b <= S; b <<= 1) {
      if (S & b) p = p * q;
      q = q * q;
    }
    int x;
    m = frexp(m * p, &x);
    e += x;
  }
}



// Sum of the 64 lanes' doubles in the same DPP order as wave_prod, broadcast from lane 63 (exact for integer values
// whose partial sums stay below 2^53: k_prep's read statistics and PL sums)
template <int CTRL, int ROWMASK>
__device__ __forceinline__ void dpp_add_step(double& v) {
  const int lo = __double2loint(v), hi = __double2hiint(v);
  const int olo = __builtin_amdgcn_update_dpp(0, lo, CTRL, ROWMASK, 0xF, false);   // rows not written: +0.0
  const int ohi = __builtin_amdgcn_update_dpp(0, hi, CTRL, ROWMASK, 0xF, false);
  v = v + __hiloint2double(ohi, olo);
}
__device__ __forceinline__ double wave_sum_exact(double v) {
  dpp_add_step<0xB1, 0xF>(v);
  dpp_add_step<0x4E, 0xF>(v);
  dpp_add_step<0x141, 0xF>(v);
  dpp_add_step<0x140, 0xF>(v);
  dpp_add_step<0x142, 0xA>(v);
  dpp_add_step<0x143, 0xC>(v);
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), 63), __builtin_amdgcn_readlane(__double2loint(v), 63));
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

#ifndef PM_LOG10_TAB
#define PM_LOG10_TAB 1   // block_logprod's log10: the table form (0: the atanh series of log10_mant)
#endif

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
  return PM_LOG10_TAB ? log10_mant_u(m, e) : log10_mant(m, e);
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
// NF: 3 = every nuclear family of the plan is a trio (the lean PF kernel's hoisting drops the second kid), 0 = any.
// NF: the lean PF kernel's persons per family when every unit is one size (3: trio plans); on EP kernels NF = 1 marks
// the ep_only plans (every family peeled: no nuclear or founder unit), whose unit loads, nuclear hoisting and lane
// products are compiled out -- fewer live registers (PM_EPO_WAVES per SIMD)
// PD: EP kernels' register tile, the largest polynomial degree evaluated from registers (PM_PD_LO / PM_PD_HI)
template <int T, int S, int NUM, bool GEN, bool ES, bool DN = false, bool PF = false, bool EP = false, bool QD = false, int NF = 0,
          int PD = PM_PD_LO>
__global__ void __launch_bounds__(T, (EP ? (NF == 1 ? (PD > PM_PD_LO ? PM_EP_WAVES : PM_EPO_WAVES) : PM_EP_WAVES)
                                     : QD ? PM_QD_WAVES : brent_waves<T, S, NUM, GEN>()))
k_brent(DevArgs A, int list) {
  constexpr int PDM = PD;
  constexpr bool EPO = EP && NF == 1;
  constexpr bool PROD = NUM != PM_NUM_EXACT;
  constexpr bool POLYK = NUM == PM_NUM_POLY && !GEN;
  __shared__ double s_lk[256];
  __shared__ double s_M[(GEN || DN) ? 100 : 1];
  __shared__ double s_red[T > 64 ? 96 : 1];
  __shared__ int s_rede[T > 64 ? 32 : 1];
  __shared__ __attribute__((aligned(16))) int s_u[POLYK && !QD ? S * T : 4];   // packed lane plan (unit_pack, lane-major)
  for (int i = threadIdx.x; i < 256; i += T) s_lk[i] = A.lktab[i];
  if constexpr (GEN || DN)
    for (int i = threadIdx.x; i < 100; i += T) s_M[i] = A.M[i];
  if constexpr (POLYK && !QD)   // (QUAD plans address families by slot and lane: no lane plan)
#pragma unroll
    for (int s = 0; s < S; s++) {
      const int4 u = A.units[s * T + threadIdx.x];
      // (NF = 34: an empty slot holds the virtual family at the planes' zero tail, pf_npad, of its half's size)
      s_u[threadIdx.x * S + s] = (NF == 34 && u.x != U_NUC) ? (A.pf_npad | ((s < S / 2 ? 4 : 3) << 24)) : unit_pack(u);
    }
  if constexpr (PF && NF == 34) {   // the virtual persons' bytes: each plane's never-written tail
    extern __shared__ uint8_t s_pf0[];
    if (A.pf_npad > 0 && threadIdx.x < 48) s_pf0[(threadIdx.x >> 4) * A.pf_stride + A.pf_npad + (threadIdx.x & 15)] = 0;
  }
  __syncthreads();
  int4 unit[S];
  if constexpr (!POLYK) {
#pragma unroll
    for (int s = 0; s < S; s++) unit[s] = EPO ? make_int4(0, 0, 0, 0) : A.units[s * T + threadIdx.x];
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
  // QD: a wave takes the grp consecutive items of one site (its configurations: one PL block) one after the other,
  // then the site grp * gridDim.x items further on, so a site's block is re-read while it is still in the XCD's L2
  // (one wave per item had the site's three reads drift apart over a persistent grid's items; qd_group 1: that order)
  const int grp = QD ? A.qd_group : 1;
  auto next_it = [&](int i) {
    if (grp <= 1) return i + (int)gridDim.x;
    return (i - A.es_it0) % grp + 1 < grp ? i + 1 : i + 1 + ((int)gridDim.x - 1) * grp;
  };
  // QD dynamic order (A.qd_ctr): the list is cut into 8 contiguous ranges, one per XCD, and the waves of XCD x
  // (block % 8, the dispatch order the static map assumes as well) claim positions from range x's counter, one per
  // item, then from the other ranges once theirs is drained.  The items in flight on an XCD are then always a
  // window of consecutive positions, where the static stride lets blocks drift apart by many items over a persistent
  // grid (FETCH 1.25x algorithmic).  Measured slower (opt-in, PM_QD_DYN=1): a site's three items then start up to an
  // item apart on three waves, and the traffic rose to 1.50x (profiles/r06o_*).  A claim is issued one item before it is resolved (its return lands under that item's Brent, and
  // an extra vector-memory operation only makes the kernel's vmcnt waits stricter), so no wait is added; the
  // blocking claims are the steals at the end.  (Grids of whole XCD rounds only: the static positions need it.)
  const bool qdyn = QD && A.qd_ctr != nullptr && gridDim.x % 8 == 0;
  const int q_len = (itEnd - A.es_it0 + 7) / 8;
  int q_x = blockIdx.x & 7, q_tries = 0, q_pend = 0;
  bool q_pend_ok = false;
  auto q_issue = [&]() {   // a speculative claim on range q_x (lane 0's VGPR)
    int v = 0;
    if (threadIdx.x == 0) v = atomicAdd(A.qd_ctr + q_x, 1);
    return v;
  };
  // (a block's first two items are static -- range positions b / 8 and nb + b / 8, nb = blocks per XCD -- so the
  // claims count from 2 nb in the home range; a steal from another range counts from 2 nb as well, its static
  // positions belonging to that range's own blocks)
  const int q_nb = (int)gridDim.x / 8;
  auto q_resolve = [&](int v) {   // the claimed list position, or -1 once every range is drained
    int p = A.es_it0 + q_x * q_len + 2 * q_nb + __builtin_amdgcn_readfirstlane(v);
    while (p >= min(A.es_it0 + (q_x + 1) * q_len, itEnd)) {
      if (++q_tries >= 8) return -1;
      q_x = (q_x + 1) & 7;
      p = A.es_it0 + q_x * q_len + 2 * q_nb + __builtin_amdgcn_readfirstlane(q_issue());
    }
    return p;
  };
  auto q_next_pos = [&]() {   // resolve the pending claim, issue the next one
    const int p = q_pend_ok ? q_resolve(q_pend) : -1;
    q_pend_ok = p >= 0 && q_tries < 8;
    if (q_pend_ok) q_pend = q_issue();
    return p;
  };
  int it_first = A.es_it0 + vb * grp;
  int q_pos1 = -1, q_next = -1;   // QD: the list positions of the next item and of the one after the current
  if constexpr (QD) {
#pragma unroll
    for (int i = 0; i < 3; i++) qvoff[i] = quad_voff(i, A.n_person);
    if (qdyn) {   // (the static first two; a block whose first is past its range takes no item -- the claims of
                  // the blocks that do take items cover every other position, the steals included)
      const int lo = A.es_it0 + q_x * q_len, hi = min(lo + q_len, itEnd);
      it_first = lo + (int)blockIdx.x / 8 < hi ? lo + (int)blockIdx.x / 8 : itEnd;
      q_pos1 = lo + q_nb + (int)blockIdx.x / 8 < hi ? lo + q_nb + (int)blockIdx.x / 8 : -1;
    } else q_pos1 = next_it(it_first) < itEnd ? next_it(it_first) : -1;
    if (it_first < itEnd) {
      q_item = items[it_first];
      quad_aux(A.ref + ((q_item >> 3) & ~3), s_qaux);
      quad_prefetch(A, q_item, qvoff, qring);
      if (q_pos1 >= 0) quad_aux(items + q_pos1, s_qaux + 64);
      if (qdyn && q_pos1 >= 0) {   // the first claim (the block's third item), resolved one item from now
        q_pend_ok = true;
        q_pend = q_issue();
      }
    }
  }
  // QD: an item's results wait in LDS and are stored after the next item's hoisting, so that they are older
  // than that item's prefetch in vmcnt order
  __shared__ double s_pend[QD ? 2 : 1];
  __shared__ int s_pendi[QD ? 3 : 1];
  for (int it = it_first; it >= 0 && it < itEnd; it = QD ? q_next : next_it(it)) {
    if (A.phase) ph_t = wall_clock64();
    const int item = QD ? q_item : items[it];
    const int site = item >> 3, cfg = item & 7;
    int r;
    if constexpr (QD) {
      __builtin_amdgcn_s_waitcnt(PM_VMCNT(3 * QD_AHEAD));   // the ref dword has landed (the item's first slots and the next index may not)
      __builtin_amdgcn_sched_barrier(0);
      r = __builtin_amdgcn_readfirstlane(((const volatile __attribute__((address_space(3))) uint8_t*)s_qaux)[site & 3]);
    } else r = A.ref[site];
    ItemCtx I;
    item_alleles(A, site, cfg, r, &I.a1, &I.a2);
    if constexpr (QD) {   // (wave-uniform: the mutation-matrix rows are scalar operands even when the claims' atomics
                          // keep the cfg-7 result fields from being scalar loads)
      I.a1 = __builtin_amdgcn_readfirstlane(I.a1);
      I.a2 = __builtin_amdgcn_readfirstlane(I.a2);
    }
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
    constexpr int NC = POLY ? ((QD && PM_QD_NC4) ? 4 : 5) : 9;
    double cond[S][NC];
    double lm0 = 1.0;   // NC = 4: the lane's product of the families' a4 (hoist_quad_t)
    int le0 = 0;
    int fl[S];
    bool hoisted = false;
    if constexpr (POLY) {
      if constexpr (PFK) {
        if (pf) {
          __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): this wave's pieces of the item's planes have landed
          if constexpr (T > 64) __syncthreads();   // ... and the other waves' pieces
          hoist_poly4_lds<S, T, NF>(A, s_u, s_pf, s_lk, cond);
          __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): every read of the buffer is done ...
          if constexpr (T > 64) __syncthreads();   // ... by every wave of the block ...
          __builtin_amdgcn_sched_barrier(0);
          prefetch_planes(A, items, it + gridDim.x, nItems, s_pf);   // ... before the next item's planes overwrite it
          hoisted = true;
        }
      }
      if constexpr (QD) {
        hoist_quad<S, NC>(A, I, pl, s_lk, s_M, cond, qring, qvoff, lm0, le0);
        hoisted = true;
        const int itn = q_pos1;   // the next item's first slots land during this item's Brent
        q_next = itn;
        // (landed: the hoisting ended with vmcnt(0)); uniform, so the next site's addresses are scalar
        const int nitem = __builtin_amdgcn_readfirstlane(((const volatile __attribute__((address_space(3))) int*)s_qaux)[64]);
        // MonomorphismLogLikelihood_denovo (the cfg-0 item, CalcAllFamLogLikelihood at f = 1,
        // NucFamGenotypeLikelihood.cpp:1086-1132): SetParentPrior(1) keeps only geno11 x geno11, so each family
        // contributes F11 * M11 * Prod_kids CalcDenovoMutLk(geno11) (:1553-1562) -- exactly the f^4 coefficient a0 the
        // cfg-1 item (a1 = ref, geno11 = (ref, ref)) has just hoisted.  One product over the slots and lanes, one log10;
        // stored with the previous item's results (before the next prefetch in vmcnt order).
        double mono_dn = 0.0;
        const bool mdn = PM_QD_MONO && A.mono_dn == 2 && cfg == 1;
        if (mdn) {
          double m; int e;
          lane_poly_top<S, NC>((const double(*)[NC])cond, m, e, lm0, le0);
          mono_dn = block_logprod<T>(m, e, s_red, s_rede, par);
        }
        if (threadIdx.x == 0) {
          if (it != it_first) {
            const int ps = s_pendi[0], pc = s_pendi[1];
            A.raw[(size_t)ps * 8 + pc] = s_pend[0];
            A.minv[ps * 8 + pc] = s_pend[1];
            A.evals[ps * 8 + pc] = s_pendi[2];
          }
          if (mdn) { A.raw[(size_t)site * 8] = mono_dn; A.minv[site * 8] = 0.0; A.evals[site * 8] = 1; }
        }
        if (itn >= 0) {
          // the position after the next item (dynamic order: the pending claim, and the next claim issued before the DMA)
          const int itnn = qdyn ? q_next_pos() : (next_it(itn) < itEnd ? next_it(itn) : -1);
          __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): s_qaux has been read before the DMA refills it
          __builtin_amdgcn_sched_barrier(0);
          quad_aux(A.ref + ((nitem >> 3) & ~3), s_qaux);
          quad_prefetch(A, nitem, qvoff, qring);
          if (itnn >= 0) quad_aux(items + itnn, s_qaux + 64);
          q_item = nitem;
          q_pos1 = itnn;
        }
      }
      if constexpr (!QD) if (!PFK && !hoisted && A.max_nuc <= 4) {
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
      if constexpr (QD || EPO) continue;
      if (PFK || DNPF_ONLY || hoisted) continue;
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
    // EPR: the register families' degrees summed (the lane's power of g) and whether any family of the wave is
    // evaluated from the coefficient buffer instead (more than PM_EPE on a lane, or D > PDM)
    int edl = 0;
    bool epmem = true;
    // EP: the lane's extended families' coefficients, peeled for this item by k_es_hoist
    const double* coef = (ES && EP) ? A.es_coef + (size_t)(it - A.es_it0) * A.max_ext * A.poly_dcap * T + threadIdx.x : nullptr;
    if constexpr (ES && EP) {
      const int cnt = A.ext_count ? A.ext_count[threadIdx.x] : 0;
      bool mem = cnt > EPE;
#pragma unroll
      for (int q = 0; q < EPE; q++) {
        const double* co = coef + (size_t)q * A.poly_dcap * T;
        ed[q] = q < cnt ? (int)co[(size_t)(A.poly_dcap - 1) * T] : -1;
        if (ed[q] > PDM) { ed[q] = -1; mem = true; }
#pragma unroll
        for (int a = 0; a <= PDM; a++) ce[q][a] = a <= ed[q] ? co[(size_t)a * T] : 0.0;
        if (ed[q] < 0) ce[q][0] = 1.0;   // (an absent family: the unit polynomial, D = 0 -- the t-form loop is branch-free)
        edl += ed[q] < 0 ? 0 : ed[q];
      }
      if constexpr (EPE > 0) epmem = __ballot(mem) != 0;
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
          lane_poly_r<S, NC>(pos_div(x, g), (g * g) * (g * g), (const double(*)[NC])cond, m, e, lm0, le0);
          tot = block_logprod<T>(m, e, s_red, s_rede, par);
        } else {
          lane_poly_top<S, NC>((const double(*)[NC])cond, m, e, lm0, le0);   // x = 1: L = a0 per family, log10(x^4) = 0
          tot = block_logprod<T>(m, e, s_red, s_rede, par);
        }
      } else if (PROD) {
        double m = 1.0; int e = 0;
        if constexpr (!EPO)
          if (!(ES && EP && A.ep_only)) lane_prod<S, GEN>(x, unit, (const double(*)[9])cond, fl, pmode, m, e);
        if constexpr (ES && EP && EPE > 0) {   // register-resident coefficients first (independent Horner chains)
          const double g = 1 - x;
          if (__builtin_amdgcn_readfirstlane((int)(g > 0.0))) {
            // EPR: every family in the one direction L = g^D sum_a c_a t^a, t = f / g (t in [1e-4, 1e4] on Brent's
            // bracket; non-negative terms, no cancellation), by FMA Horner over the PDM + 1 registers (zeros above D
            // leave the sum's bits unchanged); g^D of all the lane's families as one power g^edl (edl <= 32).  The
            // t (one division) and the powers of g are shared by the lane's families.
            // (measured and rejected: the powers as one uniform D_total log10(g) added after the reduction -- the two
            // terms then cancel on flat objectives, whose rounding noise moves Brent's minimiser off the reference's)
            const double t = pos_div(x, g);
            double gp = g, pw = 1.0;
#pragma unroll
            for (int b = 0; b < 6; b++) {
              pw = ((edl >> b) & 1) ? pw * gp : pw;
              gp = gp * gp;
            }
            // each family's value split into mantissa and exponent first (independent), then one chain of products
            // of mantissas in [0.5, 1) (no under- or overflow) and one renormalisation: bit for bit the mantissa of
            // the renormalise-after-every-factor chain (scalings by 2^k are exact), with a shorter serial path
            double mq[EPE];
#pragma unroll
            for (int q = 0; q < EPE; q++) {
              double acc = ce[q][PDM];
#pragma unroll
              for (int a = PDM - 1; a >= 0; a--) acc = fma(acc, t, ce[q][a]);
              int e1;
              mq[q] = frexp(acc, &e1);   // (a peeled family's L can be ~1e-290)
              e += e1;
            }
#pragma unroll
            for (int q = 0; q < EPE; q++) m = m * mq[q];
            int e2;
            m = frexp(m * pw, &e2);
            e += e2;
          } else {   // f = 1 (the de novo monomorphism item): the f^D coefficient of each family
#pragma unroll
            for (int q = 0; q < EPE; q++)
              if (ed[q] >= 0) {
                int e1, e2;
                const double mv = frexp(es_poly_eval_r<PDM>(ce[q], ed[q], x), &e1);
                m = frexp(m * mv, &e2);
                e += e1 + e2;
              }
          }
        }
        if (ES && A.ext_count && (EPE == 0 || epmem))   // extended families of this lane: Elston-Stewart peeling per evaluation
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
      if (++iter > A.itmax) break;   // ITMAX: numerror("ScalarMinimizer::Brent got stuck")
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
      if (!ok) { atomicExch(&A.counts[5], 1); atomicMin(&A.counts[6], site); }   // (the reference stops at the first)
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

// (the kernels below are compiled in engine.hip only; brent_inst.hip builds just the k_brent instantiations above)
#ifndef PM_BRENT_PART
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
// spw (<= PREP_SPW) sites per wave, one after the other (a block of 4 waves takes 4 x spw consecutive sites), so the
// block-level work -- one returning atomic that reserves the block's Brent items (the sites' items then go to
// consecutive slots in site order) and at most 9 counter atomics -- is shared by 4 x spw sites.  (One
// same-address atomic per site serialised k_prep: 262 144 returning atomics on counts[0] per batch.)  spw is a
// launch argument (engine.hip: PREP_SPW unless PM_PREP_SPW says otherwise).
#define PREP_SPW 8
#ifndef PREP_UNROLL
#define PREP_UNROLL 4
#endif
// VC: vcf_mode engines -- no read depth or mapping quality (PedVCF / FamilyLikelihoodSeq_VCF): dm is neither read nor
// summed, the lanes sum only the hom-ref plane's PL bytes
// MDN: the de novo monomorphism product may be formed here (A.mono_dn == 1); false compiles that path out -- its ten
// planes' bytes per chunk set the register allocation (138 -> fewer VGPRs: more waves per SIMD for the latency-bound
// chunk loop)
template <int VEC, bool SERIAL, bool VC = false, bool MDN = true>
__global__ void __launch_bounds__(256) k_prep(DevArgs A, int spw) {
  __shared__ unsigned long long s_c[9];
  __shared__ double s_lk[256];
  __shared__ double s_M[100];
  __shared__ int s_nit[4 * PREP_SPW], s_pre[4 * PREP_SPW];   // items per site of the block (0: none), exclusive prefix
  __shared__ int s_base;
  if (threadIdx.x < 9) s_c[threadIdx.x] = 0;
  if (MDN && A.mono_dn == 1) {
    s_lk[threadIdx.x] = A.lktab[threadIdx.x];
    if (threadIdx.x < 100) s_M[threadIdx.x] = A.M[threadIdx.x];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // the list and the items of a called site (main.cpp:327-437 order: quick pre-filter, else the pedigree model)
  const int list = (A.vcf || !A.unrelated) ? 0 : 1;
  const int k0 = A.vcf ? 1 : A.unrelated ? 1 : (A.denovo && !A.mono_dn) ? 0 : 1;   // first cfg (cfg 0: de novo mono)
  const int nit_called = A.vcf ? 1 : A.unrelated ? 3 : 4 - k0;
  const int site0 = blockIdx.x * 4 * spw;
  for (int j = 0; j < spw; j++) {
    const int sl = w * spw + j, site = site0 + sl;
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
      // (mono_dn == 2: the cfg-1 QUAD item forms it instead; k_prep then reads only dm and the hom-ref plane)
      const bool mdn = MDN && A.mono_dn == 1 && okref;
      double dm_m = 1.0;
      int dm_e = 0;
      const uint8_t* plane_h = pl + (size_t)h * np;
      // one chunk of VEC persons per lane: the read statistics and the PL sum (SERIAL: the serial mono sum); hr keeps
      // the hom-ref PL bytes for the de novo monomorphism product
      auto chunk = [&](int p0, uint8_t* hr) {
        uint32_t x[VEC];
        if (p0 < np) {   // np % VEC == 0: a lane's VEC persons are all present or all absent
          if constexpr (!VC) load_dwords<VEC>(dm + p0, x);
          load_bytes<VEC>(plane_h + p0, hr);
        } else {
#pragma unroll
          for (int k = 0; k < VEC; k++) { x[k] = 0; hr[k] = 0; }
        }
        // a chunk's sums in 32 bits (VEC persons: depths < 2^24 each, mapping qualities and PL bytes < 2^8), widened once
        uint32_t cp = 0;
#pragma unroll
        for (int k = 0; k < VEC; k++) cp += hr[k];
        plsum += cp;
        if constexpr (!VC) {
          uint32_t cd = 0, cm = 0, cn = 0;
#pragma unroll
          for (int k = 0; k < VEC; k++) {
            const uint32_t d = x[k] & 0xFFFFFF;
            cd += d; cm += x[k] >> 24; cn += d > 0;
          }
          dsum += cd; mqsum += cm; nsd += cn;
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
      };
      if (!mdn) {
        // unrolled: the loads of PREP_UNROLL chunks in flight together (one HBM round trip per chunk made k_prep
        // latency-bound)
#pragma unroll PREP_UNROLL
        for (int base = 0; base < np; base += 64 * VEC) {
          uint8_t hr[VEC];
          chunk(base + lane * VEC, hr);
        }
      } else
        for (int base = 0; base < np; base += 64 * VEC) {
          const int p0 = base + lane * VEC;
          uint8_t hr[VEC];
          chunk(p0, hr);
          if (p0 < np) {
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
      // integer sums < 2^53 reduced as doubles on the DPP crossbar (exact in any order; no LDS round trips)
      if constexpr (!SERIAL) {
        plsum = (long long)wave_sum_exact((double)plsum);
        mono = plsum ? -(double)plsum / 10 : 0.0;
      }
      if (!A.vcf) {   // (the VCF path's read statistics are all zero)
        dsum = (long long)wave_sum_exact((double)dsum);
        mqsum = (long long)wave_sum_exact((double)mqsum);
        nsd = (long long)wave_sum_exact((double)nsd);
      }
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
      }
    }
    if (lane == 0) s_nit[sl] = valid ? nit_called : 0;
  }
  __syncthreads();
  if (threadIdx.x == 0) {   // the block's items: one reservation, then consecutive slots in site order
    int t = 0;
    for (int i = 0; i < 4 * spw; i++) { s_pre[i] = t; t += s_nit[i]; }
    s_base = t ? atomicAdd(&A.counts[list], t) : 0;
    for (int i = 0; i < 9; i++) if (s_c[i]) atomicAdd(&A.counters[i], s_c[i]);
  }
  __syncthreads();
  // lane i of wave w writes item i of each of its sites (at most 4 items per site)
  for (int j = 0; j < spw; j++) {
    const int sl = w * spw + j;
    if (lane < s_nit[sl]) A.items[list][s_base + s_pre[sl] + lane] = ((site0 + sl) << 3) | (lane + k0);
  }
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
// log10 guess g is within 1 of that count (its error is < 1e-4 on -10 log10 q <= 100): the count is g - 1 plus the
// two tests q < thr[g - 1], q < thr[g] (adjacent thresholds: one ds_read2, no loop, no branch), the window clamped
// to [0, 100).  Identical to the reference's glibc result for every double pb.
// The guess is the bare v_log_f32 (log2, ~1 ulp) times -10 log10(2): error < 1e-5 on the range that matters; a float
// q below the normal range (where the bare instruction may read 0: +inf guess) has pb > 0.9999999999, GQ 100 anyway,
// so none of the library log10's denormal scaling and extended-precision product is needed (8 VALU instead of 16).
static __constant__ double c_gq_thr[101];   // (uploaded by engine.hip, the only unit whose kernels read it)
// (thr: the block's LDS copy of c_gq_thr -- the lookups' index diverges, so they are not scalar loads)
__device__ __forceinline__ int d_gq(double pb, const double* thr) {
  const double q = 1. - pb;
  const int g = (int)(-3.01029995664f * __builtin_amdgcn_logf((float)q) + 0.5f);   // (q = 0: +inf saturates; the select below wins)
  const int base = min(max(g - 1, 0), 98);
  const int k = base + (q < thr[base] ? 1 : 0) + (q < thr[base + 1] ? 1 : 0);
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

#ifndef PM_POST_ZINIT
#define PM_POST_ZINIT 1   // lean_nuc_post's kid sums start from their first term (0: from 0.0, the former code)
#endif
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
    // PM_POST_ZINIT: each sum starts from its first term instead of 0.0 + term (every term is +0 or positive, so
    // 0.0 + v == v bit for bit; the compiler may not drop the add itself without no-signed-zeros)
    bool h[3] = {!PM_POST_ZINIT, !PM_POST_ZINIT, !PM_POST_ZINIT};
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
      if (!z11) { const double v = (two ? q11 * lo : q11) * w; g[0] = h[0] ? g[0] + v : v; h[0] = true; }
      if (!z12) { const double v = (two ? q12 * lo : q12) * w; g[1] = h[1] ? g[1] + v : v; h[1] = true; }
      if (!z22) { const double v = (two ? q22 * lo : q22) * w; g[2] = h[2] ? g[2] + v : v; h[2] = true; }
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
#ifndef PM_POST_WAVES
#define PM_POST_WAVES 0   // k_posterior_lean: minimum waves per SIMD the register allocation must allow (0: the compiler's)
#endif
#if PM_POST_WAVES > 0
#define PM_POST_WPE __attribute__((amdgpu_waves_per_eu(PM_POST_WAVES)))
#else
#define PM_POST_WPE
#endif
template <bool VCF>
__global__ void __launch_bounds__(256) PM_POST_WPE k_posterior_lean(DevArgs A) {
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
#endif  // PM_BRENT_PART
