// engine.hip -- host side of the MI355X (gfx950) engine (pm_engine_*, the C ABI of include/polymutt_engine.h) and the
// non-Brent kernels' instantiations.  The device code is in engine_dev.h; the k_brent instantiations are compiled in
// separate units (brent_inst.hip, one object per PM_BRENT_PART) and declared extern here (brent_variants.h).
#include "engine_dev.h"
#include "brent_variants.h"

#define PM_BRENT_X(part, ...) extern template __global__ void k_brent<__VA_ARGS__>(DevArgs, int);
PM_BRENT_VARIANTS
#undef PM_BRENT_X

// ------------------------------------------------------------------------------------------------
// error reporting (thread-local, C ABI)
static thread_local std::string g_last_error;
extern "C" void pm_set_last_error(const char* msg) { g_last_error = msg ? msg : ""; }
extern "C" const char* pm_last_error(void) { return g_last_error.c_str(); }
extern "C" int pm_abi_version(void) { return PM_ABI_VERSION; }
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
  // pm_engine_submit / pm_engine_collect: the batch in flight, its results and counts landing in page-locked memory
  pm_site_result* h_res = nullptr;
  int* h_counts = nullptr;
  int pending_n = -1;
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
  int ep_dmax[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
  int itmax = 200;          // ScalarMinimizer::Brent's ITMAX (core/MathGold.cpp:98); PM_TEST_ITMAX lowers it (tests)
  int stuck_site = -1;      // the last finished batch's first site whose Brent hit ITMAX (pm_engine_stuck_site)   // [plan][class]: the largest polynomial degree of a peeled family
  int hoist_tmp = 0, hoist_waves = 4, es_chunk = 0;   // k_es_hoist: step temporaries per wave, waves per block, items per launch
  double* d_es_coef = nullptr;                        // [es_chunk][max_ext][poly_dcap][T] hoisted coefficients
  unsigned long long* d_es_prof = nullptr;            // PM_ES_PROF: es_hoist_wave cycles by part
  // the schedule compiler (es_jit.h): per plan (0, 1) and chromosome class, built on first use (0 untried, 1 ok, -1 failed)
  std::vector<int> ext_fam_h, ext_fam1_h, peel_start_h;
  std::vector<int2> steps_h;
  std::vector<int8_t> founder_h;
  std::vector<int> fam_founders_h;
  pmjit::Kernel jit[2][4];
  int jit_state[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
  int* d_jit_slots[2][4] = {{nullptr, nullptr, nullptr, nullptr}, {nullptr, nullptr, nullptr, nullptr}};   // e | sig | p0
  // the fused hoisting + Brent kernel (es_jit.h ep_brent_jit) per plan and class: 0 not tried, 1 built, -1 unavailable
  pmjit::FusedKernel fused[2][4];
  int fused_state[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
  int* d_fused_tab[2][4] = {{nullptr, nullptr, nullptr, nullptr}, {nullptr, nullptr, nullptr, nullptr}};
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
  int quad_bpc16 = 0, quad_bpc8 = 0;   // QUAD k_brent blocks resident per CU (occupancy query, first launch)
  bool units_empty = false, units1_empty = false;   // a lane plan with no nuclear or founder unit (every family peeled)
  std::vector<std::pair<const void*, int>> ep_bpc;   // EP one-wave k_brent blocks resident per CU, per instantiation
  bool all_trio = false;   // every unit of the lane plan is a 3-person nuclear family (or empty): k_brent's NF = 3
  bool split34 = false;    // plan_split34: quads in the first half of the slot rows, trios in the second (NF = 34)
  int4* d_units_q = nullptr;
  int* d_items[N_LISTS] = {nullptr, nullptr, nullptr};
  int* d_counts = nullptr;
  int* d_qctr = nullptr;     // QUAD dynamic item order: 8 per-XCD claim counters (k_brent DevArgs::qd_ctr)
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
  std::vector<std::pair<hipEvent_t, hipEvent_t>> es_events;   // the EP hoisting launches (schedule compiler or k_es_hoist)
  double es_item_ops[6] = {0, 0, 0, 0, 0, 0};   // FP64 ops of one item's hoisting over the lane plan's extended families, by variant
  bool es_grouped = false;             // es_hoist_wave tasks are a site's de novo items (the leaf steps taken once)
  bool es_ops_known = false;           // (the compiled kernels report them; the generic k_es_hoist does not)
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
// a persistent grid rounded down to whole rounds of the 8 XCDs (the kernels' XCD-aware item order needs gridDim % 8 == 0;
// they fall back to plain order otherwise), never below one block
static int xcd_grid(int g) { return g >= 8 ? g - g % 8 : std::max(g, 1); }
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

// Split plan for pedigrees of trios and quads only (config 5's 2000 mixed families): quads dealt round-robin over the lanes
// of slot rows [0, S/2), trios over rows [S/2, S), so the lean PF kernel hoists each half with its family size known
// (k_brent NF = 34).  false when either kind does not fit its half.
static bool plan_split34(const pm_pedigree* ped, int T, int S, std::vector<int4>& units) {
  if (S < 2 || S % 2) return false;
  units.assign((size_t)T * S, make_int4(U_NONE, -1, 0, 0));
  int nq = 0, nt = 0;
  for (int f = 0; f < ped->n_fam; f++) {
    const int p0 = ped->fam_start[f], n = ped->fam_start[f + 1] - p0;
    if (ped->fam_kind[f] != PM_FAM_NUCLEAR || (n != 3 && n != 4)) return false;
    int& c = n == 4 ? nq : nt;
    const int row = (n == 4 ? 0 : S / 2) + c / T;
    if (c / T >= S / 2) return false;
    units[(size_t)row * T + c % T] = make_int4(U_NUC, f, p0, n);
    c++;
  }
  return nq > 0 && nt > 0;
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
static const double kTBA[5][27] = PM_TBA_VALUES;

extern "C" {

void pm_engine_destroy(pm_engine* E) {
  if (!E) return;
  hipSetDevice(E->device);
  if (E->d_es_prof) {
    unsigned long long h[5] = {0, 0, 0, 0, 0};
    if (hipMemcpy(h, E->d_es_prof, sizeof(h), hipMemcpyDeviceToHost) == hipSuccess && (h[0] | h[1] | h[2] | h[3] | h[4]))
      fprintf(stderr, "PM_ES_PROF wave-cycles pen %llu toprest %llu leaf %llu rest %llu whole %llu\n", h[0], h[1], h[2], h[3], h[4]);
    (void)hipFree(E->d_es_prof);
  }
  void* bufs[] = {E->d_units1, E->d_ext_count1, E->d_ext_fam1, E->d_fam_founders, E->d_peel_start, E->d_ext_count, E->d_ext_fam, E->d_is_founder, E->d_steps, E->d_T10,
                  E->d_T10dn, E->d_ws, E->d_tba, E->d_units_q, E->d_poly_start, E->d_poly_lay, E->d_poly_deg, E->d_es_coef, E->d_es_pers, E->d_es_pers1, E->d_fam_perm,
                  E->d_fam_start, E->d_fam_kind, E->d_fa, E->d_mo, E->d_sex, E->d_units, E->d_lktab, E->d_M, E->d_syn,
                  E->d_pl, E->d_stage, E->d_ref, E->d_dm, E->d_res, E->d_calls, E->d_raw, E->d_minv, E->d_mono, E->d_evals,
                  E->d_items[0], E->d_items[1], E->d_items[2], E->d_counts, E->d_eval_total, E->d_row_site,
                  E->d_counters, E->d_row_blk, E->d_qctr};
  for (void* b : bufs) if (b) hipFree(b);
  for (auto& pl : E->d_jit_slots)
    for (int* b : pl) if (b) hipFree(b);
  for (auto& pl : E->d_fused_tab)
    for (int* b : pl) if (b) hipFree(b);
  for (auto& pr : E->brent_events) { hipEventDestroy(pr.first); hipEventDestroy(pr.second); }
  for (auto& pr : E->es_events) { hipEventDestroy(pr.first); hipEventDestroy(pr.second); }
  if (E->h_res) hipHostFree(E->h_res);
  if (E->h_counts) hipHostFree(E->h_counts);
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
  if (const char* s = getenv("PM_TEST_ITMAX"); s && atoi(s) > 0) E->itmax = std::min(200, atoi(s));
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
  // --- Elston-Stewart schedules and their polynomial-form layouts first: whether the polynomial form is usable
  // (es_poly) decides how many extended families a lane of the plan may hold
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
  auto fam_deg = [&](int f, int c) {   // the polynomial degree of family f in chromosome class c (0: no layout)
    return poly_start[f + 1] > poly_start[f] ? poly_lay[poly_start[f] + 2 + c] : 0;
  };
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
    // (--denovo too: the 10-state peels are hoisted by the schedule compiler's es_hoist_wave, and k_brent only
    // evaluates their coefficients; the reference-order 10-state peel of PRODUCT / EXACT numerics keeps one per lane)
    // (PM_EP_DN_ONE=1: one per lane under --denovo -- an experiment switch)
    const int per_lane = (E->es_poly && !(par->denovo && getenv("PM_EP_DN_ONE"))) ? PM_EPE : 1;
    int tmin = 1;
    while (tmin < std::min((E->n_ext + per_lane - 1) / per_lane, 256)) tmin *= 2;
    const int npref = gen ? 9 : 8;
    for (int i = 0; i < npref && !planned; i++)
      if (pref[i].x >= tmin && plan_units(ped, pref[i].x, pref[i].y, units)) { E->T = pref[i].x; E->S = pref[i].y; planned = true; }
  }
  if (!planned) { pm_engine_destroy(E); pm_set_last_error("pm_engine_create: pedigree too large for the lane plan"); return PM_EPED; }
  // mixed trio / quad pedigrees on the lean one- or two-wave 16-slot plans: the split layout (PM_NO_SPLIT34=1: off)
  if (!par->denovo && par->numerics == PM_NUM_POLY && !E->has_fp && E->n_ext == 0 && E->S == 16 && (E->T == 64 || E->T == 128) &&
      !getenv("PM_NO_SPLIT34")) {
    std::vector<int4> u2;
    if (plan_split34(ped, E->T, E->S, u2)) { units.swap(u2); E->split34 = true; }
  }
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
  E->units_empty = std::all_of(units.begin(), units.end(), [](const int4& u) { return u.x == U_NONE; });
  E->all_trio = !E->units_empty &&
                std::all_of(units.begin(), units.end(), [](const int4& u) { return u.x == U_NONE || (u.x == U_NUC && (u.w & 0xFF) == 3); });
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
    if (E->es_poly)
      for (int f = 0; f < ped->n_fam; f++)
        for (int c = 0; c < 4; c++) {
          if (ped->fam_kind[f] == PM_FAM_EXTENDED) E->ep_dmax[0][c] = std::max(E->ep_dmax[0][c], fam_deg(f, c));
          if (ped->fam_kind[f] != PM_FAM_FOUNDERS) E->ep_dmax[1][c] = std::max(E->ep_dmax[1][c], fam_deg(f, c));
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
        E->units1_empty = std::all_of(u1.begin(), u1.end(), [](const int4& u) { return u.x == U_NONE; });
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
      // hoisted coefficients of a chunk of items: every item a batch can enqueue in one list (4 per site, rounded up
      // to whole 12-item groups), <= 4 GiB.  launch_brent runs hoisting + Brent once per chunk of the list's largest
      // possible item count (4 per site), so a chunk even 4 items short of it costs an extra pair of launches per
      // list over items that do not exist (config 4's 16 384-site batches: 65 532-item chunks for 65 536, two empty
      // pairs per step).  PM_ES_CHUNK = items per chunk caps it (experiments).
      const size_t per_item = (size_t)std::max({E->max_ext * E->T, E->max_ext1 * std::max(1, E->T1), 1}) * E->poly_dcap * sizeof(double);
      const size_t want = ((size_t)4 * std::max(1, max_batch) + 11) / 12 * 12;
      E->es_chunk = (int)std::max<size_t>(1, std::min<size_t>(want, ((size_t)1 << 32) / per_item));
      if (const char* s = getenv("PM_ES_CHUNK"); s && atoi(s) > 0) E->es_chunk = std::min(E->es_chunk, atoi(s));
      if (E->es_chunk >= 12) E->es_chunk -= E->es_chunk % 12;   // whole sites of lists 0 and 1 per chunk (grouped tasks)
      // (a full-batch chunk that does not fit -- several engines per GPU, a smaller device -- falls back to the 1 GiB
      // chunk: launch_brent loops over chunks)
      if (dalloc(&E->d_es_coef, (size_t)E->es_chunk * per_item / sizeof(double)) != PM_OK) {
        (void)hipGetLastError();
        E->es_chunk = (int)std::max<size_t>(1, std::min<size_t>(E->es_chunk, ((size_t)1 << 30) / per_item));
        if (E->es_chunk >= 12) E->es_chunk -= E->es_chunk % 12;
        DALLOC(E->d_es_coef, (size_t)E->es_chunk * per_item / sizeof(double));
      }
    }
    // workspace: the Brent grids and the posterior grid are capped so each needs <= 1 GiB
    E->grid_post = E->n_cu * 8;
    if (wsmax > 0) {
      const size_t cap = (size_t)1 << 30, per_lane = (size_t)wsmax * sizeof(double);
      const size_t per_lane_b = (size_t)wsmax * sizeof(double);   // Brent grids (EP kernels use no workspace: k_es_hoist)
      E->grid_brent = (int)std::max<size_t>(E->n_cu, std::min<size_t>(E->grid_brent, cap / (per_lane_b * T)));
      E->grid_brent = xcd_grid(E->grid_brent);   // keep the XCD-aware item order exact
      if (E->T1) {
        E->grid1 = (int)std::max<size_t>(E->n_cu, std::min<size_t>(E->grid1, cap / (per_lane_b * E->T1)));
        E->grid1 = xcd_grid(E->grid1);
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
  DALLOC(E->d_qctr, 8);
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
  A.itmax = E->itmax;
  A.qd_ctr = nullptr;
  // (the QUAD plan's cfg-1 items form it from their hoisting: launch_brent takes the QUAD kernel for list 0 exactly when
  // E->quad and the plan is 64 x 8 / 64 x 16, and mono_dn_in_prep already implies the lean --denovo kernel)
  A.mono_dn = !mono_dn_in_prep(E) ? 0 : (E->quad && E->T == 64 && (E->S == 8 || E->S == 16) && !getenv("PM_MONO_DN_PREP")) ? 2 : 1;
  return A;
}

typedef void (*BrentFn)(DevArgs, int);
// numerics: PM_NUM_PRODUCT / PM_NUM_EXACT for every flavour; PM_NUM_POLY only for the lean kernel
// (the generic and ES flavours fall back to PRODUCT numerics).
// pd_hi: the plan's peeled families reach a polynomial degree above PM_PD_LO (one-wave EP plans then take the
// PM_PD_HI register tile; degrees above that are evaluated from the coefficient buffer)
static BrentFn brent_kernel(int T, int S, int num, bool gen, bool es, bool dn = false, bool pf = false, bool ep = false, bool trio = false,
                            bool epo = false, bool pd_hi = false, bool split34 = false) {
  const int n = (num == PM_NUM_POLY && gen) ? PM_NUM_PRODUCT : num;
  if (es && ep && epo && T == 64 && (S == 1 || S == 2 || S == 4)) {   // ep_only plans: the nuclear machinery compiled out
#define PMKEO(s) \
  if (S == s && pd_hi) return dn ? k_brent<64, s, PM_NUM_PRODUCT, true, true, true, false, true, false, 1, PM_PD_HI> \
                                 : k_brent<64, s, PM_NUM_PRODUCT, true, true, false, false, true, false, 1, PM_PD_HI>; \
  if (S == s) return dn ? k_brent<64, s, PM_NUM_PRODUCT, true, true, true, false, true, false, 1> \
                        : k_brent<64, s, PM_NUM_PRODUCT, true, true, false, false, true, false, 1>;
    PMKEO(1) PMKEO(2) PMKEO(4)
#undef PMKEO
  }
  if (es && ep && pd_hi && T == 64) {
#define PMKEH(s) \
  if (S == s) return dn ? k_brent<64, s, PM_NUM_PRODUCT, true, true, true, false, true, false, 0, PM_PD_HI> \
                        : k_brent<64, s, PM_NUM_PRODUCT, true, true, false, false, true, false, 0, PM_PD_HI>;
    PMKEH(1) PMKEH(2) PMKEH(4) PMKEH(8)
#undef PMKEH
  }
  if (es && ep) {   // extended families in polynomial form (PM_NUM_POLY); DN: with the 10-state (--denovo) hoisting
#define PMKEP(t, s) \
  if (T == t && S == s) return dn ? k_brent<t, s, PM_NUM_PRODUCT, true, true, true, false, true> : k_brent<t, s, PM_NUM_PRODUCT, true, true, false, false, true>;
    PMKEP(64, 1) PMKEP(64, 2) PMKEP(64, 4) PMKEP(64, 8) PMKEP(256, 1) PMKEP(256, 4) PMKEP(512, 4) PMKEP(1024, 4) PMKEP(1024, 8)
#undef PMKEP
    return nullptr;
  }
  if (dn && !gen && !es && n == PM_NUM_POLY && pf && T == 64 && S == 16)   // lean --denovo, LDS-staged hoisting only
    return k_brent<64, 16, PM_NUM_POLY, false, false, true, true>;
  if (pf && !dn && split34 && S == 16) {   // mixed trio / quad split plans
    if (T == 64) return k_brent<64, 16, PM_NUM_POLY, false, false, false, true, false, false, 34>;
    if (T == 128) return k_brent<128, 16, PM_NUM_POLY, false, false, false, true, false, false, 34>;
  }
  if (pf && !dn) {   // lean autosomal kernel with LDS plane prefetch
#define PMKP(s) if (T == 64 && S == s) return trio ? k_brent<64, s, PM_NUM_POLY, false, false, false, true, false, false, 3> \
                                                   : k_brent<64, s, PM_NUM_POLY, false, false, false, true>;
    PMKP(1) PMKP(2) PMKP(4) PMKP(8) PMKP(16)
#undef PMKP
    if (T == 128 && S == 16)   // 1025-2048 families
      return trio ? k_brent<128, 16, PM_NUM_POLY, false, false, false, true, false, false, 3> : k_brent<128, 16, PM_NUM_POLY, false, false, false, true>;
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

// The extended families of the current plan as the schedule compiler sees them (slot order e = q * T + lane).
static std::vector<pmjit::Family> jit_families(const pm_engine* E, int plan) {
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
  return fams;
}

// The schedule compiler's kernels for the current plan and chromosome class (es_jit.h), built on first use; nullptr
// when it is off (PM_NO_JIT) or failed to build (then the generic k_es_hoist / k_posterior_es run).
static const pmjit::Kernel* jit_kernel(pm_engine* E) {
  const int plan = E->use_plan1 ? 1 : 0, cls = E->chrom;
  if (!E->es_poly || getenv("PM_NO_JIT")) return nullptr;
  int& st = E->jit_state[plan][cls];
  if (st == 0) {
    st = -1;
    const std::vector<pmjit::Family> fams = jit_families(E, plan);
    std::string err;
    pmjit::Kernel& K = E->jit[plan][cls];
    // (--denovo outside vcf_mode: every de novo item is hoisted in a grouped task, launch_brent)
    const int dmode = !E->par.denovo ? 0 : (!E->vcf && !getenv("PM_ES_NOGROUP")) ? 2 : 1;
    if (!fams.empty() && pmjit::build(E->device, cls, fams, kTBA, dmode, &K, &err)) {
      const size_t ns = K.slot_e.size();
      std::vector<int> tab(3 * ns + K.pair_k.size());   // slot_e | slot_sig | slot_p0 | pair_k (pair mode)
      for (size_t i = 0; i < ns; i++) { tab[i] = K.slot_e[i]; tab[ns + i] = K.slot_sig[i]; tab[2 * ns + i] = K.slot_p0[i]; }
      std::copy(K.pair_k.begin(), K.pair_k.end(), tab.begin() + 3 * ns);
      if (dalloc(&E->d_jit_slots[plan][cls], tab.size()) == PM_OK &&
          hipMemcpy(E->d_jit_slots[plan][cls], tab.data(), sizeof(int) * tab.size(), hipMemcpyHostToDevice) == hipSuccess)
        st = 1;
    } else if (!fams.empty())
      fprintf(stderr, "polymutt: peeling-schedule compiler unavailable (%s); using the generic hoisting kernel\n", err.c_str());
  }
  return st == 1 ? &E->jit[plan][cls] : nullptr;
}

// The fused hoisting + Brent kernel for the current plan and class (bi-allelic engines, every family peeled), built on
// first use; nullptr when off (PM_NO_FUSED, PM_NO_JIT) or unavailable (then es_hoist_jit + k_brent run).
static const pmjit::FusedKernel* fused_kernel(pm_engine* E) {
  const int plan = E->use_plan1 ? 1 : 0, cls = E->chrom;
  if (!E->es_poly || getenv("PM_NO_JIT") || getenv("PM_NO_FUSED")) return nullptr;
  int& st = E->fused_state[plan][cls];
  if (st == 0) {
    st = -1;
    const std::vector<pmjit::Family> fams = jit_families(E, plan);
    std::string err;
    pmjit::FusedKernel& F = E->fused[plan][cls];
    if (!fams.empty() && pmjit::build_fused(E->device, cls, fams, kTBA, &F, &err) && F.blocks_per_cu > 0) {
      if (dalloc(&E->d_fused_tab[plan][cls], F.lane_tab.size()) == PM_OK &&
          hipMemcpy(E->d_fused_tab[plan][cls], F.lane_tab.data(), sizeof(int) * F.lane_tab.size(), hipMemcpyHostToDevice) == hipSuccess)
        st = 1;
    } else if (!fams.empty() && getenv("PM_JIT_LAYOUT"))
      fprintf(stderr, "polymutt: fused Brent kernel unavailable (%s); hoisting + k_brent\n", err.c_str());
  }
  return st == 1 ? &E->fused[plan][cls] : nullptr;
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
    A.pf_stride = A.pf_npad + 16;
    A.pf_dw = al16 ? 0 : 1;
    shmem = (size_t)3 * A.pf_stride;
  }
  // lean --denovo kernel: QUAD plans load each family's PL dwords directly (hoist_quad); other plans stage the PL
  // windows through LDS by LDS-DMA (double buffer per wave)
  A.dn_pf = 0;
  A.quad_full = E->quad_full;
  const bool quad = !gen && !unrelated && n_ext == 0 && A.denovo && E->par.numerics == PM_NUM_POLY && E->quad && T == 64 &&
                    (S == 8 || S == 16);
  if (quad) shmem = QWAVE;
  // QUAD: list 0 holds cfgs 1-3 of each called site and list 1 cfgs 4-6, consecutive and site-aligned (k_prep / k_select
  // reserve them three at a time): one wave takes a site's three in turn (PM_QD_GROUP=1: one item per step of the grid)
  A.qd_group = 1;
  if (quad && A.mono_dn == 2 && (list == 0 || list == 1)) {
    const char* eg = getenv("PM_QD_GROUP");
    A.qd_group = eg ? std::max(1, atoi(eg)) : 1;
    if (A.qd_group != 1 && A.qd_group != 3) A.qd_group = 3;
  }
  BrentFn qfn = nullptr;
  if (quad) {   // persistent grid = the blocks that are resident at once (PM_QD_WAVES per SIMD): no partial second round
    qfn = S == 16 ? k_brent<64, 16, PM_NUM_POLY, false, false, true, false, false, true>
                  : k_brent<64, 8, PM_NUM_POLY, false, false, true, false, false, true>;
    int& bpc = S == 16 ? E->quad_bpc16 : E->quad_bpc8;
    if (bpc == 0) {
      int n = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, (const void*)qfn, 64, shmem) != hipSuccess || n <= 0) {
        (void)hipGetLastError();
        n = 1024 / 64;
      }
      bpc = n;
      if (getenv("PM_QD_BPC")) bpc = std::max(1, atoi(getenv("PM_QD_BPC")));
    }
    // PM_QD_ROUNDS = R rounds of the resident blocks (default 1): a block then takes 1 / R of the items it takes in a
    // persistent grid, so the three items of a site -- started together on neighbouring blocks of one XCD -- drift
    // apart by fewer items and find the site's planes still in that XCD's L2: FETCH per dispatch 4.81 GB at R = 1, 4.24
    // at 2, 4.00 at 4, 3.96 at 8 (3.85 algorithmic), k_brent 3.19 -> 2.98 ms on one engine (profiles/r06l_*); but the
    // default three engines then interleave their launches' blocks on every XCD and the bench's wall rate drops 1.5%
    // (r06n_*), so R = 1 stays.  PM_QD_DYN=1: the per-XCD claimed item order (k_brent qd_ctr; slower, r06o_*).
    const char* ed = getenv("PM_QD_DYN");
    const bool dyn = ed && atoi(ed) != 0 && A.qd_group == 1;
    if (dyn) {
      HIP_TRY(hipMemsetAsync(E->d_qctr, 0, 8 * sizeof(int), E->stream));
      A.qd_ctr = E->d_qctr;
    }
    const char* er = getenv("PM_QD_ROUNDS");
    const int rounds = getenv("PM_QD_BPC") ? 1 : er ? std::max(1, atoi(er)) : 1;
    grid = E->n_cu * bpc * rounds;
    grid = xcd_grid(grid);   // (the XCD-aware item order)
  }
  if (!quad && !gen && !unrelated && n_ext == 0 && A.denovo && E->par.numerics == PM_NUM_POLY && E->max_nuc <= 4 && S % DN_PF_C == 0 &&
      E->n_person % 16 == 0 && E->n_person >= 16 && !getenv("PM_NO_PREFETCH")) {
    A.dn_pf = 1;
    shmem = (size_t)(T / 64) * 2 * DN_PF_BUF;
  }
  const bool ep = !unrelated && n_ext > 0 && E->es_poly && E->par.numerics == PM_NUM_POLY;
  const bool ep_only = ep && (E->use_plan1 ? E->units1_empty : E->units_empty) && !getenv("PM_NO_EP_ONLY");
  BrentFn fn = quad ? qfn
                   : brent_kernel(T, S, E->par.numerics, gen, !unrelated && n_ext > 0, A.denovo != 0, A.pf_npad > 0 || A.dn_pf, ep,
                                  E->all_trio && !unrelated && !getenv("PM_NO_TRIO"), ep_only && !getenv("PM_NO_EPO"),
                                  ep && E->ep_dmax[E->use_plan1 ? 1 : 0][E->chrom] > PM_PD_LO && !getenv("PM_NO_PD_HI"),
                                  E->split34 && !gen && !unrelated && !E->use_plan1);
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
    A.ep_only = ep_only;
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
  if (ep && T == 64) {   // EP one-wave plans: a persistent grid of exactly the resident blocks (no partial second round)
    int bpc = 0;
    for (auto& c : E->ep_bpc)
      if (c.first == (const void*)fn) bpc = c.second;
    if (bpc == 0) {
      int n = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, (const void*)fn, T, shmem) != hipSuccess || n <= 0) {
        (void)hipGetLastError();
        n = 1024 / T;
      }
      bpc = n;
      E->ep_bpc.push_back({(const void*)fn, n});
    }
    grid = std::min(grid, E->n_cu * bpc);
    grid = xcd_grid(grid);
  }
  // lean PF kernels: PM_PF_ROUNDS x the default grid (2 rounds of the resident blocks).  One-wave quad plans take 4 (8
  // rounds): less drift between the items of a site, so its planes are re-read from L2 (plain quads 27.7 -> 28.7 M
  // sites/s, k_brent frac 0.725 -> 0.76, profiles/r06m_*).  Trio plans lost 2% of wall rate with it (frac 0.70 -> 0.72:
  // the engines' launches interleave, r06p_*) and the two-wave 128 x 16 plans (config 5) gained nothing: 1
  if (A.pf_npad > 0 && !ep) {
    const char* epr = getenv("PM_PF_ROUNDS");
    const int r = epr ? std::max(1, atoi(epr)) : (T == 64 && !E->all_trio) ? 4 : 1;
    grid = xcd_grid(grid * r);
  }
  // HIP events around every Brent launch (and, for EP, every hoisting launch: pm_kernel_stats reports the two apart)
  auto mark = [&](std::vector<std::pair<hipEvent_t, hipEvent_t>>& v, bool begin) -> int {
    if (begin) {
      hipEvent_t a, b;
      HIP_TRY(hipEventCreate(&a));
      HIP_TRY(hipEventCreate(&b));
      v.push_back({a, b});
      HIP_TRY(hipEventRecord(a, E->stream));
    } else HIP_TRY(hipEventRecord(v.back().second, E->stream));
    return PM_OK;
  };
  int mrc;
  // bi-allelic engines whose every family is peeled (config 4): one fused launch per list -- each lane hoists its
  // families' polynomials into registers and the wave runs the item's Brent (es_jit.h ep_brent_jit)
  const pmjit::FusedKernel* FK = (ep && ep_only && !A.denovo && T == 64) ? fused_kernel(E) : nullptr;
  if (FK) {
    E->es_ops_known = true;   // (finish_batch: every item is bi-allelic, o[0] = one item's hoisting over every family)
    for (int v = 0; v < 6; v++) E->es_item_ops[v] = v == 0 ? FK->item_ops : 0.0;
    const int plan = E->use_plan1 ? 1 : 0;
    pmjit::FusedArgs F;
    F.items = A.items[list]; F.counts = A.counts; F.ref = A.ref; F.res = (const int*)A.res; F.pl = A.pl; F.lktab = A.lktab;
    F.lane_tab = E->d_fused_tab[plan][E->chrom];
    F.raw = A.raw; F.minv = A.minv; F.evals = A.evals; F.eval_total = A.eval_total;
    F.precision = A.precision;
    F.list = list; F.it0 = 0; F.it1 = INT_MAX; F.np = A.n_person; F.vcf = A.vcf; F.res_words = sizeof(pm_site_result) / 4;
    F.res_a1 = offsetof(pm_site_result, allele1) / 4; F.res_a2 = offsetof(pm_site_result, allele2) / 4;
    F.itmax = A.itmax; F.pad = 0;
    void* params[] = {&F};
    if ((mrc = mark(E->brent_events, true))) return mrc;
    const char* efr = getenv("PM_FUSED_ROUNDS");   // (rounds of the resident blocks: measured)
    const int frounds = efr ? std::max(1, atoi(efr)) : 1;
    HIP_TRY(hipModuleLaunchKernel(FK->fn, xcd_grid(E->n_cu * FK->blocks_per_cu * frounds), 1, 1, 64, 1, 1, 0, E->stream, params,
                                  nullptr));
    if ((mrc = mark(E->brent_events, false))) return mrc;
  } else if (ep) {   // chunks of the list (the coefficient buffer holds es_chunk items): k_es_hoist, then the chunk's Brent items
    void (*hoist)(DevArgs, int) = A.denovo ? k_es_hoist<true> : k_es_hoist<false>;
    const size_t hlds = (size_t)E->hoist_waves * (E->poly_coef + E->hoist_tmp) * sizeof(double);
    if (hlds > 64 * 1024) HIP_TRY(hipFuncSetAttribute((const void*)hoist, hipFuncAttributeMaxDynamicSharedMemorySize, (int)hlds));
    const size_t stat = (256 + 5 * 27 + (A.denovo ? 2000 : 2)) * sizeof(double);
    const int hgrid = E->n_cu * std::max(1, std::min(8, (int)((160 * 1024) / (hlds + stat))));
    const int max_items = 4 * E->last_n;
    const pmjit::Kernel* K = jit_kernel(E);
    E->es_ops_known = K != nullptr;
    if (K) {   // one item's hoisting ops over the plan's extended families (slot shapes), by variant
      for (int v = 0; v < 6; v++) {
        E->es_item_ops[v] = 0;
        for (int sg : K->slot_sig) E->es_item_ops[v] += K->shape_ops[v].empty() ? 0.0 : K->shape_ops[v][sg];
      }
    }
    for (int it0 = 0; it0 < max_items; it0 += E->es_chunk) {
      A.es_it0 = it0;
      A.es_it1 = (int)std::min<long long>((long long)it0 + E->es_chunk, INT_MAX);
      if ((mrc = mark(E->es_events, true))) return mrc;
      if (K) {   // compiled schedule: one thread (--denovo: one wave) per (item, family)
        const int plan = E->use_plan1 ? 1 : 0, ns = (int)K->slot_e.size();
        const int* tab = E->d_jit_slots[plan][E->chrom];
        pmjit::Args J;
        J.items = A.items[list]; J.counts = A.counts; J.ref = A.ref; J.res = (const int*)A.res; J.pl = A.pl; J.lktab = A.lktab;
        J.coef = A.es_coef; J.slot_e = tab; J.slot_sig = tab + ns; J.slot_p0 = tab + 2 * ns;
        J.pair_k = tab + 3 * ns; J.npairs = (int)K->pair_k.size() / 2;
        J.T10 = E->d_T10; J.T10dn = E->d_T10dn; J.tba = E->d_tba;
        J.list = list; J.it0 = A.es_it0; J.it1 = A.es_it1; J.nslots = ns; J.np = A.n_person; J.T = A.T; J.max_ext = A.max_ext;
        J.dcap = A.poly_dcap; J.vcf = A.vcf; J.res_words = sizeof(pm_site_result) / 4;
        J.res_a1 = offsetof(pm_site_result, allele1) / 4; J.res_a2 = offsetof(pm_site_result, allele2) / 4;
        J.denovo = A.denovo;
        // a site's de novo items are consecutive in lists 0 (cfgs 0-3, or 1-3 when k_prep / the QUAD item takes the
        // monomorphism) and 1 (cfgs 4-6): one task takes them together, the 10-state leaf steps once
        J.prof = nullptr;
        if (getenv("PM_ES_PROF")) {
          if (!E->d_es_prof) {
            if (int r = dalloc(&E->d_es_prof, 5)) return r;
            HIP_TRY(hipMemset(E->d_es_prof, 0, 5 * sizeof(unsigned long long)));
          }
          J.prof = E->d_es_prof;
        }
        J.group = 0;
        if (K->wave && A.denovo && !A.vcf && !getenv("PM_ES_NOGROUP")) {
          if (list == 0) J.group = A.mono_dn ? 3 : 4;
          else if (list == 1) J.group = 3;
        }
        if (list == 0) E->es_grouped = J.group > 1;   // (finish_batch's op count: lists 0 and 1 group alike)
        void* params[] = {&J};
        if (K->wave)
          HIP_TRY(hipModuleLaunchKernel(K->fn, E->n_cu * (K->blocks_per_cu > 0 ? K->blocks_per_cu : std::max(1, 16 / K->wpb)), 1, 1,
                                        64 * K->wpb, 1, 1, 0, E->stream, params, nullptr));
        else   // (a persistent grid of the resident blocks: each thread loads its next unit's PL bytes ahead)
          HIP_TRY(hipModuleLaunchKernel(K->fn, E->n_cu * (K->blocks_per_cu > 0 ? std::min(8, K->blocks_per_cu) : 8), 1, 1, 256, 1, 1, 0,
                                        E->stream, params, nullptr));
      } else hipLaunchKernelGGL(hoist, dim3(hgrid), dim3(64 * E->hoist_waves), hlds, E->stream, A, list);
      HIP_TRY(hipGetLastError());
      if ((mrc = mark(E->es_events, false))) return mrc;
      if ((mrc = mark(E->brent_events, true))) return mrc;
      hipLaunchKernelGGL(fn, dim3(grid), dim3(T), shmem, E->stream, A, list);
      HIP_TRY(hipGetLastError());
      if ((mrc = mark(E->brent_events, false))) return mrc;
    }
  } else {
    if ((mrc = mark(E->brent_events, true))) return mrc;
    hipLaunchKernelGGL(fn, dim3(grid), dim3(T), shmem, E->stream, A, list);
    HIP_TRY(hipGetLastError());
    if ((mrc = mark(E->brent_events, false))) return mrc;
  }
  return PM_OK;
}

static int run_pipeline(pm_engine* E, int n, const uint8_t* pl, const uint32_t* dm, const uint8_t* ref, pm_site_result* res,
                        pm_geno_call* calls) {
  DevArgs A = make_args(E, n, pl, dm, ref, res, calls);
  E->last_n = n;
  HIP_TRY(hipMemsetAsync(E->d_counts, 0, 16 * sizeof(int), E->stream));
  {
    // counts[4] = first emitted site, counts[6] = first stuck site (both atomicMin); counts[5] = any stuck
    static const int init[3] = {0x7fffffff, 0, 0x7fffffff};
    HIP_TRY(hipMemcpyAsync(E->d_counts + 4, init, sizeof(init), hipMemcpyHostToDevice, E->stream));
  }
  {   // persons per lane of k_prep: vector loads when n_person allows; the reference's serial mono order in EXACT
    const int np = E->n_person;
    int vmax = 8;   // measured best on 1000 quads (16 and 4 within 1%)
    // (the de novo monomorphism path compiled in only for engines that form it here: mono_dn == 1; vcf_mode never does)
    const bool mdn = A.mono_dn == 1 && !E->vcf;
    void (*prep)(DevArgs, int) = E->par.numerics == PM_NUM_EXACT ? (E->vcf ? k_prep<1, true, true, false> : mdn ? k_prep<1, true> : k_prep<1, true, false, false>)
                          : E->vcf ? ((np % 16 == 0 && vmax >= 16) ? k_prep<16, false, true, false> : (np % 8 == 0 && vmax >= 8) ? k_prep<8, false, true, false>
                                      : (np % 4 == 0 && vmax >= 4) ? k_prep<4, false, true, false> : k_prep<1, false, true, false>)
                          : mdn ? ((np % 16 == 0 && vmax >= 16) ? k_prep<16, false> : (np % 8 == 0 && vmax >= 8) ? k_prep<8, false>
                                   : (np % 4 == 0 && vmax >= 4) ? k_prep<4, false> : k_prep<1, false>)
                          : (np % 16 == 0 && vmax >= 16) ? k_prep<16, false, false, false> : (np % 8 == 0 && vmax >= 8) ? k_prep<8, false, false, false>
                          : (np % 4 == 0 && vmax >= 4) ? k_prep<4, false, false, false> : k_prep<1, false, false, false>;
    // sites per wave: PREP_SPW (PM_PREP_SPW = 1..8 overrides it; fewer sites per wave on config 4's 16 384-site
    // batches measured slower: 20.3 -> 19.7 M sites/s at 1, config 5 within noise, profiles/r05sp_ab_prep_spw.txt)
    int spw = PREP_SPW;
    if (const char* s = getenv("PM_PREP_SPW"); s && *s) spw = std::max(1, std::min(PREP_SPW, atoi(s)));
    hipLaunchKernelGGL(prep, dim3((n + 4 * spw - 1) / (4 * spw)), dim3(256), 0, E->stream, A, spw);
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
  for (auto& pr : E->es_events) {
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, pr.first, pr.second));
    E->stats.es_hoist_ms += ms;
    E->stats.es_hoist_launches++;
    hipEventDestroy(pr.first); hipEventDestroy(pr.second);
  }
  E->es_events.clear();
  return PM_OK;
}

int pm_engine_run_device(pm_engine* E, int32_t n, const uint8_t* d_pl, const uint32_t* d_dm, const uint8_t* d_ref, pm_site_result* d_res,
                         pm_geno_call* d_calls) {
  if (!E || n < 0 || n > E->max_batch) { pm_set_last_error("pm_engine_run_device: invalid arguments (n > max_batch?)"); return PM_EINVAL; }
  if (n == 0) return PM_OK;
  HIP_TRY(hipSetDevice(E->device));
  return run_pipeline(E, n, d_pl, d_dm, d_ref, d_res ? d_res : E->d_res, d_calls ? d_calls : E->d_calls);
}

// Bookkeeping after a batch's stream work has completed (counts = the batch's d_counts, already on the host).
static int finish_batch(pm_engine* E, const int* counts) {
  if (counts[4] != 0x7fffffff) E->carry_postprob = true;
  E->stats.items += (int64_t)counts[0] + counts[1] + counts[2] + counts[8];
  E->stats.site_visits += (int64_t)counts[0] / (E->vcf ? 1 : (E->par.denovo && !mono_dn_in_prep(E)) ? 4 : 3) + counts[1] / 3 +
                          counts[2] + counts[9];
  E->stats.sites += E->last_n;
  if (E->es_ops_known && (E->use_plan1 ? E->n_ext1 : E->n_ext) > 0) {
    // hoisted items by variant: under --denovo list 0 holds cfg 0 (the top variant) and cfgs 1-3 (10-state) per site,
    // list 1 cfgs 4-6 (10-state), list 2 the cfg-7 re-optimisation (bi-allelic); otherwise every item is bi-allelic
    const double* o = E->es_item_ops;
    if (E->par.denovo && !E->vcf && E->es_grouped)   // a task: one leaf prefix, then the rest per 10-state item
      E->stats.es_hoist_ops += counts[0] / 4 * (o[3] + o[5] + 3 * o[4]) + counts[1] / 3 * (o[3] + 3 * o[4]) + counts[2] * o[0];
    else if (E->par.denovo && !E->vcf)
      E->stats.es_hoist_ops += counts[0] / 4 * o[2] + (counts[0] - counts[0] / 4) * o[1] + counts[1] * o[1] + counts[2] * o[0];
    else E->stats.es_hoist_ops += ((double)counts[0] + counts[1] + counts[2]) * o[0];
  }
  int rc = collect_stats(E);
  if (rc) return rc;
  E->stuck_site = counts[5] ? counts[6] : -1;
  if (counts[5]) { pm_set_last_error("ScalarMinimizer::Brent got stuck"); return PM_EBRENT; }
  return PM_OK;
}

int pm_engine_stuck_site(pm_engine* E, int32_t* site) {
  if (!E || !site) { pm_set_last_error("pm_engine_stuck_site: invalid arguments"); return PM_EINVAL; }
  *site = E->stuck_site;
  return PM_OK;
}

// rows written for the sites before the first stuck one (rows are numbered in site order)
static int rows_before(const pm_site_result* res, int k) {
  int r = 0;
  for (int i = 0; i < k; i++) r += res[i].call_row >= 0;
  return r;
}

int pm_engine_sync(pm_engine* E) {
  if (!E) return PM_EINVAL;
  HIP_TRY(hipSetDevice(E->device));
  HIP_TRY(hipStreamSynchronize(E->stream));
  int counts[16];
  HIP_TRY(hipMemcpy(counts, E->d_counts, sizeof(counts), hipMemcpyDeviceToHost));
  return finish_batch(E, counts);
}

// Host batch -> the engine's stream, without waiting: H2D of the person-major block (asynchronous when the host
// buffers are page-locked, pm_host_alloc), transpose, the pipeline, and D2H of the per-site results and the
// batch counters into the engine's page-locked buffers.  pm_engine_collect waits and hands them out.
int pm_engine_submit(pm_engine* E, int32_t n, const uint8_t* pl, const uint32_t* dm, const uint8_t* ref) {
  if (!E || n < 0 || n > E->max_batch || (n > 0 && (!pl || !ref || (!dm && !E->vcf)))) {
    pm_set_last_error("pm_engine_submit: invalid arguments");
    return PM_EINVAL;
  }
  if (E->pending_n >= 0) { pm_set_last_error("pm_engine_submit: the previous batch has not been collected"); return PM_EINVAL; }
  HIP_TRY(hipSetDevice(E->device));
  if (!E->h_res) {
    HIP_TRY(hipHostMalloc((void**)&E->h_res, sizeof(pm_site_result) * (size_t)E->max_batch, hipHostMallocDefault));
    HIP_TRY(hipHostMalloc((void**)&E->h_counts, 16 * sizeof(int), hipHostMallocDefault));
  }
  E->pending_n = n;
  if (n == 0) return PM_OK;
  const size_t np = E->n_person;
  HIP_TRY(hipMemcpyAsync(E->d_stage, pl, (size_t)n * np * 10, hipMemcpyHostToDevice, E->stream));
  if (!E->vcf)   // (vcf_mode reads no depth: dm is neither copied nor needed, and may be NULL)
    HIP_TRY(hipMemcpyAsync(E->d_dm, dm, (size_t)n * np * 4, hipMemcpyHostToDevice, E->stream));
  HIP_TRY(hipMemcpyAsync(E->d_ref, ref, (size_t)n, hipMemcpyHostToDevice, E->stream));
  int rc = pm_engine_to_planar(E, n, E->d_stage, E->d_pl);   // the engine's genotype-planar layout
  if (rc) return rc;
  rc = run_pipeline(E, n, E->d_pl, E->d_dm, E->d_ref, E->d_res, E->d_calls);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(E->h_res, E->d_res, sizeof(pm_site_result) * n, hipMemcpyDeviceToHost, E->stream));
  HIP_TRY(hipMemcpyAsync(E->h_counts, E->d_counts, 16 * sizeof(int), hipMemcpyDeviceToHost, E->stream));
  return PM_OK;
}

int pm_engine_collect(pm_engine* E, pm_site_result* res, pm_geno_call* calls, int32_t* n_rows) {
  if (!E || !n_rows || E->pending_n < 0 || (E->pending_n > 0 && !res)) {
    pm_set_last_error("pm_engine_collect: invalid arguments (no batch submitted?)");
    return PM_EINVAL;
  }
  const int n = E->pending_n;
  E->pending_n = -1;
  *n_rows = 0;
  if (n == 0) return PM_OK;
  HIP_TRY(hipSetDevice(E->device));
  HIP_TRY(hipStreamSynchronize(E->stream));
  int counts[16];
  memcpy(counts, E->h_counts, sizeof(counts));
  const int rc = finish_batch(E, counts);
  if (rc && rc != PM_EBRENT) return rc;
  memcpy(res, E->h_res, sizeof(pm_site_result) * n);
  *n_rows = rc ? rows_before(res, E->stuck_site) : counts[3];   // PM_EBRENT: the complete sites' rows only
  const size_t np = E->n_person;
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
  return rc;
}

int pm_engine_run_vcf(pm_engine* E, int32_t n, const uint8_t* pl, const uint8_t* ref, pm_site_result* res, pm_vcf_call* calls,
                      int32_t* n_rows) {
  if (!E || !E->vcf || n < 0 || n > E->max_batch || !res || !n_rows) { pm_set_last_error("pm_engine_run_vcf: invalid arguments"); return PM_EINVAL; }
  *n_rows = 0;
  if (n == 0) return PM_OK;
  // (a pm_engine_submit batch still to be collected stays pending: the caller collects it)
  if (E->pending_n >= 0) { pm_set_last_error("pm_engine_run_vcf: a submitted batch has not been collected"); return PM_EINVAL; }
  int rc = pm_engine_submit(E, n, pl, nullptr, ref);
  E->pending_n = -1;   // (this call's own batch: collected below, or abandoned with submit's error)
  if (rc) return rc;
  HIP_TRY(hipSetDevice(E->device));
  HIP_TRY(hipStreamSynchronize(E->stream));
  int counts[16];
  memcpy(counts, E->h_counts, sizeof(counts));
  rc = finish_batch(E, counts);
  if (rc && rc != PM_EBRENT) return rc;
  memcpy(res, E->h_res, sizeof(pm_site_result) * n);
  *n_rows = rc ? rows_before(res, E->stuck_site) : counts[3];   // PM_EBRENT: the complete sites' rows only
  if (calls && counts[3] > 0)   // the device rows as they are (4 B per person)
    HIP_TRY(hipMemcpy(calls, E->d_calls, sizeof(pm_vcf_call) * E->n_person * (size_t)counts[3], hipMemcpyDeviceToHost));
  return rc;
}

int pm_engine_run(pm_engine* E, int32_t n, const uint8_t* pl, const uint32_t* dm, const uint8_t* ref, int32_t on_device,
                  pm_site_result* res, pm_geno_call* calls, int32_t* n_rows) {
  if (!E || n < 0 || n > E->max_batch || !res || !n_rows) { pm_set_last_error("pm_engine_run: invalid arguments"); return PM_EINVAL; }
  *n_rows = 0;
  if (n == 0) return PM_OK;
  if (!on_device) {   // host inputs: submit + collect
    int rc = pm_engine_submit(E, n, pl, dm, ref);
    if (rc) { E->pending_n = -1; return rc; }
    return pm_engine_collect(E, res, calls, n_rows);
  }
  HIP_TRY(hipSetDevice(E->device));
  const size_t np = E->n_person;
  int rc = pm_engine_to_planar(E, n, pl, E->d_pl);   // the engine's genotype-planar layout
  if (rc) return rc;
  rc = run_pipeline(E, n, E->d_pl, dm, ref, E->d_res, E->d_calls);
  if (rc) return rc;
  rc = pm_engine_sync(E);
  if (rc && rc != PM_EBRENT) return rc;
  HIP_TRY(hipMemcpy(res, E->d_res, sizeof(pm_site_result) * n, hipMemcpyDeviceToHost));
  int counts[16];
  HIP_TRY(hipMemcpy(counts, E->d_counts, sizeof(counts), hipMemcpyDeviceToHost));
  *n_rows = rc ? rows_before(res, E->stuck_site) : counts[3];   // PM_EBRENT: the complete sites' rows only
  if (calls && counts[3] > 0) {
    if (E->vcf) {
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
  return rc;
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

int pm_host_alloc(uint64_t bytes, void** p) {
  if (!p) return PM_EINVAL;
  *p = nullptr;
  if (bytes == 0) return PM_OK;
  HIP_TRY(hipHostMalloc(p, bytes, hipHostMallocDefault));
  return PM_OK;
}

int pm_host_free(void* p) {
  if (p) HIP_TRY(hipHostFree(p));
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
