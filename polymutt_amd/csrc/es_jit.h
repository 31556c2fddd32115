// es_jit.h -- the Elston-Stewart schedule compiler (host side of the EP hoisting).
//
// An extended family's peeling schedule (ES_Peeling, FamilyLikelihoodES.cpp:46-277) is fixed per pedigree, so
// the polynomial-form peel of a (Brent item, family) -- the bi-allelic steps of :1105-1286 run on coefficient
// vectors, see engine.hip "Elston-Stewart peeling in polynomial form" -- is compiled at engine creation into
// straight-line HIP for gfx950 (hipRTC): one device function per distinct family shape of the section's
// chromosome class, every partial and marriage-partial coefficient an SSA value (registers), the transmission
// constants folded, structurally zero terms dropped.  One thread then hoists one (item, family) -- no
// workspace, no schedule interpretation.  Families of one shape share a function; the kernel switches on it.
#pragma once
#include <cstdint>
#include <string>
#include <vector>
#include <hip/hip_runtime.h>
#include "../../include/polymutt_engine.h"

namespace pmjit {

struct Family {              // one extended family of the lane plan, in slot order e = q * T + lane
  int e;                     // slot of the plan (coefficients go to es_coef[...][e / T][...][e % T])
  int p0, n, nf;             // first person (flattened), persons, founders (Family::path: founders first)
  std::vector<int8_t> sex, founder;
  std::vector<int2> steps;   // packed schedule (engine.hip pack_steps: type | from0 | from1 | to0, to1 | slot | create | fa2mo)
};

// Arguments of the generated kernel es_hoist_jit (identical layout in the generated source).
struct Args {
  const int* items;          // the list's items (site << 3 | cfg)
  const int* counts;         // counts[list] = list size
  const uint8_t* ref;        // [site] refBase (vcf_mode: a1 | a2 << 4)
  const int* res;            // pm_site_result as int32 words (cfg-7 items read allele1/allele2)
  const uint8_t* pl;         // genotype-planar site blocks
  const double* lktab;       // [256] phred -> likelihood
  double* coef;              // es_coef
  const int* slot_e;         // [nslots] plan slot, sorted by shape
  const int* slot_sig;       // [nslots] shape index
  const int* slot_p0;        // [nslots] first person
  const double* T10;         // FamilyLikelihoodES::transmission [10][10][10] (es_hoist_wave)
  const double* T10dn;       // transmission_denovo
  const double* tba;         // transmission_BA tables [5][27]
  unsigned long long* prof;  // [5] PM_ES_PROF clock cycles (es_hoist_wave)
  const int* pair_k;         // [2 npairs] es_hoist_wave pair mode: the two slots of family pair j (Kernel::pair_k)
  int list, it0, it1, nslots, np, T, max_ext, dcap, vcf, res_words, res_a1, res_a2, denovo,
      group,                 // es_hoist_wave: items per task (the de novo items of one site share the leaf steps), 0/1 none
      npairs;
};

// Arguments of the generated posterior kernel es_post_jit (CalcPostProb_SingleExtendedPed_BA for every emitted row
// and peeled family; the families are the Kernel's slots, sorted by shape).
struct PostArgs {
  const int* counts;         // counts[3] = emitted rows
  const int* row_site;       // [row] site
  const char* res;           // pm_site_result[site] (allele1/2, maxidx, af read at the byte offsets below)
  const uint8_t* pl;
  const double* lktab;
  const double* gq_thr;      // [101] GQ thresholds (engine.hip d_gq)
  void* calls;               // pm_geno_call[row][person], or pm_vcf_call in vcf_mode
  const int* fam_p0;         // [nfams] first person (slot order, sorted by shape)
  const int* fam_sig;        // [nfams] shape
  int nfams, np, vcf, res_bytes, off_a1, off_a2, off_maxidx, off_af;
  double theta;
};

struct Kernel {
  hipFunction_t fn = nullptr;        // es_hoist_jit(Args)
  hipFunction_t fn_post = nullptr;   // es_post_jit(PostArgs)
  std::vector<int> slot_e, slot_sig, slot_p0;   // host copies (the engine uploads them)
  int n_shapes = 0;
  double compile_ms = 0;
  bool wave = false;         // --denovo: es_hoist_wave, one (item, family) per wave, blockDim = 64 wpb
  // FP64 operations of one (item, family) hoisting per shape, by variant: 0 bi-allelic, 1 10-state (de novo items),
  // 2 top (the de novo monomorphism item), 3 the leaf prefix of a grouped task, 4 / 5 its 10-state / top rest (3 + 4 ==
  // 1, 3 + 5 == 2); the bi-allelic engines fill variant 0 only
  std::vector<double> shape_ops[6];
  int wpb = 0, ws = 0;       // waves per block, workspace doubles per wave
  int blocks_per_cu = 0;     // es_hoist_wave blocks resident per CU (the runtime's occupancy; 0 unknown)
  bool pair = false;         // es_hoist_wave hoists two same-shape families per wave, one per half-wave (PM_ES_PAIR)
  std::vector<int> pair_k;   // [fpw units] slot indices of each unit of fpw same-shape slots (a short unit: its first again)
  int fpw = 1;               // families per wave (PM_ES_FPW; 2 = the pair mode)
};

// The fused Elston-Stewart Brent kernel ep_brent_jit (bi-allelic engines whose every family is peeled: config 4): one wave
// per Brent item, each lane hoisting its families' polynomials straight into registers (the shape's generated peel,
// inlined) and then running the item's whole OptimizeFrequency + Brent on them -- no es_coef round trip through HBM and
// one launch per list instead of a hoisting launch and a Brent launch.  Families sit on (row, lane) cells: sorted by
// (degree, shape), rows of `lanes` cells, so a row's register tile is its largest degree + 1 and few shapes share a row.
struct FusedArgs {
  const int* items;          // the list's items (site << 3 | cfg)
  int* counts;               // counts[list] = list size; [5] / [6] Brent stuck flag / first stuck site (atomics)
  const uint8_t* ref;        // [site] refBase (vcf_mode: a1 | a2 << 4)
  const int* res;            // pm_site_result as int32 words (cfg-7 items read allele1/allele2)
  const uint8_t* pl;         // genotype-planar site blocks
  const double* lktab;       // [256] phred -> likelihood
  const int* lane_tab;       // [rows][64] p0 | shape << 24 (-1: no family), then [64] each lane's degrees summed
  double* raw;               // [site][8] -fmin
  double* minv;              // [site][8] minimiser
  int* evals;                // [site][8] objective evaluations (the reference's count)
  unsigned long long* eval_total;
  double precision;
  int list, it0, it1, np, vcf, res_words, res_a1, res_a2, itmax, pad;
};
struct FusedKernel {
  hipFunction_t fn = nullptr;
  std::vector<int> lane_tab;   // rows * 64 + 64 ints (FusedArgs::lane_tab)
  std::vector<int> row_deg;    // each row's register tile degree
  int rows = 0, lanes = 0, n_shapes = 0, blocks_per_cu = 0;
  bool pair = false;           // two Brent items per wave, one per half-wave (rows of <= 32 cells)
  double item_ops = 0;         // FP64 operations of one item's hoisting over every family (the generated peels)
  double compile_ms = 0;
};
// The generated source of ep_brent_jit for `fams` (fills out's layout; no device needed); "" when the families do not
// fit the register tiles (then the engine keeps es_hoist_jit + k_brent).
std::string generate_fused(int chrom, const std::vector<Family>& fams, const double (*tba)[27], FusedKernel* out);
bool build_fused(int device, int chrom, const std::vector<Family>& fams, const double (*tba)[27], FusedKernel* out,
                 std::string* err);

// Packs family f's ES_Peeling schedule (pm_pedigree.steps) with its marriage-partial slots resolved the way the
// reference's partial map behaves; appends to out; returns the workspace doubles of a reference-order peel with ns
// states, -1 if it cannot be packed.
int pack_steps(const pm_pedigree* ped, int f, int ns, std::vector<int2>& out);

// The generated source of the hoisting kernel of `fams` (fills out's slot tables; no device needed).
// denovo: the wave-cooperative kernel es_hoist_wave (10-state, bi-allelic and top variants per shape) instead of the
// per-thread es_hoist_jit and es_post_jit; 2: the same for engines whose de novo items always come in grouped tasks
// (no whole 10-state / top variants: their larger workspace would set every wave's LDS slice).
std::string generate(int chrom, const std::vector<Family>& fams, const double (*tba)[27], Kernel* out, int denovo = 0);
// hipRTC compile of a generated source for gfx950 (no device needed).
// (the source may #include "brent_core.h" / "log_table.h": their text is embedded in the library)
bool compile(const std::string& src, std::vector<char>* code, std::string* err, const std::string& arch = "gfx950");

// Generates and compiles the hoisting and posterior kernels of `fams` for chromosome class `chrom` (PM_CHR_*); bi-allelic
// (3-state) peels.  tba = transmission_BA tables [5][27] (:812-924).  Returns false with a message in err.
bool build(int device, int chrom, const std::vector<Family>& fams, const double (*tba)[27], int denovo, Kernel* out,
           std::string* err);

}  // namespace pmjit
