// tests/native/jit_check.cpp -- TEST INFRASTRUCTURE: the schedule compiler (polymutt_amd/csrc/es_jit.h) without a
// device.  Loads a pedigree (.dat/.ped), builds the extended families' hoisting kernel source for every chromosome
// class as the engine would (slot order of a 64-lane plan), compiles each with hipRTC for gfx950 and prints one
// line per class: shapes, source bytes, code-object bytes, compile ms.  Exit status 1 on any failure.
//   jit_check DAT PED [--emit FILE]
#include <chrono>
#include <cstdio>
#include <string>
#include <vector>
#include "../../polymutt_amd/csrc/es_jit.h"
#include "../../polymutt_amd/host/pedigree.h"

static const double kTBA[5][27] = {   // transmission_BA tables (FamilyLikelihoodES.cpp:812-924), as the engine's
    {1, 0, 0, .5, .5, 0, 0, 1, 0, .5, .5, 0, .25, .5, .25, 0, .5, .5, 0, 1, 0, 0, .5, .5, 0, 0, 1},
    {1, 0, 0, .5, .5, 0, 0, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 0, 0, .5, .5, 0, 0, 1},
    {1, 0, 0, .5, 0, .5, 0, 0, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 0, 0, .5, 0, .5, 0, 0, 1},
    {1, 0, 0, 1, 0, 0, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 0, 0, 1, 0, 0, 1},
    {1, 0, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 0, 0, 0, 0, 1}};

int main(int argc, char** argv) {
  if (argc < 3) { fprintf(stderr, "usage: jit_check DAT PED [--emit FILE]\n"); return 2; }
  pmhost::Pedigree ped;
  try {
    ped.load(argv[1], argv[2]);
  } catch (const std::exception& e) {
    fprintf(stderr, "pedigree: %s\n", e.what());
    return 1;
  }
  const std::string emit = argc >= 5 && std::string(argv[3]) == "--emit" ? argv[4] : "";
  const pm_pedigree v = ped.view();
  std::vector<pmjit::Family> fams;
  int e = 0;
  for (int f = 0; f < v.n_fam; f++) {
    if (v.fam_kind[f] != PM_FAM_EXTENDED) continue;
    pmjit::Family F;
    F.e = e++;
    F.p0 = v.fam_start[f];
    F.n = v.fam_start[f + 1] - F.p0;
    F.nf = v.fam_founders[f];
    for (int i = 0; i < F.n; i++) { F.sex.push_back(v.sex[F.p0 + i]); F.founder.push_back(v.is_founder[F.p0 + i]); }
    if (pmjit::pack_steps(&v, f, 3, F.steps) < 0) { fprintf(stderr, "family %d: no schedule\n", f); return 1; }
    fams.push_back(F);
  }
  if (fams.empty()) { fprintf(stderr, "no extended families\n"); return 1; }
  for (int run = 0; run < 12; run++) {
    const int cls = run & 3;
    const int dn = run >= 8 ? 1 : run >= 4 ? 2 : 0;   // the --denovo engines' wave-cooperative kernel (2: grouped tasks only)
    pmjit::Kernel K;
    const std::string src = pmjit::generate(cls, fams, kTBA, &K, dn);
    if (!emit.empty() && cls == 0) {
      FILE* fh = fopen((dn ? emit + ".dn" + std::to_string(dn) : emit).c_str(), "w");
      if (fh) { fputs(src.c_str(), fh); fclose(fh); }
    }
    std::vector<char> code;
    std::string err;
    const auto t0 = std::chrono::steady_clock::now();
    if (!pmjit::compile(src, &code, &err)) { fprintf(stderr, "class %d: %s\n", cls, err.c_str()); return 1; }
    if (!emit.empty() && cls == 0) {   // the code object too (register and LDS use: llvm-readelf --notes)
      FILE* fh = fopen(((dn ? emit + ".dn" + std::to_string(dn) : emit) + ".co").c_str(), "wb");
      if (fh) { fwrite(code.data(), 1, code.size(), fh); fclose(fh); }
    }
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    std::string ops;   // FP64 operations per (item, family) of shape 0, by variant
    for (int v = 0; v < 6; v++) ops += " " + std::to_string((long long)(K.shape_ops[v].empty() ? 0 : K.shape_ops[v][0]));
    printf("class %d shapes %d families %zu source %zu code %zu compile_ms %.0f%s ops%s\n", cls, K.n_shapes, fams.size(), src.size(),
           code.size(), ms, dn ? (" denovo wpb " + std::to_string(K.wpb) + " ws " + std::to_string(K.ws)).c_str() : "", ops.c_str());
  }
  // the fused hoisting + Brent kernel of bi-allelic engines (ep_brent_jit), every class
  for (int cls = 0; cls < 4; cls++) {
    pmjit::FusedKernel F;
    const std::string src = pmjit::generate_fused(cls, fams, kTBA, &F);
    if (src.empty()) { printf("fused %d none\n", cls); continue; }
    if (!emit.empty() && cls == 0) {
      FILE* fh = fopen((emit + ".fused").c_str(), "w");
      if (fh) { fputs(src.c_str(), fh); fclose(fh); }
    }
    std::vector<char> code;
    std::string err;
    if (!pmjit::compile(src, &code, &err)) { fprintf(stderr, "fused class %d: %s\n", cls, err.c_str()); return 1; }
    if (!emit.empty() && cls == 0) {
      FILE* fh = fopen((emit + ".fused.co").c_str(), "wb");
      if (fh) { fwrite(code.data(), 1, code.size(), fh); fclose(fh); }
    }
    std::string tiles;
    for (int d : F.row_deg) tiles += " " + std::to_string(d);
    printf("fused %d shapes %d rows %d lanes %d item_ops %.0f code %zu tiles%s\n", cls, F.n_shapes, F.rows, F.lanes, F.item_ops,
           code.size(), tiles.c_str());
  }
  return 0;
}
