// synth.cpp -- synthetic workload tables and GLF dataset writer (see csrc/synth_core.h).
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>
#include <sys/stat.h>
#include "../csrc/synth_core.h"
#include "synth.h"

extern "C" void pm_synth_build_tables(pm_synth_tables* T) {
  const double perr[3] = {0.01, 0.5, 0.99};
  const double e = 0.01;
  for (int g = 0; g < 3; g++)
    for (int d = 0; d < PM_SYN_MAXDEPTH; d++) {
      double acc = 0.0, lc = 0.0;   // log C(d, k)
      for (int k = 0; k <= PM_SYN_MAXDEPTH; k++) {
        if (k <= d) {
          if (k > 0) lc += std::log((double)(d - k + 1)) - std::log((double)k);
          double lp = lc + k * std::log(perr[g]) + (d - k) * std::log(1 - perr[g]);
          acc += std::exp(lp);
        }
        T->cdf[g][d][k] = (k >= d) ? 2.0 : acc;   // last bucket always taken
      }
    }
  for (int d = 0; d < PM_SYN_MAXDEPTH; d++)
    for (int k = 0; k <= PM_SYN_MAXDEPTH; k++) {
      double l0 = k * std::log10(e) + (d - k) * std::log10(1 - e);
      double l1 = d * std::log10(0.5);
      double l2 = (d - k) * std::log10(e) + k * std::log10(1 - e);
      double mx = std::fmax(l0, std::fmax(l1, l2));
      double L[3] = {l0, l1, l2};
      for (int t = 0; t < 3; t++) {
        double v = std::nearbyint(-10.0 * (L[t] - mx));
        T->pl[d][k][t] = (uint8_t)(v > 255 ? 255 : v);
      }
    }
}

namespace pmhost {

// Family templates: per member (father, mother) family-local indices (-1 founders) and sex,
// listed in path order (founders first).
bool synth_shape(const std::string& shape, int fam, std::vector<SynthMember>& out) {
  out.clear();
  auto add = [&](int fa, int mo, int sex, int pid) { out.push_back({fa, mo, sex, pid}); };
  if (shape == "quad" || shape == "trio" || (shape == "mixed")) {
    int kids = shape == "quad" ? 2 : shape == "trio" ? 1 : (fam % 2 ? 2 : 1);
    add(-1, -1, 1, 1); add(-1, -1, 2, 2);
    for (int k = 0; k < kids; k++) add(0, 1, 1 + ((k + 2) % 2), 3 + k);
    return true;
  }
  if (shape == "ext10") {
    // GP1(m) x GP2(f) -> C1(m), C2(f); C1 x S1(f) -> K1, K2; S2(m) x C2 -> K3, K4
    // pids 1 GP1, 2 GP2, 3 C1, 4 C2, 5 S1, 6 S2, 7-10 K; path: founders 1,2,5,6 then 3,4,7,8,9,10
    add(-1, -1, 1, 1); add(-1, -1, 2, 2); add(-1, -1, 2, 5); add(-1, -1, 1, 6);
    add(0, 1, 1, 3); add(0, 1, 2, 4);
    add(4, 2, 1, 7); add(4, 2, 2, 8); add(3, 5, 1, 9); add(3, 5, 2, 10);
    return true;
  }
  if (shape == "roof") {
    // 1(m) x 2(f) -> 3(m); 4(m) x 5(f) -> 6(f); 3 x 6 -> 7, 8.  path: 1,2,4,5 then 3,6,7,8
    add(-1, -1, 1, 1); add(-1, -1, 2, 2); add(-1, -1, 1, 4); add(-1, -1, 2, 5);
    add(0, 1, 1, 3); add(2, 3, 2, 6); add(4, 5, 1, 7); add(4, 5, 2, 8);
    return true;
  }
  if (shape == "roof2") {
    // 1 x 2 -> 5(f); 3 x 4 -> 6(m); 6 x 5 -> 7, 8(m); 11 x 12 -> 9(f); 8 x 9 -> 10.  Three roofs peel first
    // (parents -> only child); the (6, 5) couple then becomes a roof itself, keyed (father, mother) like the
    // marriage partial its leaf child 7 created, so its type-3 peel runs WITH marriage partials
    // (FamilyLikelihoodES.cpp:1358-1395; plain `transmission` under --denovo, :1391).
    // path: founders 1,2,3,4,11,12 then 5,6,7,8,9,10
    add(-1, -1, 1, 1); add(-1, -1, 2, 2); add(-1, -1, 1, 3); add(-1, -1, 2, 4); add(-1, -1, 1, 11); add(-1, -1, 2, 12);
    add(0, 1, 2, 5); add(2, 3, 1, 6); add(7, 6, 1, 7); add(7, 6, 1, 8); add(4, 5, 2, 9); add(9, 10, 2, 10);
    return true;
  }
  if (shape == "ext12") {
    // 12 members, 6 founders (D = 12 on autosomes): GP1(m) x GP2(f) -> C1(m), C2(f); two roofs GP3 x GP4 -> C3(f),
    // GP5 x GP6 -> C4(m); C1 x C3 -> K1(m); C4 x C2 -> K2(f).  Peels: two leaves, two type-3 roofs, two spouse
    // steps, two more leaves, the founder couple.  path: founders 1,2,5,6,9,10 then 3,4,7,8,11,12
    add(-1, -1, 1, 1); add(-1, -1, 2, 2); add(-1, -1, 1, 5); add(-1, -1, 2, 6); add(-1, -1, 1, 9); add(-1, -1, 2, 10);
    add(0, 1, 1, 3); add(0, 1, 2, 4); add(2, 3, 2, 7); add(6, 8, 1, 8); add(4, 5, 1, 11); add(10, 7, 2, 12);
    return true;
  }
  if (shape == "ext11") {
    // 11 members, 5 founders (D = 10), mostly female middle generation: GP1(m) x GP2(f) -> C1(f), C2(m), C3(f);
    // S1(m) x C1 -> K1(f); C2 x S2(f) -> K2(f); S3(m) x C3 -> K3(m).  path: founders 1,2,6,8,10 then 3,4,5,7,9,11
    add(-1, -1, 1, 1); add(-1, -1, 2, 2); add(-1, -1, 1, 6); add(-1, -1, 2, 8); add(-1, -1, 1, 10);
    add(0, 1, 2, 3); add(0, 1, 1, 4); add(0, 1, 2, 5); add(2, 5, 2, 7); add(6, 3, 2, 9); add(4, 7, 1, 11);
    return true;
  }
  // config 4 at its stated range (8-12 members): five three-generation shapes dealt round-robin over the families
  if (shape == "extmix") {
    static const char* const mix[5] = {"ext10", "roof", "roof2", "ext12", "ext11"};
    return synth_shape(mix[fam % 5], fam, out);
  }
  if (shape == "single") { add(-1, -1, 1 + fam % 2, 1); return true; }
  // quads with an ext10 pedigree at families 256, 513, ...: a few extended families next to hundreds of
  // nuclear ones (the lane plan must pair nuclear slots with per-lane extended lists)
  if (shape == "quadext") return synth_shape(fam % 257 == 256 ? "ext10" : "quad", fam, out);
  return false;
}

// shape "<template>+dn": additionally plants a de novo het call (ref/transition) in one non-founder
// of one family at ~3% of sites, so the --denovo output path has records to check.  "+late": the first
// half of the sites are monomorphic (a site shard whose range emits nothing).  "+multi": three sections.  Files only: the device
// generator (bench) does neither.
int synth_write_dataset(const std::string& dir, const std::string& shape_arg, int nfam, int nsites, uint64_t seed,
                        std::string& err) {
  std::string shape = shape_arg;
  bool plant = false, late = false, multi = false;
  for (bool more = true; more;) {
    more = false;
    if (shape.size() > 6 && shape.compare(shape.size() - 6, 6, "+multi") == 0) { multi = more = true; shape.resize(shape.size() - 6); }
    if (shape.size() > 3 && shape.compare(shape.size() - 3, 3, "+dn") == 0) { plant = more = true; shape.resize(shape.size() - 3); }
    if (shape.size() > 5 && shape.compare(shape.size() - 5, 5, "+late") == 0) { late = more = true; shape.resize(shape.size() - 5); }
  }
  mkdir(dir.c_str(), 0755);
  static pm_synth_tables T;
  static bool built = false;
  if (!built) { pm_synth_build_tables(&T); built = true; }
  std::vector<std::vector<SynthMember>> fams(nfam);
  int np = 0;
  for (int f = 0; f < nfam; f++) {
    if (!synth_shape(shape, f, fams[f])) { err = "unknown synthetic shape " + shape; return -1; }
    np += (int)fams[f].size();
  }
  FILE* ped = fopen((dir + "/test.ped").c_str(), "w");
  FILE* gif = fopen((dir + "/test.gif").c_str(), "w");
  FILE* dat = fopen((dir + "/test.dat").c_str(), "w");
  if (!ped || !gif || !dat) { err = "cannot write dataset files in " + dir; return -1; }
  fprintf(dat, "T\tGLF_Index\n");
  fclose(dat);
  // Person numbering: global person g = family base + member; pids are "base + pid-in-template".
  std::vector<FILE*> glf(np);
  std::vector<uint64_t> gbase(nfam);
  int g = 0;
  for (int f = 0; f < nfam; f++) {
    gbase[f] = (uint64_t)g;
    const int fbase = g;
    for (size_t j = 0; j < fams[f].size(); j++) {
      const SynthMember& m = fams[f][j];
      int pid = fbase + m.pid;
      int fa = m.fa < 0 ? 0 : fbase + fams[f][m.fa].pid;
      int mo = m.mo < 0 ? 0 : fbase + fams[f][m.mo].pid;
      fprintf(ped, "F%d\t%d\t%d\t%d\t%d\t%d\n", f, pid, fa, mo, m.sex, g + 1);
      fprintf(gif, "%d p%d.glf\n", g + 1, g + 1);
      FILE* fh = fopen((dir + "/p" + std::to_string(g + 1) + ".glf").c_str(), "wb");
      if (!fh) { err = "cannot create GLF file"; return -1; }
      glf[g] = fh;
      // header: "GLF\3", u32 0 (sections follow: i32 labelLen incl. NUL, label, i32 maxPosition, records, end)
      const char magic[4] = {'G', 'L', 'F', 3};
      uint32_t zero = 0;
      fwrite(magic, 1, 4, fh); fwrite(&zero, 4, 1, fh);
      g++;
    }
  }
  fclose(ped); fclose(gif);
  std::vector<int32_t> fa, mo;
  std::vector<uint8_t> pl, hap;
  std::vector<uint32_t> dm;
  static const uint8_t iupac[5] = {0, 1, 2, 4, 8};
  // "+multi": sections "1", "X", "2" (nsites each; the site stream continues across them)
  const std::vector<std::string> labels = multi ? std::vector<std::string>{"1", "X", "2"} : std::vector<std::string>{"1"};
  for (size_t sec = 0; sec < labels.size(); sec++) {
  for (auto fh : glf) {
    const int32_t ll = (int32_t)labels[sec].size() + 1, mp = nsites;
    fwrite(&ll, 4, 1, fh); fwrite(labels[sec].c_str(), 1, ll, fh); fwrite(&mp, 4, 1, fh);
  }
  for (int s0 = 0; s0 < nsites; s0++) {
    const int s = (int)sec * nsites + s0;
    int ref; double af;
    pm_syn_site(seed, (uint64_t)s, &ref, &af);
    if (late && s0 < nsites / 2) af = 0.0;   // "+late": no polymorphism in the first half of the section
    for (int f = 0; f < nfam; f++) {
      const auto& F = fams[f];
      int n = (int)F.size();
      fa.resize(n); mo.resize(n); pl.resize((size_t)n * 10); dm.resize(n); hap.resize(n);
      for (int j = 0; j < n; j++) { fa[j] = F[j].fa; mo[j] = F[j].mo; }
      pm_syn_family(&T, seed, (uint64_t)s, ref, af, n, fa.data(), mo.data(), gbase[f], pl.data(), 10, 1, dm.data(), hap.data());
      if (plant && pm_u01(seed, (uint64_t)s, 0, 901) < 0.03 &&
          (int)(pm_u01(seed, (uint64_t)s, 0, 902) * nfam) == f) {
        int kids[64], nk = 0;
        for (int j = 0; j < n && nk < 64; j++) if (fa[j] >= 0) kids[nk++] = j;
        if (nk > 0) {
          const int j = kids[(int)(pm_u01(seed, (uint64_t)s, 0, 903) * nk) % nk];
          static const int gidx[4][4] = {{0, 1, 2, 3}, {1, 4, 5, 6}, {2, 5, 7, 8}, {3, 6, 8, 9}};
          const int alt = ref == 1 ? 3 : ref == 3 ? 1 : ref == 2 ? 4 : 2;
          uint8_t* q = pl.data() + (size_t)j * 10;
          for (int g = 0; g < 10; g++) q[g] = 255;
          q[gidx[ref - 1][ref - 1]] = 45;
          q[gidx[ref - 1][alt - 1]] = 0;
          q[gidx[alt - 1][alt - 1]] = 90;
        }
      }
      for (int j = 0; j < n; j++) {
        uint8_t rec[20];
        rec[0] = (uint8_t)(0x10 | iupac[ref]);
        uint32_t off = 1, d = dm[j] & 0xFFFFFF;
        memcpy(rec + 1, &off, 4); memcpy(rec + 5, &d, 4);
        rec[9] = (uint8_t)(dm[j] >> 24);
        memcpy(rec + 10, pl.data() + (size_t)j * 10, 10);
        fwrite(rec, 1, 20, glf[gbase[f] + j]);
      }
    }
  }
  for (auto fh : glf) { uint8_t end = 0; fwrite(&end, 1, 1, fh); }
  }
  for (auto fh : glf) fclose(fh);
  return 0;
}

}  // namespace pmhost
