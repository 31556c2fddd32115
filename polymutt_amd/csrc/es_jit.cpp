// es_jit.cpp -- see es_jit.h.
#include "es_jit.h"
#include <hip/hiprtc.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <mutex>
#include "../../include/polymutt_engine.h"
#include "jit_headers.inc"   // kBrentCoreH, kLogTableH: csrc/brent_core.h and csrc/log_table.h as text

namespace pmjit {
namespace {

constexpr int MALE = 1, FEMALE = 2;

// A homogeneous polynomial in (f, g = 1 - f) of degree d: coefficient names c[a] of f^a g^(d - a) ("" = zero).
struct Poly {
  int d = 0;
  std::vector<std::string> c;
};

std::string lit(double x) {   // exact hexadecimal literal
  char b[64];
  snprintf(b, sizeof b, "%a", x);
  return b;
}

struct Gen {
  std::string code;
  int nv = 0;
  long ops = 0;   // FP64 operations emitted (each mul, add or fma one; table loads not counted)
  std::map<std::string, std::string> memo;   // expression -> value: identical computations share one value
  std::string def(const std::string& expr) {
    auto it = memo.find(expr);
    if (it != memo.end()) return it->second;
    if (expr.compare(0, 3, "lk[") != 0) ops++;
    std::string v = "v" + std::to_string(nv++);
    code += "  const double " + v + " = " + expr + ";\n";
    memo[expr] = v;
    return v;
  }
  // acc + x * y (acc empty: x * y); "1" factors elided
  std::string mac(const std::string& acc, const std::string& x, const std::string& y) {
    const bool x1 = x == "1.0", y1 = y == "1.0";
    const std::string prod = x1 ? y : y1 ? x : "";
    if (acc.empty()) return prod.empty() ? def(x + " * " + y) : prod;
    if (!prod.empty()) return def(acc + " + " + prod);
    return def("fma(" + x + ", " + y + ", " + acc + ")");
  }
  Poly zero(int d) { Poly p; p.d = d; p.c.assign(d + 1, ""); return p; }
  Poly mul(const Poly& A, const Poly& B) {
    Poly R = zero(A.d + B.d);
    for (int a = 0; a <= R.d; a++)
      for (int u = std::max(0, a - B.d); u <= std::min(a, A.d); u++)
        if (!A.c[u].empty() && !B.c[a - u].empty()) R.c[a] = mac(R.c[a], A.c[u], B.c[a - u]);
    return R;
  }
  // sum_t w_t P_t (all of degree d)
  Poly lincomb(const std::vector<std::pair<double, const Poly*>>& terms, int d) {
    Poly R = zero(d);
    for (int a = 0; a <= d; a++)
      for (auto& t : terms) {
        if (t.first == 0.0 || t.second->c[a].empty()) continue;
        R.c[a] = mac(R.c[a], t.first == 1.0 ? std::string("1.0") : lit(t.first), t.second->c[a]);
      }
    return R;
  }
  Poly add(const Poly& A, const Poly& B) {   // same degree
    Poly R = zero(A.d);
    for (int a = 0; a <= A.d; a++) {
      if (A.c[a].empty()) R.c[a] = B.c[a];
      else if (B.c[a].empty()) R.c[a] = A.c[a];
      else R.c[a] = def(A.c[a] + " + " + B.c[a]);
    }
    return R;
  }
};

// transmission_BA of the class for an offspring of sex csex (GetTransmissionProb_BA :1059-1075)
double tba(const double (*T)[27], int chrom, int csex, int i, int j, int k) {
  const int o = i * 9 + j * 3 + k;
  if (chrom == PM_CHR_X) return csex == MALE ? T[2][o] : T[1][o];
  if (chrom == PM_CHR_Y) return csex == MALE ? T[3][o] : 1.0;
  if (chrom == PM_CHR_MT) return T[4][o];
  return T[0][o];
}

// the shape key: everything the generated code depends on
std::string shape_key(const Family& F) {
  std::string k = std::to_string(F.n) + ":" + std::to_string(F.nf) + ":";
  for (int i = 0; i < F.n; i++) {
    k += F.founder[i] ? 'F' : 'o';
    k += (char)('0' + F.sex[i]);   // (child sex of the X/Y transmission, chrY females)
  }
  for (auto& s : F.steps) k += ":" + std::to_string(s.x) + "," + std::to_string(s.y);
  return k;
}

int g_bapf = 0;           // es_hoist_jit: PL bytes of the thread's next (item, family) loaded ahead, 3 per person of the
                          // largest family (0: off, the default -- PM_ES_BAPF=1 turns it on for families of <= 12)

// One family shape's hoisting as a device function: the polynomial of FamilyLikelihoodES' BA peel in (f, g).
// fused: the ep_brent_jit form -- inlined, the D + 1 coefficients into the caller's register array out[0..D] (no degree
// word); *deg = D.
std::string gen_family(const Family& F, int chrom, const double (*T)[27], const std::string& name, double* ops,
                       bool fused = false, int* deg = nullptr) {
  Gen G;
  const int n = F.n;
  const bool X = chrom == PM_CHR_X, Y = chrom == PM_CHR_Y, MT = chrom == PM_CHR_MT;
  std::map<std::pair<int, int>, std::string> pen;   // (person, state) -> loaded likelihood
  auto penv = [&](int i, int j) {
    auto key = std::make_pair(i, j);
    auto it = pen.find(key);
    if (it != pen.end()) return it->second;
    static const char* plane[3] = {"P11", "P12", "P22"};
    std::string v = g_bapf ? G.def("lk[b[" + std::to_string(3 * i + j) + "]]")
                           : G.def(std::string("lk[") + plane[j] + "[p0 + " + std::to_string(i) + "]]");
    pen[key] = v;
    return v;
  };
  // InitializePartials_BA x SetFounderPriors_BA (:1449-1465, :666-687)
  std::vector<std::vector<Poly>> P(n, std::vector<Poly>(3));
  for (int i = 0; i < n; i++) {
    const int sx = F.sex[i];
    const bool fo = F.founder[i] && i < F.nf;
    const bool yf = Y && sx == FEMALE;
    const int d = !fo ? 0 : yf ? 0 : (((X || Y) && sx == MALE) || MT) ? 1 : 2;
    for (int j = 0; j < 3; j++) {
      Poly p = G.zero(d);
      if (yf) p.c[0] = "1.0";
      else if (!fo) p.c[0] = penv(i, j);
      else if (d == 2) p.c[2 - j] = j == 1 ? G.def("2.0 * " + penv(i, j)) : penv(i, j);   // f^2, 2fg, g^2
      else if (j != 1) p.c[j == 0 ? 1 : 0] = penv(i, j);                                    // f, 0, g
      P[i][j] = p;
    }
  }
  std::map<int, std::vector<Poly>> M;   // marriage partials by slot: [i * 3 + j]
  int fin = -1;
  for (const int2& S : F.steps) {
    const int type = S.x & 255, from0 = (S.x >> 8) & 255, from1 = (S.x >> 16) & 255, to0 = (S.x >> 24) & 255;
    const int slot = (S.y >> 8) & 255, create = (S.y >> 16) & 1, fa2mo = (S.y >> 17) & 1;
    fin = to0;
    if (type == 1) {   // peelOffspring2Parents_BA (:1105-1130): M(i, j) *= sum_k T(i, j, k) P_off[k]
      const int off = from0, csex = F.sex[off], da = P[off][0].d;
      std::vector<Poly> Sij(9);
      for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
          std::vector<std::pair<double, const Poly*>> t;
          for (int k = 0; k < 3; k++) t.push_back({tba(T, chrom, csex, i, j, k), &P[off][k]});
          Sij[i * 3 + j] = G.lincomb(t, da);
        }
      if (create || !M.count(slot)) M[slot] = Sij;
      else
        for (int e = 0; e < 9; e++) M[slot][e] = G.mul(M[slot][e], Sij[e]);
    } else if (type == 2) {   // peelSpouse2Spouse_BA (:1182-1230): P_to[i] *= sum_j P_from[j] M(j, i)
      const int sf = from0, stt = to0;
      for (int i = 0; i < 3; i++) {
        Poly sum;
        bool first = true;
        for (int j = 0; j < 3; j++) {
          Poly term = slot == 255 ? P[sf][j] : G.mul(P[sf][j], M[slot][fa2mo ? j * 3 + i : i * 3 + j]);
          sum = first ? term : G.add(sum, term);
          first = false;
        }
        P[stt][i] = G.mul(P[stt][i], sum);
      }
    } else {   // peelParents2Offspring_BA (:1260-1286): P_off[k] *= sum_ij P_fa[i] M(i, j) P_mo[j] T(i, j, k)
      const int fa = from0, mo = from1, off = to0, csex = F.sex[off];
      std::vector<Poly> W(9);
      for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
          const Poly fm = slot == 255 ? P[fa][i] : G.mul(P[fa][i], M[slot][i * 3 + j]);
          W[i * 3 + j] = G.mul(fm, P[mo][j]);
        }
      for (int k = 0; k < 3; k++) {
        std::vector<std::pair<double, const Poly*>> t;
        for (int e = 0; e < 9; e++) t.push_back({tba(T, chrom, csex, e / 3, e % 3, k), &W[e]});
        const Poly Sk = G.lincomb(t, W[0].d);
        P[off][k] = G.mul(P[off][k], Sk);
      }
    }
  }
  // CalculateLikelihood_BA (:1013-1032): the final person's partials summed
  Poly L = G.add(G.add(P[fin][0], P[fin][1]), P[fin][2]);
  if (deg) *deg = L.d;
  *ops = (double)G.ops;
  if (fused) {
    std::string out = "__device__ __forceinline__ void " + name +
                      "(const unsigned char* __restrict__ P11, const unsigned char* __restrict__ P12, "
                      "const unsigned char* __restrict__ P22, int p0, const double* __restrict__ lk, double* out) {\n" + G.code;
    for (int a = 0; a <= L.d; a++) out += "  out[" + std::to_string(a) + "] = " + (L.c[a].empty() ? "0.0" : L.c[a]) + ";\n";
    return out + "}\n";
  }
  std::string out = g_bapf ? "__device__ __forceinline__ void " + name +   // (inlined: b stays in registers)
                                 "(const unsigned int* b, const double* __restrict__ lk, double* __restrict__ out, int os, int dcap) {\n" +
                                 G.code
                           : "__device__ __attribute__((noinline)) void " + name +
                                 "(const unsigned char* __restrict__ P11, const unsigned char* __restrict__ P12, "
                                 "const unsigned char* __restrict__ P22, int p0, const double* __restrict__ lk, double* __restrict__ out, "
                                 "int os, int dcap) {\n" + G.code;
  for (int a = 0; a <= L.d; a++) out += "  out[" + std::to_string(a) + " * os] = " + (L.c[a].empty() ? "0.0" : L.c[a]) + ";\n";
  out += "  out[(dcap - 1) * os] = " + std::to_string(L.d) + ".0;\n}\n";
  return out;
}

const char* kPrologue = R"(
typedef unsigned char uint8_t;
struct Args {
  const int* items; const int* counts; const uint8_t* ref; const int* res; const uint8_t* pl; const double* lktab;
  double* coef; const int* slot_e; const int* slot_sig; const int* slot_p0;
  const double* T10; const double* T10dn; const double* tba; unsigned long long* prof; const int* pair_k;
  int list, it0, it1, nslots, np, T, max_ext, dcap, vcf, res_words, res_a1, res_a2, denovo, group, npairs;
};
__device__ __forceinline__ int gi(int b1, int b2) {
  return b1 < b2 ? (b1 - 1) * (10 - b1) / 2 + (b2 - b1) : (b2 - 1) * (10 - b2) / 2 + (b1 - b2);
}
__device__ __forceinline__ void cfg_alleles(int cfg, int r, int* a1, int* a2) {   // main.cpp:458-529, PedigreeGLF.h:14-53
  const int ts = r == 1 ? 3 : r == 2 ? 4 : r == 3 ? 1 : 2, tv1 = (r == 1 || r == 3) ? 2 : 1, tv2 = (r == 1 || r == 3) ? 4 : 3;
  switch (cfg) {
    case 0: *a1 = r; *a2 = (r == 4) ? 3 : r + 1; break;
    case 1: *a1 = r; *a2 = ts; break;
    case 2: *a1 = r; *a2 = tv1; break;
    case 3: *a1 = r; *a2 = tv2; break;
    case 4: *a1 = ts; *a2 = tv1; break;
    case 5: *a1 = ts; *a2 = tv2; break;
    default: *a1 = tv1; *a2 = tv2; break;
  }
}
)";

std::string gen_kernel(const std::vector<std::string>& shapes) {
  if (g_bapf) {   // the next unit's PL bytes are loaded before this unit is computed (one HBM round trip hidden per unit)
    std::string s = R"(
extern "C" __global__ void __launch_bounds__(256) es_hoist_jit(Args A) {
  __shared__ double lk[256];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) lk[i] = A.lktab[i];
  __syncthreads();
  const int nItems = min(A.counts[A.list], A.it1);
  if (nItems <= A.it0) return;
  const long long units = (long long)(nItems - A.it0) * A.nslots;
  const long long stride = (long long)gridDim.x * blockDim.x;
  unsigned int bn[NB];
  // unit uu's bytes b[3 i + j] = plane j (g11, g12, g22) of the family's person i (persons past the family: clamped reads
  // inside the site's block, never used)
  auto load = [&](long long uu) {
    const int uq = (int)(uu / A.nslots), k = (int)(uu - (long long)uq * A.nslots);
    const int item = A.items[A.it0 + uq];
    const int site = item >> 3, cfg = item & 7, r = A.ref[site];
    int a1, a2;
    if (A.vcf) { a1 = r & 15; a2 = r >> 4; }
    else if (cfg == 7) { a1 = A.res[(size_t)site * A.res_words + A.res_a1]; a2 = A.res[(size_t)site * A.res_words + A.res_a2]; }
    else cfg_alleles(cfg, r, &a1, &a2);
    const uint8_t* pl = A.pl + (size_t)site * A.np * 10;
    const uint8_t* P[3] = {pl + (size_t)gi(a1, a1) * A.np, pl + (size_t)gi(a1, a2) * A.np, pl + (size_t)gi(a2, a2) * A.np};
    const int p0 = A.slot_p0[k];
#pragma unroll
    for (int i = 0; i < NB / 3; i++) {
      const int pi = min(p0 + i, A.np - 1);
#pragma unroll
      for (int j = 0; j < 3; j++) bn[3 * i + j] = P[j][pi];
    }
  };
  long long u = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (u < units) load(u);
  for (; u < units; u += stride) {
    unsigned int b[NB];
#pragma unroll
    for (int i = 0; i < NB; i++) b[i] = bn[i];
    const int uq = (int)(u / A.nslots), k = (int)(u - (long long)uq * A.nslots);
    const int e = A.slot_e[k], q = e / A.T;
    double* out = A.coef + ((size_t)uq * A.max_ext + q) * A.dcap * A.T + (e - q * A.T);
    const int sig = A.slot_sig[k];
    if (u + stride < units) load(u + stride);
    switch (sig) {
)";
    for (size_t i = 0; i < shapes.size(); i++)
      s += "      case " + std::to_string(i) + ": " + shapes[i] + "(b, lk, out, A.T, A.dcap); break;\n";
    s += "    }\n  }\n}\n";
    for (size_t at; (at = s.find("NB")) != std::string::npos;) s.replace(at, 2, std::to_string(g_bapf));
    return s;
  }
  std::string s = R"(
extern "C" __global__ void __launch_bounds__(256) es_hoist_jit(Args A) {
  __shared__ double lk[256];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) lk[i] = A.lktab[i];
  __syncthreads();
  const int nItems = min(A.counts[A.list], A.it1);
  if (nItems <= A.it0) return;
  const long long units = (long long)(nItems - A.it0) * A.nslots;
  for (long long u = (long long)blockIdx.x * blockDim.x + threadIdx.x; u < units; u += (long long)gridDim.x * blockDim.x) {
    const int uq = (int)(u / A.nslots), k = (int)(u - (long long)uq * A.nslots);
    const int it = A.it0 + uq;
    const int item = A.items[it];
    const int site = item >> 3, cfg = item & 7, r = A.ref[site];
    int a1, a2;
    if (A.vcf) { a1 = r & 15; a2 = r >> 4; }
    else if (cfg == 7) { a1 = A.res[(size_t)site * A.res_words + A.res_a1]; a2 = A.res[(size_t)site * A.res_words + A.res_a2]; }
    else cfg_alleles(cfg, r, &a1, &a2);
    const uint8_t* pl = A.pl + (size_t)site * A.np * 10;
    const uint8_t* P11 = pl + (size_t)gi(a1, a1) * A.np;
    const uint8_t* P12 = pl + (size_t)gi(a1, a2) * A.np;
    const uint8_t* P22 = pl + (size_t)gi(a2, a2) * A.np;
    const int e = A.slot_e[k], q = e / A.T;
    double* out = A.coef + ((size_t)uq * A.max_ext + q) * A.dcap * A.T + (e - q * A.T);
    switch (A.slot_sig[k]) {
)";
  for (size_t i = 0; i < shapes.size(); i++)
    s += "      case " + std::to_string(i) + ": " + shapes[i] + "(P11, P12, P22, A.slot_p0[k], lk, out, A.T, A.dcap); break;\n";
  s += "    }\n  }\n}\n";
  return s;
}


// ---------------------------------------------------------------------------------------------------------------
// Genotype posteriors of one family shape (CalcPostProb_SingleExtendedPed_BA, FamilyLikelihoodSeq.cpp:171-216): for
// every person j and genotype s, the reference-order numeric BA peel at freq with j's penetrances zeroed but for s
// (FillZeroPenetrance :327-356).  The operations and their order are d_es_lk<3>'s (engine.hip), hence the
// reference's, term by term; folding x * 1 -> x, dropping + 0 and 0-products (every value is finite and >= 0) keeps
// every bit.  Computations that do not depend on j's zeroed penetrance are generated once (Gen::def memo), so the 3n
// peels of a family share their common prefix.
struct NumPeel {
  Gen& G;
  explicit NumPeel(Gen& g) : G(g) {}
  static bool is0(const std::string& x) { return x == "0.0"; }
  std::string mul(const std::string& x, const std::string& y) {
    if (is0(x) || is0(y)) return "0.0";
    if (x == "1.0") return y;
    if (y == "1.0") return x;
    return G.def(x + " * " + y);
  }
  std::string add(const std::string& acc, const std::string& x) {   // acc + x, acc "" = the sum's 0.0 start
    if (acc.empty()) return x;
    if (is0(x)) return acc;
    if (is0(acc)) return x;
    return G.def(acc + " + " + x);
  }
};

std::string gen_post_family(const Family& F, int chrom, const double (*T)[27], const std::string& name) {
  Gen G;
  NumPeel N(G);
  const int n = F.n;
  const bool X = chrom == PM_CHR_X, Y = chrom == PM_CHR_Y, MT = chrom == PM_CHR_MT;
  static const char* plane[3] = {"P11", "P12", "P22"};
  std::string body;
  // founder priors (d_es_lk: pr[] per founder, same expressions)
  const std::string q0 = G.def("fq * fq"), q1 = G.def("2 * fq * (1 - fq)"), q2 = G.def("(1 - fq) * (1 - fq)");
  const std::string h0 = "fq", h2 = G.def("1 - fq");
  std::vector<std::vector<std::string>> pen(n, std::vector<std::string>(3));
  for (int i = 0; i < n; i++)
    for (int s = 0; s < 3; s++) pen[i][s] = G.def(std::string("lk[") + plane[s] + "[p0 + " + std::to_string(i) + "]]");
  auto peel = [&](int zp, int zs) {
    std::vector<std::vector<std::string>> P(n, std::vector<std::string>(3));
    for (int i = 0; i < n; i++) {
      const int sx = F.sex[i];
      const bool fo = F.founder[i] != 0;
      std::string pr[3] = {"0.0", "0.0", "0.0"};
      if (i < F.nf) {
        pr[0] = q0; pr[1] = q1; pr[2] = q2;
        if (X && sx == MALE) { pr[0] = h0; pr[1] = "0.0"; pr[2] = h2; }
        if (Y) { if (sx == MALE) { pr[0] = h0; pr[1] = "0.0"; pr[2] = h2; } else { pr[0] = pr[1] = pr[2] = "1.0"; } }
        if (MT) { pr[0] = h0; pr[1] = "0.0"; pr[2] = h2; }
      }
      for (int s = 0; s < 3; s++) {
        const std::string pe = (zp == i && s != zs) ? std::string("0.0") : pen[i][s];
        P[i][s] = (Y && sx == FEMALE) ? std::string("1.0") : (fo ? N.mul(pr[s], pe) : pe);
      }
    }
    std::map<int, std::vector<std::string>> M;
    int fin = -1;
    for (const int2& S : F.steps) {
      const int type = S.x & 255, from0 = (S.x >> 8) & 255, from1 = (S.x >> 16) & 255, to0 = (S.x >> 24) & 255;
      const int slot = (S.y >> 8) & 255, create = (S.y >> 16) & 1, fa2mo = (S.y >> 17) & 1;
      fin = to0;
      if (type == 1) {
        const int off = from0, csex = F.sex[off];
        if (create || !M.count(slot)) M[slot].assign(9, "1.0");
        for (int i = 0; i < 3; i++)
          for (int j = 0; j < 3; j++) {
            std::string sum;
            for (int k = 0; k < 3; k++) {
              const double t = tba(T, chrom, csex, i, j, k);
              sum = N.add(sum, t == 0.0 ? std::string("0.0") : N.mul(t == 1.0 ? std::string("1.0") : lit(t), P[off][k]));
            }
            M[slot][i * 3 + j] = N.mul(M[slot][i * 3 + j], sum.empty() ? std::string("0.0") : sum);
          }
      } else if (type == 2) {
        const int sf = from0, stt = to0;
        for (int i = 0; i < 3; i++) {
          std::string sum;
          for (int j = 0; j < 3; j++) {
            if (slot == 255) sum = N.add(sum, P[sf][j]);
            else sum = N.add(sum, N.mul(P[sf][j], M[slot][fa2mo ? j * 3 + i : i * 3 + j]));
          }
          P[stt][i] = N.mul(P[stt][i], sum.empty() ? std::string("0.0") : sum);
        }
      } else {
        const int fa = from0, mo = from1, off = to0, csex = F.sex[off];
        std::string sum[3];
        for (int i = 0; i < 3; i++)
          for (int j = 0; j < 3; j++) {
            const std::string w = slot == 255 ? N.mul(P[fa][i], P[mo][j]) : N.mul(N.mul(P[fa][i], M[slot][i * 3 + j]), P[mo][j]);
            for (int k = 0; k < 3; k++) {
              const double t = tba(T, chrom, csex, i, j, k);
              sum[k] = N.add(sum[k], t == 0.0 ? std::string("0.0") : N.mul(t == 1.0 ? std::string("1.0") : lit(t), w));
            }
          }
        for (int k = 0; k < 3; k++) P[off][k] = N.mul(P[off][k], sum[k].empty() ? std::string("0.0") : sum[k]);
      }
    }
    std::string L;
    for (int i = 0; i < 3; i++) L = N.add(L, P[fin][i]);
    return L.empty() ? std::string("0.0") : L;
  };
  for (int j = 0; j < n; j++) {
    const int sx = F.sex[j];
    if (Y && sx == FEMALE) {   // CalcPostProb_SingleExtendedPed_BA: chrY females get no posterior ('.')
      body += "  emit(calls, out0 + p0 + " + std::to_string(j) + ", 0.0, 0.0, 0.0, " + std::to_string((int)PM_LBL_DOT) +
              ", thr, vcf, 1);\n";
      continue;
    }
    const std::string l0 = peel(j, 0), l1 = peel(j, 1), l2 = peel(j, 2);
    const int lab = (Y || MT || (X && sx == MALE)) ? PM_LBL_VCF_HAPLOID : PM_LBL_VCF_DIPLOID;   // d_vcf_label
    body += "  emit(calls, out0 + p0 + " + std::to_string(j) + ", " + l0 + ", " + l1 + ", " + l2 + ", " + std::to_string(lab) +
            ", thr, vcf, 0);\n";
  }
  return "__device__ __attribute__((noinline)) void " + name +
         "(const unsigned char* __restrict__ P11, const unsigned char* __restrict__ P12, const unsigned char* __restrict__ P22, "
         "int p0, const double* __restrict__ lk, double fq, const double* __restrict__ thr, void* calls, size_t out0, int vcf) {\n" +
         G.code + body + "}\n";
}

const char* kPostPrologue = R"(
struct PostArgs {
  const int* counts; const int* row_site; const char* res; const uint8_t* pl; const double* lktab; const double* gq_thr;
  void* calls; const int* fam_p0; const int* fam_sig;
  int nfams, np, vcf, res_bytes, off_a1, off_a2, off_maxidx, off_af;
  double theta;
};
struct GenoCall { double dosage; short best; short gq; signed char label; signed char pad[3]; };
struct VcfCall { signed char best; signed char gq; signed char label; signed char pad; };
// d_gq (engine.hip): GQ of OutputVCF :1818-1820 from the host's glibc thresholds, exact for every double
__device__ __forceinline__ int gq_of(double pb, const double* thr) {
  const double q = 1. - pb;
  const int g = (int)(-3.01029995664f * __builtin_amdgcn_logf((float)q) + 0.5f);   // (bare v_log_f32: see d_gq)
  const int base = min(max(g - 2, 0), 96);
  int k = base;
  for (int i = 0; i < 4; i++) k += q < thr[base + i] ? 1 : 0;
  return pb > 0.9999999999 ? 100 : k;
}
// k_posterior_es's tail: post = l / sum, best = d_best3(l), GQ of post[best], DS = post12 + 2 post22
__device__ __forceinline__ void emit(void* calls, size_t idx, double l11, double l12, double l22, int label, const double* thr,
                                     int vcf, int zero) {
  double post[3] = {0.0, 0.0, 0.0};
  int best = 0;
  if (!zero) {
    const double sum = l11 + l12 + l22;
    if (sum != 0) { post[0] = l11 / sum; post[1] = l12 / sum; post[2] = l22 / sum; }
    double m = l11;
    if (l12 > m) { m = l12; best = 1; }
    if (l22 > m) { m = l22; best = 2; }
  }
  const int gq = gq_of(post[best], thr);
  if (vcf) {
    VcfCall c; c.best = (signed char)best; c.gq = (signed char)gq; c.label = (signed char)label; c.pad = 0;
    ((VcfCall*)calls)[idx] = c;
    return;
  }
  GenoCall c; c.dosage = post[1] + post[2] * 2; c.best = (short)best; c.gq = (short)gq; c.label = (signed char)label;
  c.pad[0] = c.pad[1] = c.pad[2] = 0;
  ((GenoCall*)calls)[idx] = c;
}
)";

std::string gen_post_kernel(const std::vector<std::string>& shapes) {
  std::string s = R"(
extern "C" __global__ void __launch_bounds__(256) es_post_jit(PostArgs A) {
  __shared__ double lk[256];
  __shared__ double thr[101];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) lk[i] = A.lktab[i];
  for (int i = threadIdx.x; i < 101; i += blockDim.x) thr[i] = A.gq_thr[i];
  __syncthreads();
  const long long work = (long long)A.counts[3] * A.nfams;
  for (long long u = (long long)blockIdx.x * blockDim.x + threadIdx.x; u < work; u += (long long)gridDim.x * blockDim.x) {
    const int row = (int)(u / A.nfams), k = (int)(u - (long long)row * A.nfams);
    const int site = A.row_site[row];
    const char* R = A.res + (size_t)site * A.res_bytes;
    const int a1 = *(const int*)(R + A.off_a1), a2 = *(const int*)(R + A.off_a2);
    const double fq = (*(const int*)(R + A.off_maxidx) == 0) ? 1 - A.theta : *(const double*)(R + A.off_af);   // main.cpp:576-587
    const uint8_t* pl = A.pl + (size_t)site * A.np * 10;
    const uint8_t* P11 = pl + (size_t)gi(a1, a1) * A.np;
    const uint8_t* P12 = pl + (size_t)gi(a1, a2) * A.np;
    const uint8_t* P22 = pl + (size_t)gi(a2, a2) * A.np;
    const size_t out0 = (size_t)row * A.np;
    switch (A.fam_sig[k]) {
)";
  for (size_t i = 0; i < shapes.size(); i++)
    s += "      case " + std::to_string(i) + ": " + shapes[i] + "(P11, P12, P22, A.fam_p0[k], lk, fq, thr, A.calls, out0, A.vcf); break;\n";
  s += "    }\n  }\n}\n";
  return s;
}


// ---------------------------------------------------------------------------------------------------------------
// Wave-cooperative hoisting (--denovo engines: 10-state peels, whose marriage partials -- 100 entries x coefficients
// -- do not fit one thread's registers).  One (item, family) per wave, as engine.hip's generic k_es_hoist, but
// compiled per family shape: the workspace layout, every step's degrees and every loop bound are constants, so a
// phase is a few unrolled multiply-adds per lane between wave-level barriers, with no schedule or layout loads
// and no run-time divisions.  Variants per shape: 10-state (de novo items), bi-allelic (cfg-7 items), and "top"
// (the de novo monomorphism item: the f^D coefficient only, every degree 0).
// The de novo transmission rows of a type-1 step's pairs: from the (cache-resident) global table, or held in 20
// registers for the whole kernel (PM_ES_TR=reg: 149 VGPRs, 3 waves per SIMD; capped at 128 with 19 spilled)
bool g_tr_regs = false;
bool g_prof = false;   // PM_ES_PROF=1: es_hoist_wave accumulates per-part clock cycles into Args::prof
bool g_pack = true;    // PM_ES_PACK=0: independent type-2 steps one phase each
// PM_ES_REGP: how a type-1 phase reads the offspring coefficients a preceding type-2 phase computed -- 0 from LDS,
// 1 all by v_readlane (the non-founder is then never stored), 2 (default) every other offspring of a run by
// v_readlane and the rest from LDS: the readlanes are VALU work and the LDS reads LDS work, and the two pipes are
// best balanced half and half (ext10: 0.667 / 0.617 / 0.555 ms per hoisting launch)
int g_regp = 2;
bool g_regf = true;    // PM_ES_REGF=0: pristine founders stored and read from LDS (with PM_ES_REGP != 0)
int g_expt = 0;        // PM_ES_EXPT=1/2: timing experiments only (results wrong), see the uses
// Family pairs (PM_ES_PAIR, default on): each half-wave (32 lanes) hoists one family of a pair of same-shape families
// of the task, so every phase whose elements fit 32 lanes (type-2 steps over 10 states, founder-sparse type-1 runs
// over 30 pairs, the final sum) does two families' work per instruction; g_wl = the lanes per family (64 or 32).
// Pair mode reads partials across lanes through LDS only (no v_readlane from fixed lanes: PM_ES_REGP / REGF off).
bool g_pair = false;
// families per wave (PM_ES_FPW: 1, 2 -- the pair mode above -- or 4): g_wl = 64 / g_fpw lanes per family
int g_fpw = 1;
bool g_wspack = true;     // PM_ES_WSPACK=0: part-2 regions laid out in order instead of packed by live range
bool g_fence = true;      // PM_ES_FENCE=0: wave_sync without the wavefront-scope fences (measured 2% slower)
bool g_xcd = true;        // PM_ES_XCD=0: units dealt to the blocks in plain order
bool g_no_penp = false;   // PM_ES_PENP=0: leaf offspring partials stored and read from the workspace
// dense 10-state type-3 steps with a marriage partial (the plain transmission, quirk :1391): each child state's sum runs
// over its non-zero parent pairs from an LDS list (t3z / t3n, filled from kT3z / kT3n at kernel start); g_t3z: some
// family of the kernel uses it (PM_ES_T3Z=0, g_no_t3z: the 100-pair loop over the global table)
bool g_t3z = false;
bool g_no_t3z = false;
int g_wl = 64;
// PM_ES_FACT=1 (opt-in experiment): a dense 10-state type-1 run through T10dn = T10 * M (SetTransmissionMatrix_denovo
// :787-810) -- P' = M P per offspring coefficient (lanes over (genotype, coefficient)), then per pair 0.25 x the sum
// of P' at its four Mendelian children, instead of sum_k T10dn(e, k) P(k): the same value in real arithmetic, a
// different rounding order (not the reference's), ~3x fewer operations and no per-lane transmission-row loads
bool g_fact = false;

struct WaveGen {
  std::string code;
  void loop(int N, const std::string& body) {   // lanes over N elements x, then a wave barrier
    code += "  for (int x = lane; x < " + std::to_string(N) + "; x += 64) {\n" + body + "  }\n  wave_sync();\n";
  }
};

// ops: the FP64 operations the generated phases perform (summed over their work elements: the useful lane-operations,
// whatever the lanes' occupancy)
// part (10-state variants only): 0 the whole peel; 1 the cfg-independent prefix -- the 10-state penetrances of
// non-founders no step changes and the type-1 steps that peel them into marriage partials no cfg-dependent step
// writes (leaf steps, run first: nothing they read or write is touched by an earlier step) -- and 2 the rest (the
// other persons' partials, the other steps, the final sum).  Part 1 once and part 2 per item give part 0's values for
// the de novo items of one site (they differ only in the founder priors' genotypes; the top variant's leaf steps are
// the same degree-0 products).  Parts lay out the workspace by the 10-state variant's degrees, top or not.
std::string gen_wave_family(const Family& F, int chrom, int NS, bool top, const std::string& name, int* ws_doubles, double* ops,
                            int part = 0, int multi = 1) {
  const int n = F.n;
  const bool X = chrom == PM_CHR_X, Y = chrom == PM_CHR_Y, MT = chrom == PM_CHR_MT;
  // degrees through the peel (poly_layout's rule), capacities, temporaries (type 3 only: the W(i, j) products)
  std::vector<int> d0(n), dP(n), capP(n);
  std::map<int, int> dM, capM;
  int tmp = 1;
  // founder-sparse type-3 steps (see sp3): 10 states, one item per call, not switched off (PM_ES_SP3=0)
  const char* es3 = getenv("PM_ES_SP3");
  const bool sp3_on = NS == 10 && !(part == 2 && std::max(1, multi) > 1) && !(es3 && es3[0] == '0');
  struct StepDeg { int a, b, c, e; };
  std::vector<StepDeg> sd;
  for (int pass = (part && top) ? 0 : 1; pass < 2; pass++) {   // (pass 0: the 10-state variant's capacities)
  const bool tp = pass == 1 && top;
  sd.clear(); dM.clear();
  for (int i = 0; i < n; i++) {
    const bool fo = F.founder[i] && i < F.nf;
    const int sx = F.sex[i];
    const int dfull = !fo ? 0 : (Y && sx == FEMALE) ? 0 : (((X || Y) && sx == MALE) || MT) ? 1 : 2;
    d0[i] = dP[i] = tp ? 0 : dfull;
    capP[i] = std::max(pass ? capP[i] : 0, dP[i] + 1);
  }
  for (const int2& S : F.steps) {
    const int type = S.x & 255, from0 = (S.x >> 8) & 255, from1 = (S.x >> 16) & 255, to0 = (S.x >> 24) & 255;
    const int slot = (S.y >> 8) & 255, create = (S.y >> 16) & 1;
    StepDeg g{0, 0, 0, 0};
    if (type == 1) {
      g.a = dP[from0]; g.b = create ? 0 : dM[slot];
      dM[slot] = g.a + g.b;
      capM[slot] = std::max(capM[slot], dM[slot] + 1);
    } else if (type == 2) {
      g.a = dP[from0]; g.b = slot == 255 ? 0 : dM[slot]; g.c = dP[to0];
      dP[to0] = g.a + g.b + g.c;
      capP[to0] = std::max(capP[to0], dP[to0] + 1);
    } else {
      g.a = dP[from0]; g.b = slot == 255 ? 0 : dM[slot]; g.c = dP[from1]; g.e = dP[to0];
      dP[to0] = g.a + g.b + g.c + g.e;
      capP[to0] = std::max(capP[to0], dP[to0] + 1);
      // (the W(i, j) products: a founder-sparse step -- sp3 below -- keeps only its supports' pairs; pterms' sizes)
      auto supp = [&](int f) {
        if (!(NS == 10 && sp3_on && F.founder[f] && f < F.nf)) return NS;
        const int sx = F.sex[f];
        const int dfull = (Y && sx == FEMALE) ? 0 : (((X || Y) && sx == MALE) || MT) ? 1 : 2;
        return top ? (dfull > 0 ? 1 : 3) : dfull == 1 ? 2 : 3;
      };
      tmp = std::max(tmp, supp(from0) * supp(from1) * (g.a + g.b + g.c + 1));
    }
    sd.push_back(g);
  }
  }
  // leaf steps (part 1) and the persons only they read; pristine[s]: the founder "from" of step s still holds its
  // prior x penetrance partial (3 non-zero states), so a type-2 step sums over those 3 states only
  const int nst = (int)F.steps.size();
  std::vector<char> leaf(nst, 0), leafp(n, 0), pristine(nst, 0);
  if (NS == 10) {
    auto ty = [&](int k) { return F.steps[k].x & 255; };
    auto fr = [&](int k) { return (F.steps[k].x >> 8) & 255; };
    auto to = [&](int k) { return (F.steps[k].x >> 24) & 255; };
    auto sl = [&](int k) { return (F.steps[k].y >> 8) & 255; };
    auto fo = [&](int i) { return F.founder[i] && i < F.nf; };
    std::vector<char> isto(n, 0), touched(n, 0);
    for (int k = 0; k < nst; k++)
      if (ty(k) != 1) isto[to(k)] = 1;
    for (int k = 0; k < nst; k++) {
      if (ty(k) == 2 && fo(fr(k)) && !touched[fr(k)]) pristine[k] = 1;
      if (ty(k) != 1) touched[to(k)] = 1;
      // a leaf step reads a non-founder's penetrance partial that no step ever changes
      if (ty(k) == 1 && !fo(fr(k)) && !isto[fr(k)]) leaf[k] = 1;
    }
    // ... into a marriage partial that only leaf steps write, and that no step reads before the last of them
    for (bool changed = true; changed;) {
      changed = false;
      std::map<int, int> nonleaf_writer;
      for (int k = 0; k < nst; k++)
        if (ty(k) == 1 && !leaf[k]) nonleaf_writer[sl(k)] = 1;
      for (int k = 0; k < nst; k++) {
        if (leaf[k] && nonleaf_writer.count(sl(k))) { leaf[k] = 0; changed = true; }
        if (ty(k) == 1 || sl(k) == 255) continue;
        for (int k2 = k + 1; k2 < nst; k2++)
          if (leaf[k2] && ty(k2) == 1 && sl(k2) == sl(k)) { leaf[k2] = 0; changed = true; }
      }
    }
    for (int k = 0; k < nst; k++)
      if (leaf[k]) leafp[fr(k)] = 1;
  }
  // workspace layout: persons' partials, marriage partials, the type-3 products.  Parts put the leaf prefix's
  // regions first (a task's items share them) and give each of the M items of a part-2 function its own copy of the
  // rest, cb = c * NSZ doubles further on
  // a pristine founder's non-zero states (q: 0 g11, 1 g12, 2 g22) and their coefficient u, in the dense loop's order
  // of u at one j: prior x penetrance (SetFounderPriors), the top variant's f^D term only
  auto pterms = [&](int f) {
    const int sx = F.sex[f];
    const int dfull = (Y && sx == FEMALE) ? 0 : (((X || Y) && sx == MALE) || MT) ? 1 : 2;
    std::vector<std::pair<int, int>> t;
    if (top) {
      if (dfull > 0) t = {{0, 0}};
      else t = {{2, 0}, {1, 0}, {0, 0}};
    } else if (d0[f] == 2) t = {{2, 0}, {1, 1}, {0, 2}};
    else if (d0[f] == 1) t = {{2, 0}, {0, 1}};
    else t = {{2, 0}, {1, 0}, {0, 0}};
    return t;
  };
  // runs of consecutive type-1 steps of this part (one phase each in the 10-state code), and their founder-sparse
  // rows: when a run writes one marriage partial and its only later reader is a pristine type-2 step (the founder
  // spouse F peeled into the other), that step reads the rows of F's non-zero states only (2-3 of 10; 1 in the top
  // variant), so only those pairs are computed (lanes over F's states x the spouse's).  In part 2 a partial whose
  // writers all sit in such a run is stored compactly, row q * 10 + spouse state for F's q-th term.
  auto inpart = [&](int k2) { return !((part == 1 && !leaf[k2]) || (part == 2 && leaf[k2])); };
  auto run_of = [&](int k0) {
    std::vector<int> run;
    for (int k2 = k0; k2 < nst; k2++) {
      if (!inpart(k2)) continue;
      if ((F.steps[k2].x & 255) != 1) break;
      run.push_back(k2);
    }
    return run;
  };
  struct Sparse { std::vector<std::pair<int, int>> terms; bool father = false, compact = false; };
  auto sparse_of = [&](const std::vector<int>& run) {
    Sparse sp;
    if (NS != 10 || part == 1 || run.empty()) return sp;
    const int sl0 = (F.steps[run[0]].y >> 8) & 255;
    for (int k2 : run)
      if (((F.steps[k2].y >> 8) & 255) != sl0) return sp;
    int readers = 0, rk = -1;
    bool writes_after = false, writes_before = false;
    for (int k2 = run.back() + 1; k2 < nst; k2++) {
      if (!inpart(k2) || ((F.steps[k2].y >> 8) & 255) != sl0) continue;
      if ((F.steps[k2].x & 255) == 1) writes_after = true;
      else { readers++; rk = k2; }
    }
    for (int k2 = 0; k2 < run[0]; k2++)
      if ((F.steps[k2].x & 255) == 1 && ((F.steps[k2].y >> 8) & 255) == sl0) writes_before = true;
    if (readers == 1 && !writes_after && (F.steps[rk].x & 255) == 2 && pristine[rk]) {
      sp.terms = pterms((F.steps[rk].x >> 8) & 255);
      sp.father = (F.steps[rk].y >> 17) & 1;
      sp.compact = part == 2 && !writes_before && multi <= 1;
    }
    return sp;
  };
  std::map<int, int> crows;   // compactly stored marriage partials: slot -> rows
  if (NS == 10 && part == 2)
    for (int k = 0; k < nst; k++) {
      if (!inpart(k) || (F.steps[k].x & 255) != 1 || (k > 0 && inpart(k - 1) && (F.steps[k - 1].x & 255) == 1)) continue;
      const std::vector<int> run = run_of(k);
      const Sparse sp = sparse_of(run);
      if (sp.compact) crows[(F.steps[k].y >> 8) & 255] = 10 * (int)sp.terms.size();
    }
  const int M = part == 2 ? std::max(1, multi) : 1;
  if (g_fact && NS == 10 && M == 1)   // (PM_ES_FACT: the P' rows of a dense type-1 run in the temporaries' region)
    for (int k = 0; k < nst; k++) {
      if (!inpart(k) || (F.steps[k].x & 255) != 1) continue;
      const std::vector<int> run = run_of(k);
      int sz = 0;
      for (int k2 : run) sz += 10 * (sd[k2].a + 1);
      tmp = std::max(tmp, sz);
    }
  std::map<int, int> leafs;   // the marriage slots the leaf steps write
  for (int k = 0; k < nst; k++)
    if (leaf[k]) leafs[(F.steps[k].y >> 8) & 255] = 1;
  // (computed before the layout: persons never stored get no workspace region)
  std::vector<char> regf(n, 0), regn(n, 0), iinit(n, 0);
  // (the initial partials formed in the type-2 lanes need no cross-lane read: pair mode keeps them too)
  if (NS == 10 && part == 2 && multi <= 1 && (g_regp || g_pair)) {
    const int finp = (F.steps.back().x >> 24) & 255;
    // (pair mode: such a founder's terms read its penetrance straight from the PEN table, no v_readlane)
    for (int i = 0; i < n; i++) regf[i] = ((g_regp && g_regf) || g_pair) && F.founder[i] && i < F.nf && !leafp[i] && i != finp;
    for (int k = 0; k < nst; k++) {
      if (!inpart(k)) continue;
      const int ty2 = F.steps[k].x & 255, f0 = (F.steps[k].x >> 8) & 255, f1 = (F.steps[k].x >> 16) & 255, t0 = (F.steps[k].x >> 24) & 255;
      if (ty2 == 2) { regf[t0] = 0; if (!pristine[k]) regf[f0] = 0; }
      else if (ty2 == 3) regf[f0] = regf[f1] = regf[t0] = 0;
      else regf[f0] = 0;
    }
    // non-founders whose partial is the penetrance until one type-2 step peels a spouse into it, and is then read
    // only as a type-1 offspring (by v_readlane from that step's registers): never stored either
    std::vector<int> t2to(n, 0);
    for (int i = 0; i < n; i++) regn[i] = !(F.founder[i] && i < F.nf) && !leafp[i] && i != finp;
    for (int k = 0; k < nst; k++) {
      if (!inpart(k)) continue;
      const int ty2 = F.steps[k].x & 255, f0 = (F.steps[k].x >> 8) & 255, f1 = (F.steps[k].x >> 16) & 255, t0 = (F.steps[k].x >> 24) & 255;
      if (ty2 == 2) { t2to[t0]++; regn[f0] = 0; }
      else if (ty2 == 3) regn[f0] = regn[f1] = regn[t0] = 0;
      else if (!t2to[f0]) regn[f0] = 0;   // (a type-1 read before the type-2 step)
    }
    for (int i = 0; i < n; i++)
      if (t2to[i] != 1 || g_regp == 2 || !g_regp) regn[i] = 0;
    // persons whose first use is as the to-person of a type-2 step: their initial partial (penetrance, or prior x
    // penetrance) is formed inside that step's lanes instead of being stored and read back
    std::vector<char> seen(n, 0);
    for (int k = 0; k < nst; k++) {
      if (!inpart(k)) continue;
      const int ty2 = F.steps[k].x & 255, f0 = (F.steps[k].x >> 8) & 255, f1 = (F.steps[k].x >> 16) & 255, t0 = (F.steps[k].x >> 24) & 255;
      if (ty2 == 2 && !seen[t0] && !regf[t0]) iinit[t0] = 1;
      seen[f0] = 1;
      if (ty2 != 1) seen[t0] = 1;
      if (ty2 == 3) seen[f1] = 1;
    }
    for (int i = 0; i < n; i++)
      if (leafp[i]) iinit[i] = 0;
  }
  // leaf offspring (parts): a non-founder whose partial is its penetrance, never changed, read by leaf steps only --
  // the steps read PEN directly (the site's penetrances stay in the slice for the task), no region, no init
  std::vector<char> penp(n, 0);
  if (NS == 10 && part && !g_no_penp)
    for (int i = 0; i < n; i++) penp[i] = leafp[i] && !(F.founder[i] && i < F.nf);
  std::vector<int> po(n);
  std::map<int, int> mo;
  int off = 0, LSZ = 0;
  for (int L = part ? 1 : 0; L >= 0; L--) {
    for (int i = 0; i < n; i++)
      if (!part || leafp[i] == L) {
        po[i] = off;
        if (!regf[i] && !regn[i] && !penp[i]) off += NS * capP[i];   // (a register- or PEN-read founder / register-only non-founder: no region)
      }
    for (auto& m : capM)
      if (!part || (int)leafs.count(m.first) == L) {
        mo[m.first] = off;
        off += (crows.count(m.first) ? crows[m.first] : NS * NS) * m.second;
      }
    if (L == 1) LSZ = off;
  }
  int TB = off, NSZ = off + tmp - LSZ;
  // Part 2 (the per-item rest, the top rest): its own regions packed by live range (g_wspack, PM_ES_WSPACK=0: in
  // order).  A region is live from the phase of its first write to the phase of its last read; phases are counted
  // conservatively (consecutive steps of one type share one, a type-3 step is one, the initial partials' phase is -1,
  // the final sum the last), and a region may take the place of one whose live range ended in an earlier phase: a
  // wave_sync lies between them.  Smaller slices -> more slices in a CU's LDS -> more waves in flight.
  if (part == 2 && M == 1 && NS == 10 && !g_fact && g_wspack) {
    std::vector<int> ph(nst, -2);
    int cur = -1, prevt = -1;
    for (int k = 0; k < nst; k++) {
      if (!inpart(k)) continue;
      const int t = F.steps[k].x & 255;
      if (t != prevt || t == 3) cur++;
      prevt = t;
      ph[k] = cur;
    }
    struct Reg { int size = 0, lo = 1 << 30, hi = -3, off = 0; };
    std::map<int, Reg> rg;   // person i, marriage slot (1000 + slot), the type-3 temporaries (-1)
    auto touch = [&](int id, int size, int p) {
      Reg& r = rg[id];
      r.size = size;
      r.lo = std::min(r.lo, p);
      r.hi = std::max(r.hi, p);
    };
    auto stored = [&](int i) { return !leafp[i] && !regf[i] && !regn[i] && !penp[i]; };
    auto msize = [&](int sl) { return (crows.count(sl) ? crows[sl] : NS * NS) * capM[sl]; };
    for (int i = 0; i < n; i++)
      if (stored(i) && !iinit[i]) touch(i, NS * capP[i], -1);   // (the initial partials written up front)
    for (int k = 0; k < nst; k++) {
      if (!inpart(k)) continue;
      const int t = F.steps[k].x & 255, f0 = (F.steps[k].x >> 8) & 255, f1 = (F.steps[k].x >> 16) & 255, t0 = (F.steps[k].x >> 24) & 255;
      const int sl = (F.steps[k].y >> 8) & 255;
      if (stored(f0)) touch(f0, NS * capP[f0], ph[k]);
      if (t == 3 && stored(f1)) touch(f1, NS * capP[f1], ph[k]);
      if (t != 1 && stored(t0)) touch(t0, NS * capP[t0], ph[k]);
      if (sl != 255 && !leafs.count(sl)) touch(1000 + sl, msize(sl), ph[k]);
      if (t == 3) touch(-1, tmp, ph[k]);
    }
    const int fin_ = (F.steps.back().x >> 24) & 255;
    if (stored(fin_)) touch(fin_, NS * capP[fin_], cur + 1);
    // first fit over a few placement orders (the first write, the size, the live-range length; ties by the others),
    // keeping the smallest footprint
    std::vector<int> ids;
    for (auto& r : rg) ids.push_back(r.first);
    auto fit = [&](const std::vector<int>& order, bool commit) {
      std::vector<std::pair<int, int>> pl;   // (id, offset)
      int t_ = LSZ;
      for (int id : order) {
        const Reg& r = rg[id];
        int o = LSZ;
        for (bool moved = true; moved;) {
          moved = false;
          for (auto& q : pl) {
            const Reg& a = rg[q.first];
            const bool live = a.hi >= r.lo && r.hi >= a.lo;
            if (live && o < q.second + a.size && q.second < o + r.size) { o = q.second + a.size; moved = true; }
          }
        }
        pl.push_back({id, o});
        t_ = std::max(t_, o + r.size);
      }
      if (commit)
        for (auto& q : pl) rg[q.first].off = q.second;
      return t_;
    };
    std::vector<std::vector<int>> orders;
    for (int key = 0; key < 3; key++) {
      std::vector<int> o = ids;
      std::stable_sort(o.begin(), o.end(), [&](int a, int b) {
        const Reg &x = rg[a], &y = rg[b];
        if (key == 0 && x.lo != y.lo) return x.lo < y.lo;
        if (key == 2 && x.hi - x.lo != y.hi - y.lo) return x.hi - x.lo > y.hi - y.lo;
        if (x.size != y.size) return x.size > y.size;
        return x.lo < y.lo;
      });
      orders.push_back(o);
    }
    size_t best = 0;
    int top_ = fit(orders[0], false);
    for (size_t q = 1; q < orders.size(); q++) {
      const int t_ = fit(orders[q], false);
      if (t_ < top_) { top_ = t_; best = q; }
    }
    fit(orders[best], true);
    for (auto& a : rg)   // (the invariant the placement keeps: regions live in a common phase never share a double)
      for (auto& b : rg)
        if (a.first < b.first && a.second.hi >= b.second.lo && b.second.hi >= a.second.lo &&
            a.second.off < b.second.off + b.second.size && b.second.off < a.second.off + a.second.size) {
          fprintf(stderr, "es_jit: workspace regions %d and %d overlap while live (%s)\n", a.first, b.first, name.c_str());
          abort();
        }
    for (auto& r : rg) {
      if (r.first == -1) TB = r.second.off;
      else if (r.first >= 1000) mo[r.first - 1000] = r.second.off;
      else po[r.first] = r.second.off;
    }
    if (!rg.count(-1)) TB = top_;   // (no type-3 step: tmp = 1, above the rest)
    NSZ = std::max(1, (rg.count(-1) ? top_ : top_ + tmp) - LSZ);
  }
  // (the leaf prefix writes its own regions only -- and with PM_ES_FACT its P' rows in the temporaries' region)
  *ws_doubles = part == 1 ? (g_fact && NS == 10 ? TB + tmp : LSZ) : LSZ + M * NSZ;
  if (getenv("PM_JIT_LAYOUT")) {
    fprintf(stderr, "layout %s NS %d part %d top %d: LSZ %d NSZ %d tmp %d ws %d |", name.c_str(), NS, part, (int)top, LSZ, NSZ, tmp, *ws_doubles);
    for (int i = 0; i < n; i++) fprintf(stderr, " p%d:%d%s", i, (!regf[i] && !regn[i]) ? NS * capP[i] : 0, leafp[i] ? "L" : "");
    for (auto& m : capM) fprintf(stderr, " m%d:%d", m.first, (crows.count(m.first) ? crows[m.first] : NS * NS) * m.second);
    fprintf(stderr, " | offsets");
    for (int i = 0; i < n; i++) fprintf(stderr, " p%d@%d", i, po[i]);
    for (auto& m : capM) fprintf(stderr, " m%d@%d", m.first, mo[m.first]);
    fprintf(stderr, " tb@%d\n", TB);
  }
  auto S = [](long v) { return std::to_string(v); };
  const std::string nsS = S(NS), nsq = S(NS * NS), R = S((NS * NS + g_wl - 1) / g_wl), WL = S(g_wl);
  const bool mc = part == 2 && M > 1;   // offsets of the item's own regions carry cb (several items per call)
  auto PO = [&](int i) { return mc && !leafp[i] ? "(" + S(po[i]) + " + cb)" : S(po[i]); };
  auto MOf = [&](int s) { return mc && !leafs.count(s) ? "(" + S(mo[s]) + " + cb)" : S(mo[s]); };
  const std::string TBs = mc ? "(" + S(TB) + " + cb)" : S(TB);
  // a phase with lanes over (item c, index var < N); part 2: c's genotypes (packed 8 bits per item) and offset cb
  auto lanes = [&](int N, const std::string& var, const std::string& body) -> std::string {
    if (!mc) return "  for (int " + var + " = lane; " + var + " < " + S(N) + "; " + var + " += " + WL + ") {\n" + body + "  }\n";
    return "  for (int x_ = lane; x_ < " + S(M * N) + "; x_ += " + WL + ") {\n    const int c = x_ / " + S(N) + ", " + var + " = x_ - c * " +
           S(N) + ", cb = c * " + S(NSZ) + ";\n    const int g11 = (gg11 >> (8 * c)) & 255, g12 = (gg12 >> (8 * c)) & 255, "
           "g22 = (gg22 >> (8 * c)) & 255;\n    (void)g11; (void)g12; (void)g22; (void)cb;\n" + body + "  }\n";
  };
  // a phase with lanes over the pairs e: every item's work in the lane, unrolled
  auto items = [&](const std::string& body) -> std::string {
    if (!mc) return body;
    return "#pragma unroll\n      for (int c = 0; c < " + S(M) + "; c++) {\n      const int cb = c * " + S(NSZ) + ";\n" + body + "      }\n";
  };
  std::string code = mc ? "" : "  const int g11 = gg11, g12 = gg12, g22 = gg22;\n  (void)g11; (void)g12; (void)g22;\n";
  for (int i = 0; i < n; i++)
    if (regf[i] && !g_pair) code += "  double fp" + std::to_string(i) + " = 0.0;\n";

  // Founders whose partial this part reads only through pristine type-2 steps (their states' prior x penetrance
  // terms): the partial is never stored; lane x keeps the state's penetrance (fp<i>) and the terms take it by
  // v_readlane at the term's (wave-uniform) state -- the same value the stored partial would have held
  // InitializePartials x SetFounderPriors, one person at a time (lanes over its states)
  for (int i = 0; i < n; i++) {
    if ((part == 1 && !leafp[i]) || (part == 2 && leafp[i])) continue;
    if (regf[i]) {
      if (!g_pair) code += lanes(NS, "x", "    fp" + S(i) + " = PEN[x * " + S(n) + " + " + S(i) + "];\n");
      continue;
    }
    if (regn[i] || iinit[i] || penp[i]) continue;   // (its type-2 step forms the initial partial itself / PEN)
    const bool fo = F.founder[i] && i < F.nf;
    const int sx = F.sex[i];
    const bool yf = NS == 3 && Y && sx == FEMALE;
    const int dfull = !fo ? 0 : (Y && sx == FEMALE) ? 0 : (((X || Y) && sx == MALE) || MT) ? 1 : 2;
    const int d = d0[i];
    std::string b = "    const int o = " + PO(i) + " + x * " + S(capP[i]) + ";\n";
    for (int a = 0; a <= d; a++) b += "    W[o + " + S(a) + "] = 0.0;\n";
    if (NS == 3) {
      b += "    const double pen = PEN[(x == 0 ? g11 : x == 1 ? g12 : g22) * " + S(n) + " + " + S(i) + "];\n";
      if (yf) b += "    W[o] = 1.0;\n";
      else if (!fo) b += "    W[o] = pen;\n";
      else if (top) b += "    if (x == 0) W[o] = pen;\n";
      else if (d == 2) b += "    W[o + 2 - x] = x == 1 ? 2 * pen : pen;\n";
      else b += "    if (x != 1) W[o + (x == 0 ? 1 : 0)] = pen;\n";
    } else {
      b += "    const double pen = PEN[x * " + S(n) + " + " + S(i) + "];\n";
      b += "    const int q = x == g11 ? 0 : x == g12 ? 1 : x == g22 ? 2 : 3;\n    (void)q;\n";
      if (!fo) b += "    W[o] = pen;\n";
      else if (top && dfull > 0) b += "    if (q == 0) W[o] = pen;\n";
      else if (d == 2) b += "    if (q != 3) W[o + 2 - q] = q == 1 ? 2 * pen : pen;\n";
      else if (d == 1) b += "    if (q == 0 || q == 2) W[o + (q == 0 ? 1 : 0)] = pen;\n";
      else b += "    if (q != 3) W[o] = pen;\n";
    }
    code += lanes(NS, "x", b);
  }
  code += "  wave_sync();\n";
  // T(e = i NS + j, k) of an offspring: 10-state rows of the lane's pair(s) in registers (trow, the de novo
  // transmission), the plain transmission (quirk :1391) and the bi-allelic class tables in LDS
  auto tt = [&](int csex, const std::string& e, const std::string& k, bool plain) -> std::string {
    if (NS == 10) return plain ? "t10[(" + e + ") * 10 + " + k + "]" : "t10dn[(" + e + ") * 10 + " + k + "]";
    const int t = chrom == PM_CHR_X ? (csex == MALE ? 2 : 1) : chrom == PM_CHR_Y ? (csex == MALE ? 3 : 5) : chrom == PM_CHR_MT ? 4 : 0;
    return "tb[" + S(t * 27) + " + (" + e + ") * 3 + " + k + "]";
  };
  // founder-sparse type-3 steps (10 states, one item per call): a parent of the roof is a founder
  std::vector<char> sp3(nst, 0);
  for (int k = 0; k < nst && sp3_on; k++) {
    const int f0 = (F.steps[k].x >> 8) & 255, f1 = (F.steps[k].x >> 16) & 255;
    if ((F.steps[k].x & 255) == 3 && ((F.founder[f0] && f0 < F.nf) || (F.founder[f1] && f1 < F.nf))) sp3[k] = 1;
  }
  size_t si = 0;
  int fin = -1;
  double nops = 0;
  std::vector<char> done(nst, 0);
  double lane_slots = 0, step_ops = 0, step_eff = 1;
  std::vector<double> eff2(nst, 0.0);   // packed type-2 runs: the run's lane occupancy (10 r of WL lanes)
  std::vector<double> frac1(nst, 1.0);   // type-1 steps: the fraction of the 100 pairs computed (founder-sparse rows)
  // persons whose partial the previous phase (a type-2 phase, lanes over states) left in registers: person -> (the
  // registers' name, the first lane); a following type-1 phase takes its coefficients by v_readlane instead of
  // wave-uniform LDS reads (the LDS pipe is what bounds this kernel)
  std::map<int, std::pair<std::string, int>> regp;
  for (const int2& St : F.steps) {
    const int kstep = (int)si;
    const StepDeg g = sd[si++];
    fin = (St.x >> 24) & 255;
    if ((part == 1 && !leaf[kstep]) || (part == 2 && leaf[kstep])) continue;
    const bool emitted = done[kstep];   // (in a fused run of type-1 steps: counted here, emitted with the run's first)
    {   // this step's FP64 operations (per item), and the lane slots they occupy (PM_JIT_LAYOUT: the static lane
        // occupancy -- a phase over E elements on a family's WL lanes runs ceil(E / WL) passes of WL lanes; a packed
        // run of r type-2 steps fills 10 r of the WL lanes; PM_JIT_STEPS: per step)
      const int type = St.x & 255, slot = (St.y >> 8) & 255, create = (St.y >> 16) & 1;
      const double ns = NS, before = nops;
      auto occ = [&](double E, double lanes) { return E / (std::ceil(E / lanes) * lanes); };
      double eff = 1.0;
      if (type == 1) {
        nops += frac1[kstep] * ns * ns * ((g.a + 1) * ns + (create ? 0 : (g.a + 1) * (g.b + 1)));
        eff = occ(frac1[kstep] * ns * ns, g_wl);
      } else if (type == 2) {
        const int ds = g.a + g.b;
        if (pristine[kstep]) nops += ns * ((double)pterms((St.x >> 8) & 255).size() * (slot == 255 ? 1 : (g.b + 1)) + (g.c + 1) * (ds + 1));
        else nops += ns * ((slot == 255 ? (ds + 1) * ns : ns * (g.a + 1) * (g.b + 1)) + (g.c + 1) * (ds + 1));
        eff = eff2[kstep] > 0 ? eff2[kstep] : occ(mc ? M * ns : ns, g_wl);   // (a packed run's first step: corrected below)
      } else {
        const int dw = g.a + g.b + g.c;
        double np_ = ns * ns;   // (founder-sparse: the pairs of the founders' supports only)
        if (sp3[kstep]) {
          const int f0 = (St.x >> 8) & 255, f1 = (St.x >> 16) & 255;
          np_ = (double)((F.founder[f0] && f0 < F.nf) ? (int)pterms(f0).size() : 10) * ((F.founder[f1] && f1 < F.nf) ? (int)pterms(f1).size() : 10);
        }
        const double o1 = np_ * (g.a + 1) * (g.b + 1) * (g.c + 1) * (slot == 255 ? 1 : 2), o2 = ns * (np_ * (dw + 1) + (g.e + 1) * (dw + 1));
        nops += o1 + o2;
        eff = (o1 + o2) / (o1 / occ(np_, g_wl) + o2 / occ(mc ? M * ns : ns, g_wl));
      }
      lane_slots += (nops - before) / eff;
      step_ops = nops - before;
      step_eff = eff;
      if (getenv("PM_JIT_STEPS"))
        fprintf(stderr, "  step %s part %d M %d k %d type %d ops %.0f eff %.3f\n", name.c_str(), part, M, kstep, type, step_ops, eff);
    }
    const int type = St.x & 255, from0 = (St.x >> 8) & 255, from1 = (St.x >> 16) & 255, to0 = (St.x >> 24) & 255;
    const int slot = (St.y >> 8) & 255, create = (St.y >> 16) & 1, fa2mo = (St.y >> 17) & 1;
    if (emitted) continue;
    if (type == 1) {   // lanes over the pairs e: S(e) = sum_k T(e, k) P_off[k] in registers, then M(e) *= S(e) in place
      const int off_ = from0, csex = F.sex[off_], pcap = capP[off_], mcap = capM[slot];
      std::string b = "      double s[" + S(g.a + 1) + "];\n";
      for (int a = 0; a <= g.a; a++) {
        b += "      s[" + S(a) + "] = 0.0;\n";
        b += "#pragma unroll\n      for (int k = 0; k < " + nsS + "; k++) s[" + S(a) + "] = fma(" +
             (NS == 10 ? std::string(g_tr_regs ? "(r == 0 ? tr0[k] : tr1[k])" : "t10dn[e * 10 + k]") : tt(csex, "e", "k", false)) + ", " +
             (penp[off_] ? "PEN[k * " + S(n) + " + " + S(off_) + "]" : "W[" + PO(off_) + " + k * " + S(pcap) + " + " + S(a) + "]") + ", s[" + S(a) + "]);\n";
      }
      const std::string me = MOf(slot) + " + e * " + S(mcap);
      if (create) {
        for (int a = 0; a <= g.a; a++) b += "      W[" + me + " + " + S(a) + "] = s[" + S(a) + "];\n";
      } else {
        b += "      double m[" + S(g.b + 1) + "];\n";
        for (int c = 0; c <= g.b; c++) b += "      m[" + S(c) + "] = W[" + me + " + " + S(c) + "];\n";
        for (int a = 0; a <= g.a + g.b; a++) {
          std::string acc;
          for (int c = std::max(0, a - g.a); c <= std::min(a, g.b); c++)
            acc = acc.empty() ? "m[" + S(c) + "] * s[" + S(a - c) + "]" : "fma(m[" + S(c) + "], s[" + S(a - c) + "], " + acc + ")";
          b += "      W[" + me + " + " + S(a) + "] = " + acc + ";\n";
        }
      }
      if (NS == 10 && !mc) {
        // a run of consecutive type-1 steps (this part's; they only read offspring partials and their own marriage
        // partial) is one phase: lanes over both pairs (lane, lane + 64 < 100), one pass over k for every step of
        // the run (each offspring coefficient read from LDS once for the two pairs: wave-uniform broadcasts), then per
        // marriage partial the steps' products chained in registers and one write -- the same operations in the
        // same order as step by step
        const std::vector<int> run = run_of(kstep);
        for (int k2 : run) done[k2] = 1;
        std::vector<int> slots;   // the marriage partials the run writes, in order of first use
        for (int k2 : run) {
          const int sl2 = (F.steps[k2].y >> 8) & 255;
          if (std::find(slots.begin(), slots.end(), sl2) == slots.end()) slots.push_back(sl2);
        }
        const Sparse spi = sparse_of(run);
        const std::vector<std::pair<int, int>>& sp_terms = spi.terms;
        const bool sp_father = spi.father;
        const bool sparse = !sp_terms.empty();
        if (sparse) {   // (the run's first step was counted at 100 pairs above)
          const double fr = 10.0 * sp_terms.size() / 100.0;
          nops -= (1.0 - fr) * 100.0 * ((g.a + 1) * 10.0 + (create ? 0 : (g.a + 1) * (g.b + 1)));
          for (int k2 : run) frac1[k2] = fr;
        }
        const int nsp = 10 * (int)sp_terms.size();   // (sparse: the rows, passes of g_wl lanes over them)
        const int npair = sparse ? (nsp + g_wl - 1) / g_wl : (100 + g_wl - 1) / g_wl;
        bool fact = g_fact && !sparse;
        for (int k2 : run)
          if (regp.count((F.steps[k2].x >> 8) & 255)) fact = false;
        std::vector<int> pfo(run.size(), 0);   // PM_ES_FACT: each step's P' rows at TB + pfo[q]
        if (fact) {   // P'(m, a) = sum_k M(m, k) P(k, a); M's row m is T10dn's row of the parent pair (x x, y y), m = {x, y}
          int at = 0;
          for (size_t q = 0; q < run.size(); q++) {
            const int offq = (F.steps[run[q]].x >> 8) & 255, ga = sd[run[q]].a, na = ga + 1;
            pfo[q] = at;
            const std::string P = penp[offq] ? "PEN[k * " + S(n) + " + " + S(offq) + "]"
                                             : "W[" + PO(offq) + " + k * " + S(capP[offq]) + " + a]";
            code += lanes(10 * na, "x", "    const int m = x / " + S(na) + ", a = x - m * " + S(na) + ";\n    (void)a;\n"
                          "    const double* Mr = t10dn + kMrow[m] * 10;\n    double s = 0.0;\n#pragma unroll\n"
                          "    for (int k = 0; k < 10; k++) s = fma(Mr[k], " + P + ", s);\n    W[" + TBs + " + " + S(at) + " + x] = s;\n");
            at += 10 * na;
          }
          code += "  wave_sync();\n";
        }
        std::string c1 = "  {\n";
        if (sparse) {   // pass pr: row p = lane + pr g_wl (state o of the spouse, term qi of the founder's support); rows past
                        // the support compute an in-range pair and store nothing
          const std::string gq[3] = {"g11", "g12", "g22"};
          for (int pr = 0; pr < npair; pr++) {
            const std::string P = S(pr), qi = "qi" + P;
            std::string sF = gq[sp_terms.back().first];
            for (int q = (int)sp_terms.size() - 2; q >= 0; q--) sF = qi + " == " + S(q) + " ? " + gq[sp_terms[q].first] + " : " + sF;
            c1 += "    const int p" + P + " = lane + " + S(pr * g_wl) + ", " + qi + " = p" + P + " / 10, o" + P + " = p" + P + " - " + qi +
                  " * 10, sF" + P + " = " + sF + ";\n    const int e" + P + " = " +
                  (sp_father ? "sF" + P + " * 10 + o" + P : "o" + P + " * 10 + sF" + P) + ";\n";
          }
        } else
          for (int pr = 1; pr < npair; pr++)
            c1 += "    const int e" + S(pr) + " = lane + " + S(pr * g_wl) + ", e" + S(pr) + "c = e" + S(pr) + " < 100 ? e" + S(pr) + " : lane;\n";
        for (size_t q = 0; q < run.size(); q++) {
          const int ga = sd[run[q]].a;
          for (int pr = 0; pr < npair; pr++) {
            c1 += "    double s" + S(pr) + "_" + S(q) + "[" + S(ga + 1) + "];\n";
            for (int a = 0; a <= ga; a++) c1 += "    s" + S(pr) + "_" + S(q) + "[" + S(a) + "] = 0.0;\n";
          }
        }
        if (fact) {   // per pair: 0.25 x the P' values at its four Mendelian children (packed bytes, kMend)
          for (int pr = 0; pr < npair; pr++)
            c1 += "    const unsigned cm" + S(pr) + " = kMend[" + (pr ? "e" + S(pr) + "c" : std::string("lane")) + "];\n";
          for (size_t q = 0; q < run.size(); q++) {
            const int ga = sd[run[q]].a, na = ga + 1;
            for (int pr = 0; pr < npair; pr++)
              for (int a = 0; a <= ga; a++) {
                auto pf = [&](int t) { return "W[" + TBs + " + " + S(pfo[q] + a) + " + " + S(na) + " * ((cm" + S(pr) + " >> " + S(8 * t) + ") & 255)]"; };
                c1 += "    s" + S(pr) + "_" + S(q) + "[" + S(a) + "] = 0.25 * (((" + pf(0) + " + " + pf(1) + ") + " + pf(2) + ") + " + pf(3) + ");\n";
              }
          }
        }
        // (k unrolled by 2 only: fully unrolled, the scheduler hoists every offspring coefficient's LDS read and
        // spills)
        if (!fact) {
        c1 += "#pragma unroll 2\n    for (int k = 0; k < 10; k++) {\n";
        if (sparse) {
          c1 += "      const double t0 = t10dn[e0 * 10 + k]";
          for (int pr = 1; pr < npair; pr++) c1 += ", t" + S(pr) + " = t10dn[e" + S(pr) + " * 10 + k]";
          c1 += ";\n";
        }
        else if (npair > 2) {   // (pair mode: the rows of this lane's four pairs)
          c1 += "      const double t0 = t10dn[lane * 10 + k]";
          for (int pr = 1; pr < npair; pr++) c1 += ", t" + S(pr) + " = t10dn[e" + S(pr) + "c * 10 + k]";
          c1 += ";\n";
        } else
          c1 += g_expt == 1 ? "      const double t0 = 0.001 * k, t1 = 0.002 * k;\n"   // (timing experiment only: wrong values)
                : g_tr_regs ? "      const double t0 = tr0[k], t1 = tr1[k];\n"
                            : "      const double t0 = t10dn[lane * 10 + k], t1 = t10dn[e1c * 10 + k];\n";
        for (size_t q = 0; q < run.size(); q++) {
          const int2 Sq = F.steps[run[q]];
          const int offq = (Sq.x >> 8) & 255, ga = sd[run[q]].a;
          for (int a = 0; a <= ga; a++) {
            if (regp.count(offq) && (g_regp != 2 || q % 2 == 1)) {   // from the lanes of the type-2 phase that computed it
              const std::string v = regp[offq].first + S(a), L = S(regp[offq].second) + " + k";
              c1 += "      {\n        const double p = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(" + v + "), " + L +
                    "), __builtin_amdgcn_readlane(__double2loint(" + v + "), " + L + "));\n";
            } else
            c1 += g_expt == 2 ? "      {\n        const double p = 0.5 + 0.01 * k + " + S(a) + ";\n"   // (timing experiment only)
                              : penp[offq] ? "      {\n        const double p = PEN[k * " + S(n) + " + " + S(offq) + "];\n"
                              : "      {\n        const double p = W[" + PO(offq) + " + k * " + S(capP[offq]) + " + " + S(a) + "];\n";
            for (int pr = 0; pr < npair; pr++)
              c1 += "        s" + S(pr) + "_" + S(q) + "[" + S(a) + "] = fma(t" + S(pr) + ", p, s" + S(pr) + "_" + S(q) + "[" + S(a) + "]);\n";
            c1 += "      }\n";
          }
        }
        c1 += "    }\n";
        }
        // per pair: each marriage partial chained through its steps in registers, one write
        for (int pr = 0; pr < npair; pr++) {
          const std::string sp = "s" + S(pr) + "_", e = spi.compact ? "p" + S(pr) : sparse ? "e" + S(pr) : pr ? "e" + S(pr) : "lane";
          c1 += sparse ? "    if (p" + S(pr) + " < " + S(nsp) + ") {\n" : pr ? "    if (e" + S(pr) + " < 100) {\n" : "    {\n";
          int cid = 0;
          for (int sl2 : slots) {
            const std::string mev = MOf(sl2) + " + " + e + " * " + S(capM[sl2]);
            std::string cur;   // the register array holding the slot's current coefficients
            int dcur = -1;
            for (size_t q = 0; q < run.size(); q++) {
              const int2 Sq = F.steps[run[q]];
              if (((Sq.y >> 8) & 255) != sl2) continue;
              const int ga = sd[run[q]].a, gb = sd[run[q]].b, cr = (Sq.y >> 16) & 1;
              const std::string sq = sp + S(q);
              if (cr) { cur = sq; dcur = ga; continue; }
              if (dcur < 0) {   // the slot's coefficients so far, from LDS
                cur = "m" + S(pr) + "_" + S(cid++);
                c1 += "      double " + cur + "[" + S(gb + 1) + "];\n";
                for (int c = 0; c <= gb; c++) c1 += "      " + cur + "[" + S(c) + "] = W[" + mev + " + " + S(c) + "];\n";
                dcur = gb;
              }
              const std::string nx = "m" + S(pr) + "_" + S(cid++);
              c1 += "      double " + nx + "[" + S(ga + gb + 1) + "];\n";
              for (int a = 0; a <= ga + gb; a++) {
                std::string acc;
                for (int c = std::max(0, a - ga); c <= std::min(a, gb); c++)
                  acc = acc.empty() ? cur + "[" + S(c) + "] * " + sq + "[" + S(a - c) + "]"
                                    : "fma(" + cur + "[" + S(c) + "], " + sq + "[" + S(a - c) + "], " + acc + ")";
                c1 += "      " + nx + "[" + S(a) + "] = " + acc + ";\n";
              }
              cur = nx;
              dcur = ga + gb;
            }
            for (int a = 0; a <= dcur; a++) c1 += "      W[" + mev + " + " + S(a) + "] = " + cur + "[" + S(a) + "];\n";
          }
          c1 += "    }\n";
        }
        c1 += "  }\n  wave_sync();\n";
        code += c1;
      } else
      code += "#pragma unroll\n  for (int r = 0; r < " + R + "; r++) {\n    const int e = lane + " + WL + " * r;\n    if (e < " + nsq + ") {\n" + items(b) +
              "    }\n  }\n  wave_sync();\n";
    } else if (type == 2) {   // lanes over i: S(i) = sum_j P_from[j] M(j, i) in registers, then P_to[i] *= S(i) in place
      const int sf = from0, stt = to0, fcap = capP[sf], tcap = capP[stt];
      const int ds = g.a + g.b;
      // independent type-2 steps of one shape that follow this one (this part's): one phase, 16 lanes per step, the
      // lane's step selecting its partials' offsets
      std::vector<int> run{kstep};
      if (NS == 10 && !mc && g_pack) {
        auto sig2 = [&](int k2) {
          const int2 Q = F.steps[k2];
          const int f2 = (Q.x >> 8) & 255, t2 = (Q.x >> 24) & 255, s2 = (Q.y >> 8) & 255;
          return std::vector<int>{pristine[k2], sd[k2].a, sd[k2].b, sd[k2].c, s2 == 255, capP[f2], capP[t2], s2 == 255 ? 0 : capM[s2],
                                  d0[f2], (int)crows.count(s2), (int)regf[f2], (int)regn[t2], (int)iinit[t2], F.founder[t2] && t2 < F.nf,
                                  (F.founder[t2] && t2 < F.nf) ? ((Y && F.sex[t2] == FEMALE) ? 0 : (((X || Y) && F.sex[t2] == MALE) || MT) ? 1 : 2)
                                                               : -1};
        };
        const std::vector<int> sg0 = sig2(kstep);
        for (int k2 = kstep + 1; k2 < nst && (int)run.size() < g_wl / 16; k2++) {
          if ((part == 1 && !leaf[k2]) || (part == 2 && leaf[k2])) continue;
          const int2 Q = F.steps[k2];
          if ((Q.x & 255) != 2 || sig2(k2) != sg0) break;
          const int f2 = (Q.x >> 8) & 255, t2 = (Q.x >> 24) & 255;
          bool indep = true;
          for (int k3 : run) {
            const int f3 = (F.steps[k3].x >> 8) & 255, t3 = (F.steps[k3].x >> 24) & 255;
            if (t2 == t3 || f2 == t3 || f3 == t2) indep = false;
          }
          if (!indep) break;
          run.push_back(k2);
        }
      }
      if (run.size() > 1) {
        for (int k2 : run) eff2[k2] = (double)NS * run.size() / g_wl;
        lane_slots += step_ops / eff2[kstep] - step_ops / step_eff;
      }
      std::string OF = PO(sf), OT = PO(stt), OM = slot == 255 ? "" : MOf(slot), pre;
      if (run.size() > 1) {
        auto sel = [&](const std::function<std::string(int)>& f) {
          std::string e = f(run.back());
          for (int q = (int)run.size() - 2; q >= 0; q--) e = "q_ == " + S(q) + " ? " + f(run[q]) + " : " + e;
          return e;
        };
        pre = "      const int of_ = " + sel([&](int k2) { return PO((F.steps[k2].x >> 8) & 255); }) +
              ";\n      const int ot_ = " + sel([&](int k2) { return PO((F.steps[k2].x >> 24) & 255); }) + ";\n";
        if (slot != 255) {   // (and the marriage partial's orientation: M(i, j) or M(j, i))
          pre += "      const int om_ = " + sel([&](int k2) { return MOf((F.steps[k2].y >> 8) & 255); }) + ";\n";
          pre += "      const int si_ = " + sel([&](int k2) { return std::string((F.steps[k2].y >> 17) & 1 ? "1" : nsS); }) + ", sj_ = " +
                 sel([&](int k2) { return std::string((F.steps[k2].y >> 17) & 1 ? nsS : "1"); }) + ";\n";
        }
        OF = "of_"; OT = "ot_"; OM = "om_";
        for (int k2 : run) done[k2] = 1;
      }

      std::string b = "    double s[" + S(ds + 1) + "];\n";
      for (int a = 0; a <= ds; a++) b += "    s[" + S(a) + "] = 0.0;\n";
      if (pristine[kstep]) {
        // the founder's partial is prior x penetrance: state g11 / g12 / g22 holds one monomial, at coefficient
        // 2 - q (degree 2: q = 0, 1, 2), 1 / - / 0 (degree 1: no geno12) or 0 (degree 0); the other states are zero.
        // The sum visits j in the dense loop's order and skips the zero terms (fma(0, g, s) == s), so it is
        // bit-identical to the dense sum (q in the dense loop's coefficient order u = 0, 1, 2 at one j, should two of
        // the genotypes coincide)
        // No loop over j: the terms' states are wave-uniform, so their order by j (stable: ties keep the coefficient
        // order) is one of at most 6, chosen once by a uniform switch; each case adds the terms in that order
        const std::string gq[3] = {"g11", "g12", "g22"};
        const std::vector<std::pair<int, int>> tm = pterms(sf);
        auto term = [&](int q, int u, int qpos) {
          std::string t = "      {\n        const int j = " + gq[q] + ";\n";
          if (regf[sf]) {   // the founder's penetrance at state j from lane j (x 2 for the heterozygote's coefficient)
            auto pj = [&](int fperson) {
              const std::string v = "fp" + S(fperson);
              return "__hiloint2double(__builtin_amdgcn_readlane(__double2hiint(" + v + "), j), __builtin_amdgcn_readlane(__double2loint(" +
                     v + "), j))";
            };
            std::string pe;
            if (g_pair) {   // the penetrance the init phase would have stored, from PEN (one read: the person index selected)
              std::string who = S((F.steps[run.back()].x >> 8) & 255);
              for (int r2 = (int)run.size() - 2; r2 >= 0; r2--) who = "q_ == " + S(r2) + " ? " + S((F.steps[run[r2]].x >> 8) & 255) + " : " + who;
              pe = "PEN[j * " + S(n) + " + (" + who + ")]";
            } else {
              pe = pj((F.steps[run.back()].x >> 8) & 255);
              for (int r2 = (int)run.size() - 2; r2 >= 0; r2--) pe = "q_ == " + S(r2) + " ? " + pj((F.steps[run[r2]].x >> 8) & 255) + " : " + pe;
            }
            t += "        const double pj_ = " + pe + ";\n";
            t += (!top && d0[sf] == 2 && q == 1) ? "        const double f = 2 * pj_;\n" : "        const double f = pj_;\n";
          } else t += "        const double f = W[" + OF + " + j * " + S(fcap) + " + " + S(u) + "];\n";
          if (slot == 255) t += "        s[" + S(u) + "] += f;\n";
          else {
            const int mcap = capM[slot];
            const std::string me = crows.count(slot) ? "(" + S(qpos * 10) + " + i)"   // (compact rows)
                                 : run.size() > 1 ? "(i * si_ + j * sj_)" : fa2mo ? "(j * " + nsS + " + i)" : "(i * " + nsS + " + j)";
            for (int v = 0; v <= g.b; v++)
              t += "        s[" + S(u + v) + "] = fma(f, W[" + OM + " + " + me + " * " + S(mcap) + " + " + S(v) + "], s[" + S(u + v) + "]);\n";
          }
          return t + "      }\n";
        };
        const int nt = (int)tm.size();
        if (nt == 1) b += term(tm[0].first, tm[0].second, 0);
        else {
          // bit c of the case: term a (of pair c) is not after term b, in the terms' order a < b
          std::vector<std::pair<int, int>> prs;
          for (int a = 0; a < nt; a++)
            for (int c = a + 1; c < nt; c++) prs.push_back({a, c});
          std::string key;
          for (size_t c = 0; c < prs.size(); c++)
            key += std::string(c ? " | " : "") + "((" + gq[tm[prs[c].first].first] + " <= " + gq[tm[prs[c].second].first] + ") << " + S(c) + ")";
          b += "    switch (" + key + ") {\n";
          for (int cs = 0; cs < (1 << prs.size()); cs++) {
            std::vector<int> ord(nt);
            for (int a = 0; a < nt; a++) ord[a] = a;
            auto before = [&](int x, int y) {   // x before y in this case
              for (size_t c = 0; c < prs.size(); c++) {
                if (prs[c].first == x && prs[c].second == y) return ((cs >> c) & 1) != 0;
                if (prs[c].first == y && prs[c].second == x) return ((cs >> c) & 1) == 0;
              }
              return x < y;
            };
            std::stable_sort(ord.begin(), ord.end(), before);
            b += "      case " + S(cs) + ":\n";
            for (int a : ord) b += term(tm[a].first, tm[a].second, a);
            b += "      break;\n";
          }
          b += "    }\n";
        }
      } else if (slot == 255) {
        for (int a = 0; a <= ds; a++)
          b += "#pragma unroll\n    for (int j = 0; j < " + nsS + "; j++) s[" + S(a) + "] += W[" + OF + " + j * " + S(fcap) + " + " +
               S(a) + "];\n";
      } else {
        const int mcap = capM[slot];
        const std::string me = run.size() > 1 ? "(i * si_ + j * sj_)" : fa2mo ? "(j * " + nsS + " + i)" : "(i * " + nsS + " + j)";
        b += std::string(run.size() > 1 ? "#pragma unroll 2" : "#pragma unroll") + "\n    for (int j = 0; j < " + nsS + "; j++) {\n";
        for (int u = 0; u <= g.a; u++) b += "      const double f" + S(u) + " = W[" + OF + " + j * " + S(fcap) + " + " + S(u) + "];\n";
        for (int v = 0; v <= g.b; v++) b += "      const double g" + S(v) + " = W[" + OM + " + " + me + " * " + S(mcap) + " + " + S(v) + "];\n";
        for (int u = 0; u <= g.a; u++)
          for (int v = 0; v <= g.b; v++) b += "      s[" + S(u + v) + "] = fma(f" + S(u) + ", g" + S(v) + ", s[" + S(u + v) + "]);\n";
        b += "    }\n";
      }
      const bool keep = NS == 10 && !mc && g_regp;   // (the outputs stay in registers for a following type-1 phase)
      const bool rn = keep && regn[stt];   // (the to-person is register-only: its partial was its penetrance)
      b += "    double t[" + S(g.c + 1) + "];\n";
      if ((keep || (NS == 10 && !mc && g_pair)) && iinit[stt]) {   // the initial partial at state i (InitializePartials x SetFounderPriors)
        std::string tp = S((F.steps[run.back()].x >> 24) & 255);   // (packed: the lane group's to-person)
        for (int r2 = (int)run.size() - 2; r2 >= 0; r2--) tp = "q_ == " + S(r2) + " ? " + S((F.steps[run[r2]].x >> 24) & 255) + " : " + tp;
        const bool fo2 = F.founder[stt] && stt < F.nf;
        const int sx2 = F.sex[stt];
        const int dfull2 = !fo2 ? 0 : (Y && sx2 == FEMALE) ? 0 : (((X || Y) && sx2 == MALE) || MT) ? 1 : 2;
        const int d2 = d0[stt];
        b += "    const double pen_ = PEN[i * " + S(n) + " + (" + tp + ")];\n";
        b += "    const int qi_ = i == g11 ? 0 : i == g12 ? 1 : i == g22 ? 2 : 3;\n    (void)qi_;\n";
        for (int c = 0; c <= g.c; c++) {
          std::string v = "0.0";
          if (!fo2) v = c == 0 ? "pen_" : "0.0";
          else if (top && dfull2 > 0) v = c == 0 ? "(qi_ == 0 ? pen_ : 0.0)" : "0.0";
          else if (d2 == 2) v = c == 0 ? "(qi_ == 2 ? pen_ : 0.0)" : c == 1 ? "(qi_ == 1 ? 2 * pen_ : 0.0)" : c == 2 ? "(qi_ == 0 ? pen_ : 0.0)" : "0.0";
          else if (d2 == 1) v = c == 0 ? "(qi_ == 2 ? pen_ : 0.0)" : c == 1 ? "(qi_ == 0 ? pen_ : 0.0)" : "0.0";
          else v = c == 0 ? "(qi_ != 3 ? pen_ : 0.0)" : "0.0";
          b += "    t[" + S(c) + "] = " + v + ";\n";
        }
      } else
        for (int c = 0; c <= g.c; c++) b += "    t[" + S(c) + "] = W[" + OT + " + i * " + S(tcap) + " + " + S(c) + "];\n";
      const std::string xr = "xr" + S(kstep) + "_";
      if (keep)
        for (int a = 0; a <= g.c + ds; a++) code += "  double " + xr + S(a) + " = 0.0;\n";
      for (int a = 0; a <= g.c + ds; a++) {
        std::string acc;
        for (int c = std::max(0, a - ds); c <= std::min(a, g.c); c++)
          acc = acc.empty() ? "t[" + S(c) + "] * s[" + S(a - c) + "]" : "fma(t[" + S(c) + "], s[" + S(a - c) + "], " + acc + ")";
        if (rn) b += "    " + xr + S(a) + " = " + acc + ";\n";
        else if (keep) b += "    " + xr + S(a) + " = " + acc + ";\n    W[" + OT + " + i * " + S(tcap) + " + " + S(a) + "] = " + xr + S(a) + ";\n";
        else b += "    W[" + OT + " + i * " + S(tcap) + " + " + S(a) + "] = " + acc + ";\n";
      }
      for (size_t q = 0; q < run.size(); q++) regp.erase((F.steps[run[q]].x >> 24) & 255);
      if (keep)
        for (size_t q = 0; q < run.size(); q++) regp[(F.steps[run[q]].x >> 24) & 255] = {xr, run.size() > 1 ? 16 * (int)q : 0};
      if (run.size() > 1)
        code += "  {\n    const int q_ = lane >> 4, i = lane & 15;\n    if (q_ < " + S(run.size()) + " && i < " + nsS + ") {\n" + pre + b +
                "    }\n  }\n  wave_sync();\n";
      else code += lanes(NS, "i", b) + "  wave_sync();\n";
    } else if (sp3[kstep]) {
      // founder-sparse type-3 step (10 states): a founder's partial is prior x penetrance times whatever multiplied into
      // it -- zero outside the 1-3 states of its prior (the site's g11, g12, g22; pterms) -- so W(e) = P_fa[i] M(e) P_mo[j]
      // is zero off those pairs, and so is every term T(e, k) W(e) they would add (+0: the sums keep their bits).  Only
      // the nI x nJ pairs (i, j) in ascending e are formed (lanes over them) and summed (in the same ascending e order),
      // instead of all 100.  The states of a founder's support are sorted at run time (wave-uniform).
      regp.erase(to0);
      const int fa = from0, mo_ = from1, off_ = to0, csex = F.sex[off_];
      const int dw = g.a + g.b + g.c, ww = dw + 1;
      auto support = [&](int f, const std::string& pre) -> std::pair<int, std::string> {
        if (!(F.founder[f] && f < F.nf)) return {10, ""};
        const auto t = pterms(f);
        std::string c;
        for (size_t q = 0; q < t.size(); q++)
          c += "  int " + pre + S(q) + " = " + (t[q].first == 0 ? "g11" : t[q].first == 1 ? "g12" : "g22") + ";\n";
        auto sw = [&](int a, int b2) {
          return "  if (" + pre + S(a) + " > " + pre + S(b2) + ") { const int x_ = " + pre + S(a) + "; " + pre + S(a) + " = " + pre + S(b2) +
                 "; " + pre + S(b2) + " = x_; }\n";
        };
        if (t.size() >= 2) c += sw(0, 1);
        if (t.size() == 3) c += sw(1, 2) + sw(0, 1);
        return {(int)t.size(), c};
      };
      const std::string pI = "sI" + S(kstep) + "_", pJ = "sJ" + S(kstep) + "_";
      const auto sI = support(fa, pI), sJ = support(mo_, pJ);
      const int nI = sI.first, nJ = sJ.first, NP = nI * nJ;
      auto pick = [&](const std::string& pre, int nn, const std::string& idx) {   // the idx-th state of a support
        if (nn == 10) return idx;
        std::string r = pre + S(nn - 1);
        for (int q = nn - 2; q >= 0; q--) r = "(" + idx + " == " + S(q) + " ? " + pre + S(q) + " : " + r + ")";
        return r;
      };
      code += sI.second + sJ.second;
      std::string b = "      const int ia = p / " + S(nJ) + ", jb = p - ia * " + S(nJ) + ";\n      const int i = " + pick(pI, nI, "ia") +
                      ", j = " + pick(pJ, nJ, "jb") + ", e = i * " + nsS + " + j;\n      double w[" + S(ww) + "];\n";
      for (int a = 0; a <= dw; a++) b += "      w[" + S(a) + "] = 0.0;\n";
      for (int u = 0; u <= g.a; u++)
        for (int v = 0; v <= g.b; v++)
          for (int c = 0; c <= g.c; c++) {
            const std::string m = slot == 255 ? "" : " * W[" + MOf(slot) + " + e * " + S(capM[slot]) + " + " + S(v) + "]";
            b += "      w[" + S(u + v + c) + "] = fma(W[" + PO(fa) + " + i * " + S(capP[fa]) + " + " + S(u) + "]" + m + ", W[" +
                 PO(mo_) + " + j * " + S(capP[mo_]) + " + " + S(c) + "], w[" + S(u + v + c) + "]);\n";
          }
      for (int a = 0; a <= dw; a++) b += "      W[" + TBs + " + p * " + S(ww) + " + " + S(a) + "] = w[" + S(a) + "];\n";
      code += "#pragma unroll\n  for (int r = 0; r < " + S((NP + g_wl - 1) / g_wl) + "; r++) {\n    const int p = lane + " + WL + " * r;\n    if (p < " +
              S(NP) + ") {\n" + b + "    }\n  }\n  wave_sync();\n";
      std::string b2 = "    double s[" + S(ww) + "];\n";
      for (int a = 0; a <= dw; a++) b2 += "    s[" + S(a) + "] = 0.0;\n";
      b2 += "    for (int p = 0; p < " + S(NP) + "; p++) {\n      const int ia = p / " + S(nJ) + ", jb = p - ia * " + S(nJ) + ";\n      const int e = " +
            pick(pI, nI, "ia") + " * " + nsS + " + " + pick(pJ, nJ, "jb") + ";\n      const double t = " + tt(csex, "e", "k", slot != 255) + ";\n";
      for (int a = 0; a <= dw; a++) b2 += "      s[" + S(a) + "] = fma(t, W[" + TBs + " + p * " + S(ww) + " + " + S(a) + "], s[" + S(a) + "]);\n";
      b2 += "    }\n    double t[" + S(g.e + 1) + "];\n";
      for (int c = 0; c <= g.e; c++) b2 += "    t[" + S(c) + "] = W[" + PO(off_) + " + k * " + S(capP[off_]) + " + " + S(c) + "];\n";
      for (int a = 0; a <= g.e + dw; a++) {
        std::string acc;
        for (int c = std::max(0, a - dw); c <= std::min(a, g.e); c++)
          acc = acc.empty() ? "t[" + S(c) + "] * s[" + S(a - c) + "]" : "fma(t[" + S(c) + "], s[" + S(a - c) + "], " + acc + ")";
        b2 += "    W[" + PO(off_) + " + k * " + S(capP[off_]) + " + " + S(a) + "] = " + acc + ";\n";
      }
      code += lanes(NS, "k", b2) + "  wave_sync();\n";
    } else {   // W(e) = P_fa[i] M(e) P_mo[j] -> LDS; lanes over k: S(k) = sum_e T(e, k) W(e), P_off[k] *= S(k) in place
      regp.erase(to0);
      const int fa = from0, mo_ = from1, off_ = to0, csex = F.sex[off_];
      const int dw = g.a + g.b + g.c, ww = dw + 1;
      std::string b = "      const int i = e / " + nsS + ", j = e - i * " + nsS + ";\n      double w[" + S(ww) + "];\n";
      for (int a = 0; a <= dw; a++) b += "      w[" + S(a) + "] = 0.0;\n";
      for (int u = 0; u <= g.a; u++)
        for (int v = 0; v <= g.b; v++)
          for (int c = 0; c <= g.c; c++) {
            const std::string m = slot == 255 ? "" : " * W[" + MOf(slot) + " + e * " + S(capM[slot]) + " + " + S(v) + "]";
            b += "      w[" + S(u + v + c) + "] = fma(W[" + PO(fa) + " + i * " + S(capP[fa]) + " + " + S(u) + "]" + m + ", W[" +
                 PO(mo_) + " + j * " + S(capP[mo_]) + " + " + S(c) + "], w[" + S(u + v + c) + "]);\n";
          }
      for (int a = 0; a <= dw; a++) b += "      W[" + TBs + " + e * " + S(ww) + " + " + S(a) + "] = w[" + S(a) + "];\n";
      code += "#pragma unroll\n  for (int r = 0; r < " + R + "; r++) {\n    const int e = lane + " + WL + " * r;\n    if (e < " + nsq + ") {\n" + items(b) +
              "    }\n  }\n  wave_sync();\n";
      std::string b2 = "    double s[" + S(ww) + "];\n";
      for (int a = 0; a <= dw; a++) b2 += "    s[" + S(a) + "] = 0.0;\n";
      if (NS == 10 && slot != 255 && !g_no_t3z) {
        // the plain transmission (:1391) is the Mendelian table: 16-31 of a child state's 100 parent pairs are non-zero
        // (1, 1/2 or 1/4).  Each lane k runs over its non-zero pairs only, in ascending e (the LDS list t3z, e << 2 |
        // value code): the pairs skipped would add +0 (T = 0, W finite and >= 0), so every sum keeps its bits -- and no
        // transmission load is waited for in the 100-step loop
        g_t3z = true;
        b2 += "    const int nz_ = t3n[k];\n    for (int q_ = 0; q_ < nz_; q_++) {\n      const int pk_ = t3z[k * 32 + q_], e = pk_ >> 2;\n"
              "      const double t = (pk_ & 3) == 0 ? 1.0 : (pk_ & 3) == 1 ? 0.5 : 0.25;\n";
      } else b2 += "    for (int e = 0; e < " + nsq + "; e++) {\n      const double t = " + tt(csex, "e", "k", slot != 255) + ";\n";
      for (int a = 0; a <= dw; a++) b2 += "      s[" + S(a) + "] = fma(t, W[" + TBs + " + e * " + S(ww) + " + " + S(a) + "], s[" + S(a) + "]);\n";
      b2 += "    }\n    double t[" + S(g.e + 1) + "];\n";
      for (int c = 0; c <= g.e; c++) b2 += "    t[" + S(c) + "] = W[" + PO(off_) + " + k * " + S(capP[off_]) + " + " + S(c) + "];\n";
      for (int a = 0; a <= g.e + dw; a++) {
        std::string acc;
        for (int c = std::max(0, a - dw); c <= std::min(a, g.e); c++)
          acc = acc.empty() ? "t[" + S(c) + "] * s[" + S(a - c) + "]" : "fma(t[" + S(c) + "], s[" + S(a - c) + "], " + acc + ")";
        b2 += "    W[" + PO(off_) + " + k * " + S(capP[off_]) + " + " + S(a) + "] = " + acc + ";\n";
      }
      code += lanes(NS, "k", b2) + "  wave_sync();\n";
    }
  }
  const int D = dP[fin];
  *ops = M * (nops + (part == 1 ? 0.0 : (double)(D + 1) * NS));
  if (getenv("PM_JIT_LAYOUT"))
    fprintf(stderr, "occupancy %s part %d WL %d: %.0f FP64 ops / %.0f lane slots = %.3f\n", name.c_str(), part, g_wl, nops, lane_slots,
            lane_slots > 0 ? nops / lane_slots : 0.0);
  if (part != 1) {
    code += lanes(D + 1, "a", "    double s = 0.0;\n#pragma unroll\n    for (int i = 0; i < " + nsS + "; i++) s += W[" + PO(fin) + " + i * " +
                                  S(capP[fin]) + " + a];\n    out[" + std::string(mc ? "c * ostr + " : "") + "(size_t)a * os] = s;\n");
    code += "  if (lane < " + S(M) + ") out[" + std::string(mc ? "lane * ostr + " : "") + "(size_t)(dcap - 1) * os] = " + S(D) + ".0;\n  wave_sync();\n";
  }
  return "__device__ __forceinline__ void " + name +
         "(const uint8_t* __restrict__ pl, size_t np, const uint8_t* __restrict__ P11, const uint8_t* __restrict__ P12, "
         "const uint8_t* __restrict__ P22, int p0, int gg11, int gg12, int gg22, const double* lk, const double* __restrict__ t10, "
         "const double* __restrict__ t10dn, const double* tb, const double* tr0, const double* tr1, double* W, int lane, "
         "double* __restrict__ out, int os, int dcap, size_t ostr, const double* PEN) {\n" + code + "}\n";
}

// The site's penetrances of a family, lk[pl[g][p0 + i]] for the 10 genotypes g, into the wave's LDS table PEN[g * n + i]
// (one coalesced pass per (site, family) instead of a dependent global load per person and variant)
std::string gen_pen_fill(int n, const std::string& name) {
  const std::string N = std::to_string(n);
  return "__device__ __forceinline__ void " + name + "(const uint8_t* __restrict__ pl, size_t np, int p0, const double* lk, double* PEN, "
         "int lane) {\n  for (int e = lane; e < " + std::to_string(10 * n) + "; e += " + std::to_string(g_wl) + ") {\n    const int g = e / " + N + ", i = e - g * " + N +
         ";\n    PEN[e] = lk[pl[(size_t)g * np + p0 + i]];\n  }\n  wave_sync();\n}\n";
}

// fns: 3 variants per shape (bi-allelic, 10-state, top); parts: per shape the 10-state leaf prefix, the 10-state rest,
// the top variant's rest and (pps == 4) the 10-state rest of three items at once
std::string gen_wave_kernel(const std::vector<std::string>& fns, const std::vector<std::string>& parts, const std::vector<std::string>& pens,
                            const std::vector<int>& shape_ns, int pps, int ws, int pensz, int wpb, bool parts_only) {
  // prefetch registers per lane (0: families too large; up to 4, 8 at 16 lanes per family)
  const int npf = pensz <= (g_wl >= 32 ? 4 : 8) * g_wl ? (pensz + g_wl - 1) / g_wl : 0;
  // wave_sync: the phases' LDS hand-over inside one wave.  A wave's LDS instructions execute in issue order, so a
  // read after a write sees it without waiting for the write; only the compiler must not move accesses across
  // (g_fence, the default: wavefront-scope release / acquire fences, which wait for the outstanding LDS accesses --
  // measured 2% faster than the bare barrier, r05nf)
  std::string s = g_fence ? R"(
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
)" : R"(
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}
)";
  if (g_fact) {   // PM_ES_FACT: the four Mendelian children of parent pair e = i * 10 + j (bytes), and the pair (x x, y y)
                  // whose only child is genotype m (its T10dn row is M's row m)
    auto gi = [](int b1, int b2) { return b1 < b2 ? (b1 - 1) * (10 - b1) / 2 + (b2 - b1) : (b2 - 1) * (10 - b2) / 2 + (b1 - b2); };
    int al[10][2], at = 0;
    for (int x = 1; x <= 4; x++)
      for (int y = x; y <= 4; y++) { al[gi(x, y)][0] = x; al[gi(x, y)][1] = y; at++; }
    s += "__device__ const unsigned kMend[100] = {";
    for (int i = 0; i < 10; i++)
      for (int j = 0; j < 10; j++) {
        const int c[4] = {gi(al[i][0], al[j][0]), gi(al[i][0], al[j][1]), gi(al[i][1], al[j][0]), gi(al[i][1], al[j][1])};
        s += std::to_string((unsigned)c[0] | (unsigned)c[1] << 8 | (unsigned)c[2] << 16 | (unsigned)c[3] << 24) + "u,";
      }
    s += "};\n__device__ const int kMrow[10] = {";
    for (int m = 0; m < 10; m++) s += std::to_string(gi(al[m][0], al[m][0]) * 10 + gi(al[m][1], al[m][1])) + ",";
    s += "};\n";
    (void)at;
  }
  s += "__device__ __forceinline__ int shape_n(int sig) {\n  switch (sig) {\n";
  for (size_t i = 0; i < shape_ns.size(); i++) s += "    case " + std::to_string(i) + ": return " + std::to_string(shape_ns[i]) + ";\n";
  s += "  }\n  return 0;\n}\n";
  std::string k = R"(
extern "C" __global__ void __launch_bounds__(64 * WPB) WPEU es_hoist_wave(Args A) {   // blockDim = 64 WPB
  __shared__ double lk[256], tb[6 * 27];
  __shared__ double ws[WPB][FPW * (WSIZE + PENSZ)];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) lk[i] = A.lktab[i];
  for (int i = threadIdx.x; i < 6 * 27; i += blockDim.x) tb[i] = i < 5 * 27 ? A.tba[i] : 1.0;
T3FILL  __syncthreads();
  // FPW families per wave: lane group h (LPF lanes) hoists the unit's family h in its own slice; `lane` is the lane within
  // the group (`half`: the group, from the pair mode of two)
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & (LPF - 1);
  const int half = FPW > 1 ? (threadIdx.x & 63) / LPF : 0;
  double* W = ws[wave] + half * (WSIZE + PENSZ);
  double* PEN = W + WSIZE;   // the current (site, family)'s penetrances
  // the de novo transmission rows of this lane's marriage-partial pairs (lane, lane + 64), for every 10-state step
  double tr0[10], tr1[10];
#pragma unroll
  for (int k = 0; k < 10; k++) {
    tr0[k] = A.T10dn[lane * 10 + k];
    tr1[k] = lane + 64 < 100 ? A.T10dn[(lane + 64) * 10 + k] : 0.0;
  }
  const double* t10 = A.T10;
  const double* t10dn = A.T10dn;
  // PM_ES_PROF=1: clock cycles per wave in the pen fill, top rest, leaf prefix, 10-state rest and whole variants
  unsigned long long pc[5] = {0, 0, 0, 0, 0};
#define PCLK(c) if (PROF) { const unsigned long long t1_ = __builtin_readcyclecounter(); pc[c] += t1_ - tq; tq = t1_; }
  const int nItems = min(A.counts[A.list], A.it1);
  if (nItems <= A.it0) return;
  // a task: G consecutive items of the list -- with A.group, the de novo items of one site (list 0: cfgs 0-3, list 1:
  // cfgs 4-6), whose 10-state leaf steps are taken once per (site, family) -- on one family
  const int G = A.group > 1 ? A.group : 1;
  const int nfu = kNUnits;   // family units per task: slots, or units of FPW slots
  const long long units = ((long long)(nItems - A.it0) + G - 1) / G * nfu;
  // the next task's penetrance bytes are loaded while this one is computed (NPF per lane: 10 n <= 64 NPF)
  unsigned pb[NPF > 0 ? NPF : 1];
  long long pf_u = -1;   // the task whose bytes pb holds
  // A task's words are loaded ahead, so no load is waited for when it starts: its G item words two tasks ahead, the
  // sites' reference bytes one task ahead (both uniform); the family unit's slot words are constants of the generated
  // source (kUP0 / kUE / kUSig, per unit and half), so the penetrance-byte prefetch below has no dependent load chain
  int c_item[4], c_ref[4], n1_item[4], n1_ref[4], n2_item[4];
  auto load_items = [&](long long uu, int* it4) {
#pragma unroll
    for (int t = 0; t < 4; t++) it4[t] = -1;
    if (uu >= units) return;
    const int itn = A.it0 + (int)(uu / nfu) * G;
#pragma unroll
    for (int t = 0; t < 4; t++)
      if (t < G && itn + t < nItems) it4[t] = A.items[itn + t];
  };
  auto load_refs = [&](const int* it4, int* r4) {
#pragma unroll
    for (int t = 0; t < 4; t++) {
      const int w = __builtin_amdgcn_readfirstlane(it4[t]);
      r4[t] = w >= 0 ? (int)A.ref[w >> 3] : 0;
    }
  };
  auto prefetch = [&](long long uu, int item_w) {   // (item_w: the task's first item word, landed)
    pf_u = -1;
    if (NPF == 0 || uu >= units) return;
    const int uqn = (int)(uu / nfu), kn0 = (int)(uu - (long long)uqn * nfu);
    const int w = __builtin_amdgcn_readfirstlane(item_w);
    if (w < 0) return;
    const int sn = w >> 3;
    const int p0n = kUP0[FPW * kn0 + half];
    const int nn = shape_n(kUSig[kn0]);
    if (10 * nn > LPF * NPF) return;
    const uint8_t* pln = A.pl + (size_t)sn * A.np * 10 + p0n;
#pragma unroll
    for (int r = 0; r < (NPF > 0 ? NPF : 1); r++) {
      const int e = lane + LPF * r, g = e / nn;
      pb[r] = e < 10 * nn ? pln[(size_t)g * A.np + (e - g * nn)] : 0;
    }
    pf_u = uu;
  };
  // XCD-aware unit order: blocks are dealt round-robin over the 8 XCDs, so the units of one round are split into 8
  // contiguous ranges, one per XCD -- a task's family units (one site's penetrance rows) stay in one XCD's L2
  const long long stride = (long long)gridDim.x * WPB;
  const long long u_first = (XCD && gridDim.x % 8 == 0)
      ? (long long)(blockIdx.x % 8) * (gridDim.x / 8) * WPB + (long long)(blockIdx.x / 8) * WPB + wave
      : (long long)blockIdx.x * WPB + wave;
  load_items(u_first, c_item);
  load_refs(c_item, c_ref);
  load_items(u_first + stride, n1_item);
  load_refs(n1_item, n1_ref);
  load_items(u_first + 2 * stride, n2_item);
  prefetch(u_first, c_item[0]);
  for (long long u = u_first; u < units; u += stride) {
    const int uq = (int)(u / nfu), k0 = (int)(u - (long long)uq * nfu);
    if (u != u_first) {   // rotate: this task's words (landed a task ago), the next task's refs, the task after's items
#pragma unroll
      for (int t = 0; t < 4; t++) { c_item[t] = n1_item[t]; c_ref[t] = n1_ref[t]; n1_item[t] = n2_item[t]; }
      load_refs(n1_item, n1_ref);
      load_items(u + 2 * stride, n2_item);
    }
    // (PAIR: the unit's half -- per lane; both halves share the pair's shape)
    int leaf_site = -1, pen_site = -1;
    unsigned long long tq = PROF ? __builtin_readcyclecounter() : 0;
    for (int t = 0; t < G; t++) {
    const int it = A.it0 + uq * G + t;
    const int item = __builtin_amdgcn_readfirstlane(c_item[t]);
    if (item < 0) break;
    const int site = item >> 3, cfg = item & 7, r = __builtin_amdgcn_readfirstlane(c_ref[t]);
    int a1, a2;
    if (A.vcf) { a1 = r & 15; a2 = r >> 4; }
    else if (cfg == 7) { a1 = A.res[(size_t)site * A.res_words + A.res_a1]; a2 = A.res[(size_t)site * A.res_words + A.res_a2]; }
    else cfg_alleles(cfg, r, &a1, &a2);
    const int g11 = gi(a1, a1), g12 = gi(a1, a2), g22 = gi(a2, a2);
    const uint8_t* pl = A.pl + (size_t)site * A.np * 10;
    const uint8_t* P11 = pl + (size_t)g11 * A.np;
    const uint8_t* P12 = pl + (size_t)g12 * A.np;
    const uint8_t* P22 = pl + (size_t)g22 * A.np;
    const int e = kUE[FPW * k0 + half], q = e / A.T;
    const int sig = kUSig[k0], p0 = kUP0[FPW * k0 + half];
    double* out = A.coef + ((size_t)(it - A.it0) * A.max_ext + q) * A.dcap * A.T + (e - q * A.T);
    const int dn = A.denovo && cfg != 7, top = dn && cfg == 0 && !A.vcf;   // variant: 0 bi-allelic, 1 10-state, 2 top
    if (site != pen_site) {
      if (pf_u == u && t == 0) {   // the prefetched bytes (this task's first item)
        const int nn = shape_n(sig);
#pragma unroll
        for (int r = 0; r < (NPF > 0 ? NPF : 1); r++)
          if (lane + LPF * r < 10 * nn) PEN[lane + LPF * r] = lk[pb[r]];
        wave_sync();
        prefetch(u + stride, n1_item[0]);
      } else {
        switch (sig) {
PENS        }
      }
      pen_site = site;
      PCLK(0);
    }
    if ((G > 1 || PARTS_ONLY) && dn) {
      if (site != leaf_site) {
        leaf_site = site;
        switch (sig) {
PARTS1        }
        PCLK(2);
      }
      if (top) {
        switch (sig) {
PARTS3        }
        PCLK(1);
        continue;
      }
      if (MULTI && t + 3 <= G && it + 2 < nItems) {   // the site's three 10-state items at once (lanes over item x state)
        const int ib = __builtin_amdgcn_readfirstlane(A.items[it + 1]), ic = __builtin_amdgcn_readfirstlane(A.items[it + 2]);
        if ((ib >> 3) == site && (ic >> 3) == site && (ib & 7) != 0 && (ib & 7) != 7 && (ic & 7) != 0 && (ic & 7) != 7) {
          int b1, b2, c1, c2;
          cfg_alleles(ib & 7, r, &b1, &b2);
          cfg_alleles(ic & 7, r, &c1, &c2);
          const int G11 = g11 | gi(b1, b1) << 8 | gi(c1, c1) << 16, G12 = g12 | gi(b1, b2) << 8 | gi(c1, c2) << 16,
                    G22 = g22 | gi(b2, b2) << 8 | gi(c2, c2) << 16;
          const size_t ostr = (size_t)A.max_ext * A.dcap * A.T;
          switch (sig) {
PARTS4          }
          PCLK(3);
          t += 2;
          continue;
        }
      }
      switch (sig) {
PARTS2      }
      PCLK(3);
      continue;
    }
    leaf_site = -1;   // (the other variants' layouts overlay the leaf prefix's partials)
    switch (sig * 3 + (top ? 2 : dn ? 1 : 0)) {
)";
  k.replace(k.find("T3FILL"), 6, g_t3z ? "  for (int i = threadIdx.x; i < 330; i += blockDim.x) {\n    if (i < 320) t3z[i] = kT3z[i];\n"
                                         "    else t3n[i - 320] = kT3n[i - 320];\n  }\n" : "");
  for (size_t at; (at = k.find("WSIZE")) != std::string::npos;) k.replace(at, 5, std::to_string(ws));
  for (size_t at; (at = k.find("PENSZ")) != std::string::npos;) k.replace(at, 5, std::to_string(pensz));
  for (size_t at; (at = k.find("NPF")) != std::string::npos;) k.replace(at, 3, std::to_string(npf));
  for (size_t at; (at = k.find("LPF")) != std::string::npos;) k.replace(at, 3, std::to_string(g_wl));
  for (size_t at; (at = k.find("PAIR")) != std::string::npos;) k.replace(at, 4, g_pair ? "true" : "false");
  for (size_t at; (at = k.find("FPW")) != std::string::npos;) k.replace(at, 3, std::to_string(g_fpw));
  k.replace(k.find("XCD &&"), 3, g_xcd ? "true" : "false");
  {
    std::string cases;
    for (size_t i = 0; i < pens.size(); i++) cases += "        case " + std::to_string(i) + ": " + pens[i] + "(pl, A.np, p0, lk, PEN, lane); break;\n";
    k.replace(k.find("PENS"), 4, cases);
  }
  for (size_t at; (at = k.find("WPB")) != std::string::npos;) k.replace(at, 3, std::to_string(wpb));
  k.replace(k.find("MULTI"), 5, pps == 4 ? "true" : "false");
  k.replace(k.find("PARTS_ONLY"), 10, parts_only ? "true" : "false");
  k.replace(k.find("WPEU"), 4, "__attribute__((amdgpu_waves_per_eu(4)))");   // (<= 128 VGPRs: 4 waves per SIMD)
  const std::string call = "(pl, A.np, P11, P12, P22, p0, g11, g12, g22, lk, t10, t10dn, tb, tr0, tr1, W, lane, out, A.T, A.dcap, 0, PEN); break;\n";
  const std::string call3 = "(pl, A.np, P11, P12, P22, p0, G11, G12, G22, lk, t10, t10dn, tb, tr0, tr1, W, lane, out, A.T, A.dcap, ostr, PEN); break;\n";
  for (int p = 1; p <= 4; p++) {
    std::string cases;
    for (size_t i = 0; p <= pps && pps * i + p - 1 < parts.size(); i++)
      cases += "        case " + std::to_string(i) + ": " + parts[pps * i + p - 1] + (p == 4 ? call3 : call);
    const std::string key = "PARTS" + std::to_string(p);
    k.replace(k.find(key), key.size(), cases);
  }
  s += k;
  for (size_t i = 0; i < fns.size(); i++)
    if (!fns[i].empty()) s += "      case " + std::to_string(i) + ": " + fns[i] + call;
  s += "    }\n    PCLK(4);\n    }\n  }\n  if (PROF && lane == 0)\n    for (int c = 0; c < 5; c++) atomicAdd(A.prof + c, pc[c]);\n}\n";
  for (size_t at; (at = s.find("PROF")) != std::string::npos;) s.replace(at, 4, g_prof ? "true" : "false");
  return s;
}

std::mutex g_mu;
std::map<std::pair<int, std::string>, hipModule_t> g_modules;   // (device, source) -> module, for the process

}  // namespace

// Packs one extended family's ES_Peeling schedule for d_es_lk: marriage-partial slots are resolved the
// way the reference's partial map behaves (created by the first type-1 step of a couple, looked up by
// later type-2/3 steps, absent before that).  Returns the workspace doubles the family needs, -1 if it
// cannot be packed (family larger than 255 members).
int pack_steps(const pm_pedigree* ped, int f, int ns, std::vector<int2>& out) {
  const int p0 = ped->fam_start[f], n = ped->fam_start[f + 1] - p0;
  if (n > 255 || !ped->peel_start || !ped->steps) return -1;
  std::vector<std::pair<int, int>> keys;
  auto find = [&](int a, int b) {
    for (size_t i = 0; i < keys.size(); i++) if (keys[i].first == a && keys[i].second == b) return (int)i;
    return -1;
  };
  for (int k = ped->peel_start[f]; k < ped->peel_start[f + 1]; k++) {
    const pm_peel_step& S = ped->steps[k];
    int slot = 255, create = 0, fa2mo = 0;
    if (S.type == 1) {
      int i = find(S.to0, S.to1);
      if (i < 0) { i = (int)keys.size(); keys.push_back({S.to0, S.to1}); create = 1; }
      slot = i;
    } else if (S.type == 2) {
      int a, b;
      if (ped->sex[p0 + S.from0] == FEMALE) { a = S.to0; b = S.from0; fa2mo = 0; } else { a = S.from0; b = S.to0; fa2mo = 1; }
      const int i = find(a, b);
      slot = i < 0 ? 255 : i;
    } else if (S.type == 3) {
      const int i = find(S.from0, S.from1);
      slot = i < 0 ? 255 : i;
    } else return -1;
    if (keys.size() > 254) return -1;
    int2 e;
    e.x = (S.type & 255) | ((S.from0 & 255) << 8) | ((S.from1 & 255) << 16) | ((S.to0 & 255) << 24);
    e.y = (S.to1 & 255) | (slot << 8) | (create << 16) | (fa2mo << 17);
    out.push_back(e);
  }
  if (ped->peel_start[f + 1] == ped->peel_start[f]) return -1;
  return n * ns + (int)keys.size() * ns * ns;
}

std::string generate(int chrom, const std::vector<Family>& fams, const double (*tba)[27], Kernel* out, int denovo) {
  std::map<std::string, int> shape_of;
  for (auto& v : out->shape_ops) v.clear();
  std::vector<std::string> names, bodies, post_names, post_bodies, wave_names, wave_bodies, part_names, pen_names;
  int pensz = 1;
  std::vector<int> shape_ns;   // persons per shape
  // --denovo, PM_ES_MULTI=1: a grouped task's three 10-state items in one pass of the wave (the default: one after the other;
  // the three copies of the workspace cut the waves per CU from 14 to 6, and the kernel takes 1.95 ms instead of 1.16)
  const char* em = getenv("PM_ES_MULTI");
  const int pps = (em && em[0] == '1') ? 4 : 3;
  const char* etr = getenv("PM_ES_TR");
  g_tr_regs = etr && !strcmp(etr, "reg");
  const char* epf = getenv("PM_ES_PROF");
  g_prof = epf && epf[0] == '1';
  const char* epk = getenv("PM_ES_PACK");
  g_pack = !(epk && epk[0] == '0');
  const char* erp = getenv("PM_ES_REGP");
  g_regp = erp ? atoi(erp) : 2;
  const char* erf = getenv("PM_ES_REGF");
  g_regf = !(erf && erf[0] == '0');
  const char* eex = getenv("PM_ES_EXPT");
  g_expt = eex ? atoi(eex) : 0;
  const char* efc = getenv("PM_ES_FACT");
  g_fact = denovo != 0 && efc && efc[0] == '1';
  const char* epr = getenv("PM_ES_PAIR");
  const char* efw = getenv("PM_ES_FPW");
  g_fpw = (denovo != 0 && !(epr && epr[0] == '0') && pps == 3) ? 2 : 1;
  if (g_fpw > 1 && efw) g_fpw = atoi(efw) >= 4 ? 4 : atoi(efw) >= 2 ? 2 : 1;
  g_pair = g_fpw > 1;
  g_wl = 64 / g_fpw;
  const char* epp = getenv("PM_ES_PENP");
  g_no_penp = epp && epp[0] == '0';
  const char* efn = getenv("PM_ES_FENCE");
  g_fence = !(efn && efn[0] == '0');
  const char* exd = getenv("PM_ES_XCD");
  g_xcd = !(exd && exd[0] == '0');
  const char* ewp = getenv("PM_ES_WSPACK");
  g_wspack = !(ewp && ewp[0] == '0');
  const char* etz = getenv("PM_ES_T3Z");
  g_no_t3z = etz && etz[0] == '0';
  g_t3z = false;
  if (g_pair) { g_regp = 0; g_regf = false; g_tr_regs = false; }   // (cross-lane reads by LDS only in pair mode)
  {
    int nmax = 0;
    for (const Family& F : fams) nmax = std::max(nmax, F.n);
    const char* ebp = getenv("PM_ES_BAPF");
    // (opt-in, PM_ES_BAPF=1: measured slower, 0.105 vs 0.079 ms per config-4 launch -- 132 VGPRs, 3 waves per SIMD
    // instead of 4, r05bp)
    g_bapf = (!denovo && nmax <= 12 && ebp && ebp[0] == '1') ? 3 * nmax : 0;
  }
  int ws = 1;
  std::vector<std::pair<int, int>> order;   // (shape, index into fams)
  for (size_t i = 0; i < fams.size(); i++) {
    const std::string key = shape_key(fams[i]);
    auto it = shape_of.find(key);
    int id;
    if (it == shape_of.end()) {
      id = (int)names.size();
      shape_of[key] = id;
      names.push_back("fam" + std::to_string(id));
      double o3[6] = {0, 0, 0, 0, 0, 0};
      if (!denovo) {
        bodies.push_back(gen_family(fams[i], chrom, tba, names.back(), &o3[0]));
        post_names.push_back("post" + std::to_string(id));
        post_bodies.push_back(gen_post_family(fams[i], chrom, tba, post_names.back()));
      } else {   // variants 3 id + {0 bi-allelic, 1 10-state, 2 top}
        pen_names.push_back("wfam" + std::to_string(id) + "_pen");
        shape_ns.push_back(fams[i].n);
        wave_bodies.push_back(gen_pen_fill(fams[i].n, pen_names.back()));
        pensz = std::max(pensz, 10 * fams[i].n);
        for (int v = 0; v < 3; v++) {
          int w = 0;
          if (denovo == 2 && v > 0) {   // (grouped tasks only: the de novo items go through the parts)
            wave_names.push_back("");
            continue;
          }
          wave_names.push_back("wfam" + std::to_string(id) + "_" + std::to_string(v));
          wave_bodies.push_back(gen_wave_family(fams[i], chrom, v == 0 ? 3 : 10, v == 2, wave_names.back(), &w, &o3[v]));
          ws = std::max(ws, w);
        }
        for (int p = 1; p <= pps; p++) {   // the leaf prefix, the 10-state rest, the top rest, the 3-item rest (grouped tasks)
          int w = 0;
          double o = 0;
          part_names.push_back("wfam" + std::to_string(id) + (p == 1 ? "_leaf" : p == 2 ? "_rest" : p == 3 ? "_toprest" : "_rest3"));
          wave_bodies.push_back(gen_wave_family(fams[i], chrom, 10, p == 3, part_names.back(), &w, p < 4 ? &o3[2 + p] : &o, p == 1 ? 1 : 2,
                                                p == 4 ? 3 : 1));
          ws = std::max(ws, w);
        }
      }
      for (int v = 0; v < 6; v++) out->shape_ops[v].push_back(o3[v]);
    } else id = it->second;
    order.push_back({id, (int)i});
  }
  std::stable_sort(order.begin(), order.end(), [](const std::pair<int, int>& a, const std::pair<int, int>& b) { return a.first < b.first; });
  out->slot_e.clear(); out->slot_sig.clear(); out->slot_p0.clear(); out->pair_k.clear();
  for (auto& o : order) {
    out->slot_e.push_back(fams[o.second].e);
    out->slot_sig.push_back(o.first);
    out->slot_p0.push_back(fams[o.second].p0);
  }
  // PAIR: consecutive slots of one shape form a pair; an odd one out is paired with itself (both halves compute the
  // same family and store the same values to the same coefficients)
  // (g_fpw families per wave: consecutive slots of one shape form a unit of g_fpw, a short unit padded with its first slot)
  out->pair = g_pair;
  out->fpw = g_fpw;
  for (size_t i = 0; g_pair && i < out->slot_sig.size();) {
    size_t j = i + 1;
    while (j < out->slot_sig.size() && (int)(j - i) < g_fpw && out->slot_sig[j] == out->slot_sig[i]) j++;
    for (int f = 0; f < g_fpw; f++) out->pair_k.push_back((int)(i + f < j ? i + f : i));
    i = j;
  }
  out->n_shapes = (int)names.size();
  std::string src = kPrologue;
  if (!denovo) {
    for (auto& b : bodies) src += b;
    src += gen_kernel(names);
    src += kPostPrologue;
    for (auto& b : post_bodies) src += b;
    src += gen_post_kernel(post_names);
    out->wave = false;
  } else {
    // waves per block: as many workspace slices as fit the 64 KB of static LDS next to the tables
    const int tables = (256 + 6 * 27) * 8 + (g_t3z ? (320 + 10) * 4 : 0);
    // (one wave per SIMD: the occupancy comes from blocks per CU, build() asks the runtime for them)
    const int slice = g_fpw * (ws + pensz) * 8;   // (a unit's family slices per wave)
    // (at most 4: one wave per SIMD and block; measured on config 4 --denovo, 4 beat 1, 2, 5 and 6 even where those
    // gave more waves per CU -- profiles/r05k_ab_es_wpb.txt)
    const int fit = (64 * 1024 - tables) / slice;
    out->wpb = std::max(0, std::min(4, fit));
    if (const char* ew = getenv("PM_ES_WPB")) out->wpb = std::max(1, std::min(fit, atoi(ew)));
    // (wpb 0: a family too large for one slice -- the engine's generic kernel)
    std::string wk = gen_wave_kernel(wave_names, part_names, pen_names, shape_ns, pps, ws, pensz, std::max(1, out->wpb), denovo == 2);
    const size_t at = wk.find("extern \"C\"");   // device helpers first, then the family functions, then the kernel
    src += wk.substr(0, at);
    {   // the family units' slot words (unit = slot pair in pair mode, else slot; both halves' entries): constants
      const size_t nu = g_pair ? out->pair_k.size() / g_fpw : out->slot_e.size();
      const std::string nf = std::to_string(g_fpw * nu);
      std::string p0 = "__constant__ int kUP0[" + nf + "] = {", e = "__constant__ int kUE[" + nf + "] = {",
                  sg = "__constant__ int kUSig[" + std::to_string(nu) + "] = {";
      for (size_t u = 0; u < nu; u++) {
        for (int f = 0; f < g_fpw; f++) {
          const int k = g_pair ? out->pair_k[g_fpw * u + f] : (int)u;
          p0 += std::to_string(out->slot_p0[k]) + ",";
          e += std::to_string(out->slot_e[k]) + ",";
        }
        sg += std::to_string(out->slot_sig[g_pair ? out->pair_k[g_fpw * u] : (int)u]) + ",";
      }
      src += p0 + "};\n" + e + "};\n" + sg + "};\n__device__ constexpr int kNUnits = " + std::to_string(nu) + ";\n";
    }
    if (g_t3z) {   // the plain Mendelian T(e = i 10 + j, k)'s non-zero terms per child state k, ascending e: e << 2 | code
      auto gi = [](int b1, int b2) { return b1 < b2 ? (b1 - 1) * (10 - b1) / 2 + (b2 - b1) : (b2 - 1) * (10 - b2) / 2 + (b1 - b2); };
      std::vector<double> T(1000, 0.0);
      for (int i = 1; i <= 4; i++)
        for (int j = i; j <= 4; j++)
          for (int k = 1; k <= 4; k++)
            for (int m = k; m <= 4; m++) {
              const int g[4] = {gi(i, k), gi(i, m), gi(j, k), gi(j, m)};
              for (int t = 0; t < 4; t++) T[(gi(i, j) * 10 + gi(k, m)) * 10 + g[t]] += 0.25;
            }
      std::string z = "__shared__ int t3z[320], t3n[10];\n__device__ const int kT3z[320] = {", zn = "__device__ const int kT3n[10] = {";
      for (int k = 0; k < 10; k++) {
        int q = 0;
        for (int e = 0; e < 100; e++) {
          const double t = T[e * 10 + k];
          if (t == 0.0) continue;
          const int code = t == 1.0 ? 0 : t == 0.5 ? 1 : 2;
          if (code == 2 && t != 0.25) { fprintf(stderr, "es_jit: unexpected Mendelian entry\n"); abort(); }
          z += std::to_string(e << 2 | code) + ",";
          q++;
        }
        if (q > 32) { fprintf(stderr, "es_jit: Mendelian list over 32\n"); abort(); }
        for (; q < 32; q++) z += "0,";
        zn += std::to_string([&] { int c = 0; for (int e = 0; e < 100; e++) c += T[e * 10 + k] != 0.0; return c; }()) + ",";
      }
      src += z + "};\n" + zn + "};\n";
    }
    for (auto& b : wave_bodies) src += b;
    src += wk.substr(at);
    out->wave = true;
    out->ws = ws;
  }
  return src;
}

bool compile(const std::string& src, std::vector<char>* code, std::string* err, const std::string& arch) {
  hiprtcProgram prog;
  // the shared device headers (brent_core.h, log_table.h), embedded at build time (Makefile: build/jit_headers.inc)
  const char* hdr[] = {kBrentCoreH, kLogTableH};
  const char* hdr_names[] = {"brent_core.h", "log_table.h"};
  if (hiprtcCreateProgram(&prog, src.c_str(), "es_hoist_jit.hip", 2, hdr, hdr_names) != HIPRTC_SUCCESS) {
    *err = "hiprtcCreateProgram failed";
    return false;
  }
  // -ffp-contract=off: only the explicit fma() of the generated code fuses
  // (the device's own target -- gcnArchName without feature suffixes -- so the module always loads on it)
  const std::string off = "--offload-arch=" + arch;
  const char* opts[] = {off.c_str(), "-O3", "-ffp-contract=off", "-std=c++17"};
  const hiprtcResult rc = hiprtcCompileProgram(prog, 4, opts);
  if (rc != HIPRTC_SUCCESS) {
    size_t ls = 0;
    hiprtcGetProgramLogSize(prog, &ls);
    std::string log(ls + 1, '\0');
    hiprtcGetProgramLog(prog, &log[0]);
    *err = "hipRTC compile of the peeling kernel failed: " + log.substr(0, 2000);
    hiprtcDestroyProgram(&prog);
    return false;
  }
  size_t cs = 0;
  hiprtcGetCodeSize(prog, &cs);
  code->resize(cs);
  hiprtcGetCode(prog, code->data());
  hiprtcDestroyProgram(&prog);
  return true;
}

bool build(int device, int chrom, const std::vector<Family>& fams, const double (*tba)[27], int denovo, Kernel* out,
           std::string* err) {
  const auto t0 = std::chrono::steady_clock::now();
  const std::string src = generate(chrom, fams, tba, out, denovo);
  if (denovo && out->wpb == 0) { *err = "family workspace exceeds a block's LDS"; return false; }
  std::lock_guard<std::mutex> lock(g_mu);
  auto key = std::make_pair(device, src);
  auto it = g_modules.find(key);
  if (it == g_modules.end()) {
    std::vector<char> code;
    std::string arch = "gfx950";
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.gcnArchName[0]) {
      arch = prop.gcnArchName;
      arch = arch.substr(0, arch.find(':'));
    }
    if (!compile(src, &code, err, arch)) return false;
    hipModule_t mod;
    if (hipSetDevice(device) != hipSuccess || hipModuleLoadData(&mod, code.data()) != hipSuccess) {
      *err = "hipModuleLoadData of the peeling kernel failed";
      return false;
    }
    it = g_modules.emplace(key, mod).first;
  }
  const bool ok = denovo ? hipModuleGetFunction(&out->fn, it->second, "es_hoist_wave") == hipSuccess
                         : hipModuleGetFunction(&out->fn, it->second, "es_hoist_jit") == hipSuccess &&
                               hipModuleGetFunction(&out->fn_post, it->second, "es_post_jit") == hipSuccess;
  if (!ok) {
    *err = "hipModuleGetFunction of the generated kernels failed";
    return false;
  }
  if (denovo || g_bapf) {   // resident blocks per CU (VGPRs and LDS): the launch's grid
    int nb = 0;
    if (hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&nb, out->fn, denovo ? 64 * out->wpb : 256, 0) != hipSuccess) nb = 0;
    out->blocks_per_cu = nb;
    if (getenv("PM_JIT_LAYOUT")) fprintf(stderr, "es_hoist_wave: wpb %d ws %d blocks/CU %d\n", out->wpb, out->ws, nb);
  }
  out->compile_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return true;
}

// ---------------------------------------------------------------------------------------------------------------
// ep_brent_jit: the fused hoisting + Brent kernel (es_jit.h FusedKernel).  Layout: families sorted by (degree
// descending, shape), dealt row-major onto rows of `lanes` cells; each row's register tile holds its largest degree
// + 1 coefficients.  The lane count is chosen by a cost model of one item: hoisting = the generated peels' operations
// of every shape present in a row (a row's lanes run the shapes it holds one after the other), evaluations = about
// 30 Brent evaluations x 2 (D_row + 1) Horner operations per row; a lane's degrees summed stay <= 64 (g^D >= 1e-256
// at Brent's start b = 0.9999) and the tiles <= 64 doubles.
std::string generate_fused(int chrom, const std::vector<Family>& fams, const double (*tba)[27], FusedKernel* out) {
  const int n = (int)fams.size();
  out->lane_tab.clear(); out->row_deg.clear(); out->rows = out->lanes = out->n_shapes = 0; out->item_ops = 0;
  if (n == 0) return "";
  std::map<std::string, int> shape_of;
  std::vector<std::string> bodies;
  std::vector<int> sdeg;
  std::vector<double> sops;
  std::vector<int> sig(n);
  for (int i = 0; i < n; i++) {
    const std::string key = shape_key(fams[i]);
    auto it = shape_of.find(key);
    if (it == shape_of.end()) {
      const int id = (int)bodies.size();
      shape_of[key] = id;
      double o = 0;
      int d = 0;
      bodies.push_back(gen_family(fams[i], chrom, tba, "ffam" + std::to_string(id), &o, true, &d));
      sdeg.push_back(d);
      sops.push_back(o);
      sig[i] = id;
    } else sig[i] = it->second;
  }
  const int ns = (int)bodies.size();
  if (ns > 127) return "";
  std::vector<int> order(n);
  for (int i = 0; i < n; i++) order[i] = i;
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
    return sdeg[sig[a]] != sdeg[sig[b]] ? sdeg[sig[a]] > sdeg[sig[b]] : sig[a] < sig[b];
  });
  // Two layouts: one item per wave (rows of up to 64 cells), or two (pair: each half-wave, 32 lanes, runs its own item
  // on rows of up to 32 cells -- the evaluation's fixed part (division, power, reduction, log10, Brent's update) is then
  // shared by two items, at the price of twice the rows and of the longer of the two Brent runs).  Per-item cost model:
  // hoisting + kEvals x (2 (D_row + 1) per row + the fixed part), the pair layout's halved.
  const int kRowsMax = 8, kTile = 64, kEvals = 30;
  const double kFixed1 = 150, kFixed2 = 230, kImb = 1.1;
  const char* epair = getenv("PM_FUSED_PAIR");   // (0 / 1: force one layout)
  double best = -1;
  int best_nl = 0;
  bool pair = false;
  for (int pm = 0; pm < 2; pm++) {
    if (epair && atoi(epair) != pm) continue;
    const int lmax = pm ? 32 : 64;
    for (int nl = (n + kRowsMax - 1) / kRowsMax; nl <= lmax; nl++) {
      if (nl <= 0) continue;
      const int rows = (n + nl - 1) / nl;
      double hoist = 0, eval = pm ? kFixed2 : kFixed1;
      int tile = 0;
      std::vector<int> lane_deg(nl, 0);
      for (int r = 0; r < rows; r++) {
        std::vector<char> seen(ns, 0);
        int dmax = 0;
        for (int k = r * nl; k < std::min(n, (r + 1) * nl); k++) {
          const int sg = sig[order[k]];
          if (!seen[sg]) { seen[sg] = 1; hoist += sops[sg]; }
          dmax = std::max(dmax, sdeg[sg]);
          lane_deg[k - r * nl] += sdeg[sg];
        }
        tile += dmax + 1;
        eval += 2.0 * (dmax + 1);
      }
      if (tile > kTile || *std::max_element(lane_deg.begin(), lane_deg.end()) > 64) continue;
      const double cost = pm ? (hoist + kImb * kEvals * eval) / 2 : hoist + kEvals * eval;
      if (best < 0 || cost < best) { best = cost; best_nl = nl; pair = pm; }
    }
  }
  if (best_nl == 0) return "";
  const int nl = best_nl, rows = (n + nl - 1) / nl;
  out->lanes = nl; out->rows = rows; out->n_shapes = ns; out->pair = pair;
  out->lane_tab.assign((size_t)rows * 64 + 64, -1);
  for (int l = 0; l < 64; l++) out->lane_tab[(size_t)rows * 64 + l] = 0;
  std::vector<std::vector<int>> row_shapes(rows);
  for (int r = 0; r < rows; r++) {
    int dmax = 0;
    for (int k = r * nl; k < std::min(n, (r + 1) * nl); k++) {
      const Family& F = fams[order[k]];
      const int sg = sig[order[k]], l = k - r * nl;
      out->lane_tab[(size_t)r * 64 + l] = F.p0 | (sg << 24);
      out->lane_tab[(size_t)rows * 64 + l] += sdeg[sg];
      if (std::find(row_shapes[r].begin(), row_shapes[r].end(), sg) == row_shapes[r].end()) row_shapes[r].push_back(sg);
      dmax = std::max(dmax, sdeg[sg]);
    }
    out->row_deg.push_back(dmax);
  }
  if (pair)   // (both halves hoist the same families for their own items)
    for (int r = 0; r <= rows; r++)
      for (int l = 32; l < 64; l++) out->lane_tab[(size_t)r * 64 + l] = out->lane_tab[(size_t)r * 64 + l - 32];
  for (int i = 0; i < n; i++) out->item_ops += sops[sig[i]];
  if (getenv("PM_JIT_LAYOUT")) {
    fprintf(stderr, "ep_brent_jit: %d families, %d shapes, %d rows x %d lanes%s, tiles", n, ns, rows, nl, pair ? " (two items per wave)" : "");
    for (int r = 0; r < rows; r++) fprintf(stderr, " %d(%zu)", out->row_deg[r], row_shapes[r].size());
    fprintf(stderr, ", cost %.0f\n", best);
  }
  std::string src = kPrologue;
  src += "#include \"brent_core.h\"\n";
  src += R"(
struct FusedArgs {
  const int* items; int* counts; const uint8_t* ref; const int* res; const uint8_t* pl; const double* lktab; const int* lane_tab;
  double* raw; double* minv; int* evals; unsigned long long* eval_total;
  double precision;
  int list, it0, it1, np, vcf, res_words, res_a1, res_a2, itmax, pad;
};
)";
  for (auto& b : bodies) src += b;
  const char* wpe = getenv("PM_FUSED_WPE");   // (experiments: amdgpu_waves_per_eu of the kernel)
  src += std::string("extern \"C\" __global__ void __launch_bounds__(64) ") +
         (wpe ? "__attribute__((amdgpu_waves_per_eu(" + std::string(wpe) + ", " + std::string(wpe) + "))) " : "") +
         "ep_brent_jit(FusedArgs A) {\n";
  src += R"(  __shared__ double lk[256];
  for (int i = threadIdx.x; i < 256; i += 64) lk[i] = A.lktab[i];
  __syncthreads();
  const int lane = threadIdx.x;
  const int nItems = min(A.counts[A.list], A.it1);
  // XCD-aware item order (blocks go round-robin to the 8 XCDs): consecutive items -- one site's configurations, one
  // PL block -- on blocks of one XCD
  const int vb = (gridDim.x % 8 == 0) ? (blockIdx.x % 8) * (gridDim.x / 8) + blockIdx.x / 8 : blockIdx.x;
)";
  src += "  int ltab[" + std::to_string(rows) + "];\n";
  src += "#pragma unroll\n  for (int r = 0; r < " + std::to_string(rows) + "; r++) ltab[r] = A.lane_tab[r * 64 + lane];\n";
  src += "  const int edl = A.lane_tab[" + std::to_string(rows * 64) + " + lane];   // g^edl: the lane's degrees summed\n";
  if (!pair)
    src += R"(  unsigned long long ev_acc = 0;
  for (int it = A.it0 + vb; it < nItems; it += gridDim.x) {
    const int item = A.items[it];
)";
  else   // half-wave h takes item it0 + 2 t + h (a missing second item: the first one's data, nothing written)
    src += R"(  unsigned long long ev_acc = 0;
  const int half = lane >> 5;
  for (int t2 = vb; A.it0 + 2 * t2 < nItems; t2 += gridDim.x) {
    const int it = A.it0 + 2 * t2 + half;
    const bool valid = it < nItems;
    const int item = A.items[valid ? it : it - 1];
)";
  src += R"(

    const int site = item >> 3, cfg = item & 7, rb = A.ref[site];
    int a1, a2;
    if (A.vcf) { a1 = rb & 15; a2 = rb >> 4; }
    else if (cfg == 7) { a1 = A.res[(size_t)site * A.res_words + A.res_a1]; a2 = A.res[(size_t)site * A.res_words + A.res_a2]; }
    else cfg_alleles(cfg, rb, &a1, &a2);
    const uint8_t* pls = A.pl + (size_t)site * A.np * 10;
    const uint8_t* P11 = pls + (size_t)gi(a1, a1) * A.np;
    const uint8_t* P12 = pls + (size_t)gi(a1, a2) * A.np;
    const uint8_t* P22 = pls + (size_t)gi(a2, a2) * A.np;
)";
  for (int r = 0; r < rows; r++) {
    const int D = out->row_deg[r];
    const std::string c = "c" + std::to_string(r), R = std::to_string(r);
    src += "    double " + c + "[" + std::to_string(D + 1) + "];\n";
    src += "    if (ltab[" + R + "] < 0) {   // no family: the unit polynomial\n      " + c + "[0] = 1.0;\n";
    for (int a = 1; a <= D; a++) src += "      " + c + "[" + std::to_string(a) + "] = 0.0;\n";
    src += "    } else {\n      const int p0 = ltab[" + R + "] & 0xFFFFFF, sg = ltab[" + R + "] >> 24;\n";
    for (size_t k = 0; k < row_shapes[r].size(); k++) {
      const int sg = row_shapes[r][k];
      src += std::string(k == 0 ? "      " : " else ") +
             (k + 1 < row_shapes[r].size() ? "if (sg == " + std::to_string(sg) + ") " : "") + "{\n";
      src += "        ffam" + std::to_string(sg) + "(P11, P12, P22, p0, lk, " + c + ");\n";
      for (int a = sdeg[sg] + 1; a <= D; a++) src += "        " + c + "[" + std::to_string(a) + "] = 0.0;\n";
      src += "      }";
    }
    src += "\n    }\n";
  }
  src += R"(    PmBrent B;
    pm_brent_init(B, A.precision, A.itmax);
)";
  if (pair) src += "    bool done = !valid;\n";
  src += R"(    for (;;) {
      // every family L = g^D sum_a c_a t^a, t = f / g (non-negative terms: no cancellation), FMA Horner over the row's
      // tile (zeros above a family's own degree leave the sum's bits unchanged); the values split into mantissa and
      // exponent, multiplied in one chain with g^edl, one renormalisation -- as k_brent's EP evaluation
      const double g = 1.0 - B.x;
      const double t = pos_div(B.x, g);
)";
  {   // g^edl: the layout's distinct lane degree sums are known here -- shared squarings, one power per value, a select
    std::vector<int> vals;
    for (int l = 0; l < 64; l++) {
      const int v = out->lane_tab[(size_t)rows * 64 + l];
      if (v > 0 && std::find(vals.begin(), vals.end(), v) == vals.end()) vals.push_back(v);
    }
    std::sort(vals.begin(), vals.end());
    int top = 0;
    for (int v : vals) top = std::max(top, v);
    int nb = 0;
    while ((1 << (nb + 1)) <= top) nb++;   // the highest bit of any value
    src += "      double q0 = g;\n";
    for (int b = 1; b <= nb; b++) src += "      const double q" + std::to_string(b) + " = q" + std::to_string(b - 1) + " * q" + std::to_string(b - 1) + ";\n";
    src += "      double pw = 1.0;\n";
    for (size_t k = 0; k < vals.size(); k++) {
      std::string prod;
      for (int b = 0; b <= nb; b++)   // (ascending bits: the order of the former square-and-multiply loop)
        if ((vals[k] >> b) & 1) prod = prod.empty() ? "q" + std::to_string(b) : "(" + prod + ") * q" + std::to_string(b);
      src += "      if (edl == " + std::to_string(vals[k]) + ") pw = " + prod + ";\n";
    }
  }
  src += "      int e = 0;\n";
  for (int r = 0; r < rows; r++) {
    const int D = out->row_deg[r];
    const std::string c = "c" + std::to_string(r), R = std::to_string(r);
    src += "      double m" + R + ";\n      {\n        double acc = " + c + "[" + std::to_string(D) + "];\n";
    for (int a = D - 1; a >= 0; a--) src += "        acc = fma(acc, t, " + c + "[" + std::to_string(a) + "]);\n";
    src += "        int e1;\n        m" + R + " = frexp(acc, &e1);\n        e += e1;\n      }\n";
  }
  src += "      double m = m0";
  for (int r = 1; r < rows; r++) src += " * m" + std::to_string(r);
  src += R"(;
      int e2;
      m = frexp(m * pw, &e2);
      e += e2;
)";
  if (!pair)
    src += R"(      wave_prod(m, e);
      if (!pm_brent_feed(B, -log10_mant_u(m, e))) break;
    }
    if (lane == 0) {
)";
  else   // (a half whose Brent has ended keeps its state; the wave goes on until both have)
    src += R"(      wave_prod_pair(m, e);
      const double fx = -log10_mant_pair(m, e);
      if (!done && !pm_brent_feed(B, fx)) done = true;
      if (__ballot(!done) == 0) break;
    }
    if ((lane & 31) == 0 && valid) {
)";
  src += R"(      A.raw[(size_t)site * 8 + cfg] = -B.fmin;
      A.minv[(size_t)site * 8 + cfg] = B.mn;
      A.evals[(size_t)site * 8 + cfg] = B.nev;
      ev_acc += B.nev - 2;   // objective evaluations computed (f(a), f(c) counted only)
      if (!B.ok) { atomicExch(&A.counts[5], 1); atomicMin(&A.counts[6], site); }   // (the reference stops at the first)
    }
  }
  if ((lane & 31) == 0 && ev_acc) atomicAdd(A.eval_total, ev_acc);
}
)";
  return src;
}

bool build_fused(int device, int chrom, const std::vector<Family>& fams, const double (*tba)[27], FusedKernel* out,
                 std::string* err) {
  const auto t0 = std::chrono::steady_clock::now();
  const std::string src = generate_fused(chrom, fams, tba, out);
  if (src.empty()) { *err = "the families do not fit the fused kernel's register tiles"; return false; }
  std::lock_guard<std::mutex> lock(g_mu);
  auto key = std::make_pair(device, src);
  auto it = g_modules.find(key);
  if (it == g_modules.end()) {
    std::vector<char> code;
    std::string arch = "gfx950";
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.gcnArchName[0]) {
      arch = prop.gcnArchName;
      arch = arch.substr(0, arch.find(':'));
    }
    if (!compile(src, &code, err, arch)) return false;
    hipModule_t mod;
    if (hipSetDevice(device) != hipSuccess || hipModuleLoadData(&mod, code.data()) != hipSuccess) {
      *err = "hipModuleLoadData of the fused Brent kernel failed";
      return false;
    }
    it = g_modules.emplace(key, mod).first;
  }
  if (hipModuleGetFunction(&out->fn, it->second, "ep_brent_jit") != hipSuccess) {
    *err = "hipModuleGetFunction(ep_brent_jit) failed";
    return false;
  }
  int nb = 0;
  if (hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&nb, out->fn, 64, 0) != hipSuccess) nb = 0;
  out->blocks_per_cu = nb;
  if (getenv("PM_JIT_LAYOUT")) fprintf(stderr, "ep_brent_jit: blocks/CU %d\n", nb);
  out->compile_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return true;
}

}  // namespace pmjit
