// synth_core.h -- synthetic GLF workload of SURVEY.md section 8(d), shared bit-for-bit between the
// device generator (pm_engine_synth) and the host GLF-file writer (pmh_synth_write_dataset), so the
// GPU bench and the CPU baseline see identical sites.
//
//   refBase ~ U{1..4}; 10% of sites polymorphic with alt = transition(ref), alt AF ~ U(0.05, 0.5)
//   founders' haplotypes ~ Bernoulli(AF); non-founders inherit one random haplotype from each parent
//   depth ~ U{8..29}; alt read count ~ Binomial(depth, {0.01, 0.5, 0.99}[genotype]) (error 1%)
//   PL(11,12,22) = round(-10 (log10 L - max log10 L)) capped at 255; the other 7 genotypes = 255
//   mapQ = 60
// Randomness is a stateless counter hash of (seed, global site, person, stream), so any shard of
// sites can be generated independently on any GPU.  Binomial sampling and PL use host-built tables
// (glibc pow/log10), uploaded to the device, so both sides round identically.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define PM_HD __host__ __device__
#else
#define PM_HD
#endif

#define PM_SYN_MAXDEPTH 30   /* depth is 8..29 */

struct pm_synth_tables {
  double cdf[3][PM_SYN_MAXDEPTH][PM_SYN_MAXDEPTH + 1];   // P(nalt <= k | genotype, depth)
  uint8_t pl[PM_SYN_MAXDEPTH][PM_SYN_MAXDEPTH + 1][3];   // PL triple for (depth, nalt)
};

PM_HD static inline uint64_t pm_mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// uniform in [0,1) with 53 random bits; exact on host and device
PM_HD static inline double pm_u01(uint64_t seed, uint64_t site, uint64_t person, uint32_t stream) {
  uint64_t h = pm_mix64(seed ^ pm_mix64(site * 0x100000001B3ull ^ pm_mix64(person * 0x9E3779B1ull + stream)));
  return (double)(h >> 11) * (1.0 / 9007199254740992.0);
}

PM_HD static inline int pm_syn_ts(int r) { return r == 1 ? 3 : r == 2 ? 4 : r == 3 ? 1 : 2; }
PM_HD static inline int pm_syn_gi(int b1, int b2) {
  return b1 < b2 ? (b1 - 1) * (10 - b1) / 2 + (b2 - b1) : (b2 - 1) * (10 - b2) / 2 + (b1 - b2);
}

// Site header: refBase (1..4) and alt-allele frequency (0 for monomorphic sites).
PM_HD static inline void pm_syn_site(uint64_t seed, uint64_t site, int* ref, double* af) {
  const uint64_t S = ~0ull;   // person slot reserved for site-level streams
  *ref = 1 + (int)(pm_u01(seed, site, S, 0) * 4.0);
  bool poly = pm_u01(seed, site, S, 1) < 0.1;
  *af = poly ? 0.05 + pm_u01(seed, site, S, 2) * 0.45 : 0.0;
}

// One family's persons (path order, parents before children).  gbase = global index of the
// family's first person (used as the RNG person key).  fa/mo are family-local parent indices (-1 for
// founders).  Writes person j's genotype k at pl[j * ps + k * gs] (ps = 10, gs = 1: person-major GLF
// records; ps = 1, gs = n_person: the engine's genotype-planar site block) and dm[j].
PM_HD static inline void pm_syn_family(const pm_synth_tables* T, uint64_t seed, uint64_t site, int ref, double af, int n,
                                       const int32_t* fa, const int32_t* mo, uint64_t gbase, uint8_t* pl, size_t ps, size_t gs,
                                       uint32_t* dm, uint8_t* hap /* scratch [n] */) {
  const int alt = pm_syn_ts(ref);
  const int i0 = pm_syn_gi(ref, ref), i1 = pm_syn_gi(ref, alt), i2 = pm_syn_gi(alt, alt);
  for (int j = 0; j < n; j++) {
    const uint64_t key = gbase + (uint64_t)j;
    uint8_t h0, h1;
    if (fa[j] < 0) {
      h0 = pm_u01(seed, site, key, 0) < af;
      h1 = pm_u01(seed, site, key, 1) < af;
    } else {
      uint8_t hf = hap[fa[j]], hm = hap[mo[j]];
      h0 = (pm_u01(seed, site, key, 2) < 0.5) ? (hf & 1) : (hf >> 1);
      h1 = (pm_u01(seed, site, key, 3) < 0.5) ? (hm & 1) : (hm >> 1);
    }
    hap[j] = (uint8_t)(h0 | (h1 << 1));
    const int g = h0 + h1;
    const int depth = 8 + (int)(pm_u01(seed, site, key, 4) * 22.0);
    const double u = pm_u01(seed, site, key, 5);
    int nalt = 0;
    while (nalt < depth && u >= T->cdf[g][depth][nalt]) nalt++;
    uint8_t* rec = pl + (size_t)j * ps;
    for (int k = 0; k < 10; k++) rec[k * gs] = 255;
    rec[i0 * gs] = T->pl[depth][nalt][0];
    rec[i1 * gs] = T->pl[depth][nalt][1];
    rec[i2 * gs] = T->pl[depth][nalt][2];
    dm[j] = (uint32_t)depth | (60u << 24);
  }
}

#ifdef __cplusplus
extern "C" {
#endif
/* Host: fill the binomial CDF and PL tables with glibc arithmetic (polymutt_amd/host/synth.cpp). */
void pm_synth_build_tables(struct pm_synth_tables* T);
#ifdef __cplusplus
}
#endif
