// brent_core.h -- the device pieces of the Brent objective evaluation that the precompiled k_brent (engine_dev.h)
// and the run-time compiled Elston-Stewart Brent kernel (es_jit.cpp: ep_brent_jit, hipRTC) share, so both evaluate
// the objective and step Brent with the same instructions:
//   * pos_div: a positive quotient from the hardware reciprocal (Brent's serial path)
//   * wave_prod: the product of the 64 lanes' (mantissa, exponent) pairs on the DPP crossbar, in a fixed order
//   * log10_mant_u: log10 of a wave-uniform normalised mantissa from a 128-entry table (log_table.h)
//   * PmBrent / pm_brent_feed: OptimizeFrequency's bracketing (NucFamGenotypeLikelihood.cpp:432-441) and
//     ScalarMinimizer::Brent (core/MathGold.cpp:81-177) as a state machine fed one objective value at a time
// Self-contained (no host headers): hipRTC compiles it from the text embedded by the Makefile (build/jit_headers.inc).
#pragma once
#include "log_table.h"

#ifndef PM_LOG10_2_HI
#define PM_LOG10_2_HI 0x1.3441350800000p-2
#define PM_LOG10_2_LO 0x1.f79fef311f12bp-34
#endif

__device__ __forceinline__ double d_sign(double a, double b) { return b >= 0 ? fabs(a) : -fabs(a); }

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

// The same product over each half-wave (lanes 0-31 and 32-63: two Brent items per wave): the first five steps (rows 0+1
// end in lane 31, rows 2+3 in lane 63), then each half takes its own lane's product -- the order of wave_prod's first
// five steps.  Every lane of a half ends with that half's (m, e), m normalised.
__device__ __forceinline__ void wave_prod_pair(double& m, int& e) {
  dpp_prod_step<0xB1, 0xF>(m, e);    // quad_perm [1,0,3,2]
  dpp_prod_step<0x4E, 0xF>(m, e);    // quad_perm [2,3,0,1]
  dpp_prod_step<0x141, 0xF>(m, e);   // row_half_mirror
  dpp_prod_step<0x140, 0xF>(m, e);   // row_mirror
  dpp_prod_step<0x142, 0xA>(m, e);   // row_bcast:15 -> rows 1, 3
  const double mA = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(m), 31), __builtin_amdgcn_readlane(__double2loint(m), 31));
  const double mB = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(m), 63), __builtin_amdgcn_readlane(__double2loint(m), 63));
  const int eA = __builtin_amdgcn_readlane(e, 31), eB = __builtin_amdgcn_readlane(e, 63);
  const bool hi = (__lane_id() >> 5) != 0;
  int ev;
  m = frexp(hi ? mB : mA, &ev);
  e = (hi ? eB : eA) + ev;
}

// log10(m * 2^e) for a WAVE-UNIFORM normalised mantissa m in [0.5, 1) (or 0): the top 7 fraction bits of m pick
// c_i ~ 1 / m and L_i = -log10(c_i) (log_table.h, scalar loads at a uniform index), z = m c_i - 1 (one rounding, |z|
// < 2^-8), log10(1 + z) by a degree-6 Horner series (truncation < 5e-19); absolute error ~1e-16, like log10_mant's,
// in ~12 VALU operations instead of ~40 and without the division.  (Brent's serial path: every objective evaluation.)
static __constant__ double c_log10_tab[256] = PM_LOG10_TAB_VALUES;
__device__ __forceinline__ double log10_mant_u(double m, int e) {
  if (m == 0.0) return -__builtin_inf();   // an underflowed family product: log10(0), as the reference
  const int i = (__builtin_amdgcn_readfirstlane(__double2hiint(m)) >> 13) & 0x7F;
  const double c = c_log10_tab[2 * i], L = c_log10_tab[2 * i + 1];
  const double z = fma(m, c, -1.0);
  double p = fma(z, PM_LOG10_SER_6, PM_LOG10_SER_5);
  p = fma(z, p, PM_LOG10_SER_4);
  p = fma(z, p, PM_LOG10_SER_3);
  p = fma(z, p, PM_LOG10_SER_2);
  p = fma(z, p, PM_LOG10_SER_1);
  const double de = (double)e;
  return fma(z, p, L) + (de * PM_LOG10_2_HI + de * PM_LOG10_2_LO);
}

// log10_mant_u for a mantissa uniform over each half-wave (wave_prod_pair): the two halves' table entries by scalar loads
// at their (uniform) indices, each lane computing with its half's -- the same operations as log10_mant_u
__device__ __forceinline__ double log10_mant_pair(double m, int e) {
  const int hA = __builtin_amdgcn_readlane(__double2hiint(m), 31), hB = __builtin_amdgcn_readlane(__double2hiint(m), 63);
  const int iA = (hA >> 13) & 0x7F, iB = (hB >> 13) & 0x7F;
  const bool hi = (__lane_id() >> 5) != 0;
  const double c = hi ? c_log10_tab[2 * iB] : c_log10_tab[2 * iA];
  const double L = hi ? c_log10_tab[2 * iB + 1] : c_log10_tab[2 * iA + 1];
  const double z = fma(m, c, -1.0);
  double p = fma(z, PM_LOG10_SER_6, PM_LOG10_SER_5);
  p = fma(z, p, PM_LOG10_SER_4);
  p = fma(z, p, PM_LOG10_SER_3);
  p = fma(z, p, PM_LOG10_SER_2);
  p = fma(z, p, PM_LOG10_SER_1);
  const double de = (double)e;
  const double r = fma(z, p, L) + (de * PM_LOG10_2_HI + de * PM_LOG10_2_LO);
  return m == 0.0 ? -__builtin_inf() : r;
}

// OptimizeFrequency + Brent as a state machine (the same operations, in the same order, as k_brent's loop):
// OptimizeFrequency (NucFamGenotypeLikelihood.cpp:432-441) evaluates f(a), f(b), f(c) and calls Brent, which reads only
// f(b) (MathGold.cpp:85-93: a < c, so fa and fc are never swapped in or read) -- f(a) and f(c) are counted in nev, as
// the reference counts them, but not computed.  The caller evaluates -objective at x, feeds it, and evaluates again
// while pm_brent_feed returns true; then mn / fmin hold the minimiser, ok whether it converged (false: ITMAX, the
// reference's numerror "ScalarMinimizer::Brent got stuck", MathGold.cpp:98,175).
struct PmBrent {
  double a, c, x, mn, fmin, w, v, fw, fv, delta, d, tol;
  int phase, iter, nev, itmax;
  bool ok;
};
__device__ __forceinline__ void pm_brent_init(PmBrent& B, double tol, int itmax) {
  B.a = 0.0001; B.c = 0.5; B.x = 0.9999;   // Brent starts at b = 0.9999, outside [a, c]
  B.mn = B.fmin = B.w = B.v = B.fw = B.fv = 0.0;
  B.delta = B.d = 0.0;
  B.tol = tol;
  B.phase = 1; B.iter = 0; B.nev = 1; B.itmax = itmax;   // nev: f(a) counted
  B.ok = false;
}
__device__ __forceinline__ bool pm_brent_feed(PmBrent& B, double fx) {
  B.nev++;
  if (B.phase == 1) {   // fb; then f(c), counted only; Brent: min = b, fmin = fb (MathGold.cpp:91-93)
    B.fmin = fx; B.nev++;
    B.phase = 3; B.mn = 0.9999; B.w = B.mn; B.v = B.mn; B.fw = B.fmin; B.fv = B.fmin;
  } else {
    const double u = B.x, fu = fx;
    if (fu <= B.fmin) {
      if (u >= B.mn) B.a = B.mn; else B.c = B.mn;
      B.v = B.w; B.w = B.mn; B.mn = u;
      B.fv = B.fw; B.fw = B.fmin; B.fmin = fu;
    } else {
      if (u < B.mn) B.a = u; else B.c = u;
      if (fu <= B.fw || B.w == B.mn) { B.v = B.w; B.w = u; B.fv = B.fw; B.fw = fu; }
      else if (fu <= B.fv || B.v == B.mn || B.v == B.w) { B.v = u; B.fv = fu; }
    }
  }
  if (++B.iter > B.itmax) return false;   // ITMAX: numerror("ScalarMinimizer::Brent got stuck")
  const double middle = 0.5 * (B.a + B.c);
  const double tol1 = B.tol * fabs(B.mn) + 3.0e-10;
  const double tol2 = 2.0 * tol1;
  if (fabs(B.mn - middle) <= (tol2 - 0.5 * (B.c - B.a))) { B.ok = true; return false; }
  if (fabs(B.delta) > tol1) {
    double rr = (B.mn - B.w) * (B.fmin - B.fv);
    double q = (B.mn - B.v) * (B.fmin - B.fw);
    double p = (B.mn - B.v) * q - (B.mn - B.w) * rr;
    q = 2.0 * (q - rr);
    if (q > 0.0) p = -p;
    q = fabs(q);
    const double temp = B.delta;
    B.delta = B.d;
    if (fabs(p) >= fabs(0.5 * q * temp) || p <= q * (B.a - B.mn) || p >= q * (B.c - B.mn)) {
      B.delta = B.mn >= middle ? B.a - B.mn : B.c - B.mn;
      B.d = 0.38196601 * B.delta;
    } else {
      B.d = p / q;
      const double u = B.mn + B.d;
      if (u - B.a < tol2 || B.c - u < tol2) B.d = d_sign(tol1, middle - B.mn);
    }
  } else {
    B.delta = B.mn >= middle ? B.a - B.mn : B.c - B.mn;
    B.d = 0.38196601 * B.delta;
  }
  B.x = fabs(B.d) >= tol1 ? B.mn + B.d : B.mn + d_sign(tol1, B.d);
  return true;
}
