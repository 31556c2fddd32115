// vcf_fmt.h -- allocation-free text formatting for the per-genotype VCF columns.
//
// OutputVCF (src/NucFamGenotypeLikelihood.cpp:1751-1915) prints every genotype column with fprintf
// ("%s:%d:%d:%.2f:%d,%d,%d"); with thousands of persons per record that is most of the CLI's host time.
// These helpers append the same characters to a buffer: integers in decimal, and fixed-point values
// rounded exactly as glibc's printf does (the exact binary value rounded to `prec` decimals, ties to even).
#pragma once
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <string>

namespace pmhost {

inline void fmt_uint(std::string& out, uint64_t v) {
  char b[24];
  int n = 0;
  do { b[n++] = char('0' + v % 10); v /= 10; } while (v);
  while (n) out.push_back(b[--n]);
}

inline void fmt_int(std::string& out, int64_t v) {
  if (v < 0) { out.push_back('-'); fmt_uint(out, (uint64_t)(-(v + 1)) + 1); }
  else fmt_uint(out, (uint64_t)v);
}

// printf("%.<prec>f", v) for prec in 0..6.  v = m * 2^e exactly (m < 2^53); m * 10^prec * 2^e is split into
// an integer part and an exact remainder with 128-bit arithmetic, then rounded half-to-even.
inline void fmt_fixed(std::string& out, double v, int prec) {
  static const uint64_t kPow10[7] = {1, 10, 100, 1000, 10000, 100000, 1000000};
  if (!std::isfinite(v) || std::fabs(v) >= 1e12 || prec < 0 || prec > 6) {
    char b[64];
    snprintf(b, sizeof(b), "%.*f", prec, v);
    out += b;
    return;
  }
  const bool neg = std::signbit(v);
  const double a = std::fabs(v);
  uint64_t q = 0;
  if (a != 0.0) {
    int e;
    const double fr = std::frexp(a, &e);                       // a = fr * 2^e, fr in [0.5, 1)
    const uint64_t m = (uint64_t)std::ldexp(fr, 53);           // exact: a = m * 2^(e - 53)
    e -= 53;
    const unsigned __int128 scaled = (unsigned __int128)m * kPow10[prec];
    if (e >= 0) q = (uint64_t)(scaled << e);
    else if (-e < 127) {
      const int sh = -e;
      const unsigned __int128 one = 1;
      const unsigned __int128 mask = (one << sh) - 1, half = one << (sh - 1);
      q = (uint64_t)(scaled >> sh);
      const unsigned __int128 rem = scaled & mask;
      if (rem > half || (rem == half && (q & 1))) q++;
    }
  }
  if (neg) out.push_back('-');
  fmt_uint(out, q / kPow10[prec]);
  if (prec) {
    out.push_back('.');
    uint64_t f = q % kPow10[prec];
    char b[8];
    for (int i = prec - 1; i >= 0; i--) { b[i] = char('0' + f % 10); f /= 10; }
    out.append(b, prec);
  }
}

// Raw-pointer variants for the per-genotype columns (the caller reserves the room: at most 20 chars per integer)
inline void put_uint(char*& o, uint32_t v) {
  if (v < 10) { *o++ = char('0' + v); return; }
  if (v < 100) { *o++ = char('0' + v / 10); *o++ = char('0' + v % 10); return; }
  char b[12];
  int n = 0;
  do { b[n++] = char('0' + v % 10); v /= 10; } while (v);
  while (n) *o++ = b[--n];
}
inline void put_int(char*& o, int32_t v) {
  if (v < 0) { *o++ = '-'; put_uint(o, (uint32_t)(-(int64_t)v)); }
  else put_uint(o, (uint32_t)v);
}
inline void put_str(char*& o, const char* s) { while (*s) *o++ = *s++; }

// printf("%.2f", v): the double product v * 100 is within ~1e-14 relative of the exact one, so unless its fraction
// lies within 1e-7 of one half (where the exact binary value decides, ties to even) rounding it gives printf's
// digits; those near-ties, and values outside [0, 1e6), take fmt_fixed's exact path.
inline void put_fixed2(char*& o, double v) {
  if (!std::signbit(v) && v < 1e6) {   // (-0.0 prints "-0.00"; q < 1e8: its rounding error < 2.3e-8, below the margin)
    const double q = v * 100.0, fl = std::floor(q), fr = q - fl;
    if (std::fabs(fr - 0.5) > 1e-7) {
      const uint64_t r = (uint64_t)fl + (fr > 0.5 ? 1 : 0);
      put_uint(o, (uint32_t)(r / 100));
      *o++ = '.';
      const uint32_t c = (uint32_t)(r % 100);
      *o++ = char('0' + c / 10); *o++ = char('0' + c % 10);
      return;
    }
  }
  std::string t;
  fmt_fixed(t, v, 2);
  for (char c : t) *o++ = c;
}

}  // namespace pmhost
