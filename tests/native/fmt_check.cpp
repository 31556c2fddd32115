// fmt_check.cpp -- TEST INFRASTRUCTURE: host/vcf_fmt.h against glibc printf on random and edge values.
#include <cstdio>
#include <cstring>
#include <random>
#include "../../polymutt_amd/host/vcf_fmt.h"

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 2000000;
  std::mt19937_64 rng(12345);
  std::uniform_real_distribution<double> u(0.0, 2.0);
  long bad = 0;
  char ref[128];
  auto check = [&](double v, int prec) {
    std::string s;
    pmhost::fmt_fixed(s, v, prec);
    snprintf(ref, sizeof(ref), "%.*f", prec, v);
    if (s != ref) { if (bad < 10) printf("MISMATCH %.17g prec %d: %s vs %s\n", v, prec, s.c_str(), ref); bad++; }
    if (prec == 2) {   // the raw-pointer fast path of the genotype columns (put_fixed2)
      char buf[128], *o = buf;
      pmhost::put_fixed2(o, v);
      *o = 0;
      if (strcmp(buf, ref) != 0) { if (bad < 10) printf("MISMATCH put_fixed2 %.17g: %s vs %s\n", v, buf, ref); bad++; }
    }
  };
  for (int k = -2000; k <= 2000; k++)   // exact decimal ties and their neighbours
    for (int prec = 0; prec <= 4; prec++) {
      const double t = (k + 0.5) / 100.0;
      check(t, prec); check(std::nextafter(t, 0.0), prec); check(std::nextafter(t, 10.0), prec);
      check(k * 0.125, prec); check(k / 8.0 + 1.0 / 1024, prec);
    }
  const double edge[] = {0.0, -0.0, 1e-300, -1e-300, 0.005, 0.015, 0.025, 0.125, 0.375, 1.005, 1.995, 1.999999, 2.0, -0.004, 5e-324, 123456.789};
  for (double v : edge)
    for (int prec = 0; prec <= 6; prec++) check(v, prec);
  for (long i = 0; i < n; i++) {
    double v = u(rng);
    if (i % 3 == 0) v = std::round(v * 1000) / 1000;   // values near 3-decimal grid points
    check(v, 2);
    if (i % 7 == 0) check(-v, 2);
  }
  std::uniform_real_distribution<double> wide(0.0, 2e6);
  for (long i = 0; i < n / 4; i++) check(wide(rng), 2);   // (both sides of put_fixed2's fast-path range)
  std::string s;
  for (long v : {0L, 7L, 10L, 255L, 16777215L, -1L, -123456L}) { s.clear(); pmhost::fmt_int(s, v); snprintf(ref, sizeof(ref), "%ld", v); if (s != ref) bad++; }
  for (long v : {0L, 7L, 10L, 99L, 100L, 255L, 16777215L, -1L, -123456L, 2147483647L}) {
    char buf[32], *o = buf;
    pmhost::put_int(o, (int32_t)v);
    *o = 0;
    snprintf(ref, sizeof(ref), "%ld", v);
    if (strcmp(buf, ref) != 0) bad++;
  }
  printf("%s %ld mismatches\n", bad ? "FAIL" : "OK", bad);
  return bad ? 1 : 0;
}
