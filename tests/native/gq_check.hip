// gq_check -- test infrastructure (tests/test_gpu_gq.py): the product's device GQ (engine_dev.h d_gq, the
// threshold count around a bare-v_log_f32 guess) against the reference's expression evaluated on the host with
// glibc, (pb > 0.9999999999) ? 100 : int(-10 log10(1 - pb) + 0.5) (NucFamGenotypeLikelihood.cpp OutputVCF
// :1818-1820), over every threshold's neighbourhood (+-64 ulps of pb), the near-1 cut-off, tiny and random pb.
// Prints "gq_check: N values, M mismatches" and exits 1 on any mismatch.
#include "engine_dev.h"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

__global__ void k_gq(const double* pb, int n, const double* thr, int* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = d_gq(pb[i], thr);
}

static int ref_gq(double pb) { return pb > 0.9999999999 ? 100 : (int)(-10. * log10(1. - pb) + 0.5); }

int main() {
  double thr[101];   // the engine's thresholds (engine.hip pm_engine_create): bisection over positive bit patterns
  auto gq_of = [](double q) { return (int)(-10. * log10(q) + 0.5); };
  for (int k = 0; k <= 100; k++) {
    uint64_t lo = 1, hi = 0x3FF0000000000000ull;
    while (lo < hi) {
      const uint64_t mid = lo + (hi - lo) / 2;
      double q;
      memcpy(&q, &mid, 8);
      if (gq_of(q) <= k) hi = mid; else lo = mid + 1;
    }
    memcpy(&thr[k], &lo, 8);
  }
  std::vector<double> pb;
  for (int k = 0; k <= 100; k++) {
    double c = 1. - thr[k], lo = c, hi = c;
    pb.push_back(c);
    for (int u = 0; u < 64; u++) {
      lo = nextafter(lo, 0.0);
      hi = nextafter(hi, 2.0);
      pb.push_back(lo);
      if (hi <= 1.0) pb.push_back(hi);
    }
  }
  double c = 0.9999999999, lo = c, hi = c;
  for (int u = 0; u < 256; u++) { pb.push_back(lo); pb.push_back(hi); lo = nextafter(lo, 0.0); hi = nextafter(hi, 2.0); }
  pb.push_back(1.0);
  pb.push_back(0.0);
  for (double x = 1e-300; x < 1; x *= 3.7) pb.push_back(x);
  std::mt19937_64 rng(12345);
  std::uniform_real_distribution<double> U(0.0, 1.0);
  for (int i = 0; i < 1 << 20; i++) {
    const double u = U(rng);
    pb.push_back(i & 1 ? u : 1. - pow(10., -10.5 * u));   // uniform, and uniform in GQ
  }
  const int n = (int)pb.size();
  double *d_pb, *d_thr;
  int* d_out;
  if (hipMalloc(&d_pb, sizeof(double) * n) != hipSuccess || hipMalloc(&d_thr, sizeof(thr)) != hipSuccess ||
      hipMalloc(&d_out, sizeof(int) * n) != hipSuccess) { fprintf(stderr, "gq_check: hipMalloc failed\n"); return 2; }
  (void)hipMemcpy(d_pb, pb.data(), sizeof(double) * n, hipMemcpyHostToDevice);
  (void)hipMemcpy(d_thr, thr, sizeof(thr), hipMemcpyHostToDevice);
  k_gq<<<(n + 255) / 256, 256>>>(d_pb, n, d_thr, d_out);
  std::vector<int> out(n);
  if (hipMemcpy(out.data(), d_out, sizeof(int) * n, hipMemcpyDeviceToHost) != hipSuccess) {
    fprintf(stderr, "gq_check: kernel failed\n");
    return 2;
  }
  int bad = 0;
  for (int i = 0; i < n; i++)
    if (out[i] != ref_gq(pb[i])) {
      if (bad < 10) printf("pb=%.17g device=%d reference=%d\n", pb[i], out[i], ref_gq(pb[i]));
      bad++;
    }
  printf("gq_check: %d values, %d mismatches\n", n, bad);
  (void)hipFree(d_pb); (void)hipFree(d_thr); (void)hipFree(d_out);
  return bad ? 1 : 0;
}
