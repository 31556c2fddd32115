// tools/fp64_peak.hip -- measures the MI355X FP64 vector issue rate (mul, add, fma) that bounds k_brent.
// 8 independent dependency chains per lane, enough waves to fill every SIMD; reports ops/s
// (a mul or add = 1 op, an fma = 2 flops).  Build: hipcc -O3 --offload-arch=gfx950 -o fp64_peak fp64_peak.hip
#include <hip/hip_runtime.h>
#include <cstdio>

template <int KIND>
__global__ void __launch_bounds__(256) k_peak(double* out, int iters, double a, double b) {
  double x[8];
#pragma unroll
  for (int i = 0; i < 8; i++) x[i] = threadIdx.x * 1e-3 + i;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int r = 0; r < 16; r++)
#pragma unroll
      for (int i = 0; i < 8; i++) {
        if (KIND == 0) x[i] = x[i] * a;
        else if (KIND == 1) x[i] = x[i] + b;
        else x[i] = fma(x[i], a, b);
      }
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s += x[i];
  if (s == 1234.5) out[threadIdx.x] = s;
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  double* d;
  hipMalloc(&d, 4096);
  const int blocks = p.multiProcessorCount * 8, iters = 4096;
  const double ops = (double)blocks * 256 * iters * 16 * 8;
  const char* names[3] = {"v_mul_f64", "v_add_f64", "v_fma_f64"};
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  printf("{\"device\": \"%s\", \"cus\": %d", p.name, p.multiProcessorCount);
  for (int k = 0; k < 3; k++) {
    auto fn = k == 0 ? k_peak<0> : k == 1 ? k_peak<1> : k_peak<2>;
    hipLaunchKernelGGL(fn, dim3(blocks), dim3(256), 0, 0, d, 16, 1.0000001, 1e-9);
    hipEventRecord(e0);
    hipLaunchKernelGGL(fn, dim3(blocks), dim3(256), 0, 0, d, iters, 1.0000001, 1e-9);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    printf(", \"%s_Tops\": %.2f", names[k], ops / (ms * 1e-3) / 1e12);
  }
  printf("}\n");
  return 0;
}
