// Microbenchmark: fp64 FMA issue rate per CU (12 independent chains per thread),
// with and without DPP moves and a workgroup barrier per iteration.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int MODE>
__global__ void __launch_bounds__(512) k(double* out, int iters) {
  double a[12], w = 1.0000001;
  for (int j = 0; j < 12; ++j) a[j] = threadIdx.x * 1e-3 + j;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 5; ++r)
#pragma unroll
      for (int j = 0; j < 12; ++j) a[j] = fma(a[j], w, 1e-9);
    if (MODE >= 1) {
#pragma unroll
      for (int j = 0; j < 12; j += 3) {
        long long b = __double_as_longlong(a[j]);
        int lo = __builtin_amdgcn_update_dpp(0, (int)b, 0x138, 0xF, 0xF, true);
        int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0x138, 0xF, 0xF, true);
        a[j] = __longlong_as_double(((long long)hi << 32) | (unsigned)lo) * 0.5 + a[j] * 0.5;
      }
    }
    if (MODE >= 2) __syncthreads();
  }
  double s = 0; for (int j = 0; j < 12; ++j) s += a[j];
  out[blockIdx.x * 512 + threadIdx.x] = s;
}
int main() {
  double* d; hipMalloc(&d, 256 * 512 * 8);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const int iters = 20000;
  for (int mode = 0; mode < 3; ++mode) {
    auto f = mode == 0 ? k<0> : mode == 1 ? k<1> : k<2>;
    hipLaunchKernelGGL(f, 256, 512, 0, 0, d, 100);
    hipEventRecord(e0);
    hipLaunchKernelGGL(f, 256, 512, 0, 0, d, iters);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    double fmas = 256.0 * 512 * iters * 60;
    printf("mode %d: %.3f ms  %.1f DFMA/clk/CU at 2.4 GHz  (%.0f cycles per iteration of 60 FMA/thread)\n", mode, ms,
           fmas / 256 / (ms * 1e-3 * 2.4e9), ms * 1e-3 * 2.4e9 / iters);
  }
  return 0;
}
