// Microbenchmark: fp64 FMA throughput vs independent chains per thread
// (512-thread workgroups, one per CU: 2 waves per SIMD, as the cluster kernel).
#include <hip/hip_runtime.h>
#include <cstdio>
template <int K>
__global__ void __launch_bounds__(512) k(double* out, int iters) {
  double a[K];
  const double w = 1.0000001;
  for (int j = 0; j < K; ++j) a[j] = threadIdx.x * 1e-3 + j;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 60 / K; ++r)
#pragma unroll
      for (int j = 0; j < K; ++j) a[j] = fma(a[j], w, 1e-9);
  }
  double s = 0;
  for (int j = 0; j < K; ++j) s += a[j];
  out[blockIdx.x * 512 + threadIdx.x] = s;
}
template <int K>
static void run(double* d) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int iters = 20000;
  hipLaunchKernelGGL(k<K>, 256, 512, 0, 0, d, 100);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(k<K>, 256, 512, 0, 0, d, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  printf("chains %2d: %.3f ms, %.0f ns per 60 FMA per thread\n", K, ms, ms * 1e6 / iters);
}
int main() {
  double* d;
  (void)hipMalloc(&d, 256 * 512 * 8);
  run<1>(d); run<2>(d); run<3>(d); run<4>(d); run<6>(d); run<12>(d);
  return 0;
}
