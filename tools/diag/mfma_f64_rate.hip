// Microbenchmark: v_mfma_f64_16x16x4_f64 issue rate (register operands, NACC
// independent accumulators per wave, 256 workgroups x W waves), TFLOP/s at the
// clock the chip holds.  Build: hipcc -O3 --offload-arch=gfx950 -o tools/diag/mfma_f64_rate tools/diag/mfma_f64_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double f64x4 __attribute__((ext_vector_type(4)));
template <int NACC>
__global__ void k(double* out, int iters) {
  f64x4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = f64x4{0.0, 0.0, 0.0, 0.0};
  double a = 1.0 + threadIdx.x * 1e-9, b = 1.0 - threadIdx.x * 1e-9;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
template <int NACC>
void run(int waves) {
  double* d;
  hipMalloc(&d, 256 * 1024 * 8);
  const int iters = 20000;
  hipLaunchKernelGGL(k<NACC>, dim3(256), dim3(64 * waves), 0, 0, d, 100);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k<NACC>, dim3(256), dim3(64 * waves), 0, 0, d, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  const double flops = 256.0 * waves * iters * NACC * 16 * 16 * 4 * 2;
  printf("waves/WG %d, accumulators %d: %.3f ms, %.1f TFLOP/s\n", waves, NACC, ms, flops / (ms * 1e-3) / 1e12);
  hipFree(d);
}
int main() {
  run<1>(4); run<4>(4); run<4>(8); run<8>(4); run<8>(8);
  return 0;
}
