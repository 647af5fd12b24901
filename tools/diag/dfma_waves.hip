// Microbenchmark: fp64 FMA issue with one vs two waves per SIMD.
// Each thread runs NCH independent FMA chains, 5 FMAs per chain per iteration
// (the backward stencil's 5 FMAs per state), optionally 16 DPP moves and a
// workgroup barrier per iteration (the cluster kernel's sweep).  One workgroup
// of NT threads per CU (256 CUs).  Prints shader cycles per iteration from
// s_memtime, measured on every workgroup, median.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>
template <int NT, int NCH, int DPP, int BAR>
__global__ void __launch_bounds__(NT) k(double* out, unsigned long long* cyc, int iters) {
  double a[NCH], w = 1.0000001;
  for (int j = 0; j < NCH; ++j) a[j] = threadIdx.x * 1e-3 + j;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 5; ++r)
#pragma unroll
      for (int j = 0; j < NCH; ++j) a[j] = fma(a[j], w, 1e-9);
    if (DPP) {
#pragma unroll
      for (int j = 0; j < DPP / 2; ++j) {
        long long b = __double_as_longlong(a[j % NCH]);
        int lo = __builtin_amdgcn_update_dpp(0, (int)b, 0x138, 0xF, 0xF, true);
        int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0x130, 0xF, 0xF, true);
        a[j % NCH] = fma(__longlong_as_double(((long long)hi << 32) | (unsigned)lo), 1e-30, a[j % NCH]);
      }
    }
    if (BAR) __syncthreads();
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double s = 0;
  for (int j = 0; j < NCH; ++j) s += a[j];
  out[blockIdx.x * NT + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
template <int NT, int NCH, int DPP, int BAR>
void run(double* d, unsigned long long* c, const char* name) {
  const int iters = 20000;
  hipLaunchKernelGGL((k<NT, NCH, DPP, BAR>), 256, NT, 0, 0, d, c, 100);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL((k<NT, NCH, DPP, BAR>), 256, NT, 0, 0, d, c, iters);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> h(256);
  hipMemcpy(h.data(), c, 256 * 8, hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.end());
  const double cyc = (double)h[128] / iters;
  const double fma_per_simd = (double)(NT / 64 / 4) * NCH * 5;  // wave-FMAs per SIMD per iteration
  printf("%-34s %7.3f ms  %7.1f s_memtime cycles/iter  %5.2f cycles per wave-FMA per SIMD  (%.1f TFLOP/s)\n", name,
         ms, cyc, cyc / (fma_per_simd + (DPP ? (double)(NT / 256) * DPP / 2 : 0.0)),
         256.0 * NT * NCH * 5 * 2 * iters / (ms * 1e-3) / 1e12);
}
int main() {
  double* d; unsigned long long* c;
  hipMalloc(&d, 256 * 1024 * 8); hipMalloc(&c, 256 * 8);
  run<512, 12, 0, 0>(d, c, "2 waves/SIMD, 12 chains");
  run<256, 12, 0, 0>(d, c, "1 wave/SIMD, 12 chains");
  run<256, 24, 0, 0>(d, c, "1 wave/SIMD, 24 chains");
  run<512, 12, 16, 0>(d, c, "2 waves/SIMD, 12 chains + 16 DPP");
  run<256, 12, 16, 0>(d, c, "1 wave/SIMD, 12 chains + 16 DPP");
  run<512, 12, 16, 1>(d, c, "2 w/SIMD, 12 ch + 16 DPP + barrier");
  run<256, 12, 16, 1>(d, c, "1 w/SIMD, 12 ch + 16 DPP + barrier");
  run<256, 24, 32, 1>(d, c, "1 w/SIMD, 24 ch + 32 DPP + barrier");
  return 0;
}
