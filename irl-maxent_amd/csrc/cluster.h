// Persistent temporally blocked stencil kernels (cluster.hip): shared declarations.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"

namespace irlmx {

constexpr int kCT = 1024;    // threads per cluster workgroup
constexpr int kPairThreads = 512;  // threads per workgroup of the pair layout
constexpr int kSptMaxPair = 12;    // states per thread of the pair layout
constexpr int kTMax = 16;    // max sweeps per block (= max ghost rows)
constexpr int kSptMax = 6;   // states per thread -> extended tile <= 6144 states (no VGPR spills)
constexpr int kStripThreads = 512;  // strip kernel workgroup (2 waves per SIMD, 256 VGPRs)
constexpr int kModeFwd = 0;
constexpr int kModeBwd = 1;

struct ClusterArgs {
  int W, H, S, A;
  int R, G, C, T;          // rows per tile, ghost rows, tiles per instance, max sweeps per block
  int b0;                  // first instance of this launch
  int btot;                // instances in pub / slots / counter arrays
  int emax;                // LDS buffer length (states)
  int tab_shared;          // backward tables shared by all instances
  const double* wgt;       // forward: [B][5][S] gather weights; backward: [B'][5][S] collapsed
  const double* row_val;   // backward final sweep: [B'][A][5][S]
  const double* vin;       // forward: p0 [B][S]; backward: reward [B][S]
  const uint8_t* term;     // backward: terminal mask [B][S]
  const int32_t* bad;      // forward: non-finite policy flags [B]
  const unsigned long long* growth;  // backward: per-instance growth bound bits [B]
  double eps;
  long long max_iter;
  long long n_sweeps;      // backward: collapsed sweeps (2S - 1)
  int rescale;
  double* pub;             // [2][B][S]
  unsigned long long* slots;  // [B][3][kTMax]
  unsigned int* counter;   // [B]
  int* err;                // [1] barrier timeout
  unsigned long long* stamps;  // optional [grid][8] phase cycle counters (IRLMX_STAMPS=1), else null
  double* out;             // forward: svf [B][S]; backward: pi [B][S][A]
  int64_t* iters;
  int32_t* status;
};

struct ClusterPlan {
  int R, G, C, T, per_launch, spt, emax;
  size_t lds;
  int strip, cpl, rpt;  // strip kernel (strip.hip) shape; strip == 0: LDS kernel
  bool pair;            // LDS kernel with the pair layout (widths 64 / 128)
};

size_t strip_lds(int W, int emax, int nt);
template <int MODE>
void* strip_fn(int cpl, int rpt);

__device__ inline unsigned int ld_sc1(unsigned int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void st_sc1(double* p, double v) {  // write-through (sc1) 8-byte store
  __hip_atomic_store((unsigned long long*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline double ld_sc1(const double* p) {  // L1-bypassing (sc1) 8-byte load
  return __longlong_as_double((long long)__hip_atomic_load((unsigned long long*)p, __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT));
}

// Arrival barrier of the C tiles of one instance, in the fence-free form of
// MI355X_MICROARCH.md "Valid forms" (row 1): every payload byte is stored
// write-through (sc1) and loaded with sc1 loads, every storing wave drains
// (s_waitcnt vmcnt(0)) before the workgroup barrier, then ONE lane adds to the
// instance's arrival counter (agent scope) and polls it with sc1 loads; the
// other waves load after the workgroup barrier that lane joins.  Bounded by a
// 20 s wall-clock timeout; returns false on timeout (error word set).
__device__ inline bool instance_barrier(unsigned int* counter, unsigned int target, int* err, int* lds_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    int abort = 0;
    __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
    while (ld_sc1(counter) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > 2000000000ull) {
        abort = 1;
        atomicOr(err, 1);
        break;
      }
    }
    *lds_flag = abort;
  }
  __syncthreads();
  return *lds_flag == 0;
}

__device__ inline unsigned long long stamp_now() { return __builtin_amdgcn_s_memtime(); }

// OR of a 32-bit value over the wave (one ballot per bit that may be set).
__device__ inline unsigned wave_or_bits(unsigned v, int nbits) {
  unsigned out = 0;
  for (int b = 0; b < nbits; ++b)
    if (__ballot((v >> b) & 1u)) out |= 1u << b;
  return out;
}

bool cluster_plan(int W, int H, int B, ClusterPlan* out);
int cluster_run(int mode, const ClusterPlan& p, ClusterArgs a, int B, hipStream_t st);
__global__ void bwd_growth_kernel(const double* __restrict__ bw, int tab_shared, const double* __restrict__ reward,
                                  int S, unsigned long long* __restrict__ growth);

}  // namespace irlmx
