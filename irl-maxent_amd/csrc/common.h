// Shared device helpers for the irlmx HIP kernels (gfx950 / CDNA4, wave64).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include "../../include/irlmx.h"

namespace irlmx {

constexpr int kWave = 64;
constexpr int kStencilK = 5;  // self, +x, -x, +y, -y

void count_event(int which);  // irlmx_counters (capi.hip): IRLMX_CTR_*
// An exchange timed out and the call is rerun per sweep (capi.hip): the first
// time in a process a line on stderr, so a lost or mistagged granule does not
// pass silently as a slow success (the counter records every one).
void note_exchange_timeout(const char* shape);

// Direction k of the 5-point stencil, in the reference's action order
// (gridworld.py:47: (1,0), (-1,0), (0,1), (0,-1)); k = 0 is "stay".
__host__ __device__ inline int stencil_opposite(int k) {
  return k == 0 ? 0 : (k == 1 ? 2 : (k == 2 ? 1 : (k == 3 ? 4 : 3)));
}

// Neighbour of state s in direction k on a width x height grid (state = y*width + x).
// Off-grid neighbours map to s itself; their table weight is always zero.
__device__ inline int stencil_nbr(int s, int k, int width, int height) {
  const int x = s % width;
  const int y = s / width;
  switch (k) {
    case 1: return x + 1 < width ? s + 1 : s;
    case 2: return x > 0 ? s - 1 : s;
    case 3: return y + 1 < height ? s + width : s;
    case 4: return y > 0 ? s - width : s;
    default: return s;
  }
}

__device__ inline bool stencil_valid(int s, int k, int width, int height) {
  const int x = s % width;
  const int y = s / width;
  switch (k) {
    case 1: return x + 1 < width;
    case 2: return x > 0;
    case 3: return y + 1 < height;
    case 4: return y > 0;
    default: return true;
  }
}

// |x| as ordered bits: for non-negative doubles (and +NaN, produced by fabs)
// the unsigned 64-bit order equals the numeric order, and a NaN compares above
// +inf.  So an integer max over these bits is a NaN-propagating max, the
// semantics of np.max(np.abs(...)) that the reference's loops test against.
__device__ inline unsigned long long abs_bits(double x) {
  return (unsigned long long)__double_as_longlong(fabs(x));
}

#define kNaN (__longlong_as_double(0x7ff8000000000000LL))

__device__ inline double bits_double(unsigned long long u) {
  return __longlong_as_double((long long)u);
}

__device__ inline unsigned long long wave_max_u64(unsigned long long v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const unsigned long long o = __shfl_xor(v, off, kWave);
    v = o > v ? o : v;
  }
  return v;
}

// np.maximum / np.minimum: NaN-propagating elementwise max/min.
__device__ inline double np_maximum(double a, double b) {
  return (a != a || b != b) ? (a + b) : (a > b ? a : b);
}
__device__ inline double np_minimum(double a, double b) {
  return (a != a || b != b) ? (a + b) : (a < b ? a : b);
}

// maxent.py:260-276 -- max + log(1 + exp(min - max)); the log(1+exp) form
// (not log1p) is kept deliberately so rounding follows the reference.
__device__ inline double softmax2(double x1, double x2) {
  const double hi = np_maximum(x1, x2);
  const double lo = np_minimum(x1, x2);
  return hi + log(1.0 + exp(lo - hi));
}

// ---------------------------------------------------------------------------
// Device bounds checks (IRLMX_DEVICE_CHECKS=1 builds):
// IRLMX_DCHECK(cond, bit) records a failed check in this translation unit's
// device word and lets the caller skip the access instead of faulting the GPU;
// irlmx_device_check_failures() (capi.hip) syncs the device and returns (and
// clears) the OR of every translation unit's word.  Off by default: the macro
// is then constant-true and compiles away.
// ---------------------------------------------------------------------------
#ifndef IRLMX_DEVICE_CHECKS
#define IRLMX_DEVICE_CHECKS 0
#endif
constexpr unsigned kCheckIndex = 1;    // ELL row / column slot index outside [0, S)
constexpr unsigned kCheckGranule = 2;  // granule offset outside its buffer
constexpr unsigned kCheckTile = 4;     // tile row range / extended tile outside the grid or the LDS buffer

using DcheckTake = unsigned (*)();
bool register_dcheck(DcheckTake take);  // capi.hip

#if IRLMX_DEVICE_CHECKS
static __device__ unsigned g_dcheck;
__device__ inline bool dcheck(bool ok, unsigned bit) {
  if (!ok) atomicOr(&g_dcheck, bit);
  return ok;
}
static unsigned dcheck_take() {
  unsigned v = 0, z = 0;
  if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_dcheck), sizeof(v)) != hipSuccess) return ~0u;
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_dcheck), &z, sizeof(z)) != hipSuccess) return ~0u;
  return v;
}
static const bool g_dcheck_registered = register_dcheck(dcheck_take);
#define IRLMX_DCHECK(cond, bit) (::irlmx::dcheck((cond), (bit)))
#else
#define IRLMX_DCHECK(cond, bit) true
#endif

// Power-of-two exponent that brings the positive finite m into [0.5, 1).
__device__ inline int rescale_exponent(double m) {
  if (!(m > 0.0) || !isfinite(m)) return 0;
  int e;
  frexp(m, &e);
  return -e;
}

}  // namespace irlmx
