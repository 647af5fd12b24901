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

// ---------------------------------------------------------------------------
// np.exp / np.log for float64 as the reference's numpy computes them.  numpy
// 2.2 on an x86 host with AVX512_SKX (the image's numpy 2.2.6; SkylakeX and
// later, Zen 4 and later) evaluates contiguous float64 exp / log with SVML's
// __svml_exp8_ha / __svml_log8_ha (the loops DOUBLE_exp_AVX512_SKX /
// DOUBLE_log_AVX512_SKX call), whose results differ from a correctly rounded
// exp in ~4.6 % of arguments by one ulp -- enough to flip soft VI's argmax at
// exact-tie states.  Restated here operation for operation (same constants,
// same fma / rounding sequence); pinned bit for bit against np.exp / np.log on
// 10^7 arguments (tests/golden/npmath.npz, tools/gen_npmath.py; DESIGN.md §2
// "numpy's exp and log").  The range SVML hands to its scalar rare path (exp:
// |x| >= 707.7, NaN; log: x <= 0, inf, NaN) uses ocml, which agrees with it
// except in the last bit of some results below 1e-307 or above 1e307.
// ---------------------------------------------------------------------------
// The tables (kernels with a hot soft-VI loop stage them in LDS,
// np_stage_tables, and pass that copy: a divergent table read is then an LDS
// read instead of a global one on the sweep's dependency chain).  d[]:
//   [0, 16)  exp: 2^(j/16) as a double       [16, 32) exp: its rounding error
//   [32, 48) log: -log(R) high part          [48, 64) log: -log(R) low part
// for the 5-bit reciprocal R of the mantissa, indexed by R's top four mantissa
// bits (R < 0.75 folds a factor 2 into the exponent).
struct NpTables {
  double d[64];
  // log's reciprocal: bucket u >> 8 of the 16-bit mantissa prefix u holds
  // (#thresholds below the bucket) | (offset of the one threshold inside it,
  // or 256) << 8 -- the same function as the 16 compares (tests/test_npmath.py)
  unsigned rcp[256];
};
static __constant__ NpTables kNpTabs = {{
    0x1.0000000000000p+0, 0x1.0b5586cf9890fp+0, 0x1.172b83c7d517bp+0, 0x1.2387a6e756238p+0,
    0x1.306fe0a31b715p+0, 0x1.3dea64c123422p+0, 0x1.4bfdad5362a27p+0, 0x1.5ab07dd485429p+0,
    0x1.6a09e667f3bcdp+0, 0x1.7a11473eb0187p+0, 0x1.8ace5422aa0dbp+0, 0x1.9c49182a3f090p+0,
    0x1.ae89f995ad3adp+0, 0x1.c199bdd85529cp+0, 0x1.d5818dcfba487p+0, 0x1.ea4afa2a490dap+0,
    0x0.0p+0, 0x1.79aa65d837b6dp-54, -0x1.01b15eaa59348p-55, 0x1.68efde3a8a894p-54,
    0x1.34d754db0abb6p-55, 0x1.59f48a72a4c6dp-55, 0x1.690cebb7aafb0p-56, 0x1.063e1e21c5409p-54,
    -0x1.3b3efbf5e2228p-54, -0x1.b32dcb94da51dp-56, 0x1.db72fc1f0eab4p-55, 0x1.1affc2b91ce27p-56,
    0x1.c1a7792cb3387p-55, 0x1.36eae30af0cb3p-56, 0x1.4a385a63d07a7p-56, -0x1.ff7128fd391f0p-55,
    0x0.0p+0, -0x1.f0a30c0120000p-5, -0x1.e27076e2b0000p-4, -0x1.5ff3070a78000p-3,
    -0x1.c8ff7c79a8000p-3, -0x1.1675cababc000p-2, -0x1.4618bc21c4000p-2, -0x1.739d7f6bbc000p-2,
    0x1.269621134c000p-2, 0x1.f991c6cb38000p-3, 0x1.a93ed3c8b0000p-3, 0x1.5bf406b540000p-3,
    0x1.1178e82280000p-3, 0x1.9335e5d590000p-4, 0x1.08598b59e0000p-4, 0x1.0415d89e80000p-5,
    0x0.0p+0, 0x1.3ab33d066d1d2p-42, 0x1.a342c2af0003cp-45, -0x1.3d3c873e20a07p-43,
    -0x1.a21ac25d81ef3p-43, 0x1.9f1fc63382a8fp-42, -0x1.ec27d0b7b37b3p-42, -0x1.0069ce24c53fbp-42,
    0x1.b92783beb7677p-42, 0x1.9bcbecca0cdf3p-42, -0x1.30e486a0ac42dp-42, 0x1.ed8fdc149767ep-42,
    -0x1.b8421cc74be04p-43, 0x1.2622b8757a8fbp-42, 0x1.d034451fecdfbp-43, -0x1.77771fd187145p-42},
   {
    0x10000u, 0x10000u, 0x10000u, 0x10000u, 0x00f00u, 0x10001u, 0x10001u, 0x10001u, 0x10001u, 0x10001u, 0x10001u, 0x10001u, 0x09701u, 0x10002u, 0x10002u, 0x10002u,
    0x10002u, 0x10002u, 0x10002u, 0x10002u, 0x10002u, 0x0b402u, 0x10003u, 0x10003u, 0x10003u, 0x10003u, 0x10003u, 0x10003u, 0x10003u, 0x10003u, 0x10003u, 0x07003u,
    0x10004u, 0x10004u, 0x10004u, 0x10004u, 0x10004u, 0x10004u, 0x10004u, 0x10004u, 0x10004u, 0x0e604u, 0x10005u, 0x10005u, 0x10005u, 0x10005u, 0x10005u, 0x10005u,
    0x10005u, 0x10005u, 0x10005u, 0x10005u, 0x10005u, 0x02305u, 0x10006u, 0x10006u, 0x10006u, 0x10006u, 0x10006u, 0x10006u, 0x10006u, 0x10006u, 0x10006u, 0x10006u,
    0x10006u, 0x04306u, 0x10007u, 0x10007u, 0x10007u, 0x10007u, 0x10007u, 0x10007u, 0x10007u, 0x10007u, 0x10007u, 0x10007u, 0x10007u, 0x10007u, 0x05f07u, 0x10008u,
    0x10008u, 0x10008u, 0x10008u, 0x10008u, 0x10008u, 0x10008u, 0x10008u, 0x10008u, 0x10008u, 0x10008u, 0x10008u, 0x10008u, 0x09908u, 0x10009u, 0x10009u, 0x10009u,
    0x10009u, 0x10009u, 0x10009u, 0x10009u, 0x10009u, 0x10009u, 0x10009u, 0x10009u, 0x10009u, 0x10009u, 0x10009u, 0x10009u, 0x01509u, 0x1000au, 0x1000au, 0x1000au,
    0x1000au, 0x1000au, 0x1000au, 0x1000au, 0x1000au, 0x1000au, 0x1000au, 0x1000au, 0x1000au, 0x1000au, 0x1000au, 0x1000au, 0x1000au, 0x0070au, 0x1000bu, 0x1000bu,
    0x1000bu, 0x1000bu, 0x1000bu, 0x1000bu, 0x1000bu, 0x1000bu, 0x1000bu, 0x1000bu, 0x1000bu, 0x1000bu, 0x1000bu, 0x1000bu, 0x1000bu, 0x1000bu, 0x1000bu, 0x09c0bu,
    0x1000cu, 0x1000cu, 0x1000cu, 0x1000cu, 0x1000cu, 0x1000cu, 0x1000cu, 0x1000cu, 0x1000cu, 0x1000cu, 0x1000cu, 0x1000cu, 0x1000cu, 0x1000cu, 0x1000cu, 0x1000cu,
    0x1000cu, 0x1000cu, 0x1000cu, 0x1000cu, 0x01a0cu, 0x1000du, 0x1000du, 0x1000du, 0x1000du, 0x1000du, 0x1000du, 0x1000du, 0x1000du, 0x1000du, 0x1000du, 0x1000du,
    0x1000du, 0x1000du, 0x1000du, 0x1000du, 0x1000du, 0x1000du, 0x1000du, 0x1000du, 0x1000du, 0x1000du, 0x0d00du, 0x1000eu, 0x1000eu, 0x1000eu, 0x1000eu, 0x1000eu,
    0x1000eu, 0x1000eu, 0x1000eu, 0x1000eu, 0x1000eu, 0x1000eu, 0x1000eu, 0x1000eu, 0x1000eu, 0x1000eu, 0x1000eu, 0x1000eu, 0x1000eu, 0x1000eu, 0x1000eu, 0x1000eu,
    0x1000eu, 0x1000eu, 0x1000eu, 0x1000eu, 0x01c0eu, 0x1000fu, 0x1000fu, 0x1000fu, 0x1000fu, 0x1000fu, 0x1000fu, 0x1000fu, 0x1000fu, 0x1000fu, 0x1000fu, 0x1000fu,
    0x1000fu, 0x1000fu, 0x1000fu, 0x1000fu, 0x1000fu, 0x1000fu, 0x1000fu, 0x1000fu, 0x1000fu, 0x1000fu, 0x1000fu, 0x1000fu, 0x1000fu, 0x1000fu, 0x1000fu, 0x1000fu,
    0x0800fu, 0x10010u, 0x10010u, 0x10010u, 0x10010u, 0x10010u, 0x10010u, 0x10010u, 0x10010u, 0x10010u, 0x10010u, 0x10010u, 0x10010u, 0x10010u, 0x10010u, 0x10010u,
   }};

// Copy the tables into the workgroup's LDS copy `t` (the caller synchronises
// before the first use).
__device__ inline void np_stage_tables(NpTables* t) {
  for (int i = threadIdx.x; i < 64; i += blockDim.x) t->d[i] = kNpTabs.d[i];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) t->rcp[i] = kNpTabs.rcp[i];
}

__device__ inline double np_exp(double x, const NpTables* tt = &kNpTabs) {
  const double* t = tt->d;
  if (!(fabs(x) < 0x1.61da04cbafe44p+9)) {  // SVML's rare path
    if (x <= -746.0) return 0.0;            // underflow (-inf: soft VI's first softmax of a non-terminal state)
    if (x >= 710.0) return (double)INFINITY;
    return exp(x);                          // NaN, and the subnormal / near-overflow results
  }
  // xs = x / ln2 + shifter rounded toward zero to a multiple of 1/16 (SVML's
  // {rz-sae} fma): the round-to-nearest fma, stepped down one grid point when
  // it rounded up (the sign of the exact residual x / ln2 - N decides).
  constexpr double kShift = 0x1.8000000003ff0p+48, kInvLn2 = 0x1.71547652b82fep+0;
  double xs = __fma_rn(x, kInvLn2, kShift);
  if (__fma_rn(x, kInvLn2, kShift - xs) < 0.0) xs -= 0x1p-4;
  const double n = xs - kShift;  // k / 16, exact
  const int j = (int)(__double_as_longlong(xs) & 15);
  const double t0 = t[j], t1 = t[16 + j];
  double r = __fma_rn(-n, 0x1.62e42fefa39efp-1, x);
  r = __fma_rn(-0x1.abc9e3b39803fp-56, n, r);
  const double r2 = __dmul_rn(r, r);
  const double a = __fma_rn(r, 0x1.7411836940c04p-10, 0x1.1101cbbc265c0p-7);
  const double b = __fma_rn(r, 0x1.55557242d68fep-5, 0x1.5555553939732p-3);
  const double c = __fma_rn(r, 0x1.000000000d008p-1, 0x1.fffffffffff70p-1);
  double p = __fma_rn(r2, a, b);
  p = __fma_rn(r2, p, c);
  double q = __fma_rn(p, r, t1);
  q = __fma_rn(t0, q, t0);
  return ldexp(q, (int)floor(n));
}

// `bucket`: count the reciprocal's thresholds with one read of the 256-bucket
// table in LDS (shortest dependency chain: the single-instance grid shape and
// the numpy-order kernels) or with 16 compares (the default: no extra table
// access; grids with several states per thread, where
// the measured soft VI at 64 instances ran 46 ms with compares, 55 with the
// bucket read; tools/diag/soft_ab.py).  Same result either way.
__device__ inline double np_log(double x, const NpTables* tt = &kNpTabs, bool bucket = false) {
  const double* t = tt->d;
  if (!(x > 0.0) || isinf(x)) return log(x);  // rare path: 0, negative, inf, NaN
  int e;
  const double m = ldexp(frexp(x, &e), 1);  // [1, 2): getmant; e - 1 = getexp
  double E = (double)(e - 1);
  // R = round-to-1/32(rcp14(m)).  rcp14 reads the top 16 mantissa bits u; the
  // rounded result falls by 1/32 at each of these u (measured exhaustively over
  // all 65,536 u on an AVX-512 host: tools/gen_npmath.py).  Summed as a tree
  // (independent compares, three levels of adds): it is on the dependency chain.
  const unsigned u = (unsigned)(__double_as_longlong(m) >> 36) & 0xffffu;
  int nd;
  if (bucket) {
    const unsigned be = tt->rcp[u >> 8];
    nd = (int)(be & 0xffu) + ((u & 0xffu) >= (be >> 8) ? 1 : 0);
  } else {
    const int n0 = ((u >= 1039u) + (u >= 3223u)) + ((u >= 5556u) + (u >= 8048u));
    const int n1 = ((u >= 10726u) + (u >= 13603u)) + ((u >= 16707u) + (u >= 20063u));
    const int n2 = ((u >= 23705u) + (u >= 27669u)) + ((u >= 32007u) + (u >= 36764u));
    const int n3 = ((u >= 42010u) + (u >= 47824u)) + ((u >= 54300u) + (u >= 61568u));
    nd = (n0 + n1) + (n2 + n3);
  }
  const int idx = (16 - nd) & 15;
  const double th = t[32 + idx], tl = t[48 + idx];
  const double R = (double)(32 - nd) * 0x1p-5;
  const double r = __fma_rn(R, m, -1.0);
  if (nd > 8) E += 1.0;
  const double p1 = __fma_rn(r, 0x1.249229cee81efp-3, -0x1.55553fb28db06p-3);
  double p2 = __fma_rn(r, 0x1.c81cd309d7c70p-4, -0x1.007357e93af62p-3);
  const double r2 = __dmul_rn(r, r);
  double p3 = __fma_rn(r, 0x1.9999999cc9f5cp-3, -0x1.00000000c05bdp-2);
  p2 = __fma_rn(r2, p2, p1);
  const double r4 = __dmul_rn(r2, r2);
  const double p4 = __fma_rn(r, 0x1.5555555555466p-2, -0x1.fffffffffffc6p-2);
  p3 = __fma_rn(r2, p3, p4);
  const double hi = __fma_rn(E, 0x1.62e42fefa0000p-1, th);
  p2 = __fma_rn(r4, p2, p3);
  const double s = __dadd_rn(hi, r);
  const double rl = __dsub_rn(r, __dsub_rn(s, hi));
  p2 = __fma_rn(r2, p2, rl);
  const double lo = __fma_rn(0x1.cf79abc9e0000p-40, E, tl);
  return __dadd_rn(s, __dadd_rn(p2, lo));
}

// maxent.py:260-276 -- max + log(1 + exp(min - max)) with numpy's exp / log;
// the log(1+exp) form (not log1p) is kept deliberately so rounding follows
// the reference.
__device__ inline double softmax2(double x1, double x2, const NpTables* t = &kNpTabs, bool bucket = false) {
  const double hi = np_maximum(x1, x2);
  const double lo = np_minimum(x1, x2);
  return __dadd_rn(hi, np_log(__dadd_rn(1.0, np_exp(__dsub_rn(lo, hi), t)), t, bucket));
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
