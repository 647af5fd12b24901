// Persistent dense shape (IRLMX_SHAPE_DENSE_GRID): the two linear loops of a
// DENSE model in ONE launch, with the matrix rows held in registers for the
// whole loop instead of re-streamed every sweep:
//
//   backward  zs'[s] = exp(r[s]) * (M zs)[s], M = sum_a P_a, 2S - 1 sweeps, then
//             za[s, a] = exp(r[s]) * (P_a zs)[s]; pi = za / sum_a za   (maxent.py:143-159)
//   forward   d'[t] = p0[t] + (WT d)[t] until max|d' - d| <= eps        (maxent.py:98-112)
//
// The per-sweep dense kernels (dense.hip) pay one launch and one full read of
// the S x S matrix per sweep (S = 2048: 33.5 MB, 8.2 us per sweep).  Here every
// workgroup (512 threads, one per CU) owns RB consecutive rows of one
// instance's matrix; thread t keeps columns t, t + 512, ... (CPT of them) of
// each of its RB rows in registers (RB * CPT <= 64 doubles), so the matrix is
// read from HBM once per call.  A sweep is then:
//
//   1. gather the whole swept vector v_k: thread t polls the tagged granules of
//      its CPT columns (cluster.h gran_gather: 16-byte {lo, tag, hi, tag}
//      stores, the data is the flag, one fabric round trip);
//   2. the loop test from the gathered vector itself -- every workgroup holds all
//      of v_k and v_{k-1}, so each computes the same max|v_k - v_{k-1}| (forward)
//      or max|v_k| (backward rescale exponent) locally: no block-maximum
//      exchange and no global barrier;
//   3. RB row dots: FMA chains over the thread's columns, a DPP sum over the
//      wave (lane 63), the 8 wave partials summed in wave order through LDS;
//   4. thread r < RB publishes row r's new value as one granule.
//
// Values live in a ring of two sweeps: a workgroup publishes v_{k+1} only after
// it has gathered all of v_k, i.e. after every workgroup has published v_k and
// hence finished gathering v_{k-1}, the previous occupant of that slot.
//
// The per-state arithmetic is the per-sweep kernels' (the same fma / ldexp /
// __dmul_rn sequence); only the summation order of each row dot differs (thread
// chains of CPT terms, then the wave and workgroup trees), as the GEMM shape's
// does: results agree with the per-sweep shape to rounding, and the loop
// decisions follow the same rules (`while delta > eps` with NaN stopping,
// exactly 2S - 1 collapsed sweeps, bwd_nonfinite_rule).
//
// Co-residency: all workgroups must run at once (they wait on each other's
// granules); the rendezvous (cluster.h coresident) sends the call back to the
// per-sweep shape otherwise, as for the cluster and grid shapes.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>

#include "cluster.h"
#include "dense.h"

namespace irlmx {

void set_error(const char* fmt, ...);
int hip_fail(hipError_t e, const char* what);

namespace {

constexpr int kDG = kDenseGridThreads;
constexpr int kDGWaves = kDG / kWave;

int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return (e && *e) ? atoi(e) : dflt;
}

template <int CTRL, int ROW_MASK>
__device__ inline double dpp_f64(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, ROW_MASK, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, ROW_MASK, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}

// Sum over the wave's 64 lanes, valid in lane 63 (wave_reduce_u32's DPP
// pattern: butterflies inside each row of 16, then row_bcast:15 / :31; lanes
// a row mask disables add the `old` operand 0).  Fixed order: deterministic.
__device__ inline double wave_sum_f64(double v) {
  v += dpp_f64<0xB1, 0xF>(v);   // quad_perm [1,0,3,2]
  v += dpp_f64<0x4E, 0xF>(v);   // quad_perm [2,3,0,1]
  v += dpp_f64<0x141, 0xF>(v);  // row_half_mirror
  v += dpp_f64<0x140, 0xF>(v);  // row_mirror
  v += dpp_f64<0x142, 0xA>(v);  // row_bcast:15 -> rows 1, 3
  v += dpp_f64<0x143, 0xC>(v);  // row_bcast:31 -> rows 2, 3
  return v;
}

// a + b for two 64-lane double vectors after a cross-half exchange
// (v_permlane32_swap / v_permlane16_swap on both 32-bit halves): each lane ends
// up with the sum, over itself and its partner (lane ^ 32 / lane ^ 16), of ONE
// of the two rows -- which one, the lane's `marker` says (probe_swap)
template <int HALF>
__device__ inline double swap_sum(double a, double b) {
  const long long x = __double_as_longlong(a), y = __double_as_longlong(b);
  const unsigned xl = (unsigned)x, xh = (unsigned)(x >> 32), yl = (unsigned)y, yh = (unsigned)(y >> 32);
  auto lo = HALF == 32 ? __builtin_amdgcn_permlane32_swap(xl, yl, false, false)
                       : __builtin_amdgcn_permlane16_swap(xl, yl, false, false);
  auto hi = HALF == 32 ? __builtin_amdgcn_permlane32_swap(xh, yh, false, false)
                       : __builtin_amdgcn_permlane16_swap(xh, yh, false, false);
  const double a2 = __longlong_as_double(((long long)hi[0] << 32) | (long long)lo[0]);
  const double b2 = __longlong_as_double(((long long)hi[1] << 32) | (long long)lo[1]);
  return a2 + b2;
}
// which of the two rows a lane holds after swap_sum<HALF> (0: the first operand's)
template <int HALF>
__device__ inline int probe_swap() {
  auto p = HALF == 32 ? __builtin_amdgcn_permlane32_swap(0u, 1u, false, false)
                      : __builtin_amdgcn_permlane16_swap(0u, 1u, false, false);
  return (int)p[0];
}

// Transposed wave reduction of N row partials (N = 4, 8, 16): every exchange
// level halves the rows a lane carries instead of reducing each row over all
// 64 lanes (N = 8: 34 VALU instructions instead of 144) -- lane ^ 32 and
// lane ^ 16 by permlane swaps (no selects), lane ^ 8 (row_ror:8) and lane ^ 7
// (row_half_mirror) with the kept / sent row chosen by the lane's bit, then
// plain butterflies over the lanes left.  On return v[0] holds the full sum of
// row `row` in every lane of a group of 64 / N consecutive lanes.  Fixed order:
// deterministic.
template <int N>
__device__ inline double rows_sum(double (&v)[N], int lane, int& row) {
  static_assert(N == 4 || N == 8 || N == 16, "rows_sum: 4, 8 or 16 rows");
  const int m32 = probe_swap<32>(), m16 = probe_swap<16>();
#pragma unroll
  for (int i = 0; i < N / 2; ++i) v[i] = swap_sum<32>(v[i], v[i + N / 2]);
#pragma unroll
  for (int i = 0; i < N / 4; ++i) v[i] = swap_sum<16>(v[i], v[i + N / 4]);
  row = m32 * (N / 2) + m16 * (N / 4);
  if constexpr (N >= 8) {  // lane ^ 8: bit 3 picks the row kept
    const bool b3 = (lane >> 3) & 1;
#pragma unroll
    for (int i = 0; i < N / 8; ++i) {
      const double send = b3 ? v[i] : v[i + N / 8], keep = b3 ? v[i + N / 8] : v[i];
      v[i] = keep + dpp_f64<0x128, 0xF>(send);  // row_ror:8
    }
    row += b3 ? N / 8 : 0;
  } else {
    v[0] += dpp_f64<0x128, 0xF>(v[0]);
  }
  if constexpr (N == 16) {  // lane ^ 7 (same bits 3..5): bit 2 picks the row kept
    const bool b2 = (lane >> 2) & 1;
    const double send = b2 ? v[0] : v[1], keep = b2 ? v[1] : v[0];
    v[0] = keep + dpp_f64<0x141, 0xF>(send);  // row_half_mirror
    row += b2 ? 1 : 0;
  } else {
    v[0] += dpp_f64<0x141, 0xF>(v[0]);
  }
  v[0] += dpp_f64<0x4E, 0xF>(v[0]);  // quad_perm [2,3,0,1]
  v[0] += dpp_f64<0xB1, 0xF>(v[0]);  // quad_perm [1,0,3,2]
  return v[0];
}

__device__ inline int dg_finish_status(double delta, double eps) {
  if (delta != delta) return IRLMX_NONFINITE;
  return delta > eps ? IRLMX_MAXITER : IRLMX_OK;
}

}  // namespace

namespace {

// This workgroup's instance and index within it; false for the padding
// workgroups of an XCD-grouped grid.  XCD grouping (as the grid shape):
// workgroups are dealt round-robin over the 8 XCDs, so the workgroups of
// instance g + 8 j all come from XCD group g and its granules stay in one L2.
__device__ inline bool dg_place(const DenseGridArgs& a, int& b, int& blk) {
  int lin = blockIdx.x;
  if (a.xcd_group) {
    const int grp = blockIdx.x % 8, kk = blockIdx.x / 8;
    const int il = grp + 8 * (kk / a.bpi);
    if (il >= a.nb) return false;
    lin = il * a.bpi + kk % a.bpi;
  }
  b = lin / a.bpi;
  blk = lin % a.bpi;
  return true;
}

// Plain stores (kept in the XCD's L2) when every workgroup of the instance runs
// on one XCD -- found by exchanging XCC ids once; -1 when that exchange timed
// out.  `scratch` is a workgroup array of kDGWaves words.
__device__ inline int dg_plain(const DenseGridArgs& a, int b, int blk, unsigned salt,
                               unsigned long long* scratch, int* lflag) {
  if (!a.xcd_group) return 0;
  const int tid = threadIdx.x, wave = tid / kWave, lane = tid & (kWave - 1);
  const Gran rx = gran_rsrc(a.xgran + (size_t)b * 2 * a.bpi, 16u * (unsigned)a.bpi);
  unsigned xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  xcc &= 0xFu;
  const unsigned htag = salt | 0xFFFFFu;
  if (tid == 0) gran_store(rx, (unsigned)blk * 16u, xcc, htag, false);
  unsigned off[1] = {(unsigned)(tid < a.bpi ? tid : 0) * 16u};
  unsigned long long v[1] = {xcc};
  if (!gran_gather<1>(rx, rx, off, tid < a.bpi ? 1u : 0u, htag, v, a.gather_ticks)) *lflag = 1;
  const unsigned long long diff = wave_or_u64(tid < a.bpi ? (v[0] ^ xcc) : 0ull);
  if (lane == 0) scratch[wave] = diff;
  __syncthreads();
  if (*lflag) return -1;
  unsigned long long any = 0ull;
#pragma unroll
  for (int i = 0; i < kDGWaves; ++i) any |= scratch[i];
  __syncthreads();
  return any == 0ull ? 1 : 0;
}

}  // namespace

template <int MODE, int RB, int CPT>
__global__ void __launch_bounds__(kDG) dense_grid_kernel(DenseGridArgs a) {
  const int S = a.S;
  int b, blk;
  if (!dg_place(a, b, blk)) return;  // padding workgroup of an XCD-grouped grid
  const int tid = threadIdx.x;
  const int wave = tid / kWave, lane = tid & (kWave - 1);
  __shared__ int resident, lflag;
  __shared__ double red[2][kDGWaves][RB];  // by sweep parity (see the gather's note)
  __shared__ unsigned long long mred[2][kDGWaves];
  if (tid == 0) {
    resident = coresident(a.err + 1, a.n_resident) ? 1 : 0;
    lflag = 0;
  }
  __syncthreads();
  if (!resident) {
    if (tid == 0) atomicOr(a.err, kErrNotResident);
    return;
  }
  if (b * a.bpi + blk == a.test_drop) return;  // tests: a workgroup that stops publishing (exchange-timeout path)
  const int row0 = blk * RB;
  if (MODE == kModeFwd && a.bad[b]) {  // non-finite policy: the reference's dense product is NaN after one sweep
    if (tid < RB && row0 + tid < S) a.out[(size_t)b * S + row0 + tid] = kNaN;
    if (blk == 0 && tid == 0) { a.iters[b] = 1; a.status[b] = IRLMX_NONFINITE; }
    return;
  }
  // this workgroup's RB rows, columns tid + kDG * j
  const size_t tab = (MODE == kModeFwd || !a.shared) ? (size_t)b : 0;
  const double* mat = a.mat + tab * (size_t)S * S;
  double m[RB][CPT];
#pragma unroll
  for (int r = 0; r < RB; ++r)
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      const int row = row0 + r, c = tid + kDG * j;
      m[r][j] = (row < S && c < S) ? mat[(size_t)row * S + c] : 0.0;
    }
  // the row epilogue's constant (thread r < RB owns row row0 + r): p0 or exp(r)
  double rc = 0.0;
  if (tid < RB && row0 + tid < S) {
    const double x = a.vin[(size_t)b * S + row0 + tid];
    rc = MODE == kModeFwd ? x : exp(x);
  }
  // the swept vector at this thread's columns: forward d_0 = 0; backward zs_0 = 1[terminal]
  double cur[CPT];
  unsigned off0[CPT];
  unsigned want = 0;
#pragma unroll
  for (int j = 0; j < CPT; ++j) {
    const int c = tid + kDG * j;
    off0[j] = (unsigned)(c < S ? c : S - 1) * 16u;
    want |= (c < S ? 1u : 0u) << j;
    cur[j] = (MODE == kModeBwd && c < S && a.term[(size_t)b * S + c]) ? 1.0 : 0.0;  // maxent.py:146-147
  }
  const Gran rg = gran_rsrc(a.gran + (size_t)b * 4 * S, 32u * (unsigned)S);
  const unsigned salt = (a.salt & 0xFFFu) << 20;
  const int pl = dg_plain(a, b, blk, salt, &mred[0][0], &lflag);
  if (pl < 0) {
    if (tid == 0) atomicOr(a.err, 1);
    return;
  }
  const bool plain = pl == 1;
  const long long total = MODE == kModeBwd ? 2LL * S - 1 : -1;  // collapsed sweeps (maxent.py:154)
  double delta = 0.0;
  unsigned long long gmax = 0ull;  // backward: max |zs_k| (ordered bits; inf / NaN above every finite value)
  bool nonfinite = false;
  long long k = 0;  // sweeps done: cur = v_k
  // One workgroup barrier per sweep: the row partials of sweep k + 1 are
  // computed from v_k before the loop test on v_k is known (both go through
  // LDS at the same barrier); when the test stops the loop they are dropped.
  for (;;) {
    // row dots in chunks of up to 16 rows (bounded live registers), each chunk
    // reduced over the wave by rows_sum
    constexpr int CH = RB < 16 ? RB : 16;
#pragma unroll
    for (int r0 = 0; r0 < RB; r0 += CH) {
      double acc[CH];
#pragma unroll
      for (int r = 0; r < CH; ++r) {
        acc[r] = 0.0;
#pragma unroll
        for (int j = 0; j < CPT; ++j) acc[r] = fma(m[r0 + r][j], cur[j], acc[r]);
      }
      int row;
      const double sum = rows_sum<CH>(acc, lane, row);
      if ((lane & (kWave / CH - 1)) == 0) red[k & 1][wave][r0 + row] = sum;
    }
    __syncthreads();
    if (k > 0) {
      if (lflag) {
        if (tid == 0) atomicOr(a.err, 1);
        return;
      }
      unsigned long long mx = 0ull;
#pragma unroll
      for (int i = 0; i < kDGWaves; ++i) mx = mred[k & 1][i] > mx ? mred[k & 1][i] : mx;
      if (MODE == kModeFwd) {
        delta = bits_double(mx);
        if (!(delta > a.eps) || (a.max_iter > 0 && k >= a.max_iter)) break;  // maxent.py:108
      } else {
        gmax = mx;
        nonfinite |= mx >= 0x7FF0000000000000ull;  // bwd_nonfinite_rule
        if (k >= total) break;
      }
    }
    // sweep k + 1 at this workgroup's rows
    if (tid < RB && row0 + tid < S) {
      const int e = (MODE == kModeBwd && a.rescale && k > 0) ? rescale_exponent(bits_double(gmax)) : 0;
      double acc = red[k & 1][0][tid];
#pragma unroll
      for (int w = 1; w < kDGWaves; ++w) acc += red[k & 1][w][tid];
      const double nv = MODE == kModeFwd ? rc + acc                       // maxent.py:110
                                         : ldexp(__dmul_rn(rc, acc), e);  // maxent.py:155-156 (rescaled)
      const unsigned tag1 = salt | ((unsigned)(k + 1) & 0xFFFFFu);
      gran_store(rg, ((unsigned)((k + 1) & 1) * (unsigned)S + (unsigned)(row0 + tid)) * 16u, dbits(nv), tag1, plain);
    }
    ++k;
    // gather v_k, and its max |v_k - v_(k-1)| (forward) / max |v_k| (backward) for the next loop test.
    // red and mred alternate by sweep parity: a wave whose columns hold none of
    // this workgroup's rows can finish this gather (other workgroups' rows only)
    // and write the next partials before the owners (wave 0) have read this
    // sweep's; the slot it writes is the other one, and this one is rewritten
    // only after the next barrier, which the owners reach after their read.
    {
      const unsigned tag = salt | ((unsigned)k & 0xFFFFFu);
      unsigned off[CPT];
#pragma unroll
      for (int j = 0; j < CPT; ++j) off[j] = (unsigned)(k & 1) * 16u * (unsigned)S + off0[j];
      unsigned long long v[CPT];
      if (!gran_gather<CPT>(rg, rg, off, want, tag, v, a.gather_ticks)) lflag = 1;
      unsigned long long d = 0ull;
#pragma unroll
      for (int j = 0; j < CPT; ++j) {
        if (!((want >> j) & 1u)) continue;
        const double nv = bits_double(v[j]);
        const unsigned long long dd = MODE == kModeFwd ? abs_bits(nv - cur[j]) : abs_bits(nv);
        d = dd > d ? dd : d;
        cur[j] = nv;
      }
      d = wave_max_u64(d);
      if (lane == 0) mred[k & 1][wave] = d;
    }
  }
  if (MODE == kModeFwd) {
    // d_k at this workgroup's rows (every workgroup holds all of it)
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      const int c = tid + kDG * j;
      if (c < S && c / RB == blk) a.out[(size_t)b * S + c] = cur[j];
    }
    if (blk == 0 && tid == 0) { a.iters[b] = k; a.status[b] = dg_finish_status(delta, a.eps); }
    return;
  }
  // backward: the last of the 2S sweeps, per action (dense_bwd_final_kernel's arithmetic)
  const int A = a.A;
  const int e = a.rescale ? rescale_exponent(bits_double(gmax)) : 0;
  const double* Pb = a.P + tab * (size_t)A * S * S;
  __shared__ double za_red[kDGWaves][kDenseMaxActions];
  for (int r = 0; r < RB; ++r) {
    const int row = row0 + r;
    if (row >= S) break;
    double* pr = a.out + ((size_t)b * S + row) * A;
    if (nonfinite) {
      if (tid < A) pr[tid] = kNaN;
      continue;
    }
    for (int act = 0; act < A; ++act) {
      const double* prow = Pb + ((size_t)act * S + row) * S;
      double acc = 0.0;
#pragma unroll
      for (int j = 0; j < CPT; ++j) {
        const int c = tid + kDG * j;
        if (c < S) acc = fma(prow[c], cur[j], acc);
      }
      acc = wave_sum_f64(acc);
      if (lane == kWave - 1) za_red[wave][act] = acc;
    }
    __syncthreads();
    if (tid == 0) {
      const double er = exp(a.vin[(size_t)b * S + row]);
      double za[kDenseMaxActions];
      double zsum = 0.0;
      for (int act = 0; act < A; ++act) {
        double acc = za_red[0][act];
        for (int w = 1; w < kDGWaves; ++w) acc += za_red[w][act];
        za[act] = ldexp(__dmul_rn(er, acc), e);  // maxent.py:155
        zsum = __dadd_rn(zsum, za[act]);         // maxent.py:156
      }
      for (int act = 0; act < A; ++act) pr[act] = za[act] / zsum;  // maxent.py:159
    }
    __syncthreads();
  }
  if (blk == 0 && tid == 0) a.status[b] = IRLMX_OK;
}

// Soft VI / VI of a DENSE model (the per-sweep dense_bellman_sweep_kernel's
// statements, maxent.py:326-341, solver.py:40-50 / 95-100), one launch: the
// workgroup holds the A rows P_a[s, :] of each of its RB states (AT >= A
// compiled; the rows of actions >= A are zero), so a sweep is AT * RB row dots
// (the transposed wave reduction in chunks of 16), then thread r folds its
// state's A dots into the new value -- soft: v = phi, v = softmax(v, r + g dot_a)
// in action order; VI: max / mean of g dot_a, plus r -- and publishes it.  The
// loop test max|v_k - v_{k-1}| comes from the gathered vector, as in the
// forward.  After the stop at v_k: value = v_k and, soft, pi = exp(q - v_k)
// with q from the sweep that produced v_k (maxent.py:341).
template <bool SOFT, int AT, int RB, int CPT>
__global__ void __launch_bounds__(kDG) dense_bellman_grid_kernel(DenseGridArgs a) {
  constexpr int K = AT * RB;  // matrix rows per workgroup: (action, state)
  static_assert(K % 16 == 0 && K <= 64, "dense_bellman_grid_kernel: 16, 32, 48 or 64 rows");
  const int S = a.S, A = a.A;
  int b, blk;
  if (!dg_place(a, b, blk)) return;
  const int tid = threadIdx.x, wave = tid / kWave, lane = tid & (kWave - 1);
  __shared__ int resident, lflag;
  __shared__ double red[2][kDGWaves][K];  // by sweep parity (dense_grid_kernel's note)
  __shared__ unsigned long long mred[2][kDGWaves];
  if (tid == 0) {
    resident = coresident(a.err + 1, a.n_resident) ? 1 : 0;
    lflag = 0;
  }
  __syncthreads();
  if (!resident) {
    if (tid == 0) atomicOr(a.err, kErrNotResident);
    return;
  }
  if (b * a.bpi + blk == a.test_drop) return;  // tests: see dense_grid_kernel
  const int row0 = blk * RB;
  const size_t tab = a.shared ? 0 : (size_t)b;
  const double* Pb = a.P + tab * (size_t)A * S * S;
  double m[K][CPT];  // row act * RB + r: P_act[row0 + r, columns tid + kDG * j]
#pragma unroll
  for (int act = 0; act < AT; ++act)
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
      for (int j = 0; j < CPT; ++j) {
        const int row = row0 + r, c = tid + kDG * j;
        m[act * RB + r][j] =
            (act < A && row < S && c < S) ? Pb[((size_t)act * S + row) * S + c] : 0.0;
      }
  // thread r < RB: its state's reward and terminal reward, last value and q
  const bool owner = tid < RB && row0 + tid < S;
  const size_t srow = (size_t)b * S + row0 + (owner ? tid : 0);
  const double rr = owner ? a.vin[srow] : 0.0;
  const double ph = (SOFT && owner) ? a.phi[srow] : 0.0;
  const double v0 = SOFT ? -1e200 : 0.0;  // maxent.py:323 / solver.py:32
  double vkeep = v0, qkeep[AT];
#pragma unroll
  for (int act = 0; act < AT; ++act) qkeep[act] = 0.0;
  double cur[CPT];
  unsigned off0[CPT];
  unsigned want = 0;
#pragma unroll
  for (int j = 0; j < CPT; ++j) {
    const int c = tid + kDG * j;
    off0[j] = (unsigned)(c < S ? c : S - 1) * 16u;
    want |= (c < S ? 1u : 0u) << j;
    cur[j] = c < S ? v0 : 0.0;
  }
  const Gran rg = gran_rsrc(a.gran + (size_t)b * 4 * S, 32u * (unsigned)S);
  const unsigned salt = (a.salt & 0xFFFu) << 20;
  const int pl = dg_plain(a, b, blk, salt, &mred[0][0], &lflag);
  if (pl < 0) {
    if (tid == 0) atomicOr(a.err, 1);
    return;
  }
  const bool plain = pl == 1;
  double delta = 0.0;
  long long k = 0;  // sweeps done: cur = v_k
  for (;;) {
#pragma unroll
    for (int r0 = 0; r0 < K; r0 += 16) {
      double acc[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        acc[r] = 0.0;
#pragma unroll
        for (int j = 0; j < CPT; ++j) acc[r] = fma(m[r0 + r][j], cur[j], acc[r]);
      }
      int row;
      const double sum = rows_sum<16>(acc, lane, row);
      if ((lane & 3) == 0) red[k & 1][wave][r0 + row] = sum;
    }
    __syncthreads();
    if (k > 0) {
      if (lflag) {
        if (tid == 0) atomicOr(a.err, 1);
        return;
      }
      unsigned long long mx = 0ull;
#pragma unroll
      for (int i = 0; i < kDGWaves; ++i) mx = mred[k & 1][i] > mx ? mred[k & 1][i] : mx;
      delta = bits_double(mx);
      if (!(delta > a.eps) || (a.max_iter > 0 && k >= a.max_iter)) break;  // maxent.py:326 / solver.py:40
    }
    if (owner) {  // sweep k + 1 of this thread's state (dense_backup's arithmetic and order)
      double v = SOFT ? ph : 0.0;
#pragma unroll
      for (int act = 0; act < AT; ++act) {
        if (act >= A) break;
        double dot = red[k & 1][0][act * RB + tid];
#pragma unroll
        for (int w = 1; w < kDGWaves; ++w) dot += red[k & 1][w][act * RB + tid];
        if (SOFT) {
          qkeep[act] = __dadd_rn(rr, __dmul_rn(a.discount, dot));
          v = softmax2(v, qkeep[act]);  // maxent.py:329-333
        } else {
          const double q = __dmul_rn(a.discount, dot);  // solver.py:44
          if (a.average) v = act == 0 ? q : __dadd_rn(v, q);
          else v = act == 0 ? q : ((v != v || q <= v) ? v : q);
        }
      }
      if (!SOFT) v = __dadd_rn(rr, a.average ? v / (double)A : v);  // solver.py:47 / :99
      vkeep = v;
      const unsigned tag1 = salt | ((unsigned)(k + 1) & 0xFFFFFu);
      gran_store(rg, ((unsigned)((k + 1) & 1) * (unsigned)S + (unsigned)(row0 + tid)) * 16u, dbits(v), tag1, plain);
    }
    ++k;
    {  // gather v_k and its max |v_k - v_(k-1)| for the next loop test (the forward's ring argument)
      const unsigned tag = salt | ((unsigned)k & 0xFFFFFu);
      unsigned off[CPT];
#pragma unroll
      for (int j = 0; j < CPT; ++j) off[j] = (unsigned)(k & 1) * 16u * (unsigned)S + off0[j];
      unsigned long long v[CPT];
      if (!gran_gather<CPT>(rg, rg, off, want, tag, v, a.gather_ticks)) lflag = 1;
      unsigned long long d = 0ull;
#pragma unroll
      for (int j = 0; j < CPT; ++j) {
        if (!((want >> j) & 1u)) continue;
        const double nv = bits_double(v[j]);
        const unsigned long long dd = abs_bits(nv - cur[j]);
        d = dd > d ? dd : d;
        cur[j] = nv;
      }
      d = wave_max_u64(d);
      if (lane == 0) mred[k & 1][wave] = d;
    }
  }
  if (owner) {
    if (a.value) a.value[srow] = vkeep;
    if (SOFT)
      for (int act = 0; act < A; ++act) a.out[srow * A + act] = np_exp(qkeep[act] - vkeep);  // maxent.py:341
  }
  if (blk == 0 && tid == 0) {
    if (a.iters) a.iters[b] = k;
    a.status[b] = dg_finish_status(delta, a.eps);
  }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------

namespace {

// (RB, CPT) instantiations: RB * CPT <= 64 doubles of matrix per thread, and
// at most 256 workgroups per instance (S <= 2048 at 8 rows; 4 rows x 4 columns
// or 8 columns per thread would need more workgroups than the chip has CUs)
template <int MODE>
void* dense_grid_fn_mode(int rb, int cpt) {
#define IRLMX_DG(R, C) \
  if (rb == R && cpt == C) return (void*)&dense_grid_kernel<MODE, R, C>;
  IRLMX_DG(4, 1) IRLMX_DG(8, 1) IRLMX_DG(16, 1) IRLMX_DG(32, 1) IRLMX_DG(64, 1)
  IRLMX_DG(4, 2) IRLMX_DG(8, 2) IRLMX_DG(16, 2) IRLMX_DG(32, 2)
  IRLMX_DG(8, 4) IRLMX_DG(16, 4)
#undef IRLMX_DG
  return nullptr;
}

void* dense_grid_fn(int mode, int rb, int cpt) {
  return mode == kModeFwd ? dense_grid_fn_mode<kModeFwd>(rb, cpt) : dense_grid_fn_mode<kModeBwd>(rb, cpt);
}

int device_cus() {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  return cus;
}

// workgroups of `fn` that can run at once; IRLMX_PLAN_CUS x IRLMX_PLAN_GRID_PER_CU
// plan without a device (tools/sanitize); a launch re-checks on the device
int capacity(void* fn) {
  const int f_cus = env_int("IRLMX_PLAN_CUS", 0), f_per = env_int("IRLMX_PLAN_GRID_PER_CU", 0);
  if (f_cus > 0 && f_per > 0) return f_cus * f_per;
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)fn, kDG, 0) != hipSuccess) return 0;
  return device_cus() * per_cu;
}

std::atomic<unsigned> g_dg_salt{1};

// (AT, RB, CPT) instantiations of the Bellman kernel: AT * RB a multiple of 16,
// AT * RB * CPT <= 64 doubles, and at most 256 workgroups per instance
template <bool SOFT>
void* dense_bellman_grid_fn_s(int at, int rb, int cpt) {
#define IRLMX_DBG(T, R, C) \
  if (at == T && rb == R && cpt == C) return (void*)&dense_bellman_grid_kernel<SOFT, T, R, C>;
  IRLMX_DBG(4, 4, 1) IRLMX_DBG(4, 4, 2) IRLMX_DBG(4, 8, 1) IRLMX_DBG(4, 8, 2) IRLMX_DBG(4, 16, 1)
  IRLMX_DBG(8, 2, 1) IRLMX_DBG(8, 4, 1) IRLMX_DBG(8, 4, 2) IRLMX_DBG(8, 8, 1)
#undef IRLMX_DBG
  return nullptr;
}

int bellman_at(int A) { return A <= 4 ? 4 : (A <= 8 ? 8 : 0); }

}  // namespace

bool dense_grid_plan(int mode, int S, int B, DenseGridPlan* out) {
  if (env_int("IRLMX_DENSE_GRID", 1) == 0 || S <= 0 || B <= 0) return false;
  const int cpt = S <= kDG ? 1 : (S <= 2 * kDG ? 2 : (S <= 4 * kDG ? 4 : 0));
  if (!cpt) return false;
  const int forced = env_int("IRLMX_DENSE_GRID_RB", 0);
  const int f_cus = env_int("IRLMX_PLAN_CUS", 0);
  const int cus = f_cus > 0 ? f_cus : device_cus();
  if (cus <= 0) return false;
  // XCD groups: every instance's workgroups within one XCD (plain stores, one
  // L2; a group of 8 instances per round of the 8 XCDs).  IRLMX_DENSE_GRID_XCD
  // = 1 insists on them, 0 never takes them.
  const int fx = env_int("IRLMX_DENSE_GRID_XCD", -1);
  const bool xcd_ok = env_int("IRLMX_XCD_GROUP", 1) != 0 && fx != 0;
  // Measured preference (profiles/r03_dense_grid_bench.txt, tools/diag/dense_grid_bench.py):
  //  1. XCD-grouped, the fewest rows per workgroup that fit one XCD per instance
  //     group (0.4-0.5 us per sweep below the spread form at equal rows);
  //  2. spread over the chip at >= 8 rows and <= 128 workgroups per instance
  //     (the gather costs a whole vector per workgroup; rows are cheap with the
  //     transposed reduction), else any row count that fits one workgroup per CU.
  int pref = 8;
  while (pref < 64 && (S + pref - 1) / pref > 128) pref *= 2;
  for (int pass = 0; pass < 3; ++pass) {
    if (pass == 0 && !xcd_ok) continue;
    if (pass > 0 && fx == 1) break;
    for (int rb = pass == 1 ? pref : 4; rb <= 64; rb *= 2) {
      if (forced > 0 && rb != forced) continue;
      void* fn = dense_grid_fn(mode, rb, cpt);
      if (!fn) continue;
      const int bpi = (S + rb - 1) / rb;
      if ((long long)bpi * B > cus) continue;
      const int cap = capacity(fn);
      if ((long long)bpi * B > cap) continue;
      const bool fits = cap >= 8 && bpi <= kDG && (long long)((B + 7) / 8) * bpi <= cus / 8;
      if (pass == 0 && !fits) continue;
      *out = DenseGridPlan{rb, cpt, bpi, pass == 0 ? 1 : 0, 0};
      return true;
    }
  }
  return false;
}

// Soft VI / VI: the fewest rows per workgroup that fit (a row costs A dots and
// the fold); XCD-grouped only at <= 8 rows per workgroup (measured,
// profiles/r03_dense_bellman_grid_variants.txt: S = 256 one XCD at 8 rows 3.2 us
// per sweep vs 3.5 spread; S = 512 one XCD needs 16 rows, 4.3 vs 3.9 spread at 4).
bool dense_bellman_grid_plan(int S, int B, int A, DenseGridPlan* out) {
  if (env_int("IRLMX_DENSE_GRID", 1) == 0 || S <= 0 || B <= 0) return false;
  const int at = bellman_at(A);
  const int cpt = S <= kDG ? 1 : (S <= 2 * kDG ? 2 : 0);
  if (!at || !cpt) return false;
  const int forced = env_int("IRLMX_DENSE_GRID_RB", 0);
  const int f_cus = env_int("IRLMX_PLAN_CUS", 0);
  const int cus = f_cus > 0 ? f_cus : device_cus();
  if (cus <= 0) return false;
  const int fx = env_int("IRLMX_DENSE_GRID_XCD", -1);
  const bool xcd_ok = env_int("IRLMX_XCD_GROUP", 1) != 0 && fx != 0;
  for (int pass = 0; pass < 2; ++pass) {
    if (pass == 0 && !xcd_ok) continue;
    if (pass > 0 && fx == 1) break;
    for (int rb = 2; rb <= 16; rb *= 2) {
      if (forced > 0 && rb != forced) continue;
      void* fn = dense_bellman_grid_fn_s<true>(at, rb, cpt);
      if (!fn) continue;
      const int bpi = (S + rb - 1) / rb;
      if ((long long)bpi * B > cus) continue;
      const int cap = std::min(capacity(fn), capacity(dense_bellman_grid_fn_s<false>(at, rb, cpt)));
      if ((long long)bpi * B > cap) continue;
      const bool fits = cap >= 8 && bpi <= kDG && (long long)((B + 7) / 8) * bpi <= cus / 8 && (rb <= 8 || fx == 1);
      if (pass == 0 && !fits) continue;
      *out = DenseGridPlan{rb, cpt, bpi, pass == 0 ? 1 : 0, at};
      return true;
    }
  }
  return false;
}

static int launch_grid(void* fn, const DenseGridPlan& p, DenseGridArgs a, int rows, hipStream_t st) {
  a.rb = rows;
  a.bpi = p.bpi;
  a.nb = a.B;
  a.xcd_group = p.xcd;
  a.salt = g_dg_salt.fetch_add(1, std::memory_order_relaxed);
  // (IRLMX_TEST_NOT_RESIDENT=1, tests only: one workgroup more than launched -> the per-sweep rerun)
  a.n_resident = p.bpi * a.B + (env_int("IRLMX_TEST_NOT_RESIDENT", 0) ? 1 : 0);
  // (IRLMX_TEST_DROP_TILE / IRLMX_TEST_EXCHANGE_TIMEOUT_MS, tests only: one workgroup
  // leaves after the rendezvous, its neighbours time out -> the per-sweep rerun)
  a.test_drop = env_int("IRLMX_TEST_DROP_TILE", -1);
  const int tmo_ms = env_int("IRLMX_TEST_EXCHANGE_TIMEOUT_MS", 0);
  a.gather_ticks = tmo_ms > 0 ? (unsigned long long)tmo_ms * 100000ull : kGatherTicks;
  const int grid = p.xcd ? 8 * ((a.B + 7) / 8) * p.bpi : p.bpi * a.B;
  void* args[] = {&a};
  hipError_t e = hipLaunchKernel(fn, dim3(grid), dim3(kDG), args, 0, st);
  if (e != hipSuccess) return hip_fail(e, "dense grid launch");
  count_event(IRLMX_CTR_GRID_LAUNCHES);
  int err = 0;
  e = hipMemcpyAsync(&err, a.err, sizeof(int), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) return hip_fail(e, "dense grid sync");
  const bool timeout = err && !(err & kErrNotResident);
  if (timeout && env_int("IRLMX_STRICT_EXCHANGE", 0)) {
    set_error("dense grid shape: exchange timed out (workgroups not co-resident?)");
    return IRLMX_EHIP;
  }
  if (timeout) note_exchange_timeout("dense grid");
  if (err) {  // not all workgroups ran at once, or an exchange timed out: the per-sweep shape
    count_event(timeout ? IRLMX_CTR_RERUN_TIMEOUT : IRLMX_CTR_RERUN_NOT_RESIDENT);
    e = hipMemsetAsync(a.err, 0, 4 * sizeof(int), st);
    return e == hipSuccess ? kClusterNotResident : hip_fail(e, "dense grid err reset");
  }
  return 0;
}

int dense_bellman_grid_run(bool soft, const DenseGridPlan& p, DenseGridArgs a, hipStream_t st) {
  const int at = p.at, rb = p.rb;
  void* fn = soft ? dense_bellman_grid_fn_s<true>(at, rb, p.cpt) : dense_bellman_grid_fn_s<false>(at, rb, p.cpt);
  if (!fn) {
    set_error("dense bellman grid: no kernel for %d actions, %d rows, %d columns per thread", at, rb, p.cpt);
    return IRLMX_EINVAL;
  }
  return launch_grid(fn, p, a, rb, st);
}

int dense_grid_run(int mode, const DenseGridPlan& p, DenseGridArgs a, hipStream_t st) {
  return launch_grid(dense_grid_fn(mode, p.rb, p.cpt), p, a, p.rb, st);
}

}  // namespace irlmx
