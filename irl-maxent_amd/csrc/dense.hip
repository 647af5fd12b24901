// Dense-row kernels (IRLMX_LAYOUT_DENSE) for transition models whose rows are
// mostly nonzero -- non-grid MDPs where the ELL layout would gather ~S slots
// per state.  Each kernel is one sweep of a reference statement over all B
// instances, with the swept vector staged in LDS and the matrix rows streamed
// from HBM, one wave per output row (64 lanes x 16 B = 1 KiB per coalesced
// load, four independent FMA chains per lane, butterfly sum):
//
//   backward   zs'[s] = exp(r[s]) * (M zs)[s],  M = sum_a P_a  (maxent.py:155-156)
//   final      za[s, a] = exp(r[s]) * (P_a zs)[s]; pi = za / sum_a za (maxent.py:155-159)
//   forward    d'[t] = p0[t] + (WT d)[t],  WT[t][s] = sum_a P'[s, t, a] pi[s, a]
//                                                          (maxent.py:98-112)
//   soft VI    v'[s] = fold_a softmax(v', r[s] + g (P_a v)[s]) from phi  (maxent.py:326-338)
//   VI         v'[s] = r[s] + max_a / mean_a g (P_a v)[s]            (solver.py:40-50, 95-100)
//
// All are HBM-stream bound (S^2 doubles per sweep per table and instance).
// With one table shared by B instances the sweep is a GEMM (M . [zs_1 .. zs_B],
// or the stacked P_a for soft VI / VI); fixed_point.hip then runs it on the
// hand-written fp64 MFMA kernel below plus an epilogue, or streams M once per
// instance -- whichever the planner's measured crossover picks (dense_gemm()
// in fixed_point.hip: from 16 instances, from 4 at S >= 4096).  Up to S = 2048
// the persistent dense shape (dense_grid.hip) takes the calls the GEMM does not.
// Convergence bookkeeping follows the sweep shape of fixed_point.hip (3-slot
// max ring, done flags, host polling).

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdlib>

#include "dense.h"

namespace irlmx {

namespace {

__device__ inline int dense_finish_status(double delta, double eps) {
  if (delta != delta) return IRLMX_NONFINITE;
  return delta > eps ? IRLMX_MAXITER : IRLMX_OK;
}

// The reference's loop test for instance b before sweep `it` (fixed_point.hip
// sweep_should_stop): stop after the first sweep whose max|delta| is not > eps.
__device__ inline bool dense_should_stop(int b, long long it, int r3, double eps, long long max_iter,
                                         const DenseBufs& w, int32_t* status) {
  if (w.done[b]) return true;
  if (it == 0) return false;
  const double prev = bits_double(w.slots[b * 3 + (r3 == 0 ? 2 : r3 - 1)]);
  const bool cap = max_iter > 0 && it >= max_iter;
  if (prev > eps && !cap) return false;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    w.done[b] = 1;
    w.iters[b] = it;
    status[b] = dense_finish_status(prev, eps);
    atomicAdd(w.ndone, 1);
  }
  return true;
}

// Copy the swept vector into LDS (dense_lds_vec), else read it in place.
template <bool LDSV>
__device__ inline const double* stage(const double* __restrict__ src, double* lds, int S) {
  if constexpr (!LDSV) {
    return src;
  } else {
    if ((S & 1) == 0) {
      const double2* s2 = reinterpret_cast<const double2*>(src);
      double2* l2 = reinterpret_cast<double2*>(lds);
      for (int i = threadIdx.x; i < (S >> 1); i += blockDim.x) l2[i] = s2[i];
    } else {
      for (int i = threadIdx.x; i < S; i += blockDim.x) lds[i] = src[i];
    }
    __syncthreads();
    return lds;
  }
}

// Dot product of one matrix row with v, by one wave; every lane returns the
// same sum (the butterfly adds the same pair on both partners: commutative).
__device__ inline double wave_dot(const double* __restrict__ row, const double* __restrict__ v, int S, int lane) {
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  if ((S & 1) == 0) {
    const double2* r2 = reinterpret_cast<const double2*>(row);
    const double2* v2 = reinterpret_cast<const double2*>(v);
    const int n2 = S >> 1;
    int j = lane;
#pragma unroll kDenseUnroll
    for (; j + 64 < n2; j += 128) {
      const double2 x = r2[j];
      const double2 y = r2[j + 64];
      const double2 p = v2[j], q = v2[j + 64];
      a0 = fma(x.x, p.x, a0);
      a1 = fma(x.y, p.y, a1);
      a2 = fma(y.x, q.x, a2);
      a3 = fma(y.y, q.y, a3);
    }
    if (j < n2) {
      const double2 x = r2[j];
      const double2 p = v2[j];
      a0 = fma(x.x, p.x, a0);
      a1 = fma(x.y, p.y, a1);
    }
  } else {
    for (int j = lane; j < S; j += 64) a0 = fma(row[j], v[j], a0);
  }
  double acc = (a0 + a1) + (a2 + a3);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, kWave);
  return acc;
}

// Block-wide max of per-wave values (every lane of a wave holds the same value),
// one atomic per workgroup.
__device__ inline void block_max_slot(unsigned long long v, unsigned long long* dst) {
  __shared__ unsigned long long red[kDenseThreads / kWave];
  const int wv = threadIdx.x / kWave;
  if ((threadIdx.x & (kWave - 1)) == 0) red[wv] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long m = 0;
    for (int i = 0; i < kDenseThreads / kWave; ++i) m = red[i] > m ? red[i] : m;
    if (m) atomicMax(dst, m);
  }
}

__device__ inline size_t table_of(const DenseView& d, int b) { return d.shared ? 0 : (size_t)b; }

}  // namespace

// dense [S][S][A] -> P [A][S][S] and M [S][S] (action sum in action order)
__global__ void dense_rows_kernel(const double* __restrict__ dense, int S, int A, double* __restrict__ P,
                                  double* __restrict__ M) {
  const size_t n = (size_t)S * S;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    double acc = 0.0;
    for (int a = 0; a < A; ++a) {
      const double v = dense[i * A + a];
      P[(size_t)a * n + i] = v;
      acc += v;
    }
    M[i] = acc;
  }
}

// Forward gather matrix of instance b, transposed through LDS:
//   WT[b][t][s] = sum_a P[s, t, a] * pi[b][s][a]   (0 for terminal rows s, maxent.py:98-99)
// so that the forward sweep reads rows of WT.  32 x 32 tiles, 256 threads.
__global__ void __launch_bounds__(256) dense_fwd_weights_kernel(DenseView d, const double* __restrict__ pi,
                                                                const uint8_t* __restrict__ term,
                                                                double* __restrict__ wt) {
  __shared__ double tile[32][33];
  const int S = d.S, A = d.A, b = blockIdx.z;
  const int s0 = blockIdx.y * 32, t0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 8 rows of 32
  const double* Pb = d.P + table_of(d, b) * A * (size_t)S * S;
  const double* pib = pi + (size_t)b * S * A;
  for (int ii = ty; ii < 32; ii += 8) {
    const int s = s0 + ii, t = t0 + tx;
    double acc = 0.0;
    if (s < S && t < S && !term[(size_t)b * S + s])
      for (int a = 0; a < A; ++a) acc = fma(Pb[((size_t)a * S + s) * S + t], pib[(size_t)s * A + a], acc);
    tile[ii][tx] = acc;
  }
  __syncthreads();
  for (int jj = ty; jj < 32; jj += 8) {
    const int t = t0 + jj, s = s0 + tx;
    if (t < S && s < S) wt[((size_t)b * S + t) * S + s] = tile[tx][jj];
  }
}

// non-finite policy entries: the reference's dense product is NaN everywhere
// after one sweep (fixed_point.hip fwd_weights_kernel)
__global__ void dense_pi_check_kernel(const double* __restrict__ pi, int n, int32_t* __restrict__ bad) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (i < n && !isfinite(pi[(size_t)b * n + i])) atomicOr(&bad[b], 1);
}

template <bool LDSV>
__global__ void __launch_bounds__(kDenseThreads)
dense_fwd_sweep_kernel(DenseView d, const double* __restrict__ p0, double eps, long long max_iter,
                       int32_t* __restrict__ status, DenseBufs w, long long it, int r3) {
  extern __shared__ __attribute__((aligned(16))) double vs[];
  const int b = blockIdx.y, S = d.S;
  if (w.bad[b]) {
    if (blockIdx.x == 0 && threadIdx.x == 0 && !w.done[b]) {
      w.done[b] = 1; w.iters[b] = 1; status[b] = IRLMX_NONFINITE; atomicAdd(w.ndone, 1);
    }
    return;
  }
  if (dense_should_stop(b, it, r3, eps, max_iter, w, status)) return;
  const double* din = ((it & 1) ? w.buf1 : w.buf0) + (size_t)b * S;
  double* dout = ((it & 1) ? w.buf0 : w.buf1) + (size_t)b * S;
  const double* v = stage<LDSV>(din, vs, S);
  const int wave = threadIdx.x / kWave, lane = threadIdx.x & (kWave - 1);
  unsigned long long mx = 0ull;
  for (int i = 0; i < kDenseRowsPerWave; ++i) {
    const int t = blockIdx.x * kDenseRowsPerBlock + wave * kDenseRowsPerWave + i;
    if (t >= S) break;
    const double acc = wave_dot(w.wt + ((size_t)b * S + t) * S, v, S, lane);
    const double nv = p0[(size_t)b * S + t] + acc;   // maxent.py:110
    if (lane == 0) dout[t] = nv;
    const unsigned long long dd = abs_bits(nv - v[t]);
    mx = dd > mx ? dd : mx;
  }
  block_max_slot(mx, &w.slots[b * 3 + r3]);
  if (blockIdx.x == 0 && threadIdx.x == 0) w.slots[b * 3 + (r3 == 2 ? 0 : r3 + 1)] = 0ull;
}

__global__ void dense_bwd_init_kernel(int S, const uint8_t* __restrict__ term, double* __restrict__ buf0) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (s < S) buf0[(size_t)b * S + s] = term[(size_t)b * S + s] ? 1.0 : 0.0;   // maxent.py:146-147
}

// One collapsed backward sweep, streaming M once per instance.
template <bool LDSV>
__global__ void __launch_bounds__(kDenseThreads)
dense_bwd_sweep_kernel(DenseView d, const double* __restrict__ reward, int rescale, DenseBufs w, long long it,
                       int r3) {
  extern __shared__ __attribute__((aligned(16))) double vs[];
  const int b = blockIdx.y, S = d.S;
  const double* din = ((it & 1) ? w.buf1 : w.buf0) + (size_t)b * S;
  double* dout = ((it & 1) ? w.buf0 : w.buf1) + (size_t)b * S;
  int e = 0;
  if (rescale && it > 0) e = rescale_exponent(bits_double(w.slots[b * 3 + (r3 == 0 ? 2 : r3 - 1)]));
  const double* v = stage<LDSV>(din, vs, S);
  const double* M = d.M + table_of(d, b) * (size_t)S * S;
  const int wave = threadIdx.x / kWave, lane = threadIdx.x & (kWave - 1);
  unsigned long long mx = 0ull;
  for (int i = 0; i < kDenseRowsPerWave; ++i) {
    const int s = blockIdx.x * kDenseRowsPerBlock + wave * kDenseRowsPerWave + i;
    if (s >= S) break;
    const double acc = wave_dot(M + (size_t)s * S, v, S, lane);
    const double nv = ldexp(__dmul_rn(exp(reward[(size_t)b * S + s]), acc), e);
    if (lane == 0) {
      dout[s] = nv;
      if (!isfinite(nv)) atomicOr(&w.bad[b], 1);   // fixed_point.hip bwd_nonfinite_rule
    }
    const unsigned long long dd = abs_bits(nv);
    mx = dd > mx ? dd : mx;
  }
  if (rescale) {
    block_max_slot(mx, &w.slots[b * 3 + r3]);
    if (blockIdx.x == 0 && threadIdx.x == 0) w.slots[b * 3 + (r3 == 2 ? 0 : r3 + 1)] = 0ull;
  }
}

// Epilogue of a GEMM sweep (shared table): w.wt[b][s] = (M . zs_b)[s].
__global__ void __launch_bounds__(kDenseThreads)
dense_bwd_gemm_epilogue_kernel(int S, const double* __restrict__ reward, int rescale, DenseBufs w, long long it,
                               int r3) {
  const int b = blockIdx.y;
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  double* dout = ((it & 1) ? w.buf0 : w.buf1) + (size_t)b * S;
  int e = 0;
  if (rescale && it > 0) e = rescale_exponent(bits_double(w.slots[b * 3 + (r3 == 0 ? 2 : r3 - 1)]));
  unsigned long long mx = 0ull;
  if (s < S) {
    const double nv = ldexp(__dmul_rn(exp(reward[(size_t)b * S + s]), w.wt[(size_t)b * S + s]), e);
    dout[s] = nv;
    if (!isfinite(nv)) atomicOr(&w.bad[b], 1);
    mx = abs_bits(nv);
  }
  if (rescale) {
    for (int off = 32; off > 0; off >>= 1) {
      const unsigned long long o = __shfl_xor(mx, off, kWave);
      mx = o > mx ? o : mx;
    }
    block_max_slot(mx, &w.slots[b * 3 + r3]);
    if (blockIdx.x == 0 && threadIdx.x == 0) w.slots[b * 3 + (r3 == 2 ? 0 : r3 + 1)] = 0ull;
  }
}

// The last of the 2*S sweeps, per action: za = exp(r) * (P_a zs); pi = za / sum_a za.
template <bool LDSV>
__global__ void __launch_bounds__(kDenseThreads)
dense_bwd_final_kernel(DenseView d, const double* __restrict__ reward, int rescale, double* __restrict__ pi,
                       int32_t* __restrict__ status, DenseBufs w, long long collapsed, int r3) {
  extern __shared__ __attribute__((aligned(16))) double vs[];
  const int b = blockIdx.y, S = d.S, A = d.A;
  const int wave = threadIdx.x / kWave, lane = threadIdx.x & (kWave - 1);
  if (w.bad[b]) {  // bwd_nonfinite_rule
    for (int i = 0; i < kDenseRowsPerWave; ++i) {
      const int s = blockIdx.x * kDenseRowsPerBlock + wave * kDenseRowsPerWave + i;
      if (s < S && lane < A) pi[((size_t)b * S + s) * A + lane] = kNaN;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) status[b] = IRLMX_OK;
    return;
  }
  const double* zs = ((collapsed & 1) ? w.buf1 : w.buf0) + (size_t)b * S;
  int e = 0;
  if (rescale && collapsed > 0) e = rescale_exponent(bits_double(w.slots[b * 3 + (r3 == 0 ? 2 : r3 - 1)]));
  const double* v = stage<LDSV>(zs, vs, S);
  const double* Pb = d.P + table_of(d, b) * A * (size_t)S * S;
  for (int i = 0; i < kDenseRowsPerWave; ++i) {
    const int s = blockIdx.x * kDenseRowsPerBlock + wave * kDenseRowsPerWave + i;
    if (s >= S) break;
    const double er = exp(reward[(size_t)b * S + s]);
    double za[kDenseMaxActions];
    double zsum = 0.0;
#pragma unroll
    for (int act = 0; act < kDenseMaxActions; ++act) {
      za[act] = 0.0;
      if (act < A) {
        const double acc = wave_dot(Pb + ((size_t)act * S + s) * S, v, S, lane);
        za[act] = ldexp(__dmul_rn(er, acc), e);   // rounded product, then the sum (maxent.py:155-156)
        zsum = __dadd_rn(zsum, za[act]);
      }
    }
    double z = za[0];
#pragma unroll
    for (int act = 1; act < kDenseMaxActions; ++act) z = lane == act ? za[act] : z;
    if (lane < A) pi[((size_t)b * S + s) * A + lane] = z / zsum;   // maxent.py:159
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) status[b] = IRLMX_OK;
}

// Bellman backup of one state from its A action dots (fixed_point.hip bellman_update).
__device__ inline double dense_backup(const DenseBellman& a, int A, const double (&dots)[kDenseMaxActions], double r,
                                     double phi) {
  double v = a.soft ? phi : 0.0;
#pragma unroll
  for (int act = 0; act < kDenseMaxActions; ++act) {
    if (act >= A) break;
    if (a.soft) {
      v = softmax2(v, __dadd_rn(r, __dmul_rn(a.discount, dots[act])));   // maxent.py:329-333
    } else {
      const double q = __dmul_rn(a.discount, dots[act]);                 // solver.py:44
      if (a.average) v = act == 0 ? q : __dadd_rn(v, q);
      else v = act == 0 ? q : ((v != v || q <= v) ? v : q);
    }
  }
  if (!a.soft) v = __dadd_rn(r, a.average ? v / (double)A : v);           // solver.py:47 / :99
  return v;
}

template <bool LDSV>
__global__ void __launch_bounds__(kDenseThreads)
dense_bellman_sweep_kernel(DenseView d, DenseBellman a, DenseBufs w, long long it, int r3) {
  extern __shared__ __attribute__((aligned(16))) double vs[];
  const int b = blockIdx.y, S = d.S, A = d.A;
  if (dense_should_stop(b, it, r3, a.eps, a.max_iter, w, a.status)) return;
  const double* vin = ((it & 1) ? w.buf1 : w.buf0) + (size_t)b * S;
  double* vout = ((it & 1) ? w.buf0 : w.buf1) + (size_t)b * S;
  const double* v = stage<LDSV>(vin, vs, S);
  const double* Pb = d.P + table_of(d, b) * A * (size_t)S * S;
  const int wave = threadIdx.x / kWave, lane = threadIdx.x & (kWave - 1);
  unsigned long long mx = 0ull;
  for (int i = 0; i < kDenseRowsPerWave; ++i) {
    const int s = blockIdx.x * kDenseRowsPerBlock + wave * kDenseRowsPerWave + i;
    if (s >= S) break;
    double dots[kDenseMaxActions];
#pragma unroll
    for (int act = 0; act < kDenseMaxActions; ++act)
      dots[act] = act < A ? wave_dot(Pb + ((size_t)act * S + s) * S, v, S, lane) : 0.0;
    const double nv = dense_backup(a, A, dots, a.reward[(size_t)b * S + s], a.soft ? a.phi[(size_t)b * S + s] : 0.0);
    if (lane == 0) vout[s] = nv;
    const unsigned long long dd = abs_bits(nv - v[s]);
    mx = dd > mx ? dd : mx;
  }
  block_max_slot(mx, &w.slots[b * 3 + r3]);
  if (blockIdx.x == 0 && threadIdx.x == 0) w.slots[b * 3 + (r3 == 2 ? 0 : r3 + 1)] = 0ull;
}

// One Bellman sweep of all instances of a shared table from GEMM products:
// c[b][a * S + s] = (P_a v_b)[s], one MFMA GEMM over the stacked P_a; the
// rest of dense_bellman_sweep_kernel's update and bookkeeping, thread per state.
__global__ void __launch_bounds__(kDenseThreads)
dense_bellman_gemm_epilogue_kernel(DenseView d, DenseBellman a, DenseBufs w, const double* __restrict__ c,
                                   long long it, int r3) {
  const int b = blockIdx.y, S = d.S, A = d.A;
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (dense_should_stop(b, it, r3, a.eps, a.max_iter, w, a.status)) return;
  const double* vin = ((it & 1) ? w.buf1 : w.buf0) + (size_t)b * S;
  double* vout = ((it & 1) ? w.buf0 : w.buf1) + (size_t)b * S;
  unsigned long long mx = 0ull;
  if (s < S) {
    double dots[kDenseMaxActions];
#pragma unroll
    for (int act = 0; act < kDenseMaxActions; ++act)
      dots[act] = act < A ? c[((size_t)b * A + act) * S + s] : 0.0;
    const double nv = dense_backup(a, A, dots, a.reward[(size_t)b * S + s], a.soft ? a.phi[(size_t)b * S + s] : 0.0);
    vout[s] = nv;
    mx = abs_bits(nv - vin[s]);
  }
  for (int off = 32; off > 0; off >>= 1) {
    const unsigned long long o = __shfl_xor(mx, off, kWave);
    mx = o > mx ? o : mx;
  }
  block_max_slot(mx, &w.slots[b * 3 + r3]);
  if (blockIdx.x == 0 && threadIdx.x == 0) w.slots[b * 3 + (r3 == 2 ? 0 : r3 + 1)] = 0ull;
}

// value out; soft VI: pi = exp(q - v) with q from the last sweep's input (maxent.py:341)
template <bool LDSV>
__global__ void __launch_bounds__(kDenseThreads)
dense_bellman_finish_kernel(DenseView d, DenseBellman a, DenseBufs w) {
  extern __shared__ __attribute__((aligned(16))) double vs[];
  const int b = blockIdx.y, S = d.S, A = d.A;
  const long long it = w.iters[b];
  const double* vnew = ((it & 1) ? w.buf1 : w.buf0) + (size_t)b * S;
  const double* vold = ((it & 1) ? w.buf0 : w.buf1) + (size_t)b * S;
  const double* v = stage<LDSV>(vold, vs, S);
  const double* Pb = d.P + table_of(d, b) * A * (size_t)S * S;
  const int wave = threadIdx.x / kWave, lane = threadIdx.x & (kWave - 1);
  for (int i = 0; i < kDenseRowsPerWave; ++i) {
    const int s = blockIdx.x * kDenseRowsPerBlock + wave * kDenseRowsPerWave + i;
    if (s >= S) break;
    const double vn = vnew[s];
    if (lane == 0 && a.value) a.value[(size_t)b * S + s] = vn;
    if (a.soft) {
      const double r = a.reward[(size_t)b * S + s];
      for (int act = 0; act < A; ++act) {
        const double dot = wave_dot(Pb + ((size_t)act * S + s) * S, v, S, lane);
        const double q = __dadd_rn(r, __dmul_rn(a.discount, dot));
        if (lane == 0) a.pi[((size_t)b * S + s) * A + act] = np_exp(q - vn);
      }
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && a.iters) a.iters[b] = it;
}

// ---------------------------------------------------------------------------
// batched GEMM on the fp64 matrix cores: C[b][s] = sum_t M[s][t] * Z[b][t]
// ---------------------------------------------------------------------------
//
// One table shared by B instances (the backward sweep M . [zs_1 .. zs_B]).
// v_mfma_f64_16x16x4_f64: lane l supplies A[l & 15][k = l >> 4] and
// B[k = l >> 4][l & 15]; D[row (l >> 4) + 4 r][col l & 15] in register r
// (cdna_hip_programming.md, f64 MFMA maps).  A workgroup owns 16 ST rows of M x
// 16 NBT instances; its kGemmWaves waves split the sum over t (K) into equal
// parts and meet in LDS, summed in wave order (deterministic).  With one
// workgroup per CU, eight waves (two per SIMD: one wave's loads in flight while
// the other's MFMAs run) measured 1.1-1.7x faster than four, sixteen no better
// (S = 4096: B = 4 48.9 -> 29.1 us, B = 16 47.4 -> 33.9, B = 64 85.0 -> 79.2);
// with two or more workgroups per CU four waves stay faster (the stacked soft-VI
// GEMM at S = 4096, B = 16: 210 vs 233 us).  Per 16-wide K chunk a lane loads
// 32 contiguous bytes of each of its rows of M and Z (128 B per row across the
// four lanes of a column), and MFMA x (x = 0..3) uses element x of them: the
// k index of both operands maps to the same t = 16 c + 4 (l >> 4) + x.  M is
// read from HBM once per sweep; Z (B x S) is re-read per 32 rows of M (L2).
//
// Any S: the K tail (S % 16 != 0) is zero-padded per element -- a padded term
// is 0 * 0, exactly 0, so the sums are those of the unpadded products -- and
// rows start 16-byte aligned only when S is even (V2: two 16-byte loads per
// operand row and chunk), else the kernel loads doubles one by one.
typedef double f64x4 __attribute__((ext_vector_type(4)));
#ifndef IRLMX_GEMM_PF
#define IRLMX_GEMM_PF 1
#endif
constexpr int kGemmPrefetch = IRLMX_GEMM_PF;  // K chunks whose loads are in flight during a chunk's MFMAs

// ST 16-row tiles of M and NBT 16-instance column tiles per workgroup (sized to
// S and B so that the grid fills the chip)
template <int ST, int NBT, int kGemmWaves, bool V2>
__global__ void __launch_bounds__(kGemmWaves * kWave)
dense_gemm_kernel(const double* __restrict__ M, const double* __restrict__ Z, double* __restrict__ C, int R, int S,
                  int B) {  // M [R][S], Z [B][S] -> C [B][R]
  extern __shared__ __attribute__((aligned(16))) double part[];  // [waves][ST][NBT][4][64]
  const int wave = threadIdx.x / kWave, l = threadIdx.x & (kWave - 1);
  const int s0 = blockIdx.x * 16 * ST, b0 = blockIdx.y * 16 * NBT;
  const int i = l & 15, q = l >> 4;
  const int nchunk = (S + 15) / 16;
  const int c0 = wave * nchunk / kGemmWaves, c1 = (wave + 1) * nchunk / kGemmWaves;
  f64x4 acc[ST][NBT];
#pragma unroll
  for (int st = 0; st < ST; ++st)
#pragma unroll
    for (int bt = 0; bt < NBT; ++bt) acc[st][bt] = f64x4{0.0, 0.0, 0.0, 0.0};
  // rows of this lane (out of range: a valid row, zeroed on load)
  const double* mrow[ST];
  const double* zrow[NBT];
  bool mok[ST], zok[NBT];
#pragma unroll
  for (int st = 0; st < ST; ++st) {
    const int r = s0 + 16 * st + i;
    mok[st] = r < R;
    mrow[st] = M + (size_t)(mok[st] ? r : 0) * S;
  }
#pragma unroll
  for (int bt = 0; bt < NBT; ++bt) {
    const int r = b0 + 16 * bt + i;
    zok[bt] = r < B;
    zrow[bt] = Z + (size_t)(zok[bt] ? r : 0) * S;
  }
  // the 4 consecutive t of chunk c this lane supplies, zero beyond S
  auto load4 = [&](const double* row, int t, bool ok, double2 (&o)[2]) {
    o[0] = o[1] = make_double2(0.0, 0.0);
    if (!ok || t >= S) return;
    if (t + 3 < S) {
      if constexpr (V2) {
        o[0] = *reinterpret_cast<const double2*>(row + t);
        o[1] = *reinterpret_cast<const double2*>(row + t + 2);
      } else {
        o[0] = make_double2(row[t], row[t + 1]);
        o[1] = make_double2(row[t + 2], row[t + 3]);
      }
    } else {  // the K tail
      o[0].x = row[t];
      if (t + 1 < S) o[0].y = row[t + 1];
      if (t + 2 < S) o[1].x = row[t + 2];
    }
  };
  double2 ma[ST][2], za[NBT][2];
  auto load = [&](int c, double2 (&mo)[ST][2], double2 (&zo)[NBT][2]) {
    const int t = 16 * c + 4 * q;
    const bool tok = c < c1;
#pragma unroll
    for (int st = 0; st < ST; ++st) load4(mrow[st], t, tok && mok[st], mo[st]);
#pragma unroll
    for (int bt = 0; bt < NBT; ++bt) load4(zrow[bt], t, tok && zok[bt], zo[bt]);
  };
  auto el = [](const double2 (&v)[2], int x) { return x == 0 ? v[0].x : x == 1 ? v[0].y : x == 2 ? v[1].x : v[1].y; };
  auto mfmas = [&](const double2 (&mo)[ST][2], const double2 (&zo)[NBT][2]) {
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int st = 0; st < ST; ++st)
#pragma unroll
        for (int bt = 0; bt < NBT; ++bt)
          acc[st][bt] = __builtin_amdgcn_mfma_f64_16x16x4f64(el(mo[st], x), el(zo[bt], x), acc[st][bt], 0, 0, 0);
  };
  if constexpr (kGemmPrefetch <= 1) {
    load(c0, ma, za);
    for (int c = c0; c < c1; ++c) {
      double2 mn[ST][2], zn[NBT][2];
      load(c + 1, mn, zn);  // next chunk in flight during this chunk's MFMAs
      mfmas(ma, za);
#pragma unroll
      for (int st = 0; st < ST; ++st) { ma[st][0] = mn[st][0]; ma[st][1] = mn[st][1]; }
#pragma unroll
      for (int bt = 0; bt < NBT; ++bt) { za[bt][0] = zn[bt][0]; za[bt][1] = zn[bt][1]; }
    }
  } else {
    // a ring of kGemmPrefetch + 1 chunk buffers: kGemmPrefetch chunks in flight
    constexpr int PF = kGemmPrefetch, NR = kGemmPrefetch + 1;
    double2 mr[NR][ST][2], zr[NR][NBT][2];
#pragma unroll
    for (int p = 0; p < PF; ++p) load(c0 + p, mr[p], zr[p]);
    for (int c = c0; c < c1; c += NR) {
#pragma unroll
      for (int u = 0; u < NR; ++u) {
        load(c + u + PF, mr[(u + PF) % NR], zr[(u + PF) % NR]);
        if (c + u < c1) mfmas(mr[u], zr[u]);
      }
    }
  }
  // split-K partials -> LDS, summed in wave order
#pragma unroll
  for (int st = 0; st < ST; ++st)
#pragma unroll
    for (int bt = 0; bt < NBT; ++bt)
#pragma unroll
      for (int r = 0; r < 4; ++r) part[((((size_t)wave * ST + st) * NBT + bt) * 4 + r) * kWave + l] = acc[st][bt][r];
  __syncthreads();
  constexpr int kOut = ST * NBT * 4 * kWave;  // outputs per workgroup
  for (int e = threadIdx.x; e < kOut; e += kGemmWaves * kWave) {
    double v = part[e];
#pragma unroll
    for (int w = 1; w < kGemmWaves; ++w) v += part[(size_t)w * kOut + e];
    const int ll = e % kWave, r = (e / kWave) % 4, bt = (e / (kWave * 4)) % NBT, st = e / (kWave * 4 * NBT);
    const int row = s0 + 16 * st + (ll >> 4) + 4 * r, col = b0 + 16 * bt + (ll & 15);
    if (row < R && col < B) C[(size_t)col * R + row] = v;
  }
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------

namespace {
dim3 row_grid(const DenseView& d) { return dim3((d.S + kDenseRowsPerBlock - 1) / kDenseRowsPerBlock, d.B); }
size_t lds_bytes(int S) { return (size_t)S * sizeof(double); }

// The LDS-staged kernels take up to kDenseLdsMaxStates doubles (64 KiB) of dynamic
// LDS on top of their static words: beyond the default limit, so the attribute is
// raised once per device before the first staged launch.  If the runtime
// refuses it, the in-place (unstaged) kernels run instead: same arithmetic in
// the same order, so the same results, only without the LDS copy.
bool lds_prep() {
  static std::atomic<int> done[64];  // 0 unknown, 1 raised, 2 refused
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return false;
  const int st = done[dev].load(std::memory_order_acquire);
  if (st) return st == 1;
  const int bytes = (int)(kDenseLdsMaxStates * sizeof(double));
  bool ok = true;
  for (const void* fn : {(const void*)&dense_fwd_sweep_kernel<true>, (const void*)&dense_bwd_sweep_kernel<true>,
                         (const void*)&dense_bwd_final_kernel<true>, (const void*)&dense_bellman_sweep_kernel<true>,
                         (const void*)&dense_bellman_finish_kernel<true>})
    ok &= hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes) == hipSuccess;
  if (!ok) (void)hipGetLastError();  // the refusal is handled here; do not leave it for the launch checks
  done[dev].store(ok ? 1 : 2, std::memory_order_release);
  return ok;
}

bool lds_vec(const DenseView& d) { return dense_lds_vec(d) && lds_prep(); }
}  // namespace

void dense_rows_launch(const double* dense, int S, int A, double* P, double* M, hipStream_t st) {
  const size_t n = (size_t)S * S;
  const int blocks = (int)std::min<size_t>((n + 255) / 256, 65536);
  hipLaunchKernelGGL(dense_rows_kernel, dim3(blocks), dim3(256), 0, st, dense, S, A, P, M);
}

void dense_fwd_weights_launch(const DenseView& d, const double* pi, const uint8_t* term, DenseBufs w,
                              hipStream_t st) {
  const int nt = (d.S + 31) / 32;
  hipLaunchKernelGGL(dense_fwd_weights_kernel, dim3(nt, nt, d.B), dim3(256), 0, st, d, pi, term, w.wt);
  hipLaunchKernelGGL(dense_pi_check_kernel, dim3((d.S * d.A + 255) / 256, d.B), dim3(256), 0, st, pi, d.S * d.A,
                     w.bad);
}

void dense_fwd_sweep_launch(const DenseView& d, const double* p0, double eps, long long max_iter, int32_t* status,
                            DenseBufs w, long long it, int r3, hipStream_t st) {
  if (lds_vec(d))
    hipLaunchKernelGGL(dense_fwd_sweep_kernel<true>, row_grid(d), dim3(kDenseThreads), lds_bytes(d.S), st, d, p0, eps,
                       max_iter, status, w, it, r3);
  else
    hipLaunchKernelGGL(dense_fwd_sweep_kernel<false>, row_grid(d), dim3(kDenseThreads), 0, st, d, p0, eps, max_iter,
                       status, w, it, r3);
}

void dense_bwd_init_launch(const DenseView& d, const uint8_t* term, DenseBufs w, hipStream_t st) {
  hipLaunchKernelGGL(dense_bwd_init_kernel, dim3((d.S + 255) / 256, d.B), dim3(256), 0, st, d.S, term, w.buf0);
}

void dense_bwd_sweep_launch(const DenseView& d, const double* reward, int rescale, DenseBufs w, long long it, int r3,
                            hipStream_t st) {
  if (lds_vec(d))
    hipLaunchKernelGGL(dense_bwd_sweep_kernel<true>, row_grid(d), dim3(kDenseThreads), lds_bytes(d.S), st, d, reward,
                       rescale, w, it, r3);
  else
    hipLaunchKernelGGL(dense_bwd_sweep_kernel<false>, row_grid(d), dim3(kDenseThreads), 0, st, d, reward, rescale, w,
                       it, r3);
}

void dense_bwd_gemm_epilogue_launch(const DenseView& d, const double* reward, int rescale, DenseBufs w, long long it,
                                    int r3, hipStream_t st) {
  hipLaunchKernelGGL(dense_bwd_gemm_epilogue_kernel, dim3((d.S + kDenseThreads - 1) / kDenseThreads, d.B),
                     dim3(kDenseThreads), 0, st, d.S, reward, rescale, w, it, r3);
}

void dense_bwd_final_launch(const DenseView& d, const double* reward, int rescale, double* pi, int32_t* status,
                            DenseBufs w, long long collapsed, int r3, hipStream_t st) {
  if (lds_vec(d))
    hipLaunchKernelGGL(dense_bwd_final_kernel<true>, row_grid(d), dim3(kDenseThreads), lds_bytes(d.S), st, d, reward,
                       rescale, pi, status, w, collapsed, r3);
  else
    hipLaunchKernelGGL(dense_bwd_final_kernel<false>, row_grid(d), dim3(kDenseThreads), 0, st, d, reward, rescale,
                       pi, status, w, collapsed, r3);
}

void dense_bellman_sweep_launch(const DenseView& d, const DenseBellman& a, DenseBufs w, long long it, int r3,
                                hipStream_t st) {
  if (lds_vec(d))
    hipLaunchKernelGGL(dense_bellman_sweep_kernel<true>, row_grid(d), dim3(kDenseThreads), lds_bytes(d.S), st, d, a,
                       w, it, r3);
  else
    hipLaunchKernelGGL(dense_bellman_sweep_kernel<false>, row_grid(d), dim3(kDenseThreads), 0, st, d, a, w, it, r3);
}

hipError_t dense_bellman_gemm_sweep_launch(const DenseView& d, const DenseBellman& a, DenseBufs w, long long it,
                                           int r3, hipStream_t st) {
  const double* vin = (it & 1) ? w.buf1 : w.buf0;
  // all actions in one GEMM: the stacked P [A * S][S] times [v_1 .. v_B] -> c[b][a * S + s]
  if (hipError_t e = dense_gemm_launch(d.P, vin, w.wt, d.A * d.S, d.S, d.B, st)) return e;
  hipLaunchKernelGGL(dense_bellman_gemm_epilogue_kernel, dim3((d.S + kDenseThreads - 1) / kDenseThreads, d.B),
                     dim3(kDenseThreads), 0, st, d, a, w, w.wt, it, r3);
  return hipGetLastError();
}

void dense_bellman_finish_launch(const DenseView& d, const DenseBellman& a, DenseBufs w, hipStream_t st) {
  if (lds_vec(d))
    hipLaunchKernelGGL(dense_bellman_finish_kernel<true>, row_grid(d), dim3(kDenseThreads), lds_bytes(d.S), st, d, a,
                       w);
  else
    hipLaunchKernelGGL(dense_bellman_finish_kernel<false>, row_grid(d), dim3(kDenseThreads), 0, st, d, a, w);
}

}  // namespace irlmx

namespace irlmx {

bool dense_lds_vec(const DenseView& d) { return d.S <= kDenseLdsMaxStates && d.B > 1; }

template <int ST, int NBT, int NW>
static hipError_t gemm_go(const double* M, const double* Z, double* C, int R, int S, int B, hipStream_t st) {
  const size_t lds = (size_t)NW * ST * NBT * 4 * kWave * sizeof(double);  // up to 128 KiB (ST 2, NBT 4, 8 waves)
  const void* fn = (S % 2 == 0) ? (const void*)&dense_gemm_kernel<ST, NBT, NW, true>
                                : (const void*)&dense_gemm_kernel<ST, NBT, NW, false>;
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  const dim3 grid((R + 16 * ST - 1) / (16 * ST), (B + 16 * NBT - 1) / (16 * NBT));
  if (S % 2 == 0)
    hipLaunchKernelGGL((dense_gemm_kernel<ST, NBT, NW, true>), grid, dim3(NW * kWave), lds, st, M, Z, C, R, S, B);
  else
    hipLaunchKernelGGL((dense_gemm_kernel<ST, NBT, NW, false>), grid, dim3(NW * kWave), lds, st, M, Z, C, R, S, B);
  return hipGetLastError();
}

template <int ST, int NBT>
static hipError_t gemm_waves(const double* M, const double* Z, double* C, int R, int S, int B, hipStream_t st) {
  const long long wgs = (long long)((R + 16 * ST - 1) / (16 * ST)) * ((B + 16 * NBT - 1) / (16 * NBT));
  if (wgs >= 512) return gemm_go<ST, NBT, 4>(M, Z, C, R, S, B, st);  // several workgroups per CU
  return gemm_go<ST, NBT, 8>(M, Z, C, R, S, B, st);
}

// Tiles per workgroup (ST row tiles x NBT instance tiles of 16): the largest,
// squarest workgroup tile that still gives >= 256 workgroups (one per CU) --
// a workgroup reads 16 (ST + NBT) rows of M and Z per K chunk for 256 ST NBT
// outputs, so a 32 x 32 tile moves the least (S = 4096, B = 64: 2 x 2 tiles
// 69 us vs 1 x 4 81 us; S = 2048, B = 64: 2 x 1 26 us vs 1 x 4 on half the CUs
// 41 us, profiles/r03_dense_gemm_tiles.txt); else the most workgroups (1 x 1).
// IRLMX_GEMM_NBT forces the instance tiles (diagnostics).
static void gemm_tiles(int R, int B, int* st, int* nbt) {
  const int rt = (R + 15) / 16, ct = (B + 15) / 16;
  const char* f = getenv("IRLMX_GEMM_NBT");
  const int forced = (f && (*f == '1' || *f == '2' || *f == '4') && f[1] == 0) ? *f - '0' : 0;
  static const int cands[][2] = {{2, 4}, {2, 2}, {1, 4}, {2, 1}, {1, 2}, {1, 1}};
  for (const auto& c : cands) {
    if (forced ? c[1] != forced : (c[1] > ct || c[0] > rt)) continue;
    if ((long long)((rt + c[0] - 1) / c[0]) * ((ct + c[1] - 1) / c[1]) >= 256 || (c[0] == 1 && (forced || c[1] == 1))) {
      *st = c[0];
      *nbt = c[1];
      return;
    }
  }
  *st = 1;
  *nbt = forced ? forced : 1;
}

template <int ST>
static hipError_t gemm_nbt_go(int nbt, const double* M, const double* Z, double* C, int R, int S, int B,
                              hipStream_t st) {
  if (nbt == 1) return gemm_waves<ST, 1>(M, Z, C, R, S, B, st);
  if (nbt == 2) return gemm_waves<ST, 2>(M, Z, C, R, S, B, st);
  return gemm_waves<ST, 4>(M, Z, C, R, S, B, st);
}

hipError_t dense_gemm_launch(const double* M, const double* Z, double* C, int R, int S, int B, hipStream_t st) {
  int ts = 1, nbt = 1;
  gemm_tiles(R, B, &ts, &nbt);
  return ts == 2 ? gemm_nbt_go<2>(nbt, M, Z, C, R, S, B, st) : gemm_nbt_go<1>(nbt, M, Z, C, R, S, B, st);
}

// the kernel variant a launch of these sizes runs: {ST, NBT, waves, V2}
void dense_gemm_variant(int R, int S, int B, int* out) {
  int ts = 1, nbt = 1;
  gemm_tiles(R, B, &ts, &nbt);
  const long long wgs = (long long)((R + 16 * ts - 1) / (16 * ts)) * ((B + 16 * nbt - 1) / (16 * nbt));
  out[0] = ts;
  out[1] = nbt;
  out[2] = wgs >= 512 ? 4 : 8;
  out[3] = S % 2 == 0 ? 1 : 0;
}

}  // namespace irlmx
