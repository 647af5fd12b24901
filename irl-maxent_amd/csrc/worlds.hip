// Gridworld transition tables and policy extraction on the device.
//
// The reference builds P[from, to, action] with a Python loop over S*S*A calls
// (gridworld.py:136-140) -- about ten minutes at 128x128 and infeasible at
// 256x256.  The builders here emit the STENCIL5 row form directly:
//   row_val[b][a][k][s] = P[s, nbr_k(s), a],  k = self, +x, -x, +y, -y.
// Every value is produced by the same float64 expression as
// IcyGridWorld._transition_prob (gridworld.py:200-248), with floating-point
// contraction disabled, so the tables are bit-identical to the reference's.

#include <hip/hip_runtime.h>

#include <algorithm>

#include "common.h"

namespace irlmx {

// largest grid side / state count the 32-bit state indices of the kernels cover
constexpr int kMaxSide = 46340;                    // size * size < 2^31
constexpr long long kMaxStates = 46340LL * 46340LL;
void set_error(const char* fmt, ...);
int hip_fail(hipError_t e, const char* what);

// action offsets, gridworld.py:47
__device__ __constant__ int kActDx[4] = {1, -1, 0, 0};
__device__ __constant__ int kActDy[4] = {0, 0, 1, -1};

#pragma clang fp contract(off)
__global__ void icy_gridworld_kernel(int size, const double* __restrict__ p_slip, double* __restrict__ out) {
  const int S = size * size;
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (s >= S) return;
  const double p = p_slip[b];
  const int na = 4;
  const int fx = s % size, fy = s / size;
  const bool inner_x = 0 < fx && fx < size - 1;
  const bool inner_y = 0 < fy && fy < size - 1;
  for (int a = 0; a < na; ++a) {
    const int ax = kActDx[a], ay = kActDy[a];
    double* o = out + ((size_t)b * na + a) * kStencilK * S;
    // k = 0: staying in place (gridworld.py:226-245)
    double stay;
    const bool over = !(0 <= fx + ax && fx + ax < size) || !(0 <= fy + ay && fy + ay < size);
    if (over) {
      if (!inner_x && !inner_y) stay = 1.0 - p + 2.0 * p / na;
      else stay = 1.0 - p + p / na;
    } else if (!inner_x && !inner_y) {
      stay = 2.0 * p / na;
    } else if (!inner_x || !inner_y) {
      stay = p / na;
    } else {
      stay = 0.0;
    }
    o[s] = stay;
    // k = 1..4: the four neighbours, intended (gridworld.py:219) or slipped into (:223)
    for (int k = 1; k < kStencilK; ++k) {
      const int tx = fx + kActDx[k - 1], ty = fy + kActDy[k - 1];
      double v = 0.0;
      if (0 <= tx && tx < size && 0 <= ty && ty < size)
        v = (k - 1 == a) ? 1.0 - p + p / na : p / na;
      o[(size_t)k * S + s] = v;
    }
  }
}
#pragma clang fp contract(on)

__global__ void gridworld_kernel(int size, double* __restrict__ out) {
  const int S = size * size;
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (s >= S) return;
  const int fx = s % size, fy = s / size;
  for (int a = 0; a < 4; ++a) {
    double* o = out + ((size_t)b * 4 + a) * kStencilK * S;
    const int tx = fx + kActDx[a], ty = fy + kActDy[a];
    const bool inside = 0 <= tx && tx < size && 0 <= ty && ty < size;
    o[s] = inside ? 0.0 : 1.0;  // gridworld.py:166-168
    for (int k = 1; k < kStencilK; ++k) o[(size_t)k * S + s] = (inside && k - 1 == a) ? 1.0 : 0.0;
  }
}

// dense [S][S][A] -> STENCIL5 row form; one thread per dense element, so the
// read of the dense table is fully coalesced.
__global__ void dense_to_stencil_kernel(const double* __restrict__ dense, int width, int height, int A,
                                        double* __restrict__ out, int32_t* __restrict__ off_stencil) {
  const long long S = (long long)width * height;
  const long long n = S * S * A;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const double v = dense[i];
    if (v == 0.0) continue;
    const int a = (int)(i % A);
    const long long st = i / A;
    const int t = (int)(st % S), s = (int)(st / S);
    const int sx = s % width, sy = s / width, tx = t % width, ty = t / width;
    const int dx = tx - sx, dy = ty - sy;
    int k = -1;
    if (dx == 0 && dy == 0) k = 0;
    else if (dx == 1 && dy == 0) k = 1;
    else if (dx == -1 && dy == 0) k = 2;
    else if (dx == 0 && dy == 1) k = 3;
    else if (dx == 0 && dy == -1) k = 4;
    if (k < 0) { atomicOr(off_stencil, 1); continue; }
    out[((size_t)a * kStencilK + k) * S + s] = v;
  }
}

__global__ void optimal_policy_kernel(const int32_t* __restrict__ succ, int S, int A,
                                      const double* __restrict__ value, int64_t* __restrict__ policy) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (s >= S) return;
  const double* v = value + (size_t)b * S;
  const int32_t* row = succ + (size_t)s * A;
  // np.argmax: first maximum; a NaN counts as the maximum and the first NaN wins
  int best = 0;
  double bv = v[row[0]];
  for (int a = 1; a < A; ++a) {
    if (bv != bv) break;
    const double x = v[row[a]];
    if (x > bv || x != x) { best = a; bv = x; }
  }
  policy[(size_t)b * S + s] = best;
}

__global__ void stochastic_policy_kernel(const int32_t* __restrict__ succ, int S, int A,
                                         const double* __restrict__ wv, double* __restrict__ out) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (s >= S) return;
  const double* v = wv + (size_t)b * S;
  const int32_t* row = succ + (size_t)s * A;
  double sum = 0.0;  // np.sum over a row of < 8 entries adds sequentially
  for (int a = 0; a < A; ++a) sum += v[row[a]];
  for (int a = 0; a < A; ++a) out[((size_t)b * S + s) * A + a] = v[row[a]] / sum;  // solver.py:181
}

}  // namespace irlmx

using namespace irlmx;

extern "C" int irlmx_build_icy_gridworld(int32_t size, const double* p_slip, int32_t batch, double* row_val,
                                         void* stream) {
  if (size <= 0 || size > kMaxSide || batch <= 0 || !p_slip || !row_val) {
    set_error("build_icy_gridworld: bad arguments (size=%d, batch=%d, p_slip %s, row_val %s)", size, batch,
              p_slip ? "set" : "NULL", row_val ? "set" : "NULL");
    return IRLMX_EINVAL;
  }
  const int S = size * size;
  hipLaunchKernelGGL(icy_gridworld_kernel, dim3((S + 255) / 256, batch), dim3(256), 0, (hipStream_t)stream, size,
                     p_slip, row_val);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : hip_fail(e, "icy_gridworld_kernel");
}

extern "C" int irlmx_build_gridworld(int32_t size, int32_t batch, double* row_val, void* stream) {
  if (size <= 0 || size > kMaxSide || batch <= 0 || !row_val) {
    set_error("build_gridworld: bad arguments (size=%d, batch=%d, row_val %s)", size, batch, row_val ? "set" : "NULL");
    return IRLMX_EINVAL;
  }
  const int S = size * size;
  hipLaunchKernelGGL(gridworld_kernel, dim3((S + 255) / 256, batch), dim3(256), 0, (hipStream_t)stream, size, row_val);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : hip_fail(e, "gridworld_kernel");
}

extern "C" int irlmx_dense_to_stencil(const double* dense, int32_t width, int32_t height, int32_t n_actions,
                                      double* row_val, int32_t* off_stencil, void* stream) {
  if (width <= 0 || height <= 0 || (long long)width * height > kMaxStates || n_actions <= 0 || !dense || !row_val ||
      !off_stencil) {
    set_error("dense_to_stencil: bad arguments (width=%d, height=%d, n_actions=%d, dense %s, row_val %s, "
              "off_stencil %s)", width, height, n_actions, dense ? "set" : "NULL", row_val ? "set" : "NULL",
              off_stencil ? "set" : "NULL");
    return IRLMX_EINVAL;
  }
  hipStream_t st = (hipStream_t)stream;
  const size_t S = (size_t)width * height;
  hipError_t e = hipMemsetAsync(row_val, 0, sizeof(double) * n_actions * kStencilK * S, st);
  if (e == hipSuccess) e = hipMemsetAsync(off_stencil, 0, sizeof(int32_t), st);
  if (e != hipSuccess) return hip_fail(e, "memset");
  const long long n = (long long)S * S * n_actions;
  const long long blocks = std::min<long long>((n + 255) / 256, 256 * 64);
  hipLaunchKernelGGL(dense_to_stencil_kernel, dim3((unsigned)blocks), dim3(256), 0, st, dense, width, height,
                     n_actions, row_val, off_stencil);
  e = hipGetLastError();
  return e == hipSuccess ? 0 : hip_fail(e, "dense_to_stencil_kernel");
}

extern "C" int irlmx_optimal_policy(const int32_t* successor, int32_t n_states, int32_t n_actions, int32_t batch,
                                    const double* value, int64_t* policy, void* stream) {
  if (n_states <= 0 || n_actions <= 0 || batch <= 0 || !successor || !value || !policy) {
    set_error("optimal_policy: bad arguments (n_states=%d, n_actions=%d, batch=%d, successor %s, value %s, "
              "policy %s)", n_states, n_actions, batch, successor ? "set" : "NULL", value ? "set" : "NULL",
              policy ? "set" : "NULL");
    return IRLMX_EINVAL;
  }
  hipLaunchKernelGGL(optimal_policy_kernel, dim3((n_states + 255) / 256, batch), dim3(256), 0, (hipStream_t)stream,
                     successor, n_states, n_actions, value, policy);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : hip_fail(e, "optimal_policy_kernel");
}

extern "C" int irlmx_stochastic_policy(const int32_t* successor, int32_t n_states, int32_t n_actions, int32_t batch,
                                       const double* weighted_value, double* p_policy, void* stream) {
  if (n_states <= 0 || n_actions <= 0 || batch <= 0 || !successor || !weighted_value || !p_policy) {
    set_error("stochastic_policy: bad arguments (n_states=%d, n_actions=%d, batch=%d, successor %s, "
              "weighted_value %s, p_policy %s)", n_states, n_actions, batch, successor ? "set" : "NULL",
              weighted_value ? "set" : "NULL", p_policy ? "set" : "NULL");
    return IRLMX_EINVAL;
  }
  hipLaunchKernelGGL(stochastic_policy_kernel, dim3((n_states + 255) / 256, batch), dim3(256), 0,
                     (hipStream_t)stream, successor, n_states, n_actions, weighted_value, p_policy);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : hip_fail(e, "stochastic_policy_kernel");
}

// ---------------------------------------------------------------------------
// Dense [S][S][A] -> ELL row and column forms (any sparsity), on the device.
// Replaces the host-side conversion a dense upload of a non-grid MDP needed
// (maxent.py callers pass the reference's dense p_transition, maxent.py:98-102,
// 143).  Layout (include/irlmx.h): row form = per source state the union over
// actions of its targets, ascending; column form = per target the union of its
// sources, ascending; unused slots point at the state itself with value 0.
// ---------------------------------------------------------------------------

namespace irlmx {

// Does (s, t) carry a nonzero for some action?
__device__ inline bool ell_nz(const double* __restrict__ dense, size_t S, int A, size_t s, size_t t) {
  const double* p = dense + (s * S + t) * A;
  bool nz = false;
  for (int a = 0; a < A; ++a) nz |= p[a] != 0.0;
  return nz;
}

// One wave per source row: union sizes per row (max into k[0]) and per-target
// counts (col_count, summed over rows; its max is taken by ell_colmax_kernel).
__global__ void ell_count_kernel(const double* __restrict__ dense, int S, int A, int32_t* __restrict__ k,
                                 int32_t* __restrict__ col_count) {
  const int lane = threadIdx.x & (kWave - 1);
  const int s = blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave;
  if (s >= S) return;
  int cnt = 0;
  for (int t0 = 0; t0 < S; t0 += kWave) {
    const int t = t0 + lane;
    const bool nz = t < S && ell_nz(dense, (size_t)S, A, (size_t)s, (size_t)t);
    if (nz) atomicAdd(&col_count[t], 1);
    cnt += __popcll(__ballot(nz));
  }
  if (lane == 0) atomicMax(&k[0], cnt);
}

__global__ void ell_colmax_kernel(const int32_t* __restrict__ col_count, int S, int32_t* __restrict__ k) {
  int m = 0;
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < S; t += gridDim.x * blockDim.x) m = max(m, col_count[t]);
  atomicMax(&k[1], m);
}

// Row form: one wave per source row, slots assigned in ascending target order
// by a ballot prefix count.
__global__ void ell_rows_kernel(const double* __restrict__ dense, int S, int A, int K,
                                int32_t* __restrict__ row_idx, double* __restrict__ row_val) {
  const int lane = threadIdx.x & (kWave - 1);
  const int s = blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave;
  if (s >= S) return;
  int base = 0;
  for (int t0 = 0; t0 < S; t0 += kWave) {
    const int t = t0 + lane;
    const bool nz = t < S && ell_nz(dense, (size_t)S, A, (size_t)s, (size_t)t);
    const unsigned long long mask = __ballot(nz);
    if (nz) {
      const int slot = base + __popcll(mask & ((1ull << lane) - 1ull));
      row_idx[(size_t)slot * S + s] = t;
      for (int a = 0; a < A; ++a) row_val[((size_t)a * K + slot) * S + s] = dense[((size_t)s * S + t) * A + a];
    }
    base += __popcll(mask);
  }
  for (int slot = base + lane; slot < K; slot += kWave) {  // padding: self, value 0
    row_idx[(size_t)slot * S + s] = s;
    for (int a = 0; a < A; ++a) row_val[((size_t)a * K + slot) * S + s] = 0.0;
  }
}

// Column form: one thread per target column, scanning sources in ascending
// order (neighbouring lanes read neighbouring columns: coalesced).
__global__ void ell_cols_kernel(const double* __restrict__ dense, int S, int A, int K,
                                int32_t* __restrict__ col_idx, double* __restrict__ col_val) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= S) return;
  int slot = 0;
  for (int s = 0; s < S; ++s) {
    if (!ell_nz(dense, (size_t)S, A, (size_t)s, (size_t)t)) continue;
    col_idx[(size_t)slot * S + t] = s;
    for (int a = 0; a < A; ++a) col_val[((size_t)a * K + slot) * S + t] = dense[((size_t)s * S + t) * A + a];
    ++slot;
  }
  for (; slot < K; ++slot) {
    col_idx[(size_t)slot * S + t] = t;
    for (int a = 0; a < A; ++a) col_val[((size_t)a * K + slot) * S + t] = 0.0;
  }
}

}  // namespace irlmx

extern "C" int irlmx_dense_ell_sizes(const double* dense, int32_t n_states, int32_t n_actions, int32_t* k_out,
                                     int32_t* col_count, void* stream) {
  if (n_states <= 0 || n_states > kMaxStates || n_actions <= 0 || !dense || !k_out || !col_count) {
    set_error("dense_ell_sizes: bad arguments (n_states=%d, n_actions=%d, dense %s, k_out %s, col_count %s)",
              n_states, n_actions, dense ? "set" : "NULL", k_out ? "set" : "NULL", col_count ? "set" : "NULL");
    return IRLMX_EINVAL;
  }
  hipStream_t st = (hipStream_t)stream;
  hipError_t e = hipMemsetAsync(k_out, 0, 2 * sizeof(int32_t), st);
  if (e == hipSuccess) e = hipMemsetAsync(col_count, 0, sizeof(int32_t) * (size_t)n_states, st);
  if (e != hipSuccess) return hip_fail(e, "memset");
  const int rows_per_block = 256 / kWave;
  hipLaunchKernelGGL(ell_count_kernel, dim3((n_states + rows_per_block - 1) / rows_per_block), dim3(256), 0, st,
                     dense, n_states, n_actions, k_out, col_count);
  hipLaunchKernelGGL(ell_colmax_kernel, dim3(std::min(256, (n_states + 255) / 256)), dim3(256), 0, st, col_count,
                     n_states, k_out);
  e = hipGetLastError();
  return e == hipSuccess ? 0 : hip_fail(e, "ell_count_kernel");
}

extern "C" int irlmx_dense_to_ell(const double* dense, int32_t n_states, int32_t n_actions, int32_t k_row,
                                  int32_t k_col, int32_t* row_idx, double* row_val, int32_t* col_idx,
                                  double* col_val, void* stream) {
  if (n_states <= 0 || n_states > kMaxStates || n_actions <= 0 || k_row <= 0 || k_col <= 0 || k_row > n_states ||
      k_col > n_states || !dense || !row_idx || !row_val || !col_idx || !col_val) {
    set_error("dense_to_ell: bad arguments (n_states=%d, n_actions=%d, k_row=%d, k_col=%d; k in 1..n_states, "
              "every array non-NULL)", n_states, n_actions, k_row, k_col);
    return IRLMX_EINVAL;
  }
  hipStream_t st = (hipStream_t)stream;
  const int rows_per_block = 256 / kWave;
  hipLaunchKernelGGL(ell_rows_kernel, dim3((n_states + rows_per_block - 1) / rows_per_block), dim3(256), 0, st,
                     dense, n_states, n_actions, k_row, row_idx, row_val);
  hipLaunchKernelGGL(ell_cols_kernel, dim3((n_states + 255) / 256), dim3(256), 0, st, dense, n_states, n_actions,
                     k_col, col_idx, col_val);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : hip_fail(e, "dense_to_ell kernels");
}
