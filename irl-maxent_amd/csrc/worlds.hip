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
  if (size <= 0 || batch <= 0 || !p_slip || !row_val) { set_error("build_icy_gridworld: bad arguments"); return IRLMX_EINVAL; }
  const int S = size * size;
  hipLaunchKernelGGL(icy_gridworld_kernel, dim3((S + 255) / 256, batch), dim3(256), 0, (hipStream_t)stream, size,
                     p_slip, row_val);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : hip_fail(e, "icy_gridworld_kernel");
}

extern "C" int irlmx_build_gridworld(int32_t size, int32_t batch, double* row_val, void* stream) {
  if (size <= 0 || batch <= 0 || !row_val) { set_error("build_gridworld: bad arguments"); return IRLMX_EINVAL; }
  const int S = size * size;
  hipLaunchKernelGGL(gridworld_kernel, dim3((S + 255) / 256, batch), dim3(256), 0, (hipStream_t)stream, size, row_val);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : hip_fail(e, "gridworld_kernel");
}

extern "C" int irlmx_dense_to_stencil(const double* dense, int32_t width, int32_t height, int32_t n_actions,
                                      double* row_val, int32_t* off_stencil, void* stream) {
  if (width <= 0 || height <= 0 || n_actions <= 0 || !dense || !row_val || !off_stencil) {
    set_error("dense_to_stencil: bad arguments");
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
    set_error("optimal_policy: bad arguments");
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
    set_error("stochastic_policy: bad arguments");
    return IRLMX_EINVAL;
  }
  hipLaunchKernelGGL(stochastic_policy_kernel, dim3((n_states + 255) / 256, batch), dim3(256), 0,
                     (hipStream_t)stream, successor, n_states, n_actions, weighted_value, p_policy);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : hip_fail(e, "stochastic_policy_kernel");
}
