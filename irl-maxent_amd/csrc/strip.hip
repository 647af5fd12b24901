// Register-resident variant of the cluster kernel (cluster.hip) for grids whose
// width is 64, 128 or 256 states: the same tiles, ghost rows, blocks of sweeps,
// halo exchange and exact in-block rollback, but the state vector lives in
// registers instead of two LDS ping-pong buffers.
//
// Thread map.  Wave b of the 16 is band b of the extended tile: RPT
// consecutive rows.  Lane i holds columns i, i + 64, ... (CPL = W / 64 of
// them) of those rows, so a wave spans whole rows and a thread owns
// SPT = RPT * CPL states, with their five stencil weights, c0 and the current
// value in registers.  One sweep:
//   * horizontal neighbours: DPP wave shifts of the row's values -- wave_shr1 /
//     wave_shl1 for the same column slot, wave_ror1 / wave_rol1 for the lane-0
//     / lane-63 seam between slots; bound_ctrl zero-fills the grid edges;
//   * vertical neighbours: the thread's own registers inside its strip; the
//     rows above and below the strip are the neighbouring bands' last / first
//     rows, exchanged through a small double-buffered LDS array (one barrier
//     per sweep);
//   * the update is in place, row by row, keeping the previous row's old value.
// Per sweep and thread that is 2*CPL LDS writes + 2*CPL LDS reads instead of
// six LDS accesses per state.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>

#include "cluster.h"
#include "common.h"

namespace irlmx {

void set_error(const char* fmt, ...);
int hip_fail(hipError_t e, const char* what);

template <int CTRL>
__device__ inline double dpp_f64(double x) {
  const long long b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffLL), CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, true);
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}
constexpr int kDppShl1 = 0x130;  // lane i <- lane i + 1, lane 63 <- 0
constexpr int kDppRol1 = 0x134;  // lane 63 <- lane 0
constexpr int kDppShr1 = 0x138;  // lane i <- lane i - 1, lane 0 <- 0
constexpr int kDppRor1 = 0x13C;  // lane 0 <- lane 63

template <int MODE, int CPL, int RPT, int NT>
__global__ void __launch_bounds__(NT) strip_kernel(ClusterArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int W = 64 * CPL;
  constexpr int NB = NT / kWave;  // bands
  const int H = a.H, S = a.S;
  const int tile = blockIdx.x % a.C;
  const int inst = a.b0 + blockIdx.x / a.C;
  const int tid = threadIdx.x;
  const int band = tid / kWave, lane = tid & (kWave - 1);
  const int r0 = tile * a.R, r1 = min(H, r0 + a.R);
  const int e0 = max(0, r0 - a.G), e1 = min(H, r1 + a.G);
  const int Erows = e1 - e0;
  const int own0 = r0 - e0, own1 = r1 - e0;                 // owned ext rows
  const int pubA1 = min(own1, own0 + a.G), pubB0 = max(pubA1, own1 - a.G);
  const int base = e0 * W;
  const int row0 = band * RPT;                              // first ext row of this thread
  double* xtop = (double*)smem;                             // [2][NB][W]
  double* xbot = xtop + 2 * NB * W;                         // [2][NB][W]
  double* full = xbot + 2 * NB * W;                         // forward snapshot / backward final [emax + 2 pad]
  unsigned long long* red = (unsigned long long*)(full + a.emax + 2 * (W + 1));  // [2]
  int* lflag = (int*)(red + 2);

  const size_t iS = (size_t)inst * S;
  if (MODE == kModeFwd && a.bad[inst]) {
    for (int l = own0 * W + tid; l < own1 * W; l += NT) a.out[iS + base + l] = __longlong_as_double(0x7ff8000000000000LL);
    if (tile == 0 && tid == 0) { a.iters[inst] = 1; a.status[inst] = IRLMX_NONFINITE; }
    return;
  }

  double w[RPT][CPL][kStencilK];
  double c0[RPT][CPL];
  double v[RPT][CPL];
  const size_t wbase = (MODE == kModeBwd && a.tab_shared) ? 0 : iS * kStencilK;
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    const int row = row0 + r;
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      c0[r][c] = 0.0;
      v[r][c] = 0.0;
#pragma unroll
      for (int k = 0; k < kStencilK; ++k) w[r][c][k] = 0.0;
      if (row < Erows) {
        const int s = base + row * W + lane + 64 * c;
        c0[r][c] = MODE == kModeFwd ? a.vin[iS + s] : exp(a.vin[iS + s]);
        if (MODE == kModeBwd) v[r][c] = a.term[iS + s] ? 1.0 : 0.0;
#pragma unroll
        for (int k = 0; k < kStencilK; ++k) w[r][c][k] = a.wgt[wbase + (size_t)k * S + s];
      }
#pragma unroll
      for (int k = 0; k < kStencilK; ++k) asm volatile("" : "+v"(w[r][c][k]));
      asm volatile("" : "+v"(c0[r][c]));
    }
  }
  if (MODE == kModeFwd)
    for (int l = tid; l < Erows * W; l += NT) full[l] = 0.0;  // block-0 snapshot: d = 0
  if (tid < 2) red[tid] = 0ull;
  if (tid == 0) lflag[0] = 0;

  int T = a.T;
  if (MODE == kModeBwd) {
    const double g = bits_double(a.growth[inst]);
    if (a.rescale && g > 2.0 && isfinite(g)) {
      const int cap = (int)floor(900.0 / log2(g)) - 1;
      T = max(1, min(T, cap));
    }
  }
  __syncthreads();

  const double eps = a.eps;
  int par = 0;
  auto sweep = [&](int i, unsigned& flags, bool want_max) {
    unsigned long long mx = 0ull;
    double* xt = xtop + par * NB * W;
    double* xb = xbot + par * NB * W;
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      xt[band * W + lane + 64 * c] = v[0][c];
      xb[band * W + lane + 64 * c] = v[RPT - 1][c];
    }
    __syncthreads();
    double up[CPL], dn[CPL];
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      up[c] = band > 0 ? xb[(band - 1) * W + lane + 64 * c] : 0.0;
      dn[c] = band < NB - 1 ? xt[(band + 1) * W + lane + 64 * c] : 0.0;
    }
    double prev[CPL];
#pragma unroll
    for (int c = 0; c < CPL; ++c) prev[c] = up[c];
#pragma unroll
    for (int r = 0; r < RPT; ++r) {
      double L[CPL], Rr[CPL];
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        double l = dpp_f64<kDppShr1>(v[r][c]);
        double rr = dpp_f64<kDppShl1>(v[r][c]);
        if (c > 0) {  // lane 0 of slot c: column 64c - 1 = lane 63 of slot c - 1
          const double seam = dpp_f64<kDppRor1>(v[r][c - 1]);
          l = lane == 0 ? seam : l;
        }
        if (c < CPL - 1) {  // lane 63 of slot c: column 64c + 64 = lane 0 of slot c + 1
          const double seam = dpp_f64<kDppRol1>(v[r][c + 1]);
          rr = lane == kWave - 1 ? seam : rr;
        }
        L[c] = l;
        Rr[c] = rr;
      }
      const bool owned = row0 + r >= own0 && row0 + r < own1;
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        const double self = v[r][c];
        const double down = r == RPT - 1 ? dn[c] : v[r + 1][c];
        double acc = fma(w[r][c][0], self, 0.0);
        acc = fma(w[r][c][1], Rr[c], acc);
        acc = fma(w[r][c][2], L[c], acc);
        acc = fma(w[r][c][3], down, acc);
        acc = fma(w[r][c][4], prev[c], acc);
        const double nv = MODE == kModeFwd ? c0[r][c] + acc : c0[r][c] * acc;
        prev[c] = self;
        v[r][c] = nv;
        if (owned) {
          if (MODE == kModeFwd) {
            const double d = fabs(nv - self);
            flags |= ((d > eps) ? 1u : 0u) << i;
            flags |= ((d != d) ? 1u : 0u) << (16 + i);
          } else if (want_max) {
            const unsigned long long d = abs_bits(nv);
            mx = d > mx ? d : mx;
          }
        }
      }
    }
    par ^= 1;
    return mx;
  };

  unsigned int* slots = (unsigned int*)(a.slots + (size_t)inst * 3 * kTMax);
  unsigned long long* slots64 = a.slots + (size_t)inst * 3 * kTMax;
  const size_t pubStride = (size_t)a.btot * S;
  long long done = 0;
  const long long total = MODE == kModeBwd ? a.n_sweeps : -1;
  unsigned long long st_acc[5] = {0, 0, 0, 0, 0};
  const bool stamps = a.stamps != nullptr && tid == 0;
  unsigned long long ts = stamps ? stamp_now() : 0;
  auto stamp = [&](int k) {
    if (stamps) { const unsigned long long t = stamp_now(); st_acc[k] += t - ts; ts = t; }
  };
  auto stamp_flush = [&]() {
    if (stamps) for (int k = 0; k < 5; ++k) a.stamps[(size_t)blockIdx.x * 8 + k] = st_acc[k];
  };

  for (int m = 0;; ++m) {
    int Tm = T;
    if (MODE == kModeBwd) Tm = (int)min<long long>((long long)T, total - done);
    unsigned flags = 0;
    unsigned long long mx = 0ull;
    for (int i = 0; i < Tm; ++i) mx = sweep(i, flags, i == Tm - 1);
    stamp(0);
    if (stamps) st_acc[4] += 1;
    if (MODE == kModeFwd) {
      const unsigned wf = wave_or_bits(flags, 16 + Tm) & (((1u << Tm) - 1) | (((1u << Tm) - 1) << 16));
      if (lane == 0 && wf) atomicOr((unsigned*)&red[m & 1], wf);
    } else if (a.rescale) {
      mx = wave_max_u64(mx);
      if (lane == 0 && mx) atomicMax(&red[m & 1], mx);
    }
    double* pubm = a.pub + (size_t)(m & 1) * pubStride + iS;
#pragma unroll
    for (int r = 0; r < RPT; ++r) {
      const int row = row0 + r;
      if ((row >= own0 && row < pubA1) || (row >= pubB0 && row < own1)) {
#pragma unroll
        for (int c = 0; c < CPL; ++c) st_sc1(&pubm[base + row * W + lane + 64 * c], v[r][c]);
      }
    }
    __syncthreads();
    if (tid == 0) {
      const unsigned long long s = red[m & 1];
      if (MODE == kModeFwd) {
        if (s) atomicOr(&slots[m % 3], (unsigned)s);
      } else if (s) {
        atomicMax(&slots64[(m % 3) + 3], s);
      }
      if (tile == 0) {
        __hip_atomic_store(&slots[(m + 1) % 3], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&slots64[((m + 1) % 3) + 3], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    stamp(1);
    if (!instance_barrier(&a.counter[inst], (unsigned)(a.C * (m + 1)), a.err, &lflag[0])) return;
    stamp(2);
    if (tid == 0) red[(m + 1) & 1] = 0ull;
    if (MODE == kModeFwd) {
      const unsigned msk = __hip_atomic_load(&slots[m % 3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      int conv = 0;
      bool nan_stop = false;
      for (int i = 0; i < Tm; ++i) {
        const bool cap = a.max_iter > 0 && done + i + 1 >= a.max_iter;
        nan_stop = (msk >> (16 + i)) & 1u;
        if (nan_stop || !((msk >> i) & 1u) || cap) { conv = i + 1; break; }
      }
      if (conv) {
        // exact stop inside the block: replay `conv` sweeps from the block-start snapshot
#pragma unroll
        for (int r = 0; r < RPT; ++r)
#pragma unroll
          for (int c = 0; c < CPL; ++c)
            v[r][c] = row0 + r < Erows ? full[(row0 + r) * W + lane + 64 * c] : 0.0;
        unsigned scratch = 0;
        for (int i = 0; i < conv; ++i) sweep(i, scratch, false);
#pragma unroll
        for (int r = 0; r < RPT; ++r) {
          const int row = row0 + r;
          if (row >= own0 && row < own1)
#pragma unroll
            for (int c = 0; c < CPL; ++c) a.out[iS + base + row * W + lane + 64 * c] = v[r][c];
        }
        stamp(3);
        stamp_flush();
        if (tile == 0 && tid == 0) {
          const bool big = (msk >> (conv - 1)) & 1u;
          a.iters[inst] = done + conv;
          a.status[inst] = nan_stop ? IRLMX_NONFINITE : (big ? IRLMX_MAXITER : IRLMX_OK);
        }
        return;
      }
    }
    done += Tm;
    int e_scale = 0;
    if (MODE == kModeBwd && a.rescale)
      e_scale = rescale_exponent(bits_double(
          __hip_atomic_load(&slots64[(m % 3) + 3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)));
#pragma unroll
    for (int r = 0; r < RPT; ++r) {
      const int row = row0 + r;
      if (row < Erows) {
        const bool ghost = row < own0 || row >= own1;
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
          const int l = row * W + lane + 64 * c;
          double x = ghost ? ld_sc1(&pubm[base + l]) : v[r][c];
          if (MODE == kModeBwd && e_scale) x = ldexp(x, e_scale);
          v[r][c] = x;
          if (MODE == kModeFwd) full[l] = x;  // block-start snapshot for an exact rollback
        }
      }
    }
    __syncthreads();
    stamp(3);
    if (MODE == kModeBwd && done >= total) break;
  }
  stamp_flush();

  if (MODE == kModeBwd) {
    // last of the 2*S sweeps, per action, from a padded LDS copy of the state
    const int pad = W + 1;
    for (int i = tid; i < Erows * W + 2 * pad; i += NT) full[i] = 0.0;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < RPT; ++r)
      if (row0 + r < Erows)
#pragma unroll
        for (int c = 0; c < CPL; ++c) full[pad + (row0 + r) * W + lane + 64 * c] = v[r][c];
    __syncthreads();
    const int A = a.A;
    const size_t tb = a.tab_shared ? 0 : (size_t)inst;
    for (int l = own0 * W + tid; l < own1 * W; l += NT) {
      const int s = base + l;
      const double* q = full + l + 1;
      const double er = exp(a.vin[iS + s]);
      double za[8];
      double zsum = 0.0;
      for (int act = 0; act < A; ++act) {
        const double* rv = a.row_val + ((tb * A + act) * kStencilK) * (size_t)S + s;
        double acc = fma(rv[0], q[W], 0.0);
        acc = fma(rv[(size_t)1 * S], q[W + 1], acc);
        acc = fma(rv[(size_t)2 * S], q[W - 1], acc);
        acc = fma(rv[(size_t)3 * S], q[2 * W], acc);
        acc = fma(rv[(size_t)4 * S], q[0], acc);
        za[act] = er * acc;
        zsum += za[act];
      }
      for (int act = 0; act < A; ++act) a.out[(iS + s) * A + act] = za[act] / zsum;
    }
    if (tile == 0 && tid == 0) a.status[inst] = IRLMX_OK;
  }
}

size_t strip_lds(int W, int emax, int nt) {
  return (size_t)4 * (nt / kWave) * W * sizeof(double) + (size_t)(emax + 2 * (W + 1)) * sizeof(double) + 64;
}

// (CPL, RPT) shapes with 512-thread workgroups (8 bands): every listed shape
// compiles without VGPR spills (tools/kernel_resources.py).
template <int MODE>
void* strip_fn(int cpl, int rpt) {
#define IRLMX_STRIP(C_, R_) if (cpl == C_ && rpt == R_) return (void*)&strip_kernel<MODE, C_, R_, kStripThreads>;
  IRLMX_STRIP(1, 4) IRLMX_STRIP(1, 8) IRLMX_STRIP(2, 2) IRLMX_STRIP(2, 4) IRLMX_STRIP(4, 1) IRLMX_STRIP(4, 2)
#undef IRLMX_STRIP
  return nullptr;
}
template void* strip_fn<kModeFwd>(int, int);
template void* strip_fn<kModeBwd>(int, int);

}  // namespace irlmx
