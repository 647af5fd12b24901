// Persistent, temporally blocked stencil sweeps for state spaces too large
// for one CU (e.g. 128x128 grids): forward SVF (maxent.py:63-114) and the
// non-causal backward pass (maxent.py:119-159).
//
// Decomposition.  An instance's width x height grid is cut into C row tiles of
// R rows.  Each tile is owned by one 1024-thread workgroup (one per CU, all
// co-resident), which keeps its tile plus G ghost rows on either side in LDS
// (two ping-pong float64 buffers) and the per-state stencil weights of that
// extended tile in registers.  A block of T <= G sweeps runs entirely on chip:
// after sweep i the rows that are still exact shrink by one on each ghost side,
// so after T sweeps the owned rows are exact.  Then the tiles of an instance
// exchange state through HBM:
//
//   publish : every tile stores its owned rows into pub[parity][instance]
//             (plain stores), each storing wave drains (s_waitcnt vmcnt(0)),
//             the workgroup barriers, one lane does an agent-scope release and
//             a relaxed agent-scope add on the instance's arrival counter;
//   consume : that lane polls the counter (relaxed, s_sleep, bounded by a
//             wall-clock timeout), issues one agent-scope acquire, the
//             workgroup barriers, then plain loads of the ghost rows.
//   (MI355X_MICROARCH.md "Workgroup dispatch ... visibility", Valid forms.)
//
// Convergence (forward).  Each tile reduces max|d_new - d_old| over its owned
// states for every sweep of the block and max-combines it into the
// instance's per-sweep slots (3-slot ring of blocks).  After the exchange every
// tile reads the same slots and so takes the same decision: if the first sweep
// with !(delta > eps) lies inside the block, every tile reloads the
// block-start state (the previous block's publication, still intact thanks to
// the double buffer) and re-runs exactly that many sweeps -- the same
// arithmetic in the same order, so the result is the one the reference's loop
// stops at.
//
// Rescaling (backward).  The partition vector grows geometrically.  A first
// pass bounds the per-sweep growth g of each instance; blocks are capped at
// T_eff sweeps so that g^T_eff stays below 2^900, and at every block boundary
// all tiles multiply their values by the same power of two derived from the
// instance-wide maximum: ratio-exact, like the single-workgroup kernel.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>

#include "cluster.h"
#include "common.h"

namespace irlmx {

void set_error(const char* fmt, ...);
int hip_fail(hipError_t e, const char* what);

__device__ inline unsigned int ld_acq_relaxed(unsigned int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Arrival barrier of the C tiles of one instance (see file comment).  Returns
// false on timeout (then the error word is set and the caller exits).
__device__ inline bool instance_barrier(unsigned int* counter, unsigned int target, int* err, int* lds_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its stores
  __syncthreads();
  if (threadIdx.x == 0) {
    int abort = 0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
    while (ld_acq_relaxed(counter) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > 2000000000ull) {  // 20 s
        abort = 1;
        atomicOr(err, 1);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    *lds_flag = abort;
  }
  __syncthreads();
  return *lds_flag == 0;
}

// LDS buffer layout: [W + 1 zeros][E states][W + 1 zeros].  With the pads, the
// five stencil reads of state l are q[0], q[W-1], q[W], q[W+1], q[2W] for
// q = buf + l + 1: one address register per state and constant offsets (the
// pads are never written and stay 0; their stencil weight is 0 or the row they
// feed is a ghost row that is no longer exact).
template <int MODE, int SPT, int WT>
__global__ void __launch_bounds__(kCT) cluster_kernel(ClusterArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int W = WT ? WT : a.W;
  const int H = a.H, S = a.S;
  const int tile = blockIdx.x % a.C;
  const int inst = a.b0 + blockIdx.x / a.C;
  const int tid = threadIdx.x;
  const int r0 = tile * a.R, r1 = min(H, r0 + a.R);
  const int e0 = max(0, r0 - a.G), e1 = min(H, r1 + a.G);
  const int E = (e1 - e0) * W;
  const int own0 = (r0 - e0) * W, own1 = (r1 - e0) * W;
  const int base = e0 * W;
  const int pad = W + 1;
  const int blen = a.emax + 2 * pad;
  double* bufA = (double*)smem;
  double* bufB = bufA + blen;
  unsigned long long* red = (unsigned long long*)(bufB + blen);  // [2][kTMax]
  int* lflag = (int*)(red + 2 * kTMax);                          // [4]

  const size_t iS = (size_t)inst * S;
  if (MODE == kModeFwd && a.bad[inst]) {
    // non-finite policy: the reference's dense product is NaN after one sweep
    for (int l = own0 + tid; l < own1; l += kCT) a.out[iS + base + l] = __longlong_as_double(0x7ff8000000000000LL);
    if (tile == 0 && tid == 0) { a.iters[inst] = 1; a.status[inst] = IRLMX_NONFINITE; }
    return;
  }

  // ---- per-state constants into registers --------------------------------
  double w[SPT][kStencilK];
  double c0[SPT];  // forward: p0; backward: exp(r), applied after the row sum as in the other shapes
  const size_t wbase = (MODE == kModeBwd && a.tab_shared) ? 0 : iS * kStencilK;
#pragma unroll
  for (int j = 0; j < SPT; ++j) {
    const int l = tid + j * kCT;
    c0[j] = 0.0;
#pragma unroll
    for (int k = 0; k < kStencilK; ++k) w[j][k] = 0.0;
    if (l < E) {
      const int s = base + l;
      c0[j] = MODE == kModeFwd ? a.vin[iS + s] : exp(a.vin[iS + s]);
#pragma unroll
      for (int k = 0; k < kStencilK; ++k) w[j][k] = a.wgt[wbase + (size_t)k * S + s];
    }
  }
  for (int i = tid; i < 2 * blen; i += kCT) bufA[i] = 0.0;
  __syncthreads();
  for (int l = tid; l < E; l += kCT) {
    double v0 = 0.0;
    if (MODE == kModeBwd) v0 = a.term[iS + base + l] ? 1.0 : 0.0;
    bufA[pad + l] = v0;
    bufB[pad + l] = v0;
  }
  if (tid < 2 * kTMax) red[tid] = 0ull;
  if (tid == 0) lflag[0] = 0;

  int T = a.T;
  if (MODE == kModeBwd) {
    // cap the block so the growth over T sweeps stays below 2^900
    const double g = bits_double(a.growth[inst]);
    if (a.rescale && g > 2.0 && isfinite(g)) {
      const int cap = (int)floor(900.0 / log2(g)) - 1;
      T = max(1, min(T, cap));
    }
  }
  __syncthreads();

  // one Jacobi sweep over the extended tile; the owned-row maximum goes to *rslot
  auto sweep = [&](const double* din, double* dout, unsigned long long* rslot) {
    unsigned long long mx = 0ull;
#pragma unroll
    for (int j = 0; j < SPT; ++j) {
      const int l = tid + j * kCT;
      if (l < E) {
        const double* q = din + l + 1;
        const double self = q[W];
        double acc = fma(w[j][0], self, 0.0);  // same association as the fused/sweep shapes
        acc = fma(w[j][1], q[W + 1], acc);
        acc = fma(w[j][2], q[W - 1], acc);
        acc = fma(w[j][3], q[2 * W], acc);
        acc = fma(w[j][4], q[0], acc);
        const double nv = MODE == kModeFwd ? __dadd_rn(c0[j], acc) : __dmul_rn(c0[j], acc);
        dout[pad + l] = nv;
        if (l >= own0 && l < own1) {
          const unsigned long long d = MODE == kModeFwd ? abs_bits(nv - self) : abs_bits(nv);
          mx = d > mx ? d : mx;
        }
      }
    }
    mx = wave_max_u64(mx);
    if ((tid & (kWave - 1)) == 0 && mx) atomicMax(rslot, mx);
    __syncthreads();
  };

  unsigned long long* slots = a.slots + (size_t)inst * 3 * kTMax;
  const size_t pubStride = (size_t)a.btot * S;  // pub[parity] stride

  double* cur = bufA;
  double* oth = bufB;
  long long done = 0;  // sweeps completed before the current block
  const long long total = MODE == kModeBwd ? a.n_sweeps : -1;
  for (int m = 0;; ++m) {
    int Tm = T;
    if (MODE == kModeBwd) Tm = (int)min<long long>((long long)T, total - done);
    unsigned long long* rset = red + (m & 1) * kTMax;
    // ---- T_m sweeps on chip ----------------------------------------------
    for (int i = 0; i < Tm; ++i) {
      sweep(cur, oth, &rset[i]);
      double* t = cur; cur = oth; oth = t;
    }
    // ---- publish owned rows, combine per-sweep maxima, arrive --------------
    double* pubm = a.pub + (size_t)(m & 1) * pubStride + iS;
    for (int l = own0 + tid; l < own1; l += kCT) pubm[base + l] = cur[pad + l];
    if (tid == 0) {
      unsigned long long* sl = slots + (m % 3) * kTMax;
      for (int i = 0; i < Tm; ++i)
        if (rset[i]) atomicMax(&sl[i], rset[i]);
      if (tile == 0) {
        unsigned long long* nx = slots + ((m + 1) % 3) * kTMax;
        for (int i = 0; i < kTMax; ++i) __hip_atomic_store(&nx[i], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    if (!instance_barrier(&a.counter[inst], (unsigned)(a.C * (m + 1)), a.err, &lflag[0])) return;
    // every tile now sees every tile's publication and maxima of block m;
    // the other maxima set was last read before this barrier: clear it for block m + 1
    if (tid < kTMax) red[((m + 1) & 1) * kTMax + tid] = 0ull;
    unsigned long long* sl = slots + (m % 3) * kTMax;
    if (MODE == kModeFwd) {
      int conv = 0;
      double dl = 0.0;
      for (int i = 0; i < Tm; ++i) {
        dl = bits_double(__hip_atomic_load(&sl[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        const bool cap = a.max_iter > 0 && done + i + 1 >= a.max_iter;
        if (!(dl > a.eps) || cap) { conv = i + 1; break; }
      }
      if (conv) {
        // exact stop inside the block: replay `conv` sweeps from the block-start state
        const double* src = m == 0 ? nullptr : a.pub + (size_t)((m - 1) & 1) * pubStride + iS;
        for (int l = tid; l < E; l += kCT) cur[pad + l] = src ? src[base + l] : 0.0;
        __syncthreads();
        unsigned long long* scratch = red + ((m + 1) & 1) * kTMax;
        for (int i = 0; i < conv; ++i) {
          sweep(cur, oth, scratch);
          double* t = cur; cur = oth; oth = t;
        }
        for (int l = own0 + tid; l < own1; l += kCT) a.out[iS + base + l] = cur[pad + l];
        if (tile == 0 && tid == 0) {
          a.iters[inst] = done + conv;
          a.status[inst] = dl != dl ? IRLMX_NONFINITE : (dl > a.eps ? IRLMX_MAXITER : IRLMX_OK);
        }
        return;
      }
    }
    done += Tm;
    // ---- refresh ghost rows from the neighbours' publications ---------------
    int e_scale = 0;
    if (MODE == kModeBwd && a.rescale)
      e_scale = rescale_exponent(bits_double(__hip_atomic_load(&sl[Tm - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)));
    for (int l = tid; l < E; l += kCT) {
      double v = (l >= own0 && l < own1) ? cur[pad + l] : pubm[base + l];
      if (MODE == kModeBwd && e_scale) v = ldexp(v, e_scale);
      cur[pad + l] = v;
    }
    __syncthreads();
    if (MODE == kModeBwd && done >= total) break;
  }

  if (MODE == kModeBwd) {
    // last of the 2*S sweeps, per action: za = exp(r) * (P_a zs); pi = za / sum_a za
    const int A = a.A;
    const size_t tb = a.tab_shared ? 0 : (size_t)inst;
    for (int l = own0 + tid; l < own1; l += kCT) {
      const int s = base + l;
      const double* q = cur + l + 1;
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
        za[act] = __dmul_rn(er, acc);  // rounded product, then the sum: no contraction into an fma
        zsum = __dadd_rn(zsum, za[act]);
      }
      for (int act = 0; act < A; ++act) a.out[(iS + s) * A + act] = za[act] / zsum;
    }
    if (tile == 0 && tid == 0) a.status[inst] = IRLMX_OK;
  }
}

}  // namespace irlmx

namespace irlmx {

// Per-instance bound on the backward's per-sweep growth: max_s exp(r_s) * sum_k bw[k][s].
__global__ void bwd_growth_kernel(const double* __restrict__ bw, int tab_shared, const double* __restrict__ reward,
                                  int S, unsigned long long* __restrict__ growth) {
  const int b = blockIdx.x;
  const double* wb = bw + (tab_shared ? 0 : (size_t)b * kStencilK * S);
  unsigned long long mx = 0ull;
  for (int s = threadIdx.x; s < S; s += blockDim.x) {
    double row = 0.0;
    for (int k = 0; k < kStencilK; ++k) row += wb[(size_t)k * S + s];
    mx = max(mx, abs_bits(exp(reward[(size_t)b * S + s]) * row));
  }
  __shared__ unsigned long long red[16];
  mx = wave_max_u64(mx);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x / 64] = mx;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < (int)(blockDim.x / 64); ++i) mx = max(mx, red[i]);
    growth[b] = mx;
  }
}

static int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return (e && *e) ? atoi(e) : dflt;
}

static int device_cus() {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  return cus;
}

static size_t cluster_lds(int emax, int W) {
  return 2 * (size_t)(emax + 2 * (W + 1)) * sizeof(double) + 2 * kTMax * sizeof(unsigned long long) + 16;
}

// Tile plan for a width x height stencil grid and B instances: the fewest
// sequential launches first, then the most sweeps per exchange (G), then the
// smallest extended tile.  IRLMX_CLUSTER_R / _G force a plan (tests).
bool cluster_plan(int W, int H, int B, ClusterPlan* out) {
  if (env_int("IRLMX_CLUSTER", 1) == 0) return false;
  const int cus = device_cus();
  if (cus <= 0) return false;
  const int rows_cap = kCT * kSptMax / W;
  const int fR = env_int("IRLMX_CLUSTER_R", 0), fG = env_int("IRLMX_CLUSTER_G", 0);
  double best = 1e300;
  bool ok = false;
  for (int G = kTMax; G >= 1; --G) {
    if (fG && G != fG) continue;
    for (int R = std::min(H, rows_cap - 2 * G); R >= 1; --R) {
      if (fR && R != fR) continue;
      const int C = (H + R - 1) / R;
      const int ext = std::min(H, R + 2 * G);
      const int E = ext * W;
      const int spt = (E + kCT - 1) / kCT;
      if (spt > kSptMax) continue;
      const int per = cus / C;
      if (per < 1) continue;
      const int nl = (B + per - 1) / per;
      const double cost = nl * (double)spt * (G + 8.0) / G;
      if (cost < best - 1e-9) {
        best = cost;
        ok = true;
        *out = ClusterPlan{R, G, C, G, std::min(per, B), spt, spt * kCT, cluster_lds(spt * kCT, W)};
      }
    }
  }
  return ok;
}

template <int MODE, int WT>
static void* cluster_fn_w(int spt) {
  switch (spt) {
    case 1: return (void*)&cluster_kernel<MODE, 1, WT>;
    case 2: return (void*)&cluster_kernel<MODE, 2, WT>;
    case 3: return (void*)&cluster_kernel<MODE, 3, WT>;
    case 4: return (void*)&cluster_kernel<MODE, 4, WT>;
    case 5: return (void*)&cluster_kernel<MODE, 5, WT>;
    case 6: return (void*)&cluster_kernel<MODE, 6, WT>;
  }
  return nullptr;
}

// grid widths with compile-time LDS offsets; any other width uses WT = 0
template <int MODE>
static void* cluster_fn(int spt, int W) {
  switch (W) {
    case 64: return cluster_fn_w<MODE, 64>(spt);
    case 128: return cluster_fn_w<MODE, 128>(spt);
    case 256: return cluster_fn_w<MODE, 256>(spt);
  }
  return cluster_fn_w<MODE, 0>(spt);
}

// Launch the cluster kernel over all instances, `per_launch` at a time, then
// check the barrier-timeout word (synchronises the stream).
int cluster_run(int mode, const ClusterPlan& p, ClusterArgs a, int B, hipStream_t st) {
  void* fn = mode == kModeFwd ? cluster_fn<kModeFwd>(p.spt, a.W) : cluster_fn<kModeBwd>(p.spt, a.W);
  if (!fn) { set_error("cluster: no kernel for spt=%d", p.spt); return IRLMX_EINVAL; }
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)p.lds);
  if (e != hipSuccess) return hip_fail(e, "cluster hipFuncSetAttribute");
  int per_cu = 0;
  e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)fn, kCT, p.lds);
  if (e != hipSuccess) return hip_fail(e, "cluster occupancy");
  const int resident = per_cu * device_cus();
  if (p.C * p.per_launch > resident) {
    set_error("cluster: %d workgroups cannot be co-resident (%d)", p.C * p.per_launch, resident);
    return IRLMX_EINVAL;
  }
  a.R = p.R; a.G = p.G; a.C = p.C; a.T = p.T; a.emax = p.emax; a.btot = B;
  for (int b0 = 0; b0 < B; b0 += p.per_launch) {
    const int nb = std::min(p.per_launch, B - b0);
    a.b0 = b0;
    void* args[] = {&a};
    e = hipLaunchKernel(fn, dim3(nb * p.C), dim3(kCT), args, p.lds, st);
    if (e != hipSuccess) return hip_fail(e, "cluster launch");
  }
  int err = 0;
  e = hipMemcpyAsync(&err, a.err, sizeof(int), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) return hip_fail(e, "cluster sync");
  if (err) { set_error("cluster: instance barrier timed out (workgroups not co-resident?)"); return IRLMX_EHIP; }
  return 0;
}

}  // namespace irlmx
