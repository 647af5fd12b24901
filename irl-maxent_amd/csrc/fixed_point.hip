// Fixed-point sweeps of the MaxEnt-IRL inner loop on gfx950.
//
//   backward  (maxent.py:119-159)  zs <- exp(r) * sum_a P_a zs, 2*S sweeps, then za/zs
//   forward   (maxent.py:63-114)   d  <- p0 + sum_a P'_a^T (pi_a * d) until max|dd| <= eps
//   soft VI   (maxent.py:279-341)  v  <- fold_a softmax(v, r + g P_a v) until max|dv| <= eps
//   VI        (solver.py:9-104)    v  <- r + max_a / mean_a (g P_a v) until max|dv| <= eps
//
// Two execution shapes, chosen per call from the state count S:
//
//  * fused: one workgroup owns one instance for the WHOLE loop.  The two
//    ping-pong state vectors live in LDS (2*S*8 B <= 64 KiB at S = 4096), each
//    thread keeps the weights and neighbour indices of its SPT states in
//    registers, and a sweep costs one workgroup barrier: the convergence test
//    max|new - old| is a wave shuffle-max plus one LDS atomic max into a
//    3-slot ring, so there is no host round trip until the loop has converged.
//  * sweep: S too large for one CU.  One launch per sweep over all B
//    instances; vectors in HBM, per-instance max|delta| by one global atomic
//    per workgroup into a 3-slot ring, and a per-instance done flag that
//    freezes an instance once converged, so the host can enqueue sweeps in
//    chunks and only polls a done counter between chunks.
//
// The convergence word is the raw bits of |x| as uint64: for non-negative
// doubles integer order is numeric order and NaN sorts above +inf, so the
// integer max reproduces np.max(np.abs(.)) including NaN propagation, and
// `!(delta > eps)` stops on NaN exactly like the reference's `while delta > eps`.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <initializer_list>
#include <type_traits>
#include <vector>

#include "cluster.h"
#include "common.h"
#include "dense.h"

namespace irlmx {

void set_error(const char* fmt, ...);
int hip_fail(hipError_t e, const char* what);

constexpr int kFusedMaxStates = 4096;

static int getenv_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return (e && *e) ? atoi(e) : dflt;
}

// Largest S run by the fused shape; IRLMX_FUSED_MAX_STATES lowers it (tests use
// 0 to drive every size through the sweep shape).
static int fused_max_states() {
  const char* e = getenv("IRLMX_FUSED_MAX_STATES");
  if (!e || !*e) return kFusedMaxStates;
  const int v = atoi(e);
  return v < kFusedMaxStates ? v : kFusedMaxStates;
}
constexpr int kMaxActions = 8;
constexpr int kSweepThreads = 256;

// ---------------------------------------------------------------------------
// model views
// ---------------------------------------------------------------------------

struct Model {
  int S, A, K, W, H, B, stencil, shared, Kc, dense;
  int props;  // irlmx_mdp.props: IRLMX_PROPS_KNOWN | IRLMX_PROP_* from irlmx_mdp_properties, or 0 (unknown)
  const double* row_val;
  const int32_t* row_idx;
  const int32_t* col_idx;
  const double* col_val;
};

static Model make_model(const irlmx_mdp* m) {
  Model o;
  o.S = m->n_states;
  o.A = m->n_actions;
  o.stencil = m->layout == IRLMX_LAYOUT_STENCIL5;
  o.dense = m->layout == IRLMX_LAYOUT_DENSE;
  o.K = o.stencil ? kStencilK : (o.dense ? m->n_states : m->k_row);
  o.Kc = o.stencil ? kStencilK : (o.dense ? m->n_states : m->k_col);
  o.W = m->width;
  o.H = m->height;
  o.B = m->batch;
  o.shared = m->shared != 0;
  o.row_val = m->row_val;
  o.row_idx = m->row_idx;
  o.col_idx = m->col_idx;
  o.col_val = m->col_val;
  o.props = m->props;
  return o;
}

__device__ inline size_t inst_of(const Model& m, int b) { return m.shared ? 0 : (size_t)b; }

// neighbour (row form) of s in slot k
__device__ inline int row_nbr(const Model& m, int b, int s, int k) {
  if (m.stencil) return stencil_nbr(s, k, m.W, m.H);
  const int t = m.row_idx[(inst_of(m, b) * m.K + k) * m.S + s];
  return IRLMX_DCHECK(t >= 0 && t < m.S, kCheckIndex) ? t : s;
}

__device__ inline double row_val(const Model& m, int b, int a, int k, int s) {
  return m.row_val[((inst_of(m, b) * m.A + a) * m.K + k) * m.S + s];
}

// source (column form) of target t in slot k
__device__ inline int col_src(const Model& m, int b, int t, int k) {
  if (m.stencil) return stencil_nbr(t, k, m.W, m.H);
  const int s = m.col_idx[(inst_of(m, b) * m.Kc + k) * m.S + t];
  return IRLMX_DCHECK(s >= 0 && s < m.S, kCheckIndex) ? s : t;
}

// ---------------------------------------------------------------------------
// workspace carving
// ---------------------------------------------------------------------------

struct Ws {
  double* wgt;                // forward: [B][Kc][S] gather weights; backward: [B][K][S] reward-folded
  int32_t* bad;               // [B] forward: policy has a non-finite entry
  double* buf0;               // [B][S]   sweep path ping
  double* buf1;               // [B][S]   sweep path pong
  unsigned long long* slots;  // [B][3]
  int32_t* done;              // [B]
  int64_t* iters;             // [B]
  int32_t* ndone;             // [1]
  // cluster shape (stencil layouts too large for one CU); sizes as carve() takes them:
  unsigned long long* gran;   // cluster: [B][gran_inst_len(W, H)] x 16 B (two padded halo parities, cluster.h);
                              // grid: [B][3][S] x 16 B; dense grid: [B][2][S] x 16 B
  unsigned long long* sgran;  // cluster: [B][kSumRows][H] x 16 B (tile summaries by block % kSumSlots,
                              // then the XCC ids and the forward's full flags, cluster.h); grid: [B][4][bpi]; dense grid: [B][bpi] x 16 B
  unsigned long long* growth; // [2][B] growth / decay bounds (bwd_growth_kernel)
  int* err;                   // [4]: error bits, rendezvous counters
  size_t total;
};

static size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

static bool use_fused(const Model& m, int op);

// Persistent grid shape (soft VI / VI on stencil grids too large for one CU):
// states per thread and workgroups per instance; false when it does not apply.
struct GridPlan {
  int spt, bpi, xcd;
};
static bool grid_plan(const Model& m, int op, GridPlan* out);
// Persistent dense shape (dense_grid.hip) for this call, if it applies.
static bool dense_grid(const Model& m, int op, DenseGridPlan* out);

static Ws carve(const Model& m, int op, void* base) {
  Ws w;
  size_t off = 0;
  char* p = (char*)base;
  auto take = [&](size_t bytes) {
    char* r = p ? p + off : nullptr;
    off += align256(bytes);
    return (void*)r;
  };
  const size_t B = m.B, S = m.S;
  size_t nw = 0;
  if (op == IRLMX_OP_FORWARD) nw = B * m.Kc * S;  // dense: the per-instance gather matrices WT [B][S][S]
  if (op == IRLMX_OP_BACKWARD) nw = m.dense ? B * S : B * m.K * S;  // reward-folded; dense: the GEMM product
  if ((op == IRLMX_OP_SOFT_BACKWARD || op == IRLMX_OP_VALUE_ITERATION) && m.dense && m.shared)
    nw = (size_t)m.A * B * S;  // the per-action GEMM products of a shared dense table
  w.wgt = (double*)take(nw * sizeof(double));
  w.bad = (int32_t*)take(B * sizeof(int32_t));
  const bool sweep = !use_fused(m, op);
  w.buf0 = (double*)take(sweep ? B * S * sizeof(double) : 0);
  w.buf1 = (double*)take(sweep ? B * S * sizeof(double) : 0);
  w.slots = (unsigned long long*)take(B * 3 * sizeof(unsigned long long));
  w.done = (int32_t*)take(B * sizeof(int32_t));
  w.iters = (int64_t*)take(B * sizeof(int64_t));
  w.ndone = (int32_t*)take(sizeof(int32_t) * 4);
  const bool cl = sweep && m.stencil && (op == IRLMX_OP_FORWARD || op == IRLMX_OP_BACKWARD);
  GridPlan gp{0, 0, 0};
  const bool gr = sweep && grid_plan(m, op, &gp);
  DenseGridPlan dp{0, 0, 0, 0};
  const bool dg = sweep && dense_grid(m, op, &dp);
  // cluster halo exchange: [B][gran_inst_len] and [B][kSumRows][H] 16-byte granule pairs;
  // grid shape: [B][3][S] value and [B][3][bpi] block-delta granules;
  // dense grid shape: [B][2][S] value and [B][bpi] XCC-id granules
  const size_t gcl = cl ? B * gran_inst_len(m.W, m.H) * 16 : 0;   // cluster.h kGranRowPad layout
  w.gran = (unsigned long long*)take(std::max(gcl, dg ? 2 * B * S * 16 : (gr ? 3 * B * S * 16 : 0)));
  w.sgran = (unsigned long long*)take(cl ? kSumRows * B * (size_t)m.H * 16
                                         : (gr ? 4 * B * (size_t)gp.bpi * 16 : (dg ? B * (size_t)dp.bpi * 16 : 0)));
  w.growth = (unsigned long long*)take(cl ? 2 * B * sizeof(unsigned long long) : 0);
  w.err = (int*)take(cl || gr || dg ? 4 * sizeof(int) : 0);
  w.total = off;
  return w;
}

// ---------------------------------------------------------------------------
// weight preparation
// ---------------------------------------------------------------------------

// Gather weights of the forward pass, one per (target t, slot k):
//   w[k][t] = sum_a P[s, t, a] * pi[s, a]  over non-terminal sources s = src_k(t)
// (P' of maxent.py:98-99 has the terminal rows cleared).  Any non-finite
// policy entry makes the reference's dense dgemv return NaN everywhere after
// one sweep (0 * NaN inside the dot), so such instances are flagged in `bad`.
__global__ void fwd_weights_kernel(Model m, const double* __restrict__ pi,
                                   const uint8_t* __restrict__ term, double* __restrict__ w,
                                   int32_t* __restrict__ bad) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (t >= m.S) return;
  const int S = m.S, A = m.A;
  const double* pib = pi + (size_t)b * S * A;
  const uint8_t* tb = term + (size_t)b * S;
  bool nonfinite = false;
  for (int a = 0; a < A; ++a) nonfinite |= !isfinite(pib[(size_t)t * A + a]);
  for (int k = 0; k < m.Kc; ++k) {
    double acc = 0.0;
    if (m.stencil) {
      if (stencil_valid(t, k, m.W, m.H)) {
        const int s = stencil_nbr(t, k, m.W, m.H);
        const int kk = stencil_opposite(k);  // direction from s back to t
        if (!tb[s])
          for (int a = 0; a < A; ++a) acc = fma(row_val(m, b, a, kk, s), pib[(size_t)s * A + a], acc);
      }
    } else {
      const int s = col_src(m, b, t, k);
      if (!tb[s]) {
        const size_t base = inst_of(m, b) * A;
        for (int a = 0; a < A; ++a)
          acc = fma(m.col_val[((base + a) * m.Kc + k) * S + t], pib[(size_t)s * A + a], acc);
      }
    }
    w[((size_t)b * m.Kc + k) * S + t] = acc;
  }
  if (nonfinite) atomicOr(&bad[b], 1);
}

// bwd_nonfinite_rule.  The reference's backward product is dense (maxent.py:155:
// P_a.dot(zs) over all S columns), so one non-finite partition value makes
// 0 * inf = NaN appear in every row within a sweep, and the returned policy is
// NaN everywhere.  The compact products here touch only stored neighbours, so
// every shape records "some zs value of the 2S - 1 collapsed sweeps was
// non-finite" (fused and sweep shapes: per sweep) and then writes NaN for the
// whole instance.  With rescaling on, values turn non-finite only through
// non-finite weights (a reward of +inf or NaN), which bwd_weights_kernel flags
// (the cluster shape fills such instances with NaN after its sweeps,
// bwd_nan_fill_kernel); calls without rescaling (the reference's overflow) do
// not run on the cluster shape.
// Collapsed, reward-folded backward weights of instance b:
//   w[b][k][s] = exp(r[b][s]) * sum_a P[s, target_k(s), a]
// so one backward sweep is zs'[s] = sum_k w[b][k][s] * zs[target_k(s)]
// (maxent.py:155-156 with the action sum and exp(r) taken out of the loop).
// Every shape (fused, sweep, cluster) uses these same weights in the same
// order, so the shapes stay bit-identical to each other.
__global__ void bwd_weights_kernel(Model m, const double* __restrict__ reward, double* __restrict__ w,
                                   int32_t* __restrict__ bad) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (s >= m.S) return;
  const size_t bi = m.shared ? 0 : (size_t)b;  // table instance
  const double er = exp(reward[(size_t)b * m.S + s]);
  bool nf = false;
  for (int k = 0; k < m.K; ++k) {
    double acc = 0.0;
    for (int a = 0; a < m.A; ++a)
      acc += m.row_val[((bi * m.A + a) * m.K + k) * m.S + s];
    const double wk = __dmul_rn(er, acc);
    nf |= !isfinite(wk);
    w[((size_t)b * m.K + k) * m.S + s] = wk;
  }
  // non-finite weights make some partition value non-finite within two sweeps,
  // and the reference's dense product then NaN everywhere (bwd_nonfinite_rule)
  if (nf) atomicOr(&bad[b], 1);
}

// bwd_nonfinite_rule for the cluster shape: NaN policy for flagged instances
__global__ void bwd_nan_fill_kernel(Model m, const int32_t* __restrict__ bad, double* __restrict__ pi) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (i < m.S * m.A && bad[b]) pi[(size_t)b * m.S * m.A + i] = kNaN;
}

// ---------------------------------------------------------------------------
// fused (one workgroup per instance) kernels
// ---------------------------------------------------------------------------

struct FwdArgs {
  Model m;
  const double* w;  // [B][Kc][S]
  const int32_t* bad;
  const double* p0;
  double eps;
  long long max_iter;
  double* out;
  int64_t* iters;
  int32_t* status;
};

__device__ inline int finish_status(double delta, double eps) {
  if (delta != delta) return IRLMX_NONFINITE;
  return delta > eps ? IRLMX_MAXITER : IRLMX_OK;
}

// The reference's fixed-point loops stop after the first sweep whose
// max|x_new - x| is not > eps, NaN included (maxent.py:108, :335, solver.py:49).
// run_deferred keeps that rule without a per-sweep reduction: each lane records
// per sweep i "some |x_new - x| > eps" (bit i) and "some |x_new - x| is NaN"
// (bit 32 + i) for its states (record_delta), and the workgroup ORs the bits
// once per block of kDeferBlock sweeps.  If the block holds the stopping sweep
// k, restore() puts the block-start state back (LDS and registers; save() took
// it) and sweeps 0..k are replayed -- the same arithmetic, so the same bits.
// sweep(it, pos, bits) runs one sweep from buffer parity it & 1 and records at
// bit pos (the helpers put the barrier after it); slot[0..2] are zero on entry.
// Returns the status (OK, NONFINITE, MAXITER); `it` counts the sweeps done.
// One call site of sweep(), so it is inlined once.  run_each is the per-sweep
// form for kernels whose registers have no room for the block bookkeeping: the
// same bits, reduced every sweep with two ballots (no cross-lane shuffles).
constexpr int kDeferBlock = 32;
__device__ inline void record_delta(unsigned long long& bits, int pos, double d, double eps) {
  bits |= ((d > eps) ? 1ull : 0ull) << pos;
  bits |= ((d != d) ? 1ull : 0ull) << (32 + pos);
}
template <class Sweep, class Save, class Restore>
__device__ __attribute__((always_inline)) inline int run_deferred(long long max_iter, unsigned long long* slot,
                                                                  long long& it, Sweep&& sweep, Save&& save,
                                                                  Restore&& restore) {
  const int tid = threadIdx.x;
  for (int blk = 0;; ++blk) {
    save();
    int nb = kDeferBlock;
    if (max_iter > 0) nb = (int)min<long long>(nb, max_iter - it);
    int k = -1;
    unsigned nan = 0u;
    for (int pass = 0; pass < 2; ++pass) {  // the block, then (stop inside it) the replay
      unsigned long long bits = 0ull;
      const int cnt = pass == 0 ? nb : k + 1;
      for (int i = 0; i < cnt; ++i) {
        sweep(it + i, i, bits);
        __syncthreads();
      }
      if (pass == 1) break;
      bits = wave_or_u64(bits);
      if ((tid & (kWave - 1)) == 0 && bits) atomicOr(&slot[blk & 1], bits);
      if (tid == 0) slot[(blk & 1) ^ 1] = 0ull;  // last read in the previous block, before this block's barriers
      __syncthreads();
      const unsigned long long all = slot[blk & 1];
      const unsigned gt = (unsigned)all;
      nan = (unsigned)(all >> 32);
      const unsigned live = nb >= 32 ? 0xFFFFFFFFu : ((1u << nb) - 1u);
      const unsigned stop = (~gt | nan) & live;
      if (!stop) break;
      k = __builtin_ctz(stop);
      restore();
    }
    if (k >= 0) {
      it += k + 1;
      return ((nan >> k) & 1u) ? IRLMX_NONFINITE : IRLMX_OK;
    }
    it += nb;
    if (max_iter > 0 && it >= max_iter) return IRLMX_MAXITER;
  }
}
template <class Sweep>
__device__ __attribute__((always_inline)) inline int run_each(long long max_iter, unsigned long long* slot,
                                                              long long& it, Sweep&& sweep) {
  const int tid = threadIdx.x;
  for (int r3 = 0;; r3 = r3 == 2 ? 0 : r3 + 1) {
    unsigned long long bits = 0ull;
    sweep(it, 0, bits);
    const unsigned long long w = (__builtin_amdgcn_ballot_w64((bits & 1ull) != 0ull) ? 1ull : 0ull) |
                                 (__builtin_amdgcn_ballot_w64((bits >> 32) != 0ull) ? (1ull << 32) : 0ull);
    if ((tid & (kWave - 1)) == 0 && w) atomicOr(&slot[r3], w);
    if (tid == 0) slot[r3 == 2 ? 0 : r3 + 1] = 0ull;  // read two sweeps ago
    __syncthreads();
    const unsigned long long all = slot[r3];
    ++it;
    if (all >> 32) return IRLMX_NONFINITE;
    if (!(all & 1ull)) return IRLMX_OK;
    if (max_iter > 0 && it >= max_iter) return IRLMX_MAXITER;
  }
}

// one barrier per sweep; LDS: two S-vectors + 3 convergence slots
template <int SPT, int KMAX>
__global__ void __launch_bounds__(1024) fwd_fused_kernel(FwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const Model& m = a.m;
  const int S = m.S, K = m.Kc;
  const int b = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
  double* bufA = (double*)smem;
  double* bufB = bufA + S;
  unsigned long long* slot = (unsigned long long*)(bufB + S);
  double* snap = (double*)(slot + 4);  // run_deferred's block-start state (LDS: the registers are taken)

  if (a.bad[b]) {  // non-finite policy: the reference yields NaN after one sweep
    for (int s = tid; s < S; s += nt) a.out[(size_t)b * S + s] = __longlong_as_double(0x7ff8000000000000LL);
    if (tid == 0) { a.iters[b] = 1; a.status[b] = IRLMX_NONFINITE; }
    return;
  }

  double w[SPT][KMAX];
  int nb[SPT][KMAX];
  double p0[SPT], cur[SPT];
  const double* wb = a.w + (size_t)b * K * S;
#pragma unroll
  for (int j = 0; j < SPT; ++j) {
    const int s = tid + j * nt;
    cur[j] = 0.0;
    p0[j] = 0.0;
#pragma unroll
    for (int k = 0; k < KMAX; ++k) { w[j][k] = 0.0; nb[j][k] = 0; }
    if (s < S) {
      p0[j] = a.p0[(size_t)b * S + s];
#pragma unroll
      for (int k = 0; k < KMAX; ++k)
        if (k < K) { w[j][k] = wb[(size_t)k * S + s]; nb[j][k] = col_src(m, b, s, k); }
    }
  }
  for (int s = tid; s < S; s += nt) bufA[s] = 0.0;
  if (tid < 3) slot[tid] = 0ull;
  __syncthreads();

  long long it = 0;
  auto sweep = [&](long long it, int pos, unsigned long long& bits) __attribute__((always_inline)) {
    const double* din = (it & 1) ? bufB : bufA;
    double* dout = (it & 1) ? bufA : bufB;
#pragma unroll
    for (int j = 0; j < SPT; ++j) {
      const int s = tid + j * nt;
      if (s < S) {
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k < KMAX; ++k)
          if (k < K) acc = fma(w[j][k], din[nb[j][k]], acc);
        const double nv = p0[j] + acc;
        dout[s] = nv;
        record_delta(bits, pos, fabs(nv - cur[j]), a.eps);
        cur[j] = nv;
      }
    }
  };
  // (the widest ELL rows fill the registers: the per-sweep reduction there)
  int status;
  if constexpr (SPT * KMAX < 32) {
    status = run_deferred(
        a.max_iter, slot, it, sweep,
        [&]() {
#pragma unroll
          for (int j = 0; j < SPT; ++j)
            if (tid + j * nt < S) snap[tid + j * nt] = cur[j];
        },
        [&]() {
          double* d0 = (it & 1) ? bufB : bufA;
#pragma unroll
          for (int j = 0; j < SPT; ++j)
            if (tid + j * nt < S) d0[tid + j * nt] = cur[j] = snap[tid + j * nt];
          __syncthreads();
        });
  } else {
    // the per-sweep max reduction (these kernels sit at the register limit)
    int r3 = 0;
    double delta = 0.0;
    for (;;) {
      const double* din = (it & 1) ? bufB : bufA;
      double* dout = (it & 1) ? bufA : bufB;
      unsigned long long mx = 0ull;
#pragma unroll
      for (int j = 0; j < SPT; ++j) {
        const int s = tid + j * nt;
        if (s < S) {
          double acc = 0.0;
#pragma unroll
          for (int k = 0; k < KMAX; ++k)
            if (k < K) acc = fma(w[j][k], din[nb[j][k]], acc);
          const double nv = p0[j] + acc;
          dout[s] = nv;
          const unsigned long long d = abs_bits(nv - cur[j]);
          mx = d > mx ? d : mx;
          cur[j] = nv;
        }
      }
      mx = wave_max_u64(mx);
      if ((tid & (kWave - 1)) == 0 && mx) atomicMax(&slot[r3], mx);
      if (tid == 0) slot[r3 == 2 ? 0 : r3 + 1] = 0ull;
      __syncthreads();
      delta = bits_double(slot[r3]);
      r3 = r3 == 2 ? 0 : r3 + 1;
      ++it;
      if (!(delta > a.eps)) break;
      if (a.max_iter > 0 && it >= a.max_iter) break;
    }
    status = finish_status(delta, a.eps);
  }
#pragma unroll
  for (int j = 0; j < SPT; ++j) {
    const int s = tid + j * nt;
    if (s < S) a.out[(size_t)b * S + s] = cur[j];
  }
  if (tid == 0) { a.iters[b] = it; a.status[b] = status; }
}

struct BwdArgs {
  Model m;
  const double* w;  // [B][K][S] collapsed, reward-folded weights
  const double* reward;
  const uint8_t* term;
  int rescale;
  double* pi;  // [B][S][A]
  int32_t* status;
};

template <int SPT, int KMAX>
__global__ void __launch_bounds__(1024) bwd_fused_kernel(BwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const Model& m = a.m;
  const int S = m.S, K = m.K, A = m.A;
  const int b = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
  double* bufA = (double*)smem;
  double* bufB = bufA + S;
  unsigned long long* slot = (unsigned long long*)(bufB + S);

  double w[SPT][KMAX];
  int nb[SPT][KMAX];
  const double* wb = a.w + (size_t)b * K * S;
#pragma unroll
  for (int j = 0; j < SPT; ++j) {
    const int s = tid + j * nt;
#pragma unroll
    for (int k = 0; k < KMAX; ++k) { w[j][k] = 0.0; nb[j][k] = 0; }
    if (s < S) {
#pragma unroll
      for (int k = 0; k < KMAX; ++k)
        if (k < K) { w[j][k] = wb[(size_t)k * S + s]; nb[j][k] = row_nbr(m, b, s, k); }
    }
  }
  for (int s = tid; s < S; s += nt) bufA[s] = a.term[(size_t)b * S + s] ? 1.0 : 0.0;
  if (tid < 3) slot[tid] = 0ull;
  __syncthreads();

  // 2*S sweeps in all (maxent.py:154): the first 2*S - 1 on the action-summed
  // table, the last one per action because it also produces za.
  const long long collapsed = 2LL * S - 1;
  int e = 0, r3 = 0;
  bool nf = false;  // some partition value went non-finite (see bwd_nonfinite_rule)
  for (long long it = 0; it < collapsed; ++it) {
    const double* din = (it & 1) ? bufB : bufA;
    double* dout = (it & 1) ? bufA : bufB;
    if (a.rescale && it > 0) e = rescale_exponent(bits_double(slot[r3 == 0 ? 2 : r3 - 1]));
    unsigned long long mx = 0ull;
#pragma unroll
    for (int j = 0; j < SPT; ++j) {
      const int s = tid + j * nt;
      if (s < S) {
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k < KMAX; ++k)
          if (k < K) acc = fma(w[j][k], din[nb[j][k]], acc);
        const double nv = ldexp(acc, e);
        dout[s] = nv;
        const unsigned long long d = abs_bits(nv);
        mx = d > mx ? d : mx;
        nf |= !isfinite(nv);
      }
    }
    if (a.rescale) {
      mx = wave_max_u64(mx);
      if ((tid & (kWave - 1)) == 0 && mx) atomicMax(&slot[r3], mx);
      if (tid == 0) slot[r3 == 2 ? 0 : r3 + 1] = 0ull;
    }
    __syncthreads();
    r3 = r3 == 2 ? 0 : r3 + 1;
  }
  const double* zs = (collapsed & 1) ? bufB : bufA;
  if (a.rescale && collapsed > 0) e = rescale_exponent(bits_double(slot[r3 == 0 ? 2 : r3 - 1]));
  const bool all_nan = __syncthreads_or(nf);
#pragma unroll
  for (int j = 0; j < SPT; ++j) {
    const int s = tid + j * nt;
    if (s < S && all_nan) {
      for (int act = 0; act < A; ++act) a.pi[((size_t)b * S + s) * A + act] = kNaN;
    } else if (s < S) {
      const double er = exp(a.reward[(size_t)b * S + s]);
      double za[kMaxActions];
      double zsum = 0.0;
      for (int act = 0; act < A; ++act) {
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k < KMAX; ++k)
          if (k < K) acc = fma(row_val(m, b, act, k, s), zs[nb[j][k]], acc);
        za[act] = ldexp(__dmul_rn(er, acc), e);  // rounded product, then the sum (maxent.py:155-156)
        zsum = __dadd_rn(zsum, za[act]);
      }
      for (int act = 0; act < A; ++act) a.pi[((size_t)b * S + s) * A + act] = za[act] / zsum;
    }
  }
  if (tid == 0) a.status[b] = IRLMX_OK;
}

// ---------------------------------------------------------------------------
// backward pass in numpy's floating-point order (irlmx_backward_maxent_numpy_order)
// ---------------------------------------------------------------------------
//
// maxent.py:142-159 with every rounding where numpy / OpenBLAS put it on a
// Haswell-family x86-64 host (oracle/blas_order.c states and pins the order):
// p[a].dot(zs) per action -- four lane accumulators by column % 4 over the
// first S & ~3 columns (fma lanes for rows s < S & ~3, rounded-product lanes
// for the last row when S % 4 == 1; blocks of 2048 columns), lane sum
// (l0 + l2) + (l1 + l3), the last column fused on -- then er * dot rounded,
// zs = ((za0 + za1) + za2) + za3, and za / zs after exactly 2 S sweeps.  No
// rescaling: it overflows to NaN exactly where the reference does.  er is the
// caller's np.exp(reward) (ocml's exp may differ from numpy's in the last bit).
// One workgroup per instance; zs ping-pongs in LDS (S <= 4096).

constexpr int kNpBlock = 2048;  // OpenBLAS dgemv_t NBMAX

struct NpArgs {
  Model m;
  const double* er;     // [B][S] exp(reward), numpy's
  const uint8_t* term;  // [B][S]
  double* pi;           // [B][S][A]
  int32_t* status;
};

// one lane term: fma lanes (dgemv_kernel_4x4) or product-then-add lanes (dgemv_kernel_4x1)
__device__ inline void np_lane(double (&l)[2][4], int c, double v, double x, bool fused) {
  double& acc = l[c >= kNpBlock ? 1 : 0][c & 3];
  acc = fused ? fma(v, x, acc) : __dadd_rn(acc, __dmul_rn(v, x));
}

// p[a][s, :] . x in OpenBLAS dgemv_t order, from the row's stored entries in
// ascending column order (zero entries are exact no-ops while x is finite)
template <int LAYOUT>
__device__ double np_row_dot(const Model& m, int b, int a, int s, const double* x) {
  const int S = m.S, m1 = S & ~3;
  const bool fused = s < m1;
  double l[2][4] = {{0.0, 0.0, 0.0, 0.0}, {0.0, 0.0, 0.0, 0.0}};
  double tail_v = 0.0;
  bool tail = false;
  auto put = [&](int c, double v) {
    if (c < m1) np_lane(l, c, v, x[c], fused);
    // S % 4 == 1: the one column c = S - 1 (an unused ELL slot may repeat it with value 0)
    else if (!tail || v != 0.0) { tail = true; tail_v = v; }
  };
  if (LAYOUT == IRLMX_LAYOUT_STENCIL5) {
    // ascending columns: -y, -x, self, +x, +y (k = 4, 2, 0, 1, 3)
    constexpr int order[kStencilK] = {4, 2, 0, 1, 3};
#pragma unroll
    for (int i = 0; i < kStencilK; ++i) {
      const int k = order[i];
      if (stencil_valid(s, k, m.W, m.H)) put(stencil_nbr(s, k, m.W, m.H), row_val(m, b, a, k, s));
    }
  } else if (LAYOUT == IRLMX_LAYOUT_ELL) {
    for (int k = 0; k < m.K; ++k) put(row_nbr(m, b, s, k), row_val(m, b, a, k, s));
  } else {
    const double* row = m.row_val + ((inst_of(m, b) * m.A + a) * (size_t)S + s) * S;
    for (int c = 0; c < S; ++c) put(c, row[c]);
  }
  double y = __dadd_rn(0.0, __dadd_rn(__dadd_rn(l[0][0], l[0][2]), __dadd_rn(l[0][1], l[0][3])));
  if (m1 > kNpBlock) y = __dadd_rn(y, __dadd_rn(__dadd_rn(l[1][0], l[1][2]), __dadd_rn(l[1][1], l[1][3])));
  if (tail) y = fma(tail_v, x[S - 1], y);
  return y;
}

// p'[a][:, t] . x in OpenBLAS dgemv_n order (numpy's P_a.T.dot(x), maxent.py:109;
// oracle/blas_order.c blas_order_dgemv_cols): for t < S & ~3 the sources in
// groups of four, each group one chain c = fma(.., c) in source order 4g + 1,
// 4g, 4g + 2, 4g + 3 (its first term a rounded product), added to the sum group
// after group; a last source s = S - 1 (S % 4 == 1) as a rounded product added
// last; the last output t = S - 1 one fma chain over the sources in order.
// Zero entries (terminal sources, unused slots) are exact no-ops while x is
// finite, so only stored entries are visited.  xs(s) = pi[s, a] * d[s], rounded.
constexpr int kNpColMax = 32;  // ELL column slots the numpy-order forward supports

template <int LAYOUT, typename XS>
__device__ double np_col_dot(const Model& m, int b, int a, int t, const uint8_t* term, XS xs) {
  const int S = m.S, n4 = S & ~3;
  if (LAYOUT == IRLMX_LAYOUT_DENSE) {
    const double* col = m.row_val + (inst_of(m, b) * m.A + a) * (size_t)S * S + t;  // P[s, t, a] at s * S
    auto v = [&](int s) { return term[s] ? 0.0 : col[(size_t)s * S]; };
    double out = 0.0;
    if (t >= n4) {
      for (int s = 0; s < S; ++s) out = fma(v(s), xs(s), out);
      return out;
    }
    for (int s = 0; s < n4; s += 4) {
      double c = __dmul_rn(v(s + 1), xs(s + 1));
      c = fma(v(s), xs(s), c);
      c = fma(v(s + 2), xs(s + 2), c);
      c = fma(v(s + 3), xs(s + 3), c);
      out = __dadd_rn(out, c);
    }
    for (int s = n4; s < S; ++s) out = __dadd_rn(out, __dmul_rn(v(s), xs(s)));
    return out;
  }
  // stored entries of column t, ascending by source
  constexpr int KM = LAYOUT == IRLMX_LAYOUT_STENCIL5 ? kStencilK : kNpColMax;
  int src[KM];
  double val[KM];
  int n = 0;
  if (LAYOUT == IRLMX_LAYOUT_STENCIL5) {
    constexpr int order[kStencilK] = {4, 2, 0, 1, 3};  // sources t - W, t - 1, t, t + 1, t + W
#pragma unroll
    for (int i = 0; i < kStencilK; ++i) {
      const int k = order[i];
      if (!stencil_valid(t, k, m.W, m.H)) continue;
      const int s = stencil_nbr(t, k, m.W, m.H);
      if (term[s]) continue;
      src[n] = s;
      val[n] = row_val(m, b, a, stencil_opposite(k), s);  // P[s, t, a]
      ++n;
    }
  } else {
    for (int k = 0; k < m.Kc && k < kNpColMax; ++k) {
      const int s = col_src(m, b, t, k);
      const double v = m.col_val[((inst_of(m, b) * m.A + a) * m.Kc + k) * S + t];
      if (term[s] || v == 0.0) continue;
      int j = n++;  // insertion by source (unused slots repeat t with value 0 and are skipped)
      for (; j > 0 && src[j - 1] > s; --j) { src[j] = src[j - 1]; val[j] = val[j - 1]; }
      src[j] = s;
      val[j] = v;
    }
  }
  double out = 0.0;
  if (t >= n4) {
    for (int i = 0; i < n; ++i) out = fma(val[i], xs(src[i]), out);
    return out;
  }
  int i = 0;
  while (i < n && src[i] < n4) {
    const int g = src[i] >> 2;
    int e = i;
    while (e < n && src[e] < n4 && (src[e] >> 2) == g) ++e;
    double c = 0.0;
    constexpr int qorder[4] = {1, 0, 2, 3};
#pragma unroll
    for (int qi = 0; qi < 4; ++qi)
      for (int j = i; j < e; ++j)
        if ((src[j] & 3) == qorder[qi]) c = fma(val[j], xs(src[j]), c);
    out = __dadd_rn(out, c);
    i = e;
  }
  for (; i < n; ++i) out = __dadd_rn(out, __dmul_rn(val[i], xs(src[i])));
  return out;
}

struct NpFwdArgs {
  Model m;
  const double* p0;     // [B][S]
  const uint8_t* term;  // [B][S]
  const double* pi;     // [B][S][A]
  double eps;
  long long max_iter;
  double* svf;          // [B][S]
  int64_t* iters;
  int32_t* status;
};

// Forward in numpy's order (irlmx_forward_svf_numpy_order): maxent.py:105-114
// with every rounding where numpy puts it -- x_a = pi[:, a] * d, y_a = P'_a^T x_a
// (np_col_dot), d_ = p0 + (((y_0 + y_1) + y_2) + ...), delta = max|d_ - d| -- so
// the SVF and the sweep count are bit-identical to the reference's on a
// Haswell-family host.  A non-finite policy or value meets the zero entries of
// the dense product (0 * NaN): every later entry is NaN, as in the reference.
template <int LAYOUT>
__global__ void __launch_bounds__(1024) fwd_numpy_order_kernel(NpFwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const Model& m = a.m;
  const int S = m.S, A = m.A;
  const int b = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
  double* const buf0 = (double*)smem;  // (two named LDS pointers, not an array: ds_* accesses, not flat)
  double* const buf1 = buf0 + S;
  unsigned long long* slot = (unsigned long long*)(buf1 + S);  // [3] delta ring
  int* bad = (int*)(slot + 3);                                     // [2] sticky non-finite, by parity
  const double* pi = a.pi + (size_t)b * S * A;
  const double* p0 = a.p0 + (size_t)b * S;
  const uint8_t* term = a.term + (size_t)b * S;
  bool nf = false;
  for (int s = tid; s < S; s += nt) {
    buf0[s] = 0.0;  // maxent.py:105
    for (int act = 0; act < A; ++act) nf |= !isfinite(pi[(size_t)s * A + act]);
  }
  if (tid < 3) slot[tid] = 0ull;
  if (tid < 2) bad[tid] = 0;
  __syncthreads();
  if (nf) bad[1] = 1;  // a non-finite policy: the first sweep's product is NaN everywhere
  __syncthreads();
  long long it = 0;
  int r3 = 0;
  double delta = 0.0;
  for (;;) {
    const double* d = ((it & 1) ? buf1 : buf0);
    double* dn = ((it & 1) ? buf0 : buf1);
    const bool poisoned = bad[(it & 1) ^ 1] != 0;  // written in the previous sweep (or above)
    unsigned long long mx = 0ull;
    bool nfo = false;
    for (int t = tid; t < S; t += nt) {
      double v = 0.0;
      for (int act = 0; act < A; ++act) {
        auto xs = [&](int s) { return __dmul_rn(pi[(size_t)s * A + act], d[s]); };  // maxent.py:109
        const double y = poisoned ? kNaN : np_col_dot<LAYOUT>(m, b, act, t, term, xs);
        v = act == 0 ? y : __dadd_rn(v, y);  // np.array(d_).sum(axis=0)
      }
      const double nv = __dadd_rn(p0[t], v);  // maxent.py:110
      dn[t] = nv;
      nfo |= !isfinite(nv);
      const unsigned long long dd = abs_bits(nv - d[t]);
      mx = dd > mx ? dd : mx;
    }
    if (nfo) bad[it & 1] = 1;
    mx = wave_max_u64(mx);
    if ((tid & (kWave - 1)) == 0 && mx) atomicMax(&slot[r3], mx);
    if (tid == 0) slot[r3 == 2 ? 0 : r3 + 1] = 0ull;
    __syncthreads();
    delta = bits_double(slot[r3]);
    r3 = r3 == 2 ? 0 : r3 + 1;
    ++it;
    if (!(delta > a.eps)) break;  // maxent.py:108
    if (a.max_iter > 0 && it >= a.max_iter) break;
  }
  const double* d = ((it & 1) ? buf1 : buf0);
  for (int t = tid; t < S; t += nt) a.svf[(size_t)b * S + t] = d[t];
  if (tid == 0) {
    a.iters[b] = it;
    a.status[b] = finish_status(delta, a.eps);
  }
}

// The same forward for a STENCIL5 model with TPT targets per thread (512
// threads; S <= 1024, A <= 4): each thread keeps its targets' sources, the
// processing order of np_col_dot and every P[s, t, a] and pi[s, a] it
// multiplies in registers, so a sweep is five LDS reads per target and the
// chains -- no global load, no index arithmetic (the general kernel re-derives
// them every sweep, ~15 us per sweep at 64 states).
constexpr int kNpCachedThreads = 512;
constexpr int kNpCachedMaxStates = 2 * kNpCachedThreads;
constexpr int kNpCachedMaxActions = 4;
template <int TPT>
__global__ void __launch_bounds__(kNpCachedThreads) fwd_numpy_order_cached_kernel(NpFwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const Model& m = a.m;
  const int S = m.S, A = m.A, n4 = S & ~3;
  const int b = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
  double* const buf0 = (double*)smem;  // (two named LDS pointers, not an array: ds_* accesses, not flat)
  double* const buf1 = buf0 + S;
  unsigned long long* slot = (unsigned long long*)(buf1 + S);
  int* bad = (int*)(slot + 3);
  const double* pi = a.pi + (size_t)b * S * A;
  const uint8_t* term = a.term + (size_t)b * S;
  // per target j: entries in processing order; kind: 0 chain continues, 1 chain
  // starts (the previous chain's sum added first), 2 tail source (rounded
  // product added), 3 tail output (one fma chain).  (Every array is indexed by
  // compile-time constants only: registers, not scratch.)
  int src[TPT][kStencilK], kind[TPT][kStencilK], n[TPT];
  double val[TPT][kNpCachedMaxActions][kStencilK], pw[TPT][kNpCachedMaxActions][kStencilK], p0t[TPT];
  constexpr int order[kStencilK] = {4, 2, 0, 1, 3};  // candidate sources t - W, t - 1, t, t + 1, t + W
#pragma unroll
  for (int j = 0; j < TPT; ++j) {
    const int t = tid + j * nt;
    n[j] = 0;
    p0t[j] = 0.0;
#pragma unroll
    for (int p = 0; p < kStencilK; ++p) {
      src[j][p] = 0;
      kind[j][p] = 0;
#pragma unroll
      for (int act = 0; act < kNpCachedMaxActions; ++act) { val[j][act][p] = 0.0; pw[j][act][p] = 0.0; }
    }
    if (t >= S) continue;
    p0t[j] = a.p0[(size_t)b * S + t];
    int cs[kStencilK], key[kStencilK];
    bool ok[kStencilK];
#pragma unroll
    for (int i = 0; i < kStencilK; ++i) {
      ok[i] = stencil_valid(t, order[i], m.W, m.H);
      cs[i] = stencil_nbr(t, order[i], m.W, m.H);
      ok[i] = ok[i] && !term[cs[i]];  // P' rows of terminal states are zero (maxent.py:99)
      // processing key: group, then source order 4g + 1, 4g, 4g + 2, 4g + 3; tail sources after
      const int q = cs[i] & 3;
      key[i] = t >= n4 ? cs[i] : (cs[i] < n4 ? 4 * (cs[i] >> 2) + (q == 1 ? 0 : q == 0 ? 1 : q) : 4 * S + cs[i]);
    }
#pragma unroll
    for (int i = 0; i < kStencilK; ++i) {
      if (!ok[i]) continue;
      int pos = 0;
      bool first = true;  // lowest key of its group among the valid sources
#pragma unroll
      for (int q = 0; q < kStencilK; ++q) {
        pos += (ok[q] && key[q] < key[i]) ? 1 : 0;
        first = first && !(ok[q] && key[q] < key[i] && (cs[q] >> 2) == (cs[i] >> 2));
      }
      const int kd = t >= n4 ? 3 : (cs[i] >= n4 ? 2 : (first ? 1 : 0));
#pragma unroll
      for (int p = 0; p < kStencilK; ++p)
        if (pos == p) {
          src[j][p] = cs[i];
          kind[j][p] = kd;
#pragma unroll
          for (int act = 0; act < kNpCachedMaxActions; ++act) {
            val[j][act][p] = act < A ? row_val(m, b, act, stencil_opposite(order[i]), cs[i]) : 0.0;
            pw[j][act][p] = act < A ? pi[(size_t)cs[i] * A + act] : 0.0;
          }
        }
      ++n[j];
    }
  }
  bool nf = false;
  for (int s = tid; s < S; s += nt) {
    buf0[s] = 0.0;  // maxent.py:105
    for (int act = 0; act < A; ++act) nf |= !isfinite(pi[(size_t)s * A + act]);
  }
  if (tid < 3) slot[tid] = 0ull;
  if (tid < 2) bad[tid] = 0;
  __syncthreads();
  if (nf) bad[1] = 1;
  __syncthreads();
  // convergence deferred over blocks of sweeps, replay of the stopping block
  // (run_deferred); the poison flags bad[] are part of the block-start state
  long long it = 0;
  auto sweep = [&](long long it, int pos, unsigned long long& bits) __attribute__((always_inline)) {
    const double* d = ((it & 1) ? buf1 : buf0);
    double* dn = ((it & 1) ? buf0 : buf1);
    const bool poisoned = bad[(it & 1) ^ 1] != 0;
    bool nfo = false;
#pragma unroll
    for (int j = 0; j < TPT; ++j) {
      const int t = tid + j * nt;
      if (t >= S) continue;
      double dv[kStencilK];
#pragma unroll
      for (int i = 0; i < kStencilK; ++i) dv[i] = d[src[j][i]];  // (unused entries: src 0, selected away below)
      // all actions' chains side by side, branch-free (the entries' kinds differ
      // between lanes): every step computes its candidates and selects, so the
      // four independent chains interleave instead of diverging
      double out[kNpCachedMaxActions], c[kNpCachedMaxActions];
#pragma unroll
      for (int act = 0; act < kNpCachedMaxActions; ++act) { out[act] = 0.0; c[act] = 0.0; }
      bool open = false;
#pragma unroll
      for (int i = 0; i < kStencilK; ++i) {
        const int kd = i < n[j] ? kind[j][i] : -1;  // -1: no entry
        const bool flush = open && (kd == 1 || kd == 2);
#pragma unroll
        for (int act = 0; act < kNpCachedMaxActions; ++act) {
          // every candidate computed, then selected: a conditional operator
          // around an arithmetic call compiles to an exec-mask branch per step
          const double vv = val[j][act][i];
          const double x = __dmul_rn(pw[j][act][i], dv[i]);  // maxent.py:109
          const double oc = __dadd_rn(out[act], c[act]);
          const double o1 = flush ? oc : out[act];
          const double cf = fma(vv, x, kd == 1 ? 0.0 : c[act]);
          const double f3 = fma(vv, x, out[act]);
          const double a2 = __dadd_rn(o1, __dmul_rn(vv, x));
          c[act] = (kd == 0 || kd == 1) ? cf : c[act];
          out[act] = kd == 3 ? f3 : (kd == 2 ? a2 : o1);
        }
        open = kd == 1 ? true : (kd == 2 ? false : open);
      }
      double v = 0.0;
#pragma unroll
      for (int act = 0; act < kNpCachedMaxActions; ++act) {
        if (act >= A) break;
        const double oc = __dadd_rn(out[act], c[act]);
        const double o = open ? oc : out[act];
        const double y = poisoned ? kNaN : o;
        v = act == 0 ? y : __dadd_rn(v, y);  // np.array(d_).sum(axis=0)
      }
      const double nv = __dadd_rn(p0t[j], v);  // maxent.py:110
      dn[t] = nv;
      nfo |= !isfinite(nv);
      record_delta(bits, pos, fabs(nv - d[t]), a.eps);
    }
    if (nfo) bad[it & 1] = 1;
  };
  double keep[TPT];
  int bad0 = 0, bad1 = 0;
  const int status = run_deferred(
      a.max_iter, slot, it, sweep,
      [&]() {
        const double* d0 = ((it & 1) ? buf1 : buf0);
#pragma unroll
        for (int j = 0; j < TPT; ++j) keep[j] = tid + j * nt < S ? d0[tid + j * nt] : 0.0;
        bad0 = bad[0];
        bad1 = bad[1];
      },
      [&]() {
        double* d0w = ((it & 1) ? buf1 : buf0);
#pragma unroll
        for (int j = 0; j < TPT; ++j)
          if (tid + j * nt < S) d0w[tid + j * nt] = keep[j];
        __syncthreads();  // every lane past its reads of bad[] before they are restored
        if (tid == 0) { bad[0] = bad0; bad[1] = bad1; }
        __syncthreads();
      });
  for (int t = tid; t < S; t += nt) a.svf[(size_t)b * S + t] = ((it & 1) ? buf1 : buf0)[t];
  if (tid == 0) {
    a.iters[b] = it;
    a.status[b] = status;
  }
}

// A thread's stencil rows in registers for the numpy-order kernels (TPT states
// per thread, A <= 4): per state j and candidate column i (ascending: -y, -x,
// self, +x, +y) the column, its dgemv lane (column % 4; 4 = the last column
// S - 1 of an S % 4 == 1 grid, fused on after the lane sum; -1 = off-grid) and
// P[s, c, a] -- np_row_dot's arithmetic without re-deriving indices or
// re-loading P every sweep.  Static indices only: registers, not scratch.
template <int TPT>
struct NpStencilRows {
  int col[TPT][kStencilK], lane[TPT][kStencilK];
  double val[TPT][kNpCachedMaxActions][kStencilK];

  __device__ __attribute__((always_inline)) void load(const Model& m, int b, int tid, int nt) {
    constexpr int order[kStencilK] = {4, 2, 0, 1, 3};
    const int S = m.S, m1 = S & ~3;
#pragma unroll
    for (int j = 0; j < TPT; ++j) {
      const int s = tid + j * nt;
#pragma unroll
      for (int i = 0; i < kStencilK; ++i) {
        const bool ok = s < S && stencil_valid(s, order[i], m.W, m.H);
        col[j][i] = ok ? stencil_nbr(s, order[i], m.W, m.H) : 0;
        lane[j][i] = ok ? (col[j][i] < m1 ? (col[j][i] & 3) : 4) : -1;
#pragma unroll
        for (int act = 0; act < kNpCachedMaxActions; ++act)
          val[j][act][i] = (ok && act < m.A) ? row_val(m, b, act, order[i], s) : 0.0;
      }
    }
  }
  // the vector at state j's columns
  __device__ __attribute__((always_inline)) void gather(int j, const double* v, double (&x)[kStencilK]) const {
#pragma unroll
    for (int i = 0; i < kStencilK; ++i) x[i] = lane[j][i] >= 0 ? v[col[j][i]] : 0.0;
  }
  // p[act][s, :] . v in OpenBLAS dgemv_t order (fused: rows s < S & ~3)
  __device__ __attribute__((always_inline)) double dot(int j, int act, bool fused, const double (&x)[kStencilK]) const {
    double l[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int i = 0; i < kStencilK; ++i)  // ascending columns within a lane
        if (lane[j][i] == q)
          l[q] = fused ? fma(val[j][act][i], x[i], l[q]) : __dadd_rn(l[q], __dmul_rn(val[j][act][i], x[i]));
    double y = __dadd_rn(0.0, __dadd_rn(__dadd_rn(l[0], l[2]), __dadd_rn(l[1], l[3])));
#pragma unroll
    for (int i = 0; i < kStencilK; ++i)
      if (lane[j][i] == 4) y = fma(val[j][act][i], x[i], y);
    return y;
  }
};

// The numpy-order backward for a STENCIL5 model with TPT states per thread
// (512 threads; S <= 1024, A <= 4), the rows in registers (NpStencilRows).
template <int TPT>
__global__ void __launch_bounds__(kNpCachedThreads) bwd_numpy_order_cached_kernel(NpArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const Model& m = a.m;
  const int S = m.S, A = m.A, m1 = S & ~3;
  const int b = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
  double* const zbuf0 = (double*)smem;  // (two named LDS pointers, not an array: ds_* accesses, not flat)
  double* const zbuf1 = zbuf0 + S;
  int* bad = (int*)(zbuf1 + S);
  const double* er = a.er + (size_t)b * S;
  double* pi = a.pi + (size_t)b * S * A;
  NpStencilRows<TPT> rows;
  rows.load(m, b, tid, nt);
  double ers[TPT];
#pragma unroll
  for (int j = 0; j < TPT; ++j) ers[j] = tid + j * nt < S ? er[tid + j * nt] : 0.0;
  for (int s = tid; s < S; s += nt) zbuf0[s] = a.term[(size_t)b * S + s] ? 1.0 : 0.0;  // maxent.py:146-147
  if (tid < 2) bad[tid] = 0;
  __syncthreads();
  const long long n = 2LL * S;  // maxent.py:154
  for (long long it = 0; it < n; ++it) {
    const double* zin = ((it & 1) ? zbuf1 : zbuf0);
    double* zout = ((it & 1) ? zbuf0 : zbuf1);
    if (it > 0 && bad[(it - 1) & 1]) {  // the reference's overflow: NaN from here on (bwd_numpy_order_kernel)
      for (int s = tid; s < S; s += nt)
        for (int act = 0; act < A; ++act) pi[(size_t)s * A + act] = kNaN;
      if (tid == 0) a.status[b] = IRLMX_OK;
      return;
    }
    bool nf = false;
#pragma unroll
    for (int j = 0; j < TPT; ++j) {
      const int s = tid + j * nt;
      if (s >= S) continue;
      double x[kStencilK];
      rows.gather(j, zin, x);
      double z = 0.0;
#pragma unroll
      for (int act = 0; act < kNpCachedMaxActions; ++act) {
        if (act >= A) break;
        const double za = __dmul_rn(ers[j], rows.dot(j, act, s < m1, x));  // maxent.py:155
        z = act == 0 ? za : __dadd_rn(z, za);                               // maxent.py:156
        if (it == n - 1) pi[(size_t)s * A + act] = za;
      }
      zout[s] = z;
      nf |= !isfinite(z);
    }
    if (nf) bad[it & 1] = 1;
    __syncthreads();
  }
  const double* zs = ((n & 1) ? zbuf1 : zbuf0);
  for (int s = tid; s < S; s += nt)
    for (int act = 0; act < A; ++act) pi[(size_t)s * A + act] = pi[(size_t)s * A + act] / zs[s];  // maxent.py:159
  if (tid == 0) a.status[b] = IRLMX_OK;
}

template <int LAYOUT>
__global__ void __launch_bounds__(1024) bwd_numpy_order_kernel(NpArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const Model& m = a.m;
  const int S = m.S, A = m.A;
  const int b = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
  double* const zbuf0 = (double*)smem;  // (two named LDS pointers, not an array: ds_* accesses, not flat)
  double* const zbuf1 = zbuf0 + S;
  int* bad = (int*)(zbuf1 + S);  // [2] sticky: sweep k's output had a non-finite value (slot k & 1)
  const double* er = a.er + (size_t)b * S;
  double* pi = a.pi + (size_t)b * S * A;
  for (int s = tid; s < S; s += nt) zbuf0[s] = a.term[(size_t)b * S + s] ? 1.0 : 0.0;  // maxent.py:146-147
  if (tid < 2) bad[tid] = 0;
  __syncthreads();
  const long long n = 2LL * S;  // maxent.py:154
  for (long long it = 0; it < n; ++it) {
    const double* zin = ((it & 1) ? zbuf1 : zbuf0);
    double* zout = ((it & 1) ? zbuf0 : zbuf1);
    // a non-finite zs meets a zero entry of every dense row (0 * inf): the
    // reference's next dots are all NaN (a DENSE row visits every column itself)
    const bool poisoned = LAYOUT != IRLMX_LAYOUT_DENSE && it > 0 && bad[(it - 1) & 1];
    if (poisoned) {
      // from here every dot, za and zs is NaN (the overflow the reference hits at
      // about 13 x 13 and unit reward): the policy is NaN, no need to sweep on
      for (int s = tid; s < S; s += nt)
        for (int act = 0; act < A; ++act) pi[(size_t)s * A + act] = kNaN;
      if (tid == 0) a.status[b] = IRLMX_OK;
      return;
    }
    bool nf = false;
    for (int s = tid; s < S; s += nt) {
      double z = 0.0;
      for (int act = 0; act < A; ++act) {
        const double dot = np_row_dot<LAYOUT>(m, b, act, s, zin);
        const double za = __dmul_rn(er[s], dot);                 // maxent.py:155
        z = act == 0 ? za : __dadd_rn(z, za);                    // maxent.py:156
        if (it == n - 1) pi[(size_t)s * A + act] = za;
      }
      zout[s] = z;
      nf |= !isfinite(z);
    }
    if (nf) bad[it & 1] = 1;
    __syncthreads();
  }
  const double* zs = ((n & 1) ? zbuf1 : zbuf0);
  for (int s = tid; s < S; s += nt)
    for (int act = 0; act < A; ++act) pi[(size_t)s * A + act] = pi[(size_t)s * A + act] / zs[s];  // maxent.py:159
  if (tid == 0) a.status[b] = IRLMX_OK;
}

struct SoftArgs {
  Model m;
  const double* reward;
  const double* phi;  // soft: terminal reward; unused by VI
  double discount;
  double eps;
  long long max_iter;
  int average;  // VI only
  double* pi;   // soft only, [B][S][A]
  double* value;
  int64_t* iters;
  int32_t* status;
};

// per-state Bellman update shared by the fused and the sweep shapes.
// NB: neighbour lookup; CACHED uses the per-thread register copy.
template <bool SOFT, int KMAX, bool CACHED>
__device__ inline double bellman_update(const SoftArgs& a, int b, int s, const int* nb,
                                        const double* vin, double r, double phi) {
  const Model& m = a.m;
  const int K = m.K, A = m.A;
  double v = SOFT ? phi : 0.0;
#pragma unroll 1
  for (int act = 0; act < A; ++act) {
    double dot = 0.0;
    if (CACHED) {
#pragma unroll
      for (int k = 0; k < KMAX; ++k)
        if (k < K) dot = fma(row_val(m, b, act, k, s), vin[nb[k]], dot);
    } else {
      for (int k = 0; k < K; ++k) dot = fma(row_val(m, b, act, k, s), vin[row_nbr(m, b, s, k)], dot);
    }
    if (SOFT) {
      v = softmax2(v, __dadd_rn(r, __dmul_rn(a.discount, dot)));  // maxent.py:329-333
    } else {
      const double q = __dmul_rn(a.discount, dot);  // solver.py:44
      if (a.average) v = act == 0 ? q : __dadd_rn(v, q);
      else v = act == 0 ? q : ((v != v || q <= v) ? v : q);
    }
  }
  if (!SOFT) v = __dadd_rn(r, a.average ? v / (double)A : v);  // solver.py:47 / :99
  return v;
}

template <int KMAX, bool CACHED>
__device__ inline void soft_policy_row(const SoftArgs& a, int b, int s, const int* nb,
                                       const double* vold, double vnew, double r) {
  const Model& m = a.m;
#pragma unroll 1
  for (int act = 0; act < m.A; ++act) {
    double dot = 0.0;
    if (CACHED) {
#pragma unroll
      for (int k = 0; k < KMAX; ++k)
        if (k < m.K) dot = fma(row_val(m, b, act, k, s), vold[nb[k]], dot);
    } else {
      for (int k = 0; k < m.K; ++k) dot = fma(row_val(m, b, act, k, s), vold[row_nbr(m, b, s, k)], dot);
    }
    const double q = __dadd_rn(r, __dmul_rn(a.discount, dot));
    a.pi[((size_t)b * m.S + s) * m.A + act] = np_exp(q - vnew);  // maxent.py:341
  }
}

template <bool SOFT, int SPT, int KMAX>
__device__ __forceinline__ void bellman_fused_body(const SoftArgs& a, unsigned char* smem) {
  const Model& m = a.m;
  const int S = m.S, K = m.K;
  const int b = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
  double* bufA = (double*)smem;
  double* bufB = bufA + S;
  unsigned long long* slot = (unsigned long long*)(bufB + S);
  double* snap = (double*)(slot + 4);  // run_deferred's block-start state (LDS: the registers are taken)

  int nb[SPT][KMAX];
  double r[SPT], phi[SPT], cur[SPT];
  const double v0 = SOFT ? -1e200 : 0.0;  // maxent.py:323 / solver.py:32
#pragma unroll
  for (int j = 0; j < SPT; ++j) {
    const int s = tid + j * nt;
    r[j] = 0.0;
    phi[j] = 0.0;
    cur[j] = v0;
#pragma unroll
    for (int k = 0; k < KMAX; ++k) nb[j][k] = 0;
    if (s < S) {
      r[j] = a.reward[(size_t)b * S + s];
      if (SOFT) phi[j] = a.phi[(size_t)b * S + s];
#pragma unroll
      for (int k = 0; k < KMAX; ++k)
        if (k < K) nb[j][k] = row_nbr(m, b, s, k);
    }
  }
  for (int s = tid; s < S; s += nt) bufA[s] = v0;
  if (tid < 3) slot[tid] = 0ull;
  __syncthreads();

  long long it = 0;
  auto sweep = [&](long long it, int pos, unsigned long long& bits) __attribute__((always_inline)) {
    const double* vin = (it & 1) ? bufB : bufA;
    double* vout = (it & 1) ? bufA : bufB;
#pragma unroll
    for (int j = 0; j < SPT; ++j) {
      const int s = tid + j * nt;
      if (s < S) {
        const double v = bellman_update<SOFT, KMAX, true>(a, b, s, nb[j], vin, r[j], phi[j]);
        vout[s] = v;
        record_delta(bits, pos, fabs(v - cur[j]), a.eps);
        cur[j] = v;
      }
    }
  };
  // (VI converges in tens of sweeps, where a block's overshoot and replay cost
  // more than a reduction per sweep; the widest rows fill the registers: per-
  // sweep bits there too)
  int status;
  if constexpr (SOFT && SPT * KMAX < 32) {
    status = run_deferred(
        a.max_iter, slot, it, sweep,
        [&]() {
#pragma unroll
          for (int j = 0; j < SPT; ++j)
            if (tid + j * nt < S) snap[tid + j * nt] = cur[j];
        },
        [&]() {
          double* v0w = (it & 1) ? bufB : bufA;
#pragma unroll
          for (int j = 0; j < SPT; ++j)
            if (tid + j * nt < S) v0w[tid + j * nt] = cur[j] = snap[tid + j * nt];
          __syncthreads();
        });
  } else {
    status = run_each(a.max_iter, slot, it, sweep);
  }
  const double* vold = (it & 1) ? bufA : bufB;  // input of the last sweep
#pragma unroll
  for (int j = 0; j < SPT; ++j) {
    const int s = tid + j * nt;
    if (s < S) {
      if (a.value) a.value[(size_t)b * S + s] = cur[j];
      if (SOFT) soft_policy_row<KMAX, true>(a, b, s, nb[j], vold, cur[j], r[j]);
    }
  }
  if (tid == 0) {
    if (a.iters) a.iters[b] = it;
    a.status[b] = status;
  }
}

// Soft VI / VI in numpy's floating-point order (irlmx_soft_backward /
// irlmx_value_iteration with IRLMX_NUMPY_ORDER): every p[a].dot(v) as
// np_row_dot sums it, then the per-sweep kernel's statements.  VI has no
// transcendental function, so its values are bit-identical to the reference's
// on a Haswell-family host; soft VI's exp / log are ocml's (numpy's SIMD exp /
// log may differ in the last bit), its dot products follow numpy's order.
template <bool SOFT, int LAYOUT>
__global__ void __launch_bounds__(1024) bellman_numpy_order_kernel(SoftArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const Model& m = a.m;
  const int S = m.S, A = m.A;
  const int b = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
  __shared__ NpTables npt_lds;
  const NpTables* const npt = &npt_lds;
  double* const buf0 = (double*)smem;  // (two named LDS pointers, not an array: ds_* accesses, not flat)
  double* const buf1 = buf0 + S;
  unsigned long long* slot = (unsigned long long*)(buf1 + S);
  const double v0 = SOFT ? -1e200 : 0.0;  // maxent.py:323 / solver.py:29
  const double* rw = a.reward + (size_t)b * S;
  for (int s = tid; s < S; s += nt) buf0[s] = v0;
  if (tid < 3) slot[tid] = 0ull;
  if (SOFT) np_stage_tables(&npt_lds);  // numpy exp / log tables in LDS (common.h)
  __syncthreads();
  long long it = 0;
  int r3 = 0;
  double delta = 0.0;
  for (;;) {
    const double* vin = ((it & 1) ? buf1 : buf0);
    double* vout = ((it & 1) ? buf0 : buf1);
    unsigned long long mx = 0ull;
    for (int s = tid; s < S; s += nt) {
      const double r = rw[s];
      double v = SOFT ? a.phi[(size_t)b * S + s] : 0.0;
      for (int act = 0; act < A; ++act) {
        const double dot = np_row_dot<LAYOUT>(m, b, act, s, vin);
        if (SOFT) {
          v = softmax2(v, __dadd_rn(r, __dmul_rn(a.discount, dot)), npt, true);  // maxent.py:329-333
        } else {
          const double q = __dmul_rn(a.discount, dot);  // solver.py:44
          if (a.average) v = act == 0 ? q : __dadd_rn(v, q);
          else v = act == 0 ? q : ((v != v || q <= v) ? v : q);
        }
      }
      if (!SOFT) v = __dadd_rn(r, a.average ? v / (double)A : v);  // solver.py:47 / :99
      vout[s] = v;
      const unsigned long long d = abs_bits(v - vin[s]);
      mx = d > mx ? d : mx;
    }
    mx = wave_max_u64(mx);
    if ((tid & (kWave - 1)) == 0 && mx) atomicMax(&slot[r3], mx);
    if (tid == 0) slot[r3 == 2 ? 0 : r3 + 1] = 0ull;
    __syncthreads();
    delta = bits_double(slot[r3]);
    r3 = r3 == 2 ? 0 : r3 + 1;
    ++it;
    if (!(delta > a.eps)) break;
    if (a.max_iter > 0 && it >= a.max_iter) break;
  }
  const double* vold = ((it & 1) ? buf0 : buf1);  // input of the last sweep
  const double* vnew = ((it & 1) ? buf1 : buf0);
  for (int s = tid; s < S; s += nt) {
    if (a.value) a.value[(size_t)b * S + s] = vnew[s];
    if (SOFT)
      for (int act = 0; act < A; ++act) {
        const double q = __dadd_rn(rw[s], __dmul_rn(a.discount, np_row_dot<LAYOUT>(m, b, act, s, vold)));
        a.pi[((size_t)b * S + s) * A + act] = np_exp(q - vnew[s], npt);  // maxent.py:341
      }
  }
  if (tid == 0) {
    if (a.iters) a.iters[b] = it;
    a.status[b] = finish_status(delta, a.eps);
  }
}

// Soft VI / VI in numpy's order for a STENCIL5 model with TPT states per
// thread (512 threads; S <= 1024, A <= 4), the rows in registers (NpStencilRows).
template <bool SOFT, int TPT>
__global__ void __launch_bounds__(kNpCachedThreads) bellman_numpy_order_cached_kernel(SoftArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const Model& m = a.m;
  const int S = m.S, A = m.A, m1 = S & ~3;
  const int b = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
  __shared__ NpTables npt_lds;
  const NpTables* const npt = &npt_lds;
  double* const buf0 = (double*)smem;  // (two named LDS pointers, not an array: ds_* accesses, not flat)
  double* const buf1 = buf0 + S;
  unsigned long long* slot = (unsigned long long*)(buf1 + S);
  const double v0 = SOFT ? -1e200 : 0.0;  // maxent.py:323 / solver.py:29
  NpStencilRows<TPT> rows;
  rows.load(m, b, tid, nt);
  double rr[TPT], ph[TPT];
#pragma unroll
  for (int j = 0; j < TPT; ++j) {
    const int s = tid + j * nt;
    rr[j] = s < S ? a.reward[(size_t)b * S + s] : 0.0;
    ph[j] = (SOFT && s < S) ? a.phi[(size_t)b * S + s] : 0.0;
  }
  for (int s = tid; s < S; s += nt) buf0[s] = v0;
  if (tid < 3) slot[tid] = 0ull;
  if (SOFT) np_stage_tables(&npt_lds);  // numpy exp / log tables in LDS (common.h)
  __syncthreads();
  // convergence deferred over blocks of sweeps, replay of the stopping block
  // (run_deferred: the stop after the first sweep whose max|v_new - v| is not
  // > eps, NaN included -- solver.py:49, maxent.py:335)
  long long it = 0;
  auto sweep = [&](long long it, int pos, unsigned long long& bits) __attribute__((always_inline)) {
    const double* vin = ((it & 1) ? buf1 : buf0);
    double* vout = ((it & 1) ? buf0 : buf1);
#pragma unroll
    for (int j = 0; j < TPT; ++j) {
      const int s = tid + j * nt;
      if (s >= S) continue;
      double x[kStencilK];
      rows.gather(j, vin, x);
      double v = SOFT ? ph[j] : 0.0;
#pragma unroll
      for (int act = 0; act < kNpCachedMaxActions; ++act) {
        if (act >= A) break;
        const double dot = rows.dot(j, act, s < m1, x);
        if (SOFT) {
          v = softmax2(v, __dadd_rn(rr[j], __dmul_rn(a.discount, dot)), npt, true);  // maxent.py:329-333
        } else {
          const double q = __dmul_rn(a.discount, dot);  // solver.py:44
          if (a.average) v = act == 0 ? q : __dadd_rn(v, q);
          else v = act == 0 ? q : ((v != v || q <= v) ? v : q);
        }
      }
      if (!SOFT) v = __dadd_rn(rr[j], a.average ? v / (double)A : v);  // solver.py:47 / :99
      vout[s] = v;
      record_delta(bits, pos, fabs(v - vin[s]), a.eps);
    }
  };
  // (VI: a reduction per sweep, as in bellman_fused_body)
  double keep[TPT];
  int status;
  if constexpr (SOFT) {
    status = run_deferred(
        a.max_iter, slot, it, sweep,
        [&]() {
          const double* v0p = ((it & 1) ? buf1 : buf0);
#pragma unroll
          for (int j = 0; j < TPT; ++j) keep[j] = tid + j * nt < S ? v0p[tid + j * nt] : 0.0;
        },
        [&]() {
          double* v0w = ((it & 1) ? buf1 : buf0);
#pragma unroll
          for (int j = 0; j < TPT; ++j)
            if (tid + j * nt < S) v0w[tid + j * nt] = keep[j];
          __syncthreads();
        });
  } else {
    status = run_each(a.max_iter, slot, it, sweep);
  }
  const double* vold = ((it & 1) ? buf0 : buf1);  // input of the last sweep
  const double* vnew = ((it & 1) ? buf1 : buf0);
#pragma unroll
  for (int j = 0; j < TPT; ++j) {
    const int s = tid + j * nt;
    if (s >= S) continue;
    if (a.value) a.value[(size_t)b * S + s] = vnew[s];
    if (SOFT) {
      double x[kStencilK];
      rows.gather(j, vold, x);
#pragma unroll
      for (int act = 0; act < kNpCachedMaxActions; ++act) {
        if (act >= A) break;
        const double q = __dadd_rn(rr[j], __dmul_rn(a.discount, rows.dot(j, act, s < m1, x)));
        a.pi[((size_t)b * S + s) * A + act] = np_exp(q - vnew[s], npt);  // maxent.py:341
      }
    }
  }
  if (tid == 0) {
    if (a.iters) a.iters[b] = it;
    a.status[b] = status;
  }
}

template <int SPT, int KMAX>
__global__ void __launch_bounds__(1024) soft_fused_kernel(SoftArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bellman_fused_body<true, SPT, KMAX>(a, smem);
}

template <int SPT, int KMAX>
__global__ void __launch_bounds__(1024) vi_fused_kernel(SoftArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bellman_fused_body<false, SPT, KMAX>(a, smem);
}

// ---------------------------------------------------------------------------
// sweep (one launch per sweep, all instances) kernels
// ---------------------------------------------------------------------------

__device__ inline void block_max_to(unsigned long long v, unsigned long long* dst) {
  __shared__ unsigned long long red[kSweepThreads / kWave];
  v = wave_max_u64(v);
  const int wv = threadIdx.x / kWave;
  if ((threadIdx.x & (kWave - 1)) == 0) red[wv] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long m = 0;
    for (int i = 0; i < (int)(blockDim.x / kWave); ++i) m = red[i] > m ? red[i] : m;
    if (m) atomicMax(dst, m);
  }
}

// Common prologue: decides whether instance b converged after the previous
// sweep (`it` sweeps done so far); the first workgroup records the outcome.
__device__ inline bool sweep_should_stop(int b, long long it, int r3, double eps, long long max_iter,
                                         const Ws& ws, int32_t* status) {
  if (ws.done[b]) return true;
  if (it == 0) return false;
  const double prev = bits_double(ws.slots[b * 3 + (r3 == 0 ? 2 : r3 - 1)]);
  const bool cap = max_iter > 0 && it >= max_iter;
  if (prev > eps && !cap) return false;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    ws.done[b] = 1;
    ws.iters[b] = it;
    status[b] = finish_status(prev, eps);
    atomicAdd(ws.ndone, 1);
  }
  return true;
}

__global__ void __launch_bounds__(kSweepThreads)
fwd_sweep_kernel(FwdArgs a, Ws ws, long long it, int r3) {
  const Model& m = a.m;
  const int b = blockIdx.y;
  if (ws.bad[b]) {
    if (blockIdx.x == 0 && threadIdx.x == 0 && !ws.done[b]) {
      ws.done[b] = 1; ws.iters[b] = 1; a.status[b] = IRLMX_NONFINITE; atomicAdd(ws.ndone, 1);
    }
    return;
  }
  if (sweep_should_stop(b, it, r3, a.eps, a.max_iter, ws, a.status)) return;
  const int S = m.S;
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  const double* din = ((it & 1) ? ws.buf1 : ws.buf0) + (size_t)b * S;
  double* dout = ((it & 1) ? ws.buf0 : ws.buf1) + (size_t)b * S;
  unsigned long long d = 0ull;
  if (s < S) {
    const double* wb = a.w + (size_t)b * m.Kc * S;
    double acc = 0.0;
    for (int k = 0; k < m.Kc; ++k) acc = fma(wb[(size_t)k * S + s], din[col_src(m, b, s, k)], acc);
    const double nv = a.p0[(size_t)b * S + s] + acc;
    dout[s] = nv;
    d = abs_bits(nv - din[s]);
  }
  block_max_to(d, &ws.slots[b * 3 + r3]);
  if (blockIdx.x == 0 && threadIdx.x == 0) ws.slots[b * 3 + (r3 == 2 ? 0 : r3 + 1)] = 0ull;
}

__global__ void fwd_finish_kernel(FwdArgs a, Ws ws) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  const int S = a.m.S;
  if (s >= S) return;
  double v;
  if (ws.bad[b]) v = __longlong_as_double(0x7ff8000000000000LL);
  else v = ((ws.iters[b] & 1) ? ws.buf1 : ws.buf0)[(size_t)b * S + s];
  a.out[(size_t)b * S + s] = v;
  if (s == 0) a.iters[b] = ws.iters[b];
}

__global__ void __launch_bounds__(kSweepThreads)
bwd_sweep_kernel(BwdArgs a, Ws ws, long long it, int r3) {
  const Model& m = a.m;
  const int S = m.S;
  const int b = blockIdx.y;
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  const double* din = ((it & 1) ? ws.buf1 : ws.buf0) + (size_t)b * S;
  double* dout = ((it & 1) ? ws.buf0 : ws.buf1) + (size_t)b * S;
  int e = 0;
  if (a.rescale && it > 0) e = rescale_exponent(bits_double(ws.slots[b * 3 + (r3 == 0 ? 2 : r3 - 1)]));
  unsigned long long d = 0ull;
  if (s < S) {
    const double* wb = a.w + (size_t)b * m.K * S;
    double acc = 0.0;
    for (int k = 0; k < m.K; ++k) acc = fma(wb[(size_t)k * S + s], din[row_nbr(m, b, s, k)], acc);
    const double nv = ldexp(acc, e);
    dout[s] = nv;
    d = abs_bits(nv);
    if (!isfinite(nv)) atomicOr(&ws.bad[b], 1);  // bwd_nonfinite_rule
  }
  if (a.rescale) {
    block_max_to(d, &ws.slots[b * 3 + r3]);
    if (blockIdx.x == 0 && threadIdx.x == 0) ws.slots[b * 3 + (r3 == 2 ? 0 : r3 + 1)] = 0ull;
  }
}

__global__ void bwd_init_kernel(BwdArgs a, Ws ws) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (s >= a.m.S) return;
  ws.buf0[(size_t)b * a.m.S + s] = a.term[(size_t)b * a.m.S + s] ? 1.0 : 0.0;
}

__global__ void bwd_final_kernel(BwdArgs a, Ws ws, long long collapsed, int r3) {
  const Model& m = a.m;
  const int S = m.S, A = m.A;
  const int b = blockIdx.y;
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= S) return;
  if (ws.bad[b]) {  // bwd_nonfinite_rule
    for (int act = 0; act < A; ++act) a.pi[((size_t)b * S + s) * A + act] = kNaN;
    if (s == 0) a.status[b] = IRLMX_OK;
    return;
  }
  const double* zs = ((collapsed & 1) ? ws.buf1 : ws.buf0) + (size_t)b * S;
  int e = 0;
  if (a.rescale && collapsed > 0) e = rescale_exponent(bits_double(ws.slots[b * 3 + (r3 == 0 ? 2 : r3 - 1)]));
  const double er = exp(a.reward[(size_t)b * S + s]);
  double za[kMaxActions];
  double zsum = 0.0;
  for (int act = 0; act < A; ++act) {
    double acc = 0.0;
    for (int k = 0; k < m.K; ++k) acc = fma(row_val(m, b, act, k, s), zs[row_nbr(m, b, s, k)], acc);
    za[act] = ldexp(__dmul_rn(er, acc), e);
    zsum = __dadd_rn(zsum, za[act]);
  }
  for (int act = 0; act < A; ++act) a.pi[((size_t)b * S + s) * A + act] = za[act] / zsum;
  if (s == 0) a.status[b] = IRLMX_OK;
}

template <bool SOFT>
__global__ void __launch_bounds__(kSweepThreads)
bellman_sweep_kernel(SoftArgs a, Ws ws, long long it, int r3) {
  const Model& m = a.m;
  const int b = blockIdx.y;
  if (sweep_should_stop(b, it, r3, a.eps, a.max_iter, ws, a.status)) return;
  const int S = m.S;
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  const double* vin = ((it & 1) ? ws.buf1 : ws.buf0) + (size_t)b * S;
  double* vout = ((it & 1) ? ws.buf0 : ws.buf1) + (size_t)b * S;
  unsigned long long d = 0ull;
  if (s < S) {
    const double r = a.reward[(size_t)b * S + s];
    const double phi = SOFT ? a.phi[(size_t)b * S + s] : 0.0;
    const double v = bellman_update<SOFT, 1, false>(a, b, s, nullptr, vin, r, phi);
    vout[s] = v;
    d = abs_bits(v - vin[s]);
  }
  block_max_to(d, &ws.slots[b * 3 + r3]);
  if (blockIdx.x == 0 && threadIdx.x == 0) ws.slots[b * 3 + (r3 == 2 ? 0 : r3 + 1)] = 0ull;
}

template <bool SOFT>
__global__ void bellman_finish_kernel(SoftArgs a, Ws ws) {
  const Model& m = a.m;
  const int S = m.S;
  const int b = blockIdx.y;
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= S) return;
  const long long it = ws.iters[b];
  const double* vnew = ((it & 1) ? ws.buf1 : ws.buf0) + (size_t)b * S;
  const double* vold = ((it & 1) ? ws.buf0 : ws.buf1) + (size_t)b * S;
  if (a.value) a.value[(size_t)b * S + s] = vnew[s];
  if (SOFT) soft_policy_row<1, false>(a, b, s, nullptr, vold, vnew[s], a.reward[(size_t)b * S + s]);
  if (s == 0 && a.iters) a.iters[b] = it;
}

// ---------------------------------------------------------------------------
// persistent grid shape: soft VI / VI on stencil grids with S > 4096
// ---------------------------------------------------------------------------
//
// One launch runs the whole loop.  Every workgroup owns SPT * kGridThreads
// states of one instance, keeps their weights, reward and terminal reward in
// registers, and exchanges values with the rest of the instance every sweep
// through tagged granules in HBM (cluster.h: one 16-byte write-through store
// {lo, tag, hi, tag} per value, tag = call salt | sweep; readers poll their
// five stencil neighbours with sc1 loads until the tags match -- the data is
// the flag, one fabric round trip per sweep and no global barrier).  The
// convergence word travels the same way: each workgroup publishes the max
// |v_new - v_old| of its states as one granule, and with sweep k's neighbour
// values every workgroup also gathers all of sweep k's block maxima, so all of
// them take the reference's decision (`while delta > eps`, NaN included: the
// maxima are ordered bits, fixed_point.hip header) at the same sweep.  Values
// and maxima live in rings of three sweeps: a workgroup can only write sweep
// k + 3 after every workgroup of the instance has published sweep k + 2, i.e.
// finished reading sweep k.  Per-state arithmetic is bellman_update's, in the
// same order: results bit-identical to the fused and per-sweep shapes.
constexpr int kGridThreads = 256;
constexpr int kGridMaxActions = 5;

struct GridArgs {
  unsigned long long* gran;   // [B][3][S] x 16 B
  unsigned long long* dgran;  // [B][4][bpi] x 16 B: three sweeps of block maxima + the XCC ids
  int* err;
  int bpi;
  int nb;                     // instances
  int xcd_group;              // workgroups dealt to XCD groups (see the kernel)
  unsigned salt;
  int n_resident;             // workgroups that must run at once (coresident(), cluster.h)
};

// every workgroup of the launch running at once, or none goes on (the err[1..2]
// counters; err bit kErrNotResident tells the host to rerun per sweep)
__device__ inline bool grid_coresident(const GridArgs& g) {
  __shared__ int resident;
  if (threadIdx.x == 0) resident = coresident(g.err + 1, g.n_resident) ? 1 : 0;
  __syncthreads();
  if (!resident && threadIdx.x == 0) atomicOr(g.err, kErrNotResident);
  return resident != 0;
}

template <bool SOFT, int SPT, int KMAX>
__global__ void __launch_bounds__(kGridThreads) bellman_grid_kernel(SoftArgs a, GridArgs g) {
  const Model& m = a.m;
  const int S = m.S, A = m.A, Kr = m.K;  // Kr <= KMAX slots: the stencil's five or the ELL row form's
  // XCD grouping (as cluster.hip): workgroups are dealt round-robin over the 8
  // XCDs, so the workgroups of instance g + 8 j are all taken from XCD group g
  // and its hand-offs can stay in one L2 (checked below; speed only).  The grid
  // is padded to 8 equal groups; padding workgroups leave at once.
  int lin = blockIdx.x;
  if (g.xcd_group) {
    const int grp = blockIdx.x % 8, kk = blockIdx.x / 8;
    const int il = grp + 8 * (kk / g.bpi);
    if (il >= g.nb) return;
    lin = il * g.bpi + kk % g.bpi;
  }
  const int b = lin / g.bpi, blk = lin % g.bpi, tid = threadIdx.x;
  __shared__ NpTables npt_lds;
  const NpTables* const npt = &npt_lds;
  if (SOFT) np_stage_tables(&npt_lds);  // numpy exp / log tables in LDS (common.h); grid_coresident synchronises
  if (!grid_coresident(g)) return;
  constexpr int K = KMAX;
  __shared__ unsigned long long red_in[kGridThreads / kWave], red_out[kGridThreads / kWave];
  __shared__ int lflag;
  int sidx[SPT];
  bool ok[SPT];
  int nb[SPT][K];
  double w[SPT][kGridMaxActions][K];
  double r[SPT], phi[SPT], cur[SPT], q[SPT][kGridMaxActions];
  const double v0 = SOFT ? -1e200 : 0.0;  // maxent.py:323 / solver.py:32
#pragma unroll
  for (int j = 0; j < SPT; ++j) {
    const int s = (blk * SPT + j) * kGridThreads + tid;
    sidx[j] = s;
    ok[j] = s < S;
    const int ss = ok[j] ? s : 0;
    r[j] = a.reward[(size_t)b * S + ss];
    phi[j] = SOFT ? a.phi[(size_t)b * S + ss] : 0.0;
    cur[j] = v0;
#pragma unroll
    for (int k = 0; k < K; ++k) nb[j][k] = k < Kr ? row_nbr(m, b, ss, k) : ss;
#pragma unroll
    for (int act = 0; act < kGridMaxActions; ++act) {
      q[j][act] = 0.0;
#pragma unroll
      for (int k = 0; k < K; ++k) w[j][act][k] = (act < A && k < Kr) ? row_val(m, b, act, k, ss) : 0.0;
    }
  }
  if (tid == 0) lflag = 0;
  const Gran rg = gran_rsrc(g.gran + (size_t)b * 6 * S, 48u * (unsigned)S);
  const Gran rd = gran_rsrc(g.dgran + (size_t)b * 8 * g.bpi, 64u * (unsigned)g.bpi);
  const unsigned salt = (g.salt & 0xFFFu) << 20;
  // hand-off store form: write-through (sc1) in general; plain stores (kept in the
  // XCD's L2, where the readers' sc1 loads are served) when every workgroup of
  // the instance runs on the same XCD -- found by exchanging XCC ids once
  bool plain = false;
  {
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    xcc &= 0xFu;
    const unsigned htag = salt | 0xFFFFFu;
    if (tid == 0) gran_store(rd, (3u * (unsigned)g.bpi + (unsigned)blk) * 16u, xcc, htag, false);
    unsigned off[1] = {(3u * (unsigned)g.bpi + (unsigned)tid) * 16u};
    unsigned long long v[1] = {xcc};
    if (!gran_gather<1>(rd, rd, off, tid < g.bpi ? 1u : 0u, htag, v)) lflag = 1;
    const unsigned long long diff = wave_or_u64(tid < g.bpi ? (v[0] ^ xcc) : 0ull);
    if ((tid & (kWave - 1)) == 0) red_in[tid / kWave] = diff;
    __syncthreads();
    if (lflag) {
      if (tid == 0) atomicOr(g.err, 1);
      return;
    }
    unsigned long long any = 0ull;
#pragma unroll
    for (int i = 0; i < kGridThreads / kWave; ++i) any |= red_in[i];
    plain = g.xcd_group && any == 0ull;
    __syncthreads();
  }
  double delta = 0.0;
  long long k = 0;  // sweeps done: cur = v_k
  for (;;) {
    double nv[SPT][K];
    if (k == 0) {
#pragma unroll
      for (int j = 0; j < SPT; ++j)
#pragma unroll
        for (int kk = 0; kk < K; ++kk) nv[j][kk] = v0;
    } else {
      // sweep k's neighbour values and (threads < bpi) all block maxima, one round trip
      const unsigned tag = salt | ((unsigned)k & 0xFFFFFu);
      const unsigned slot = (unsigned)(k % 3);
      unsigned off[SPT * K + 1];
      using mask_t = typename std::conditional<(SPT * K + 1 > 32), unsigned long long, unsigned>::type;
      mask_t want = 0;
#pragma unroll
      for (int j = 0; j < SPT; ++j)
#pragma unroll
        for (int kk = 0; kk < K; ++kk) {
          off[j * K + kk] = (slot * (unsigned)S + (unsigned)nb[j][kk]) * 16u;
          want |= (mask_t)(ok[j] && kk < Kr ? 1u : 0u) << (j * K + kk);
        }
      off[SPT * K] = (slot * (unsigned)g.bpi + (unsigned)tid) * 16u;
      want |= (mask_t)(tid < g.bpi ? 1u : 0u) << (SPT * K);
      unsigned long long v[SPT * K + 1];
      if (!gran_gather<SPT * K + 1>(rg, rd, off, want, tag, v)) lflag = 1;
#pragma unroll
      for (int j = 0; j < SPT; ++j)
#pragma unroll
        for (int kk = 0; kk < K; ++kk) nv[j][kk] = (ok[j] && kk < Kr) ? bits_double(v[j * K + kk]) : 0.0;
      unsigned long long d = tid < g.bpi ? v[SPT * K] : 0ull;
      d = wave_max_u64(d);
      if ((tid & (kWave - 1)) == 0) red_in[tid / kWave] = d;
      __syncthreads();
      if (lflag) {
        if (tid == 0) atomicOr(g.err, 1);
        return;
      }
      unsigned long long mx = 0ull;
#pragma unroll
      for (int i = 0; i < kGridThreads / kWave; ++i) mx = red_in[i] > mx ? red_in[i] : mx;
      delta = bits_double(mx);
      if (!(delta > a.eps) || (a.max_iter > 0 && k >= a.max_iter)) break;  // maxent.py:326 / solver.py:40
    }
    // sweep k + 1 (bellman_update's arithmetic and order)
    unsigned long long dmax = 0ull;
    const unsigned tag1 = salt | ((unsigned)(k + 1) & 0xFFFFFu);
    const unsigned slot1 = (unsigned)((k + 1) % 3);
#pragma unroll
    for (int j = 0; j < SPT; ++j) {
      double v = SOFT ? phi[j] : 0.0;
#pragma unroll
      for (int act = 0; act < kGridMaxActions; ++act) {
        if (act >= A) break;
        double dot = 0.0;
#pragma unroll
        for (int kk = 0; kk < K; ++kk)
          if (kk < Kr) dot = fma(w[j][act][kk], nv[j][kk], dot);
        if (SOFT) {
          q[j][act] = __dadd_rn(r[j], __dmul_rn(a.discount, dot));
          v = softmax2(v, q[j][act], npt, SPT == 1);  // maxent.py:329-333
        } else {
          const double qq = __dmul_rn(a.discount, dot);  // solver.py:44
          if (a.average) v = act == 0 ? qq : __dadd_rn(v, qq);
          else v = act == 0 ? qq : ((v != v || qq <= v) ? v : qq);
        }
      }
      if (!SOFT) v = __dadd_rn(r[j], a.average ? v / (double)A : v);  // solver.py:47 / :99
      if (ok[j]) {
        const unsigned long long d = abs_bits(v - cur[j]);
        dmax = d > dmax ? d : dmax;
        gran_store(rg, (slot1 * (unsigned)S + (unsigned)sidx[j]) * 16u, dbits(v), tag1, plain);
      }
      cur[j] = v;
    }
    dmax = wave_max_u64(dmax);
    if ((tid & (kWave - 1)) == 0) red_out[tid / kWave] = dmax;
    __syncthreads();
    if (tid == 0) {
      unsigned long long mx = 0ull;
      for (int i = 0; i < kGridThreads / kWave; ++i) mx = red_out[i] > mx ? red_out[i] : mx;
      gran_store(rd, (slot1 * (unsigned)g.bpi + (unsigned)blk) * 16u, mx, tag1, plain);
    }
    ++k;
  }
#pragma unroll
  for (int j = 0; j < SPT; ++j) {
    if (!ok[j]) continue;
    const size_t o = (size_t)b * S + sidx[j];
    if (a.value) a.value[o] = cur[j];
    if (SOFT)
      for (int act = 0; act < A; ++act) a.pi[o * A + act] = np_exp(q[j][act] - cur[j], npt);  // maxent.py:341
  }
  if (blk == 0 && tid == 0) {
    if (a.iters) a.iters[b] = k;
    a.status[b] = finish_status(delta, a.eps);
  }
}

// The grid shape for the linear loops of ELL models (generic sparsity, S > 4096):
// the forward (MODE kModeFwd: d <- p0 + sum_k w[k] d[src_k], until max|dd| <= eps;
// fwd_sweep_kernel's arithmetic) and the backward (kModeBwd: 2S - 1 collapsed
// sweeps zs <- ldexp(sum_k w[k] zs[nbr_k], e), e from the previous sweep's
// maximum, then the per-action sweep; bwd_sweep_kernel / bwd_final_kernel's
// arithmetic).  Same exchange as bellman_grid_kernel; the block maxima carry
// max|dd| (forward) or max|zs| (backward: the rescale exponent, and a NaN /
// inf there is bwd_nonfinite_rule's flag -- ordered bits sort them above every
// finite value).
struct LinearGridArgs {
  Model m;
  const double* w;      // [B][K][S] forward gather weights / reward-folded backward weights
  const double* vin;    // forward: p0 [B][S]; backward: reward [B][S]
  const uint8_t* term;  // backward: terminal mask
  const int32_t* bad;   // [B] non-finite policy (forward) / weights (backward)
  double eps;
  long long max_iter;
  int rescale;
  double* out;          // forward: svf [B][S]; backward: pi [B][S][A]
  int64_t* iters;
  int32_t* status;
};

template <int MODE, int SPT, int KMAX>
__global__ void __launch_bounds__(kGridThreads) linear_grid_kernel(LinearGridArgs a, GridArgs g) {
  const Model& m = a.m;
  const int S = m.S;
  const int Kr = MODE == kModeFwd ? m.Kc : m.K;
  int lin = blockIdx.x;
  if (g.xcd_group) {
    const int grp = blockIdx.x % 8, kk = blockIdx.x / 8;
    const int il = grp + 8 * (kk / g.bpi);
    if (il >= g.nb) return;
    lin = il * g.bpi + kk % g.bpi;
  }
  const int b = lin / g.bpi, blk = lin % g.bpi, tid = threadIdx.x;
  if (!grid_coresident(g)) return;
  constexpr int K = KMAX;
  __shared__ unsigned long long red_in[kGridThreads / kWave], red_out[kGridThreads / kWave];
  __shared__ int lflag;
  int sidx[SPT];
  bool ok[SPT];
  int nb[SPT][K];
  double w[SPT][K], c0[SPT], cur[SPT];
  if (MODE == kModeFwd && a.bad[b]) {  // non-finite policy: the reference's dense product is NaN after one sweep
#pragma unroll
    for (int j = 0; j < SPT; ++j) {
      const int s = (blk * SPT + j) * kGridThreads + tid;
      if (s < S) a.out[(size_t)b * S + s] = kNaN;
    }
    if (blk == 0 && tid == 0) { a.iters[b] = 1; a.status[b] = IRLMX_NONFINITE; }
    return;
  }
#pragma unroll
  for (int j = 0; j < SPT; ++j) {
    const int s = (blk * SPT + j) * kGridThreads + tid;
    sidx[j] = s;
    ok[j] = s < S;
    const int ss = ok[j] ? s : 0;
    c0[j] = MODE == kModeFwd ? a.vin[(size_t)b * S + ss] : 0.0;
    cur[j] = MODE == kModeBwd ? (a.term[(size_t)b * S + ss] ? 1.0 : 0.0) : 0.0;  // maxent.py:146-147 / d = 0
#pragma unroll
    for (int k = 0; k < K; ++k) {
      nb[j][k] = k < Kr ? (MODE == kModeFwd ? col_src(m, b, ss, k) : row_nbr(m, b, ss, k)) : ss;
      w[j][k] = k < Kr ? a.w[((size_t)b * Kr + k) * S + ss] : 0.0;
    }
  }
  if (tid == 0) lflag = 0;
  const Gran rg = gran_rsrc(g.gran + (size_t)b * 6 * S, 48u * (unsigned)S);
  const Gran rd = gran_rsrc(g.dgran + (size_t)b * 8 * g.bpi, 64u * (unsigned)g.bpi);
  const unsigned salt = (g.salt & 0xFFFu) << 20;
  bool plain = false;
  {  // XCC ids (bellman_grid_kernel)
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    xcc &= 0xFu;
    const unsigned htag = salt | 0xFFFFFu;
    if (tid == 0) gran_store(rd, (3u * (unsigned)g.bpi + (unsigned)blk) * 16u, xcc, htag, false);
    unsigned off[1] = {(3u * (unsigned)g.bpi + (unsigned)tid) * 16u};
    unsigned long long v[1] = {xcc};
    if (!gran_gather<1>(rd, rd, off, tid < g.bpi ? 1u : 0u, htag, v)) lflag = 1;
    const unsigned long long diff = wave_or_u64(tid < g.bpi ? (v[0] ^ xcc) : 0ull);
    if ((tid & (kWave - 1)) == 0) red_in[tid / kWave] = diff;
    __syncthreads();
    if (lflag) {
      if (tid == 0) atomicOr(g.err, 1);
      return;
    }
    unsigned long long any = 0ull;
#pragma unroll
    for (int i = 0; i < kGridThreads / kWave; ++i) any |= red_in[i];
    plain = g.xcd_group && any == 0ull;
    __syncthreads();
  }
  // backward: publish the start vector as sweep 0 (its neighbours read it)
  const long long total = MODE == kModeBwd ? 2LL * S - 1 : -1;
  double delta = 0.0;
  unsigned long long gmax = 0ull;  // backward: max |zs| of the vector the next sweep reads
  bool nonfinite = false;
  long long k = 0;
  if (MODE == kModeBwd) {
    const unsigned tag0 = salt | 1u;  // tag of sweep k: salt | (k + 1), never 0 (a zeroed workspace)
    unsigned long long dm = 0ull;
#pragma unroll
    for (int j = 0; j < SPT; ++j)
      if (ok[j]) {
        gran_store(rg, (unsigned)sidx[j] * 16u, dbits(cur[j]), tag0, plain);
        const unsigned long long d = abs_bits(cur[j]);
        dm = d > dm ? d : dm;
      }
    dm = wave_max_u64(dm);
    if ((tid & (kWave - 1)) == 0) red_out[tid / kWave] = dm;
    __syncthreads();
    if (tid == 0) {
      unsigned long long mx = 0ull;
      for (int i = 0; i < kGridThreads / kWave; ++i) mx = red_out[i] > mx ? red_out[i] : mx;
      gran_store(rd, (unsigned)blk * 16u, mx, tag0, plain);
    }
  }
  double nv[SPT][K];  // the neighbours' values of the vector the next sweep reads
  for (;;) {
    if (MODE == kModeFwd && k == 0) {
#pragma unroll
      for (int j = 0; j < SPT; ++j)
#pragma unroll
        for (int kk = 0; kk < K; ++kk) nv[j][kk] = 0.0;
    } else {
      const unsigned tag = salt | ((unsigned)(k + 1) & 0xFFFFFu);
      const unsigned slot = (unsigned)(k % 3);
      unsigned off[SPT * K + 1];
      using mask_t = typename std::conditional<(SPT * K + 1 > 32), unsigned long long, unsigned>::type;
      mask_t want = 0;
#pragma unroll
      for (int j = 0; j < SPT; ++j)
#pragma unroll
        for (int kk = 0; kk < K; ++kk) {
          off[j * K + kk] = (slot * (unsigned)S + (unsigned)nb[j][kk]) * 16u;
          want |= (mask_t)(ok[j] && kk < Kr ? 1u : 0u) << (j * K + kk);
        }
      off[SPT * K] = (slot * (unsigned)g.bpi + (unsigned)tid) * 16u;
      want |= (mask_t)(tid < g.bpi ? 1u : 0u) << (SPT * K);
      unsigned long long v[SPT * K + 1];
      if (!gran_gather<SPT * K + 1>(rg, rd, off, want, tag, v)) lflag = 1;
#pragma unroll
      for (int j = 0; j < SPT; ++j)
#pragma unroll
        for (int kk = 0; kk < K; ++kk) nv[j][kk] = (ok[j] && kk < Kr) ? bits_double(v[j * K + kk]) : 0.0;
      unsigned long long d = tid < g.bpi ? v[SPT * K] : 0ull;
      d = wave_max_u64(d);
      if ((tid & (kWave - 1)) == 0) red_in[tid / kWave] = d;
      __syncthreads();
      if (lflag) {
        if (tid == 0) atomicOr(g.err, 1);
        return;
      }
      unsigned long long mx = 0ull;
#pragma unroll
      for (int i = 0; i < kGridThreads / kWave; ++i) mx = red_in[i] > mx ? red_in[i] : mx;
      if (MODE == kModeFwd) {
        delta = bits_double(mx);
        if (!(delta > a.eps) || (a.max_iter > 0 && k >= a.max_iter)) break;  // maxent.py:108
      } else {
        gmax = mx;
        nonfinite |= mx >= 0x7FF0000000000000ull;  // some |zs| is inf or NaN
        if (k >= total) break;  // neighbours of zs_{2S-1} gathered: the per-action sweep
      }
    }
    const int e = (MODE == kModeBwd && a.rescale && k > 0) ? rescale_exponent(bits_double(gmax)) : 0;
    unsigned long long dmax = 0ull;
    const unsigned tag1 = salt | ((unsigned)(k + 2) & 0xFFFFFu);
    const unsigned slot1 = (unsigned)((k + 1) % 3);
#pragma unroll
    for (int j = 0; j < SPT; ++j) {
      double acc = 0.0;
#pragma unroll
      for (int kk = 0; kk < K; ++kk)
        if (kk < Kr) acc = fma(w[j][kk], nv[j][kk], acc);
      const double v = MODE == kModeFwd ? c0[j] + acc : ldexp(acc, e);
      if (ok[j]) {
        const unsigned long long d = MODE == kModeFwd ? abs_bits(v - cur[j]) : abs_bits(v);
        dmax = d > dmax ? d : dmax;
        gran_store(rg, (slot1 * (unsigned)S + (unsigned)sidx[j]) * 16u, dbits(v), tag1, plain);
      }
      cur[j] = v;
    }
    dmax = wave_max_u64(dmax);
    if ((tid & (kWave - 1)) == 0) red_out[tid / kWave] = dmax;
    __syncthreads();
    if (tid == 0) {
      unsigned long long mx = 0ull;
      for (int i = 0; i < kGridThreads / kWave; ++i) mx = red_out[i] > mx ? red_out[i] : mx;
      gran_store(rd, (slot1 * (unsigned)g.bpi + (unsigned)blk) * 16u, mx, tag1, plain);
    }
    ++k;
  }
  if (MODE == kModeFwd) {
#pragma unroll
    for (int j = 0; j < SPT; ++j)
      if (ok[j]) a.out[(size_t)b * S + sidx[j]] = cur[j];
    if (blk == 0 && tid == 0) { a.iters[b] = k; a.status[b] = finish_status(delta, a.eps); }
  } else {
    // the last of the 2*S sweeps, per action (bwd_final_kernel's arithmetic)
    const int A = m.A;
    const int e = a.rescale ? rescale_exponent(bits_double(gmax)) : 0;
    const bool all_nan = nonfinite || a.bad[b];
#pragma unroll
    for (int j = 0; j < SPT; ++j) {
      if (!ok[j]) continue;
      const int s = sidx[j];
      double* pr = a.out + ((size_t)b * S + s) * A;
      if (all_nan) {
        for (int act = 0; act < A; ++act) pr[act] = kNaN;
        continue;
      }
      const double er = exp(a.vin[(size_t)b * S + s]);
      double za[kMaxActions];
      double zsum = 0.0;
      for (int act = 0; act < A; ++act) {
        double acc = 0.0;
        for (int kk = 0; kk < Kr; ++kk) acc = fma(row_val(m, b, act, kk, s), nv[j][kk], acc);
        za[act] = ldexp(__dmul_rn(er, acc), e);
        zsum = __dadd_rn(zsum, za[act]);
      }
      for (int act = 0; act < A; ++act) pr[act] = za[act] / zsum;
    }
    if (blk == 0 && tid == 0) a.status[b] = IRLMX_OK;
  }
}

template <bool SOFT>
static void* bellman_grid_fn(int spt, int kmax) {
  if (kmax == 5) {
    switch (spt) {
      case 1: return (void*)&bellman_grid_kernel<SOFT, 1, 5>;
      case 2: return (void*)&bellman_grid_kernel<SOFT, 2, 5>;
      case 4: return (void*)&bellman_grid_kernel<SOFT, 4, 5>;
    }
  } else if (kmax == 8) {
    switch (spt) {
      case 1: return (void*)&bellman_grid_kernel<SOFT, 1, 8>;
      case 2: return (void*)&bellman_grid_kernel<SOFT, 2, 8>;
    }
  } else if (kmax == 16 && spt == 1) {
    return (void*)&bellman_grid_kernel<SOFT, 1, 16>;
  }
  return nullptr;
}
// slots per state the grid kernels hold in registers: the linear loops up to 32
// (ELL rows / columns of generic sparse models), the Bellman loops up to 16
// (their A x K weights)
static int grid_kmax_of(int K, int cap) {
  const int k = K <= 5 ? 5 : (K <= 8 ? 8 : (K <= 16 ? 16 : (K <= 32 ? 32 : 0)));
  return k <= cap ? k : 0;
}
static int grid_kmax(const Model& m) { return grid_kmax_of(m.K, 16); }
static int grid_kmax_lin(const Model& m) { return grid_kmax_of(m.K, 32); }
static int grid_kmax_fwd(const Model& m) { return grid_kmax_of(m.Kc, 32); }

template <int MODE>
static void* linear_grid_fn(int spt, int kmax) {
  if (kmax == 5) {
    switch (spt) {
      case 1: return (void*)&linear_grid_kernel<MODE, 1, 5>;
      case 2: return (void*)&linear_grid_kernel<MODE, 2, 5>;
      case 4: return (void*)&linear_grid_kernel<MODE, 4, 5>;
    }
  } else if (kmax == 8) {
    switch (spt) {
      case 1: return (void*)&linear_grid_kernel<MODE, 1, 8>;
      case 2: return (void*)&linear_grid_kernel<MODE, 2, 8>;
    }
  } else if (kmax == 16) {
    switch (spt) {
      case 1: return (void*)&linear_grid_kernel<MODE, 1, 16>;
      case 2: return (void*)&linear_grid_kernel<MODE, 2, 16>;
    }
  } else if (kmax == 32 && spt == 1) {
    return (void*)&linear_grid_kernel<MODE, 1, 32>;
  }
  return nullptr;
}

static void* grid_fn(const Model& m, int op, int spt) {
  switch (op) {
    case IRLMX_OP_SOFT_BACKWARD: return bellman_grid_fn<true>(spt, grid_kmax(m));
    case IRLMX_OP_VALUE_ITERATION: return bellman_grid_fn<false>(spt, grid_kmax(m));
    case IRLMX_OP_FORWARD: return linear_grid_fn<kModeFwd>(spt, grid_kmax_fwd(m));
    case IRLMX_OP_BACKWARD: return linear_grid_fn<kModeBwd>(spt, grid_kmax_lin(m));
  }
  return nullptr;
}

static int grid_capacity(void* fn) {
  // IRLMX_PLAN_CUS x IRLMX_PLAN_GRID_PER_CU: planning without a device (the
  // host-side sanitizer build, tools/sanitize); a launch always re-checks
  // co-residency on the device (coresident()), so a wrong figure cannot hang
  const int f_cus = getenv_int("IRLMX_PLAN_CUS", 0), f_per = getenv_int("IRLMX_PLAN_GRID_PER_CU", 0);
  if (f_cus > 0 && f_per > 0) return f_cus * f_per;
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)fn, kGridThreads, 0) != hipSuccess) return 0;
  return cus * per_cu;
}

// the smallest states-per-thread whose grid is co-resident (all workgroups must
// run at once: they wait on each other's granules); IRLMX_GRID=0 disables
static bool grid_plan(const Model& m, int op, GridPlan* out) {
  if (m.dense || getenv_int("IRLMX_GRID", 1) == 0) return false;
  if (m.S <= fused_max_states()) return false;  // one workgroup holds it: the fused shape
  if (op == IRLMX_OP_SOFT_BACKWARD || op == IRLMX_OP_VALUE_ITERATION) {
    if (m.A > kGridMaxActions || !grid_kmax(m)) return false;
  } else if (op == IRLMX_OP_FORWARD || op == IRLMX_OP_BACKWARD) {
    // stencil grids run the cluster shape; ELL rows / columns of at most 32 slots here
    if (m.stencil || !(op == IRLMX_OP_FORWARD ? grid_kmax_fwd(m) : grid_kmax_lin(m)) || m.A > kMaxActions) return false;
  } else {
    return false;
  }
  for (int spt = 1; spt <= 4; spt *= 2) {
    void* fn = grid_fn(m, op, spt);
    if (!fn) continue;
    const int bpi = (m.S + spt * kGridThreads - 1) / (spt * kGridThreads);
    if (bpi > kGridThreads) continue;  // the block maxima are gathered one per thread
    const int cap = grid_capacity(fn);
    // XCD groups: ceil(B / 8) instances per group, each group within one XCD's
    // share -- only from 8 instances on: fewer would leave XCDs idle (one 128x128
    // instance: soft VI 3.5 ms grouped on one XCD vs 3.1 ms spread, 812 sweeps)
    const bool xcd = getenv_int("IRLMX_XCD_GROUP", 1) != 0 && cap >= 8 && m.B >= 8 &&
                     (long long)((m.B + 7) / 8) * bpi <= cap / 8;
    if (xcd || (long long)bpi * m.B <= cap) {
      *out = GridPlan{spt, bpi, xcd ? 1 : 0};
      return true;
    }
  }
  return false;
}

static std::atomic<unsigned> g_grid_salt{1};

// one persistent launch of the grid shape, then its exchange-timeout word
// (synchronises the stream, like cluster_run)
static int grid_launch(const Model& m, int op, const GridPlan& gp, void** args, const Ws& ws, hipStream_t st) {
  const int grid = gp.xcd ? 8 * ((m.B + 7) / 8) * gp.bpi : gp.bpi * m.B;
  hipError_t e = hipLaunchKernel(grid_fn(m, op, gp.spt), dim3(grid), dim3(kGridThreads), args, 0, st);
  if (e != hipSuccess) return hip_fail(e, "grid launch");
  count_event(IRLMX_CTR_GRID_LAUNCHES);
  int err = 0;
  e = hipMemcpyAsync(&err, ws.err, sizeof(int), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) return hip_fail(e, "grid sync");
  // not all workgroups could run at once, or (after a passed rendezvous) one was
  // descheduled long enough for an exchange to time out: clear the words and
  // rerun on the per-sweep shape (cluster_run treats both cases the same way)
  const bool timeout = err && !(err & kErrNotResident);
  if (timeout && getenv_int("IRLMX_STRICT_EXCHANGE", 0)) {
    set_error("grid shape: exchange timed out (workgroups not co-resident?)");
    return IRLMX_EHIP;
  }
  if (timeout) note_exchange_timeout("grid");
  if (err) {
    count_event(timeout ? IRLMX_CTR_RERUN_TIMEOUT : IRLMX_CTR_RERUN_NOT_RESIDENT);
    e = hipMemsetAsync(ws.err, 0, 4 * sizeof(int), st);
    return e == hipSuccess ? kClusterNotResident : hip_fail(e, "grid err reset");
  }
  return 0;
}

static GridArgs grid_args(const Model& m, const GridPlan& gp, const Ws& ws) {
  // (IRLMX_TEST_NOT_RESIDENT=1, tests only: one workgroup more than launched -> the per-sweep rerun)
  return GridArgs{ws.gran, ws.sgran, ws.err, gp.bpi, m.B, gp.xcd, g_grid_salt.fetch_add(1, std::memory_order_relaxed),
                  gp.bpi * m.B + (getenv_int("IRLMX_TEST_NOT_RESIDENT", 0) ? 1 : 0)};
}

__global__ void fill_kernel(double* p, size_t n, double v) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

// ---------------------------------------------------------------------------
// host-side dispatch
// ---------------------------------------------------------------------------

struct FusedShape {
  int spt;
  int kmax;
  int threads;
};

static int pick_kmax(int K) {
  if (K <= 5) return 5;
  if (K <= 8) return 8;
  if (K <= 16) return 16;
  if (K <= 32) return 32;
  return 0;
}

// (SPT, KMAX) pairs instantiated per op: every pair listed compiles without
// VGPR spills at __launch_bounds__(1024) (tools/kernel_resources.py); the soft
// pass carries fp64 exp/log inline and so keeps fewer states per thread.
static constexpr bool fused_pair_ok(int op, int spt, int kmax) {
  switch (op) {
    case IRLMX_OP_FORWARD:
    case IRLMX_OP_BACKWARD:
      return (kmax == 5 && spt <= 4) || (kmax == 8 && spt <= 2) || (kmax == 16 && spt <= 2) ||
             (kmax == 32 && spt == 1);
    case IRLMX_OP_SOFT_BACKWARD:
      return (kmax == 5 && spt <= 2) || (kmax == 8 && spt == 1) || (kmax == 16 && spt == 1);
    case IRLMX_OP_VALUE_ITERATION:
      return (kmax == 5 && spt <= 4) || (kmax == 8 && spt <= 4) || (kmax == 16 && spt == 1) ||
             (kmax == 32 && spt == 1);
  }
  return false;
}

static bool fused_shape(const Model& m, int op, FusedShape* out) {
  if (m.dense || m.S > fused_max_states() || m.A > kMaxActions) return false;
  // Grids of width 64 / 128 run the forward and backward passes on the cluster
  // shape even when they fit one CU: its register-resident pair layouts sweep
  // 4-5x faster than the general-sparsity fused kernel, and a single instance
  // then spreads over several CUs (cluster.hip).
  if ((op == IRLMX_OP_FORWARD || op == IRLMX_OP_BACKWARD) && m.stencil && (m.W == 64 || m.W == 128) &&
      getenv_int("IRLMX_CLUSTER", 1) != 0)
    return false;
  const int K = op == IRLMX_OP_FORWARD ? m.Kc : m.K;
  const int kmax = pick_kmax(K);
  if (!kmax) return false;
  int spt = 1;
  while ((m.S + spt - 1) / spt > 1024) spt *= 2;
  if (!fused_pair_ok(op, spt, kmax)) return false;
  const int per = (m.S + spt - 1) / spt;
  out->spt = spt;
  out->kmax = kmax;
  out->threads = std::min(1024, ((per + kWave - 1) / kWave) * kWave);
  return true;
}

static bool use_fused(const Model& m, int op) {
  FusedShape f;
  return fused_shape(m, op, &f);
}

// two S-vectors, the convergence slots and (run_deferred) the block-start snapshot
static size_t fused_lds(const Model& m) { return 3 * (size_t)m.S * sizeof(double) + 4 * sizeof(unsigned long long); }

// Kernel-pointer getters: only the (SPT, KMAX) pairs fused_pair_ok() admits
// are instantiated.
#define IRLMX_FUSED_GETTER(NAME, KERNEL_T, OP, ARGS_T)                    \
  template <int S_, int K_>                                               \
  static void (*NAME())(ARGS_T) {                                         \
    if constexpr (fused_pair_ok(OP, S_, K_)) return &KERNEL_T<S_, K_>;    \
    else return nullptr;                                                  \
  }
IRLMX_FUSED_GETTER(fwd_fused_ptr, fwd_fused_kernel, IRLMX_OP_FORWARD, FwdArgs)
IRLMX_FUSED_GETTER(bwd_fused_ptr, bwd_fused_kernel, IRLMX_OP_BACKWARD, BwdArgs)
IRLMX_FUSED_GETTER(soft_fused_ptr, soft_fused_kernel, IRLMX_OP_SOFT_BACKWARD, SoftArgs)
IRLMX_FUSED_GETTER(vi_fused_ptr, vi_fused_kernel, IRLMX_OP_VALUE_ITERATION, SoftArgs)

#define IRLMX_DISPATCH_FUSED(GETTER, SHAPE, B, LDS, STREAM, ARGS)                                   \
  do {                                                                                                \
    void (*kfn)(decltype(ARGS)) = nullptr;                                                           \
    const int _s = (SHAPE).spt, _k = (SHAPE).kmax;                                                    \
    if (_s == 1 && _k == 5) kfn = GETTER<1, 5>();                                                     \
    else if (_s == 2 && _k == 5) kfn = GETTER<2, 5>();                                                \
    else if (_s == 4 && _k == 5) kfn = GETTER<4, 5>();                                                \
    else if (_s == 1 && _k == 8) kfn = GETTER<1, 8>();                                                \
    else if (_s == 2 && _k == 8) kfn = GETTER<2, 8>();                                                \
    else if (_s == 4 && _k == 8) kfn = GETTER<4, 8>();                                                \
    else if (_s == 1 && _k == 16) kfn = GETTER<1, 16>();                                              \
    else if (_s == 2 && _k == 16) kfn = GETTER<2, 16>();                                              \
    else if (_s == 1 && _k == 32) kfn = GETTER<1, 32>();                                              \
    if (!kfn) { set_error("no fused kernel for spt=%d kmax=%d", _s, _k); return IRLMX_EINVAL; }       \
    hipError_t _e = hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                        (int)(LDS));                                                  \
    if (_e != hipSuccess) return hip_fail(_e, "hipFuncSetAttribute");                                \
    hipLaunchKernelGGL(kfn, dim3(B), dim3((SHAPE).threads), (LDS), (STREAM), ARGS);                   \
    _e = hipGetLastError();                                                                           \
    if (_e != hipSuccess) return hip_fail(_e, #GETTER);                                               \
  } while (0)

static int validate(const irlmx_mdp* mdp) {
  if (!mdp) { set_error("mdp is NULL"); return IRLMX_EINVAL; }
  const Model m = make_model(mdp);
  if (m.S <= 0 || m.A <= 0 || m.B <= 0) { set_error("bad sizes S=%d A=%d B=%d", m.S, m.A, m.B); return IRLMX_EINVAL; }
  if (m.A > kMaxActions) { set_error("n_actions=%d exceeds %d", m.A, kMaxActions); return IRLMX_EINVAL; }
  if (!m.row_val) { set_error("row_val is NULL"); return IRLMX_EINVAL; }
  if (m.stencil) {
    if (m.W <= 0 || m.H <= 0 || (long long)m.W * m.H != m.S) {
      set_error("stencil grid %dx%d != %d states", m.W, m.H, m.S);
      return IRLMX_EINVAL;
    }
  } else if (mdp->layout == IRLMX_LAYOUT_ELL) {
    if (!m.row_idx || m.K <= 0) { set_error("ELL row form missing"); return IRLMX_EINVAL; }
    if (m.K > m.S) { set_error("ELL k_row=%d out of range (1..%d)", m.K, m.S); return IRLMX_EINVAL; }
  } else if (m.dense) {
    if (!m.col_val) { set_error("DENSE action-summed rows (col_val) missing"); return IRLMX_EINVAL; }
    if ((long long)m.S * m.S * m.A > (1LL << 40)) { set_error("DENSE table too large (S=%d)", m.S); return IRLMX_EINVAL; }
  } else {
    set_error("unknown layout %d", mdp->layout);
    return IRLMX_EINVAL;
  }
  return 0;
}

// Required array arguments of an entry point: NULL is rejected before any work
// is enqueued (a null device pointer would fault the GPU).
struct Arg {
  const void* p;
  const char* name;  // nullptr: optional argument
};
static int need_all(const char* fn, std::initializer_list<Arg> args) {
  for (const Arg& a : args)
    if (a.name && !a.p) {
      set_error("%s: %s is NULL", fn, a.name);
      return IRLMX_EINVAL;
    }
  return 0;
}

static int check_ws(const Model& m, int op, size_t bytes, void* ws) {
  const size_t need = carve(m, op, nullptr).total;
  if (bytes < need || (need && !ws)) {
    set_error("workspace too small: need %zu bytes, got %zu", need, bytes);
    return IRLMX_EWORKSPACE;
  }
  return 0;
}

// Host poll loop of the sweep shape: enqueue `chunk` sweeps, read the done
// counter, repeat.  Converged instances skip their sweeps, so over-enqueueing
// costs only empty launches.
template <typename LaunchOne>
static int run_until_done(const Ws& ws, int B, hipStream_t st, LaunchOne&& one) {
  long long it = 0;
  int r3 = 0;
  long long chunk = 32;
  for (;;) {
    for (long long c = 0; c < chunk; ++c) {
      one(it, r3);
      ++it;
      r3 = r3 == 2 ? 0 : r3 + 1;
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "sweep launch");
    int32_t nd = 0;
    e = hipMemcpyAsync(&nd, ws.ndone, sizeof(int32_t), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return hip_fail(e, "poll");
    if (nd >= B) return 0;
    if (chunk < 4096) chunk *= 2;
  }
}

// ---------------------------------------------------------------------------
// dense-row path (dense.hip)
// ---------------------------------------------------------------------------

static DenseView dense_view(const Model& m) { return DenseView{m.S, m.A, m.B, m.shared, m.row_val, m.col_val}; }

static DenseBufs dense_bufs(const Ws& ws) {
  return DenseBufs{ws.buf0, ws.buf1, ws.slots, ws.done, ws.iters, ws.ndone, ws.bad, ws.wgt};
}

// Shared table, B instances: the collapsed backward sweep is the GEMM
// M [S x S] . ZS [S x B].  Measured on MI355X (tools/diag/dense_bench.py,
// profiles/r02_dense_gemm_bench.txt, microseconds per sweep):
//
//            streaming (VALU)      hand-written fp64 MFMA     rocBLAS dgemm (round 2, since dropped)
//   S=2048   B=4 16  B=16 40  B=64 112   16 / 19 / 43           117 / 117 / 117
//   S=4096   B=4 81  B=16 303 B=64 1227  29 / 34 / 80           447 / 448 / 450
//
// Streaming re-reads M from the 256 MB last-level cache, so it wins for few
// instances while M is small; the MFMA kernel (dense.hip dense_gemm_kernel, any
// S: zero-padded K tail) wins from 16 instances on, and from 4 on once M leaves
// that cache (S >= 4096).  IRLMX_DENSE_GEMM_MIN=<B> forces the batch threshold.
static bool dense_gemm(const Model& m) {
  if (!m.dense || !m.shared) return false;
  const int forced = getenv_int("IRLMX_DENSE_GEMM_MIN", 0);
  if (forced > 0) return m.B >= forced;
  return m.B >= 16 || (m.S >= 4096 && m.B >= 4);
}

// The persistent dense shape takes the forward and the collapsed backward
// whenever the rows fit in registers at one workgroup per CU (dense_grid.hip);
// a backward that the planner gives to the GEMM keeps it.
static bool dense_grid(const Model& m, int op, DenseGridPlan* out) {
  if (!m.dense) return false;
  if (op != IRLMX_OP_FORWARD && dense_gemm(m)) return false;
  if (op == IRLMX_OP_SOFT_BACKWARD || op == IRLMX_OP_VALUE_ITERATION) return dense_bellman_grid_plan(m.S, m.B, m.A, out);
  if (op != IRLMX_OP_FORWARD && op != IRLMX_OP_BACKWARD) return false;
  return dense_grid_plan(op == IRLMX_OP_FORWARD ? kModeFwd : kModeBwd, m.S, m.B, out);
}

static DenseGridArgs dense_grid_args(const Model& m, const Ws& ws) {
  DenseGridArgs a{};
  a.S = m.S; a.A = m.A; a.B = m.B; a.shared = m.shared;
  a.gran = ws.gran; a.xgran = ws.sgran; a.err = ws.err;
  return a;
}

static int dense_backward(const Model& m, const double* reward, const uint8_t* terminal, int rescale,
                          double* p_action, int32_t* status, const Ws& ws, hipStream_t st) {
  const DenseView d = dense_view(m);
  const DenseBufs w = dense_bufs(ws);
  DenseGridPlan dp;
  if (dense_grid(m, IRLMX_OP_BACKWARD, &dp)) {  // one persistent launch, M's rows in registers
    DenseGridArgs a = dense_grid_args(m, ws);
    a.mat = m.col_val; a.P = m.row_val; a.vin = reward; a.term = terminal;
    a.rescale = rescale; a.out = p_action; a.status = status;
    const int rc = dense_grid_run(kModeBwd, dp, a, st);
    if (rc != kClusterNotResident) return rc;  // else: the per-sweep shape below
  }
  count_event(IRLMX_CTR_SWEEP_CALLS);
  dense_bwd_init_launch(d, terminal, w, st);
  const long long collapsed = 2LL * m.S - 1;
  const bool gemm = dense_gemm(m);
  int r3 = 0;
  for (long long it = 0; it < collapsed; ++it) {
    if (gemm) {
      // C [B][S] = ZS . M^T on the hand-written fp64 MFMA kernel, then the per-state update
      const double* zin = (it & 1) ? ws.buf1 : ws.buf0;
      if (hipError_t e = dense_gemm_launch(m.col_val, zin, ws.wgt, m.S, m.S, m.B, st)) return hip_fail(e, "dense gemm");
      dense_bwd_gemm_epilogue_launch(d, reward, rescale, w, it, r3, st);
    } else {
      dense_bwd_sweep_launch(d, reward, rescale, w, it, r3, st);
    }
    if (hipError_t e = hipGetLastError()) return hip_fail(e, "dense backward sweep");
    r3 = r3 == 2 ? 0 : r3 + 1;
  }
  dense_bwd_final_launch(d, reward, rescale, p_action, status, w, collapsed, r3, st);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : hip_fail(e, "dense backward");
}

}  // namespace irlmx

using namespace irlmx;

extern "C" int irlmx_dense_to_rows(const double* dense, int32_t n_states, int32_t n_actions, double* p_rows,
                                   double* m_rows, void* stream) {
  if (!dense || !p_rows || !m_rows || n_states <= 0 || n_actions <= 0 || n_actions > kMaxActions) {
    set_error("dense_to_rows: bad arguments (n_states=%d, n_actions=%d in 1..%d, dense %s, p_rows %s, m_rows %s)",
              n_states, n_actions, kMaxActions, dense ? "set" : "NULL", p_rows ? "set" : "NULL",
              m_rows ? "set" : "NULL");
    return IRLMX_EINVAL;
  }
  dense_rows_launch(dense, n_states, n_actions, p_rows, m_rows, (hipStream_t)stream);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : hip_fail(e, "dense_to_rows");
}

namespace irlmx {
// The backward's tables fit the compact-weight cluster layout (cluster.hip,
// LAY 4: width 256 only)?  From the model's properties when the caller supplied
// them (irlmx_mdp_properties, checked once per table), else checked on the
// device per call (bwd_compact_ok_kernel), one int of device memory as the flag;
// that synchronises the stream.  IRLMX_COMPACT=0 turns the layout off.
static bool bwd_compact_check(const Model& m, int* flag, hipStream_t st) {
  if (hipMemsetAsync(flag, 0, sizeof(int), st) != hipSuccess) return false;
  hipLaunchKernelGGL(bwd_compact_ok_kernel, dim3((m.S + 255) / 256, m.shared ? 1 : m.B), dim3(256), 0, st,
                     m.row_val, m.W, m.H, m.A, flag);
  int h = 1;
  if (hipMemcpyAsync(&h, flag, sizeof(int), hipMemcpyDeviceToHost, st) != hipSuccess) return false;
  if (hipStreamSynchronize(st) != hipSuccess) return false;
  return h == 0;
}
static bool bwd_compact(const Model& m, int* flag, hipStream_t st) {
  if (!m.stencil || m.W != 256 || getenv_int("IRLMX_COMPACT", 1) == 0) return false;
  if (m.props & IRLMX_PROPS_KNOWN) return (m.props & IRLMX_PROP_COMPACT) != 0;
  return bwd_compact_check(m, flag, st);
}
}  // namespace irlmx

extern "C" size_t irlmx_workspace_bytes(const irlmx_mdp* mdp, int32_t op) {
  if (validate(mdp)) return 0;
  return carve(make_model(mdp), op, nullptr).total;
}

extern "C" int irlmx_execution_plan(const irlmx_mdp* mdp, int32_t op, int64_t* plan) {
  if (int rc = validate(mdp)) return rc;
  if (!plan) { set_error("plan is NULL"); return IRLMX_EINVAL; }
  // (a backward call with rescale = 0 never takes the cluster shape: see irlmx_backward_maxent)
  const bool no_rescale = op > 0 && (op & IRLMX_PLAN_NO_RESCALE) != 0;
  if (no_rescale) op &= ~IRLMX_PLAN_NO_RESCALE;
  if (op < IRLMX_OP_BACKWARD || op > IRLMX_OP_VALUE_ITERATION) { set_error("unknown op %d", op); return IRLMX_EINVAL; }
  if (no_rescale && op != IRLMX_OP_BACKWARD) { set_error("IRLMX_PLAN_NO_RESCALE applies to IRLMX_OP_BACKWARD only"); return IRLMX_EINVAL; }
  const Model m = make_model(mdp);
  for (int i = 0; i < IRLMX_PLAN_LEN; ++i) plan[i] = 0;
  FusedShape fs;
  if (fused_shape(m, op, &fs)) {
    plan[0] = IRLMX_SHAPE_FUSED;
    plan[5] = fs.spt;
    plan[7] = fs.threads;
    plan[8] = 1;
    plan[9] = (int64_t)fused_lds(m);
    return 0;
  }
  ClusterPlan cp;
  const int mode = op == IRLMX_OP_FORWARD ? kModeFwd : kModeBwd;
  bool compact = false;
  if (op == IRLMX_OP_BACKWARD && m.stencil && m.W == 256 && (m.props & IRLMX_PROPS_KNOWN)) {
    compact = bwd_compact(m, nullptr, nullptr);  // (the table's structure, from its properties)
  } else if (op == IRLMX_OP_BACKWARD && m.stencil && m.W == 256) {  // (data-dependent: checked on the device)
    int* flag = nullptr;
    if (hipMalloc((void**)&flag, sizeof(int)) == hipSuccess) {
      compact = bwd_compact(m, flag, nullptr);
      (void)hipFree(flag);
    }
  }
  if (m.stencil && (op == IRLMX_OP_FORWARD || (op == IRLMX_OP_BACKWARD && !no_rescale && m.A <= kMaxActions)) &&
      cluster_plan(m.W, m.H, m.B, mode, &cp, compact)) {
    plan[0] = IRLMX_SHAPE_CLUSTER;
    plan[1] = cp.R; plan[2] = cp.G; plan[3] = cp.C; plan[4] = cp.per_launch; plan[5] = cp.spt;
    plan[6] = cp.pair; plan[7] = cp.nt; plan[8] = (m.B + cp.per_launch - 1) / cp.per_launch;
    plan[9] = (int64_t)cp.lds;
    return 0;
  }
  GridPlan gp;
  if (grid_plan(m, op, &gp)) {
    plan[0] = IRLMX_SHAPE_GRID;
    plan[2] = gp.xcd;   // (the G column: 1 = workgroups grouped by XCD)
    plan[3] = gp.bpi;
    plan[4] = m.B;
    plan[5] = gp.spt;
    plan[7] = kGridThreads;
    plan[8] = 1;
    return 0;
  }
  DenseGridPlan dp;
  if (dense_grid(m, op, &dp)) {
    plan[0] = IRLMX_SHAPE_DENSE_GRID;
    plan[1] = dp.rb;    // (the R column: matrix rows per workgroup)
    plan[2] = dp.xcd;
    plan[3] = dp.bpi;
    plan[4] = m.B;
    plan[5] = dp.cpt;   // columns per thread
    plan[6] = dp.at;    // soft VI / VI: actions compiled per state (0: forward / backward)
    plan[7] = kDenseGridThreads;
    plan[8] = 1;
    return 0;
  }
  if (m.dense) {
    const bool gemm = op != IRLMX_OP_FORWARD && dense_gemm(m);
    plan[0] = gemm ? IRLMX_SHAPE_DENSE_GEMM : IRLMX_SHAPE_DENSE;
    plan[7] = kDenseThreads;
    plan[9] = dense_lds_vec(dense_view(m)) ? (int64_t)m.S * 8 : 0;
    return 0;
  }
  plan[0] = IRLMX_SHAPE_SWEEP;
  plan[7] = kSweepThreads;
  return 0;
}

extern "C" int irlmx_forward_svf(const irlmx_mdp* mdp, const double* p_initial, const uint8_t* terminal,
                                 const double* p_action, double eps, int64_t max_iter, double* svf,
                                 int64_t* iterations, int32_t* status, void* workspace,
                                 size_t workspace_bytes, void* stream) {
  if (int rc = validate(mdp)) return rc;
  const Model m = make_model(mdp);
  if (!m.stencil && !m.dense && (!m.col_idx || !m.col_val || m.Kc <= 0)) { set_error("ELL column form missing"); return IRLMX_EINVAL; }
  if (!m.stencil && !m.dense && m.Kc > m.S) { set_error("ELL k_col=%d out of range (1..%d)", m.Kc, m.S); return IRLMX_EINVAL; }
  if (int rc = need_all("forward_svf", {{p_initial, "p_initial"}, {terminal, "terminal"}, {p_action, "p_action"},
                                        {svf, "svf"}, {iterations, "iterations"}, {status, "status"}}))
    return rc;
  if (int rc = check_ws(m, IRLMX_OP_FORWARD, workspace_bytes, workspace)) return rc;
  hipStream_t st = (hipStream_t)stream;
  Ws ws = carve(m, IRLMX_OP_FORWARD, workspace);
  hipError_t e = hipMemsetAsync(workspace, 0, ws.total, st);
  if (e != hipSuccess) return hip_fail(e, "workspace memset");
  const dim3 g((m.S + 255) / 256, m.B);
  if (!m.dense) hipLaunchKernelGGL(fwd_weights_kernel, g, dim3(256), 0, st, m, p_action, terminal, ws.wgt, ws.bad);
  FwdArgs a{m, ws.wgt, ws.bad, p_initial, eps, (long long)max_iter, svf, iterations, status};
  FusedShape fs;
  if (fused_shape(m, IRLMX_OP_FORWARD, &fs)) {
    IRLMX_DISPATCH_FUSED(fwd_fused_ptr, fs, m.B, fused_lds(m), st, a);
    return 0;
  }
  if (m.dense) {  // dense rows (dense.hip): per-instance gather matrices WT, one launch per sweep
    const DenseView d = dense_view(m);
    const DenseBufs w = dense_bufs(ws);
    dense_fwd_weights_launch(d, p_action, terminal, w, st);
    DenseGridPlan dp;
    if (dense_grid(m, IRLMX_OP_FORWARD, &dp)) {  // one persistent launch, WT's rows in registers
      DenseGridArgs ga = dense_grid_args(m, ws);
      ga.mat = ws.wgt; ga.vin = p_initial; ga.bad = ws.bad; ga.eps = eps; ga.max_iter = (long long)max_iter;
      ga.out = svf; ga.iters = iterations; ga.status = status;
      const int rc = dense_grid_run(kModeFwd, dp, ga, st);
      if (rc != kClusterNotResident) return rc;  // else: the per-sweep shape below
    }
    count_event(IRLMX_CTR_SWEEP_CALLS);
    int rc = run_until_done(ws, m.B, st, [&](long long it, int r3) {
      dense_fwd_sweep_launch(d, p_initial, eps, (long long)max_iter, status, w, it, r3, st);
    });
    if (rc) return rc;
    hipLaunchKernelGGL(fwd_finish_kernel, g, dim3(256), 0, st, a, ws);
    e = hipGetLastError();
    return e == hipSuccess ? 0 : hip_fail(e, "dense forward");
  }
  ClusterPlan cp;
  bool persistent = true;  // false once a persistent launch found its workgroups not co-resident
  if (m.stencil && cluster_plan(m.W, m.H, m.B, kModeFwd, &cp)) {
    ClusterArgs ca{};
    ca.W = m.W; ca.H = m.H; ca.S = m.S; ca.A = m.A;
    ca.wgt = ws.wgt; ca.vin = p_initial; ca.bad = ws.bad;
    ca.eps = eps; ca.max_iter = (long long)max_iter;
    ca.gran = ws.gran; ca.sgran = ws.sgran; ca.err = ws.err;
    ca.out = svf; ca.iters = iterations; ca.status = status;
    const int rc = cluster_run(kModeFwd, cp, ca, m.B, st);
    if (rc != kClusterNonFinite && rc != kClusterNotResident) return rc;
    // an instance turned non-finite (rare): the cluster shape's convergence bits
    // drop NaN deltas, so rerun the call on the per-sweep shape, whose
    // bookkeeping is exact (same arithmetic, bit-identical results); likewise
    // when the tiles could not all run at once (another kernel holds CUs)
    persistent = rc != kClusterNotResident;
    if (rc == kClusterNonFinite) count_event(IRLMX_CTR_RERUN_NONFINITE);
    e = hipMemsetAsync(workspace, 0, ws.total, st);
    if (e != hipSuccess) return hip_fail(e, "workspace memset");
    hipLaunchKernelGGL(fwd_weights_kernel, g, dim3(256), 0, st, m, p_action, terminal, ws.wgt, ws.bad);
  }
  GridPlan gp;
  if (persistent && grid_plan(m, IRLMX_OP_FORWARD, &gp)) {  // ELL models: one persistent launch
    LinearGridArgs la{m, ws.wgt, p_initial, nullptr, ws.bad, eps, (long long)max_iter, 0, svf, iterations, status};
    GridArgs ga = grid_args(m, gp, ws);
    void* args[] = {&la, &ga};
    const int rc = grid_launch(m, IRLMX_OP_FORWARD, gp, args, ws, st);
    if (rc != kClusterNotResident) return rc;  // else: the per-sweep shape below
  }
  const dim3 gs((m.S + kSweepThreads - 1) / kSweepThreads, m.B);
  count_event(IRLMX_CTR_SWEEP_CALLS);
  int rc = run_until_done(ws, m.B, st, [&](long long it, int r3) {
    hipLaunchKernelGGL(fwd_sweep_kernel, gs, dim3(kSweepThreads), 0, st, a, ws, it, r3);
  });
  if (rc) return rc;
  hipLaunchKernelGGL(fwd_finish_kernel, g, dim3(256), 0, st, a, ws);
  e = hipGetLastError();
  return e == hipSuccess ? 0 : hip_fail(e, "fwd_finish");
}

extern "C" int irlmx_backward_maxent(const irlmx_mdp* mdp, const double* reward, const uint8_t* terminal,
                                     int32_t rescale, double* p_action, int32_t* status, void* workspace,
                                     size_t workspace_bytes, void* stream) {
  if (int rc = validate(mdp)) return rc;
  const Model m = make_model(mdp);
  if (int rc = need_all("backward_maxent",
                        {{reward, "reward"}, {terminal, "terminal"}, {p_action, "p_action"}, {status, "status"}}))
    return rc;
  if (int rc = check_ws(m, IRLMX_OP_BACKWARD, workspace_bytes, workspace)) return rc;
  hipStream_t st = (hipStream_t)stream;
  Ws ws = carve(m, IRLMX_OP_BACKWARD, workspace);
  hipError_t e = hipMemsetAsync(workspace, 0, ws.total, st);
  if (e != hipSuccess) return hip_fail(e, "workspace memset");
  if (m.dense) return dense_backward(m, reward, terminal, rescale, p_action, status, ws, st);
  hipLaunchKernelGGL(bwd_weights_kernel, dim3((m.S + 255) / 256, m.B), dim3(256), 0, st, m, reward, ws.wgt, ws.bad);
  BwdArgs a{m, ws.wgt, reward, terminal, rescale, p_action, status};
  FusedShape fs;
  if (fused_shape(m, IRLMX_OP_BACKWARD, &fs)) {
    IRLMX_DISPATCH_FUSED(bwd_fused_ptr, fs, m.B, fused_lds(m), st, a);
    return 0;
  }
  ClusterPlan cp;
  bool persistent = true;  // false once a persistent launch found its workgroups not co-resident
  // (without rescaling the partition vector overflows like the reference's: such
  // calls take the per-sweep shape, whose non-finite bookkeeping is per sweep)
  if (m.stencil && m.A <= kMaxActions && rescale &&
      cluster_plan(m.W, m.H, m.B, kModeBwd, &cp, m.W == 256 && bwd_compact(m, ws.err + 3, st))) {
    hipLaunchKernelGGL(bwd_growth_kernel, dim3(m.B), dim3(1024), 0, st, ws.wgt, m.W, m.S, m.B, ws.growth);
    ClusterArgs ca{};
    ca.W = m.W; ca.H = m.H; ca.S = m.S; ca.A = m.A;
    ca.tab_shared = m.shared ? 1 : 0;
    ca.wgt = ws.wgt; ca.row_val = m.row_val; ca.vin = reward; ca.term = terminal; ca.growth = ws.growth;
    ca.n_sweeps = 2LL * m.S - 1; ca.rescale = rescale;
    ca.gran = ws.gran; ca.sgran = ws.sgran; ca.err = ws.err;
    ca.out = p_action; ca.status = status;
    const int rc = cluster_run(kModeBwd, cp, ca, m.B, st);
    if (rc != kClusterNotResident) {
      if (rc) return rc;
      // instances with non-finite weights: all NaN (bwd_nonfinite_rule), outside the sweep kernel
      hipLaunchKernelGGL(bwd_nan_fill_kernel, dim3((m.S * m.A + 255) / 256, m.B), dim3(256), 0, st, m, ws.bad,
                         p_action);
      e = hipGetLastError();
      return e == hipSuccess ? 0 : hip_fail(e, "backward nan fill");
    }
    // the tiles could not all run at once (another kernel holds CUs): rerun on
    // the per-sweep shape (same arithmetic, bit-identical results)
    persistent = false;
    e = hipMemsetAsync(workspace, 0, ws.total, st);
    if (e != hipSuccess) return hip_fail(e, "workspace memset");
    hipLaunchKernelGGL(bwd_weights_kernel, dim3((m.S + 255) / 256, m.B), dim3(256), 0, st, m, reward, ws.wgt, ws.bad);
  }
  GridPlan gp;
  if (persistent && grid_plan(m, IRLMX_OP_BACKWARD, &gp)) {  // ELL models: one persistent launch
    LinearGridArgs la{m, ws.wgt, reward, terminal, ws.bad, 0.0, 0, rescale, p_action, nullptr, status};
    GridArgs ga = grid_args(m, gp, ws);
    void* args[] = {&la, &ga};
    const int rc = grid_launch(m, IRLMX_OP_BACKWARD, gp, args, ws, st);
    if (rc != kClusterNotResident) return rc;  // else: the per-sweep shape below
  }
  const dim3 g((m.S + kSweepThreads - 1) / kSweepThreads, m.B);
  count_event(IRLMX_CTR_SWEEP_CALLS);
  hipLaunchKernelGGL(bwd_init_kernel, g, dim3(kSweepThreads), 0, st, a, ws);
  const long long collapsed = 2LL * m.S - 1;
  int r3 = 0;
  for (long long it = 0; it < collapsed; ++it) {
    hipLaunchKernelGGL(bwd_sweep_kernel, g, dim3(kSweepThreads), 0, st, a, ws, it, r3);
    r3 = r3 == 2 ? 0 : r3 + 1;
  }
  hipLaunchKernelGGL(bwd_final_kernel, g, dim3(kSweepThreads), 0, st, a, ws, collapsed, r3);
  e = hipGetLastError();
  return e == hipSuccess ? 0 : hip_fail(e, "backward");
}

// np_row_dot sums an ELL row's entries in slot order, which is numpy's order
// only when every action's nonzero entries sit in ascending column order
// (irlmx_dense_to_ell's layout; unused slots, value 0, are exact no-ops
// anywhere).  One thread per (table instance, row): *bad set on a violation.
__global__ void np_ell_ascending_kernel(Model m, int* bad) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (s >= m.S) return;
  for (int a = 0; a < m.A; ++a) {
    int last = -1;
    for (int k = 0; k < m.K; ++k) {
      if (row_val(m, b, a, k, s) == 0.0) continue;
      const int c = m.row_idx[((size_t)b * m.K + k) * m.S + s];
      if (c <= last) { atomicOr(bad, 1); return; }
      last = c;
    }
  }
}

// Whether every ELL row holds its nonzero entries in ascending column order
// (np_ell_ascending_kernel), into *sorted; synchronises the stream.
static int ell_rows_sorted(const Model& m, hipStream_t st, bool* sorted) {
  int* flag = nullptr;
  hipError_t e = hipMallocAsync((void**)&flag, sizeof(int), st);
  if (e != hipSuccess) return hip_fail(e, "ELL row-order check");
  int h = 0;
  e = hipMemsetAsync(flag, 0, sizeof(int), st);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(np_ell_ascending_kernel, dim3((m.S + 255) / 256, m.shared ? 1 : m.B), dim3(256), 0, st, m,
                       flag);
    e = hipMemcpyAsync(&h, flag, sizeof(int), hipMemcpyDeviceToHost, st);
  }
  (void)hipFreeAsync(flag, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) return hip_fail(e, "ELL row-order check");
  *sorted = h == 0;
  return 0;
}

// The numpy-order row dots' precondition on an ELL model (above); other
// layouts visit their entries in column order by construction.  From the
// model's properties when the caller supplied them (irlmx_mdp_properties: once
// per table), else checked on the device per call (synchronises).
static int np_check_ell_rows(const Model& m, const char* fn, hipStream_t st) {
  if (m.stencil || m.dense) return 0;
  bool sorted = true;
  if (m.props & IRLMX_PROPS_KNOWN) sorted = (m.props & IRLMX_PROP_ELL_SORTED) != 0;
  else if (int rc = ell_rows_sorted(m, st, &sorted)) return rc;
  if (!sorted) {
    set_error("%s: an ELL row holds its nonzero entries out of ascending column order (numpy's order needs "
              "irlmx_dense_to_ell's slot layout)", fn);
    return IRLMX_EINVAL;
  }
  return 0;
}

extern "C" int irlmx_mdp_properties(const irlmx_mdp* mdp, int32_t* props, void* stream) {
  if (int rc = validate(mdp)) return rc;
  if (!props) { set_error("mdp_properties: props is NULL"); return IRLMX_EINVAL; }
  Model m = make_model(mdp);
  m.props = 0;
  hipStream_t st = (hipStream_t)stream;
  int32_t p = IRLMX_PROPS_KNOWN;
  if (m.stencil) {
    int* flag = nullptr;
    hipError_t e = hipMallocAsync((void**)&flag, sizeof(int), st);
    if (e != hipSuccess) return hip_fail(e, "mdp_properties");
    const bool compact = bwd_compact_check(m, flag, st);
    e = hipFreeAsync(flag, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return hip_fail(e, "mdp_properties");
    if (compact) p |= IRLMX_PROP_COMPACT;
  } else if (!m.dense) {
    bool sorted = false;
    if (int rc = ell_rows_sorted(m, st, &sorted)) return rc;
    if (sorted) p |= IRLMX_PROP_ELL_SORTED;
  }
  *props = p;
  return 0;
}

extern "C" int irlmx_backward_maxent_numpy_order(const irlmx_mdp* mdp, const double* exp_reward,
                                                 const uint8_t* terminal, double* p_action, int32_t* status,
                                                 void* stream) {
  if (int rc = validate(mdp)) return rc;
  const Model m = make_model(mdp);
  if (int rc = need_all("backward_maxent_numpy_order", {{exp_reward, "exp_reward"}, {terminal, "terminal"},
                                                        {p_action, "p_action"}, {status, "status"}}))
    return rc;
  if (m.S > kFusedMaxStates || (m.S & 3) > 1) {
    set_error("backward_maxent_numpy_order: numpy's order is restated for S <= %d with S %% 4 in {0, 1}, got S=%d",
              kFusedMaxStates, m.S);
    return IRLMX_EINVAL;
  }
  hipStream_t st = (hipStream_t)stream;
  if (int rc = np_check_ell_rows(m, "backward_maxent_numpy_order", st)) return rc;
  NpArgs a{m, exp_reward, terminal, p_action, status};
  const bool cached = m.stencil && m.S <= kNpCachedMaxStates && m.A <= kNpCachedMaxActions;
  void (*fn)(NpArgs) = cached ? (m.S <= kNpCachedThreads ? bwd_numpy_order_cached_kernel<1>
                                                         : bwd_numpy_order_cached_kernel<2>)
                              : m.stencil ? bwd_numpy_order_kernel<IRLMX_LAYOUT_STENCIL5>
                                          : (m.dense ? bwd_numpy_order_kernel<IRLMX_LAYOUT_DENSE>
                                                     : bwd_numpy_order_kernel<IRLMX_LAYOUT_ELL>);
  const size_t lds = 2 * (size_t)m.S * sizeof(double) + 2 * sizeof(int);
  hipError_t e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return hip_fail(e, "hipFuncSetAttribute");
  const int nthr = cached ? std::min(kNpCachedThreads, ((m.S + kWave - 1) / kWave) * kWave)
                          : (m.S >= 1024 ? 1024 : ((m.S + kWave - 1) / kWave) * kWave);
  hipLaunchKernelGGL(fn, dim3(m.B), dim3(nthr), lds, st, a);
  e = hipGetLastError();
  return e == hipSuccess ? 0 : hip_fail(e, "backward_maxent_numpy_order");
}

static int bellman_common(const irlmx_mdp* mdp, const double* reward, const double* phi, double discount,
                          double eps, int64_t max_iter, int average, double* p_action, double* value,
                          int64_t* iterations, int32_t* status, void* workspace, size_t workspace_bytes,
                          void* stream, bool soft) {
  if (int rc = validate(mdp)) return rc;
  const Model m = make_model(mdp);
  const int op = soft ? IRLMX_OP_SOFT_BACKWARD : IRLMX_OP_VALUE_ITERATION;
  if (int rc = need_all(soft ? "soft_backward" : "value_iteration",
                        {{reward, "reward"}, {phi, soft ? "terminal_reward" : nullptr},
                         {p_action, soft ? "p_action" : nullptr}, {value, soft ? nullptr : "value"},
                         {iterations, "iterations"}, {status, "status"}}))
    return rc;
  if (int rc = check_ws(m, op, workspace_bytes, workspace)) return rc;
  hipStream_t st = (hipStream_t)stream;
  Ws ws = carve(m, op, workspace);
  hipError_t e = hipMemsetAsync(workspace, 0, ws.total, st);
  if (e != hipSuccess) return hip_fail(e, "workspace memset");
  SoftArgs a{m, reward, phi, discount, eps, (long long)max_iter, average, p_action, value, iterations, status};
  FusedShape fs;
  if (fused_shape(m, op, &fs)) {
    if (soft) IRLMX_DISPATCH_FUSED(soft_fused_ptr, fs, m.B, fused_lds(m), st, a);
    else IRLMX_DISPATCH_FUSED(vi_fused_ptr, fs, m.B, fused_lds(m), st, a);
    return 0;
  }
  const dim3 g((m.S + kSweepThreads - 1) / kSweepThreads, m.B);
  // the Bellman sweep is a latency chain per state (A dots, A softmax folds):
  // smaller workgroups spread one instance over more CUs (IRLMX_BELLMAN_THREADS)
  const int bt = std::max(64, std::min(kSweepThreads, getenv_int("IRLMX_BELLMAN_THREADS", kSweepThreads)));
  const dim3 gb((m.S + bt - 1) / bt, m.B);
  const size_t n = (size_t)m.B * m.S;
  hipLaunchKernelGGL(fill_kernel, dim3((n + 255) / 256), dim3(256), 0, st, ws.buf0, n, soft ? -1e200 : 0.0);
  if (m.dense) {  // dense rows (dense.hip)
    const DenseView d = dense_view(m);
    const DenseBufs w = dense_bufs(ws);
    const DenseBellman db{reward, phi, discount, eps, (long long)max_iter, average, soft ? 1 : 0, p_action, value,
                          iterations, status};
    const bool gemm = dense_gemm(m);  // the P . [v_1 .. v_B] products on the MFMA kernel
    DenseGridPlan dp;
    if (dense_grid(m, op, &dp)) {  // one persistent launch, the A rows of each state in registers
      DenseGridArgs ga = dense_grid_args(m, ws);
      ga.P = m.row_val; ga.vin = reward; ga.phi = phi; ga.discount = discount; ga.average = average;
      ga.value = value; ga.eps = eps; ga.max_iter = (long long)max_iter;
      ga.out = p_action; ga.iters = iterations; ga.status = status;
      const int rc = dense_bellman_grid_run(soft, dp, ga, st);
      if (rc != kClusterNotResident) return rc;  // else: the per-sweep shape below
    }
    hipError_t gerr = hipSuccess;
    count_event(IRLMX_CTR_SWEEP_CALLS);
    int rc = run_until_done(ws, m.B, st, [&](long long it, int r3) {
      if (gemm) {
        const hipError_t e = dense_bellman_gemm_sweep_launch(d, db, w, it, r3, st);
        if (e != hipSuccess && gerr == hipSuccess) gerr = e;
      } else {
        dense_bellman_sweep_launch(d, db, w, it, r3, st);
      }
    });
    if (gerr != hipSuccess) return hip_fail(gerr, "dense gemm");
    if (rc) return rc;
    dense_bellman_finish_launch(d, db, w, st);
    e = hipGetLastError();
    return e == hipSuccess ? 0 : hip_fail(e, "dense bellman");
  }
  GridPlan gp;
  if (grid_plan(m, op, &gp)) {  // persistent grid shape: one launch for the whole loop
    GridArgs ga = grid_args(m, gp, ws);
    void* args[] = {&a, &ga};
    const int rc = grid_launch(m, op, gp, args, ws, st);
    if (rc != kClusterNotResident) return rc;  // else: the per-sweep shape below
  }
  count_event(IRLMX_CTR_SWEEP_CALLS);
  int rc = run_until_done(ws, m.B, st, [&](long long it, int r3) {
    if (soft) hipLaunchKernelGGL(bellman_sweep_kernel<true>, gb, dim3(bt), 0, st, a, ws, it, r3);
    else hipLaunchKernelGGL(bellman_sweep_kernel<false>, gb, dim3(bt), 0, st, a, ws, it, r3);
  });
  if (rc) return rc;
  if (soft) hipLaunchKernelGGL(bellman_finish_kernel<true>, g, dim3(kSweepThreads), 0, st, a, ws);
  else hipLaunchKernelGGL(bellman_finish_kernel<false>, g, dim3(kSweepThreads), 0, st, a, ws);
  e = hipGetLastError();
  return e == hipSuccess ? 0 : hip_fail(e, "bellman finish");
}

extern "C" int irlmx_soft_backward(const irlmx_mdp* mdp, const double* reward, const double* terminal_reward,
                                   double discount, double eps, int64_t max_iter, double* p_action,
                                   double* value, int64_t* iterations, int32_t* status, void* workspace,
                                   size_t workspace_bytes, void* stream) {
  return bellman_common(mdp, reward, terminal_reward, discount, eps, max_iter, 0, p_action, value, iterations,
                        status, workspace, workspace_bytes, stream, true);
}

extern "C" int irlmx_value_iteration(const irlmx_mdp* mdp, const double* reward, double discount, double eps,
                                     int32_t average, int64_t max_iter, double* value, int64_t* iterations,
                                     int32_t* status, void* workspace, size_t workspace_bytes, void* stream) {
  return bellman_common(mdp, reward, nullptr, discount, eps, max_iter, average, nullptr, value, iterations,
                        status, workspace, workspace_bytes, stream, false);
}

extern "C" int irlmx_forward_svf_numpy_order(const irlmx_mdp* mdp, const double* p_initial,
                                             const uint8_t* terminal, const double* p_action, double eps,
                                             int64_t max_iter, double* svf, int64_t* iterations, int32_t* status,
                                             void* stream) {
  if (int rc = validate(mdp)) return rc;
  const Model m = make_model(mdp);
  if (int rc = need_all("forward_svf_numpy_order", {{p_initial, "p_initial"}, {terminal, "terminal"},
                                                    {p_action, "p_action"}, {svf, "svf"},
                                                    {iterations, "iterations"}, {status, "status"}}))
    return rc;
  if (m.S > kFusedMaxStates || (m.S & 3) > 1) {
    set_error("forward_svf_numpy_order: numpy's order is restated for S <= %d with S %% 4 in {0, 1}, got S=%d",
              kFusedMaxStates, m.S);
    return IRLMX_EINVAL;
  }
  if (mdp->layout == IRLMX_LAYOUT_ELL && (!m.col_idx || !m.col_val || m.Kc <= 0 || m.Kc > kNpColMax)) {
    set_error("forward_svf_numpy_order: ELL column form missing or k_col > %d", kNpColMax);
    return IRLMX_EINVAL;
  }
  NpFwdArgs a{m, p_initial, terminal, p_action, eps, (long long)max_iter, svf, iterations, status};
  const bool cached = m.stencil && m.S <= kNpCachedMaxStates && m.A <= kNpCachedMaxActions;
  void (*k)(NpFwdArgs) = cached ? (m.S <= kNpCachedThreads ? fwd_numpy_order_cached_kernel<1>
                                                           : fwd_numpy_order_cached_kernel<2>)
                                : m.stencil ? fwd_numpy_order_kernel<IRLMX_LAYOUT_STENCIL5>
                                            : (m.dense ? fwd_numpy_order_kernel<IRLMX_LAYOUT_DENSE>
                                                       : fwd_numpy_order_kernel<IRLMX_LAYOUT_ELL>);
  const size_t lds = 2 * (size_t)m.S * sizeof(double) + 3 * sizeof(unsigned long long) + 2 * sizeof(int);
  hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return hip_fail(e, "hipFuncSetAttribute");
  const int nthr = cached ? std::min(kNpCachedThreads, ((m.S + kWave - 1) / kWave) * kWave)
                          : (m.S >= 1024 ? 1024 : ((m.S + kWave - 1) / kWave) * kWave);
  hipLaunchKernelGGL(k, dim3(m.B), dim3(nthr), lds, (hipStream_t)stream, a);
  e = hipGetLastError();
  return e == hipSuccess ? 0 : hip_fail(e, "forward_svf_numpy_order");
}

// Soft VI / VI in numpy's order: one workgroup per instance (S <= 4096, S % 4 in {0, 1}).
static int bellman_numpy_order(const irlmx_mdp* mdp, const double* reward, const double* phi, double discount,
                               double eps, int64_t max_iter, int average, double* p_action, double* value,
                               int64_t* iterations, int32_t* status, void* stream, bool soft) {
  if (int rc = validate(mdp)) return rc;
  const Model m = make_model(mdp);
  const char* fn = soft ? "soft_backward_numpy_order" : "value_iteration_numpy_order";
  if (int rc = need_all(fn, {{reward, "reward"}, {phi, soft ? "terminal_reward" : nullptr},
                             {p_action, soft ? "p_action" : nullptr}, {value, soft ? nullptr : "value"},
                             {iterations, "iterations"}, {status, "status"}}))
    return rc;
  if (m.S > kFusedMaxStates || (m.S & 3) > 1) {
    set_error("%s: numpy's order is restated for S <= %d with S %% 4 in {0, 1}, got S=%d", fn, kFusedMaxStates, m.S);
    return IRLMX_EINVAL;
  }
  if (int rc = np_check_ell_rows(m, fn, (hipStream_t)stream)) return rc;
  SoftArgs a{m, reward, phi, discount, eps, (long long)max_iter, average, p_action, value, iterations, status};
  void (*k)(SoftArgs) = nullptr;
  const bool cached = m.stencil && m.S <= kNpCachedMaxStates && m.A <= kNpCachedMaxActions;
  if (cached) {
    if (m.S <= kNpCachedThreads) k = soft ? bellman_numpy_order_cached_kernel<true, 1>
                                          : bellman_numpy_order_cached_kernel<false, 1>;
    else k = soft ? bellman_numpy_order_cached_kernel<true, 2> : bellman_numpy_order_cached_kernel<false, 2>;
  } else if (m.stencil) k = soft ? bellman_numpy_order_kernel<true, IRLMX_LAYOUT_STENCIL5>
                          : bellman_numpy_order_kernel<false, IRLMX_LAYOUT_STENCIL5>;
  else if (m.dense) k = soft ? bellman_numpy_order_kernel<true, IRLMX_LAYOUT_DENSE>
                             : bellman_numpy_order_kernel<false, IRLMX_LAYOUT_DENSE>;
  else k = soft ? bellman_numpy_order_kernel<true, IRLMX_LAYOUT_ELL> : bellman_numpy_order_kernel<false, IRLMX_LAYOUT_ELL>;
  const size_t lds = 2 * (size_t)m.S * sizeof(double) + 4 * sizeof(unsigned long long);
  hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return hip_fail(e, "hipFuncSetAttribute");
  const int nthr = cached ? std::min(kNpCachedThreads, ((m.S + kWave - 1) / kWave) * kWave)
                          : (m.S >= 1024 ? 1024 : ((m.S + kWave - 1) / kWave) * kWave);
  hipLaunchKernelGGL(k, dim3(m.B), dim3(nthr), lds, (hipStream_t)stream, a);
  e = hipGetLastError();
  return e == hipSuccess ? 0 : hip_fail(e, fn);
}

extern "C" int irlmx_soft_backward_numpy_order(const irlmx_mdp* mdp, const double* reward,
                                               const double* terminal_reward, double discount, double eps,
                                               int64_t max_iter, double* p_action, double* value,
                                               int64_t* iterations, int32_t* status, void* stream) {
  return bellman_numpy_order(mdp, reward, terminal_reward, discount, eps, max_iter, 0, p_action, value, iterations,
                             status, stream, true);
}

extern "C" int irlmx_value_iteration_numpy_order(const irlmx_mdp* mdp, const double* reward, double discount,
                                                 double eps, int32_t average, int64_t max_iter, double* value,
                                                 int64_t* iterations, int32_t* status, void* stream) {
  return bellman_numpy_order(mdp, reward, nullptr, discount, eps, max_iter, average, nullptr, value, iterations,
                             status, stream, false);
}

extern "C" int irlmx_dense_gemm(const double* m, const double* z, double* c, int32_t rows, int32_t n, int32_t batch,
                                void* stream) {
  if (!m || !z || !c || rows <= 0 || n <= 0 || batch <= 0) {
    set_error("dense_gemm: bad arguments (rows=%d, n=%d, batch=%d, m %s, z %s, c %s)", rows, n, batch,
              m ? "set" : "NULL", z ? "set" : "NULL", c ? "set" : "NULL");
    return IRLMX_EINVAL;
  }
  const hipError_t e = dense_gemm_launch(m, z, c, rows, n, batch, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "dense_gemm");
}

extern "C" int irlmx_dense_gemm_variant(int32_t rows, int32_t n, int32_t batch, int32_t* variant) {
  if (!variant || rows <= 0 || n <= 0 || batch <= 0) {
    set_error("dense_gemm_variant: bad arguments");
    return IRLMX_EINVAL;
  }
  int v[4];
  dense_gemm_variant(rows, n, batch, v);
  for (int i = 0; i < 4; ++i) variant[i] = v[i];
  return 0;
}
