// Persistent temporally blocked stencil kernels (cluster.hip): shared declarations.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"

namespace irlmx {

constexpr int kCT = 1024;          // threads per workgroup, per-state layout
constexpr int kSptMax = 6;         // states per thread, per-state layout (no VGPR spills at 128 VGPRs)
constexpr int kPairThreads = 512;  // threads per workgroup, pair layouts (256 VGPRs)
constexpr int kSptMaxPair = 12;    // states per thread, pair layouts -> extended tile <= 6144 states
constexpr int kSptMaxQuadFwd = 12;  // forward with column quads (register budget)
// backward with column quads: 16 states per lane (32 rows at width 256; ~30
// VGPRs spill to scratch, yet 3.8 % faster at config 4 than 12: G = 8 ghost
// rows instead of 4 halve the exchanges)
constexpr int kSptMaxQuadBwd = 16;
// backward with column quads and compact weights (layout 4, width 256): three
// weights per state instead of five, so 20 states per lane fit the registers
constexpr int kSptMaxQuadBwdCW = 20;
constexpr int kTMax = 16;          // max sweeps per block (= max ghost rows)
constexpr int kSoloBwdT = 256;     // backward sweeps per block of a solo tile (no ghost rows)
#ifndef IRLMX_RESCALE_EVERY
#define IRLMX_RESCALE_EVERY 32
#endif
constexpr int kRescaleEvery = IRLMX_RESCALE_EVERY;  // backward: max blocks between rescales
constexpr size_t kMaxLdsBytes = 160 * 1024;  // LDS per CU (one workgroup per CU)
// Tile-summary granule slots per instance, indexed by block % kSumSlots.  A
// backward tile reads the other tiles' summaries only on rescale blocks (at
// most kRescaleEvery apart), so between two such blocks a tile can run ahead
// of a distant tile by up to kRescaleEvery blocks; its summary for block
// m + kRescaleEvery must not land in the slot a slow tile is still polling for
// block m.  (The period is also capped per instance so that the partition
// vector neither grows nor shrinks by more than 2^900 between two rescales:
// cluster.hip, p_max.)
constexpr int kSumSlots = kRescaleEvery < 8 ? 8 : kRescaleEvery + 1;
static_assert(kSumSlots > kRescaleEvery, "summary slots must outlast the rescale period");
// Rows of an instance's summary granules (sgran): [0, kSumSlots) block summaries,
// kSumSlots the tiles' XCC ids, kSumSlots + 1 the forward's full convergence
// flags of a replayed block (cluster.hip, "cheap convergence proof").
constexpr int kSumRows = kSumSlots + 2;
constexpr int kXccRow = kSumSlots, kFullRow = kSumSlots + 1;
constexpr size_t kClusterStaticLds = 128;     // cluster_kernel's own __shared__ variables (resident flag, stamps)
constexpr int kModeFwd = 0;
constexpr int kModeBwd = 1;

struct ClusterArgs {
  int W, H, S, A;
  int R, G, C, T;          // rows per tile, ghost rows, tiles per instance, max sweeps per block
  int b0;                  // first instance of this launch
  int nb;                  // instances in this launch
  int btot;                // instances in the granule arrays
  int emax;                // LDS buffer length (states)
  int tab_shared;          // backward tables shared by all instances
  const double* wgt;       // forward: [B][5][S] gather weights; backward: [B][5][S] collapsed, reward-folded
  const double* row_val;   // backward final sweep: [B'][A][5][S]
  const double* vin;       // forward: p0 [B][S]; backward: reward [B][S]
  const uint8_t* term;     // backward: terminal mask [B][S]
  const int32_t* bad;      // forward: non-finite policy flags [B]
  const unsigned long long* growth;  // backward: per-instance growth / decay bound bits [2][B]
  double eps;
  long long max_iter;
  long long n_sweeps;      // backward: collapsed sweeps (2S - 1)
  int rescale;
  unsigned long long* gran;   // [B][gran_inst_len] x 16-byte tagged granule pairs (halo rows, see kGranRowPad)
  unsigned long long* sgran;  // [B][kSumRows][H] x 16-byte tagged granule pairs (tile summaries, XCC ids, full flags)
  int xcd_group;           // number the tiles of an instance within one XCD group
  unsigned salt;           // per-launch granule tag salt
  int* err;                // [0]: exchange timeout (1), non-finite (2), not co-resident (4); [1..2]: rendezvous
  int n_resident;          // workgroups of this launch that must run at once (coresident())
  unsigned long long gather_ticks;  // exchange timeout (s_memrealtime ticks; kGatherTicks unless a test shortens it)
  int test_drop;           // tests only (IRLMX_TEST_DROP_TILE): this workgroup leaves after the rendezvous, else -1
  int eager_summary;       // A/B and tests (IRLMX_EAGER_SUMMARY=1): wait for every tile's summary every block
  unsigned long long* stamps;  // optional [grid][8] phase cycle counters (IRLMX_STAMPS=1), else null
  double* out;             // forward: svf [B][S]; backward: pi [B][S][A]
  int64_t* iters;
  int32_t* status;
};

struct ClusterPlan {
  int R, G, C, T, per_launch, spt, emax;
  size_t lds;
  int pair;             // in-tile layout: 0 per state, 1 pair rows, 2 column pairs, 3 column quads,
                        // 4 column quads with compact weights (backward, width 256)
  int nt;               // threads per workgroup
};

// Tagged granules (cdna_hip_programming.md Guideline 16, form R2: the data is
// the flag).  A 64-bit value v travels as one 16-byte sc1 store of
// {lo32(v), tag, hi32(v), tag}; each 8-byte half is an untorn {value, tag}
// granule, so a reader that sees tag == the block's epoch in both halves (sc1
// loads: L1 bypassed, no acquire needed) holds the value of that block.  No
// counter, no fence, one fabric round trip per exchange.  Tag = per-launch
// salt | (block + 1); the workspace is also zeroed before every call.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#ifndef IRLMX_POLL_SLEEP
#define IRLMX_POLL_SLEEP 1   // s_sleep units (64 cycles) between polling passes
#endif
constexpr int kGatherPerThread = 4;

// Halo granule layout per instance: [2 parities][S states (+ kGranRowPad per
// row)] x 16 B.  At width 128 the parities and the instances sit a few 128-B
// lines further apart than their power-of-two sizes (24 and 40 granules); other
// widths keep the power-of-two distances.  Measured (DESIGN.md section 4 "Halo
// granule layout", profiles/r06_pad_ab.txt, r06_pmc_writeback.txt): the offsets
// make the L2 write dirty granule lines back 4x as often (config 3's backward
// 3.1 -> 12 GB of WRITE_SIZE per launch, no extra evictions) yet run config 3's
// backward 0.5-0.7 % faster on three boxes; at width 256 (config 4) the
// unpadded layout is ~1 % faster.  IRLMX_GRAN_PAR_PAD / _INST_PAD (>= 0) force
// one layout at every width.
#ifndef IRLMX_GRAN_ROW_PAD
#define IRLMX_GRAN_ROW_PAD 0
#endif
#ifndef IRLMX_GRAN_PAR_PAD
#define IRLMX_GRAN_PAR_PAD -1
#endif
#ifndef IRLMX_GRAN_INST_PAD
#define IRLMX_GRAN_INST_PAD -1
#endif
constexpr int kGranRowPad = IRLMX_GRAN_ROW_PAD;                   // extra granules per row (8: one 128-B line)
__host__ __device__ inline size_t gran_par_pad(int W) { return IRLMX_GRAN_PAR_PAD >= 0 ? IRLMX_GRAN_PAR_PAD : (W == 128 ? 24 : 0); }
__host__ __device__ inline size_t gran_inst_pad(int W) { return IRLMX_GRAN_INST_PAD >= 0 ? IRLMX_GRAN_INST_PAD : (W == 128 ? 40 : 0); }
__host__ __device__ inline size_t gran_par_len(int W, int H) {
  return (size_t)H * (W + kGranRowPad) + gran_par_pad(W);
}
__host__ __device__ inline size_t gran_inst_len(int W, int H) { return 2 * gran_par_len(W, H) + gran_inst_pad(W); }

// A granule buffer: its descriptor (and, in IRLMX_DEVICE_CHECKS builds, its
// byte length for the offset checks).
struct Gran {
  __amdgpu_buffer_rsrc_t r;
#if IRLMX_DEVICE_CHECKS
  unsigned bytes;
#endif
};
__device__ inline Gran gran_rsrc(const void* base, unsigned bytes) {
  Gran g;
  g.r = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
#if IRLMX_DEVICE_CHECKS
  g.bytes = bytes;
#endif
  return g;
}
#if IRLMX_DEVICE_CHECKS
__device__ inline bool gran_in(const Gran& g, unsigned off) { return g.bytes >= 16u && off <= g.bytes - 16u; }
#endif
__device__ inline unsigned long long dbits(double v) { return (unsigned long long)__double_as_longlong(v); }
// sc1 (write-through) store, or a plain store when every reader shares this XCD's L2
__device__ inline void gran_store(const Gran& g, unsigned off, unsigned long long v, unsigned tag, bool plain) {
  if (!IRLMX_DCHECK(gran_in(g, off), kCheckGranule)) return;
  const u32x4 x = {(unsigned)v, tag, (unsigned)(v >> 32), tag};
  if (plain) __builtin_amdgcn_raw_buffer_store_b128(x, g.r, (int)off, 0, 0);
  else __builtin_amdgcn_raw_buffer_store_b128(x, g.r, (int)off, 0, 16 /* sc1 */);
}
// Poll the granule pairs selected by `want` (bit k: entry k; the last entry
// through rsrc `rl`, the others through `r`) until all carry `tag`; false
// after `limit` ticks of s_memrealtime (100 MHz; default 20 s).  Every pending
// load of a pass is in flight at once.
constexpr unsigned long long kGatherTicks = 2000000000ull;
// (mask type M: 32-bit, or 64-bit for more than 32 entries)
template <int N, typename M>
__device__ inline bool gran_gather(const Gran& r, const Gran& rl, const unsigned (&off)[N],
                                   M want, unsigned tag, unsigned long long (&v)[N],
                                   unsigned long long limit = kGatherTicks) {
  static_assert(N <= 8 * (int)sizeof(M), "gran_gather: mask too narrow");
  M pending = want;
#if IRLMX_DEVICE_CHECKS
#pragma unroll
  for (int k = 0; k < N; ++k) {
    if (((pending >> k) & 1u) && !IRLMX_DCHECK(gran_in(k == N - 1 ? rl : r, off[k]), kCheckGranule)) {
      pending &= ~((M)1 << k);  // skipped: the value reads as 0
      v[k] = 0ull;
    }
  }
#endif
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (pending) {
    u32x4 x[N];
#pragma unroll
    for (int k = 0; k < N; ++k)
      if ((pending >> k) & 1u)
        x[k] = __builtin_amdgcn_raw_buffer_load_b128(k == N - 1 ? rl.r : r.r, (int)off[k], 0, 16 /* sc1 */);
#pragma unroll
    for (int k = 0; k < N; ++k)
      if (((pending >> k) & 1u) && x[k].y == tag && x[k].w == tag) {
        v[k] = ((unsigned long long)x[k].z << 32) | x[k].x;
        pending &= ~((M)1 << k);
      }
    if (!pending) break;
    if (__builtin_amdgcn_s_memrealtime() - t0 > limit) return false;
    __builtin_amdgcn_s_sleep(IRLMX_POLL_SLEEP);
  }
  return true;
}

// Co-residency rendezvous of a persistent launch (cluster and grid shapes),
// thread 0 of every participating workgroup: count in ctr[0] ("arrived") and
// wait for all n, then count in ctr[1] ("committed") and wait for all n.  The
// hand-offs assume that all workgroups run at once; when another kernel or
// process holds CUs, some start only after others have left, and without this
// check they would spin until the exchange timeout.  A workgroup that does not
// see all arrivals within kArriveTicks leaves without committing, so nobody
// passes the second phase and the host reruns the call on the per-sweep shape.
// A workgroup that committed saw every arrival; the rest commit within a poll
// of the last arrival, well inside the second phase's longer limit, so either
// all workgroups pass or none does.  ctr is zeroed before every launch.
constexpr unsigned long long kArriveTicks = 10000000ull;  // 100 ms of s_memrealtime (100 MHz)
constexpr int kErrNotResident = 4;                        // err bit: the rendezvous failed
__device__ inline bool coresident(int* ctr, int n) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int ph = 0; ph < 2; ++ph) {
    atomicAdd(&ctr[ph], 1);
    while (__hip_atomic_load(&ctr[ph], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < n) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > (ph + 1) * kArriveTicks) return false;
      __builtin_amdgcn_s_sleep(2);
    }
  }
  return true;
}

__device__ inline unsigned long long stamp_now() { return __builtin_amdgcn_s_memtime(); }

// Wave-wide reduction of a 32-bit value with DPP (no LDS): butterflies inside
// each row of 16 lanes, then row_bcast:15 / row_bcast:31 carry the row results
// up to lane 63, whose value is returned (wave-uniform).  OP 0: max, 1: or;
// both have identity 0.
template <int OP>
__device__ inline unsigned wave_reduce_u32(unsigned v) {
  auto op = [](unsigned x, unsigned y) { return OP == 0 ? (x > y ? x : y) : (x | y); };
  v = op(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false));   // quad_perm [1,0,3,2]
  v = op(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false));   // quad_perm [2,3,0,1]
  v = op(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false));  // row_half_mirror
  v = op(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false));  // row_mirror
  v = op(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false));  // row_bcast:15 -> rows 1, 3
  v = op(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false));  // row_bcast:31 -> rows 2, 3
  return (unsigned)__builtin_amdgcn_readlane((int)v, 63);
}

// Backward rescale summary as a 32-bit code, monotone in |m|: 0 for m == 0,
// kCodeNonFinite for inf / NaN, else frexp exponent + kCodeBias.  The max of
// codes is the code of the max, and code_exponent(code(max)) ==
// rescale_exponent(max) (common.h), so tiles can combine codes instead of
// 64-bit maxima.
constexpr unsigned kCodeBias = 1100u, kCodeNonFinite = 0x1FFFu;
__device__ inline unsigned scale_code(double m) {
  if (!isfinite(m)) return kCodeNonFinite;  // inf or NaN (checked first: NaN > 0 is false)
  if (!(m > 0.0)) return 0u;
  int e;
  frexp(m, &e);
  return (unsigned)(e + (int)kCodeBias);
}
__device__ inline int code_exponent(unsigned c) {
  return (c == 0u || c == kCodeNonFinite) ? 0 : -((int)c - (int)kCodeBias);
}
__device__ inline unsigned long long wave_or_u64(unsigned long long v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v |= __shfl_xor(v, off, kWave);
  return v;
}

// cluster_run's result when a forward instance turned non-finite: the call must
// be rerun on the per-sweep shape (exact NaN bookkeeping; cluster.hip)
constexpr int kClusterNonFinite = 1;
// cluster_run's result when the launch's workgroups could not all run at once
// (coresident()): the call must be rerun on a shape without hand-offs
constexpr int kClusterNotResident = 2;

// compact: the backward's weights have the structure layout 4 needs
// (bwd_compact_ok_kernel); the planner then considers it at width 256
bool cluster_plan(int W, int H, int B, int mode, ClusterPlan* out, bool compact = false);
int cluster_run(int mode, const ClusterPlan& p, ClusterArgs a, int B, hipStream_t st);
__global__ void bwd_growth_kernel(const double* __restrict__ bw, int W, int S, int B,
                                  unsigned long long* __restrict__ growth);
__global__ void bwd_compact_ok_kernel(const double* __restrict__ row_val, int W, int H, int A, int* __restrict__ bad);

}  // namespace irlmx
