// Persistent, temporally blocked stencil sweeps for state spaces too large
// for one CU (e.g. 128x128 grids): forward SVF (maxent.py:63-114) and the
// non-causal backward pass (maxent.py:119-159).
//
// Decomposition.  An instance's width x height grid is cut into C row tiles of
// R rows.  Each tile is owned by one workgroup (one per CU, all co-resident),
// which keeps its tile plus G ghost rows on either side on chip (LDS and/or
// registers, by layout -- see cluster_kernel) and the per-state stencil
// weights of that extended tile in registers.  A block of T <= G sweeps runs
// entirely on chip: after sweep i the rows that are still exact shrink by one
// on each ghost side, so after T sweeps the owned rows are exact.  Then the
// tiles of an instance exchange halos.
//
// Exchange (cluster.h "Tagged granules").  Every tile stores the owned rows
// within G of its edges as {value, tag} granules (tag = call salt | block + 1)
// plus one granule with its 32-bit block summary; every thread then polls its
// ghost granules (and threads < C all tiles' summaries) with sc1 loads until
// the tags match.  The data is the flag: one round trip, no counter, no fence
// (cdna_hip_programming.md Guideline 16, R2).  Two parities of buffers: a tile
// cannot publish block m + 2 before every tile has read block m + 1's
// summaries, which each tile publishes only after reading block m.  Granules
// are written through (sc1) unless all C tiles are found on one XCD (plain
// stores then stay in that XCD's L2, where the sc1 loads are served).
//
// Convergence (forward).  Per sweep i of a block a tile records "some owned
// |delta| > eps" (bit i; a running fmax per lane) and, once per block, "some
// owned value is non-finite" (bit 31); the OR over tiles arrives with the
// exchange, so every tile takes the same decision: if the first sweep with
// !(delta > eps) lies inside the block, every tile reloads the block-start
// state (an LDS snapshot) and re-runs exactly that many sweeps -- the same
// arithmetic in the same order, so the result is the one the reference's loop
// stops at.  Bit 31 hands the call back to the host (exact NaN bookkeeping on
// the per-sweep shape, see the kernel).
//
// Rescaling (backward).  The partition vector grows geometrically.  A first
// pass bounds the per-sweep growth g of each instance; blocks are capped at
// T_eff sweeps so that g^T_eff stays below 2^900, and at every block boundary
// all tiles multiply their values by the same power of two derived from the
// instance-wide maximum: ratio-exact, like the single-workgroup kernel.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "cluster.h"
#include "common.h"

namespace irlmx {

void set_error(const char* fmt, ...);
int hip_fail(hipError_t e, const char* what);

// LDS buffer layout: [W + 1 zeros][E states][W + 1 zeros].  With the pads, the
// five stencil reads of state l are q[0], q[W-1], q[W], q[W+1], q[2W] for
// q = buf + l + 1: one address register per state and constant offsets (the
// pads are never written and stay 0; their stencil weight is 0 or the row they
// feed is a ghost row that is no longer exact).
//
// Per-sweep convergence bookkeeping (forward): the reference stops after the
// first sweep whose max|d_new - d_old| is not > eps, NaN included.  Threads
// collect "some |delta| > eps" per sweep (bit i) in a register, and the tile
// ORs the bits once per block (DPP wave reduction, one LDS atomic per wave) --
// no per-sweep reduction.  NaN: see the kernel's bookkeeping comment.
//
// PAIR (widths 64 and 128): thread slot jp holds the horizontally adjacent
// states 2p, 2p + 1 (p = tid + jp * NT) and keeps their values in registers
// between sweeps.  A wave then spans 64 consecutive pairs, so the horizontal
// neighbours of a pair are the neighbouring lanes' registers (DPP wave shifts;
// at a row edge the neighbour lane belongs to another row or is zero-filled,
// and the stencil weight there is 0), and each sweep reads only the pairs
// above and below (two ds_read_b128) and writes its own (one ds_write_b128):
// a third of the LDS traffic of the per-state form.
template <int CTRL>
__device__ inline double dpp_shift_f64(double x) {
  const long long b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffLL), CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, true);
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}

//
// COLS (LAY == 2; widths 64 / 128): the pair layout turned into column
// strips.  Lane cp of band bb (W / 2 lanes per band, NT / (W / 2) bands) holds
// the column pair 2 cp, 2 cp + 1 of the SPT / 2 consecutive rows of its band,
// all in registers.  Vertical neighbours are then the thread's own registers
// except at the band's top and bottom row, which go through a small
// double-buffered LDS boundary array -- per sweep one 16-byte write and one
// read at each band edge instead of three 16-byte accesses per pair.
//
// LAY == 3 is the same with four columns per lane (CPL = 4): half the DPP
// moves per state, and at width 256 one band row is one wave.
//
// LAY == 4 (backward, width 256): column quads with compact weights.  For the
// gridworld tables the collapsed coefficients sum_a P[s, n, a] of the +x and
// -x neighbours are equal wherever both are in the grid, the self coefficient
// is 0 off the grid border, and an off-grid neighbour's coefficient is 0
// (checked per call on the table: bwd_compact_ok_kernel).  A state then keeps
// three weights in registers -- w_x for both horizontal neighbours, w_+y, w_-y
// -- instead of five:
//   * an off-grid horizontal neighbour reads 0 (the DPP shift's zero fill at
//     lanes 0 and 63, where one band row is one wave), so fma(w_x, 0, acc) ==
//     acc == fma(0, garbage, acc) of the five-weight chain;
//   * the self term fma(w_0, v, 0) (+0 off the border): columns 0 and CPL - 1
//     take w_0 from two per-row registers that hold it only in lane 0 / HW - 1
//     (x = 0 / W - 1) and on the border rows y = 0 / H - 1, else 0; the middle
//     columns from one 16-byte LDS entry per row that is 0 except on a border
//     row.  No branch: the sweep stays one straight-line block (a per-row
//     branch measured 2.3x slower, the FMA chains of different rows no longer
//     interleaving).
// The FMA chain is the five-weight one, operand for operand, so the results
// are bit-identical, with three weight registers per state instead of five.
// The LDS band-edge array aliases the tile buffer, which the backward touches
// only between blocks.
template <int MODE, int SPT, int WT, int LAY, int NT>
__global__ void __launch_bounds__(NT) cluster_kernel(ClusterArgs a) {
  constexpr bool PAIR = LAY >= 1, COLS = LAY >= 2;
  constexpr bool CW = LAY == 4;                          // compact weights (see above)
  constexpr int CPL = LAY >= 3 ? 4 : 2;                  // COLS: columns per lane
  static_assert(LAY != 1 || (SPT % 2 == 0 && (WT == 64 || WT == 128)), "pair rows: even SPT, width 64/128");
  static_assert(LAY != 2 || (SPT % 2 == 0 && (WT == 64 || WT == 128)), "column pairs: even SPT, width 64/128");
  static_assert(LAY != 3 || (SPT % 4 == 0 && (WT == 128 || WT == 256)), "column quads: SPT % 4, width 128/256");
  static_assert(LAY != 4 || (MODE == kModeBwd && SPT % 4 == 0 && WT == 256), "compact weights: backward, width 256");
  constexpr int RW = COLS ? SPT / CPL : 1;               // COLS: rows per band
  constexpr int HW = COLS ? WT / CPL : 1;                // COLS: lanes per band
  constexpr int NB = COLS ? NT / HW : 1;                 // COLS: bands
  constexpr int QW = CPL / 2;                            // COLS: double2 per lane per row
#ifndef IRLMX_FWD_PROOF
#define IRLMX_FWD_PROOF 1
#endif
  // Forward, column layouts: per-sweep bookkeeping on band row kProofRow only
  // (the cheap proof of "not converged"; the block loop replays a block with
  // full bookkeeping when some sweep is left unproven).  IRLMX_FWD_PROOF=0: full
  // bookkeeping every sweep, as before round 6.
  constexpr bool kProof = MODE == kModeFwd && COLS && IRLMX_FWD_PROOF;
  constexpr int kProofRow = RW / 2;
#ifndef IRLMX_LDS_SIDES
#define IRLMX_LDS_SIDES -1
#endif
  // COLS pairs: band edge rows' side neighbours from LDS (for quads, where 2 of
  // 3 rows are edge rows, the exposed LDS latency costs more than the DPP moves).
  // Forward only since round 5's backward schedule (store fence, unpinned
  // barrier): DPP moves there are faster -- config 3's backward 22.09 / 22.13 ->
  // 21.99 / 21.99 ms, config 2's 2.57 -> 2.40 ms -- while the forward keeps the
  // LDS reads (one 128x128 instance 13.42 -> 13.82 ms per 20,000 sweeps with DPP;
  // profiles/r05_ab_c3_sched.txt).  IRLMX_LDS_SIDES: -1 that rule, 0 never, 1 always.
  constexpr bool kLdsSides = COLS && CPL == 2 && (IRLMX_LDS_SIDES < 0 ? MODE == kModeFwd : IRLMX_LDS_SIDES != 0);
#ifndef IRLMX_COLS_RELOAD
#define IRLMX_COLS_RELOAD 0
#endif
  // COLS: register state through the LDS tile at every block boundary (see the publish step)
  constexpr bool kReload = COLS && IRLMX_COLS_RELOAD;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int W = WT ? WT : a.W;
  const int H = a.H, S = a.S;
  // XCD-grouped numbering (a.xcd_group): workgroups are dealt round-robin over
  // the 8 XCDs, so blockIdx % 8 names an XCD group; all C tiles of an instance
  // are taken from one group (instance g + 8 j of group g), which lets their
  // halo hand-offs stay inside one L2 when the dealing is as observed (checked
  // at run time below; speed only).  The grid is padded to 8 equal groups; the
  // padding workgroups leave at once.
  int lin = blockIdx.x;  // = local instance * C + tile
  if (a.xcd_group) {
    const int g = blockIdx.x % 8, k = blockIdx.x / 8;
    const int il = g + 8 * (k / a.C);
    if (il >= a.nb) return;
    lin = il * a.C + k % a.C;
  }
  const int tile = lin % a.C;
  const int inst = a.b0 + lin / a.C;
  const int tid = threadIdx.x;
  {  // every workgroup of the launch running at once, or none goes on (coresident())
    __shared__ int resident;
    if (tid == 0) resident = coresident(a.err + 1, a.n_resident) ? 1 : 0;
    __syncthreads();
    if (!resident) {
      if (tid == 0) atomicOr(a.err, kErrNotResident);
      return;
    }
  }
  if (lin == a.test_drop) return;  // tests: a workgroup that stops publishing (exchange-timeout path)
  const int r0 = tile * a.R, r1 = min(H, r0 + a.R);
  const int e0 = max(0, r0 - a.G), e1 = min(H, r1 + a.G);
  const int E = (e1 - e0) * W;
  // device checks: the tile's rows inside the grid, its extended tile inside the
  // LDS buffer and the register slots (a failing workgroup leaves; its
  // neighbours' exchange then times out and the host reruns per sweep)
  if (!IRLMX_DCHECK(0 <= e0 && e0 <= r0 && r0 < r1 && r1 <= e1 && e1 <= H && E <= a.emax && E <= SPT * NT,
                    kCheckTile))
    return;
  const int own0 = (r0 - e0) * W, own1 = (r1 - e0) * W;
  // owned rows other tiles read as ghosts: within G rows of either tile edge
  const int pubA1 = min(own1, own0 + a.G * W), pubB0 = max(pubA1, own1 - a.G * W);
  const int base = e0 * W;
  const int pad = PAIR ? W : W + 1;  // pair layout keeps every pair 16-byte aligned
  const int blen = a.emax + 2 * pad;
  const int cp = COLS ? tid % HW : 0, bb = COLS ? tid / HW : 0;  // COLS: column group, band
  // state index of register slot j
  auto slot_state = [&](int j) {
    if (COLS) return (bb * RW + j / CPL) * W + CPL * cp + j % CPL;
    return PAIR ? 2 * (tid + (j >> 1) * NT) + (j & 1) : tid + j * NT;
  };
  double* bufA = (double*)smem;
  // COLS keeps a single tile buffer (ghost staging, the backward's final sweep)
  double* bufB = bufA + (COLS ? 0 : blen);
  double* snap = bufB + blen;                                            // forward: block-start state
  // COLS: band edge rows [2 parities][NB + 2 (zero band at both ends)][2: top, bottom][HW][QW] double2;
  // CW: aliasing the tile buffer (used only inside a block's sweeps; the tile
  // buffer only between blocks), the zero bands replaced by one zero row zrow
  constexpr int kBndLen = COLS ? 2 * (NB + 2) * 2 * HW * QW : 0;
  double2* bnd = CW ? (double2*)bufA : (double2*)(snap + (MODE == kModeFwd ? a.emax : 0));
  unsigned char* tail = CW ? (unsigned char*)bufA + max((size_t)blen * sizeof(double), (size_t)kBndLen * sizeof(double2))
                           : (unsigned char*)(bnd + kBndLen);
  double2* wmid = (double2*)tail;                                        // CW: [NB][RW][HW] middle columns' w_0 per band row (0 off rows 0 / H - 1)
  double2* zrow = wmid + (CW ? NB * RW * HW : 0);                        // CW: [HW][QW] zeros
  unsigned long long* red = (unsigned long long*)(zrow + (CW ? HW * QW : 0));  // [3]
  int* lflag = (int*)(red + 3);                                          // [4]

  const size_t iS = (size_t)inst * S;
  if (MODE == kModeFwd && a.bad[inst]) {
    // non-finite policy: the reference's dense product is NaN after one sweep
    for (int l = own0 + tid; l < own1; l += NT) a.out[iS + base + l] = __longlong_as_double(0x7ff8000000000000LL);
    if (tile == 0 && tid == 0) { a.iters[inst] = 1; a.status[inst] = IRLMX_NONFINITE; }
    return;
  }

  // ---- per-state constants into registers --------------------------------
  double w[CW ? 1 : SPT][kStencilK];  // forward: gather weights; backward: reward-folded weights
  double wc[CW ? SPT : 1][3];         // CW: w_x (both horizontal neighbours), w_+y, w_-y
  double edge_w[CW ? 2 * RW : 1];     // CW: per band row, w_0 of columns 0 / CPL-1 (x-border lanes, border rows; else 0)
  double c0[MODE == kModeFwd ? SPT : 1];  // forward: p0
  const size_t wbase = iS * kStencilK;
#pragma unroll
  for (int j = 0; j < SPT; ++j) {
    const int l = slot_state(j);
    if (MODE == kModeFwd) c0[MODE == kModeFwd ? j : 0] = 0.0;
    if constexpr (CW) {
#pragma unroll
      for (int k = 0; k < 3; ++k) wc[j][k] = 0.0;
      if (l < E) {
        const int s = base + l;
        const int x = s % W;
        wc[j][0] = a.wgt[wbase + (size_t)(x + 1 < W ? 1 : 2) * S + s];
        wc[j][1] = a.wgt[wbase + (size_t)3 * S + s];
        wc[j][2] = a.wgt[wbase + (size_t)4 * S + s];
      }
#pragma unroll
      for (int k = 0; k < 3; ++k) asm volatile("" : "+v"(wc[j][k]));
    } else {
#pragma unroll
      for (int k = 0; k < kStencilK; ++k) w[j][k] = 0.0;
      if (l < E) {
        const int s = base + l;
        if (MODE == kModeFwd) c0[MODE == kModeFwd ? j : 0] = a.vin[iS + s];
#pragma unroll
        for (int k = 0; k < kStencilK; ++k) w[j][k] = a.wgt[wbase + (size_t)k * S + s];
      }
      // pin the constants in registers: without this the compiler re-loads them
      // from global memory inside every sweep (rematerialisation of invariant loads)
#pragma unroll
      for (int k = 0; k < kStencilK; ++k) asm volatile("" : "+v"(w[j][k]));
      if (MODE == kModeFwd) asm volatile("" : "+v"(c0[MODE == kModeFwd ? j : 0]));
    }
  }
  if constexpr (CW) {
#pragma unroll
    for (int r = 0; r < RW; ++r) {
      edge_w[2 * r] = 0.0;
      edge_w[2 * r + 1] = 0.0;
      const int l0 = slot_state(r * CPL), l3 = slot_state(r * CPL + CPL - 1);
      const int y = e0 + l0 / W;
      const bool brow = l0 < E && (y == 0 || y == H - 1);
      if ((cp == 0 || brow) && l0 < E) edge_w[2 * r] = a.wgt[wbase + base + l0];
      if ((cp == HW - 1 || brow) && l3 < E) edge_w[2 * r + 1] = a.wgt[wbase + base + l3];
      asm volatile("" : "+v"(edge_w[2 * r]));
      asm volatile("" : "+v"(edge_w[2 * r + 1]));
    }
  }
  // one sweep's new value from the weighted sum: forward p0 + sum, backward the sum
  auto finish = [&](int j, double acc) { return MODE == kModeFwd ? c0[MODE == kModeFwd ? j : 0] + acc : acc; };
  // forward: does any slot of this wave hold a nonzero p0 (NaN counts)?  Wave-uniform (SGPR).
  bool wave_p0 = true;
  if constexpr (MODE == kModeFwd) {
    bool mine = false;
#pragma unroll
    for (int j = 0; j < SPT; ++j) mine |= !(c0[MODE == kModeFwd ? j : 0] == 0.0);
#ifndef IRLMX_FWD_P0_SKIP
#define IRLMX_FWD_P0_SKIP 1
#endif
    wave_p0 = !IRLMX_FWD_P0_SKIP || __builtin_amdgcn_readfirstlane(__builtin_amdgcn_ballot_w64(mine) != 0ull ? 1 : 0) != 0;
  }
  for (int i = tid; i < (COLS ? 1 : 2) * blen; i += NT) bufA[i] = 0.0;
  for (int i = tid; i < kBndLen; i += NT) bnd[i] = make_double2(0.0, 0.0);
  if constexpr (CW) {
    static_assert(!CW || CPL == 4, "compact weights: column quads");
    for (int i = tid; i < HW * QW; i += NT) zrow[i] = make_double2(0.0, 0.0);
#pragma unroll
    for (int r = 0; r < RW; ++r) {  // w_0 of columns 1, 2 of this lane's band row r: nonzero on rows 0 / H - 1 only
      const int l1 = slot_state(r * CPL + 1);
      const int y = e0 + l1 / W;
      const bool brow = l1 < E && (y == 0 || y == H - 1);
      wmid[(bb * RW + r) * HW + cp] = brow ? make_double2(a.wgt[wbase + base + l1], a.wgt[wbase + base + l1 + 1])
                                           : make_double2(0.0, 0.0);
    }
  }
  __syncthreads();
  for (int l = tid; l < E; l += NT) {
    double v0 = 0.0;
    if (MODE == kModeBwd) v0 = a.term[iS + base + l] ? 1.0 : 0.0;
    bufA[pad + l] = v0;
    bufB[pad + l] = v0;
    if (MODE == kModeFwd) snap[l] = v0;
  }
  if (tid < 3) red[tid] = 0ull;
  if (tid == 0) lflag[0] = 0;
  double cv[PAIR ? SPT : 1];  // pair layout: this thread's states, kept across sweeps
#pragma unroll
  for (int j = 0; j < (PAIR ? SPT : 1); ++j) {
    const int l = slot_state(j);
    cv[j] = (PAIR && MODE == kModeBwd && l < E) ? (a.term[iS + base + l] ? 1.0 : 0.0) : 0.0;
  }
  // reload the register copy from an LDS buffer (after a ghost refresh or a rollback)
  auto reload = [&](const double* buf) {
    if (PAIR) {
#pragma unroll
      for (int j = 0; j < (PAIR ? SPT : 1); ++j) cv[j] = buf[pad + slot_state(j)];
    }
  };

  // per-slot predicates as bit masks (bit j: register slot j)
  unsigned own_bits = 0, pub_bits = 0, ext_bits = 0;
#pragma unroll
  for (int j = 0; j < SPT; ++j) {
    const int l = slot_state(j);
    const bool own = l >= own0 && l < own1;
    own_bits |= (own ? 1u : 0u) << j;
    ext_bits |= (l < E ? 1u : 0u) << j;
    pub_bits |= (((l >= own0 && l < pubA1) || (l >= pubB0 && l < own1)) ? 1u : 0u) << j;
  }

  // Opaque per use, so the compiler does not hoist per-slot SGPR masks out of
  // the loops (SGPR pressure).  When a wave covers exactly one row per slot
  // (pair rows at width 128; column strips with 64 lanes per band row) the
  // predicates are wave-uniform: kept in an SGPR they turn into scalar
  // branches instead of per-lane selects.
  constexpr bool kUniformSlots = LAY == 1 ? WT == 128 : (COLS && HW == 64);
  auto slot_bits = [&](unsigned b) {
    if constexpr (kUniformSlots) {
      b = (unsigned)__builtin_amdgcn_readfirstlane((int)b);
      asm volatile("" : "+s"(b));
    } else {
      asm volatile("" : "+v"(b));
    }
    return b;
  };

  int T = a.T;
  // Backward rescaling period: blocks between rescales (see the block loop).
  // Between two rescales the partition vector neither grows nor shrinks by more
  // than 2^900: its maximum grows at most by g = max_s sum_k w_k(s) per sweep
  // and shrinks at most by d = the smallest positive weight (when every state is
  // some state's stencil operand with a positive weight -- checked by
  // bwd_growth_kernel -- the state holding the maximum feeds at least d times it
  // into the next sweep; otherwise short blocks, rescaled every block).  The
  // sweeps between rescales, T * p_max, are capped at 900 / log2 of either rate
  // -- which shortens the solo backward's 256-sweep blocks (kSoloBwdT) where
  // the rewards are very negative (decay) or the growth is near 2 per sweep.
  int p_max = 1;
  if (MODE == kModeBwd) {
    const double g = bits_double(a.growth[inst]);
    const double d = bits_double(a.growth[a.btot + inst]);
    if (a.rescale && isfinite(g)) {
      int cap = 1 << 20;
      if (g > 1.0) cap = max(1, (int)floor(900.0 / log2(g)) - 1);
      if (d > 0.0 && d < 1.0) cap = min(cap, max(1, (int)floor(900.0 / -log2(d)) - 1));
      // no decay bound (a state feeds nobody, bwd_growth_kernel): blocks of at
      // most kTMax sweeps, rescaled every block (the round-3 cadence)
      if (d < 0.0) cap = min(cap, kTMax);
      T = max(1, min(T, cap));
      p_max = d < 0.0 ? 1 : max(1, min(kRescaleEvery, cap / T));
    }
  }
  __syncthreads();

  const double eps = a.eps;
  // Forward convergence bookkeeping per sweep i of a block: bit i of `flags`
  // = "the running fmax of this lane's owned |delta| exceeds eps" (two VALU
  // instructions per state).  The reference stops at the first sweep whose
  // np.max(|delta|) is not > eps, NaN included; fmax drops NaN, so the bits
  // are exact unless some |delta| is NaN.  A non-finite value is sticky (every
  // sweep multiplies a state's own value by its self weight, and 0 * inf =
  // NaN), so a non-finite owned value at the block's end (bit 31, checked once
  // per block) covers that case: the instance is then handed back to the host,
  // which reruns the call on the per-sweep shape with exact NaN bookkeeping
  // (bit-identical arithmetic; fixed_point.hip irlmx_forward_svf).
  // One Jacobi sweep over the extended tile.  (Backward: the owned maximum for
  // the block-end rescale is taken once after the block's last sweep.)
  // Every slot l < SPT * NT is swept, also l >= E: those have zero weights and
  // zero c0, read only zeros (buffers are zero-filled and hold emax + 2 pads),
  // and stay 0 -- which is what state E - 1's down-neighbour must read.  No
  // per-state branch, so all LDS reads of a sweep can be in flight together.
  auto sweep = [&](const double* __restrict__ din, double* __restrict__ dout, int i, unsigned& flags) {
    const unsigned ob = slot_bits(own_bits);
    double dmax = 0.0;
    auto account = [&](int j, double nv, double self) {
      if (MODE == kModeFwd && ((ob >> j) & 1u)) dmax = fmax(dmax, fabs(nv - self));
    };
    if constexpr (PAIR && !COLS) {
#pragma unroll
      for (int jp = 0; jp < SPT / 2; ++jp) {
        const int l = 2 * (tid + jp * NT);
        const double2 up = *reinterpret_cast<const double2*>(din + l);           // row above (pad = W)
        const double2 dn = *reinterpret_cast<const double2*>(din + 2 * W + l);   // row below
        const double va = cv[2 * jp], vb = cv[2 * jp + 1];
        const double lft = dpp_shift_f64<0x138>(vb);  // wave_shr1: left neighbour of state a
        const double rgt = dpp_shift_f64<0x130>(va);  // wave_shl1: right neighbour of state b
        const double* wa = w[CW ? 0 : 2 * jp];
        const double* wb = w[CW ? 0 : 2 * jp + 1];
        double acc = fma(wa[0], va, 0.0);
        acc = fma(wa[1], vb, acc);
        acc = fma(wa[2], lft, acc);
        acc = fma(wa[3], dn.x, acc);
        acc = fma(wa[4], up.x, acc);
        const double na = finish(2 * jp, acc);
        acc = fma(wb[0], vb, 0.0);
        acc = fma(wb[1], rgt, acc);
        acc = fma(wb[2], va, acc);
        acc = fma(wb[3], dn.y, acc);
        acc = fma(wb[4], up.y, acc);
        const double nb = finish(2 * jp + 1, acc);
        *reinterpret_cast<double2*>(dout + W + l) = make_double2(na, nb);
        account(2 * jp, na, va);
        account(2 * jp + 1, nb, vb);
        cv[2 * jp] = na;
        cv[2 * jp + 1] = nb;
      }
    } else {
#pragma unroll
      for (int j = 0; j < SPT; ++j) {
        const int l = tid + j * NT;
        const double* q = din + l + 1;
        const double self = q[W];
        double acc = fma(w[CW ? 0 : j][0], self, 0.0);
        acc = fma(w[CW ? 0 : j][1], q[W + 1], acc);
        acc = fma(w[CW ? 0 : j][2], q[W - 1], acc);
        acc = fma(w[CW ? 0 : j][3], q[2 * W], acc);
        acc = fma(w[CW ? 0 : j][4], q[0], acc);
        const double nv = finish(j, acc);
        dout[pad + l] = nv;
        account(j, nv, self);
      }
    }
    if (MODE == kModeFwd) flags |= ((dmax > eps) ? 1u : 0u) << i;
    __syncthreads();
  };

  // COLS sweep between two register arrays (src -> dst): no register copies for
  // the old values the neighbouring rows still need; callers alternate the
  // arrays, two sweeps per loop iteration.
  double cw[COLS ? SPT : 1];
  // band edge row e (0: top, 1: bottom) of band slot `band` (0 and NB + 1 are
  // the zero bands) in parity buffer `par`
  auto bnd_at = [&](int par, int band, int e) { return bnd + ((((size_t)par * (NB + 2) + band) * 2 + e) * HW + cp) * QW; };
  // kSplitEdges (column pairs): the same storage per edge row as two arrays of
  // HW doubles (column 0, column 1), so that the side reads -- the neighbour
  // lanes' last / first column -- are 8-byte strided (no bank conflicts; the
  // double2 form reads them at a 16-byte stride)
#ifndef IRLMX_SPLIT_EDGES
#define IRLMX_SPLIT_EDGES 0
#endif
  constexpr bool kSplitEdges = kLdsSides && IRLMX_SPLIT_EDGES;
  auto edge_row = [&](int par, int band, int e) {
    return reinterpret_cast<double*>(bnd + (((size_t)par * (NB + 2) + band) * 2 + e) * HW * QW);
  };
  // p0tag (std::integral_constant<bool, P0>): with P0 false the forward's "p0 +"
  // is left out -- exact where every p0 of the wave's slots is +-0: the FMA
  // chain starts from fma(w, v, +0.0), which is never -0.0, so 0.0 + acc == acc
  // bit for bit (NaN and inf included).
  //
  // fulltag (std::integral_constant<bool, FULL>): the forward's owned-delta
  // bookkeeping on every owned slot (FULL) or only on the slots of band row
  // kProofRow, the cheap proof of "not converged" (see the block loop).
  auto cols_sweep = [&](const double (&src)[COLS ? SPT : 1], double (&dst)[COLS ? SPT : 1], int i,
                        unsigned& flags, auto p0tag, auto fulltag) {
    constexpr bool kP0 = decltype(p0tag)::value;
    constexpr bool kFull = decltype(fulltag)::value;
    if constexpr (COLS) {
      const unsigned ob = slot_bits(own_bits);
      double dmax = 0.0;
#ifndef IRLMX_CW_PREFETCH
#define IRLMX_CW_PREFETCH 1
#endif
      // CW: the middle columns' self weights of every row, read at the top of
      // the sweep (constant LDS data: ahead of the edge-row stores and the
      // barrier) so that no row's FMA chain starts by waiting for its read
      double2 wm_pf[CW && IRLMX_CW_PREFETCH ? RW : 1];
      if constexpr (CW && IRLMX_CW_PREFETCH) {
#pragma unroll
        for (int r = 0; r < RW; ++r) wm_pf[r] = wmid[(bb * RW + r) * HW + cp];
      }
#ifndef IRLMX_FWD_BRANCH_ACCOUNT
#define IRLMX_FWD_BRANCH_ACCOUNT 1
#endif
#ifndef IRLMX_FWD_BRANCH_SPT_MAX
#define IRLMX_FWD_BRANCH_SPT_MAX 12
#endif
      // With wave-uniform slot predicates (IRLMX_FWD_BRANCH_ACCOUNT): a scalar
      // branch per slot around the owned-delta update instead of computing it
      // for every slot and selecting -- the empty asm keeps the compiler from
      // speculating the body back into selects.  One 128² instance's forward
      // 0.736 -> 0.713 us per sweep, config 5 forward 127.0 -> 122.4 ms, same
      // sweep counts.  Round 5: at 12 states per lane too (config 3's and the
      // batched causal forward; two VGPRs spill, outside the sweep loop): B = 64
      // at 128x128, 3,000 sweeps 3.19 -> 3.01 ms, three alternations on one box.
#ifndef IRLMX_FWD_BALLOT_ACCOUNT
#define IRLMX_FWD_BALLOT_ACCOUNT 0
#endif
#ifndef IRLMX_FWD_NO_ACCOUNT
#define IRLMX_FWD_NO_ACCOUNT 0   // timing experiments only: every sweep counts as not converged
#endif
      // IRLMX_FWD_BALLOT_ACCOUNT=1 (round 6, measured slower): no branch and no
      // select -- per slot one f64 subtract and one compare whose lane mask (a
      // ballot, SGPRs) is ANDed with the slot's ownership and ORed into a
      // wave-uniform mask, the sweep one straight-line block.  The same bit as
      // the fmax form's (NaN > eps is false, as fmax drops NaN), but each
      // compare-to-SGPR feeds a scalar OR: config 3's plan 11.4k -> 14.4k cycles
      // of sweeps per 8-sweep block, one 128x128 instance 6.9k -> 9.1k.
      constexpr bool kBallotAccount = MODE == kModeFwd && IRLMX_FWD_BALLOT_ACCOUNT;
      unsigned long long anyv = 0ull;
      auto account = [&](int j, double nv, double self) {
        if (!kFull && j / CPL != kProofRow) return;   // (compile-time after unrolling)
        if constexpr (MODE == kModeFwd && IRLMX_FWD_NO_ACCOUNT) {
          (void)j; (void)nv; (void)self;
        } else if constexpr (kBallotAccount) {
          bool big = ((ob >> j) & 1u) != 0u;
          big = big & (fabs(nv - self) > eps);
          anyv |= __builtin_amdgcn_ballot_w64(big);
        } else if constexpr (MODE == kModeFwd && kUniformSlots && SPT <= IRLMX_FWD_BRANCH_SPT_MAX && IRLMX_FWD_BRANCH_ACCOUNT) {
          if ((ob >> j) & 1u) {
            asm volatile("");
            dmax = fmax(dmax, fabs(nv - self));
          }
        } else if (MODE == kModeFwd && ((ob >> j) & 1u)) {
          dmax = fmax(dmax, fabs(nv - self));
        }
      };
      if constexpr (kSplitEdges) {  // band edge rows (old values) out: column 0 / column 1 arrays
        double* t = edge_row(i & 1, bb + 1, 0);
        double* u = edge_row(i & 1, bb + 1, 1);
        t[cp] = src[0]; t[HW + cp] = src[1];
        u[cp] = src[SPT - 2]; u[HW + cp] = src[SPT - 1];
      } else {  // band edge rows (old values) out
        double2* t = bnd_at(i & 1, bb + 1, 0);
        double2* u = bnd_at(i & 1, bb + 1, 1);
#pragma unroll
        for (int q = 0; q < QW; ++q) {
          t[q] = make_double2(src[2 * q], src[2 * q + 1]);
          u[q] = make_double2(src[SPT - CPL + 2 * q], src[SPT - CPL + 2 * q + 1]);
        }
      }
#ifndef IRLMX_PIN_STORES
#define IRLMX_PIN_STORES -1
#endif
      // Column pairs: issue the band-edge stores before the first interior rows'
      // FMAs, which then cover the stores' completion ahead of the barrier (the
      // scheduler otherwise sinks the stores below most of those FMAs).  Faster
      // for the backward at up to 8 states per lane -- config 2's solo backward
      // 2.81 -> 2.56 ms, one 128x128 instance 17.16 -> 16.70 ms -- slower at 12
      // (config 3: 22.51 -> 23.6 ms), neutral for the forward
      // (profiles/r05_ab_pin_stores.txt).  IRLMX_PIN_STORES: -1 that rule, 0 never, 1 always.
      // Config 3's backward (column pairs, 12 states per lane) is fastest with
      // the store fence, both interior steps before the barrier and the barrier
      // unpinned: 22.57 / 22.64 -> 22.24 / 22.23 ms (two alternations; at 8
      // states per lane the same set is slower, config 2 2.57 -> 2.67 ms;
      // profiles/r05_ab_c3_sched.txt)
      constexpr bool kBwdPairs12 = CPL == 2 && MODE == kModeBwd && SPT >= 12;
      constexpr bool kPinStores =
          IRLMX_PIN_STORES < 0 ? (CPL == 2 && MODE == kModeBwd && (SPT <= 8 || kBwdPairs12)) : IRLMX_PIN_STORES != 0;
      if constexpr (kPinStores) __builtin_amdgcn_sched_barrier(0);
      if (MODE == kModeFwd && i == 0) {
        // forward: the block-start state into the LDS snapshot (for a stop inside
        // the block), here rather than at the block boundary so that the stores
        // overlap the first sweep's arithmetic
        const unsigned xb = slot_bits(ext_bits);
#pragma unroll
        for (int jp = 0; jp < SPT / 2; ++jp)
          if ((xb >> (2 * jp)) & 1u)
            *reinterpret_cast<double2*>(snap + slot_state(2 * jp)) = make_double2(src[2 * jp], src[2 * jp + 1]);
      }
      double above[CPL], below[CPL];  // bottom row of the band above, top row of the band below
      // The band's own top / bottom rows are in the edge array too, so their
      // horizontal neighbours (the last column of lane cp - 1, the first of lane
      // cp + 1) can be LDS reads instead of DPP moves: 8 fewer VALU instructions
      // per sweep at 6 rows per band (config 3 backward 24.69 -> 24.40 ms).  A band row spans the full width, so lane 0 is
      // x = 0 and lane HW - 1 is x = W - 1, whose out-of-row neighbour (weight 0)
      // reads an adjacent, finite array entry.
      double side[2][2];  // [top, bottom][left, right]
      // (which: 1 = the row above, 2 = the row below, 3 = both; sync: the barrier first)
#ifndef IRLMX_PIN_BARRIER
#define IRLMX_PIN_BARRIER -1
#endif
      // Column pairs: keep the instruction scheduler from moving the interior
      // rows' FMAs across the barrier (it hoisted the barrier to the top of the
      // loop body; config 3 backward 24.4 -> 23.0 ms on one box).  Column
      // quads are faster unpinned (267.6 vs 273.6 ms at config 4).
      // (IRLMX_PIN_BARRIER: -1 pairs only, 0 never, 1 always.)
      constexpr bool kPin = IRLMX_PIN_BARRIER < 0 ? (CPL == 2 && !kBwdPairs12) : IRLMX_PIN_BARRIER != 0;
      auto edges_in = [&](int which = 3, bool sync = true) {
        if (kPin && sync) __builtin_amdgcn_sched_barrier(0);
        if (sync) __syncthreads();
        if (kPin && sync) __builtin_amdgcn_sched_barrier(0);
        if constexpr (kSplitEdges) {
          const double* t = edge_row(i & 1, bb, 1);
          const double* u = edge_row(i & 1, bb + 2, 0);
          if (which & 1) { above[0] = t[cp]; above[1] = t[HW + cp]; }
          if (which & 2) { below[0] = u[cp]; below[1] = u[HW + cp]; }
#pragma unroll
          for (int e = 0; e < 2; ++e) {  // left: column 1 of lane cp - 1; right: column 0 of lane cp + 1
            const double* o = edge_row(i & 1, bb + 1, e);
            side[e][0] = o[HW + cp - 1];
            side[e][1] = o[cp + 1];
          }
          return;
        }
        const double2* t = (CW && bb == 0) ? zrow + cp * QW : bnd_at(i & 1, bb, 1);
        const double2* u = (CW && bb == NB - 1) ? zrow + cp * QW : bnd_at(i & 1, bb + 2, 0);
#pragma unroll
        for (int q = 0; q < QW; ++q) {
          if (which & 1) {
            const double2 x = t[q];
            above[2 * q] = x.x; above[2 * q + 1] = x.y;
          }
          if (which & 2) {
            const double2 y = u[q];
            below[2 * q] = y.x; below[2 * q + 1] = y.y;
          }
        }
        if constexpr (kLdsSides) {
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const double* o = reinterpret_cast<const double*>(bnd_at(i & 1, bb + 1, e));
            side[e][0] = o[-1];
            side[e][1] = o[CPL];
          }
        }
      };
      // rows j1 and j2 (j2 == j1: one row) at once: up to 2 * CPL independent FMA chains
      auto rows = [&](int j1, int j2) {
        const bool two = j2 != j1;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          if (h == 1 && !two) break;
          const int jr = h == 0 ? j1 : j2;
          const double* v = src + jr * CPL;
          const double* up = jr == 0 ? above : src + (jr > 0 ? jr - 1 : 0) * CPL;
          const double* dn = jr == RW - 1 ? below : src + (jr + 1 < RW ? jr + 1 : RW - 1) * CPL;
          const bool edge_row = kLdsSides && (jr == 0 || jr == RW - 1);
          const int er = jr == 0 ? 0 : 1;
          const double lft = edge_row ? side[er][0] : dpp_shift_f64<0x138>(v[CPL - 1]);  // wave_shr1: left of column 0
          const double rgt = edge_row ? side[er][1] : dpp_shift_f64<0x130>(v[0]);        // wave_shl1: right of column CPL - 1
          double acc[CPL];
          if constexpr (CW) {
            // the five-weight chain with w_1 = w_2 = w_x and the self term as
            // described at the top of the kernel
            const double2 wm = IRLMX_CW_PREFETCH ? wm_pf[IRLMX_CW_PREFETCH ? jr : 0] : wmid[(bb * RW + jr) * HW + cp];
            acc[0] = fma(edge_w[2 * jr], v[0], 0.0);
            acc[1] = fma(wm.x, v[1], 0.0);
            acc[2] = fma(wm.y, v[2], 0.0);
            acc[CPL - 1] = fma(edge_w[2 * jr + 1], v[CPL - 1], 0.0);
#pragma unroll
            for (int c = 0; c < CPL; ++c) acc[c] = fma(wc[jr * CPL + c][0], c + 1 < CPL ? v[c + 1 < CPL ? c + 1 : 0] : rgt, acc[c]);
#pragma unroll
            for (int c = 0; c < CPL; ++c) acc[c] = fma(wc[jr * CPL + c][0], c > 0 ? v[c > 0 ? c - 1 : 0] : lft, acc[c]);
#pragma unroll
            for (int c = 0; c < CPL; ++c) acc[c] = fma(wc[jr * CPL + c][1], dn[c], acc[c]);
#pragma unroll
            for (int c = 0; c < CPL; ++c) acc[c] = fma(wc[jr * CPL + c][2], up[c], acc[c]);
          } else {
#pragma unroll
            for (int c = 0; c < CPL; ++c) acc[c] = fma(w[CW ? 0 : jr * CPL + c][0], v[c], 0.0);
#pragma unroll
            for (int c = 0; c < CPL; ++c) acc[c] = fma(w[CW ? 0 : jr * CPL + c][1], c + 1 < CPL ? v[c + 1 < CPL ? c + 1 : 0] : rgt, acc[c]);
#pragma unroll
            for (int c = 0; c < CPL; ++c) acc[c] = fma(w[CW ? 0 : jr * CPL + c][2], c > 0 ? v[c > 0 ? c - 1 : 0] : lft, acc[c]);
#pragma unroll
            for (int c = 0; c < CPL; ++c) acc[c] = fma(w[CW ? 0 : jr * CPL + c][3], dn[c], acc[c]);
#pragma unroll
            for (int c = 0; c < CPL; ++c) acc[c] = fma(w[CW ? 0 : jr * CPL + c][4], up[c], acc[c]);
          }
#pragma unroll
          for (int c = 0; c < CPL; ++c) {
            dst[jr * CPL + c] = kP0 ? finish(jr * CPL + c, acc[c]) : acc[c];
            account(jr * CPL + c, dst[jr * CPL + c], v[c]);
          }
        }
      };
      // interior rows first (all their operands are registers), the band's
      // bottom and top rows last; with two columns per lane, two rows at a
      // time.  The first kPre interior steps run between the edge-row stores
      // and the barrier (they hide the stores' completion and the other waves'
      // arrival), the rest while the edge reads after the barrier are in flight.
      constexpr int step = CPL == 2 ? 2 : 1;
      constexpr int n_int = RW >= 3 ? (RW - 2 + step - 1) / step : 0;
#ifndef IRLMX_KPRE
#define IRLMX_KPRE -1
#endif
      // (IRLMX_KPRE >= 0: experiments, interior steps before the barrier.)  The
      // compact-weight quads run all their interior rows before the barrier:
      // config 4's backward 193.3 / 189.8 -> 186.5 / 183.8 ms (two alternations;
      // config 3's column pairs are slower that way, 22.50 -> 22.54-22.64 ms,
      // profiles/r05_ab_c4_sched.txt)
      // (config 3's backward: both interior steps, see kBwdPairs12; the
      // forward in column pairs at <= 8 states per lane -- config 5's one
      // instance, 6 per lane -- none: 14.25 / 14.30 -> 13.59 / 13.56 ms per
      // 20,000 sweeps, but config 3's forward at 12 is slower that way)
      constexpr int kPre = IRLMX_KPRE >= 0 ? (IRLMX_KPRE < n_int ? IRLMX_KPRE : n_int)
                           : (CW || kBwdPairs12) ? n_int
                           : (CPL == 2 && MODE == kModeFwd && SPT <= 8) ? 0
                                                                       : (n_int + 1) / 2;
      // IRLMX_QUAD_LAZY_ABOVE (quads): the row below is read at the barrier, the
      // row above only before the band's top row, so the two edge rows are never
      // live together (four doubles less register pressure; the hot loop has no
      // scratch either way -- DESIGN.md section 4 "Registers").
#ifndef IRLMX_QUAD_LAZY_ABOVE
#define IRLMX_QUAD_LAZY_ABOVE 0
#endif
      constexpr bool kLazy = CPL == 4 && IRLMX_QUAD_LAZY_ABOVE;
      constexpr int kFirst = kLazy ? 2 : 3;
#pragma unroll
      for (int s = 0; s < n_int; ++s) {
        if (s == kPre) edges_in(kFirst);
        const int jp = 1 + s * step;
        rows(jp, jp + step - 1 <= RW - 2 ? jp + step - 1 : jp);
      }
      if constexpr (kPre >= n_int) edges_in(kFirst);
      if constexpr (RW >= 2) {
        if constexpr (CPL == 2) rows(RW - 1, 0);
        else { rows(RW - 1, RW - 1); if constexpr (kLazy) edges_in(1, false); rows(0, 0); }
      } else {
        if constexpr (kLazy) edges_in(1, false);
        rows(0, 0);
      }
      if constexpr (MODE == kModeFwd && IRLMX_FWD_NO_ACCOUNT) flags |= 1u << i;
      else if constexpr (kBallotAccount) flags |= (anyv != 0ull ? 1u : 0u) << i;
      else if (MODE == kModeFwd) flags |= ((dmax > eps) ? 1u : 0u) << i;
    }
  };

  // Halo exchange in tagged granules (cluster.h): this instance's region of
  // a.gran is [2 parities][H rows][W + kGranRowPad] x 16 B (cluster.h), of a.sgran [kSumRows][H tiles] x 16 B
  // (summaries by block % kSumSlots, then the XCC ids and the full forward flags).
  const size_t gpl = gran_par_len(W, H);
  const Gran rg = gran_rsrc(a.gran + (size_t)inst * 2 * gran_inst_len(W, H), 32u * (unsigned)gpl);
  constexpr int kRG = WT ? WT + kGranRowPad : 0;  // granules per row (compile-time where the width is)
  const unsigned rgw = WT ? kRG : (unsigned)(W + kGranRowPad);
  const unsigned gbase = (unsigned)e0 * rgw;
  // granule index of extended-tile state l in the parity-0 half
  auto gidx = [&](int l) { return gbase + (unsigned)(l / W) * rgw + (unsigned)(l % W); };
  const Gran rs = gran_rsrc(a.sgran + (size_t)inst * 2 * kSumRows * a.H, 16u * kSumRows * (unsigned)a.H);
  const int ng0 = own0, ng = own0 + (E - own1);  // ghost states: [0, own0) and [own1, E)
  const unsigned salt = (a.salt & 0xFFFu) << 20;  // per call: a stale granule of an earlier call never matches
  // Hand-off store form: write-through (sc1) in general; plain stores (kept in
  // the XCD's L2, where the readers' sc1 loads are served) when every tile of
  // the instance runs on the same XCD -- found by exchanging XCC ids once.
  bool plain = false;
  {
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    xcc &= 0xFu;
    const unsigned htag = salt | 0xFFFFFu;
    if (tid == 0) gran_store(rs, ((unsigned)kXccRow * (unsigned)a.H + (unsigned)tile) * 16u, xcc, htag, false);
    bool ok = true;
    if (tid < kWave) {
      unsigned long long diff = 0ull;
      for (int t0 = 0; t0 < a.C; t0 += kWave) {
        unsigned long long v[1] = {xcc};
        unsigned off[1] = {((unsigned)kXccRow * (unsigned)a.H + (unsigned)(t0 + tid)) * 16u};
        ok &= gran_gather<1>(rs, rs, off, t0 + tid < a.C ? 1u : 0u, htag, v, a.gather_ticks);
        diff |= v[0] ^ xcc;
      }
      diff = wave_or_u64(diff);
      if (tid == 0) { red[2] = diff; lflag[1] = ok ? 0 : 1; }
    }
    __syncthreads();
    if (lflag[1]) { if (tid == 0) atomicOr(a.err, 1); return; }
    plain = a.xcd_group && red[2] == 0ull;
    __syncthreads();
  }

  double* cur = bufA;
  double* oth = bufB;
  long long done = 0;  // sweeps completed before the current block
  // phase cycle counters (thread 0): sweeps, summary + publish, exchange wait, refresh, blocks
  // (in LDS, thread 0 only: as registers they are live across the sweep loop and
  // push the quad kernels over their register budget)
  __shared__ unsigned long long st_acc[8], ts_l[1];  // st_acc[5], [6]: sub-phases of 1
  const bool stamps = a.stamps != nullptr && tid == 0;
  if (stamps) {
    for (int k = 0; k < 8; ++k) st_acc[k] = 0ull;
    ts_l[0] = stamp_now();
  }
  unsigned long long& ts = ts_l[0];
  auto stamp = [&](int k) {
    if (stamps) { const unsigned long long t = stamp_now(); st_acc[k] += t - ts; ts = t; }
  };
  auto stamp_flush = [&]() {
    if (stamps) {
      for (int k = 0; k < 5; ++k) a.stamps[(size_t)lin * 8 + k] = st_acc[k];
      a.stamps[(size_t)lin * 8 + 5] = plain ? 1 : 0;
      a.stamps[(size_t)lin * 8 + 6] = st_acc[5];
      a.stamps[(size_t)lin * 8 + 7] = st_acc[6];
    }
  };
  const long long total = MODE == kModeBwd ? a.n_sweeps : -1;
  int rescale_in = 1;  // backward: blocks until the next rescale
  // n sweeps from the current state (registers for PAIR layouts, else `cur`)
  auto run_sweeps = [&](int n, unsigned& fl) {
    if constexpr (COLS) {
      int i = 0;
      for (; i + 1 < n; i += 2) {
        cols_sweep(cv, cw, i, fl, std::true_type{}, std::true_type{});
        cols_sweep(cw, cv, i + 1, fl, std::true_type{}, std::true_type{});
      }
      if (i < n) {
        cols_sweep(cv, cw, i, fl, std::true_type{}, std::true_type{});
#pragma unroll
        for (int j = 0; j < (COLS ? SPT : 1); ++j) cv[j] = cw[j];
      }
    } else {
      for (int i = 0; i < n; ++i) {
        sweep(cur, oth, i, fl);
        double* t = cur; cur = oth; oth = t;
      }
    }
  };
  // back to the block-start state (forward: the LDS snapshot)
  auto restore = [&]() {
    for (int l = tid; l < E; l += NT) cur[pad + l] = snap[l];
    __syncthreads();
    reload(cur);
  };
  // COLS forward: the n sweeps of a block in registers (fulltag: see cols_sweep).
  // (The backward keeps its own copy of this loop in the block loop: written
  // through this lambda, its schedule changed -- fewer interior FMAs between the
  // band-edge stores and the barrier -- and config 3's backward lost 7.8 %,
  // 22.0 -> 23.8 ms, profiles/r06_forward_ab.txt.)
  auto block_sweeps = [&](unsigned& fl, const int n, auto fulltag) {
    if constexpr (COLS && MODE == kModeFwd) {
      auto go = [&](auto p0tag) {
        int i = 0;
        for (; i + 1 < n; i += 2) {
          cols_sweep(cv, cw, i, fl, p0tag, fulltag);
          cols_sweep(cw, cv, i + 1, fl, p0tag, fulltag);
        }
        if (i < n) {
          cols_sweep(cv, cw, i, fl, p0tag, fulltag);
#pragma unroll
          for (int j = 0; j < (COLS ? SPT : 1); ++j) cv[j] = cw[j];
        }
      };
      // (the full-bookkeeping replay, rare, keeps the p0 add everywhere: one copy less of the loop)
      if (MODE == kModeFwd && ((decltype(fulltag)::value && kProof) || wave_p0)) go(std::true_type{});
      else go(std::false_type{});
    }
  };
  for (int m = 0;; ++m) {
    int Tm = T;
    if (MODE == kModeBwd) Tm = (int)min<long long>((long long)T, total - done);
    // ---- T_m sweeps on chip ----------------------------------------------
    unsigned flags = 0;
    // Backward: rescale at the end of this block?  Every block until the
    // partition vector is seen growing (a non-positive rescale exponent after
    // the first blocks), then every p_max blocks, and always at the last block.
    // Rescaling by a power of two is exact, so the period changes no result
    // while values stay in range; blocks in between publish a zero code.
    const bool resc = MODE == kModeBwd && a.rescale && (rescale_in <= 1 || done + Tm >= total);
    double mxd = 0.0;
    if constexpr (COLS) {
      if constexpr (MODE == kModeBwd) {
        int i = 0;
        for (; i + 1 < Tm; i += 2) {
          cols_sweep(cv, cw, i, flags, std::false_type{}, std::true_type{});
          cols_sweep(cw, cv, i + 1, flags, std::false_type{}, std::true_type{});
        }
        if (i < Tm) {
          cols_sweep(cv, cw, i, flags, std::false_type{}, std::true_type{});
#pragma unroll
          for (int j = 0; j < (COLS ? SPT : 1); ++j) cv[j] = cw[j];
        }
      } else {
        // forward: the p0 add only in waves holding a nonzero p0 (the start states:
        // one wave of the launch at config 3), a wave-uniform scalar branch around
        // the whole block, so each sweep stays one straight-line block
        block_sweeps(flags, Tm, std::integral_constant<bool, !kProof>{});
      }
#ifndef IRLMX_POST_SWEEP_BARRIER
#define IRLMX_POST_SWEEP_BARRIER 0
#endif
      // CW: the band-edge array aliases the tile buffer the publication is
      // staged in, so the last sweep's edge reads must be done first.  The other
      // layouts' staging writes touch nothing a sweep reads (the tile buffer is
      // read only between blocks, behind the barriers there), so their waves go
      // on to the publication as they finish (IRLMX_POST_SWEEP_BARRIER=1: the r04
      // barrier here, A/B)
      if constexpr (CW || IRLMX_POST_SWEEP_BARRIER) __syncthreads();
    } else {
      run_sweeps(Tm, flags);
    }
    if (MODE == kModeFwd) {  // non-finite owned value at the block end: bit 31 (see above)
      const unsigned ob = slot_bits(own_bits);
      bool nf = false;
#pragma unroll
      for (int j = 0; j < SPT; ++j)
        if ((ob >> j) & 1u) nf |= !isfinite(PAIR ? cv[PAIR ? j : 0] : cur[pad + slot_state(j)]);
      if (nf) flags |= 1u << 31;
    }
    if (resc) {  // owned maximum of the block's last sweep (fmax: a NaN is skipped, inf kept)
      const unsigned ob = slot_bits(own_bits);
#pragma unroll
      for (int j = 0; j < SPT; ++j)
        if ((ob >> j) & 1u) mxd = fmax(mxd, fabs(PAIR ? cv[PAIR ? j : 0] : cur[pad + slot_state(j)]));
    }
    stamp(0);
    if (stamps) st_acc[4] += 1;
    // ---- publish the halo rows, tagged with the block ------------------------
    const unsigned tag = salt | (((unsigned)m + 1u) & 0xFFFFFu);
    const unsigned gpar = (unsigned)(m & 1) * (unsigned)gpl;
    // one tile per instance (C == 1: a 64x64 grid fits one CU): no halo, the
    // block summary is the tile's own -- no hand-off at all.  (Compiled in for
    // width 64 only: wider grids never fit one tile, and their kernels keep the
    // exchange code exactly as scheduled without this branch.)
    const bool solo = WT == 64 && a.C == 1;
    auto store_rows = [&]() {  // from the LDS tile, spread evenly over all threads
      for (int l = own0 + tid; l < pubA1; l += NT)
        gran_store(rg, (gpar + gidx(l)) * 16u, dbits(cur[pad + l]), tag, plain);
      for (int l = pubB0 + tid; l < own1; l += NT)
        gran_store(rg, (gpar + gidx(l)) * 16u, dbits(cur[pad + l]), tag, plain);
    };
    if constexpr (COLS) {
      // a band's rows sit in one wave: stage them in the LDS tile first, so that
      // the stores spread over all waves after the barrier below.  kReload: all
      // owned rows, and the register state is read back from the tile after the
      // exchange -- it is then not live across the exchange code, which fits the
      // kernels in their register budget without scratch spills.
      const unsigned pb = slot_bits(kReload ? own_bits : pub_bits);
#pragma unroll
      for (int jp = 0; jp < SPT / 2; ++jp)
        if ((pb >> (2 * jp)) & 1u)
          *reinterpret_cast<double2*>(cur + pad + slot_state(2 * jp)) =
              make_double2(cv[PAIR ? 2 * jp : 0], cv[PAIR ? 2 * jp + 1 : 0]);
    } else if constexpr (PAIR) {
      const unsigned pb = slot_bits(pub_bits);
#pragma unroll
      for (int j = 0; j < SPT; ++j)  // per register slot: all stores of a thread in flight together
        if ((pb >> j) & 1u)
          gran_store(rg, (gpar + gidx(slot_state(j))) * 16u, dbits(cv[PAIR ? j : 0]), tag, plain);
    } else {
      store_rows();
    }
    if (stamps) { const unsigned long long t = stamp_now(); st_acc[5] += t - ts; }
    // ---- per-tile summary of the block (32 bits), while the halo is in flight --
    // forward: bit i / 16 + i = some owned |delta| > eps / NaN at sweep i;
    // backward: scale code (cluster.h) of the owned maximum of the last sweep
    unsigned* red32 = (unsigned*)red;  // [0..1]: tile summary by parity, [2..3]: instance summary
    if (tid == 0) red32[2 + ((m + 1) & 1)] = 0u;  // last read in block m - 1
    if (MODE == kModeFwd) {
      const unsigned wf = wave_reduce_u32<1>(flags) & (((1u << Tm) - 1) | (1u << 31));
      if ((tid & (kWave - 1)) == 0 && wf) atomicOr(&red32[m & 1], wf);
    } else if (resc) {
      const unsigned wc = wave_reduce_u32<0>(scale_code(mxd));
      if ((tid & (kWave - 1)) == 0 && wc) atomicMax(&red32[m & 1], wc);
    }
    if (stamps) { const unsigned long long t = stamp_now(); st_acc[6] += t - ts; }
    __syncthreads();  // the tile summary in red32[m & 1] (and COLS: the staged rows) complete
    if (!solo) {
      if (tid == 0) gran_store(rs, ((unsigned)(m % kSumSlots) * (unsigned)a.H + (unsigned)tile) * 16u, red32[m & 1], tag, plain);
#ifndef IRLMX_PAIR_BATCHED_PUBLISH
#define IRLMX_PAIR_BATCHED_PUBLISH 0
#endif
      if constexpr (COLS && CPL == 2 && !IRLMX_PAIR_BATCHED_PUBLISH) {
        store_rows();
      } else if constexpr (COLS) {
        // column quads (width 256: 8 rows per thread): the staged rows, kPub per
        // thread at a time, all LDS reads in flight before the stores (the plain
        // loop waits out one LDS round trip per row): config 4 backward 302.6 ->
        // 293.6 ms; no gain for column pairs at width 128 (23.5 vs 23.7 ms)
#ifndef IRLMX_KPUB
#define IRLMX_KPUB 4
#endif
        constexpr int kPub = IRLMX_KPUB;
        const int nA = pubA1 - own0, ntot = nA + (own1 - pubB0);
        for (int k0 = 0; k0 < ntot; k0 += kPub * NT) {
          int ls[kPub];
          double vv[kPub];
#pragma unroll
          for (int i = 0; i < kPub; ++i) {
            const int k = k0 + tid + i * NT;
            ls[i] = k < nA ? own0 + k : (k < ntot ? pubB0 + (k - nA) : -1);
            vv[i] = cur[pad + (ls[i] >= 0 ? ls[i] : 0)];
          }
#pragma unroll
          for (int i = 0; i < kPub; ++i)
            if (ls[i] >= 0) gran_store(rg, (gpar + gidx(ls[i])) * 16u, dbits(vv[i]), tag, plain);
        }
      }
    }
    stamp(1);
    // ---- gather this tile's ghost rows and (threads < C) every tile's summary,
    // ---- all polls of a thread in flight together: one round trip --------------
    bool ok = true;
    constexpr int GPT = PAIR ? kGatherPerThread : 1;  // ghost granules in flight per thread
    // Every tile's summary is waited for only when the block needs it (the
    // forward's convergence bits, the backward's rescale blocks -- resc is the
    // same in every tile of an instance): between rescales a backward tile
    // waits for its two neighbours' rows alone, not for the slowest of the
    // instance's C tiles.  (a.eager_summary: every block, for A/B tests.)
    const bool need_summary = a.eager_summary || MODE == kModeFwd || resc;
    auto gather = [&]() {
      for (int k0 = 0; k0 < max(ng, 1); k0 += GPT * NT) {
        unsigned off[GPT + 1];
        int ls[GPT];
        unsigned want = 0;
#pragma unroll
        for (int i = 0; i < GPT; ++i) {
          const int k = k0 + tid + i * NT;
          ls[i] = k < ng0 ? k : own1 + (k - ng0);
          off[i] = (gpar + gidx(ls[i])) * 16u;
          want |= (k < ng ? 1u : 0u) << i;
        }
        off[GPT] = ((unsigned)(m % kSumSlots) * (unsigned)a.H + (unsigned)tid) * 16u;
        want |= (k0 == 0 && tid < a.C && need_summary ? 1u : 0u) << GPT;
        unsigned long long v[GPT + 1];
        ok &= gran_gather<GPT + 1>(rg, rs, off, want, tag, v, a.gather_ticks);
#pragma unroll
        for (int i = 0; i < GPT; ++i)
          if ((want >> i) & 1u) cur[pad + ls[i]] = bits_double(v[i]);
        if ((want >> GPT) & 1u) {
          if (MODE == kModeFwd) atomicOr(&red32[2 + (m & 1)], (unsigned)v[GPT]);
          else atomicMax(&red32[2 + (m & 1)], (unsigned)v[GPT]);
        }
      }
    };
    if (!solo) gather();
    else if (tid == 0) red32[2 + (m & 1)] = red32[m & 1];
    if (!ok) { lflag[0] = 1; atomicOr(a.err, 1); }
    __syncthreads();
    if (lflag[0]) return;  // exchange timed out (reported through a.err)
    const unsigned summary =
        MODE == kModeFwd ? (unsigned)__builtin_amdgcn_readfirstlane((int)red32[2 + (m & 1)]) : red32[2 + (m & 1)];
    if (tid == 0) red32[m & 1] = 0u;  // next-but-one block's tile summary (read above)
    stamp(2);
    if (MODE == kModeFwd) {
      unsigned msk = summary;
      if (msk >> 31) {
        // a non-finite value: every tile of the instance sees the same bit and
        // leaves; the host reruns the call with exact NaN bookkeeping
        stamp_flush();
        if (tile == 0 && tid == 0) atomicOr(a.err, 2);
        return;
      }
      int conv = 0;
      const unsigned live = (1u << Tm) - 1;
      if constexpr (kProof) {
        // Cheap convergence proof.  The block's sweeps kept the owned-delta
        // bookkeeping on band row kProofRow only: a set bit i proves "some owned
        // |delta| > eps at sweep i" (a subset's maximum is at most the
        // maximum), a clear one proves nothing.  If every sweep is proven, the
        // instance is not converged anywhere in the block -- the common case.
        // Otherwise (every tile sees the same OR), every tile replays the block
        // from its start with full bookkeeping -- registers from the LDS
        // snapshot; the tile buffer keeps the ghost rows just gathered -- which
        // recomputes the same values bit for bit, and the tiles exchange the
        // exact flags in a second summary round (row kFullRow).  The stop
        // decision below then uses those.  Typically two blocks of a call
        // replay: the first (the start distribution has not reached the proof
        // rows yet) and the stopping one.
        if ((msk & live) != live) {
          if (tid == 0) { lflag[2] = 0; lflag[3] = 0; }
          const unsigned xb = slot_bits(ext_bits);
#pragma unroll
          for (int j = 0; j < (COLS ? SPT : 1); ++j) cv[j] = ((xb >> j) & 1u) ? snap[slot_state(j)] : 0.0;
          unsigned ff = 0;
          block_sweeps(ff, Tm, std::true_type{});
          const unsigned wf = wave_reduce_u32<1>(ff) & live;
          __syncthreads();   // (lflag[2..3] zeroed; every wave's sweeps done)
          if ((tid & (kWave - 1)) == 0 && wf) atomicOr(reinterpret_cast<unsigned*>(&lflag[2]), wf);
          __syncthreads();
          bool ok2 = true;
          if (!solo) {
            if (tid == 0)
              gran_store(rs, ((unsigned)kFullRow * (unsigned)a.H + (unsigned)tile) * 16u, (unsigned)lflag[2], tag,
                         plain);
            if (tid < a.C) {
              unsigned long long v[1];
              const unsigned off[1] = {((unsigned)kFullRow * (unsigned)a.H + (unsigned)tid) * 16u};
              ok2 = gran_gather<1>(rs, rs, off, 1u, tag, v, a.gather_ticks);
              if (ok2) atomicOr(reinterpret_cast<unsigned*>(&lflag[3]), (unsigned)v[0]);
            }
          } else if (tid == 0) {
            lflag[3] = lflag[2];
          }
          if (!ok2) { lflag[0] = 1; atomicOr(a.err, 1); }
          __syncthreads();
          if (lflag[0]) return;  // exchange timed out (reported through a.err)
          msk = (unsigned)__builtin_amdgcn_readfirstlane(lflag[3]);
        }
      }
      if ((msk & live) != live || (a.max_iter > 0 && done + Tm >= a.max_iter)) {
        for (int i = 0; i < Tm; ++i) {
          const bool cap = a.max_iter > 0 && done + i + 1 >= a.max_iter;
          if (!((msk >> i) & 1u) || cap) { conv = i + 1; break; }
        }
      }
      if (conv) {
        // exact stop inside the block: replay `conv` sweeps from the block-start state
        restore();
        unsigned scratch = 0;
        run_sweeps(conv, scratch);
        if (COLS) {
          const unsigned ob = slot_bits(own_bits);
#pragma unroll
          for (int j = 0; j < SPT; ++j)
            if ((ob >> j) & 1u) a.out[iS + base + slot_state(j)] = cv[PAIR ? j : 0];
        } else {
          for (int l = own0 + tid; l < own1; l += NT) a.out[iS + base + l] = cur[pad + l];
        }
        stamp(3);
        stamp_flush();
        if (tile == 0 && tid == 0) {
          const bool big = (msk >> (conv - 1)) & 1u;
          a.iters[inst] = done + conv;
          a.status[inst] = big ? IRLMX_MAXITER : IRLMX_OK;
        }
        return;
      }
    }
    done += Tm;
    // ---- rescale (backward), snapshot (forward), register copy (pair) --------
    const int e_scale = resc ? code_exponent(summary) : 0;
    if (MODE == kModeBwd) rescale_in = resc ? ((e_scale <= 0 && m >= 3) ? p_max : 1) : rescale_in - 1;
    if constexpr (PAIR) {
      const unsigned ob = slot_bits(own_bits), xb = slot_bits(ext_bits);
#pragma unroll
      for (int jp = 0; jp < SPT / 2; ++jp) {  // pairs: own / ext predicates hold for both states
        const int l = slot_state(2 * jp);
        const bool own = (ob >> (2 * jp)) & 1u, ext = (xb >> (2 * jp)) & 1u;
        double2 v = make_double2(cv[PAIR ? 2 * jp : 0], cv[PAIR ? 2 * jp + 1 : 0]);
        if (kReload) v = ext ? *reinterpret_cast<const double2*>(cur + pad + l) : make_double2(0.0, 0.0);
        else if (!own && ext) v = *reinterpret_cast<const double2*>(cur + pad + l);  // gathered ghost pair
        if (MODE == kModeBwd && e_scale) {
          v.x = ldexp(v.x, e_scale);
          v.y = ldexp(v.y, e_scale);
          if (ext && !COLS) *reinterpret_cast<double2*>(cur + pad + l) = v;
        }
        if (MODE == kModeFwd && ext && !COLS) *reinterpret_cast<double2*>(snap + l) = v;  // COLS: in the first sweep
        cv[PAIR ? 2 * jp : 0] = v.x;
        cv[PAIR ? 2 * jp + 1 : 0] = v.y;
      }
    } else if (MODE == kModeFwd || e_scale) {
      for (int l = tid; l < E; l += NT) {
        double v = cur[pad + l];
        if (MODE == kModeBwd) cur[pad + l] = v = ldexp(v, e_scale);
        if (MODE == kModeFwd) snap[l] = v;
      }
    }
    // Column layouts (not CW) refresh only their own register slots from the
    // tile buffer, and the next block's sweeps touch only registers and the
    // band-edge array: a wave may start them while others still refresh (the
    // next block's staging writes owned rows, its gather writes ghost rows only
    // after the post-staging barrier).  Measured (tools/diag/ab_passes.py, three
    // alternations on one box): one 128x128 instance's forward 14.53 -> 14.17 ms
    // per 20,000 sweeps without this barrier, but config 3's backward 22.50 ->
    // 22.77 ms -- so only the forward drops it.  (IRLMX_POST_SWEEP_BARRIER=1: as r04.)
    if constexpr (!COLS || CW || MODE == kModeBwd || IRLMX_POST_SWEEP_BARRIER) __syncthreads();
    stamp(3);
    if (MODE == kModeBwd && done >= total) break;
  }
  stamp_flush();

  if (MODE == kModeBwd) {
    if (COLS) {  // the register state into the LDS tile for the final per-action sweep
      const unsigned xb = slot_bits(ext_bits);
#pragma unroll
      for (int jp = 0; jp < SPT / 2; ++jp)
        if ((xb >> (2 * jp)) & 1u)
          *reinterpret_cast<double2*>(cur + pad + slot_state(2 * jp)) = make_double2(cv[PAIR ? 2 * jp : 0], cv[PAIR ? 2 * jp + 1 : 0]);
      if constexpr (CW) {
        // the pads and unused slots around the extended tile held band-edge rows
        // (aliasing): back to 0, the value an off-grid neighbour reads below
        for (int l = tid; l < pad; l += NT) cur[l] = 0.0;
        for (int l = pad + E + tid; l < blen; l += NT) cur[l] = 0.0;
      }
      __syncthreads();
    }
    // last of the 2*S sweeps, per action: za = exp(r) * (P_a zs); pi = za / sum_a za
    const int A = a.A;
    const size_t tb = a.tab_shared ? 0 : (size_t)inst;
    for (int l = own0 + tid; l < own1; l += NT) {
      const int s = base + l;
      const double* q = cur + l + (pad - W);
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

}  // namespace irlmx

namespace irlmx {

// Per-instance bounds on the backward's per-sweep growth and decay (reward-folded
// weights, fixed_point.hip bwd_weights_kernel): growth[b] = max_s sum_k bw[b][k][s],
// growth[B + b] = the smallest positive weight (both as float64 bits; the
// weights are non-negative, so the bits order like the values).  The decay bound
// rests on every state feeding some state with a positive weight (its value is
// a stencil operand of itself or of an in-grid neighbour): then the state holding
// the maximum passes at least that weight times it into the next sweep.  A table
// with a state that feeds nobody (its neighbours' weights towards it are all 0)
// has no such bound: growth[B + b] = kNoDecayBound, and the kernel falls back to
// short blocks rescaled every block (cluster_kernel, p_max).
constexpr unsigned long long kNoDecayBound = 0xBFF0000000000000ull;  // bits of -1.0
__global__ void bwd_growth_kernel(const double* __restrict__ bw, int W, int S, int B,
                                  unsigned long long* __restrict__ growth) {
  const int b = blockIdx.x;
  const double* wb = bw + (size_t)b * kStencilK * S;
  unsigned long long mx = 0ull, mn = ~0ull;
  unsigned dead = 0u;  // some state feeds no state with a positive weight
  for (int s = threadIdx.x; s < S; s += blockDim.x) {
    double row = 0.0;
    for (int k = 0; k < kStencilK; ++k) {
      const double x = wb[(size_t)k * S + s];
      row += x;
      if (x > 0.0) mn = min(mn, abs_bits(x));
    }
    mx = max(mx, abs_bits(row));
    // s is slot k's neighbour of: itself (0), s - 1 (+x, 1), s + 1 (-x, 2), s - W (+y, 3), s + W (-y, 4)
    const int x = s % W;
    const bool feeds = wb[s] > 0.0 || (x > 0 && wb[(size_t)1 * S + s - 1] > 0.0) ||
                       (x + 1 < W && wb[(size_t)2 * S + s + 1] > 0.0) ||
                       (s >= W && wb[(size_t)3 * S + s - W] > 0.0) ||
                       (s + W < S && wb[(size_t)4 * S + s + W] > 0.0);
    dead |= feeds ? 0u : 1u;
  }
  __shared__ unsigned long long red[2][16];
  __shared__ unsigned dead_l;
  if (threadIdx.x == 0) dead_l = 0u;
  __syncthreads();
  if (dead) atomicOr(&dead_l, 1u);
  mx = wave_max_u64(mx);
  mn = ~wave_max_u64(~mn);
  if ((threadIdx.x & 63) == 0) { red[0][threadIdx.x / 64] = mx; red[1][threadIdx.x / 64] = mn; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < (int)(blockDim.x / 64); ++i) { mx = max(mx, red[0][i]); mn = min(mn, red[1][i]); }
    growth[b] = mx;
    // no positive weight: no decay at all (0); a state that feeds nobody: no bound
    growth[B + b] = dead_l ? kNoDecayBound : (mn == ~0ull ? 0ull : mn);
  }
}

// Does the backward of these STENCIL5 tables fit the compact-weight layout
// (cluster_kernel LAY == 4)?  With c_k(s) = sum_a row_val[a][k][s] summed as
// bwd_weights_kernel sums it (so the reward-folded weights inherit every
// equality): c_+x == c_-x wherever both neighbours are in the grid, and
// c_self == 0 off the grid border.  Any violation sets *bad.  One block row of
// threads per table instance (grid.y).
__global__ void bwd_compact_ok_kernel(const double* __restrict__ row_val, int W, int H, int A, int* __restrict__ bad) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  const int S = W * H;
  if (s >= S) return;
  const double* rv = row_val + (size_t)blockIdx.y * A * kStencilK * S;
  double c[kStencilK];
  for (int k = 0; k < kStencilK; ++k) {
    double acc = 0.0;
    for (int a = 0; a < A; ++a) acc += rv[((size_t)a * kStencilK + k) * S + s];
    c[k] = acc;
  }
  const int x = s % W, y = s / W;
  const bool ix = x > 0 && x < W - 1, iy = y > 0 && y < H - 1;
  bool ok = !ix || (dbits(c[1]) == dbits(c[2]));
  if (ix && iy) ok = ok && dbits(c[0]) == 0ull;
  if (!ok) atomicOr(bad, 1);
}

static std::atomic<unsigned> g_salt{1};  // per-launch tag salt (cluster.h granules)

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

// CUs the planner plans for: the device's, or IRLMX_PLAN_CUS (tests: a planner
// that believes in more CUs than exist produces a grid that cannot be
// co-resident, which cluster_run must reject; the host-side sanitizer build
// plans without a device).  The co-residency check always uses device_cus().
static int plan_cus() {
  const int forced = env_int("IRLMX_PLAN_CUS", 0);
  return forced > 0 ? forced : device_cus();
}

// Can the C tiles of each of nb instances sit in one XCD group (<= CUs / 8
// workgroups per group, one per CU)?
static bool xcd_groupable(int nb, int C) {
  const int cus = plan_cus();
  return cus >= 8 && ((nb + 7) / 8) * C <= cus / 8;
}

static size_t cluster_lds(int emax, int W, int layout, int nt, int mode) {
  const size_t buf = (size_t)(emax + 2 * (W + 1)) * sizeof(double);  // one padded tile buffer
  const size_t snap = mode == kModeFwd ? (size_t)emax * sizeof(double) : 0;  // forward block-start state
  if (layout >= 2) {
    // column strips: one tile buffer (ghost staging, final sweep) + snapshot +
    // band edge rows [2][NB + 2][2][W / CPL lanes] of CPL doubles + summary words
    const int cpl = layout >= 3 ? 4 : 2;
    const size_t bnd = 2 * (size_t)(nt / (W / cpl) + 2) * 2 * W * sizeof(double);
    if (layout == 4) {
      // compact weights: the edge rows alias the tile buffer (the kernel's
      // padded buffer is emax + 2 W doubles); + the middle columns' self
      // weights per band row (16 B per lane and row) and one zero edge row
      const size_t tb = (size_t)(emax + 2 * W) * sizeof(double);
      return std::max(tb, bnd) + (size_t)emax / 4 * 16 + W * sizeof(double) + 64;
    }
    return buf + snap + bnd + 64;
  }
  // ping-pong buffers + snapshot + summary words
  return 2 * buf + snap + 64;
}

// Tile plan for a width x height stencil grid and B instances: the fewest
// sequential launches first, then the most sweeps per exchange (G), then the
// smallest extended tile.  IRLMX_CLUSTER_R / _G force a plan (tests).
bool cluster_plan(int W, int H, int B, int mode, ClusterPlan* out, bool compact) {
  if (env_int("IRLMX_CLUSTER", 1) == 0) return false;
  const int cus = plan_cus();
  if (cus <= 0) return false;
  const int fR = env_int("IRLMX_CLUSTER_R", 0), fG = env_int("IRLMX_CLUSTER_G", 0);
  // in-tile layout (IRLMX_PAIR forces one): widths 64 / 128 column pairs (2;
  // 1 = pair rows, 3 = column quads at 128), width 256 backward column quads
  // (3), other widths per state (0)
  int layout = 0;
  const int env_layout = env_int("IRLMX_PAIR", -1);
  if (W == 64 || W == 128) layout = env_layout >= 0 ? std::min(env_layout, W == 128 ? 3 : 2) : 2;
  // (the forward's column quads fit only 8 states per lane: too few rows per
  // tile at width 256, so its forward stays per state)
  // (compact: the backward's tables fit layout 4, column quads with three
  // weights per state -- checked per call; IRLMX_PAIR=3 forces the five-weight quads)
  const bool cw = compact && W == 256 && mode == kModeBwd && env_int("IRLMX_COMPACT", 1) != 0;
  if (W == 256)
    layout = env_layout >= 0 ? (env_layout == 4 && cw ? 4 : (env_layout >= 3 ? 3 : 0))
                             : (mode == kModeBwd ? (cw ? 4 : 3) : 0);
  const bool pair = layout > 0;
  const int nt = pair ? kPairThreads : kCT;
  // register budget per lane: the forward's convergence bookkeeping needs more
  // (IRLMX_SPT_MAX: experiments only)
  const int spt_max = env_int("IRLMX_SPT_MAX", !pair ? kSptMax
                                              : layout == 4 ? kSptMaxQuadBwdCW
                                              : layout == 3 ? (mode == kModeFwd ? kSptMaxQuadFwd : kSptMaxQuadBwd)
                                                            : kSptMaxPair);
  const int rows_cap = nt * spt_max / W;
  double best = 1e300;
  bool ok = false;
  // Column-pair backward at width 128: plans with G = 8 ghost rows measured as
  // fast as or faster than the cost model's choice at every working-set size of
  // the full run (tools/diag/g8_plans.py, one MI355X: 9-16 instances 17.5 ->
  // 16.4 ms, 17-24 20.4 -> 19.2, 33-40 24.3 -> 23.2; within 0.7 % elsewhere),
  // so the search is restricted to G = 8 there, unless nothing fits.
  // (At most 8 instances keep the model's choice, (4, 14, 32) for one 128x128
  // instance: 0.4-2.3 % faster than (8, 8, 16) on two boxes.)
  const bool prefer8 = !fG && mode == kModeBwd && layout == 2 && W == 128 && B > 8 && env_int("IRLMX_PLAN_G8", 1) != 0;
  for (int pass = prefer8 ? 0 : 1; pass < 2 && !ok; ++pass)
  for (int G = kTMax; G >= 1; --G) {
    if (fG && G != fG) continue;
    if (pass == 0 && G != 8) continue;
    for (int R = std::min(H, rows_cap - 2 * G); R >= 1; --R) {
      if (fR && R != fR) continue;
      const int C = (H + R - 1) / R;
      const int ext = std::min(H, R + 2 * G);
      const int E = ext * W;
      int spt = (E + nt - 1) / nt;
      if (pair) spt = (spt + (layout >= 3 ? 3 : 1)) / (layout >= 3 ? 4 : 2) * (layout >= 3 ? 4 : 2);
      if (spt > spt_max) continue;
      const size_t lds = cluster_lds(spt * nt, W, layout, nt, mode);
      if (lds + kClusterStaticLds > kMaxLdsBytes) continue;
      const int per = cus / C;
      if (per < 1) continue;
      const int nl = (B + per - 1) / per;
      // cycles per sweep (measured on MI355X, tools/diag/pair_bench.py): ~110 per
      // state slot per sweep, plus one halo exchange per block of G sweeps,
      // ~5k cycles inside one L2, ~11k across XCDs.  (Two 256-thread
      // workgroups per CU, each exchanging while the other sweeps, measured
      // 1.5x slower at config 3: the exchange of a half-size tile costs as much
      // as a full one and the two workgroups stay in phase.)
      // (a single tile per instance needs no hand-off: ~0.8k cycles of block
      // bookkeeping; a sweep takes at least ~850 cycles of barrier, LDS and
      // FMA-chain latency however few states a lane holds)
      const bool solo = C == 1 && W == 64 && layout > 0;
      double xchg = solo ? 800.0 : xcd_groupable(std::min(per, B), C) ? 5000.0 : 11000.0;
      // the forward's block end waits for the convergence words of all C tiles
      // of an instance: ~120 cycles more per tile (measured at one 128x128 /
      // 64x64 instance, C = 8..32: tools/diag/plan_bench.py)
      if (mode == kModeFwd && !solo) xchg += 120.0 * (C - 16);
      // (the forward's convergence bookkeeping: ~165 cycles per slot)
      // A solo tile has no ghost rows, so its block length is free: the backward
      // runs blocks of kSoloBwdT sweeps (IRLMX_SOLO_T; the growth cap still
      // bounds it), amortising the ~1.9k cycles of per-block bookkeeping
      // (rescale test, summary, register refresh) over 16x more sweeps: config 2
      // backward 3.42 -> 2.77 ms.  (The forward's per-sweep convergence bits
      // hold 16 sweeps per block.)
      const int T = (solo && mode == kModeBwd) ? std::max(1, env_int("IRLMX_SOLO_T", kSoloBwdT)) : G;
      const double cost = nl * (std::max((mode == kModeFwd ? 165.0 : 110.0) * spt, 850.0) * T + xchg) / T;
      if (cost < best - 1e-9) {
        best = cost;
        ok = true;
        *out = ClusterPlan{R, G, C, T, std::min(per, B), spt, spt * nt, lds, layout, nt};
      }
    }
  }
  return ok;
}

template <int MODE, int WT>
static void* cluster_fn_w(int spt) {
  switch (spt) {
    case 1: return (void*)&cluster_kernel<MODE, 1, WT, 0, kCT>;
    case 2: return (void*)&cluster_kernel<MODE, 2, WT, 0, kCT>;
    case 3: return (void*)&cluster_kernel<MODE, 3, WT, 0, kCT>;
    case 4: return (void*)&cluster_kernel<MODE, 4, WT, 0, kCT>;
    case 5: return (void*)&cluster_kernel<MODE, 5, WT, 0, kCT>;
    case 6: return (void*)&cluster_kernel<MODE, 6, WT, 0, kCT>;
  }
  return nullptr;
}

template <int MODE, int WT, int LAY>
static void* cluster_fn_pair(int spt) {
  switch (spt) {
    case 2: return (void*)&cluster_kernel<MODE, 2, WT, LAY, kPairThreads>;
    case 4: return (void*)&cluster_kernel<MODE, 4, WT, LAY, kPairThreads>;
    case 6: return (void*)&cluster_kernel<MODE, 6, WT, LAY, kPairThreads>;
    case 8: return (void*)&cluster_kernel<MODE, 8, WT, LAY, kPairThreads>;
    case 10: return (void*)&cluster_kernel<MODE, 10, WT, LAY, kPairThreads>;
    case 12: return (void*)&cluster_kernel<MODE, 12, WT, LAY, kPairThreads>;
  }
  return nullptr;
}

// pair layout for widths 64 / 128 (even states per thread); compile-time LDS
// offsets for widths 64 / 128 / 256; any other width uses WT = 0
template <int MODE, int WT>
static void* cluster_fn_quad(int spt) {
  switch (spt) {
    case 4: return (void*)&cluster_kernel<MODE, 4, WT, 3, kPairThreads>;
    case 8: return (void*)&cluster_kernel<MODE, 8, WT, 3, kPairThreads>;
    case 12: return (void*)&cluster_kernel<MODE, 12, WT, 3, kPairThreads>;
    case 16:  // backward only (kSptMaxQuadFwd: the forward does not fit its registers)
      if constexpr (MODE == kModeBwd) return (void*)&cluster_kernel<MODE, 16, WT, 3, kPairThreads>;
      return nullptr;
  }
  return nullptr;
}

template <int MODE>
static void* cluster_fn(int spt, int W, int layout, int) {
  if (layout == 4) {
    if constexpr (MODE == kModeBwd) {
      if (W != 256) return nullptr;
      switch (spt) {
        case 8: return (void*)&cluster_kernel<MODE, 8, 256, 4, kPairThreads>;
        case 12: return (void*)&cluster_kernel<MODE, 12, 256, 4, kPairThreads>;
        case 16: return (void*)&cluster_kernel<MODE, 16, 256, 4, kPairThreads>;
        case 20: return (void*)&cluster_kernel<MODE, 20, 256, 4, kPairThreads>;
      }
    }
    return nullptr;
  }
  if (layout == 3) {
    if (W == 128) return cluster_fn_quad<MODE, 128>(spt);
    if (W == 256) return cluster_fn_quad<MODE, 256>(spt);
    return nullptr;
  }
  if (layout == 1 || layout == 2) {
    if (W == 64) return layout == 1 ? cluster_fn_pair<MODE, 64, 1>(spt) : cluster_fn_pair<MODE, 64, 2>(spt);
    if (W == 128) return layout == 1 ? cluster_fn_pair<MODE, 128, 1>(spt) : cluster_fn_pair<MODE, 128, 2>(spt);
    return nullptr;
  }
  switch (W) {
    case 64: return cluster_fn_w<MODE, 64>(spt);
    case 128: return cluster_fn_w<MODE, 128>(spt);
    case 256: return cluster_fn_w<MODE, 256>(spt);
  }
  return cluster_fn_w<MODE, 0>(spt);
}

// Launch the cluster kernel over all instances, `per_launch` at a time, then
// check the exchange-timeout word (synchronises the stream).
int cluster_run(int mode, const ClusterPlan& plan, ClusterArgs a, int B, hipStream_t st) {
  ClusterPlan p = plan;
  void* fn;
  fn = mode == kModeFwd ? cluster_fn<kModeFwd>(p.spt, a.W, p.pair, p.nt) : cluster_fn<kModeBwd>(p.spt, a.W, p.pair, p.nt);
  const int nt = p.nt;
  if (!fn) { set_error("cluster: no kernel for spt=%d", p.spt); return IRLMX_EINVAL; }
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)p.lds);
  if (e != hipSuccess) return hip_fail(e, "cluster hipFuncSetAttribute");
  int per_cu = 0;
  e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)fn, nt, p.lds);
  if (e != hipSuccess) return hip_fail(e, "cluster occupancy");
  const int resident = per_cu * device_cus();
  if (p.C * p.per_launch > resident) {
    set_error("cluster: %d workgroups cannot be co-resident (%d)", p.C * p.per_launch, resident);
    return IRLMX_EINVAL;
  }
  a.R = p.R; a.G = p.G; a.C = p.C; a.T = p.T; a.emax = p.emax; a.btot = B;
  unsigned long long* stamps = nullptr;
  const int nwg = p.C * std::min(p.per_launch, B);
  if (env_int("IRLMX_STAMPS", 0)) {  // diagnostics only: phase cycle counters per workgroup
    e = hipMallocAsync((void**)&stamps, sizeof(unsigned long long) * 8 * nwg, st);
    if (e != hipSuccess) return hip_fail(e, "stamps alloc");
    (void)hipMemsetAsync(stamps, 0, sizeof(unsigned long long) * 8 * nwg, st);
  }
  a.stamps = stamps;
  // IRLMX_TEST_NOT_RESIDENT=1 (tests only): wait for one workgroup more than
  // the launch has, i.e. take the not-co-resident path deterministically
  const int extra = env_int("IRLMX_TEST_NOT_RESIDENT", 0) ? 1 : 0;
  // IRLMX_TEST_DROP_TILE=<workgroup> and IRLMX_TEST_EXCHANGE_TIMEOUT_MS=<ms> (tests
  // only): one workgroup leaves after the rendezvous, so its neighbours' exchange
  // times out (after the shortened limit) and the call takes the rerun path
  a.test_drop = env_int("IRLMX_TEST_DROP_TILE", -1);
  a.eager_summary = env_int("IRLMX_EAGER_SUMMARY", 0) ? 1 : 0;
  const int tmo_ms = env_int("IRLMX_TEST_EXCHANGE_TIMEOUT_MS", 0);
  a.gather_ticks = tmo_ms > 0 ? (unsigned long long)tmo_ms * 100000ull : kGatherTicks;
  for (int b0 = 0; b0 < B; b0 += p.per_launch) {
    const int nb = std::min(p.per_launch, B - b0);
    a.b0 = b0;
    a.nb = nb;
    a.n_resident = nb * p.C + extra;
    if (b0 > 0) {  // fresh rendezvous counters for this launch (err[1..2])
      e = hipMemsetAsync(a.err + 1, 0, 2 * sizeof(int), st);
      if (e != hipSuccess) return hip_fail(e, "cluster rendezvous reset");
    }
    a.xcd_group = xcd_groupable(nb, p.C) && env_int("IRLMX_XCD_GROUP", 1) != 0;
    a.salt = g_salt.fetch_add(1, std::memory_order_relaxed);
    void* args[] = {&a};
    const int grid = a.xcd_group ? 8 * ((nb + 7) / 8) * p.C : nb * p.C;
    e = hipLaunchKernel(fn, dim3(grid), dim3(nt), args, p.lds, st);
    if (e != hipSuccess) return hip_fail(e, "cluster launch");
    count_event(IRLMX_CTR_CLUSTER_LAUNCHES);
  }
  int err = 0;
  e = hipMemcpyAsync(&err, a.err, sizeof(int), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) return hip_fail(e, "cluster sync");
  if (stamps) {
    unsigned long long* h = (unsigned long long*)malloc(sizeof(unsigned long long) * 8 * nwg);
    (void)hipMemcpy(h, stamps, sizeof(unsigned long long) * 8 * nwg, hipMemcpyDeviceToHost);
    double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int g = 0; g < nwg; ++g)
      for (int k = 0; k < 8; ++k) acc[k] += (double)h[(size_t)g * 8 + k] / nwg;
    fprintf(stderr, "[irlmx stamps] %s%s mode=%d R=%d G=%d C=%d spt=%d blocks=%.0f  cycles/block: sweeps %.0f  publish %.0f  "
                    "wait %.0f  refresh %.0f  same-xcd %.2f  (publish: stores %.0f, summary %.0f)\n", "lds", p.pair == 4 ? "-quads-cw" : p.pair == 3 ? "-quads" : (p.pair == 2 ? "-cols" : (p.pair == 1 ? "-pair" : "")), mode, p.R, p.G, p.C, p.spt,
            acc[4], acc[0] / acc[4], acc[1] / acc[4], acc[2] / acc[4], acc[3] / acc[4], acc[5], acc[6] / acc[4],
            (acc[7] - acc[6]) / acc[4]);
    if (p.C <= 8) {  // per tile position: the interior tiles carry ghost rows on both sides
      for (int t = 0; t < p.C; ++t) {
        double ta[5] = {0, 0, 0, 0, 0};
        int n = 0;
        for (int g = t; g < nwg; g += p.C, ++n)
          for (int k = 0; k < 5; ++k) ta[k] += (double)h[(size_t)g * 8 + k];
        if (n && ta[4] > 0)
          fprintf(stderr, "[irlmx stamps]   tile %d: sweeps %.0f  publish %.0f  wait %.0f  refresh %.0f\n", t,
                  ta[0] / ta[4], ta[1] / ta[4], ta[2] / ta[4], ta[3] / ta[4]);
      }
    }
    free(h);
    (void)hipFree(stamps);
  }
  if (err & kErrNotResident) {
    count_event(IRLMX_CTR_RERUN_NOT_RESIDENT);
    return kClusterNotResident;
  }
  // A halo exchange that timed out (20 s): every workgroup passed the rendezvous,
  // but one was descheduled later (e.g. compute-wave save/restore on a GPU shared
  // with another process) and its neighbours gave up waiting for its granules.
  // The call is rerun on the per-sweep shape like a failed rendezvous, so a
  // caller on a shared GPU still gets the same answers; the counter records it.
  // IRLMX_STRICT_EXCHANGE=1 reports it as an error instead (tests).
  if (err & 1) {
    if (env_int("IRLMX_STRICT_EXCHANGE", 0)) {
      set_error("cluster: halo exchange timed out (workgroups not co-resident?)");
      return IRLMX_EHIP;
    }
    count_event(IRLMX_CTR_RERUN_TIMEOUT);
    note_exchange_timeout("cluster");
    return kClusterNotResident;
  }
  return (err & 2) ? kClusterNonFinite : 0;
}

}  // namespace irlmx
