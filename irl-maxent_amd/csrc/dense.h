// Dense-row path (IRLMX_LAYOUT_DENSE): shared declarations between dense.hip
// (kernels) and fixed_point.hip (the per-sweep drivers and the C ABI).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"

namespace irlmx {

// A dense model: B instances over one table (shared) or B tables.
struct DenseView {
  int S, A, B, shared;
  const double* P;  // [B'][A][S][S]: P[s, t, a] at [a][s][t]
  const double* M;  // [B'][S][S]:    sum_a P[s, t, a]
};

// Per-sweep state, the same conventions as the sweep shape (fixed_point.hip Ws):
// ping-pong vectors, a 3-slot ring of per-instance max|.| words, done flags.
struct DenseBufs {
  double* buf0;               // [B][S]
  double* buf1;               // [B][S]
  unsigned long long* slots;  // [B][3]
  int32_t* done;              // [B]
  int64_t* iters;             // [B]
  int32_t* ndone;             // [1]
  int32_t* bad;               // [B] non-finite policy (forward) / partition value (backward)
  double* wt;                 // forward: [B][S][S] per-instance gather matrix WT[t][s]; GEMM: [B][S] product
};

struct DenseBellman {  // soft VI (maxent.py:326-338) / VI (solver.py:40-50)
  const double* reward;
  const double* phi;
  double discount;
  double eps;
  long long max_iter;
  int average;
  int soft;
  double* pi;
  double* value;
  int64_t* iters;
  int32_t* status;
};

constexpr int kDenseMaxActions = 8;
// rows of a dense kernel launch: 4 waves x kDenseRowsPerWave rows per workgroup
constexpr int kDenseThreads = 256;
// Build-time knobs (tools/diag/build_variant.sh -D...; tools/diag/dense_bench.py,
// profiles/r02_dense_variants.txt, microseconds per sweep at B = 1):
//                         S=2048 bwd / fwd    S=4096 bwd / fwd
//   LDS vector, unroll 1     8.97 / 9.86        29.3 / 30.3
//   LDS vector, unroll 4     8.40 / 9.12        26.2 / 27.1
//   global vector, unroll 4  8.18 / 9.31        24.8 / 26.5
//   one row per wave         10.9 / 12.0        31.3 / 32.7
// Unrolling lets a wave issue the loads of four row chunks before their FMAs
// (same FMA order, bit-identical).  Reading the swept vector through L1/L2
// instead of staging it in LDS drops the per-block prologue and its barrier at
// one instance; with several instances the vector re-reads compete with the
// row streams in L1/L2 (S = 2048, B = 16: backward 36 us with LDS, 47 without;
// forward 108 vs 158), so there it is staged (dense_lds_vec).
#ifndef IRLMX_DENSE_RPW
#define IRLMX_DENSE_RPW 2
#endif
#ifndef IRLMX_DENSE_UNROLL
#define IRLMX_DENSE_UNROLL 4
#endif
constexpr int kDenseRowsPerWave = IRLMX_DENSE_RPW;
constexpr int kDenseUnroll = IRLMX_DENSE_UNROLL;  // wave_dot: loop iterations whose loads issue together
constexpr int kDenseRowsPerBlock = (kDenseThreads / kWave) * kDenseRowsPerWave;
constexpr int kDenseLdsMaxStates = 8192;  // the swept vector fits in LDS up to here (64 KiB)

// Stage the swept vector in LDS?
bool dense_lds_vec(const DenseView& d);

void dense_rows_launch(const double* dense, int S, int A, double* P, double* M, hipStream_t st);
void dense_fwd_weights_launch(const DenseView& d, const double* pi, const uint8_t* term, DenseBufs w,
                              hipStream_t st);
void dense_fwd_sweep_launch(const DenseView& d, const double* p0, double eps, long long max_iter, int32_t* status,
                            DenseBufs w, long long it, int r3, hipStream_t st);
void dense_bwd_init_launch(const DenseView& d, const uint8_t* term, DenseBufs w, hipStream_t st);
void dense_bwd_sweep_launch(const DenseView& d, const double* reward, int rescale, DenseBufs w, long long it, int r3,
                            hipStream_t st);
// shared table, all B instances: the epilogue of a GEMM sweep (w.wt = M . ZS)
void dense_bwd_gemm_epilogue_launch(const DenseView& d, const double* reward, int rescale, DenseBufs w, long long it,
                                    int r3, hipStream_t st);
void dense_bwd_final_launch(const DenseView& d, const double* reward, int rescale, double* pi, int32_t* status,
                            DenseBufs w, long long collapsed, int r3, hipStream_t st);
void dense_bellman_sweep_launch(const DenseView& d, const DenseBellman& a, DenseBufs w, long long it, int r3,
                                hipStream_t st);
void dense_bellman_finish_launch(const DenseView& d, const DenseBellman& a, DenseBufs w, hipStream_t st);
// shared table: the sweep's A products P_a . [v_1 .. v_B] on the MFMA kernel (w.wt = [B][A][S]) + the update
hipError_t dense_bellman_gemm_sweep_launch(const DenseView& d, const DenseBellman& a, DenseBufs w, long long it,
                                           int r3, hipStream_t st);
// C[b][r] = sum_t M[r][t] Z[b][t], M [R][S], Z [B][S], on the fp64 matrix cores (any S; rows of M and Z
// contiguous); returns the attribute / launch error, if any
hipError_t dense_gemm_launch(const double* M, const double* Z, double* C, int R, int S, int B, hipStream_t st);
// {ST row tiles, NBT instance tiles, waves, 16-byte loads} of the launch dense_gemm_launch makes
void dense_gemm_variant(int R, int S, int B, int* out);

// Persistent dense shape (dense_grid.hip): the forward / collapsed backward loop
// in one launch, each workgroup holding rb rows of its instance's matrix in
// registers (columns t + 512 j, j < cpt), values exchanged as tagged granules.
constexpr int kDenseGridThreads = 512;
struct DenseGridPlan {
  int rb, cpt, bpi, xcd;  // rows per workgroup, columns per thread, workgroups per instance, XCD grouping
  int at;                 // soft VI / VI: actions compiled (4 or 8), else 0
};
struct DenseGridArgs {
  int S, A, B, shared;
  const double* mat;          // forward: WT [B][S][S]; backward: M [B'][S][S]
  const double* P;            // backward final sweep: [B'][A][S][S]
  const double* vin;          // forward: p0 [B][S]; backward, soft VI, VI: reward [B][S]
  const uint8_t* term;        // backward: terminal mask [B][S]
  const int32_t* bad;         // forward: non-finite policy [B]
  const double* phi;          // soft VI: terminal reward [B][S]
  double discount;            // soft VI / VI
  int average;                // VI: mean over actions (solver.py:99) instead of the max
  double* value;              // soft VI / VI: value out [B][S] (optional for soft VI)
  double eps;
  long long max_iter;
  int rescale;
  double* out;                // forward: svf [B][S]; backward, soft VI: pi [B][S][A]
  int64_t* iters;
  int32_t* status;
  unsigned long long* gran;   // [B][2][S] x 16-byte granules
  unsigned long long* xgran;  // [B][bpi] x 16-byte granules (XCC ids)
  int* err;                   // [0] timeout (1) / not co-resident (4); [1..2] rendezvous
  int rb, bpi, nb, xcd_group; // (set by dense_grid_run)
  unsigned salt;
  int n_resident;
  unsigned long long gather_ticks;  // exchange timeout (kGatherTicks unless a test shortens it)
  int test_drop;              // tests only (IRLMX_TEST_DROP_TILE): this workgroup leaves after the rendezvous, else -1
};
// mode: kModeFwd / kModeBwd (cluster.h).  False when the rows do not fit in
// registers at one workgroup per CU (IRLMX_DENSE_GRID=0 disables the shape,
// IRLMX_DENSE_GRID_RB forces the rows per workgroup).
bool dense_grid_plan(int mode, int S, int B, DenseGridPlan* out);
// 0, kClusterNotResident (rerun per sweep; err words cleared) or an IRLMX_E* code
int dense_grid_run(int mode, const DenseGridPlan& p, DenseGridArgs a, hipStream_t st);
// Soft VI / VI (maxent.py:326-341, solver.py:40-50 / 95-100) of a DENSE model in
// one persistent launch: each workgroup holds the A rows P_a of its rb states
// (A <= 8; A * rb * cpt <= 64 doubles per thread)
bool dense_bellman_grid_plan(int S, int B, int A, DenseGridPlan* out);
int dense_bellman_grid_run(bool soft, const DenseGridPlan& p, DenseGridArgs a, hipStream_t st);

}  // namespace irlmx
