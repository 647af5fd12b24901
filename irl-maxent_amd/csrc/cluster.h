// Persistent temporally blocked stencil kernels (cluster.hip): shared declarations.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace irlmx {

constexpr int kCT = 1024;    // threads per cluster workgroup
constexpr int kTMax = 16;    // max sweeps per block (= max ghost rows)
constexpr int kSptMax = 6;   // states per thread -> extended tile <= 6144 states (no VGPR spills)
constexpr int kModeFwd = 0;
constexpr int kModeBwd = 1;

struct ClusterArgs {
  int W, H, S, A;
  int R, G, C, T;          // rows per tile, ghost rows, tiles per instance, max sweeps per block
  int b0;                  // first instance of this launch
  int btot;                // instances in pub / slots / counter arrays
  int emax;                // LDS buffer length (states)
  int tab_shared;          // backward tables shared by all instances
  const double* wgt;       // forward: [B][5][S] gather weights; backward: [B'][5][S] collapsed
  const double* row_val;   // backward final sweep: [B'][A][5][S]
  const double* vin;       // forward: p0 [B][S]; backward: reward [B][S]
  const uint8_t* term;     // backward: terminal mask [B][S]
  const int32_t* bad;      // forward: non-finite policy flags [B]
  const unsigned long long* growth;  // backward: per-instance growth bound bits [B]
  double eps;
  long long max_iter;
  long long n_sweeps;      // backward: collapsed sweeps (2S - 1)
  int rescale;
  double* pub;             // [2][B][S]
  unsigned long long* slots;  // [B][3][kTMax]
  unsigned int* counter;   // [B]
  int* err;                // [1] barrier timeout
  unsigned long long* stamps;  // optional [grid][8] phase cycle counters (IRLMX_STAMPS=1), else null
  double* out;             // forward: svf [B][S]; backward: pi [B][S][A]
  int64_t* iters;
  int32_t* status;
};

struct ClusterPlan {
  int R, G, C, T, per_launch, spt, emax;
  size_t lds;
};

bool cluster_plan(int W, int H, int B, ClusterPlan* out);
int cluster_run(int mode, const ClusterPlan& p, ClusterArgs a, int B, hipStream_t st);
__global__ void bwd_growth_kernel(const double* __restrict__ bw, int tab_shared, const double* __restrict__ reward,
                                  int S, unsigned long long* __restrict__ growth);

}  // namespace irlmx
