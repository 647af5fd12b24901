// Host-side sanitizer driver ("Race detection / sanitizers").
//
// Built by tools/sanitize/Makefile: every irl-maxent_amd/csrc/*.hip source is
// compiled with its host code instrumented by AddressSanitizer +
// UndefinedBehaviorSanitizer (device code as usual: no GPU sanitizer) and linked
// with this driver.  It runs without a GPU: the planner is told the device shape
// through its test overrides (IRLMX_PLAN_CUS = 256 CUs, IRLMX_PLAN_GRID_PER_CU),
// and no call below gets past argument validation and planning, so nothing is
// ever enqueued.  What it exercises under the sanitizers:
//
//  * the tile planner (cluster.hip cluster_plan: R / G / C / states per lane /
//    LDS budget), the fused / grid / dense shape choice and the workspace
//    carving (fixed_point.hip carve) for widths 5..256, rectangular grids,
//    batches 1..256, all four ops, stencil / ELL / DENSE layouts -- through the
//    C ABI's irlmx_execution_plan and irlmx_workspace_bytes, with invariants
//    checked on every plan;
//  * every argument-validation path of every entry point (null models, bad
//    sizes, unknown layouts, NULL arrays, short workspaces), with the error text.
//
// Exit status 0 and "host_check ok" on success.

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/irlmx.h"

static int g_fail = 0;
static long long g_checks = 0;

#define CHECK(cond, ...)                                                  \
  do {                                                                    \
    ++g_checks;                                                           \
    if (!(cond)) {                                                        \
      if (g_fail < 50) {                                                  \
        fprintf(stderr, "FAIL %s:%d (%s): ", __FILE__, __LINE__, #cond);  \
        fprintf(stderr, __VA_ARGS__);                                     \
        fputc('\n', stderr);                                              \
      }                                                                   \
      ++g_fail;                                                           \
    }                                                                     \
  } while (0)

// Never dereferenced by the host code under test: it only checks pointers for NULL.
static double g_fake[16];
static void* fake() { return (void*)g_fake; }

static irlmx_mdp stencil(int w, int h, int a, int b, int shared) {
  irlmx_mdp m;
  memset(&m, 0, sizeof(m));
  m.layout = IRLMX_LAYOUT_STENCIL5;
  m.n_states = w * h;
  m.n_actions = a;
  m.width = w;
  m.height = h;
  m.k_row = m.k_col = 5;
  m.batch = b;
  m.shared = shared;
  m.row_val = g_fake;
  return m;
}

static irlmx_mdp ell(int s, int a, int k_row, int k_col, int b) {
  irlmx_mdp m;
  memset(&m, 0, sizeof(m));
  m.layout = IRLMX_LAYOUT_ELL;
  m.n_states = s;
  m.n_actions = a;
  m.k_row = k_row;
  m.k_col = k_col;
  m.batch = b;
  m.shared = 1;
  m.row_val = g_fake;
  m.row_idx = (const int32_t*)g_fake;
  m.col_idx = (const int32_t*)g_fake;
  m.col_val = g_fake;
  return m;
}

static irlmx_mdp dense(int s, int a, int b) {
  irlmx_mdp m = ell(s, a, s, s, b);
  m.layout = IRLMX_LAYOUT_DENSE;
  return m;
}

static const int kCus = 256;
static long long g_shapes[7];

// Invariants of one plan (include/irlmx.h, IRLMX_PLAN_LEN fields).
static void check_plan(const irlmx_mdp& m, int op, const int64_t* p, const char* what) {
  const int64_t shape = p[0];
  CHECK(shape >= IRLMX_SHAPE_FUSED && shape <= IRLMX_SHAPE_DENSE_GRID, "%s: shape %lld", what, (long long)shape);
  if (shape == IRLMX_SHAPE_FUSED) {
    CHECK(p[7] >= 64 && p[7] <= 1024 && p[7] % 64 == 0, "%s: fused threads %lld", what, (long long)p[7]);
    CHECK(p[5] * p[7] >= m.n_states, "%s: fused spt %lld x %lld < S %d", what, (long long)p[5], (long long)p[7],
          m.n_states);
    CHECK(p[9] <= 160 * 1024, "%s: fused LDS %lld", what, (long long)p[9]);
  } else if (shape == IRLMX_SHAPE_CLUSTER) {
    const int64_t R = p[1], G = p[2], C = p[3], per = p[4], spt = p[5], lay = p[6], nt = p[7], nl = p[8];
    const int H = m.height, W = m.width;
    CHECK(m.layout == IRLMX_LAYOUT_STENCIL5 && (op == IRLMX_OP_BACKWARD || op == IRLMX_OP_FORWARD), "%s", what);
    CHECK(R >= 1 && R <= H && G >= 1 && G <= 16, "%s: R %lld G %lld", what, (long long)R, (long long)G);
    CHECK(C == (H + R - 1) / R, "%s: C %lld for H %d R %lld", what, (long long)C, H, (long long)R);
    CHECK(per >= 1 && per * C <= kCus && per <= m.batch, "%s: per_launch %lld x C %lld", what, (long long)per,
          (long long)C);
    CHECK(nl == (m.batch + per - 1) / per, "%s: launches %lld", what, (long long)nl);
    const int64_t ext = (R + 2 * G < H ? R + 2 * G : H);
    CHECK(spt * nt >= ext * W, "%s: %lld slots < extended tile %lld", what, (long long)(spt * nt),
          (long long)(ext * W));
    CHECK(nt == 512 || nt == 1024, "%s: threads %lld", what, (long long)nt);
    CHECK(lay >= 0 && lay <= 3 && (lay == 0 || W == 64 || W == 128 || W == 256), "%s: layout %lld", what,
          (long long)lay);
    CHECK(p[9] > 0 && p[9] <= 160 * 1024, "%s: LDS %lld", what, (long long)p[9]);
  } else if (shape == IRLMX_SHAPE_GRID) {
    CHECK(p[3] >= 1 && p[4] == m.batch && p[7] == 256, "%s: grid bpi %lld", what, (long long)p[3]);
    CHECK(p[5] * p[7] * p[3] >= m.n_states, "%s: grid covers %lld < S", what, (long long)(p[5] * p[7] * p[3]));
  } else if (shape == IRLMX_SHAPE_DENSE || shape == IRLMX_SHAPE_DENSE_GEMM) {
    CHECK(m.layout == IRLMX_LAYOUT_DENSE, "%s: dense shape for layout %d", what, m.layout);
  } else if (shape == IRLMX_SHAPE_DENSE_GRID) {
    const int64_t rb = p[1], bpi = p[3], cpt = p[5], at = p[6];
    const bool bellman = op == IRLMX_OP_SOFT_BACKWARD || op == IRLMX_OP_VALUE_ITERATION;
    CHECK(m.layout == IRLMX_LAYOUT_DENSE, "%s", what);
    CHECK(p[7] == 512 && p[4] == m.batch && p[8] == 1, "%s: dense grid threads %lld", what, (long long)p[7]);
    CHECK(bellman ? (at >= m.n_actions && (at == 4 || at == 8)) : at == 0, "%s: dense grid actions %lld", what,
          (long long)at);
    CHECK(rb >= (bellman ? 2 : 4) && rb <= 64 && rb * cpt * (bellman ? at : 1) <= 64,
          "%s: dense grid rb %lld cpt %lld", what, (long long)rb, (long long)cpt);
    CHECK(cpt * 512 >= m.n_states && bpi == (m.n_states + rb - 1) / rb, "%s: dense grid covers", what);
    CHECK(bpi * m.batch <= kCus, "%s: dense grid %lld x %d workgroups", what, (long long)bpi, m.batch);
  }
}

static void plan_and_workspace(const irlmx_mdp& m, const char* tag) {
  for (int op = IRLMX_OP_BACKWARD; op <= IRLMX_OP_VALUE_ITERATION; ++op) {
    char what[160];
    snprintf(what, sizeof(what), "%s op %d S %d B %d", tag, op, m.n_states, m.batch);
    int64_t plan[IRLMX_PLAN_LEN];
    for (auto& v : plan) v = -7;
    const int rc = irlmx_execution_plan(&m, op, plan);
    CHECK(rc == 0, "%s: plan rc %d (%s)", what, rc, irlmx_last_error());
    if (rc == 0) check_plan(m, op, plan, what);
    if (rc == 0 && plan[0] >= 0 && plan[0] < 7) ++g_shapes[plan[0]];
    if (op == IRLMX_OP_BACKWARD) {
      int64_t p2[IRLMX_PLAN_LEN];
      CHECK(irlmx_execution_plan(&m, op | IRLMX_PLAN_NO_RESCALE, p2) == 0, "%s: no-rescale plan", what);
      CHECK(p2[0] != IRLMX_SHAPE_CLUSTER, "%s: rescale=0 backward planned on the cluster shape", what);
    }
    const size_t ws = irlmx_workspace_bytes(&m, op);
    const size_t floor = (op == IRLMX_OP_BACKWARD || op == IRLMX_OP_FORWARD)
                             ? (size_t)m.batch * sizeof(int32_t)  // at least the per-instance flags
                             : 0;
    CHECK(ws >= floor && ws < (size_t(1) << 44), "%s: workspace %zu", what, ws);
    CHECK(ws % 256 == 0, "%s: workspace %zu not 256-aligned", what, ws);
  }
}

static int run_bwd(const irlmx_mdp* m, void* reward, void* term, void* pi, void* status, void* ws, size_t n) {
  return irlmx_backward_maxent(m, (const double*)reward, (const uint8_t*)term, 1, (double*)pi, (int32_t*)status, ws,
                               n, nullptr);
}

static void expect(int rc, int want, const char* msg_part, const char* what) {
  CHECK(rc == want, "%s: rc %d, want %d (%s)", what, rc, want, irlmx_last_error());
  CHECK(strstr(irlmx_last_error(), msg_part) != nullptr, "%s: message '%s' lacks '%s'", what, irlmx_last_error(),
        msg_part);
}

static void error_paths() {
  irlmx_mdp good = stencil(5, 5, 4, 1, 1);
  void* f = fake();
  const size_t need = irlmx_workspace_bytes(&good, IRLMX_OP_BACKWARD);
  expect(run_bwd(nullptr, f, f, f, f, f, need), IRLMX_EINVAL, "mdp is NULL", "null mdp");
  struct Bad {
    const char* name;
    irlmx_mdp m;
    const char* msg;
  };
  std::vector<Bad> bad;
  irlmx_mdp m = good; m.n_states = 0; bad.push_back({"S=0", m, "bad sizes"});
  m = good; m.n_actions = 9; bad.push_back({"A=9", m, "exceeds"});
  m = good; m.batch = -1; bad.push_back({"B<0", m, "bad sizes"});
  m = good; m.row_val = nullptr; bad.push_back({"row_val", m, "row_val is NULL"});
  m = good; m.width = 4; bad.push_back({"grid", m, "stencil grid"});
  m = good; m.width = -5; m.height = -5; bad.push_back({"negative grid", m, "stencil grid"});
  m = good; m.layout = 9; bad.push_back({"layout", m, "unknown layout"});
  m = ell(25, 4, 30, 3, 1); bad.push_back({"ell k_row", m, "out of range"});
  m = ell(25, 4, 3, 3, 1); m.row_idx = nullptr; bad.push_back({"ell row_idx", m, "ELL row form missing"});
  m = dense(25, 4, 1); m.col_val = nullptr; bad.push_back({"dense col_val", m, "missing"});
  m = dense(1 << 20, 4, 1); bad.push_back({"dense size", m, "too large"});
  for (const Bad& b : bad) {
    expect(run_bwd(&b.m, f, f, f, f, f, need), IRLMX_EINVAL, b.msg, b.name);
    int64_t plan[IRLMX_PLAN_LEN];
    expect(irlmx_execution_plan(&b.m, IRLMX_OP_FORWARD, plan), IRLMX_EINVAL, b.msg, b.name);
    int32_t props = 0;
    expect(irlmx_mdp_properties(&b.m, &props, nullptr), IRLMX_EINVAL, b.msg, b.name);
    CHECK(irlmx_workspace_bytes(&b.m, IRLMX_OP_FORWARD) == 0, "%s: workspace of an invalid model", b.name);
  }
  expect(run_bwd(&good, nullptr, f, f, f, f, need), IRLMX_EINVAL, "reward is NULL", "null reward");
  expect(run_bwd(&good, f, f, f, nullptr, f, need), IRLMX_EINVAL, "status is NULL", "null status");
  expect(run_bwd(&good, f, f, f, f, f, need - 1), IRLMX_EWORKSPACE, "workspace too small", "short workspace");
  expect(run_bwd(&good, f, f, f, f, nullptr, need), IRLMX_EWORKSPACE, "workspace too small", "null workspace");
  expect(irlmx_forward_svf(&good, (double*)f, (uint8_t*)f, (double*)f, 1e-5, 0, (double*)f, nullptr, (int32_t*)f, f,
                           1 << 30, nullptr),
         IRLMX_EINVAL, "iterations is NULL", "forward null iterations");
  expect(irlmx_soft_backward(&good, (double*)f, nullptr, 0.7, 1e-5, 0, (double*)f, nullptr, (int64_t*)f,
                             (int32_t*)f, f, 1 << 30, nullptr),
         IRLMX_EINVAL, "terminal_reward is NULL", "soft null phi");
  expect(irlmx_value_iteration(&good, (double*)f, 0.9, 1e-3, 0, 0, nullptr, (int64_t*)f, (int32_t*)f, f, 1 << 30,
                               nullptr),
         IRLMX_EINVAL, "value is NULL", "vi null value");
  int64_t plan[IRLMX_PLAN_LEN];
  expect(irlmx_execution_plan(&good, 0, plan), IRLMX_EINVAL, "unknown op 0", "op 0");
  expect(irlmx_execution_plan(&good, -1, plan), IRLMX_EINVAL, "unknown op -1", "op -1");
  expect(irlmx_execution_plan(&good, IRLMX_OP_FORWARD | IRLMX_PLAN_NO_RESCALE, plan), IRLMX_EINVAL, "NO_RESCALE",
         "no-rescale forward");
  expect(irlmx_execution_plan(&good, IRLMX_OP_FORWARD, nullptr), IRLMX_EINVAL, "plan is NULL", "null plan");
  expect(irlmx_mdp_properties(nullptr, (int32_t*)f, nullptr), IRLMX_EINVAL, "mdp is NULL", "props null mdp");
  expect(irlmx_mdp_properties(&good, nullptr, nullptr), IRLMX_EINVAL, "props is NULL", "props null out");
  expect(irlmx_numpy_math(2, (double*)f, (double*)f, 4, nullptr), IRLMX_EINVAL, "unknown op 2", "npmath op");
  expect(irlmx_numpy_math(IRLMX_NPMATH_EXP, (double*)f, (double*)f, -1, nullptr), IRLMX_EINVAL, "< 0", "npmath n");
  expect(irlmx_numpy_math(IRLMX_NPMATH_LOG, nullptr, (double*)f, 4, nullptr), IRLMX_EINVAL, "NULL", "npmath null");
  expect(irlmx_numpy_math(IRLMX_NPMATH_EXP, nullptr, nullptr, 0, nullptr), IRLMX_OK, "", "npmath empty");
  expect(irlmx_build_icy_gridworld(0, (double*)f, 1, (double*)f, nullptr), IRLMX_EINVAL, "size=0", "icy size");
  expect(irlmx_build_gridworld(50000, 1, (double*)f, nullptr), IRLMX_EINVAL, "size=50000", "grid size");
  expect(irlmx_dense_to_stencil((double*)f, 5, 5, 4, (double*)f, nullptr, nullptr), IRLMX_EINVAL, "off_stencil NULL",
         "stencil flag");
  expect(irlmx_dense_to_rows((double*)f, 25, 9, (double*)f, (double*)f, nullptr), IRLMX_EINVAL, "n_actions=9",
         "rows actions");
  expect(irlmx_dense_ell_sizes((double*)f, 0, 4, (int32_t*)f, (int32_t*)f, nullptr), IRLMX_EINVAL, "n_states=0",
         "ell sizes");
  expect(irlmx_dense_to_ell((double*)f, 25, 4, 26, 3, (int32_t*)f, (double*)f, (int32_t*)f, (double*)f, nullptr),
         IRLMX_EINVAL, "k_row=26", "ell k");
  expect(irlmx_optimal_policy((int32_t*)f, 25, 4, 1, nullptr, (int64_t*)f, nullptr), IRLMX_EINVAL, "value NULL",
         "argmax value");
  expect(irlmx_stochastic_policy((int32_t*)f, 25, 0, 1, (double*)f, (double*)f, nullptr), IRLMX_EINVAL,
         "n_actions=0", "stochastic actions");
  int64_t ctr[IRLMX_COUNTERS_LEN + 4];
  CHECK(irlmx_counters(ctr, IRLMX_COUNTERS_LEN + 4) == IRLMX_COUNTERS_LEN, "counters length");
  CHECK(irlmx_counters(nullptr, 3) == IRLMX_COUNTERS_LEN, "counters length (NULL)");
}

int main() {
  setenv("IRLMX_PLAN_CUS", "256", 1);          // the MI355X's CU count, without a device
  setenv("IRLMX_PLAN_GRID_PER_CU", "4", 1);
  CHECK(irlmx_abi_version() == IRLMX_ABI_VERSION, "abi version");
  error_paths();

  std::vector<int> widths, batches;
  for (int w = 5; w <= 40; ++w) widths.push_back(w);
  for (int w = 41; w <= 256; w += 9) widths.push_back(w);
  for (int w : {48, 63, 64, 65, 96, 127, 128, 129, 192, 255, 256}) widths.push_back(w);
  for (int b = 1; b <= 16; ++b) batches.push_back(b);
  for (int b : {17, 31, 32, 33, 63, 64, 65, 100, 127, 128, 129, 200, 255, 256}) batches.push_back(b);
  long long plans = 0;
  for (int w : widths) {
    for (int b : batches) {
      for (int shared = 0; shared <= 1; ++shared) {
        plan_and_workspace(stencil(w, w, 4, b, shared), "square");
        plan_and_workspace(stencil(w, w, 5, b, shared), "square A=5");
        plans += 8;
      }
      if (w % 3 == 0) {  // rectangles: wide and tall
        plan_and_workspace(stencil(w, 2 * w + 1, 4, b, 0), "tall");
        plan_and_workspace(stencil(2 * w, w, 4, b, 0), "wide");
        plans += 8;
      }
    }
  }
  // generic sparsity and dense rows: state counts around the fused / grid boundaries
  for (int s : {5, 25, 100, 1000, 4095, 4096, 4097, 10000, 16384, 40000}) {
    for (int k : {1, 2, 5, 8, 9, 16, 17, 32, 33}) {
      if (k > s) continue;
      for (int b : {1, 3, 16, 64, 256}) {
        plan_and_workspace(ell(s, 4, k, k, b), "ell");
        plan_and_workspace(ell(s, 4, k, (k % 5) + 1, b), "ell skew");
        plans += 8;
      }
    }
  }
  for (int s : {7, 64, 301, 1040, 2048, 4096, 8192})
    for (int b : {1, 3, 4, 15, 16, 17, 64}) {
      plan_and_workspace(dense(s, 4, b), "dense");
      plans += 4;
    }
  if (g_fail) {
    fprintf(stderr, "host_check: %d of %lld checks failed\n", g_fail, g_checks);
    return 1;
  }
  CHECK(g_shapes[IRLMX_SHAPE_CLUSTER] > 1000 && g_shapes[IRLMX_SHAPE_GRID] > 100 && g_shapes[IRLMX_SHAPE_FUSED] > 100 &&
            g_shapes[IRLMX_SHAPE_DENSE_GEMM] > 0 && g_shapes[IRLMX_SHAPE_DENSE] > 0 &&
            g_shapes[IRLMX_SHAPE_DENSE_GRID] > 0,
        "every shape planned: fused %lld cluster %lld sweep %lld dense %lld gemm %lld grid %lld dense-grid %lld",
        g_shapes[0], g_shapes[1], g_shapes[2], g_shapes[3], g_shapes[4], g_shapes[5], g_shapes[6]);
  if (g_fail) {
    fprintf(stderr, "host_check: %d of %lld checks failed\n", g_fail, g_checks);
    return 1;
  }
  printf("host_check ok: %lld plans, %lld checks; shapes fused %lld cluster %lld sweep %lld dense %lld dense-gemm %lld "
         "grid %lld dense-grid %lld\n", plans, g_checks, g_shapes[0], g_shapes[1], g_shapes[2], g_shapes[3], g_shapes[4],
         g_shapes[5], g_shapes[6]);
  return 0;
}
