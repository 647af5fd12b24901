// Error reporting and version of the irlmx C ABI.  No C++ exception crosses
// the ABI: failures return a negative code and leave a thread-local message.

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <vector>

#include "common.h"

namespace irlmx {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int hip_fail(hipError_t e, const char* what) {
  set_error("%s: %s (%d)", what, hipGetErrorString(e), (int)e);
  return IRLMX_EHIP;
}

static std::atomic<long long> g_counters[IRLMX_COUNTERS_LEN];

void count_event(int which) {
  if (which >= 0 && which < IRLMX_COUNTERS_LEN) g_counters[which].fetch_add(1, std::memory_order_relaxed);
}

void note_exchange_timeout(const char* shape) {
  static std::atomic<bool> told{false};
  if (!told.exchange(true))
    fprintf(stderr,
            "irlmx: %s shape: an exchange timed out (a workgroup descheduled or a lost granule); the call was rerun "
            "on the per-sweep shape (counter rerun_timeout; IRLMX_STRICT_EXCHANGE=1 makes it an error)\n", shape);
}

__global__ void numpy_math_kernel(int op, const double* __restrict__ x, double* __restrict__ y, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = op == IRLMX_NPMATH_EXP ? np_exp(x[i]) : np_log(x[i]);
}

static std::vector<DcheckTake>& dcheck_registry() {
  static std::vector<DcheckTake> r;
  return r;
}

bool register_dcheck(DcheckTake take) {
  dcheck_registry().push_back(take);
  return true;
}

}  // namespace irlmx

extern "C" int irlmx_device_checks_enabled(void) { return IRLMX_DEVICE_CHECKS; }

extern "C" int64_t irlmx_device_check_failures(void) {
  if (!IRLMX_DEVICE_CHECKS) return 0;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  unsigned v = 0;
  for (auto take : irlmx::dcheck_registry()) v |= take();
  return (int64_t)v;
}

extern "C" int irlmx_abi_version(void) { return IRLMX_ABI_VERSION; }

extern "C" int irlmx_numpy_math(int32_t op, const double* x, double* y, int64_t n, void* stream) {
  if (op != IRLMX_NPMATH_EXP && op != IRLMX_NPMATH_LOG) {
    irlmx::set_error("unknown op %d", op);
    return IRLMX_EINVAL;
  }
  if (n < 0) {
    irlmx::set_error("n = %lld < 0", (long long)n);
    return IRLMX_EINVAL;
  }
  if (n == 0) return IRLMX_OK;
  if (!x || !y) {
    irlmx::set_error("x or y is NULL");
    return IRLMX_EINVAL;
  }
  const int64_t blocks = (n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096;
  hipLaunchKernelGGL(irlmx::numpy_math_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, op, x, y, n);
  if (hipError_t e = hipGetLastError(); e != hipSuccess) return irlmx::hip_fail(e, "numpy_math_kernel");
  return IRLMX_OK;
}

extern "C" const char* irlmx_last_error(void) { return irlmx::g_err; }

extern "C" int irlmx_counters(int64_t* out, int32_t n) {
  if (out)
    for (int i = 0; i < n && i < IRLMX_COUNTERS_LEN; ++i)
      out[i] = irlmx::g_counters[i].load(std::memory_order_relaxed);
  return IRLMX_COUNTERS_LEN;
}
