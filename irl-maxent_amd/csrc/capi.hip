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

extern "C" const char* irlmx_last_error(void) { return irlmx::g_err; }

extern "C" int irlmx_counters(int64_t* out, int32_t n) {
  if (out)
    for (int i = 0; i < n && i < IRLMX_COUNTERS_LEN; ++i)
      out[i] = irlmx::g_counters[i].load(std::memory_order_relaxed);
  return IRLMX_COUNTERS_LEN;
}
