// Error reporting and version of the irlmx C ABI.  No C++ exception crosses
// the ABI: failures return a negative code and leave a thread-local message.

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>

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

}  // namespace irlmx

extern "C" int irlmx_abi_version(void) { return IRLMX_ABI_VERSION; }

extern "C" const char* irlmx_last_error(void) { return irlmx::g_err; }
