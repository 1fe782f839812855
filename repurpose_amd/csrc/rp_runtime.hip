// Error plumbing and version of the C ABI (include/rp_api.h).
#include <stdarg.h>
#include <string.h>

#include "rp_common.h"

static thread_local char g_err[1024] = "";

void rp_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int rp_check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    rp_set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return RP_ERR_LAUNCH;
  }
  return RP_OK;
}

extern "C" int rp_version(void) { return 1; }

extern "C" int rp_last_error(char* buf, size_t n) {
  if (!buf || n == 0) return RP_ERR_ARG;
  strncpy(buf, g_err, n - 1);
  buf[n - 1] = '\0';
  return RP_OK;
}
