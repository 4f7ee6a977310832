// Error plumbing and version for the C ABI (include/liteasr_hip.h).
#include <stdarg.h>
#include <stdio.h>

#include "common.h"

static thread_local char g_err[512] = "";

void lasr_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int lasr_check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    lasr_set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return LASR_ERR_LAUNCH;
  }
  return LASR_OK;
}

extern "C" const char* lasr_last_error(void) { return g_err; }
extern "C" int lasr_version(void) { return 1; }
