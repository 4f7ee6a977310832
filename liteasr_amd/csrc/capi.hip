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

static const uint64_t* g_drop_ctr = nullptr;
const uint64_t* lasr_dropout_counter() { return g_drop_ctr; }
extern "C" int lasr_set_dropout_counter(const uint64_t* dev_counter) {
  g_drop_ctr = dev_counter;
  return LASR_OK;
}

__global__ void counter_add_kernel(uint64_t* c, uint64_t v) { c[0] += v; }
extern "C" int lasr_counter_add(uint64_t* dev_counter, uint64_t v, void* stream) {
  counter_add_kernel<<<1, 1, 0, (hipStream_t)stream>>>(dev_counter, v);
  return lasr_check_launch("counter_add");
}

// Multiplier of kept elements for drop probability p (common.h mkdrop): callers that apply a
// stored keep mask (the GEMM gate, aux_act = LASR_ACT_GATE) scale by this.
extern "C" float lasr_dropout_scale(float p) { return mkdrop(p, 0).scale; }
