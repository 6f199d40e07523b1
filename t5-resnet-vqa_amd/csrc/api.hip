// Error reporting and version for the C ABI (include/vqa_hip.h).
#include <stdarg.h>
#include <stdio.h>

#include "common.h"

namespace {
thread_local char g_err[512] = "";
}

namespace vqa {
int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail((int)e, "%s: launch failed: %s", what, hipGetErrorString(e));
  return VQA_OK;
}
}  // namespace vqa

extern "C" int vqa_abi_version(void) { return VQA_ABI_VERSION; }
extern "C" const char* vqa_last_error(void) { return g_err; }
