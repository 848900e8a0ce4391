// C-ABI plumbing: thread-local error text, launch checks, version.
#include "common.h"

#include <cstring>

namespace vqgnn {

static thread_local char g_err[512] = {0};

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

void clear_error() { g_err[0] = 0; }

int check_launch(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return VQGNN_ERR_LAUNCH;
  }
  return VQGNN_OK;
}

}  // namespace vqgnn

extern "C" const char* vqgnn_last_error(void) { return vqgnn::g_err; }
extern "C" int vqgnn_version(void) { return 500; }
