// C-ABI plumbing: error reporting and version (see include/nbp.h).
#include <stdarg.h>
#include <string.h>

#include "nbp_common.h"

namespace nbp {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return NBP_ERR_LAUNCH;
  }
  return NBP_OK;
}

}  // namespace nbp

extern "C" {

const char* nbp_last_error_string(void) { return nbp::g_err; }

int nbp_version(void) { return NBP_VERSION; }

}  // extern "C"
