// C-ABI plumbing: error reporting and version (see include/nbp.h).
#include <stdarg.h>
#include <string.h>

#include <vector>

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

// Per-launch timing of the entries that issue several kernel instances per call (nbp_launch_timing): while on, each
// such launch is bracketed by HIP events on its stream and recorded with its kernel instance name and its algorithmic
// FLOPs / bytes.  Off (the default) it costs one thread-local test per launch.
struct LaunchRec {
  const char* name;
  hipEvent_t e0, e1;
  double flops, bytes;
};
static thread_local std::vector<LaunchRec> g_lrec;
static thread_local bool g_ltiming = false;
static thread_local hipEvent_t g_lt_open = nullptr;

void lt_begin(hipStream_t st) {
  if (!g_ltiming) return;
  hipEvent_t e;
  if (hipEventCreate(&e) != hipSuccess) return;
  hipEventRecord(e, st);
  g_lt_open = e;
}

void lt_end(hipStream_t st, const char* name, double flops, double bytes) {
  if (!g_ltiming || !g_lt_open) return;
  hipEvent_t e;
  if (hipEventCreate(&e) != hipSuccess) return;
  hipEventRecord(e, st);
  g_lrec.push_back(LaunchRec{name, g_lt_open, e, flops, bytes});
  g_lt_open = nullptr;
}

static void lt_clear() {
  for (LaunchRec& r : g_lrec) {
    hipEventDestroy(r.e0);
    hipEventDestroy(r.e1);
  }
  g_lrec.clear();
}

}  // namespace nbp

extern "C" {

int nbp_launch_timing(int on) {
  nbp::lt_clear();
  nbp::g_ltiming = on != 0;
  return NBP_OK;
}

int nbp_launch_timing_count(void) { return (int)nbp::g_lrec.size(); }

int nbp_launch_timing_get(int i, char* name, int cap, double* out) {
  NBP_REQUIRE(i >= 0 && i < (int)nbp::g_lrec.size() && name && cap > 0 && out, "nbp_launch_timing_get: bad args");
  const nbp::LaunchRec& r = nbp::g_lrec[i];
  float ms = 0.f;
  if (hipEventSynchronize(r.e1) != hipSuccess || hipEventElapsedTime(&ms, r.e0, r.e1) != hipSuccess) {
    nbp::set_error("nbp_launch_timing_get: event query failed");
    return NBP_ERR_LAUNCH;
  }
  snprintf(name, cap, "%s", r.name);
  out[0] = ms;
  out[1] = r.flops;
  out[2] = r.bytes;
  return NBP_OK;
}

const char* nbp_last_error_string(void) { return nbp::g_err; }

int nbp_version(void) { return NBP_VERSION; }

}  // extern "C"
