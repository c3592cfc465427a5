// Thread-local error reporting shared by every libgvl entry point.
#include "capi_util.h"
#include "../../include/gvl.h"

#include <string>

namespace {
thread_local std::string g_last_error;
thread_local hipEvent_t g_ev_start = nullptr, g_ev_stop = nullptr;
}

namespace gvl {
void set_error(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
}

int num_cus() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  if (cached[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    cached[dev] = n;
  }
  return cached[dev];
}

bool take_launch_events(hipEvent_t* start, hipEvent_t* stop) {
  if (!g_ev_start || !g_ev_stop) return false;
  *start = g_ev_start;
  *stop = g_ev_stop;
  g_ev_start = g_ev_stop = nullptr;
  return true;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: HIP launch failed: %s", what, hipGetErrorString(e));
    return -2;
  }
  return 0;
}
}  // namespace gvl

extern "C" {
const char* gvl_last_error(void) { return g_last_error.c_str(); }
int gvl_abi_version(void) { return GVL_ABI_VERSION; }
int gvl_set_launch_events(void* start, void* stop) {
  g_ev_start = reinterpret_cast<hipEvent_t>(start);
  g_ev_stop = reinterpret_cast<hipEvent_t>(stop);
  return 0;
}
}
