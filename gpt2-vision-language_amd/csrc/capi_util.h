// Host-side helpers for the libgvl C-ABI: thread-local error text, launch checks.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdint.h>

namespace gvl {
void set_error(const char* fmt, ...);
int check_launch(const char* what);
int num_cus();  // compute units of the current device (cached per device)
inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }
inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }
inline bool aligned8(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 7u) == 0; }

// Kernel timing armed by gvl_set_launch_events: the next launch_timed() binds the pair to
// its own dispatch (hipExtLaunchKernelGGL), so elapsed(start, stop) is the kernel's execution
// interval as the dispatch records it (the source rocprofv3's kernel trace reads), not the
// span between two stream markers around it.
bool take_launch_events(hipEvent_t* start, hipEvent_t* stop);

template <typename K, typename... Args>
inline void launch_timed(K kernel, dim3 grid, dim3 block, uint32_t lds, hipStream_t s,
                         Args... args) {
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (take_launch_events(&e0, &e1))
    hipExtLaunchKernelGGL(kernel, grid, block, lds, s, e0, e1, 0, args...);
  else
    hipLaunchKernelGGL(kernel, grid, block, lds, s, args...);
}
}  // namespace gvl

#define GVL_REQUIRE(cond, ...)          \
  do {                                  \
    if (!(cond)) {                      \
      gvl::set_error(__VA_ARGS__);      \
      return -1;                        \
    }                                   \
  } while (0)

#define GVL_LAUNCH_CHECK(name) \
  do {                         \
    int _rc = gvl::check_launch(name); \
    if (_rc) return _rc;       \
  } while (0)
