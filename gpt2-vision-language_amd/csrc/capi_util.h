// Host-side helpers for the libgvl C-ABI: thread-local error text, launch checks.
#pragma once
#include <hip/hip_runtime.h>
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
