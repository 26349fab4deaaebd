// nsgpu_internal.h — host-side helpers shared by the libnsgpu translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include "../../include/nsgpu.h"

namespace nsgpu {

// Sets the thread-local last-error string returned by nsgpu_last_error() and returns `code`.
int set_error(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));

}  // namespace nsgpu

#define NSGPU_HIP(call)                                                                              \
  do {                                                                                              \
    hipError_t e_ = (call);                                                                         \
    if (e_ != hipSuccess)                                                                           \
      return ::nsgpu::set_error(NSGPU_EHIP, "%s:%d %s: %s", __FILE__, __LINE__, #call, hipGetErrorString(e_)); \
  } while (0)
