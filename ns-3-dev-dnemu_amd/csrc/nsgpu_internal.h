// nsgpu_internal.h — host-side helpers shared by the libnsgpu translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
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

// The RCCL communicator of a partitioned run (one rank per GPU process): nsgpu_comm_init (nsgpu_p2p.hip);
// the partitioned p2p and Wi-Fi engines issue their collectives on it.
struct nsgpu_comm {
  ncclComm_t comm = nullptr;
  int nranks = 0, rank = 0;
};

#define NCCL_TRY(x)                                                                            \
  do {                                                                                         \
    ncclResult_t r_ = (x);                                                                     \
    if (r_ != ncclSuccess) return ::nsgpu::set_error(NSGPU_EHIP, "%s: %s", #x, ncclGetErrorString(r_)); \
  } while (0)
