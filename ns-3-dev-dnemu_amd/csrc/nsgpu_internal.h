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

// DefaultSimulatorImpl's m_uid is a uint32 that wraps to 0 after 0xffffffff (default-simulator-impl.cc:52-56,
// 188-219).  No engine replicates the wrap: a Schedule call that would take uid 0xffffffff (the
// engines' "none" marker) or a wrapped one fails with NSGPU_ERANGE before any such event is dispatched.  The
// counter (the next uid) may reach UID_NEXT_MAX; every uid handed out stays below it.
constexpr uint64_t UID_NEXT_MAX = 0xffffffffull;
inline int uid_range_error(const char *where) {
  return set_error(NSGPU_ERANGE, "%s: the uid counter would pass 0xfffffffe (DefaultSimulatorImpl's uint32 m_uid "
                                 "wraps there, which the engines do not replicate)", where);
}

// The attached p2p engine's first setup uid (its scenario's uid_first, or 4): nsgpu_sim_attach_p2p checks it
// against a start set with nsgpu_sim_set_next_uid.
}  // namespace nsgpu
struct nsgpu_p2p;
struct nsgpu_wifil;
struct nsgpu_wifil_end;
namespace nsgpu {
uint32_t p2p_first_uid(const nsgpu_p2p *h);
// The closed-loop PHY's last epoch's EndReceive with this uid (false: none), and a phy's node (the runtime's
// EndReceive hand-back, nsgpu_sim_wifi_set_end_handler).
bool wifil_epoch_end(const nsgpu_wifil *h, uint32_t uid, nsgpu_wifil_end *out);
uint32_t wifil_node(const nsgpu_wifil *h, uint32_t phy);
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
