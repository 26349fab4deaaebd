/*
 * nsgpu_types.h — plain-old-data types shared by the nsgpu C-ABI (include/nsgpu.h)
 * and its test checker (oracle/).  No torch types, no C++ across the ABI.
 *
 * Event key layout follows ns-3's Scheduler::EventKey
 *   (reference: src/core/model/scheduler.h:58-63):
 *     uint64 m_ts; uint32 m_uid; uint32 m_context
 * and the ordering is (ts, uid) ONLY (scheduler.h:105-121) — context is payload.
 */
#ifndef NSGPU_TYPES_H
#define NSGPU_TYPES_H

#include <stdint.h>

#if defined(__HIP__)
#define NSGPU_HD __host__ __device__
#else
#define NSGPU_HD
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* Scheduler::EventKey + Scheduler::Event (scheduler.h:58-68): 24 bytes. */
typedef struct nsgpu_event {
  uint64_t ts;       /* absolute time, in Time resolution units (ns) */
  uint32_t uid;      /* global schedule counter, starts at 4 (default-simulator-impl.cc:52-56) */
  uint32_t context;  /* node id, 0xffffffff = no node (default-simulator-impl.cc:60) */
  uint64_t handle;   /* opaque EventImpl* (host closure) — never dereferenced on device */
} nsgpu_event;

/* ns-3 EventId (event-id.h:46-83): (impl, ts, context, uid). */
typedef struct nsgpu_event_id {
  uint64_t impl;
  uint64_t ts;
  uint32_t context;
  uint32_t uid;
} nsgpu_event_id;

/* Propagation loss model kinds (src/propagation/model/propagation-loss-model.cc). */
enum nsgpu_loss_kind {
  NSGPU_LOSS_NONE = 0,
  NSGPU_LOSS_LOG_DISTANCE = 1, /* p0 = exponent, p1 = reference distance, p2 = reference loss  (:464-491) */
  NSGPU_LOSS_FRIIS = 2,        /* p0 = lambda, p1 = system loss, p2 = min distance            (:197-239) */
  NSGPU_LOSS_FIXED_RSS = 3,    /* p0 = fixed rss dBm                                          (:718-723) */
  NSGPU_LOSS_RANGE = 4         /* p0 = max range m; beyond it -1000 dBm                       (:822-834) */
};

typedef struct nsgpu_loss_model {
  int32_t kind;
  int32_t pad_;
  double p0, p1, p2;
} nsgpu_loss_model;

/* A PropagationLossModel chain (PropagationLossModel::CalcRxPower, :64-74): up to 4 links. */
#define NSGPU_MAX_LOSS_CHAIN 4
typedef struct nsgpu_loss_chain {
  int32_t n;
  int32_t pad_;
  nsgpu_loss_model m[NSGPU_MAX_LOSS_CHAIN];
} nsgpu_loss_chain;

/* Result record of one broadcast fan-out receiver (YansWifiChannel::Send, yans-wifi-channel.cc:77-115):
 * the ScheduleWithContext(dstNode, delay, &YansWifiChannel::Receive, this, j, copy, rxPowerDbm, ...) call. */
typedef struct nsgpu_rx_record {
  uint64_t ts;       /* now + delay */
  uint32_t uid;      /* uid_base + rank among surviving receivers (list order) */
  uint32_t context;  /* destination node id */
  uint32_t phy;      /* index j into the channel's phy list */
  uint32_t pad_;
  double rx_dbm;     /* CalcRxPower (txPowerDbm, sender, receiver) */
} nsgpu_rx_record;

/* Order-sensitive digest of a dispatch sequence: sum over k of mix(k, ts_k, uid_k).
 * Used to compare long dispatch orders (pop order) without moving whole logs. */
NSGPU_HD static inline uint64_t nsgpu_mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
NSGPU_HD static inline uint64_t nsgpu_dispatch_digest_term(uint64_t rank, uint64_t ts, uint32_t uid) {
  return nsgpu_mix64(rank * 0x9e3779b97f4a7c15ULL ^ nsgpu_mix64(ts ^ ((uint64_t)uid << 40) ^ (uint64_t)uid));
}

#ifdef __cplusplus
}
#endif
#endif /* NSGPU_TYPES_H */
