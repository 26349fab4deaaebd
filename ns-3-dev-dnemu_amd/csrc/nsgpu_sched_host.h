// nsgpu_sched_host.h — HipBatchScheduler's state and its per-event host paths (shared by
// nsgpu_sched.hip, which owns the device side, and nsgpu_simimpl.hip, which calls the per-event paths
// inline instead of through the C-ABI).
//
// Semantics are MapScheduler's (map-scheduler.cc:51-100): Insert, IsEmpty, PeekNext, RemoveNext,
// Remove, ordered by (ts, uid) (scheduler.h:105-121).  Layout, two levels:
//   * device: one sorted array D of 24-byte Scheduler::Event records {ts, uid, context, impl} in HBM;
//   * host:   the FRONT — the next B events of D, copied out in one transfer into pinned memory and
//             consumed by an index — plus a binary heap H for inserts whose key is below the front's
//             last key (they pop in order with the front), and the STAGE, a pinned ring of every other
//             insert, appended to with one store.
// When the front and H run dry, one refill (sched_refill) sorts the stage on the device (the sort
// kernel reads the pinned ring directly), merges it into D and writes the next B merged events
// straight into the pinned front: one device round trip per B dispatches.  B adapts to the measured
// round trip R and the pending count P: an insert lands in H with probability ~B / 2P, so the per-event
// cost R / B + c_heap * B / P is smallest at B = sqrt (R * P / c_heap).  Removes are lazy: the uid is
// recorded and the event is dropped when it surfaces (uids are unique, scheduler.h:58-63).
#pragma once
#include <algorithm>
#include <unordered_set>
#include <vector>
#include "nsgpu_internal.h"

namespace nsgpu {

__host__ __device__ __forceinline__ bool ev_less(const nsgpu_event &a, const nsgpu_event &b) {
  return a.ts < b.ts || (a.ts == b.ts && a.uid < b.uid);
}

}  // namespace nsgpu

struct nsgpu_sched {
  hipStream_t stream = nullptr;
  uint32_t batch_fixed = 0;  // 0: adaptive front size
  // device: live events are d_main[d_head, d_n)
  nsgpu_event *d_main = nullptr, *d_tmp = nullptr, *d_stage2 = nullptr, *d_stage3 = nullptr;
  uint64_t cap = 0, tmp_cap = 0, stage2_cap = 0, stage3_cap = 0;
  uint64_t d_head = 0, d_n = 0;
  // pinned host buffers (device-visible): the front and the stage ring
  nsgpu_event *h_front = nullptr, *h_stage = nullptr;
  uint64_t front_cap = 0, front_n = 0, front_i = 0;
  uint64_t stage_cap = 0, stage_n = 0;
  nsgpu_event front_bound{};  // the largest key copied to the front
  std::vector<nsgpu_event> heap;
  std::unordered_set<uint32_t> removed;
  uint64_t size = 0;
  // adaptivity / statistics
  double refill_ns = 30000.0;  // running estimate of one refill's wall time
  uint64_t refills = 0;
};

namespace nsgpu {

int sched_refill(nsgpu_sched *s);       // nsgpu_sched.hip: flush the stage, copy the next front out
int sched_grow_stage(nsgpu_sched *s);   // nsgpu_sched.hip: double the pinned stage ring

struct SchedHeapGreater {
  bool operator()(const nsgpu_event &a, const nsgpu_event &b) const { return ev_less(b, a); }
};

// Scheduler::Insert of one event.
__host__ inline int sched_insert1(nsgpu_sched *s, const nsgpu_event &ev) {
  const bool active = s->front_i < s->front_n || !s->heap.empty();
  if (active && ev_less(ev, s->front_bound)) {  // below a key already on the host: pops in order with it
    s->heap.push_back(ev);
    std::push_heap(s->heap.begin(), s->heap.end(), SchedHeapGreater());
  } else {
    if (s->stage_n == s->stage_cap) {
      const int rc = sched_grow_stage(s);
      if (rc) return rc;
    }
    s->h_stage[s->stage_n++] = ev;
  }
  s->size++;
  return NSGPU_OK;
}

// Pops (pop) or peeks the smallest live event into *out.  Returns 1 if found; *rc carries an error.
__host__ inline int sched_next(nsgpu_sched *s, nsgpu_event *out, bool pop, int *rc) {
  *rc = NSGPU_OK;
  for (;;) {
    const bool hf = s->front_i < s->front_n;
    const bool hh = !s->heap.empty();
    if (!hf && !hh) {
      if (s->stage_n == 0 && s->d_n == s->d_head) return 0;
      if ((*rc = sched_refill(s))) return 0;
      continue;
    }
    const bool from_front = hf && (!hh || ev_less(s->h_front[s->front_i], s->heap.front()));
    const nsgpu_event e = from_front ? s->h_front[s->front_i] : s->heap.front();
    bool dead = false;
    if (!s->removed.empty()) {
      auto it = s->removed.find(e.uid);
      if (it != s->removed.end()) {
        dead = true;
        s->removed.erase(it);
      }
    }
    if (dead || pop) {
      if (from_front) {
        s->front_i++;
      } else {
        std::pop_heap(s->heap.begin(), s->heap.end(), SchedHeapGreater());
        s->heap.pop_back();
      }
    }
    if (dead) continue;
    *out = e;
    return 1;
  }
}

__host__ inline int sched_remove_next1(nsgpu_sched *s, nsgpu_event *out) {
  int rc;
  if (!sched_next(s, out, true, &rc)) return rc ? rc : set_error(NSGPU_ESTATE, "RemoveNext on an empty scheduler");
  s->size--;
  return NSGPU_OK;
}

}  // namespace nsgpu
