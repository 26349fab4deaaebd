// nsgpu_simimpl.hip — the host half of HipSimulatorImpl: DefaultSimulatorImpl's semantics
// (default-simulator-impl.cc:49-353) over the HipBatchScheduler (nsgpu_sched), for events whose
// closures stay on the host.  ns3::HipSimulatorImpl forwards its SimulatorImpl
// virtuals here with ns-3's own EventImpl* as the opaque handle; this C-ABI version carries a
// C callback + argument instead so the same semantics can be exercised without an ns-3 tree.
//   uid allocation from 4, ScheduleDestroy consuming a uid (:235-242), Now/Context/Uid updated
//   before Invoke (:117-131), cancelled events still dequeued (event-impl.cc:34-41), IsExpired's
//   rule (:304-332), Remove of destroy events (:256-268), Stop / Stop (Time) (:167-183).
#include <deque>
#include <vector>
#include "nsgpu_internal.h"

namespace {
struct HostEvent {  // EventImpl: closure + cancel flag (+ refcount held by ids/queue)
  nsgpu_event_fn fn;
  void *user;
  uint64_t arg;
  bool cancelled;
  bool is_stop;
};
}  // namespace

struct nsgpu_sim {
  nsgpu_sched *events = nullptr;
  bool stop = false;
  uint32_t uid = 4;
  uint32_t cur_uid = 0;
  uint64_t cur_ts = 0;
  uint32_t cur_ctx = 0xffffffffu;
  uint64_t dispatched = 0, cancelled = 0;
  std::deque<nsgpu_event_id> destroy_events;
  std::vector<HostEvent *> arena;  // EventImpls live until the simulator is freed (EventId keeps them valid)
  HostEvent *make(nsgpu_event_fn fn, void *user, uint64_t arg, bool is_stop = false) {
    HostEvent *e = new HostEvent{fn, user, arg, false, is_stop};
    arena.push_back(e);
    return e;
  }
  static HostEvent *impl(const nsgpu_event_id &id) { return (HostEvent *)(uintptr_t)id.impl; }
  int insert(uint64_t ts, uint32_t ctx, HostEvent *e, nsgpu_event_id *id) {
    nsgpu_event ev{ts, uid, ctx, (uint64_t)(uintptr_t)e};
    if (id) *id = nsgpu_event_id{(uint64_t)(uintptr_t)e, ts, ctx, uid};
    uid++;
    return nsgpu_sched_insert(events, &ev, 1);
  }
  bool is_expired(const nsgpu_event_id &ev) const {
    if (ev.uid == 2) {
      if (impl(ev) == nullptr || impl(ev)->cancelled) return true;
      for (auto &d : destroy_events)
        if (d.impl == ev.impl && d.ts == ev.ts && d.context == ev.context && d.uid == ev.uid) return false;
      return true;
    }
    return impl(ev) == nullptr || ev.ts < cur_ts || (ev.ts == cur_ts && ev.uid <= cur_uid) || impl(ev)->cancelled;
  }
};

using nsgpu::set_error;

extern "C" {

int nsgpu_sim_create(uint32_t batch, void *stream, nsgpu_sim **out) {
  if (!out) return set_error(NSGPU_EINVAL, "nsgpu_sim_create: null");
  nsgpu_sim *s = new nsgpu_sim();
  int rc = nsgpu_sched_create(batch, stream, &s->events);
  if (rc) {
    delete s;
    return rc;
  }
  *out = s;
  return NSGPU_OK;
}

int nsgpu_sim_free(nsgpu_sim *s) {
  if (!s) return NSGPU_OK;
  nsgpu_sched_destroy(s->events);
  for (HostEvent *e : s->arena) delete e;
  delete s;
  return NSGPU_OK;
}

int nsgpu_sim_schedule(nsgpu_sim *s, int64_t delay, nsgpu_event_fn fn, void *user, uint64_t arg,
                       nsgpu_event_id *id) {  // :188-204
  const int64_t t = delay + (int64_t)s->cur_ts;
  if (t < 0 || t < (int64_t)s->cur_ts) return set_error(NSGPU_EINVAL, "Schedule: negative absolute time");
  return s->insert((uint64_t)t, s->cur_ctx, s->make(fn, user, arg), id);
}

int nsgpu_sim_schedule_with_context(nsgpu_sim *s, uint32_t ctx, int64_t delay, nsgpu_event_fn fn, void *user,
                                    uint64_t arg) {  // :206-219
  return s->insert(s->cur_ts + (uint64_t)delay, ctx, s->make(fn, user, arg), nullptr);
}

int nsgpu_sim_schedule_now(nsgpu_sim *s, nsgpu_event_fn fn, void *user, uint64_t arg, nsgpu_event_id *id) {
  return s->insert(s->cur_ts, s->cur_ctx, s->make(fn, user, arg), id);  // :221-233
}

int nsgpu_sim_schedule_destroy(nsgpu_sim *s, nsgpu_event_fn fn, void *user, uint64_t arg, nsgpu_event_id *id) {
  HostEvent *e = s->make(fn, user, arg);  // :235-242
  nsgpu_event_id d{(uint64_t)(uintptr_t)e, s->cur_ts, 0xffffffffu, 2};
  s->destroy_events.push_back(d);
  s->uid++;
  if (id) *id = d;
  return NSGPU_OK;
}

int nsgpu_sim_is_expired(nsgpu_sim *s, const nsgpu_event_id *id, int *expired) {
  *expired = s->is_expired(*id) ? 1 : 0;
  return NSGPU_OK;
}

int nsgpu_sim_cancel(nsgpu_sim *s, const nsgpu_event_id *id) {  // :292-302
  if (!s->is_expired(*id)) nsgpu_sim::impl(*id)->cancelled = true;
  return NSGPU_OK;
}

int nsgpu_sim_remove(nsgpu_sim *s, const nsgpu_event_id *id) {  // :256-290
  if (id->uid == 2) {
    for (auto i = s->destroy_events.begin(); i != s->destroy_events.end(); i++) {
      if (i->impl == id->impl && i->ts == id->ts && i->context == id->context && i->uid == id->uid) {
        s->destroy_events.erase(i);
        break;
      }
    }
    return NSGPU_OK;
  }
  if (s->is_expired(*id)) return NSGPU_OK;
  nsgpu_event ev{id->ts, id->uid, id->context, id->impl};
  int rc = nsgpu_sched_remove(s->events, &ev);
  if (rc) return rc;
  nsgpu_sim::impl(*id)->cancelled = true;
  return NSGPU_OK;
}

int nsgpu_sim_run(nsgpu_sim *s) {  // :153-165 + ProcessOneEvent :117-131
  s->stop = false;
  for (;;) {
    int empty = 0;
    int rc = nsgpu_sched_is_empty(s->events, &empty);
    if (rc) return rc;
    if (empty || s->stop) break;
    nsgpu_event next;
    if ((rc = nsgpu_sched_remove_next(s->events, &next))) return rc;
    if (next.ts < s->cur_ts) return set_error(NSGPU_ESTATE, "event in the past (ts %llu < now %llu)",
                                              (unsigned long long)next.ts, (unsigned long long)s->cur_ts);
    s->cur_ts = next.ts;
    s->cur_ctx = next.context;
    s->cur_uid = next.uid;
    s->dispatched++;
    HostEvent *e = (HostEvent *)(uintptr_t)next.handle;
    if (e->cancelled) {
      s->cancelled++;
      continue;
    }
    if (e->is_stop) s->stop = true;
    else e->fn(e->user, e->arg);
  }
  return NSGPU_OK;
}

int nsgpu_sim_stop(nsgpu_sim *s) {
  s->stop = true;
  return NSGPU_OK;
}

int nsgpu_sim_stop_at(nsgpu_sim *s, int64_t delay) {  // Stop (Time): Schedule (time, &Simulator::Stop)
  return s->insert(s->cur_ts + (uint64_t)delay, s->cur_ctx, s->make(nullptr, nullptr, 0, true), nullptr);
}

int nsgpu_sim_destroy(nsgpu_sim *s) {  // :76-91
  while (!s->destroy_events.empty()) {
    HostEvent *e = nsgpu_sim::impl(s->destroy_events.front());
    s->destroy_events.pop_front();
    if (!e->cancelled) e->fn(e->user, e->arg);
  }
  return NSGPU_OK;
}

int nsgpu_sim_state(nsgpu_sim *s, uint64_t *now, uint32_t *context, uint64_t *dispatched, uint32_t *next_uid) {
  if (now) *now = s->cur_ts;
  if (context) *context = s->cur_ctx;
  if (dispatched) *dispatched = s->dispatched;
  if (next_uid) *next_uid = s->uid;
  return NSGPU_OK;
}

}  // extern "C"
