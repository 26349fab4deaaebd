// nsgpu_simimpl.hip — the host-closure runtime behind ns3::HipSimulatorImpl: events whose closures
// stay on the host (EventImpl*), kept in the device-resident HipBatchScheduler (nsgpu_sched), dispatched
// in WINDOWS, optionally interleaved with a GPU-resident p2p engine in one (ts, uid) order.
//
// Contract (the reference semantics it keeps — default-simulator-impl.cc:49-353 — are listed so the
// parity tests can cite them): uids from 4, ScheduleDestroy consumes one (:235-242); Now / Context / uid
// are set before a closure runs (:117-131); a cancelled event is still dequeued and counted
// (event-impl.cc:34-41); IsExpired's rule (:304-332); Stop / Stop (Time) (:167-183).
//
// Windows (nsgpu_sim_pop_window): with host closures only, a window is every pending event of the
// smallest timestamp — an event a closure schedules has a larger uid, so it sorts after the whole
// window, and events the window's closures Remove are skipped.  With an attached engine
// (nsgpu_sim_attach_p2p) the engine first dispatches every device event below the next host event's
// key (nsgpu_p2p_advance pauses its window pipeline there), then that host event is the window.  The
// runtime owns the uid counter and the dispatch rank; the engine continues from them at every advance.
#include <deque>
#include <vector>
#include <unordered_set>
#include "nsgpu_internal.h"

namespace {
struct HostEvent {  // a C-callback closure + cancel flag (nsgpu_sim_schedule*); raw handles are the caller's
  nsgpu_event_fn fn;
  void *user;
  uint64_t arg;
  bool cancelled;
  bool is_stop;
};
constexpr uint64_t RAW = 1;  // handle tag: a caller-owned handle (nsgpu_sim_insert), not a HostEvent
}  // namespace

struct nsgpu_sim {
  nsgpu_sched *events = nullptr;
  nsgpu_p2p *p2p = nullptr;
  void *stream = nullptr;
  bool stop = false, ended = false;
  uint32_t uid = 4;
  uint32_t cur_uid = 0;
  uint64_t cur_ts = 0;
  uint32_t cur_ctx = 0xffffffffu;
  uint64_t dispatched = 0, cancelled = 0, digest = 0, host_dispatched = 0;
  uint64_t *log_ts = nullptr;  // optional pop-order log of the host dispatches (global ranks)
  uint32_t *log_uid = nullptr, *log_ctx = nullptr;
  uint64_t log_cap = 0;
  std::deque<nsgpu_event_id> destroy_events;
  std::vector<HostEvent *> arena;              // live until the runtime is freed (EventIds stay valid)
  std::vector<nsgpu_event> win;                // the current window
  size_t win_next = 0;                         // first event of it not yet begun
  std::unordered_set<uint32_t> win_removed;    // window events a closure removed
  uint32_t p2p_seq = 0, p2p_seq_uid = 0;       // trace sink calls the running closure made on the engine
  HostEvent *make(nsgpu_event_fn fn, void *user, uint64_t arg, bool is_stop = false) {
    HostEvent *e = new HostEvent{fn, user, arg, false, is_stop};
    arena.push_back(e);
    return e;
  }
  static HostEvent *impl(const nsgpu_event_id &id) { return (HostEvent *)(uintptr_t)id.impl; }
  int insert(uint64_t ts, uint32_t ctx, uint64_t handle, uint32_t *out_uid) {
    nsgpu_event ev{ts, uid, ctx, handle};
    if (out_uid) *out_uid = uid;
    uid++;
    return nsgpu_sched_insert(events, &ev, 1);
  }
  bool in_window(uint32_t u) const {
    for (size_t i = win_next; i < win.size(); i++)
      if (win[i].uid == u) return true;
    return false;
  }
  // the time part of IsExpired (:304-332): the event's key is not after the one being dispatched
  bool key_expired(uint64_t ts, uint32_t u) const { return ts < cur_ts || (ts == cur_ts && u <= cur_uid); }
  bool is_expired(const nsgpu_event_id &ev) const {
    if (ev.uid == 2) {
      if (impl(ev) == nullptr || impl(ev)->cancelled) return true;
      for (auto &d : destroy_events)
        if (d.impl == ev.impl && d.ts == ev.ts && d.context == ev.context && d.uid == ev.uid) return false;
      return true;
    }
    return impl(ev) == nullptr || key_expired(ev.ts, ev.uid) || impl(ev)->cancelled;
  }
};

using nsgpu::set_error;

extern "C" {

int nsgpu_sim_create(uint32_t batch, void *stream, nsgpu_sim **out) {
  if (!out) return set_error(NSGPU_EINVAL, "nsgpu_sim_create: null");
  nsgpu_sim *s = new nsgpu_sim();
  s->stream = stream;
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

// The GPU-resident p2p engine joins this runtime's order: its setup-time events hold uids 4.. (their
// Schedule calls precede the program's), so the runtime continues from the engine's post-setup uid.
int nsgpu_sim_attach_p2p(nsgpu_sim *s, nsgpu_p2p *h) {
  if (!s || !h) return set_error(NSGPU_EINVAL, "nsgpu_sim_attach_p2p: null");
  uint64_t n = 0;
  nsgpu_sched_size(s->events, &n);
  if (n || s->dispatched || s->uid != 4) return set_error(NSGPU_ESTATE, "nsgpu_sim_attach_p2p: attach before scheduling");
  uint32_t u = 0;
  int rc = nsgpu_p2p_setup_uid(h, &u);
  if (rc) return rc;
  s->p2p = h;
  s->uid = u;
  return NSGPU_OK;
}

int nsgpu_sim_set_log(nsgpu_sim *s, uint64_t *ts, uint32_t *uid, uint32_t *ctx, uint64_t cap) {
  if (!s) return set_error(NSGPU_EINVAL, "nsgpu_sim_set_log: null");
  s->log_ts = ts, s->log_uid = uid, s->log_ctx = ctx, s->log_cap = (ts && uid && ctx) ? cap : 0;
  return NSGPU_OK;
}

int nsgpu_sim_schedule(nsgpu_sim *s, int64_t delay, nsgpu_event_fn fn, void *user, uint64_t arg,
                       nsgpu_event_id *id) {  // :188-204
  const int64_t t = delay + (int64_t)s->cur_ts;
  if (t < 0 || t < (int64_t)s->cur_ts) return set_error(NSGPU_EINVAL, "Schedule: negative absolute time");
  HostEvent *e = s->make(fn, user, arg);
  uint32_t u;
  const int rc = s->insert((uint64_t)t, s->cur_ctx, (uint64_t)(uintptr_t)e, &u);
  if (id) *id = nsgpu_event_id{(uint64_t)(uintptr_t)e, (uint64_t)t, s->cur_ctx, u};
  return rc;
}

int nsgpu_sim_schedule_with_context(nsgpu_sim *s, uint32_t ctx, int64_t delay, nsgpu_event_fn fn, void *user,
                                    uint64_t arg) {  // :206-219
  return s->insert(s->cur_ts + (uint64_t)delay, ctx, (uint64_t)(uintptr_t)s->make(fn, user, arg), nullptr);
}

int nsgpu_sim_schedule_now(nsgpu_sim *s, nsgpu_event_fn fn, void *user, uint64_t arg, nsgpu_event_id *id) {
  return nsgpu_sim_schedule(s, 0, fn, user, arg, id);  // :221-233
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
  nsgpu_sim::impl(*id)->cancelled = true;
  return nsgpu_sim_remove_key(s, id->ts, id->uid, id->context, id->impl);
}

// ---- raw handles (ns3::HipSimulatorImpl: the handle is an EventImpl*, never dereferenced here) ----
int nsgpu_sim_insert(nsgpu_sim *s, uint64_t ts, uint32_t ctx, uint64_t handle, uint32_t *uid) {
  if (!s || (handle & RAW)) return set_error(NSGPU_EINVAL, "nsgpu_sim_insert: null runtime or odd handle");
  if (ts < s->cur_ts) return set_error(NSGPU_EINVAL, "nsgpu_sim_insert: event in the past");
  return s->insert(ts, ctx, handle | RAW, uid);
}

int nsgpu_sim_consume_uid(nsgpu_sim *s, uint32_t *uid) {  // ScheduleDestroy's uid (:235-242)
  if (!s) return set_error(NSGPU_EINVAL, "nsgpu_sim_consume_uid: null");
  if (uid) *uid = s->uid;
  s->uid++;
  return NSGPU_OK;
}

int nsgpu_sim_key_expired(nsgpu_sim *s, uint64_t ts, uint32_t uid, int *expired) {
  if (!s || !expired) return set_error(NSGPU_EINVAL, "nsgpu_sim_key_expired: null");
  *expired = s->key_expired(ts, uid) ? 1 : 0;
  return NSGPU_OK;
}

// Scheduler::Remove of a pending event (the caller checked it is not expired).
int nsgpu_sim_remove_key(nsgpu_sim *s, uint64_t ts, uint32_t uid, uint32_t ctx, uint64_t handle) {
  if (!s) return set_error(NSGPU_EINVAL, "nsgpu_sim_remove_key: null");
  if (s->in_window(uid)) {  // popped with the current window, not dispatched yet
    s->win_removed.insert(uid);
    return NSGPU_OK;
  }
  nsgpu_event ev{ts, uid, ctx, handle};
  return nsgpu_sched_remove(s->events, &ev);
}

// The next window (see the file header).  *n = 0: nothing is left to dispatch (the queue is empty and
// the attached engine, if any, has run out), or a Stop was dispatched.
int nsgpu_sim_pop_window(nsgpu_sim *s, nsgpu_event *out, uint32_t cap, uint32_t *n) {
  if (!s || !out || !n || cap == 0) return set_error(NSGPU_EINVAL, "nsgpu_sim_pop_window: bad arguments");
  *n = 0;
  s->win.clear();
  s->win_next = 0;
  s->win_removed.clear();
  if (s->stop || s->ended) return NSGPU_OK;
  int rc;
  nsgpu_event e;
  uint64_t size = 0;
  if ((rc = nsgpu_sched_size(s->events, &size))) return rc;
  if (s->p2p) {
    bool have = false;
    if (size) {
      if ((rc = nsgpu_sched_peek_next(s->events, &e))) return rc;
      have = true;
    }
    int ended = 0;
    rc = nsgpu_p2p_advance(s->p2p, have ? e.ts : ~0ull, have ? e.uid : 0u, &s->uid, &s->dispatched, &ended, s->stream);
    if (rc) return rc;
    if (ended) {  // the device dispatched Simulator::Stop, or nothing is pending anywhere
      s->ended = true;
      return NSGPU_OK;
    }
    if (!have) return NSGPU_OK;
    if ((rc = nsgpu_sched_remove_next(s->events, &e))) return rc;
    out[0] = e;
    s->win.push_back(e);
    *n = 1;
    return NSGPU_OK;
  }
  if (!size) return NSGPU_OK;
  if ((rc = nsgpu_sched_remove_next(s->events, &e))) return rc;
  out[0] = e;
  s->win.push_back(e);
  uint32_t k = 1;
  while (k < cap) {
    if ((rc = nsgpu_sched_size(s->events, &size))) return rc;
    if (!size) break;
    nsgpu_event f;
    if ((rc = nsgpu_sched_peek_next(s->events, &f))) return rc;
    if (f.ts != e.ts) break;
    if ((rc = nsgpu_sched_remove_next(s->events, &f))) return rc;
    out[k++] = f;
    s->win.push_back(f);
  }
  *n = k;
  return NSGPU_OK;
}

// Window event i is being dispatched: 0 = run its closure, 1 = a closure of this window removed it
// (skip it), 2 = a Stop was dispatched before it (it stays pending).  Sets Now / Context / the
// current uid and accounts the dispatch (rank, digest, log) for a dispatched one.
int nsgpu_sim_begin(nsgpu_sim *s, const nsgpu_event *e, int *skip) {
  if (!s || !e || !skip) return set_error(NSGPU_EINVAL, "nsgpu_sim_begin: null");
  if (s->win_next < s->win.size() && s->win[s->win_next].uid == e->uid) s->win_next++;
  if (s->win_removed.count(e->uid)) {
    *skip = 1;
    return NSGPU_OK;
  }
  if (s->stop) {
    *skip = 2;
    return nsgpu_sched_insert(s->events, e, 1);
  }
  *skip = 0;
  s->cur_ts = e->ts;
  s->cur_ctx = e->context;
  s->cur_uid = e->uid;
  const uint64_t rank = s->dispatched++;
  s->host_dispatched++;
  s->digest += nsgpu_dispatch_digest_term(rank, e->ts, e->uid);
  if (rank < s->log_cap) {
    s->log_ts[rank] = e->ts;
    s->log_uid[rank] = e->uid;
    s->log_ctx[rank] = e->context;
  }
  return NSGPU_OK;
}

int nsgpu_sim_run(nsgpu_sim *s) {  // Run (:153-165): windows of closures (and device events)
  s->stop = false;
  std::vector<nsgpu_event> w(1024);
  for (;;) {
    uint32_t n = 0;
    int rc = nsgpu_sim_pop_window(s, w.data(), (uint32_t)w.size(), &n);
    if (rc) return rc;
    if (n == 0) break;
    for (uint32_t i = 0; i < n; i++) {
      int skip = 0;
      if ((rc = nsgpu_sim_begin(s, &w[i], &skip))) return rc;
      if (skip) continue;
      if (w[i].handle & RAW) return set_error(NSGPU_ESTATE, "nsgpu_sim_run: a raw handle (dispatch it with nsgpu_sim_pop_window)");
      HostEvent *e = (HostEvent *)(uintptr_t)w[i].handle;
      if (e->cancelled) {  // still dequeued and counted (event-impl.cc:34-41)
        s->cancelled++;
        continue;
      }
      if (e->is_stop) s->stop = true;
      else e->fn(e->user, e->arg);
    }
  }
  return NSGPU_OK;
}

int nsgpu_sim_stop(nsgpu_sim *s) {
  s->stop = true;
  return NSGPU_OK;
}

int nsgpu_sim_stop_at(nsgpu_sim *s, int64_t delay) {  // Stop (Time): Schedule (time, &Simulator::Stop)
  return s->insert(s->cur_ts + (uint64_t)delay, s->cur_ctx, (uint64_t)(uintptr_t)s->make(nullptr, nullptr, 0, true),
                   nullptr);
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

// Next () / IsFinished (): the time of the next host event (device events of an attached engine
// are not counted: they never outlive Run); *empty = 1 when none is pending.
int nsgpu_sim_next(nsgpu_sim *s, uint64_t *ts, int *empty) {
  if (!s || !ts || !empty) return set_error(NSGPU_EINVAL, "nsgpu_sim_next: null");
  uint64_t n = 0;
  int rc = nsgpu_sched_size(s->events, &n);
  if (rc) return rc;
  *empty = n == 0;
  *ts = 0;
  if (n) {
    nsgpu_event e;
    if ((rc = nsgpu_sched_peek_next(s->events, &e))) return rc;
    *ts = e.ts;
  }
  return NSGPU_OK;
}

// Stop () sets the flag that ends the current Run at the next dispatch; Run clears it (:153-165).
int nsgpu_sim_set_stop(nsgpu_sim *s, int stop) {
  if (!s) return set_error(NSGPU_EINVAL, "nsgpu_sim_set_stop: null");
  s->stop = stop != 0;
  return NSGPU_OK;
}

// DoDispose: hands back up to `cap` pending events (not dispatched) so the caller can release them.
int nsgpu_sim_drain(nsgpu_sim *s, nsgpu_event *out, uint32_t cap, uint32_t *n) {
  if (!s || !out || !n) return set_error(NSGPU_EINVAL, "nsgpu_sim_drain: null");
  *n = 0;
  for (uint32_t k = 0; k < cap; k++) {
    uint64_t size = 0;
    int rc = nsgpu_sched_size(s->events, &size);
    if (rc) return rc;
    if (!size) break;
    if ((rc = nsgpu_sched_remove_next(s->events, &out[k]))) return rc;
    *n = k + 1;
  }
  return NSGPU_OK;
}

int nsgpu_sim_current_uid(nsgpu_sim *s, uint32_t *uid) {
  if (!s || !uid) return set_error(NSGPU_EINVAL, "nsgpu_sim_current_uid: null");
  *uid = s->cur_uid;
  return NSGPU_OK;
}

int nsgpu_sim_host_stats(nsgpu_sim *s, uint64_t *host_dispatched, uint64_t *cancelled, uint64_t *digest) {
  if (!s) return set_error(NSGPU_EINVAL, "nsgpu_sim_host_stats: null");
  if (host_dispatched) *host_dispatched = s->host_dispatched;
  if (cancelled) *cancelled = s->cancelled;
  if (digest) *digest = s->digest;
  return NSGPU_OK;
}

// A host closure's UdpSocket::Send on application `app` of the attached engine (now, with the uid
// of the closure being dispatched; its Schedule calls take the runtime's next uids).
int nsgpu_sim_p2p_send(nsgpu_sim *s, uint32_t app) {
  if (!s || !s->p2p) return set_error(NSGPU_ESTATE, "nsgpu_sim_p2p_send: no engine attached");
  uint32_t seq = s->p2p_seq_uid == s->cur_uid ? s->p2p_seq : 0;
  int rc = nsgpu_p2p_inject_send(s->p2p, app, s->cur_ts, s->cur_uid, s->cur_ctx, &s->uid, &seq, s->stream);
  s->p2p_seq_uid = s->cur_uid;
  s->p2p_seq = seq;
  return rc;
}

}  // extern "C"
