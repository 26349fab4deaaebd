// nsgpu_simimpl.hip — the host-closure runtime behind ns3::HipSimulatorImpl: events whose closures
// stay on the host (EventImpl*), kept in the device-resident HipBatchScheduler (nsgpu_sched), dispatched
// in WINDOWS, optionally interleaved with a GPU-resident p2p engine or the closed-loop Wi-Fi PHY
// (nsgpu_wifil) in one (ts, uid) order.
//
// Contract (the reference semantics it keeps — default-simulator-impl.cc:49-353 — are listed so the
// parity tests can cite them): uids from 4, ScheduleDestroy consumes one (:235-242); Now / Context / uid
// are set before a closure runs (:117-131); a cancelled event is still dequeued and counted
// (event-impl.cc:34-41); IsExpired's rule (:304-332); Stop / Stop (Time) (:167-183); IsFinished is
// "queue empty or stopped" (:133-137) and RunOneEvent dispatches one event whatever the stop flag says
// (:167-170); Destroy pops the destroy list from the front until it is empty, so a destroy event
// scheduled or removed by a destroy closure is honoured (:79-92, :256-268).
//
// Windows (nsgpu_sim_pop_window): with host closures only, a window is every pending event of the
// smallest timestamp — an event a closure schedules has a larger uid, so it sorts after the whole
// window, and events the window's closures Remove are skipped.  With an attached engine
// (nsgpu_sim_attach_p2p) the engine first dispatches every device event below the next host event's
// key (nsgpu_p2p_advance pauses its window pipeline there), then that host event is the window.  The
// runtime owns the uid counter and the dispatch rank; the engine continues from them at every advance.
//
// Inserts go straight into the scheduler's pinned stage ring (nsgpu_sched_host.h: one store each, no
// device call); the ring is sorted and merged on the device once per front refill.  C-callback closures
// live in a slab whose slots are recycled at dispatch / removal; an EventId names a slot and its
// generation, so an id of a recycled slot reads as expired.
#include <deque>
#include <vector>
#include <unordered_set>
#include "nsgpu_sched_host.h"

namespace {
struct HostEvent {  // a C-callback closure + cancel flag (nsgpu_sim_schedule*); raw handles are the caller's
  nsgpu_event_fn fn;
  void *user;
  uint64_t arg;
  uint32_t gen;  // bumped when the slot is released
  bool cancelled, is_stop, live;
};
struct DestroyEv {  // an entry of the destroy list (DefaultSimulatorImpl::m_destroyEvents)
  uint64_t handle;  // slab handle, or a caller's raw handle with RAW set
  uint64_t ts;      // the EventId's ts (ScheduleDestroy's Now)
};
constexpr uint64_t RAW = 1;  // handle tag: a caller-owned handle (nsgpu_sim_insert), not a HostEvent
}  // namespace

struct nsgpu_sim {
  nsgpu_sched *events = nullptr;
  nsgpu_p2p *p2p = nullptr;
  nsgpu_wifil *wifi = nullptr;  // closed-loop Wi-Fi PHY (nsgpu_sim_attach_wifi)
  void *stream = nullptr;
  bool stop = false, ended = false, dev_stopped = false;
  uint32_t uid = 4;
  uint32_t uid_first = 4;  // m_uid before the program's first Schedule call (nsgpu_sim_set_next_uid)
  bool uid_set = false;    // uid_first was set explicitly (an attached engine must start there too)
  nsgpu_wifi_end_fn wifi_end_fn = nullptr;  // the EndReceive hand-back (nsgpu_sim_wifi_set_end_handler)
  void *wifi_end_user = nullptr;
  uint64_t wifi_listen_n = 0;                // phys listened to
  std::vector<uint8_t> lis_on;
  bool uid_spent = false;  // a Schedule call hit the uid limit (a closure's call fails; the run then fails too)
  uint32_t cur_uid = 0;
  uint64_t cur_ts = 0;
  uint32_t cur_ctx = 0xffffffffu;
  uint64_t dispatched = 0, cancelled = 0, digest = 0, host_dispatched = 0;
  uint64_t *log_ts = nullptr;  // optional pop-order log of the host dispatches (global ranks)
  uint32_t *log_uid = nullptr, *log_ctx = nullptr;
  uint64_t log_cap = 0;
  std::deque<DestroyEv> destroy_events;
  std::vector<HostEvent> slab;                 // C-callback closures; handle = (gen << 32 | slot) << 1
  std::vector<uint32_t> free_slots;
  std::vector<nsgpu_event> win;                // the current window
  size_t win_next = 0;                         // first event of it not yet begun
  std::unordered_set<uint32_t> win_removed;    // window events a closure removed
  uint32_t p2p_seq = 0, p2p_seq_uid = 0;       // trace sink calls the running closure made on the engine

  uint64_t make(nsgpu_event_fn fn, void *user, uint64_t arg, bool is_stop = false) {
    uint32_t i;
    if (!free_slots.empty()) {
      i = free_slots.back();
      free_slots.pop_back();
    } else {
      i = (uint32_t)slab.size();
      slab.push_back(HostEvent{nullptr, nullptr, 0, 1, false, false, false});
    }
    HostEvent &e = slab[i];
    e.fn = fn, e.user = user, e.arg = arg, e.cancelled = false, e.is_stop = is_stop, e.live = true;
    return (((uint64_t)e.gen << 32) | i) << 1;
  }
  // the live closure a slab handle names, or null (released slot, other generation, raw handle)
  HostEvent *get(uint64_t handle) {
    if (handle & RAW) return nullptr;
    const uint32_t i = (uint32_t)(handle >> 1), g = (uint32_t)(handle >> 33);
    if (i >= slab.size() || !slab[i].live || slab[i].gen != g) return nullptr;
    return &slab[i];
  }
  void release(uint64_t handle) {
    HostEvent *e = get(handle);
    if (!e) return;
    e->live = false;
    e->gen++;
    free_slots.push_back((uint32_t)(handle >> 1));
  }
  int spent(const char *where) {
    uid_spent = true;
    return nsgpu::uid_range_error(where);
  }
  int insert(uint64_t ts, uint32_t ctx, uint64_t handle, uint32_t *out_uid) {
    if (uid >= nsgpu::UID_NEXT_MAX) return spent("nsgpu_sim: Schedule");
    const nsgpu_event ev{ts, uid, ctx, handle};
    if (out_uid) *out_uid = uid;
    uid++;
    return nsgpu::sched_insert1(events, ev);
  }
  bool in_window(uint32_t u) const {
    for (size_t i = win_next; i < win.size(); i++)
      if (win[i].uid == u) return true;
    return false;
  }
  // the time part of IsExpired (:304-332): the event's key is not after the one being dispatched
  bool key_expired(uint64_t ts, uint32_t u) const { return ts < cur_ts || (ts == cur_ts && u <= cur_uid); }
  bool destroy_pending(uint64_t handle, uint64_t ts) const {
    for (const DestroyEv &d : destroy_events)
      if (d.handle == handle && d.ts == ts) return true;
    return false;
  }
  bool is_expired(const nsgpu_event_id &ev) {
    HostEvent *e = get(ev.impl);
    if (ev.uid == 2) return e == nullptr || e->cancelled || !destroy_pending(ev.impl, ev.ts);
    return e == nullptr || key_expired(ev.ts, ev.uid) || e->cancelled;
  }
  // the attached engine's pending events (Next / IsFinished)
  int device_pending(uint64_t *n, uint64_t *next_ts) {
    *n = 0;
    *next_ts = ~0ull;
    if (wifi) return nsgpu_wifil_pending(wifi, n, next_ts);
    if (!p2p || ended) return NSGPU_OK;
    int stopped = 0;
    return nsgpu_p2p_pending(p2p, n, next_ts, &stopped, stream);
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
  delete s;
  return NSGPU_OK;
}

// The GPU-resident p2p engine joins this runtime's order: its setup-time events hold uids 4.. (their
// Schedule calls precede the program's), so the runtime continues from the engine's post-setup uid.
int nsgpu_sim_attach_p2p(nsgpu_sim *s, nsgpu_p2p *h) {
  if (!s || !h) return set_error(NSGPU_EINVAL, "nsgpu_sim_attach_p2p: null");
  if (s->events->size || s->dispatched || s->uid != s->uid_first)
    return set_error(NSGPU_ESTATE, "nsgpu_sim_attach_p2p: attach before scheduling");
  if (s->uid_set && nsgpu::p2p_first_uid(h) != s->uid_first)  // (two starts that disagree)
    return set_error(NSGPU_ESTATE, "nsgpu_sim_attach_p2p: the engine's setup starts at uid %u, this runtime was set "
                                   "to start at %u", nsgpu::p2p_first_uid(h), s->uid_first);
  uint32_t u = 0;
  int rc = nsgpu_p2p_setup_uid(h, &u);
  if (rc) return rc;
  s->p2p = h;
  s->uid = u;
  return NSGPU_OK;
}

int nsgpu_sim_adopt_p2p(nsgpu_sim *s, nsgpu_p2p *h) {
  if (!s || !h) return set_error(NSGPU_EINVAL, "nsgpu_sim_adopt_p2p: null");
  if (s->p2p || s->wifi) return set_error(NSGPU_ESTATE, "nsgpu_sim_adopt_p2p: an engine is attached already");
  if (s->dispatched) return set_error(NSGPU_ESTATE, "nsgpu_sim_adopt_p2p: events were dispatched already");
  uint32_t u = 0;
  int rc = nsgpu_p2p_setup_uid(h, &u);
  if (rc) return rc;
  if (u != s->uid)
    return set_error(NSGPU_ESTATE, "nsgpu_sim_adopt_p2p: the engine's setup ends at uid %u, this runtime is at %u "
                                   "(the setup list does not mirror the program's Schedule calls)", u, s->uid);
  s->p2p = h;
  return NSGPU_OK;
}

// The closed-loop Wi-Fi PHY joins this runtime's order: its events are scheduled at run time only (the
// host closures' SendPacket calls), so it takes no setup uids.
int nsgpu_sim_attach_wifi(nsgpu_sim *s, nsgpu_wifil *h) {
  if (!s || !h) return set_error(NSGPU_EINVAL, "nsgpu_sim_attach_wifi: null");
  if (s->p2p || s->wifi) return set_error(NSGPU_ESTATE, "nsgpu_sim_attach_wifi: an engine is attached already");
  s->wifi = h;
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
  const uint64_t h = s->make(fn, user, arg);
  uint32_t u = 0;
  const int rc = s->insert((uint64_t)t, s->cur_ctx, h, &u);
  if (rc) {
    s->release(h);
    return rc;
  }
  if (id) *id = nsgpu_event_id{h, (uint64_t)t, s->cur_ctx, u};
  return rc;
}

int nsgpu_sim_schedule_with_context(nsgpu_sim *s, uint32_t ctx, int64_t delay, nsgpu_event_fn fn, void *user,
                                    uint64_t arg) {  // :206-219
  const uint64_t h = s->make(fn, user, arg);
  const int rc = s->insert(s->cur_ts + (uint64_t)delay, ctx, h, nullptr);
  if (rc) s->release(h);
  return rc;
}

int nsgpu_sim_schedule_now(nsgpu_sim *s, nsgpu_event_fn fn, void *user, uint64_t arg, nsgpu_event_id *id) {
  return nsgpu_sim_schedule(s, 0, fn, user, arg, id);  // :221-233
}

int nsgpu_sim_schedule_destroy(nsgpu_sim *s, nsgpu_event_fn fn, void *user, uint64_t arg, nsgpu_event_id *id) {
  if (s->uid >= nsgpu::UID_NEXT_MAX) return s->spent("nsgpu_sim_schedule_destroy");
  const uint64_t h = s->make(fn, user, arg);  // :235-242
  s->destroy_events.push_back(DestroyEv{h, s->cur_ts});
  s->uid++;
  if (id) *id = nsgpu_event_id{h, s->cur_ts, 0xffffffffu, 2};
  return NSGPU_OK;
}

int nsgpu_sim_is_expired(nsgpu_sim *s, const nsgpu_event_id *id, int *expired) {
  *expired = s->is_expired(*id) ? 1 : 0;
  return NSGPU_OK;
}

int nsgpu_sim_cancel(nsgpu_sim *s, const nsgpu_event_id *id) {  // :292-302
  if (!s->is_expired(*id)) s->get(id->impl)->cancelled = true;
  return NSGPU_OK;
}

int nsgpu_sim_remove(nsgpu_sim *s, const nsgpu_event_id *id) {  // :256-290
  if (id->uid == 2) {
    for (auto i = s->destroy_events.begin(); i != s->destroy_events.end(); i++) {
      if (i->handle == id->impl && i->ts == id->ts) {
        s->destroy_events.erase(i);
        s->release(id->impl);
        break;
      }
    }
    return NSGPU_OK;
  }
  if (s->is_expired(*id)) return NSGPU_OK;
  const int rc = nsgpu_sim_remove_key(s, id->ts, id->uid, id->context, id->impl);
  s->release(id->impl);  // (the queue entry, dropped when it surfaces, is never dereferenced)
  return rc;
}

// ---- raw handles (ns3::HipSimulatorImpl: the handle is an EventImpl*, never dereferenced here) ----
int nsgpu_sim_insert(nsgpu_sim *s, uint64_t ts, uint32_t ctx, uint64_t handle, uint32_t *uid) {
  if (!s || (handle & RAW)) return set_error(NSGPU_EINVAL, "nsgpu_sim_insert: null runtime or odd handle");
  if (ts < s->cur_ts) return set_error(NSGPU_EINVAL, "nsgpu_sim_insert: event in the past");
  return s->insert(ts, ctx, handle | RAW, uid);
}

// m_uid before anything is scheduled: the uids below `uid` count as consumed by Schedule calls this runtime did
// not see (default-simulator-impl.cc:52-56 starts at 4).  Only on a fresh runtime.
int nsgpu_sim_set_next_uid(nsgpu_sim *s, uint32_t uid) {
  if (!s) return set_error(NSGPU_EINVAL, "nsgpu_sim_set_next_uid: null");
  if (s->events->size || s->dispatched || s->uid != s->uid_first || !s->destroy_events.empty() || s->p2p || s->wifi)
    return set_error(NSGPU_ESTATE, "nsgpu_sim_set_next_uid: the runtime has scheduled or attached something already");
  if (uid < 4) return set_error(NSGPU_EINVAL, "nsgpu_sim_set_next_uid: uids 0, 1, 2 (and 3) are reserved");
  s->uid = s->uid_first = uid;
  s->uid_set = true;
  return NSGPU_OK;
}

int nsgpu_sim_consume_uid(nsgpu_sim *s, uint32_t *uid) {  // ScheduleDestroy's uid (:235-242)
  if (!s) return set_error(NSGPU_EINVAL, "nsgpu_sim_consume_uid: null");
  if (s->uid >= nsgpu::UID_NEXT_MAX) return s->spent("nsgpu_sim_consume_uid");
  if (uid) *uid = s->uid;
  s->uid++;
  return NSGPU_OK;
}

// The destroy list of raw handles (DefaultSimulatorImpl::m_destroyEvents, :235-242, :79-92, :256-268,
// :306-322): the runtime keeps the list, the caller keeps the reference each entry holds.
int nsgpu_sim_destroy_insert(nsgpu_sim *s, uint64_t handle, uint64_t *ts) {  // ScheduleDestroy
  if (!s || (handle & RAW)) return set_error(NSGPU_EINVAL, "nsgpu_sim_destroy_insert: null runtime or odd handle");
  if (s->uid >= nsgpu::UID_NEXT_MAX) return s->spent("nsgpu_sim_destroy_insert");
  s->destroy_events.push_back(DestroyEv{handle | RAW, s->cur_ts});
  s->uid++;
  if (ts) *ts = s->cur_ts;
  return NSGPU_OK;
}

int nsgpu_sim_destroy_pop(nsgpu_sim *s, uint64_t *handle, int *found) {  // Destroy: front, then pop_front
  if (!s || !handle || !found) return set_error(NSGPU_EINVAL, "nsgpu_sim_destroy_pop: null");
  *found = 0;
  while (!s->destroy_events.empty()) {
    const DestroyEv d = s->destroy_events.front();
    s->destroy_events.pop_front();
    if (!(d.handle & RAW)) return set_error(NSGPU_ESTATE, "nsgpu_sim_destroy_pop: a callback destroy event (nsgpu_sim_destroy)");
    *handle = d.handle & ~RAW;
    *found = 1;
    return NSGPU_OK;
  }
  return NSGPU_OK;
}

int nsgpu_sim_destroy_remove(nsgpu_sim *s, uint64_t handle, uint64_t ts, int *found) {  // Remove (uid 2)
  if (!s || !found) return set_error(NSGPU_EINVAL, "nsgpu_sim_destroy_remove: null");
  *found = 0;
  for (auto i = s->destroy_events.begin(); i != s->destroy_events.end(); i++) {
    if (i->handle == (handle | RAW) && i->ts == ts) {
      s->destroy_events.erase(i);
      *found = 1;
      break;
    }
  }
  return NSGPU_OK;
}

int nsgpu_sim_destroy_pending(nsgpu_sim *s, uint64_t handle, uint64_t ts, int *pending) {  // IsExpired (uid 2)
  if (!s || !pending) return set_error(NSGPU_EINVAL, "nsgpu_sim_destroy_pending: null");
  *pending = s->destroy_pending(handle | RAW, ts) ? 1 : 0;
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
// the attached engine, if any, has run out), or a Stop was dispatched.  `force`: pop even after a Stop
// (RunOneEvent).
static int pop_window(nsgpu_sim *s, nsgpu_event *out, uint32_t cap, uint32_t *n, bool force) {
  *n = 0;
  if (s->uid_spent) return nsgpu::uid_range_error("nsgpu_sim: Run after a Schedule call failed at the uid limit");
  s->win.clear();
  s->win_next = 0;
  if (!s->win_removed.empty()) s->win_removed.clear();
  if (s->stop && !force) return NSGPU_OK;
  int rc;
  nsgpu_event e;
  nsgpu_sched *q = s->events;
  // RunOneEvent (ProcessOneEvent, :167-170) dispatches exactly one event; an attached engine dispatches its
  // events in windows (one advance can run any number of them), so one-event steps are refused there
  if (force && (s->wifi || (s->p2p && !s->ended)))
    return set_error(NSGPU_ESTATE, "RunOneEvent: not supported while a GPU-resident engine is attached (it "
                                   "dispatches its events in windows)");
  // a Run after the Run that the device's Simulator::Stop ended: the reference resumes (:153-165), this
  // engine cannot (its final window's children were not queued) — fail instead of dropping the host events
  if (s->dev_stopped && !force && q->size)
    return set_error(NSGPU_ESTATE, "Run: the attached engine dispatched Simulator::Stop; resuming with %llu host "
                                   "event(s) pending is not supported", (unsigned long long)q->size);
  if (s->wifi) {  // the PHY's events below the next host event's key, then that host event (one per window)
    for (;;) {
      bool have = false;
      if (q->size) {
        if (!nsgpu::sched_next(q, &e, false, &rc)) return rc ? rc : set_error(NSGPU_ESTATE, "pop_window: lost events");
        have = true;
      }
      uint64_t bts = have ? e.ts : ~0ull;
      uint32_t buid = have ? e.uid : 0u;
      // the EndReceive hand-back: a listened phy's next EndReceive before the host event runs inside the order
      // (its own epoch, through its key), and the device never runs past a time where one not yet scheduled could
      // fall (a pending Receive that may sync) before that Receive has run
      bool handback = false, partial = false;
      nsgpu_wifil_next nx;
      if (s->wifi_end_fn && s->wifi_listen_n) {
        if ((rc = nsgpu_wifil_next_end(s->wifi, &nx))) return rc;
        const bool before_host = !have || nx.ts < e.ts || (nx.ts == e.ts && nx.uid < e.uid);
        if (nx.found && before_host && nx.ts <= nx.ts_potential) {  // (a later sync's uid is larger: at an equal ts
          bts = nx.ts;                                              //  the known one is first)
          buid = nx.uid + 1u;
          handback = true;
        } else if (nx.ts_potential != ~0ull && (!have || nx.ts_potential < e.ts) &&
                   (!nx.found || nx.ts_potential < nx.ts)) {  // (a host event at that ts was scheduled before the sync)
          bts = nx.ts_potential;
          buid = 0u;
          partial = true;
        }
      }
      rc = nsgpu_wifil_advance(s->wifi, bts, buid, &s->uid, &s->dispatched, &s->digest, s->log_ts, s->log_uid,
                               s->log_ctx, s->log_cap);
      if (rc == NSGPU_ERANGE) s->uid_spent = true;  // (sticky: the epoch's EndReceives would take wrapped uids)
      if (rc) return rc;
      if (handback) {
        nsgpu_wifil_end end;
        if (!nsgpu::wifil_epoch_end(s->wifi, nx.uid, &end))
          return set_error(NSGPU_ESTATE, "EndReceive hand-back: EndReceive %u of phy %u was not dispatched", nx.uid, nx.phy);
        if (!(end.flags & NSGPU_WIFI_END_CANCELLED)) {
          s->cur_ts = end.ts;  // (YansWifiPhy::EndReceive's Now (), its EventImpl's uid and context)
          s->cur_uid = end.uid;
          s->cur_ctx = nsgpu::wifil_node(s->wifi, end.phy);
          s->wifi_end_fn(s->wifi_end_user, &end);
          if (s->uid_spent) return nsgpu::uid_range_error("nsgpu_sim: EndReceive hand-back");
        }
        continue;
      }
      if (partial) continue;
      if (!have) return NSGPU_OK;
      if ((rc = nsgpu::sched_remove_next1(q, &e))) return rc;
      out[0] = e;
      s->win.push_back(e);
      *n = 1;
      return NSGPU_OK;
    }
  }
  if (s->p2p && !s->ended) {
    bool have = false;
    if (q->size) {
      if (!nsgpu::sched_next(q, &e, false, &rc)) return rc ? rc : set_error(NSGPU_ESTATE, "pop_window: lost events");
      have = true;
    }
    int ended = 0;
    rc = nsgpu_p2p_advance(s->p2p, have ? e.ts : ~0ull, have ? e.uid : 0u, &s->uid, &s->dispatched, &ended, s->stream);
    if (rc == NSGPU_ERANGE) s->uid_spent = true;
    if (rc) return rc;
    if (ended) {  // the device dispatched Simulator::Stop, or nothing is pending on the device
      uint64_t pn = 0, pts = 0;
      int stopped = 0;
      if ((rc = nsgpu_p2p_pending(s->p2p, &pn, &pts, &stopped, s->stream))) return rc;
      s->ended = true;
      if (stopped) {  // the device Stop ends this Run (:153-165); the engine cannot resume after it
        s->dev_stopped = true;
        return NSGPU_OK;
      }
    } else {
      if (!have) return NSGPU_OK;
      if ((rc = nsgpu::sched_remove_next1(q, &e))) return rc;
      out[0] = e;
      s->win.push_back(e);
      *n = 1;
      return NSGPU_OK;
    }
    if (!have) return NSGPU_OK;  // (the device drained: the host queue continues alone below)
  } else if (s->dev_stopped && !force) {
    return NSGPU_OK;
  }
  if (!q->size) return NSGPU_OK;
  if ((rc = nsgpu::sched_remove_next1(q, &e))) return rc;
  out[0] = e;
  s->win.push_back(e);
  uint32_t k = 1;
  while (k < cap && q->size) {
    nsgpu_event f;
    if (!nsgpu::sched_next(q, &f, false, &rc)) return rc ? rc : set_error(NSGPU_ESTATE, "pop_window: lost events");
    if (f.ts != e.ts) break;
    if ((rc = nsgpu::sched_remove_next1(q, &f))) return rc;
    out[k++] = f;
    s->win.push_back(f);
  }
  *n = k;
  return NSGPU_OK;
}

int nsgpu_sim_pop_window(nsgpu_sim *s, nsgpu_event *out, uint32_t cap, uint32_t *n) {
  if (!s || !out || !n || cap == 0) return set_error(NSGPU_EINVAL, "nsgpu_sim_pop_window: bad arguments");
  return pop_window(s, out, cap, n, false);
}

// RunOneEvent (:167-170): the next event, whatever the stop flag says.
int nsgpu_sim_pop_one(nsgpu_sim *s, nsgpu_event *out, uint32_t *n) {
  if (!s || !out || !n) return set_error(NSGPU_EINVAL, "nsgpu_sim_pop_one: bad arguments");
  return pop_window(s, out, 1, n, true);
}

// Window event i is being dispatched: 0 = run its closure, 1 = a closure of this window removed it
// (skip it), 2 = a Stop was dispatched before it (it stays pending).  Sets Now / Context / the
// current uid and accounts the dispatch (rank, digest, log) for a dispatched one.
int nsgpu_sim_begin(nsgpu_sim *s, const nsgpu_event *e, int *skip) {
  if (!s || !e || !skip) return set_error(NSGPU_EINVAL, "nsgpu_sim_begin: null");
  if (s->win_next < s->win.size() && s->win[s->win_next].uid == e->uid) s->win_next++;
  if (!s->win_removed.empty() && s->win_removed.count(e->uid)) {
    *skip = 1;
    return NSGPU_OK;
  }
  if (s->stop && s->win.size() > 1) {  // (a one-event window was popped for this dispatch: RunOneEvent)
    *skip = 2;
    return nsgpu::sched_insert1(s->events, *e);
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

// Dispatches the popped window of C-callback closures.
static int run_window(nsgpu_sim *s, const nsgpu_event *w, uint32_t n) {
  for (uint32_t i = 0; i < n; i++) {
    int skip = 0;
    int rc = nsgpu_sim_begin(s, &w[i], &skip);
    if (rc) return rc;
    if (skip) continue;
    if (w[i].handle & RAW) return set_error(NSGPU_ESTATE, "nsgpu_sim_run: a raw handle (dispatch it with nsgpu_sim_pop_window)");
    HostEvent *e = s->get(w[i].handle);
    if (!e) return set_error(NSGPU_ESTATE, "nsgpu_sim_run: a dispatched event names a released closure");
    const HostEvent c = *e;
    s->release(w[i].handle);
    if (c.cancelled) {  // still dequeued and counted (event-impl.cc:34-41)
      s->cancelled++;
      continue;
    }
    if (c.is_stop) s->stop = true;
    else c.fn(c.user, c.arg);
  }
  return NSGPU_OK;
}

int nsgpu_sim_run(nsgpu_sim *s) {  // Run (:153-165): windows of closures (and device events)
  // A later Run continues after Stop (:153-165); the device pipeline cannot restart after a Stop it
  // dispatched itself (its final window's children are not queued), so that case fails loudly.
  if (s->dev_stopped)
    return set_error(NSGPU_ESTATE, "nsgpu_sim_run: the attached engine dispatched Simulator::Stop; resuming after a "
                                   "device-side Stop is not supported");
  s->stop = false;
  std::vector<nsgpu_event> w(1024);
  for (;;) {
    uint32_t n = 0;
    int rc = pop_window(s, w.data(), (uint32_t)w.size(), &n, false);
    if (rc) return rc;
    if (n == 0) break;
    if ((rc = run_window(s, w.data(), n))) return rc;
  }
  return s->wifi ? nsgpu_wifil_flush(s->wifi, &s->digest) : NSGPU_OK;  // (the epochs' digest terms still summing)
}

int nsgpu_sim_run_one(nsgpu_sim *s) {  // RunOneEvent (:167-170)
  nsgpu_event e;
  uint32_t n = 0;
  int rc = pop_window(s, &e, 1, &n, true);
  if (rc || n == 0) return rc;
  return run_window(s, &e, 1);
}

int nsgpu_sim_stop(nsgpu_sim *s) {
  s->stop = true;
  return NSGPU_OK;
}

int nsgpu_sim_stop_at(nsgpu_sim *s, int64_t delay) {  // Stop (Time): Schedule (time, &Simulator::Stop)
  return s->insert(s->cur_ts + (uint64_t)delay, s->cur_ctx, s->make(nullptr, nullptr, 0, true), nullptr);
}

int nsgpu_sim_destroy(nsgpu_sim *s) {  // :79-92 — a destroy closure may schedule or remove destroy events
  while (!s->destroy_events.empty()) {
    const DestroyEv d = s->destroy_events.front();
    s->destroy_events.pop_front();
    if (d.handle & RAW) return set_error(NSGPU_ESTATE, "nsgpu_sim_destroy: a raw destroy handle (nsgpu_sim_destroy_pop)");
    HostEvent *e = s->get(d.handle);
    if (!e) continue;
    const HostEvent c = *e;
    s->release(d.handle);
    if (!c.cancelled) c.fn(c.user, c.arg);
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

// Next (): the time of the next event, host or device (an attached engine's pending events count);
// *empty = 1 when none is pending anywhere.
int nsgpu_sim_next(nsgpu_sim *s, uint64_t *ts, int *empty) {
  if (!s || !ts || !empty) return set_error(NSGPU_EINVAL, "nsgpu_sim_next: null");
  uint64_t dn = 0, dts = ~0ull;
  int rc = s->device_pending(&dn, &dts);
  if (rc) return rc;
  *ts = dn ? dts : ~0ull;
  if (s->events->size) {
    nsgpu_event e;
    if (!nsgpu::sched_next(s->events, &e, false, &rc)) return rc ? rc : set_error(NSGPU_ESTATE, "next: lost events");
    if (e.ts < *ts) *ts = e.ts;
  }
  *empty = (s->events->size == 0 && dn == 0) ? 1 : 0;
  if (*empty) *ts = 0;
  return NSGPU_OK;
}

// IsFinished () (:133-137): nothing pending (host or device), or Stop was called / dispatched.
int nsgpu_sim_is_finished(nsgpu_sim *s, int *finished) {
  if (!s || !finished) return set_error(NSGPU_EINVAL, "nsgpu_sim_is_finished: null");
  if (s->stop || s->dev_stopped) {
    *finished = 1;
    return NSGPU_OK;
  }
  uint64_t ts = 0;
  int empty = 1;
  const int rc = nsgpu_sim_next(s, &ts, &empty);
  *finished = empty;
  return rc;
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
  for (uint32_t k = 0; k < cap && s->events->size; k++) {
    const int rc = nsgpu::sched_remove_next1(s->events, &out[k]);
    if (rc) return rc;
    s->release(out[k].handle);
    *n = k + 1;
  }
  return NSGPU_OK;
}

int nsgpu_sim_current_uid(nsgpu_sim *s, uint32_t *uid) {
  if (!s || !uid) return set_error(NSGPU_EINVAL, "nsgpu_sim_current_uid: null");
  *uid = s->cur_uid;
  return NSGPU_OK;
}

int nsgpu_sim_sched_stats(nsgpu_sim *s, uint64_t *refills, uint64_t *front, double *refill_us) {
  if (!s) return set_error(NSGPU_EINVAL, "nsgpu_sim_sched_stats: null");
  return nsgpu_sched_stats(s->events, refills, front, refill_us);
}

int nsgpu_sim_host_stats(nsgpu_sim *s, uint64_t *host_dispatched, uint64_t *cancelled, uint64_t *digest) {
  if (!s) return set_error(NSGPU_EINVAL, "nsgpu_sim_host_stats: null");
  if (host_dispatched) *host_dispatched = s->host_dispatched;
  if (cancelled) *cancelled = s->cancelled;
  if (s->wifi) {
    int rc = nsgpu_wifil_flush(s->wifi, &s->digest);
    if (rc) return rc;
  }
  if (digest) *digest = s->digest;
  return NSGPU_OK;
}

// Closures held by the runtime (live slab slots): scheduled, destroy-listed or not yet released.
int nsgpu_sim_live_closures(nsgpu_sim *s, uint64_t *n) {
  if (!s || !n) return set_error(NSGPU_EINVAL, "nsgpu_sim_live_closures: null");
  *n = s->slab.size() - s->free_slots.size();
  return NSGPU_OK;
}

// A host closure's YansWifiPhy::SendPacket on `phy` of the attached Wi-Fi PHY (now; YansWifiChannel::Send's
// receiver loop takes the runtime's next uids, one per receiver).
int nsgpu_sim_wifi_send(nsgpu_sim *s, uint32_t phy, uint32_t size, double dbm, uint32_t modclass, uint64_t rate,
                        uint32_t bw, uint32_t preamble) {
  if (!s || !s->wifi) return set_error(NSGPU_ESTATE, "nsgpu_sim_wifi_send: no Wi-Fi PHY attached");
  uint32_t n = 0;
  int rc = nsgpu_wifil_receivers(s->wifi, phy, &n);
  if (rc) return rc;
  if ((uint64_t)s->uid + n > nsgpu::UID_NEXT_MAX) return s->spent("nsgpu_sim_wifi_send");
  rc = nsgpu_wifil_send(s->wifi, s->cur_ts, s->uid, phy, size, dbm, modclass, rate, bw, preamble);
  if (rc) return rc;
  s->uid += n;
  return NSGPU_OK;
}

int nsgpu_sim_wifi_set_end_handler(nsgpu_sim *s, nsgpu_wifi_end_fn fn, void *user) {
  if (!s) return set_error(NSGPU_EINVAL, "nsgpu_sim_wifi_set_end_handler: null");
  s->wifi_end_fn = fn;
  s->wifi_end_user = user;
  return NSGPU_OK;
}

int nsgpu_sim_wifi_listen(nsgpu_sim *s, uint32_t phy, int on) {
  if (!s || !s->wifi) return set_error(NSGPU_ESTATE, "nsgpu_sim_wifi_listen: no Wi-Fi PHY attached");
  if (s->lis_on.size() <= phy) s->lis_on.resize((size_t)phy + 1, 0);
  const uint8_t v = on ? 1 : 0;
  int rc = nsgpu_wifil_listen(s->wifi, phy, on);
  if (rc) return rc;
  if (s->lis_on[phy] != v) {
    s->wifi_listen_n += v ? 1 : (uint64_t)-1;
    s->lis_on[phy] = v;
  }
  return NSGPU_OK;
}

// MobilityModel::SetPosition of `phy`'s node from the running closure: the later SendPackets' fan-outs see it.
int nsgpu_sim_wifi_set_position(nsgpu_sim *s, uint32_t phy, double x, double y, double z) {
  if (!s || !s->wifi) return set_error(NSGPU_ESTATE, "nsgpu_sim_wifi_set_position: no Wi-Fi PHY attached");
  return nsgpu_wifil_set_position(s->wifi, phy, x, y, z);
}

// WifiPhyStateHelper::GetState of `phy` at Now (the device has run every event before the running closure).
int nsgpu_sim_wifi_state(nsgpu_sim *s, uint32_t phy, nsgpu_wifil_phy_state *out) {
  if (!s || !s->wifi) return set_error(NSGPU_ESTATE, "nsgpu_sim_wifi_state: no Wi-Fi PHY attached");
  return nsgpu_wifil_get_state(s->wifi, phy, s->cur_ts, out);
}

// A host closure's UdpSocket::Send on application `app` of the attached engine (now, with the uid
// of the closure being dispatched; its Schedule calls take the runtime's next uids).
int nsgpu_sim_p2p_send(nsgpu_sim *s, uint32_t app) {
  if (!s || !s->p2p) return set_error(NSGPU_ESTATE, "nsgpu_sim_p2p_send: no engine attached");
  // (an engine that has run out — nothing pending on the device, or a device Stop — is not advanced
  // again, so a datagram handed to it would never be dispatched)
  if (s->ended)
    return set_error(NSGPU_ESTATE, "nsgpu_sim_p2p_send: the attached engine has finished (no device event was "
                                   "pending when a host event was next); the datagram would never be sent");
  uint32_t seq = s->p2p_seq_uid == s->cur_uid ? s->p2p_seq : 0;
  int rc = nsgpu_p2p_inject_send(s->p2p, app, s->cur_ts, s->cur_uid, s->cur_ctx, &s->uid, &seq, s->stream);
  if (rc == NSGPU_ERANGE) return s->spent("nsgpu_sim_p2p_send");
  s->p2p_seq_uid = s->cur_uid;
  s->p2p_seq = seq;
  return rc;
}

}  // extern "C"
