// nsref_sched.cc — CPU ORACLE (test infrastructure only; see nsref.h header).
// Restatement of the sequential engine: DefaultSimulatorImpl (src/core/model/default-simulator-impl.cc)
// over MapScheduler (map-scheduler.cc), HeapScheduler (heap-scheduler.cc) or ListScheduler
// (list-scheduler.cc), with EventImpl's ref-counted, cancellable closure (event-impl.cc:34-53).
// Also utils/bench-simulator.cc's Bench (config 1), used as the CPU baseline ("port").
#include "nsref.h"
#include <map>
#include <vector>
#include <list>
#include <deque>
#include <chrono>
#include <stdio.h>
#include <stdlib.h>

#include "nsref_engine.hpp"

namespace {
struct StopEvent : EventImpl {  // Simulator::Stop scheduled by Stop (Time) (:179-183)
  nsref_sim *s;
  explicit StopEvent(nsref_sim *x) : s(x) {}
  void Notify() override { s->m_stop = true; }
};
}  // namespace

extern "C" {

nsref_sim *nsref_sim_new(int scheduler) { return new nsref_sim(scheduler); }
void nsref_sim_free(nsref_sim *s) { delete s; }
void nsref_sim_set_uid(nsref_sim *s, uint32_t uid) { s->m_uid = uid; }
nsgpu_event_id nsref_sim_schedule(nsref_sim *s, int64_t delay, nsref_fn fn, void *user, uint64_t arg) {
  EventImpl *e = new CEvent(fn, user, arg);
  s->pin(e);
  return s->Schedule(delay, e);
}
void nsref_sim_schedule_with_context(nsref_sim *s, uint32_t ctx, int64_t delay, nsref_fn fn, void *user,
                                     uint64_t arg) {
  s->ScheduleWithContext(ctx, delay, new CEvent(fn, user, arg));
}
nsgpu_event_id nsref_sim_schedule_now(nsref_sim *s, nsref_fn fn, void *user, uint64_t arg) {
  EventImpl *e = new CEvent(fn, user, arg);
  s->pin(e);
  return s->ScheduleNow(e);
}
nsgpu_event_id nsref_sim_schedule_destroy(nsref_sim *s, nsref_fn fn, void *user, uint64_t arg) {
  EventImpl *e = new CEvent(fn, user, arg);
  s->pin(e);
  return s->ScheduleDestroy(e);
}
void nsref_sim_remove(nsref_sim *s, const nsgpu_event_id *id) { s->Remove(*id); }
void nsref_sim_cancel(nsref_sim *s, const nsgpu_event_id *id) { s->Cancel(*id); }
int nsref_sim_is_expired(nsref_sim *s, const nsgpu_event_id *id) { return s->IsExpired(*id) ? 1 : 0; }
void nsref_sim_run(nsref_sim *s) { s->Run(); }
void nsref_sim_run_one(nsref_sim *s) { s->RunOneEvent(); }
int nsref_sim_is_finished(nsref_sim *s) { return s->IsFinished() ? 1 : 0; }
void nsref_sim_stop(nsref_sim *s) { s->m_stop = true; }
void nsref_sim_stop_at(nsref_sim *s, int64_t delay) { s->Schedule(delay, new StopEvent(s)); }
void nsref_sim_destroy(nsref_sim *s) { s->Destroy(); }
uint64_t nsref_sim_now(nsref_sim *s) { return s->m_currentTs; }
uint32_t nsref_sim_context(nsref_sim *s) { return s->m_currentContext; }
uint64_t nsref_sim_delay_left(nsref_sim *s, const nsgpu_event_id *id) {  // :247-254
  return s->IsExpired(*id) ? 0 : id->ts - s->m_currentTs;
}
uint64_t nsref_sim_dispatched(nsref_sim *s) { return s->m_dispatched; }
uint32_t nsref_sim_next_uid(nsref_sim *s) { return s->m_uid; }
void nsref_sim_set_log(nsref_sim *s, uint64_t *ts, uint32_t *uid, uint32_t *ctx, uint64_t cap) {
  s->log_ts = ts;
  s->log_uid = uid;
  s->log_ctx = ctx;
  s->log_cap = cap;
}

}  // extern "C"

// ---------------- utils/bench-simulator.cc ----------------
namespace {
struct Bench;
struct BenchCb : EventImpl {  // MakeEvent (&Bench::Cb, this)
  Bench *b;
  explicit BenchCb(Bench *x) : b(x) {}
  void Notify() override;
};
struct Bench {  // bench-simulator.cc:32-45
  const uint64_t *dist;
  uint32_t n;
  uint32_t m_current = 0;
  uint32_t m_n = 0;
  uint32_t m_total;
  nsref_sim *sim;
  void Cb() {  // :109-127
    if (m_n > m_total) return;
    if (m_current == n) m_current = 0;
    sim->Schedule((int64_t)dist[m_current], new BenchCb(this));  // NanoSeconds (*m_current)
    m_current++;
    m_n++;
  }
};
void BenchCb::Notify() { b->Cb(); }
}  // namespace

extern "C" int nsref_churn_run(const uint64_t *dist_ns, uint32_t n, uint32_t total, int scheduler,
                               uint64_t *log_ts, uint32_t *log_uid, uint64_t log_cap, nsref_churn_result *out) {
  nsref_sim sim(scheduler);
  sim.log_ts = log_ts;
  sim.log_uid = log_uid;
  sim.log_cap = log_ts ? log_cap : 0;
  Bench b;
  b.dist = dist_ns;
  b.n = n;
  b.m_total = total;
  b.sim = &sim;
  auto t0 = std::chrono::steady_clock::now(), t1 = t0;
  // Simulator::Run; the order-sensitive digest of the pop order is folded in by ProcessOneEvent
  sim.want_digest = true;
  int rc = 0;
  try {
    for (uint32_t i = 0; i < n; i++) sim.Schedule((int64_t)dist_ns[i], new BenchCb(&b));  // RunBench :84-88
    t1 = std::chrono::steady_clock::now();
    sim.Run();
  } catch (const CalendarCrash &) {
    rc = -3;  // where the reference's CalendarScheduler crashes
    sim.crashed = true;
  }
  auto t2 = std::chrono::steady_clock::now();
  const uint64_t digest = sim.m_digest, last_ts = sim.m_currentTs;
  out->dispatched = sim.m_dispatched;
  out->holds = b.m_n;
  out->final_ts = last_ts;
  out->digest = digest;
  out->next_uid = sim.m_uid;
  out->pad_ = 0;
  out->init_seconds = std::chrono::duration<double>(t1 - t0).count();
  out->run_seconds = std::chrono::duration<double>(t2 - t1).count();
  return rc;
}
