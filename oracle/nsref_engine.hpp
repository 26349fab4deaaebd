// nsref_engine.hpp — CPU ORACLE internals (test infrastructure only; see nsref.h header).
// The restated sequential engine shared by nsref_sched.cc and nsref_p2p.cc.
#pragma once
#include "nsref.h"
#include <map>
#include <vector>
#include <list>
#include <deque>
#include <stdlib.h>

namespace nsref_detail {

struct Key {  // Scheduler::EventKey — scheduler.h:58-63
  uint64_t ts;
  uint32_t uid;
  uint32_t ctx;
};
// operator< (scheduler.h:105-121): (ts, uid) only.
struct KeyLess {
  bool operator()(const Key &a, const Key &b) const {
    if (a.ts < b.ts) return true;
    if (a.ts == b.ts && a.uid < b.uid) return true;
    return false;
  }
};

// EventImpl (event-impl.cc:34-53): Invoke runs Notify unless cancelled.
struct EventImpl {
  virtual ~EventImpl() {}
  virtual void Notify() = 0;
  void Invoke() {
    if (!cancelled) Notify();
  }
  void Ref() { ++refs; }
  void Unref() {
    if (--refs == 0) delete this;
  }
  int refs = 1;
  bool cancelled = false;
};

struct CEvent : EventImpl {  // closure made by MakeEvent (make-event.h:76+), here a C callback
  nsref_fn fn;
  void *user;
  uint64_t arg;
  CEvent(nsref_fn f, void *u, uint64_t a) : fn(f), user(u), arg(a) {}
  void Notify() override { fn(user, arg); }
};

struct Event {  // Scheduler::Event (scheduler.h:64-68)
  EventImpl *impl;
  Key key;
};

// ---- schedulers ----
struct Scheduler {
  virtual ~Scheduler() {}
  virtual void Insert(const Event &ev) = 0;
  virtual bool IsEmpty() const = 0;
  virtual Event PeekNext() const = 0;
  virtual Event RemoveNext() = 0;
  virtual void Remove(const Event &ev) = 0;
};

struct MapScheduler : Scheduler {  // map-scheduler.cc:51-100
  std::map<Key, EventImpl *, KeyLess> m_list;
  void Insert(const Event &ev) override {
    auto r = m_list.insert(std::make_pair(ev.key, ev.impl));
    if (!r.second) abort();  // NS_ASSERT (result.second)
  }
  bool IsEmpty() const override { return m_list.empty(); }
  Event PeekNext() const override {
    auto i = m_list.begin();
    return Event{i->second, i->first};
  }
  Event RemoveNext() override {
    auto i = m_list.begin();
    Event ev{i->second, i->first};
    m_list.erase(i);
    return ev;
  }
  void Remove(const Event &ev) override {
    auto i = m_list.find(ev.key);
    m_list.erase(i);
  }
};

struct HeapScheduler : Scheduler {  // heap-scheduler.cc:44-217 (1-based binary heap, H5 Remove quirk kept)
  std::vector<Event> m_heap;
  HeapScheduler() { m_heap.push_back(Event{nullptr, {0, 0, 0}}); }
  bool Less(uint32_t a, uint32_t b) const { return KeyLess()(m_heap[a].key, m_heap[b].key); }
  uint32_t Last() const { return (uint32_t)m_heap.size() - 1; }
  bool IsBottom(uint32_t id) const { return id >= m_heap.size(); }
  void Exch(uint32_t a, uint32_t b) { std::swap(m_heap[a], m_heap[b]); }
  void BottomUp() {
    uint32_t index = Last();
    while (index != 1 && Less(index, index / 2)) {
      Exch(index, index / 2);
      index = index / 2;
    }
  }
  void TopDown(uint32_t start) {  // heap-scheduler.cc:141-172
    uint32_t index = start;
    uint32_t right = index * 2 + 1;
    while (!IsBottom(right)) {
      uint32_t left = index * 2;
      uint32_t tmp = Less(left, right) ? left : right;
      if (Less(index, tmp)) return;
      Exch(index, tmp);
      index = tmp;
      right = index * 2 + 1;
    }
    if (IsBottom(index)) return;
    uint32_t left = index * 2;
    if (IsBottom(left)) return;
    if (Less(index, left)) return;
    Exch(index, left);
  }
  void Insert(const Event &ev) override {
    m_heap.push_back(ev);
    BottomUp();
  }
  bool IsEmpty() const override { return m_heap.size() == 1; }
  Event PeekNext() const override { return m_heap[1]; }
  Event RemoveNext() override {
    Event next = m_heap[1];
    Exch(1, Last());
    m_heap.pop_back();
    TopDown(1);
    return next;
  }
  void Remove(const Event &ev) override {  // heap-scheduler.cc:201-217: swap with last, TopDown only
    for (uint32_t i = 1; i < m_heap.size(); i++) {
      if (ev.key.uid == m_heap[i].key.uid) {
        Exch(i, Last());
        m_heap.pop_back();
        TopDown(i);
        return;
      }
    }
    abort();
  }
};

struct ListScheduler : Scheduler {  // list-scheduler.cc:50-96: sorted std::list, insert scans from front
  std::list<Event> m_events;
  void Insert(const Event &ev) override {
    for (auto i = m_events.begin(); i != m_events.end(); i++) {
      if (KeyLess()(ev.key, i->key)) {
        m_events.insert(i, ev);
        return;
      }
    }
    m_events.push_back(ev);
  }
  bool IsEmpty() const override { return m_events.empty(); }
  Event PeekNext() const override { return m_events.front(); }
  Event RemoveNext() override {
    Event e = m_events.front();
    m_events.pop_front();
    return e;
  }
  void Remove(const Event &ev) override {
    for (auto i = m_events.begin(); i != m_events.end(); i++) {
      if (i->key.uid == ev.key.uid) {
        m_events.erase(i);
        return;
      }
    }
    abort();
  }
};

// CalendarScheduler (calendar-scheduler.cc:45-348): Brown's calendar queue, buckets of sorted lists,
// resized by doubling/halving with a width sampled from the next events.  SURVEY H3: the "no event
// within one year" fallback of DoRemoveNext starts from a sentinel whose ts is 0xffffffff (the
// initializer `{0, {~0u, ~0u}}` puts ~0u in the 64-bit m_ts), so once every pending event is later than
// 2^32 ns the sentinel wins, an arbitrary (or empty) bucket is popped and the impl-less sentinel is
// returned: the reference crashes there (free(): invalid pointer / null Invoke).  The restatement throws
// CalendarCrash at that point instead of reproducing the undefined behaviour.
struct CalendarCrash {};

struct CalendarScheduler : Scheduler {
  typedef std::list<Event> Bucket;
  std::vector<Bucket> m_buckets;
  uint32_t m_nBuckets = 0;
  uint64_t m_width = 0, m_lastPrio = 0, m_bucketTop = 0;
  uint32_t m_lastBucket = 0;
  uint32_t m_qSize = 0;
  CalendarScheduler() { Init(2, 1, 0); }
  void Init(uint32_t nBuckets, uint64_t width, uint64_t startPrio) {  // :57-69
    m_buckets.assign(nBuckets, Bucket());
    m_nBuckets = nBuckets;
    m_width = width;
    m_lastPrio = startPrio;
    m_lastBucket = Hash(startPrio);
    m_bucketTop = (startPrio / width + 1) * width;
  }
  uint32_t Hash(uint64_t ts) const { return (uint32_t)((ts / m_width) % m_nBuckets); }  // :81-86
  void DoInsert(const Event &ev) {  // :88-107: before the first later key of the bucket
    Bucket &b = m_buckets[Hash(ev.key.ts)];
    for (auto i = b.begin(); i != b.end(); ++i)
      if (KeyLess()(ev.key, i->key)) {
        b.insert(i, ev);
        return;
      }
    b.push_back(ev);
  }
  void Insert(const Event &ev) override {  // :109-115
    DoInsert(ev);
    m_qSize++;
    ResizeUp();
  }
  bool IsEmpty() const override { return m_qSize == 0; }
  static Event Sentinel() { return Event{nullptr, {0xffffffffull, 0xffffffffu, 0u}}; }
  Event PeekNext() const override {  // :121-150
    uint32_t i = m_lastBucket;
    uint64_t bucketTop = m_bucketTop;
    Event minEvent = Sentinel();
    do {
      if (!m_buckets[i].empty()) {
        const Event &next = m_buckets[i].front();
        if (next.key.ts < bucketTop) return next;
        if (KeyLess()(next.key, minEvent.key)) minEvent = next;
      }
      i++;
      i %= m_nBuckets;
      bucketTop += m_width;
    } while (i != m_lastBucket);
    if (minEvent.impl == nullptr) throw CalendarCrash();
    return minEvent;
  }
  Event DoRemoveNext() {  // :152-188
    uint32_t i = m_lastBucket;
    uint64_t bucketTop = m_bucketTop;
    Event minEvent = Sentinel();
    do {
      if (!m_buckets[i].empty()) {
        Event next = m_buckets[i].front();
        if (next.key.ts < bucketTop) {
          m_lastBucket = i;
          m_lastPrio = next.key.ts;
          m_bucketTop = bucketTop;
          m_buckets[i].pop_front();
          return next;
        }
        if (KeyLess()(next.key, minEvent.key)) minEvent = next;
      }
      i++;
      i %= m_nBuckets;
      bucketTop += m_width;
    } while (i != m_lastBucket);
    if (minEvent.impl == nullptr) throw CalendarCrash();  // H3
    m_lastPrio = minEvent.key.ts;
    m_lastBucket = Hash(minEvent.key.ts);
    m_bucketTop = (minEvent.key.ts / m_width + 1) * m_width;
    m_buckets[m_lastBucket].pop_front();
    return minEvent;
  }
  Event RemoveNext() override {  // :190-203
    Event ev = DoRemoveNext();
    m_qSize--;
    ResizeDown();
    return ev;
  }
  void Remove(const Event &ev) override {  // :205-226
    Bucket &b = m_buckets[Hash(ev.key.ts)];
    for (auto i = b.begin(); i != b.end(); ++i)
      if (i->key.uid == ev.key.uid) {
        b.erase(i);
        m_qSize--;
        ResizeDown();
        return;
      }
    abort();
  }
  void ResizeUp() {  // :228-236
    if (m_qSize > m_nBuckets * 2 && m_nBuckets < 32768) Resize(m_nBuckets * 2);
  }
  void ResizeDown() {  // :237-244
    if (m_qSize < m_nBuckets / 2) Resize(m_nBuckets / 2);
  }
  uint64_t CalculateNewWidth() {  // :246-322 (returned through uint32_t, as the reference does)
    if (m_qSize < 2) return 1;
    uint32_t nSamples = m_qSize <= 5 ? m_qSize : 5 + m_qSize / 10;
    if (nSamples > 25) nSamples = 25;
    std::vector<Event> samples;
    const uint32_t lastBucket = m_lastBucket;
    const uint64_t bucketTop = m_bucketTop, lastPrio = m_lastPrio;
    for (uint32_t i = 0; i < nSamples; i++) samples.push_back(DoRemoveNext());
    for (const Event &e : samples) DoInsert(e);
    m_lastBucket = lastBucket;
    m_bucketTop = bucketTop;
    m_lastPrio = lastPrio;
    uint64_t totalSeparation = 0;
    for (uint32_t k = 1; k < samples.size(); k++) totalSeparation += samples[k].key.ts - samples[k - 1].key.ts;
    const uint64_t twiceAvg = totalSeparation / (nSamples - 1) * 2;
    totalSeparation = 0;
    for (uint32_t k = 1; k < samples.size(); k++) {
      const uint64_t diff = samples[k].key.ts - samples[k - 1].key.ts;
      if (diff <= twiceAvg) totalSeparation += diff;
    }
    totalSeparation *= 3;
    if (totalSeparation < 1) totalSeparation = 1;
    return (uint32_t)totalSeparation;
  }
  void DoResize(uint32_t newSize, uint64_t newWidth) {  // :323-339
    std::vector<Bucket> old;
    old.swap(m_buckets);
    Init(newSize, newWidth, m_lastPrio);
    for (auto &b : old)
      for (const Event &e : b) DoInsert(e);
  }
  void Resize(uint32_t newSize) { DoResize(newSize, CalculateNewWidth()); }  // :340-348
};

}  // namespace nsref_detail
using namespace nsref_detail;

// ---- DefaultSimulatorImpl (default-simulator-impl.cc:49-353) ----
struct nsref_sim {
  Scheduler *m_events;
  bool m_stop = false;
  uint32_t m_uid = 4;  // uids 0,1,2 reserved (:52-56)
  uint32_t m_currentUid = 0;
  uint64_t m_currentTs = 0;
  uint32_t m_currentContext = 0xffffffff;
  int64_t m_unscheduledEvents = 0;
  uint64_t m_dispatched = 0;
  uint64_t m_cancelled = 0;   // dispatches of cancelled events
  uint64_t m_digest = 0;      // order-sensitive digest of the pop order (when want_digest)
  bool want_digest = false;
  std::deque<nsgpu_event_id> m_destroyEvents;  // EventId list (:235-242)
  std::vector<EventImpl *> m_pinned;           // impls an EventId was handed out for (kept alive, like Ptr<>)
  uint64_t *log_ts = nullptr;
  uint32_t *log_uid = nullptr, *log_ctx = nullptr;
  uint64_t log_cap = 0;

  explicit nsref_sim(int sched) {
    if (sched == NSREF_SCHED_HEAP) m_events = new HeapScheduler();
    else if (sched == NSREF_SCHED_LIST) m_events = new ListScheduler();
    else if (sched == NSREF_SCHED_CALENDAR) m_events = new CalendarScheduler();
    else m_events = new MapScheduler();
  }
  bool crashed = false;  // the scheduler reached a point where the reference crashes
  ~nsref_sim() {
    // DoDispose (:66-75): drain and unref (after a restated crash the pending events are leaked)
    try {
      while (!crashed && !m_events->IsEmpty()) m_events->RemoveNext().impl->Unref();
    } catch (const CalendarCrash &) {
    }
    delete m_events;
    for (EventImpl *e : m_pinned) e->Unref();
  }
  void pin(EventImpl *e) {
    e->Ref();
    m_pinned.push_back(e);
  }

  void ProcessOneEvent() {  // :117-131
    Event next = m_events->RemoveNext();
    if (next.key.ts < m_currentTs) abort();
    m_unscheduledEvents--;
    m_currentTs = next.key.ts;
    m_currentContext = next.key.ctx;
    m_currentUid = next.key.uid;
    if (m_dispatched < log_cap) {
      log_ts[m_dispatched] = next.key.ts;
      log_uid[m_dispatched] = next.key.uid;
      if (log_ctx) log_ctx[m_dispatched] = next.key.ctx;
    }
    if (want_digest) m_digest += nsgpu_dispatch_digest_term(m_dispatched, next.key.ts, next.key.uid);
    if (next.impl->cancelled) m_cancelled++;
    m_dispatched++;
    next.impl->Invoke();
    next.impl->Unref();
  }
  void Run() {  // :153-165
    m_stop = false;
    while (!m_events->IsEmpty() && !m_stop) ProcessOneEvent();
  }
  bool IsFinished() const { return m_events->IsEmpty() || m_stop; }  // :133-137
  void RunOneEvent() {  // :167-170 (RemoveNext on an empty queue asserts)
    if (m_events->IsEmpty()) abort();
    ProcessOneEvent();
  }
  nsgpu_event_id Schedule(int64_t delay, EventImpl *event) {  // :188-204
    int64_t tAbsolute = delay + (int64_t)m_currentTs;
    if (tAbsolute < 0 || tAbsolute < (int64_t)m_currentTs) abort();  // NS_ASSERTs
    Event ev;
    ev.impl = event;
    ev.key.ts = (uint64_t)tAbsolute;
    ev.key.ctx = m_currentContext;
    ev.key.uid = m_uid;
    m_uid++;
    m_unscheduledEvents++;
    m_events->Insert(ev);
    return nsgpu_event_id{(uint64_t)(uintptr_t)event, ev.key.ts, ev.key.ctx, ev.key.uid};
  }
  void ScheduleWithContext(uint32_t context, int64_t delay, EventImpl *event) {  // :206-219
    Event ev;
    ev.impl = event;
    ev.key.ts = m_currentTs + delay;
    ev.key.ctx = context;
    ev.key.uid = m_uid;
    m_uid++;
    m_unscheduledEvents++;
    m_events->Insert(ev);
  }
  nsgpu_event_id ScheduleNow(EventImpl *event) {  // :221-233
    Event ev;
    ev.impl = event;
    ev.key.ts = m_currentTs;
    ev.key.ctx = m_currentContext;
    ev.key.uid = m_uid;
    m_uid++;
    m_unscheduledEvents++;
    m_events->Insert(ev);
    return nsgpu_event_id{(uint64_t)(uintptr_t)event, ev.key.ts, ev.key.ctx, ev.key.uid};
  }
  nsgpu_event_id ScheduleDestroy(EventImpl *event) {  // :235-242
    nsgpu_event_id id{(uint64_t)(uintptr_t)event, m_currentTs, 0xffffffffu, 2};
    m_destroyEvents.push_back(id);
    m_uid++;
    return id;
  }
  static bool same(const nsgpu_event_id &a, const nsgpu_event_id &b) {  // EventId operator== (event-id.cc)
    return a.impl == b.impl && a.ts == b.ts && a.context == b.context && a.uid == b.uid;
  }
  static EventImpl *impl(const nsgpu_event_id &id) { return (EventImpl *)(uintptr_t)id.impl; }
  bool IsExpired(const nsgpu_event_id &ev) const {  // :304-332
    if (ev.uid == 2) {
      if (impl(ev) == nullptr || impl(ev)->cancelled) return true;
      for (auto &d : m_destroyEvents)
        if (same(d, ev)) return false;
      return true;
    }
    if (impl(ev) == nullptr || ev.ts < m_currentTs || (ev.ts == m_currentTs && ev.uid <= m_currentUid) ||
        impl(ev)->cancelled)
      return true;
    return false;
  }
  void Remove(const nsgpu_event_id &id) {  // :256-290
    if (id.uid == 2) {
      for (auto i = m_destroyEvents.begin(); i != m_destroyEvents.end(); i++) {
        if (same(*i, id)) {
          m_destroyEvents.erase(i);
          break;
        }
      }
      return;
    }
    if (IsExpired(id)) return;
    Event event;
    event.impl = impl(id);
    event.key.ts = id.ts;
    event.key.ctx = id.context;
    event.key.uid = id.uid;
    m_events->Remove(event);
    event.impl->cancelled = true;
    event.impl->Unref();
    m_unscheduledEvents--;
  }
  void Cancel(const nsgpu_event_id &id) {  // :292-302
    if (!IsExpired(id)) impl(id)->cancelled = true;
  }
  void Destroy() {  // :76-91
    while (!m_destroyEvents.empty()) {
      EventImpl *ev = impl(m_destroyEvents.front());
      m_destroyEvents.pop_front();
      if (!ev->cancelled) ev->Invoke();
    }
  }
};

