// sched_bench — utils/bench-simulator.cc's hold model (config 1) driven through libnsgpu's C-ABI exactly
// as the ns-3 plugins call it, the closures staying on the host:
//   mode "scheduler": ns3::HipBatchScheduler under DefaultSimulatorImpl — one nsgpu_sched_insert per
//                     Schedule (n = 1), one nsgpu_sched_remove_next per dispatch;
//   mode "simimpl":   ns3::HipSimulatorImpl (hip-simulator-impl.cc) — Run pops windows
//                     (nsgpu_sim_pop_window) and calls nsgpu_sim_begin per event; Bench::Cb's
//                     Simulator::Schedule is the plugin's Schedule: Now and GetContext through
//                     nsgpu_sim_state, then nsgpu_sim_insert.
// Either way every event is a heap-allocated closure with a virtual Invoke and a reference count
// (MakeEvent / EventImpl::Unref), as the oracle's timed MapScheduler run allocates them.
// It measures that integration path, not the GPU-resident churn kernel (nsgpu_hold_run).  Prints one JSON
// line: events, seconds of the event loop, digest (the nsgpu_dispatch_digest_term sum, equal to the
// oracle's MapScheduler run of the same distribution), refills of the front.
//
// usage: sched_bench <distribution file (one delay in ns per line)> <holds> <mode> [batch, 0 = adaptive]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "nsgpu.h"

static void die(const char *what) {
  std::fprintf(stderr, "sched_bench: %s: %s\n", what, nsgpu_last_error());
  std::exit(1);
}

namespace {
struct EventImpl {  // ns3::EventImpl: ref count + cancel flag + virtual Notify
  int refs = 1;
  bool cancelled = false;
  virtual ~EventImpl() {}
  virtual void Notify() = 0;
  void Invoke() {
    if (!cancelled) Notify();
  }
  void Unref() {
    if (--refs == 0) delete this;
  }
};

struct Bench {  // bench-simulator.cc:32-45, Cb :109-127
  const std::vector<uint64_t> *dist;
  uint64_t cur = 0, n = 0, total = 0;
  nsgpu_sched *sched = nullptr;  // scheduler mode
  nsgpu_sim *rt = nullptr;       // simimpl mode
  uint32_t uid = 4;
  uint64_t now = 0;
  uint32_t ctx = 0xffffffffu;
  void Schedule(uint64_t delay);
  void Cb() {
    if (n > total) return;
    if (cur == dist->size()) cur = 0;
    Schedule((*dist)[cur]);
    cur++;
    n++;
  }
};
struct BenchCb : EventImpl {
  Bench *b;
  explicit BenchCb(Bench *x) : b(x) {}
  void Notify() override { b->Cb(); }
};

void Bench::Schedule(uint64_t delay) {
  EventImpl *ev = new BenchCb(this);
  if (rt) {  // HipSimulatorImpl::Schedule: NowTs (), GetContext (), Enqueue -> nsgpu_sim_insert
    uint64_t t = 0;
    uint32_t c = 0;
    if (nsgpu_sim_state(rt, &t, nullptr, nullptr, nullptr)) die("state");
    if (nsgpu_sim_state(rt, nullptr, &c, nullptr, nullptr)) die("state");
    uint32_t u = 0;
    if (nsgpu_sim_insert(rt, t + delay, c, (uint64_t)(uintptr_t)ev, &u)) die("insert");
  } else {  // DefaultSimulatorImpl::Schedule -> HipBatchScheduler::Insert
    const nsgpu_event e{now + delay, uid++, ctx, (uint64_t)(uintptr_t)ev};
    if (nsgpu_sched_insert(sched, &e, 1)) die("insert");
  }
}
}  // namespace

int main(int argc, char **argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s dist.txt holds scheduler|simimpl [batch]\n", argv[0]);
    return 2;
  }
  std::vector<uint64_t> d;
  {
    FILE *f = std::fopen(argv[1], "r");
    if (!f) die("open distribution");
    unsigned long long v;
    while (std::fscanf(f, "%llu", &v) == 1) d.push_back(v);
    std::fclose(f);
  }
  const uint64_t total = std::strtoull(argv[2], nullptr, 10);
  const bool simimpl = std::strcmp(argv[3], "simimpl") == 0;
  const uint32_t batch = argc > 4 ? (uint32_t)std::strtoul(argv[4], nullptr, 10) : 0u;
  if (d.empty()) die("empty distribution");
  if (nsgpu_set_device(0)) die("nsgpu_set_device");
  Bench b;
  b.dist = &d;
  b.total = total;
  if (simimpl) {
    if (nsgpu_sim_create(batch, nullptr, &b.rt)) die("nsgpu_sim_create");
  } else {
    if (nsgpu_sched_create(batch, nullptr, &b.sched)) die("nsgpu_sched_create");
  }
  // RunBench (bench-simulator.cc:79-107): Schedule (NanoSeconds (d[i]), &Bench::Cb) for i < N
  for (uint64_t i = 0; i < d.size(); i++) b.Schedule(d[i]);
  const auto t0 = std::chrono::steady_clock::now();
  uint64_t k = 0, digest = 0;
  if (simimpl) {  // HipSimulatorImpl::Run
    std::vector<nsgpu_event> w(4096);
    if (nsgpu_sim_set_stop(b.rt, 0)) die("set_stop");
    for (;;) {
      uint32_t n = 0;
      if (nsgpu_sim_pop_window(b.rt, w.data(), (uint32_t)w.size(), &n)) die("pop_window");
      if (n == 0) break;
      for (uint32_t i = 0; i < n; i++) {
        int skip = 0;
        if (nsgpu_sim_begin(b.rt, &w[i], &skip)) die("begin");
        if (skip) continue;
        EventImpl *ev = (EventImpl *)(uintptr_t)(w[i].handle & ~1ull);
        ev->Invoke();
        ev->Unref();
      }
    }
    if (nsgpu_sim_host_stats(b.rt, &k, nullptr, &digest)) die("host_stats");
  } else {  // DefaultSimulatorImpl::Run over HipBatchScheduler
    for (;;) {
      int empty = 0;
      if (nsgpu_sched_is_empty(b.sched, &empty)) die("is_empty");
      if (empty) break;
      nsgpu_event e;
      if (nsgpu_sched_remove_next(b.sched, &e)) die("remove_next");
      digest += nsgpu_dispatch_digest_term(k, e.ts, e.uid);
      b.now = e.ts;
      b.ctx = e.context;
      EventImpl *ev = (EventImpl *)(uintptr_t)e.handle;
      ev->Invoke();
      ev->Unref();
      k++;
    }
  }
  const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  uint64_t refills = 0, front = 0;
  double refill_us = 0;
  if (simimpl) {  // (the runtime's host-closure queue: the same front-batch scheduler)
    nsgpu_sim_sched_stats(b.rt, &refills, &front, &refill_us);
    nsgpu_sim_free(b.rt);
  } else {
    nsgpu_sched_stats(b.sched, &refills, &front, &refill_us);
    nsgpu_sched_destroy(b.sched);
  }
  std::printf("{\"mode\": \"%s\", \"what\": \"host-structure throughput (host closures; no GPU-resident events)\", \"events\": %llu, \"seconds\": %.6f, \"digest\": %llu, \"batch\": %u, "
              "\"pending\": %llu, \"refills\": %llu, \"front\": %llu, \"refill_us\": %.2f}\n",
              simimpl ? "simimpl" : "scheduler", (unsigned long long)k, secs, (unsigned long long)digest, batch,
              (unsigned long long)d.size(), (unsigned long long)refills, (unsigned long long)front, refill_us);
  return 0;
}
