// sched_bench — utils/bench-simulator.cc's hold model (config 1) driven through HipBatchScheduler's C-ABI
// exactly as ns3::HipBatchScheduler calls it from DefaultSimulatorImpl: one nsgpu_sched_insert per
// Schedule (n = 1) and one nsgpu_sched_remove_next per dispatched event, the closures staying on the host.
// It measures that integration path (host closures, device-sorted pending set), not the GPU-resident
// churn kernel (nsgpu_hold_run).  Prints one JSON line: events, seconds of the event loop, digest (the
// nsgpu_dispatch_digest_term sum, equal to the oracle's MapScheduler run of the same distribution).
//
// usage: sched_bench <distribution file (one delay in ns per line)> <holds> [batch]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "nsgpu.h"

static void die(const char *what) {
  std::fprintf(stderr, "sched_bench: %s: %s\n", what, nsgpu_last_error());
  std::exit(1);
}

int main(int argc, char **argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s dist.txt holds [batch]\n", argv[0]);
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
  const uint32_t batch = argc > 3 ? (uint32_t)std::strtoul(argv[3], nullptr, 10) : 4096u;
  if (d.empty()) die("empty distribution");
  if (nsgpu_set_device(0)) die("nsgpu_set_device");
  nsgpu_sched *s = nullptr;
  if (nsgpu_sched_create(batch, nullptr, &s)) die("nsgpu_sched_create");
  const uint64_t n = d.size();
  // RunBench (bench-simulator.cc:79-107): Schedule (NanoSeconds (d[i]), &Bench::Cb) for i < N
  uint32_t uid = 4;
  for (uint64_t i = 0; i < n; i++) {
    const nsgpu_event e{d[i], uid++, 0xffffffffu, 0};
    if (nsgpu_sched_insert(s, &e, 1)) die("insert");
  }
  // Simulator::Run with Bench::Cb (:109-127): the k-th dispatch schedules now + d[k mod N] while k <= total
  const auto t0 = std::chrono::steady_clock::now();
  uint64_t k = 0, digest = 0;
  for (;;) {
    int empty = 0;
    if (nsgpu_sched_is_empty(s, &empty)) die("is_empty");
    if (empty) break;
    nsgpu_event e;
    if (nsgpu_sched_remove_next(s, &e)) die("remove_next");
    digest += nsgpu_dispatch_digest_term(k, e.ts, e.uid);
    if (k <= total) {
      const nsgpu_event c{e.ts + d[k % n], uid++, 0xffffffffu, 0};
      if (nsgpu_sched_insert(s, &c, 1)) die("insert");
    }
    k++;
  }
  const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  nsgpu_sched_destroy(s);
  std::printf("{\"events\": %llu, \"seconds\": %.6f, \"digest\": %llu, \"batch\": %u, \"pending\": %llu}\n",
              (unsigned long long)k, secs, (unsigned long long)digest, batch, (unsigned long long)n);
  return 0;
}
