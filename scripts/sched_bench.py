"""HipBatchScheduler (ns3::Scheduler over nsgpu_sched_*) on config 1's hold model, against the oracle's
MapScheduler / HeapScheduler on the same distribution (one host core each).  Prints one JSON line.

The GPU side is build/sched_bench (scripts/sched_bench.cc): one C-ABI call per Schedule and per dispatch,
as the ns-3 plugin makes them.  Its digest must equal the oracle's (same pop order)."""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "oracle")]
import nsref  # noqa: E402

DIST = os.path.join(REPO, "tests", "golden", "bench_dist_u01_10k.txt")
holds = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
out = {"workload": f"bench-simulator hold model: 10000 pending, U[0,1) s delays, {holds} holds"}
dist = nsref.load_distribution(DIST)  # ReadDistribution: seconds -> ns
ns_file = os.path.join(tempfile.mkdtemp(), "dist_ns.txt")
np.savetxt(ns_file, dist, fmt="%d")
for batch in (1024, 4096, 16384):
    r = subprocess.run([os.path.join(REPO, "ns-3-dev-dnemu_amd", "build", "sched_bench"), ns_file, str(holds),
                        str(batch)], capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        raise SystemExit(r.stderr)
    g = json.loads(r.stdout.strip().splitlines()[-1])
    out[f"hip_batch_scheduler_b{batch}"] = {"events_per_s": g["events"] / g["seconds"], "seconds": g["seconds"],
                                           "digest": g["digest"], "events": g["events"]}
    print(json.dumps({f"b{batch}": out[f"hip_batch_scheduler_b{batch}"]}), flush=True)  # (progress)
for name, sched in (("map", nsref.SCHED_MAP), ("heap", nsref.SCHED_HEAP)):
    res, _, _ = nsref.churn_run(dist, holds, scheduler=sched)
    out[f"oracle_{name}"] = {"events_per_s": res.dispatched / res.run_seconds, "seconds": res.run_seconds,
                             "digest": res.digest, "events": res.dispatched}
out["digest_match"] = all(v["digest"] == out["oracle_map"]["digest"] and v["events"] == out["oracle_map"]["events"]
                          for k, v in out.items() if k.startswith("hip_batch"))
print(json.dumps(out))
