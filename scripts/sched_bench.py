"""The host-closure plugin path on config 1's hold model — ns3::HipSimulatorImpl's call sequence (simimpl)
and ns3::HipBatchScheduler's under DefaultSimulatorImpl (scheduler) — against the oracle's MapScheduler /
HeapScheduler on the same distribution (one host core each).  Prints one JSON line.

The GPU side is build/sched_bench (scripts/sched_bench.cc): the C-ABI calls the ns-3 plugins make, one
heap-allocated closure per event as in the oracle.  Its digest must equal the oracle's (same pop order)."""
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
holds = int(sys.argv[1]) if len(sys.argv) > 1 else 5_000_000
out = {"workload": f"bench-simulator hold model: 10000 pending, U[0,1) s delays, {holds} holds"}
dist = nsref.load_distribution(DIST)  # ReadDistribution: seconds -> ns
ns_file = os.path.join(tempfile.mkdtemp(), "dist_ns.txt")
np.savetxt(ns_file, dist, fmt="%d")
runs = [("simimpl", 0), ("scheduler", 0), ("scheduler", 4096)]
for mode, batch in runs:
    r = subprocess.run([os.path.join(REPO, "ns-3-dev-dnemu_amd", "build", "sched_bench"), ns_file, str(holds),
                        mode, str(batch)], capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        raise SystemExit(r.stderr)
    g = json.loads(r.stdout.strip().splitlines()[-1])
    key = f"hip_{mode}_" + (f"b{batch}" if batch else "adaptive")
    out[key] = dict(g, events_per_s=g["events"] / g["seconds"])
    print(json.dumps({key: out[key]}), flush=True)  # (progress)
for name, sched in (("map", nsref.SCHED_MAP), ("heap", nsref.SCHED_HEAP)):
    res, _, _ = nsref.churn_run(dist, holds, scheduler=sched)
    out[f"oracle_{name}"] = {"events_per_s": res.dispatched / res.run_seconds, "seconds": res.run_seconds,
                             "digest": res.digest, "events": res.dispatched}
out["digest_match"] = all(v["digest"] == out["oracle_map"]["digest"] and v["events"] == out["oracle_map"]["events"]
                          for k, v in out.items() if k.startswith("hip_"))
print(json.dumps(out))
