"""Config 4 weak-scaled to 128 x 128N in N row bands (bench.py's --gpus N layout) as a LOOPBACK group of N
partitions on one GPU (nsgpu_p2p_group_*: the partitioned algorithm with device copies in place of RCCL).

One GPU runs every partition's kernels in turn, so the run time is not a multi-GPU number; what it measures is
each partition's per-window kernel cost at N ranks — the part of the window that grows with N (k_gtile ranks
this rank's records against every rank's).  Run it under `rocprofv3 --kernel-trace --stats` for per-kernel
averages.  Usage: python scripts/p2p_group_scale.py N [grid] [steps]"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ns-3-dev-dnemu_amd"))

import p2p  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    g = int(sys.argv[2]) if len(sys.argv) > 2 else 128
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    sc = p2p.grid(g, g * n)
    grp = p2p.LoopbackGroup(sc, n)
    res = grp.run()  # (warm-up: graphs built)
    t0 = time.perf_counter()
    for _ in range(steps):
        res = grp.run()
    dt = (time.perf_counter() - t0) / steps
    st = res[0]
    print(json.dumps({"partitions": n, "grid": [g, g * n], "events": int(st.dispatched), "windows": int(st.windows),
                      "s_per_run": dt, "us_per_window_all_partitions": dt * 1e6 / max(int(st.windows), 1)}),
          flush=True)


if __name__ == "__main__":
    main()
