"""Times the config-5 dumbbell partitioned the way simple-distributed.cc assigns system ids, all
partitions on one GPU (loopback group), against the oracle; checks counters and digest.
Usage: python scripts/dumbbell_dist_timing.py <leaves per side> <partitions>"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "ns-3-dev-dnemu_amd"), os.path.join(REPO, "oracle")]
import numpy as np  # noqa: E402

import nsref  # noqa: E402
import p2p  # noqa: E402

n, k = int(sys.argv[1]), int(sys.argv[2])
sc = p2p.dumbbell(n)
s = sc.c_struct()
st = p2p.P2PStats()
devc = np.zeros(s.n_devices, p2p.DEV_COUNTERS_DTYPE)
appc = np.zeros(s.n_apps, p2p.APP_COUNTERS_DTYPE)
cpu_s, _ = nsref.p2p_run(s, st, devc, appc, 0)
grp = p2p.LoopbackGroup(sc, k, owner=p2p.dumbbell_owner(n, k))
t0 = time.time()
gst, gdevc, gappc, _ = grp.run()
wall = time.time() - t0
ok = gst.digest == st.digest and gst.dispatched == st.dispatched and np.array_equal(gdevc, devc) and \
    np.array_equal(gappc, appc)
print(f"dumbbell-dist nodes={sc.n_nodes} parts={k} events={st.dispatched} windows={gst.windows} gpu_s={wall:.3f} "
      f"oracle_run_s={cpu_s:.3f} bit_exact={ok}", flush=True)
sys.exit(0 if ok else 1)
