"""Diagnostic: per-phase cycle split of the packed hold kernel (s_memtime stamps, wave 0 view)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ns-3-dev-dnemu_amd"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import nsgpu  # noqa: E402
from bench import load_distribution, DIST_FILE  # noqa: E402

dist = load_distribution(DIST_FILE)
prof = nsgpu.DeviceBuffer(7 * 8)
prof.zero()
nsgpu.check(nsgpu.lib().nsgpu_hold_set_profile(prof.ptr))
h = nsgpu.HoldRun(dist, int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000)
h.launch()
st, _, _ = h.result()
cyc = prof.download(np.uint64, 7)
names = ["A+B1 cand/scan", "B2 ballot", "C commit", "D rank/search", "E chunk/scan", "F write", "-"]
tot = cyc[:6].sum()
print("rounds", st.rounds, "cycles/round", tot / st.rounds)
for n, c in zip(names, cyc[:6]):
    print(f"{n:16s} {c / st.rounds:9.1f} cyc/round  {100 * c / tot:5.1f}%")
nsgpu.check(nsgpu.lib().nsgpu_hold_set_profile(None))
t = nsgpu.Timer()
t.start(None)
h.launch()
t.stop(None)
print("unprofiled ms", t.elapsed_ms(), "events", st.dispatched)
