"""Diagnostic: first divergence between the wide engine's pop log and the oracle's on a scenario
(tests/test_gpu_wide.py's burst case by default).  Writes gpurun_out/wide_debug.npz."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "ns-3-dev-dnemu_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402
import nsgpu  # noqa: E402
import p2p  # noqa: E402
from test_gpu_trace import oracle_full  # noqa: E402

nsgpu.check(nsgpu.lib().nsgpu_set_device(0))
rows = cols = 64
n = rows * cols
rng = np.random.default_rng(3)
flows = [(int(s), int(d)) for s, d in zip(rng.integers(0, n, 4500), rng.integers(0, n, 4500)) if s != d]
sc = p2p.grid(rows, cols, flows=flows, stop_ns=130_000_000, sim_stop_ns=140_000_000)
cap = 600_000
o = oracle_full(sc, cap)
for narrow in (False, True):
    if narrow:
        os.environ["NSGPU_P2P_NARROW"] = "1"
    eng = p2p.Engine(sc, log_cap=cap)
    os.environ.pop("NSGPU_P2P_NARROW", None)
    st, devc, appc, (lts, luid, lctx) = eng.run(log_n=cap)
    m = min(int(st.dispatched), int(o[0].dispatched))
    ots, ouid, octx = o[3]
    bad = np.nonzero((lts[:m] != ots[:m]) | (luid[:m] != ouid[:m]) | (lctx[:m] != octx[:m]))[0]
    print(f"narrow={narrow} wide={eng.wide()} dispatched gpu {st.dispatched} oracle {o[0].dispatched} windows {st.windows} "
          f"refits {st.refits} max_window {st.max_window} next_uid {st.next_uid}/{o[0].next_uid} first_bad {bad[:5]}")
    if len(bad):
        b = int(bad[0])
        for k in range(max(0, b - 3), min(m, b + 8)):
            print(k, "gpu", int(lts[k]), int(luid[k]), int(lctx[k]), " oracle", int(ots[k]), int(ouid[k]), int(octx[k]))
    eng.close()
