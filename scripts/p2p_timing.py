"""Diagnostic: GPU p2p engine timing on grids vs the oracle (events/s)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "ns-3-dev-dnemu_amd"), os.path.join(REPO, "oracle")]
import numpy as np  # noqa: E402
import nsgpu  # noqa: E402
import nsref  # noqa: E402
import p2p  # noqa: E402

for n in [int(a) for a in sys.argv[1:]] or [16, 32, 64, 128]:
    t0 = time.time()
    g = p2p.grid(n, n)
    tb = time.time() - t0
    s = g.c_struct()
    st = p2p.P2PStats()
    devc = np.zeros(s.n_devices, p2p.DEV_COUNTERS_DTYPE)
    appc = np.zeros(s.n_apps, p2p.APP_COUNTERS_DTYPE)
    osecs, _ = nsref.p2p_run(s, st, devc, appc)
    eng = p2p.Engine(g)
    eng.reset()
    eng.launch()
    eng.results()
    tm = nsgpu.Timer()
    eng.reset()
    tm.start(None)
    eng.launch()
    tm.stop(None)
    ms = tm.elapsed_ms()
    gst, gdevc, gappc, _ = eng.results()
    ok = gst.digest == st.digest and gst.dispatched == st.dispatched
    print(f"grid {n}x{n}: build {tb:.2f}s events {gst.dispatched} windows {gst.windows} maxw {gst.max_window} "
          f"gpu {ms:.1f} ms = {gst.dispatched / ms / 1e3:.2f} Mev/s | oracle {osecs:.3f}s = "
          f"{st.dispatched / osecs / 1e6:.2f} Mev/s | match {ok}", flush=True)
