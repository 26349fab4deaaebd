"""Diagnostic: GPU time of the p2p window pipeline on an n x n grid (HIP events on the engine stream)."""
import ctypes as C
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "ns-3-dev-dnemu_amd")]
import nsgpu  # noqa: E402
import p2p  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 128
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
eng = p2p.Engine(p2p.grid(n, n))
for i in range(reps):
    t0 = time.perf_counter()
    st, _, _, _ = eng.run()
    wall = time.perf_counter() - t0
    ms = C.c_double()
    nsgpu.check(nsgpu.lib().nsgpu_p2p_last_run_ms(eng.h, C.byref(ms)))
    print(f"grid {n}: events {st.dispatched} windows {st.windows} digest {st.digest:#x}  gpu {ms.value:.1f} ms "
          f"({1e3 * ms.value / max(st.windows, 1):.1f} us/window, {st.dispatched / ms.value / 1e3:.2f} M ev/s)  "
          f"wall {wall * 1e3:.1f} ms")
