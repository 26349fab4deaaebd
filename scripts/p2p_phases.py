"""Diagnostic: in-kernel phase times of the p2p window pipeline (lib/libnsgpu_prof.so, NSGPU_LIB)."""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("NSGPU_LIB", os.path.join(REPO, "ns-3-dev-dnemu_amd", "lib", "libnsgpu_prof.so"))
sys.path[:0] = [os.path.join(REPO, "ns-3-dev-dnemu_amd")]
import numpy as np  # noqa: E402
import nsgpu  # noqa: E402
import p2p  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 128
eng = p2p.Engine(p2p.grid(n, n))
eng.run()
buf = np.zeros(64, np.uint64)
nsgpu.check(nsgpu.lib().nsgpu_p2p_phase_read(buf.ctypes.data, 64, 1))
st, _, _, _ = eng.run()
ms = C.c_double()
nsgpu.check(nsgpu.lib().nsgpu_p2p_last_run_ms(eng.h, C.byref(ms)))
nsgpu.check(nsgpu.lib().nsgpu_p2p_phase_read(buf.ctypes.data, 64, 1))
w = max(int(st.windows), 1)
print(f"grid {n}: {st.dispatched} events, {w} windows, {ms.value:.1f} ms ({1e3 * ms.value / w:.2f} us/window)")
names = {0: "k2_pa: entry -> last-window slot loads", 1: "k2_pa: append + partition", 2: "k2_pa: publish_min+digest",
         8: "k2_handle: entry -> ctl (block 0)", 9: "k2_handle: body (block 0: holders)",
         16: "k2_scan: entry -> slot loads", 17: "k2_scan: rank scatter to LDS", 18: "k2_scan: scan",
         19: "k2_scan: sinfo stores", 20: "k2_scan: bookkeeping"}
for i, nm in names.items():
    print(f"  {nm:32s} {buf[i] * 10.0 / w / 1e3:8.3f} us/window")
prof = eng.profile(sample_every=4)
print("  kernel us/launch (hipExtLaunchKernel events):", {k: round(v[0] * 1e3, 2) for k, v in prof.items()})
