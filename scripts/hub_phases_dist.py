"""Diagnostic: hub_phases.py for the partitioned engine (config 5 through one loopback partition): the hub
blocks' phase totals over the run (lib/libnsgpu_prof.so; g_phase[22..31])."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("NSGPU_LIB", os.path.join(REPO, "ns-3-dev-dnemu_amd", "lib", "libnsgpu_prof.so"))
sys.path[:0] = [os.path.join(REPO, "ns-3-dev-dnemu_amd")]
import numpy as np  # noqa: E402
import nsgpu  # noqa: E402
import p2p  # noqa: E402

nsgpu.check(nsgpu.lib().nsgpu_set_device(0))
grp = p2p.LoopbackGroup(p2p.dumbbell(499_999), 1)
grp.run()
buf = np.zeros(64, np.uint64)
nsgpu.check(nsgpu.lib().nsgpu_p2p_phase_read(buf.ctypes.data, 64, 1))
st, _, _, _ = grp.run()
nsgpu.check(nsgpu.lib().nsgpu_p2p_phase_read(buf.ctypes.data, 64, 1))
calls = max(int(buf[28]), 1)
print(f"partitioned dumbbell x1: {st.dispatched} events, {st.windows} windows, {calls} hub-block calls")
for i, nm in ((22, "wait for the holders"), (24, "window scan + sort"), (25, "node parts"), (23, "segment ops -> LDS"),
              (26, "device steps"), (27, "publish / totals")):
    print(f"  {nm:20s} total {buf[i] * 10.0 / 1e3:10.1f} us, {buf[i] * 10.0 / calls / 1e3:8.3f} us per hub call")
print(f"  events in hub calls {int(buf[30])}, serial node parts {int(buf[29])}; serial loop time {buf[31] * 10.0 / 1e3:.1f} us")
