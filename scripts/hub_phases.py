"""Diagnostic: where the hub blocks' time goes on the dumbbell (config 5 shape; lib/libnsgpu_prof.so):
thread 0 of every hub block adds its phase times (s_memrealtime, 100 MHz) into g_phase[24..28]."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("NSGPU_LIB", os.path.join(REPO, "ns-3-dev-dnemu_amd", "lib", "libnsgpu_prof.so"))
sys.path[:0] = [os.path.join(REPO, "ns-3-dev-dnemu_amd")]
import numpy as np  # noqa: E402
import nsgpu  # noqa: E402
import p2p  # noqa: E402

leaves = int(sys.argv[1]) if len(sys.argv) > 1 else 499_999
nsgpu.check(nsgpu.lib().nsgpu_set_device(0))
eng = p2p.Engine(p2p.dumbbell(leaves))
eng.run()
buf = np.zeros(64, np.uint64)
nsgpu.check(nsgpu.lib().nsgpu_p2p_phase_read(buf.ctypes.data, 64, 1))
st, _, _, _ = eng.run()
nsgpu.check(nsgpu.lib().nsgpu_p2p_phase_read(buf.ctypes.data, 64, 1))
w = max(int(st.windows), 1)
calls = max(int(buf[28]), 1)
print(f"dumbbell {leaves} leaves: {st.dispatched} events, {w} windows, {calls} hub-block calls ({calls / w:.2f} a window)")
for i, nm in ((22, "wait for the holders"), (24, "window scan + sort"), (25, "node parts"), (23, "segment ops -> LDS"),
              (26, "device steps"), (27, "publish / totals")):
    print(f"  {nm:20s} {buf[i] * 10.0 / calls / 1e3:8.3f} us per hub call")
print(f"  events in hub calls {int(buf[30])} ({int(buf[30]) / calls:.0f} a call), of them serial node parts {int(buf[29])}; "
      f"serial loop time {buf[31] * 10.0 / calls / 1e3:.3f} us per hub call")
