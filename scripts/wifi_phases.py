"""Diagnostic: where the per-phy Wi-Fi kernel's wave time goes (lib/libnsgpu_prof.so, NSGPU_PHASE_PROF):
s_memtime deltas between the loop's sections, summed over waves (lane 0 of each)."""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("NSGPU_LIB", os.path.join(REPO, "ns-3-dev-dnemu_amd", "lib", "libnsgpu_prof.so"))
sys.path[:0] = [os.path.join(REPO, "ns-3-dev-dnemu_amd")]
import nsgpu  # noqa: E402
import wifi  # noqa: E402

nsgpu.check(nsgpu.lib().nsgpu_set_device(0))
stop = float(sys.argv[1]) if len(sys.argv) > 1 else 0.5
eng = wifi.Engine(wifi.wifi_grid(n_side=100, stop_s=stop))
eng.run()
buf = (C.c_ulonglong * 16)()
f = nsgpu.lib().nsgpu_wifi_phase_read
f.restype = C.c_int
nsgpu.check(f(buf, 1))
eng.run()
st = eng.stats()
nsgpu.check(f(buf, 0))
names = ["pending EndReceive choice", "SendPacket/EndReceive", "NiChanges: end entry, running sums", "state/sync", "CCA",
         "counters/digest", "kind decision, operands", "NiChanges: eager cursor", "NiChanges: fold / start", "scan for the next Receive"]
tot = sum(buf[:10])
print(f"dispatched {st.dispatched}, store {eng.store()}")
for i, n in enumerate(names):
    print(f"  {n:24s} {buf[i] / tot * 100:6.1f} %")
print(f"  slowest wave / mean wave: {buf[14] / (tot / max(buf[15], 1)):.2f} ({buf[15]} waves)")
