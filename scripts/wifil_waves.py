"""Diagnostic: k_wl_stepw's waves on the closed-loop bench workload (lib/libnsgpu_prof.so, NSGPU_PHASE_PROF):
lifetime by events per wave, the longest wave, the epoch span and dispatch spread, and the wave's sections
(s_memtime ticks: 100 MHz constant clock on gfx950)."""
import ctypes as C
import os
import sys
import types

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("NSGPU_LIB", os.path.join(REPO, "ns-3-dev-dnemu_amd", "lib", "libnsgpu_prof.so"))
sys.path[:0] = [REPO, os.path.join(REPO, "ns-3-dev-dnemu_amd"), os.path.join(REPO, "tests")]
import nsgpu  # noqa: E402
import bench  # noqa: E402

stop = float(sys.argv[1]) if len(sys.argv) > 1 else 0.05
args = types.SimpleNamespace(wifi_side=100, wifi_loop_stop=stop)
w = bench.WifiLoop(args, None)
buf = (C.c_ulonglong * 28)()
f = nsgpu.lib().nsgpu_wifil_prof_read
f.restype = C.c_int
nsgpu.check(f(buf))
disp, _dig, info = w.run(w.sc)
nsgpu.check(f(buf))
sw, sw2 = buf[8:24], buf[24:28]
epochs = info["epochs"]
print(f"dispatched {disp}, epochs {epochs}, us/epoch (host clock) {info['us_per_epoch']:.1f}")
waves = sum(sw[0:5])
for c in range(5):
    n = sw[c]
    print(f"  waves with {c}{'+' if c == 4 else ''} events: {n / max(epochs, 1):8.1f} per epoch, mean lifetime "
          f"{sw[5 + c] / max(n, 1):8.1f} ticks")
print(f"  longest wave {sw[10]} ticks ({sw[11]} events)")
print(f"  epoch span (last end - first start) {sw[12] / max(epochs, 1):.1f} ticks, dispatch spread "
      f"{sw[15] / max(epochs, 1):.1f} ticks")
print(f"  sections per wave: loads {sw2[1] / waves:.1f}, event loop {sw2[2] / waves:.1f}, flush + write-backs "
      f"{sw2[3] / waves:.1f} ticks")
