"""Diagnostic: k_wl_stepw's waves on the closed-loop bench workload (lib/libnsgpu_prof.so, NSGPU_PHASE_PROF):
per-wave s_memtime stamps (shader clock ticks) of WREC_E consecutive epochs, recorded without atomics — the
epoch span, when waves start (dispatch), lifetimes by events, and the waves' sections (loads / event loop /
flush and write-backs)."""
import ctypes as C
import os
import sys
import types

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("NSGPU_LIB", os.path.join(REPO, "ns-3-dev-dnemu_amd", "lib", "libnsgpu_prof.so"))
sys.path[:0] = [REPO, os.path.join(REPO, "ns-3-dev-dnemu_amd"), os.path.join(REPO, "tests")]
import nsgpu  # noqa: E402
import bench  # noqa: E402

WREC_E, WREC_P = 8, 16384
stop = float(sys.argv[1]) if len(sys.argv) > 1 else 0.05
target = int(sys.argv[2]) if len(sys.argv) > 2 else 400
args = types.SimpleNamespace(wifi_side=100, wifi_loop_stop=stop)
w = bench.WifiLoop(args, None)
f = nsgpu.lib().nsgpu_wifil_prof_waves
f.restype = C.c_int
f.argtypes = [C.c_uint32, C.c_void_p]
nsgpu.check(f(target, None))
disp, _dig, info = w.run(w.sc)
rec = np.zeros((WREC_E, WREC_P, 5), np.uint64)
nsgpu.check(f(target, rec.ctypes.data))
n = w.sc["phys"].n_phy
print(f"dispatched {disp}, epochs {info['epochs']}, us/epoch (host clock) {info['us_per_epoch']:.1f}")
for e in range(WREC_E):
    r = rec[e, :n].astype(np.int64)
    if not r[:, 3].any():
        continue
    t0 = r[:, 0].min()
    st, en, ev = r[:, 0] - t0, r[:, 3] - t0, r[:, 4]
    life = en - st
    print(f"epoch {target + e}: span {en.max()} ticks, last start {st.max()}, events {ev.sum()}, "
          f"life p50 {np.percentile(life, 50):.0f} p90 {np.percentile(life, 90):.0f} max {life.max()} "
          f"(events {ev[life.argmax()]}, phy {life.argmax()}, start {st[life.argmax()]})")
    for c in range(4):
        m = ev == c if c < 3 else ev >= 3
        if m.any():
            print(f"    {c}{'+' if c == 3 else ''} events: {m.sum():5d} waves, life mean {life[m].mean():8.0f}, sections "
                  f"loads {(r[m, 1] - r[m, 0]).mean():7.0f} loop {(r[m, 2] - r[m, 1]).mean():7.0f} "
                  f"flush {(r[m, 3] - r[m, 2]).mean():7.0f}")
    q = np.percentile(st, [10, 50, 90])
    print(f"    starts p10 {q[0]:.0f} p50 {q[1]:.0f} p90 {q[2]:.0f}; waves ending after 90% of the span: "
          f"{(en > 0.9 * en.max()).sum()}")
