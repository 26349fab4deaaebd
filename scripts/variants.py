"""Diagnostic: config 4 (wide engine) per-run time and per-kernel window times for each library variant given
on the command line (paths; each in its own process, NSGPU_LIB)."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys, time, json
sys.path[:0] = [os.path.join(sys.argv[1], "ns-3-dev-dnemu_amd")]
import nsgpu, p2p, ctypes as C
nsgpu.check(nsgpu.lib().nsgpu_set_device(0))
eng = p2p.Engine(p2p.grid(int(sys.argv[2]), int(sys.argv[2])))
best = None
for _ in range(4):
    st, _, _, _ = eng.run()
    ms = C.c_double()
    nsgpu.check(nsgpu.lib().nsgpu_p2p_last_run_ms(eng.h, C.byref(ms)))
    best = ms.value if best is None else min(best, ms.value)
prof = eng.profile(sample_every=4)
print(json.dumps({"lib": os.environ["NSGPU_LIB"], "windows": int(st.windows), "dispatched": int(st.dispatched),
                  "digest": int(st.digest), "run_ms": round(best, 2),
                  "us_per_window": round(1e3 * best / max(int(st.windows), 1), 2),
                  "kernel_us": {k: round(v[0] * 1e3, 2) for k, v in prof.items()}}))
'''
n = os.environ.get("GRID", "128")
for lib in sys.argv[1:]:
    env = dict(os.environ, NSGPU_LIB=os.path.abspath(lib))
    r = subprocess.run([sys.executable, "-c", CHILD, REPO, n], env=env, capture_output=True, text=True, timeout=240)
    print(r.stdout.strip() or r.stderr[-800:], flush=True)
