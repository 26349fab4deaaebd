"""Diagnostic: the deferred accounting's phases in one sampled window (lib/libnsgpu_prof.so, NSGPU_LIB):
records arrived, block scan, per-rank arrays + lookups + barrier, resolve/log/digest (s_memrealtime, 10 ns)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("NSGPU_LIB", os.path.join(REPO, "ns-3-dev-dnemu_amd", "lib", "libnsgpu_prof.so"))
sys.path[:0] = [os.path.join(REPO, "ns-3-dev-dnemu_amd")]
import numpy as np  # noqa: E402
import nsgpu  # noqa: E402
import p2p  # noqa: E402

eng = p2p.Engine(p2p.grid(128, 128))
eng.set_eager(True)
for rep in range(2):
    buf = np.zeros(64, np.uint64)
    nsgpu.check(nsgpu.lib().nsgpu_p2p_phase_read(buf.ctypes.data, buf.size, 1))
    eng.run()
    nsgpu.check(nsgpu.lib().nsgpu_p2p_phase_read(buf.ctypes.data, buf.size, 1))
    for i, name in ((16, "records arrived"), (18, "block scan"), (20, "arrays + lookups + barrier"),
                    (22, "resolve / log / digest")):
        n = max(int(buf[i + 1]), 1)
        print(f"rep {rep} {name:28s} {buf[i] * 0.01 / n:8.2f} us  (n={int(buf[i + 1])})", flush=True)
