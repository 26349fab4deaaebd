"""Diagnostic: how many exact chain compares (two order words tied between distinct records) k2_rank made
over a whole run of tests/test_gpu_wide.py's lockstep scenario (lib/libnsgpu_prof.so)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("NSGPU_LIB", os.path.join(REPO, "ns-3-dev-dnemu_amd", "lib", "libnsgpu_prof.so"))
sys.path[:0] = [os.path.join(REPO, "ns-3-dev-dnemu_amd")]
import numpy as np  # noqa: E402
import nsgpu  # noqa: E402
import p2p  # noqa: E402

nsgpu.check(nsgpu.lib().nsgpu_set_device(0))
cols = 8
sc = p2p.grid(2, cols, flows=[(0, cols - 1), (cols, 2 * cols - 1)], rate_bps=20_000_000, qmax=100,
              stop_ns=160_000_000, sim_stop_ns=180_000_000)
eng = p2p.Engine(sc)
buf = np.zeros(64, np.uint64)
nsgpu.check(nsgpu.lib().nsgpu_p2p_phase_read(buf.ctypes.data, 64, 1))
st, _, _, _ = eng.run()
nsgpu.check(nsgpu.lib().nsgpu_p2p_phase_read(buf.ctypes.data, 64, 1))
print(f"wide {eng.wide()} windows {st.windows} dispatched {st.dispatched}: exact chain compares {buf[61]}")
