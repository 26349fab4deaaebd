"""Diagnostic: where k2_rank's time goes in window 1000 of config 4's wide engine (lib/libnsgpu_prof.so):
per-block phase means (s_memrealtime, 10 ns) and the sampled window's sizes and tie counts."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("NSGPU_LIB", os.path.join(REPO, "ns-3-dev-dnemu_amd", "lib", "libnsgpu_prof.so"))
sys.path[:0] = [os.path.join(REPO, "ns-3-dev-dnemu_amd")]
import numpy as np  # noqa: E402
import nsgpu  # noqa: E402
import p2p  # noqa: E402

nsgpu.check(nsgpu.lib().nsgpu_set_device(0))
eng = p2p.Engine(p2p.grid(128, 128))
eng.run()
buf = np.zeros(64, np.uint64)
nsgpu.check(nsgpu.lib().nsgpu_p2p_phase_read(buf.ctypes.data, 64, 1))
st, _, _, _ = eng.run()
nsgpu.check(nsgpu.lib().nsgpu_p2p_phase_read(buf.ctypes.data, 64, 1))
print(f"windows {st.windows}; sampled window: N {buf[57]} Lt {buf[58]} tiles {buf[59]} ties(word2) {buf[56]} "
      f"max depth {buf[60]}")
for i, nm in ((48, "entry -> local_prefix"), (50, "tile loads"), (52, "compare loop"), (54, "atomic + sync")):
    n = max(int(buf[i + 1]), 1)
    print(f"  {nm:24s} {buf[i] * 10.0 / n / 1e3:8.3f} us per block-mark (n={int(buf[i + 1])})")
prof = eng.profile(sample_every=4)
print({k: round(v[0] * 1e3, 2) for k, v in prof.items()})
