"""Diagnostic: per-kernel window times of config 4's wide engine for a library given by NSGPU_LIB."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "ns-3-dev-dnemu_amd")]
import nsgpu  # noqa: E402
import p2p  # noqa: E402

nsgpu.check(nsgpu.lib().nsgpu_set_device(0))
eng = p2p.Engine(p2p.grid(128, 128))
st, _, _, _ = eng.run()
prof = eng.profile(sample_every=4)
print(os.environ.get("NSGPU_LIB", "default"), st.windows, {k: round(v[0] * 1e3, 2) for k, v in prof.items()})
