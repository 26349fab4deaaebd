"""Diagnostic: per-window-phase cycle split of the p2p engine kernel (s_memtime, wave 0 view)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "ns-3-dev-dnemu_amd")]
import numpy as np  # noqa: E402
import nsgpu  # noqa: E402
import p2p  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 128
eng = p2p.Engine(p2p.grid(n, n))
prof = nsgpu.DeviceBuffer(16 * 8)
prof.zero()
nsgpu.check(nsgpu.lib().nsgpu_p2p_set_profile(eng.h, prof.ptr))
st, _, _, _ = eng.run()
cyc = prof.download(np.uint64, 16)
names = {0: "1 reduce", 1: "2 count/bisect", 2: "3 partition", 7: "4a histogram", 8: "4b sort", 3: "4c group",
         4: "5 handlers", 6: "6 uids/append"}
order = [0, 1, 2, 7, 8, 3, 4, 6]
tot = sum(cyc[i] for i in order)
print(f"grid {n}: windows {st.windows} events {st.dispatched} cycles/window {tot / st.windows:.0f}")
for i in order:
    print(f"  {names[i]:16s} {cyc[i] / st.windows:10.0f} cyc/window  {100 * cyc[i] / tot:5.1f}%")
print(f"  bitonic fallback windows: {cyc[9]}")
