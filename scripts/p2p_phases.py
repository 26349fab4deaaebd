"""Diagnostic: in-kernel phase times of the p2p window pipeline (lib/libnsgpu_prof.so, NSGPU_LIB)."""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("NSGPU_LIB", os.path.join(REPO, "ns-3-dev-dnemu_amd", "lib", "libnsgpu_prof.so"))
sys.path[:0] = [os.path.join(REPO, "ns-3-dev-dnemu_amd")]
import numpy as np  # noqa: E402
import nsgpu  # noqa: E402
import p2p  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 128
eng = p2p.Engine(p2p.grid(n, n))
eng.run()
buf = np.zeros(64, np.uint64)
nsgpu.check(nsgpu.lib().nsgpu_p2p_phase_read(buf.ctypes.data, 64, 1))
st, _, _, _ = eng.run()
ms = C.c_double()
nsgpu.check(nsgpu.lib().nsgpu_p2p_last_run_ms(eng.h, C.byref(ms)))
nsgpu.check(nsgpu.lib().nsgpu_p2p_phase_read(buf.ctypes.data, 64, 1))
w = max(int(st.windows), 1)
print(f"grid {n}: {st.dispatched} events, {w} windows, {ms.value:.1f} ms ({1e3 * ms.value / w:.2f} us/window)")
names = {0: "k_pa: entry->ctl", 1: "k_pa: sweep", 2: "k_pa: publish_min+digest",
         8: "handle_rank: entry->ctl", 9: "handle_rank: body (block 0)",
         12: "handle: holder+node_cnt (lane max)", 13: "handle: gather+sort (lane max)",
         14: "handle: event loop (lane max)",
         16: "scan: entry->W", 17: "scan: slot loads+lds", 18: "scan: scan", 19: "scan: sinfo stores",
         20: "scan: bookkeeping", 24: "append: entry->ctl", 25: "append: body", 26: "append: publish"}
for i, nm in names.items():
    print(f"  {nm:32s} {buf[i] * 10.0 / w / 1e3:8.3f} us/window")
print(f"  holders in block 0: {buf[15] / w:.1f} per window")
print(f"  max handle thread {buf[10] * 10.0 / 1e3:.2f} us, max rank thread {buf[11] * 10.0 / 1e3:.2f} us")
