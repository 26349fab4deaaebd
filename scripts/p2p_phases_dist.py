"""Diagnostic: k_pa in-kernel phase times (block 0), single-GPU engine vs partitioned engine on one
rank (RCCL, one member), lib/libnsgpu_prof.so."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("NSGPU_LIB", os.path.join(REPO, "ns-3-dev-dnemu_amd", "lib", "libnsgpu_prof.so"))
sys.path[:0] = [os.path.join(REPO, "ns-3-dev-dnemu_amd")]
import numpy as np  # noqa: E402
import nsgpu  # noqa: E402
import p2p  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 128
sc = p2p.grid(n, n)
buf = np.zeros(64, np.uint64)
comm = p2p.Comm(p2p.Comm.unique_id(), 1, 0)
for name, eng in [("single", p2p.Engine(sc)),
                  ("partitioned x1", p2p.DistEngine(sc, np.zeros(sc.n_nodes, np.uint32), 0, 1, comm))]:
    eng.run()
    nsgpu.check(nsgpu.lib().nsgpu_p2p_phase_read(buf.ctypes.data, 64, 1))
    st, _, _, _ = eng.run()
    nsgpu.check(nsgpu.lib().nsgpu_p2p_phase_read(buf.ctypes.data, 64, 1))
    w = max(int(st.windows), 1)
    print(f"{name}: {st.dispatched} events, {w} windows")
    for i, nm in {0: "k_pa: entry->slot loads", 1: "k_pa: sweep", 2: "k_pa: publish_min+digest",
                  8: "handle_rank: entry->ctl", 9: "handle_rank: body (block 0)"}.items():
        print(f"  {nm:32s} {buf[i] * 10.0 / w / 1e3:8.3f} us/window")
