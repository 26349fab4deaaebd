"""Diagnostic (not product): config 4's run with the window pipeline replayed from its hipGraph (the
default; NSGPU_P2P_EAGER unset) under rocprofv3 --kernel-trace, with scripts/segv_dump.so's SIGSEGV
handler installed after the profiler's, so that a crash prints library-relative frames.  Round 2 saw a
SIGSEGV here (gpurun_out/measure/rocprof_p2p.log) and switched profiling to eager launches.
usage: rocprofv3 --kernel-trace --stats -d <dir> -- python3 scripts/rocprof_graph_probe.py [runs]"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "ns-3-dev-dnemu_amd")]
seg = ctypes.CDLL(os.path.join(REPO, "scripts", "segv_dump.so"))
seg.segv_dump_install()
import nsgpu  # noqa: E402
import p2p  # noqa: E402

nsgpu.check(nsgpu.lib().nsgpu_set_device(0))
runs = int(sys.argv[1]) if len(sys.argv) > 1 else 2
eng = p2p.Engine(p2p.grid(128, 128))
for r in range(runs):
    st, _, _, _ = eng.run()
    print(f"run {r}: {st.dispatched} events, {st.windows} windows, digest {st.digest}", flush=True)
print("graph replay under the tracer: no fault", flush=True)
