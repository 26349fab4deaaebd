"""Diagnostic: per-block spans of the window kernels at sampled windows across one scenario's run
(lib/libnsgpu_prof.so).  Usage: python scripts/p2p_blocks_sweep.py dumbbell|grid [step] [n] [first] [count]
Each sample re-runs the engine with the per-block stamps aimed at window w (nsgpu_p2p_phase_read(-w)) and
prints, per kernel, the span and each role's median / latest block end (us), with the window's size from the phase words."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("NSGPU_LIB", os.path.join(REPO, "ns-3-dev-dnemu_amd", "lib", "libnsgpu_prof.so"))
sys.path[:0] = [os.path.join(REPO, "ns-3-dev-dnemu_amd")]
import numpy as np  # noqa: E402
import nsgpu  # noqa: E402
import p2p  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "dumbbell"
step = int(sys.argv[2]) if len(sys.argv) > 2 else 50
sc = p2p.dumbbell(int(sys.argv[3]) if len(sys.argv) > 3 else 499_999) if kind == "dumbbell" else \
    p2p.grid(int(sys.argv[3]) if len(sys.argv) > 3 else 128, int(sys.argv[3]) if len(sys.argv) > 3 else 128)
nsgpu.check(nsgpu.lib().nsgpu_set_device(0))
eng = p2p.Engine(sc)
eng.set_eager(True)
st, _, _, _ = eng.run()
W = int(st.windows)
print(f"{kind}: {st.dispatched} events, {W} windows; sampling every {step}", flush=True)
BLK = 2048
buf = np.zeros(64 + 3 * BLK * 2, np.uint64)
wide = eng.wide()
nslot = (4096 + 4096) // 256 if wide else 16
roles = {0: [("slot", 0, nslot), ("pool", nslot, 256)],
         1: [("holder", 0, 64), ("hub", 64, 96), ("maint", 96, 224), ("rank", 224, 1248)],
         2: [("book", 0, 1), ("sdef", 1, 5), ("tiles", 5, 256)] if wide else [("scan", 0, 1)]}
names = ("k2_pa", "k2_handle", "k2_rank" if wide else "k2_scan")
first = int(sys.argv[4]) if len(sys.argv) > 4 else 1
count = int(sys.argv[5]) if len(sys.argv) > 5 else W
for w in list(range(first, W, step))[:count]:
    nsgpu.check(nsgpu.lib().nsgpu_p2p_phase_read(buf.ctypes.data, 64, -w))
    eng.run()
    nsgpu.check(nsgpu.lib().nsgpu_p2p_phase_read(buf.ctypes.data, buf.size, 0))
    blk = buf[64:].reshape(3, BLK, 2).astype(np.int64)
    parts = []
    for k, name in enumerate(names):
        b = blk[k]
        ok = b[:, 1] > 0
        if not ok.any():
            parts.append(f"{name} -")
            continue
        t0 = b[ok, 0].min()
        rs = []
        for rn, lo, hi in roles[k]:
            r = b[lo:hi][ok[lo:hi]]
            if len(r):
                en = (r[:, 1] - t0) * 0.01
                rs.append(f"{rn} {np.median(en):.1f}/{en.max():.1f}")
        parts.append(f"{name} {(b[ok, 1].max() - t0) * 0.01:.1f} ({', '.join(rs)})")
    print(f"w {w:5d}: pool end {int(buf[46]):8d} gen0 {int(buf[47]):5d} | " + " | ".join(parts), flush=True)
