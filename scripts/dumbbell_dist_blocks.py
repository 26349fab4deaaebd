"""Diagnostic: per-block spans of the partitioned engine's k2_pa / k2_handle at sampled windows of config 5
(one loopback partition, eager launches, lib/libnsgpu_prof.so), printing the windows whose k2_handle span
exceeds a threshold with each role's median / latest block end (us).
Usage: python scripts/dumbbell_dist_blocks.py [step] [first] [last] [threshold_us]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("NSGPU_LIB", os.path.join(REPO, "ns-3-dev-dnemu_amd", "lib", "libnsgpu_prof.so"))
os.environ.setdefault("NSGPU_P2P_EAGER", "1")
sys.path[:0] = [os.path.join(REPO, "ns-3-dev-dnemu_amd")]
import numpy as np  # noqa: E402
import nsgpu  # noqa: E402
import p2p  # noqa: E402

step = int(sys.argv[1]) if len(sys.argv) > 1 else 20
first = int(sys.argv[2]) if len(sys.argv) > 2 else 1
last = int(sys.argv[3]) if len(sys.argv) > 3 else 1 << 30
thr = float(sys.argv[4]) if len(sys.argv) > 4 else 200.0
nsgpu.check(nsgpu.lib().nsgpu_set_device(0))
sc = p2p.dumbbell(499_999)
grp = p2p.LoopbackGroup(sc, 1)
st, _, _, _ = grp.run()
W = int(st.windows)
print(f"dumbbell partitioned x1: {st.dispatched} events, {W} windows", flush=True)
BLK = 2048
buf = np.zeros(64 + 3 * BLK * 2, np.uint64)
roles = {1: [("holder", 0, 64), ("hub", 64, 96), ("maint", 96, 224)]}
for w in range(first, min(W, last), step):
    nsgpu.check(nsgpu.lib().nsgpu_p2p_phase_read(buf.ctypes.data, 64, -w))
    grp.run()
    nsgpu.check(nsgpu.lib().nsgpu_p2p_phase_read(buf.ctypes.data, buf.size, 0))
    blk = buf[64:].reshape(3, BLK, 2).astype(np.int64)
    b = blk[1]
    ok = b[:, 1] > 0
    if not ok.any():
        continue
    t0 = b[ok, 0].min()
    span = (b[ok, 1].max() - t0) * 0.01
    if span < thr:
        continue
    rs = []
    for rn, lo, hi in roles[1]:
        r = b[lo:hi][ok[lo:hi]]
        if len(r):
            en = (r[:, 1] - t0) * 0.01
            rs.append(f"{rn} {np.median(en):.1f}/{en.max():.1f} (block {lo + int(np.argmax(en))})")
    print(f"w {w:5d}: gen0 {int(buf[47]):5d} words {[int(x) for x in buf[32:48]]} | k2_handle {span:.1f}: " + ", ".join(rs),
          flush=True)
