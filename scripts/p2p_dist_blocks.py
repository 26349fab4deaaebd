"""Diagnostic: per-block start / end times of the partitioned engine's k2_pa<DIST> and k2_handle in one
sampled window (lib/libnsgpu_prof.so), one loopback rank on the 128x128 grid: which roles finish last."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("NSGPU_LIB", os.path.join(REPO, "ns-3-dev-dnemu_amd", "lib", "libnsgpu_prof.so"))
sys.path[:0] = [os.path.join(REPO, "ns-3-dev-dnemu_amd")]
import numpy as np  # noqa: E402
import nsgpu  # noqa: E402
import p2p  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 128
grp = p2p.LoopbackGroup(p2p.grid(n, n), 1)
BLK = 2048
buf = np.zeros(64 + 3 * BLK * 2, np.uint64)
nsgpu.check(nsgpu.lib().nsgpu_p2p_phase_read(buf.ctypes.data, 64, 1))
grp.run()
nsgpu.check(nsgpu.lib().nsgpu_p2p_phase_read(buf.ctypes.data, buf.size, 0))
blk = buf[64:].reshape(3, BLK, 2).astype(np.int64)
wide = grp.members[0].wide()
nslot = (4096 + 4096) // 256 if wide else 16  # (wide: gen-0 slots, then the local records' dense list)
roles = {0: [("slot", 0, 16), ("lslot", 16, nslot), ("remote", nslot, nslot + 1), ("pool", nslot + 1, 256)],
         1: [("holder", 0, 64), ("hub", 64, 96), ("maint", 96, 224)],
         2: [("book", 0, 1), ("stack", 1, 2), ("gen0", 2, 66), ("local", 66, 130)]}
for k, name in ((0, "k2_pa<DIST>"), (1, "k2_handle"), (2, "k_dfin2")):
    b = blk[k]
    ok = b[:, 1] > 0
    if not ok.any():
        print(f"{name}: no blocks recorded")
        continue
    t0 = b[ok, 0].min()
    print(f"{name}: blocks {ok.sum()}, span {(b[ok, 1].max() - t0) * 0.01:.2f} us (s_memrealtime, 10 ns)")
    for rn, lo, hi in roles[k]:
        r = b[lo:hi][ok[lo:hi]]
        if len(r) == 0:
            continue
        st, en = (r[:, 0] - t0) * 0.01, (r[:, 1] - t0) * 0.01
        print(f"  {rn:7s} n={len(r):5d} start {st.min():6.2f}..{st.max():6.2f}  end p50 {np.median(en):6.2f} "
              f"max {en.max():6.2f}  dur p50 {np.median(en - st):6.2f} max {(en - st).max():6.2f} us")
    slow = np.argsort(-(b[:, 1] - t0) * ok)[:12]
    print("  slowest: " + " ".join(f"{i}:{(b[i, 0] - t0) * 0.01:.1f}-{(b[i, 1] - t0) * 0.01:.1f}" for i in slow))
ph = buf[:64]
marks = {32: "snapshot issued", 34: "bound/publish (waits snapshot)", 36: "digest/log/classify (waits slot data)",
         38: "block_alloc2 (atomics+barriers)", 40: "writes (node-table atomics)", 42: "loop exit", 44: "publish_min+digest"}
print("k2_pa slot blocks, mean per block (sampled window):")
for i, nm in marks.items():
    c = max(int(ph[i + 1]), 1)
    print(f"  {nm:40s} {ph[i] * 0.01 / c:6.2f} us  (n={int(ph[i + 1])})")
print(f"k2_pa inputs (sampled window): pool end {int(buf[46])}, last window gen-0 {int(buf[47])}, local {int(buf[48])}; "
      f"pool entries taken {int(buf[49])}, pool chunks swept {int(buf[50])}")
print("k2_pa pool blocks, mean per block (sampled window):")
for i, nm in ((52, "run control + barrier"), (54, "pool sweep"), (62, "publish_min + digest")):
    c = max(int(buf[i + 1]), 1)
    print(f"  {nm:40s} {buf[i] * 0.01 / c:6.2f} us  (n={int(buf[i + 1])})")
