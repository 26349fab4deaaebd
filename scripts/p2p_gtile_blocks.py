"""Diagnostic: k_gtile's per-block stamps in one sampled window of the partitioned 128x128 grid on one loopback
rank (lib/libnsgpu_prof.so): dispatch ramp, prologue trip, column-tile trip, compares, atomics."""
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
BLK, GTB = 2048, 8192
buf = np.zeros(64 + 3 * BLK * 2 + GTB * 8, np.uint64)
nsgpu.check(nsgpu.lib().nsgpu_p2p_phase_read(buf.ctypes.data, 64, 1))
grp.run()
nsgpu.check(nsgpu.lib().nsgpu_p2p_phase_read(buf.ctypes.data, buf.size, 0))
g = buf[64 + 3 * BLK * 2:].reshape(GTB, 8).astype(np.int64)
ok = g[:, 4] > 0
print(f"k_gtile blocks recorded {ok.sum()}")
g = g[ok]
t0 = g[:, 0].min()
us = lambda x: (x - t0) * 0.01  # noqa: E731
st, en = us(g[:, 0]), us(g[:, 4])
print(f"span {en.max():.2f} us; start p10/p50/p90/max {np.percentile(st, 10):.2f} {np.median(st):.2f} "
      f"{np.percentile(st, 90):.2f} {st.max():.2f}; end p50/p90/max {np.median(en):.2f} {np.percentile(en, 90):.2f} {en.max():.2f}")
work = g[:, 2] > 0
for nm, a, b in (("prologue (hdr trip)", 0, 1), ("tile loads + barrier", 1, 2), ("compares", 2, 3), ("atomics (returned)", 3, 4)):
    m = work if a >= 1 else np.ones(len(g), bool)
    d = (g[m, b] - g[m, a]) * 0.01
    d = d[(g[m, a] > 0) & (g[m, b] > 0)]
    if len(d):
        print(f"  {nm:24s} n={len(d):5d} p50 {np.median(d):6.2f} p90 {np.percentile(d, 90):6.2f} max {d.max():6.2f} us")
kind = g[:, 6]
for nm, k in (("gen x gen", 0), ("gen row x local col", 1), ("local row x gen col", 2), ("local x local", 3)):
    m = work & ((kind & 3) == k)
    if not m.any():
        continue
    ti = ((kind & 4) > 0) & m
    dl, dc = (g[m, 2] - g[m, 1]) * 0.01, (g[m, 3] - g[m, 2]) * 0.01
    print(f"  {nm:20s} n={m.sum():5d} (ties {ti.sum():4d}) loads p50 {np.median(dl):5.2f} max {dl.max():5.2f}  "
          f"compares p50 {np.median(dc):5.2f} p90 {np.percentile(dc, 90):5.2f} max {dc.max():5.2f}  end max {en[m].max():6.2f}")
    if ti.any():
        dt = (g[ti, 3] - g[ti, 2]) * 0.01
        print(f"      with ties: compares p50 {np.median(dt):5.2f} max {dt.max():5.2f}")
idle = ~work
print(f"  idle blocks {idle.sum()}: dur p50 {np.median(en[idle] - st[idle]) if idle.any() else 0:.2f} us, "
      f"start p50 {np.median(st[idle]) if idle.any() else 0:.2f}")
for x in range(8):
    m = g[:, 5] == x
    if m.any():
        print(f"  xcc {x}: blocks {m.sum():5d} start max {st[m].max():6.2f} end max {en[m].max():6.2f}")
# a timeline: blocks started / finished per 1-us bucket
h0, _ = np.histogram(st, bins=np.arange(0, en.max() + 1))
h1, _ = np.histogram(en, bins=np.arange(0, en.max() + 1))
print("  started per us:  " + " ".join(str(int(x)) for x in h0))
print("  finished per us: " + " ".join(str(int(x)) for x in h1))
