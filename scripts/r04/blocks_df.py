"""Diagnostic: per-block start / end times of k2_pa, k2_handle and k2_rank<true> in one sampled window of the
deferred pipeline (lib/libnsgpu_prof.so, NSGPU_LIB), k2_pa's slot-block phase marks and the deferred
accounting's phases (s_memrealtime, 10 ns)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("NSGPU_LIB", os.path.join(REPO, "ns-3-dev-dnemu_amd", "lib", "libnsgpu_prof.so"))
sys.path[:0] = [os.path.join(REPO, "ns-3-dev-dnemu_amd")]
import numpy as np  # noqa: E402
import nsgpu  # noqa: E402
import p2p  # noqa: E402

eng = p2p.Engine(p2p.grid(128, 128))
eng.set_eager(True)
BLK = 2048
SDEF = {22: "records arrived", 24: "block scan", 26: "LDS arrays + prefixes + barrier", 28: "resolve/log/digest",
        30: "clears"}
for rep in range(2):
    buf = np.zeros(64 + 3 * BLK * 2, np.uint64)
    nsgpu.check(nsgpu.lib().nsgpu_p2p_phase_read(buf.ctypes.data, buf.size, 1))
    eng.run()
    nsgpu.check(nsgpu.lib().nsgpu_p2p_phase_read(buf.ctypes.data, buf.size, 1))
    blk = buf[64:].reshape(3, BLK, 2).astype(np.int64)
    print(f"rep {rep}")
    for k, name in enumerate(("k2_pa", "k2_handle", "k2_rank")):
        b = blk[k]
        ok = np.nonzero(b[:, 1] > 0)[0]
        if len(ok) == 0:
            continue
        t0 = b[ok, 0].min()
        print(f"{name}: blocks {len(ok)} (max index {ok.max()}), span {(b[ok, 1].max() - t0) * 0.01:.2f} us")
        for lo in range(0, ok.max() + 1, 64):
            sel = ok[(ok >= lo) & (ok < lo + 64)]
            if len(sel) == 0:
                continue
            st, en = (b[sel, 0] - t0) * 0.01, (b[sel, 1] - t0) * 0.01
            print(f"  blocks {lo:5d}+{len(sel):3d} start {st.min():6.2f}..{st.max():6.2f}  end p50 {np.median(en):6.2f}"
                  f" max {en.max():6.2f}  dur p50 {np.median(en - st):6.2f} max {(en - st).max():6.2f}")
        order = ok[np.argsort(-(b[ok, 1] - t0))][:12]
        print("  slowest:", " ".join(f"{i}:{(b[i, 0] - t0) * 0.01:.1f}-{(b[i, 1] - t0) * 0.01:.1f}" for i in order))
        if k == 0:
            print("  slot blocks:", " ".join(f"{i}:{(b[i, 1] - t0) * 0.01:.1f}" for i in range(32)))
        if k == 2:
            print("  book (0), accounting (1):", " ".join(f"{i}:{(b[i, 0] - t0) * 0.01:.1f}-{(b[i, 1] - t0) * 0.01:.1f}"
                                                      for i in (0, 1)))
    ph = buf[:64]
    print(f"  rank-tile ties (chain compares) over the run: {int(ph[61])}")
    for i in range(22, 64, 2):
        if ph[i + 1]:
            nm = SDEF.get(i, "")
            print(f"  mark {i:2d} {nm:32s}: {ph[i] * 0.01 / ph[i + 1]:7.2f} us mean (n={int(ph[i + 1])})")
