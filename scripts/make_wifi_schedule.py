"""Writes tests/golden/wifi_grid100_schedule.csv: the committed transmission schedule of the 100x100
Wi-Fi grid parity test (tests/test_gpu_wifi.py).  300 broadcast frames of 1064 B (a 1000-B UDP datagram)
at DSSS 1 Mbps from random phys of the 10,000, at random ns instants in [0, 60 ms) — about 43 frames
on the air at once, so receivers see syncs, drops in RX and TX, and CCA-busy extensions.  No phy starts
a frame while its previous one is still on the air.  Rows are (ts_ns, phy) in (ts, setup uid) order."""
import os

import numpy as np

FRAME_US = 192 + 1064 * 8


def main():
    rng = np.random.default_rng(20261016)
    rows, on_air = [], {}
    while len(rows) < 300:
        s, t = int(rng.integers(0, 10000)), int(rng.integers(0, 60_000_000))
        if any(t <= e and t + FRAME_US * 1000 >= b for b, e in on_air.get(s, [])):
            continue
        on_air.setdefault(s, []).append((t, t + FRAME_US * 1000))
        rows.append((t, s))
    rows.sort()
    out = os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "wifi_grid100_schedule.csv")
    with open(out, "w") as f:
        f.write("ts_ns,phy\n")
        for t, s in rows:
            f.write(f"{t},{s}\n")


if __name__ == "__main__":
    main()
