"""Diagnostic: the closed-loop Wi-Fi PHY (nsgpu_wifil behind nsgpu_sim) at config-3 scale — n_side^2 phys,
the MAC stand-in of tests/wifi_loop_harness.py (send when IDLE, else back off), broadcast period and Stop
from argv — timed on the GPU, optionally against the oracle (argv[4] = 1)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "ns-3-dev-dnemu_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402
import nsgpu  # noqa: E402
import wifi  # noqa: E402
from wifi_loop_harness import run_gpu, run_oracle, scenario  # noqa: E402

nsgpu.check(nsgpu.lib().nsgpu_set_device(0))
n_side = int(sys.argv[1]) if len(sys.argv) > 1 else 100
period = int(float(sys.argv[2]) * 1e9) if len(sys.argv) > 2 else 1_000_000_000
stop = int(float(sys.argv[3]) * 1e9) if len(sys.argv) > 3 else 200_000_000
with_oracle = len(sys.argv) > 4 and sys.argv[4] == "1"
sc = scenario(n_side=n_side, spacing=100.0, seed=11, period=period, stop_ns=stop, size=1000, tx_cap=1 << 20,
              rxq_cap=1024, ni_cap=1024)
t0 = time.perf_counter()
glog, gends, gphys, gtot, keep = run_gpu(sc, log_cap=1 << 22)
t1 = time.perf_counter()
print(f"gpu: {n_side}x{n_side} phys, period {period} ns, stop {stop} ns: dispatched {gtot['dispatched']} "
      f"sends {gtot['sends']} busy {gtot['busy']} ends {len(gends)} in {t1 - t0:.2f} s "
      f"({gtot['dispatched'] / (t1 - t0) / 1e6:.1f} M ev/s)", flush=True)
if with_oracle:
    t2 = time.perf_counter()
    olog, oends, ophys, otot = run_oracle(sc, log_cap=1 << 22)
    t3 = time.perf_counter()
    same = all(gtot[f] == otot[f] for f in ("dispatched", "digest", "next_uid", "final_ts", "sends", "busy"))
    print(f"oracle: {otot['dispatched']} in {t3 - t2:.2f} s ({otot['dispatched'] / (t3 - t2) / 1e6:.1f} M ev/s); "
          f"totals match: {same}", flush=True)
