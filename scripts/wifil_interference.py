"""Diagnostic: the closed-loop Wi-Fi line measured 75 us an epoch alone and 111 us as the
p2p-grid bench's secondary.  This runs the wifi-loop workload (bench.WifiLoop) in one process after each of the
steps the bench takes before it and prints its us per epoch, so the step that slows it shows up.
Usage (GPU box): python scripts/wifil_interference.py [stages...]"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "ns-3-dev-dnemu_amd"))

import bench  # noqa: E402
import nsgpu  # noqa: E402


def args_ns():
    return argparse.Namespace(grid=128, holds=5_000_000, dumbbell_leaves=499_999, fanout_tx=1024, wifi_side=100,
                              wifi_stop=2.0, wifi_loop_stop=0.2, wifi_mac="native")


def loop(tag, args, stream, reps=3):
    wl = bench.WifiLoop(args, stream.handle)
    wl.step()
    us = []
    for _ in range(reps):
        t0 = time.perf_counter()
        wl.step()
        us.append(round(wl.result()[2]["us_per_epoch"], 1))
    wl.close()
    print(f"{tag:40s} us/epoch {us}", flush=True)


def main():
    nsgpu.check(nsgpu.lib().nsgpu_set_device(0))
    args = args_ns()
    stream = nsgpu.Stream()
    stages = sys.argv[1:] or ["fresh", "p2p", "profile", "close_p2p", "wifi_grid", "dumbbell"]
    if stages[0] == "nofresh":  # (the first loop only after the next stage: stream creation order as in bench.py)
        stages = stages[1:]
    g = None
    for st in stages:
        if st == "fresh":
            pass
        elif st == "p2p":
            g = bench.P2PGrid(args, stream.handle)
            g.step()
            stream.sync()
        elif st == "p2p_norun":  # created, never run
            g = bench.P2PGrid(args, stream.handle)
        elif st == "p2p6":  # the bench primary's warmup + 5 timed steps
            g = bench.P2PGrid(args, stream.handle)
            for _ in range(6):
                g.step()
            stream.sync()
        elif st == "profile":
            g.roofline(50.0, 7_599_361)
        elif st == "close_p2p":
            g.close()
            g = None
        elif st == "wifi_grid":
            w = bench.WifiGrid(args, stream.handle)
            w.step()
            stream.sync()
            w.close()
        elif st == "wifi_grid_open":
            w = bench.WifiGrid(args, stream.handle)
            w.step()
            stream.sync()
        elif st == "dumbbell":
            d = bench.P2PDumbbell(args, stream.handle)
            d.step()
            stream.sync()
            d.close()
        elif st == "cpu_p2p":  # the p2p-grid line's CPU baseline (the oracle's full run, one host core)
            g = g or bench.P2PGrid(args, stream.handle)
            g.cpu_baseline()
        elif st == "cpu_wifi":  # the wifi-grid secondary's CPU baseline (oracle sample + a GPU sample engine)
            w = bench.WifiGrid(args, stream.handle)
            w.step()
            stream.sync()
            w.cpu_baseline()
            w.close()
        elif st == "cpu_oracle_wifi":  # only its oracle part
            import wifi
            import numpy as np
            nsref = bench.oracle()
            sc = wifi.wifi_grid(n_side=100, stop_s=0.1)
            stt = wifi.WifiStats()
            nsref.wifi_run(sc.c_struct(), stt, np.zeros(sc.n_phy, wifi.PHY_COUNTERS_DTYPE),
                           np.zeros(len(sc.tx), np.uint32), wifi.END_RECORD_DTYPE)
        elif st == "probe":
            print("probe", nsgpu.probe_latency(), flush=True)
        loop(f"after {st}", args, stream)


if __name__ == "__main__":
    main()
