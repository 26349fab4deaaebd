"""bench.py — simulated events/s of the nsgpu engine on MI355X (driver contract: one JSON line).

Workload (round 1): SURVEY §8(d) config 1, utils/bench-simulator.cc churn — 10,000 pending
events, delays U[0,1) s (tests/golden/bench_dist_u01_10k.txt), 5e6 holds, MapScheduler pop
order, run entirely on the device (nsgpu_hold_run).  One step = one full bench-simulator run
(10,000 inserts + 5,010,001 dispatches); inputs are resident in HBM before the timed region.

The churn is one logical process (all events have context 0xffffffff), so it does not shard:
with --gpus N every rank runs an independent replica ("replicas only") and `value`
is the events of all ranks divided by the slowest rank's time.

roofline: the dominant kernel is hold_run; algorithmic bytes = 72 B per dispatched event
(24 B insert + 24 B window read + 24 B dispatch write) x events per launch,
divided by the kernel's average duration measured with HIP events on its stream.
cpu_baseline: the oracle's restatement of DefaultSimulatorImpl + MapScheduler + Bench::Cb
("port"), on one host core, same distribution and hold count.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "ns-3-dev-dnemu_amd"))

METRIC = "simulated events/sec (whole node) at 1/2/4/8 GPUs; speedup vs ns-3 CPU"
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
BYTES_PER_EVENT = 72    # SURVEY §8(d) event-queue algorithmic bytes
DIST_FILE = os.path.join(REPO, "tests", "golden", "bench_dist_u01_10k.txt")
TOTAL_HOLDS = 5_000_000


def load_distribution(path):
    """bench-simulator ReadDistribution (bench-simulator.cc:59-76): (uint64_t)(seconds * 1e9)."""
    import numpy as np
    vals = []
    for tok in open(path).read().split():
        try:
            vals.append(float(tok))
        except ValueError:
            pass
    return (np.array(vals, dtype=np.float64) * 1000000000).astype(np.uint64)


def cpu_baseline(dist, total):
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import nsref
    runs = []
    for _ in range(3):
        res, _, _ = nsref.churn_run(dist, total, nsref.SCHED_MAP)
        runs.append(res)
    best = min(runs, key=lambda r: r.run_seconds)
    return {
        "value": best.dispatched / best.run_seconds,
        "unit": "events/s",
        "cores": 1,
        "kind": "port",
        "sample": f"full config-1 run ({len(dist)} pending, {total} holds, {best.dispatched} dispatches), "
                  "oracle restatement of DefaultSimulatorImpl+MapScheduler+Bench::Cb, g++ -O2, best of 3, "
                  f"Simulator::Run only ({best.run_seconds:.3f} s)",
        "digest_match": None,
        "_digest": best.digest,
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--holds", type=int, default=TOTAL_HOLDS)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist_pg = None
    if world > 1:
        import torch
        import torch.distributed as tdist
        torch.cuda.set_device(local_rank)
        tdist.init_process_group("nccl")
        dist_pg = tdist

    import numpy as np
    import nsgpu

    nsgpu.check(nsgpu.lib().nsgpu_set_device(local_rank))
    dist = load_distribution(DIST_FILE)
    stream = nsgpu.Stream()
    run = nsgpu.HoldRun(dist, args.holds, stream=stream.handle)
    timer = nsgpu.Timer()

    for _ in range(args.warmup):
        run.launch()
    stream.sync()

    def barrier():
        if dist_pg is not None:
            import torch
            torch.cuda.synchronize()
            dist_pg.barrier()
            torch.cuda.synchronize()

    barrier()
    stream.sync()
    t0 = time.perf_counter()
    timer.start(stream.handle)
    for _ in range(args.steps):
        run.launch()
    timer.stop(stream.handle)
    stream.sync()
    barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms_total = timer.elapsed_ms()
    st, _, _ = run.result()

    if dist_pg is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local_rank}")
        dist_pg.all_reduce(t, op=dist_pg.ReduceOp.MAX)
        elapsed = float(t.item())

    events_per_step = int(st.dispatched)
    value = events_per_step * args.steps * world / elapsed
    kernel_ms = kernel_ms_total / args.steps  # one hold_run launch per step (+ a tiny init-rank kernel)
    achieved = BYTES_PER_EVENT * events_per_step / (kernel_ms / 1e3) / 1e9

    traffic = None
    tpath = os.path.join(REPO, "profiles", "traffic_hold_run.json")
    if os.path.exists(tpath):
        try:
            traffic = json.load(open(tpath)).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "events/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic",
            "config": {
                "workload": f"bench-simulator churn (config 1): {len(dist)} pending, U[0,1) s delays, "
                            f"{args.holds} holds, MapScheduler (ts,uid) order, GPU-resident Bench::Cb",
                "events_per_step": events_per_step,
                "parallelism": "replicas" if world > 1 else "single",
                "rounds_per_step": int(st.rounds),
                "max_batch": int(st.max_batch),
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBPS,
                "traffic": traffic,
                "kernel": "nsgpu::hold_run",
                "kernel_ms": kernel_ms,
                "bytes_per_event": BYTES_PER_EVENT,
            },
        }
        if not args.no_cpu_baseline:
            cb = cpu_baseline(dist, args.holds)
            cb["digest_match"] = bool(cb.pop("_digest") == st.digest)
            out["cpu_baseline"] = cb
            out["speedup_vs_cpu"] = value / world / cb["value"]
        print(json.dumps(out), flush=True)

    if dist_pg is not None:
        dist_pg.destroy_process_group()


if __name__ == "__main__":
    main()
