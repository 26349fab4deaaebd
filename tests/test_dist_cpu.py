"""Host side of a partitioned (multi-GPU) p2p run, on CPU (there is no GPU here): the node partition
(Node (systemId) blocks), the merge of per-rank results, and a world-size-2 gloo job driving them the
way bench.py --gpus N drives its ranks (bootstrap broadcast of the RCCL id, result exchange,
max-over-ranks timing).  The per-rank results are synthetic arrays in the shapes nsgpu_p2p_results
returns; the engines themselves are covered on the GPU by tests/test_gpu_p2p_dist.py."""
import os
import socket

import numpy as np
import pytest

import p2p


def test_owner_blocks_partition():
    for n, k in [(16, 1), (16, 2), (100, 3), (16384, 8), (7, 7)]:
        o = p2p.owner_blocks(n, k)
        assert o.dtype == np.uint32 and len(o) == n
        assert np.all(np.diff(o.astype(np.int64)) >= 0)  # contiguous id blocks
        assert set(o.tolist()) == set(range(k))
        counts = np.bincount(o, minlength=k)
        assert counts.max() - counts.min() <= 1  # balanced
    with pytest.raises(ValueError):
        p2p.owner_blocks(4, 0)


def test_weak_scaled_grid_row_bands():
    """grid(rows, cols * N) in N row bands (the bench layout): the bands are whole rows, the cut is
    the column links between bands, and every column flow crosses every band."""
    rows, cols, world = 8, 4 * 2, 2
    sc = p2p.grid(rows, cols)
    owner = p2p.owner_blocks(sc.n_nodes, world)
    ys = np.arange(sc.n_nodes) // cols
    assert np.array_equal(owner, (ys * world // rows).astype(np.uint32))
    dev = np.array(sc.dev)
    cut = owner[dev[:, 0]] != owner[dev[dev[:, 1], 0]]
    assert cut.sum() == 2 * cols  # one column link per column between the two bands, two devices each
    for a in sc.apps:
        if a["kind"] == p2p.APP_ONOFF:
            assert owner[a["node"]] == 0 and owner[a["dst"]] == world - 1


def _rank_results(sc, world, rank, total=40):
    s = sc.c_struct()
    st = p2p.stats_from_dict(dict(dispatched=total, cancelled=rank, digest=(1 << 63) + rank, final_ts=999,
                                  next_uid=77, windows=5, ttl_drops=rank, no_route_drops=0, max_window=9,
                                  unreach_drops=1, refits=rank))
    devc = np.zeros(s.n_devices, p2p.DEV_COUNTERS_DTYPE)
    devc["tx_packets"] = 100 + rank  # this rank's value everywhere; only its own rows are meaningful
    appc = np.zeros(s.n_apps, p2p.APP_COUNTERS_DTYPE)
    appc["rx_bytes"] = 1000 + rank
    k = np.arange(total)
    mine = k % world == rank  # this rank dispatched the global ranks k with k % world == rank
    ts = np.where(mine, 1000 + k, 0).astype(np.uint64)
    uid = np.where(mine, 4 + k, 0).astype(np.uint32)
    ctx = np.where(mine, k % 7, 0).astype(np.uint32)
    return st, devc, appc, (ts, uid, ctx)


def _check_merge(sc, world, per_rank):
    s = sc.c_struct()
    owner = p2p.owner_blocks(sc.n_nodes, world)
    st, devc, appc, (ts, uid, ctx) = p2p.merge_results(per_rank, owner, s)
    assert st.dispatched == 40 and st.next_uid == 77 and st.windows == 5  # run-global: rank 0's
    assert st.cancelled == sum(range(world)) and st.unreach_drops == world  # per-rank tallies: summed
    assert st.digest == ((world << 63) + sum(range(world))) & ((1 << 64) - 1)  # modulo 2^64
    assert np.array_equal(devc["tx_packets"], 100 + owner[s._keep["dev_node"]])
    assert np.array_equal(appc["rx_bytes"], 1000 + owner[s._keep["app_node"]])
    k = np.arange(40)
    assert np.array_equal(ts, 1000 + k) and np.array_equal(uid, 4 + k) and np.array_equal(ctx, k % 7)


def test_merge_results_single_process():
    sc = p2p.grid(4, 6)
    _check_merge(sc, 3, [_rank_results(sc, 3, r) for r in range(3)])


def _free_port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def _worker(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch
    import torch.distributed as td
    td.init_process_group("gloo")
    try:
        # bootstrap: rank 0's RCCL unique id reaches every rank (bench.py P2PGridDist)
        uid = [os.urandom(128) if rank == 0 else None]
        td.broadcast_object_list(uid, src=0)
        sc = p2p.grid(4, 4 * world)
        st, devc, appc, log = _rank_results(sc, world, rank)
        parts = [None] * world
        td.all_gather_object(parts, (uid[0], p2p.stats_to_dict(st), devc, appc, log))
        assert all(p[0] == uid[0] for p in parts)
        per_rank = [(p2p.stats_from_dict(d), dc, ac, lg) for _u, d, dc, ac, lg in parts]
        _check_merge(sc, world, per_rank)
        # the digest of the run is the sum of the ranks' shares (bench.py P2PGridDist.result)
        digests = [None] * world
        td.all_gather_object(digests, int(st.digest))
        assert sum(digests) & ((1 << 64) - 1) == ((world << 63) + sum(range(world))) & ((1 << 64) - 1)
        # max-over-ranks timing (bench.py)
        t = torch.tensor([float(rank + 1)], dtype=torch.float64)
        td.all_reduce(t, op=td.ReduceOp.MAX)
        assert t.item() == float(world)
        td.barrier()
    finally:
        td.destroy_process_group()


def test_gloo_world2_orchestration():
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(2, _free_port()), nprocs=2, join=True)


# ---------------------------------------------------------------- the ranks' engine plans, one process each
def _plan_worker(rank, world, port, workload, leaves, skew):
    """One rank of a partitioned run's bootstrap as bench.py does it (bench.dist_scenario + bench.check_plans, the
    RCCL id broadcast), minus the GPU calls: every rank builds its scenario and owner map itself and computes its
    engine plan (nsgpu_p2p_dist_plan, the host half of nsgpu_p2p_create_dist).  skew: rank 1 builds a different
    grid (a rank whose plan disagrees must make every rank fail before any collective)."""
    import sys
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if repo not in sys.path:
        sys.path.insert(0, repo)
    import torch.distributed as td
    import bench
    td.init_process_group("gloo")
    try:
        args = bench.parser().parse_args(["--workload", workload, "--dumbbell-leaves", str(leaves)])
        if skew and rank == 1:
            args.grid = 64
        sc, owner = bench.dist_scenario(args, workload, rank, world)
        try:
            plan = bench.check_plans(sc, owner, rank, world, td)
        except RuntimeError as e:
            assert skew and "plans differ" in str(e), e
            return
        assert not skew, "a skewed rank went unnoticed"
        uid = [os.urandom(128) if rank == 0 else None]  # (bench: rank 0's RCCL unique id to every rank)
        td.broadcast_object_list(uid, src=0)
        plans = [None] * world
        td.all_gather_object(plans, plan)
        assert p2p.plan_mismatch(plans) == {}
        # what the collectives carry: X0 16 B, X1 the fixed summary, X2 at least the largest cut between two
        # ranks (x3 for wide windows) per peer, at most CAPX_MAX records
        s = sc.c_struct()
        dn, dp = s._keep["dev_node"], s._keep["dev_peer"]
        po, qo = owner[dn], owner[dn[dp]]
        cut = np.zeros((world, world), np.int64)
        np.add.at(cut, (po[po != qo], qo[po != qo]), 1)
        need = int(cut.max()) * (3 if plan["wide"] else 1)
        assert plan["x0_bytes"] == 16 and plan["x1_bytes"] > 0
        assert plan["x2_records"] == min((need + 15) // 16 * 16, 1024)
        assert plan["x2_bytes"] == 16 + 40 * plan["x2_records"]  # (X2Hdr + 40-B event records)
        # every setup event is exactly one rank's (Simulator::Stop rank 0's), window 0's bound the whole setup's
        whole = p2p.dist_plan(sc, None, 0, 1)
        assert sum(p["n_init"] for p in plans) == whole["n_init"]
        for f in ("red0_tmin", "red0_wend", "stop_ts", "uid_init", "lookahead"):
            assert plan[f] == whole[f], f
        td.barrier()
    finally:
        td.destroy_process_group()


@pytest.mark.parametrize("workload,world,leaves,skew", [
    ("p2p-grid", 2, 0, False),       # config 4 weak-scaled: 128 x 256 in 2 row bands
    ("p2p-grid", 4, 0, False),       # 128 x 512 in 4
    ("dumbbell", 4, 499_999, False),  # config 5 at BASELINE size: 1,000,000 nodes, simple-distributed.cc's owners
    ("dumbbell", 2, 20_000, False),
    ("p2p-grid", 2, 0, True),        # rank 1 builds another grid: both ranks fail before any collective
])
def test_gloo_ranks_build_equal_plans(workload, world, leaves, skew):
    """a per-rank size mismatch is an RCCL hang at N > 1 that no single-process test sees.
    Each gloo process builds the partitioned scenario on its own, and the ranks' plans must agree field for field
    (except each rank's own setup events and pool)."""
    import torch.multiprocessing as mp
    mp.spawn(_plan_worker, args=(world, _free_port(), workload, leaves or 499_999, skew), nprocs=world, join=True)


def test_wifi_receiver_partitions():
    """The Wi-Fi split's receiver blocks (wifi.partitions, bench.py wifi-grid --gpus N): contiguous,
    covering every phy once, balanced, empty blocks allowed when there are more partitions than phys."""
    import wifi
    for n, k in [(10_000, 1), (10_000, 2), (10_000, 8), (3, 5), (7, 3)]:
        r = wifi.partitions(n, k)
        assert len(r) == k and r[0][0] == 0 and r[-1][1] == n
        assert all(a[1] == b[0] for a, b in zip(r, r[1:]))
        sizes = [e - b for b, e in r]
        assert min(sizes) >= 0 and max(sizes) - min(sizes) <= 1
