"""Partitioned (multi-GPU) p2p engine vs the SEQUENTIAL oracle.

The partitions run on one GPU through the loopback transport (device copies in place of the RCCL
collectives, nsgpu_p2p_group_*) and through RCCL with one rank.  Bit-exact: the merged (ts, uid,
context) pop order, dispatch count, cancelled dispatches, digest, final time, next uid and every
per-device / per-application counter — the partitioned run reproduces DefaultSimulatorImpl's
sequential order and uids, which DistributedSimulatorImpl itself does not (its uids are per rank)."""
import numpy as np
import pytest

import nsref
import p2p
from test_gpu_p2p import assert_same

pytestmark = pytest.mark.gpu


def oracle(sc, log_cap=0):
    s = sc.c_struct()
    st = p2p.P2PStats()
    devc = np.zeros(s.n_devices, p2p.DEV_COUNTERS_DTYPE)
    appc = np.zeros(s.n_apps, p2p.APP_COUNTERS_DTYPE)
    _, olog = nsref.p2p_run(s, st, devc, appc, log_cap)
    return st, devc, appc, olog


@pytest.mark.parametrize("nranks", [1, 2, 3, 4])
def test_grid_full_pop_order(nranks):
    sc = p2p.grid(8, 8)
    o = oracle(sc, 60000)
    grp = p2p.LoopbackGroup(sc, nranks, log_cap=60000)
    assert all(m.wide() for m in grp.members)  # (wide windows: local records ranked across the ranks)
    g = grp.run(log_n=60000)
    assert_same(o, g)


@pytest.mark.parametrize("nranks", [2, 4])
def test_wide_and_narrow_partitioned_windows_agree(nranks, monkeypatch):
    """The same 24x24 grid through wide partitioned windows (same-node TransmitCompletes run inside the window as
    local records, ordered across ranks by their chain words in X1Loc) and through narrow ones
    (NSGPU_P2P_NARROW=1): both equal the oracle's full pop log, and the wide run takes fewer windows."""
    sc = p2p.grid(24, 24)
    o = oracle(sc, 400000)
    wide = p2p.LoopbackGroup(sc, nranks, log_cap=400000)
    assert all(m.wide() for m in wide.members)
    gw = wide.run(log_n=400000)
    assert_same(o, gw)
    monkeypatch.setenv("NSGPU_P2P_NARROW", "1")
    narrow = p2p.LoopbackGroup(sc, nranks, log_cap=400000)
    assert not any(m.wide() for m in narrow.members)
    gn = narrow.run(log_n=400000)
    assert_same(o, gn)
    assert gw[0].windows < gn[0].windows, (gw[0].windows, gn[0].windows)


def test_config4_grid_partitioned_rccl_counters_digest():
    """The partitioned bench line's workload on one RCCL rank (128x128, wide windows): every counter, the digest,
    final time and next uid equal the oracle's."""
    sc = p2p.grid(128, 128)
    o = oracle(sc)
    comm = p2p.Comm(p2p.Comm.unique_id(), 1, 0)
    eng = p2p.DistEngine(sc, np.zeros(sc.n_nodes, np.uint32), 0, 1, comm)
    assert eng.wide()
    assert_same(o, eng.run(), log=False)


@pytest.mark.parametrize("seed", range(3))
def test_random_topologies_two_partitions(seed):
    sc = p2p.random_topology(15, 25, 8, seed)
    o = oracle(sc, 300000)
    g = p2p.LoopbackGroup(sc, 2, log_cap=300000).run(log_n=300000)
    assert_same(o, g)


def test_random_topology_interleaved_owners():
    """Owners need not be blocks: every other node on the other rank (most links cut)."""
    sc = p2p.random_topology(15, 25, 8, 7)
    owner = (np.arange(sc.n_nodes) % 2).astype(np.uint32)
    o = oracle(sc, 300000)
    g = p2p.LoopbackGroup(sc, 2, owner=owner, log_cap=300000).run(log_n=300000)
    assert_same(o, g)


def test_congested_drops_three_partitions():
    sc = p2p.grid(5, 5, bps=1_000_000, qmax=5, rate_bps=2_000_000, stop_ns=400_000_000, sim_stop_ns=500_000_000)
    o = oracle(sc, 200000)
    g = p2p.LoopbackGroup(sc, 3, log_cap=200000).run(log_n=200000)
    assert o[1]["drop_packets"].sum() > 0
    assert_same(o, g)


def test_window_cut_agreement():
    """48x48: the setup windows overflow WCAP on each rank, and the X0 agreement cuts every rank's
    window at the smallest fitting bound."""
    sc = p2p.grid(48, 48)
    o = oracle(sc)
    g = p2p.LoopbackGroup(sc, 2).run()
    assert g[0].refits > 0
    assert_same(o, g, log=False)


def test_weak_scaled_grid_four_partitions():
    """The bench's weak-scaling layout at small size: grid(rows, cols * N) in N row bands, every
    column flow crossing every band."""
    sc = p2p.grid(16, 16 * 4)
    o = oracle(sc)
    g = p2p.LoopbackGroup(sc, 4).run()
    assert_same(o, g, log=False)


def test_rccl_single_rank():
    sc = p2p.grid(12, 12)
    o = oracle(sc, 100000)
    comm = p2p.Comm(p2p.Comm.unique_id(), 1, 0)
    eng = p2p.DistEngine(sc, np.zeros(sc.n_nodes, np.uint32), 0, 1, comm, log_cap=100000)
    g = eng.run(log_n=100000)
    assert_same(o, g)
    g2 = eng.run(log_n=100000)  # (graph replay of the same engine)
    assert_same(o, g2)


@pytest.mark.parametrize("nranks", [2, 3])
def test_incast_sorted_run_cuts_a_same_ts_group(nranks):
    """A partitioned sorted run (nsgpu_p2p_win.h): 5,000 leaves send to one hub at the same instant, so its
    windows hold 5,000 same-ts Receives whose DoForwardUp leaves are zero-delay children: more than a rank's
    WCAP, so the window becomes a run sorted once per rank and dispatched in chunks; chunks cut that same-ts group
    (its leaves queued), the chunk that ends it ends the run, and the rest returns to pending.  The hub and 4,000
    leaves on rank 0, the last 1,000 leaves over the other ranks (X2 holds at most 1,024 remote events a peer a
    window).  Full pop log."""
    sc = p2p.incast(5000, stop_ns=1_020_000_000, sim_stop_ns=1_040_000_000)
    owner = np.zeros(sc.n_nodes, np.uint32)
    owner[4001:] = 1 + (np.arange(1000) * (nranks - 1)) // 1000
    o = oracle(sc, 400000)
    g = p2p.LoopbackGroup(sc, nranks, owner=owner, log_cap=400000).run(log_n=400000)
    assert g[0].refits > 0
    assert_same(o, g)
