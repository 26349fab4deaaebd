"""Wide windows of the single p2p engine: windows bounded by the cross-node lookahead,
a node's same-node TransmitCompletes running inside the window as local records, ranked after the handlers
(k2_rank, by their chains up to a gen-0 ancestor) and given their uids from their parents' child prefixes
(k2_scan).

Every run is compared with the oracle's sequential DefaultSimulatorImpl restatement — full (ts, uid,
context) pop log, counters and trace records — and with the same engine forced narrow
(NSGPU_P2P_NARROW=1).  Cases: the config-4 shape, a congested grid (TransmitComplete chains: local records
of local records), random topologies, ICMP TTL expiry, host closures cutting wide windows, and a start
burst larger than a window (a widened window trimmed back to its narrow bound, k_renarrow)."""
import os

import numpy as np
import pytest

import p2p
from test_gpu_trace import assert_same_run, gpu_full, oracle_full

pytestmark = pytest.mark.gpu


def narrow_engine(sc, log_cap=0):
    os.environ["NSGPU_P2P_NARROW"] = "1"
    try:
        return p2p.Engine(sc, log_cap=log_cap)
    finally:
        del os.environ["NSGPU_P2P_NARROW"]


def check_wide_and_narrow(sc, log_cap, trace_cap, expect_wide=True):
    o = oracle_full(sc, log_cap)
    eng = p2p.Engine(sc)
    if expect_wide is not None:  # (wide needs Lx <= 8 tx_min: chains of local records stay short)
        assert eng.wide() == expect_wide
    eng.close()
    g = gpu_full(sc, log_cap, trace_cap)
    assert_same_run(sc, o, g)
    n = narrow_engine(sc, log_cap)
    assert not n.wide()
    nst, ndevc, nappc, nlog = n.run(log_n=log_cap)
    assert nst.digest == o[0].digest and nst.dispatched == o[0].dispatched
    assert np.array_equal(ndevc, o[1]) and np.array_equal(nappc, o[2])
    return g[0], nst


def test_config4_shape_wide_has_fewer_windows():
    sc = p2p.grid(16, 16, stop_ns=600_000_000, sim_stop_ns=650_000_000)
    gst, nst = check_wide_and_narrow(sc, 400_000, 2_000_000)
    assert gst.windows < nst.windows * 0.6, (gst.windows, nst.windows)


def test_lockstep_deep_chains_tie_break():
    """Two identical rows, each saturated by a flow along it (20 Mb/s offered to 10 Mb/s links): the sources'
    TransmitComplete chains run up to 3 deep inside each window, in lockstep across the rows, so local records
    of one ts whose parents and grandparents share their ts meet — their two order words tie and k2_rank falls
    back to the exact chain compare (the gen-0 ancestors' uids decide)."""
    cols = 8
    sc = p2p.grid(2, cols, flows=[(0, cols - 1), (cols, 2 * cols - 1)], rate_bps=20_000_000, qmax=100,
                  stop_ns=160_000_000, sim_stop_ns=180_000_000)
    check_wide_and_narrow(sc, 400_000, 2_000_000)


def test_congested_grid_transmit_complete_chains():
    """Every node of the top row sends 2 Mb/s to one bottom corner: the corner's column links saturate, the
    queues back up and drop, and TransmitComplete chains (a local record's TransmitStart making the next
    local record) run inside each window."""
    rows, cols = 8, 8
    flows = [(x, (rows - 1) * cols) for x in range(1, cols)]
    sc = p2p.grid(rows, cols, flows=flows, rate_bps=2_000_000, qmax=10, stop_ns=400_000_000,
                  sim_stop_ns=450_000_000)
    o = oracle_full(sc, 0)
    assert o[1]["drop_packets"].sum() > 0
    check_wide_and_narrow(sc, 300_000, 2_000_000)


@pytest.mark.parametrize("seed", range(5))
def test_random_topologies(seed):
    sc = p2p.random_topology(30, 60, 12, seed)
    check_wide_and_narrow(sc, 300_000, 2_000_000, expect_wide=None)


def test_icmp_ttl_expiry_grid():
    sc = p2p.grid(10, 10, ttl=5, icmp=True, stop_ns=300_000_000, sim_stop_ns=350_000_000)
    check_wide_and_narrow(sc, 300_000, 2_000_000, expect_wide=None)  # (58-B errors: Lx > 8 tx_min, narrow)


def test_start_burst_larger_than_a_window_is_trimmed_narrow():
    """4,500 flows start at the same instant on a 64 x 64 grid: the first windows overflow WCAP and become
    sorted runs; a widened one is trimmed back to its narrow bound before it runs."""
    rows = cols = 64
    n = rows * cols
    rng = np.random.default_rng(3)
    flows = [(int(s), int(d)) for s, d in zip(rng.integers(0, n, 4500), rng.integers(0, n, 4500)) if s != d]
    sc = p2p.grid(rows, cols, flows=flows, stop_ns=130_000_000, sim_stop_ns=140_000_000)
    o = oracle_full(sc, 0)
    g = p2p.Engine(sc)
    assert g.wide()
    gst, gdevc, gappc, _ = g.run()
    assert gst.refits > 0  # (sorted runs happened)
    for f in ("dispatched", "cancelled", "digest", "final_ts", "next_uid"):
        assert getattr(gst, f) == getattr(o[0], f), f
    assert np.array_equal(gdevc, o[1]) and np.array_equal(gappc, o[2])


def test_dumbbell_router_degree_keeps_narrow():
    """A router with more than 16 devices: the engine stays narrow (a node's pending local records are its
    busy devices' TransmitCompletes, bounded by LQ = 16)."""
    sc = p2p.dumbbell(40)
    assert not p2p.Engine(sc).wide()


@pytest.mark.parametrize("narrow", [False, True])
def test_host_closures_cut_windows(narrow):
    """Host probes (nsgpu_sim) between device events cap the windows at their keys and send datagrams
    (test_gpu_mixed's harness, which runs wide engines by default), here in both window modes."""
    from test_gpu_mixed import check_same, flows_grid, run_gpu, run_oracle
    sc = flows_grid()
    app_send = [i for i, a in enumerate(sc.apps) if a["kind"] == p2p.APP_ONOFF][1]
    app_obs = [i for i, a in enumerate(sc.apps) if a["kind"] == p2p.APP_SINK][0]
    o = run_oracle(sc, 150_000_000, 5_300_001, 30, app_send, app_obs, 400000)
    if narrow:
        os.environ["NSGPU_P2P_NARROW"] = "1"
    try:
        g = run_gpu(sc, 150_000_000, 5_300_001, 30, app_send, app_obs, 400000, 400000)
    finally:
        os.environ.pop("NSGPU_P2P_NARROW", None)
    check_same(sc, o, g)
