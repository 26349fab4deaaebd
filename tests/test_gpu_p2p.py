"""GPU-resident point-to-point subset vs the oracle (configs 2/4 handler chain).

Bit-exact: the full (ts, uid, context) pop order on small scenarios; dispatch count, cancelled
dispatches, digest, final time, next uid and every per-device / per-application counter on the
larger grids."""
import numpy as np
import pytest

import nsref
import p2p

pytestmark = pytest.mark.gpu


def both(sc, log_cap=0):
    s = sc.c_struct()
    st = p2p.P2PStats()
    devc = np.zeros(s.n_devices, p2p.DEV_COUNTERS_DTYPE)
    appc = np.zeros(s.n_apps, p2p.APP_COUNTERS_DTYPE)
    _, olog = nsref.p2p_run(s, st, devc, appc, log_cap)
    eng = p2p.Engine(sc, log_cap=log_cap)
    gst, gdevc, gappc, glog = eng.run(log_n=log_cap)
    return (st, devc, appc, olog), (gst, gdevc, gappc, glog)


def assert_same(o, g, log=True):
    st, devc, appc, olog = o
    gst, gdevc, gappc, glog = g
    for f in ("dispatched", "cancelled", "digest", "final_ts", "next_uid", "ttl_drops", "no_route_drops"):
        assert getattr(gst, f) == getattr(st, f), (f, getattr(gst, f), getattr(st, f))
    assert np.array_equal(gdevc, devc)
    assert np.array_equal(gappc, appc)
    if log:
        n = int(min(st.dispatched, len(olog[0])))
        for a, b, name in zip(glog, olog, ("ts", "uid", "ctx")):
            assert np.array_equal(a[:n], b[:n]), name


@pytest.mark.parametrize("seed", range(6))
def test_random_topologies_full_pop_order(seed):
    sc = p2p.random_topology(15, 25, 8, seed)
    o, g = both(sc, log_cap=300000)
    assert_same(o, g)


def test_grid_8x8_full_pop_order():
    o, g = both(p2p.grid(8, 8), log_cap=60000)
    assert_same(o, g)


def test_grid_congested_drops():
    # 1 Mb/s links with 4 sources per destination column: DropTail overflows
    g = p2p.grid(5, 5, bps=1_000_000, qmax=5, rate_bps=2_000_000, stop_ns=400_000_000,
                 sim_stop_ns=500_000_000)
    o, gg = both(g, log_cap=200000)
    assert o[1]["drop_packets"].sum() > 0
    assert_same(o, gg)


def test_grid_32x32_counters_digest():
    o, g = both(p2p.grid(32, 32))
    assert_same(o, g, log=False)


def test_eager_launches_match_graph_replays():
    """The kernels launched one by one (profiling mode) compute exactly what the graph replays do."""
    sc = p2p.grid(12, 12)
    eng = p2p.Engine(sc, log_cap=100000)
    a = eng.run(log_n=100000)
    eng.set_eager(True)
    b = eng.run(log_n=100000)
    assert_same((a[0], a[1], a[2], a[3]), b)
    prof = eng.profile(sample_every=2)
    assert set(prof) >= {"k2_pa", "k2_handle", "k2_scan"}
    assert all(ms >= 0 for ms, _ in prof.values())
    c = eng.results()
    assert c[0].digest == a[0].digest and c[0].dispatched == a[0].dispatched


def test_grid_128x128_counters_digest():
    """The bench workload itself (config 4): every counter, the digest, final time and next uid."""
    o, g = both(p2p.grid(128, 128))
    assert_same(o, g, log=False)


def test_setup_list_from_journal_app_before_a_device():
    """A program that installs an application on a node before one more link (its journal has an
    Application::Start between two NetDevice::Starts): the setup list nsgpu_setup_from_journal derives from
    the classified journal runs on the engine exactly as on the oracle, full pop order."""
    from test_setup_journal_cpu import app_before_link
    sc = app_before_link()
    j, devs, napp = p2p.scenario_journal(sc)
    setup, _owned, _dmap, _amap, _stop = p2p.setup_from_journal(j, devs, napp)
    sc.setup = setup
    o, g = both(sc, log_cap=20000)
    assert o[2]["rx_packets"][0] > 0
    assert_same(o, g)


def test_stop_before_start_bounded_by_a_far_stop():
    """r04c's scenario (OnOff StartTime 0.1 s, StopTime 0.02 s: the flow never stops, application.cc:87-95) with
    an explicit Simulator::Stop at 3 s: full pop log = the oracle's (without the Stop the run is unbounded in ns-3
    too; tests/test_p2p_oracle.py pins the semantics)."""
    sc = p2p.grid(2, 2, start_ns=100_000_000, stop_ns=20_000_000, sim_stop_ns=3_000_000_000, flows=[(0, 3)])
    o, g = both(sc, log_cap=20_000)
    assert o[2]["tx_packets"].sum() > 300
    assert_same(o, g)


@pytest.mark.parametrize("which", ["grid", "random", "dumbbell_hubs", "partitioned", "traced"])
def test_poisoned_device_memory(which, monkeypatch):
    """r04b: the fault came from device memory a previous engine had dirtied (create did not zero the deferred
    pipeline's arrays).  NSGPU_P2P_POISON=1 fills every array with 0xa5 bytes when it is allocated, before create
    initialises it: each pipeline (deferred, hub blocks, partitioned, traced) must still equal the oracle."""
    monkeypatch.setenv("NSGPU_P2P_POISON", "1")
    if which == "grid":
        sc = p2p.grid(12, 12)
        eng = p2p.Engine(sc, log_cap=60_000)
        assert eng.wide()
        o = both(sc, log_cap=60_000)[0]
        assert_same(o, eng.run(log_n=60_000))
    elif which == "random":
        o, g = both(p2p.random_topology(15, 25, 8, 3), log_cap=300_000)
        assert_same(o, g)
    elif which == "dumbbell_hubs":
        o, g = both(p2p.dumbbell(2000), log_cap=0)
        assert_same(o, g, log=False)
    elif which == "partitioned":
        sc = p2p.grid(6, 6)
        o = both(sc, log_cap=0)[0]
        st = p2p.LoopbackGroup(sc, 3).run()[0]
        assert (st.dispatched, st.digest, st.next_uid) == (o[0].dispatched, o[0].digest, o[0].next_uid)
    else:
        from test_gpu_trace import assert_same_trace, oracle_trace
        import trace
        g = p2p.grid(4, 4, qmax=3, rate_bps=4_000_000, stop_ns=300_000_000, sim_stop_ns=400_000_000,
                     flows=[(0, 15), (1, 15), (4, 15), (5, 15)])
        _ost, odevc, otr = oracle_trace(g)
        eng = p2p.Engine(g)
        eng.set_trace(len(otr) + 16)
        _st, gdevc, _appc, _log = eng.run()
        assert np.array_equal(gdevc, odevc)
        assert_same_trace(g, otr, trace.sort_records(eng.trace()))
