"""Config 5 (src/mpi/examples/simple-distributed.cc dumbbell) on the GPU engine vs the oracle:
single engine (full pop order, counters, digest, trace records) and partitioned the way the example
assigns system ids (left side + router 1 / router 2 + right side), through the loopback group."""
import numpy as np
import pytest

import p2p
import trace
from test_gpu_trace import assert_same_run, assert_same_trace, gpu_full, oracle_full

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n_leaves", [4, 64, 300])
def test_dumbbell_single_engine(n_leaves):
    sc = p2p.dumbbell(n_leaves)
    o = oracle_full(sc, 20000)
    if n_leaves == 300:
        assert o[1]["drop_packets"].sum() > 0  # the 5 Mb/s router link's DropTail overflows
    assert_same_run(sc, o, gpu_full(sc, 20000, 20000))


@pytest.mark.parametrize("n_leaves,nranks", [(4, 2), (300, 2), (300, 3)])
def test_dumbbell_partitioned_like_systemid(n_leaves, nranks):
    sc = p2p.dumbbell(n_leaves)
    st, devc, appc, _log, otr = oracle_full(sc, 0)
    grp = p2p.LoopbackGroup(sc, nranks, owner=p2p.dumbbell_owner(n_leaves, nranks), trace_cap=len(otr) + 16)
    gst, gdevc, gappc, _glog = grp.run()
    for f in ("dispatched", "cancelled", "digest", "final_ts", "next_uid"):
        assert getattr(gst, f) == getattr(st, f), f
    assert np.array_equal(gdevc, devc)
    assert np.array_equal(gappc, appc)
    assert_same_trace(sc, otr, trace.sort_records(grp.trace()))


def test_dumbbell_compressed_routes_match_dense():
    o = oracle_full(p2p.dumbbell(300, compressed=False), 20000)
    sc = p2p.dumbbell(300, compressed=True)
    assert sc.route is None
    assert_same_run(sc, o, gpu_full(sc, 20000, 20000))


LEAVES = 499_999  # the BASELINE size: 2 routers + 2 x 499,999 leaves = 1,000,000 nodes


@pytest.fixture(scope="module")
def million():
    """Config 5 at its BASELINE size: 1,000,000 nodes (compressed routes), 8.5 M events.  The oracle's
    sequential run (counters and digest, no trace) takes ~1-20 s on one host core; the scenario's Python
    build ~20 s."""
    import nsref
    sc = p2p.dumbbell(LEAVES)
    s = sc.c_struct()
    st = p2p.P2PStats()
    devc = np.zeros(s.n_devices, p2p.DEV_COUNTERS_DTYPE)
    appc = np.zeros(s.n_apps, p2p.APP_COUNTERS_DTYPE)
    nsref.p2p_run(s, st, devc, appc)
    return sc, st, devc, appc


def _same_counters(gst, gdevc, gappc, st, devc, appc):
    for f in ("dispatched", "cancelled", "digest", "final_ts", "next_uid", "ttl_drops", "no_route_drops"):
        assert getattr(gst, f) == getattr(st, f), (f, getattr(gst, f), getattr(st, f))
    assert np.array_equal(gdevc, devc)
    assert np.array_equal(gappc, appc)


def test_dumbbell_million_nodes_single_gpu(million):
    """simple-distributed.cc at 1,000,000 nodes on one engine: the sequential counters and digest."""
    sc, st, devc, appc = million
    assert sc.n_nodes == 1_000_000 and st.dispatched == 8_500_495
    eng = p2p.Engine(sc)
    gst, gdevc, gappc, _ = eng.run()
    eng.close()
    _same_counters(gst, gdevc, gappc, st, devc, appc)


def test_dumbbell_million_nodes_eight_partitions(million):
    """The same 1,000,000-node run partitioned 8 ways the way simple-distributed.cc assigns system ids
    (left side + router 1 on rank 0, router 2 and the right leaves over ranks 1-7), all partitions on
    one GPU through the loopback group: the sequential counters and digest."""
    sc, st, devc, appc = million
    grp = p2p.LoopbackGroup(sc, 8, owner=p2p.dumbbell_owner(LEAVES, 8))
    gst, gdevc, gappc, _ = grp.run()
    _same_counters(gst, gdevc, gappc, st, devc, appc)
