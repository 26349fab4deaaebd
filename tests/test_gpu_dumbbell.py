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


LEAVES = 4_095  # 8,192 nodes; the BASELINE size (499,999 per side) is DESIGN.md 4.3's open item


@pytest.fixture(scope="module")
def million():
    """A large config-5 dumbbell: 2 routers + 2 x 4,095 leaves = 8,192 nodes (compressed routes).
    The dumbbell's two routers are hub nodes: a window holds up to WCAP of their events, which one
    holder thread walks with the O(W) per-event slot scan, so run time grows with
    the leaf count squared; the BASELINE's 1,000,000 nodes does not finish in a test's time yet
    (65,536 nodes: 53 s on one MI355X, bit-exact)."""
    sc = p2p.dumbbell(LEAVES)
    st, devc, appc, _log, _tr = oracle_full(sc, 0)
    return sc, st, devc, appc


def _same_counters(gst, gdevc, gappc, st, devc, appc):
    for f in ("dispatched", "cancelled", "digest", "final_ts", "next_uid", "ttl_drops", "no_route_drops"):
        assert getattr(gst, f) == getattr(st, f), (f, getattr(gst, f), getattr(st, f))
    assert np.array_equal(gdevc, devc)
    assert np.array_equal(gappc, appc)


def test_dumbbell_large_single_gpu(million):
    sc, st, devc, appc = million
    assert sc.n_nodes == 2 * LEAVES + 2 and st.dispatched > 60_000
    gst, gdevc, gappc, _ = p2p.Engine(sc).run()
    _same_counters(gst, gdevc, gappc, st, devc, appc)


def test_dumbbell_large_eight_partitions(million):
    """Partitioned 8 ways (left side + router 1 on rank 0, router 2 and the right leaves over ranks
    1-7) through the loopback group: the sequential counters and digest."""
    sc, st, devc, appc = million
    grp = p2p.LoopbackGroup(sc, 8, owner=p2p.dumbbell_owner(LEAVES, 8))
    gst, gdevc, gappc, _ = grp.run()
    _same_counters(gst, gdevc, gappc, st, devc, appc)
