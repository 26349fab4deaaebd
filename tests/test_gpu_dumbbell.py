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
