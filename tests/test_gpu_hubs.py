"""Hub nodes and sorted runs of the single-GPU engine (nsgpu_p2p_win.h) against the oracle.

* a node with more than CH window events is run by a hub block (forwarding routers: the dumbbell;
  a node that is also the PacketSink: incast, whose local deliveries run zero-delay DoForwardUp
  leaves inline);
* a hub with more than HUBL events in a window, or a window larger than WCAP, is dispatched as a
  radix-sorted run in chunks — with more than WCAP same-time deliveries to one sink a chunk boundary
  cuts a same-time group, whose DoForwardUp leaves are then queued (K_FWD_UP_D).
Every case compares the full (ts, uid, context) pop log, counters and trace records bit for bit."""
import numpy as np
import pytest

import p2p
from test_gpu_trace import assert_same_run, gpu_full, oracle_full

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n_src", [40, 300, 5000])
def test_incast_sink_hub(n_src):
    sc = p2p.incast(n_src)
    o = oracle_full(sc, 400000)
    assert o[2]["rx_packets"][0] > 0
    assert_same_run(sc, o, gpu_full(sc, 400000, 2_000_000))


def test_incast_congested_drops():
    """The hub's own uplinks are idle, but every leaf queue overflows: 8 Mb/s of offered load on 1 Mb/s."""
    sc = p2p.incast(64, bps=1_000_000, qmax=5, rate_bps=8_000_000)
    o = oracle_full(sc, 200000)
    assert o[1]["drop_packets"].sum() > 0
    assert_same_run(sc, o, gpu_full(sc, 200000, 1_000_000))


def test_dumbbell_router_hub_over_hubl():
    """2,000 leaves: router 1 takes 2,000 same-time Receives in a window of at most WCAP events, more
    than a hub block sorts in LDS: the window is dispatched as a sorted run."""
    sc = p2p.dumbbell(2000)
    o = oracle_full(sc, 100000)
    assert_same_run(sc, o, gpu_full(sc, 100000, 200000))


def test_dumbbell_65536_nodes_single_gpu():
    """Config 5's dumbbell at 65,536 nodes (2 routers + 2 x 32,767 leaves, compressed routes): the
    sequential counters and digest."""
    n = 32_767
    sc = p2p.dumbbell(n)
    o = oracle_full(sc, 0)
    st, devc, appc = o[0], o[1], o[2]
    gst, gdevc, gappc, _ = p2p.Engine(sc).run()
    for f in ("dispatched", "cancelled", "digest", "final_ts", "next_uid", "ttl_drops", "no_route_drops"):
        assert getattr(gst, f) == getattr(st, f), (f, getattr(gst, f), getattr(st, f))
    assert np.array_equal(gdevc, devc)
    assert np.array_equal(gappc, appc)


def test_dumbbell_65536_nodes_eight_partitions():
    """The same 65,536-node dumbbell partitioned 8 ways the way simple-distributed.cc assigns system ids
    (left side + router 1 on rank 0; router 2 and the right leaves over ranks 1-7), all partitions on
    one GPU through the loopback group: the sequential counters and digest."""
    n = 32_767
    sc = p2p.dumbbell(n)
    st, devc, appc, _log, _tr = oracle_full(sc, 0)
    grp = p2p.LoopbackGroup(sc, 8, owner=p2p.dumbbell_owner(n, 8))
    gst, gdevc, gappc, _ = grp.run()
    for f in ("dispatched", "cancelled", "digest", "final_ts", "next_uid", "ttl_drops", "no_route_drops"):
        assert getattr(gst, f) == getattr(st, f), (f, getattr(gst, f), getattr(st, f))
    assert np.array_equal(gdevc, devc)
    assert np.array_equal(gappc, appc)
