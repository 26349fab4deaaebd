"""GPU-resident trace sink records vs the oracle (trace-record replay).

The GPU p2p engine records every ascii trace sink call (TxQueue Enqueue/Dequeue/Drop, MacRx) of a
run; ordered by (ts, uid, seq) the records must equal the oracle's bit for bit, and the trace codec
must turn both into the same ascii and pcap bytes.  The oracle's records are pinned against the
unmodified reference's first.cc ascii/pcap md5s (tests/test_trace_oracle.py)."""
import hashlib

import numpy as np
import pytest

import nsref
import p2p
import trace

pytestmark = pytest.mark.gpu

FIELDS = ("ts", "uid", "seq", "kind", "dev", "app", "ipid", "size", "ttl")


def oracle_trace(sc):
    s = sc.c_struct()
    st = p2p.P2PStats()
    devc = np.zeros(s.n_devices, p2p.DEV_COUNTERS_DTYPE)
    appc = np.zeros(s.n_apps, p2p.APP_COUNTERS_DTYPE)
    _secs, _log, tr = nsref.p2p_run_trace(s, st, devc, appc, 0)
    return st, devc, trace.sort_records(tr)


def assert_same_trace(sc, otr, gtr):
    assert len(gtr) == len(otr)
    for f in FIELDS:
        assert np.array_equal(gtr[f], otr[f]), f
    codec = trace.Codec(sc)
    assert hashlib.md5(codec.ascii(gtr).encode()).hexdigest() == hashlib.md5(codec.ascii(otr).encode()).hexdigest()
    gp, op = codec.pcaps(gtr), codec.pcaps(otr)
    assert gp.keys() == op.keys()
    for k in op:
        assert gp[k] == op[k], k


def gpu_trace(sc, cap):
    eng = p2p.Engine(sc)
    eng.set_trace(cap)
    st, devc, _appc, _log = eng.run()
    return st, devc, trace.sort_records(eng.trace())


@pytest.mark.parametrize("seed", range(4))
def test_random_topology_trace(seed):
    sc = p2p.random_topology(15, 25, 8, seed)
    ost, odevc, otr = oracle_trace(sc)
    gst, gdevc, gtr = gpu_trace(sc, len(otr) + 16)
    assert gst.digest == ost.digest
    assert np.array_equal(gdevc, odevc)
    assert_same_trace(sc, otr, gtr)


def test_grid_congested_trace_with_drops():
    g = p2p.grid(4, 4, qmax=3, rate_bps=4_000_000, stop_ns=300_000_000, sim_stop_ns=400_000_000,
                 flows=[(0, 15), (1, 15), (4, 15), (5, 15)])
    _ost, odevc, otr = oracle_trace(g)
    assert (otr["kind"] == trace.TR_DROP).sum() > 0
    _gst, gdevc, gtr = gpu_trace(g, len(otr))
    assert np.array_equal(gdevc, odevc)
    assert_same_trace(g, otr, gtr)


def test_grid_8x8_trace():
    g = p2p.grid(8, 8)
    _ost, _odevc, otr = oracle_trace(g)
    _gst, _gdevc, gtr = gpu_trace(g, len(otr))
    assert_same_trace(g, otr, gtr)


def test_trace_capacity_overflow_is_reported():
    g = p2p.grid(4, 4)
    eng = p2p.Engine(g)
    eng.set_trace(8)
    eng.run()
    with pytest.raises(Exception):
        eng.trace()


@pytest.mark.parametrize("nranks", [2, 3])
def test_partitioned_trace_union(nranks):
    """Each partition records the sink calls of its own nodes; their union is the sequential trace."""
    g = p2p.grid(6, 6, qmax=4, rate_bps=2_000_000, stop_ns=300_000_000, sim_stop_ns=400_000_000)
    _ost, _odevc, otr = oracle_trace(g)
    grp = p2p.LoopbackGroup(g, nranks, trace_cap=len(otr) + 16)
    grp.run()
    assert_same_trace(g, otr, trace.sort_records(grp.trace()))
