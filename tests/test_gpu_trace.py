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


# ---------------------------------------------------------------- UDP echo (config 1: first.cc)
def gpu_full(sc, log_cap, trace_cap, kinds=nsref.TRACE_DEVICE_KINDS):
    eng = p2p.Engine(sc, log_cap=log_cap)
    eng.set_trace(trace_cap, kinds)
    st, devc, appc, log = eng.run(log_n=log_cap)
    return st, devc, appc, log, trace.sort_records(eng.trace())


def oracle_full(sc, log_cap, kinds=nsref.TRACE_DEVICE_KINDS):
    s = sc.c_struct()
    st = p2p.P2PStats()
    devc = np.zeros(s.n_devices, p2p.DEV_COUNTERS_DTYPE)
    appc = np.zeros(s.n_apps, p2p.APP_COUNTERS_DTYPE)
    _secs, log, tr = nsref.p2p_run_trace(s, st, devc, appc, log_cap, kinds=kinds)
    return st, devc, appc, log, trace.sort_records(tr)


def assert_same_run(sc, o, g):
    st, devc, appc, olog, otr = o
    gst, gdevc, gappc, glog, gtr = g
    for f in ("dispatched", "cancelled", "digest", "final_ts", "next_uid", "ttl_drops", "no_route_drops"):
        assert getattr(gst, f) == getattr(st, f), (f, getattr(gst, f), getattr(st, f))
    assert np.array_equal(gdevc, devc)
    assert np.array_equal(gappc, appc)
    n = int(min(st.dispatched, len(olog[0])))
    for a, b, name in zip(glog, olog, ("ts", "uid", "ctx")):
        assert np.array_equal(a[:n], b[:n]), name
    assert_same_trace(sc, otr, gtr)


def test_first_cc_on_gpu_matches_reference_md5s():
    """examples/tutorial/first.cc on the GPU engine: the 19 events of the reference run and its
    ascii / pcap files byte for byte (md5s recorded from the unmodified reference)."""
    import json
    import os
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "survey_reference_runs.json")) as f:
        ref = json.load(f)["first_cc"]
    sc = p2p.first_cc()
    o = oracle_full(sc, 64)
    g = gpu_full(sc, 64, 64)
    assert_same_run(sc, o, g)
    gst, _gdevc, gappc, _glog, gtr = g
    assert gst.dispatched == ref["events_dispatched"] == 19
    assert int(gappc["rx_packets"].sum()) == ref["received_lines"]
    codec = trace.Codec(sc)
    assert hashlib.md5(codec.ascii(gtr).encode()).hexdigest() == ref["ascii_md5"]
    pc = codec.pcaps(gtr)
    assert hashlib.md5(pc[(0, 0)]).hexdigest() == ref["node0_pcap_md5"]
    assert hashlib.md5(pc[(1, 0)]).hexdigest().startswith(ref["node1_pcap_md5_prefix"])


def test_echo_count_interval_and_stop_cancel_gpu():
    sc = p2p.Scenario(2)
    da, db = sc.link(0, 1, 5_000_000, 2_000_000)
    sc.install_stack()
    sc.assign_link(da, db, p2p.ip("10.1.1.0"))
    sc.add_echo_server(1, 1_000_000_000, 10_000_000_000)
    sc.add_echo_client(0, 1, 2_000_000_000, 2_600_000_000, count=3, interval_ns=500_000_000,
                       remote_addr=sc.dev_addr[db])
    sc.route_bfs()
    o = oracle_full(sc, 256)
    assert o[0].cancelled == 1
    assert_same_run(sc, o, gpu_full(sc, 256, 256))


def echo_grid(rows, cols, interval_ns, count, qmax=100):
    """A grid with UdpEchoServers on the bottom row and UdpEchoClients on the top row (one pair per
    column, diagonal partner), plus the column OnOff flows' PacketSinks replaced by the servers."""
    g = p2p.grid(rows, cols, qmax=qmax, flows=[])
    for c in range(cols):
        g.add_echo_server((rows - 1) * cols + c, 50_000_000, 900_000_000)
    for c in range(cols):
        dst = (rows - 1) * cols + (cols - 1 - c)
        g.add_echo_client(c, dst, 100_000_000 + 1_000_000 * c, 800_000_000, count=count, interval_ns=interval_ns,
                          size=512)
    g.route_bfs()
    return g


@pytest.mark.parametrize("interval_ns,count,qmax", [(200_000_000, 3, 100), (300_000, 40, 4)])
def test_echo_grid(interval_ns, count, qmax):
    g = echo_grid(4, 4, interval_ns, count, qmax)
    o = oracle_full(g, 100000)
    assert o[2]["rx_packets"].sum() > 0
    if qmax == 4:
        assert o[1]["drop_packets"].sum() > 0
    assert_same_run(g, o, gpu_full(g, 100000, 200000))


@pytest.mark.parametrize("nranks", [2])
def test_echo_grid_partitioned(nranks):
    g = echo_grid(4, 4, 300_000, 40, 4)
    _st, _devc, _appc, _log, otr = oracle_full(g, 0)
    grp = p2p.LoopbackGroup(g, nranks, trace_cap=len(otr) + 16)
    grp.run()
    assert_same_trace(g, otr, trace.sort_records(grp.trace()))


def halfway_link():
    """Two nodes, 10 Mb/s, delay 1,991,400 ns, a 4.096 Mb/s CBR OnOff from 1.1 s to 1.9 s: sends every 1 ms,
    Receive / MacRx at ... 5,000 ns (transmission 433,600 + delay) — GetSeconds () of those lies half-way
    between two 6-digit decimals, where ns-3's int64x64 path and ts / 1e9 round apart on ~6 % of them
    (trace-helper.cc:306-390, nstime.h:419-431)."""
    sc = p2p.Scenario(2)
    da, db = sc.link(0, 1, 10_000_000, 1_991_400)
    sc.install_stack()
    sc.assign_link(da, db, p2p.ip("10.1.1.0"))
    sc.add_sink(1, 0, 2_500_000_000)
    sc.add_onoff(0, 1, 1_100_000_000, 1_900_000_000, rate_bps=4_096_000, on_s=1e9, off_s=0.0,
                 remote_addr=sc.dev_addr[db])
    sc.route_bfs()
    return sc


def test_halfway_timestamps_gpu_equals_oracle_line_for_line():
    sc = halfway_link()
    o = oracle_full(sc, 4096)
    g = gpu_full(sc, 4096, 8192)
    assert_same_run(sc, o, g)
    gtr = g[4]
    naive = ["%g" % (int(t) / 1e9) for t in gtr["ts"]]
    ns3 = [trace.seconds_text(int(t)) for t in gtr["ts"]]
    assert sum(a != b for a, b in zip(naive, ns3)) > 0  # the run does land on half-way timestamps
    cc = p2p.TraceCodec(sc)
    assert cc.ascii(gtr) == trace.Codec(sc).ascii(o[4])
