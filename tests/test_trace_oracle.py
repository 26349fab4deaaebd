"""Trace replay pinned against the reference's own output (no GPU).

examples/tutorial/first.cc run by the oracle (restated DefaultSimulatorImpl + p2p/IPv4/UDP chain with
UdpEchoClient/UdpEchoServer) records its ascii trace sink calls; the trace codec (ns-3-dev-dnemu_amd/
trace.py) turns them into ns-3's ascii and pcap bytes, whose md5s must equal the ones recorded from
the unmodified reference (tests/golden/survey_reference_runs.json, SURVEY.md:408): 19 events, the
EnableAsciiAll (stream) file, and both EnablePcapAll files."""
import hashlib
import json
import os

import numpy as np

import nsref
import p2p
import trace

HERE = os.path.dirname(os.path.abspath(__file__))


def run_trace(sc, log_cap=0):
    s = sc.c_struct()
    st = p2p.P2PStats()
    devc = np.zeros(s.n_devices, p2p.DEV_COUNTERS_DTYPE)
    appc = np.zeros(s.n_apps, p2p.APP_COUNTERS_DTYPE)
    _secs, log, tr = nsref.p2p_run_trace(s, st, devc, appc, log_cap)
    return st, devc, appc, log, trace.sort_records(tr)


def reference_first():
    with open(os.path.join(HERE, "golden", "survey_reference_runs.json")) as f:
        return json.load(f)["first_cc"]


def test_first_cc_events_and_traces_match_reference():
    ref = reference_first()
    sc = p2p.first_cc()
    st, devc, appc, (lts, luid, lctx), tr = run_trace(sc, log_cap=64)
    assert st.dispatched == ref["events_dispatched"] == 19
    # the two "Received ..." log lines: server and client HandleRead
    assert int(appc["rx_packets"].sum()) == ref["received_lines"]
    assert st.cancelled == 0 and st.final_ts == 10_000_000_000  # the Stop events of both applications
    codec = trace.Codec(sc)
    text = codec.ascii(tr)
    assert hashlib.md5(text.encode()).hexdigest() == ref["ascii_md5"]
    pc = codec.pcaps(tr)
    assert hashlib.md5(pc[(0, 0)]).hexdigest() == ref["node0_pcap_md5"]
    assert hashlib.md5(pc[(1, 0)]).hexdigest().startswith(ref["node1_pcap_md5_prefix"])


def test_first_cc_trace_content():
    sc = p2p.first_cc()
    _st, _devc, _appc, _log, tr = run_trace(sc)
    lines = trace.Codec(sc).ascii(tr).splitlines()
    assert [ln[:1] for ln in lines] == ["+", "-", "r", "+", "-", "r"]
    # request 2 s -> node 1 after txTime (1054 B at 5 Mb/s = 1.6864 ms) + 2 ms; the echo leaves at once
    assert [int(t) for t in tr["ts"]] == [2_000_000_000] * 2 + [2_003_686_400] * 3 + [2_007_372_800]
    assert "10.1.1.1 > 10.1.1.2" in lines[0] and "49153 > 9" in lines[0]
    assert "10.1.1.2 > 10.1.1.1" in lines[3] and "9 > 49153" in lines[3]


def test_echo_count_interval_and_stop_cancel():
    """MaxPackets 3, Interval 0.5 s, client stopped at 2.6 s: 2 requests sent, the third Send cancelled
    (StopApplication: Simulator::Cancel (m_sendEvent)) but still dispatched (H16)."""
    sc = p2p.Scenario(2)
    da, db = sc.link(0, 1, 5_000_000, 2_000_000)
    sc.install_stack()
    sc.assign_link(da, db, p2p.ip("10.1.1.0"))
    sc.add_echo_server(1, 1_000_000_000, 10_000_000_000)
    sc.add_echo_client(0, 1, 2_000_000_000, 2_600_000_000, count=3, interval_ns=500_000_000,
                       remote_addr=sc.dev_addr[db])
    sc.route_bfs()
    st, devc, appc, _log, tr = run_trace(sc)
    assert st.cancelled == 1
    assert appc["tx_packets"].tolist() == [2, 2] and appc["rx_packets"].tolist() == [2, 2]
    # IPv4 identification counts each node's originated datagrams
    req = tr[(tr["kind"] == trace.TR_ENQUEUE) & ((tr["app"] & trace.PKT_REPLY) == 0)]
    rep = tr[(tr["kind"] == trace.TR_ENQUEUE) & ((tr["app"] & trace.PKT_REPLY) != 0)]
    assert req["ipid"].tolist() == [0, 1] and rep["ipid"].tolist() == [0, 1]


def test_grid_trace_conservation():
    """Trace records agree with the counters: one '+' per enqueue, '-' per dequeue, 'd' per drop, 'r' per
    device receive; pcap files hold one record per dequeue and receive of their device."""
    g = p2p.grid(4, 4, qmax=3, rate_bps=4_000_000, stop_ns=300_000_000, sim_stop_ns=400_000_000,
                 flows=[(0, 15), (1, 15), (4, 15), (5, 15)])
    st, devc, appc, _log, tr = run_trace(g)
    for kind, field in ((trace.TR_ENQUEUE, "enq_packets"), (trace.TR_DEQUEUE, "deq_packets"),
                        (trace.TR_DROP, "drop_packets"), (trace.TR_RX, "rx_packets")):
        got = np.bincount(tr["dev"][tr["kind"] == kind], minlength=len(g.dev))
        assert np.array_equal(got, devc[field]), field
    assert devc["drop_packets"].sum() > 0
    codec = trace.Codec(g)
    pc = codec.pcaps(tr)
    for d in range(len(g.dev)):
        f = pc[(codec.dev_node[d], codec.ifindex[d])]
        n = 0
        off = 24
        while off < len(f):
            ln = int.from_bytes(f[off + 8:off + 12], "little")
            off += 16 + ln
            n += 1
        assert n == devc["deq_packets"][d] + devc["rx_packets"][d]
    text = codec.ascii(tr)
    assert text.count("\n") == len(tr)
