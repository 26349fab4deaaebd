"""Ipv4L3Protocol Tx / Rx / Drop trace records in the oracle and the trace codec.

InternetStackHelper::EnableAsciiIpv4All hooks Ipv4L3Protocol's Tx (SendRealOut, ipv4-l3-protocol.cc:764),
Rx (Receive :455) and Drop (DROP_NO_ROUTE :505, DROP_TTL_EXPIRED :835) sources on every interface and
prints "<t|r|d> <seconds> /NodeList/<n>/$ns3::Ipv4L3Protocol/<Tx|Rx|Drop>(<interface>) <packet>"
(internet-stack-helper.cc:650-730 with INTERFACE_CONTEXT, :187).  The reference's test suites hold no
Ipv4 ascii trace fixture, so the known answers below are derived by hand from those call sites: the
line format is parity unpinned against a reference run; the GPU engine's records are checked against
this oracle bit for bit (tests/test_gpu_icmp.py, tests/test_gpu_trace.py)."""
import numpy as np
import pytest

import nsref
import p2p
import trace
from test_icmp_oracle import icmp_scenario, line

ALL = nsref.TRACE_DEVICE_KINDS | nsref.TRACE_IPV4_KINDS
FIELDS = ("ts", "uid", "kind", "dev", "app", "ipid", "size", "ttl")


def run(sc, kinds=ALL):
    s = sc.c_struct()
    st = p2p.P2PStats()
    devc = np.zeros(s.n_devices, p2p.DEV_COUNTERS_DTYPE)
    appc = np.zeros(s.n_apps, p2p.APP_COUNTERS_DTYPE)
    _secs, _log, tr = nsref.p2p_run_trace(s, st, devc, appc, 0, kinds=kinds)
    return st, trace.sort_records(tr)


def ipv4_lines(sc, tr):
    return [ln for ln in trace.Codec(sc).ascii(tr).splitlines() if "Ipv4L3Protocol" in ln]


UDP = ("ns3::Ipv4Header (tos 0x0 DSCP Default ECN Not-ECT ttl %d id 0 protocol 17 offset (bytes) 0 flags [none] "
       "length: 1052 %s) ns3::UdpHeader (length: 1032 %s) Payload (size=1024)")
TE = ("ns3::Ipv4Header (tos 0x0 DSCP Default ECN Not-ECT ttl 64 id 0 protocol 1 offset (bytes) 0 flags [none] "
      "length: 56 10.1.1.2 > 10.1.1.1) ns3::Icmpv4Header (type=11, code=0) ns3::Icmpv4TimeExceeded (tos 0x0 DSCP "
      "Default ECN Not-ECT ttl 0 id 0 protocol 17 offset (bytes) 0 flags [none] length: 1052 10.1.1.1 > 10.1.2.2 "
      "org data=192 1 0 9 4 8 0 0 )")


def test_time_exceeded_ipv4_lines():
    """TTL 1 through node 1: node 0 sends (Tx on interface 1), node 1 receives (Rx(1)), sends the time
    exceeded error back (Tx(1)) and then drops the request on its forwarding route's interface (Drop(2),
    the header as received, TTL 1); node 0 receives the error (Rx(1))."""
    sc = line(3, client_ttl=1)
    _st, tr = run(sc)
    assert ipv4_lines(sc, tr) == [
        "t 2 /NodeList/0/$ns3::Ipv4L3Protocol/Tx(1) " + UDP % (1, "10.1.1.1 > 10.1.2.2", "49153 > 9"),
        "r 2.00369 /NodeList/1/$ns3::Ipv4L3Protocol/Rx(1) " + UDP % (1, "10.1.1.1 > 10.1.2.2", "49153 > 9"),
        "t 2.00369 /NodeList/1/$ns3::Ipv4L3Protocol/Tx(1) " + TE,
        "d 2.00369 /NodeList/1/$ns3::Ipv4L3Protocol/Drop(2) " + UDP % (1, "10.1.1.1 > 10.1.2.2", "49153 > 9"),
        "r 2.00578 /NodeList/0/$ns3::Ipv4L3Protocol/Rx(1) " + TE]
    # inside node 1's Receive event: MacRx, Rx, the error's Tx, Enqueue, Dequeue, then the Drop
    ev = tr[tr["ts"] == tr["ts"][tr["kind"] == trace.TR_IP_DROP][0]]
    assert list(ev["kind"]) == [trace.TR_RX, trace.TR_IP_RX, trace.TR_IP_TX, trace.TR_ENQUEUE, trace.TR_DEQUEUE,
                                trace.TR_IP_DROP]
    assert list(ev["seq"]) == list(range(6))


def test_echo_round_trip_ipv4_lines():
    """A reply travels back: the server's Tx carries the reply's own header (TTL 64, server -> client),
    the forwarding node's Tx the decremented TTL."""
    sc = line(3, server=True)
    _st, tr = run(sc)
    lines = ipv4_lines(sc, tr)
    assert [ln.split(" ")[0] for ln in lines] == ["t", "r", "t", "r", "t", "r", "t", "r"]
    assert lines[2].startswith("t 2.00369 /NodeList/1/$ns3::Ipv4L3Protocol/Tx(2) ")
    assert UDP % (63, "10.1.1.1 > 10.1.2.2", "49153 > 9") in lines[2]
    assert lines[4].startswith("t 2.00737 /NodeList/2/$ns3::Ipv4L3Protocol/Tx(1) ")
    assert UDP % (64, "10.1.2.2 > 10.1.1.1", "9 > 49153") in lines[4]


def test_first_cc_ipv4_records_leave_the_device_stream_unchanged():
    """first.cc with both helpers on one stream: the device lines are the EnableAsciiAll file's (the md5
    pinned in tests/test_trace_oracle.py), the Ipv4 lines interleave in call order."""
    sc = p2p.first_cc()
    _st, dev_only = run(sc, nsref.TRACE_DEVICE_KINDS)
    _st, both = run(sc)
    codec = trace.Codec(sc)
    assert [ln for ln in codec.ascii(both).splitlines() if "Ipv4L3Protocol" not in ln] == \
        codec.ascii(dev_only).splitlines()
    assert [ln.split(" ")[0] + " " + ln.split(" ")[2] for ln in ipv4_lines(sc, both)] == [
        "t /NodeList/0/$ns3::Ipv4L3Protocol/Tx(1)", "r /NodeList/1/$ns3::Ipv4L3Protocol/Rx(1)",
        "t /NodeList/1/$ns3::Ipv4L3Protocol/Tx(1)", "r /NodeList/0/$ns3::Ipv4L3Protocol/Rx(1)"]
    assert codec.pcaps(both) == codec.pcaps(dev_only)


@pytest.mark.parametrize("seed,icmp", [(1, True), (2, True), (5, False)])
def test_ipv4_record_properties(seed, icmp):
    sc = icmp_scenario(seed, icmp)
    st, dev_only = run(sc, nsref.TRACE_DEVICE_KINDS)
    st2, tr = run(sc)
    assert st.digest == st2.digest
    k = tr["kind"]
    # the device records are the same calls, in the same order
    rest = tr[k < trace.TR_IP_TX]
    for f in FIELDS:
        assert np.array_equal(rest[f], dev_only[f]), f
    # every received frame reaches Ipv4L3Protocol::Receive; every Tx goes to the device's Send (enqueue or
    # queue drop) with the same descriptor
    assert (k == trace.TR_IP_RX).sum() == (k == trace.TR_RX).sum()
    assert (k == trace.TR_IP_TX).sum() == ((k == trace.TR_ENQUEUE) | (k == trace.TR_DROP)).sum()
    nxt = np.flatnonzero(k == trace.TR_IP_TX) + 1
    for f in ("dev", "app", "ipid", "ttl"):
        assert np.array_equal(tr[f][nxt], tr[f][nxt - 1]), f
    assert np.array_equal(tr["size"][nxt], tr["size"][nxt - 1] + 2)
    # drops: TTL expiries (TTL 1 as received) and forwarding without a route
    drops = tr[k == trace.TR_IP_DROP]
    assert st.ttl_drops <= len(drops) <= st.ttl_drops + st.no_route_drops
    assert st.ttl_drops > 0
    assert ((drops["ttl"] & 255) == 1).sum() == st.ttl_drops
    assert ((drops["app"] & trace.PKT_ICMP) != 0).sum() == 0 or icmp
    # a Drop is the last call of its event
    idx = np.flatnonzero(k == trace.TR_IP_DROP)
    last = (idx == len(tr) - 1) | (tr["uid"][np.minimum(idx + 1, len(tr) - 1)] != tr["uid"][idx]) | \
        (tr["ts"][np.minimum(idx + 1, len(tr) - 1)] != tr["ts"][idx])
    assert last.all()
    text = trace.Codec(sc).ascii(tr)
    assert text.count("$ns3::Ipv4L3Protocol/Drop(") == len(drops)
