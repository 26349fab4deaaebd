"""ICMP errors in the oracle's p2p handler chain and the trace codec.

Ipv4L3Protocol::IpForward's TTL expiry sends Icmpv4L4Protocol::SendTimeExceededTtl and LocalDeliver's
RX_ENDPOINT_UNREACH sends SendDestUnreachPort (ipv4-l3-protocol.cc, icmpv4-l4-protocol.cc:131-160); the
56-byte error is routed back to the offending datagram's source like any IPv4 packet.  The reference's
test suites hold no ICMP fixture, so the known answers below are derived by hand from those call sites
and Icmpv4*::Print / Serialize (icmpv4.cc:91-94, 311-347, 405-446): parity unpinned against a reference
run; the GPU engine is checked against this oracle bit for bit (tests/test_gpu_icmp.py)."""
import re

import numpy as np
import pytest

import nsref
import p2p
import trace


def line(n, client_ttl=64, server=False, client_stop_ns=10_000_000_000):
    """n nodes in a line, 5 Mb/s / 2 ms links 10.1.(i+1).0/24, a one-shot UdpEchoClient 0 -> n-1."""
    sc = p2p.Scenario(n, icmp=True)
    links = [sc.link(i, i + 1, 5_000_000, 2_000_000) for i in range(n - 1)]
    sc.install_stack()
    for i, (a, b) in enumerate(links):
        sc.assign_link(a, b, p2p.ip("10.1.%d.0" % (i + 1)))
    if server:
        sc.add_echo_server(n - 1, 1_000_000_000, 20_000_000_000)
    sc.add_echo_client(0, n - 1, 2_000_000_000, client_stop_ns, count=1, ttl=client_ttl)
    sc.route_bfs()
    return sc


def run(sc, log_cap=0):
    s = sc.c_struct()
    st = p2p.P2PStats()
    devc = np.zeros(s.n_devices, p2p.DEV_COUNTERS_DTYPE)
    appc = np.zeros(s.n_apps, p2p.APP_COUNTERS_DTYPE)
    _secs, log, tr = nsref.p2p_run_trace(s, st, devc, appc, log_cap)
    return st, devc, appc, log, trace.sort_records(tr)


def icmp_lines(sc, tr):
    return [ln for ln in trace.Codec(sc).ascii(tr).splitlines() if "Icmpv4" in ln]


UDP_1052 = "protocol 17 offset (bytes) 0 flags [none] length: 1052"
IP = "ns3::Ipv4Header (tos 0x0 DSCP Default ECN Not-ECT ttl %d id %d protocol 1 offset (bytes) 0 flags [none] length: 56 %s)"
PPP = "ns3::PppHeader (Point-to-Point Protocol: IP (0x0021)) "


def test_time_exceeded_at_first_router():
    """TTL 1: node 1's IpForward drops the request and node 1 sends type 11 code 0 back to 10.1.1.1 from its
    interface on that route (10.1.1.2); it is enqueued at the request's arrival (2 s + 1054 B at 5 Mb/s + 2 ms)
    and received at node 0 one 58-byte frame time (92.8 us) + 2 ms later."""
    sc = line(3, client_ttl=1)
    st, _devc, _appc, _log, tr = run(sc)
    assert (st.ttl_drops, st.unreach_drops, st.icmp_sent) == (1, 0, 1)
    te = ("ns3::Icmpv4Header (type=11, code=0) ns3::Icmpv4TimeExceeded (tos 0x0 DSCP Default ECN Not-ECT ttl 0 id 0 "
          + UDP_1052 + " 10.1.1.1 > 10.1.2.2 org data=192 1 0 9 4 8 0 0 )")
    assert icmp_lines(sc, tr) == [
        "+ 2.00369 /NodeList/1/DeviceList/0/$ns3::PointToPointNetDevice/TxQueue/Enqueue " + PPP
        + IP % (64, 0, "10.1.1.2 > 10.1.1.1") + " " + te,
        "- 2.00369 /NodeList/1/DeviceList/0/$ns3::PointToPointNetDevice/TxQueue/Dequeue " + PPP
        + IP % (64, 0, "10.1.1.2 > 10.1.1.1") + " " + te,
        "r 2.00578 /NodeList/0/DeviceList/0/$ns3::PointToPointNetDevice/MacRx " + IP % (64, 0, "10.1.1.2 > 10.1.1.1")
        + " " + te]
    rx = tr[(tr["kind"] == trace.TR_RX) & ((tr["app"] & trace.PKT_ICMP) != 0)]
    # DataRate::CalculateTxTime's double 58 * 8 / 5e6 = 9.28e-05 s truncates to 92,799 ns in Seconds ()
    assert int(rx["ts"][0]) == 2_000_000_000 + 1_686_400 + 2_000_000 + 92_799 + 2_000_000
    # PPP 0x0021 | IPv4 (len 56, id 0, ttl 64, proto 1, csum 0) | type 11 code 0 csum 0, 4 unused | the
    # request's IPv4 header with TTL 0 | its first 8 bytes (UDP 49153 > 9, length 1032, checksum 0)
    assert trace.Codec(sc).packet_bytes(rx[0]).hex() == (
        "0021" "45000038" "00000000" "40010000" "0a010102" "0a010101" "0b000000" "00000000"
        "4500041c" "00000000" "00110000" "0a010101" "0a010202" "c0010009" "04080000")


def test_port_unreachable_at_destination():
    """No socket bound at node 2: LocalDeliver's RX_ENDPOINT_UNREACH sends type 3 code 3 (next-hop MTU 0)
    with the request's header as received (TTL 63), forwarded by node 1 (TTL 63 on the second link)."""
    sc = line(3)
    st, _devc, _appc, _log, tr = run(sc)
    assert (st.ttl_drops, st.unreach_drops, st.icmp_sent) == (0, 1, 1)
    du = ("ns3::Icmpv4Header (type=3, code=3) ns3::Icmpv4DestinationUnreachable (tos 0x0 DSCP Default ECN Not-ECT "
          "ttl 63 id 0 " + UDP_1052 + " 10.1.1.1 > 10.1.2.2 org data=192 1 0 9 4 8 0 0 )")
    lines = icmp_lines(sc, tr)
    assert [ln.split(" ")[:3] for ln in lines] == [
        ["+", "2.00737", "/NodeList/2/DeviceList/0/$ns3::PointToPointNetDevice/TxQueue/Enqueue"],
        ["-", "2.00737", "/NodeList/2/DeviceList/0/$ns3::PointToPointNetDevice/TxQueue/Dequeue"],
        ["r", "2.00947", "/NodeList/1/DeviceList/1/$ns3::PointToPointNetDevice/MacRx"],
        ["+", "2.00947", "/NodeList/1/DeviceList/0/$ns3::PointToPointNetDevice/TxQueue/Enqueue"],
        ["-", "2.00947", "/NodeList/1/DeviceList/0/$ns3::PointToPointNetDevice/TxQueue/Dequeue"],
        ["r", "2.01156", "/NodeList/0/DeviceList/0/$ns3::PointToPointNetDevice/MacRx"]]
    assert lines[0].endswith(PPP + IP % (64, 0, "10.1.2.2 > 10.1.1.1") + " " + du)
    assert lines[-1].endswith("MacRx " + IP % (63, 0, "10.1.2.2 > 10.1.1.1") + " " + du)
    e = tr[(tr["kind"] == trace.TR_ENQUEUE) & ((tr["app"] & trace.PKT_ICMP) != 0)][0]
    assert trace.Codec(sc).packet_bytes(e).hex() == (
        "0021" "45000038" "00000000" "40010000" "0a010202" "0a010101" "03030000" "00000000"
        "4500041c" "00000000" "3f110000" "0a010101" "0a010202" "c0010009" "04080000")


def test_echo_reply_to_a_stopped_client():
    """The client stops before its reply returns: the reply finds no endpoint at node 0, which sends the port
    unreachable back to the server (10.1.2.2) with its own second IPv4 identification (id 1)."""
    sc = line(3, server=True, client_stop_ns=2_001_000_000)
    st, _devc, appc, _log, tr = run(sc)
    assert (st.unreach_drops, st.icmp_sent) == (1, 1)
    assert appc["rx_packets"].sum() == 1  # the server's
    lines = icmp_lines(sc, tr)
    assert lines[0].startswith("+ 2.01475 /NodeList/0/DeviceList/0/")
    assert lines[0].endswith(PPP + IP % (64, 1, "10.1.1.1 > 10.1.2.2") + " ns3::Icmpv4Header (type=3, code=3) "
                             "ns3::Icmpv4DestinationUnreachable (tos 0x0 DSCP Default ECN Not-ECT ttl 63 id 0 "
                             + UDP_1052 + " 10.1.2.2 > 10.1.1.1 org data=0 9 192 1 4 8 0 0 )")
    assert lines[-1].startswith("r 2.01893 /NodeList/2/DeviceList/0/")


def test_echo_reply_time_exceeded_after_64_hops():
    """A 70-node line: the request (TTL 255) reaches the server, whose reply leaves with the default TTL 64
    and expires at its 64th forwarder, node 5, which sends type 11 from 10.1.6.1 to the server."""
    sc = line(70, client_ttl=255, server=True)
    st, _devc, _appc, _log, tr = run(sc)
    assert (st.ttl_drops, st.icmp_sent) == (1, 1)
    lines = icmp_lines(sc, tr)
    assert lines[0].startswith("+ 2.49029 /NodeList/5/DeviceList/1/")
    assert IP % (64, 0, "10.1.6.1 > 10.1.69.2") in lines[0]
    assert "ttl 0 id 0 " + UDP_1052 + " 10.1.69.2 > 10.1.1.1 org data=0 9 192 1 4 8 0 0 )" in lines[0]
    assert lines[-1].startswith("r 2.62423 /NodeList/69/DeviceList/0/")
    assert IP % (1, 0, "10.1.6.1 > 10.1.69.2") in lines[-1]


def icmp_scenario(seed, icmp=True):
    return p2p.random_topology(30, 60, 10, seed, ttl=3, icmp=icmp, sink_window=(150_000_000, 600_000_000))


@pytest.mark.parametrize("seed", range(3))
def test_random_topologies_icmp_properties(seed):
    """Every non-ICMP TTL expiry and unbound arrival sends exactly one error (ICMP packets carry TTL 64 and
    never expire here, and an error reaching its destination is consumed); each error's destination is the
    embedded datagram's source, a time exceeded embeds TTL 0, a port unreachable a positive one; and the
    errors' frames are 58 bytes with IPv4 protocol 1."""
    sc = icmp_scenario(seed)
    st, _devc, _appc, _log, tr = run(sc)
    assert st.icmp_sent > 0 and st.icmp_sent == st.ttl_drops + st.unreach_drops
    codec = trace.Codec(sc)
    pat = re.compile(r"length: 56 (\S+) > (\S+)\) ns3::Icmpv4Header \(type=(\d+), code=(\d+)\) ns3::Icmpv4(\w+) "
                     r"\(tos 0x0 DSCP Default ECN Not-ECT ttl (\d+) id \d+ protocol 17 offset \(bytes\) 0 flags "
                     r"\[none\] length: \d+ (\S+) > (\S+) org data=(\d+ ){8}\)$")
    icmp = tr[(tr["app"] & trace.PKT_ICMP) != 0]
    assert len(icmp) > 0
    for ln in icmp_lines(sc, tr):
        m = pat.search(ln)
        assert m, ln
        _src, dst, typ, code, name, ottl, osrc, _odst, _ = m.groups()
        assert dst == osrc
        if name == "TimeExceeded":
            assert (typ, code, ottl) == ("11", "0", "0")
        else:
            assert (name, typ, code) == ("DestinationUnreachable", "3", "3") and int(ottl) > 0
    for r in icmp[:200]:
        b = codec.packet_bytes(r)
        assert len(b) == 58 and b[2 + 9] == 1 and int(r["size"]) == (56 if r["kind"] == trace.TR_RX else 58)
    off = run(icmp_scenario(seed, icmp=False))[0]
    assert off.icmp_sent == 0 and (off.ttl_drops, off.unreach_drops) != (0, 0)


def test_icmp_pcap_round_trip():
    sc = icmp_scenario(0)
    tr = run(sc)[4]
    pcs = trace.Codec(sc).pcaps(tr)
    n_icmp = 0
    for blob in pcs.values():
        _hdr, recs = trace.pcap_read(blob)
        n_icmp += sum(1 for *_t, data in recs if data[2 + 9] == 1)
    # the sniffer sees every ICMP frame at PhyTxBegin (after Dequeue) and before MacRx
    is_icmp = (tr["app"] & trace.PKT_ICMP) != 0
    assert n_icmp == int((is_icmp & ((tr["kind"] == trace.TR_DEQUEUE) | (tr["kind"] == trace.TR_RX))).sum()) > 0
