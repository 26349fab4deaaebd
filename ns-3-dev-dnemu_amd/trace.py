"""Trace replay: ns-3 ascii and pcap trace files from nsgpu_trace_record streams.

The engines (the GPU p2p engine, and the oracle that checks it) record one nsgpu_trace_record per
call of a default ascii trace sink (include/nsgpu_types.h); this module turns the records into the
bytes ns-3 writes, host side and after the run:

  * ascii: AsciiTraceHelper::Default{Enqueue,Dequeue,Drop,Receive}SinkWithContext
    (src/network/helper/trace-helper.cc:303-390) as connected by PointToPointHelper::EnableAsciiInternal
    with a stream (src/point-to-point/helper/point-to-point-helper.cc:186-219, EnableAsciiAll (stream)):
    "<c> <Now ().GetSeconds ()> <context> <packet>" where the packet prints through its metadata
    (Packet::Print, src/network/model/packet.cc:427-476) as
    ns3::PppHeader (...) ns3::Ipv4Header (...) ns3::UdpHeader (...) Payload (size=N);
    PppHeader::Print (ppp-header.cc:57-72), Ipv4Header::Print (ipv4-header.cc:301-338, this fork's
    DSCP/ECN fields), UdpHeader::Print (udp-header.cc:156-162).
  * pcap: PcapHelper::CreateFile (DLT_PPP, snaplen 65535) + the PromiscSniffer sink
    (point-to-point-helper.cc:81-110): one file per device, PcapFileWrapper::Write (Time, Packet)
    (pcap-file-wrapper.cc:104-111: GetMicroSeconds () split into s / us), the serialized bytes
    PPP (2) + IPv4 (20, checksum 0: ChecksumEnabled is false) + UDP (8, checksum 0) + zero payload.

The packet descriptor of a record (flow, IPv4 identification, size, TTL) plus the scenario's
addressing (Scenario.dev_addr, application ports) determine every byte.  Pinned against the
reference's own first.cc output (tests/golden/survey_reference_runs.json: ascii and pcap md5s).
"""
import struct

import numpy as np

import p2p

TR_ENQUEUE, TR_DEQUEUE, TR_DROP, TR_RX = 0, 1, 2, 3
TR_IP_TX, TR_IP_RX, TR_IP_DROP = 4, 5, 6  # Ipv4L3Protocol Tx / Rx / Drop (InternetStackHelper::EnableAsciiIpv4)
_L3 = (TR_RX, TR_IP_TX, TR_IP_RX, TR_IP_DROP)  # records of the packet without its PppHeader
PKT_REPLY = 0x80000000
PKT_ICMP, PKT_ICMP_UNREACH, PKT_ICMP_OF_REPLY, PKT_APP = 0x40000000, 0x20000000, 0x10000000, 0x0FFFFFFF
TRACE_RECORD_DTYPE = p2p.TRACE_RECORD_DTYPE  # nsgpu_trace_record
_CHAR = {TR_ENQUEUE: "+", TR_DEQUEUE: "-", TR_DROP: "d", TR_RX: "r", TR_IP_TX: "t", TR_IP_RX: "r", TR_IP_DROP: "d"}
_SOURCE = {TR_ENQUEUE: "TxQueue/Enqueue", TR_DEQUEUE: "TxQueue/Dequeue", TR_DROP: "TxQueue/Drop", TR_RX: "MacRx",
           TR_IP_TX: "Tx", TR_IP_RX: "Rx", TR_IP_DROP: "Drop"}
PPP_HDR = 2


def dotted(a):
    return "%d.%d.%d.%d" % (a >> 24, (a >> 16) & 255, (a >> 8) & 255, a & 255)


def sort_records(tr):
    """Trace order: the pop order of the dispatching event (ts, uid), then call order inside it."""
    tr = np.asarray(tr, dtype=TRACE_RECORD_DTYPE)
    return tr[np.lexsort((tr["seq"], tr["uid"], tr["ts"]))]


# ---------------- pcap file format (PcapFile, src/network/utils/pcap-file.cc) ----------------
PCAP_MAGIC = 0xa1b2c3d4
DLT_EN10MB, DLT_PPP = 1, 9


def pcap_file_header(snaplen=65535, linktype=DLT_PPP, tz=0):
    """PcapFile::Init (pcap-file.cc:300-346): magic, version 2.4, thiszone, sigfigs 0, snaplen, network
    (native little-endian, no swap)."""
    return struct.pack("<IHHiIII", PCAP_MAGIC, 2, 4, tz, 0, snaplen, linktype)


def pcap_record(sec, usec, data, total_len=None, snaplen=65535):
    """PcapFile::WritePacketHeader + Write (pcap-file.cc:348-381): inclLen = min (totalLen, snapLen),
    origLen = totalLen, then the first inclLen bytes of the packet."""
    total = len(data) if total_len is None else total_len
    incl = min(total, snaplen)
    return struct.pack("<IIII", sec, usec, incl, total) + bytes(data[:incl])


def pcap_read(buf):
    """(file header fields, [(sec, usec, inclLen, origLen, data)]) of a native-endian pcap file."""
    magic, vmaj, vmin, tz, sig, snap, link = struct.unpack_from("<IHHiIII", buf, 0)
    assert magic == PCAP_MAGIC, hex(magic)
    recs, off = [], 24
    while off + 16 <= len(buf):
        sec, usec, incl, orig = struct.unpack_from("<IIII", buf, off)
        recs.append((sec, usec, incl, orig, bytes(buf[off + 16:off + 16 + incl])))
        off += 16 + incl
    return (vmaj, vmin, tz, sig, snap, link), recs


def pcap_diff(a, b, snaplen=65535):
    """PcapFile::Diff (pcap-file.cc:465-535): (differ, sec, usec) — the time of the first record whose
    timestamp, read length or data differ (reading at most snaplen bytes of each), or of the last record
    read when one file ends first."""
    _ha, ra = pcap_read(a)
    _hb, rb = pcap_read(b)
    sec = usec = 0
    for i in range(max(len(ra), len(rb))):
        if (i < len(ra)) != (i < len(rb)):
            return True, sec, usec
        s1, u1, _i1, _o1, d1 = ra[i]
        s2, u2, _i2, _o2, d2 = rb[i]
        sec, usec = s1, u1
        if (s1, u1) != (s2, u2) or d1[:snaplen] != d2[:snaplen]:
            return True, sec, usec
    return False, sec, usec


_M64 = (1 << 64) - 1


def _umul_by_invert(a, b):
    """int64x64_t::UmulByInvert (int64x64-128.cc:103-118): hi = ah * bh is NOT shifted back."""
    ah, al, bh, bl = a >> 64, a & _M64, b >> 64, b & _M64
    return (ah * bh + (((ah * bl + al * bh) & ((1 << 128) - 1)) >> 64)) & ((1 << 128) - 1)


def _invert(v):
    """int64x64_t::Invert (int64x64-128.cc:119-134) via Divu (:67-92)."""
    a = 1 << 64
    quo, rem = divmod(a, v)
    r = quo << 64
    if rem >> 64 == 0:
        r += (rem << 64) // v
    else:
        r += rem // (v >> 64)
    if _umul_by_invert(v << 64, r) >> 64 != 1:
        r += 1
    return r


_INV_1E9 = _invert(1_000_000_000)


def get_seconds(ts_ns):
    """Time::GetSeconds () at NS resolution: To (S) = int64x64_t (ts).MulByInvert (Invert (1e9)), then the
    two-rounding GetDouble (nstime.h:419-431, int64x64-128.cc:94-134, int64x64-128.h:83-95) — not ts / 1e9,
    which differs at half-way timestamps (840,877,500 ns: 0.8408774999999999 in ns-3)."""
    ts = int(ts_ns)
    v = _umul_by_invert(abs(ts) << 64, _INV_1E9)
    r = float(v >> 64) + float(v & _M64) / 18446744073709551615.0
    return -r if ts < 0 else r


def seconds_text(ts_ns):
    """std::ostream << double (precision 6, %g) of Time::GetSeconds ()."""
    return "%g" % get_seconds(ts_ns)


class Codec:
    """Addressing of a p2p.Scenario as ns-3 would print it: interface indices, addresses, ports."""

    def __init__(self, sc):
        self.sc = sc
        self.dev_node = [d[0] for d in sc.dev]
        # Node::AddDevice order fixes GetIfIndex: point-to-point devices and the loopback (setup list)
        self.ifindex = {}
        nxt = [0] * sc.n_nodes
        for kind, k in sc.setup:
            if kind == p2p.SETUP_DEVICE:
                n = sc.dev[k][0]
                self.ifindex[k] = nxt[n]
                nxt[n] += 1
            elif kind == p2p.SETUP_NOOP:  # LoopbackNetDevice
                nxt[k] += 1
        # ephemeral ports of the sender sockets: Ipv4EndPointDemux::AllocateEphemeralPort (49153, 49154, ...
        # per node, ipv4-end-point-demux.cc:350-370) in StartApplication order (start time, then app order)
        self.eport = {}
        per_node = {}
        order = sorted((a["start"], i) for i, a in enumerate(sc.apps) if a["kind"] in p2p.SENDERS)
        for _t, i in order:
            n = sc.apps[i]["node"]
            per_node[n] = per_node.get(n, 49152) + 1
            self.eport[i] = per_node[n]
        self.echo_server = {a["node"]: i for i, a in enumerate(sc.apps) if a["kind"] == p2p.APP_ECHO_SERVER}
        # an application without an explicit remote address targets its node's first interface
        self.first_addr = {}
        for d in sorted(self.ifindex, key=lambda d: self.ifindex[d]):
            self.first_addr.setdefault(self.dev_node[d], sc.dev_addr.get(d, 0))
        self.slot = sc.dst_slot

    def _out_addr(self, node, dst_node):
        d = int(self.sc.next_hop(node, self.slot[dst_node]))
        return self.sc.dev_addr.get(d, 0)

    def _walk(self, node, dst_node, hops):
        """The node a datagram from `node` towards `dst_node` reaches after `hops` hops."""
        for _ in range(hops):
            d = int(self.sc.next_hop(node, self.slot[dst_node]))
            node = self.dev_node[int(self.sc.dev[d][1])]
        return node

    def icmp_fields(self, r):
        """An ICMP error record (include/nsgpu_types.h NSGPU_PKT_ICMP): its own (src, dst) and the offending
        datagram's embedded IPv4 header (src, dst, sport, dport, ttl, id, length)."""
        a = int(r["app"])
        fa = a & PKT_APP
        of_reply = bool(a & PKT_ICMP_OF_REPLY)
        A = self.sc.apps[fa]
        osrc, odst, osp, odp = self.headers(fa | (PKT_REPLY if of_reply else 0))
        sender, dest = (A["dst"], A["node"]) if of_reply else (A["node"], A["dst"])
        if a & PKT_ICMP_UNREACH:  # LocalDeliver at the datagram's destination
            origin = dest
        else:  # IpForward where the TTL reached 0: the sender's TTL-th hop
            t0 = self.sc.apps[self.echo_server[sender]]["ttl"] if of_reply else A["ttl"]
            origin = self._walk(sender, dest, t0)
        own_src = self._out_addr(origin, sender)
        return own_src, osrc, (osrc, odst, osp, odp, (int(r["ttl"]) >> 8) & 255, int(r["ipid"]) >> 16,
                               int(r["ttl"]) >> 16)

    def headers(self, app_word):
        """(src, dst, sport, dport) of a datagram of flow app_word."""
        a = app_word & ~PKT_REPLY
        A = self.sc.apps[a]
        req_src = self._out_addr(A["node"], A["dst"])
        req_dst = A["remote_addr"] if A["remote_addr"] is not None else self.first_addr.get(A["dst"], 0)
        if app_word & PKT_REPLY:  # UdpEchoServer::HandleRead -> SendTo (packet, 0, from)
            return self._out_addr(A["dst"], A["node"]), req_src, A["remote_port"], self.eport[a]
        return req_src, req_dst, self.eport[a], A["remote_port"]

    # ---------------- ascii ----------------
    @staticmethod
    def _ipv4_text(ttl, ipid, proto, length, src, dst):
        """Ipv4Header::Print (ipv4-header.cc:301-338, this fork's DSCP/ECN fields)."""
        return ("tos 0x0 DSCP Default ECN Not-ECT ttl %d id %d protocol %d offset (bytes) 0 flags [none] length: %d "
                "%s > %s" % (ttl & 255, ipid & 0xffff, proto, length, dotted(src), dotted(dst)))

    def packet_text(self, r):
        if int(r["app"]) & PKT_ICMP:
            return self.icmp_text(r)
        src, dst, sp, dp = self.headers(int(r["app"]))
        ip_len = int(r["size"]) - (0 if r["kind"] in _L3 else PPP_HDR)
        parts = []
        if r["kind"] not in _L3:
            parts.append("ns3::PppHeader (Point-to-Point Protocol: IP (0x0021))")
        parts.append("ns3::Ipv4Header (tos 0x0 DSCP Default ECN Not-ECT ttl %d id %d protocol 17 offset (bytes) 0 "
                     "flags [none] length: %d %s > %s)" % (int(r["ttl"]) & 255, int(r["ipid"]) & 0xffff, ip_len,
                                                           dotted(src), dotted(dst)))
        parts.append("ns3::UdpHeader (length: %d %d > %d)" % (ip_len - 20, sp, dp))
        parts.append("Payload (size=%d)" % (ip_len - 28))
        return " ".join(parts)

    def icmp_text(self, r):
        """Icmpv4Header::Print + Icmpv4TimeExceeded / Icmpv4DestinationUnreachable::Print (icmpv4.cc:91-94,
        336-347, 435-446): the embedded header, then " org data=" and its 8 payload bytes, each followed
        by a space."""
        own_src, own_dst, (osrc, odst, osp, odp, ottl, oid, olen) = self.icmp_fields(r)
        ip_len = int(r["size"]) - (0 if r["kind"] in _L3 else PPP_HDR)
        unreach = bool(int(r["app"]) & PKT_ICMP_UNREACH)
        data = struct.pack(">HHHH", osp, odp, olen - 20, 0)
        parts = []
        if r["kind"] not in _L3:
            parts.append("ns3::PppHeader (Point-to-Point Protocol: IP (0x0021))")
        parts.append("ns3::Ipv4Header (%s)" % self._ipv4_text(int(r["ttl"]), int(r["ipid"]), 1, ip_len, own_src, own_dst))
        parts.append("ns3::Icmpv4Header (type=%d, code=%d)" % ((3, 3) if unreach else (11, 0)))
        parts.append("ns3::%s (%s org data=%s)" % (
            "Icmpv4DestinationUnreachable" if unreach else "Icmpv4TimeExceeded",
            self._ipv4_text(ottl, oid, 17, olen, osrc, odst), "".join("%d " % b for b in data)))
        return " ".join(parts)

    def ascii(self, tr):
        """The ascii file of a sorted record stream, as one string: PointToPointHelper::EnableAsciiAll
        (stream) lines for the device records and InternetStackHelper::EnableAsciiIpv4All (stream) lines
        (internet-stack-helper.cc:650-730, INTERFACE_CONTEXT: "<c> <s> /NodeList/<n>/$ns3::Ipv4L3Protocol/
        <Tx|Rx|Drop>(<interface>) <packet>", the packet from its Ipv4Header on) for the Ipv4 records, in
        record order (both helpers given one stream)."""
        out = []
        for r in tr:
            d = int(r["dev"])
            k = int(r["kind"])
            if k >= TR_IP_TX:
                ctx = "/NodeList/%d/$ns3::Ipv4L3Protocol/%s(%d)" % (self.dev_node[d], _SOURCE[k], self.sc.dev_ifindex[d])
            else:
                ctx = "/NodeList/%d/DeviceList/%d/$ns3::PointToPointNetDevice/%s" % (
                    self.dev_node[d], self.ifindex[d], _SOURCE[k])
            out.append("%s %s %s %s\n" % (_CHAR[int(r["kind"])], seconds_text(int(r["ts"])), ctx, self.packet_text(r)))
        return "".join(out)

    # ---------------- pcap ----------------
    def packet_bytes(self, r):
        """Serialized packet with its PPP header (what the sniffer sees)."""
        if int(r["app"]) & PKT_ICMP:  # IPv4 (protocol 1) + Icmpv4Header + TimeExceeded / DestinationUnreachable
            own_src, own_dst, (osrc, odst, osp, odp, ottl, oid, olen) = self.icmp_fields(r)
            ip_len = int(r["size"]) - (0 if r["kind"] in _L3 else PPP_HDR)
            unreach = bool(int(r["app"]) & PKT_ICMP_UNREACH)
            ipv4 = struct.pack(">BBHHHBBHII", 0x45, 0, ip_len, int(r["ipid"]) & 0xffff, 0, int(r["ttl"]) & 255, 1, 0,
                               own_src, own_dst)
            icmp = struct.pack(">BBH", *((3, 3, 0) if unreach else (11, 0, 0))) + bytes(4)  # unused / next-hop MTU 0
            org = struct.pack(">BBHHHBBHII", 0x45, 0, olen, oid & 0xffff, 0, ottl, 17, 0, osrc, odst)
            return struct.pack(">H", 0x0021) + ipv4 + icmp + org + struct.pack(">HHHH", osp, odp, olen - 20, 0)
        src, dst, sp, dp = self.headers(int(r["app"]))
        ip_len = int(r["size"]) - (0 if r["kind"] in _L3 else PPP_HDR)
        ipv4 = struct.pack(">BBHHHBBHII", 0x45, 0, ip_len, int(r["ipid"]) & 0xffff, 0, int(r["ttl"]) & 255, 17, 0,
                           src, dst)
        udp = struct.pack(">HHHH", sp, dp, ip_len - 20, 0)
        return struct.pack(">H", 0x0021) + ipv4 + udp + bytes(ip_len - 28)

    def pcaps(self, tr):
        """EnablePcapAll: {(node, ifindex): file bytes} for every point-to-point device."""
        files = {}
        for d in range(len(self.sc.dev)):
            files[(self.dev_node[d], self.ifindex[d])] = bytearray(pcap_file_header(65535, DLT_PPP))
        for r in tr:
            if r["kind"] not in (TR_DEQUEUE, TR_RX):  # the sniffer runs after Dequeue and before MacRx
                continue
            d = int(r["dev"])
            pkt = self.packet_bytes(r)
            us = int(r["ts"]) // 1000
            f = files[(self.dev_node[d], self.ifindex[d])]
            f += pcap_record(us // 1000000, us % 1000000, pkt)
        return {k: bytes(v) for k, v in files.items()}
