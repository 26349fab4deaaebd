// nsgpu_trace.cc — the trace codec of the GPU-resident p2p subset, in the product library: nsgpu_trace_record
// streams (one record per call of a default trace sink, include/nsgpu_types.h) -> the bytes ns-3's default
// sinks write.  Host code (the records are small and written once per run); C-ABI in include/nsgpu.h.
//
//   ascii  AsciiTraceHelper::Default{Enqueue,Dequeue,Drop,Receive}SinkWithContext
//          (src/network/helper/trace-helper.cc:303-390) as PointToPointHelper::EnableAsciiInternal connects
//          them (src/point-to-point/helper/point-to-point-helper.cc:186-219): "<c> <Now ().GetSeconds ()>
//          <context> <packet>", the packet printed through its metadata (Packet::Print,
//          src/network/model/packet.cc:427-476): PppHeader::Print (ppp-header.cc:57-72), Ipv4Header::Print
//          (ipv4-header.cc:301-338, this fork's DSCP / ECN fields), UdpHeader::Print (udp-header.cc:156-162),
//          Icmpv4Header / Icmpv4TimeExceeded / Icmpv4DestinationUnreachable::Print (icmpv4.cc:91-94,
//          336-347, 435-446); Ipv4L3Protocol Tx / Rx / Drop lines as InternetStackHelper::EnableAsciiIpv4
//          Internal connects them (internet-stack-helper.cc:650-730).
//   pcap   PcapHelper::CreateFile (DLT_PPP, snaplen 65535; pcap-file.cc:300-346) + the PromiscSniffer sink
//          (point-to-point-helper.cc:81-110): PcapFileWrapper::Write (Time, Packet) (pcap-file-wrapper.cc:
//          104-111: GetMicroSeconds () split into s / us; pcap-file.cc:348-381), the serialized packet PPP (2)
//          + IPv4 (20, checksum 0: ChecksumEnabled is false) + UDP (8, checksum 0) + zero payload, or the ICMP
//          error (IPv4 protocol 1, the Icmpv4Header, 4 unused bytes, the offending IPv4 header and 8 bytes).
//
// Every byte follows from the record's packet descriptor (flow, IPv4 identification, size, TTL), the
// scenario (devices, routes, applications) and its addressing (nsgpu_trace_addressing).  Pinned by the
// reference's first.cc md5s and known.pcap (tests/test_trace_codec_cpu.py).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <new>
#include <string>
#include <vector>

#include "nsgpu.h"

namespace nsgpu {
int set_error(int code, const char *fmt, ...);
}
using nsgpu::set_error;

struct nsgpu_trace_codec {
  uint32_t n_nodes = 0, n_devices = 0, n_apps = 0, n_dst = 0;
  std::vector<uint32_t> dev_node, dev_peer, dev_addr, dev_ipif, ifindex;
  std::vector<uint32_t> route, route_def, route_exc_slot, route_exc_dev;
  std::vector<uint64_t> route_exc_off;
  std::vector<uint32_t> app_kind, app_node, app_dst, app_dst_slot, app_src_slot, app_ttl, app_raddr, app_rport;
  std::vector<uint32_t> eport, first_addr;
  std::vector<int32_t> echo_server;  // per node: its UdpEchoServer application (the last one), -1: none

  uint32_t next_hop(uint32_t n, uint32_t slot) const {
    if (!route.empty()) return route[(uint64_t)n * n_dst + slot];
    const uint64_t lo = route_exc_off[n], hi = route_exc_off[n + 1];
    const auto b = route_exc_slot.begin();
    const auto it = std::lower_bound(b + lo, b + hi, slot);
    if (it != b + hi && *it == slot) return route_exc_dev[it - b];
    return route_def[n];
  }
  uint32_t out_addr(uint32_t node, uint32_t slot) const {  // the address of the route's output interface
    if (slot == 0xffffffffu) return 0;
    const uint32_t d = next_hop(node, slot);
    return d < n_devices ? dev_addr[d] : 0;
  }
};

namespace {

constexpr uint32_t PPP = 2;
const char *const kChar[7] = {"+", "-", "d", "r", "t", "r", "d"};
const char *const kSource[7] = {"TxQueue/Enqueue", "TxQueue/Dequeue", "TxQueue/Drop", "MacRx", "Tx", "Rx", "Drop"};

bool l3_record(uint32_t k) {  // records of the packet without its PppHeader (MacRx, Ipv4 sinks)
  return k == NSGPU_TR_RX || k == NSGPU_TR_IP_TX || k == NSGPU_TR_IP_RX || k == NSGPU_TR_IP_DROP;
}

struct Hdr {
  uint32_t src, dst, sport, dport;
};

// (src, dst, sport, dport) of a datagram of flow `word` (| NSGPU_PKT_REPLY: UdpEchoServer::HandleRead ->
// SendTo (packet, 0, from), back to the client's ephemeral port)
Hdr headers(const nsgpu_trace_codec &c, uint32_t word) {
  const uint32_t a = word & NSGPU_PKT_APP;
  const uint32_t req_src = c.out_addr(c.app_node[a], c.app_dst_slot[a]);
  const uint32_t req_dst = c.app_raddr[a] ? c.app_raddr[a] : c.first_addr[c.app_dst[a]];
  if (word & NSGPU_PKT_REPLY) return Hdr{c.out_addr(c.app_dst[a], c.app_src_slot[a]), req_src, c.app_rport[a], c.eport[a]};
  return Hdr{req_src, req_dst, c.eport[a], c.app_rport[a]};
}

struct IcmpF {
  uint32_t own_src, own_dst;
  uint32_t osrc, odst, osp, odp, ottl, oid, olen;
};

// An ICMP error record: its own (src, dst) and the offending datagram's embedded header.
IcmpF icmp_fields(const nsgpu_trace_codec &c, const nsgpu_trace_record &r) {
  const uint32_t a = r.app;
  const uint32_t fa = a & NSGPU_PKT_APP;
  const bool of_reply = (a & NSGPU_PKT_ICMP_OF_REPLY) != 0;
  const Hdr h = headers(c, fa | (of_reply ? NSGPU_PKT_REPLY : 0u));
  const uint32_t sender = of_reply ? c.app_dst[fa] : c.app_node[fa];
  const uint32_t dest_slot = of_reply ? c.app_src_slot[fa] : c.app_dst_slot[fa];
  const uint32_t sender_slot = of_reply ? c.app_dst_slot[fa] : c.app_src_slot[fa];
  uint32_t origin;
  if (a & NSGPU_PKT_ICMP_UNREACH) {  // LocalDeliver at the datagram's destination
    origin = of_reply ? c.app_node[fa] : c.app_dst[fa];
  } else {  // IpForward where the TTL reached 0: the sender's TTL-th hop
    uint32_t t0 = c.app_ttl[fa];
    if (of_reply) {
      const int32_t es = c.echo_server[sender];
      t0 = es >= 0 ? c.app_ttl[es] : 0;
    }
    origin = sender;
    for (uint32_t k = 0; k < t0; k++) origin = c.dev_node[c.dev_peer[c.next_hop(origin, dest_slot)]];
  }
  IcmpF f;
  f.own_src = c.out_addr(origin, sender_slot);
  f.own_dst = h.src;
  f.osrc = h.src, f.odst = h.dst, f.osp = h.sport, f.odp = h.dport;
  f.ottl = (r.ttl >> 8) & 255, f.oid = r.ipid >> 16, f.olen = r.ttl >> 16;
  return f;
}

// Time::GetSeconds () at the default NS resolution, as ns-3 computes it (not ts / 1e9): ToDouble (S) = To (S)
// .GetDouble () (nstime.h:419-431); To (S) with toMul false is int64x64_t (ts).MulByInvert (Invert (1e9))
// (int64x64-128.cc:94-134), then the two-rounding GetDouble (int64x64-128.h:83-95).  ts / 1e9 differs at
// half-way timestamps: 840,877,500 ns is 0.8408774999999999 here and prints 0.840877, not 0.840878.
typedef unsigned __int128 u128;
u128 divu128(u128 a, u128 b) {  // int64x64_t::Divu (int64x64-128.cc:67-92)
  u128 quo = a / b, rem = a % b;
  u128 result = quo << 64;
  u128 div;
  if ((rem >> 64) == 0) {
    rem <<= 64;
    div = b;
  } else {
    div = b >> 64;
  }
  return result + rem / div;
}
u128 umul_by_invert(u128 a, u128 b) {  // int64x64_t::UmulByInvert (int64x64-128.cc:103-118)
  const u128 lo = ~(u128)0 >> 64;
  const u128 ah = a >> 64, bh = b >> 64, al = a & lo, bl = b & lo;
  return ah * bh + ((ah * bl + al * bh) >> 64);
}
u128 invert_1e9() {  // int64x64_t::Invert (1e9) (int64x64-128.cc:119-134)
  const uint64_t v = 1000000000ULL;
  u128 r = divu128((u128)1 << 64, v);
  const u128 t = umul_by_invert((u128)v << 64, r);
  if ((uint64_t)(t >> 64) != 1) r += 1;
  return r;
}
}  // namespace

extern "C" double nsgpu_time_get_seconds(int64_t ts) {
  static const u128 inv = invert_1e9();
  const bool neg = ts < 0;
  const u128 a = (u128)(neg ? -(__int128)ts : (__int128)ts) << 64;
  const u128 v = umul_by_invert(a, inv);  // MulByInvert: the magnitude, sign restored below
  const uint64_t hi = (uint64_t)(v >> 64), lo = (uint64_t)v;
  double flo = (double)lo;
  flo /= 18446744073709551615.0;  // HP128_MAX_64
  double r = (double)hi;
  r += flo;
  return neg ? -r : r;
}

namespace {

void dotted(std::string &o, uint32_t a) {
  char b[20];
  std::snprintf(b, sizeof b, "%u.%u.%u.%u", a >> 24, (a >> 16) & 255, (a >> 8) & 255, a & 255);
  o += b;
}

void ipv4_text(std::string &o, uint32_t ttl, uint32_t ipid, uint32_t proto, uint32_t len, uint32_t src, uint32_t dst) {
  char b[160];
  std::snprintf(b, sizeof b,
                "tos 0x0 DSCP Default ECN Not-ECT ttl %u id %u protocol %u offset (bytes) 0 flags [none] length: %u ",
                ttl & 255, ipid & 0xffff, proto, len);
  o += b;
  dotted(o, src);
  o += " > ";
  dotted(o, dst);
}

void packet_text(const nsgpu_trace_codec &c, const nsgpu_trace_record &r, std::string &o) {
  const uint32_t ip_len = r.size - (l3_record(r.kind) ? 0 : PPP);
  if (!l3_record(r.kind)) o += "ns3::PppHeader (Point-to-Point Protocol: IP (0x0021)) ";
  char b[96];
  if (r.app & NSGPU_PKT_ICMP) {
    const IcmpF f = icmp_fields(c, r);
    const bool unreach = (r.app & NSGPU_PKT_ICMP_UNREACH) != 0;
    o += "ns3::Ipv4Header (";
    ipv4_text(o, r.ttl, r.ipid, 1, ip_len, f.own_src, f.own_dst);
    std::snprintf(b, sizeof b, ") ns3::Icmpv4Header (type=%d, code=%d) ns3::%s (", unreach ? 3 : 11, unreach ? 3 : 0,
                  unreach ? "Icmpv4DestinationUnreachable" : "Icmpv4TimeExceeded");
    o += b;
    ipv4_text(o, f.ottl, f.oid, 17, f.olen, f.osrc, f.odst);
    const uint8_t data[8] = {(uint8_t)(f.osp >> 8), (uint8_t)f.osp, (uint8_t)(f.odp >> 8), (uint8_t)f.odp,
                             (uint8_t)((f.olen - 20) >> 8), (uint8_t)(f.olen - 20), 0, 0};
    o += " org data=";
    for (uint8_t x : data) {
      std::snprintf(b, sizeof b, "%u ", (unsigned)x);
      o += b;
    }
    o += ")";
    return;
  }
  const Hdr h = headers(c, r.app);
  o += "ns3::Ipv4Header (";
  ipv4_text(o, r.ttl, r.ipid, 17, ip_len, h.src, h.dst);
  std::snprintf(b, sizeof b, ") ns3::UdpHeader (length: %u %u > %u) Payload (size=%u)", ip_len - 20, h.sport, h.dport,
                ip_len - 28);
  o += b;
}

void line(const nsgpu_trace_codec &c, const nsgpu_trace_record &r, std::string &o) {
  const uint32_t k = r.kind, d = r.dev;
  char b[128];
  o += kChar[k];
  std::snprintf(b, sizeof b, " %g ", nsgpu_time_get_seconds(r.ts));  // std::ostream << double: precision 6, %g
  o += b;
  if (k >= NSGPU_TR_IP_TX)
    std::snprintf(b, sizeof b, "/NodeList/%u/$ns3::Ipv4L3Protocol/%s(%u) ", c.dev_node[d], kSource[k], c.dev_ipif[d]);
  else
    std::snprintf(b, sizeof b, "/NodeList/%u/DeviceList/%u/$ns3::PointToPointNetDevice/%s ", c.dev_node[d],
                  c.ifindex[d], kSource[k]);
  o += b;
  packet_text(c, r, o);
  o += "\n";
}

inline void be16(std::vector<uint8_t> &o, uint32_t v) {
  o.push_back((uint8_t)(v >> 8));
  o.push_back((uint8_t)v);
}
inline void be32(std::vector<uint8_t> &o, uint32_t v) {
  be16(o, v >> 16);
  be16(o, v & 0xffff);
}
inline void le32(std::vector<uint8_t> &o, uint32_t v) {
  for (int i = 0; i < 4; i++) o.push_back((uint8_t)(v >> (8 * i)));
}
void ipv4_bytes(std::vector<uint8_t> &o, uint32_t len, uint32_t ipid, uint32_t ttl, uint32_t proto, uint32_t src,
                uint32_t dst) {
  o.push_back(0x45);
  o.push_back(0);
  be16(o, len);
  be16(o, ipid & 0xffff);
  be16(o, 0);
  o.push_back((uint8_t)(ttl & 255));
  o.push_back((uint8_t)proto);
  be16(o, 0);
  be32(o, src);
  be32(o, dst);
}

// The serialized packet with its PPP header (what the PromiscSniffer sees).
void packet_bytes(const nsgpu_trace_codec &c, const nsgpu_trace_record &r, std::vector<uint8_t> &o) {
  const uint32_t ip_len = r.size - (l3_record(r.kind) ? 0 : PPP);
  be16(o, 0x0021);
  if (r.app & NSGPU_PKT_ICMP) {
    const IcmpF f = icmp_fields(c, r);
    const bool unreach = (r.app & NSGPU_PKT_ICMP_UNREACH) != 0;
    ipv4_bytes(o, ip_len, r.ipid, r.ttl, 1, f.own_src, f.own_dst);
    o.push_back(unreach ? 3 : 11);
    o.push_back(unreach ? 3 : 0);
    be16(o, 0);
    be32(o, 0);  // unused / next-hop MTU 0
    ipv4_bytes(o, f.olen, f.oid, f.ottl, 17, f.osrc, f.odst);
    be16(o, f.osp);
    be16(o, f.odp);
    be16(o, f.olen - 20);
    be16(o, 0);
    return;
  }
  const Hdr h = headers(c, r.app);
  ipv4_bytes(o, ip_len, r.ipid, r.ttl, 17, h.src, h.dst);
  be16(o, h.sport);
  be16(o, h.dport);
  be16(o, ip_len - 20);
  be16(o, 0);
  o.insert(o.end(), ip_len - 28, 0);
}

bool record_ok(const nsgpu_trace_codec &c, const nsgpu_trace_record &r) {
  if (r.kind > NSGPU_TR_IP_DROP || r.dev >= c.n_devices) return false;
  if ((r.app & NSGPU_PKT_APP) >= c.n_apps) return false;
  const uint32_t ip_len = r.size - (l3_record(r.kind) ? 0 : PPP);
  return r.size >= (l3_record(r.kind) ? 0 : PPP) && ip_len >= 28u;
}

// PcapFile::Init (pcap-file.cc:300-346): magic, version 2.4, thiszone 0, sigfigs 0, snaplen, network
// (native little-endian, no swap)
void pcap_header(std::vector<uint8_t> &o, uint32_t linktype, uint32_t snaplen) {
  le32(o, 0xa1b2c3d4u);
  o.push_back(2), o.push_back(0), o.push_back(4), o.push_back(0);
  le32(o, 0), le32(o, 0), le32(o, snaplen), le32(o, linktype);
}
// PcapFile::WritePacketHeader + Write (pcap-file.cc:348-381): inclLen = min (totalLen, snapLen), origLen =
// totalLen, then the first inclLen bytes of the data
void pcap_rec(std::vector<uint8_t> &o, uint32_t sec, uint32_t usec, const uint8_t *data, uint32_t len, uint32_t orig,
              uint32_t snaplen) {
  const uint32_t incl = std::min(std::min(orig, snaplen), len);
  le32(o, sec), le32(o, usec), le32(o, incl), le32(o, orig);
  o.insert(o.end(), data, data + incl);
}

int copy_out(const void *src, uint64_t n, void *out, uint64_t cap, uint64_t *len) {
  *len = n;
  if (!out) return NSGPU_OK;  // (a size query)
  if (cap < n) return set_error(NSGPU_EINVAL, "nsgpu_trace: output buffer of %llu bytes, %llu needed",
                                (unsigned long long)cap, (unsigned long long)n);
  if (n) std::memcpy(out, src, n);
  return NSGPU_OK;
}

}  // namespace

extern "C" {

int nsgpu_trace_codec_create(const nsgpu_p2p_scenario *sc, const nsgpu_trace_addressing *ad, nsgpu_trace_codec **out) {
  if (!sc || !ad || !out) return set_error(NSGPU_EINVAL, "nsgpu_trace_codec_create: null");
  if (!sc->dev_node || !sc->dev_peer || !ad->dev_addr || !ad->dev_ip_ifindex || (sc->n_apps && (!ad->app_remote_addr ||
      !ad->app_remote_port || !sc->app_kind || !sc->app_node || !sc->app_dst_node || !sc->app_dst_slot || !sc->app_ttl ||
      !sc->app_start_ns)) || (sc->n_setup && (!sc->setup_kind || !sc->setup_index)))
    return set_error(NSGPU_EINVAL, "nsgpu_trace_codec_create: missing scenario / addressing arrays");
  if (!sc->route && !(sc->route_default && sc->route_exc_off && sc->route_exc_slot && sc->route_exc_dev))
    return set_error(NSGPU_EINVAL, "nsgpu_trace_codec_create: no route table");
  nsgpu_trace_codec *c = new (std::nothrow) nsgpu_trace_codec();
  if (!c) return set_error(NSGPU_ENOMEM, "nsgpu_trace_codec_create: out of memory");
  const uint32_t N = sc->n_nodes, D = sc->n_devices, A = sc->n_apps;
  c->n_nodes = N, c->n_devices = D, c->n_apps = A, c->n_dst = sc->n_dst;
  c->dev_node.assign(sc->dev_node, sc->dev_node + D);
  c->dev_peer.assign(sc->dev_peer, sc->dev_peer + D);
  c->dev_addr.assign(ad->dev_addr, ad->dev_addr + D);
  c->dev_ipif.assign(ad->dev_ip_ifindex, ad->dev_ip_ifindex + D);
  if (sc->route) {
    c->route.assign(sc->route, sc->route + (uint64_t)N * sc->n_dst);
  } else {
    c->route_def.assign(sc->route_default, sc->route_default + N);
    c->route_exc_off.assign(sc->route_exc_off, sc->route_exc_off + N + 1);
    const uint64_t ne = sc->route_exc_off[N];
    c->route_exc_slot.assign(sc->route_exc_slot, sc->route_exc_slot + ne);
    c->route_exc_dev.assign(sc->route_exc_dev, sc->route_exc_dev + ne);
  }
  for (uint32_t d = 0; d < D; d++)
    if (c->dev_node[d] >= N || c->dev_peer[d] >= D) {
      delete c;
      return set_error(NSGPU_EINVAL, "nsgpu_trace_codec_create: device %u names a node / peer out of range", d);
    }
  if (A) {
    c->app_kind.assign(sc->app_kind, sc->app_kind + A);
    c->app_node.assign(sc->app_node, sc->app_node + A);
    c->app_dst.assign(sc->app_dst_node, sc->app_dst_node + A);
    c->app_dst_slot.assign(sc->app_dst_slot, sc->app_dst_slot + A);
    c->app_ttl.assign(sc->app_ttl, sc->app_ttl + A);
    c->app_raddr.assign(ad->app_remote_addr, ad->app_remote_addr + A);
    c->app_rport.assign(ad->app_remote_port, ad->app_remote_port + A);
    c->app_src_slot.assign(A, 0xffffffffu);
    if (sc->app_src_slot) c->app_src_slot.assign(sc->app_src_slot, sc->app_src_slot + A);
  }
  for (uint32_t a = 0; a < A; a++)
    if (c->app_node[a] >= N || ((c->app_kind[a] == NSGPU_APP_ONOFF || c->app_kind[a] == NSGPU_APP_ECHO_CLIENT) &&
                                c->app_dst[a] >= N)) {
      delete c;
      return set_error(NSGPU_EINVAL, "nsgpu_trace_codec_create: application %u names a node out of range", a);
    }
  // Node::AddDevice order fixes GetIfIndex: the point-to-point devices and each node's LoopbackNetDevice
  // (NSGPU_SETUP_NOOP), in the setup list's order
  c->ifindex.assign(D, 0);
  std::vector<uint32_t> nxt(N, 0);
  for (uint32_t i = 0; i < sc->n_setup; i++) {
    const uint32_t k = sc->setup_index[i];
    if (sc->setup_kind[i] == NSGPU_SETUP_DEVICE && k < D) c->ifindex[k] = nxt[c->dev_node[k]]++;
    else if (sc->setup_kind[i] == NSGPU_SETUP_NOOP && k < N) nxt[k]++;
  }
  // the sender sockets' ephemeral ports: Ipv4EndPointDemux::AllocateEphemeralPort (49153, 49154, ... per node,
  // ipv4-end-point-demux.cc:350-370) in StartApplication order (start time, then application order)
  c->eport.assign(A, 0);
  std::vector<std::pair<int64_t, uint32_t>> order;
  for (uint32_t a = 0; a < A; a++)
    if (c->app_kind[a] == NSGPU_APP_ONOFF || c->app_kind[a] == NSGPU_APP_ECHO_CLIENT) order.push_back({sc->app_start_ns[a], a});
  std::sort(order.begin(), order.end());
  std::vector<uint32_t> port(N, 49152);
  for (const auto &o : order) c->eport[o.second] = ++port[c->app_node[o.second]];
  c->echo_server.assign(N, -1);
  for (uint32_t a = 0; a < A; a++)
    if (c->app_kind[a] == NSGPU_APP_ECHO_SERVER) c->echo_server[c->app_node[a]] = (int32_t)a;
  // an application without an explicit remote address targets its destination's first interface
  c->first_addr.assign(N, 0);
  std::vector<uint32_t> best(N, 0xffffffffu);
  for (uint32_t d = 0; d < D; d++) {
    const uint32_t n = c->dev_node[d];
    if (c->ifindex[d] < best[n]) {
      best[n] = c->ifindex[d];
      c->first_addr[n] = c->dev_addr[d];
    }
  }
  *out = c;
  return NSGPU_OK;
}

int nsgpu_trace_codec_free(nsgpu_trace_codec *c) {
  delete c;
  return NSGPU_OK;
}

int nsgpu_trace_sort(nsgpu_trace_record *rec, uint64_t n) {
  if (!rec && n) return set_error(NSGPU_EINVAL, "nsgpu_trace_sort: null");
  std::stable_sort(rec, rec + n, [](const nsgpu_trace_record &a, const nsgpu_trace_record &b) {
    if (a.ts != b.ts) return a.ts < b.ts;
    if (a.uid != b.uid) return a.uid < b.uid;
    return a.seq < b.seq;
  });
  return NSGPU_OK;
}

int nsgpu_trace_line(const nsgpu_trace_codec *c, const nsgpu_trace_record *r, char *out, uint64_t cap, uint64_t *len) {
  if (!c || !r || !len) return set_error(NSGPU_EINVAL, "nsgpu_trace_line: null");
  if (!record_ok(*c, *r)) return set_error(NSGPU_EINVAL, "nsgpu_trace_line: malformed record");
  std::string o;
  line(*c, *r, o);
  return copy_out(o.data(), o.size(), out, cap, len);
}

int nsgpu_trace_packet(const nsgpu_trace_codec *c, const nsgpu_trace_record *r, uint8_t *out, uint64_t cap,
                       uint64_t *len) {
  if (!c || !r || !len) return set_error(NSGPU_EINVAL, "nsgpu_trace_packet: null");
  if (!record_ok(*c, *r)) return set_error(NSGPU_EINVAL, "nsgpu_trace_packet: malformed record");
  std::vector<uint8_t> o;
  packet_bytes(*c, *r, o);
  return copy_out(o.data(), o.size(), out, cap, len);
}

int nsgpu_trace_ascii(const nsgpu_trace_codec *c, const nsgpu_trace_record *rec, uint64_t n, char *out, uint64_t cap,
                      uint64_t *len) {
  if (!c || (!rec && n) || !len) return set_error(NSGPU_EINVAL, "nsgpu_trace_ascii: null");
  std::string o;
  o.reserve(n * 200);
  for (uint64_t i = 0; i < n; i++) {
    if (!record_ok(*c, rec[i])) return set_error(NSGPU_EINVAL, "nsgpu_trace_ascii: record %llu is malformed", (unsigned long long)i);
    line(*c, rec[i], o);
  }
  return copy_out(o.data(), o.size(), out, cap, len);
}

int nsgpu_trace_pcap(const nsgpu_trace_codec *c, const nsgpu_trace_record *rec, uint64_t n, uint32_t dev, uint8_t *out,
                     uint64_t cap, uint64_t *len) {
  if (!c || (!rec && n) || !len) return set_error(NSGPU_EINVAL, "nsgpu_trace_pcap: null");
  if (dev >= c->n_devices) return set_error(NSGPU_EINVAL, "nsgpu_trace_pcap: device %u out of range", dev);
  std::vector<uint8_t> o;
  pcap_header(o, 9, 65535);  // PcapHelper::CreateFile (DLT_PPP, snaplen 65535)
  std::vector<uint8_t> pk;
  for (uint64_t i = 0; i < n; i++) {
    const nsgpu_trace_record &r = rec[i];
    if (r.dev != dev || (r.kind != NSGPU_TR_DEQUEUE && r.kind != NSGPU_TR_RX)) continue;  // the sniffer's calls
    if (!record_ok(*c, r)) return set_error(NSGPU_EINVAL, "nsgpu_trace_pcap: record %llu is malformed", (unsigned long long)i);
    pk.clear();
    packet_bytes(*c, r, pk);
    const uint64_t us = r.ts / 1000;  // (Time::GetMicroSeconds, PcapFileWrapper::Write)
    pcap_rec(o, (uint32_t)(us / 1000000), (uint32_t)(us % 1000000), pk.data(), (uint32_t)pk.size(), (uint32_t)pk.size(),
             65535);
  }
  return copy_out(o.data(), o.size(), out, cap, len);
}

// ---- Wi-Fi sniffer records ----
int nsgpu_wifi_sniff_power(const nsgpu_wifil_end *e, double rx_noise_figure_db, double *signal_dbm, double *noise_dbm) {
  if (!e || !signal_dbm || !noise_dbm) return set_error(NSGPU_EINVAL, "nsgpu_wifi_sniff_power: null");
  // yans-wifi-phy.cc:788-789 (RatioToDb: 10 log10, wifi-utils / yans-wifi-phy.cc)
  *signal_dbm = 10.0 * std::log10(e->rx_w) + 30;
  *noise_dbm = 10.0 * std::log10(e->rx_w / e->snr) - rx_noise_figure_db + 30;
  return NSGPU_OK;
}

namespace {
// RadiotapHeader as PcapSniffTxEvent / PcapSniffRxEvent build it (radiotap-header.cc:69-138: fields in bit
// order, little-endian, after the 8-byte header; setters at :231-380)
void radiotap(std::vector<uint8_t> &o, const nsgpu_wifi_sniff &r) {
  const bool rx = r.kind == 1;
  const uint32_t present = 0x1u | 0x2u | 0x4u | 0x8u | (rx ? 0x20u | 0x40u : 0u);
  const uint16_t length = (uint16_t)(8 + 8 + 1 + 1 + 4 + (rx ? 2 : 0));
  o.push_back(0), o.push_back(0);
  o.push_back((uint8_t)length), o.push_back((uint8_t)(length >> 8));
  le32(o, present);
  const uint64_t tsft = r.ts / 1000;  // Simulator::Now ().GetMicroSeconds ()
  for (int i = 0; i < 8; i++) o.push_back((uint8_t)(tsft >> (8 * i)));
  o.push_back((uint8_t)(0x10u | (r.short_preamble ? 0x02u : 0u)));  // FCS included, short preamble
  o.push_back((uint8_t)r.rate);
  uint16_t cf = 0;
  switch (r.rate) {
    case 2: case 4: case 10: case 22: cf |= 0x0020; break;  // CCK (1, 2, 5.5, 11 Mb/s)
    default: cf |= 0x0040; break;                           // OFDM
  }
  cf |= r.freq_mhz < 2500 ? 0x0080 : 0x0100;
  o.push_back((uint8_t)r.freq_mhz), o.push_back((uint8_t)(r.freq_mhz >> 8));
  o.push_back((uint8_t)cf), o.push_back((uint8_t)(cf >> 8));
  if (rx) {
    auto dbm8 = [](double v) -> uint8_t {
      if (v > 127) return (uint8_t)127;
      if (v < -128) return (uint8_t)(int8_t)-128;
      return (uint8_t)(int8_t)std::floor(v + 0.5);
    };
    o.push_back(dbm8(r.signal_dbm));
    o.push_back(dbm8(r.noise_dbm));
  }
}
}  // namespace

int nsgpu_wifi_pcap(uint32_t dlt, const nsgpu_wifi_sniff *rec, uint64_t n, uint32_t phy, const uint64_t *frame_off,
                    const uint8_t *frames, uint8_t *out, uint64_t cap, uint64_t *len) {
  if (!len || (n && (!rec || !frame_off || !frames))) return set_error(NSGPU_EINVAL, "nsgpu_wifi_pcap: null");
  if (dlt != 105 && dlt != 127)
    return set_error(NSGPU_EINVAL, "nsgpu_wifi_pcap: data link type %u (105: IEEE802_11, 127: radiotap)", dlt);
  std::vector<uint8_t> o, pk;
  pcap_header(o, dlt, 65535);
  for (uint64_t i = 0; i < n; i++) {
    const nsgpu_wifi_sniff &r = rec[i];
    if (r.phy != phy) continue;
    if (r.kind > 1 || frame_off[r.tx + 1] < frame_off[r.tx])
      return set_error(NSGPU_EINVAL, "nsgpu_wifi_pcap: record %llu is malformed", (unsigned long long)i);
    pk.clear();
    if (dlt == 127) radiotap(pk, r);
    pk.insert(pk.end(), frames + frame_off[r.tx], frames + frame_off[r.tx + 1]);
    const uint64_t us = r.ts / 1000;
    pcap_rec(o, (uint32_t)(us / 1000000), (uint32_t)(us % 1000000), pk.data(), (uint32_t)pk.size(),
             (uint32_t)pk.size(), 65535);
  }
  return copy_out(o.data(), o.size(), out, cap, len);
}

int nsgpu_wifi_ascii(const nsgpu_wifi_sniff *rec, uint64_t n, const uint32_t *phy_node, const uint32_t *phy_device,
                     const uint64_t *text_off, const char *text, char *out, uint64_t cap, uint64_t *len) {
  if (!len || (n && (!rec || !phy_node || !phy_device || !text_off || !text)))
    return set_error(NSGPU_EINVAL, "nsgpu_wifi_ascii: null");
  std::string o;
  char b[160];
  for (uint64_t i = 0; i < n; i++) {
    const nsgpu_wifi_sniff &r = rec[i];
    if (r.kind > 1) return set_error(NSGPU_EINVAL, "nsgpu_wifi_ascii: record %llu is malformed", (unsigned long long)i);
    std::snprintf(b, sizeof b, "%s %g /NodeList/%u/DeviceList/%u/$ns3::WifiNetDevice/Phy/State/%s ", r.kind ? "r" : "t",
                  nsgpu_time_get_seconds(r.ts), phy_node[r.phy], phy_device[r.phy], r.kind ? "RxOk" : "Tx");
    o += b;
    o.append(text + text_off[r.tx], text + text_off[r.tx + 1]);
    o += "\n";
  }
  return copy_out(o.data(), o.size(), out, cap, len);
}

int nsgpu_pcap_file(uint32_t linktype, uint32_t snaplen, uint64_t n, const uint32_t *sec, const uint32_t *usec,
                    const uint32_t *orig_len, const uint64_t *off, const uint8_t *data, uint8_t *out, uint64_t cap,
                    uint64_t *len) {
  if (!len || (n && (!sec || !usec || !orig_len || !off || !data))) return set_error(NSGPU_EINVAL, "nsgpu_pcap_file: null");
  std::vector<uint8_t> o;
  pcap_header(o, linktype, snaplen);
  for (uint64_t i = 0; i < n; i++) {
    if (off[i + 1] < off[i]) return set_error(NSGPU_EINVAL, "nsgpu_pcap_file: offsets decrease at %llu", (unsigned long long)i);
    pcap_rec(o, sec[i], usec[i], data + off[i], (uint32_t)(off[i + 1] - off[i]), orig_len[i], snaplen);
  }
  return copy_out(o.data(), o.size(), out, cap, len);
}

}  // extern "C"
