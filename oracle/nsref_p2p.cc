// nsref_p2p.cc — CPU ORACLE (test infrastructure only; see nsref.h header).
// Sequential restatement of the point-to-point / DropTail / IPv4-forward / UDP handler chain and of
// the OnOff + PacketSink applications, driven by the restated DefaultSimulatorImpl + MapScheduler.
// Every Schedule* call is made in the same order as the reference code makes it, so uids,
// timestamps and the pop order follow the reference:
//   setup:     NodeListPriv::Add (node-list.cc:124-131), Node::AddDevice (node.cc:111-123),
//              Node::AddApplication (node.cc:137-145), Node::DoStart (node.cc:183-199),
//              Application::DoStart (application.cc:87-95)
//   OnOff:     onoff-application.cc:132-252 (StartApplication, CancelEvents, StartSending, StopSending,
//              ScheduleNextTx, ScheduleStartEvent, ScheduleStopEvent, SendPacket)
//   device:    point-to-point-net-device.cc:206-269 (TransmitStart, TransmitComplete), :304-346 (Receive),
//              :462-518 (Send); point-to-point-channel.cc:82-103 (TransmitStart)
//   queue:     queue.cc:61-200, drop-tail-queue.cc:83-132
//   IPv4:      ipv4-l3-protocol.cc:434-537 (Receive), :815-841 (IpForward: TTL), static next-hop routing
//   UDP/sink:  udp-l4-protocol.cc:312-407 -> udp-socket-impl.cc:864-905 -> PacketSink (no events)
//   echo:      udp-echo-client.cc (StartApplication, StopApplication, ScheduleTransmit, Send, HandleRead),
//              udp-echo-server.cc (StartApplication, StopApplication, HandleRead -> SendTo)
//   IPv4 id:   Ipv4L3Protocol::BuildHeader (ipv4-l3-protocol.cc): m_identification++ per originated packet
//   traces:    the ascii default sinks hooked by PointToPointHelper::EnableAsciiInternal
//              (point-to-point-helper.cc:113-219): Queue Enqueue/Dequeue/Drop (queue.cc:61-97,
//              drop-tail-queue.cc:83-100), device MacRx (point-to-point-net-device.cc:304-346)
// Packet sizes: payload + 8 (UDP) + 20 (IPv4) + 2 (PPP, added in PointToPointNetDevice::Send).
#include <vector>
#include <deque>
#include <chrono>
#include <functional>
#include <string.h>
#include <stdio.h>
#include "nsref_engine.hpp"

namespace {

struct Pkt {
  uint32_t app;   // sending application (| NSGPU_PKT_REPLY: an echo on its way back to this client)
  uint32_t ipid;  // IPv4 identification (the sending node's m_identification)
  uint32_t size;  // current size in bytes (headers included as they are added)
  uint32_t ttl;
};

struct Model;

struct Dev {
  bool busy = false;  // m_txMachineState == BUSY
  Pkt cur{};
  std::deque<Pkt> q;  // DropTailQueue::m_packets
  nsgpu_dev_counters c{};
};

struct App {
  bool started = false;  // Object::m_started
  bool sink_active = false;
  nsgpu_event_id sendEvent{0, 0, 0, 0};       // OnOffApplication::m_sendEvent
  nsgpu_event_id startStopEvent{0, 0, 0, 0};  // m_startStopEvent
  uint64_t lastStartTime = 0;
  uint32_t residualBits = 0;
  uint32_t totBytes = 0;
  uint32_t sent = 0;  // UdpEchoClient::m_sent
  nsgpu_app_counters c{};
};

struct Model {
  nsref_sim sim{NSREF_SCHED_MAP};
  nsgpu_p2p_scenario s;
  std::vector<Dev> dev;
  std::vector<App> app;
  std::vector<std::vector<uint32_t>> node_apps;
  std::vector<int32_t> sink_of_node;
  std::vector<uint32_t> node_ipid;  // Ipv4L3Protocol::m_identification
  std::vector<nsgpu_trace_record> *trace = nullptr;
  uint16_t tr_seq = 0;
  uint32_t tr_uid = 0;
  uint64_t tr_ts = ~0ull;
  uint32_t tr_kinds = 0xfu;  // nsgpu_trace_kind bits recorded (nsref_p2p_set_trace_kinds)
  void tr(uint8_t kind, uint32_t d, const Pkt &p) {
    if (!trace || !((tr_kinds >> kind) & 1u)) return;
    if (sim.m_currentUid != tr_uid || sim.m_currentTs != tr_ts) {  // a new dispatched event
      tr_uid = sim.m_currentUid;
      tr_ts = sim.m_currentTs;
      tr_seq = 0;
    }
    nsgpu_trace_record r{};
    r.ts = sim.m_currentTs;
    r.uid = sim.m_currentUid;
    r.seq = tr_seq++;
    r.kind = kind;
    r.dev = d;
    r.app = p.app;
    r.ipid = p.ipid;
    r.size = p.size;
    r.ttl = p.ttl;
    trace->push_back(r);
  }
  // The node a packet is addressed to: an echo reply goes back to its client, an ICMP error to the
  // offending datagram's sender (icmpv4-l4-protocol.cc:131-160: SendMessage (p, header.GetSource (), ...)).
  uint32_t pkt_dst_node(const Pkt &p) const {
    if (p.app & NSGPU_PKT_ICMP) {
      const uint32_t fa = p.app & NSGPU_PKT_APP;
      return (p.app & NSGPU_PKT_ICMP_OF_REPLY) ? s.app_dst_node[fa] : s.app_node[fa];
    }
    return (p.app & NSGPU_PKT_REPLY) ? s.app_node[p.app & ~NSGPU_PKT_REPLY] : s.app_dst_node[p.app];
  }
  // static next hop of node n towards route slot k: the dense table, or the compressed one
  // (per-node default + ascending (slot, device) exceptions; include/nsgpu_types.h)
  uint32_t next_hop(uint32_t n, uint32_t k) const {
    if (s.route) return s.route[(uint64_t)n * s.n_dst + k];
    uint64_t lo = s.route_exc_off[n], hi = s.route_exc_off[n + 1];
    while (lo < hi) {
      const uint64_t mid = (lo + hi) / 2;
      if (s.route_exc_slot[mid] < k) lo = mid + 1;
      else hi = mid;
    }
    if (lo < s.route_exc_off[n + 1] && s.route_exc_slot[lo] == k) return s.route_exc_dev[lo];
    return s.route_default[n];
  }
  uint32_t src_slot(uint32_t a) const { return s.app_src_slot ? s.app_src_slot[a] : 0xffffffffu; }
  uint32_t pkt_dst_slot(const Pkt &p) const {
    if (p.app & NSGPU_PKT_ICMP) {
      const uint32_t fa = p.app & NSGPU_PKT_APP;
      return (p.app & NSGPU_PKT_ICMP_OF_REPLY) ? s.app_dst_slot[fa] : src_slot(fa);
    }
    return (p.app & NSGPU_PKT_REPLY) ? src_slot(p.app & ~NSGPU_PKT_REPLY) : s.app_dst_slot[p.app];
  }
  uint64_t ttl_drops = 0, no_route_drops = 0, unreach_drops = 0, icmp_sent = 0;

  template <class F>
  struct Ev : EventImpl {
    F f;
    explicit Ev(F x) : f(x) {}
    void Notify() override { f(); }
  };
  template <class F>
  nsgpu_event_id schedule(int64_t delay, F f) { return sim.Schedule(delay, new Ev<F>(f)); }
  template <class F>
  void schedule_ctx(uint32_t ctx, int64_t delay, F f) { sim.ScheduleWithContext(ctx, delay, new Ev<F>(f)); }
  bool running(const nsgpu_event_id &id) { return !sim.IsExpired(id); }  // EventId::IsRunning
  void cancel(const nsgpu_event_id &id) { sim.Cancel(id); }

  // ---------------- Queue / DropTailQueue ----------------
  bool enqueue(uint32_t d, const Pkt &p) {  // Queue::Enqueue -> DropTailQueue::DoEnqueue
    Dev &D = dev[d];
    if (D.q.size() >= s.dev_qmax[d]) {  // Drop (p): m_nTotalDroppedPackets++, bytes
      tr(NSGPU_TR_DROP, d, p);
      D.c.drop_packets++;
      D.c.drop_bytes += p.size;
      return false;
    }
    D.q.push_back(p);
    tr(NSGPU_TR_ENQUEUE, d, p);
    D.c.enq_packets++;
    D.c.enq_bytes += p.size;
    return true;
  }
  bool dequeue(uint32_t d, Pkt &out) {
    Dev &D = dev[d];
    if (D.q.empty()) return false;
    out = D.q.front();
    D.q.pop_front();
    tr(NSGPU_TR_DEQUEUE, d, out);
    D.c.deq_packets++;
    return true;
  }

  // ---------------- PointToPointNetDevice / PointToPointChannel ----------------
  void transmit_start(uint32_t d, const Pkt &p) {  // point-to-point-net-device.cc:206-234
    Dev &D = dev[d];
    D.busy = true;
    D.cur = p;
    D.c.tx_packets++;
    // Time txTime = Seconds (m_bps.CalculateTxTime (p->GetSize ())) (data-rate.cc:224-227)
    const double tx_s = static_cast<double>(p.size) * 8 / s.dev_bps[d];
    const int64_t txTime = nsref_seconds(tx_s);
    const int64_t txCompleteTime = txTime + s.dev_ifg_ns[d];
    schedule(txCompleteTime, [this, d]() { transmit_complete(d); });
    // PointToPointChannel::TransmitStart (point-to-point-channel.cc:82-103)
    const uint32_t peer = s.dev_peer[d];
    schedule_ctx(s.dev_node[peer], txTime + s.dev_delay_ns[d], [this, peer, p]() { receive(peer, p); });
  }
  void transmit_complete(uint32_t d) {  // :236-269
    Dev &D = dev[d];
    D.busy = false;
    Pkt p;
    if (!dequeue(d, p)) return;
    transmit_start(d, p);
  }
  void device_send(uint32_t d, Pkt p) {  // :462-518
    p.size += 2;  // AddHeader (PppHeader)
    Dev &D = dev[d];
    if (!D.busy) {
      if (enqueue(d, p)) {
        Pkt q;
        dequeue(d, q);
        transmit_start(d, q);
      }
      // else MacTxDrop: counted by the queue's drop counters
    } else {
      enqueue(d, p);
    }
  }
  void receive(uint32_t d, Pkt p) {  // :304-346 (no error model)
    dev[d].c.rx_packets++;
    p.size -= 2;  // ProcessHeader strips the PPP header
    tr(NSGPU_TR_RX, d, p);  // m_macRxTrace
    tr(NSGPU_TR_IP_RX, d, p);  // Ipv4L3Protocol::Receive: m_rxTrace (ipv4-l3-protocol.cc:455)
    ip_receive(s.dev_node[d], p, d);
  }
  // SendRealOut: m_txTrace (the packet with its IPv4 header), then the interface's device (:764-765)
  void ip_out(uint32_t out, const Pkt &p) {
    tr(NSGPU_TR_IP_TX, out, p);
    device_send(out, p);
  }
  // m_dropTrace (header, packet, reason, ipv4, interface): the header as received; a UDP datagram's
  // record keeps its 16-bit id (an ICMP descriptor's packs the embedded one too)
  void ip_drop(uint32_t d, Pkt p) {
    if (!(p.app & NSGPU_PKT_ICMP)) p.ipid &= 0xffffu;
    tr(NSGPU_TR_IP_DROP, d, p);
  }

  // ---------------- IPv4 + UDP ----------------
  // ---------------- ICMP (icmpv4-l4-protocol.cc:85-160, icmpv4.cc:306-440) ----------------
  // The error about datagram p (p's IPv4 header as embedded: TTL, identification, length) is a 56-byte
  // IPv4 packet (Icmpv4Header 4 + TimeExceeded / DestinationUnreachable 4 + header 20 + 8 payload bytes)
  // sent from node n to p's sender with the default TTL 64: SendMessage -> RouteOutput ->
  // Ipv4L3Protocol::Send (m_identification++); no route: "drop icmp message".
  void icmp_send(uint32_t n, const Pkt &p, bool unreach) {
    const uint32_t of = (p.app & NSGPU_PKT_REPLY) ? NSGPU_PKT_ICMP_OF_REPLY : 0u;
    Pkt e{NSGPU_PKT_ICMP | (unreach ? NSGPU_PKT_ICMP_UNREACH : 0u) | of | (p.app & NSGPU_PKT_APP),
          (p.ipid & 0xffffu) << 16, 56u, 64u | ((p.ttl & 0xffu) << 8) | (p.size << 16)};
    const uint32_t k = pkt_dst_slot(e);
    const uint32_t out = k == 0xffffffffu ? 0xffffffffu : next_hop(n, k);
    if (out == 0xffffffffu) {
      no_route_drops++;
      return;
    }
    e.ipid |= node_ipid[n]++ & 0xffffu;
    icmp_sent++;
    ip_out(out, e);
  }

  void ip_receive(uint32_t n, Pkt p, uint32_t rx_dev) {  // Ipv4L3Protocol::Receive -> RouteInput
    if (pkt_dst_node(p) == n) {  // LocalDeliver -> UdpL4Protocol::Receive (udp-l4-protocol.cc:312-407)
      // an ICMP error ends in Icmpv4L4Protocol::Receive -> HandleTimeExceeded / HandleDestUnreach ->
      // UdpL4Protocol::ReceiveIcmp -> the endpoint's (null) ICMP callback: nothing is scheduled
      if (p.app & NSGPU_PKT_ICMP) return;
      // the bound endpoint: the client's own socket for an echo reply, else the node's sink / echo server
      const int32_t k = (p.app & NSGPU_PKT_REPLY) ? (int32_t)(p.app & ~NSGPU_PKT_REPLY) : sink_of_node[n];
      if (k < 0 || !app[k].sink_active) {  // no bound endpoint: RX_ENDPOINT_UNREACH
        unreach_drops++;
        if (s.icmp) icmp_send(n, p, true);  // Ipv4L3Protocol::LocalDeliver: SendDestUnreachPort (ip, copy)
        return;
      }
      // Ipv4EndPoint::ForwardUp: ScheduleNow (&Ipv4EndPoint::DoForwardUp) (ipv4-end-point.cc:112-120)
      sim.ScheduleNow(new Ev<std::function<void()>>([this, k, p, n]() {
        // DoForwardUp -> UdpSocketImpl::ForwardUp -> PacketSink / UdpEchoClient / UdpEchoServer::HandleRead
        if (!app[k].sink_active) return;
        app[k].c.rx_packets++;
        app[k].c.rx_bytes += p.size - 28;
        if (s.app_kind[k] == NSGPU_APP_ECHO_SERVER) {  // socket->SendTo (packet, 0, from)
          Pkt r{p.app | NSGPU_PKT_REPLY, 0, p.size, s.app_ttl[k]};
          app[k].c.tx_packets++;
          app[k].c.tx_bytes += p.size - 28;
          ip_send(n, r);
        }
      }));
      return;
    }
    const uint32_t out = next_hop(n, pkt_dst_slot(p));
    if (out == 0xffffffffu) {  // DROP_NO_ROUTE (:505)
      no_route_drops++;
      ip_drop(rx_dev, p);
      return;
    }
    // IpForward (ipv4-l3-protocol.cc:815-841)
    const Pkt received = p;
    p.ttl -= 1;
    if ((p.ttl & 0xffu) == 0) {  // DROP_TTL_EXPIRED, after SendTimeExceededTtl (never about an ICMP message)
      ttl_drops++;
      if (s.icmp && !(p.app & NSGPU_PKT_ICMP)) icmp_send(n, p, false);
      ip_drop(out, received);  // (:835: the forwarding route's interface, the header as received)
      return;
    }
    ip_out(out, p);
  }
  void ip_send(uint32_t n, Pkt p) {  // UdpSocketImpl::DoSendTo (RouteOutput) -> Ipv4L3Protocol::Send
    const uint32_t out = next_hop(n, pkt_dst_slot(p));
    if (out == 0xffffffffu) {
      no_route_drops++;
      return;
    }
    p.ipid = node_ipid[n]++;  // BuildHeader: SetIdentification (m_identification++)
    ip_out(out, p);
  }

  // ---------------- OnOffApplication ----------------
  void cancel_events(uint32_t a) {  // :165-178
    App &A = app[a];
    if (running(A.sendEvent)) {
      const int64_t delta = (int64_t)sim.m_currentTs - (int64_t)A.lastStartTime;
      uint64_t d[2], inv[2], t[2], r[2], b[2];
      nsref_i64x64_from_int(delta, d);
      nsref_i64x64_invert(1000000000ull, inv);
      nsref_i64x64_mul_by_invert(d, inv, t);  // delta.To (Time::S)
      nsref_i64x64_from_parts((int64_t)s.app_rate_bps[a], 0, r);
      nsref_i64x64_mul(t, r, b);  // * m_cbrRate.GetBitRate ()
      A.residualBits += (uint32_t)nsref_i64x64_get_high(b);
    }
    cancel(A.sendEvent);
    cancel(A.startStopEvent);
  }
  void schedule_start_event(uint32_t a) {  // :209-215
    app[a].startStopEvent = schedule(nsref_seconds(s.app_off_s[a]), [this, a]() { start_sending(a); });
  }
  void schedule_stop_event(uint32_t a) {  // :217-223
    app[a].startStopEvent = schedule(nsref_seconds(s.app_on_s[a]), [this, a]() { stop_sending(a); });
  }
  void schedule_next_tx(uint32_t a) {  // :193-207
    App &A = app[a];
    if (s.app_max_bytes[a] == 0 || A.totBytes < s.app_max_bytes[a]) {
      const uint32_t bits = s.app_pkt_size[a] * 8 - A.residualBits;
      const int64_t nextTime = nsref_seconds(bits / static_cast<double>(s.app_rate_bps[a]));
      A.sendEvent = schedule(nextTime, [this, a]() { send_packet(a); });
    } else {
      stop_application(a);
    }
  }
  void start_sending(uint32_t a) {  // :180-185
    app[a].lastStartTime = sim.m_currentTs;
    schedule_next_tx(a);
    schedule_stop_event(a);
  }
  void stop_sending(uint32_t a) {  // :187-191
    cancel_events(a);
    schedule_start_event(a);
  }
  void send_packet(uint32_t a) {  // :226-236
    App &A = app[a];
    Pkt p{a, 0, s.app_pkt_size[a] + 8 + 20, s.app_ttl[a]};
    A.c.tx_packets++;
    A.c.tx_bytes += s.app_pkt_size[a];
    ip_send(s.app_node[a], p);
    A.totBytes += s.app_pkt_size[a];
    A.lastStartTime = sim.m_currentTs;
    A.residualBits = 0;
    schedule_next_tx(a);
  }
  // ---------------- UdpEchoClient ----------------
  void echo_send(uint32_t a) {  // UdpEchoClient::Send
    App &A = app[a];
    A.c.tx_packets++;
    A.c.tx_bytes += s.app_pkt_size[a];
    ip_send(s.app_node[a], Pkt{a, 0, s.app_pkt_size[a] + 8 + 20, s.app_ttl[a]});  // m_socket->Send (p)
    ++A.sent;
    if (A.sent < s.app_count[a])  // ScheduleTransmit (m_interval)
      A.sendEvent = schedule(s.app_interval_ns[a], [this, a]() { echo_send(a); });
  }

  void start_application(uint32_t a) {  // :132-150 (socket setup schedules nothing)
    if (s.app_kind[a] == NSGPU_APP_SINK || s.app_kind[a] == NSGPU_APP_ECHO_SERVER) {  // Bind (port)
      app[a].sink_active = true;
      return;
    }
    if (s.app_kind[a] == NSGPU_APP_ECHO_CLIENT) {  // Bind, Connect, SetRecvCallback, ScheduleTransmit (0)
      app[a].sink_active = true;
      app[a].sendEvent = schedule(0, [this, a]() { echo_send(a); });
      return;
    }
    cancel_events(a);
    schedule_start_event(a);
  }
  void stop_application(uint32_t a) {  // :152-163
    if (s.app_kind[a] == NSGPU_APP_SINK || s.app_kind[a] == NSGPU_APP_ECHO_SERVER) {  // m_socket->Close ()
      app[a].sink_active = false;
      return;
    }
    if (s.app_kind[a] == NSGPU_APP_ECHO_CLIENT) {  // Close; Simulator::Cancel (m_sendEvent)
      app[a].sink_active = false;
      cancel(app[a].sendEvent);
      return;
    }
    cancel_events(a);
  }

  // ---------------- setup ----------------
  void app_object_start(uint32_t a) {  // Object::Start -> Application::DoStart (application.cc:87-95)
    if (app[a].started) return;
    app[a].started = true;
    schedule(s.app_start_ns[a], [this, a]() { start_application(a); });
    if (s.app_stop_ns[a] != 0) schedule(s.app_stop_ns[a], [this, a]() { stop_application(a); });
  }
  void node_start(uint32_t n) {  // Node::DoStart: devices (no events), then applications in order
    for (uint32_t a : node_apps[n]) app_object_start(a);
  }
  void setup() {
    if (s.uid_first) sim.m_uid = s.uid_first;  // the program's earlier Schedule calls consumed the uids below it
    dev.resize(s.n_devices);
    app.resize(s.n_apps);
    node_apps.assign(s.n_nodes, {});
    sink_of_node.assign(s.n_nodes, -1);
    node_ipid.assign(s.n_nodes, 0);
    for (uint32_t a = 0; a < s.n_apps; a++) {
      node_apps[s.app_node[a]].push_back(a);
      if (s.app_kind[a] == NSGPU_APP_SINK || s.app_kind[a] == NSGPU_APP_ECHO_SERVER)
        sink_of_node[s.app_node[a]] = (int32_t)a;
    }
    for (uint32_t i = 0; i < s.n_setup; i++) {
      const uint32_t k = s.setup_index[i];
      switch (s.setup_kind[i]) {
        case NSGPU_SETUP_NODE:  // NodeListPriv::Add
          schedule_ctx(k, 0, [this, k]() { node_start(k); });
          break;
        case NSGPU_SETUP_DEVICE:  // Node::AddDevice -> NetDevice::Start (already started by Node::Start)
          schedule_ctx(s.dev_node[k], 0, []() {});
          break;
        case NSGPU_SETUP_APP:  // Node::AddApplication -> Application::Start (Object::Start is idempotent)
          schedule_ctx(s.app_node[k], 0, [this, k]() { app_object_start(k); });
          break;
        case NSGPU_SETUP_STOP:  // Simulator::Stop (Time) (default-simulator-impl.cc:179-183)
          schedule(s.stop_ns, [this]() { sim.m_stop = true; });
          break;
        case NSGPU_SETUP_NOOP:  // e.g. LoopbackNetDevice added by Ipv4L3Protocol::SetupLoopback
          schedule_ctx(k, 0, []() {});
          break;
        default:  // a setup call consuming a uid without a queued event (ScheduleDestroy)
          sim.m_uid++;
      }
    }
  }
};

uint32_t g_trace_kinds = 0xfu;

}  // namespace

// The trace kinds the next runs record (bit k = nsgpu_trace_kind k; default 0xf, the device sinks):
// nsgpu_p2p_set_trace_kinds' counterpart.
extern "C" void nsref_p2p_set_trace_kinds(uint32_t mask) { g_trace_kinds = mask; }

extern "C" int nsref_p2p_run_trace(const nsgpu_p2p_scenario *sc, nsgpu_p2p_stats *stats,
                                   nsgpu_dev_counters *devc, nsgpu_app_counters *appc, uint64_t *log_ts,
                                   uint32_t *log_uid, uint32_t *log_ctx, uint64_t log_cap, double *run_seconds,
                                   nsgpu_trace_record *trace, uint64_t trace_cap, uint64_t *trace_n) {
  Model *m = new Model();
  std::vector<nsgpu_trace_record> tv;
  if (trace_n) m->trace = &tv;
  m->tr_kinds = g_trace_kinds;
  m->s = *sc;
  m->sim.want_digest = true;
  m->sim.log_ts = log_ts;
  m->sim.log_uid = log_uid;
  m->sim.log_ctx = log_ctx;
  m->sim.log_cap = log_ts ? log_cap : 0;
  m->setup();
  auto t0 = std::chrono::steady_clock::now();
  m->sim.Run();
  auto t1 = std::chrono::steady_clock::now();
  if (run_seconds) *run_seconds = std::chrono::duration<double>(t1 - t0).count();
  memset(stats, 0, sizeof(*stats));
  stats->dispatched = m->sim.m_dispatched;
  stats->cancelled = m->sim.m_cancelled;
  stats->digest = m->sim.m_digest;
  stats->final_ts = m->sim.m_currentTs;
  stats->next_uid = m->sim.m_uid;
  stats->ttl_drops = m->ttl_drops;
  stats->no_route_drops = m->no_route_drops;
  stats->unreach_drops = m->unreach_drops;
  stats->icmp_sent = m->icmp_sent;
  if (devc)
    for (uint32_t d = 0; d < sc->n_devices; d++) devc[d] = m->dev[d].c;
  if (appc)
    for (uint32_t a = 0; a < sc->n_apps; a++) appc[a] = m->app[a].c;
  if (trace_n) {
    *trace_n = tv.size();
    for (uint64_t i = 0; i < tv.size() && i < trace_cap; i++) trace[i] = tv[i];
  }
  delete m;
  return 0;
}

// A host application interleaved with the handler chain (the mixed-mode contract of nsgpu_sim +
// nsgpu_p2p): a closure scheduled with Simulator::Schedule (t0) right after setup, which, every `period`
// for `count` rounds, reads application app_obs's counters (a trace / stats callback) and sends one
// datagram of application app_send's flow through its socket now (UdpSocket::Send from a host
// application: onoff-application.cc:226-236's send without the OnOff state), then re-schedules itself.
extern "C" int nsref_p2p_run_probe(const nsgpu_p2p_scenario *sc, int64_t t0, int64_t period, uint32_t count,
                                   uint32_t app_send, uint32_t app_obs, nsgpu_app_counters *samples,
                                   nsgpu_p2p_stats *stats, nsgpu_dev_counters *devc, nsgpu_app_counters *appc,
                                   uint64_t *log_ts, uint32_t *log_uid, uint32_t *log_ctx, uint64_t log_cap,
                                   nsgpu_trace_record *trace, uint64_t trace_cap, uint64_t *trace_n) {
  Model *m = new Model();
  std::vector<nsgpu_trace_record> tv;
  if (trace_n) m->trace = &tv;
  m->tr_kinds = g_trace_kinds;
  m->s = *sc;
  m->sim.want_digest = true;
  m->sim.log_ts = log_ts;
  m->sim.log_uid = log_uid;
  m->sim.log_ctx = log_ctx;
  m->sim.log_cap = log_ts ? log_cap : 0;
  m->setup();
  uint32_t k = 0;
  std::function<void()> probe = [&]() {
    samples[k] = m->app[app_obs].c;
    App &A = m->app[app_send];
    A.c.tx_packets++;
    A.c.tx_bytes += sc->app_pkt_size[app_send];
    m->ip_send(sc->app_node[app_send], Pkt{app_send, 0, sc->app_pkt_size[app_send] + 8 + 20, sc->app_ttl[app_send]});
    if (++k < count) m->schedule(period, [&]() { probe(); });
  };
  if (count) m->schedule(t0, [&]() { probe(); });
  m->sim.Run();
  memset(stats, 0, sizeof(*stats));
  stats->dispatched = m->sim.m_dispatched;
  stats->cancelled = m->sim.m_cancelled;
  stats->digest = m->sim.m_digest;
  stats->final_ts = m->sim.m_currentTs;
  stats->next_uid = m->sim.m_uid;
  stats->ttl_drops = m->ttl_drops;
  stats->no_route_drops = m->no_route_drops;
  stats->unreach_drops = m->unreach_drops;
  stats->icmp_sent = m->icmp_sent;
  if (devc)
    for (uint32_t d = 0; d < sc->n_devices; d++) devc[d] = m->dev[d].c;
  if (appc)
    for (uint32_t a = 0; a < sc->n_apps; a++) appc[a] = m->app[a].c;
  if (trace_n) {
    *trace_n = tv.size();
    for (uint64_t i = 0; i < tv.size() && i < trace_cap; i++) trace[i] = tv[i];
  }
  delete m;
  return 0;
}

// A host application's datagrams at given times: right after setup, Simulator::Schedule (ts[k], send k) for k in
// order; send k is UdpSocket::Send of one datagram of application app[k]'s flow (as the probe's send above).  The
// replay of a reference pcap's sends (tests/olsr_replay.py: OLSR HELLOs over point-to-point).
extern "C" int nsref_p2p_run_sends(const nsgpu_p2p_scenario *sc, uint64_t n, const int64_t *ts, const uint32_t *app,
                                   nsgpu_p2p_stats *stats, nsgpu_dev_counters *devc, nsgpu_app_counters *appc,
                                   uint64_t *log_ts, uint32_t *log_uid, uint32_t *log_ctx, uint64_t log_cap,
                                   nsgpu_trace_record *trace, uint64_t trace_cap, uint64_t *trace_n) {
  Model *m = new Model();
  std::vector<nsgpu_trace_record> tv;
  if (trace_n) m->trace = &tv;
  m->tr_kinds = g_trace_kinds;
  m->s = *sc;
  m->sim.want_digest = true;
  m->sim.log_ts = log_ts;
  m->sim.log_uid = log_uid;
  m->sim.log_ctx = log_ctx;
  m->sim.log_cap = log_ts ? log_cap : 0;
  m->setup();
  for (uint64_t k = 0; k < n; k++) {
    const uint32_t a = app[k];
    m->schedule(ts[k], [m, sc, a]() {
      App &A = m->app[a];
      A.c.tx_packets++;
      A.c.tx_bytes += sc->app_pkt_size[a];
      m->ip_send(sc->app_node[a], Pkt{a, 0, sc->app_pkt_size[a] + 8 + 20, sc->app_ttl[a]});
    });
  }
  m->sim.Run();
  memset(stats, 0, sizeof(*stats));
  stats->dispatched = m->sim.m_dispatched;
  stats->cancelled = m->sim.m_cancelled;
  stats->digest = m->sim.m_digest;
  stats->final_ts = m->sim.m_currentTs;
  stats->next_uid = m->sim.m_uid;
  stats->ttl_drops = m->ttl_drops;
  stats->no_route_drops = m->no_route_drops;
  stats->unreach_drops = m->unreach_drops;
  stats->icmp_sent = m->icmp_sent;
  if (devc)
    for (uint32_t d = 0; d < sc->n_devices; d++) devc[d] = m->dev[d].c;
  if (appc)
    for (uint32_t a = 0; a < sc->n_apps; a++) appc[a] = m->app[a].c;
  if (trace_n) {
    *trace_n = tv.size();
    for (uint64_t i = 0; i < tv.size() && i < trace_cap; i++) trace[i] = tv[i];
  }
  delete m;
  return 0;
}

extern "C" int nsref_p2p_run(const nsgpu_p2p_scenario *sc, nsgpu_p2p_stats *stats, nsgpu_dev_counters *devc,
                             nsgpu_app_counters *appc, uint64_t *log_ts, uint32_t *log_uid, uint32_t *log_ctx,
                             uint64_t log_cap, double *run_seconds) {
  return nsref_p2p_run_trace(sc, stats, devc, appc, log_ts, log_uid, log_ctx, log_cap, run_seconds, nullptr, 0,
                             nullptr);
}
