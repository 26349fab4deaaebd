/*
 * nsgpu_types.h — plain-old-data types shared by the nsgpu C-ABI (include/nsgpu.h)
 * and its test checker (oracle/).  No torch types, no C++ across the ABI.
 *
 * Event key layout follows ns-3's Scheduler::EventKey
 *   (reference: src/core/model/scheduler.h:58-63):
 *     uint64 m_ts; uint32 m_uid; uint32 m_context
 * and the ordering is (ts, uid) ONLY (scheduler.h:105-121) — context is payload.
 */
#ifndef NSGPU_TYPES_H
#define NSGPU_TYPES_H

#include <stdint.h>

#if defined(__HIP__)
#define NSGPU_HD __host__ __device__
#else
#define NSGPU_HD
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* Scheduler::EventKey + Scheduler::Event (scheduler.h:58-68): 24 bytes. */
typedef struct nsgpu_event {
  uint64_t ts;       /* absolute time, in Time resolution units (ns) */
  uint32_t uid;      /* global schedule counter, starts at 4 (default-simulator-impl.cc:52-56) */
  uint32_t context;  /* node id, 0xffffffff = no node (default-simulator-impl.cc:60) */
  uint64_t handle;   /* opaque EventImpl* (host closure) — never dereferenced on device */
} nsgpu_event;

/* ns-3 EventId (event-id.h:46-83): (impl, ts, context, uid). */
typedef struct nsgpu_event_id {
  uint64_t impl;
  uint64_t ts;
  uint32_t context;
  uint32_t uid;
} nsgpu_event_id;

/* Propagation loss model kinds (src/propagation/model/propagation-loss-model.cc). */
enum nsgpu_loss_kind {
  NSGPU_LOSS_NONE = 0,
  NSGPU_LOSS_LOG_DISTANCE = 1, /* p0 = exponent, p1 = reference distance, p2 = reference loss  (:464-491) */
  NSGPU_LOSS_FRIIS = 2,        /* p0 = lambda, p1 = system loss, p2 = min distance            (:197-239) */
  NSGPU_LOSS_FIXED_RSS = 3,    /* p0 = fixed rss dBm                                          (:718-723) */
  NSGPU_LOSS_RANGE = 4         /* p0 = max range m; beyond it -1000 dBm                       (:822-834) */
};

typedef struct nsgpu_loss_model {
  int32_t kind;
  int32_t pad_;
  double p0, p1, p2;
} nsgpu_loss_model;

/* A PropagationLossModel chain (PropagationLossModel::CalcRxPower, :64-74): up to 4 links. */
#define NSGPU_MAX_LOSS_CHAIN 4
typedef struct nsgpu_loss_chain {
  int32_t n;
  int32_t pad_;
  nsgpu_loss_model m[NSGPU_MAX_LOSS_CHAIN];
} nsgpu_loss_chain;

/* Result record of one broadcast fan-out receiver (YansWifiChannel::Send, yans-wifi-channel.cc:77-115):
 * the ScheduleWithContext(dstNode, delay, &YansWifiChannel::Receive, this, j, copy, rxPowerDbm, ...) call. */
typedef struct nsgpu_rx_record {
  uint64_t ts;       /* now + delay */
  uint32_t uid;      /* uid_base + rank among surviving receivers (list order) */
  uint32_t context;  /* destination node id */
  uint32_t phy;      /* index j into the channel's phy list */
  uint32_t pad_;
  double rx_dbm;     /* CalcRxPower (txPowerDbm, sender, receiver) */
} nsgpu_rx_record;

/* SpectrumModels a MultiModelSpectrumChannel knows, indexed in ascending SpectrumModelUid order (the
 * iteration order of its m_rxSpectrumModelInfoMap, multi-model-spectrum-channel.cc:246-249): model m has
 * the bands [band_off[m], band_off[m+1]) of fl / fh (BandInfo, Hz).  Pointers are device memory. */
typedef struct nsgpu_spectrum_models {
  int32_t n_models;
  int32_t max_bands;          /* largest band count of any model (the PSD stride) */
  const uint32_t *band_off;   /* [n_models + 1] */
  const double *fl, *fh;      /* [band_off[n_models]] */
} nsgpu_spectrum_models;

/* One PropagationLoss trace call of a spectrum channel's StartTx: m_propagationLossTrace (txPhy, rxPhy,
 * -gainDb), fired for every receiver before the MaxLossDb cut (multi-model-spectrum-channel.cc:290-291,
 * single-model-spectrum-channel.cc:145-146). */
typedef struct nsgpu_loss_trace {
  uint32_t rx_phy;
  uint32_t pad_;
  double loss_db;
} nsgpu_loss_trace;

/* ---------------- point-to-point scenario (GPU-resident p2p / DropTail / IPv4 / UDP subset) ----------------
 * A topology of PointToPointNetDevices joined by PointToPointChannels, IPv4 forwarding by static
 * next-hop tables, OnOff (UDP, constant on/off times) sources and PacketSink sinks.  All arrays are
 * host pointers; devices and applications are listed in ns-3 creation order (Node::AddDevice /
 * Node::AddApplication), which fixes the setup-time uids (node-list.cc:124-131, node.cc:111-145). */
enum nsgpu_app_kind { NSGPU_APP_ONOFF = 0, NSGPU_APP_SINK = 1, NSGPU_APP_ECHO_CLIENT = 2, NSGPU_APP_ECHO_SERVER = 3 };
/* UdpEchoClient (udp-echo-client.cc): app_dst_node = the server's node, app_pkt_size = PacketSize,
 * app_count = MaxPackets, app_interval_ns = Interval, app_src_slot = the route-table slot of the
 * client's own node (the echo comes back there).  UdpEchoServer (udp-echo-server.cc): the node's bound
 * UDP endpoint, like a PacketSink; HandleRead sends every datagram back to its sender.  A node has
 * at most one bound endpoint (PacketSink or UdpEchoServer). */

typedef struct nsgpu_p2p_scenario {
  uint32_t n_nodes;
  uint32_t n_devices;
  uint32_t n_apps;
  uint32_t n_dst;              /* columns of the route table (destination slots) */
  /* devices (PointToPointNetDevice + DropTailQueue), index = creation order */
  const uint32_t *dev_node;    /* owning node */
  const uint32_t *dev_peer;    /* device at the other end of the channel */
  const uint64_t *dev_bps;     /* DataRate (bit/s), point-to-point-net-device.cc:57 */
  const int64_t  *dev_ifg_ns;  /* InterframeGap */
  const int64_t  *dev_delay_ns;/* PointToPointChannel Delay of the device's channel */
  const uint32_t *dev_qmax;    /* DropTailQueue MaxPackets (PACKETS mode), drop-tail-queue.cc:37-43 */
  /* IPv4 static routing: route[node * n_dst + slot] = output device, or 0xffffffff = no route */
  const uint32_t *route;
  /* applications in AddApplication order */
  const uint32_t *app_kind;    /* nsgpu_app_kind */
  const uint32_t *app_node;
  const int64_t  *app_start_ns;
  const int64_t  *app_stop_ns; /* 0 = never (application.cc:90-93) */
  /* OnOff parameters (ignored for sinks), onoff-application.cc:47-86 */
  const uint32_t *app_dst_node;
  const uint32_t *app_dst_slot;
  const uint64_t *app_rate_bps;
  const uint32_t *app_pkt_size;
  const double   *app_on_s;    /* ConstantVariable OnTime (seconds; converted by Seconds () at each use) */
  const double   *app_off_s;   /* ConstantVariable OffTime */
  const uint32_t *app_max_bytes;
  const uint32_t *app_ttl;     /* IP TTL of the flow's packets */
  int64_t stop_ns;             /* Simulator::Stop (Seconds (x)) from main, as ns */
  /* Setup-time Schedule calls in program order (they fix every later uid):
   *   NSGPU_SETUP_NODE k   NodeListPriv::Add      -> ScheduleWithContext (k, 0, &Node::Start)
   *   NSGPU_SETUP_DEVICE d Node::AddDevice        -> ScheduleWithContext (node, 0, &NetDevice::Start)
   *   NSGPU_SETUP_APP a    Node::AddApplication   -> ScheduleWithContext (node, 0, &Application::Start)
   *   NSGPU_SETUP_STOP     Simulator::Stop (t)    -> Schedule (t, &Simulator::Stop), context 0xffffffff
   *   NSGPU_SETUP_UID      any other setup call that consumes one uid without a dispatched event */
  uint32_t n_setup;
  /* 1: ICMP errors are generated (Ipv4L3Protocol::IpForward TTL expiry -> Icmpv4L4Protocol::
   * SendTimeExceededTtl, LocalDeliver RX_ENDPOINT_UNREACH -> SendDestUnreachPort; ipv4-l3-protocol.cc,
   * icmpv4-l4-protocol.cc:85-160) and routed back to the offending datagram's sender through
   * app_src_slot; the lookahead then also covers the 58-byte ICMP frames.  0: the triggers are only
   * counted (ttl_drops / unreach_drops), i.e. the scenario asserts they never happen. */
  uint32_t icmp;
  const uint32_t *setup_kind;
  const uint32_t *setup_index;
  /* UdpEchoClient parameters (NULL when the scenario has no echo client) */
  const uint32_t *app_count;
  const int64_t  *app_interval_ns;
  /* route-table slot of each sending application's own node: where an echo reply and (icmp = 1) an
   * ICMP error about the application's datagrams are routed; 0xffffffff: none */
  const uint32_t *app_src_slot;
  /* Compressed next-hop table, used when `route` is NULL (large topologies: the dense table is
   * n_nodes x n_dst): node n forwards towards slot k through route_exc_dev[j] for the j in
   * [route_exc_off[n], route_exc_off[n + 1]) with route_exc_slot[j] == k (slots ascending within a
   * node), else through route_default[n] (0xffffffff: no route). */
  const uint32_t *route_default;   /* n_nodes */
  const uint64_t *route_exc_off;   /* n_nodes + 1 */
  const uint32_t *route_exc_slot;
  const uint32_t *route_exc_dev;
  /* DefaultSimulatorImpl::m_uid before the first setup call (0: 4, the reference's start, :52-56) — a program
   * whose earlier Schedule calls consumed uids; the engine refuses to pass 0xfffffffe (NSGPU_ERANGE) */
  uint32_t uid_first;
  uint32_t pad_uid_;
} nsgpu_p2p_scenario;

/* Packet descriptor flags (the descriptor {app, ipid, size, ttl} of a datagram): an echo reply
 * travelling back to its client (app) ... */
#define NSGPU_PKT_REPLY 0x80000000u
/* ... or an ICMP error about a datagram of flow (app & NSGPU_PKT_APP), travelling back to that datagram's
 * sender: NSGPU_PKT_ICMP_UNREACH = destination unreachable (port), else time exceeded (TTL);
 * NSGPU_PKT_ICMP_OF_REPLY = the offending datagram was an echo reply.  An ICMP descriptor packs the
 * offending datagram's IPv4 header fields: ipid = own | offending << 16 (16 bits each), size = 56 (the
 * ICMP packet's IPv4 length), ttl = own TTL | offending TTL << 8 | offending IPv4 length << 16. */
#define NSGPU_PKT_ICMP 0x40000000u
#define NSGPU_PKT_ICMP_UNREACH 0x20000000u
#define NSGPU_PKT_ICMP_OF_REPLY 0x10000000u
#define NSGPU_PKT_APP 0x0fffffffu

/* ---------------- trace records (ascii / pcap replay) ----------------
 * One record per call of a default ascii trace sink of PointToPointHelper::EnableAsciiInternal
 * (point-to-point-helper.cc:113-219, trace-helper.cc:303-390): TxQueue/Enqueue "+", TxQueue/Dequeue
 * "-", TxQueue/Drop "d", MacRx "r".  The pcap PromiscSniffer calls are implied: every Dequeue is
 * followed by the sniffer on the same device (Send :462-518, TransmitComplete :236-269), every MacRx is
 * preceded by it (Receive :304-346, packet with the PPP header).  Records are written unordered; the
 * trace order is (ts, uid, seq): the pop order of the dispatched event, then call order inside it. */
enum nsgpu_trace_kind { NSGPU_TR_ENQUEUE = 0, NSGPU_TR_DEQUEUE = 1, NSGPU_TR_DROP = 2, NSGPU_TR_RX = 3,
                        /* Ipv4L3Protocol's trace sources as InternetStackHelper::EnableAsciiIpv4 hooks them
                         * (internet-stack-helper.cc:593-730, every interface): "t" Tx (SendRealOut,
                         * ipv4-l3-protocol.cc:764, the packet with its new IPv4 header), "r" Rx (Receive
                         * :455, as received), "d" Drop (DROP_TTL_EXPIRED :835 — after the time exceeded an
                         * ICMP-enabled node sends —, DROP_NO_ROUTE :505; the received header; a UDP datagram's ipid & 0xffff).
                         * dev: the sending device (Tx), the receiving one (Rx, DROP_NO_ROUTE), the forwarding
                         * route's (DROP_TTL_EXPIRED: IpForward's interface); size: the IPv4 length. */
                        NSGPU_TR_IP_TX = 4, NSGPU_TR_IP_RX = 5, NSGPU_TR_IP_DROP = 6 };
typedef struct nsgpu_trace_record {
  uint64_t ts;    /* Now () of the call (ns) */
  uint32_t uid;   /* uid of the dispatched event that made the call */
  uint16_t seq;   /* call index inside that event */
  uint8_t  kind;  /* nsgpu_trace_kind */
  uint8_t  pad_;
  uint32_t dev;   /* device (its queue) */
  /* the packet as the sink sees it: flow (| NSGPU_PKT_REPLY), IPv4 identification, size in bytes
   * (PPP header included except for MacRx), IPv4 TTL */
  uint32_t app, ipid, size, ttl;
  uint32_t pad2_;
} nsgpu_trace_record;  /* 40 bytes */

enum nsgpu_setup_kind { NSGPU_SETUP_NODE = 0, NSGPU_SETUP_DEVICE = 1, NSGPU_SETUP_APP = 2, NSGPU_SETUP_STOP = 3,
                        NSGPU_SETUP_UID = 4, NSGPU_SETUP_NOOP = 5 };
/* NSGPU_SETUP_NOOP k: ScheduleWithContext (k, 0, <no-op>) — e.g. the LoopbackNetDevice that
 * Ipv4L3Protocol::SetupLoopback adds to every node (ipv4-l3-protocol.cc:227-244 -> node.cc:118). */

/* Counters of a p2p run (both the oracle and the GPU engine fill this). */
typedef struct nsgpu_p2p_stats {
  uint64_t dispatched;        /* RemoveNext calls, setup and cancelled ones included */
  uint64_t cancelled;         /* dispatches of cancelled events */
  uint64_t digest;            /* order-sensitive digest of the (ts, uid) pop order */
  uint64_t final_ts;          /* Now () when Run returned */
  uint32_t next_uid;          /* DefaultSimulatorImpl::m_uid when Run returned */
  uint32_t windows;           /* GPU: parallel dispatch windows (0 for the oracle) */
  uint64_t ttl_drops;
  uint64_t no_route_drops;
  uint64_t max_window;
  uint64_t unreach_drops;     /* UDP datagrams with no bound endpoint */
  uint64_t refits;            /* GPU: windows cut back to the window capacity (0 for the oracle) */
  uint64_t icmp_sent;         /* ICMP errors sent (scenario icmp = 1) */
} nsgpu_p2p_stats;

/* Per-device counters: Queue (queue.cc:61-200) + device. */
typedef struct nsgpu_dev_counters {
  uint32_t enq_packets, enq_bytes;     /* m_nTotalReceivedPackets/Bytes */
  uint32_t drop_packets, drop_bytes;   /* m_nTotalDroppedPackets/Bytes */
  uint32_t deq_packets, tx_packets;    /* Dequeue calls returning a packet; TransmitStart calls */
  uint32_t rx_packets, pad_;           /* PointToPointNetDevice::Receive calls */
} nsgpu_dev_counters;

/* Per-application counters: OnOff sent packets/bytes, PacketSink received packets/bytes. */
typedef struct nsgpu_app_counters {
  uint32_t tx_packets, rx_packets;
  uint64_t tx_bytes, rx_bytes;
} nsgpu_app_counters;

/* Order-sensitive digest of a dispatch sequence: sum over k of mix(k, ts_k, uid_k).
 * Used to compare long dispatch orders (pop order) without moving whole logs. */
NSGPU_HD static inline uint64_t nsgpu_mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
NSGPU_HD static inline uint64_t nsgpu_dispatch_digest_term(uint64_t rank, uint64_t ts, uint32_t uid) {
  return nsgpu_mix64(rank * 0x9e3779b97f4a7c15ULL ^ nsgpu_mix64(ts ^ ((uint64_t)uid << 40) ^ (uint64_t)uid));
}

/* ---------------- Wi-Fi PHY receive subset ----------------
 * YansWifiChannel::Send (yans-wifi-channel.cc:77-115) -> YansWifiChannel::Receive (:117-122) ->
 * YansWifiPhy::StartReceivePacket (yans-wifi-phy.cc:399-496) with its InterferenceHelper
 * (interference-helper.cc:129-212, 365-391) and WifiPhyStateHelper (wifi-phy-state-helper.cc:123-185,
 * 255-322, 392-416), EndReceive's state part (yans-wifi-phy.cc:770-799: NotifyRxEnd + DoSwitchFromRx)
 * and SendPacket's (:499-522).  The scenario is a PHY harness in the style of wifi-test.cc:181-260:
 * every transmission is a SendPacket call scheduled before Run (its uid is a setup uid), so the
 * transmission schedule is an input; the MAC, its DCF and EndReceive's m_random draw stay on the host
 * (SURVEY H13).  Channel switching is not modelled (no SWITCHING state). */
enum nsgpu_wifi_modclass { NSGPU_WIFI_DSSS = 0, NSGPU_WIFI_OFDM = 1, NSGPU_WIFI_ERP_OFDM = 2 };
enum nsgpu_wifi_store { NSGPU_WIFI_STORE_AUTO = 0, NSGPU_WIFI_STORE_LDS = 1, NSGPU_WIFI_STORE_HBM = 2,
                        NSGPU_WIFI_STORE_MASK = 3, NSGPU_WIFI_INLINE_RX = 4, NSGPU_WIFI_UNSORTED_RX = 8 };
enum nsgpu_wifi_preamble { NSGPU_WIFI_PREAMBLE_LONG = 0, NSGPU_WIFI_PREAMBLE_SHORT = 1 };

typedef struct nsgpu_wifi_scenario {
  int64_t n_phy;                /* YansWifiChannel::m_phyList, in Add order */
  const double *x, *y, *z;      /* ConstantPositionMobilityModel positions */
  const uint32_t *channel;      /* GetChannelNumber () */
  const uint32_t *node;         /* context of the Receive events (0xffffffff: no NetDevice) */
  nsgpu_loss_chain loss;
  double speed;                 /* ConstantSpeedPropagationDelayModel Speed */
  double rx_gain_db;            /* YansWifiPhy RxGain (default 1) */
  double ed_threshold_dbm;      /* EnergyDetectionThreshold (default -96) */
  double cca_threshold_dbm;     /* CcaMode1Threshold (default -99) */
  int64_t n_tx;                 /* SendPacket calls, in (ts, uid) order */
  const uint64_t *tx_ts;
  const uint32_t *tx_uid;       /* setup uids: all below uid_start */
  const uint32_t *tx_phy;
  const uint32_t *tx_size;      /* packet->GetSize () at the PHY */
  const double *tx_dbm;         /* GetPowerDbm (txPowerLevel) + TxGain: the channel's txPowerDbm */
  const uint32_t *tx_modclass;  /* the payload WifiMode (wifi-phy.cc:236-301) */
  const uint64_t *tx_rate_bps;
  const uint32_t *tx_bw_hz;
  const uint32_t *tx_preamble;  /* nsgpu_wifi_preamble */
  uint32_t uid_start;           /* DefaultSimulatorImpl::m_uid when Run starts */
  uint32_t ni_cap;              /* NiChanges capacity per phy (GPU); a longer list fails the run */
  uint64_t stop_ts;             /* Simulator::Stop event (ts, uid); stop_ts = ~0: none */
  uint32_t stop_uid;
  uint32_t pad_;
} nsgpu_wifi_scenario;

/* Outcome of one Receive event (StartReceivePacket's switch, yans-wifi-phy.cc:416-478). */
enum nsgpu_wifi_rx_outcome { NSGPU_WIFI_SYNC = 0, NSGPU_WIFI_DROP_RX = 1, NSGPU_WIFI_DROP_TX = 2,
                             NSGPU_WIFI_DROP_ED = 3, NSGPU_WIFI_NOT_RUN = 255 };
#define NSGPU_WIFI_F_CCA_EVAL   1u  /* maybeCcaBusy: GetEnergyDuration (CcaMode1Threshold) evaluated */
#define NSGPU_WIFI_F_CCA_SWITCH 2u  /* ... and non-zero: SwitchMaybeToCcaBusy */
#define NSGPU_WIFI_F_NEAR_ED    4u  /* rxPowerW within 1e-9 (relative) of EnergyDetectionThreshold */
#define NSGPU_WIFI_F_NEAR_CCA   8u  /* a noise+interference sum within 1e-9 of CcaMode1Threshold */

/* One Receive event, at slot [tx * n_phy + phy] (the sender's own slot stays NOT_RUN). */
typedef struct nsgpu_wifi_rx_log {
  uint64_t ts;       /* send time + delay */
  uint32_t uid;      /* uid base of the transmission + rank among the receivers */
  uint8_t outcome;   /* nsgpu_wifi_rx_outcome */
  uint8_t flags;     /* NSGPU_WIFI_F_* */
  uint16_t pad_;
  int64_t cca_ns;    /* GetEnergyDuration result when evaluated, else 0 */
} nsgpu_wifi_rx_log;

/* One EndReceive event (the Simulator::Schedule of a syncing StartReceivePacket, yans-wifi-phy.cc:469-471). */
#define NSGPU_WIFI_END_CANCELLED  1u  /* SendPacket while in Rx cancelled it (:510-514); still dispatched */
#define NSGPU_WIFI_END_DISPATCHED 2u  /* before the Stop event */
typedef struct nsgpu_wifi_end_record {
  uint64_t ts;
  uint64_t sync_ts;  /* the Receive event that synced */
  uint32_t uid;
  uint32_t phy;
  uint32_t tx;       /* transmission index of the packet */
  uint32_t flags;
} nsgpu_wifi_end_record;

typedef struct nsgpu_wifi_phy_counters {
  uint32_t rx, sync, drop_rx, drop_tx, drop_ed, cca_switches, end, end_cancelled;
  uint32_t ni_len;   /* NiChanges length when the run ended */
  uint32_t ni_max;
  int64_t end_tx, end_rx, end_cca_busy;  /* WifiPhyStateHelper m_endTx / m_endRx / m_endCcaBusy */
  double first_power;                    /* InterferenceHelper::m_firstPower */
  uint32_t rxing, pad_;
} nsgpu_wifi_phy_counters;

typedef struct nsgpu_wifi_stats {
  uint64_t dispatched;      /* SendPacket + Receive + EndReceive (+ Stop) dispatches, cancelled ones included */
  uint64_t tx, rx, sync, drop_rx, drop_tx, drop_ed, cca_evals, cca_switches, end, end_cancelled;
  uint64_t ni_inserts;      /* NiChange entries inserted */
  uint64_t near_threshold;  /* Receive events flagged NEAR_ED or NEAR_CCA */
  uint64_t digest;          /* sum of nsgpu_wifi_term over the dispatched events */
  uint64_t final_ts;        /* Now () when Run returned */
  uint32_t next_uid;        /* m_uid when Run returned */
  uint32_t ni_max;
} nsgpu_wifi_stats;

/* Digest term of a dispatched event: SendPacket (0, ts, uid, uid base of its fan-out, 0); Receive
 * (1, ts, tx, phy, outcome | (flags & 3) << 8 | cca_ns << 16); EndReceive (2, ts, uid, phy, cancelled);
 * Stop (3, ts, uid, 0, 0).  A Receive's uid is base + rank, so the SendPacket term pins it. */
NSGPU_HD static inline uint64_t nsgpu_wifi_term(uint64_t kind, uint64_t ts, uint64_t a, uint64_t b, uint64_t c) {
  return nsgpu_mix64(nsgpu_mix64(ts ^ (kind << 60)) + nsgpu_mix64(a * 0x9e3779b97f4a7c15ULL + b) +
                     c * 0xd1b54a32d192ed03ULL);
}

/* ---- closed-loop Wi-Fi PHY (nsgpu_wifil_*, attached to nsgpu_sim: SendPacket from host closures) ---- */
typedef struct nsgpu_wifil_config {
  int64_t n_phy;                /* YansWifiChannel::m_phyList, in Add order */
  const double *x, *y, *z;      /* ConstantPositionMobilityModel positions */
  const uint32_t *channel;      /* GetChannelNumber () */
  const uint32_t *node;         /* context of the Receive / EndReceive events */
  nsgpu_loss_chain loss;
  double speed;                 /* ConstantSpeedPropagationDelayModel Speed */
  double rx_gain_db;            /* YansWifiPhy RxGain (default 1) */
  double ed_threshold_dbm;      /* EnergyDetectionThreshold (default -96) */
  double cca_threshold_dbm;     /* CcaMode1Threshold (default -99) */
  double rx_noise_figure_db;    /* RxNoiseFigure (default 7): InterferenceHelper::SetNoiseFigure (DbToRatio) */
  uint32_t error_model;         /* nsgpu_wifil_error_model */
  uint32_t ni_cap;              /* NiChanges entries per phy (power of two); a longer list fails the run */
  uint32_t rxq_cap;             /* pending Receive events per phy (power of two) */
  uint32_t pad_;
  uint64_t tx_cap;              /* SendPacket calls over the run */
} nsgpu_wifil_config;
enum nsgpu_wifil_error_model { NSGPU_WIFIL_NIST = 0, NSGPU_WIFIL_YANS = 1 };  /* (YansWifiPhyHelper::Default: Nist) */

/* One EndReceive (yans-wifi-phy.cc:770-799): InterferenceHelper::CalculateSnrPer's result, for the host's
 * m_random draw (a cancelled one carries no snr / per). */
typedef struct nsgpu_wifil_end {
  uint64_t ts;
  uint32_t uid, phy;
  double snr, per;
  uint32_t tx;     /* the transmission (SendPacket call) it receives */
  uint32_t flags;  /* NSGPU_WIFI_END_CANCELLED */
  double rx_w;     /* the event's received power (InterferenceHelper::Event::GetRxPowerW): with snr, the
                    * MonitorSnifferRx signal / noise dBm of an Ok reception (yans-wifi-phy.cc:788-789) */
} nsgpu_wifil_end;

/* WifiPhyStateHelper of one phy at Now (wifi-phy-state-helper.cc:159-183). */
enum nsgpu_wifil_state { NSGPU_WIFIL_IDLE = 0, NSGPU_WIFIL_RX = 1, NSGPU_WIFIL_TX = 2, NSGPU_WIFIL_CCA_BUSY = 3 };
typedef struct nsgpu_wifil_phy_state {
  uint32_t state;  /* nsgpu_wifil_state */
  uint32_t rxing;
  int64_t end_tx, end_rx, end_cca_busy;
  int64_t delay_until_idle;  /* GetDelayUntilIdle (:122-151) */
} nsgpu_wifil_phy_state;

#ifdef __cplusplus
}
#endif
#endif /* NSGPU_TYPES_H */
