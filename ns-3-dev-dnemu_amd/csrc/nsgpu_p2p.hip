// nsgpu_p2p.hip — GPU-resident point-to-point / DropTail / IPv4-forward / UDP subset (configs 2, 4).
//
// Event semantics follow the reference code line by line (restated independently in
// oracle/nsref_p2p.cc, which is the parity checker):
//   setup      node-list.cc:124-131, node.cc:111-145,183-199, application.cc:87-95
//   OnOff      onoff-application.cc:132-252      PacketSink: no events
//   device     point-to-point-net-device.cc:206-269,304-346,462-518; point-to-point-channel.cc:82-103
//   queue      queue.cc:61-200, drop-tail-queue.cc:83-132
//   IPv4/UDP   ipv4-l3-protocol.cc:434-537,815-841 (static next-hop routes, TTL)
//
// Engine (MI355X).  The simulation advances in conservative windows; each window is a fixed pipeline
// of short multi-CU kernels (a CU is 64 lanes per clock, so no phase may live on one CU), replayed
// from a hipGraph of NWIN windows until the device-side `done` flag is set:
//   k_reduce     W_end = min over pending e of (ts_e + L(kind_e)), L = the smallest delay any child of
//                that kind of handler can have: DefaultSimulatorImpl's uids make a child sort after every
//                pending event with ts <= its own, so every pending event with ts <= W_end is safe;
//   k_partition  window keys ((ts - tmin) << 32 | uid, capped at the Simulator::Stop key) -> window
//                list, the rest -> the other pool buffer (wave-aggregated atomic slots);
//   k_refit      only when the window overflowed WCAP: bisection for the largest key prefix that fits
//                (a key prefix of a safe window is safe), single workgroup;
//   k_rank       dispatch rank of every window key by tiled all-pairs counting (WCAP^2 / 256 CUs);
//   k_scatter    rank order; per-node chains through node_head (one atomicExch per event);
//   k_handle     the chain holder of each node runs that node's events in rank order, so node state
//                (device tx state, DropTail rings, OnOff state, sink counters) needs no atomics;
//                children go to per-rank slots in Schedule-call order;
//   k_scan       exclusive scans of child counts in rank order (uids), run bookkeeping;
//   k_append     digest/log of the dispatch order, children -> pool with the uids DefaultSimulatorImpl
//                would assign.
#include "nsgpu_device.h"
#include "nsgpu_internal.h"

namespace nsgpu {

enum EvKind : uint32_t {
  K_NODE_START = 1,     // Node::Start (setup)
  K_DEV_START = 2,      // NetDevice::Start (setup, no-op: started by Node::Start)
  K_APPOBJ_START = 3,   // Application::Start (setup)
  K_APP_START = 4,      // Application::StartApplication
  K_APP_STOP = 5,       // Application::StopApplication
  K_START_SENDING = 6,  // OnOffApplication::StartSending   (gen in bits 8..31)
  K_STOP_SENDING = 7,   // OnOffApplication::StopSending    (gen)
  K_SEND = 8,           // OnOffApplication::SendPacket     (gen)
  K_TX_COMPLETE = 9,    // PointToPointNetDevice::TransmitComplete
  K_RECEIVE = 10,       // PointToPointNetDevice::Receive
  K_STOP = 11,          // Simulator::Stop
  K_FWD_UP = 12,        // Ipv4EndPoint::DoForwardUp -> UdpSocketImpl::ForwardUp -> PacketSink (zero-delay leaf)
  K_NKINDS = 13
};

constexpr int WCAP = 4096;       // events per window
constexpr int TB = 256;          // threads per block, pool sweeps and k_rank
constexpr int RB = 64;           // threads per block, per-rank kernels (spread over CUs)
constexpr int NT = WCAP / TB;    // rank tiles per side
constexpr int GRID_POOL = 256;   // blocks of the pool sweeps (grid-stride)
constexpr int SCAN_THREADS = 1024;
constexpr int CH = 16;           // chain entries a handler thread sorts in LDS
constexpr int NWIN = 32;         // windows per graph replay
constexpr uint32_t NOCTX = 0xffffffffu;
constexpr uint32_t NOCHAIN = 0xffffffffu;

struct Pkt {
  uint32_t app, seq, size, ttl;
};

// Device-resident run control (one per engine); every field is written by one kernel of the window
// pipeline and read by later ones, never read and written by different blocks of one kernel except
// through atomics.
struct Ctl {
  uint64_t P;                  // pending events in pool `cur`
  uint64_t K;                  // dispatched so far
  uint64_t tmin, wend, stopts; // window reduction (atomicMin); ~0 between windows
  uint64_t bound, span, inline_lim;
  uint64_t windows, max_window, last_ts, max_windows;
  uint64_t digest, cancelled, ttl_drops, no_route, unreach;
  uint64_t K0, tmin0, inline_lim0;  // the window k_append works on (set by k_scan)
  uint32_t uid, cur, W, nxtP, overflow, done, stop_seen, scan_ran;
  uint32_t stopuid, uid0, W0, Pbase, total_children, total_inline, pad0, pad1;
};

// Device-resident model + engine state (all pointers are HBM).
struct P2PDev {
  // scenario
  uint32_t n_nodes, n_devices, n_apps, n_dst, qcap, maxc;
  const uint32_t *dev_node, *dev_peer, *dev_qmax;
  const uint64_t *dev_bps;
  const int64_t *dev_ifg, *dev_delay;
  const uint32_t *route;
  const uint32_t *app_kind, *app_node, *app_dst_node, *app_dst_slot, *app_pkt_size, *app_max_bytes, *app_ttl;
  const int64_t *app_start, *app_stop;
  const uint64_t *app_rate;
  const double *app_on_s, *app_off_s;
  const uint32_t *node_app_off, *node_app_list;  // CSR: apps of each node in AddApplication order
  int64_t lookahead[K_NKINDS];
  // model state
  uint32_t *dev_busy, *q_head, *q_count;
  Pkt *q_buf;
  nsgpu_dev_counters *devc;
  uint32_t *app_flags;    // bit0 started, bit1 sink active, bit2 send live, bit3 start/stop live
  uint32_t *app_send_gen, *app_ss_gen, *app_residual, *app_tot, *app_seq;
  uint64_t *app_last_start;
  nsgpu_app_counters *appc;
  // event pools (double-buffered SoA)
  uint64_t *ev_ts[2];
  uint32_t *ev_uid[2], *ev_ctx[2], *ev_kind[2], *ev_a[2];
  Pkt *ev_pkt[2];
  uint64_t pool_cap;
  // the window (WCAP entries each): partition order (w*), rank order (s*, link, counts, prefixes)
  uint64_t *wkey, *skey;
  uint32_t *wpi, *wrank, *spi, *sctx, *link, *nchild, *ninl, *cpref, *ipref, *gbnd;
  uint32_t *node_head;  // per-node chain head of the current window (NOCHAIN between windows)
  // children of the current window: slot = rank * maxc + j
  uint64_t *ch_ts;
  uint32_t *ch_ctx, *ch_kind, *ch_a;
  Pkt *ch_pkt;
  // run control / outputs
  uint32_t n_init;    // initial pending count (pool 0)
  uint32_t uid_init;  // m_uid after setup
  Ctl *C;
  uint32_t *error;  // non-zero = capacity exceeded (code)
  uint64_t *log_ts;
  uint32_t *log_uid, *log_ctx;
  uint64_t log_cap;
};

// ---------------- wave / block helpers ----------------
__device__ __forceinline__ uint64_t wave_min64(uint64_t v) {
  for (int o = 32; o > 0; o >>= 1) {
    uint64_t w = __shfl_xor(v, o);
    v = w < v ? w : v;
  }
  return v;
}
__device__ __forceinline__ uint64_t wave_max64(uint64_t v) {
  for (int o = 32; o > 0; o >>= 1) {
    uint64_t w = __shfl_xor(v, o);
    v = w > v ? w : v;
  }
  return v;
}
__device__ __forceinline__ uint32_t wave_sum32(uint32_t v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ uint32_t wave_exscan32(uint32_t v, int lane) {
  uint32_t inc = v;
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t w = __shfl_up(inc, o);
    if (lane >= o) inc += w;
  }
  return inc - v;
}
// Block exclusive scan of one value per thread (NTH threads); *total = block sum.
template <int NTH>
__device__ __forceinline__ uint32_t block_exscan(uint32_t v, uint32_t *wsum, uint32_t *total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint32_t ex = wave_exscan32(v, lane);
  if (lane == 63) wsum[wid] = ex + v;
  __syncthreads();
  uint32_t off = 0, tot = 0;
  for (int w = 0; w < NTH / 64; w++) {
    const uint32_t s = wsum[w];
    off += w < wid ? s : 0;
    tot += s;
  }
  __syncthreads();
  *total = tot;
  return off + ex;
}

// ---------------- model (runs on the thread that owns the event's node) ----------------
struct Emit {
  const P2PDev *M;
  uint64_t now;
  uint32_t ctx;
  uint32_t slot0;  // rank * maxc
  uint32_t n;
  __device__ void child(int64_t delay, uint32_t ctx_, uint32_t kind, uint32_t a, Pkt p) {
    const uint32_t s = slot0 + n++;
    M->ch_ts[s] = now + (uint64_t)delay;
    M->ch_ctx[s] = ctx_;
    M->ch_kind[s] = kind;
    M->ch_a[s] = a;
    M->ch_pkt[s] = p;
  }
};

__device__ __forceinline__ int64_t tx_time(const P2PDev &M, uint32_t d, uint32_t size) {
  // Seconds (m_bps.CalculateTxTime (size)): static_cast<double>(bytes)*8/m_bps (data-rate.cc:224-227)
  return seconds_to_ts(static_cast<double>(size) * 8 / (double)M.dev_bps[d]);
}

__device__ void transmit_start(const P2PDev &M, Emit &E, uint32_t d, const Pkt &p) {
  M.dev_busy[d] = 1;
  M.devc[d].tx_packets++;
  const int64_t txTime = tx_time(M, d, p.size);
  E.child(txTime + M.dev_ifg[d], E.ctx, K_TX_COMPLETE, d, Pkt{0, 0, 0, 0});  // Schedule (txCompleteTime)
  const uint32_t peer = M.dev_peer[d];
  E.child(txTime + M.dev_delay[d], M.dev_node[peer], K_RECEIVE, peer, p);   // channel ScheduleWithContext
}

__device__ bool enqueue(const P2PDev &M, uint32_t d, const Pkt &p) {
  const uint32_t cnt = M.q_count[d];
  if (cnt >= M.dev_qmax[d]) {
    M.devc[d].drop_packets++;
    M.devc[d].drop_bytes += p.size;
    return false;
  }
  const uint32_t pos = (M.q_head[d] + cnt) % M.qcap;
  M.q_buf[(uint64_t)d * M.qcap + pos] = p;
  M.q_count[d] = cnt + 1;
  M.devc[d].enq_packets++;
  M.devc[d].enq_bytes += p.size;
  return true;
}

__device__ bool dequeue(const P2PDev &M, uint32_t d, Pkt &out) {
  const uint32_t cnt = M.q_count[d];
  if (cnt == 0) return false;
  const uint32_t h = M.q_head[d];
  out = M.q_buf[(uint64_t)d * M.qcap + h];
  M.q_head[d] = (h + 1) % M.qcap;
  M.q_count[d] = cnt - 1;
  M.devc[d].deq_packets++;
  return true;
}

__device__ void device_send(const P2PDev &M, Emit &E, uint32_t d, Pkt p) {
  p.size += 2;  // PppHeader
  if (M.dev_busy[d] == 0) {
    if (enqueue(M, d, p)) {
      Pkt q;
      dequeue(M, d, q);
      transmit_start(M, E, d, q);
    }
  } else {
    enqueue(M, d, p);
  }
}

__device__ void ip_send(const P2PDev &M, Emit &E, uint32_t n, const Pkt &p, uint64_t *no_route) {
  const uint32_t out = M.route[(uint64_t)n * M.n_dst + M.app_dst_slot[p.app]];
  if (out == 0xffffffffu) {
    (*no_route)++;
    return;
  }
  device_send(M, E, out, p);
}

__device__ void ip_receive(const P2PDev &M, Emit &E, uint32_t n, Pkt p, int32_t sink, uint64_t *ttl_drops,
                           uint64_t *no_route, uint64_t *unreach) {
  if (M.app_dst_node[p.app] == n) {  // LocalDeliver -> UdpL4Protocol::Receive (udp-l4-protocol.cc:312-407)
    if (sink < 0 || !(M.app_flags[sink] & 2u)) {  // no bound endpoint: RX_ENDPOINT_UNREACH
      (*unreach)++;
      return;
    }
    // Ipv4EndPoint::ForwardUp: ScheduleNow (&Ipv4EndPoint::DoForwardUp) (ipv4-end-point.cc:112-120)
    E.child(0, E.ctx, K_FWD_UP, (uint32_t)sink, p);
    return;
  }
  const uint32_t out = M.route[(uint64_t)n * M.n_dst + M.app_dst_slot[p.app]];
  if (out == 0xffffffffu) {
    (*no_route)++;
    return;
  }
  p.ttl -= 1;  // IpForward
  if (p.ttl == 0) {
    (*ttl_drops)++;
    return;
  }
  device_send(M, E, out, p);
}

// int64x64 residual-bits update of OnOffApplication::CancelEvents (onoff-application.cc:170-173):
// bits = (delta.To (Time::S) * GetBitRate ()).GetHigh (); To(S) = int64x64 (delta) MulByInvert Invert (1e9).
__device__ __forceinline__ u128 umul_by_invert(u128 a, u128 b) {
  const u128 LO = (((u128)1) << 64) - 1;
  u128 ah = a >> 64, bh = b >> 64, al = a & LO, bl = b & LO;
  u128 hi = ah * bh;
  u128 mid = ah * bl + al * bh;
  mid >>= 64;
  return hi + mid;
}
__device__ __forceinline__ u128 divu(u128 a, u128 b) {
  u128 quo = a / b;
  u128 rem = a % b;
  u128 result = quo << 64;
  u128 tmp = rem >> 64;
  u128 div;
  if (tmp == 0) {
    rem = rem << 64;
    div = b;
  } else {
    div = b >> 64;
  }
  quo = rem / div;
  return result + quo;
}
__device__ int64_t residual_bits(int64_t delta_ns, uint64_t rate) {
  // Invert (1e9) (int64x64-128.cc:119-134)
  u128 one = ((u128)1) << 64;
  i128 inv = (i128)divu(one, (u128)1000000000ull);
  {
    i128 tmp = ((i128)1000000000ll) << 64;
    u128 r = umul_by_invert((u128)tmp, (u128)inv);
    if ((int64_t)(r >> 64) != 1) inv += 1;
  }
  // MulByInvert (delta)
  i128 v = ((i128)delta_ns) << 64;
  bool neg = v < 0;
  u128 a = neg ? (u128)(-v) : (u128)v;
  u128 t = umul_by_invert(a, (u128)inv);
  i128 ts = neg ? -(i128)t : (i128)t;
  // Mul by int64x64_t (rate): Umul with the '|=' combine (int64x64-128.cc:20-57)
  i128 rb = ((i128)rate) << 64;
  bool negA = ts < 0;
  u128 ua = negA ? (u128)(-ts) : (u128)ts, ub = (u128)rb;
  const u128 LO = (((u128)1) << 64) - 1;
  u128 aL = ua & LO, bL = ub & LO, aH = (ua >> 64) & LO, bH = (ub >> 64) & LO;
  u128 loPart = aL * bL;
  u128 midPart = aL * bH + aH * bL;
  u128 res = (loPart >> 64) + (midPart & LO);
  u128 hiPart = aH * bH;
  res |= ((hiPart & LO) << 64) + (midPart & ~LO);
  i128 r = negA ? -(i128)res : (i128)res;
  bool rn = r < 0;
  i128 x = rn ? -r : r;
  x >>= 64;
  int64_t h = (int64_t)x;
  return rn ? -h : h;
}

__device__ void cancel_events(const P2PDev &M, uint32_t a, uint64_t now) {
  uint32_t f = M.app_flags[a];
  if (f & 4u) {  // m_sendEvent.IsRunning ()
    const int64_t delta = (int64_t)now - (int64_t)M.app_last_start[a];
    M.app_residual[a] += (uint32_t)residual_bits(delta, M.app_rate[a]);
  }
  M.app_flags[a] = f & ~(4u | 8u);  // Cancel (m_sendEvent); Cancel (m_startStopEvent)
}

__device__ void schedule_start_event(const P2PDev &M, Emit &E, uint32_t a) {
  const uint32_t g = (M.app_ss_gen[a] + 1) & 0xffffffu;
  M.app_ss_gen[a] = g;
  M.app_flags[a] |= 8u;
  E.child(seconds_to_ts(M.app_off_s[a]), E.ctx, K_START_SENDING | (g << 8), a, Pkt{0, 0, 0, 0});
}
__device__ void schedule_stop_event(const P2PDev &M, Emit &E, uint32_t a) {
  const uint32_t g = (M.app_ss_gen[a] + 1) & 0xffffffu;
  M.app_ss_gen[a] = g;
  M.app_flags[a] |= 8u;
  E.child(seconds_to_ts(M.app_on_s[a]), E.ctx, K_STOP_SENDING | (g << 8), a, Pkt{0, 0, 0, 0});
}
__device__ void stop_application(const P2PDev &M, uint32_t a, uint64_t now) {
  if (M.app_kind[a] == NSGPU_APP_SINK) {
    M.app_flags[a] &= ~2u;
    return;
  }
  cancel_events(M, a, now);
}
__device__ void schedule_next_tx(const P2PDev &M, Emit &E, uint32_t a) {
  const uint32_t maxb = M.app_max_bytes[a];
  if (maxb == 0 || M.app_tot[a] < maxb) {
    const uint32_t bits = M.app_pkt_size[a] * 8 - M.app_residual[a];
    const int64_t next = seconds_to_ts(bits / static_cast<double>(M.app_rate[a]));
    const uint32_t g = (M.app_send_gen[a] + 1) & 0xffffffu;
    M.app_send_gen[a] = g;
    M.app_flags[a] |= 4u;
    E.child(next, E.ctx, K_SEND | (g << 8), a, Pkt{0, 0, 0, 0});
  } else {
    stop_application(M, a, E.now);
  }
}
__device__ void appobj_start(const P2PDev &M, Emit &E, uint32_t a) {  // Application::DoStart
  uint32_t f = M.app_flags[a];
  if (f & 1u) return;
  M.app_flags[a] = f | 1u;
  E.child(M.app_start[a], E.ctx, K_APP_START, a, Pkt{0, 0, 0, 0});
  if (M.app_stop[a] != 0) E.child(M.app_stop[a], E.ctx, K_APP_STOP, a, Pkt{0, 0, 0, 0});
}

// Runs one event; returns true if it was a cancelled dispatch.
__device__ __noinline__ bool run_event(const P2PDev &M, Emit &E, uint32_t kind_word, uint32_t a, const Pkt &pkt, int32_t sink,
                          uint64_t *ttl_drops, uint64_t *no_route, uint64_t *unreach, bool *stop) {
  const uint32_t kind = kind_word & 0xffu;
  const uint32_t gen = kind_word >> 8;
  switch (kind) {
    case K_NODE_START: {
      for (uint32_t i = M.node_app_off[a]; i < M.node_app_off[a + 1]; i++) appobj_start(M, E, M.node_app_list[i]);
      return false;
    }
    case K_DEV_START:
      return false;
    case K_APPOBJ_START:
      appobj_start(M, E, a);
      return false;
    case K_APP_START:
      if (M.app_kind[a] == NSGPU_APP_SINK) {
        M.app_flags[a] |= 2u;
      } else {
        cancel_events(M, a, E.now);
        schedule_start_event(M, E, a);
      }
      return false;
    case K_APP_STOP:
      stop_application(M, a, E.now);
      return false;
    case K_START_SENDING: {
      const uint32_t f = M.app_flags[a];
      if (!((f & 8u) && M.app_ss_gen[a] == gen)) return true;  // cancelled
      M.app_flags[a] = f & ~8u;
      M.app_last_start[a] = E.now;
      schedule_next_tx(M, E, a);
      schedule_stop_event(M, E, a);
      return false;
    }
    case K_STOP_SENDING: {
      const uint32_t f = M.app_flags[a];
      if (!((f & 8u) && M.app_ss_gen[a] == gen)) return true;
      M.app_flags[a] = f & ~8u;
      cancel_events(M, a, E.now);
      schedule_start_event(M, E, a);
      return false;
    }
    case K_SEND: {
      const uint32_t f = M.app_flags[a];
      if (!((f & 4u) && M.app_send_gen[a] == gen)) return true;
      M.app_flags[a] = f & ~4u;
      const uint32_t sz = M.app_pkt_size[a];
      Pkt p{a, M.app_seq[a]++, sz + 8 + 20, M.app_ttl[a]};
      M.appc[a].tx_packets++;
      M.appc[a].tx_bytes += sz;
      ip_send(M, E, M.app_node[a], p, no_route);
      M.app_tot[a] += sz;
      M.app_last_start[a] = E.now;
      M.app_residual[a] = 0;
      schedule_next_tx(M, E, a);
      return false;
    }
    case K_TX_COMPLETE: {
      M.dev_busy[a] = 0;
      Pkt p;
      if (dequeue(M, a, p)) transmit_start(M, E, a, p);
      return false;
    }
    case K_RECEIVE: {
      M.devc[a].rx_packets++;
      Pkt p = pkt;
      p.size -= 2;
      ip_receive(M, E, M.dev_node[a], p, sink, ttl_drops, no_route, unreach);
      return false;
    }
    case K_FWD_UP:  // DoForwardUp -> UdpSocketImpl::ForwardUp -> PacketSink::HandleRead (a = sink app)
      if (M.app_flags[a] & 2u) {
        M.appc[a].rx_packets++;
        M.appc[a].rx_bytes += pkt.size - 28;
      }
      return false;
    case K_STOP:
      *stop = true;
      return false;
    default:
      return false;
  }
}

// ================================ window pipeline ================================
// Window bound from the reduction: packed key bound, span, Stop key (shared by k_partition/k_refit).
struct WinBound {
  uint64_t tmin, span, bound, stop_packed;
};
__device__ __forceinline__ WinBound window_bound(const Ctl &C) {
  WinBound b;
  b.tmin = C.tmin;
  uint64_t span = C.wend - b.tmin;
  if (span > 0xfffffffeull) span = 0xfffffffeull;
  b.span = span;
  b.bound = (span << 32) | 0xffffffffull;
  b.stop_packed = ~0ull;
  if (C.stopts != ~0ull && C.stopts - b.tmin <= span) {
    // Stop caps the window at its own key (it is dispatched; later events are not)
    b.stop_packed = ((C.stopts - b.tmin) << 32) | C.stopuid;
    b.bound = b.stop_packed < b.bound ? b.stop_packed : b.bound;
  }
  return b;
}
__device__ __forceinline__ void publish_bound(Ctl &C, const WinBound &b) {
  C.bound = b.bound;
  C.span = b.span;
  // zero-delay leaf children (Ipv4EndPoint::DoForwardUp) run inside the window; when the window ends
  // at the Stop event, those at the Stop's ts sort after it and are never dispatched
  const bool has_stop = b.stop_packed != ~0ull && b.bound >= b.stop_packed;
  C.inline_lim = has_stop ? (b.stop_packed >> 32) : ~0ull;
}

// ---- k_reduce: tmin, W_end, the pending Stop ----
__global__ __launch_bounds__(TB) void k_reduce(const P2PDev *__restrict__ Mp) {
  const P2PDev &M = *Mp;
  Ctl &C = *M.C;
  if (blockIdx.x == 0 && threadIdx.x == 0) C.scan_ran = 0;
  if (C.done) return;
  const uint64_t P = C.P;
  const int cur = C.cur;
  const uint64_t *ts = M.ev_ts[cur];
  const uint32_t *kindv = M.ev_kind[cur];
  uint64_t tmin = ~0ull, wend = ~0ull;
  for (uint64_t i = (uint64_t)blockIdx.x * TB + threadIdx.x; i < P; i += (uint64_t)gridDim.x * TB) {
    const uint64_t t = ts[i];
    const uint32_t k = kindv[i] & 0xffu;
    tmin = t < tmin ? t : tmin;
    const uint64_t e = t + (uint64_t)M.lookahead[k];
    wend = e < wend ? e : wend;
    if (k == K_STOP) {  // at most one Stop event is pending
      C.stopts = t;
      C.stopuid = M.ev_uid[cur][i];
    }
  }
  __shared__ uint64_t s0[TB / 64], s1[TB / 64];
  tmin = wave_min64(tmin);
  wend = wave_min64(wend);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    s0[wid] = tmin;
    s1[wid] = wend;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < TB / 64; w++) {
      tmin = s0[w] < tmin ? s0[w] : tmin;
      wend = s1[w] < wend ? s1[w] : wend;
    }
    if (tmin != ~0ull) atomicMin((unsigned long long *)&C.tmin, (unsigned long long)tmin);
    if (wend != ~0ull) atomicMin((unsigned long long *)&C.wend, (unsigned long long)wend);
  }
}

// Classifies pool entry i against the window bound and moves it: window -> (wkey, wpi) list,
// otherwise -> the other pool buffer.  All 64 lanes of the wave must call it (ballots).
__device__ __forceinline__ void partition_one(const P2PDev &M, Ctl &C, const WinBound &b, int cur, uint64_t i,
                                              bool valid) {
  const int lane = threadIdx.x & 63;
  uint64_t t = 0, pk = 0;
  bool in = false;
  if (valid) {
    t = M.ev_ts[cur][i];
    pk = ((t - b.tmin) << 32) | M.ev_uid[cur][i];
    in = (t - b.tmin <= b.span) && pk <= b.bound;
  }
  const uint64_t bin = __ballot(valid && in), bout = __ballot(valid && !in);
  uint32_t basein = 0, baseout = 0;
  if (lane == 0) {
    if (bin) basein = atomicAdd(&C.W, (uint32_t)__popcll(bin));
    if (bout) baseout = atomicAdd(&C.nxtP, (uint32_t)__popcll(bout));
  }
  basein = __shfl(basein, 0);
  baseout = __shfl(baseout, 0);
  const uint64_t below = (1ull << lane) - 1ull;
  if (valid && in) {
    const uint32_t slot = basein + (uint32_t)__popcll(bin & below);
    if (slot < (uint32_t)WCAP) {
      M.wkey[slot] = pk;
      M.wpi[slot] = (uint32_t)i;
    } else {
      C.overflow = 1;
    }
  } else if (valid) {
    const uint64_t o = baseout + (uint64_t)__popcll(bout & below);
    const int nxt = cur ^ 1;
    if (o < M.pool_cap) {
      M.ev_ts[nxt][o] = t;
      M.ev_uid[nxt][o] = M.ev_uid[cur][i];
      M.ev_ctx[nxt][o] = M.ev_ctx[cur][i];
      M.ev_kind[nxt][o] = M.ev_kind[cur][i];
      M.ev_a[nxt][o] = M.ev_a[cur][i];
      M.ev_pkt[nxt][o] = M.ev_pkt[cur][i];
    } else {
      atomicOr(M.error, 1u);
    }
  }
}

// ---- k_partition ----
__global__ __launch_bounds__(TB) void k_partition(const P2PDev *__restrict__ Mp) {
  const P2PDev &M = *Mp;
  Ctl &C = *M.C;
  if (C.done) return;
  const WinBound b = window_bound(C);
  if (blockIdx.x == 0 && threadIdx.x == 0) publish_bound(C, b);
  const uint64_t P = C.P;
  const int cur = C.cur;
  for (uint64_t i0 = (uint64_t)blockIdx.x * TB; i0 < P; i0 += (uint64_t)gridDim.x * TB) {
    const uint64_t i = i0 + threadIdx.x;
    partition_one(M, C, b, cur, i, i < P);
  }
}

// ---- k_refit: the window overflowed WCAP; cut it to the largest key prefix that fits ----
__global__ __launch_bounds__(SCAN_THREADS) void k_refit(const P2PDev *__restrict__ Mp) {
  const P2PDev &M = *Mp;
  Ctl &C = *M.C;
  if (C.done || !C.overflow) return;
  __shared__ uint32_t wc[SCAN_THREADS / 64];
  WinBound b = window_bound(C);
  const uint64_t P = C.P;
  const int cur = C.cur;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  auto count_le = [&](uint64_t bnd) -> uint32_t {
    uint32_t c = 0;
    for (uint64_t i = threadIdx.x; i < P; i += SCAN_THREADS) {
      const uint64_t t = M.ev_ts[cur][i];
      if (t - b.tmin <= b.span) c += ((((t - b.tmin) << 32) | M.ev_uid[cur][i]) <= bnd);
    }
    c = wave_sum32(c);
    if (lane == 0) wc[wid] = c;
    __syncthreads();
    uint32_t tot = 0;
    for (int w = 0; w < SCAN_THREADS / 64; w++) tot += wc[w];
    __syncthreads();
    return tot;
  };
  uint64_t lo_b = 0, hi_b = b.bound;  // count (hi_b) > WCAP
  while (hi_b - lo_b > 1) {
    const uint64_t mid = lo_b + (hi_b - lo_b) / 2;
    if (count_le(mid) <= (uint32_t)WCAP) lo_b = mid;
    else hi_b = mid;
  }
  b.bound = lo_b;
  __syncthreads();
  if (threadIdx.x == 0) {
    C.W = 0;
    C.nxtP = 0;
    C.overflow = 0;
    publish_bound(C, b);
  }
  __syncthreads();
  for (uint64_t i0 = 0; i0 < P; i0 += SCAN_THREADS) {
    const uint64_t i = i0 + threadIdx.x;
    partition_one(M, C, b, cur, i, i < P);
  }
}

// ---- k_rank: rank of each window key = # of smaller keys (keys are distinct: uids) ----
__global__ __launch_bounds__(TB) void k_rank(const P2PDev *__restrict__ Mp) {
  const P2PDev &M = *Mp;
  const Ctl &C = *M.C;
  if (C.done) return;
  const uint32_t W = C.W;
  const uint32_t ti = blockIdx.x / NT, tj = blockIdx.x % NT;
  if (ti * TB >= W || tj * TB >= W) return;
  __shared__ uint64_t tk[TB];
  const uint32_t j = tj * TB + threadIdx.x;
  tk[threadIdx.x] = j < W ? M.wkey[j] : ~0ull;
  __syncthreads();
  const uint32_t i = ti * TB + threadIdx.x;
  if (i >= W) return;
  const uint64_t x = M.wkey[i];
  uint32_t c = 0;
#pragma unroll 16
  for (int y = 0; y < TB; y++) c += tk[y] < x;
  if (c) atomicAdd(&M.wrank[i], c);
}

// ---- k_scatter: rank order; per-node chains ----
__global__ __launch_bounds__(RB) void k_scatter(const P2PDev *__restrict__ Mp) {
  const P2PDev &M = *Mp;
  const Ctl &C = *M.C;
  if (C.done) return;
  const uint32_t i = blockIdx.x * RB + threadIdx.x;
  if (i >= C.W) return;
  const uint32_t r = M.wrank[i];
  M.wrank[i] = 0;
  const uint32_t pi = M.wpi[i];
  M.skey[r] = M.wkey[i];
  M.spi[r] = pi;
  const uint32_t c = M.ev_ctx[C.cur][pi];
  M.sctx[r] = c;
  M.link[r] = c < M.n_nodes ? atomicExch(&M.node_head[c], r) : NOCHAIN;
}

// ---- k_handle: the node's last exchanger runs the node's chain in rank order ----
// Zero-delay leaf children (K_FWD_UP: Ipv4EndPoint::DoForwardUp, ipv4-end-point.cc:112-120) run at
// their key position: after the node's events with ts <= theirs, before the first with a larger ts.
__global__ __launch_bounds__(RB) void k_handle(const P2PDev *__restrict__ Mp,
                                               const int32_t *__restrict__ sink_of_node) {
  const P2PDev &M = *Mp;
  Ctl &C = *M.C;
  if (C.done) return;
  const uint32_t W = C.W;
  const uint32_t r0 = blockIdx.x * RB + threadIdx.x;
  if (r0 >= W) return;
  const uint32_t c = M.sctx[r0];
  if (c < M.n_nodes) {
    if (M.node_head[c] != r0) return;  // not the chain holder
    M.node_head[c] = NOCHAIN;
  }
  __shared__ uint32_t chs[RB * CH];
  uint32_t *my = &chs[threadIdx.x * CH];
  uint32_t n = 0;
  for (uint32_t x = r0; x != NOCHAIN; x = M.link[x]) {
    if (n < (uint32_t)CH) my[n] = x;
    n++;
  }
  const bool small = n <= (uint32_t)CH;
  if (small)
    for (uint32_t a = 1; a < n; a++) {  // insertion sort: ascending rank
      const uint32_t v = my[a];
      uint32_t b = a;
      while (b > 0 && my[b - 1] > v) {
        my[b] = my[b - 1];
        b--;
      }
      my[b] = v;
    }
  const uint64_t tmin = C.tmin;
  const uint64_t inline_lim = C.inline_lim;
  const int cur = C.cur;
  const int32_t sink = c < M.n_nodes ? sink_of_node[c] : -1;
  uint64_t cancelled = 0, ttl_drops = 0, no_route = 0, unreach = 0;
  bool stop = false;
  int64_t last = -1;
  uint32_t ts0_it = 0, pending = 0;
  uint64_t cur_rel = 0;
  auto rank_at = [&](uint32_t it) -> uint32_t {
    if (small) return my[it];
    uint32_t best = NOCHAIN;  // it-th smallest: the smallest rank above `last`
    for (uint32_t x = r0; x != NOCHAIN; x = M.link[x])
      if ((int64_t)x > last && x < best) best = x;
    return best;
  };
  for (uint32_t it = 0; it <= n; it++) {
    const uint32_t r = it < n ? rank_at(it) : NOCHAIN;
    const uint64_t rel = it < n ? (M.skey[r] >> 32) : ~0ull;
    if (it > 0 && rel > cur_rel && pending) {
      // flush the inline children of this node's events at cur_rel (chain positions [ts0_it, it))
      for (uint32_t jt = ts0_it; jt < it; jt++) {
        const uint32_t x = small ? my[jt] : NOCHAIN;
        uint32_t xr = x;
        if (!small) {  // recover the jt-th rank by selection (long chains only)
          int64_t lst = -1;
          for (uint32_t s = 0; s <= jt; s++) {
            uint32_t best = NOCHAIN;
            for (uint32_t y = r0; y != NOCHAIN; y = M.link[y])
              if ((int64_t)y > lst && y < best) best = y;
            lst = best;
          }
          xr = (uint32_t)lst;
        }
        const uint32_t ncr = M.nchild[xr];
        for (uint32_t j = 0; j < ncr; j++) {
          const uint32_t sl = xr * M.maxc + j;
          if ((M.ch_kind[sl] & 0xffu) != K_FWD_UP) continue;
          Emit E0;
          E0.M = &M;
          E0.now = tmin + cur_rel;
          E0.ctx = c;
          E0.slot0 = 0;
          E0.n = 0;
          bool st0 = false;
          run_event(M, E0, M.ch_kind[sl], M.ch_a[sl], M.ch_pkt[sl], sink, &ttl_drops, &no_route, &unreach, &st0);
        }
      }
      pending = 0;
    }
    if (it == n) break;
    if (it == 0 || rel > cur_rel) {
      ts0_it = it;
      cur_rel = rel;
    }
    const uint32_t pi = M.spi[r];
    Emit E;
    E.M = &M;
    E.now = tmin + rel;
    E.ctx = c;
    E.slot0 = r * M.maxc;
    E.n = 0;
    bool st = false;
    cancelled += run_event(M, E, M.ev_kind[cur][pi], M.ev_a[cur][pi], M.ev_pkt[cur][pi], sink, &ttl_drops,
                           &no_route, &unreach, &st);
    stop |= st;
    uint32_t ni = 0;
    if (rel < inline_lim)
      for (uint32_t j = 0; j < E.n; j++) ni += (M.ch_kind[E.slot0 + j] & 0xffu) == K_FWD_UP;
    M.nchild[r] = E.n;
    M.ninl[r] = ni;
    pending += ni;
    last = r;
  }
  if (stop) C.stop_seen = 1;
  if (cancelled) atomicAdd((unsigned long long *)&C.cancelled, (unsigned long long)cancelled);
  if (ttl_drops) atomicAdd((unsigned long long *)&C.ttl_drops, (unsigned long long)ttl_drops);
  if (no_route) atomicAdd((unsigned long long *)&C.no_route, (unsigned long long)no_route);
  if (unreach) atomicAdd((unsigned long long *)&C.unreach, (unsigned long long)unreach);
}

// ---- k_scan: child / inline prefixes in rank order, same-ts groups, run bookkeeping ----
__global__ __launch_bounds__(SCAN_THREADS) void k_scan(const P2PDev *__restrict__ Mp) {
  const P2PDev &M = *Mp;
  Ctl &C = *M.C;
  if (C.done) return;
  constexpr int RPT = WCAP / SCAN_THREADS;
  __shared__ uint32_t wsum[SCAN_THREADS / 64];
  __shared__ uint32_t gstart[WCAP];
  const uint32_t W = C.W;
  const int tid = threadIdx.x;
  uint32_t nc[RPT], ni[RPT], hd[RPT], sc = 0, si = 0, sh = 0;
  uint64_t prev_rel = 0;
  if (tid * RPT < (int)W && tid > 0) prev_rel = M.skey[tid * RPT - 1] >> 32;
#pragma unroll
  for (int q = 0; q < RPT; q++) {
    const uint32_t r = tid * RPT + q;
    nc[q] = ni[q] = hd[q] = 0;
    if (r < W) {
      nc[q] = M.nchild[r];
      ni[q] = M.ninl[r];
      const uint64_t rel = M.skey[r] >> 32;
      hd[q] = r == 0 || rel != prev_rel;
      prev_rel = rel;
    }
    sc += nc[q];
    si += ni[q];
    sh += hd[q];
  }
  uint32_t tc, tinl, ng;
  uint32_t bc = block_exscan<SCAN_THREADS>(sc, wsum, &tc);
  uint32_t bi = block_exscan<SCAN_THREADS>(si, wsum, &tinl);
  uint32_t bh = block_exscan<SCAN_THREADS>(sh, wsum, &ng);
  uint32_t g[RPT];
#pragma unroll
  for (int q = 0; q < RPT; q++) {
    const uint32_t r = tid * RPT + q;
    bh += hd[q];
    g[q] = bh - 1;  // same-ts group of rank r
    if (r < W) {
      M.cpref[r] = bc;
      M.ipref[r] = bi;
      if (hd[q]) gstart[g[q]] = r;
    }
    bc += nc[q];
    bi += ni[q];
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < RPT; q++) {
    const uint32_t r = tid * RPT + q;
    if (r < W) {
      const uint32_t first = gstart[g[q]];
      const uint32_t last = (g[q] + 1 < ng ? gstart[g[q] + 1] : W) - 1;
      M.gbnd[r] = first | (last << 16);
    }
  }
  if (tid == 0) {
    C.K0 = C.K;
    C.uid0 = C.uid;
    C.W0 = W;
    C.Pbase = C.nxtP;
    C.tmin0 = C.tmin;
    C.inline_lim0 = C.inline_lim;
    C.total_children = tc;
    C.total_inline = tinl;
    // (inline children at the Stop's ts are scheduled — uids consumed — but never dispatched; the run
    //  ends with this window, so the pool bookkeeping only has to be right for other windows)
    const uint64_t newP = (uint64_t)C.nxtP + tc - tinl;
    C.K += W + tinl;
    C.uid += tc;
    C.P = newP;
    C.cur ^= 1;
    C.windows++;
    if (W > C.max_window) C.max_window = W;
    C.tmin = ~0ull;
    C.wend = ~0ull;
    C.stopts = ~0ull;
    C.W = 0;
    C.nxtP = 0;
    bool done = C.stop_seen || newP == 0;
    if (newP > M.pool_cap) {
      atomicOr(M.error, 1u);
      done = true;
    }
    if (C.windows >= C.max_windows && !done) {
      atomicOr(M.error, 4u);
      done = true;
    }
    C.scan_ran = 1;
    if (done) C.done = 1;
  }
}

// ---- k_append: dispatch ranks (digest, log), children -> pool ----
__global__ __launch_bounds__(RB) void k_append(const P2PDev *__restrict__ Mp) {
  const P2PDev &M = *Mp;
  Ctl &C = *M.C;
  if (!C.scan_ran) return;
  const uint32_t W = C.W0;
  const uint32_t r = blockIdx.x * RB + threadIdx.x;
  if (blockIdx.x * RB >= W) return;  // whole block idle (uniform)
  uint64_t digest = 0;
  if (r < W) {
    const uint64_t K0 = C.K0, tmin = C.tmin0, inline_lim = C.inline_lim0;
    const uint32_t uid0 = C.uid0, tinl = C.total_inline;
    const uint64_t pk = M.skey[r];
    const uint64_t rel = pk >> 32;
    const uint64_t t = tmin + rel;
    const uint32_t u = (uint32_t)pk;
    const uint32_t gb = M.gbnd[r];
    const uint32_t first = gb & 0xffffu, last = gb >> 16;
    const uint32_t ip = M.ipref[r], cp = M.cpref[r];
    // dispatch rank of main event r = r + #inline children with ts < ts_r; of the i-th inline child
    // of r = (#main events with ts <= ts_r) + iprefix[r] + i  (inline children are key-sorted by r)
    const uint64_t rk = K0 + r + (tinl ? M.ipref[first] : 0);
    digest += digest_term(rk, t, u);
    if (rk < M.log_cap) {
      M.log_ts[rk] = t;
      M.log_uid[rk] = u;
      M.log_ctx[rk] = M.sctx[r];
    }
    if (r == W - 1) C.last_ts = t;
    const uint32_t ncr = M.nchild[r];
    uint32_t ii = 0;
    uint64_t o = (uint64_t)C.Pbase + (cp - ip);  // non-inline children before this rank
    const int dst = C.cur;                       // (already flipped by k_scan: the next pool)
    for (uint32_t j = 0; j < ncr; j++) {
      const uint32_t sl = r * M.maxc + j;
      const uint32_t cu = uid0 + cp + j;
      const uint32_t kw = M.ch_kind[sl];
      if ((kw & 0xffu) == K_FWD_UP) {
        if (rel < inline_lim) {  // dispatched inside this window
          const uint64_t crk = K0 + last + 1 + ip + ii;
          digest += digest_term(crk, t, cu);
          if (crk < M.log_cap) {
            M.log_ts[crk] = t;
            M.log_uid[crk] = cu;
            M.log_ctx[crk] = M.ch_ctx[sl];
          }
          ii++;
        }
        continue;  // never re-queued
      }
      if (o < M.pool_cap) {
        M.ev_ts[dst][o] = M.ch_ts[sl];
        M.ev_uid[dst][o] = cu;
        M.ev_ctx[dst][o] = M.ch_ctx[sl];
        M.ev_kind[dst][o] = kw;
        M.ev_a[dst][o] = M.ch_a[sl];
        M.ev_pkt[dst][o] = M.ch_pkt[sl];
      } else {
        atomicOr(M.error, 1u);
      }
      o++;
    }
  }
  digest = wave_sum64(digest);
  if ((threadIdx.x & 63) == 0 && digest) atomicAdd((unsigned long long *)&C.digest, (unsigned long long)digest);
}

}  // namespace nsgpu
// ====================================================================================================
// Host side: scenario upload, setup-time event list, launch, results.
// ====================================================================================================
#include <vector>
#include <algorithm>
#include <string.h>

using namespace nsgpu;

struct nsgpu_p2p {
  P2PDev M;
  nsgpu_p2p_scenario sc;
  std::vector<void *> allocs;
  int32_t *sink_of_node = nullptr;
  P2PDev *d_M = nullptr;  // device copy of M (kernel argument by pointer)
  Ctl C0{};               // run control after reset
  uint64_t max_windows = ~0ull;
  hipStream_t s = nullptr;  // engine stream (graph capture and replay)
  hipGraphExec_t gexec = nullptr;
  hipEvent_t ev[2] = {nullptr, nullptr}, t0 = nullptr, t1 = nullptr;
  uint32_t *done_host = nullptr;  // pinned, 2 slots
  float last_ms = 0.f;
  // pristine initial pool (device) for resets
  uint64_t *init_ts = nullptr;
  uint32_t *init_uid = nullptr, *init_ctx = nullptr, *init_kind = nullptr, *init_a = nullptr;
  uint32_t n_apps = 0;
};

namespace {
template <class T>
int dalloc(nsgpu_p2p *h, T **p, size_t n) {
  void *q = nullptr;
  hipError_t e = hipMalloc(&q, (n ? n : 1) * sizeof(T));
  if (e != hipSuccess) return set_error(NSGPU_ENOMEM, "nsgpu_p2p: hipMalloc(%zu): %s", n * sizeof(T),
                                        hipGetErrorString(e));
  h->allocs.push_back(q);
  *p = (T *)q;
  return NSGPU_OK;
}
template <class T>
int dupload(nsgpu_p2p *h, const T **dst, const T *src, size_t n) {
  T *p;
  int rc = dalloc(h, &p, n);
  if (rc) return rc;
  if (n) NSGPU_HIP(hipMemcpy(p, src, n * sizeof(T), hipMemcpyHostToDevice));
  *dst = p;
  return NSGPU_OK;
}
}  // namespace

#define TRY(x)            \
  do {                    \
    int rc_ = (x);        \
    if (rc_) {            \
      nsgpu_p2p_destroy(h); \
      return rc_;         \
    }                     \
  } while (0)

extern "C" int nsgpu_p2p_destroy(nsgpu_p2p *h) {
  if (!h) return NSGPU_OK;
  if (h->s) (void)hipStreamSynchronize(h->s);
  if (h->gexec) (void)hipGraphExecDestroy(h->gexec);
  for (hipEvent_t e : {h->ev[0], h->ev[1], h->t0, h->t1})
    if (e) (void)hipEventDestroy(e);
  if (h->done_host) (void)hipHostFree(h->done_host);
  if (h->s) (void)hipStreamDestroy(h->s);
  for (void *p : h->allocs) (void)hipFree(p);
  delete h;
  return NSGPU_OK;
}

extern "C" int nsgpu_p2p_create(const nsgpu_p2p_scenario *sc, uint64_t pool_cap, uint64_t log_cap,
                                nsgpu_p2p **out) {
  if (!sc || !out) return set_error(NSGPU_EINVAL, "nsgpu_p2p_create: null");
  *out = nullptr;
  const uint32_t N = sc->n_nodes, D = sc->n_devices, A = sc->n_apps;
  if (N == 0 || !sc->setup_kind || !sc->setup_index) return set_error(NSGPU_EINVAL, "nsgpu_p2p_create: empty");
  // ---- validation (host arrays) ----
  uint32_t qcap = 1;
  for (uint32_t d = 0; d < D; d++) {
    if (sc->dev_node[d] >= N || sc->dev_peer[d] >= D || sc->dev_peer[sc->dev_peer[d]] != d)
      return set_error(NSGPU_EINVAL, "nsgpu_p2p_create: device %u: bad node/peer", d);
    if (sc->dev_bps[d] == 0) return set_error(NSGPU_EINVAL, "nsgpu_p2p_create: device %u: zero DataRate", d);
    if (sc->dev_delay_ns[d] < 0 || sc->dev_ifg_ns[d] < 0)
      return set_error(NSGPU_EINVAL, "nsgpu_p2p_create: device %u: negative delay", d);
    qcap = std::max(qcap, sc->dev_qmax[d]);
  }
  std::vector<uint32_t> napps(N + 1, 0);
  std::vector<int32_t> sink(N, -1);
  uint32_t min_pkt = 0xffffffffu;
  for (uint32_t a = 0; a < A; a++) {
    if (sc->app_node[a] >= N) return set_error(NSGPU_EINVAL, "nsgpu_p2p_create: app %u: bad node", a);
    napps[sc->app_node[a] + 1]++;
    if (sc->app_kind[a] == NSGPU_APP_SINK) {
      if (sink[sc->app_node[a]] >= 0)
        return set_error(NSGPU_EINVAL, "nsgpu_p2p_create: node %u has two PacketSinks", sc->app_node[a]);
      sink[sc->app_node[a]] = (int32_t)a;
    } else {
      if (sc->app_dst_node[a] >= N || sc->app_dst_slot[a] >= sc->n_dst || sc->app_rate_bps[a] == 0 ||
          sc->app_pkt_size[a] == 0 || sc->app_ttl[a] == 0 || sc->app_dst_node[a] == sc->app_node[a])
        return set_error(NSGPU_EINVAL, "nsgpu_p2p_create: OnOff %u: bad destination/rate/size/ttl", a);
      min_pkt = std::min(min_pkt, sc->app_pkt_size[a]);
    }
  }
  uint32_t maxapps = 0;
  for (uint32_t n = 0; n < N; n++) maxapps = std::max(maxapps, napps[n + 1]);
  for (uint32_t n = 0; n < N; n++) napps[n + 1] += napps[n];
  std::vector<uint32_t> node_list(A), fill(napps.begin(), napps.end() - 1);
  for (uint32_t a = 0; a < A; a++) node_list[fill[sc->app_node[a]]++] = a;
  // ---- lookahead per event kind: the smallest delay a child of that kind can get ----
  const int64_t INFL = (int64_t)1 << 61;
  int64_t tx_min = INFL;
  if (min_pkt != 0xffffffffu)
    for (uint32_t d = 0; d < D; d++)
      tx_min = std::min(tx_min, seconds_to_ts(static_cast<double>(min_pkt + 30) * 8 / (double)sc->dev_bps[d]));
  int64_t send_ivl = INFL;
  for (uint32_t a = 0; a < A; a++)
    if (sc->app_kind[a] == NSGPU_APP_ONOFF)
      send_ivl = std::min(send_ivl, seconds_to_ts((sc->app_pkt_size[a] * 8) / static_cast<double>(sc->app_rate_bps[a])));
  nsgpu_p2p *h = new nsgpu_p2p();
  h->sc = *sc;
  h->n_apps = A;
  P2PDev &M = h->M;
  memset(&M, 0, sizeof(M));
  M.n_nodes = N;
  M.n_devices = D;
  M.n_apps = A;
  M.n_dst = sc->n_dst;
  M.qcap = qcap;
  M.maxc = std::max(3u, 2 * maxapps);
  for (int k = 0; k < K_NKINDS; k++) M.lookahead[k] = INFL;
  M.lookahead[K_NODE_START] = 0;     // children at app start/stop times (may be 0)
  M.lookahead[K_APPOBJ_START] = 0;
  M.lookahead[K_APP_START] = 0;      // StartSending after OffTime (may be 0)
  M.lookahead[K_START_SENDING] = 0;  // first send after residual-shortened interval
  M.lookahead[K_STOP_SENDING] = 0;   // StartSending after OffTime
  M.lookahead[K_SEND] = std::min(tx_min, send_ivl);
  M.lookahead[K_TX_COMPLETE] = tx_min;
  M.lookahead[K_RECEIVE] = tx_min;
  // ---- scenario upload ----
  TRY(dupload(h, &M.dev_node, sc->dev_node, D));
  TRY(dupload(h, &M.dev_peer, sc->dev_peer, D));
  TRY(dupload(h, &M.dev_qmax, sc->dev_qmax, D));
  TRY(dupload(h, &M.dev_bps, sc->dev_bps, D));
  TRY(dupload(h, &M.dev_ifg, sc->dev_ifg_ns, D));
  TRY(dupload(h, &M.dev_delay, sc->dev_delay_ns, D));
  TRY(dupload(h, &M.route, sc->route, (size_t)N * sc->n_dst));
  TRY(dupload(h, &M.app_kind, sc->app_kind, A));
  TRY(dupload(h, &M.app_node, sc->app_node, A));
  TRY(dupload(h, &M.app_dst_node, sc->app_dst_node, A));
  TRY(dupload(h, &M.app_dst_slot, sc->app_dst_slot, A));
  TRY(dupload(h, &M.app_pkt_size, sc->app_pkt_size, A));
  TRY(dupload(h, &M.app_max_bytes, sc->app_max_bytes, A));
  TRY(dupload(h, &M.app_ttl, sc->app_ttl, A));
  TRY(dupload(h, &M.app_start, sc->app_start_ns, A));
  TRY(dupload(h, &M.app_stop, sc->app_stop_ns, A));
  TRY(dupload(h, &M.app_rate, sc->app_rate_bps, A));
  TRY(dupload(h, &M.app_on_s, sc->app_on_s, A));
  TRY(dupload(h, &M.app_off_s, sc->app_off_s, A));
  TRY(dupload(h, &M.node_app_off, napps.data(), N + 1));
  TRY(dupload(h, &M.node_app_list, node_list.data(), A));
  const int32_t *sinkp;
  TRY(dupload(h, &sinkp, sink.data(), N));
  h->sink_of_node = (int32_t *)sinkp;
  // ---- state ----
  TRY(dalloc(h, &M.dev_busy, D));
  TRY(dalloc(h, &M.q_head, D));
  TRY(dalloc(h, &M.q_count, D));
  TRY(dalloc(h, &M.q_buf, (size_t)D * qcap));
  TRY(dalloc(h, &M.devc, D));
  TRY(dalloc(h, &M.app_flags, A));
  TRY(dalloc(h, &M.app_send_gen, A));
  TRY(dalloc(h, &M.app_ss_gen, A));
  TRY(dalloc(h, &M.app_residual, A));
  TRY(dalloc(h, &M.app_tot, A));
  TRY(dalloc(h, &M.app_seq, A));
  TRY(dalloc(h, &M.app_last_start, A));
  TRY(dalloc(h, &M.appc, A));
  TRY(dalloc(h, &M.node_head, N));
  // ---- setup-time events (node-list.cc:124-131, node.cc:111-145, default-simulator-impl.cc:179-183) ----
  std::vector<uint64_t> its;
  std::vector<uint32_t> iuid, ictx, ikind, ia;
  uint32_t uid = 4;
  for (uint32_t i = 0; i < sc->n_setup; i++) {
    const uint32_t k = sc->setup_index[i];
    switch (sc->setup_kind[i]) {
      case NSGPU_SETUP_NODE:
        if (k >= N) { nsgpu_p2p_destroy(h); return set_error(NSGPU_EINVAL, "setup: node %u", k); }
        its.push_back(0); iuid.push_back(uid); ictx.push_back(k); ikind.push_back(K_NODE_START); ia.push_back(k);
        break;
      case NSGPU_SETUP_DEVICE:
        if (k >= D) { nsgpu_p2p_destroy(h); return set_error(NSGPU_EINVAL, "setup: device %u", k); }
        its.push_back(0); iuid.push_back(uid); ictx.push_back(sc->dev_node[k]); ikind.push_back(K_DEV_START); ia.push_back(k);
        break;
      case NSGPU_SETUP_APP:
        if (k >= A) { nsgpu_p2p_destroy(h); return set_error(NSGPU_EINVAL, "setup: app %u", k); }
        its.push_back(0); iuid.push_back(uid); ictx.push_back(sc->app_node[k]); ikind.push_back(K_APPOBJ_START); ia.push_back(k);
        break;
      case NSGPU_SETUP_NOOP:
        if (k >= N) { nsgpu_p2p_destroy(h); return set_error(NSGPU_EINVAL, "setup: noop node %u", k); }
        its.push_back(0); iuid.push_back(uid); ictx.push_back(k); ikind.push_back(K_DEV_START); ia.push_back(k);
        break;
      case NSGPU_SETUP_STOP:
        if (sc->stop_ns < 0) { nsgpu_p2p_destroy(h); return set_error(NSGPU_EINVAL, "setup: negative stop"); }
        its.push_back((uint64_t)sc->stop_ns); iuid.push_back(uid); ictx.push_back(NOCTX); ikind.push_back(K_STOP); ia.push_back(0);
        break;
      default:
        break;  // consumes a uid, no event
    }
    uid++;
  }
  M.n_init = (uint32_t)its.size();
  M.uid_init = uid;
  M.pool_cap = pool_cap ? pool_cap : std::max<uint64_t>(4ull * M.n_init + 65536, 1ull << 20);
  if (M.n_init > M.pool_cap) { nsgpu_p2p_destroy(h); return set_error(NSGPU_EINVAL, "pool_cap < setup events"); }
  for (int b = 0; b < 2; b++) {
    TRY(dalloc(h, &M.ev_ts[b], M.pool_cap));
    TRY(dalloc(h, &M.ev_uid[b], M.pool_cap));
    TRY(dalloc(h, &M.ev_ctx[b], M.pool_cap));
    TRY(dalloc(h, &M.ev_kind[b], M.pool_cap));
    TRY(dalloc(h, &M.ev_a[b], M.pool_cap));
    TRY(dalloc(h, &M.ev_pkt[b], M.pool_cap));
  }
  const size_t chn = (size_t)WCAP * M.maxc;
  TRY(dalloc(h, &M.ch_ts, chn));
  TRY(dalloc(h, &M.ch_ctx, chn));
  TRY(dalloc(h, &M.ch_kind, chn));
  TRY(dalloc(h, &M.ch_a, chn));
  TRY(dalloc(h, &M.ch_pkt, chn));
  TRY(dalloc(h, &M.wkey, WCAP));
  TRY(dalloc(h, &M.skey, WCAP));
  for (uint32_t **p : {&M.wpi, &M.wrank, &M.spi, &M.sctx, &M.link, &M.nchild, &M.ninl, &M.cpref, &M.ipref, &M.gbnd})
    TRY(dalloc(h, p, WCAP));
  TRY(dalloc(h, &M.C, 1));
  TRY(dalloc(h, &M.error, 4));
  M.log_cap = log_cap;
  TRY(dalloc(h, &M.log_ts, log_cap));
  TRY(dalloc(h, &M.log_uid, log_cap));
  TRY(dalloc(h, &M.log_ctx, log_cap));
  const uint64_t *c_ts;
  const uint32_t *c_uid, *c_ctx, *c_kind, *c_a;
  TRY(dupload(h, &c_ts, its.data(), its.size()));
  TRY(dupload(h, &c_uid, iuid.data(), iuid.size()));
  TRY(dupload(h, &c_ctx, ictx.data(), ictx.size()));
  TRY(dupload(h, &c_kind, ikind.data(), ikind.size()));
  TRY(dupload(h, &c_a, ia.data(), ia.size()));
  h->init_ts = (uint64_t *)c_ts;
  h->init_uid = (uint32_t *)c_uid;
  h->init_ctx = (uint32_t *)c_ctx;
  h->init_kind = (uint32_t *)c_kind;
  h->init_a = (uint32_t *)c_a;
  // run control after reset
  Ctl &C0 = h->C0;
  memset(&C0, 0, sizeof(C0));
  C0.P = M.n_init;
  C0.uid = uid;
  C0.tmin = C0.wend = C0.stopts = ~0ull;
  C0.max_windows = h->max_windows;
  C0.done = M.n_init == 0;
  TRY(dalloc(h, &h->d_M, 1));
  if (hipStreamCreateWithFlags(&h->s, hipStreamNonBlocking) != hipSuccess) {
    h->s = nullptr;
    nsgpu_p2p_destroy(h);
    return set_error(NSGPU_EHIP, "nsgpu_p2p_create: hipStreamCreate failed");
  }
  for (hipEvent_t *e : {&h->ev[0], &h->ev[1]})
    if (hipEventCreateWithFlags(e, hipEventDisableTiming) != hipSuccess) {
      *e = nullptr;
      nsgpu_p2p_destroy(h);
      return set_error(NSGPU_EHIP, "nsgpu_p2p_create: hipEventCreate failed");
    }
  for (hipEvent_t *e : {&h->t0, &h->t1})
    if (hipEventCreate(e) != hipSuccess) {
      *e = nullptr;
      nsgpu_p2p_destroy(h);
      return set_error(NSGPU_EHIP, "nsgpu_p2p_create: hipEventCreate failed");
    }
  if (hipHostMalloc((void **)&h->done_host, 2 * sizeof(uint32_t), hipHostMallocDefault) != hipSuccess) {
    h->done_host = nullptr;
    nsgpu_p2p_destroy(h);
    return set_error(NSGPU_ENOMEM, "nsgpu_p2p_create: hipHostMalloc failed");
  }
  if (hipMemcpy(h->d_M, &h->M, sizeof(P2PDev), hipMemcpyHostToDevice) != hipSuccess) {
    nsgpu_p2p_destroy(h);
    return set_error(NSGPU_EHIP, "nsgpu_p2p_create: upload failed");
  }
  *out = h;
  return NSGPU_OK;
}

// Restores the initial (post-setup) state on the device, asynchronously.
extern "C" int nsgpu_p2p_reset(nsgpu_p2p *h, void *stream) {
  if (!h) return set_error(NSGPU_EINVAL, "nsgpu_p2p_reset: null");
  hipStream_t s = (hipStream_t)stream;
  P2PDev &M = h->M;
  const uint32_t D = M.n_devices, A = M.n_apps, n0 = M.n_init;
  NSGPU_HIP(hipMemcpyAsync(M.ev_ts[0], h->init_ts, n0 * sizeof(uint64_t), hipMemcpyDeviceToDevice, s));
  NSGPU_HIP(hipMemcpyAsync(M.ev_uid[0], h->init_uid, n0 * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
  NSGPU_HIP(hipMemcpyAsync(M.ev_ctx[0], h->init_ctx, n0 * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
  NSGPU_HIP(hipMemcpyAsync(M.ev_kind[0], h->init_kind, n0 * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
  NSGPU_HIP(hipMemcpyAsync(M.ev_a[0], h->init_a, n0 * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
  NSGPU_HIP(hipMemsetAsync(M.dev_busy, 0, D * sizeof(uint32_t), s));
  NSGPU_HIP(hipMemsetAsync(M.q_head, 0, D * sizeof(uint32_t), s));
  NSGPU_HIP(hipMemsetAsync(M.q_count, 0, D * sizeof(uint32_t), s));
  NSGPU_HIP(hipMemsetAsync(M.devc, 0, D * sizeof(nsgpu_dev_counters), s));
  NSGPU_HIP(hipMemsetAsync(M.app_flags, 0, A * sizeof(uint32_t), s));
  NSGPU_HIP(hipMemsetAsync(M.app_send_gen, 0, A * sizeof(uint32_t), s));
  NSGPU_HIP(hipMemsetAsync(M.app_ss_gen, 0, A * sizeof(uint32_t), s));
  NSGPU_HIP(hipMemsetAsync(M.app_residual, 0, A * sizeof(uint32_t), s));
  NSGPU_HIP(hipMemsetAsync(M.app_tot, 0, A * sizeof(uint32_t), s));
  NSGPU_HIP(hipMemsetAsync(M.app_seq, 0, A * sizeof(uint32_t), s));
  NSGPU_HIP(hipMemsetAsync(M.app_last_start, 0, A * sizeof(uint64_t), s));
  NSGPU_HIP(hipMemsetAsync(M.appc, 0, A * sizeof(nsgpu_app_counters), s));
  NSGPU_HIP(hipMemsetAsync(M.node_head, 0xff, M.n_nodes * sizeof(uint32_t), s));
  NSGPU_HIP(hipMemsetAsync(M.wrank, 0, WCAP * sizeof(uint32_t), s));
  NSGPU_HIP(hipMemsetAsync(M.error, 0, 4 * sizeof(uint32_t), s));
  NSGPU_HIP(hipMemcpyAsync(M.C, &h->C0, sizeof(Ctl), hipMemcpyHostToDevice, s));
  return NSGPU_OK;
}

static int build_graph(nsgpu_p2p *h) {
  // NWIN windows of the pipeline; kernels read every run-dependent value from the device (Ctl), so
  // one instantiated graph serves every run of this engine
  hipGraph_t g = nullptr;
  NSGPU_HIP(hipStreamBeginCapture(h->s, hipStreamCaptureModeThreadLocal));
  for (int w = 0; w < NWIN; w++) {
    hipLaunchKernelGGL(k_reduce, dim3(GRID_POOL), dim3(TB), 0, h->s, h->d_M);
    hipLaunchKernelGGL(k_partition, dim3(GRID_POOL), dim3(TB), 0, h->s, h->d_M);
    hipLaunchKernelGGL(k_refit, dim3(1), dim3(SCAN_THREADS), 0, h->s, h->d_M);
    hipLaunchKernelGGL(k_rank, dim3(NT * NT), dim3(TB), 0, h->s, h->d_M);
    hipLaunchKernelGGL(k_scatter, dim3(WCAP / RB), dim3(RB), 0, h->s, h->d_M);
    hipLaunchKernelGGL(k_handle, dim3(WCAP / RB), dim3(RB), 0, h->s, h->d_M, h->sink_of_node);
    hipLaunchKernelGGL(k_scan, dim3(1), dim3(SCAN_THREADS), 0, h->s, h->d_M);
    hipLaunchKernelGGL(k_append, dim3(WCAP / RB), dim3(RB), 0, h->s, h->d_M);
  }
  hipError_t e = hipStreamEndCapture(h->s, &g);
  if (e != hipSuccess) return set_error(NSGPU_EHIP, "nsgpu_p2p: graph capture: %s", hipGetErrorString(e));
  e = hipGraphInstantiate(&h->gexec, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  if (e != hipSuccess) {
    h->gexec = nullptr;
    return set_error(NSGPU_EHIP, "nsgpu_p2p: graph instantiate: %s", hipGetErrorString(e));
  }
  return NSGPU_OK;
}

// Runs the simulation to completion (blocking): graph replays of NWIN windows on the engine stream,
// ordered after the work already queued on `stream`; work queued on `stream` later runs after it.
extern "C" int nsgpu_p2p_run(nsgpu_p2p *h, void *stream) {
  if (!h) return set_error(NSGPU_EINVAL, "nsgpu_p2p_run: null");
  if (!h->gexec) {
    int rc = build_graph(h);
    if (rc) return rc;
  }
  hipStream_t cs = (hipStream_t)stream;
  NSGPU_HIP(hipEventRecord(h->ev[0], cs));
  NSGPU_HIP(hipStreamWaitEvent(h->s, h->ev[0], 0));
  NSGPU_HIP(hipEventRecord(h->t0, h->s));
  h->done_host[0] = h->done_host[1] = 0;
  // two replays in flight: replay i+1 is queued before the done flag of replay i is examined
  for (uint64_t it = 0;; it++) {
    NSGPU_HIP(hipGraphLaunch(h->gexec, h->s));
    NSGPU_HIP(hipMemcpyAsync(&h->done_host[it & 1], &h->M.C->done, sizeof(uint32_t), hipMemcpyDeviceToHost, h->s));
    NSGPU_HIP(hipEventRecord(h->ev[it & 1], h->s));
    if (it > 0) {
      NSGPU_HIP(hipEventSynchronize(h->ev[(it - 1) & 1]));
      if (h->done_host[(it - 1) & 1]) break;
    }
  }
  NSGPU_HIP(hipEventRecord(h->t1, h->s));
  NSGPU_HIP(hipEventSynchronize(h->t1));
  NSGPU_HIP(hipEventElapsedTime(&h->last_ms, h->t0, h->t1));
  NSGPU_HIP(hipEventRecord(h->ev[0], h->s));
  NSGPU_HIP(hipStreamWaitEvent(cs, h->ev[0], 0));
  return NSGPU_OK;
}

extern "C" int nsgpu_p2p_last_run_ms(nsgpu_p2p *h, double *gpu_ms) {
  if (!h || !gpu_ms) return set_error(NSGPU_EINVAL, "nsgpu_p2p_last_run_ms: null");
  *gpu_ms = h->last_ms;
  return NSGPU_OK;
}

extern "C" int nsgpu_p2p_results(nsgpu_p2p *h, nsgpu_p2p_stats *stats, nsgpu_dev_counters *devc,
                                 nsgpu_app_counters *appc, uint64_t *log_ts, uint32_t *log_uid, uint32_t *log_ctx,
                                 uint64_t log_n, uint32_t *error, void *stream) {
  if (!h) return set_error(NSGPU_EINVAL, "nsgpu_p2p_results: null");
  hipStream_t s = (hipStream_t)stream;
  const P2PDev &M = h->M;
  Ctl c;
  NSGPU_HIP(hipMemcpyAsync(&c, M.C, sizeof(Ctl), hipMemcpyDeviceToHost, s));
  if (devc) NSGPU_HIP(hipMemcpyAsync(devc, M.devc, M.n_devices * sizeof(*devc), hipMemcpyDeviceToHost, s));
  if (appc) NSGPU_HIP(hipMemcpyAsync(appc, M.appc, M.n_apps * sizeof(*appc), hipMemcpyDeviceToHost, s));
  if (log_n > M.log_cap) log_n = M.log_cap;
  if (log_ts && log_n) NSGPU_HIP(hipMemcpyAsync(log_ts, M.log_ts, log_n * 8, hipMemcpyDeviceToHost, s));
  if (log_uid && log_n) NSGPU_HIP(hipMemcpyAsync(log_uid, M.log_uid, log_n * 4, hipMemcpyDeviceToHost, s));
  if (log_ctx && log_n) NSGPU_HIP(hipMemcpyAsync(log_ctx, M.log_ctx, log_n * 4, hipMemcpyDeviceToHost, s));
  uint32_t err = 0;
  NSGPU_HIP(hipMemcpyAsync(&err, M.error, 4, hipMemcpyDeviceToHost, s));
  NSGPU_HIP(hipStreamSynchronize(s));
  if (stats) {
    memset(stats, 0, sizeof(*stats));
    stats->dispatched = c.K;
    stats->digest = c.digest;
    stats->cancelled = c.cancelled;
    stats->final_ts = c.last_ts;
    stats->next_uid = c.uid;
    stats->windows = (uint32_t)c.windows;
    stats->ttl_drops = c.ttl_drops;
    stats->no_route_drops = c.no_route;
    stats->max_window = c.max_window;
    stats->unreach_drops = c.unreach;
  }
  if (error) *error = err;
  if (err) return set_error(NSGPU_ENOMEM, "nsgpu_p2p: engine capacity exceeded (code %u: 1 = event pool, "
                                          "4 = window limit, 8 = window cut)", err);
  return NSGPU_OK;
}
