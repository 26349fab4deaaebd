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
// Engine (MI355X): one persistent 1024-thread workgroup runs the whole simulation in windows.
// Pending events live in HBM (SoA, double-buffered pool).  Per window:
//   1. W_end = min over pending e of (ts_e + L(kind_e)), L = the smallest delay any child of that
//      kind of handler can have (DefaultSimulatorImpl's uids make a child sort after every pending
//      event with ts <= its own ts, so every pending event with ts <= W_end is safe to dispatch);
//      a Simulator::Stop event caps the window at its key; an over-full window is cut to its first
//      WCAP keys by bisection (a key prefix of a safe window is safe);
//   2. window keys are packed ((ts - tmin) << 32 | uid) and bitonic-sorted -> global dispatch rank;
//   3. a second sort on (context << 32 | rank) groups the window by logical process (node); the
//      first thread of each group runs that node's events sequentially in rank order, so node
//      state (device tx state, DropTail rings, OnOff state, sink counters) needs no atomics;
//   4. handlers write their children (in Schedule-call order) to per-rank slots; an exclusive scan
//      of child counts in rank order gives each child the uid DefaultSimulatorImpl would assign;
//      children are appended to the next pool.
#include "nsgpu_device.h"
#include "nsgpu_internal.h"
#include "nsgpu_sort.h"

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

constexpr int P2P_THREADS = 512;
constexpr int WCAP = SORT_N;  // events per window
constexpr int RPT = WCAP / P2P_THREADS;  // window ranks per thread
constexpr uint32_t NOCTX = 0xffffffffu;
constexpr uint32_t NOCHAIN = 0xffffffffu;

struct Pkt {
  uint32_t app, seq, size, ttl;
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
  // children of the current window: slot = rank * maxc + j
  uint64_t *ch_ts;
  uint32_t *ch_ctx, *ch_kind, *ch_a;
  Pkt *ch_pkt;
  // run state / outputs
  uint32_t n_init;         // initial pending count (pool 0)
  uint32_t uid_init;       // m_uid after setup
  nsgpu_p2p_stats *stats;
  uint32_t *error;         // non-zero = capacity exceeded (code)
  uint64_t *log_ts;
  uint32_t *log_uid, *log_ctx;
  uint64_t log_cap;
  uint64_t max_windows;
  uint64_t *prof;  // diagnostic: per-phase s_memtime cycle sums (wave 0 view), or null
  uint32_t *node_head;  // per-node chain head of the current window (NOCHAIN between windows)
};

struct P2PLds {
  SortLds sort;
  uint32_t nchild[WCAP];
  uint32_t ninl[WCAP];     // inline (zero-delay leaf) children dispatched inside the window, per rank
  uint32_t iprefix[WCAP];  // exclusive prefix of ninl in rank order
  uint32_t wsum[P2P_THREADS / 64];
  uint64_t wmin[P2P_THREADS / 64];
  uint64_t wmin2[P2P_THREADS / 64];
  uint32_t wcnt[P2P_THREADS / 64];
  uint32_t wcnt2[P2P_THREADS / 64];
  uint32_t stop_flag;
};

// ---------------- block reductions / scans (1024 threads) ----------------
__device__ __forceinline__ uint64_t wave_min64(uint64_t v) {
  for (int o = 32; o > 0; o >>= 1) {
    uint64_t w = __shfl_xor(v, o);
    v = w < v ? w : v;
  }
  return v;
}
__device__ __forceinline__ uint32_t wave_sum32(uint32_t v) {
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
// Block exclusive scan of one value per thread; returns the exclusive prefix, *total = block sum.
__device__ __forceinline__ uint32_t block_exscan(uint32_t v, uint32_t *wsum, uint32_t *total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint32_t ex = wave_exscan32(v, lane);
  if (lane == 63) wsum[wid] = ex + v;
  __syncthreads();
  uint32_t off = 0, tot = 0;
  for (int w = 0; w < P2P_THREADS / 64; w++) {
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

__global__ __launch_bounds__(P2P_THREADS) void p2p_run(const P2PDev *__restrict__ Mp, const int32_t *__restrict__ sink_of_node) {
  const P2PDev &M = *Mp;  // in global memory: fields come through scalar loads, not 70 SGPR kernel args
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  P2PLds &L = *reinterpret_cast<P2PLds *>(smem_raw);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const uint64_t INF = ~0ull;

  uint64_t P = M.n_init;
  int cur = 0;
  uint64_t K = 0;            // dispatched so far
  uint32_t uid = M.uid_init; // next uid
  uint64_t digest = 0, cancelled = 0, ttl_drops = 0, no_route = 0, unreach = 0;
  uint64_t windows = 0, max_window = 0, last_ts = 0;
  if (tid == 0) L.stop_flag = 0;
  __syncthreads();
  uint64_t pacc[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t tprev = M.prof ? __builtin_amdgcn_s_memtime() : 0;
#define PSTAMP(i)                                        \
  if (M.prof) {                                          \
    const uint64_t tnow_ = __builtin_amdgcn_s_memtime(); \
    pacc[i] += tnow_ - tprev;                            \
    tprev = tnow_;                                       \
  }

  while (P > 0) {
    if (windows >= M.max_windows) {
      if (tid == 0) atomicOr(M.error, 4u);
      break;
    }
    const uint64_t *ts = M.ev_ts[cur];
    const uint32_t *uidv = M.ev_uid[cur];
    const uint32_t *kindv = M.ev_kind[cur];
    PSTAMP(6);
    // ---- 1. tmin, W_end = min (ts + L(kind)), stop key ----
    uint64_t tmin = INF, wend = INF, stopkey = INF;
    for (uint64_t i = tid; i < P; i += P2P_THREADS) {
      const uint64_t t = ts[i];
      const uint32_t k = kindv[i] & 0xffu;
      tmin = t < tmin ? t : tmin;
      const uint64_t e = t + (uint64_t)M.lookahead[k];
      wend = e < wend ? e : wend;
      if (k == K_STOP) stopkey = t;  // at most one Stop event is pending
    }
    tmin = wave_min64(tmin);
    wend = wave_min64(wend);
    stopkey = wave_min64(stopkey);
    if (lane == 0) {
      L.wmin[wid] = tmin;
      L.wmin2[wid] = wend;
      L.sort.k[0][wid] = stopkey;
    }
    __syncthreads();
    tmin = INF;
    wend = INF;
    stopkey = INF;
    for (int w = 0; w < P2P_THREADS / 64; w++) {
      tmin = L.wmin[w] < tmin ? L.wmin[w] : tmin;
      wend = L.wmin2[w] < wend ? L.wmin2[w] : wend;
      stopkey = L.sort.k[0][w] < stopkey ? L.sort.k[0][w] : stopkey;
    }
    __syncthreads();
    // packed key bound: ((ts - tmin) << 32) | uid <= bound
    uint64_t span = wend - tmin;
    if (span > 0xfffffffeull) span = 0xfffffffeull;
    uint64_t bound = (span << 32) | 0xffffffffull;
    uint64_t stop_packed = INF;
    if (stopkey != INF && stopkey - tmin <= span) {
      // Stop caps the window at its own key (it is dispatched; later events are not)
      for (uint64_t i = tid; i < P; i += P2P_THREADS)
        if ((kindv[i] & 0xffu) == K_STOP) L.sort.k[1][0] = ((ts[i] - tmin) << 32) | uidv[i];
      __syncthreads();
      stop_packed = L.sort.k[1][0];
      bound = stop_packed < bound ? stop_packed : bound;
      __syncthreads();
    }
    PSTAMP(0);
    // ---- count; if the window would exceed WCAP, bisect for the largest key bound that fits ----
    // (any key prefix of a safe window is safe: its children still sort after every kept event)
    auto count_le = [&](uint64_t bnd) -> uint32_t {
      uint32_t c = 0;
      for (uint64_t i = tid; i < P; i += P2P_THREADS) {
        const uint64_t t = ts[i];
        if (t - tmin <= span) c += ((((t - tmin) << 32) | uidv[i]) <= bnd);
      }
      c = wave_sum32(c);
      if (lane == 0) L.wcnt[wid] = c;
      __syncthreads();
      uint32_t tot = 0;
      for (int w = 0; w < P2P_THREADS / 64; w++) tot += L.wcnt[w];
      __syncthreads();
      return tot;
    };
    uint32_t cnt = count_le(bound);
    if (cnt > (uint32_t)WCAP) {
      uint64_t lo_b = 0, hi_b = bound;  // count (hi_b) > WCAP
      while (hi_b - lo_b > 1) {
        const uint64_t mid = lo_b + (hi_b - lo_b) / 2;
        if (count_le(mid) <= (uint32_t)WCAP) lo_b = mid;
        else hi_b = mid;
      }
      bound = lo_b;
      cnt = count_le(bound);
    }
    const uint32_t W = cnt;
    // zero-delay leaf children (Ipv4EndPoint::DoForwardUp) run inside the window; when the window
    // ends at the Stop event, those at the Stop's ts sort after it and are never dispatched
    const bool has_stop = stop_packed != INF && bound >= stop_packed;
    const uint64_t inline_ts_limit = has_stop ? (stop_packed >> 32) : INF;  // relative ts (exclusive)
    PSTAMP(1);
    // ---- 2. partition: window -> LDS list (packed key, pool index); rest -> next pool ----
    const int nxt = cur ^ 1;
    {
      // each thread handles a contiguous range of the pool; window slots by block scan
      const uint64_t per = (P + P2P_THREADS - 1) / P2P_THREADS;
      const uint64_t i0 = (uint64_t)tid * per, i1 = i0 + per < P ? i0 + per : P;
      uint32_t nin = 0, nout = 0;
      for (uint64_t i = i0; i < i1; i++) {
        const uint64_t t = ts[i];
        const bool in = (t - tmin <= span) && ((((t - tmin) << 32) | uidv[i]) <= bound);
        nin += in;
        nout += !in;
      }
      uint32_t tot_in, tot_out;
      uint32_t win_off = block_exscan(nin, L.wsum, &tot_in);
      uint32_t out_off = block_exscan(nout, L.wsum, &tot_out);
      for (uint64_t i = i0; i < i1; i++) {
        const uint64_t t = ts[i];
        const uint64_t pk = ((t - tmin) << 32) | uidv[i];
        const bool in = (t - tmin <= span) && (pk <= bound);
        if (in) {
          L.sort.k[0][win_off] = pk;
          L.sort.v[0][win_off] = (uint32_t)i;
          win_off++;
        } else {
          M.ev_ts[nxt][out_off] = t;
          M.ev_uid[nxt][out_off] = uidv[i];
          M.ev_ctx[nxt][out_off] = M.ev_ctx[cur][i];
          M.ev_kind[nxt][out_off] = kindv[i];
          M.ev_a[nxt][out_off] = M.ev_a[cur][i];
          M.ev_pkt[nxt][out_off] = M.ev_pkt[cur][i];
          out_off++;
        }
      }
      P = tot_out;  // survivors; children are appended after them
    }
    // clear the bucket histogram (sort.v[1]) and fill counters (nchild)
    for (int i = tid; i < WCAP; i += P2P_THREADS) {
      L.sort.v[1][i] = 0;
      L.nchild[i] = 0;
    }
    __syncthreads();
    PSTAMP(2);
    // ---- 3. dispatch rank: bucket sort of the packed keys by relative ts (bitonic if a bucket is crowded) ----
    {
      uint64_t rmax = 0;
      for (int i = tid; i < (int)W; i += P2P_THREADS) {
        const uint64_t r = L.sort.k[0][i] >> 32;
        rmax = r > rmax ? r : rmax;
      }
      for (int o = 32; o > 0; o >>= 1) {
        const uint64_t w = __shfl_xor(rmax, o);
        rmax = w > rmax ? w : rmax;
      }
      if (lane == 0) L.wmin[wid] = rmax;
      __syncthreads();
      rmax = 0;
      for (int w = 0; w < P2P_THREADS / 64; w++) rmax = L.wmin[w] > rmax ? L.wmin[w] : rmax;
      const uint64_t denom = rmax + 1;
      for (int i = tid; i < (int)W; i += P2P_THREADS) {
        const uint32_t bk = (uint32_t)(((L.sort.k[0][i] >> 32) * (uint64_t)WCAP) / denom);
        atomicAdd(&L.sort.v[1][bk], 1u);
      }
      __syncthreads();
      // exclusive scan of the 4096 bucket counts (4 per thread) and the largest bucket
      uint32_t bc[RPT], bs = 0, bmax = 0;
#pragma unroll
      for (int q = 0; q < RPT; q++) {
        bc[q] = L.sort.v[1][tid * RPT + q];
        bs += bc[q];
        bmax = bc[q] > bmax ? bc[q] : bmax;
      }
      uint32_t btot;
      uint32_t bstart = block_exscan(bs, L.wsum, &btot);
#pragma unroll
      for (int q = 0; q < RPT; q++) {
        L.sort.v[1][tid * RPT + q] = bstart;
        bstart += bc[q];
      }
      for (int o = 32; o > 0; o >>= 1) {
        const uint32_t w = __shfl_xor(bmax, o);
        bmax = w > bmax ? w : bmax;
      }
      if (lane == 0) L.wcnt[wid] = bmax;
      __syncthreads();
      bmax = 0;
      for (int w = 0; w < P2P_THREADS / 64; w++) bmax = L.wcnt[w] > bmax ? L.wcnt[w] : bmax;
      PSTAMP(7);
      if (bmax > 32) {
        if (M.prof) pacc[9]++;
        // crowded buckets (equal timestamps: lockstep sources, the setup burst at ts 0): wave-run
        // sort + cross-run ranking
        __syncthreads();
        run_rank_sort<P2P_THREADS>(L.sort, W);
      } else {
        // scatter into buckets (sort.k[1] keys, ninl pool indices), then sort each bucket in place
        for (int i = tid; i < (int)W; i += P2P_THREADS) {
          const uint64_t pk = L.sort.k[0][i];
          const uint32_t bk = (uint32_t)(((pk >> 32) * (uint64_t)WCAP) / denom);
          const uint32_t pos = L.sort.v[1][bk] + atomicAdd(&L.nchild[bk], 1u);
          L.sort.k[1][pos] = pk;
          L.ninl[pos] = L.sort.v[0][i];
        }
        __syncthreads();
#pragma unroll 1
        for (int q = 0; q < RPT; q++) {
          const uint32_t bk = tid * RPT + q;
          const uint32_t c = L.nchild[bk];
          if (c > 1) {
            const uint32_t s0 = L.sort.v[1][bk];
            for (uint32_t x = s0 + 1; x < s0 + c; x++) {  // insertion sort (c <= 32)
              const uint64_t kx = L.sort.k[1][x];
              const uint32_t vx = L.ninl[x];
              uint32_t y = x;
              while (y > s0 && L.sort.k[1][y - 1] > kx) {
                L.sort.k[1][y] = L.sort.k[1][y - 1];
                L.ninl[y] = L.ninl[y - 1];
                y--;
              }
              L.sort.k[1][y] = kx;
              L.ninl[y] = vx;
            }
          }
        }
        __syncthreads();
        for (int r = tid; r < (int)W; r += P2P_THREADS) {
          L.sort.k[0][r] = L.sort.k[1][r];
          L.sort.v[0][r] = L.ninl[r];
        }
      }
      __syncthreads();
      PSTAMP(8);
    }
    // ---- group by node: per-node chains through a global head array (one atomicExch per event) ----
    // (sort.k[1] is free after the sort: it holds each rank's context)
    uint32_t *const Lctx = reinterpret_cast<uint32_t *>(&L.sort.k[1][0]);
#pragma unroll
    for (int q = 0; q < RPT; q++) {
      const int r = tid + P2P_THREADS * q;
      if (r < (int)W) {
        const uint32_t c = M.ev_ctx[cur][L.sort.v[0][r]];
        Lctx[r] = c;
        L.sort.v[1][r] = c < M.n_nodes ? atomicExch(&M.node_head[c], (uint32_t)r) : NOCHAIN;
      }
      if (r < WCAP) {
        L.nchild[r] = 0;
        L.ninl[r] = 0;
      }
    }
    __syncthreads();
    PSTAMP(3);
    // ---- 4. handlers: the node's last exchanger walks the node's chain in rank order ----
    // Zero-delay leaf children (K_FWD_UP: Ipv4EndPoint::DoForwardUp, ipv4-end-point.cc:112-120) run at
    // their key position: after the node's events with ts <= theirs, before the first with a larger ts.
#pragma unroll 1
    for (int q = 0; q < RPT; q++) {
      const int r0 = tid + P2P_THREADS * q;
      if (r0 >= (int)W) continue;
      const uint32_t c = Lctx[r0];
      if (c < M.n_nodes) {
        const uint32_t head = __hip_atomic_load(&M.node_head[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (head != (uint32_t)r0) continue;  // not the chain holder
        __hip_atomic_store(&M.node_head[c], NOCHAIN, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      const int32_t sink = c < M.n_nodes ? sink_of_node[c] : -1;
      uint32_t n = 0;
      for (uint32_t x = (uint32_t)r0; x != NOCHAIN; x = L.sort.v[1][x]) n++;
      int64_t last = -1;
      uint32_t ts0_rank = 0, pending = 0;
      uint64_t cur_rel = 0;
      for (uint32_t it = 0; it <= n; it++) {
        uint32_t r = NOCHAIN;
        if (it < n)
          for (uint32_t x = (uint32_t)r0; x != NOCHAIN; x = L.sort.v[1][x])
            if ((int64_t)x > last && x < r) r = x;
        const uint64_t rel = it < n ? (L.sort.k[0][r] >> 32) : INF;
        if (it > 0 && rel > cur_rel && pending) {
          // flush the inline children of this node's events at cur_rel (ranks in [ts0_rank, r))
          for (uint32_t x = (uint32_t)r0; x != NOCHAIN; x = L.sort.v[1][x]) {
            if (x < ts0_rank || x >= r) continue;
            const uint32_t ncr = L.nchild[x];
            for (uint32_t j = 0; j < ncr; j++) {
              const uint32_t sl = x * M.maxc + j;
              if ((M.ch_kind[sl] & 0xffu) != K_FWD_UP) continue;
              Emit E0;
              E0.M = &M;
              E0.now = tmin + cur_rel;
              E0.ctx = c;
              E0.slot0 = 0;
              E0.n = 0;
              bool st0 = false;
              run_event(M, E0, M.ch_kind[sl], M.ch_a[sl], M.ch_pkt[sl], sink, &ttl_drops, &no_route, &unreach,
                        &st0);
            }
          }
          pending = 0;
        }
        if (it == n) break;
        if (it == 0 || rel > cur_rel) {
          ts0_rank = r;
          cur_rel = rel;
        }
        const uint32_t pi = L.sort.v[0][r];
        Emit E;
        E.M = &M;
        E.now = tmin + rel;
        E.ctx = c;
        E.slot0 = r * M.maxc;
        E.n = 0;
        bool stop = false;
        const bool was_cancelled = run_event(M, E, M.ev_kind[cur][pi], M.ev_a[cur][pi], M.ev_pkt[cur][pi], sink,
                                             &ttl_drops, &no_route, &unreach, &stop);
        cancelled += was_cancelled;
        L.nchild[r] = E.n;
        if (stop) L.stop_flag = 1;
        uint32_t ni = 0;
        if (rel < inline_ts_limit)
          for (uint32_t j = 0; j < E.n; j++) ni += (M.ch_kind[E.slot0 + j] & 0xffu) == K_FWD_UP;
        L.ninl[r] = ni;
        pending += ni;
        last = r;
      }
    }
    __syncthreads();
    PSTAMP(4);
    // ---- 5. uids: exclusive scan of child counts in rank order; dispatch ranks; children -> next pool ----
    uint32_t nc[RPT], ni4[RPT], tsum = 0, isum = 0;
#pragma unroll
    for (int q = 0; q < RPT; q++) {
      nc[q] = L.nchild[tid * RPT + q];
      ni4[q] = L.ninl[tid * RPT + q];
      tsum += nc[q];
      isum += ni4[q];
    }
    uint32_t total_children, total_inline;
    uint32_t base = block_exscan(tsum, L.wsum, &total_children);
    uint32_t ibase = block_exscan(isum, L.wsum, &total_inline);
    {
      uint32_t ib = ibase;
#pragma unroll
      for (int q = 0; q < RPT; q++) {
        L.iprefix[tid * RPT + q] = ib;
        ib += ni4[q];
      }
    }
    __syncthreads();
    // dispatch rank of main event r = r + #inline children with ts < ts_r; of the i-th inline child
    // of r = (#main events with ts <= ts_r) + iprefix[r] + i  (inline children are key-sorted by r)
    auto first_same = [&](uint32_t r, uint64_t rel) -> uint32_t {
      uint32_t lo = 0, hi = r;
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if ((L.sort.k[0][mid] >> 32) < rel) lo = mid + 1;
        else hi = mid;
      }
      return lo;
    };
    auto last_same = [&](uint32_t r, uint64_t rel) -> uint32_t {
      uint32_t lo = r + 1, hi = W;
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if ((L.sort.k[0][mid] >> 32) <= rel) lo = mid + 1;
        else hi = mid;
      }
      return lo - 1;
    };
#pragma unroll 1
    for (int q = 0; q < RPT; q++) {
      const uint32_t r = tid * RPT + q;
      if (r < W) {
        const uint64_t pk = L.sort.k[0][r];
        const uint64_t rel = pk >> 32;
        const uint64_t t = tmin + rel;
        const uint32_t u = (uint32_t)pk;
        const bool dup_prev = r > 0 && (L.sort.k[0][r - 1] >> 32) == rel;
        const uint32_t f = total_inline ? (dup_prev ? first_same(r, rel) : r) : r;
        const uint64_t rk = K + r + (total_inline ? L.iprefix[f] : 0);
        digest += digest_term(rk, t, u);
        if (rk < M.log_cap) {
          M.log_ts[rk] = t;
          M.log_uid[rk] = u;
          M.log_ctx[rk] = M.ev_ctx[cur][L.sort.v[0][r]];
        }
        if (r == W - 1) last_ts = t;
        uint32_t lastr = 0;
        const uint32_t nir = L.ninl[r], ncr = L.nchild[r];
        if (nir) lastr = (r + 1 < W && (L.sort.k[0][r + 1] >> 32) == rel) ? last_same(r, rel) : r;
        uint32_t ii = 0, nonin = base - (ibase);  // non-inline children before this rank
        for (uint32_t j = 0; j < ncr; j++) {
          const uint32_t sl = r * M.maxc + j;
          const uint32_t cu = uid + base + j;
          if ((M.ch_kind[sl] & 0xffu) == K_FWD_UP) {
            if (rel < inline_ts_limit) {  // dispatched inside this window
              const uint64_t crk = K + lastr + 1 + L.iprefix[r] + ii;
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
          const uint64_t o = P + nonin;
          nonin++;
          if (o < M.pool_cap) {
            M.ev_ts[nxt][o] = M.ch_ts[sl];
            M.ev_uid[nxt][o] = cu;
            M.ev_ctx[nxt][o] = M.ch_ctx[sl];
            M.ev_kind[nxt][o] = M.ch_kind[sl];
            M.ev_a[nxt][o] = M.ch_a[sl];
            M.ev_pkt[nxt][o] = M.ch_pkt[sl];
          } else {
            atomicOr(M.error, 1u);
          }
        }
        base += ncr;
        ibase += nir;
      }
    }
    // (inline children at the Stop's ts are scheduled — uids consumed — but never dispatched; the run
    //  ends with this window, so the pool bookkeeping below only has to be right for other windows)
    K += W + total_inline;
    uid += total_children;
    P += total_children - total_inline;
    cur = nxt;
    windows++;
    max_window = W > max_window ? W : max_window;
    __syncthreads();
    if (L.stop_flag) break;
    if (P > M.pool_cap) {
      if (tid == 0) atomicOr(M.error, 1u);
      break;
    }
    __threadfence_block();
  }

  if (M.prof && tid == 0)
    for (int i = 0; i < 16; i++) M.prof[i] = pacc[i];
#undef PSTAMP
  // ---- reduce and publish counters ----
  __syncthreads();
  uint64_t vals[5] = {digest, cancelled, ttl_drops, no_route, unreach};
  for (int k = 0; k < 5; k++) {
    uint64_t v = vals[k];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if (lane == 0) L.wmin[wid] = v;
    __syncthreads();
    if (tid == 0) {
      uint64_t s = 0;
      for (int w = 0; w < P2P_THREADS / 64; w++) s += L.wmin[w];
      vals[k] = s;
    }
    __syncthreads();
  }
  // last dispatched ts: carried by the thread that saw rank W-1 of the final window
  if (last_ts) atomicMax((unsigned long long *)&M.stats->final_ts, (unsigned long long)last_ts);
  if (tid == 0) {
    M.stats->dispatched = K;
    M.stats->digest = vals[0];
    M.stats->cancelled = vals[1];
    M.stats->ttl_drops = vals[2];
    M.stats->no_route_drops = vals[3];
    M.stats->unreach_drops = vals[4];
    M.stats->next_uid = uid;
    M.stats->windows = (uint32_t)windows;
    M.stats->max_window = max_window;
  }
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
  TRY(dalloc(h, &M.stats, 1));
  TRY(dalloc(h, &M.error, 4));
  M.log_cap = log_cap;
  TRY(dalloc(h, &M.log_ts, log_cap));
  TRY(dalloc(h, &M.log_uid, log_cap));
  TRY(dalloc(h, &M.log_ctx, log_cap));
  M.max_windows = ~0ull;
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
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void *)p2p_run, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)sizeof(P2PLds));
    if (e != hipSuccess) {
      nsgpu_p2p_destroy(h);
      return set_error(NSGPU_EHIP, "hipFuncSetAttribute(p2p_run, %zu B LDS): %s", sizeof(P2PLds),
                       hipGetErrorString(e));
    }
    attr = true;
  }
  TRY(dalloc(h, &h->d_M, 1));
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
  NSGPU_HIP(hipMemsetAsync(M.stats, 0, sizeof(nsgpu_p2p_stats), s));
  NSGPU_HIP(hipMemsetAsync(M.error, 0, 4 * sizeof(uint32_t), s));
  return NSGPU_OK;
}

extern "C" int nsgpu_p2p_set_profile(nsgpu_p2p *h, uint64_t *d_phase_cycles) {
  if (!h) return set_error(NSGPU_EINVAL, "nsgpu_p2p_set_profile: null");
  h->M.prof = d_phase_cycles;
  return NSGPU_OK;
}

extern "C" int nsgpu_p2p_run(nsgpu_p2p *h, void *stream) {
  if (!h) return set_error(NSGPU_EINVAL, "nsgpu_p2p_run: null");
  NSGPU_HIP(hipMemcpyAsync(h->d_M, &h->M, sizeof(P2PDev), hipMemcpyHostToDevice, (hipStream_t)stream));
  hipLaunchKernelGGL(p2p_run, dim3(1), dim3(P2P_THREADS), sizeof(P2PLds), (hipStream_t)stream, h->d_M,
                     h->sink_of_node);
  NSGPU_HIP(hipGetLastError());
  return NSGPU_OK;
}

extern "C" int nsgpu_p2p_results(nsgpu_p2p *h, nsgpu_p2p_stats *stats, nsgpu_dev_counters *devc,
                                 nsgpu_app_counters *appc, uint64_t *log_ts, uint32_t *log_uid, uint32_t *log_ctx,
                                 uint64_t log_n, uint32_t *error, void *stream) {
  if (!h) return set_error(NSGPU_EINVAL, "nsgpu_p2p_results: null");
  hipStream_t s = (hipStream_t)stream;
  const P2PDev &M = h->M;
  if (stats) NSGPU_HIP(hipMemcpyAsync(stats, M.stats, sizeof(*stats), hipMemcpyDeviceToHost, s));
  if (devc) NSGPU_HIP(hipMemcpyAsync(devc, M.devc, M.n_devices * sizeof(*devc), hipMemcpyDeviceToHost, s));
  if (appc) NSGPU_HIP(hipMemcpyAsync(appc, M.appc, M.n_apps * sizeof(*appc), hipMemcpyDeviceToHost, s));
  if (log_n > M.log_cap) log_n = M.log_cap;
  if (log_ts && log_n) NSGPU_HIP(hipMemcpyAsync(log_ts, M.log_ts, log_n * 8, hipMemcpyDeviceToHost, s));
  if (log_uid && log_n) NSGPU_HIP(hipMemcpyAsync(log_uid, M.log_uid, log_n * 4, hipMemcpyDeviceToHost, s));
  if (log_ctx && log_n) NSGPU_HIP(hipMemcpyAsync(log_ctx, M.log_ctx, log_n * 4, hipMemcpyDeviceToHost, s));
  uint32_t err = 0;
  NSGPU_HIP(hipMemcpyAsync(&err, M.error, 4, hipMemcpyDeviceToHost, s));
  NSGPU_HIP(hipStreamSynchronize(s));
  if (error) *error = err;
  if (err) return set_error(NSGPU_ENOMEM, "nsgpu_p2p: engine capacity exceeded (code %u: 1 = event pool, "
                                          "4 = window limit, 8 = window cut)", err);
  return NSGPU_OK;
}
