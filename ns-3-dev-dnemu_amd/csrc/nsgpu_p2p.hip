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
// Engines (MI355X).  The simulation advances in conservative windows: W_end = min over pending e of
// (ts_e + L(kind_e)), L = the smallest delay any child of that kind of handler can have, capped at
// the Simulator::Stop key; DefaultSimulatorImpl's uids make a child sort after every pending event
// with ts <= its own, so every pending event with key <= that bound is safe to dispatch.
//   * single GPU: nsgpu_p2p_win.h — k2_pa / k2_handle / k2_scan per window (in-place pool, hub blocks,
//     sorted runs for windows larger than WCAP), replayed from a hipGraph;
//   * partitioned (one rank per GPU, or a loopback group on one GPU): the same k2_pa / k2_handle over
//     each rank's nodes, then k_gtile / k_dfin2 below, with the X0 / X1 / X2 exchanges.
#include <hip/hip_ext.h>
#include <stddef.h>
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
  K_FWD_UP_Q = 13,      // DoForwardUp -> UdpEchoServer / UdpEchoClient::HandleRead (queued: it schedules)
  K_FWD_UP_D = 14,      // a PacketSink DoForwardUp queued like any event: its ts group is cut by a run chunk
  K_NKINDS = 15
};

constexpr int WCAP = 4096;       // events per window
constexpr int TB = 256;          // threads per block, pool sweeps
constexpr int HB = 64;           // threads per block, per-slot kernels (spread over CUs)
constexpr int NHB = WCAP / HB;   // holder blocks of k2_handle
constexpr int RJ = 256;          // keys per rank tile column
constexpr int NJT = WCAP / RJ;   // rank tile columns
constexpr int RTR = 1;           // window keys (rows) per thread of a rank tile (4: same traffic, slower)
constexpr int NRT = WCAP / (HB * RTR);  // rank tile rows
constexpr int NRB = NRT * NJT;   // rank tile blocks (k2_handle)
#ifndef GRID_POOL_N
#define GRID_POOL_N 128  // (r06, with 128-record slot blocks: 128 against 256 blocks, config 4 +1.4 %: ab/p2p_knobs2.log)
#endif
#ifndef GRID_POOL_BIG_N
#define GRID_POOL_BIG_N 256  // (config 5's 5 M-entry pool on one engine: 256 / 128 / 96 / 64 blocks 120.6 / 114.6 / 110.9 / 101.3 M
#endif                       //  ev/s, ab/p2p_pool_blocks.log; config 4 flat from 64 to 128)
constexpr int GRID_POOL_BIG = GRID_POOL_BIG_N;  // ... the single engine's, when the pool capacity is above 2^20 entries
constexpr int GRID_POOL = GRID_POOL_N;
#ifndef GRID_POOL_DIST_N
#define GRID_POOL_DIST_N GRID_POOL_N
#endif
constexpr int GRID_POOL_DIST = GRID_POOL_DIST_N;  // k2_pa<DIST>'s whole grid (slot, remote, chunk and pool blocks)   // blocks of the pool sweep (grid-stride; r06: 1,024 measured slower on
                                         // config 4 and on the dumbbell's 5 M-entry pool: per-block reductions)
#ifndef PA_SLOT_LANES
#define PA_SLOT_LANES 128        // k2_pa (single engine): last-window records per slot block (r06: 128 against 256,
                                 // config 4 +0.7 %, k2_pa ~10.3 -> ~9.8 us; profiles/r06/ab/p2p_tail_replays_slot_lanes.log)
#endif
constexpr int SCAN_THREADS = 1024;
constexpr int CH = 16;           // events of one node a handler thread sorts in LDS
constexpr int NSLOT = 7;         // per-node slot table entries
constexpr int NTAB = NSLOT + 1;  // words per node table record (count + slots)
#ifndef NWIN_N
#define NWIN_N 32
#endif
#ifndef NWIN_TAIL_N
#define NWIN_TAIL_N 2  // (2 / 4 / 8 / none: 160.4 / 159.9 / 160.3 / 159.5 M ev/s on config 4, interleaved)
#endif
constexpr int NWIN = NWIN_N;     // windows per graph replay
constexpr int NWIN_TAIL = NWIN_TAIL_N;  // ... near the end of a run (drive)
constexpr uint32_t NOCTX = 0xffffffffu;
constexpr uint32_t LOCALBIT = 0x80000000u;  // child record kind: run inside the window as a local record
// a Receive whose node another rank owns (partitioned engines; set by the device step from its record, so
// that k2_pa and k_dfin2 need no owner lookup per child; only K_RECEIVE kind words carry it: their upper bits
// hold no generation)
constexpr uint32_t REMOTEBIT = 0x40000000u;

// Packet descriptor: flow (sending app), IPv4 identification (Ipv4L3Protocol::m_identification of
// the originating node), size in bytes with the headers added so far, IPv4 TTL.
struct Pkt {
  uint32_t app, ipid, size, ttl;
};

// Per-device record of the transmit path: the tx state (busy, queue count / head), the static
// parameters a TransmitStart / TransmitComplete reads and the device's counters, in ONE 128-B line —
// a device step touches one line instead of eleven scattered SoA words (each a separate line fetch
// from another XCD's writes: measured 2.8 -> 1.6 MB HBM fetch per k2_handle launch on config 4).
struct DevRec {
  uint32_t busy, cnt, head, qmax;  // PointToPointNetDevice m_txMachineState, DropTail count / ring head, MaxPackets
  uint32_t peer, peer_node, rkind, pad1;  // rkind: the Receive child's kind word (K_RECEIVE | REMOTEBIT when
  uint64_t bps;                            //   another rank owns the peer's node)
  int64_t ifg, delay;              // InterframeGap, channel Delay
  uint64_t pad2;
  nsgpu_dev_counters c;            // (copied out strided by nsgpu_p2p_results / _counters)
  uint64_t pad3[4];
};
static_assert(sizeof(DevRec) == 128 && offsetof(DevRec, c) == 64, "DevRec is one 128-B line");

// Reduction of a pending set: the next window's bound (atomicMin), the pending Stop.
struct Red {
  uint64_t tmin, wend, stopts;
  uint32_t stopuid, pad;
  uint64_t wendw;  // the wide bound: min over pending of ts + lookw (cross-node lookahead; wide engines)
};

// A deferred window's dispatch bases: what k2_sdef needs once the window's records are staged in rank order.
struct WInfo {
  uint64_t K0, tmin, ilim;  // dispatches before the window, its tmin and inline limit
  uint32_t uid0, N, W, Lt;  // the uid its first child takes; records (gen-0 W + local Lt)
};

// A staged record of a deferred window, at its rank: key (rel ts << 32 | its uid — resolved at staging when it
// was provisional; a local record's key has uid 0: its uid is its parent's child prefix + j, resolved by
// k2_sdef), counts (children | inline children << 9 | the record's dense index << 18), and for a local record
// its parent (the parent's dense index | child index << 24), for a gen-0 record its first inline leaf (its
// context | child index << 24; a local record has none).  Its context is kept beside it (stx).  Stage arrays (and the child prefixes cpt) are indexed by stg_pos(rank): k2_sdef's
// thread t owns the 8 consecutive ranks 8t..8t+7 and loads its q-th one from q * 1024 + t, so every load and
// store of a wave is coalesced.
struct Stg {
  uint64_t key;
  uint32_t cnt, par;
};
static_assert(sizeof(Stg) == 16, "Stg");
constexpr uint32_t STG_NT = 1024;  // k2_sdef's threads (its rank slices)
// Provisional uids (deferred windows): child j of the record of rank r of window n, before window n's child
// prefix is known, is PROV | (n & 1) << 30 | r << 8 | j — above every resolved uid (< UID_DF_LIMIT, checked), so
// keys compare as the final uids do; resolved to uid0(n) + cpt[n & 1][r] + j.
constexpr uint32_t PROV = 0x80000000u, PROV_MAXC = 256, UID_DF_LIMIT = 0x3fe00000u;
// A window's children take at most NMAX x PROV_MAXC = 2^21 uids, so a deferred window that starts below
// UID_DF_SOFT ends below UID_DF_LIMIT; the window that reaches UID_DF_SOFT pauses the deferred pipeline
// (MODE_UIDX) and the scanning pipeline runs the rest of the run (df_usable is false from there on).
constexpr uint32_t UID_DF_SOFT = UID_DF_LIMIT - (1u << 22);
// DefaultSimulatorImpl's m_uid is a uint32 that wraps to 0 after 0xffffffff (default-simulator-impl.cc:52-56,
// 188-219); the wrapped uids would sort before every earlier one at equal ts and uid 2 would read as a
// ScheduleDestroy id.  The engines do not replicate that: a window whose children would take uid 0xffffffff
// or a wrapped one fails the run (error 2048) before any of them runs.  (0xffffffff itself is kept free: it is
// the "none" marker of several engine records.)
constexpr uint64_t UID_MAX_NEXT = nsgpu::UID_NEXT_MAX;
__device__ __forceinline__ uint32_t prov_uid(uint64_t win, uint32_t r, uint32_t j) {
  return PROV | ((uint32_t)(win & 1) << 30) | (r << 8) | j;
}

// Device-resident run control (one per engine).  Every field is written by one kernel of the
// window pipeline and read by later ones, never read and written by different blocks of one kernel
// except through atomics.  Window k: red[(k + 1) & 1] holds the pending set's reduction that bounds
// it; its leftovers and children fold into red[k & 1].
struct Ctl {
  Red red[2];
  uint64_t K;                          // dispatched so far (after the last scanned window)
  uint64_t tmin, bound, inline_lim;    // current window (k2_pa / the partitioned cut)
  uint64_t windows, max_window, last_ts, max_windows, refits;
  uint64_t digest, cancelled, ttl_drops, no_route, unreach, icmp;
  uint64_t pK0, ptmin, pinline_lim;    // the last scanned window, appended by the next k2_pa
  // (W, nxtP, overflow, prep): a partitioned rank's X0 payload, sent from here — its window candidates,
  // (unused), a hub too large for a block, the window is the cut of the last one
  uint32_t puid0, pW, uid, hdl;
  uint32_t W, nxtP, overflow, prep;  // (16-B aligned: the X0 payload)
  uint32_t done, stop_seen, pvalid, pinl;
  // ---- single-GPU engine (k2_*: in-place pool, sorted runs, hub blocks) ----
  uint64_t P_end, live, nfree;  // pool scan range, live pool entries, free-stack entries
  uint64_t r0, rW;              // sorted run: start of the next chunk, run length
  uint64_t split_lo, split_hi;  // run chunk: rel ts of a same-ts group cut at its start / end (~0: none)
  uint64_t wkmax;               // largest window key of the forming window (radix sort width)
  uint64_t npush, nF;           // this window: pool slots freed, children parked in the fresh buffer
  uint32_t mode, rt, nhub, wbase;  // engine mode, red[] accumulating index, hub nodes, chunk base
  uint32_t force_run, hcap;        // a hub too large to sort in a block: dispatch the window as a run;
                                   // the window is cut at the next host event (pause after it)
  uint64_t hts, hrel;              // next host event (nsgpu_p2p_advance): ts (~0: none); the rel ts of the
  uint32_t huid, gt_tinl;          //   window's last timestamp (W_end or the host event's); the host uid;
  uint32_t gt_lown, gt_pad;        //   k_gtile -> k_dfin2: the merged window's inline children, this rank's
                                   //   local records (from the X1 headers: k_dfin2's record blocks read none)
  uint64_t pchild;                 // children of the last scanned window that stay pending (not inline)
  // ---- wide windows (nsgpu_p2p_win.h; partitioned: k_gtile / k_dfin2): same-node TransmitCompletes run inside ----
  uint64_t lim_rel;   // a TransmitComplete child with rel ts < lim_rel is a local record of this window
  uint64_t nbound;    // the narrow bound of the forming window (an overflowing wide window is trimmed to it)
  uint64_t tn0;       // trace records before this window's handlers (the local records' uid patch)
  uint64_t span_t;    // adaptive span target of wide windows (kept between the narrow and the wide bound)
  uint32_t plt;       // local records of the last scanned window (lrec)
  uint32_t renarrow;  // the overflowing window is wide: trim its sorted run to nbound (host step)
  // ---- sorted runs: the chunk being dispatched ends at rnext; rtrim: the run ends after it (k_trim) ----
  uint64_t rnext;
  uint32_t rtrim, pad5;
  // ---- deferred dispatch accounting (single wide engine, nsgpu_p2p_win.h "deferred windows") ----
  uint64_t acc_tc, acc_tinl;  // this window's children / inline children (k2_handle accumulates)
  uint32_t pdf;               // the window the next k2_pa appends is staged (1) or appended from sinfo (0)
  uint32_t sflag;             // k2_pa staged a window for k2_sdef: 1 | (its window index & 3) << 1 (k2_pa writes
                              // it every window; k2_sdef's blocks only read it)
  uint32_t rk_W, rk_go;       // k2_handle's snapshot for k2_rank (window size; it was handled, normally)
  uint64_t rk_win, rk_lim;    //   (its window index, lim_rel): k2_rank's bookkeeping block rewrites C.W etc.
  WInfo winfo[4];             // window n's dispatch bases (k2_rank's bookkeeping), at n & 3
  // ---- partitioned sorted runs (a window some rank cannot hold: every rank sorts its candidates once and the
  // run is dispatched in chunks cut at a common key; k_drun_*, k2_pa's chunk role, k_dfin2) ----
  uint32_t drun, drpad;       // a run is being dispatched (every rank alike)
  uint64_t dr0, drW, dr1;     // this rank's run: next entry, length (rn_* arrays); past the chunk being formed
  uint64_t drg;               // the next chunk's cut key (from the ranks' fitting and head keys, k_dfin2)
  uint64_t drlo;              // the next chunk continues the same-ts group the last one cut: its rel ts (~0: no)
  uint32_t drtrim, dtrim;     // the next chunk ends that group and the run after it; the run ended so: the next
                              // k2_pa returns this rank's entries left that are not in the pool to pending
  uint64_t drn_tmin, drn_wend;  // the pending set's reduction at the run's start, its own entries included (k2_pa
  uint64_t drn_stopts;          // folds it into every chunk's instead of sweeping the pool)
  uint32_t drn_stopuid, drpad2;
  uint64_t drb_tmin, drb_span, drb_bound, drb_stop, drb_nbound, drb_lim;  // the run window's bound (WinBound)
  uint64_t drn_wendw;  // (wide partitioned engines) the wide bound's part of drn_*
  uint64_t drcut;      // (wide partitioned engines) the run's candidates up to the narrow bound (k_drun_trim)
  // ---- hub windows of the narrow engines: the hub events' stateless node parts by their slots' threads ----
  uint32_t hub_rdy;    // holder blocks done with them (k2_pa zeroes it; the hub blocks wait for NHB)
  uint32_t hub_ser;    // some hub event's node part touches node state (its hub block runs those serially)
};

static_assert(offsetof(Ctl, prep) == offsetof(Ctl, W) + 12 && offsetof(Ctl, W) % 16 == 0, "the X0 payload");

// Device-resident model + engine state (all pointers are HBM).  Passed to the kernels by value.
// A window record's place in the dispatch order, for the wide windows' ranking (k2_rank): the chain of
// records from it up to its gen-0 ancestor (a local record is a same-node TransmitComplete run inside the
// window; its parent is the event whose TransmitStart made it).  A gen-0 record is a chain of length 0.
// Order (ts, uid): a local record's uid is its parent's child prefix + its child index, so among records of
// one ts the gen-0 ones come first (older uids), and local ones follow their parents' order, then j.
constexpr int LKD = 8;  // chain levels kept: a record and up to 7 local ancestors (create: Lx <= 8 tx_min)
struct LKey {
  uint32_t rel[LKD];  // rel[t]: rel ts of the chain's level-t record (level 0: this one)
  uint32_t uid;       // the gen-0 ancestor's uid (level `depth`)
  uint32_t depth;     // local records in the chain (0: a gen-0 record)
  uint32_t pad[2];
  uint8_t j[16];      // j[t]: the level-t local record's child index in its parent
};
static_assert(sizeof(LKey) == 64, "LKey: four 16-B loads");

struct P2PDev {
  // scenario
  uint32_t n_nodes, n_devices, n_apps, n_dst, qcap, maxc;
  const uint32_t *dev_node;
  const uint32_t *route;  // dense [node][slot], or null: the compressed table below
  const uint32_t *route_def, *route_exc_slot, *route_exc_dev;
  const uint64_t *route_exc_off;
  const uint32_t *app_kind, *app_node, *app_dst_node, *app_dst_slot, *app_pkt_size, *app_max_bytes, *app_ttl;
  const int64_t *app_start, *app_stop;
  const uint64_t *app_rate;
  const double *app_on_s, *app_off_s;
  const uint32_t *app_count, *app_src_slot;  // UdpEchoClient MaxPackets, route slot of its own node
  const int64_t *app_interval;               // UdpEchoClient Interval
  const uint32_t *node_app_off, *node_app_list;  // CSR: apps of each node in AddApplication order
  const int32_t *sink_of_node;                    // PacketSink of each node (-1: none)
  uint32_t icmp;                                  // ICMP errors are generated (scenario icmp)
  int64_t lookahead[K_NKINDS];
  int64_t lookw[K_NKINDS];  // wide windows: the smallest delay of a child that does not run in the window
  uint32_t wide, pad_w;     // wide windows on
  // model state
  DevRec *dev;  // per-device tx state + transmit parameters (one record per device)
  Pkt *q_buf;
  uint32_t *app_flags;    // bit0 started, bit1 sink active, bit2 send live, bit3 start/stop live
  uint32_t *app_send_gen, *app_ss_gen, *app_residual, *app_tot;
  uint32_t *node_ipid;    // Ipv4L3Protocol::m_identification per node
  uint64_t *app_last_start;
  nsgpu_app_counters *appc;
  // pending pool (double-buffered SoA)
  uint64_t *ev_ts[2];
  uint32_t *ev_uid[2], *ev_ctx[2], *ev_kind[2], *ev_a[2];
  Pkt *ev_pkt[2];
  uint64_t pool_cap;
  // the current window (WCAP slots): slot records (k2_pa) ...
  uint64_t *wkey;
  uint32_t *wctx, *wkind, *wa, *widx;
  Pkt *wpkt;
  // ... handler outputs: child counts and child records (slot * maxc + j, Schedule-call order) ...
  uint32_t *nchild, *ninl;
  uint64_t *ch_ts;
  uint32_t *ch_ctx, *ch_kind, *ch_a;
  Pkt *ch_pkt;
  // ... dispatch info per slot (k2_scan / k_dfin2), and the keys / contexts kept for the next k2_pa
  // (which rewrites wkey / wctx with the next window while it appends this one)
  uint4 *sinfo;
  uint64_t *pwkey;
  uint32_t *pwctx;
  uint32_t *wrank;  // rank accumulators of the current window (0 between windows)
  // per-node slot tables of the current window, one 32-B record per node: [0] the node's window
  // events (0 between windows), [1 .. NSLOT] their first slots (one line per node, not two)
  uint32_t *node_tab;
  // partitioned run (dist != 0): this engine owns the nodes n with owner[n] == rank
  uint32_t dist, rank, nranks, pad_d;
  const uint32_t *owner;
  uint64_t *x0_send, *x0_recv;  // X0: 16 B per rank (x0_send points at the run control's X0 payload)
  uint64_t *xk_send, *xk_recv;  // the cut's exchange (host-driven): one rank's largest fitting key (16 B)
  uint8_t *x1_send, *x1_recv;   // X1: X1B bytes per rank (header, the rank's records in dispatch order: SEnt)
  uint8_t *x1_own;              // this rank's window lists, not exchanged: X1Ent x WCAP, then X1Loc x XLCAP
  uint8_t *x2_send, *x2_recv;   // X2: x2b bytes per peer
  uint32_t capx, pad_x;         // X2 records per peer per window (the run's largest cut between two ranks)
  uint64_t x2b;                 // X2 bytes per peer
  uint32_t *gacc;               // k_gtile's accumulators: 2 x NACC packed 64-bit words
  // run control / outputs
  uint32_t n_init;    // initial pending count (pool 0)
  uint32_t uid_init;  // m_uid after setup
  Ctl *C;
  uint32_t *error;  // non-zero = capacity exceeded (code)
  uint64_t *log_ts;
  uint32_t *log_uid, *log_ctx;
  uint64_t log_cap;
  // ascii/pcap trace sink calls (nsgpu_p2p_set_trace; null: tracing off), unordered
  nsgpu_trace_record *trace;
  uint64_t trace_cap;
  unsigned long long *trace_n;
  uint32_t trace_kinds, pad_tk;  // nsgpu_trace_kind bits recorded (nsgpu_p2p_set_trace_kinds)
  // ---- single-GPU engine (k2_*) ----
  uint64_t runcap;        // capacity of the window record arrays (a sorted run may hold the whole pool)
  uint32_t *wsrc;         // pool slot each window record came from (NOSRC: a child of the last window)
  uint64_t *f_ts;         // fresh buffer: children of the last window that stay pending (moved into
  uint32_t *f_uid, *f_ctx, *f_kind, *f_a;  // the pool by k2_handle's maintenance blocks)
  Pkt *f_pkt;
  uint64_t fcap;
  uint32_t *fstack;       // free pool slots (stack)
  uint32_t *hub_list;     // nodes with more than CH window events (hub blocks)
  struct HubEv *hx;       // hub blocks: per-slot node-part results
  uint64_t *hub_key;      // hub blocks: the hub's events in key order (NHUB x WCAP)
  uint32_t *hub_slot;     // (then WCAP more: hub_mark.  P2PDev is passed by value: one more pointer here made the
                          //  compiler copy the whole struct into scratch, 1.4 KB a lane, in k2_handle)
  uint64_t *s_key2;       // radix sort / compaction scratch
  uint32_t *s_val, *s_val2, *s_hist, *g_u32;
  Pkt *g_pkt;
  uint64_t *cmp_cnt;      // compaction: live entries written
  // ---- wide windows: local records (same-node TransmitCompletes run inside the window) ----
  uint32_t *wpar;         // local record: parent record | child index << 24
  uint32_t *lcnt;         // local records per region this window (one region per holder / hub block)
  uint32_t *lrec;         // the last scanned window's local records (dense list, C.plt of them)
  LKey *lkey;             // [LCAP] the local records' chains (k2_rank: the rare exact compare)
  ulonglong2 *lkw;        // [LCAP] their chain order packed into two words (lk_word, lk_word2)
  uint4 *ldat;            // [LMAX] the window's local records in dense order (k2_rank -> k2_scan): record,
                          // child counts (n | inline << 16), rel ts, parent (wpar)
  uint32_t *lrank;        // [LMAX] their rank accumulators (k2_rank; 0 between windows)
  // ---- deferred windows (wrank / lrank are then 2 x WTOT / 2 x LMAX: by window parity) ----
  struct Stg *stage;      // [NMAX] a window's records by stg_pos(rank) (k2_pa stages, k2_sdef reads)
  uint32_t *stx;          // [NMAX] their contexts (stg_pos)
  uint2 *sleaf;           // [NMAX][maxc] their further inline leaves: (context, child index) (by rank, entry 0 unused)
  uint32_t *cpt;          // [2][NMAX] child prefix by rank (k2_sdef): provisional uids resolve through it
  uint32_t *ldpd;         // [LMAX] the dense list's parents as dense indices | child index << 24 (k2_rank -> k2_pa)
  uint32_t sdef_fold;     // df_sdef runs as k2_rank's blocks 1 .. NSDEF (1) or as its own kernel k2_sdef (0)
  // ---- partitioned sorted runs: this rank's candidates of the run window, in key order (runcap each) ----
  uint64_t *rn_key;
  uint32_t *rn_ctx, *rn_kind, *rn_a, *rn_src;
  Pkt *rn_pkt;
};

// ---------------- wave / block helpers ----------------
// Wave reductions (every lane of the wave active; the result in every lane): within each row of 16 lanes by DPP
// moves — quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror: each step pairs a lane with one of the other
// half of its group, so after four steps every lane holds its row's value — then the four rows' values read into
// scalars (v_readlane).  (The __shfl_xor butterflies were 6 dependent ds_bpermute rounds, LDS-latency each: the
// holders' five counter sums alone cost config 4 ~0.5 us a window.)
template <int CTRL>
__device__ __forceinline__ uint32_t dpp32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xf, 0xf, false);
}
template <int CTRL>
__device__ __forceinline__ uint64_t dpp64(uint64_t v) {
  return ((uint64_t)dpp32<CTRL>((uint32_t)(v >> 32)) << 32) | dpp32<CTRL>((uint32_t)v);
}
__device__ __forceinline__ uint32_t rl32(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); }
__device__ __forceinline__ uint64_t rl64(uint64_t v, int l) { return ((uint64_t)rl32((uint32_t)(v >> 32), l) << 32) | rl32((uint32_t)v, l); }
constexpr int DPP_X1 = 0xB1, DPP_X2 = 0x4E, DPP_HMIRROR = 0x141, DPP_MIRROR = 0x140;
__device__ __forceinline__ uint64_t wave_min64(uint64_t v) {
  uint64_t w;
  w = dpp64<DPP_X1>(v), v = w < v ? w : v;
  w = dpp64<DPP_X2>(v), v = w < v ? w : v;
  w = dpp64<DPP_HMIRROR>(v), v = w < v ? w : v;
  w = dpp64<DPP_MIRROR>(v), v = w < v ? w : v;
  const uint64_t a = rl64(v, 0), b = rl64(v, 16), c = rl64(v, 32), d = rl64(v, 48);
  const uint64_t x = a < b ? a : b, y = c < d ? c : d;
  return x < y ? x : y;
}
__device__ __forceinline__ uint64_t wave_max64(uint64_t v) {
  uint64_t w;
  w = dpp64<DPP_X1>(v), v = w > v ? w : v;
  w = dpp64<DPP_X2>(v), v = w > v ? w : v;
  w = dpp64<DPP_HMIRROR>(v), v = w > v ? w : v;
  w = dpp64<DPP_MIRROR>(v), v = w > v ? w : v;
  const uint64_t a = rl64(v, 0), b = rl64(v, 16), c = rl64(v, 32), d = rl64(v, 48);
  const uint64_t x = a > b ? a : b, y = c > d ? c : d;
  return x > y ? x : y;
}
__device__ __forceinline__ uint32_t wave_sum32(uint32_t v) {
  v += dpp32<DPP_X1>(v);
  v += dpp32<DPP_X2>(v);
  v += dpp32<DPP_HMIRROR>(v);
  v += dpp32<DPP_MIRROR>(v);
  return rl32(v, 0) + rl32(v, 16) + rl32(v, 32) + rl32(v, 48);
}
__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
  v += dpp64<DPP_X1>(v);
  v += dpp64<DPP_X2>(v);
  v += dpp64<DPP_HMIRROR>(v);
  v += dpp64<DPP_MIRROR>(v);
  return rl64(v, 0) + rl64(v, 16) + rl64(v, 32) + rl64(v, 48);
}
// Inclusive wave scans by DPP (every lane active): row_shr 1 / 2 / 4 / 8 within each row of 16 (a lane without a
// source adds 0), then row_bcast:15 (rows 1 and 3 add the previous row's last lane) and row_bcast:31 (rows 2 and 3
// add lane 31) — six DPP steps instead of six ds_bpermute rounds.
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ uint32_t dppm32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWS, 0xf, false);
}
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ uint64_t dppm64(uint64_t v) {
  return ((uint64_t)dppm32<CTRL, ROWS>((uint32_t)(v >> 32)) << 32) | dppm32<CTRL, ROWS>((uint32_t)v);
}
__device__ __forceinline__ uint32_t wave_incscan32(uint32_t v) {
  v += dppm32<0x111>(v);
  v += dppm32<0x112>(v);
  v += dppm32<0x114>(v);
  v += dppm32<0x118>(v);
  v += dppm32<0x142, 0xa>(v);
  v += dppm32<0x143, 0xc>(v);
  return v;
}
__device__ __forceinline__ uint64_t wave_incscan64(uint64_t v) {
  v += dppm64<0x111>(v);
  v += dppm64<0x112>(v);
  v += dppm64<0x114>(v);
  v += dppm64<0x118>(v);
  v += dppm64<0x142, 0xa>(v);
  v += dppm64<0x143, 0xc>(v);
  return v;
}
__device__ __forceinline__ uint32_t wave_exscan32(uint32_t v, int lane) {
  (void)lane;
  return wave_incscan32(v) - v;
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
// Children of the event being run go to its slot's child records in Schedule-call order; the ones
// that stay pending fold into the next window's reduction (tmn, wnd).
struct Emit {
  uint64_t now;
  uint32_t ctx;
  uint32_t slot0;  // slot * maxc
  uint32_t n;
  uint64_t *ch_ts;
  uint32_t *ch_ctx, *ch_kind, *ch_a;
  Pkt *ch_pkt;
  const int64_t *lookahead, *lookw;
  uint64_t tmn, wnd, wndw;
  uint64_t lim_abs;  // wide window: a TransmitComplete child before it is a local record (0: none)
  uint32_t uid;      // uid of the event being run (its trace records; a local record's: its record index, tloc)
  bool tloc = false; // the event is a local record whose uid k2_scan assigns later (k_tpatch resolves its records)
  uint32_t trseq;    // trace sink calls made by it so far
  bool demote;       // the event's ts group is cut by a run chunk: its DoForwardUp leaves are queued
  int32_t lj;        // the local child this event made (an event makes at most one TransmitComplete): its
  uint32_t la, lctx; //   index (-1: none), device and context
  uint64_t lts;
  __device__ __forceinline__ void child(int64_t delay, uint32_t ctx_, uint32_t kind, uint32_t a, Pkt p) {
    if (demote && kind == K_FWD_UP) kind = K_FWD_UP_D;
    const uint32_t s = slot0 + n++;
    const uint64_t ts = now + (uint64_t)delay;
    // a same-node TransmitComplete inside a wide window runs in it (the node's holder takes it next)
    const bool local = kind == K_TX_COMPLETE && ts < lim_abs;
    ch_ts[s] = ts;
    ch_ctx[s] = ctx_;
    ch_kind[s] = local ? (kind | LOCALBIT) : kind;
    if (local) {
      lj = (int32_t)(s - slot0);
      lts = ts;
      la = a;
      lctx = ctx_;
    }
    ch_a[s] = a;
    ch_pkt[s] = p;
    if ((kind & 0xffu) != K_FWD_UP && !local) {  // DoForwardUp is a leaf run inside the window, never re-queued
      tmn = ts < tmn ? ts : tmn;
      const uint64_t e = ts + (uint64_t)lookahead[kind & 0xffu];
      wnd = e < wnd ? e : wnd;
      if (lookw) {  // (wide engines)
        const uint64_t ew = ts + (uint64_t)lookw[kind & 0xffu];
        wndw = ew < wndw ? ew : wndw;
      }
    }
  }
};

// Run statistics of one handler thread.
struct HStat {
  uint32_t cancelled, ttl_drops, no_route, unreach, icmp;  // (one holder's window: 32 bits; 64-bit fields were spilled to scratch)
  bool stop;
};

// Device step of an event (second phase of every handler, run by all lanes together so the wave
// does not serialise one copy per event kind):
//   SEND  PointToPointNetDevice::Send (point-to-point-net-device.cc:462-518): PppHeader, enqueue
//         (DropTail: queue.cc:61-97, drop-tail-queue.cc:83-100), and if the device is idle dequeue
//         + TransmitStart;
//   KICK  TransmitComplete (:304-346): device idle, dequeue, TransmitStart if a packet was queued.
// TransmitStart (:206-269) + PointToPointChannel::TransmitStart (point-to-point-channel.cc:82-103):
//   Schedule (txTime + ifg, TransmitComplete); ScheduleWithContext (peer node, txTime + delay, Receive).
enum : uint32_t { ACT_NONE = 0, ACT_SEND = 1, ACT_KICK = 2 };

// One ascii trace sink call (AsciiTraceHelper::Default*SinkWithContext, trace-helper.cc:303-390, as
// hooked by PointToPointHelper::EnableAsciiInternal, point-to-point-helper.cc:113-219): appended
// unordered; the host orders the records by (ts, uid, seq).
__device__ __forceinline__ void trace_call(const P2PDev &M, Emit &E, uint32_t kind, uint32_t d, const Pkt &p) {
  if (!M.trace || !((M.trace_kinds >> kind) & 1u)) return;
  nsgpu_trace_record r;
  r.ts = E.now;
  r.uid = E.uid;
  r.seq = (uint16_t)E.trseq++;
  r.kind = (uint8_t)kind;
  r.pad_ = E.tloc ? 1 : 0;  // (k_tpatch replaces a local record's index by its uid and clears the flag)
  r.dev = d;
  r.app = p.app;
  r.ipid = p.ipid;
  r.size = p.size;
  r.ttl = p.ttl;
  r.pad2_ = 0;
  const unsigned long long i = atomicAdd(M.trace_n, 1ull);
  if (i < M.trace_cap) M.trace[i] = r;
}
struct Act {
  uint32_t op, dev;
  Pkt p;
};
// Ipv4L3Protocol::m_dropTrace (ipv4-l3-protocol.cc:505,835): the datagram as received (a UDP datagram's
// 16-bit identification); d = the receiving device (DROP_NO_ROUTE) or the forwarding route's
// (DROP_TTL_EXPIRED).
__device__ __forceinline__ void trace_ip_drop(const P2PDev &M, Emit &E, uint32_t d, Pkt p) {
  if (!(p.app & NSGPU_PKT_ICMP)) p.ipid &= 0xffffu;
  trace_call(M, E, NSGPU_TR_IP_DROP, d, p);
}
// The TTL-expired datagram a time-exceeded error e was made from (icmp_error below embeds its flow, reply
// flag, identification and length; it arrived with TTL 1): its Drop record follows the error's Send.
__device__ __forceinline__ void trace_te_drop(const P2PDev &M, Emit &E, uint32_t d, const Pkt &e) {
  const uint32_t app = (e.app & NSGPU_PKT_APP) | ((e.app & NSGPU_PKT_ICMP_OF_REPLY) ? NSGPU_PKT_REPLY : 0u);
  trace_call(M, E, NSGPU_TR_IP_DROP, d, Pkt{app, e.ipid >> 16, e.ttl >> 16, 1u});
}

__device__ __forceinline__ void device_act(const P2PDev &M, Emit &E, const Act &act) {
  if (act.op == ACT_NONE) return;
  const uint32_t d = act.dev;
  // every operand of the step at once
  const DevRec dr = M.dev[d];
  const uint32_t busy = dr.busy, cnt = dr.cnt, head = dr.head, qmax = dr.qmax;
  nsgpu_dev_counters dc = dr.c;
  const uint64_t bps = dr.bps;
  const int64_t ifg = dr.ifg, delay = dr.delay;
  const uint32_t peer = dr.peer;
  const uint32_t peer_node = dr.peer_node;
  Pkt *qb = M.q_buf + (uint64_t)d * M.qcap;
  uint32_t ncnt = cnt, nhead = head, nbusy = busy;
  bool go = false;
  Pkt tx{0, 0, 0, 0};
  if (act.op == ACT_SEND) {
    trace_call(M, E, NSGPU_TR_IP_TX, d, act.p);  // SendRealOut: m_txTrace, then the device's Send
    Pkt p = act.p;
    p.size += 2;  // PppHeader
    if (cnt >= qmax) {
      trace_call(M, E, NSGPU_TR_DROP, d, p);  // Queue::Drop: m_traceDrop
      dc.drop_packets++;
      dc.drop_bytes += p.size;
    } else {
      trace_call(M, E, NSGPU_TR_ENQUEUE, d, p);  // Queue::Enqueue: m_traceEnqueue
      dc.enq_packets++;
      dc.enq_bytes += p.size;
      if (busy == 0) {  // Enqueue + Dequeue: the head of the queue leaves at once
        if (cnt == 0) {
          tx = p;  // (the ring slot would be written and read back: skip it)
        } else {
          qb[(head + cnt) % M.qcap] = p;
          tx = qb[head];
        }
        nhead = (head + 1) % M.qcap;
        trace_call(M, E, NSGPU_TR_DEQUEUE, d, tx);  // Queue::Dequeue: m_traceDequeue
        dc.deq_packets++;
        go = true;
      } else {
        qb[(head + cnt) % M.qcap] = p;
        ncnt = cnt + 1;
      }
    }
  } else {  // ACT_KICK
    nbusy = 0;
    if (cnt > 0) {
      tx = qb[head];
      nhead = (head + 1) % M.qcap;
      ncnt = cnt - 1;
      trace_call(M, E, NSGPU_TR_DEQUEUE, d, tx);
      dc.deq_packets++;
      go = true;
    }
  }
  if (go) {
    nbusy = 1;
    dc.tx_packets++;
    // Seconds (m_bps.CalculateTxTime (size)): static_cast<double>(bytes)*8/m_bps (data-rate.cc:224-227)
    const int64_t txTime = seconds_to_ts(static_cast<double>(tx.size) * 8 / (double)bps);
    E.child(txTime + ifg, E.ctx, K_TX_COMPLETE, d, Pkt{0, 0, 0, 0});
    E.child(txTime + delay, peer_node, dr.rkind, peer, tx);
  }
  if (nbusy != busy) M.dev[d].busy = nbusy;
  if (ncnt != cnt) M.dev[d].cnt = ncnt;
  if (nhead != head) M.dev[d].head = nhead;
  M.dev[d].c = dc;
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
// Invert (1e9) (int64x64-128.cc:119-134): the same steps, evaluated at compile time (per call, its 128-bit
// divisions took thousands of instructions a lane; a wave of OnOff StopApplications paid them in every window)
constexpr u128 c_umul_by_invert(u128 a, u128 b) {
  const u128 LO = (((u128)1) << 64) - 1;
  return (a >> 64) * (b >> 64) + (((a >> 64) * (b & LO) + (a & LO) * (b >> 64)) >> 64);
}
constexpr u128 c_divu(u128 a, u128 b) {
  const u128 quo = a / b, rem = a % b;
  const bool small = (rem >> 64) == 0;
  return (quo << 64) + (small ? (rem << 64) / b : rem / (b >> 64));
}
constexpr i128 c_invert_1e9() {
  i128 inv = (i128)c_divu(((u128)1) << 64, (u128)1000000000ull);
  const u128 r = c_umul_by_invert((u128)(((i128)1000000000ll) << 64), (u128)inv);
  if ((int64_t)(r >> 64) != 1) inv += 1;
  return inv;
}
__device__ __noinline__ int64_t residual_bits(int64_t delta_ns, uint64_t rate) {
  constexpr i128 inv = c_invert_1e9();
  static_assert((uint64_t)((u128)inv >> 64) == 0x44b82fa09ull && (uint64_t)(u128)inv == 0xb5a52cb98b405448ull,
                "Invert (1e9)");
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

__device__ __forceinline__ void cancel_events(const P2PDev &M, uint32_t a, uint64_t now) {
  uint32_t f = M.app_flags[a];
  if (f & 4u) {  // m_sendEvent.IsRunning ()
    const int64_t delta = (int64_t)now - (int64_t)M.app_last_start[a];
    M.app_residual[a] += (uint32_t)residual_bits(delta, M.app_rate[a]);
  }
  M.app_flags[a] = f & ~(4u | 8u);  // Cancel (m_sendEvent); Cancel (m_startStopEvent)
}

__device__ __forceinline__ void schedule_start_event(const P2PDev &M, Emit &E, uint32_t a) {
  const uint32_t g = (M.app_ss_gen[a] + 1) & 0xffffffu;
  M.app_ss_gen[a] = g;
  M.app_flags[a] |= 8u;
  E.child(seconds_to_ts(M.app_off_s[a]), E.ctx, K_START_SENDING | (g << 8), a, Pkt{0, 0, 0, 0});
}
__device__ __forceinline__ void schedule_stop_event(const P2PDev &M, Emit &E, uint32_t a) {
  const uint32_t g = (M.app_ss_gen[a] + 1) & 0xffffffu;
  M.app_ss_gen[a] = g;
  M.app_flags[a] |= 8u;
  E.child(seconds_to_ts(M.app_on_s[a]), E.ctx, K_STOP_SENDING | (g << 8), a, Pkt{0, 0, 0, 0});
}
__device__ __forceinline__ void stop_application(const P2PDev &M, uint32_t a, uint64_t now) {
  const uint32_t k = M.app_kind[a];
  if (k == NSGPU_APP_SINK || k == NSGPU_APP_ECHO_SERVER) {  // m_socket->Close ()
    M.app_flags[a] &= ~2u;
    return;
  }
  if (k == NSGPU_APP_ECHO_CLIENT) {  // UdpEchoClient::StopApplication: Close; Simulator::Cancel (m_sendEvent)
    M.app_flags[a] &= ~(2u | 4u);
    return;
  }
  cancel_events(M, a, now);
}
// OnOffApplication::ScheduleNextTx (onoff-application.cc:228-252); the child is returned, not
// emitted: in SendPacket it is scheduled after the packet's device children.
struct Post {
  bool valid;
  int64_t delay;
  uint32_t kind, a;
};
__device__ __forceinline__ Post schedule_next_tx(const P2PDev &M, uint32_t a, uint64_t now) {
  Post po{false, 0, 0, 0};
  const uint32_t maxb = M.app_max_bytes[a];
  if (maxb == 0 || M.app_tot[a] < maxb) {
    const uint32_t bits = M.app_pkt_size[a] * 8 - M.app_residual[a];
    const uint32_t g = (M.app_send_gen[a] + 1) & 0xffffffu;
    M.app_send_gen[a] = g;
    M.app_flags[a] |= 4u;
    po.valid = true;
    po.delay = seconds_to_ts(bits / static_cast<double>(M.app_rate[a]));
    po.kind = K_SEND | (g << 8);
    po.a = a;
  } else {
    stop_application(M, a, now);
  }
  return po;
}
__device__ __forceinline__ void appobj_start(const P2PDev &M, Emit &E, uint32_t a) {  // Application::DoStart
  uint32_t f = M.app_flags[a];
  if (f & 1u) return;
  M.app_flags[a] = f | 1u;
  E.child(M.app_start[a], E.ctx, K_APP_START, a, Pkt{0, 0, 0, 0});
  if (M.app_stop[a] != 0) E.child(M.app_stop[a], E.ctx, K_APP_STOP, a, Pkt{0, 0, 0, 0});
}

// Addressing of a packet descriptor: the node it is addressed to and that node's route-table slot.
// An echo reply (NSGPU_PKT_REPLY) travels back to its client's node; an ICMP error (NSGPU_PKT_ICMP) to the
// offending datagram's sender (icmpv4-l4-protocol.cc:131-160: SendMessage (p, header.GetSource (), ...)).
__device__ __forceinline__ uint32_t pkt_dst_node(const P2PDev &M, const Pkt &p) {
  if (p.app & NSGPU_PKT_ICMP) {
    const uint32_t fa = p.app & NSGPU_PKT_APP;
    return (p.app & NSGPU_PKT_ICMP_OF_REPLY) ? M.app_dst_node[fa] : M.app_node[fa];
  }
  if (p.app & NSGPU_PKT_REPLY) return M.app_node[p.app & ~NSGPU_PKT_REPLY];
  return M.app_dst_node[p.app];
}
__device__ __forceinline__ uint32_t pkt_dst_slot(const P2PDev &M, const Pkt &p) {
  if (p.app & NSGPU_PKT_ICMP) {
    const uint32_t fa = p.app & NSGPU_PKT_APP;
    return (p.app & NSGPU_PKT_ICMP_OF_REPLY) ? M.app_dst_slot[fa] : M.app_src_slot[fa];
  }
  if (p.app & NSGPU_PKT_REPLY) return M.app_src_slot[p.app & ~NSGPU_PKT_REPLY];
  return M.app_dst_slot[p.app];
}
// The ICMP error about datagram p (its IPv4 header as the error embeds it): Icmpv4TimeExceeded /
// Icmpv4DestinationUnreachable + the 4-byte Icmpv4Header over the offending header and 8 payload bytes:
// a 56-byte IPv4 packet with the default TTL 64 (icmpv4.cc:306-309,407-410; Ipv4L3Protocol::Send).
__device__ __forceinline__ Pkt icmp_error(const Pkt &p, bool unreach) {
  const uint32_t of = (p.app & NSGPU_PKT_REPLY) ? NSGPU_PKT_ICMP_OF_REPLY : 0u;
  return Pkt{NSGPU_PKT_ICMP | (unreach ? NSGPU_PKT_ICMP_UNREACH : 0u) | of | (p.app & NSGPU_PKT_APP),
             (p.ipid & 0xffffu) << 16, 56u, 64u | ((p.ttl & 0xffu) << 8) | (p.size << 16)};
}

// Ipv4 route lookup: the static next-hop device of node n towards route-table slot `slot`.
__device__ __forceinline__ uint32_t route_at(const P2PDev &M, uint32_t n, uint32_t slot) {
  if (slot == 0xffffffffu) return 0xffffffffu;
  if (M.route) return M.route[(uint64_t)n * M.n_dst + slot];
  // compressed: binary search of the node's exceptions (a dumbbell router holds one per leaf); a node
  // with an exception for every slot has them at their slot's position (ascending, distinct)
  const uint64_t e1 = M.route_exc_off[n + 1];
  uint64_t lo = M.route_exc_off[n], hi = e1;
  if (hi - lo == M.n_dst) return M.route_exc_dev[lo + slot];
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (M.route_exc_slot[mid] < slot) lo = mid + 1;
    else hi = mid;
  }
  return (lo < e1 && M.route_exc_slot[lo] == slot) ? M.route_exc_dev[lo] : M.route_def[n];
}
// ... towards the packet's destination.
__device__ __forceinline__ uint32_t route_of(const P2PDev &M, uint32_t n, const Pkt &p) {
  return route_at(M, n, pkt_dst_slot(M, p));
}

// Icmpv4L4Protocol::SendMessage (icmpv4-l4-protocol.cc:85-129): RouteOutput towards the error's
// destination, then Ipv4L3Protocol::Send from node n (its m_identification++); no route: dropped.
__device__ __forceinline__ Act icmp_act(const P2PDev &M, uint32_t n, Pkt e, HStat &hs) {
  const uint32_t out = route_of(M, n, e);
  if (out == 0xffffffffu) {
    hs.no_route++;
    return Act{ACT_NONE, 0, Pkt{0, 0, 0, 0}};
  }
  e.ipid |= M.node_ipid[n]++ & 0xffffu;
  hs.icmp++;
  return Act{ACT_SEND, out, e};
}

// One event: the kind-specific first phase (node part: node and application state, its own children),
// then the device step, then a trailing child.  The node part never reads device queue / tx state and
// the device step never reads node state, so a hub node's events can run them in two passes.
struct NodeOut {
  Act act;
  Post post;
  bool cancelled;
  uint32_t xdrop;  // forwarding device + 1 of a TTL-expired datagram whose time-exceeded error is act:
                   // its Drop record follows the device step (0: none)
};
// A Receive's addressing (pkt_dst_node, pkt_dst_slot), loaded ahead of the event by its caller.
struct DstHint {
  bool valid;
  uint32_t node, slot;
};
// rx_atomic: the device's rx counter is added with an atomic (hub blocks: other lanes add to it too;
// holders: a no-return atomic, so the event does not wait for the counter's line).
__device__ __forceinline__ NodeOut node_part(const P2PDev &M, Emit &E, uint32_t kind_word, uint32_t a,
                                             const Pkt &pkt, int32_t sink, HStat &hs, bool rx_atomic = false,
                                             DstHint hint = DstHint{false, 0, 0}) {
  const uint32_t kind = kind_word & 0xffu;
  const uint32_t gen = kind_word >> 8;
  Act act{ACT_NONE, 0, Pkt{0, 0, 0, 0}};
  Post post{false, 0, 0, 0};
  bool cancelled = false;
  uint32_t xdrop = 0;
  if (kind == K_RECEIVE) {  // PointToPointNetDevice::Receive -> Ipv4L3Protocol::Receive (ipv4-l3-protocol.cc:434-537)
    if (rx_atomic) atomicAdd(&M.dev[a].c.rx_packets, 1u);
    else M.dev[a].c.rx_packets++;
    Pkt p = pkt;
    p.size -= 2;                             // ProcessHeader strips the PppHeader
    trace_call(M, E, NSGPU_TR_RX, a, p);     // m_macRxTrace
    trace_call(M, E, NSGPU_TR_IP_RX, a, p);  // Ipv4L3Protocol::Receive: m_rxTrace (:455)
    // the receiving node: the context ScheduleWithContext gave the Receive (point-to-point-channel.cc:100)
    const uint32_t n = E.ctx < M.n_nodes ? E.ctx : M.dev_node[a];
    const bool reply = (p.app & NSGPU_PKT_REPLY) != 0;
    const uint32_t fa = p.app & ~NSGPU_PKT_REPLY;
    if ((hint.valid ? hint.node : pkt_dst_node(M, p)) == n) {
      // LocalDeliver -> UdpL4Protocol::Receive (udp-l4-protocol.cc:312-407): the bound endpoint is the
      // client's own socket for an echo reply, else the node's PacketSink / UdpEchoServer.  An ICMP error
      // ends in Icmpv4L4Protocol::Receive -> UdpL4Protocol::ReceiveIcmp (no event, no counter).
      const int32_t k = reply ? (int32_t)fa : sink;
      if (p.app & NSGPU_PKT_ICMP) {
      } else if (k < 0 || !(M.app_flags[k] & 2u)) {  // no bound endpoint: RX_ENDPOINT_UNREACH
        hs.unreach++;
        if (M.icmp) act = icmp_act(M, n, icmp_error(p, true), hs);  // SendDestUnreachPort (ip, copy)
      } else {
        // Ipv4EndPoint::ForwardUp: ScheduleNow (&Ipv4EndPoint::DoForwardUp) (ipv4-end-point.cc:112-120);
        // run inline for a PacketSink, queued for the echo applications (their HandleRead schedules)
        const bool q = reply || M.app_kind[k] == NSGPU_APP_ECHO_SERVER;
        E.child(0, E.ctx, q ? K_FWD_UP_Q : K_FWD_UP, (uint32_t)k, p);
      }
    } else {
      const uint32_t out = hint.valid ? route_at(M, n, hint.slot) : route_of(M, n, p);
      if (out == 0xffffffffu) {
        hs.no_route++;
        trace_ip_drop(M, E, a, p);  // DROP_NO_ROUTE
      } else {
        p.ttl -= 1;  // IpForward (:815-841)
        if ((p.ttl & 0xffu) == 0) {
          hs.ttl_drops++;  // (no ICMP about an ICMP message)
          if (M.icmp && !(p.app & NSGPU_PKT_ICMP)) act = icmp_act(M, n, icmp_error(p, false), hs);
          if (act.op == ACT_SEND) {
            xdrop = out + 1;
          } else {
            p.ttl += 1;
            trace_ip_drop(M, E, out, p);  // DROP_TTL_EXPIRED (:835: on the forwarding route's interface)
          }
        } else {
          act = Act{ACT_SEND, out, p};
        }
      }
    }
  } else if (kind == K_TX_COMPLETE) {
    act = Act{ACT_KICK, a, Pkt{0, 0, 0, 0}};
  } else if (kind == K_SEND) {  // OnOffApplication::SendPacket (onoff-application.cc:254-270)
    const uint32_t f = M.app_flags[a];
    if (!((f & 4u) && M.app_send_gen[a] == gen)) {
      cancelled = true;
    } else if (M.app_kind[a] == NSGPU_APP_ECHO_CLIENT) {  // UdpEchoClient::Send (udp-echo-client.cc)
      M.app_flags[a] = f & ~4u;
      const uint32_t sz = M.app_pkt_size[a];
      Pkt p{a, 0, sz + 8 + 20, M.app_ttl[a]};
      M.appc[a].tx_packets++;
      M.appc[a].tx_bytes += sz;
      const uint32_t an = M.app_node[a];
      const uint32_t out = route_of(M, an, p);  // m_socket->Send (p)
      if (out == 0xffffffffu) {
        hs.no_route++;
      } else {
        p.ipid = M.node_ipid[an]++;
        act = Act{ACT_SEND, out, p};
      }
      const uint32_t sent = ++M.app_tot[a];  // ++m_sent
      if (sent < M.app_count[a]) {           // ScheduleTransmit (m_interval)
        const uint32_t g = (M.app_send_gen[a] + 1) & 0xffffffu;
        M.app_send_gen[a] = g;
        M.app_flags[a] |= 4u;
        post = Post{true, M.app_interval[a], K_SEND | (g << 8), a};
      }
    } else {
      M.app_flags[a] = f & ~4u;
      const uint32_t sz = M.app_pkt_size[a];
      Pkt p{a, 0, sz + 8 + 20, M.app_ttl[a]};
      M.appc[a].tx_packets++;
      M.appc[a].tx_bytes += sz;
      const uint32_t an = M.app_node[a];
      const uint32_t out = route_of(M, an, p);  // UdpSocketImpl::DoSendTo: RouteOutput
      if (out == 0xffffffffu) {
        hs.no_route++;
      } else {
        p.ipid = M.node_ipid[an]++;  // Ipv4L3Protocol::BuildHeader: SetIdentification (m_identification++)
        act = Act{ACT_SEND, out, p};
      }
      M.app_tot[a] += sz;
      M.app_last_start[a] = E.now;
      M.app_residual[a] = 0;
      post = schedule_next_tx(M, a, E.now);
    }
  } else {
    switch (kind) {
      case K_NODE_START:
        for (uint32_t i = M.node_app_off[a]; i < M.node_app_off[a + 1]; i++) appobj_start(M, E, M.node_app_list[i]);
        break;
      case K_APPOBJ_START:
        appobj_start(M, E, a);
        break;
      case K_APP_START:
        if (M.app_kind[a] == NSGPU_APP_SINK || M.app_kind[a] == NSGPU_APP_ECHO_SERVER) {  // Bind (port)
          M.app_flags[a] |= 2u;
        } else if (M.app_kind[a] == NSGPU_APP_ECHO_CLIENT) {
          // UdpEchoClient::StartApplication: Bind, Connect, SetRecvCallback, ScheduleTransmit (Seconds (0))
          const uint32_t g = (M.app_send_gen[a] + 1) & 0xffffffu;
          M.app_send_gen[a] = g;
          M.app_flags[a] |= 2u | 4u;
          E.child(0, E.ctx, K_SEND | (g << 8), a, Pkt{0, 0, 0, 0});
        } else {
          cancel_events(M, a, E.now);
          schedule_start_event(M, E, a);
        }
        break;
      case K_APP_STOP:
        stop_application(M, a, E.now);
        break;
      case K_START_SENDING: {  // onoff-application.cc:196-206
        const uint32_t f = M.app_flags[a];
        if (!((f & 8u) && M.app_ss_gen[a] == gen)) {
          cancelled = true;
          break;
        }
        M.app_flags[a] = f & ~8u;
        M.app_last_start[a] = E.now;
        post = schedule_next_tx(M, a, E.now);
        if (post.valid) E.child(post.delay, E.ctx, post.kind, post.a, Pkt{0, 0, 0, 0});
        post.valid = false;
        schedule_stop_event(M, E, a);
        break;
      }
      case K_STOP_SENDING: {  // onoff-application.cc:208-216
        const uint32_t f = M.app_flags[a];
        if (!((f & 8u) && M.app_ss_gen[a] == gen)) {
          cancelled = true;
          break;
        }
        M.app_flags[a] = f & ~8u;
        cancel_events(M, a, E.now);
        schedule_start_event(M, E, a);
        break;
      }
      case K_FWD_UP:  // DoForwardUp -> UdpSocketImpl::ForwardUp -> PacketSink::HandleRead (a = sink app)
      case K_FWD_UP_D:
        if (M.app_flags[a] & 2u) {
          M.appc[a].rx_packets++;
          M.appc[a].rx_bytes += pkt.size - 28;
        }
        break;
      case K_FWD_UP_Q:  // DoForwardUp -> UdpSocketImpl::ForwardUp -> UdpEcho{Server,Client}::HandleRead (a = endpoint app)
        if (M.app_flags[a] & 2u) {
          M.appc[a].rx_packets++;
          M.appc[a].rx_bytes += pkt.size - 28;
          if (M.app_kind[a] == NSGPU_APP_ECHO_SERVER) {  // socket->SendTo (packet, 0, from)
            Pkt r{pkt.app | NSGPU_PKT_REPLY, 0, pkt.size, M.app_ttl[a]};
            M.appc[a].tx_packets++;
            M.appc[a].tx_bytes += pkt.size - 28;
            const uint32_t an = M.app_node[a];
            const uint32_t out = route_of(M, an, r);
            if (out == 0xffffffffu) {
              hs.no_route++;
            } else {
              r.ipid = M.node_ipid[an]++;
              act = Act{ACT_SEND, out, r};
            }
          }
        }
        break;
      case K_STOP:
        hs.stop = true;
        break;
      default:  // K_DEV_START: no-op
        break;
    }
  }
  return NodeOut{act, post, cancelled, xdrop};
}
__device__ __forceinline__ bool run_event(const P2PDev &M, Emit &E, uint32_t kind_word, uint32_t a, const Pkt &pkt,
                                          int32_t sink, HStat &hs) {
  const NodeOut o = node_part(M, E, kind_word, a, pkt, sink, hs);
  device_act(M, E, o.act);
  if (o.xdrop) trace_te_drop(M, E, o.xdrop - 1, o.act.p);
  if (o.post.valid) E.child(o.post.delay, E.ctx, o.post.kind, o.post.a, Pkt{0, 0, 0, 0});
  return o.cancelled;
}

// Diagnostic build (-DNSGPU_PHASE_PROF, lib/libnsgpu_prof.so only): thread 0 of block 0 of each
// pipeline kernel accumulates s_memrealtime (100 MHz) deltas between phase marks into g_phase.
#ifdef NSGPU_PHASE_PROF
__device__ uint64_t g_phase[64];
#define PH_BEGIN() uint64_t ph_t_ = (threadIdx.x == 0 && blockIdx.x == 0) ? __builtin_amdgcn_s_memrealtime() : 0
#define PH_MARK(i)                                                                      \
  do {                                                                                  \
    if (threadIdx.x == 0 && blockIdx.x == 0) {                                          \
      const uint64_t t_ = __builtin_amdgcn_s_memrealtime();                             \
      atomicAdd((unsigned long long *)&g_phase[i], (unsigned long long)(t_ - ph_t_));   \
      ph_t_ = t_;                                                                       \
    }                                                                                   \
  } while (0)
// hub blocks (k2_handle): thread 0 of every hub block adds its phase times into g_phase[24..27], calls in [28]
#define HUB_T0() uint64_t hub_t_ = threadIdx.x == 0 ? __builtin_amdgcn_s_memrealtime() : 0
#define HUB_MARK(i)                                                                     \
  do {                                                                                  \
    if (threadIdx.x == 0) {                                                             \
      const uint64_t t_ = __builtin_amdgcn_s_memrealtime();                             \
      atomicAdd((unsigned long long *)&g_phase[i], (unsigned long long)(t_ - hub_t_));  \
      hub_t_ = t_;                                                                      \
    }                                                                                   \
  } while (0)
#else
#define PH_BEGIN() (void)0
#define PH_MARK(i) (void)0
#define HUB_T0() (void)0
#define HUB_MARK(i) (void)0
#endif
// Per-block start / end times (s_memrealtime) of the window kernels in one sampled window
// (diagnostic build only): g_blk[kernel][block] = {start, end}, window g_blk_win.
#ifdef NSGPU_PHASE_PROF
constexpr int BLK_MAX = 2048;
__device__ uint64_t g_blk[3][BLK_MAX][2];
__device__ uint64_t g_blk_win = 1000;
#define BLK_T0() uint64_t bt0_ = __builtin_amdgcn_s_memrealtime(), btm_ = bt0_
// per-block phase mark in the sampled window: g_phase[i] += time since the block's previous mark
#define BLK_MARK(i, win)                                                                         \
  do {                                                                                           \
    if (threadIdx.x == 0 && (win) == g_blk_win) {                                                \
      const uint64_t t_ = __builtin_amdgcn_s_memrealtime();                                      \
      atomicAdd((unsigned long long *)&g_phase[i], (unsigned long long)(t_ - btm_));             \
      atomicAdd((unsigned long long *)&g_phase[(i) + 1], 1ull);                                  \
      btm_ = t_;                                                                                 \
    }                                                                                            \
  } while (0)
// k_gtile's per-block stamps in the sampled window: g_gt[block] = {start, prologue done, first tile in LDS,
// first tile compared, end (after its atomics returned)}
constexpr int GT_BLK_MAX = 8192;
__device__ uint64_t g_gt[GT_BLK_MAX][8];
#define BLK_REC(k, win)                                                                          \
  do {                                                                                           \
    if (threadIdx.x == 0 && (win) == g_blk_win && blockIdx.x < (uint32_t)BLK_MAX) {              \
      g_blk[k][blockIdx.x][0] = bt0_;                                                            \
      g_blk[k][blockIdx.x][1] = __builtin_amdgcn_s_memrealtime();                                \
    }                                                                                            \
  } while (0)
#else
#define BLK_T0() (void)0
#define BLK_REC(k, win) (void)0
#define BLK_MARK(i, win) (void)0
#endif

// ================================ window pipeline ================================
// Window bound of a pending set's reduction: packed key bound, span, Stop key.
struct WinBound {
  uint64_t tmin, span, bound, stop_packed;
  uint64_t nbound;  // the narrow bound (span = the narrow lookahead's)
  uint64_t lim;     // local records: a TransmitComplete child with rel ts < lim runs in the window (0: none)
};
// wide: wide windows — the span is span_t clamped between the narrow bound (min over
// pending of ts + lookahead) and the wide one (ts + lookw, nsgpu_p2p_create); a same-node TransmitComplete
// before the window's end then runs inside it (local record).
__device__ __forceinline__ WinBound window_bound(const Red &R, bool wide = false, uint64_t span_t = 0) {
  WinBound b;
  b.tmin = R.tmin;
  uint64_t span = R.wend - b.tmin;
  if (span > 0xfffffffeull) span = 0xfffffffeull;
  const uint64_t nspan = span;
  if (wide && R.tmin != ~0ull && R.wendw != ~0ull && R.wendw > R.wend) {
    uint64_t wspan = R.wendw - b.tmin;
    if (wspan > 0xfffffffeull) wspan = 0xfffffffeull;
    span = span_t < wspan ? span_t : wspan;
    span = span > nspan ? span : nspan;
  }
  b.span = span;
  b.bound = (span << 32) | 0xffffffffull;
  b.nbound = (nspan << 32) | 0xffffffffull;
  // a local child at the window's end could tie with a cross-node child there: strictly before it
  b.lim = span > nspan ? span : 0;
  b.stop_packed = ~0ull;
  if (R.stopts != ~0ull && R.stopts - b.tmin <= span) {
    // Stop caps the window at its own key (it is dispatched; later events are not); a child at the Stop's
    // ts sorts after it (a larger uid)
    b.stop_packed = ((R.stopts - b.tmin) << 32) | R.stopuid;
    b.bound = b.stop_packed < b.bound ? b.stop_packed : b.bound;
    b.nbound = b.stop_packed < b.nbound ? b.stop_packed : b.nbound;
    b.lim = (R.stopts - b.tmin) < b.lim ? (R.stopts - b.tmin) : b.lim;
  }
  return b;
}
__device__ __forceinline__ void publish_bound(Ctl &C, const WinBound &b) {
  C.tmin = b.tmin;
  C.bound = b.bound;
  C.nbound = b.nbound;
  C.lim_rel = b.lim;
  // zero-delay leaf children (Ipv4EndPoint::DoForwardUp) run inside the window; when the window ends
  // at the Stop event, those at the Stop's ts sort after it and are never dispatched
  const bool has_stop = b.stop_packed != ~0ull && b.bound >= b.stop_packed;
  C.inline_lim = has_stop ? (b.stop_packed >> 32) : ~0ull;
}

// Reduces (tmn, wnd) over the workgroup and one lane folds them into R (atomicMin): one atomic
// pair per workgroup, not per wave (a word takes ~11 ns per atomic).  All threads must call it.
// WIDE: the wide bound (wndw) as well.
template <int NTH, bool WIDE = false>
__device__ __forceinline__ void publish_min(Red &R, uint64_t tmn, uint64_t wnd, uint64_t wndw = ~0ull) {
  tmn = wave_min64(tmn);
  wnd = wave_min64(wnd);
  if constexpr (WIDE) wndw = wave_min64(wndw);
  if constexpr (NTH > 64) {
    __shared__ uint64_t s0[NTH / 64], s1[NTH / 64], s2[NTH / 64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) {
      s0[wid] = tmn;
      s1[wid] = wnd;
      if constexpr (WIDE) s2[wid] = wndw;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    for (int w = 1; w < NTH / 64; w++) {
      tmn = s0[w] < tmn ? s0[w] : tmn;
      wnd = s1[w] < wnd ? s1[w] : wnd;
      if constexpr (WIDE) wndw = s2[w] < wndw ? s2[w] : wndw;
    }
  } else if ((threadIdx.x & 63) != 0) {
    return;
  }
  if (tmn != ~0ull) atomicMin((unsigned long long *)&R.tmin, (unsigned long long)tmn);
  if (wnd != ~0ull) atomicMin((unsigned long long *)&R.wend, (unsigned long long)wnd);
  if (WIDE && wndw != ~0ull) atomicMin((unsigned long long *)&R.wendw, (unsigned long long)wndw);
}

// A pending event in registers.
struct Ev {
  uint64_t ts;
  uint32_t uid, ctx, kind, a;
  Pkt p;
};

// ---- exchange records of a partitioned run (fixed sizes: they are captured into the window graph) ----
// X1: a rank's window summary, allgathered.  LbtsMessage's role (distributed-simulator-impl.h:36-84:
// rx/tx counts, smallest next time) is played by the pending-set reduction `red` and the counts.
struct X1Hdr {
  uint32_t W, tc, tinl, needc;  // window events, their children, their inline children; pool compaction wanted
  uint32_t L, pad1;           // wide windows: this rank's local records (X1Loc entries)
  uint64_t lastkey;           // largest window key
  Red red;                    // reduction of this rank's pending set after the window (next LBTS)
  uint64_t rkey, rrem, rhead; // sorted run: this rank's fitting key for the next chunk (~0: the rest fits), entries
                              // left, the first one's key (~0: none)
  uint64_t pad2[4];
};
static_assert(sizeof(X1Hdr) == 128, "X1 records: the loopback transport copies 16-byte words");
struct X1Ent {  // one window event: key and child counts (children | inline children << 16)
  uint64_t key;
  uint32_t cnt, pad;
};
// Wide windows: one rank's local records (same-node TransmitCompletes run inside the window), compacted by
// k2_handle.  Their order words (lkw) decide every pair from different gen-0 ancestors exactly once the chain
// depth is at most 2 (the partitioned wide span is kept below 3 tx_min, nsgpu_p2p_create_dist), except a
// depth-2 word's clamped ancestor uid: `anc` holds it whole.  Records of one ancestor are on one rank, where
// their exact chains are (lkey[rec]).
struct X1Loc {
  uint64_t w1, w2;     // lkw: (rel ts, local, parent rel ts), (ancestor uid, child index / ...)
  uint32_t cnt, rec;   // children | inline children << 16; the record on its rank
  uint32_t anc, par;   // the gen-0 ancestor's uid; the parent's accumulator row | child index << 24 (k_dfin2)
};
static_assert(sizeof(X1Loc) == 32, "X1Loc");
constexpr int XLCAP = 4096;  // local records of one rank's window (LMAX)
constexpr int NACC = WCAP + XLCAP;  // k_gtile's accumulator rows: gen-0 slots, then local records (compact order)
// One record of a rank's window in that rank's dispatch order (k_gsort), as another rank's k_gsearch compares its
// own records with it: the order key (rel ts, gen-0 before local, then a gen-0 record's uid / a local record's
// order words and ancestor uid: records of different ranks never tie on it) and the exclusive prefixes of its
// rank's children / inline children before it.  Entry n (n = the rank's records) is a sentinel with the totals.
struct SEnt {
  uint64_t k0;  // rel ts << 32 | (gen-0: uid; local: the low word of its first order word)
  uint64_t b;   // local: its second order word (gen-0: 0)
  uint32_t c, L;  // local: the gen-0 ancestor's uid, 1 (gen-0: 0, 0)
  uint32_t cp, ip;
};
static_assert(sizeof(SEnt) == 32, "SEnt");
// X1 (all-gathered): the header and the sorted records; the rank's own lists stay in x1_own.
constexpr size_t X1B = sizeof(X1Hdr) + sizeof(SEnt) * (NACC + 1);
constexpr size_t X1OWN = sizeof(X1Ent) * WCAP + sizeof(X1Loc) * XLCAP;
static_assert(X1B % 16 == 0, "k_copies moves 16-byte words");
// X2: remote events for one peer (children whose node another rank owns), all-to-all; the record is
// the pending event itself, uid included (mpi-interface.cc:414-506 sends {rx ns, node, dev, packet}).
struct X2Hdr {
  uint32_t n, pad[3];
};
// X2 records per peer: a device starts at most one transmission per narrow window (its TransmitComplete is a
// child, and children sort after the window) — three per wide one (its local TransmitCompletes start the next
// ones: chain depth <= 2) — and Receive is the only child scheduled on another node, so rank p sends rank q at
// most that many records per window per device of p whose peer q owns (nsgpu_p2p_create_dist sizes X2 to the
// largest such cut, rounded up to 16; at most CAPX_MAX).
constexpr int CAPX_MAX = 1024;
constexpr size_t X0B = 16;  // X0: one rank's largest fitting window bound (+ pad)
constexpr int MAXR = 64;    // ranks
static_assert(MAXR <= 64 && HB == 64, "per-rank summaries are read one lane per rank in one-wave blocks");
static_assert((uint64_t)MAXR * NACC <= (1u << 21), "k_gtile's packed rank fields");
__device__ __forceinline__ X1Hdr *x1hdr(uint8_t *b, uint32_t q) { return (X1Hdr *)(b + (size_t)q * X1B); }
__device__ __forceinline__ SEnt *x1srt(uint8_t *b, uint32_t q) { return (SEnt *)(b + (size_t)q * X1B + sizeof(X1Hdr)); }
__device__ __forceinline__ X1Ent *x1ent(const P2PDev &M) { return (X1Ent *)M.x1_own; }
__device__ __forceinline__ X1Loc *x1loc(const P2PDev &M) { return (X1Loc *)(M.x1_own + sizeof(X1Ent) * WCAP); }
__device__ __forceinline__ X2Hdr *x2hdr(const P2PDev &M, uint8_t *b, uint32_t q) {
  return (X2Hdr *)(b + (size_t)q * M.x2b);
}
__device__ __forceinline__ Ev *x2rec(const P2PDev &M, uint8_t *b, uint32_t q) {
  return (Ev *)(b + (size_t)q * M.x2b + sizeof(X2Hdr));
}

constexpr int PFC = 4;  // children per slot k2_pa loads ahead


// Rank tile t: rows [ti * HB * RTR, +HB * RTR) of the window (RTR keys per thread) against the RJ keys
// of column tile tj: each row's count of smaller keys is added to its rank (keys are distinct: uids).
// Wide rows: each column tile's keys are loaded by NRT blocks, not WCAP / HB.
// (wr: the rank accumulators of the window's parity, wrank_of)
__device__ __forceinline__ void rank_tile(const P2PDev &M, const Ctl &C, uint32_t t, uint32_t *wr) {
  const uint32_t ti = t / NJT, tj = t % NJT;
  __shared__ uint64_t tk[RJ];
  // the window size first: a config-4 window fills ~1/4 of the WCAP x WCAP tiles, and the tiles past
  // it load nothing (these blocks are off the launch's critical path, the holders are on it)
  const uint32_t W = C.W;
  const uint32_t r0 = ti * HB * RTR;
  if (r0 >= W || tj * RJ >= W) return;  // uniform over the block
#pragma unroll
  for (int q = 0; q < RJ / HB; q++) {  // (slots past W hold stale keys: padded with a key after every row's)
    const uint32_t j = tj * RJ + q * HB + threadIdx.x;
    tk[q * HB + threadIdx.x] = j < W ? M.wkey[j] : ~0ull;
  }
  uint64_t x[RTR];
#pragma unroll
  for (int r = 0; r < RTR; r++) {
    const uint32_t i = r0 + r * HB + threadIdx.x;
    x[r] = i < W ? M.wkey[i] : 0;
  }
  __syncthreads();
  uint32_t c[RTR] = {};
#pragma unroll 16
  for (int y = 0; y < RJ; y++) {
    const uint64_t k = tk[y];
#pragma unroll
    for (int r = 0; r < RTR; r++) c[r] += k < x[r];
  }
#pragma unroll
  for (int r = 0; r < RTR; r++) {
    const uint32_t i = r0 + r * HB + threadIdx.x;
    if (i < W && c[r]) atomicAdd(&wr[i], c[r]);
  }
}

#include "nsgpu_p2p_win.h"

// ================================ partitioned run (multi-GPU) ================================
// DistributedSimulatorImpl (src/mpi/model/distributed-simulator-impl.cc:146-326) gives every rank
// the nodes of its system id and grants it min over ranks of (next ts) + lookahead after an
// MPI_Allgather of LbtsMessage (:276-313); remote packets travel as {rx ns, node, dev, serialized
// packet} (mpi-interface.cc:414-506).  Here every rank runs the single-GPU engine's window kernels
// over its own nodes, and three fixed-size collectives per window (RCCL, captured into the window
// graph with the kernels) make the partitioned run reproduce the SEQUENTIAL pop order — uids
// included, which DistributedSimulatorImpl itself does not (its uids are per rank):
//   k2_pa<true>  as single-GPU (in-place pool), plus the remote events of the last X2;
//   X0           allgather of every rank's window size and hub flag (16 B, straight from Ctl);
//   k2_handle    holders and hub blocks (no rank tiles), writing this rank's X1 summary and entries —
//                unless some rank's window does not fit: then nothing runs and the window becomes a
//                partitioned sorted run (every rank sorts its candidates once; chunks cut at the smallest
//                of the ranks' fitting keys, nsgpu_p2p_win.h);
//   X1           allgather of the summaries;
//   k_gtile      per own event, over the merged windows: # smaller keys (global dispatch rank) and the
//                child / inline-child sums below it and below its same-ts group (uid prefixes);
//   k_dfin2      own events' dispatch info, remote children -> X2 with their final uids, the pool
//                bookkeeping, and the run bookkeeping from the merged summaries: the LBTS (the next
//                window's bound), `done`, a compaction every rank makes;
//   X2           all-to-all of remote events.

// ---- partitioned sorted runs: the host step that starts one (nsgpu_p2p_win.h, "partitioned sorted runs") ----
// The window that did not fit (C.W candidates in the window records, relative to its tmin) is sorted by key into
// rn_* (k_rs_*), after its node-table entries are cleared (k_drun_clear: the chunks claim them again); k_drun_start
// keeps the window's bound and sends this rank's fitting key (its WCAP-th entry's key; ~0 when all fit) and size,
// and after their all-gather k_drun_first moves the first chunk in.  The candidates that came from the pool stay
// there until their chunk runs (its maintenance tombstones them); the others live in the run only.
__global__ __launch_bounds__(256) void k_drun_clear(const P2PDev M) {
  const Ctl &C = *M.C;
  const uint64_t W = C.W;
  const uint64_t nt = W < (uint64_t)WCAP ? W : (uint64_t)WCAP;  // (k2_write claims slots below WCAP only)
  for (uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x; s < nt; s += (uint64_t)gridDim.x * 256) {
    const uint32_t c = lp_of(M, M.wctx[s], M.wkind[s], M.wa[s]);
    if (c < M.n_nodes) M.node_tab[(uint64_t)c * NTAB] = 0;
  }
}
__global__ void k_drun_start(const P2PDev M, uint64_t n) {
  Ctl &C = *M.C;
  if (M.wide) n = C.drcut < n ? C.drcut : n;  // (k_drun_trim: the run is the window's narrow part)
  const WinBound b = window_bound(C.rt ? C.red[0] : C.red[1]);  // (the bound k2_pa formed the window with)
  C.drb_tmin = b.tmin;
  C.drb_span = b.span;
  C.drb_bound = b.bound;
  C.drb_stop = b.stop_packed;
  C.drb_nbound = b.nbound;
  C.drb_lim = b.lim;
  C.dr0 = C.dr1 = 0;
  C.drW = n;
  C.W = 0;
  C.nhub = 0;
  C.overflow = 0;
  C.drlo = ~0ull;
  C.drtrim = 0;
  C.dtrim = 0;
  {  // the pending set outside the run, as the overflowing window's k2_pa reduced it (the run's entries: k_drun_red)
    const Red r = x1hdr(M.x1_send, 0)->red;
    C.drn_tmin = r.tmin;
    C.drn_wend = r.wend;
    C.drn_stopts = r.stopts;
    C.drn_stopuid = r.stopuid;
    C.drn_wendw = r.wendw;
  }
  M.xk_send[0] = n > (uint64_t)WCAP ? M.rn_key[WCAP - 1] : ~0ull;  // (this rank's fitting key)
  M.xk_send[1] = n ? M.rn_key[0] : ~0ull;                           // (its head key)
}
// During the run the pool is not swept: the pending set's reduction at its start (k_drun_start) and the run's
// entries' (all of them: conservative, some are dispatched before the run ends) are folded into every chunk's; the
// chunks' children fold in as they are parked.  So the first window after the run is bounded safely.
__global__ __launch_bounds__(256) void k_drun_red(const P2PDev M, uint64_t n) {
  Ctl &C = *M.C;
  const uint64_t tmin = C.drb_tmin;
  uint64_t tmn = ~0ull, wnd = ~0ull, wndw = ~0ull;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    const uint64_t ts = tmin + (M.rn_key[i] >> 32);
    const uint32_t kd = (M.rn_kind[i] & 0xffu) % K_NKINDS;
    const uint64_t x = ts + (uint64_t)M.lookahead[kd], xw = ts + (uint64_t)M.lookw[kd];
    tmn = ts < tmn ? ts : tmn;
    wnd = x < wnd ? x : wnd;
    wndw = xw < wndw ? xw : wndw;
  }
  tmn = wave_min64(tmn);
  wnd = wave_min64(wnd);
  wndw = wave_min64(wndw);
  if ((threadIdx.x & 63) == 0) {
    if (tmn != ~0ull) atomicMin((unsigned long long *)&C.drn_tmin, (unsigned long long)tmn);
    if (wnd != ~0ull) atomicMin((unsigned long long *)&C.drn_wend, (unsigned long long)wnd);
    if (M.wide && wndw != ~0ull) atomicMin((unsigned long long *)&C.drn_wendw, (unsigned long long)wndw);
  }
}
// A widened window some rank cannot hold (wide partitioned engines): the run must be a narrow window (every child
// of a run event sorts after every run event), so the sorted candidates past the window's narrow bound leave it —
// those from the pool stay there, the others (children, remote events) are parked in the fresh buffer, which the
// next handled window's maintenance moves into the pool; k_drun_red folds every candidate into the reduction.
__global__ __launch_bounds__(1024) void k_drun_trim(const P2PDev M, uint64_t n) {
  Ctl &C = *M.C;
  const uint64_t nb = C.nbound, tmin = C.tmin;
  __shared__ uint64_t s_cut;
  if (threadIdx.x == 0) {  // the first candidate past the narrow bound (rn_key is sorted)
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
      const uint64_t mid = (lo + hi) >> 1;
      if (M.rn_key[mid] <= nb) lo = mid + 1;
      else hi = mid;
    }
    s_cut = lo;
  }
  __syncthreads();
  const uint64_t cut = s_cut;
  for (uint64_t i = cut + threadIdx.x; i < n; i += 1024) {
    if (M.rn_src[i] != NOSRC) continue;  // (still in the pool)
    const uint64_t fi = atomicAdd((unsigned long long *)&C.nF, 1ull);
    if (fi >= M.fcap) {
      atomicOr(M.error, 1u);
      continue;
    }
    const uint64_t k = M.rn_key[i];
    M.f_ts[fi] = tmin + (k >> 32);
    M.f_uid[fi] = (uint32_t)k;
    M.f_ctx[fi] = M.rn_ctx[i];
    M.f_kind[fi] = M.rn_kind[i];
    M.f_a[fi] = M.rn_a[i];
    M.f_pkt[fi] = M.rn_pkt[i];
  }
  if (threadIdx.x == 0) C.drcut = cut;
}
// The next chunk's cut key from the ranks' smallest fitting key fk and smallest head key hk (every rank computes
// the same): a chunk that continues the same-ts group the last one cut (gp: the last chunk's key) takes more of
// that group, and when the rest of the group fits, exactly the rest — and the run ends after it (its queued
// DoForwardUp leaves at that ts are pending: they sort before every later run entry); otherwise the chunk backs
// off to the start of the group its fitting key would cut, unless that group alone fills it.
struct DrunCut {
  uint64_t g, lo;
  uint32_t trim;
};
__device__ __forceinline__ DrunCut drun_cut(uint64_t fk, uint64_t hk, uint64_t gp) {
  const uint64_t T0 = hk >> 32, gend = (T0 << 32) | 0xffffffffull;
  if (gp != ~0ull && (uint32_t)gp != 0xffffffffu && (gp >> 32) == T0)  // (a real key's uid is below 0xffffffff)
    return fk >= gend ? DrunCut{gend, T0, 1u} : DrunCut{fk, T0, 0u};
  if (fk != ~0ull && (fk >> 32) > T0) return DrunCut{((fk >> 32) << 32) - 1, ~0ull, 0u};
  return DrunCut{fk, ~0ull, 0u};
}
__global__ __launch_bounds__(TB) void k_drun_first(const P2PDev M) {
  Ctl &C = *M.C;
  uint64_t fk = ~0ull, hk = ~0ull;
  for (uint32_t q = 0; q < M.nranks; q++) {
    fk = M.xk_recv[2 * q] < fk ? M.xk_recv[2 * q] : fk;
    hk = M.xk_recv[2 * q + 1] < hk ? M.xk_recv[2 * q + 1] : hk;
  }
  const uint64_t g = drun_cut(fk, hk, ~0ull).g;
  drun_chunk<TB>(M, C, (uint64_t)blockIdx.x * TB + threadIdx.x, 0, C.drW, g);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const WinBound b = drun_bound(C, g);
    publish_bound(C, b);
    C.split_lo = ~0ull;  // (leaves at a cut group's ts are queued: pending events of that ts sort before them)
    C.split_hi = drun_cuts_group(g, C.drb_bound) ? (g >> 32) : b.span;
    C.hrel = C.split_hi;
    C.hcap = 0;
    C.drun = 1;
    C.drg = g;
    C.prep = 1;  // (the next k2_pa finds the window formed: it appended the last window already)
    C.mode = MODE_NORMAL;
  }
}

#ifndef GT_CT
#define GT_CT 1  // column tiles of one k_gtile work item (more: fewer atomics, but the compares bound it)
#endif
#ifndef GT_GJ
#define GT_GJ 64  // columns of one k_gtile tile (smaller tiles, more waves a SIMD to interleave: 256 -> 64 columns
                   // took a wide window's k_gtile from 25 to 17 us)
#endif
constexpr int GJ = GT_GJ;
static_assert(GJ <= 64, "k_gtile's packed column counts (7-bit count field)");
#ifndef GT_GTB
#define GT_GTB 8192
#endif
constexpr int GTB = GT_GTB;  // blocks of k_gtile (grid-stride over tiles: a wide window's ~5,600 tiles in one round)
// The partitioned window's dispatch order, in three steps (r06; before, k_gtile compared every row with every
// rank's records, so its work grew with the ranks: 12.6 / 19.6 / 40.6 / 52.8 us a window at 1 / 2 / 4 / 8
// loopback partitions, profiles/r06/gtile_scale/):
//   k_gtile (before the X1 exchange): this rank's records among themselves, all pairs in tiles;
//   k_gsort (more than one rank): each record into the rank's X1 at its rank there (SEnt: its order key and the
//     exclusive prefixes of the children / inline children before it, a sentinel with the totals after them);
//   k_gsearch (after the exchange): a record's place among another rank's records is a binary search of that
//     rank's sorted list (records of different ranks never tie), its counts and prefixes read at that place.
// Rows: this rank's window records — its W gen-0 slots, then (WIDE) its L local records in X1Loc order; columns:
// this rank's, in column tiles of GJ (its gen-0 tiles, then its local tiles).  Per row, over the rank's window: the
// records before it (its rank), those of a smaller ts, those of ts <= its own (its same-ts group's end), and the
// children / inline children of the records before it and before its group (uid and dispatch prefixes).  A gen-0
// record precedes a local one of equal ts; two local records compare by their order words, a tie by the ancestor
// uid, then (same ancestor: same node, this rank) by their exact chains.
template <bool WIDE>
__global__ __launch_bounds__(HB, 6) void k_gtile(const P2PDev M) {  // (6 waves a SIMD: 73 VGPRs; 8 spilled)
  Ctl &C = *M.C;
  // the run control and every rank's window size in one trip (the sizes loaded before the test: a load after a
  // branch on C.hdl waited for it)
  const uint32_t hdl = C.hdl, W = C.pW;
  const X1Hdr *hs = x1hdr(M.x1_send, 0);  // (this rank's summary: the tiles rank its records among themselves)
  const uint32_t L0 = WIDE ? hs->L : 0u, tq0 = hs->tinl;
#ifdef NSGPU_PHASE_PROF
  const uint64_t gt_t0 = __builtin_amdgcn_s_memrealtime();
  const bool gt_rec = C.windows == g_blk_win && blockIdx.x < (uint32_t)GT_BLK_MAX;
  uint64_t gt_t[4] = {0, 0, 0, 0}, gt_kind = 0;
#define GT_MARK(k)                                                       \
  do {                                                                   \
    if (gt_rec && !gt_t[k]) gt_t[k] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define GT_MARK(k) (void)0
#endif
  if (!hdl) return;  // (k2_handle ran nothing: a cut, a pause, the end)
  // a column tile in LDS: its rel ts (the common test), child counts, and the fine key an equal ts needs — a
  // gen-0 record's uid; a local record's order words' low part and second word (ties: ancestor uid, record)
  // a column's child counts packed for the row's before-sum (tpb: 1 | children << 7 | inline children << 29 — over
  // one tile of GJ <= 64 columns the three fields stay within 7, 22 and 22 bits) and its inline children alone
  // (read four columns at a time as 16-B vectors)
  __shared__ __align__(16) uint32_t tts[GJ], tni[GJ], tfa[GJ];
  __shared__ __align__(16) uint64_t tpb[GJ], tfb[GJ];  // (tfb: a gen-0 column's whole key, a local one's w2)
  __shared__ uint32_t tu[WIDE ? GJ : 1], tr[WIDE ? GJ : 1];
  const uint32_t L = L0;
  const uint32_t ng = (W + GJ - 1) / GJ;  // (column tiles: the gen-0 records', then the local records')
  if (blockIdx.x == 0 && threadIdx.x == 0) {  // (for k_dfin2: its record blocks then read no X1 header, and its
    C.gt_tinl = tq0;                          //  block 0, the only reader left, resets this rank's header; more
    C.gt_lown = L;                            //  ranks: k_gsearch sums every rank's inline children)
  }
  GT_MARK(0);
  const uint32_t njt = ng + (L + GJ - 1) / GJ, NR = W + L;
  // a work item: one row tile against GT_CT consecutive column tiles, summed in registers (one pair of atomics per
  // row and item: the accumulators' atomics, not the compares, bound the kernel)
  const uint32_t nseg = (njt + GT_CT - 1) / GT_CT;
  const uint32_t nrt = (NR + HB - 1) / HB;
  const uint64_t T = (uint64_t)nrt * nseg;
  for (uint64_t t = blockIdx.x; t < T; t += gridDim.x) {  // (uniform over the block)
   // the local rows' tiles first (the last row tiles): their loads and compares take about twice a gen-0
   // tile's, and the blocks dispatched first start first
   const uint32_t ti = nrt - 1u - (uint32_t)(t / nseg), sg = (uint32_t)(t % nseg);
   const uint32_t i = ti * HB + threadIdx.x;
   const bool lrow = WIDE && i >= W;
   uint32_t tx = 0, fax = 0, xu = 0, xrec = 0;
   uint64_t fbx = 0;
   if (i < NR) {
     if (lrow) {
       const X1Loc e = x1loc(M)[i - W];
       tx = (uint32_t)(e.w1 >> 32), fax = (uint32_t)e.w1, fbx = e.w2, xu = e.anc, xrec = e.rec;
     } else {
       const uint64_t key = M.wkey[i];
       tx = (uint32_t)(key >> 32), fax = (uint32_t)key;
     }
   }
   uint32_t gr = 0, cp = 0, ip = 0, ipf = 0, lp = 0;
   const uint32_t tj1 = (sg + 1) * GT_CT < njt ? (sg + 1) * GT_CT : njt;
   for (uint32_t tj = sg * GT_CT; tj < tj1; tj++) {
    const bool ltile = WIDE && tj >= ng;  // a tile of the local records
    const uint32_t j0 = (ltile ? tj - ng : tj) * GJ, nq = ltile ? L : W;
    const uint32_t n = nq - j0 < (uint32_t)GJ ? nq - j0 : (uint32_t)GJ;
    if (ltile) {
      const X1Loc *E = x1loc(M) + j0;
      for (uint32_t k = threadIdx.x; k < (uint32_t)GJ; k += HB) {  // (padding: a ts after every row's)
        const bool in = k < n;
        const uint64_t w1 = in ? E[k].w1 : ~0ull;
        tts[k] = (uint32_t)(w1 >> 32);
        tfa[k] = (uint32_t)w1;
        tfb[k] = in ? E[k].w2 : ~0ull;
        const uint32_t c = in ? E[k].cnt : 0u;
        tpb[k] = 1ull | (uint64_t)(c & 0xffffu) << 7 | (uint64_t)(c >> 16) << 29;
        tni[k] = c >> 16;
        tu[k] = in ? E[k].anc : 0u;
        tr[k] = in ? E[k].rec : 0u;
      }
    } else {
      const X1Ent *E = x1ent(M) + j0;
      for (uint32_t k = threadIdx.x; k < (uint32_t)GJ; k += HB) {
        const uint64_t key = k < n ? E[k].key : ~0ull;
        tts[k] = (uint32_t)(key >> 32);
        tfa[k] = (uint32_t)key;
        tfb[k] = key;
        const uint32_t c = k < n ? E[k].cnt : 0u;
        tpb[k] = 1ull | (uint64_t)(c & 0xffffu) << 7 | (uint64_t)(c >> 16) << 29;
        tni[k] = c >> 16;
      }
    }
    __syncthreads();
    GT_MARK(1);
#ifdef NSGPU_PHASE_PROF
    gt_kind |= (ltile ? 1u : 0u) | (__any(lrow) ? 2u : 0u) | (__any(i < NR) ? 8u : 0u);
#endif
    if (i < NR) {
      // per column: earlier ts -> before (and in ipf); equal ts -> the fine key: gen-0 x gen-0 by uid, a gen-0
      // record before a local one, local x local by the order words (their ties after the loop)
      // (the compares bound the kernel: one 64-bit add of the packed counts a column instead of three selects)
      uint64_t ab = 0;
      // columns y0..y0+3: rel ts, inline children, packed counts (and, FA / FB, the fine key's parts)
      struct Col4 {
        uint32_t ts[4], ni[4], fa[4];
        uint64_t pb[4], fb[4];
      };
      auto col4 = [&](uint32_t y0, bool FA, bool FB) {
        Col4 c;
        const uint4 a = *(const uint4 *)&tts[y0], b = *(const uint4 *)&tni[y0];
        const ulonglong2 p0 = *(const ulonglong2 *)&tpb[y0], p1 = *(const ulonglong2 *)&tpb[y0 + 2];
        c.ts[0] = a.x, c.ts[1] = a.y, c.ts[2] = a.z, c.ts[3] = a.w;
        c.ni[0] = b.x, c.ni[1] = b.y, c.ni[2] = b.z, c.ni[3] = b.w;
        c.pb[0] = p0.x, c.pb[1] = p0.y, c.pb[2] = p1.x, c.pb[3] = p1.y;
#pragma unroll
        for (int k = 0; k < 4; k++) {  // (opaque: else the selects below become a masked load each, and a wait)
          asm("" : "+v"(c.pb[k]));
          asm("" : "+v"(c.ni[k]));
        }
        if (FA) {
          const uint4 f = *(const uint4 *)&tfa[y0];
          c.fa[0] = f.x, c.fa[1] = f.y, c.fa[2] = f.z, c.fa[3] = f.w;
        }
        if (FB) {
          const ulonglong2 f0 = *(const ulonglong2 *)&tfb[y0], f1 = *(const ulonglong2 *)&tfb[y0 + 2];
          c.fb[0] = f0.x, c.fb[1] = f0.y, c.fb[2] = f1.x, c.fb[3] = f1.y;
        }
        return c;
      };
      auto acc = [&](const Col4 &c, int k, bool bef, bool lt, bool le) {
        ab += bef ? c.pb[k] : 0ull;
        lp += le;
        ipf += lt ? c.ni[k] : 0u;
      };
      if (!ltile && !lrow) {  // (the whole keys in one 64-bit compare)
        const uint64_t kx = (uint64_t)tx << 32 | fax;
#pragma unroll 2
        for (uint32_t y0 = 0; y0 < (uint32_t)GJ; y0 += 4) {
          const Col4 c = col4(y0, false, true);
#pragma unroll
          for (int k = 0; k < 4; k++) acc(c, k, c.fb[k] < kx, c.ts[k] < tx, c.ts[k] <= tx);
        }
      } else if (!lrow) {  // gen-0 row, local columns: before iff an earlier ts
#pragma unroll 4
        for (uint32_t y0 = 0; y0 < (uint32_t)GJ; y0 += 4) {
          const Col4 c = col4(y0, false, false);
#pragma unroll
          for (int k = 0; k < 4; k++) {
            const bool lt = c.ts[k] < tx;
            acc(c, k, lt, lt, c.ts[k] <= tx);
          }
        }
      } else if (!ltile) {  // local row, gen-0 columns: before iff ts <= the row's
#pragma unroll 4
        for (uint32_t y0 = 0; y0 < (uint32_t)GJ; y0 += 4) {
          const Col4 c = col4(y0, false, false);
#pragma unroll
          for (int k = 0; k < 4; k++) {
            const bool le = c.ts[k] <= tx;
            acc(c, k, le, c.ts[k] < tx, le);
          }
        }
      } else {  // local x local
        const int self = (i - W >= j0 && i - W < j0 + n) ? (int)(i - W - j0) : -1;
        bool tie = false;
#pragma unroll 2
        for (uint32_t y0 = 0; y0 < (uint32_t)GJ; y0 += 4) {
          const Col4 c = col4(y0, true, true);
#pragma unroll
          for (int k = 0; k < 4; k++) {
            const bool lt = c.ts[k] < tx, eq = c.ts[k] == tx;
            const bool ea = eq & (c.fa[k] == fax);
            tie |= ea & (c.fb[k] == fbx) & ((int)(y0 + k) != self);
            acc(c, k, lt | (eq & (c.fa[k] < fax)) | (ea & (c.fb[k] < fbx)), lt, lt | eq);
          }
        }
#ifdef NSGPU_PHASE_PROF
        gt_kind |= __any(tie) ? 4u : 0u;
#endif
        if (tie) {  // (rare: equal words — a clamped ancestor uid, or one ancestor's chains)
          for (uint32_t y = 0; y < n; y++) {
            if (tts[y] != tx || tfa[y] != fax || tfb[y] != fbx || (int)y == self) continue;
            const bool lt = tu[y] != xu ? tu[y] < xu : lk_before(M.lkey[tr[y] - LBASE], M.lkey[xrec - LBASE]);
            if (lt) ab += tpb[y];
          }
        }
      }
      gr += (uint32_t)(ab & 0x7fu);
      cp += (uint32_t)((ab >> 7) & 0x3fffffu);
      ip += (uint32_t)((ab >> 29) & 0x3fffffu);
    }
    GT_MARK(2);
    __syncthreads();
   }
   if (i < NR) {
     // two packed 64-bit accumulators instead of five words: (rank, group end, inline prefix: each at
     // most MAXR x NACC < 2^21) and (child prefix < 2^32, the group's inline prefix)
     unsigned long long *A = reinterpret_cast<unsigned long long *>(M.gacc);
     const uint32_t row = lrow ? (uint32_t)WCAP + (i - W) : i;
     const uint64_t w0 = (uint64_t)gr | ((uint64_t)lp << 21) | ((uint64_t)ip << 42);
     const uint64_t w1 = (uint64_t)cp | ((uint64_t)ipf << 32);
     if (w0) atomicAdd(&A[row], (unsigned long long)w0);
     if (w1) atomicAdd(&A[NACC + row], (unsigned long long)w1);
   }
  }
#ifdef NSGPU_PHASE_PROF
  __builtin_amdgcn_s_waitcnt(0);
  if (gt_rec && threadIdx.x == 0) {
    g_gt[blockIdx.x][0] = gt_t0;
    for (int k = 0; k < 3; k++) g_gt[blockIdx.x][1 + k] = gt_t[k];
    g_gt[blockIdx.x][4] = __builtin_amdgcn_s_memrealtime();
    uint32_t xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
    g_gt[blockIdx.x][5] = xcc;
    g_gt[blockIdx.x][6] = gt_kind;
  }
#endif
#undef GT_MARK
}

// k_gsort: this rank's records into its X1 list at their ranks among themselves (k_gtile's accumulators hold only
// this rank's contributions until k_gsearch), with the prefixes before each and the totals after the last.
template <bool WIDE>
__global__ __launch_bounds__(256) void k_gsort(const P2PDev M) {
  const Ctl &C = *M.C;
  const uint32_t hdl = C.hdl, W = C.pW;
  const uint32_t L = WIDE ? x1hdr(M.x1_send, 0)->L : 0u;
  if (!hdl) return;
  const uint32_t NR = W + L, i = blockIdx.x * 256 + threadIdx.x;
  SEnt *S = x1srt(M.x1_send, 0);
  if (NR == 0) {
    if (i == 0) S[0] = SEnt{~0ull, ~0ull, ~0u, 1u, 0u, 0u};
    return;
  }
  if (i >= NR) return;
  const uint64_t *A = reinterpret_cast<const uint64_t *>(M.gacc);
  const bool lrow = WIDE && i >= W;
  const uint32_t row = lrow ? (uint32_t)WCAP + (i - W) : i;
  const uint64_t w0 = A[row], w1 = A[NACC + row];
  SEnt e;
  uint32_t cnt;
  if (lrow) {
    const X1Loc x = x1loc(M)[i - W];
    e = SEnt{x.w1, x.w2, x.anc, 1u, 0u, 0u};
    cnt = x.cnt;
  } else {
    const X1Ent x = x1ent(M)[i];
    e = SEnt{x.key, 0ull, 0u, 0u, 0u, 0u};
    cnt = x.cnt;
  }
  const uint32_t gr = (uint32_t)(w0 & 0x1fffffu);
  e.cp = (uint32_t)w1;
  e.ip = (uint32_t)(w0 >> 42);
  if (gr < NR) S[gr] = e;
  else atomicOr(M.error, 64u);  // (ranks among the rank's own records are a permutation)
  if (gr == NR - 1) S[NR] = SEnt{~0ull, ~0ull, ~0u, 1u, e.cp + (cnt & 0xffffu), e.ip + (cnt >> 16)};
}

// Record e of another rank before this rank's record x, in the merged dispatch order: earlier rel ts, then a gen-0
// record before a local one, then (gen-0) the uid, (local) the order words and the ancestor uid.
__device__ __forceinline__ bool sent_before(uint64_t ek0, uint32_t eL, uint64_t eb, uint32_t ec, uint64_t xk0, uint32_t xL,
                                            uint64_t xb, uint32_t xc) {
  if ((ek0 >> 32) != (xk0 >> 32)) return (ek0 >> 32) < (xk0 >> 32);
  if (eL != xL) return eL < xL;
  if ((uint32_t)ek0 != (uint32_t)xk0) return (uint32_t)ek0 < (uint32_t)xk0;
  if (eb != xb) return eb < xb;
  return ec < xc;
}
constexpr int GS_T = 256;             // k_gsearch: rows a block (one peer rank per blockIdx.y)
constexpr int GS_STEP = 32;           // every GS_STEP-th record of the peer's list sampled into LDS
constexpr int GS_NS = NACC / GS_STEP + 1;
// k_gsearch: this rank's records against each other rank's sorted list — three searches a (row, peer): the
// records before the row, those of a smaller ts, those of ts <= its own — first over the list's samples in LDS,
// then within GS_STEP entries in the list (five trips); the counts and the prefixes found there are added to the
// row's accumulators (k_gtile's packing).  Block (0, 0) also sums every rank's inline children for k_dfin2.
template <bool WIDE>
__global__ __launch_bounds__(GS_T) void k_gsearch(const P2PDev M) {
  Ctl &C = *M.C;
  const uint32_t hdl = C.hdl, W = C.pW;
  const uint32_t L = WIDE ? x1hdr(M.x1_send, 0)->L : 0u;
  const uint32_t q = blockIdx.y < M.rank ? blockIdx.y : blockIdx.y + 1u;  // (the peer)
  const X1Hdr *hq = x1hdr(M.x1_recv, q);
  const uint32_t nq = hq->W + (WIDE ? hq->L : 0u);
  const uint32_t tq = threadIdx.x < M.nranks ? x1hdr(M.x1_recv, threadIdx.x)->tinl : 0u;
  if (!hdl) return;
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x < 64) {  // (wave 0: one lane per rank)
    const uint32_t tg = wave_sum32(tq);
    if (threadIdx.x == 0) C.gt_tinl = tg;
  }
  const uint32_t NR = W + L, i = blockIdx.x * GS_T + threadIdx.x;
  if (blockIdx.x * GS_T >= NR) return;  // (block-uniform)
  const SEnt *S = x1srt(M.x1_recv, q);
  __shared__ uint64_t s_k0[GS_NS], s_b[GS_NS];
  __shared__ uint32_t s_c[GS_NS], s_L[GS_NS];
  const uint32_t ns = (nq + GS_STEP - 1) / GS_STEP;
  for (uint32_t k = threadIdx.x; k < ns; k += GS_T) {
    const SEnt e = S[k * GS_STEP];
    s_k0[k] = e.k0, s_b[k] = e.b, s_c[k] = e.c, s_L[k] = e.L;
  }
  __syncthreads();
  if (i >= NR) return;
  const bool lrow = WIDE && i >= W;
  uint64_t xk0, xb = 0;
  uint32_t xc = 0, xL = 0;
  if (lrow) {
    const X1Loc x = x1loc(M)[i - W];
    xk0 = x.w1, xb = x.w2, xc = x.anc, xL = 1u;
  } else {
    xk0 = x1ent(M)[i].key;
  }
  const uint32_t xts = (uint32_t)(xk0 >> 32);
  // the samples: how many satisfy each predicate (a prefix of them: the list is sorted)
  uint32_t lo[3] = {0, 0, 0}, cn[3] = {ns, ns, ns};
  while (cn[0] | cn[1] | cn[2]) {
#pragma unroll
    for (int k = 0; k < 3; k++) {
      if (!cn[k]) continue;
      const uint32_t h = cn[k] >> 1, m = lo[k] + h;
      const uint32_t ets = (uint32_t)(s_k0[m] >> 32);
      const bool p = k == 0 ? sent_before(s_k0[m], s_L[m], s_b[m], s_c[m], xk0, xL, xb, xc) : k == 1 ? ets < xts : ets <= xts;
      if (p) lo[k] = m + 1, cn[k] -= h + 1;
      else cn[k] = h;
    }
  }
  // within the list: entries ((c - 1) * STEP, min (c * STEP, nq)) after the last satisfying sample c - 1
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const uint32_t c = lo[k];
    if (c == 0) {
      cn[k] = 0;
    } else {
      lo[k] = (c - 1) * GS_STEP + 1;
      const uint32_t hi = c * GS_STEP < nq ? c * GS_STEP : nq;
      cn[k] = hi > lo[k] ? hi - lo[k] : 0u;
    }
  }
  while (cn[0] | cn[1] | cn[2]) {  // (the three searches' loads in flight together)
    uint32_t m[3];
    uint64_t ek0[3];
#pragma unroll
    for (int k = 0; k < 3; k++) m[k] = lo[k] + (cn[k] >> 1);
    const SEnt e0 = S[m[0]];
    ek0[0] = e0.k0;
    ek0[1] = S[m[1]].k0;
    ek0[2] = S[m[2]].k0;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      if (!cn[k]) continue;
      const uint32_t h = cn[k] >> 1, ets = (uint32_t)(ek0[k] >> 32);
      const bool p = k == 0 ? sent_before(e0.k0, e0.L, e0.b, e0.c, xk0, xL, xb, xc) : k == 1 ? ets < xts : ets <= xts;
      if (p) lo[k] = m[k] + 1, cn[k] -= h + 1;
      else cn[k] = h;
    }
  }
  const uint32_t p = lo[0], plt = lo[1], ple = lo[2];  // (<= nq: entry nq is the sentinel)
  const SEnt ep = S[p];
  const uint32_t ipf = S[plt].ip;
  if (p < nq && ep.k0 == xk0 && ep.L == xL && ep.b == xb && ep.c == xc) atomicOr(M.error, 64u);  // (a tie: impossible)
  unsigned long long *A = reinterpret_cast<unsigned long long *>(M.gacc);
  const uint32_t row = lrow ? (uint32_t)WCAP + (i - W) : i;
  const uint64_t w0 = (uint64_t)p | ((uint64_t)ple << 21) | ((uint64_t)ep.ip << 42);
  const uint64_t w1 = (uint64_t)ep.cp | ((uint64_t)ipf << 32);
  if (w0) atomicAdd(&A[row], (unsigned long long)w0);
  if (w1) atomicAdd(&A[NACC + row], (unsigned long long)w1);
}

// Block 0 also does the pool bookkeeping (k2_scan's) and, last, the run bookkeeping; the other blocks
// read only fields block 0 leaves alone (pW, puid0, hdl, done < 2).  WIDE: threads WCAP.. take this rank's local
// records (X1Loc order): a local record's uid is its parent's child prefix + its child index.
constexpr int DF2_FB = 2;  // k_dfin2's blocks before the record blocks (the books, the free-stack move)
template <bool WIDE>
__global__ __launch_bounds__(HB) void k_dfin2(const P2PDev M) {
  Ctl &C = *M.C;
  BLK_T0();
#ifdef NSGPU_PHASE_PROF
  const uint64_t c_win = C.windows;  // (diagnostic: block stamps in g_blk[2], the partitioned path runs no k2_scan)
#endif
  const uint32_t hdl = C.hdl, W = C.pW;  // (tested after the loads below: a load after a branch on it waited for it)
  const uint32_t tinl_g = C.gt_tinl, Lown = WIDE ? C.gt_lown : 0u;  // (k_gtile's, from the X1 headers)
  // block 0: every rank's X1 header at once, one lane per rank (HB = one wave)
  const uint32_t lq = threadIdx.x;
  const X1Hdr *lh = x1hdr(M.x1_recv, lq < M.nranks ? lq : 0u);
  const bool lv = lq < M.nranks;
  const uint32_t l_q = (WIDE && lv && blockIdx.x == 0) ? lh->L : 0u;  // (the ranks' local records)
  // (block 0: the rest of the summaries and the run control, for the run bookkeeping, in the same trip)
  struct Bk {
    uint64_t nF, nfree, npush, pK0, ptmin, windows, P_end, live, inline_lim, max_windows, max_window, drg, dr1;
    uint64_t bound, span_t;
    uint32_t nhub, puid0, rt, drtrim, drun;
  } bk{};
  if (blockIdx.x <= 1)  // (block 1: the free-stack move and the hubs' tables, beside block 0's bookkeeping)
    bk = Bk{C.nF, C.nfree, C.npush, C.pK0, C.ptmin, C.windows, C.P_end, C.live, C.inline_lim, C.max_windows,
            C.max_window, C.drg, C.dr1, WIDE ? C.bound : 0, WIDE ? C.span_t : 0, C.nhub, C.puid0, C.rt, C.drtrim,
            C.drun};
  uint32_t hW = 0, htc = 0, hneedc = 0, hsuid = 0;
  uint64_t hlk = 0, htmin = ~0ull, hwend = ~0ull, hwendw = ~0ull, hsts = ~0ull, hrkey = ~0ull, hrrem = 0,
           hrhead = ~0ull;
  if (blockIdx.x == 0 && lv) {
    hW = lh->W;
    htc = lh->tc;
    hneedc = lh->needc;
    hlk = lh->lastkey;
    htmin = lh->red.tmin;
    hwend = lh->red.wend;
    hwendw = lh->red.wendw;
    hsts = lh->red.stopts;
    hsuid = lh->red.stopuid;
    hrkey = lh->rkey;
    hrrem = lh->rrem;
    hrhead = lh->rhead;
  }
  // the record's accumulators, record and first children, all loaded before anything waits — with the headers,
  // before the arrival's wait (WIDE: thread WCAP + k takes local record k of this rank, its record index from
  // the X1Loc list: one more trip; its parent's child prefix needs the parent's accumulator, one more)
  // (block 0 keeps the books, block 1 moves the free stack: the records are the next blocks' — block 0 was the
  //  kernel's tail with the books after its own records, block 1 with the stack move after its records)
  const bool rec_block = blockIdx.x >= (uint32_t)DF2_FB;
  const uint32_t ti = (rec_block ? blockIdx.x - (uint32_t)DF2_FB : 0u) * HB + threadIdx.x;
  const bool loc = WIDE && ti >= (uint32_t)WCAP;
  uint64_t *A = reinterpret_cast<uint64_t *>(M.gacc);
  uint64_t w0, w1, wk;
  uint32_t s = ti, wc, ncr, ckw[PFC], cctx[PFC], wpar = 0;
  {  // (speculative: every thread loads, whether or not its record exists — the indices stay in range)
    uint64_t lw1 = 0;
    if (loc) {
      const X1Loc e = x1loc(M)[ti - WCAP];
      s = e.rec < (uint32_t)WTOT ? e.rec : (uint32_t)WTOT - 1u;
      lw1 = e.w1;
      wpar = e.par;
    }
    w0 = A[ti];
    w1 = A[NACC + ti];
    wk = loc ? lw1 : M.wkey[s];
    wc = M.wctx[s];
    ncr = M.nchild[s];
#pragma unroll
    for (int j = 0; j < PFC; j++) {  // (a child index past maxc loads the slot's last one: in range, ignored)
      const uint32_t sl = s * M.maxc + min((uint32_t)j, M.maxc - 1u);
      ckw[j] = M.ch_kind[sl];
      cctx[j] = M.ch_ctx[sl];
    }
  }
  if (!hdl) return;  // (k2_handle ran nothing: a cut, a pause, the end)
  // X1 is all-gathered in place (x1_send is this rank's slot of x1_recv): block 0, the kernel's only reader of the
  // headers (k_gtile's reads ended with its launch), resets this rank's for the next window once its loads have
  // returned (one wave: the wave's wait covers every lane)
  if (blockIdx.x == 0) {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_s_waitcnt(0);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    X1Hdr *hs = x1hdr(M.x1_send, 0);
    hs->W = hs->tc = hs->tinl = hs->needc = 0;
    hs->L = 0;
    hs->lastkey = 0;
    hs->red.tmin = hs->red.wend = hs->red.stopts = hs->red.wendw = ~0ull;
    hs->red.stopuid = 0;
    hs->rkey = ~0ull;
    hs->rrem = 0;
  }
  const bool vs = rec_block && (loc ? ti - (uint32_t)WCAP < Lown : ti < W);
  if (vs) {
    if (!WIDE) {  // (wide: k2_handle zeroes them — a local record reads its parent's below)
      A[ti] = 0;
      A[NACC + ti] = 0;
    }
    const uint32_t gr = (uint32_t)(w0 & 0x1fffffu), lp = (uint32_t)((w0 >> 21) & 0x1fffffu),
                   ip = (uint32_t)(w0 >> 42), cp = (uint32_t)w1, ipf = (uint32_t)(w1 >> 32);
    // as k2_scan: (dispatch rank rel. K0, rank of the first inline child, child prefix, inline prefix)
    M.sinfo[s] = make_uint4(gr + (tinl_g ? ipf : 0), lp + ip, cp, ip);
    if (loc) {  // uid = the parent's child prefix + the child index (DefaultSimulatorImpl::Schedule order)
      const uint32_t prow = wpar & 0xffffffu;  // (k_xlcompact: the parent's row, gen-0 slot or WCAP + compact index)
      const uint32_t pcp = (uint32_t)A[NACC + (prow < (uint32_t)NACC ? prow : 0u)];
      M.pwkey[s] = ((wk >> 32) << 32) | (uint32_t)(C.puid0 + pcp + (wpar >> 24));
      M.lrec[ti - WCAP] = s;
    } else {
      M.pwkey[s] = wk;
    }
    M.pwctx[s] = wc;
    const uint32_t uid0 = C.puid0;
    // the record's children on other ranks' nodes -> X2 (one rank: none).  Their kinds eight at a time (one
    // dependent load a child past the first PFC held a record with many children ~10 us: the kernel's tail)
    constexpr int KB = 8;
    static_assert(PFC <= KB, "the preloaded kinds fit the first batch");
    for (uint32_t j0 = 0; M.nranks > 1 && j0 < ncr; j0 += KB) {
      uint32_t kwv[KB];
#pragma unroll
      for (int q = 0; q < KB; q++) {
        const uint32_t j = j0 + q;
        kwv[q] = (j0 == 0 && q < PFC) ? ckw[q < PFC ? q : 0] : j < ncr ? M.ch_kind[s * M.maxc + j] : 0u;
      }
#pragma unroll
      for (int q = 0; q < KB; q++) {
        const uint32_t j = j0 + q, kw = kwv[q];
        if (j >= ncr || (kw & 0xffu) == K_FWD_UP) continue;
        if (!(kw & REMOTEBIT)) continue;  // (a Receive on another rank's node: the device step marked it)
        const uint32_t sl = s * M.maxc + j;
        const uint32_t ctx = (j0 == 0 && q < PFC) ? cctx[q < PFC ? q : 0] : M.ch_ctx[sl];
        const uint32_t qr = M.owner[ctx];
        const uint32_t pos = atomicAdd(&x2hdr(M, M.x2_send, qr)->n, 1u);
        if (pos < M.capx)
          x2rec(M, M.x2_send, qr)[pos] = Ev{M.ch_ts[sl], uid0 + cp + j, ctx, kw, M.ch_a[sl], M.ch_pkt[sl]};
        else
          atomicOr(M.error, 16u);
      }
    }
  }
  // ---- pool bookkeeping (k2_scan's): the free stack loses the slots the fresh children took and gains
  // the window's; its pushed part is moved down over the popped hole; the hubs' slot tables are cleared
  const uint64_t nF = bk.nF, nfree = bk.nfree, npush = bk.npush;
  const uint64_t consumed = nF < nfree ? nF : nfree;
  const uint64_t mv = consumed < npush ? consumed : npush;
  const uint32_t nh = bk.nhub < (uint32_t)MAXHUB ? bk.nhub : (uint32_t)MAXHUB;
  if (blockIdx.x == 1) {  // the free-stack move and the hubs' slot tables (the two ranges are disjoint: eight
    constexpr int SB = 8;  // loads in flight a lane, then the stores)
    for (uint64_t i0 = threadIdx.x; i0 < mv; i0 += (uint64_t)HB * SB) {
      uint32_t v[SB];
#pragma unroll
      for (int k = 0; k < SB; k++) {
        const uint64_t i = i0 + (uint64_t)k * HB;
        v[k] = i < mv ? M.fstack[nfree + npush - mv + i] : 0u;
      }
#pragma unroll
      for (int k = 0; k < SB; k++) {
        const uint64_t i = i0 + (uint64_t)k * HB;
        if (i < mv) M.fstack[nfree - consumed + i] = v[k];
      }
    }
    for (uint32_t h = threadIdx.x; h < nh; h += HB) M.node_tab[(uint64_t)M.hub_list[h] * NTAB] = 0;
  }
  if (blockIdx.x != 0) {
    BLK_REC(2, c_win);
    return;
  }
  // the ranks' summaries, reduced across the lanes (rank q's in lane q)
  const uint32_t Wg = wave_sum32(hW), tcg = wave_sum32(htc), Lg = WIDE ? wave_sum32(l_q) : 0u;
  const uint32_t needc = __ballot(hneedc != 0) ? 1u : 0u;
  // a partitioned sorted run: entries left on some rank -> the next chunk (drun_cut), unless the chunk just
  // run ended the run (it ended a cut same-ts group)
  const bool drun_more = __ballot(hrrem != 0) != 0;
  const uint64_t drfk = wave_min64(hrrem != 0 ? hrkey : ~0ull), drhk = wave_min64(hrrem != 0 ? hrhead : ~0ull);
  const uint64_t lk = wave_max64(hW ? hlk : 0ull);
  Red rg{~0ull, ~0ull, ~0ull, 0, 0, ~0ull};
  rg.tmin = wave_min64(htmin);
  rg.wend = wave_min64(hwend);
  if (WIDE) rg.wendw = wave_min64(hwendw);
  // wide windows: the adaptive span keeps every rank's window inside its capacity (WCAP gen-0, NMAX records;
  // k2_scan's rule, from the largest rank's counts so that every rank forms the same bound)
  const uint64_t mxW = WIDE ? wave_max64(hW) : 0, mxN = WIDE ? wave_max64((uint64_t)hW + l_q) : 0;
  {  // the pending Stop: the smallest stopts, the first rank holding it
    rg.stopts = wave_min64(hsts);
    const uint64_t m = __ballot(lv && hsts == rg.stopts && rg.stopts != ~0ull);
    const int first = m ? __ffsll((unsigned long long)m) - 1 : 0;
    rg.stopuid = __shfl(hsuid, first);
  }
  if (threadIdx.x != 0) return;  // (the reductions above took the whole wave)
  C.K = bk.pK0 + Wg + Lg + tinl_g;
  if (WIDE) {
    C.plt = Lown;  // (the next k2_pa appends them from lrec)
    if (!bk.drun) {  // (a run's chunks are narrow)
      const uint64_t span = bk.bound >> 32;
      if (mxN > (uint64_t)(7 * NMAX / 8) || mxW > (uint64_t)(7 * WCAP / 8)) C.span_t = span - span / 4;
      else if (mxN < (uint64_t)(3 * NMAX / 4) && mxW < (uint64_t)(3 * WCAP / 4) && bk.span_t < (1ull << 40))
        C.span_t = bk.span_t + bk.span_t / 8 + 1;
    }
  }
  C.uid = bk.puid0 + tcg;
  if (Wg) C.last_ts = bk.ptmin + (lk >> 32);
  const uint32_t rt = bk.rt;
  C.red[rt] = rg;  // bounds the next window (k2_pa reads red[rt ^ 1] after the flip)
  C.rt = rt ^ 1;
  const uint64_t windows = bk.windows + 1;
  C.windows = windows;
  if (Wg + Lg > bk.max_window) C.max_window = Wg + Lg;
  const uint64_t P_end = bk.P_end + (nF > nfree ? nF - nfree : 0);
  C.nfree = nfree - consumed + npush;
  C.P_end = P_end;
  C.live = bk.live - npush + nF;
  C.npush = 0;
  C.nF = 0;
  C.nhub = 0;
  C.W = 0;
  C.overflow = 0;
  C.prep = 0;
  {
    const bool go = drun_more && !bk.drtrim;
    const DrunCut dc = go ? drun_cut(drfk, drhk, bk.drg) : DrunCut{~0ull, ~0ull, 0u};
    C.drun = go ? 1u : 0u;
    C.dr0 = bk.dr1;  // (the chunk just run ended there; k2_pa reads dr0 at its start)
    C.drg = dc.g;
    C.drlo = dc.lo;
    C.drtrim = dc.trim;
    C.dtrim = drun_more && bk.drtrim ? 1u : 0u;  // (the next k2_pa returns the run's entries left to pending)
  }
  // the window that held Simulator::Stop ends the run (every rank knows it from the bound), as does an
  // empty pending set on every rank (a run's entries from the fresh buffer are pending outside the pool)
  bool done = bk.inline_lim != ~0ull || (rg.tmin == ~0ull && !drun_more);
  if (P_end > M.pool_cap) {
    atomicOr(M.error, 1u);
    done = true;
  }
  if (windows >= bk.max_windows && !done) {
    atomicOr(M.error, 4u);
    done = true;
  }
  if ((uint64_t)bk.puid0 + tcg > UID_MAX_NEXT) {  // (every rank: tcg is the merged window's)
    atomicOr(M.error, 2048u);
    done = true;
  }
  if (done) C.done = 1;
  else if (needc && !drun_more) C.mode = MODE_COMPACT;  // (every rank: the pipelines stay in step; a run's
                                                         //  pool entries keep their slots until it ends)
  BLK_REC(2, c_win);
}

// Loopback transport (nsgpu_p2p_group_*: every partition on one device): one block per copy.
struct CopyDesc {
  const uint8_t *src;
  uint8_t *dst;
  uint64_t bytes;  // multiple of 16
};
__global__ __launch_bounds__(256) void k_copies(const CopyDesc *__restrict__ d) {
  const CopyDesc c = d[blockIdx.x];
  const uint4 *src = (const uint4 *)c.src;
  uint4 *dst = (uint4 *)c.dst;
  for (uint64_t i = threadIdx.x; i < c.bytes / 16; i += 256) dst[i] = src[i];
}

}  // namespace nsgpu
// ====================================================================================================
// Host side: scenario upload, setup-time event list, launch, results.
// ====================================================================================================
#include <vector>
#include <algorithm>
#include <string.h>
#include <stdlib.h>
#include <rccl/rccl.h>

using namespace nsgpu;

// (nsgpu_comm, NCCL_TRY: nsgpu_internal.h)

extern "C" int nsgpu_comm_unique_id(uint8_t *id) {
  if (!id) return set_error(NSGPU_EINVAL, "nsgpu_comm_unique_id: null");
  ncclUniqueId u;
  NCCL_TRY(ncclGetUniqueId(&u));
  memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
  return NSGPU_OK;
}

extern "C" int nsgpu_comm_init(const uint8_t *id, int nranks, int rank, nsgpu_comm **out) {
  if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks)
    return set_error(NSGPU_EINVAL, "nsgpu_comm_init: bad arguments");
  ncclUniqueId u;
  memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
  nsgpu_comm *c = new nsgpu_comm();
  const ncclResult_t r = ncclCommInitRank(&c->comm, nranks, u, rank);
  if (r != ncclSuccess) {
    delete c;
    return set_error(NSGPU_EHIP, "ncclCommInitRank: %s", ncclGetErrorString(r));
  }
  c->nranks = nranks;
  c->rank = rank;
  *out = c;
  return NSGPU_OK;
}

extern "C" int nsgpu_comm_destroy(nsgpu_comm *c) {
  if (!c) return NSGPU_OK;
  if (c->comm) (void)ncclCommDestroy(c->comm);
  delete c;
  return NSGPU_OK;
}

struct nsgpu_p2p {
  P2PDev M;
  nsgpu_p2p_scenario sc;  // (its host pointers are the caller's: not used after nsgpu_p2p_create)
  std::vector<uint32_t> app_kind;
  std::vector<void *> allocs;
  Ctl C0{};               // run control after reset
  uint32_t uid_hint = 4;  // the run control's uid as last seen by the host (the deferred pipeline starts below UID_DF_SOFT)
  uint64_t max_windows = ~0ull;
  hipStream_t s = nullptr;  // engine stream (graph capture and replay)
  hipGraphExec_t gexec = nullptr;
  hipGraphExec_t gexec_df = nullptr;  // the deferred pipeline's replay (single wide engine, untraced)
  hipGraphExec_t gtail[2] = {nullptr, nullptr};  // NWIN_TAIL-window replays (plain, deferred): a run's last windows
  hipEvent_t ev[2] = {nullptr, nullptr}, t0 = nullptr, t1 = nullptr;
  uint32_t *done_host = nullptr;  // pinned, 2 slots
  Ctl *snap = nullptr;            // pinned, 2 run-control snapshots (single engine)
  float last_ms = 0.f;
  bool eager = getenv("NSGPU_P2P_EAGER") != nullptr;  // kernels one by one instead of graph replays
  // NSGPU_P2P_POISON=1: every device array is filled with 0xa5 bytes when allocated, before create initialises
  // it (a deterministic stand-in for device memory a previous engine dirtied: create must zero what it reads)
  bool poison = [] {
    const char *e = getenv("NSGPU_P2P_POISON");
    return e && e[0] == '1';
  }();
  // pristine initial pool (device) for resets
  uint64_t *init_ts = nullptr;
  uint32_t *init_uid = nullptr, *init_ctx = nullptr, *init_kind = nullptr, *init_a = nullptr;
  const DevRec *dev_init = nullptr;  // device records after reset (tx state idle)
  uint32_t n_apps = 0;
  // partitioned run
  nsgpu_comm *comm = nullptr;  // RCCL transport (null: a loopback group member)
  X1Hdr x1h0{};                // empty X1 summary (reset template)
};

namespace {
template <class T>
int dalloc(nsgpu_p2p *h, T **p, size_t n) {
  void *q = nullptr;
  hipError_t e = hipMalloc(&q, (n ? n : 1) * sizeof(T));
  if (e != hipSuccess) return set_error(NSGPU_ENOMEM, "nsgpu_p2p: hipMalloc(%zu): %s", n * sizeof(T),
                                        hipGetErrorString(e));
  h->allocs.push_back(q);
  if (h->poison) NSGPU_HIP(hipMemset(q, 0xa5, (n ? n : 1) * sizeof(T)));
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
  if (h->gexec_df) (void)hipGraphExecDestroy(h->gexec_df);
  for (hipGraphExec_t g : h->gtail)
    if (g) (void)hipGraphExecDestroy(g);
  for (hipEvent_t e : {h->ev[0], h->ev[1], h->t0, h->t1})
    if (e) (void)hipEventDestroy(e);
  if (h->done_host) (void)hipHostFree(h->done_host);
  if (h->snap) (void)hipHostFree(h->snap);
  if (h->s) (void)hipStreamDestroy(h->s);
  for (void *p : h->allocs) (void)hipFree(p);
  delete h;
  return NSGPU_OK;
}

// What a rank's engine is built from, computed on the host before any device allocation (create_engine) and
// exposed as nsgpu_p2p_dist_plan: every rank of a partitioned run must get the same lookaheads, window capacities
// and exchange sizes — a mismatch would be a collective of different sizes (an RCCL hang), which the multi-process
// CPU tests check (tests/test_dist_cpu.py).
struct EnginePlan {
  uint32_t qcap = 1, maxapps = 0, maxc = 3, wide = 0;
  bool has_echo = false;
  std::vector<uint32_t> napps, node_list;
  std::vector<int32_t> sink;
  int64_t tx_min = 0, lx = 0, send_ivl = 0;
  int64_t lookahead[K_NKINDS], lookw[K_NKINDS];
  // the setup-time events (this rank's, partitioned) and the bound of window 0 (the whole setup: every rank)
  std::vector<uint64_t> its;
  std::vector<uint32_t> iuid, ictx, ikind, ia;
  Red red0{};
  uint32_t n_init = 0, uid_init = 0;
  uint64_t pool_cap = 0;
  uint32_t capx = 0;  // partitioned: X2 records per peer per window
  uint64_t x2b = 0;   // partitioned: X2 bytes per peer
};

static int plan_engine(const nsgpu_p2p_scenario *sc, const uint32_t *owner, int rank, int nranks, uint64_t pool_cap,
                       EnginePlan &P) {
  if (!sc) return set_error(NSGPU_EINVAL, "nsgpu_p2p_create: null");
  const uint32_t N = sc->n_nodes, D = sc->n_devices, A = sc->n_apps;
  if (N == 0 || !sc->setup_kind || !sc->setup_index) return set_error(NSGPU_EINVAL, "nsgpu_p2p_create: empty");
  // ---- validation (host arrays) ----
  uint32_t &qcap = P.qcap;
  qcap = 1;
  for (uint32_t d = 0; d < D; d++) {
    if (sc->dev_node[d] >= N || sc->dev_peer[d] >= D || sc->dev_peer[sc->dev_peer[d]] != d)
      return set_error(NSGPU_EINVAL, "nsgpu_p2p_create: device %u: bad node/peer", d);
    if (sc->dev_bps[d] == 0) return set_error(NSGPU_EINVAL, "nsgpu_p2p_create: device %u: zero DataRate", d);
    if (sc->dev_delay_ns[d] < 0 || sc->dev_ifg_ns[d] < 0)
      return set_error(NSGPU_EINVAL, "nsgpu_p2p_create: device %u: negative delay", d);
    qcap = std::max(qcap, sc->dev_qmax[d]);
  }
  if (owner) {
    if (nranks < 1 || nranks > MAXR || rank < 0 || rank >= nranks ||
        (uint64_t)nranks * CAPX_MAX + TB + 2 * WCAP >= (uint64_t)GRID_POOL_DIST * TB)  // (k2_pa: slot, remote, chunk blocks)
      return set_error(NSGPU_EINVAL, "nsgpu_p2p_create_dist: rank %d of %d (at most %d ranks)", rank, nranks,
                       (int)(((uint64_t)GRID_POOL_DIST * TB - TB - 2 * WCAP - 1) / CAPX_MAX));
    for (uint32_t n = 0; n < N; n++)
      if (owner[n] >= (uint32_t)nranks) return set_error(NSGPU_EINVAL, "nsgpu_p2p_create_dist: node %u: owner %u", n, owner[n]);
  }
  if (!sc->route) {  // compressed next-hop table
    if (!sc->route_default || !sc->route_exc_off || !sc->route_exc_slot || !sc->route_exc_dev ||
        sc->route_exc_off[0] != 0)
      return set_error(NSGPU_EINVAL, "nsgpu_p2p_create: no route table");
    for (uint32_t n = 0; n < N; n++) {
      if (sc->route_exc_off[n + 1] < sc->route_exc_off[n])
        return set_error(NSGPU_EINVAL, "nsgpu_p2p_create: route_exc_off not ascending at node %u", n);
      if (sc->route_default[n] != 0xffffffffu && sc->route_default[n] >= D)
        return set_error(NSGPU_EINVAL, "nsgpu_p2p_create: node %u: bad default route", n);
      for (uint64_t j = sc->route_exc_off[n]; j < sc->route_exc_off[n + 1]; j++)
        if ((j > sc->route_exc_off[n] && sc->route_exc_slot[j] <= sc->route_exc_slot[j - 1]) ||
            sc->route_exc_slot[j] >= sc->n_dst || (sc->route_exc_dev[j] != 0xffffffffu && sc->route_exc_dev[j] >= D))
          return set_error(NSGPU_EINVAL, "nsgpu_p2p_create: node %u: bad route exception %llu", n,
                           (unsigned long long)j);
    }
  }
  std::vector<uint32_t> &napps = P.napps;
  std::vector<int32_t> &sink = P.sink;
  napps.assign(N + 1, 0);
  sink.assign(N, -1);
  uint32_t min_pkt = 0xffffffffu;
  bool &has_echo = P.has_echo;
  has_echo = false;
  int64_t echo_ivl = (int64_t)1 << 61;
  for (uint32_t a = 0; a < A; a++) {
    if (sc->app_node[a] >= N) return set_error(NSGPU_EINVAL, "nsgpu_p2p_create: app %u: bad node", a);
    napps[sc->app_node[a] + 1]++;
    const uint32_t ak = sc->app_kind[a];
    if (ak == NSGPU_APP_SINK || ak == NSGPU_APP_ECHO_SERVER) {  // the node's bound UDP endpoint
      if (sink[sc->app_node[a]] >= 0)
        return set_error(NSGPU_EINVAL, "nsgpu_p2p_create: node %u has two bound endpoints", sc->app_node[a]);
      sink[sc->app_node[a]] = (int32_t)a;
      if (ak == NSGPU_APP_ECHO_SERVER) {
        if (sc->app_ttl[a] == 0) return set_error(NSGPU_EINVAL, "nsgpu_p2p_create: UdpEchoServer %u: ttl", a);
        has_echo = true;
      }
    } else if (ak == NSGPU_APP_ECHO_CLIENT) {
      if (!sc->app_count || !sc->app_interval_ns || !sc->app_src_slot || sc->app_dst_node[a] >= N ||
          sc->app_dst_slot[a] >= sc->n_dst || sc->app_src_slot[a] >= sc->n_dst || sc->app_pkt_size[a] == 0 ||
          sc->app_ttl[a] == 0 || sc->app_dst_node[a] == sc->app_node[a] || sc->app_interval_ns[a] < 0)
        return set_error(NSGPU_EINVAL, "nsgpu_p2p_create: UdpEchoClient %u: bad destination/size/ttl/interval", a);
      has_echo = true;
      min_pkt = std::min(min_pkt, sc->app_pkt_size[a]);
      echo_ivl = std::min(echo_ivl, sc->app_interval_ns[a]);
    } else if (ak != NSGPU_APP_ONOFF) {
      return set_error(NSGPU_EINVAL, "nsgpu_p2p_create: app %u: unknown kind %u", a, ak);
    } else {
      if (sc->app_dst_node[a] >= N || sc->app_dst_slot[a] >= sc->n_dst || sc->app_rate_bps[a] == 0 ||
          sc->app_pkt_size[a] == 0 || sc->app_ttl[a] == 0 || sc->app_dst_node[a] == sc->app_node[a] ||
          (sc->app_src_slot && sc->app_src_slot[a] != 0xffffffffu && sc->app_src_slot[a] >= sc->n_dst))
        return set_error(NSGPU_EINVAL, "nsgpu_p2p_create: OnOff %u: bad destination/rate/size/ttl/source slot", a);
      min_pkt = std::min(min_pkt, sc->app_pkt_size[a]);
    }
    // SendRealOut fragments a datagram above the device MTU (ipv4-l3-protocol.cc:722-731; PointToPointNetDevice
    // Mtu 1500): not modelled, so payloads are bounded by 1500 - 20 (IPv4) - 8 (UDP)
    if (ak == NSGPU_APP_ECHO_CLIENT || ak == NSGPU_APP_ONOFF) {
      if (sc->app_pkt_size[a] > 1472)
        return set_error(NSGPU_EINVAL, "nsgpu_p2p_create: app %u: %u-byte payload needs IPv4 fragmentation", a,
                         sc->app_pkt_size[a]);
    }
    if (A > NSGPU_PKT_APP) return set_error(NSGPU_EINVAL, "nsgpu_p2p_create: more than 2^28 applications");
  }
  uint32_t &maxapps = P.maxapps;
  maxapps = 0;
  for (uint32_t n = 0; n < N; n++) maxapps = std::max(maxapps, napps[n + 1]);
  for (uint32_t n = 0; n < N; n++) napps[n + 1] += napps[n];
  std::vector<uint32_t> &node_list = P.node_list, fill(napps.begin(), napps.end() - 1);
  node_list.assign(A, 0);
  for (uint32_t a = 0; a < A; a++) node_list[fill[sc->app_node[a]]++] = a;
  // ---- lookahead per event kind: the smallest delay a child of that kind can get ----
  const int64_t INFL = (int64_t)1 << 61;
  int64_t tx_min = INFL;
  if (min_pkt != 0xffffffffu)
    for (uint32_t d = 0; d < D; d++) {
      tx_min = std::min(tx_min, seconds_to_ts(static_cast<double>(min_pkt + 30) * 8 / (double)sc->dev_bps[d]));
      // an ICMP error is a 56-byte IPv4 packet (+2 PPP)
      if (sc->icmp) tx_min = std::min(tx_min, seconds_to_ts(static_cast<double>(56 + 2) * 8 / (double)sc->dev_bps[d]));
    }
  int64_t send_ivl = INFL;
  for (uint32_t a = 0; a < A; a++)
    if (sc->app_kind[a] == NSGPU_APP_ONOFF)
      send_ivl = std::min(send_ivl, seconds_to_ts((sc->app_pkt_size[a] * 8) / static_cast<double>(sc->app_rate_bps[a])));
  P.tx_min = tx_min;
  P.send_ivl = send_ivl;
  P.maxc = std::max(3u, 2 * maxapps);
  for (int k = 0; k < K_NKINDS; k++) P.lookahead[k] = INFL;
  P.lookahead[K_NODE_START] = 0;     // children at app start/stop times (may be 0)
  P.lookahead[K_APPOBJ_START] = 0;
  P.lookahead[K_APP_START] = 0;      // StartSending after OffTime (may be 0)
  P.lookahead[K_START_SENDING] = 0;  // first send after residual-shortened interval
  P.lookahead[K_STOP_SENDING] = 0;   // StartSending after OffTime
  P.lookahead[K_SEND] = std::min(std::min(tx_min, send_ivl), echo_ivl);
  P.lookahead[K_TX_COMPLETE] = tx_min;
  P.lookahead[K_RECEIVE] = tx_min;
  P.lookahead[K_FWD_UP_Q] = tx_min;  // UdpEchoServer reply: device children
  // A datagram for a UDP echo endpoint is delivered by a queued zero-delay DoForwardUp (its handler
  // schedules): the window must then end at the delivering Receive's time, so that the DoForwardUp is
  // the next window's first event at that time.
  if (has_echo) P.lookahead[K_RECEIVE] = 0;
  // Wide windows (nsgpu_p2p_win.h): an event on another node is at least one transmission
  // plus its channel delay away — Lx = min over devices of (smallest frame's tx time + delay) — and a
  // same-node TransmitComplete before the window's end runs inside the window (a local record), so only
  // the children that are neither bound the window: lookw = lookahead with tx_min replaced by Lx.
  int64_t lx = INFL;
  if (min_pkt != 0xffffffffu)
    for (uint32_t d = 0; d < D; d++) {
      int64_t t = seconds_to_ts(static_cast<double>(min_pkt + 30) * 8 / (double)sc->dev_bps[d]);
      if (sc->icmp) t = std::min(t, seconds_to_ts(static_cast<double>(56 + 2) * 8 / (double)sc->dev_bps[d]));
      lx = std::min(lx, t + sc->dev_delay_ns[d]);
    }
  for (int k = 0; k < K_NKINDS; k++) P.lookw[k] = P.lookahead[k];
  P.lookw[K_SEND] = std::min(std::min(lx, send_ivl), echo_ivl);
  P.lookw[K_TX_COMPLETE] = lx;
  P.lookw[K_RECEIVE] = has_echo ? 0 : lx;
  P.lookw[K_FWD_UP_Q] = lx;
  {  // a node's pending local records are its busy devices' TransmitCompletes: at most its degree
    std::vector<uint32_t> deg(N, 0);
    uint32_t dmax = 0;
    for (uint32_t d = 0; d < D; d++) dmax = std::max(dmax, ++deg[sc->dev_node[d]]);
    const char *nw = getenv("NSGPU_P2P_NARROW");
    // (a chain of same-node TransmitCompletes inside a window is shorter than Lx / tx_min: LKD levels)
    P.wide = (dmax <= (uint32_t)LQ && lx > tx_min && lx <= (int64_t)LKD * tx_min && lx < INFL &&
              !(nw && nw[0] == '1')) ? 1u : 0u;
    // partitioned: the ranks order each other's local records by their two order words (k_gtile), which are
    // exact for chains of at most 2 levels below a gen-0 event (the ancestor uid in X1Loc): the wide span is
    // kept below 3 tx_min, so a third level (3 transmissions after its gen-0 event) never falls in a window
    if (owner && P.wide)
      for (int k = 0; k < K_NKINDS; k++) P.lookw[k] = std::min<int64_t>(P.lookw[k], 3 * tx_min - 1);
  }
  P.lx = lx;
  // ---- setup-time events (node-list.cc:124-131, node.cc:111-145, default-simulator-impl.cc:179-183) ----
  std::vector<uint64_t> &its = P.its;
  std::vector<uint32_t> &iuid = P.iuid, &ictx = P.ictx, &ikind = P.ikind, &ia = P.ia;
  uint32_t uid = sc->uid_first ? sc->uid_first : 4u;  // (DefaultSimulatorImpl: m_uid (4), :52-56)
  if ((uint64_t)uid + sc->n_setup > UID_MAX_NEXT) {
    return set_error(NSGPU_EINVAL, "nsgpu_p2p_create: the setup calls' uids would pass 0xfffffffe");
  }
  for (uint32_t i = 0; i < sc->n_setup; i++) {
    const uint32_t k = sc->setup_index[i];
    switch (sc->setup_kind[i]) {
      case NSGPU_SETUP_NODE:
        if (k >= N) { return set_error(NSGPU_EINVAL, "setup: node %u", k); }
        its.push_back(0); iuid.push_back(uid); ictx.push_back(k); ikind.push_back(K_NODE_START); ia.push_back(k);
        break;
      case NSGPU_SETUP_DEVICE:
        if (k >= D) { return set_error(NSGPU_EINVAL, "setup: device %u", k); }
        its.push_back(0); iuid.push_back(uid); ictx.push_back(sc->dev_node[k]); ikind.push_back(K_DEV_START); ia.push_back(k);
        break;
      case NSGPU_SETUP_APP:
        if (k >= A) { return set_error(NSGPU_EINVAL, "setup: app %u", k); }
        its.push_back(0); iuid.push_back(uid); ictx.push_back(sc->app_node[k]); ikind.push_back(K_APPOBJ_START); ia.push_back(k);
        break;
      case NSGPU_SETUP_NOOP:
        if (k >= N) { return set_error(NSGPU_EINVAL, "setup: noop node %u", k); }
        its.push_back(0); iuid.push_back(uid); ictx.push_back(k); ikind.push_back(K_DEV_START); ia.push_back(k);
        break;
      case NSGPU_SETUP_STOP:
        if (sc->stop_ns < 0) { return set_error(NSGPU_EINVAL, "setup: negative stop"); }
        its.push_back((uint64_t)sc->stop_ns); iuid.push_back(uid); ictx.push_back(NOCTX); ikind.push_back(K_STOP); ia.push_back(0);
        break;
      default:
        break;  // consumes a uid, no event
    }
    uid++;
  }
  // reduction of the whole initial pending set: window 0 is bounded by red[1] on every rank
  Red &red0 = P.red0;
  red0 = Red{~0ull, ~0ull, ~0ull, 0, 0, ~0ull};
  for (size_t i = 0; i < its.size(); i++) {
    red0.tmin = std::min<uint64_t>(red0.tmin, its[i]);
    red0.wend = std::min<uint64_t>(red0.wend, its[i] + (uint64_t)P.lookahead[ikind[i] & 0xffu]);
    red0.wendw = std::min<uint64_t>(red0.wendw, its[i] + (uint64_t)P.lookw[ikind[i] & 0xffu]);
    if ((ikind[i] & 0xffu) == K_STOP) {
      red0.stopts = its[i];
      red0.stopuid = iuid[i];
    }
  }
  if (owner) {  // this rank's initial events (Simulator::Stop: rank 0)
    size_t k = 0;
    for (size_t i = 0; i < its.size(); i++) {
      const bool mine = ictx[i] == NOCTX ? rank == 0 : owner[ictx[i]] == (uint32_t)rank;
      if (!mine) continue;
      its[k] = its[i], iuid[k] = iuid[i], ictx[k] = ictx[i], ikind[k] = ikind[i], ia[k] = ia[i];
      k++;
    }
    its.resize(k), iuid.resize(k), ictx.resize(k), ikind.resize(k), ia.resize(k);
  }
  P.n_init = (uint32_t)its.size();
  P.uid_init = uid;
  P.pool_cap = pool_cap ? pool_cap : std::max<uint64_t>(4ull * P.n_init + 65536, 1ull << 20);
  if (P.n_init > P.pool_cap) { return set_error(NSGPU_EINVAL, "pool_cap < setup events"); }
  if (owner) {
    {  // X2 capacity: the largest number of devices of one rank whose peer another rank owns
      std::vector<uint32_t> cut((size_t)nranks * nranks, 0);
      for (uint32_t d = 0; d < D; d++) {
        const uint32_t p = owner[sc->dev_node[d]], q = owner[sc->dev_node[sc->dev_peer[d]]];
        if (p != q) cut[(size_t)p * nranks + q]++;
      }
      uint32_t mx = 1;
      for (uint32_t c : cut) mx = std::max(mx, c);
      if (P.wide) mx *= 3;  // (wide: a device's gen-0 TransmitStart and up to two local ones, chain depth <= 2)
      P.capx = std::min<uint32_t>((mx + 15) / 16 * 16, CAPX_MAX);
      P.x2b = sizeof(X2Hdr) + sizeof(Ev) * (uint64_t)P.capx;
    }
  }
  return NSGPU_OK;
}

// owner == null: the whole scenario on this device; otherwise the partition `rank` of `nranks`
// (node n belongs to rank owner[n]).
static int create_engine(const nsgpu_p2p_scenario *sc, const uint32_t *owner, int rank, int nranks,
                         nsgpu_comm *comm, uint64_t pool_cap, uint64_t log_cap, nsgpu_p2p **out) {
  if (!out) return set_error(NSGPU_EINVAL, "nsgpu_p2p_create: null");
  *out = nullptr;
  EnginePlan P;
  if (int rcp = plan_engine(sc, owner, rank, nranks, pool_cap, P)) return rcp;
  const uint32_t N = sc->n_nodes, D = sc->n_devices, A = sc->n_apps;
  const uint32_t qcap = P.qcap;
  const std::vector<uint32_t> &napps = P.napps, &node_list = P.node_list;
  const std::vector<int32_t> &sink = P.sink;
  nsgpu_p2p *h = new nsgpu_p2p();
  h->sc = *sc;
  h->app_kind.assign(sc->app_kind, sc->app_kind + A);
  h->n_apps = A;
  P2PDev &M = h->M;
  memset(&M, 0, sizeof(M));
  M.n_nodes = N;
  M.n_devices = D;
  M.n_apps = A;
  M.n_dst = sc->n_dst;
  M.qcap = qcap;
  M.maxc = P.maxc;
  for (int k = 0; k < K_NKINDS; k++) M.lookahead[k] = P.lookahead[k], M.lookw[k] = P.lookw[k];
  M.wide = P.wide;
  // ---- scenario upload ----
  TRY(dupload(h, &M.dev_node, sc->dev_node, D));
  if (sc->route) {
    TRY(dupload(h, &M.route, sc->route, (size_t)N * sc->n_dst));
  } else {
    const uint64_t ne = sc->route_exc_off[N];
    TRY(dupload(h, &M.route_def, sc->route_default, N));
    TRY(dupload(h, &M.route_exc_off, sc->route_exc_off, N + 1));
    TRY(dupload(h, &M.route_exc_slot, sc->route_exc_slot, ne));
    TRY(dupload(h, &M.route_exc_dev, sc->route_exc_dev, ne));
  }
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
  {
    std::vector<uint32_t> cnt(A, 0), src(A, 0);
    std::vector<int64_t> ivl(A, 0);
    for (uint32_t a = 0; a < A; a++) {
      src[a] = sc->app_src_slot ? sc->app_src_slot[a] : 0xffffffffu;
      if (sc->app_kind[a] == NSGPU_APP_ECHO_CLIENT) {
        cnt[a] = sc->app_count[a];
        ivl[a] = sc->app_interval_ns[a];
      }
    }
    TRY(dupload(h, &M.app_count, cnt.data(), A));
    TRY(dupload(h, &M.app_interval, ivl.data(), A));
    TRY(dupload(h, &M.app_src_slot, src.data(), A));
  }
  TRY(dupload(h, &M.node_app_off, napps.data(), N + 1));
  TRY(dupload(h, &M.node_app_list, node_list.data(), A));
  const int32_t *sinkp;
  TRY(dupload(h, &sinkp, sink.data(), N));
  M.sink_of_node = sinkp;
  M.icmp = sc->icmp ? 1u : 0u;
  M.trace_kinds = 0xfu;
  // ---- state ----
  {  // the device records' reset image: tx state idle, the static parameters
    std::vector<DevRec> dr(D);
    for (uint32_t d = 0; d < D; d++) {
      DevRec r{};
      r.qmax = sc->dev_qmax[d];
      r.peer = sc->dev_peer[d];
      r.peer_node = sc->dev_node[sc->dev_peer[d]];
      r.rkind = K_RECEIVE | ((owner && owner[r.peer_node] != (uint32_t)rank) ? REMOTEBIT : 0u);
      r.bps = sc->dev_bps[d];
      r.ifg = sc->dev_ifg_ns[d];
      r.delay = sc->dev_delay_ns[d];
      dr[d] = r;
    }
    const DevRec *init;
    TRY(dupload(h, &init, dr.data(), D));
    h->dev_init = init;
    TRY(dalloc(h, &M.dev, D));
  }
  TRY(dalloc(h, &M.q_buf, (size_t)D * qcap));
  TRY(dalloc(h, &M.app_flags, A));
  TRY(dalloc(h, &M.app_send_gen, A));
  TRY(dalloc(h, &M.app_ss_gen, A));
  TRY(dalloc(h, &M.app_residual, A));
  TRY(dalloc(h, &M.app_tot, A));
  TRY(dalloc(h, &M.node_ipid, N));
  TRY(dalloc(h, &M.app_last_start, A));
  TRY(dalloc(h, &M.appc, A));
  TRY(dalloc(h, &M.node_tab, (size_t)N * NTAB));
  const std::vector<uint64_t> &its = P.its;
  const std::vector<uint32_t> &iuid = P.iuid, &ictx = P.ictx, &ikind = P.ikind, &ia = P.ia;
  const uint32_t uid = P.uid_init;
  const Red red0 = P.red0;
  M.n_init = P.n_init;
  M.uid_init = P.uid_init;
  M.pool_cap = P.pool_cap;
  for (int b = 0; b < 2; b++) {
    TRY(dalloc(h, &M.ev_ts[b], M.pool_cap));
    TRY(dalloc(h, &M.ev_uid[b], M.pool_cap));
    TRY(dalloc(h, &M.ev_ctx[b], M.pool_cap));
    TRY(dalloc(h, &M.ev_kind[b], M.pool_cap));
    TRY(dalloc(h, &M.ev_a[b], M.pool_cap));
    TRY(dalloc(h, &M.ev_pkt[b], M.pool_cap));
  }
  const size_t chn = (size_t)WTOT * M.maxc;  // children of gen-0 and local records
  TRY(dalloc(h, &M.ch_ts, chn));
  TRY(dalloc(h, &M.ch_ctx, chn));
  TRY(dalloc(h, &M.ch_kind, chn));
  TRY(dalloc(h, &M.ch_a, chn));
  TRY(dalloc(h, &M.ch_pkt, chn));
  // window records: a whole sorted run (single engine), a whole window before its cut (partitioned)
  M.fcap = (size_t)NMAX * M.maxc;  // children parked in one window: at most every record's
  M.runcap = M.pool_cap + M.fcap;
  if (M.runcap >= 0xffffffffull) {
    nsgpu_p2p_destroy(h);
    return set_error(NSGPU_EINVAL, "nsgpu_p2p_create: pool_cap too large for 32-bit slots");
  }
  TRY(dalloc(h, &M.wkey, M.runcap));
  TRY(dalloc(h, &M.wpkt, M.runcap));
  for (uint32_t **p : {&M.wctx, &M.wkind, &M.wa}) TRY(dalloc(h, p, M.runcap));
  TRY(dalloc(h, &M.pwkey, WTOT));
  TRY(dalloc(h, &M.sinfo, WTOT));
  TRY(dalloc(h, &M.widx, WCAP));
  for (uint32_t **p : {&M.nchild, &M.ninl, &M.pwctx, &M.wpar}) TRY(dalloc(h, p, WTOT));
  TRY(dalloc(h, &M.wrank, 2 * (size_t)WTOT));  // (by window parity)
  TRY(dalloc(h, &M.lcnt, NLR));
  TRY(dalloc(h, &M.lrec, NMAX));  // (k2_pa loads lrec[k] speculatively: zeroed, every entry stays < WTOT)
  TRY(dalloc(h, &M.lkey, LCAP));
  TRY(dalloc(h, &M.lkw, LCAP));
  TRY(dalloc(h, &M.ldat, LMAX));
  TRY(dalloc(h, &M.lrank, 2 * (size_t)LMAX));
  // deferred windows (single wide engine): staged records, their leaves, child prefixes, dense map
  if (M.wide) {
    TRY(dalloc(h, &M.stage, NMAX));
    TRY(dalloc(h, &M.sleaf, (size_t)NMAX * M.maxc));
    TRY(dalloc(h, &M.stx, NMAX));
    TRY(dalloc(h, &M.cpt, 2 * (size_t)NMAX));
    TRY(dalloc(h, &M.ldpd, LMAX));
    const char *e = getenv("NSGPU_P2P_SDEF_KERNEL");  // (diagnostic: the accounting as its own kernel)
    M.sdef_fold = (e && e[0] == '1') ? 0u : 1u;
  }
  // (k2_pa loads lrec / ldat entries speculatively and follows their record index: zeroed, every entry
  // stays < WTOT; the deferred pipeline's arrays start zeroed too, so a stale entry is always in range)
  bool zok = hipMemset(M.lrec, 0, NMAX * sizeof(uint32_t)) == hipSuccess &&
             hipMemset(M.lcnt, 0, NLR * sizeof(uint32_t)) == hipSuccess &&
             hipMemset(M.ldat, 0, LMAX * sizeof(uint4)) == hipSuccess;
  if (zok && M.wide)
    zok = hipMemset(M.stage, 0, (size_t)NMAX * sizeof(Stg)) == hipSuccess &&
          hipMemset(M.sleaf, 0, (size_t)NMAX * M.maxc * sizeof(uint2)) == hipSuccess &&
          hipMemset(M.stx, 0, (size_t)NMAX * sizeof(uint32_t)) == hipSuccess &&
          hipMemset(M.cpt, 0, 2 * (size_t)NMAX * sizeof(uint32_t)) == hipSuccess &&
          hipMemset(M.ldpd, 0, (size_t)LMAX * sizeof(uint32_t)) == hipSuccess;
  if (!zok) {
    nsgpu_p2p_destroy(h);
    return set_error(NSGPU_EHIP, "nsgpu_p2p_create: hipMemset failed");
  }
  // in-place pool, fresh buffer, free stack, hub blocks, compaction; radix sort scratch (single engine)
  TRY(dalloc(h, &M.wsrc, M.runcap));
  TRY(dalloc(h, &M.f_ts, M.fcap));
  for (uint32_t **p : {&M.f_uid, &M.f_ctx, &M.f_kind, &M.f_a}) TRY(dalloc(h, p, M.fcap));
  TRY(dalloc(h, &M.f_pkt, M.fcap));
  TRY(dalloc(h, &M.fstack, M.pool_cap));
  TRY(dalloc(h, &M.hub_list, MAXHUB));
  TRY(dalloc(h, &M.hx, WCAP));
  TRY(dalloc(h, &M.hub_key, (size_t)NHUB * WCAP));
  TRY(dalloc(h, &M.hub_slot, (size_t)(NHUB + 1) * WCAP));  // (+ hub_mark's WCAP)
  TRY(dalloc(h, &M.cmp_cnt, 1));
  {  // radix sort scratch: the single engine's sorted runs, a partitioned rank's run (sorted once per run)
    TRY(dalloc(h, &M.s_key2, M.runcap));
    for (uint32_t **p : {&M.s_val, &M.s_val2}) TRY(dalloc(h, p, M.runcap));
    TRY(dalloc(h, &M.s_hist, 256 * ((M.runcap + RS_TILE - 1) / RS_TILE)));
    if (!owner) {  // (the single engine gathers in place through these; a partitioned rank into rn_*)
      TRY(dalloc(h, &M.g_u32, M.runcap));
      TRY(dalloc(h, &M.g_pkt, M.runcap));
    }
  }
  if (owner) {
    TRY(dalloc(h, &M.rn_key, M.runcap));
    for (uint32_t **p : {&M.rn_ctx, &M.rn_kind, &M.rn_a, &M.rn_src}) TRY(dalloc(h, p, M.runcap));
    TRY(dalloc(h, &M.rn_pkt, M.runcap));
    M.dist = 1;
    M.rank = (uint32_t)rank;
    M.nranks = (uint32_t)nranks;
    TRY(dupload(h, &M.owner, owner, N));
    TRY(dalloc(h, &M.x0_recv, 2 * (size_t)nranks));
    TRY(dalloc(h, &M.xk_send, 2));
    TRY(dalloc(h, &M.xk_recv, 2 * (size_t)nranks));
    TRY(dalloc(h, &M.x1_recv, X1B * nranks));
    TRY(dalloc(h, &M.x1_own, X1OWN));
    M.x1_send = M.x1_recv + (size_t)rank * X1B;  // (in place: NCCL moves only the other ranks' slots)
    if ((uint64_t)nranks * WCAP * M.maxc >= (1ull << 32))  // (k_gtile's packed child prefix)
      return set_error(NSGPU_EINVAL, "nsgpu_p2p_create_dist: %d ranks x %u children per event", nranks, M.maxc);
    M.capx = P.capx;
    M.x2b = P.x2b;
    TRY(dalloc(h, &M.x2_send, M.x2b * nranks));
    TRY(dalloc(h, &M.x2_recv, M.x2b * nranks));
    TRY(dalloc(h, &M.gacc, 4 * (size_t)NACC));
    h->comm = comm;
    memset(&h->x1h0, 0, sizeof(X1Hdr));
    h->x1h0.red.tmin = h->x1h0.red.wend = h->x1h0.red.stopts = h->x1h0.red.wendw = ~0ull;
    h->x1h0.rkey = ~0ull;
  }
  TRY(dalloc(h, &M.C, 1));
  if (owner) M.x0_send = reinterpret_cast<uint64_t *>(&M.C->W);  // X0 sends (W, nxtP, overflow, prep)
  if (owner && nranks == 1) {  // one rank: its exchanges are its own payloads in place (no copies in the window)
    M.x0_recv = M.x0_send;
    M.x2_recv = M.x2_send;  // (with one rank no child is remote: X2 stays empty)
  }
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
  C0.uid = uid;
  // reduction of the initial pool: window 0 is bounded by red[1] (k2_pa / k2_handle fold later
  // pending sets in for the next windows)
  C0.red[0].tmin = C0.red[0].wend = C0.red[0].stopts = C0.red[0].wendw = ~0ull;
  C0.red[0].stopuid = 0;
  C0.red[1] = red0;
  C0.max_windows = h->max_windows;
  C0.done = red0.tmin == ~0ull ? 2 : 0;  // (no event anywhere)
  C0.P_end = C0.live = M.n_init;  // single engine: the in-place pool starts as the setup events
  C0.hts = ~0ull;                 // no host closure pending (nsgpu_p2p_advance sets one)
  C0.hrel = ~0ull;
  C0.rt = 0;                      // window 0 is bounded by red[1] and folds into red[0]
  C0.span_t = ~0ull >> 2;         // wide windows start at their widest (adapted to the capacity)
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
  if (hipHostMalloc((void **)&h->snap, 2 * sizeof(Ctl), hipHostMallocDefault) != hipSuccess) {
    h->snap = nullptr;
    nsgpu_p2p_destroy(h);
    return set_error(NSGPU_ENOMEM, "nsgpu_p2p_create: hipHostMalloc failed");
  }
  if (hipHostMalloc((void **)&h->done_host, 2 * sizeof(uint32_t), hipHostMallocDefault) != hipSuccess) {
    h->done_host = nullptr;
    nsgpu_p2p_destroy(h);
    return set_error(NSGPU_ENOMEM, "nsgpu_p2p_create: hipHostMalloc failed");
  }
  *out = h;
  return NSGPU_OK;
}

extern "C" int nsgpu_p2p_create(const nsgpu_p2p_scenario *sc, uint64_t pool_cap, uint64_t log_cap,
                                nsgpu_p2p **out) {
  return create_engine(sc, nullptr, 0, 1, nullptr, pool_cap, log_cap, out);
}

extern "C" int nsgpu_p2p_create_dist(const nsgpu_p2p_scenario *sc, const uint32_t *node_owner, int rank,
                                     int nranks, nsgpu_comm *comm, uint64_t pool_cap, uint64_t log_cap,
                                     nsgpu_p2p **out) {
  if (!node_owner) return set_error(NSGPU_EINVAL, "nsgpu_p2p_create_dist: null owner map");
  if (comm && (comm->nranks != nranks || comm->rank != rank))
    return set_error(NSGPU_EINVAL, "nsgpu_p2p_create_dist: communicator is rank %d of %d", comm->rank, comm->nranks);
  return create_engine(sc, node_owner, rank, nranks, comm, pool_cap, log_cap, out);
}

extern "C" int nsgpu_p2p_dist_plan(const nsgpu_p2p_scenario *sc, const uint32_t *node_owner, int rank, int nranks,
                                   uint64_t pool_cap, nsgpu_p2p_plan *out) {
  if (!sc || !out) return set_error(NSGPU_EINVAL, "nsgpu_p2p_dist_plan: null");
  static_assert(K_NKINDS <= 16, "nsgpu_p2p_plan holds 16 kinds");
  EnginePlan P;
  if (int rc = plan_engine(sc, node_owner, rank, nranks, pool_cap, P)) return rc;
  memset(out, 0, sizeof(*out));
  out->wide = P.wide;
  out->maxc = P.maxc;
  out->wcap = WCAP;
  out->xlcap = XLCAP;
  if (node_owner) {
    out->x0_bytes = X0B;
    out->x1_bytes = X1B;
    out->x2_bytes = P.x2b;
    out->x2_records = P.capx;
  }
  out->n_kinds = K_NKINDS;
  for (int k = 0; k < K_NKINDS; k++) out->lookahead[k] = P.lookahead[k], out->lookw[k] = P.lookw[k];
  out->tx_min = P.tx_min;
  out->lx = P.lx;
  out->red0_tmin = P.red0.tmin;
  out->red0_wend = P.red0.wend;
  out->red0_wendw = P.red0.wendw;
  out->stop_ts = P.red0.stopts;
  out->stop_uid = P.red0.stopuid;
  out->uid_init = P.uid_init;
  out->n_init = P.n_init;
  out->pool_cap = P.pool_cap;
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
  NSGPU_HIP(hipMemcpyAsync(M.dev, h->dev_init, D * sizeof(DevRec), hipMemcpyDeviceToDevice, s));
  NSGPU_HIP(hipMemsetAsync(M.app_flags, 0, A * sizeof(uint32_t), s));
  NSGPU_HIP(hipMemsetAsync(M.app_send_gen, 0, A * sizeof(uint32_t), s));
  NSGPU_HIP(hipMemsetAsync(M.app_ss_gen, 0, A * sizeof(uint32_t), s));
  NSGPU_HIP(hipMemsetAsync(M.app_residual, 0, A * sizeof(uint32_t), s));
  NSGPU_HIP(hipMemsetAsync(M.app_tot, 0, A * sizeof(uint32_t), s));
  NSGPU_HIP(hipMemsetAsync(M.node_ipid, 0, M.n_nodes * sizeof(uint32_t), s));
  if (M.trace) NSGPU_HIP(hipMemsetAsync(M.trace_n, 0, sizeof(unsigned long long), s));
  NSGPU_HIP(hipMemsetAsync(M.app_last_start, 0, A * sizeof(uint64_t), s));
  NSGPU_HIP(hipMemsetAsync(M.appc, 0, A * sizeof(nsgpu_app_counters), s));
  NSGPU_HIP(hipMemsetAsync(M.node_tab, 0, (size_t)M.n_nodes * NTAB * sizeof(uint32_t), s));
  NSGPU_HIP(hipMemsetAsync(M.wrank, 0, 2 * WTOT * sizeof(uint32_t), s));
  NSGPU_HIP(hipMemsetAsync(M.lrank, 0, 2 * LMAX * sizeof(uint32_t), s));
  NSGPU_HIP(hipMemsetAsync(M.lcnt, 0, NLR * sizeof(uint32_t), s));
  NSGPU_HIP(hipMemsetAsync(M.error, 0, 4 * sizeof(uint32_t), s));
  if (M.dist) {
    const size_t R = M.nranks;
    if (M.x0_recv != M.x0_send) NSGPU_HIP(hipMemsetAsync(M.x0_recv, 0, X0B * R, s));
    NSGPU_HIP(hipMemsetAsync(M.xk_send, 0, 16, s));
    NSGPU_HIP(hipMemsetAsync(M.xk_recv, 0, 16 * R, s));
    NSGPU_HIP(hipMemsetAsync(M.x1_recv, 0, X1B * R, s));
    NSGPU_HIP(hipMemsetAsync(M.x1_own, 0, X1OWN, s));
    NSGPU_HIP(hipMemcpyAsync(M.x1_send, &h->x1h0, sizeof(X1Hdr), hipMemcpyHostToDevice, s));  // (its own slot)
    NSGPU_HIP(hipMemsetAsync(M.x2_send, 0, M.x2b * R, s));
    if (M.x2_recv != M.x2_send) NSGPU_HIP(hipMemsetAsync(M.x2_recv, 0, M.x2b * R, s));
    NSGPU_HIP(hipMemsetAsync(M.gacc, 0, 4 * NACC * sizeof(uint32_t), s));
  }
  if (M.log_cap) {  // (partitioned: every rank writes only the entries it dispatches, the union is the log;
                    //  mixed runs: the ranks of host dispatches stay unwritten)
    NSGPU_HIP(hipMemsetAsync(M.log_ts, 0, M.log_cap * 8, s));
    NSGPU_HIP(hipMemsetAsync(M.log_uid, 0, M.log_cap * 4, s));
    NSGPU_HIP(hipMemsetAsync(M.log_ctx, 0, M.log_cap * 4, s));
  }
  NSGPU_HIP(hipMemcpyAsync(M.C, &h->C0, sizeof(Ctl), hipMemcpyHostToDevice, s));
  h->uid_hint = h->C0.uid;
  return NSGPU_OK;
}

// The window pipeline, in launch order (graph capture, eager runs and the per-kernel profile).
namespace {
constexpr int NKERN = 6;
const char *const KERNEL_NAMES[NKERN] = {"k2_pa", "k2_handle", "k2_rank", "k2_scan", "k_tpatch", "k2_sdef"};
// ev0 / ev1: optional HIP events the command processor records at the kernel's start and end
// (hipExtLaunchKernelGGL: no separate marker packets between the pipeline's kernels).
// Kernel k of the single engine's window (KERNEL_NAMES); a wide engine places its local records after
// its handlers (k2_rank) and, traced, patches their trace uids (k_tpatch).  Returns
// whether kernel k is part of this engine's window.
// (NSGPU_P2P_PLAIN_LAUNCH=1, diagnostic: plain launches instead of hipExtLaunchKernelGGL where no events are asked)
bool plain_launch() {
  static const bool p = [] {
    const char *e = getenv("NSGPU_P2P_PLAIN_LAUNCH");
    return e && e[0] == '1';
  }();
  return p;
}
#define NSGPU_KLAUNCH(K, G, B, S, E0, E1, ...)                         \
  do {                                                                \
    if (plain_launch() && !(E0)) hipLaunchKernelGGL(K, G, B, 0, S, __VA_ARGS__); \
    else hipExtLaunchKernelGGL(K, G, B, 0, S, E0, E1, 0, __VA_ARGS__);  \
  } while (0)
bool launch_kernel(nsgpu_p2p *h, int k, hipStream_t s, bool df, hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr) {
  const bool wide = h->M.wide != 0;
  switch (k) {
    case 0:
      if (df) NSGPU_KLAUNCH((k2_pa<false, true, true>), dim3(pa_grid_rt<true>(h->M)), dim3(TB), s, ev0, ev1, h->M);
      else if (wide) NSGPU_KLAUNCH((k2_pa<false, true>), dim3(pa_grid_rt<true>(h->M)), dim3(TB), s, ev0, ev1, h->M);
      else NSGPU_KLAUNCH((k2_pa<false, false>), dim3(pa_grid_rt<false>(h->M)), dim3(TB), s, ev0, ev1, h->M);
      return true;
    case 1:
      if (wide) NSGPU_KLAUNCH(k2_handle<true>, dim3(K2_GRID), dim3(HB), s, ev0, ev1, h->M);
      else NSGPU_KLAUNCH(k2_handle<false>, dim3(K2_GRID), dim3(HB), s, ev0, ev1, h->M);
      return true;
    case 2:
      if (!wide) return false;
      if (df) NSGPU_KLAUNCH(k2_rank<true>, dim3(RK_GRID_DF), dim3(RKT_DF), s, ev0, ev1, h->M);
      else NSGPU_KLAUNCH(k2_rank<false>, dim3(RK_GRID), dim3(RKT), s, ev0, ev1, h->M);
      return true;
    case 3:
      if (df) return false;  // (the deferred pipeline: df_book in k2_rank, the accounting in k2_sdef)
      if (wide) NSGPU_KLAUNCH(k2_scan<true>, dim3(1), dim3(SCAN_THREADS), s, ev0, ev1, h->M);
      else NSGPU_KLAUNCH(k2_scan<false>, dim3(1), dim3(SCAN_THREADS), s, ev0, ev1, h->M);
      return true;
    case 4:
      if (!(wide && h->M.trace)) return false;
      NSGPU_KLAUNCH(k_tpatch, dim3(64), dim3(256), s, ev0, ev1, h->M);
      return true;
    default:  // k2_sdef(n) after k2_rank(n + 1): window n was staged by k2_pa(n + 1) (folded: k2_rank's blocks 1 .. NSDEF)
      if (!df || h->M.sdef_fold) return false;
      NSGPU_KLAUNCH(k2_sdef, dim3(NSDEF), dim3(SCAN_THREADS), s, ev0, ev1, h->M);
      return true;
  }
}
// Diagnostic mode (eager launches with NSGPU_P2P_DEBUG=1): after every kernel the stream is drained (a
// fault is reported with the kernel and window that raised it) and k_dbg checks the engine's invariants
// (pool, free stack, fresh buffer, window records, children), so that a broken state is reported by the
// kernel that made it instead of faulting a later one.
// In graph mode (NSGPU_P2P_DEBUG=2) k_dbg runs after every kernel of the replay (`at`: window << 8 | kernel)
// and a broken invariant also ends the run (done = 2, error 1024) so that the next kernels do nothing.
__global__ __launch_bounds__(256) void k_dbg(const P2PDev M, unsigned long long *out, unsigned long long at = 0) {
  Ctl &C = *M.C;
  const uint64_t i0 = (uint64_t)blockIdx.x * 256 + threadIdx.x, st = (uint64_t)gridDim.x * 256;
  if (at && out[0]) return;  // (graph mode: the first violation is kept)
  auto bad = [&](unsigned long long code, unsigned long long a, unsigned long long b) {
    if (atomicCAS(&out[0], 0ull, code) == 0ull) {
      out[1] = a;
      out[2] = b;
      out[3] = at | ((unsigned long long)C.windows << 32);
      if (at) {
        atomicOr(M.error, 1024u);
        C.done = 2;
      }
    }
  };
  const uint64_t Pe = C.P_end, nfree = C.nfree, nF = C.nF, W = C.W;
  if (i0 == 0) {
    if (Pe > M.pool_cap) bad(1, Pe, M.pool_cap);
    if (nfree + C.npush > M.pool_cap) bad(2, nfree, C.npush);
    if (C.live > Pe + nF) bad(3, C.live, Pe);
    if (nF > M.fcap) bad(4, nF, M.fcap);
    if (W > M.runcap) bad(5, W, M.runcap);
  }
  const uint64_t P = Pe < M.pool_cap ? Pe : M.pool_cap;
  for (uint64_t p = i0; p < P; p += st)
    if (M.ev_ts[0][p] != TOMB && ((M.ev_ctx[0][p] >= M.n_nodes && M.ev_ctx[0][p] != ~0u) ||
                                  (M.ev_kind[0][p] & 0xffu) >= (uint32_t)K_NKINDS))
      bad(10, p, M.ev_ctx[0][p]);
  const uint64_t F = nF < M.fcap ? nF : M.fcap;
  for (uint64_t f = i0; f < F; f += st)
    if (M.f_ctx[f] >= M.n_nodes && M.f_ctx[f] != ~0u) bad(30, f, M.f_ctx[f]);
  const uint64_t NF = nfree < M.pool_cap ? nfree : M.pool_cap;
  for (uint64_t j = i0; j < NF; j += st)
    if (M.fstack[j] >= P) bad(40, j, M.fstack[j]);
  const uint64_t Wm = W < (uint64_t)WCAP ? W : (uint64_t)WCAP;
  if (C.mode != MODE_RUN)
    for (uint64_t s = i0; s < Wm; s += st) {
      if (M.wctx[s] >= M.n_nodes && M.wctx[s] != ~0u) bad(20, s, M.wctx[s]);
      if (M.nchild[s] > M.maxc) bad(21, s, M.nchild[s]);
    }
}
unsigned long long *g_dbg_out = nullptr;
int dbg_alloc() {  // (before any capture)
  if (!g_dbg_out) {
    NSGPU_HIP(hipMalloc(&g_dbg_out, 4 * sizeof(unsigned long long)));
    NSGPU_HIP(hipMemset(g_dbg_out, 0, 4 * sizeof(unsigned long long)));
  }
  return NSGPU_OK;
}
int launch_windows_dbg(nsgpu_p2p *h, hipStream_t s, bool df) {
  if (const int rd = dbg_alloc()) return rd;
  unsigned long long *dout = g_dbg_out;
  if (!h->eager) {  // graph capture: checks as graph nodes
    for (int w = 0; w < NWIN; w++)
      for (int k = 0; k < NKERN; k++)
        if (launch_kernel(h, k, s, df)) hipLaunchKernelGGL(k_dbg, dim3(256), dim3(256), 0, s, h->M, dout, (unsigned long long)(w << 8 | k | 0x80000000u));
    return NSGPU_OK;
  }
  static int lines = 0;
  static const bool trace_c = getenv("NSGPU_P2P_DEBUG_TRACE") != nullptr;
  for (int w = 0; w < NWIN; w++) {
    Ctl c{};
    NSGPU_HIP(hipMemcpyAsync(&c, h->M.C, sizeof(Ctl), hipMemcpyDeviceToHost, s));
    NSGPU_HIP(hipStreamSynchronize(s));
    if (trace_c && (lines < 400 || c.windows % 10000 == 0) && lines < 2000) {
      lines++;
      fprintf(stderr, "[p2p dbg] df %d win %llu mode %u done %u live %llu P_end %llu nfree %llu pvalid %u pchild %llu "
              "hts %llu hcap %u tmin %llu W %u K %llu uid %u stop %u\n", (int)df, (unsigned long long)c.windows, c.mode,
              c.done, (unsigned long long)c.live, (unsigned long long)c.P_end, (unsigned long long)c.nfree, c.pvalid,
              (unsigned long long)c.pchild, (unsigned long long)c.hts, c.hcap, (unsigned long long)c.tmin, c.W,
              (unsigned long long)c.K, c.uid, c.stop_seen);
    }
    for (int k = 0; k < NKERN; k++) {
      if (!launch_kernel(h, k, s, df)) continue;
      hipError_t e = hipStreamSynchronize(s);
      if (e != hipSuccess)
        return set_error(NSGPU_EHIP, "nsgpu_p2p debug: %s faulted in window %llu (df %d, mode %u): %s", KERNEL_NAMES[k],
                         (unsigned long long)c.windows, (int)df, c.mode, hipGetErrorString(e));
      NSGPU_HIP(hipMemsetAsync(dout, 0, 4 * sizeof(unsigned long long), s));
      hipLaunchKernelGGL(k_dbg, dim3(256), dim3(256), 0, s, h->M, dout);
      unsigned long long o[4] = {};
      NSGPU_HIP(hipMemcpyAsync(o, dout, sizeof(o), hipMemcpyDeviceToHost, s));
      NSGPU_HIP(hipStreamSynchronize(s));
      if (o[0])
        return set_error(NSGPU_EHIP, "nsgpu_p2p debug: invariant %llu broken after %s in window %llu (df %d, mode %u): "
                         "%llu %llu", o[0], KERNEL_NAMES[k], (unsigned long long)c.windows, (int)df, c.mode, o[1], o[2]);
    }
  }
  return NSGPU_OK;
}
int launch_windows(nsgpu_p2p *h, hipStream_t s, bool df, int nwin = NWIN) {
  static const int dbg = [] {
    const char *e = getenv("NSGPU_P2P_DEBUG");
    return e ? atoi(e) : 0;
  }();
  if ((dbg == 1 && h->eager) || (dbg == 2 && !h->eager)) return launch_windows_dbg(h, s, df);
  for (int w = 0; w < nwin; w++)
    for (int k = 0; k < NKERN; k++) launch_kernel(h, k, s, df);
  return NSGPU_OK;
}
// The deferred pipeline is used for untraced single wide engines (NSGPU_P2P_NODEFER=1: never).
bool df_usable(const nsgpu_p2p *h) {
  static const bool off = [] {
    const char *e = getenv("NSGPU_P2P_NODEFER");
    return e && e[0] == '1';
  }();
  return h->M.wide && !h->M.dist && !h->M.trace && h->M.maxc <= PROV_MAXC && h->M.n_nodes < (1u << 24) && !off;
}
// When the deferred pipeline paused itself (a sorted run, a compaction, a host closure) after window n's
// bookkeeping: window n's dispatch accounting from its records (k2_scan<true, true>: sinfo for the next
// k2_pa), and every provisional uid still pending resolved (k_xlate); the other pipeline can take over.
int df_flush(nsgpu_p2p *h, hipStream_t s) {
  hipLaunchKernelGGL((k2_scan<true, true>), dim3(1), dim3(SCAN_THREADS), 0, s, h->M);
  hipLaunchKernelGGL(k_xlate, dim3(1024), dim3(256), 0, s, h->M);
  NSGPU_HIP(hipGetLastError());
  return NSGPU_OK;
}
}  // namespace

// The host-driven steps of the single engine (rare; on the engine stream, after the pipeline has
// paused itself): the radix sort that turns an overflowing window into a sorted run, and the pool
// compaction.  `c` is the run control the pause left.
static int host_step(nsgpu_p2p *h, const Ctl &c, hipStream_t s) {
  const P2PDev &M = h->M;
  if (c.mode == MODE_SORT) {
    const uint64_t n = c.rW;
    NSGPU_HIP(hipMemsetAsync(M.cmp_cnt, 0, sizeof(uint64_t), s));
    hipLaunchKernelGGL(k_rs_or, dim3((uint32_t)std::min<uint64_t>((n + 255) / 256, 2048)), dim3(256), 0, s, M.wkey, n,
                       (unsigned long long *)M.cmp_cnt);
    uint64_t kor = 0;
    NSGPU_HIP(hipMemcpyAsync(&kor, M.cmp_cnt, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    NSGPU_HIP(hipStreamSynchronize(s));
    const int bits = kor ? 64 - __builtin_clzll(kor) : 1;
    const int passes = (bits + 7) / 8;
    const uint32_t ntiles = (uint32_t)((n + RS_TILE - 1) / RS_TILE);
    uint64_t *kin = M.wkey, *kout = M.s_key2;
    uint32_t *vin = nullptr, *vout = M.s_val;
    for (int p = 0; p < passes; p++) {
      hipLaunchKernelGGL(k_rs_hist, dim3(ntiles), dim3(RS_T), 0, s, kin, n, 8 * p, M.s_hist, ntiles);
      hipLaunchKernelGGL(k_rs_scan, dim3(1), dim3(1024), 0, s, M.s_hist, (uint64_t)256 * ntiles);
      hipLaunchKernelGGL(k_rs_scatter, dim3(ntiles), dim3(RS_T), 0, s, kin, vin, kout, vout, n, 8 * p, M.s_hist,
                         ntiles);
      std::swap(kin, kout);
      vin = vout;
      vout = vin == M.s_val ? M.s_val2 : M.s_val;
    }
    if (kin != M.wkey) NSGPU_HIP(hipMemcpyAsync(M.wkey, kin, n * sizeof(uint64_t), hipMemcpyDeviceToDevice, s));
    if (vin) {
      const uint32_t gg = (uint32_t)std::min<uint64_t>((n + 255) / 256, 8192);
      for (uint32_t *a : {M.wctx, M.wkind, M.wa}) {
        hipLaunchKernelGGL(k_rs_gather<uint32_t>, dim3(gg), dim3(256), 0, s, vin, a, M.g_u32, n);
        NSGPU_HIP(hipMemcpyAsync(a, M.g_u32, n * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
      }
      hipLaunchKernelGGL(k_rs_gather<Pkt>, dim3(gg), dim3(256), 0, s, vin, M.wpkt, M.g_pkt, n);
      NSGPU_HIP(hipMemcpyAsync(M.wpkt, M.g_pkt, n * sizeof(Pkt), hipMemcpyDeviceToDevice, s));
    }
    if (c.renarrow) hipLaunchKernelGGL(k_renarrow, dim3(1), dim3(1024), 0, s, M);  // (a widened window)
    hipLaunchKernelGGL(k_after_sort, dim3(1), dim3(1024), 0, s, M);
    NSGPU_HIP(hipGetLastError());
  } else if (c.mode == MODE_UIDX) {  // (the deferred pipeline handed over: nothing to do on the host)
    hipLaunchKernelGGL(k_after_uidx, dim3(1), dim3(1), 0, s, M);
    NSGPU_HIP(hipGetLastError());
  } else if (c.mode == MODE_TRIM) {  // a run ends after a cut same-ts group: the rest goes back to the pool
    hipLaunchKernelGGL(k_trim, dim3(1), dim3(1024), 0, s, M);
    NSGPU_HIP(hipGetLastError());
  } else if (c.mode == MODE_COMPACT) {
    NSGPU_HIP(hipMemsetAsync(M.cmp_cnt, 0, sizeof(uint64_t), s));
    hipLaunchKernelGGL(k_cmp, dim3(1024), dim3(256), 0, s, M, c.P_end);
    NSGPU_HIP(hipGetLastError());
    uint64_t live = 0;
    NSGPU_HIP(hipMemcpyAsync(&live, M.cmp_cnt, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    NSGPU_HIP(hipStreamSynchronize(s));
    if (live != c.live) return set_error(NSGPU_EHIP, "nsgpu_p2p: compaction found %llu live events, expected %llu",
                                          (unsigned long long)live, (unsigned long long)c.live);
    NSGPU_HIP(hipMemcpyAsync(M.ev_ts[0], M.ev_ts[1], live * 8, hipMemcpyDeviceToDevice, s));
    NSGPU_HIP(hipMemcpyAsync(M.ev_uid[0], M.ev_uid[1], live * 4, hipMemcpyDeviceToDevice, s));
    NSGPU_HIP(hipMemcpyAsync(M.ev_ctx[0], M.ev_ctx[1], live * 4, hipMemcpyDeviceToDevice, s));
    NSGPU_HIP(hipMemcpyAsync(M.ev_kind[0], M.ev_kind[1], live * 4, hipMemcpyDeviceToDevice, s));
    NSGPU_HIP(hipMemcpyAsync(M.ev_a[0], M.ev_a[1], live * 4, hipMemcpyDeviceToDevice, s));
    NSGPU_HIP(hipMemcpyAsync(M.ev_pkt[0], M.ev_pkt[1], live * sizeof(Pkt), hipMemcpyDeviceToDevice, s));
    hipLaunchKernelGGL(k_after_compact, dim3(1), dim3(1), 0, s, M, live);
    NSGPU_HIP(hipGetLastError());
  }
  return NSGPU_OK;
}

// The exchanges of a partitioned window.  A one-rank job has nothing to exchange: its "all-gather" and
// "all-to-all" are a device copy of its own slot (no RCCL call, so the window graph is all kernels and copies).
static int x_allgather(nsgpu_p2p *h, const void *send, void *recv, size_t bytes, hipStream_t s) {
  if (h->M.nranks == 1) {
    if (send != recv) NSGPU_HIP(hipMemcpyAsync(recv, send, bytes, hipMemcpyDeviceToDevice, s));
    return NSGPU_OK;
  }
  NCCL_TRY(ncclAllGather(send, recv, bytes, ncclUint8, h->comm->comm, s));
  return NSGPU_OK;
}
static int x_alltoall(nsgpu_p2p *h, const void *send, void *recv, size_t bytes, hipStream_t s) {
  if (h->M.nranks == 1) {
    if (send != recv && bytes) NSGPU_HIP(hipMemcpyAsync(recv, send, bytes, hipMemcpyDeviceToDevice, s));
    return NSGPU_OK;
  }
  NCCL_TRY(ncclAllToAll(send, recv, bytes, ncclUint8, h->comm->comm, s));
  return NSGPU_OK;
}

// The partitioned window's kernels (narrow, or wide: local records ranked across the ranks through X1Loc).
static void dist_pa(const P2PDev &M, hipStream_t s) {
  if (M.wide) hipLaunchKernelGGL((k2_pa<true, true>), dim3(GRID_POOL_DIST), dim3(TB), 0, s, M);
  else hipLaunchKernelGGL((k2_pa<true, false>), dim3(GRID_POOL_DIST), dim3(TB), 0, s, M);
}
static void dist_handle(const P2PDev &M, hipStream_t s) {
  if (M.wide) {
    hipLaunchKernelGGL((k2_handle<true, true>), dim3(K2_GRID_W), dim3(HB), 0, s, M);
    hipLaunchKernelGGL(k_xlcompact, dim3(NLR), dim3(HB), 0, s, M);
  }
  else hipLaunchKernelGGL(k2_handle<false>, dim3(K2_GRID), dim3(HB), 0, s, M);
}
// Before the X1 exchange: this rank's records ranked among themselves and, with more ranks, sorted into its X1.
static void dist_rank(const P2PDev &M, hipStream_t s) {
  if (M.wide) hipLaunchKernelGGL(k_gtile<true>, dim3(GTB), dim3(HB), 0, s, M);
  else hipLaunchKernelGGL(k_gtile<false>, dim3(GTB), dim3(HB), 0, s, M);
  if (M.nranks > 1) {
    if (M.wide) hipLaunchKernelGGL(k_gsort<true>, dim3(NACC / 256), dim3(256), 0, s, M);
    else hipLaunchKernelGGL(k_gsort<false>, dim3(NACC / 256), dim3(256), 0, s, M);
  }
}
// After it: the other ranks' records before each of this rank's (binary searches), then the window's books.
static void dist_rank_fin(const P2PDev &M, hipStream_t s) {
  if (M.nranks > 1) {
    const dim3 g(NACC / GS_T, M.nranks - 1);
    if (M.wide) hipLaunchKernelGGL(k_gsearch<true>, g, dim3(GS_T), 0, s, M);
    else hipLaunchKernelGGL(k_gsearch<false>, g, dim3(GS_T), 0, s, M);
  }
  if (M.wide) hipLaunchKernelGGL(k_dfin2<true>, dim3(DF2_FB + NACC / HB), dim3(HB), 0, s, M);
  else hipLaunchKernelGGL(k_dfin2<false>, dim3(DF2_FB + NHB), dim3(HB), 0, s, M);
}
// The partitioned window (one RCCL member): 4 kernels and 3 collectives, on stream s.
static int launch_windows_dist(nsgpu_p2p *h, hipStream_t s, int nwin = NWIN) {
  const P2PDev &M = h->M;
  int rc = NSGPU_OK;
  for (int w = 0; w < nwin && !rc; w++) {
    dist_pa(M, s);
    rc = x_allgather(h, M.x0_send, M.x0_recv, X0B, s);
    dist_handle(M, s);
    dist_rank(M, s);
    if (!rc) rc = x_allgather(h, M.x1_send, M.x1_recv, X1B, s);
    dist_rank_fin(M, s);
    if (!rc) rc = x_alltoall(h, M.x2_send, M.x2_recv, M.x2b, s);
  }
  return rc;
}

// The partitioned engine's host-driven steps (every rank makes the same ones: the pause that asks for them is
// decided from exchanged data): the pool compaction, and the start of a partitioned sorted run — a window some
// rank cannot hold (MODE_CUT): every rank sorts its candidates (drun_sort), the ranks' fitting keys are
// all-gathered (`gather`) and every rank moves the first chunk in (k_drun_first); the later chunks are formed
// by the window pipeline itself.
static int host_step(nsgpu_p2p *h, const Ctl &c, hipStream_t s);
static int drun_sort(nsgpu_p2p *h, uint64_t W, hipStream_t s) {
  const P2PDev &M = h->M;
  const uint64_t n = W < M.runcap ? W : M.runcap;
  hipLaunchKernelGGL(k_drun_clear, dim3(64), dim3(256), 0, s, M);
  if (n) {  // LSD radix sort of the keys (as host_step's MODE_SORT), the records gathered into rn_*
    NSGPU_HIP(hipMemsetAsync(M.cmp_cnt, 0, sizeof(uint64_t), s));
    hipLaunchKernelGGL(k_rs_or, dim3((uint32_t)std::min<uint64_t>((n + 255) / 256, 2048)), dim3(256), 0, s, M.wkey, n,
                       (unsigned long long *)M.cmp_cnt);
    uint64_t kor = 0;
    NSGPU_HIP(hipMemcpyAsync(&kor, M.cmp_cnt, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    NSGPU_HIP(hipStreamSynchronize(s));
    const int bits = kor ? 64 - __builtin_clzll(kor) : 1;
    const int passes = (bits + 7) / 8;
    const uint32_t ntiles = (uint32_t)((n + RS_TILE - 1) / RS_TILE);
    const uint64_t *kin = M.wkey;
    uint64_t *kout = (passes & 1) ? M.rn_key : M.s_key2;  // (alternating so that the last pass writes rn_key)
    uint32_t *vin = nullptr, *vout = M.s_val;
    for (int p = 0; p < passes; p++) {
      hipLaunchKernelGGL(k_rs_hist, dim3(ntiles), dim3(RS_T), 0, s, kin, n, 8 * p, M.s_hist, ntiles);
      hipLaunchKernelGGL(k_rs_scan, dim3(1), dim3(1024), 0, s, M.s_hist, (uint64_t)256 * ntiles);
      hipLaunchKernelGGL(k_rs_scatter, dim3(ntiles), dim3(RS_T), 0, s, kin, vin, kout, vout, n, 8 * p, M.s_hist,
                         ntiles);
      kin = kout;
      kout = kout == M.rn_key ? M.s_key2 : M.rn_key;
      vin = vout;
      vout = vin == M.s_val ? M.s_val2 : M.s_val;
    }
    const uint32_t gg = (uint32_t)std::min<uint64_t>((n + 255) / 256, 8192);
    hipLaunchKernelGGL(k_rs_gather<uint32_t>, dim3(gg), dim3(256), 0, s, vin, M.wctx, M.rn_ctx, n);
    hipLaunchKernelGGL(k_rs_gather<uint32_t>, dim3(gg), dim3(256), 0, s, vin, M.wkind, M.rn_kind, n);
    hipLaunchKernelGGL(k_rs_gather<uint32_t>, dim3(gg), dim3(256), 0, s, vin, M.wa, M.rn_a, n);
    hipLaunchKernelGGL(k_rs_gather<uint32_t>, dim3(gg), dim3(256), 0, s, vin, M.wsrc, M.rn_src, n);
    hipLaunchKernelGGL(k_rs_gather<Pkt>, dim3(gg), dim3(256), 0, s, vin, M.wpkt, M.rn_pkt, n);
  }
  if (n && M.wide) hipLaunchKernelGGL(k_drun_trim, dim3(1), dim3(1024), 0, s, M, n);
  hipLaunchKernelGGL(k_drun_start, dim3(1), dim3(1), 0, s, M, n);
  if (n) hipLaunchKernelGGL(k_drun_red, dim3((uint32_t)std::min<uint64_t>((n + 255) / 256, 1024)), dim3(256), 0, s, M, n);
  NSGPU_HIP(hipGetLastError());
  return NSGPU_OK;
}
template <class G>
static int host_step_dist(const Ctl &c, hipStream_t s, G gather, nsgpu_p2p *h) {
  if (c.mode != MODE_CUT) return host_step(h, c, s);
  int rc = drun_sort(h, c.W, s);
  if (!rc) rc = gather();
  if (rc) return rc;
  hipLaunchKernelGGL(k_drun_first, dim3(WCAP / TB), dim3(TB), 0, s, h->M);
  NSGPU_HIP(hipGetLastError());
  return NSGPU_OK;
}

static int build_graph(nsgpu_p2p *h, bool df = false, bool tail = false) {
  // NWIN windows of the pipeline (tail: NWIN_TAIL, single engine); kernels read every run-dependent value from the
  // device (Ctl), so one instantiated graph serves every run of this engine
  hipGraphExec_t &gx = tail ? h->gtail[df ? 1 : 0] : df ? h->gexec_df : h->gexec;
  hipGraph_t g = nullptr;
  if (const int rd = dbg_alloc()) return rd;
  NSGPU_HIP(hipStreamBeginCapture(h->s, h->M.dist ? hipStreamCaptureModeRelaxed : hipStreamCaptureModeThreadLocal));
  int rc = NSGPU_OK;
  if (h->M.dist) rc = launch_windows_dist(h, h->s);
  else launch_windows(h, h->s, df, tail ? NWIN_TAIL : NWIN);
  hipError_t e = hipStreamEndCapture(h->s, &g);
  if (rc != NSGPU_OK || e != hipSuccess) {
    if (g) (void)hipGraphDestroy(g);
    (void)hipGetLastError();
    if (rc != NSGPU_OK) return rc;
    return set_error(NSGPU_EHIP, "nsgpu_p2p: graph capture: %s", hipGetErrorString(e));
  }
  e = hipGraphInstantiate(&gx, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  if (e != hipSuccess) {
    gx = nullptr;
    return set_error(NSGPU_EHIP, "nsgpu_p2p: graph instantiate: %s", hipGetErrorString(e));
  }
  return NSGPU_OK;
}

// A run that set the engine's error word: capacity exceeded (the simulation is truncated).
static int engine_error(uint32_t err) {
  return set_error((err & 2048u) ? NSGPU_ERANGE : NSGPU_ENOMEM, "nsgpu_p2p: engine capacity exceeded (code %u: 1 = event pool, 4 = window limit, "
                                 "8 = window cut, 16 = a window's remote events beyond the X2 capacity, 32 = local "
                                 "records, 64 = window records, 256 = deferred uid resolution (internal), 512 = uids "
                                 "beyond the deferred pipeline's range (internal), 2048 = the uid counter would pass "
                                 "0xfffffffe: DefaultSimulatorImpl's uint32 m_uid wraps there, which the engine does "
                                 "not replicate)", err);
}

// The run control into a pinned snapshot after a replay: a copy-engine transfer (hipMemcpyAsync), or with
// NSGPU_P2P_SNAPK=1 one wave of k_snap on the same queue (no hand-over to the copy engine between replays).
static hipError_t snapshot(const Ctl *c, Ctl *out, hipStream_t s) {
  static const bool kern = [] {
    const char *e = getenv("NSGPU_P2P_SNAPK");
    return e && e[0] == '1';
  }();
  if (!kern) return hipMemcpyAsync(out, c, sizeof(Ctl), hipMemcpyDeviceToHost, s);
  hipLaunchKernelGGL(k_snap, dim3(1), dim3(64), 0, s, c, out);
  return hipGetLastError();
}

// Replays the single engine's window pipeline until the run is over (done >= 2) or the pipeline paused
// for a host closure (*paused).  Two replays in flight: replay i+1 is queued before the run control
// after replay i is examined; a pipeline that paused itself (host-driven sort or compaction, a host
// closure) makes the replay queued behind it a no-op, and the step runs once that replay has drained.
static int drive(nsgpu_p2p *h, bool *paused) {
  *paused = false;
  int cur = 0;
  bool have_prev = false;
  // the deferred pipeline while the engine runs normal windows; after a pause (which it flushes) the other
  // pipeline until a replay ends in a normal window
  const bool dfu = df_usable(h);
  bool df = dfu && h->uid_hint < UID_DF_SOFT;
  bool df_of[2] = {false, false};
  if (df && !h->eager && !h->gexec_df) {
    const int rc = build_graph(h, true);
    if (rc) return rc;
  }
  // The run's last windows in replays of NWIN_TAIL: a replay queued behind the final window is a no-op that still
  // launches its kernels (~1.5 x NWIN of them trail the run).  The tail starts once the examined snapshots' pace
  // (simulated ns a window) puts Simulator::Stop within the windows already queued plus one replay.  Speed only:
  // the windows are the same whatever a replay holds.
  const uint64_t stop_ts = h->C0.red[1].stopts;
  bool tail = false;
  uint64_t w_last = 0, t_last = 0;
  int queued = 0;  // windows of the replay in flight behind the examined one
  for (;;) {
    const int nw = tail ? NWIN_TAIL : NWIN;
    if (h->eager) {
      const int rc = launch_windows(h, h->s, df, nw);
      if (rc) return rc;
      NSGPU_HIP(hipGetLastError());
    } else {
      hipGraphExec_t gx = tail ? h->gtail[df ? 1 : 0] : df ? h->gexec_df : h->gexec;
      if (tail && !gx) {
        const int rc = build_graph(h, df, true);
        if (rc) return rc;
        gx = h->gtail[df ? 1 : 0];
      }
      NSGPU_HIP(hipGraphLaunch(gx, h->s));
    }
    queued = nw;
    df_of[cur] = df;
    NSGPU_HIP(snapshot(h->M.C, &h->snap[cur], h->s));
    NSGPU_HIP(hipEventRecord(h->ev[cur], h->s));
    if (have_prev) {
      NSGPU_HIP(hipEventSynchronize(h->ev[cur ^ 1]));
      const Ctl &c = h->snap[cur ^ 1];
      if (c.done >= 2) break;  // 2: the final window is appended
      if (!tail && stop_ts != ~0ull && c.mode == MODE_NORMAL && c.windows > w_last && c.tmin > t_last &&
          c.tmin != ~0ull && t_last != 0) {
        const double pace = (double)(c.tmin - t_last) / (double)(c.windows - w_last);
        const double left = stop_ts > c.tmin ? (double)(stop_ts - c.tmin) / pace : 0.0;
        if (left < (double)(queued + NWIN)) tail = true;
      }
      if (c.mode == MODE_NORMAL && c.tmin != ~0ull) w_last = c.windows, t_last = c.tmin;
      if (c.mode >= MODE_SORT) {
        NSGPU_HIP(hipEventSynchronize(h->ev[cur]));
        if (df_of[cur ^ 1]) {  // (the pause came from the deferred pipeline: its last window is not accounted yet)
          int rc = df_flush(h, h->s);
          if (!rc) {
            NSGPU_HIP(hipMemcpyAsync(&h->snap[cur], h->M.C, sizeof(Ctl), hipMemcpyDeviceToHost, h->s));
            NSGPU_HIP(hipStreamSynchronize(h->s));
          }
          if (rc) return rc;
        }
        df = false;
        if (h->snap[cur].mode == MODE_HOST) {
          *paused = true;
          break;
        }
        const int rc = host_step(h, h->snap[cur], h->s);
        if (rc) return rc;
        have_prev = false;
        continue;
      }
      if (!df && dfu && c.mode == MODE_NORMAL && c.uid < UID_DF_SOFT) {  // a normal window ended the replay: back
                                                                        // to the deferred pipeline
        // (not in a sorted run's chunks: those belong to the other pipeline until the run is over)
        if (!h->eager && !h->gexec_df) {
          const int rc = build_graph(h, true);
          if (rc) return rc;
        }
        df = true;
      }
    }
    have_prev = true;
    cur ^= 1;
  }
  NSGPU_HIP(hipStreamSynchronize(h->s));
  return NSGPU_OK;
}

// Replays the partitioned window pipeline until the run is over, as drive(): two replays in flight;
// a pause (a cut, a compaction: every rank pauses in the same window) runs its host step once the
// replay queued behind it has drained.
static int drive_dist(nsgpu_p2p *h) {
  int cur = 0;
  bool have_prev = false;
  auto gather = [h]() -> int { return x_allgather(h, h->M.xk_send, h->M.xk_recv, 16, h->s); };
  for (;;) {
    if (h->eager) {
      const int rc = launch_windows_dist(h, h->s);
      if (rc) return rc;
      NSGPU_HIP(hipGetLastError());
    } else {
      NSGPU_HIP(hipGraphLaunch(h->gexec, h->s));
    }
    NSGPU_HIP(hipMemcpyAsync(&h->snap[cur], h->M.C, sizeof(Ctl), hipMemcpyDeviceToHost, h->s));
    NSGPU_HIP(hipEventRecord(h->ev[cur], h->s));
    if (have_prev) {
      NSGPU_HIP(hipEventSynchronize(h->ev[cur ^ 1]));
      const Ctl &c = h->snap[cur ^ 1];
      if (c.done >= 2) break;  // 2: the final window is appended
      if (c.mode >= MODE_SORT) {
        NSGPU_HIP(hipEventSynchronize(h->ev[cur]));
        const int rc = host_step_dist(h->snap[cur], h->s, gather, h);
        if (rc) return rc;
        have_prev = false;
        continue;
      }
    }
    have_prev = true;
    cur ^= 1;
  }
  NSGPU_HIP(hipStreamSynchronize(h->s));
  return NSGPU_OK;
}

// ---- mixed host / device runs: the host-closure runtime (nsgpu_sim) drives the engine ----
uint32_t nsgpu::p2p_first_uid(const nsgpu_p2p *h) { return h->sc.uid_first ? h->sc.uid_first : 4u; }

extern "C" int nsgpu_p2p_setup_uid(nsgpu_p2p *h, uint32_t *uid) {
  if (!h || !uid) return set_error(NSGPU_EINVAL, "nsgpu_p2p_setup_uid: null");
  *uid = h->C0.uid;
  return NSGPU_OK;
}

extern "C" int nsgpu_p2p_advance(nsgpu_p2p *h, uint64_t hts, uint32_t huid, uint32_t *uid, uint64_t *dispatched,
                                 int *ended, void *stream) {
  if (!h || !uid || !dispatched || !ended) return set_error(NSGPU_EINVAL, "nsgpu_p2p_advance: null");
  if (h->M.dist) return set_error(NSGPU_ESTATE, "nsgpu_p2p_advance: single-device engines only");
  *ended = 0;
  if (!h->eager && !h->gexec) {
    const int rc = build_graph(h);
    if (rc) return rc;
  }
  hipStream_t cs = (hipStream_t)stream;
  NSGPU_HIP(hipEventRecord(h->ev[0], cs));
  NSGPU_HIP(hipStreamWaitEvent(h->s, h->ev[0], 0));
  uint32_t err0 = 0;
  NSGPU_HIP(hipMemcpyAsync(&h->snap[0], h->M.C, sizeof(Ctl), hipMemcpyDeviceToHost, h->s));
  NSGPU_HIP(hipMemcpyAsync(&err0, h->M.error, 4, hipMemcpyDeviceToHost, h->s));
  NSGPU_HIP(hipStreamSynchronize(h->s));
  if (err0) return engine_error(err0);  // (sticky: e.g. a refused inject_send at the uid limit)
  if (h->snap[0].done >= 2) {
    *ended = 1;
    return NSGPU_OK;
  }
  hipLaunchKernelGGL(k_host_resume, dim3(1), dim3(1), 0, h->s, h->M, hts, huid, *uid, *dispatched);
  NSGPU_HIP(hipGetLastError());
  h->uid_hint = *uid;
  bool paused = false;
  const int rc = drive(h, &paused);
  if (rc) return rc;
  uint32_t err = 0;
  NSGPU_HIP(hipMemcpyAsync(&h->snap[0], h->M.C, sizeof(Ctl), hipMemcpyDeviceToHost, h->s));
  NSGPU_HIP(hipMemcpyAsync(&err, h->M.error, 4, hipMemcpyDeviceToHost, h->s));
  NSGPU_HIP(hipStreamSynchronize(h->s));
  if (err) return engine_error(err);
  *uid = h->snap[0].uid;
  h->uid_hint = *uid;
  *dispatched = h->snap[0].K;
  *ended = paused ? 0 : 1;
  NSGPU_HIP(hipEventRecord(h->ev[0], h->s));
  NSGPU_HIP(hipStreamWaitEvent(cs, h->ev[0], 0));
  return NSGPU_OK;
}

// The attached engine's pending device events (Next / IsFinished of the runtime): how many, the
// smallest timestamp among them, and whether a device-dispatched Simulator::Stop ended the run.
extern "C" int nsgpu_p2p_pending(nsgpu_p2p *h, uint64_t *n, uint64_t *next_ts, int *stopped, void *stream) {
  if (!h || !n || !next_ts || !stopped) return set_error(NSGPU_EINVAL, "nsgpu_p2p_pending: null");
  if (h->M.dist) return set_error(NSGPU_ESTATE, "nsgpu_p2p_pending: single-device engines only");
  hipStream_t cs = (hipStream_t)stream;
  NSGPU_HIP(hipEventRecord(h->ev[0], cs));
  NSGPU_HIP(hipStreamWaitEvent(h->s, h->ev[0], 0));
  NSGPU_HIP(hipMemcpyAsync(&h->snap[0], h->M.C, sizeof(Ctl), hipMemcpyDeviceToHost, h->s));
  NSGPU_HIP(hipStreamSynchronize(h->s));
  const Ctl &c = h->snap[0];
  *stopped = c.stop_seen ? 1 : 0;
  if (c.done >= 1) {  // (1: the final window is dispatched, its children are not queued)
    *n = 0;
    *next_ts = ~0ull;
    return NSGPU_OK;
  }
  *n = c.live + (c.pvalid ? c.pchild : 0) + (c.mode == MODE_RUN ? c.rW - c.r0 : 0);
  *next_ts = c.red[0].tmin < c.red[1].tmin ? c.red[0].tmin : c.red[1].tmin;
  return NSGPU_OK;
}

extern "C" int nsgpu_p2p_inject_send(nsgpu_p2p *h, uint32_t app, uint64_t now, uint32_t cur_uid, uint32_t cur_ctx,
                                     uint32_t *uid, uint32_t *trace_seq, void *stream) {
  if (!h || !uid || !trace_seq) return set_error(NSGPU_EINVAL, "nsgpu_p2p_inject_send: null");
  if (h->M.dist) return set_error(NSGPU_ESTATE, "nsgpu_p2p_inject_send: single-device engines only");
  if (app >= h->M.n_apps || h->app_kind[app] != NSGPU_APP_ONOFF)
    return set_error(NSGPU_EINVAL, "nsgpu_p2p_inject_send: app %u is not an OnOff flow", app);
  hipStream_t s = h->s;
  hipStream_t cs = (hipStream_t)stream;
  NSGPU_HIP(hipEventRecord(h->ev[0], cs));
  NSGPU_HIP(hipStreamWaitEvent(s, h->ev[0], 0));
  NSGPU_HIP(hipMemcpyAsync(&h->snap[0], h->M.C, sizeof(Ctl), hipMemcpyDeviceToHost, s));
  NSGPU_HIP(hipStreamSynchronize(s));
  if (h->snap[0].mode != MODE_HOST) return set_error(NSGPU_ESTATE, "nsgpu_p2p_inject_send: the engine is not paused for a host closure");
  hipLaunchKernelGGL(k_set_uid, dim3(1), dim3(1), 0, s, h->M, *uid);  // (the host closures' Schedule calls)
  // (the room is checked on the device before any child is written: a refused send leaves the sticky uid error)
  if ((uint64_t)*uid > UID_MAX_NEXT) return nsgpu::uid_range_error("nsgpu_p2p_inject_send");
  hipLaunchKernelGGL(k_inject, dim3(1), dim3(1), 0, s, h->M, app, now, cur_uid, cur_ctx, *trace_seq,
                     (uint64_t)(UID_MAX_NEXT - *uid), h->M.s_val);
  NSGPU_HIP(hipGetLastError());
  uint32_t outv[3];
  NSGPU_HIP(hipMemcpyAsync(outv, h->M.s_val, sizeof(outv), hipMemcpyDeviceToHost, s));
  NSGPU_HIP(hipStreamSynchronize(s));
  if (outv[2]) return nsgpu::uid_range_error("nsgpu_p2p_inject_send");
  *uid = outv[0];
  *trace_seq = outv[1];
  return NSGPU_OK;
}

extern "C" int nsgpu_p2p_counters(nsgpu_p2p *h, nsgpu_dev_counters *devc, nsgpu_app_counters *appc, void *stream) {
  if (!h) return set_error(NSGPU_EINVAL, "nsgpu_p2p_counters: null");
  hipStream_t cs = (hipStream_t)stream;
  NSGPU_HIP(hipStreamSynchronize(h->s));
  if (devc)
    NSGPU_HIP(hipMemcpy2DAsync(devc, sizeof(*devc), &h->M.dev[0].c, sizeof(DevRec), sizeof(*devc), h->M.n_devices,
                               hipMemcpyDeviceToHost, cs));
  if (appc) NSGPU_HIP(hipMemcpyAsync(appc, h->M.appc, h->M.n_apps * sizeof(*appc), hipMemcpyDeviceToHost, cs));
  NSGPU_HIP(hipStreamSynchronize(cs));
  return NSGPU_OK;
}

extern "C" int nsgpu_p2p_run(nsgpu_p2p *h, void *stream) {
  if (!h) return set_error(NSGPU_EINVAL, "nsgpu_p2p_run: null");
  if (h->M.dist && !h->comm)
    return set_error(NSGPU_ESTATE, "nsgpu_p2p_run: a loopback partition runs with its group (nsgpu_p2p_group_run)");
  if (!h->eager && !h->gexec) {
    int rc = build_graph(h);
    if (rc && h->M.dist) {  // RCCL collectives that refuse stream capture: launch them eagerly
      h->eager = true;
      rc = NSGPU_OK;
    }
    if (rc) return rc;
  }
  hipStream_t cs = (hipStream_t)stream;
  NSGPU_HIP(hipEventRecord(h->ev[0], cs));
  NSGPU_HIP(hipStreamWaitEvent(h->s, h->ev[0], 0));
  NSGPU_HIP(hipEventRecord(h->t0, h->s));
  h->done_host[0] = h->done_host[1] = 0;
  if (h->M.dist) {
    const int rc = drive_dist(h);
    if (rc) return rc;
  } else {
    bool paused = false;
    const int rc = drive(h, &paused);
    if (rc) return rc;
    if (paused) return set_error(NSGPU_ESTATE, "nsgpu_p2p_run: paused for a host closure (use nsgpu_p2p_advance)");
  }
  NSGPU_HIP(hipEventRecord(h->t1, h->s));
  uint32_t err = 0;
  NSGPU_HIP(hipMemcpyAsync(&err, h->M.error, 4, hipMemcpyDeviceToHost, h->s));
  NSGPU_HIP(hipEventSynchronize(h->t1));
  NSGPU_HIP(hipStreamSynchronize(h->s));
  NSGPU_HIP(hipEventElapsedTime(&h->last_ms, h->t0, h->t1));
  if (err & 1024u) {  // (debug mode 2: a graph-resident check stopped the run)
    unsigned long long o[4] = {};
    NSGPU_HIP(hipMemcpy(o, g_dbg_out, sizeof(o), hipMemcpyDeviceToHost));
    return set_error(NSGPU_EHIP, "nsgpu_p2p debug (graph): invariant %llu broken after %s (window %llu of the replay, "
                     "C.windows %llu): %llu %llu", o[0], KERNEL_NAMES[o[3] & 0xff], (o[3] >> 8) & 0xff, o[3] >> 32, o[1],
                     o[2]);
  }
  if (err) return engine_error(err);
  NSGPU_HIP(hipEventRecord(h->ev[0], h->s));
  NSGPU_HIP(hipStreamWaitEvent(cs, h->ev[0], 0));
  return NSGPU_OK;
}

extern "C" int nsgpu_p2p_phase_read(uint64_t *out, int n, int reset) {
#ifdef NSGPU_PHASE_PROF
  if (!out || n <= 0) return set_error(NSGPU_EINVAL, "nsgpu_p2p_phase_read: null");
  if (n > 64) {  // the rest: the per-block times of the sampled window (g_blk)
    const int nb = std::min(n - 64, 3 * BLK_MAX * 2);
    NSGPU_HIP(hipMemcpyFromSymbol(out + 64, HIP_SYMBOL(g_blk), nb * sizeof(uint64_t)));
    const int ng = std::min(n - 64 - 3 * BLK_MAX * 2, GT_BLK_MAX * 8);  // (then k_gtile's stamps)
    if (ng > 0) NSGPU_HIP(hipMemcpyFromSymbol(out + 64 + 3 * BLK_MAX * 2, HIP_SYMBOL(g_gt), ng * sizeof(uint64_t)));
    n = 64;
  }
  NSGPU_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase), n * sizeof(uint64_t)));
  if (reset) {
    uint64_t z[64] = {0};
    NSGPU_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_phase), z, sizeof(z)));
  }
  if (reset < 0) {  // (-w: the window the per-block stamps sample from now on; its old stamps cleared)
    const uint64_t w = (uint64_t)(-(int64_t)reset);
    NSGPU_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_blk_win), &w, sizeof(w)));
    std::vector<uint64_t> zb(3 * BLK_MAX * 2, 0);
    NSGPU_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_blk), zb.data(), zb.size() * sizeof(uint64_t)));
  }
  return NSGPU_OK;
#else
  (void)out, (void)n, (void)reset;
  return set_error(NSGPU_ESTATE, "nsgpu_p2p_phase_read: library built without NSGPU_PHASE_PROF");
#endif
}

// Trace sink records (ascii/pcap replay): a device buffer of `cap` records, cleared by every reset.
// The kernels take the engine descriptor by value, so an instantiated graph is rebuilt.
extern "C" int nsgpu_p2p_set_trace(nsgpu_p2p *h, uint64_t cap) {
  if (!h) return set_error(NSGPU_EINVAL, "nsgpu_p2p_set_trace: null");
  if (h->M.trace) return set_error(NSGPU_ESTATE, "nsgpu_p2p_set_trace: tracing is already on");
  if (cap == 0) return set_error(NSGPU_EINVAL, "nsgpu_p2p_set_trace: zero capacity");
  nsgpu_trace_record *tb = nullptr;
  unsigned long long *tn = nullptr;
  int rc = dalloc(h, &tb, cap);
  if (!rc) rc = dalloc(h, &tn, 1);
  if (rc) return rc;
  h->M.trace = tb;
  h->M.trace_n = tn;
  if (h->M.dist) h->M.wide = 0;  // (a traced partitioned engine runs narrow windows: its local records' trace
                                 //  uids would need the single engine's patch pass)
  NSGPU_HIP(hipMemset(h->M.trace_n, 0, sizeof(unsigned long long)));
  h->M.trace_cap = cap;
  if (h->gexec) {
    (void)hipGraphExecDestroy(h->gexec);
    h->gexec = nullptr;
  }
  if (h->gexec_df) {  // (traced engines run the other pipeline)
    (void)hipGraphExecDestroy(h->gexec_df);
    h->gexec_df = nullptr;
  }
  for (hipGraphExec_t &g : h->gtail)
    if (g) {
      (void)hipGraphExecDestroy(g);
      g = nullptr;
    }
  return NSGPU_OK;
}

// Which trace sinks the runs record (bit k = nsgpu_trace_kind k).
extern "C" int nsgpu_p2p_set_trace_kinds(nsgpu_p2p *h, uint32_t mask) {
  if (!h) return set_error(NSGPU_EINVAL, "nsgpu_p2p_set_trace_kinds: null");
  if (mask & ~0x7fu) return set_error(NSGPU_EINVAL, "nsgpu_p2p_set_trace_kinds: unknown kind bits 0x%x", mask);
  h->M.trace_kinds = mask;
  for (hipGraphExec_t *g : {&h->gexec, &h->gexec_df, &h->gtail[0], &h->gtail[1]})
    if (*g) {
      (void)hipGraphExecDestroy(*g);
      *g = nullptr;
    }
  return NSGPU_OK;
}

// Copies the trace records of the last run (unordered; *n = how many the run made, which may exceed
// both the buffer and `cap`: NSGPU_ENOMEM then).
extern "C" int nsgpu_p2p_trace_read(nsgpu_p2p *h, nsgpu_trace_record *out, uint64_t cap, uint64_t *n, void *stream) {
  if (!h || !n) return set_error(NSGPU_EINVAL, "nsgpu_p2p_trace_read: null");
  if (!h->M.trace) return set_error(NSGPU_ESTATE, "nsgpu_p2p_trace_read: tracing is off (nsgpu_p2p_set_trace)");
  hipStream_t s = (hipStream_t)stream;
  unsigned long long total = 0;
  NSGPU_HIP(hipMemcpyAsync(&total, h->M.trace_n, sizeof(total), hipMemcpyDeviceToHost, s));
  NSGPU_HIP(hipStreamSynchronize(s));
  *n = total;
  const uint64_t m = std::min<uint64_t>(std::min<uint64_t>(total, h->M.trace_cap), cap);
  if (m && out) {
    NSGPU_HIP(hipMemcpyAsync(out, h->M.trace, m * sizeof(nsgpu_trace_record), hipMemcpyDeviceToHost, s));
    NSGPU_HIP(hipStreamSynchronize(s));
  }
  if (total > h->M.trace_cap || (out && total > cap))
    return set_error(NSGPU_ENOMEM, "nsgpu_p2p_trace_read: %llu records, buffer %llu", total,
                     (unsigned long long)std::min<uint64_t>(h->M.trace_cap, cap));
  return NSGPU_OK;
}

extern "C" int nsgpu_p2p_set_eager(nsgpu_p2p *h, int eager) {
  if (!h) return set_error(NSGPU_EINVAL, "nsgpu_p2p_set_eager: null");
  h->eager = eager != 0;
  return NSGPU_OK;
}

extern "C" int nsgpu_p2p_kernel_count(int *n) {
  if (!n) return set_error(NSGPU_EINVAL, "nsgpu_p2p_kernel_count: null");
  *n = NKERN;
  return NSGPU_OK;
}

extern "C" const char *nsgpu_p2p_kernel_name(int k) { return k >= 0 && k < NKERN ? KERNEL_NAMES[k] : nullptr; }

// Per-kernel device time: runs the simulation to completion with the pipeline's kernels launched
// one by one on the engine stream; in every `sample_every`-th window each kernel is bracketed by
// two HIP events on that stream, and kernel_ms[k] / launches[k] accumulate the bracketed time and
// the bracketed launches of kernel k (NKERN entries each).  Other windows run unbracketed.
extern "C" int nsgpu_p2p_profile(nsgpu_p2p *h, void *stream, uint32_t sample_every, double *kernel_ms,
                                 uint64_t *launches) {
  if (!h || !kernel_ms || !launches) return set_error(NSGPU_EINVAL, "nsgpu_p2p_profile: null");
  if (h->M.dist) return set_error(NSGPU_ESTATE, "nsgpu_p2p_profile: single-device engines only");
  if (sample_every == 0) sample_every = 1;
  for (int k = 0; k < NKERN; k++) kernel_ms[k] = 0.0, launches[k] = 0;
  // up to NS sampled windows; the events are read after the run (no synchronisation in between
  // beyond the done-flag checks every NWIN windows that nsgpu_p2p_run makes too)
  constexpr int NS = 512;
  std::vector<hipEvent_t> ev(2 * NKERN * NS, nullptr);
  int rc = NSGPU_OK;
  for (auto &e : ev)
    if (hipEventCreate(&e) != hipSuccess) {
      e = nullptr;
      rc = set_error(NSGPU_EHIP, "nsgpu_p2p_profile: hipEventCreate failed");
      break;
    }
  hipStream_t cs = (hipStream_t)stream;
  if (rc == NSGPU_OK && (hipEventRecord(h->ev[0], cs) != hipSuccess || hipStreamWaitEvent(h->s, h->ev[0], 0) != hipSuccess))
    rc = set_error(NSGPU_EHIP, "nsgpu_p2p_profile: stream join failed");
  int ns = 0;
  bool used[NKERN] = {};  // the engine's window launches kernel k (its events are recorded)
  const bool dfu = df_usable(h);
  bool df = dfu && h->uid_hint < UID_DF_SOFT;
  // the run control is read after every window (so no sampled pass is a paused no-op and the
  // host-driven steps run as soon as the pipeline asks)
  for (uint64_t w = 0; rc == NSGPU_OK; w++) {
    const bool sample = (w % sample_every) == 0 && ns < NS;
    for (int k = 0; k < NKERN; k++) {
      if (sample) used[k] |= launch_kernel(h, k, h->s, df, ev[(2 * ns) * NKERN + k], ev[(2 * ns + 1) * NKERN + k]);
      else launch_kernel(h, k, h->s, df);
    }
    if (sample) ns++;
    if (hipGetLastError() != hipSuccess) {
      rc = set_error(NSGPU_EHIP, "nsgpu_p2p_profile: launch failed");
      break;
    }
    if (hipMemcpyAsync(&h->snap[0], h->M.C, sizeof(Ctl), hipMemcpyDeviceToHost, h->s) != hipSuccess ||
        hipStreamSynchronize(h->s) != hipSuccess) {
      rc = set_error(NSGPU_EHIP, "nsgpu_p2p_profile: sync failed");
      break;
    }
    if (h->snap[0].done >= 2) break;  // the final window is appended
    if (h->snap[0].mode >= MODE_SORT) {
      if (df) {  // (the deferred pipeline paused: flush its last window first)
        rc = df_flush(h, h->s);
        if (rc == NSGPU_OK && (hipMemcpyAsync(&h->snap[0], h->M.C, sizeof(Ctl), hipMemcpyDeviceToHost, h->s) != hipSuccess ||
                               hipStreamSynchronize(h->s) != hipSuccess))
          rc = set_error(NSGPU_EHIP, "nsgpu_p2p_profile: sync failed");
        df = false;
      }
      if (rc == NSGPU_OK) rc = host_step(h, h->snap[0], h->s);
    } else if (!df && dfu && h->snap[0].mode == MODE_NORMAL && h->snap[0].uid < UID_DF_SOFT) {  // (sorted-run
                                                                                             //  chunks stay on the other pipeline)
      df = true;
    }
  }
  if (rc == NSGPU_OK) {
    for (int i = 0; i < ns; i++)
      for (int k = 0; k < NKERN; k++) {
        float ms = 0.f;
        if (used[k] && hipEventElapsedTime(&ms, ev[(2 * i) * NKERN + k], ev[(2 * i + 1) * NKERN + k]) == hipSuccess) {
          kernel_ms[k] += ms;
          launches[k]++;
        }
      }
  }
  for (auto e : ev)
    if (e) (void)hipEventDestroy(e);
  (void)hipEventRecord(h->ev[0], h->s);
  (void)hipStreamWaitEvent(cs, h->ev[0], 0);
  return rc;
}

// Whether the engine runs wide windows (node degree <= LQ, not NSGPU_P2P_NARROW=1; a traced partitioned engine
// runs narrow ones).
extern "C" int nsgpu_p2p_get_wide(nsgpu_p2p *h, int *wide) {
  if (!h || !wide) return set_error(NSGPU_EINVAL, "nsgpu_p2p_get_wide: null");
  *wide = h->M.wide ? 1 : 0;
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
  if (devc)
    NSGPU_HIP(hipMemcpy2DAsync(devc, sizeof(*devc), &M.dev[0].c, sizeof(DevRec), sizeof(*devc), M.n_devices,
                               hipMemcpyDeviceToHost, s));
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
    stats->icmp_sent = c.icmp;
    stats->refits = c.refits;
  }
  if (error) *error = err;
  if (err) return engine_error(err);
  return NSGPU_OK;
}

// ====================================================================================================
// Loopback group: every partition of one scenario on this device, the collectives replaced by
// device-to-device copies (k_copies) on one stream — the partitioned algorithm's parity harness on
// a single GPU.  Members are nsgpu_p2p_create_dist engines with comm == NULL, rank i at index i.
// ====================================================================================================
struct nsgpu_p2p_group {
  std::vector<nsgpu_p2p *> m;
  CopyDesc *d_x[4] = {nullptr, nullptr, nullptr, nullptr};  // X0, X1, X2, the cut's keys: n x n copies each
  hipStream_t s = nullptr;
  hipGraphExec_t gexec = nullptr;
  hipEvent_t ev[2] = {nullptr, nullptr};
  uint32_t *done_host = nullptr;
  Ctl *snap = nullptr;  // pinned, 2 run-control snapshots of member 0 (the pauses are run-global)
};

static void launch_windows_group(nsgpu_p2p_group *g, hipStream_t s, int nwin = NWIN) {
  const unsigned n = (unsigned)g->m.size();
  for (int w = 0; w < nwin; w++) {
    for (auto *h : g->m) dist_pa(h->M, s);
    hipLaunchKernelGGL(k_copies, dim3(n * n), dim3(256), 0, s, (const CopyDesc *)g->d_x[0]);
    for (auto *h : g->m) dist_handle(h->M, s);
    for (auto *h : g->m) dist_rank(h->M, s);
    hipLaunchKernelGGL(k_copies, dim3(n * n), dim3(256), 0, s, (const CopyDesc *)g->d_x[1]);
    for (auto *h : g->m) dist_rank_fin(h->M, s);
    hipLaunchKernelGGL(k_copies, dim3(n * n), dim3(256), 0, s, (const CopyDesc *)g->d_x[2]);
  }
}

extern "C" int nsgpu_p2p_group_destroy(nsgpu_p2p_group *g) {
  if (!g) return NSGPU_OK;
  if (g->s) (void)hipStreamSynchronize(g->s);
  if (g->gexec) (void)hipGraphExecDestroy(g->gexec);
  for (hipEvent_t e : {g->ev[0], g->ev[1]})
    if (e) (void)hipEventDestroy(e);
  if (g->done_host) (void)hipHostFree(g->done_host);
  if (g->snap) (void)hipHostFree(g->snap);
  for (CopyDesc *d : g->d_x)
    if (d) (void)hipFree(d);
  if (g->s) (void)hipStreamDestroy(g->s);
  delete g;
  return NSGPU_OK;
}

extern "C" int nsgpu_p2p_group_create(nsgpu_p2p **members, int n, nsgpu_p2p_group **out) {
  if (!members || !out || n < 1) return set_error(NSGPU_EINVAL, "nsgpu_p2p_group_create: bad arguments");
  *out = nullptr;
  for (int i = 0; i < n; i++) {
    const nsgpu_p2p *h = members[i];
    if (!h || !h->M.dist || h->comm || h->M.nranks != (uint32_t)n || h->M.rank != (uint32_t)i)
      return set_error(NSGPU_EINVAL, "nsgpu_p2p_group_create: member %d is not loopback partition %d of %d", i, i, n);
  }
  nsgpu_p2p_group *g = new nsgpu_p2p_group();
  g->m.assign(members, members + n);
  std::vector<CopyDesc> x[4];
  for (int r = 0; r < n; r++)
    for (int q = 0; q < n; q++) {
      const P2PDev &R = members[r]->M, &Q = members[q]->M;
      x[0].push_back(CopyDesc{(const uint8_t *)Q.x0_send, (uint8_t *)(R.x0_recv + 2 * q), X0B});
      x[1].push_back(CopyDesc{Q.x1_send, R.x1_recv + (size_t)q * X1B, X1B});
      x[2].push_back(CopyDesc{Q.x2_send + (size_t)r * Q.x2b, R.x2_recv + (size_t)q * R.x2b, Q.x2b});
      x[3].push_back(CopyDesc{(const uint8_t *)Q.xk_send, (uint8_t *)(R.xk_recv + 2 * q), 16});
    }
  for (int k = 0; k < 4; k++) {
    if (hipMalloc(&g->d_x[k], x[k].size() * sizeof(CopyDesc)) != hipSuccess ||
        hipMemcpy(g->d_x[k], x[k].data(), x[k].size() * sizeof(CopyDesc), hipMemcpyHostToDevice) != hipSuccess) {
      nsgpu_p2p_group_destroy(g);
      return set_error(NSGPU_ENOMEM, "nsgpu_p2p_group_create: copy descriptors");
    }
  }
  if (hipStreamCreateWithFlags(&g->s, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&g->ev[0], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&g->ev[1], hipEventDisableTiming) != hipSuccess ||
      hipHostMalloc((void **)&g->done_host, 2 * sizeof(uint32_t), hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc((void **)&g->snap, 2 * sizeof(Ctl), hipHostMallocDefault) != hipSuccess) {
    nsgpu_p2p_group_destroy(g);
    return set_error(NSGPU_EHIP, "nsgpu_p2p_group_create: stream / events");
  }
  *out = g;
  return NSGPU_OK;
}

extern "C" int nsgpu_p2p_group_reset(nsgpu_p2p_group *g, void *stream) {
  if (!g) return set_error(NSGPU_EINVAL, "nsgpu_p2p_group_reset: null");
  for (nsgpu_p2p *h : g->m) {
    const int rc = nsgpu_p2p_reset(h, stream);
    if (rc) return rc;
  }
  return NSGPU_OK;
}

// The host-driven steps of a group (host_step_dist's, every member): the cut's keys go through k_copies.
static int group_host_step(nsgpu_p2p_group *g, const Ctl &c0) {
  hipStream_t s = g->s;
  if (c0.mode == MODE_CUT) {  // a partitioned sorted run (host_step_dist's steps, every member)
    for (auto *h : g->m) {
      Ctl c;
      NSGPU_HIP(hipMemcpyAsync(&c, h->M.C, sizeof(Ctl), hipMemcpyDeviceToHost, s));
      NSGPU_HIP(hipStreamSynchronize(s));
      const int rc = drun_sort(h, c.W, s);
      if (rc) return rc;
    }
    const unsigned n = (unsigned)g->m.size();
    hipLaunchKernelGGL(k_copies, dim3(n * n), dim3(256), 0, s, (const CopyDesc *)g->d_x[3]);
    for (auto *h : g->m) hipLaunchKernelGGL(k_drun_first, dim3(WCAP / TB), dim3(TB), 0, s, h->M);
    NSGPU_HIP(hipGetLastError());
    return NSGPU_OK;
  }
  for (auto *h : g->m) {
    Ctl c;
    NSGPU_HIP(hipMemcpyAsync(&c, h->M.C, sizeof(Ctl), hipMemcpyDeviceToHost, s));
    NSGPU_HIP(hipStreamSynchronize(s));
    const int rc = host_step(h, c, s);
    if (rc) return rc;
  }
  return NSGPU_OK;
}

// Runs every partition to the end of the simulation (blocking), like nsgpu_p2p_run.
extern "C" int nsgpu_p2p_group_run(nsgpu_p2p_group *g, void *stream) {
  if (!g) return set_error(NSGPU_EINVAL, "nsgpu_p2p_group_run: null");
  // NSGPU_P2P_EAGER: the replays' kernels launched one by one (rocprofv3's kernel tracer does not follow graphs)
  static const bool eager = getenv("NSGPU_P2P_EAGER") != nullptr;
  if (!eager && !g->gexec) {
    hipGraph_t gr = nullptr;
    NSGPU_HIP(hipStreamBeginCapture(g->s, hipStreamCaptureModeThreadLocal));
    launch_windows_group(g, g->s);
    hipError_t e = hipStreamEndCapture(g->s, &gr);
    if (e != hipSuccess) return set_error(NSGPU_EHIP, "nsgpu_p2p_group: graph capture: %s", hipGetErrorString(e));
    e = hipGraphInstantiate(&g->gexec, gr, nullptr, nullptr, 0);
    (void)hipGraphDestroy(gr);
    if (e != hipSuccess) {
      g->gexec = nullptr;
      return set_error(NSGPU_EHIP, "nsgpu_p2p_group: graph instantiate: %s", hipGetErrorString(e));
    }
  }
  hipStream_t cs = (hipStream_t)stream;
  NSGPU_HIP(hipEventRecord(g->ev[0], cs));
  NSGPU_HIP(hipStreamWaitEvent(g->s, g->ev[0], 0));
  // as drive_dist: member 0's run control decides (done and the pauses are run-global)
  const Ctl *C0 = g->m[0]->M.C;
  int cur = 0;
  bool have_prev = false;
  for (;;) {
    if (eager) launch_windows_group(g, g->s);
    else NSGPU_HIP(hipGraphLaunch(g->gexec, g->s));
    NSGPU_HIP(hipGetLastError());
    NSGPU_HIP(hipMemcpyAsync(&g->snap[cur], C0, sizeof(Ctl), hipMemcpyDeviceToHost, g->s));
    NSGPU_HIP(hipEventRecord(g->ev[cur], g->s));
    if (have_prev) {
      NSGPU_HIP(hipEventSynchronize(g->ev[cur ^ 1]));
      const Ctl &c = g->snap[cur ^ 1];
      if (c.done >= 2) break;
      if (c.mode >= MODE_SORT) {
        NSGPU_HIP(hipEventSynchronize(g->ev[cur]));
        const int rc = group_host_step(g, g->snap[cur]);
        if (rc) return rc;
        have_prev = false;
        continue;
      }
    }
    have_prev = true;
    cur ^= 1;
  }
  NSGPU_HIP(hipEventRecord(g->ev[0], g->s));
  NSGPU_HIP(hipEventSynchronize(g->ev[0]));
  NSGPU_HIP(hipStreamWaitEvent(cs, g->ev[0], 0));
  uint32_t err = 0;
  for (nsgpu_p2p *m : g->m) {  // (as nsgpu_p2p_run: a member's error word fails the run)
    uint32_t e = 0;
    NSGPU_HIP(hipMemcpy(&e, m->M.error, 4, hipMemcpyDeviceToHost));
    err |= e;
  }
  if (err) return engine_error(err);
  return NSGPU_OK;
}
