// nsgpu_p2p_win.h — the single-GPU window pipeline of the GPU-resident p2p subset (included by
// nsgpu_p2p.hip inside namespace nsgpu, after the shared model code).
//
// Per conservative window three kernels, replayed from a hipGraph:
//   k2_pa      appends the last window (dispatch log / digest; its children get their uids) and forms
//              the next one: every pending event with key <= the bound (W_end = min over pending of
//              ts + lookahead(kind), capped at Simulator::Stop's key) becomes a window record.  The
//              pending pool is kept IN PLACE: it is only read (ts, uid, kind) — window events are
//              tombstoned afterwards and their slots reused, children that stay pending are parked
//              in a fresh buffer and moved into free slots by k2_handle.
//   k2_handle  the holder of each node runs the node's window events in key order; nodes with more
//              than CH events (hubs: a dumbbell router) get a whole block that takes the node's
//              events in key order, runs their node parts (stateless forwarding in parallel,
//              node-state work serially) and then the device steps with the device state kept in
//              registers.  Other blocks rank the window keys (all-pairs counting) and do the pool
//              maintenance.
//   k2_scan    rank order, exclusive scans of child counts (uids), run bookkeeping.
// A window larger than WCAP (config 5's hundreds of thousands of same-time events) is a SORTED RUN:
// k2_scan pauses the graph, the host radix-sorts the window records by key (k_rs_*), and the run is
// then dispatched in rank-order chunks of WCAP — every child of a run event sorts after every run
// event (the window rule), so chunks need no re-selection.  A zero-delay PacketSink DoForwardUp
// whose ts group a chunk boundary cuts is queued like any other event (K_FWD_UP_D) instead of being
// run inline, which keeps its (ts, uid) position.  When the pool holds many tombstones the host
// compacts it (k_cmp).

enum : uint32_t { MODE_NORMAL = 0, MODE_RUN = 1, MODE_SORT = 2, MODE_COMPACT = 3, MODE_HOST = 4, MODE_CUT = 5,
                  MODE_TRIM = 6, MODE_UIDX = 7 };  // UIDX: the deferred pipeline hands over (uids near UID_DF_SOFT)
constexpr uint64_t TOMB = ~0ull;        // ev_ts of a free pool slot
constexpr uint32_t NOSRC = 0xffffffffu;
constexpr int NHUB = 32;                // hub blocks of k2_handle
#ifndef NMB_N
#define NMB_N 128
#endif
constexpr int NMB = NMB_N;              // maintenance blocks of k2_handle
constexpr int MAXHUB = WCAP / (CH + 1) + 1;
constexpr int K2_GRID_W = NHB + NHUB + NMB;  // holders, hub blocks, pool maintenance
constexpr int K2_GRID = K2_GRID_W + NRB;       // + rank tiles (single engine; partitioned: k_gtile ranks)
// ---- wide windows: local records (a node's same-node TransmitCompletes run inside the window) ----
constexpr int LQ = 16;                   // a node's pending local records: its busy devices' (degree <= LQ)
constexpr int LR = 128;                  // local records of one holder block per window (its region)
constexpr int LRH = 512;                 // ... of one hub block
constexpr int NLR = NHB + NHUB;          // regions: holder blocks, then hub blocks
constexpr uint32_t LBASE = WCAP;         // local records live at [LBASE, LBASE + LCAP) of the record arrays
constexpr int LCAP = NHB * LR + NHUB * LRH;
constexpr int WTOT = WCAP + LCAP;        // record index space (gen-0 slots + local regions)
constexpr int NMAX = 8192;               // records of one window, gen-0 + local (k2_scan's LDS capacity)
static_assert(NMAX == 8 * STG_NT, "stage slices");
// The run control through the vector memory path.  A kernel's first reads of Ctl come from lines another XCD
// wrote (one memory trip).  As scalar loads they hold back every later scalar load (a scalar wait cannot
// single out one load), so the kernel-argument pointers of the slot loads wait for the run control and the
// slot loads go out one trip late; as vector loads they are in flight together.
__device__ __forceinline__ Ctl *vec_ctl(Ctl *p) {
  typedef __attribute__((address_space(1))) Ctl GCtl;
  GCtl *g = (GCtl *)p;
  asm volatile("" : "+v"(g));
  return (Ctl *)g;  // (a global pointer: global, not flat, loads)
}
// a staged rank's position in the stage arrays and cpt (k2_sdef's thread r / 8 loads it as its (r % 8)-th)
__device__ __forceinline__ uint32_t stg_pos(uint32_t r) { return (r & 7u) * STG_NT + (r >> 3); }
// a rank's word in k2_sdef's per-rank LDS arrays: one pad word per 64, so a wave's 8-strided accesses
// (lane l, rank 8l + q) fall in 64 different banks
__device__ __forceinline__ uint32_t lds_pad(uint32_t r) { return r + (r >> 6); }
constexpr int NMAX_PAD = NMAX + NMAX / 64;
constexpr int LMAX = NMAX - WCAP;        // local records of one window
static_assert(LMAX == XLCAP, "a partitioned rank's X1Loc list holds its window's local records");
constexpr int SLOTG = WCAP + LMAX;       // k2_pa's slot-role threads (single engine): gen-0 slots, then local
static_assert(LCAP < (1 << 24) && WTOT < (1 << 24), "wpar packs a record index in 24 bits");
// Rank accumulators of window `win` (by parity: a deferred window's ranks are read after the next window's
// ranking has begun).  wrank: 2 x WTOT, lrank: 2 x LMAX.
__device__ __forceinline__ uint32_t *wrank_of(const P2PDev &M, uint64_t win) { return M.wrank + (win & 1) * WTOT; }
__device__ __forceinline__ uint32_t *lrank_of(const P2PDev &M, uint64_t win) { return M.lrank + (win & 1) * LMAX; }

__device__ __forceinline__ uint32_t region_base(uint32_t r) {
  return LBASE + (r < (uint32_t)NHB ? r * LR : NHB * LR + (r - NHB) * LRH);
}
// Dense record d of a window of W gen-0 records and local regions with prefix pre[] (NLR + 1 entries).
__device__ __forceinline__ uint32_t dense_rec(uint32_t d, uint32_t W, const uint32_t *pre) {
  if (d < W) return d;
  const uint32_t k = d - W;
  uint32_t lo = 0, hi = NLR;  // the region r with pre[r] <= k < pre[r + 1]
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (pre[mid] <= k) lo = mid;
    else hi = mid;
  }
  return region_base(lo) + (k - pre[lo]);
}

// Node-part result of one hub event (k2_handle hub blocks, between the two passes).
struct HubEv {
  uint32_t op, dev;
  Pkt p;
  int64_t pdelay;      // trailing child (OnOffApplication::ScheduleNextTx after SendPacket)
  uint32_t pkind, pa;  // pkind == 0: none
  uint32_t n, seq;     // children and trace sink calls the node part made
  uint32_t cancelled, pad;  // pad: the node part's inline DoForwardUp children
  uint32_t ctx, xdrop;      // the event's context (its Schedule calls inherit it); NodeOut::xdrop
};

constexpr int HUBL = 1024;  // events of a hub a block sorts in LDS (more: the window is dispatched as a run)

// A handled window slot's child counts.  A partitioned rank also fills the slot's X1 entry (key, counts)
// and accumulates its summary's totals per thread (x1_totals folds them).
struct X1Acc {
  uint32_t tc, ti;
  uint64_t lk;
};
__device__ __forceinline__ void slot_done(const P2PDev &M, uint32_t s, uint64_t key, uint32_t n, uint32_t ni,
                                          X1Acc &xa) {
  M.nchild[s] = n;
  M.ninl[s] = ni;
  xa.tc += n;  // (the window's totals: a partitioned rank's X1 summary, the single engine's k2_rank bookkeeping)
  xa.ti += ni;
  if (M.dist && s < (uint32_t)WCAP) {  // (a local record's entry: X1Loc, compacted at its block's end)
    x1ent(M)[s] = X1Ent{key, n | (ni << 16), 0};
    xa.lk = key > xa.lk ? key : xa.lk;
  }
}
// All lanes of the wave call it.
__device__ __forceinline__ void x1_totals(const P2PDev &M, X1Acc xa) {
  if (!M.dist) {  // single engine: the window's child totals (the deferred bookkeeping advances uid / K by them)
    xa.tc = wave_sum32(xa.tc);
    xa.ti = wave_sum32(xa.ti);
    if ((threadIdx.x & 63) == 0) {
      if (xa.tc) atomicAdd((unsigned long long *)&M.C->acc_tc, (unsigned long long)xa.tc);
      if (xa.ti) atomicAdd((unsigned long long *)&M.C->acc_tinl, (unsigned long long)xa.ti);
    }
    return;
  }
  xa.tc = wave_sum32(xa.tc);
  xa.ti = wave_sum32(xa.ti);
  xa.lk = wave_max64(xa.lk);
  if ((threadIdx.x & 63) == 0) {
    X1Hdr *h = x1hdr(M.x1_send, 0);
    if (xa.tc) atomicAdd(&h->tc, xa.tc);
    if (xa.ti) atomicAdd(&h->tinl, xa.ti);
    if (xa.lk) atomicMax((unsigned long long *)&h->lastkey, (unsigned long long)xa.lk);
  }
}

// Wave-aggregated counter allocation: one index per lane with `want` (active lanes only).
__device__ __forceinline__ uint32_t wave_alloc32(uint32_t *ctr, bool want) {
  const uint64_t m = __ballot(want);
  const int lane = threadIdx.x & 63;
  uint32_t base = 0;
  if (m) {
    const int first = __ffsll((unsigned long long)m) - 1;
    if (lane == first) base = atomicAdd(ctr, (uint32_t)__popcll(m));
    base = rl32(base, first);  // (first is uniform: a readlane, not a ds_bpermute)
  }
  return base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
}
__device__ __forceinline__ uint64_t wave_alloc64(uint64_t *ctr, bool want) {
  const uint64_t m = __ballot(want);
  const int lane = threadIdx.x & 63;
  unsigned long long base = 0;
  if (m) {
    const int first = __ffsll((unsigned long long)m) - 1;
    if (lane == first) base = atomicAdd((unsigned long long *)ctr, (unsigned long long)__popcll(m));
    base = rl64(base, first);
  }
  return (uint64_t)base + (uint64_t)__popcll(m & ((1ull << lane) - 1ull));
}

constexpr uint32_t NOHOLD = 0xffffffffu;  // widx of a window event no holder runs (NetDevice::Start)

// The node whose state an event touches (its logical process).  Events scheduled by the handlers carry
// it as their context; a host closure runs in context 0xffffffff and Simulator::Schedule inherits the
// current context, so e.g. the TransmitComplete of a datagram a host closure sent has none
// (point-to-point-net-device.cc:226, default-simulator-impl.cc:188-204).
__device__ __forceinline__ uint32_t lp_of(const P2PDev &M, uint32_t ctx, uint32_t kind_word, uint32_t a) {
  if (ctx != NOCTX) return ctx;
  switch (kind_word & 0xffu) {
    case K_TX_COMPLETE:
    case K_RECEIVE:
      return M.dev_node[a];
    case K_NODE_START:
      return a;
    case K_STOP:
    case K_DEV_START:
      return NOCTX;
    default:
      return M.app_node[a];
  }
}

// Window record `slot` of node `ctx` -> the node's slot table (local slot index); the node that
// reaches CH + 1 events becomes a hub.  NetDevice::Start is a no-op (the device was started by
// Node::Start): it is dispatched (logged, uid-ranked) but no holder runs it — a dumbbell router has
// one per leaf link at time 0.  In two halves: the claim issues the count atomic, the finish (late in
// the kernel, once the atomic's value is back) stores the slot, so a wave does not wait for the atomic.
struct NtClaim {
  uint32_t slot, c, idx;  // c == NOSRC: nothing to finish
};
__device__ __forceinline__ NtClaim node_table_claim(const P2PDev &M, uint32_t slot, uint32_t ctx, uint32_t kind) {
  if ((kind & 0xffu) == K_DEV_START) {  // (k2_handle writes its zero child counts: k2_pa still reads the
    M.widx[slot] = NOHOLD;               //  last window's counts of this slot)
    return NtClaim{slot, NOSRC, 0};
  }
  if (ctx < M.n_nodes) return NtClaim{slot, ctx, atomicAdd(&M.node_tab[(uint64_t)ctx * NTAB], 1u)};
  M.widx[slot] = 0;
  return NtClaim{slot, NOSRC, 0};
}
// sorted: a partitioned run's chunk (key order: its hub blocks take a hub's events in slot order, no HUBL limit)
__device__ __forceinline__ void node_table_finish(const P2PDev &M, Ctl &C, const NtClaim &p, bool sorted = false) {
  if (p.c == NOSRC) return;
  const uint32_t idx = p.idx;
  if (idx < (uint32_t)NSLOT) M.node_tab[(uint64_t)p.c * NTAB + 1 + idx] = p.slot;
  if (idx == (uint32_t)CH) {
    const uint32_t hh = atomicAdd(&C.nhub, 1u);
    if (hh < (uint32_t)MAXHUB) M.hub_list[hh] = p.c;
  }
  if (idx == (uint32_t)HUBL && !sorted) {  // too many for a hub block: a sorted run (single engine or partitioned)
    if (M.dist) C.overflow = 1;
    else C.force_run = 1;
  }
  M.widx[p.slot] = idx;
}
__device__ __forceinline__ void node_table_add(const P2PDev &M, Ctl &C, uint32_t slot, uint32_t ctx, uint32_t kind) {
  node_table_finish(M, C, node_table_claim(M, slot, ctx, kind));
}
// node_table_claim for the wave's lanes with `on` (every lane of the wave calls it), the lanes whose node is the
// first such lane's claimed with ONE atomic: a sorted run's chunk holds a hub's thousands of events, and their
// count atomics on one word serialised (~10 ns each: k2_pa 51 us a chunk at a dumbbell router).  Which of a node's
// slots gets which index does not matter (the holder sorts its node's events by key; a hub's block scans them).
__device__ __forceinline__ NtClaim node_table_claim_wave(const P2PDev &M, uint32_t slot, uint32_t ctx, uint32_t kind,
                                                         bool on) {
  const bool dev_start = (kind & 0xffu) == K_DEV_START;
  const bool nd = on && !dev_start && ctx < M.n_nodes;  // (a node's count claim)
  const uint64_t mn = __ballot(nd);
  NtClaim cl{slot, NOSRC, 0};
  bool done = false;
  if (mn) {
    const int lead = __ffsll((unsigned long long)mn) - 1;
    const uint32_t c0 = rl32(ctx, lead);  // (lead is uniform)
    const bool same = nd && ctx == c0;
    const uint64_t ms = __ballot(same);
    const int lane = threadIdx.x & 63;
    uint32_t base = 0;
    if (lane == lead) base = atomicAdd(&M.node_tab[(uint64_t)c0 * NTAB], (uint32_t)__popcll(ms));
    base = rl32(base, lead);
    if (same) {
      cl = NtClaim{slot, ctx, base + (uint32_t)__popcll(ms & ((1ull << lane) - 1ull))};
      done = true;
    }
  }
  if (on && !done) cl = node_table_claim(M, slot, ctx, kind);
  return cl;
}

// A pending event against the window bound: window record (normal mode, key <= bound), else pending:
// a child (src == NOSRC) is parked in the fresh buffer, a pool entry stays where it is; both fold
// into the next window's reduction.
template <bool WIDE>
__device__ __forceinline__ void k2_classify(const int64_t *look, const WinBound &b, bool run, bool valid, const Ev &e,
                                            uint32_t src, Red &R, uint64_t &tmn, uint64_t &wnd, uint64_t &wndw,
                                            bool &in, bool &park) {
  const uint64_t pk = ((e.ts - b.tmin) << 32) | e.uid;
  in = valid && !run && (e.ts - b.tmin <= b.span) && pk <= b.bound;
  park = valid && !in && src == NOSRC;
  if (valid && !in) {
    tmn = e.ts < tmn ? e.ts : tmn;
    const uint32_t kd = (e.kind & 0xffu) % K_NKINDS;
    const uint64_t x = e.ts + (uint64_t)look[kd];
    wnd = x < wnd ? x : wnd;
    if constexpr (WIDE) {
      const uint64_t xw = e.ts + (uint64_t)look[K_NKINDS + kd];
      wndw = xw < wndw ? xw : wndw;
    }
    if ((e.kind & 0xffu) == K_STOP) {  // at most one Stop event is pending
      R.stopts = e.ts;
      R.stopuid = e.uid;
    }
  }
}

// Writes a classified event: window record `slot`, or fresh-buffer entry `fi` (a parked child).  Returns
// the window record's node-table claim (to finish later in the kernel).
__device__ __forceinline__ NtClaim k2_write(const P2PDev &M, Ctl &C, const WinBound &b, const Ev &e, uint32_t src,
                                            bool in, bool park, uint32_t slot, uint64_t fi) {
  NtClaim cl{0, NOSRC, 0};
  if (in) {
    if (slot < M.runcap) {
      M.wkey[slot] = ((e.ts - b.tmin) << 32) | e.uid;
      M.wctx[slot] = e.ctx;
      M.wkind[slot] = e.kind;
      M.wa[slot] = e.a;
      M.wpkt[slot] = e.p;
      M.wsrc[slot] = src;
      if (slot < (uint32_t)WCAP) cl = node_table_claim(M, slot, lp_of(M, e.ctx, e.kind, e.a), e.kind);
    } else {
      atomicOr(M.error, 1u);
    }
  } else if (park) {
    if (fi < M.fcap) {
      M.f_ts[fi] = e.ts;
      M.f_uid[fi] = e.uid;
      M.f_ctx[fi] = e.ctx;
      M.f_kind[fi] = e.kind;
      M.f_a[fi] = e.a;
      M.f_pkt[fi] = e.p;
    } else {
      atomicOr(M.error, 1u);
    }
  }
  return cl;
}

// Block-wide allocation of window slots (C.W) and fresh-buffer entries (C.nF): per-thread counts in,
// each thread's first index out, ONE atomic per counter per block (a device-scope atomic on a shared
// word costs ~10 ns and they serialise: per-wave allocation cost k2_pa ~3 us a window).  Every thread
// of the block calls it.
template <int NT>
__device__ __forceinline__ void block_alloc2(Ctl &C, uint32_t nw, uint32_t nf, uint32_t &w0, uint64_t &f0) {
  __shared__ uint64_t s_w[NT / 64];
  __shared__ uint64_t s_base[2];
  const uint64_t v = (uint64_t)nw | ((uint64_t)nf << 32);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint64_t inc = wave_incscan64(v);
  if (lane == 63) s_w[wid] = inc;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t tot = 0;
    for (int w = 0; w < NT / 64; w++) {
      const uint64_t x = s_w[w];
      s_w[w] = tot;
      tot += x;
    }
    const uint32_t tw = (uint32_t)tot, tf = (uint32_t)(tot >> 32);
    s_base[0] = tw ? atomicAdd(&C.W, tw) : 0u;
    s_base[1] = tf ? (uint64_t)atomicAdd((unsigned long long *)&C.nF, (unsigned long long)tf) : 0ull;
  }
  __syncthreads();
  const uint64_t ex = s_w[wid] + inc - v;
  w0 = (uint32_t)s_base[0] + (uint32_t)ex;
  f0 = s_base[1] + (ex >> 32);
  __syncthreads();  // (s_w / s_base are reused by the next call)
}

// The end of the sorted-run chunk that starts at r0 (a run is dispatched in rank-order chunks of at most
// WCAP).  A chunk does not end inside a same-ts group unless the group alone fills it: the chunk's
// DoForwardUp leaves at a cut group's ts are queued (K_FWD_UP_D, their uids sort after the whole group), so
// a chunk that continues a cut group ends with the group and the run ends there (*trim: the rest of the
// run goes back to the pool, k_trim) — the queued leaves are then dispatched before any later event.
// Every thread of the block calls it.
template <int NT>
__device__ void run_chunk_end(const P2PDev &M, uint64_t r0, uint64_t rW, uint64_t &r1_out, bool &trim_out) {
  __shared__ unsigned long long s_r1;
  __shared__ uint32_t s_trim;
  const uint64_t r1 = r0 + (uint64_t)WCAP < rW ? r0 + (uint64_t)WCAP : rW;
  const uint64_t t0 = M.wkey[r0] >> 32, tl = M.wkey[r1 - 1] >> 32;
  const bool cont = r0 > 0 && (M.wkey[r0 - 1] >> 32) == t0;
  const bool cut = r1 < rW && (M.wkey[r1] >> 32) == tl;
  if (threadIdx.x == 0) {
    s_r1 = r1;
    s_trim = 0;
  }
  __syncthreads();
  if (cont && tl != t0) {  // the continued group ends inside [r0, r1): the chunk ends with it
    for (uint64_t i = r0 + threadIdx.x; i < r1; i += NT)
      if ((M.wkey[i] >> 32) > t0) {
        atomicMin(&s_r1, (unsigned long long)i);
        break;
      }
    if (threadIdx.x == 0) s_trim = 1;
  } else if (!cont && cut) {  // back off to the start of the group the chunk would cut (unless it fills it)
    for (uint64_t i = r0 + threadIdx.x; i < r1; i += NT)
      if ((M.wkey[i] >> 32) == tl) {
        if (i > r0) atomicMin(&s_r1, (unsigned long long)i);
        break;
      }
  }
  __syncthreads();
  r1_out = s_r1;
  trim_out = s_trim != 0;
  __syncthreads();
}

// ---- partitioned sorted runs (DIST) ----
// A window some rank cannot hold (more than WCAP candidates, or a hub beyond HUBL) becomes a sorted run: every
// rank sorts its candidates once (host step: k_drun_clear, k_rs_*, k_drun_start; the run lives in rn_*), and the
// run is dispatched in chunks — chunk k is every rank's run entries with key <= g_k, g_k the smallest of the
// ranks' fitting keys (the key of a rank's WCAP-th remaining entry; none when the rest fits).  A key prefix of a
// safe window is safe, and every child of a run event sorts after the whole run (the run window was bounded by
// the pending set's lookahead), so the chunks are the sequential order's windows; their children stay pending
// until the run ends.  The first chunk is formed after the exchange of the fitting keys (k_drun_first), every
// later one by k2_pa with g from the last window's X1 summaries (k_dfin2): no host step per chunk.

// A chunk cut at g ends inside a same-ts group (g is a real key: its uid part is below 0xffffffff; a back-off or
// group-end cut is ((ts << 32) | 0xffffffff)): its DoForwardUp leaves at that ts are queued.
__device__ __forceinline__ bool drun_cuts_group(uint64_t g, uint64_t bound) {
  return g < bound && (uint32_t)g != 0xffffffffu;
}
// The chunk's bound: the run window's, capped at the cut key g.
__device__ __forceinline__ WinBound drun_bound(const Ctl &C, uint64_t g) {
  WinBound b;
  b.tmin = C.drb_tmin;
  b.span = C.drb_span;
  b.bound = C.drb_bound < g ? C.drb_bound : g;
  b.stop_packed = C.drb_stop;
  b.nbound = C.drb_nbound;
  b.lim = C.drb_lim;
  return b;
}
// Thread t (< WCAP, NT per block, every thread of the block calls it): run entry r0 + t, if its key is <= g,
// becomes window record t (the entries <= g are a prefix: the run is sorted); the block's count goes to C.W.
// The thread of the chunk's last entry (thread 0 when the chunk is empty) advances the run and puts this rank's
// fitting key for the next chunk and its entries left into the rank's X1 summary.
template <int NT>
__device__ void drun_chunk(const P2PDev &M, Ctl &C, uint64_t t, uint64_t r0, uint64_t rW, uint64_t g) {
  const uint64_t i = r0 + t;
  const bool take = t < (uint64_t)WCAP && i < rW && M.rn_key[i] <= g;
  const bool next = t + 1 < (uint64_t)WCAP && i + 1 < rW && M.rn_key[i + 1] <= g;
  uint32_t cc = NOSRC, ck = 0;
  if (take) {
    const uint64_t key = M.rn_key[i];
    const uint32_t ctx = M.rn_ctx[i], kind = M.rn_kind[i], a = M.rn_a[i];
    M.wkey[t] = key;
    M.wctx[t] = ctx;
    M.wkind[t] = kind;
    M.wa[t] = a;
    M.wpkt[t] = M.rn_pkt[i];
    M.wsrc[t] = M.rn_src[i];
    cc = lp_of(M, ctx, kind, a);
    ck = kind;
  }
  const NtClaim cl = node_table_claim_wave(M, (uint32_t)t, cc, ck, take);  // (a hub's claims aggregated)
  const uint32_t nb = (uint32_t)__syncthreads_count(take);
  if (threadIdx.x == 0 && nb) atomicAdd(&C.W, nb);
  node_table_finish(M, C, cl, true);
  if ((take && !next) || (t == 0 && !take)) {
    const uint64_t r1 = take ? i + 1 : r0;
    C.dr1 = r1;  // (k_dfin2 advances dr0: this kernel's other blocks may still be loading it)
    X1Hdr *hs = x1hdr(M.x1_send, 0);
    hs->rrem = rW - r1;
    hs->rkey = rW - r1 > (uint64_t)WCAP ? M.rn_key[r1 + WCAP - 1] : ~0ull;
    hs->rhead = rW > r1 ? M.rn_key[r1] : ~0ull;
    if (g < C.drb_bound) C.refits++;
  }
}

// ---- k2_pa ----
// DIST: a partitioned rank's variant: children on other ranks' nodes are skipped (they travel through
// X2), the remote events the last X2 brought are classified like children (a role of whole blocks
// after the slot blocks), the rank's reduction goes to its X1 summary, and a window the host cut
// (the first chunk of a partitioned sorted run, k_drun_first: C.prep) is already formed; during such a run
// (C.drun) every k2_pa moves the run's next chunk in, and children, remote events and the pool stay pending.
// WIDE: wide windows (the last window's local records are appended too; partitioned: their sinfo / pwkey /
// lrec come from k_dfin2).
// k2_pa's grid (single engine): the slot blocks, then as many blocks of the pool sweep as GRID_POOL leaves
template <bool WIDE>
constexpr int pa_grid() {
  constexpr int nsg = WIDE ? SLOTG : WCAP;
  return nsg / PA_SLOT_LANES + GRID_POOL - nsg / TB;
}
// ... at run time: a large pool (the default capacity is 2^20 entries; config 5's holds millions) sweeps with more blocks
template <bool WIDE>
inline int pa_grid_rt(const P2PDev &M) {
  return pa_grid<WIDE>() + (M.pool_cap > (1ull << 20) ? GRID_POOL_BIG - GRID_POOL : 0);
}
// DF: the deferred pipeline's variant (single wide engine): when the last window is staged (C.pdf) its records
// are written in rank order to the stage for k2_sdef and its children get provisional uids (no dispatch log
// here); the pool's provisional uids of the window before it are resolved as the pool is read.
template <bool DIST, bool WIDE, bool DF = false>
__global__ __launch_bounds__(TB) void k2_pa(const P2PDev M) {
  static_assert(!DF || WIDE, "deferred windows are the wide engine's");
  PH_BEGIN();
  BLK_T0();
  Ctl &C = *vec_ctl(M.C);
#ifdef NSGPU_PHASE_PROF
  const uint64_t c_win = C.windows;
#endif
  if (blockIdx.x == 0 && threadIdx.x == 0) {  // (k2_handle's hub-window handshake: this window's)
    C.hub_rdy = 0;
    C.hub_ser = 0;
  }
  // slot role: one thread per record of the last window — its gen-0 slots, then (single engine) its local
  // records (the dense list lrec), SL of them in each of the first NSGB blocks (roles are block-uniform:
  // a slot block's lanes past SL take part in its barriers only)
  constexpr uint32_t NSG = WIDE ? (uint32_t)SLOTG : (uint32_t)WCAP;
  constexpr uint32_t SL = DIST ? (uint32_t)TB : (uint32_t)PA_SLOT_LANES, NSGB = NSG / SL;
  const bool slot_block = blockIdx.x < NSGB;
  const bool slot_role = slot_block && threadIdx.x < SL;
  const uint64_t g = slot_block ? (uint64_t)blockIdx.x * SL + threadIdx.x
                                : NSG + (uint64_t)(blockIdx.x - NSGB) * TB + threadIdx.x;
  const uint32_t rrb = DIST ? (M.nranks * M.capx + TB - 1) / TB : 0u;  // remote-event blocks
  const bool remote_role = DIST && !slot_block && blockIdx.x < NSGB + rrb;
  // Everything this kernel reads of the run control and of the last window's slot, loaded at once:
  // these lines were written by k2_scan on another XCD, so every dependent level is a trip to memory.
  // (The slot arrays are WCAP long: a slot past the last window's size is loaded and ignored.)
  const uint32_t c_done = C.done, c_mode = C.mode, rt = C.rt, c_pvalid = C.pvalid, c_pW = C.pW, c_huid = C.huid;
  const uint32_t uid0 = C.puid0, c_plt = WIDE ? C.plt : 0u;
  const uint32_t c_prep = DIST ? C.prep : 0u;  // (with the rest: its test after the slot loads cost a second trip)
  const Red red0 = C.red[0], red1 = C.red[1];
  const uint64_t hts = C.hts, c_ptmin = C.ptmin, K0 = C.pK0, ilim = C.pinline_lim, c_P = C.P_end;
  const uint64_t c_span_t = WIDE ? C.span_t : 0;
  const uint32_t c_pdf = DF ? C.pdf : 0u;
  // partitioned sorted run: this window is a chunk (children, remote events and the pool stay pending)
  const bool drun = DIST && C.drun != 0;
  const uint64_t c_dr0 = DIST ? C.dr0 : 0, c_drW = DIST ? C.drW : 0, c_drg = DIST ? C.drg : 0;
  const uint64_t c_drlo = DIST ? C.drlo : ~0ull;
  const bool dtrim = DIST && C.dtrim != 0;  // a run ended after a cut group: its entries left outside the pool
  const uint64_t c_wn = DF ? C.windows : 0;  // (this window's index: the last one is c_wn - 1)
  // (branch-free, two loads into two registers: as one select of two branch loads the compiler reused one register,
  // and the second branch's address write waited for the first branch's load — s_waitcnt vmcnt(0) — so wave 0 sat a
  // whole trip on the run control before it issued the slot loads below)
  const int64_t look_a = M.lookahead[threadIdx.x < K_NKINDS ? threadIdx.x : 0u];
  const int64_t look_w = WIDE ? M.lookw[threadIdx.x >= K_NKINDS && threadIdx.x < 2 * K_NKINDS ? threadIdx.x - K_NKINDS : 0u]
                              : 0;
  const int64_t look_mine = threadIdx.x < K_NKINDS ? look_a : threadIdx.x < 2 * K_NKINDS ? look_w : 0;
  uint32_t xw_u[4] = {0, 0, 0, 0};  // (window c_wn - 2's uid base: the pool's provisional uids; all four
  if (DF) {                          //  loaded with the run control, picked once C.windows is back)
#pragma unroll
    for (int k = 0; k < 4; k++) xw_u[k] = C.winfo[k].uid0;
  }
  uint64_t spk = 0;
  uint4 si = make_uint4(0, 0, 0, 0);
  uint32_t ncr = 0, sctx = 0;
  // the first PFC children, field by field (an Ev array here was kept in scratch, and each child's scratch
  // store waited for its loads: one memory trip per child)
  uint64_t cts[PFC];
  uint32_t cctx[PFC], ckind[PFC], ca[PFC];
  uint4 cpk[PFC];
  constexpr int NPEND = 4;  // node-table claims a thread keeps pending (PFC children, or PPT pool entries)
  static_assert(PFC <= NPEND, "pending claims");
  NtClaim pend[NPEND];
#pragma unroll
  for (int q = 0; q < NPEND; q++) pend[q] = NtClaim{0, NOSRC, 0};
  // the record this slot-role thread appends: gen-0 slot g, or local record lrec[g - WCAP] (lrec holds
  // record indices from earlier windows past C.plt: loaded speculatively, always in range).  DF: the dense
  // local entry ldat (record, child counts, rel ts, parent) instead, and both parities' rank accumulators
  uint4 ldd = make_uint4((uint32_t)g, 0, 0, 0);
  uint32_t rk2[2] = {0, 0}, ninl0 = 0, lpd = 0;
  if (DF && WIDE && g >= (uint64_t)WCAP && slot_role) {
    ldd = M.ldat[g - WCAP];
    lpd = M.ldpd[g - WCAP];  // (its parent as a dense index: k2_sdef finds the parent's rank in LDS)
  }
  // (a speculative entry past the last window's records is followed too: clamped into the record space)
  const uint32_t rec =
      (WIDE && g >= (uint64_t)WCAP && slot_role) ? min(DF ? ldd.x : M.lrec[g - WCAP], (uint32_t)WTOT - 1u) : (uint32_t)g;
  if (slot_role) {  // the slot and its first children (the children first: a register copy of an early-arriving
    const uint32_t s = rec;  // slot field made the wave wait for it before the later loads were issued)
#pragma unroll
    for (int j = 0; j < PFC; j++) {  // (a child index past maxc loads the slot's last one: in range, ignored)
      const uint32_t sl = s * M.maxc + min((uint32_t)j, M.maxc - 1u);
      cts[j] = M.ch_ts[sl];
      cctx[j] = M.ch_ctx[sl];
      ckind[j] = M.ch_kind[sl];
      ca[j] = M.ch_a[sl];
      cpk[j] = *(const uint4 *)&M.ch_pkt[sl];
    }
    if (DF) {  // (branch-free: a branch here made the wave wait for these before issuing the child loads)
      const bool gz = g < (uint64_t)WCAP;
      const uint32_t *wr = (gz ? M.wrank : M.lrank - WCAP) + g;
      rk2[0] = wr[0];
      rk2[1] = wr[gz ? (uint32_t)WTOT : (uint32_t)LMAX];
      ninl0 = M.ninl[gz ? (uint32_t)g : 0u];  // (a local record's is not used)
    }
    spk = M.pwkey[s];
    si = M.sinfo[s];
    ncr = M.nchild[s];
    sctx = M.pwctx[s];
  }
  if (DIST) {
    if (blockIdx.x == 0 && threadIdx.x < M.nranks) x2hdr(M, M.x2_send, threadIdx.x)->n = 0;  // (X2 has sent them)
    if (c_prep) return;
  }
  // k2_sdef's flag, every window (its blocks only read it: a block may start after another finished)
  if (DF && g == 0)
    C.sflag = (c_done < 2 && c_mode < MODE_SORT && c_mode != MODE_RUN && c_pdf && c_pvalid)
                  ? 1u | (uint32_t)(((c_wn - 1) & 3) << 1) : 0u;
  if (c_done >= 2 || c_mode >= MODE_SORT) return;
  // the kinds' lookaheads in LDS (a per-child lookup of the kernel-argument table was a memory trip each)
  __shared__ int64_t s_look[2 * K_NKINDS];
  if (threadIdx.x < 2 * K_NKINDS) s_look[threadIdx.x] = look_mine;
  __syncthreads();
  if (slot_block) BLK_MARK(32, c_win);  // snapshot + slot loads issued (waits at first use)
  if (!slot_block && !remote_role) BLK_MARK(52, c_win);  // (pool blocks: the run control, the barrier)
  const bool run = c_mode == MODE_RUN;
  const bool partition = c_done == 0;
  Red &R = DIST ? x1hdr(M.x1_send, 0)->red : C.red[rt];
  WinBound b = drun ? drun_bound(C, c_drg) : window_bound(rt ? red0 : red1, WIDE && !run, c_span_t);
  // a pending host closure (nsgpu_p2p_advance) cuts the window at its key, like Simulator::Stop: the
  // window holds the device events before it, and the pipeline pauses for the host after the window
  bool hcap = false;
  uint64_t hrel = ~0ull;
  if (hts != ~0ull && !run) {
    if (hts < b.tmin || b.tmin == ~0ull) {
      b.bound = 0;  // (every device key is >= 4: uids start at 4)
      b.nbound = 0;
      b.lim = 0;
      hcap = true;
    } else if (hts - b.tmin <= b.span) {
      const uint64_t hk = ((hts - b.tmin) << 32) | c_huid;
      if (hk <= b.bound) {
        b.bound = hk;
        hcap = true;
        hrel = hts - b.tmin;
        b.nbound = hk < b.nbound ? hk : b.nbound;
        b.lim = hrel < b.lim ? hrel : b.lim;  // (a child at the host event's ts sorts after it)
      }
    }
  }
  if (!run && partition && g == 0) {
    publish_bound(C, b);
    if (WIDE && M.trace) C.tn0 = *M.trace_n;  // (the local records' trace uids are patched from here on)
    // the window's last timestamp (W_end, or the host event's): other children of this window can land
    // there with smaller uids than a DoForwardUp leaf its events schedule, so those leaves are queued
    // (K_FWD_UP_D), not run inline; a leaf of an earlier timestamp has every same-time event in the window
    // (a run chunk cut inside a same-ts group: that group's ts)
    const uint64_t edge = hcap ? hrel : (drun && drun_cuts_group(c_drg, C.drb_bound)) ? (c_drg >> 32) : b.span;
    C.split_lo = drun ? c_drlo : ~0ull;  // (a chunk continuing a cut group queues that group's leaves too)
    C.split_hi = edge;
    C.hrel = edge;
    C.hcap = hcap;
  }
  const uint32_t pW = c_pvalid ? c_pW : 0;
#ifndef PA_PPT
#define PA_PPT 2  // (4: config 4 149.5 M ev/s, 2: 153 M — twice the pool blocks, each half the claims and writes)
#endif
  constexpr int PPT = PA_PPT;  // (pool entries a thread reads a chunk)
  {  // a pool block past the pool's end (most of them: the pool holds a few thousand entries) has nothing to do
    const uint64_t pb = blockIdx.x - (uint64_t)(NSGB + rrb);
    if (!slot_block && !remote_role && partition && !run && !drun && !(DIST && dtrim && pb < (uint64_t)(WCAP / TB)) &&
        pb * TB * PPT >= c_P)
      return;
  }
#ifdef NSGPU_PHASE_PROF
  if (c_win == g_blk_win && blockIdx.x == 0 && threadIdx.x == 0) {  // (diagnostic: the window's inputs)
    g_phase[46] = c_P;
    g_phase[47] = pW;
    g_phase[48] = c_plt;
  }
#endif
  PH_MARK(0);
  uint64_t tmn = ~0ull, wnd = ~0ull, wndw = ~0ull, digest = 0;
  uint32_t xw_uid0 = xw_u[0];  // (window c_wn - 2's uid base: its provisional uids resolve in this kernel)
#pragma unroll
  for (int k = 1; k < 4; k++)
    if ((uint64_t)k == ((c_wn + 2) & 3)) xw_uid0 = xw_u[k];
  Stg st_pending{0, 0, 0};
  if (slot_block) {
    // ---- record `rec` of the last window: dispatch rank (log, digest), inline children, children -> pending
    const bool vs = slot_role && (g < (uint64_t)WCAP ? g < pW : (c_pvalid && g - WCAP < c_plt));
    const uint32_t s = rec;
    const bool loc = WIDE && g >= (uint64_t)WCAP;
    const bool stg = DF && c_pdf;  // the last window is staged for k2_sdef (deferred dispatch accounting)
    const uint64_t rel = (stg && loc) ? (uint64_t)ldd.z : spk >> 32;
    const uint64_t t = c_ptmin + rel;
    const uint32_t pn = (uint32_t)((c_wn - 1) & 1);  // (DF: the last window's parity)
    const uint32_t srank = pn ? rk2[1] : rk2[0];
    BLK_MARK(34, c_win);  // bound, publish_bound
    if (stg && vs && srank >= (uint32_t)NMAX) atomicOr(M.error, 256u);
    const bool sw = stg && vs && srank < (uint32_t)NMAX;  // the record is staged at its rank (k2_sdef logs it)
    if (sw) {
      // a provisional uid (a child of the window before) resolves now: k2_sdef ran for that window.  The
      // prefix's load is issued here and the stage is written after the children, so its trip overlaps theirs
      uint32_t ku = (uint32_t)spk;
      if (!loc && (ku & PROV)) {
        const uint32_t tag = (ku >> 30) & 1u;
        if (tag != (uint32_t)(c_wn & 1)) atomicOr(M.error, 256u);
        ku = xw_uid0 + M.cpt[(uint64_t)tag * NMAX + stg_pos(((ku & 0x3fffffffu) >> 8) % NMAX)] + (ku & 0xffu);
      }
      const uint32_t cc = loc ? ldd.y : (ncr | (ninl0 << 16));
      const uint32_t dn = loc ? pW + (uint32_t)(g - WCAP) : (uint32_t)g;  // (its dense index)
      st_pending = Stg{loc ? (rel << 32) : ((spk >> 32) << 32 | ku), (cc & 0x1ffu) | ((cc >> 16) << 9) | (dn << 18),
                       loc ? lpd : 0u};
      M.stx[stg_pos(srank)] = sctx;
    } else if (vs) {
      const uint64_t rk = K0 + si.x;
      digest += digest_term(rk, t, (uint32_t)spk);
      if (rk < M.log_cap) {
        M.log_ts[rk] = t;
        M.log_uid[rk] = (uint32_t)spk;
        M.log_ctx[rk] = sctx;
      }
    }
    // the slot's children in groups of PFC, one block allocation per group (block-uniform loop)
    const uint32_t nl = vs ? ncr : 0u;
    uint32_t ii = 0;
    for (uint32_t j0 = 0; __syncthreads_or(j0 < nl); j0 += PFC) {
      if (j0) {  // (the last group's claims: finished now, their atomics had a block allocation's time)
#pragma unroll
        for (int q = 0; q < PFC; q++) node_table_finish(M, C, pend[q]);
      }
      Ev ge[PFC];
      bool gin[PFC], gpk[PFC];
      uint32_t cw = 0, cf = 0;
#pragma unroll
      for (int q = 0; q < PFC; q++) {
        const uint32_t j = j0 + q;
        const bool has = j < nl;
        Ev e{0, 0, 0, 0, 0, Pkt{0, 0, 0, 0}};
        bool valid = false;
        if (has) {
          if (j0 == 0) {
            e = Ev{cts[q], 0, cctx[q], ckind[q], ca[q], Pkt{cpk[q].x, cpk[q].y, cpk[q].z, cpk[q].w}};
          } else {
            const uint32_t sl = s * M.maxc + j;
            e = Ev{M.ch_ts[sl], 0, M.ch_ctx[sl], M.ch_kind[sl], M.ch_a[sl], M.ch_pkt[sl]};
          }
          e.uid = stg ? prov_uid(c_wn - 1, srank, j) : uid0 + si.z + j;
          if ((e.kind & 0xffu) == K_FWD_UP) {  // leaf: dispatched inside its window (or never), not queued
            if (stg) {
              if (rel < ilim && srank < (uint32_t)NMAX) {  // (k2_sdef logs it after its group)
                if (ii) M.sleaf[(uint64_t)srank * M.maxc + ii] = make_uint2(e.ctx, j);
                else st_pending.par = e.ctx | (j << 24);  // (a gen-0 record's: local records have no leaves)
                ii++;
              }
            } else if (rel < ilim) {
              const uint64_t crk = K0 + si.y + ii;
              digest += digest_term(crk, t, e.uid);
              if (crk < M.log_cap) {
                M.log_ts[crk] = t;
                M.log_uid[crk] = e.uid;
                M.log_ctx[crk] = e.ctx;
              }
              ii++;
            }
          } else if (!WIDE || !(e.kind & LOCALBIT)) {  // (partitioned: a child on another rank's node goes there through X2)
            valid = partition && (!DIST || !(e.kind & REMOTEBIT));  // (remote Receives go through X2)
          }  // (a local record's child ran in the last window itself)
        }
        k2_classify<WIDE>(s_look, b, run || drun, valid, e, NOSRC, R, tmn, wnd, wndw, gin[q], gpk[q]);
        ge[q] = e;
        cw += gin[q];
        cf += gpk[q];
      }
      BLK_MARK(36, c_win);  // digest/log, classify (slot data arrived)
      uint32_t w0;
      uint64_t f0;
      block_alloc2<TB>(C, cw, cf, w0, f0);
      BLK_MARK(38, c_win);  // block allocation (atomics)
#pragma unroll
      for (int q = 0; q < PFC; q++) {
        pend[q] = k2_write(M, C, b, ge[q], NOSRC, gin[q], gpk[q], w0, f0);
        w0 += gin[q];
        f0 += gpk[q];
      }
      BLK_MARK(40, c_win);  // writes (node-table atomics)
    }
    if (sw) M.stage[stg_pos(srank)] = st_pending;  // (one stage: df_sdef(n - 1) was done with it before k2_pa(n + 1))
  } else if (DIST && remote_role) {
    // ---- remote events the last X2 brought (partitioned): record idx % capx from rank idx / capx
    if (partition) {
      const uint64_t idx = g - NSG;
      const uint32_t q = (uint32_t)(idx / M.capx), rec = (uint32_t)(idx % M.capx);
      // the record and its peer's count in one trip (the record loaded whether or not it is valid: in range)
      const uint32_t qc = q < M.nranks ? q : 0u;
      const uint32_t nq = x2hdr(M, M.x2_recv, qc)->n;
      Ev e = x2rec(M, M.x2_recv, qc)[rec];
      const bool valid = q < M.nranks && rec < nq;
      if (valid) e.kind &= ~REMOTEBIT;  // (its sender's mark: this rank owns it)
      else e = Ev{0, 0, 0, 0, 0, Pkt{0, 0, 0, 0}};
      bool gin, gpk;
      k2_classify<WIDE>(s_look, b, drun, valid, e, NOSRC, R, tmn, wnd, wndw, gin, gpk);
      uint32_t w0;
      uint64_t f0;
      block_alloc2<TB>(C, gin, gpk, w0, f0);
      pend[0] = k2_write(M, C, b, e, NOSRC, gin, gpk, w0, f0);
    }
  } else if (partition && !run && drun) {
    // ---- a partitioned run's chunk (the pool is not swept during the run: its reduction is folded below)
    const uint64_t pb = blockIdx.x - (uint64_t)(NSGB + rrb);
    if (pb < (uint64_t)(WCAP / TB)) drun_chunk<TB>(M, C, pb * TB + threadIdx.x, c_dr0, c_drW, c_drg);
  } else if (partition && !run) {
    // ---- the pool, in place: read (ts, uid, kind) of every slot; window events are copied out.
    // Chunks of PPT x TB entries per block (loads of a chunk all in flight), one allocation per chunk;
    // blocks past the pool's end returned above.
    const uint64_t P = c_P;
    const uint64_t pb = blockIdx.x - (uint64_t)(NSGB + rrb), npb = gridDim.x - (uint64_t)(NSGB + rrb);
    static_assert(PPT <= NPEND, "pending claims");
    // after a partitioned run that ended at a cut group, the first WCAP / TB of these blocks return its entries
    // left that are not in the pool (children / remote events of the run's window) to pending: window records or
    // parked, as the children above (then they sweep the pool too)
    if (DIST && dtrim && pb < (uint64_t)(WCAP / TB)) {
      for (uint64_t c0 = c_dr0 + pb * TB; __syncthreads_or(c0 < c_drW); c0 += (uint64_t)(WCAP / TB) * TB) {
        const uint64_t i = c0 + threadIdx.x;
        const bool valid = i < c_drW && M.rn_src[i] == NOSRC;
        Ev e{0, 0, 0, 0, 0, Pkt{0, 0, 0, 0}};
        if (valid) {
          const uint64_t k = M.rn_key[i];
          e = Ev{C.drb_tmin + (k >> 32), (uint32_t)k, M.rn_ctx[i], M.rn_kind[i], M.rn_a[i], M.rn_pkt[i]};
        }
        bool gin, gpk;
        k2_classify<WIDE>(s_look, b, false, valid, e, NOSRC, R, tmn, wnd, wndw, gin, gpk);
        uint32_t w0;
        uint64_t f0;
        block_alloc2<TB>(C, gin, gpk, w0, f0);
        node_table_finish(M, C, k2_write(M, C, b, e, NOSRC, gin, gpk, w0, f0));
      }
    }
    // the key fields only: most pool entries stay pending (the window entries' second load overlaps the block
    // allocation, and the pool's other 24 B a slot are not fetched for the rest).  A large pool takes several
    // chunks a block: the next chunk's keys are loaded before this one is classified (its trip overlaps this
    // chunk's allocation and writes)
    uint64_t nts[PPT];
    uint32_t nuid[PPT], nkind[PPT];
#pragma unroll
    for (int q = 0; q < PPT; q++) {
      const uint64_t i = pb * TB * PPT + (uint64_t)q * TB + threadIdx.x;
      nts[q] = TOMB;
      if (i < P) nts[q] = M.ev_ts[0][i], nuid[q] = M.ev_uid[0][i], nkind[q] = M.ev_kind[0][i];
    }
    for (uint64_t c0 = pb * TB * PPT; c0 < P; c0 += npb * TB * PPT) {  // block-uniform trip count
#pragma unroll
      for (int q = 0; q < PPT; q++) node_table_finish(M, C, pend[q]);  // (the last chunk's)
#pragma unroll
      for (int q = 0; q < PPT; q++) pend[q].c = NOSRC;
      Ev ge[PPT];
      bool gin[PPT], gpk[PPT];
      uint32_t cw = 0;
#pragma unroll
      for (int q = 0; q < PPT; q++) ge[q] = Ev{nts[q], nuid[q], 0, nkind[q], 0, Pkt{0, 0, 0, 0}};
#pragma unroll
      for (int q = 0; q < PPT; q++) {  // (the next chunk's keys)
        const uint64_t i = c0 + npb * TB * PPT + (uint64_t)q * TB + threadIdx.x;
        nts[q] = TOMB;
        if (i < P) nts[q] = M.ev_ts[0][i], nuid[q] = M.ev_uid[0][i], nkind[q] = M.ev_kind[0][i];
      }
      if (DF) {  // children the window before the last one parked: their uids resolve now (k2_sdef ran for it)
#pragma unroll
        for (int q = 0; q < PPT; q++) {
          const uint64_t i = c0 + (uint64_t)q * TB + threadIdx.x;
          const uint32_t u = ge[q].uid;
          if (ge[q].ts != TOMB && (u & PROV)) {
            const uint32_t tag = (u >> 30) & 1u;
            if (tag != (uint32_t)(c_wn & 1)) atomicOr(M.error, 256u);
            ge[q].uid = xw_uid0 + M.cpt[(uint64_t)tag * NMAX + stg_pos(((u & 0x3fffffffu) >> 8) % NMAX)] + (u & 0xffu);
            M.ev_uid[0][i] = ge[q].uid;
          }
        }
      }
#pragma unroll
      for (int q = 0; q < PPT; q++) {
        const uint64_t i = c0 + (uint64_t)q * TB + threadIdx.x;
        k2_classify<WIDE>(s_look, b, drun, ge[q].ts != TOMB, ge[q], (uint32_t)i, R, tmn, wnd, wndw, gin[q], gpk[q]);
        cw += gin[q];
        if (gin[q]) {  // the window entry's record (its loads overlap the block allocation below)
          ge[q].ctx = M.ev_ctx[0][i];
          ge[q].a = M.ev_a[0][i];
          ge[q].p = M.ev_pkt[0][i];
        }
      }
      uint32_t w0 = 0;
      uint64_t f0 = 0;
      if (__syncthreads_or(cw != 0)) block_alloc2<TB>(C, cw, 0u, w0, f0);  // (most chunks of a large pool: none)
#ifdef NSGPU_PHASE_PROF
      if (c_win == g_blk_win) {  // (diagnostic: pool entries taken, pool chunks swept)
        if (cw) atomicAdd((unsigned long long *)&g_phase[49], (unsigned long long)cw);
        if (threadIdx.x == 0) atomicAdd((unsigned long long *)&g_phase[50], 1ull);
      }
#endif
#pragma unroll
      for (int q = 0; q < PPT; q++) {
        const uint64_t i = c0 + (uint64_t)q * TB + threadIdx.x;
        pend[q] = k2_write(M, C, b, ge[q], (uint32_t)i, gin[q], false, w0, 0);
        w0 += gin[q];
      }
    }
  } else if (partition && run) {
    // ---- the next chunk of the sorted run: per-node slot tables, chunk bounds
    const uint64_t r0 = C.r0, rW = C.rW, rn = C.rnext;
    const uint32_t Wc = (uint32_t)(rn - r0);  // (run_chunk_end: at most WCAP)
    const uint64_t s = g - NSG;
    if (s == 0) {
      C.W = Wc;
      C.wbase = (uint32_t)r0;
      const uint64_t r1 = r0 + Wc;
      const uint64_t klo = M.wkey[r0] >> 32, khi = M.wkey[r1 - 1] >> 32;
      C.split_lo = (r0 > 0 && (M.wkey[r0 - 1] >> 32) == klo) ? klo : ~0ull;
      C.split_hi = (r1 < rW && (M.wkey[r1] >> 32) == khi) ? khi : C.hrel;
    }
    {  // (every lane: the claims of one node are aggregated over the wave)
      const bool on = s < Wc;
      const uint32_t kw = on ? M.wkind[r0 + s] : 0u;
      const uint32_t c = on ? lp_of(M, M.wctx[r0 + s], kw, M.wa[r0 + s]) : NOSRC;
      node_table_finish(M, C, node_table_claim_wave(M, (uint32_t)s, c, kw, on));
    }
  }
  PH_MARK(1);
  if (slot_block) BLK_MARK(42, c_win);
  if (!slot_block && !remote_role) BLK_MARK(54, c_win);  // (pool blocks: the sweep)
  if (drun && g == 0) {  // the pending set of the run's start and the run's entries (k_drun_start, k_drun_red)
    const uint64_t a = C.drn_tmin, w = C.drn_wend, st = C.drn_stopts;
    tmn = a < tmn ? a : tmn;
    wnd = w < wnd ? w : wnd;
    if (WIDE) {
      const uint64_t ww = C.drn_wendw;
      wndw = ww < wndw ? ww : wndw;
    }
    if (st != ~0ull) {
      R.stopts = st;
      R.stopuid = C.drn_stopuid;
    }
  }
  publish_min<TB, WIDE>(R, tmn, wnd, wndw);
  digest = wave_sum64(digest);
  {  // one digest atomic per block
    __shared__ uint64_t s_dg[TB / 64];
    if ((threadIdx.x & 63) == 0) s_dg[threadIdx.x >> 6] = digest;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint64_t dg = 0;
      for (int w = 0; w < TB / 64; w++) dg += s_dg[w];
      if (dg) atomicAdd((unsigned long long *)&C.digest, (unsigned long long)dg);
    }
  }
  // the node-table claims still pending (their atomics overlapped the reductions above)
#pragma unroll
  for (int q = 0; q < NPEND; q++) node_table_finish(M, C, pend[q]);
  PH_MARK(2);
  if (slot_block) BLK_MARK(44, c_win);  // publish_min, digest
  if (!slot_block && !remote_role) BLK_MARK(62, c_win);  // (pool blocks: publish_min, digest)
  BLK_REC(0, c_win);
}

// ---- k2_handle: holders ----
// The roles of k2_handle's blocks share one LDS buffer (holders: per-thread sort lists; hub blocks:
// the hub's list), so that every block of the launch is resident at once.
constexpr int K2_LDS_WORDS = HB * CH * 3;                // holders: sort lists (12 KB; >= HUBL * 3)
constexpr int K2_LDS_WORDS_W = K2_LDS_WORDS + HB * LQ * 4;  // wide engines: + local queues (28 KB)
static_assert(HUBL * 3 <= K2_LDS_WORDS, "hub list does not fit the shared buffer");
// Run control a window kernel reads, loaded once at its entry (all fields at once: one memory trip).
struct HCtl {
  uint64_t tmin, inline_lim, slo, shi;
  uint64_t lim;         // wide window: a TransmitComplete child with rel ts < lim is a local record (0: none)
  const int64_t *look;  // the kinds' lookaheads, then (wide) their wide lookaheads, in LDS (a child's lookup of
                        // the kernel-argument table was a dependent memory load each)
};
// Slot i0's window record, loaded ahead (speculatively at base 0; reloaded for a run chunk).
struct SlotPre {
  uint32_t widx, ctx, kind, a;
  uint64_t key;
  Pkt pkt;
};

// A local record's chain order packed into two words (lexicographic), the LKey compare only for a tie:
// word 1 = rel ts, local, the parent's rel ts; word 2 = a gen-0 parent's uid and the child index (exact:
// records tie only with themselves), or a local parent's: its parent's rel ts and class, and that one's
// uid or parent rel ts (clamped: a tie falls back to the LKey compare).
__device__ __forceinline__ uint64_t lk_word(const LKey &k) {
  const uint32_t r1 = k.rel[1] < 0x7fffffffu ? k.rel[1] : 0x7fffffffu;
  return ((uint64_t)k.rel[0] << 32) | 0x80000000u | r1;
}
__device__ __forceinline__ uint64_t lk_word2(const LKey &k) {
  if (k.depth == 1) return ((uint64_t)k.uid << 8) | k.j[0];
  const bool g2 = k.depth == 2;  // (the grandparent is the gen-0 ancestor)
  const uint32_t r2 = k.rel[2] < 0x7fffffffu ? k.rel[2] : 0x7fffffffu;
  // (a provisional uid, deferred windows: above every real one, squeezed into the field's top 2^21 values)
  const uint32_t nx = g2 ? ((k.uid & PROV) ? 0x3fe00000u | (k.uid & 0x1fffffu) : k.uid) : k.rel[3];
  return (1ull << 63) | ((uint64_t)r2 << 31) | ((g2 ? 0ull : 1ull) << 30) | (nx < 0x3fffffffu ? nx : 0x3fffffffu);
}
// The local record of child E.lj of record `par` (a same-node TransmitComplete inside a wide window, marked
// LOCALBIT by Emit::child): slot k of the caller's region (counter *cnt: LDS, shared by a holder block's
// threads, or a hub block's lane 0), written like a window record; its key holds the rel ts (its uid is
// assigned by k2_scan: uid0 + the parent's child prefix + j).  NOSRC: the region is full (error 32).
__device__ __forceinline__ uint32_t local_record(const P2PDev &M, const Emit &E, uint32_t par, uint64_t tmin,
                                                 uint32_t region, uint32_t *cnt, bool atomic, uint64_t par_key) {
  const uint32_t cap = region < (uint32_t)NHB ? (uint32_t)LR : (uint32_t)LRH;
  const uint32_t k = atomic ? atomicAdd(cnt, 1u) : (*cnt)++;
  if (k >= cap) {
    atomicOr(M.error, 32u);
    return NOSRC;
  }
  const uint32_t rec = region_base(region) + k;
  M.wkey[rec] = ((E.lts - tmin) << 32) | 0xffffffffull;
  M.wctx[rec] = E.lctx;
  M.wkind[rec] = K_TX_COMPLETE;
  M.wa[rec] = E.la;
  M.wpkt[rec] = Pkt{0, 0, 0, 0};
  M.wpar[rec] = par | ((uint32_t)E.lj << 24);
  // its chain for k2_rank: the parent's, one level up
  LKey x;
  if (par < LBASE) {  // (par_key: the gen-0 parent's window key, wkey[par])
    const uint64_t pk = par_key;
    x.rel[1] = (uint32_t)(pk >> 32);
    x.uid = (uint32_t)pk;
    x.depth = 1;
  } else {
    const LKey p = M.lkey[par - LBASE];
#pragma unroll
    for (int t = 0; t + 1 < LKD; t++) x.rel[t + 1] = p.rel[t];
#pragma unroll
    for (int t = 0; t + 1 < 16; t++) x.j[t + 1] = p.j[t];
    x.uid = p.uid;
    x.depth = p.depth + 1;
    if (x.depth >= (uint32_t)LKD) atomicOr(M.error, 32u);  // (create keeps chains shorter: Lx <= LKD tx_min)
  }
  x.rel[0] = (uint32_t)(E.lts - tmin);
  x.j[0] = (uint8_t)E.lj;
  x.pad[0] = x.pad[1] = 0;
  M.lkey[rec - LBASE] = x;
  M.lkw[rec - LBASE] = make_ulonglong2(lk_word(x), lk_word2(x));
  return rec;
}
// A node's pending local records, sorted by rel ts (ties: creation order = the parents' order); head qh.
// Each entry: rel ts, record, and the record's context and device (so running it reads no record field).
struct LQ4 {
  uint32_t *rel, *rec, *ctx, *dev;
  uint32_t stride;
  __device__ __forceinline__ void move(uint32_t to, uint32_t from) const {
    rel[to * stride] = rel[from * stride];
    rec[to * stride] = rec[from * stride];
    ctx[to * stride] = ctx[from * stride];
    dev[to * stride] = dev[from * stride];
  }
};
__device__ __forceinline__ void lq_push(const P2PDev &M, const LQ4 &q, uint32_t &qh, uint32_t &nq, uint32_t rel,
                                        uint32_t rec, uint32_t ctx, uint32_t dev) {
  if (nq == (uint32_t)LQ && qh > 0) {  // compact the consumed head away
    for (uint32_t i = qh; i < nq; i++) q.move(i - qh, i);
    nq -= qh;
    qh = 0;
  }
  if (nq == (uint32_t)LQ) {
    atomicOr(M.error, 32u);
    return;
  }
  uint32_t p = nq;
  while (p > qh && q.rel[(p - 1) * q.stride] > rel) {
    q.move(p, p - 1);
    p--;
  }
  q.rel[p * q.stride] = rel;
  q.rec[p * q.stride] = rec;
  q.ctx[p * q.stride] = ctx;
  q.dev[p * q.stride] = dev;
  nq++;
}

// Device state of the device a holder's or a hub's serial device pass is on, in registers.
struct DevCache {
  uint32_t d, busy, cnt, head, qmax, peer, peer_node, rkind;
  uint64_t bps;
  int64_t ifg, delay;
  uint32_t q[6];  // enq_packets, enq_bytes, drop_packets, drop_bytes, deq_packets, tx_packets
  __device__ __forceinline__ void flush(const P2PDev &M) {
    if (d == NOSRC) return;
    M.dev[d].busy = busy;
    M.dev[d].cnt = cnt;
    M.dev[d].head = head;
    uint32_t *w = reinterpret_cast<uint32_t *>(&M.dev[d].c);  // not rx_packets: the node pass adds it atomically
    *reinterpret_cast<uint4 *>(w) = make_uint4(q[0], q[1], q[2], q[3]);
    *reinterpret_cast<uint2 *>(w + 4) = make_uint2(q[4], q[5]);
  }
  __device__ __forceinline__ void load(const P2PDev &M, uint32_t dd) {
    d = dd;
    const DevRec dr = M.dev[d];
    busy = dr.busy;
    cnt = dr.cnt;
    head = dr.head;
    qmax = dr.qmax;
    bps = dr.bps;
    ifg = dr.ifg;
    delay = dr.delay;
    peer = dr.peer;
    peer_node = dr.peer_node;
    rkind = dr.rkind;
    const uint32_t *w = reinterpret_cast<const uint32_t *>(&M.dev[d].c);
    const uint4 a = *reinterpret_cast<const uint4 *>(w);
    const uint2 b2 = *reinterpret_cast<const uint2 *>(w + 4);
    q[0] = a.x, q[1] = a.y, q[2] = a.z, q[3] = a.w, q[4] = b2.x, q[5] = b2.y;
  }
};

// device_act with the device state in a register cache (the same steps, point-to-point-net-device.cc
// :206-269,462-518, queue.cc:61-97, drop-tail-queue.cc:83-100).
__device__ __forceinline__ void device_act_cached(const P2PDev &M, Emit &E, const Act &act, DevCache &D) {
  if (act.op == ACT_NONE) return;
  if (D.d != act.dev) {
    D.flush(M);
    D.load(M, act.dev);
  }
  const uint32_t d = act.dev;
  Pkt *qb = M.q_buf + (uint64_t)d * M.qcap;
  bool go = false;
  Pkt tx{0, 0, 0, 0};
  if (act.op == ACT_SEND) {
    trace_call(M, E, NSGPU_TR_IP_TX, d, act.p);
    Pkt p = act.p;
    p.size += 2;  // PppHeader
    if (D.cnt >= D.qmax) {
      trace_call(M, E, NSGPU_TR_DROP, d, p);
      D.q[2]++;
      D.q[3] += p.size;
    } else {
      trace_call(M, E, NSGPU_TR_ENQUEUE, d, p);
      D.q[0]++;
      D.q[1] += p.size;
      if (D.busy == 0) {
        if (D.cnt == 0) {
          tx = p;
        } else {
          qb[(D.head + D.cnt) % M.qcap] = p;
          tx = qb[D.head];
        }
        D.head = (D.head + 1) % M.qcap;
        trace_call(M, E, NSGPU_TR_DEQUEUE, d, tx);
        D.q[4]++;
        go = true;
      } else {
        qb[(D.head + D.cnt) % M.qcap] = p;
        D.cnt++;
      }
    }
  } else {  // ACT_KICK
    D.busy = 0;
    if (D.cnt > 0) {
      tx = qb[D.head];
      D.head = (D.head + 1) % M.qcap;
      D.cnt--;
      trace_call(M, E, NSGPU_TR_DEQUEUE, d, tx);
      D.q[4]++;
      go = true;
    }
  }
  if (go) {
    D.busy = 1;
    D.q[5]++;
    const int64_t txTime = seconds_to_ts(static_cast<double>(tx.size) * 8 / (double)D.bps);
    E.child(txTime + D.ifg, E.ctx, K_TX_COMPLETE, d, Pkt{0, 0, 0, 0});
    E.child(txTime + D.delay, D.peer_node, D.rkind, D.peer, tx);
  }
}

template <bool WIDE>
__device__ __forceinline__ void handle_node2(const P2PDev &M, Ctl &C, uint32_t i0, uint32_t W, uint32_t base, Red &R,
                                             uint32_t *lds, const HCtl &hc, SlotPre sp, uint32_t *lcnt_sh) {
  uint32_t *chs = lds;
  uint64_t *chk = reinterpret_cast<uint64_t *>(lds + HB * CH);
  uint64_t tmn = ~0ull, wnd = ~0ull, wndw = ~0ull;
  HStat hs{0, 0, 0, 0, false};
  if (base != 0 && i0 < W) {
    sp.ctx = M.wctx[base + i0];
    sp.kind = M.wkind[base + i0];
    sp.a = M.wa[base + i0];
    sp.key = M.wkey[base + i0];
    sp.pkt = M.wpkt[base + i0];
  }
  X1Acc xa{0, 0, 0};
  const uint32_t wi = i0 < W ? sp.widx : 1u;
  if (wi == NOHOLD) slot_done(M, i0, sp.key, 0, 0, xa);  // NetDevice::Start: dispatched, no children
  if (wi == 0) {  // the holder
    const uint32_t c = lp_of(M, sp.ctx, sp.kind, sp.a);
    // its own event's addressing, if a Receive, loaded beside the node table (the node's only event, or
    // one of them: used when it runs)
    DstHint h0{false, 0, 0};
    if ((sp.kind & 0xffu) == K_RECEIVE) h0 = DstHint{true, pkt_dst_node(M, sp.pkt), pkt_dst_slot(M, sp.pkt)};
    uint32_t n = 1;
    int32_t sink = -1;
    if (c < M.n_nodes) {
      n = M.node_tab[(uint64_t)c * NTAB];
      sink = M.sink_of_node[c];
    }
    if (n <= (uint32_t)CH) {  // (a hub's events are its hub block's)
      if (c < M.n_nodes) M.node_tab[(uint64_t)c * NTAB] = 0;
      const uint64_t key0 = sp.key;
      uint32_t *my = &chs[threadIdx.x * CH];
      uint64_t *mk = &chk[threadIdx.x * CH];
      my[0] = i0;
      mk[0] = key0;
      if (n > 1) {
        const uint32_t ns = n < (uint32_t)NSLOT ? n : (uint32_t)NSLOT;
        for (uint32_t j = 0; j < ns; j++) my[j] = M.node_tab[(uint64_t)c * NTAB + 1 + j];
        if (n > (uint32_t)NSLOT) {  // the rest: window entries of node c not in the table
          uint32_t m = NSLOT;
          for (uint32_t x = 0; x < W && m < n; x++)
            if (M.widx[x] >= (uint32_t)NSLOT && M.widx[x] != NOHOLD &&
                lp_of(M, M.wctx[base + x], M.wkind[base + x], M.wa[base + x]) == c)
              my[m++] = x;
        }
        for (uint32_t j = 0; j < n; j++) mk[j] = M.wkey[base + my[j]];
        for (uint32_t a = 1; a < n; a++) {  // insertion sort by key
          const uint32_t v = my[a];
          const uint64_t kv = mk[a];
          uint32_t bb = a;
          while (bb > 0 && mk[bb - 1] > kv) {
            my[bb] = my[bb - 1];
            mk[bb] = mk[bb - 1];
            bb--;
          }
          my[bb] = v;
          mk[bb] = kv;
        }
      }
      const uint64_t tmin = hc.tmin, inline_lim = hc.inline_lim, slo = hc.slo, shi = hc.shi;
      Emit E;
      E.ctx = c;
      E.ch_ts = M.ch_ts;
      E.ch_ctx = M.ch_ctx;
      E.ch_kind = M.ch_kind;
      E.ch_a = M.ch_a;
      E.ch_pkt = M.ch_pkt;
      E.lookahead = hc.look;
      E.lookw = WIDE ? hc.look + K_NKINDS : nullptr;
      E.tmn = ~0ull;
      E.wnd = ~0ull;
      E.wndw = ~0ull;
      E.lim_abs = WIDE && hc.lim ? tmin + hc.lim : 0;
      // the node's events in key order: its gen-0 window events (sorted above) merged with the local records
      // its own TransmitStarts make (a gen-0 event first at equal ts: its uid is older)
      uint32_t *qrel = lds + HB * CH * 3 + threadIdx.x;
      const LQ4 lq{qrel, qrel + HB * LQ, qrel + 2 * HB * LQ, qrel + 3 * HB * LQ, (uint32_t)HB};
      // the node's device state in registers across its events (every device step of a node's events is
      // on one of its own devices; the Receive's rx counter is not cached)
      DevCache D;
      D.d = NOSRC;
      uint32_t qh = 0, nq = 0, it = 0, ts0_it = 0, pending = 0;
      uint64_t cur_rel = 0;
      bool started = false;
      for (;;) {
        const bool hg = it < n, hl = WIDE && qh < nq;
        const uint64_t relg = hg ? (mk[it] >> 32) : ~0ull;
        const bool take_l = hl && (uint64_t)qrel[qh * HB] < relg;
        const uint64_t rel = take_l ? (uint64_t)qrel[qh * HB] : relg;
        if (started && rel > cur_rel && pending) {
          // flush the inline children of this node's gen-0 events at cur_rel (positions [ts0_it, it))
          for (uint32_t jt = ts0_it; jt < it; jt++) {
            const uint32_t xr = my[jt];
            const uint32_t ncr = M.nchild[xr];
            for (uint32_t j = 0; j < ncr; j++) {
              const uint32_t sl = xr * M.maxc + j;
              if ((E.ch_kind[sl] & 0xffu) != K_FWD_UP) continue;
              const uint32_t sa = E.ch_a[sl];  // DoForwardUp -> PacketSink::HandleRead
              if (M.app_flags[sa] & 2u) {
                M.appc[sa].rx_packets++;
                M.appc[sa].rx_bytes += E.ch_pkt[sl].size - 28;
              }
            }
          }
          pending = 0;
        }
        if (!hg && !hl) break;
        if (!started || rel > cur_rel) {
          ts0_it = it;
          cur_rel = rel;
          started = true;
        }
        uint32_t s, kw, a;
        Pkt pk{0, 0, 0, 0};
        uint64_t key = 0;
        DstHint hint{false, 0, 0};
        if (WIDE && take_l) {  // a local record: PointToPointNetDevice::TransmitComplete
          s = lq.rec[qh * HB];
          E.ctx = lq.ctx[qh * HB];
          a = lq.dev[qh * HB];
          qh++;
          kw = K_TX_COMPLETE;
          E.uid = s, E.tloc = true;
          E.demote = false;
        } else {
          s = my[it];
          key = mk[it];
          it++;
          if (s == i0) {  // (the holder's own event: loaded at entry)
            E.ctx = sp.ctx;
            kw = sp.kind;
            a = sp.a;
            pk = sp.pkt;
            hint = h0;
          } else {
            E.ctx = M.wctx[base + s];  // (Schedule calls inherit the event's context)
            kw = M.wkind[base + s];
            a = M.wa[base + s];
            pk = M.wpkt[base + s];
          }
          E.uid = (uint32_t)key, E.tloc = false;
          E.demote = rel == slo || rel == shi;
        }
        E.now = tmin + rel;
        E.slot0 = s * M.maxc;
        E.n = 0;
        E.trseq = 0;
        E.lj = -1;
        {  // run_event with the device step on the cached state
          const NodeOut o = node_part(M, E, kw, a, pk, sink, hs, true, hint);
          device_act_cached(M, E, o.act, D);
          if (o.xdrop) trace_te_drop(M, E, o.xdrop - 1, o.act.p);
          if (o.post.valid) E.child(o.post.delay, E.ctx, o.post.kind, o.post.a, Pkt{0, 0, 0, 0});
          hs.cancelled += o.cancelled;
        }
        uint32_t ni = 0;
        if (rel < inline_lim)
          for (uint32_t j = 0; j < E.n; j++) ni += (E.ch_kind[E.slot0 + j] & 0xffu) == K_FWD_UP;
        slot_done(M, s, key, E.n, ni, xa);
        pending += ni;
        if (WIDE && E.lj >= 0) {
          const uint32_t r2 = local_record(M, E, s, tmin, blockIdx.x, lcnt_sh, true, key);
          if (r2 != NOSRC) lq_push(M, lq, qh, nq, (uint32_t)(E.lts - tmin), r2, E.lctx, E.la);
        }
      }
      D.flush(M);
      tmn = E.tmn;
      wnd = E.wnd;
      wndw = E.wndw;
    }
  }
  publish_min<HB, WIDE>(R, tmn, wnd, wndw);
  x1_totals(M, xa);
  if (hs.stop) C.stop_seen = 1;
  // the counters summed over the wave first: one atomic per thread on one word serialised over the window (4,096
  // cancelled OnOff events at a dumbbell's 5 s: 37-54 us a window)
  // (only in a wave that has any: config 4's windows have none, and the sums unconditionally cost its holders
  // ~0.5 us a window — 152.3 -> 149.3 M ev/s, interleaved A/B in gpurun_out/r06ab2)
  if (__any((hs.cancelled | hs.ttl_drops | hs.no_route | hs.unreach | hs.icmp) != 0)) {
    const uint64_t cn = wave_sum64(hs.cancelled), td = wave_sum64(hs.ttl_drops), nr = wave_sum64(hs.no_route),
                   ur = wave_sum64(hs.unreach), ic = wave_sum64(hs.icmp);
    if ((threadIdx.x & 63) == 0) {
      if (cn) atomicAdd((unsigned long long *)&C.cancelled, (unsigned long long)cn);
      if (td) atomicAdd((unsigned long long *)&C.ttl_drops, (unsigned long long)td);
      if (nr) atomicAdd((unsigned long long *)&C.no_route, (unsigned long long)nr);
      if (ur) atomicAdd((unsigned long long *)&C.unreach, (unsigned long long)ur);
      if (ic) atomicAdd((unsigned long long *)&C.icmp, (unsigned long long)ic);
    }
  }
}

// ---- k2_handle: hub blocks ----
// Events whose node part touches no node state: TransmitComplete, and a Receive that IpForward
// sends on (its node is not the datagram's destination).
__device__ __forceinline__ bool stateless_event(const P2PDev &M, uint32_t c, uint32_t kind, const Pkt &p) {
  if (kind == K_TX_COMPLETE || kind == K_DEV_START) return true;  // (NetDevice::Start: no-op)
  if (kind != K_RECEIVE) return false;
  if (M.icmp && (p.ttl & 0xffu) <= 1u) return false;  // a TTL expiry sends an ICMP error: m_identification++
  return pkt_dst_node(M, p) != c;
}

__device__ __forceinline__ void bitonic_sort_lds(uint64_t *k, uint32_t *v, uint32_t n) {
  uint32_t P = 1;
  while (P < n) P <<= 1;
  for (uint32_t i = n + threadIdx.x; i < P; i += HB) k[i] = ~0ull;
  __syncthreads();
  for (uint32_t kk = 2; kk <= P; kk <<= 1)
    for (uint32_t j = kk >> 1; j > 0; j >>= 1) {
      for (uint32_t i = threadIdx.x; i < P; i += HB) {
        const uint32_t l = i ^ j;
        if (l > i) {
          const bool asc = (i & kk) == 0;
          const uint64_t a = k[i], bb = k[l];
          if ((a > bb) == asc) {
            k[i] = bb;
            k[l] = a;
            const uint32_t t = v[i];
            v[i] = v[l];
            v[l] = t;
          }
        }
      }
      __syncthreads();
    }
}

// ---- parallel device steps of one device (a hub whose device steps all use one queue) ----
// With c = the queue length while the device transmits and c = -1 while it is idle (idle implies an
// empty queue), Send is c -> min (c + 1, qmax) (c == qmax: Queue::Drop; c == -1: Enqueue + Dequeue +
// TransmitStart at once) and TransmitComplete is c -> c - 1 (a dequeue + TransmitStart if c >= 1).
// Maps of the form x -> clamp (x + a, lo, hi) are closed under composition, so a wave scan of the
// segments' composed maps gives every event its input state; a second scan of enqueue / dequeue counts
// gives the ring positions.  Results (traces, counters, children, state) equal the serial pass's.
struct CMap {
  int32_t a, lo, hi;
};
__device__ __forceinline__ int32_t clampi(int32_t x, int32_t l, int32_t h) { return x < l ? l : (x > h ? h : x); }
constexpr int32_t CBIG = 1 << 28;
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ CMap cmap_dpp(const CMap &x) {  // (rows / lanes without a source: the identity map)
  return CMap{__builtin_amdgcn_update_dpp(0, x.a, CTRL, ROWS, 0xf, false),
              __builtin_amdgcn_update_dpp(-CBIG, x.lo, CTRL, ROWS, 0xf, false),
              __builtin_amdgcn_update_dpp(CBIG, x.hi, CTRL, ROWS, 0xf, false)};
}
__device__ __forceinline__ CMap cmap_then(const CMap &f, const CMap &g) {  // g after f
  return CMap{f.a + g.a, clampi(f.lo + g.a, g.lo, g.hi), clampi(f.hi + g.a, g.lo, g.hi)};
}

// Returns false (nothing done) when the batch would reuse a ring slot (more enqueues than the ring
// holds beyond the queued packets): the serial pass runs instead.
// hops[j], hsl[j]: the op and the slot of the list's event j (hub_node gathered the lane's segment into LDS).
template <bool WIDE>
__device__ __forceinline__ bool hub_device_scan(const P2PDev &M, Emit &E, uint32_t c, uint32_t d, const uint32_t *gs,
                                const uint64_t *gk, uint32_t n, uint32_t j0s, uint32_t j1s, uint64_t tmin, HStat &hs,
                                X1Acc &xa, const uint8_t *hops, const uint16_t *hsl) {
  const int lane = threadIdx.x;
  const DevRec dr = M.dev[d];
  const int32_t qmax = (int32_t)dr.qmax;
  const uint32_t busy0 = dr.busy, cnt0 = dr.cnt, head0 = dr.head, qcap = M.qcap;
  const int32_t c0 = busy0 ? (int32_t)cnt0 : -1;
  const uint64_t bps = dr.bps;
  const int64_t ifg = dr.ifg, delay = dr.delay;
  const uint32_t peer = dr.peer, peer_node = dr.peer_node, rkind = dr.rkind;
  Pkt *qb = M.q_buf + (uint64_t)d * qcap;
  // pass A: the segment's composed map and its enqueue / dequeue counts
  CMap f{0, -CBIG, CBIG};
  for (uint32_t j = j0s; j < j1s; j++) {
    const uint32_t op = hops[j];
    if (op == ACT_SEND) f = cmap_then(f, CMap{1, -CBIG, qmax});
    else if (op == ACT_KICK) f = cmap_then(f, CMap{-1, -CBIG, CBIG});
  }
  // the lanes' inclusive composition by DPP (a lane without a source composes with the identity map)
  CMap inc = f;
  inc = cmap_then(cmap_dpp<0x111>(inc), inc);
  inc = cmap_then(cmap_dpp<0x112>(inc), inc);
  inc = cmap_then(cmap_dpp<0x114>(inc), inc);
  inc = cmap_then(cmap_dpp<0x118>(inc), inc);
  inc = cmap_then(cmap_dpp<0x142, 0xa>(inc), inc);
  inc = cmap_then(cmap_dpp<0x143, 0xc>(inc), inc);
  const CMap ex = cmap_dpp<0x138>(inc);  // (wave_shr:1: the exclusive one; lane 0 the identity)
  const int32_t cin = clampi(c0 + ex.a, ex.lo, ex.hi);
  const int32_t cfin = clampi(c0 + (int32_t)rl32((uint32_t)inc.a, 63), (int32_t)rl32((uint32_t)inc.lo, 63), (int32_t)rl32((uint32_t)inc.hi, 63));
  uint32_t ne = 0, nd = 0;
  {
    int32_t x = cin;
    for (uint32_t j = j0s; j < j1s; j++) {
      const uint32_t op = hops[j];
      if (op == ACT_SEND) {
        if (x < qmax) ne++;
        if (x == -1) nd++;
        x = x + 1 < qmax ? x + 1 : qmax;
      } else if (op == ACT_KICK) {
        if (x >= 1) nd++;
        x -= 1;
      }
    }
  }
  const uint32_t ebefore = wave_exscan32(ne, lane), dbefore = wave_exscan32(nd, lane);
  const uint32_t dtot = rl32(dbefore + nd, 63), etot = rl32(ebefore + ne, 63);
  if (cnt0 + etot > qcap) return false;
  // pass B1: enqueued packets into the ring (before any TransmitComplete reads one).  The lane's segment in
  // batches: the slots from LDS (hsl), the batch's packets loaded at once (one memory trip a batch, not one an
  // event: the loop's ring stores kept the next event's loads behind them)
  constexpr int B1B = WIDE ? 1 : 8;  // (the wide kernel has no registers to spare)
  {
    int32_t x = cin;
    uint32_t e = ebefore;
    for (uint32_t jb = j0s; jb < j1s; jb += B1B) {
      Pkt pb[B1B];
      uint32_t qi[B1B];
#pragma unroll
      for (int u = 0; u < B1B; u++) {  // (the state walk over the batch's ops: which enqueue, where)
        const uint32_t j = jb + (uint32_t)u;
        qi[u] = NOSRC;
        if (j < j1s) {
          const uint32_t op = hops[j];
          if (op == ACT_SEND) {
            if (x >= 0 && x < qmax) qi[u] = (head0 + cnt0 + e) % qcap;
            if (x < qmax) e++;
            x = x + 1 < qmax ? x + 1 : qmax;
          } else if (op == ACT_KICK) {
            x -= 1;
          }
        }
      }
#pragma unroll
      for (int u = 0; u < B1B; u++)
        if (qi[u] != NOSRC) pb[u] = M.hx[hsl[jb + u]].p;
#pragma unroll
      for (int u = 0; u < B1B; u++)
        if (qi[u] != NOSRC) {
          Pkt p = pb[u];
          p.size += 2;
          qb[qi[u]] = p;
        }
    }
  }
  __syncthreads();
  // pass B2: traces, counters, TransmitStart children, trailing children (B2B events a batch: their records and
  // ring reads in one memory trip)
  constexpr int B2B = WIDE ? 1 : 4;
  uint32_t q0 = 0, q1 = 0, q2 = 0, q3 = 0, q4 = 0, q5 = 0;
  {
    int32_t x = cin;
    uint32_t dq = dbefore;
    for (uint32_t jb = j0s; jb < j1s; jb += B2B) {
      uint32_t sb[B2B], ri[B2B];
      uint64_t kb[B2B];
      HubEv hb[B2B];
      Pkt tq[B2B];
      {
        int32_t xx = x;
        uint32_t dd = dq;
#pragma unroll
        for (int u = 0; u < B2B; u++) {  // (each TransmitComplete's dequeue position, from the ops)
          const uint32_t j = jb + (uint32_t)u;
          ri[u] = NOSRC;
          sb[u] = 0;
          if (j < j1s) {
            sb[u] = hsl[j];
            const uint32_t op = hops[j];
            if (op == ACT_SEND) {
              if (xx == -1) dd++;
              xx = xx + 1 < qmax ? xx + 1 : qmax;
            } else if (op == ACT_KICK) {
              if (xx >= 1) ri[u] = (head0 + dd++) % qcap;
              xx -= 1;
            }
          }
        }
      }
#pragma unroll
      for (int u = 0; u < B2B; u++) {
        const uint32_t j = jb + (uint32_t)u;
        if (j < j1s) {
          kb[u] = gk[j];
          hb[u] = M.hx[sb[u]];
        }
        if (ri[u] != NOSRC) tq[u] = qb[ri[u]];
      }
#pragma unroll
      for (int u = 0; u < B2B; u++) {
        const uint32_t j = jb + (uint32_t)u;
        if (j >= j1s) break;
        const uint32_t s = sb[u];
        const uint64_t key = kb[u];
        const HubEv &h = hb[u];
        E.ctx = h.ctx;
        E.now = tmin + (key >> 32);
        E.slot0 = s * M.maxc;
        E.n = h.n;
        E.uid = (uint32_t)key, E.tloc = false;
        E.trseq = h.seq;
        E.demote = false;
        hs.cancelled += h.cancelled;
        bool go = false;
        Pkt tx{0, 0, 0, 0};
        if (h.op == ACT_SEND) {
          trace_call(M, E, NSGPU_TR_IP_TX, d, h.p);
          Pkt p = h.p;
          p.size += 2;  // PppHeader
          if (x >= qmax) {
            trace_call(M, E, NSGPU_TR_DROP, d, p);
            q2++;
            q3 += p.size;
          } else {
            trace_call(M, E, NSGPU_TR_ENQUEUE, d, p);
            q0++;
            q1 += p.size;
            if (x == -1) {  // Enqueue + Dequeue: the packet leaves at once
              tx = p;
              trace_call(M, E, NSGPU_TR_DEQUEUE, d, tx);
              q4++;
              dq++;
              go = true;
            }
          }
          x = x + 1 < qmax ? x + 1 : qmax;
        } else if (h.op == ACT_KICK) {
          if (x >= 1) {
            tx = tq[u];
            trace_call(M, E, NSGPU_TR_DEQUEUE, d, tx);
            q4++;
            dq++;
            go = true;
          }
          x -= 1;
        }
        if (go) {
          q5++;
          const int64_t txTime = seconds_to_ts(static_cast<double>(tx.size) * 8 / (double)bps);
          E.child(txTime + ifg, h.ctx, K_TX_COMPLETE, d, Pkt{0, 0, 0, 0});
          E.child(txTime + delay, peer_node, rkind, peer, tx);
        }
        if (h.xdrop) trace_te_drop(M, E, h.xdrop - 1, h.p);
        if (h.pkind) E.child(h.pdelay, h.ctx, h.pkind, h.pa, Pkt{0, 0, 0, 0});
        slot_done(M, s, key, E.n, 0, xa);
      }
    }
  }
  q0 = wave_sum32(q0), q1 = wave_sum32(q1), q2 = wave_sum32(q2), q3 = wave_sum32(q3), q4 = wave_sum32(q4),
  q5 = wave_sum32(q5);
  if (lane == 0) {
    M.dev[d].busy = cfin >= 0 ? 1u : 0u;
    M.dev[d].cnt = cfin >= 0 ? (uint32_t)cfin : 0u;
    M.dev[d].head = (head0 + dtot) % qcap;
    uint32_t *w = reinterpret_cast<uint32_t *>(&M.dev[d].c);  // not rx_packets: the node pass adds it atomically
    const uint4 a = *reinterpret_cast<const uint4 *>(w);
    const uint2 b2 = *reinterpret_cast<const uint2 *>(w + 4);
    *reinterpret_cast<uint4 *>(w) = make_uint4(a.x + q0, a.y + q1, a.z + q2, a.w + q3);
    *reinterpret_cast<uint2 *>(w + 4) = make_uint2(b2.x + q4, b2.y + q5);
  }
  return true;
}

// ---- hub windows of the narrow engines: the stateless node parts by the slots' own threads ----
// A hub block is one wave; its pass over the hub's node parts took 64 events a round, each round a chain of
// four dependent memory trips (slot -> record -> destination -> route): ~160 us for a run chunk of 4,000 events
// at a dumbbell router.  Those node parts touch no node state, so in a window with hubs every slot's own thread
// of the holder blocks runs its event's, if it is a hub's (the same steps as hub_node's lanes), into hx, and marks
// the slot's hub (hub_mark: the hub block's list is then one array's scan); a node part that touches node state is
// left to the hub block (HOP_SER, hub_ser), which runs those serially in key order as before.  Each holder block
// then signals the hub blocks (hub_rdy), which wait for all NHB before they read hx / hub_mark (lower block indices
// are dispatched first: the holder blocks are running or done when a hub block waits).
constexpr uint32_t HOP_SER = 0xffu;  // hx[s].op: the node part is the hub block's (serial, node state)
__device__ __forceinline__ uint32_t *hub_mark(const P2PDev &M) { return M.hub_slot + (uint64_t)NHUB * WCAP; }
__device__ __forceinline__ void hub_help(const P2PDev &M, Ctl &C, uint32_t i0, uint32_t W, uint32_t base,
                                         const HCtl &hc, SlotPre &sp) {
  uint32_t mark = NOSRC;
  bool ser = false;
  HStat hs{0, 0, 0, 0, false};
  if (i0 < W) {
    if (base != 0) {  // (a run chunk's records: handle_node2 reloads them too)
      sp.ctx = M.wctx[base + i0];
      sp.kind = M.wkind[base + i0];
      sp.a = M.wa[base + i0];
      sp.key = M.wkey[base + i0];
      sp.pkt = M.wpkt[base + i0];
    }
    const uint32_t kind = sp.kind & 0xffu;
    if (sp.widx != NOHOLD) {
      const uint32_t c = lp_of(M, sp.ctx, sp.kind, sp.a);
      uint32_t dn = 0, ds = 0;  // (a Receive's addressing, loaded with the node's count)
      if (kind == K_RECEIVE) {
        dn = pkt_dst_node(M, sp.pkt);
        ds = pkt_dst_slot(M, sp.pkt);
      }
      if (c < M.n_nodes && M.node_tab[(uint64_t)c * NTAB] > (uint32_t)CH) {
        mark = c;
        const bool sl = kind == K_TX_COMPLETE || kind == K_DEV_START ||
                        (kind == K_RECEIVE && !(M.icmp && (sp.pkt.ttl & 0xffu) <= 1u) && dn != c);
        if (!sl) {
          ser = true;
          M.hx[i0].op = HOP_SER;
        } else {
          Emit E;
          E.now = hc.tmin + (sp.key >> 32);
          E.uid = (uint32_t)sp.key, E.tloc = false;
          E.trseq = 0;
          HubEv h{ACT_NONE, 0, Pkt{0, 0, 0, 0}, 0, 0, 0, 0, 0, 0, 0, sp.ctx, 0};
          if (kind == K_TX_COMPLETE) {
            h.op = ACT_KICK;
            h.dev = sp.a;
          } else if (kind == K_RECEIVE) {  // PointToPointNetDevice::Receive -> Ipv4L3Protocol::Receive -> IpForward
            const uint32_t out = route_at(M, c, ds);
            atomicAdd(&M.dev[sp.a].c.rx_packets, 1u);
            Pkt p = sp.pkt;
            p.size -= 2;
            trace_call(M, E, NSGPU_TR_RX, sp.a, p);
            trace_call(M, E, NSGPU_TR_IP_RX, sp.a, p);
            if (out == 0xffffffffu) {
              hs.no_route++;
              trace_ip_drop(M, E, sp.a, p);
            } else {
              p.ttl -= 1;
              if (p.ttl == 0) {  // (ICMP off: a stateless event)
                hs.ttl_drops++;
                trace_ip_drop(M, E, out, Pkt{p.app, p.ipid, p.size, 1u});
              } else {
                h.op = ACT_SEND;
                h.dev = out;
                h.p = p;
              }
            }
          }
          h.seq = E.trseq;
          M.hx[i0] = h;
        }
      }
    }
    hub_mark(M)[i0] = mark;
  }
  const uint64_t nr = wave_sum64(hs.no_route), td = wave_sum64(hs.ttl_drops);
  const bool anyser = __ballot(ser) != 0;
  if (threadIdx.x == 0) {
    if (nr) atomicAdd((unsigned long long *)&C.no_route, (unsigned long long)nr);
    if (td) atomicAdd((unsigned long long *)&C.ttl_drops, (unsigned long long)td);
    if (anyser) atomicOr(&C.hub_ser, 1u);
    __threadfence();  // (HB = one wave: the block's writes, released before the signal)
    atomicAdd(&C.hub_rdy, 1u);
  }
}

// A hub node's window events, by one block: (1) its events in key order (slot order in a sorted run
// chunk; otherwise at most HUBL of them, bitonic-sorted in LDS) into the block's global scratch list;
// (2a) node parts without node state (TransmitComplete; Receive -> IpForward) in parallel; (2b) the
// other node parts serially in key order; (3) the device steps and trailing children serially in key
// order, the device state in registers.  Node parts never read device state and device steps never
// read node state (node_part), so this is the sequential order's result.
template <bool WIDE>
__device__ __forceinline__ void hub_node(const P2PDev &M, Ctl &C, uint32_t c, uint32_t W, uint32_t base, bool sorted, Red &R,
                         uint32_t hb, uint32_t *lds, const HCtl &hc, uint32_t *lcnt_sh, bool helped) {
  const int lane = threadIdx.x;
  const uint64_t below = (1ull << lane) - 1ull;
  uint64_t *gk = M.hub_key + (uint64_t)hb * WCAP;
  uint32_t *gs = M.hub_slot + (uint64_t)hb * WCAP;
  HUB_T0();
  uint32_t ser = 1;  // (helped: some hub event's node part is left to its hub block)
  if (!WIDE && helped) {  // the holder blocks ran the stateless node parts (hub_help): wait for all of them
    if (lane == 0)
      while (__hip_atomic_load(&C.hub_rdy, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (uint32_t)NHB)
        __builtin_amdgcn_s_sleep(2);
    __syncthreads();
    __threadfence();
    ser = __hip_atomic_load(&C.hub_ser, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    HUB_MARK(22);  // (the wait for the holder blocks)
  }
  // 1. the node's window events, in slot order (HSB batches of HB window entries a memory trip; the wide
  //    kernel has no registers to spare: one there).  helped: the slots marked with this hub, HMB batches a trip
  constexpr int HSB = WIDE ? 1 : 4;
  constexpr int HMB = 8;
  uint32_t n = 0;
  if (!WIDE && helped) {
    for (uint32_t x0 = 0; x0 < W; x0 += HB * HMB) {
      uint32_t hm[HMB];
      uint64_t hk[HMB];
#pragma unroll
      for (int u = 0; u < HMB; u++) {  // (the keys loaded with the marks: in range, used for this hub's)
        const uint32_t x = x0 + (uint32_t)(u * HB) + lane;
        hm[u] = x < W ? hub_mark(M)[x] : NOSRC;
        hk[u] = M.wkey[base + (x < W ? x : 0u)];
      }
#pragma unroll
      for (int u = 0; u < HMB; u++) {
        const uint32_t x = x0 + (uint32_t)(u * HB) + lane;
        const bool m = hm[u] == c;
        const uint64_t bm = __ballot(m);
        if (m) {
          const uint32_t p = n + (uint32_t)__popcll(bm & below);
          gs[p] = x;
          gk[p] = hk[u];
        }
        n += (uint32_t)__popcll(bm);
      }
    }
  }
  for (uint32_t x0 = 0; x0 < ((!WIDE && helped) ? 0u : W); x0 += HB * HSB) {
    uint32_t bi[HSB], bc[HSB], bk[HSB], ba[HSB];
#pragma unroll
    for (int u = 0; u < HSB; u++) {
      const uint32_t x = x0 + (uint32_t)(u * HB) + lane;
      bi[u] = NOHOLD;
      if (x < W) {
        bi[u] = M.widx[x];
        bc[u] = M.wctx[base + x];
        bk[u] = M.wkind[base + x];
        ba[u] = M.wa[base + x];
      }
    }
#pragma unroll
    for (int u = 0; u < HSB; u++) {
      const uint32_t x = x0 + (uint32_t)(u * HB) + lane;
      const bool m = x < W && bi[u] != NOHOLD && lp_of(M, bc[u], bk[u], ba[u]) == c;
      const uint64_t bm = __ballot(m);
      if (m) {
        const uint32_t p = n + (uint32_t)__popcll(bm & below);
        gs[p] = x;
        gk[p] = M.wkey[base + x];
      }
      n += (uint32_t)__popcll(bm);
    }
  }
  __syncthreads();
  if (!sorted) {  // (n <= HUBL here: a larger hub makes its window a sorted run, k2_pa)
    uint64_t *lk = reinterpret_cast<uint64_t *>(lds);
    uint32_t *ls = lds + 2 * HUBL;
    for (uint32_t j = lane; j < n; j += HB) {
      lk[j] = gk[j];
      ls[j] = gs[j];
    }
    __syncthreads();
    bitonic_sort_lds(lk, ls, n);
    for (uint32_t j = lane; j < n; j += HB) {
      gk[j] = lk[j];
      gs[j] = ls[j];
    }
    __syncthreads();
  }
  HUB_MARK(24);  // (the window scan and the sort)
  const uint64_t tmin = hc.tmin, inline_lim = hc.inline_lim, slo = hc.slo, shi = hc.shi;
  const int32_t sink = M.sink_of_node[c];
  Emit E;
  E.ctx = c;
  E.ch_ts = M.ch_ts;
  E.ch_ctx = M.ch_ctx;
  E.ch_kind = M.ch_kind;
  E.ch_a = M.ch_a;
  E.ch_pkt = M.ch_pkt;
  E.lookahead = hc.look;
  E.lookw = WIDE ? hc.look + K_NKINDS : nullptr;
  E.tmn = ~0ull;
  E.wnd = ~0ull;
  E.wndw = ~0ull;
  E.lim_abs = WIDE && hc.lim ? hc.tmin + hc.lim : 0;
  E.lj = -1;
  E.demote = false;
  HStat hs{0, 0, 0, 0, false};
  // the passes go through the list 64 events at a time: every lane loads one event's record into
  // LDS (one memory round trip per batch), then the serial work reads LDS
  // (LDS words: key [0, 2 HB), slot [2 HB, 3 HB), then the hub events at 11 HB)
  uint64_t *b_key = reinterpret_cast<uint64_t *>(lds);  // [HB]
  uint32_t *b_s = lds + 2 * HB;
  HubEv *b_h = reinterpret_cast<HubEv *>(lds + 11 * HB);  // [HB]
  // 2. node parts: the stateless ones (TransmitComplete, NetDevice::Start, Receive -> IpForward: rx
  //    counter, MacRx trace, route, TTL) by their own lane, the others serially by lane 0 in key order.
  //    NBT batches of HB events per round: each dependent step (slot -> record -> destination -> route)
  //    is one memory trip for all of them.
  constexpr int NBT = WIDE ? 1 : 2;  // (the wide kernel has no registers to spare: its hubs stay one batch a round)
  if (!WIDE && helped) {
    // the holder blocks ran the stateless ones (hub_help); the rest (HOP_SER), serially by lane 0 in key order
    for (uint32_t j0 = 0; ser && j0 < n; j0 += HB) {
      const uint32_t j = j0 + lane;
      uint32_t op = 0;
      if (j < n) op = M.hx[gs[j]].op;
      uint64_t m = __ballot(j < n && op == HOP_SER);
      if (lane == 0) {
        while (m) {
          const uint32_t q = j0 + (uint32_t)(__ffsll((unsigned long long)m) - 1);
          m &= m - 1;
          const uint32_t s = gs[q];
          const uint64_t key = gk[q], rel = key >> 32;
          const uint32_t kw = M.wkind[base + s], a = M.wa[base + s], ctx = M.wctx[base + s];
          const Pkt pk = M.wpkt[base + s];
          E.ctx = ctx;
          E.now = tmin + rel;
          E.slot0 = s * M.maxc;
          E.n = 0;
          E.uid = (uint32_t)key, E.tloc = false;
          E.trseq = 0;
          E.demote = rel == slo || rel == shi;
          const NodeOut o = node_part(M, E, kw, a, pk, sink, hs, true);
          uint32_t ni = 0;
          for (uint32_t jj = 0; jj < E.n; jj++) ni += (M.ch_kind[E.slot0 + jj] & 0xffu) == K_FWD_UP;
          M.hx[s] = HubEv{o.act.op, o.act.dev, o.act.p, o.post.delay, o.post.valid ? o.post.kind : 0u, o.post.a, E.n,
                          E.trseq, o.cancelled ? 1u : 0u, ni, ctx, o.xdrop};
        }
      }
      __syncthreads();
    }
  } else {
    uint64_t *c_key = reinterpret_cast<uint64_t *>(lds);  // [HB * NBT]
    uint32_t *c_s = lds + 2 * HB * NBT, *c_kind = lds + 3 * HB * NBT, *c_a = lds + 4 * HB * NBT,
             *c_ctx = lds + 6 * HB * NBT;
    Pkt *c_pkt = reinterpret_cast<Pkt *>(lds + 7 * HB * NBT);  // [HB * NBT]
    static_assert(11 * HB * NBT <= K2_LDS_WORDS, "hub node-part batch does not fit the shared buffer");
    for (uint32_t j0 = 0; j0 < n; j0 += HB * NBT) {
      uint32_t s_[NBT], kw_[NBT], a_[NBT], ctx_[NBT], dn_[NBT], ds_[NBT], out_[NBT];
      uint64_t key_[NBT];
      Pkt p_[NBT];
#pragma unroll
      for (int u = 0; u < NBT; u++) {
        const uint32_t j = j0 + (uint32_t)(u * HB) + lane;
        if (j < n) {
          s_[u] = gs[j];
          key_[u] = gk[j];
        }
      }
#pragma unroll
      for (int u = 0; u < NBT; u++) {
        const uint32_t j = j0 + (uint32_t)(u * HB) + lane;
        if (j < n) {
          kw_[u] = M.wkind[base + s_[u]];
          a_[u] = M.wa[base + s_[u]];
          ctx_[u] = M.wctx[base + s_[u]];
          p_[u] = M.wpkt[base + s_[u]];
        }
      }
#pragma unroll
      for (int u = 0; u < NBT; u++) {  // (stateless_event's and route_of's addressing)
        const uint32_t j = j0 + (uint32_t)(u * HB) + lane;
        dn_[u] = ds_[u] = 0;
        if (j < n && (kw_[u] & 0xffu) == K_RECEIVE) {
          dn_[u] = pkt_dst_node(M, p_[u]);
          ds_[u] = pkt_dst_slot(M, p_[u]);
        }
      }
#pragma unroll
      for (int u = 0; u < NBT; u++) {
        const uint32_t j = j0 + (uint32_t)(u * HB) + lane;
        out_[u] = 0xffffffffu;
        if (j < n && (kw_[u] & 0xffu) == K_RECEIVE && dn_[u] != c) out_[u] = route_at(M, c, ds_[u]);
      }
      // stateless_event, with the destination loaded above; the others' positions as wave masks (lane 0
      // visits only those: a scan of every position's flag in LDS cost ~80 ns an event)
      bool sl_[NBT];
      uint64_t ser_[NBT];
#pragma unroll
      for (int u = 0; u < NBT; u++) {
        const uint32_t j = j0 + (uint32_t)(u * HB) + lane;
        const uint32_t kind = kw_[u] & 0xffu;
        sl_[u] = j < n && (kind == K_TX_COMPLETE || kind == K_DEV_START ||
                           (kind == K_RECEIVE && !(M.icmp && (p_[u].ttl & 0xffu) <= 1u) && dn_[u] != c));
        ser_[u] = __ballot(j < n && !sl_[u]);
      }
#pragma unroll
      for (int u = 0; u < NBT; u++) {
        const uint32_t j = j0 + (uint32_t)(u * HB) + lane;
        if (j >= n) continue;
        const uint32_t s = s_[u], kw = kw_[u], a = a_[u], ctx = ctx_[u], bq = (uint32_t)(u * HB) + lane;
        const uint64_t key = key_[u];
        Pkt p = p_[u];
        const uint32_t kind = kw & 0xffu;
        const bool sl = sl_[u];
        c_ctx[bq] = ctx;
        c_s[bq] = s;
        c_key[bq] = key;
        c_kind[bq] = kw;
        c_a[bq] = a;
        c_pkt[bq] = p;
        if (sl) {
          E.now = tmin + (key >> 32);
          E.uid = (uint32_t)key, E.tloc = false;
          E.trseq = 0;
          HubEv h{ACT_NONE, 0, Pkt{0, 0, 0, 0}, 0, 0, 0, 0, 0, 0, 0, ctx, 0};
          if (kind == K_TX_COMPLETE) {
            h.op = ACT_KICK;
            h.dev = a;
          } else if (kind == K_RECEIVE) {  // PointToPointNetDevice::Receive -> Ipv4L3Protocol::Receive -> IpForward
            atomicAdd(&M.dev[a].c.rx_packets, 1u);
            p.size -= 2;
            trace_call(M, E, NSGPU_TR_RX, a, p);
            trace_call(M, E, NSGPU_TR_IP_RX, a, p);
            const uint32_t out = out_[u];
            if (out == 0xffffffffu) {
              hs.no_route++;
              trace_ip_drop(M, E, a, p);
            } else {
              p.ttl -= 1;
              if (p.ttl == 0) {  // (ICMP off: stateless_event)
                hs.ttl_drops++;
                trace_ip_drop(M, E, out, Pkt{p.app, p.ipid, p.size, 1u});
              } else {
                h.op = ACT_SEND;
                h.dev = out;
                h.p = p;
              }
            }
          }
          h.seq = E.trseq;
          M.hx[s] = h;
        }
      }
      __syncthreads();
#ifdef NSGPU_PHASE_PROF
      const uint64_t ser_t0 = __builtin_amdgcn_s_memrealtime();
#endif
      uint64_t any = 0;
#pragma unroll
      for (int u = 0; u < NBT; u++) any |= ser_[u];
      if (lane == 0 && any) {
#ifdef NSGPU_PHASE_PROF
        atomicAdd((unsigned long long *)&g_phase[30], (unsigned long long)(n - j0 < (uint32_t)(HB * NBT) ? n - j0 : (uint32_t)(HB * NBT)));
#endif
#pragma unroll 1
        for (int u = 0; u < NBT; u++) {
          uint64_t m = 0;
#pragma unroll
          for (int k = 0; k < NBT; k++) m = k == u ? ser_[k] : m;  // (a select chain: no indexed registers)
          while (m) {
            const uint32_t q = (uint32_t)(u * HB) + (uint32_t)(__ffsll((unsigned long long)m) - 1);
            m &= m - 1;
#ifdef NSGPU_PHASE_PROF
            atomicAdd((unsigned long long *)&g_phase[29], 1ull);
#endif
            const uint32_t s = c_s[q];
            const uint64_t rel = c_key[q] >> 32;
            E.ctx = c_ctx[q];
            E.now = tmin + rel;
            E.slot0 = s * M.maxc;
            E.n = 0;
            E.uid = (uint32_t)c_key[q], E.tloc = false;
            E.trseq = 0;
            E.demote = rel == slo || rel == shi;
            const NodeOut o = node_part(M, E, c_kind[q], c_a[q], c_pkt[q], sink, hs, true);
            uint32_t ni = 0;
            for (uint32_t jj = 0; jj < E.n; jj++) ni += (M.ch_kind[E.slot0 + jj] & 0xffu) == K_FWD_UP;
            M.hx[s] = HubEv{o.act.op, o.act.dev, o.act.p, o.post.delay, o.post.valid ? o.post.kind : 0u, o.post.a, E.n,
                            E.trseq, o.cancelled ? 1u : 0u, ni, c_ctx[q], o.xdrop};
          }
        }
      }
      __syncthreads();
#ifdef NSGPU_PHASE_PROF
      if (lane == 0) atomicAdd((unsigned long long *)&g_phase[31], (unsigned long long)(__builtin_amdgcn_s_memrealtime() - ser_t0));
#endif
    }
  }
  HUB_MARK(25);  // (node parts)
  // 3. device steps and trailing children.  When every device step of the hub is on one device and no
  //    event has inline children (a dumbbell router's burst), the steps are resolved in parallel
  //    (hub_device_scan); otherwise serially in key order with the device state in registers.
  const uint32_t mseg = (n + HB - 1) / HB, j0s = lane * mseg, j1s = j0s + mseg < n ? j0s + mseg : n;
  uint32_t dmin = NOSRC, dmax = 0, inl = 0;
  // the lane's segment: devices, inline flags, and its ops into LDS for the device scan (HSO events a
  // memory trip; past the serial pass's batch arrays)
  uint8_t *hops = reinterpret_cast<uint8_t *>(lds + 2048);
  uint16_t *hsl = reinterpret_cast<uint16_t *>(lds);  // (the slots, for the device scan's batches)
  static_assert(2048 + WCAP / 4 <= K2_LDS_WORDS && WCAP <= 4096, "hub ops / slots do not fit the shared buffer");
  constexpr int HSO = WIDE ? 1 : 8;
  for (uint32_t j = j0s; j < j1s; j += HSO) {
    uint32_t sl[HSO], op[HSO], dv[HSO], pd[HSO];
#pragma unroll
    for (int u = 0; u < HSO; u++)
      if (j + u < j1s) sl[u] = gs[j + u];
#pragma unroll
    for (int u = 0; u < HSO; u++)
      if (j + u < j1s) {
        const HubEv *hp = M.hx + sl[u];
        op[u] = hp->op;
        dv[u] = hp->dev;
        pd[u] = hp->pad;
      }
#pragma unroll
    for (int u = 0; u < HSO; u++)
      if (j + u < j1s) {
        hops[j + u] = (uint8_t)op[u];
        hsl[j + u] = (uint16_t)sl[u];
        if (op[u] != ACT_NONE) {
          dmin = dv[u] < dmin ? dv[u] : dmin;
          dmax = dv[u] > dmax ? dv[u] : dmax;
        }
        inl |= pd[u];
      }
  }
  HUB_MARK(23);  // (the segments' ops into LDS)
  dmin = (uint32_t)wave_min64(dmin);
  dmax = (uint32_t)wave_max64(dmax);
  inl = (uint32_t)wave_sum32(inl != 0 ? 1u : 0u) != 0 ? 1u : 0u;
  // (not in a wide window: a TransmitStart there makes a local record the scan cannot place)
  bool fast = dmin != NOSRC && dmin == dmax && inl == 0 && (!WIDE || hc.lim == 0) && M.dev[dmin].qmax >= 1 &&
              !(M.dev[dmin].busy == 0 && M.dev[dmin].cnt != 0);
  X1Acc xa{0, 0, 0};
  if (fast) fast = hub_device_scan<WIDE>(M, E, c, dmin, gs, gk, n, j0s, j1s, tmin, hs, xa, hops, hsl);
  if (!fast) {
    DevCache D;
    D.d = NOSRC;
    uint32_t ts0_it = 0, pending = 0;
    uint64_t cur_rel = 0;
    bool started = false;
    // local records (wide windows) of this hub, lane 0's queue: merged with the gen-0 events by rel ts
    __shared__ uint32_t hq_rel[LQ], hq_rec[LQ], hq_ctx[LQ], hq_dev[LQ];
    const LQ4 hq{hq_rel, hq_rec, hq_ctx, hq_dev, 1u};
    uint32_t qh = 0, nq = 0;
    // the inline DoForwardUp leaves of this node's gen-0 events at cur_rel (positions [ts0_it, it)), before
    // anything at a later ts
    auto flush = [&](uint32_t it) {
      for (uint32_t jt = ts0_it; jt < it; jt++) {
        const uint32_t xr = gs[jt];
        const uint32_t ncr = M.nchild[xr];
        for (uint32_t jj = 0; jj < ncr; jj++) {
          const uint32_t sl = xr * M.maxc + jj;
          if ((M.ch_kind[sl] & 0xffu) != K_FWD_UP) continue;
          const uint32_t sa = M.ch_a[sl];
          if (M.app_flags[sa] & 2u) {
            M.appc[sa].rx_packets++;
            M.appc[sa].rx_bytes += M.ch_pkt[sl].size - 28;
          }
        }
      }
      pending = 0;
    };
    auto new_local = [&](uint32_t par) {
      if (!WIDE || E.lj < 0) return;
      const uint32_t r2 = local_record(M, E, par, tmin, NHB + hb, lcnt_sh, false, par < LBASE ? M.wkey[par] : 0ull);
      if (r2 != NOSRC) lq_push(M, hq, qh, nq, (uint32_t)(E.lts - tmin), r2, E.lctx, E.la);
    };
    // the local records due before rel (at equal ts the gen-0 event first); `it`: the next gen-0 position
    auto run_locals = [&](uint64_t rel, uint32_t it) {
      while (WIDE && qh < nq && (uint64_t)hq_rel[qh] < rel) {
        const uint64_t lrel = hq_rel[qh];
        if (started && lrel > cur_rel && pending) flush(it);
        if (!started || lrel > cur_rel) {
          ts0_it = it;
          cur_rel = lrel;
          started = true;
        }
        const uint32_t s = hq_rec[qh], la = hq_dev[qh];
        E.ctx = hq_ctx[qh++];
        E.now = tmin + lrel;
        E.slot0 = s * M.maxc;
        E.n = 0;
        E.uid = s, E.tloc = true;
        E.trseq = 0;
        E.demote = false;
        E.lj = -1;
        device_act_cached(M, E, Act{ACT_KICK, la, Pkt{0, 0, 0, 0}}, D);  // TransmitComplete
        slot_done(M, s, 0, E.n, 0, xa);
        new_local(s);
      }
    };
    for (uint32_t j0 = 0; j0 <= n; j0 += HB) {
      const uint32_t j = j0 + lane;
      if (j < n) {
        const uint32_t s = gs[j];
        b_s[lane] = s;
        b_key[lane] = gk[j];
        b_h[lane] = M.hx[s];
      }
      __syncthreads();
      if (lane == 0) {
        const uint32_t nb = n - j0 < (uint32_t)HB ? n - j0 : (uint32_t)HB;
        for (uint32_t q = 0; q <= nb; q++) {
          const uint32_t it = j0 + q;
          if (q == nb && it < n) break;  // (the next batch continues; the final flush runs at it == n)
          const uint64_t key = it < n ? b_key[q] : ~0ull;
          const uint64_t rel = it < n ? (key >> 32) : ~0ull;
          run_locals(rel, it);
          if (started && rel > cur_rel && pending) flush(it);
          if (it == n) break;
          if (!started || rel > cur_rel) {
            ts0_it = it;
            cur_rel = rel;
            started = true;
          }
          const uint32_t s = b_s[q];
          const HubEv h = b_h[q];
          E.ctx = h.ctx;
          E.now = tmin + rel;
          E.slot0 = s * M.maxc;
          E.n = h.n;
          E.uid = (uint32_t)key, E.tloc = false;
          E.trseq = h.seq;
          E.demote = rel == slo || rel == shi;
          E.lj = -1;
          hs.cancelled += h.cancelled;
          device_act_cached(M, E, Act{h.op, h.dev, h.p}, D);
          if (h.xdrop) trace_te_drop(M, E, h.xdrop - 1, h.p);
          if (h.pkind) E.child(h.pdelay, h.ctx, h.pkind, h.pa, Pkt{0, 0, 0, 0});
          const uint32_t ni = rel < inline_lim ? h.pad : 0u;
          slot_done(M, s, key, E.n, ni, xa);
          pending += ni;
          new_local(s);
        }
      }
      __syncthreads();
    }
    if (lane == 0) D.flush(M);
  }
  HUB_MARK(26);  // (device steps: the parallel scan or the serial pass)
  publish_min<HB, WIDE>(R, E.tmn, E.wnd, E.wndw);
  x1_totals(M, xa);
  const uint64_t nr = wave_sum64(hs.no_route), td = wave_sum64(hs.ttl_drops), cn = wave_sum64(hs.cancelled),
                 ur = wave_sum64(hs.unreach), ic = wave_sum64(hs.icmp);
  const bool stop = __ballot(hs.stop) != 0;
  if (lane == 0) {
    if (stop) C.stop_seen = 1;
    if (cn) atomicAdd((unsigned long long *)&C.cancelled, (unsigned long long)cn);
    if (td) atomicAdd((unsigned long long *)&C.ttl_drops, (unsigned long long)td);
    if (nr) atomicAdd((unsigned long long *)&C.no_route, (unsigned long long)nr);
    if (ur) atomicAdd((unsigned long long *)&C.unreach, (unsigned long long)ur);
    if (ic) atomicAdd((unsigned long long *)&C.icmp, (unsigned long long)ic);
  }
  __syncthreads();
  HUB_MARK(27);  // (publish, totals)
#ifdef NSGPU_PHASE_PROF
  if (threadIdx.x == 0) atomicAdd((unsigned long long *)&g_phase[28], 1ull);
#endif
}

// ---- k2_handle: pool maintenance (tombstones, free slots, fresh children -> pool) ----
__device__ __forceinline__ void maintain(const P2PDev &M, Ctl &C, uint32_t mb, bool run, bool handle, uint32_t W, uint64_t nfree,
                         uint64_t nF, uint64_t Pe) {
  const uint64_t tstride = (uint64_t)NMB * HB;
  if (!run) {
    for (uint64_t w0 = (uint64_t)mb * HB; w0 < W; w0 += tstride) {  // wave-uniform
      const uint64_t s = w0 + threadIdx.x;
      const uint32_t src = s < W ? M.wsrc[s] : NOSRC;
      const bool f = src != NOSRC;
      if (f) M.ev_ts[0][src] = TOMB;
      const uint64_t p = wave_alloc64(&C.npush, f);
      if (f) M.fstack[nfree + p] = src;
    }
    if (!handle) {  // the window becomes a sorted run: its slot tables are not used
      const uint64_t ws = W < (uint32_t)WCAP ? W : (uint32_t)WCAP;
      for (uint64_t s = (uint64_t)mb * HB + threadIdx.x; s < ws; s += tstride) {
        const uint32_t c = M.wctx[s];
        if (c < M.n_nodes) M.node_tab[(uint64_t)c * NTAB] = 0;
      }
    }
  }
  for (uint64_t j = (uint64_t)mb * HB + threadIdx.x; j < nF; j += tstride) {
    const uint64_t dst = j < nfree ? (uint64_t)M.fstack[nfree - 1 - j] : Pe + (j - nfree);
    if (dst < M.pool_cap) {
      M.ev_ts[0][dst] = M.f_ts[j];
      M.ev_uid[0][dst] = M.f_uid[j];
      M.ev_ctx[0][dst] = M.f_ctx[j];
      M.ev_kind[0][dst] = M.f_kind[j];
      M.ev_a[0][dst] = M.f_a[j];
      M.ev_pkt[0][dst] = M.f_pkt[j];
    } else {
      atomicOr(M.error, 1u);
    }
  }
}

// WIDE: the single engine's wide windows (local records: k2_rank places them after the handlers).
// Partitioned wide windows, after k2_handle: region bx's local records (its count in lcnt) into this rank's X1Loc
// list, compacted in region order (each block's offset: the prefix of the region counts, all loaded in one trip —
// no allocation atomic).  (Inside k2_handle this code made the kernel spill 1.3 KB of scratch a lane.)
__global__ __launch_bounds__(HB) void k_xlcompact(const P2PDev M) {
  static_assert(NLR <= 2 * HB, "two region counts a lane");
  const Ctl &C = *M.C;
  const uint32_t hdl = C.hdl, tid = threadIdx.x, bx = blockIdx.x;
  const uint64_t lim = C.lim_rel;
  const uint32_t a0 = M.lcnt[tid], a1 = tid + HB < (uint32_t)NLR ? M.lcnt[tid + HB] : 0u;
  // the region's first HB records, loaded with the counts (speculatively: a region holds at least HB, so the
  // indices are in range; the counts decide which are written)
  static_assert(LR >= HB && LRH >= HB, "a region's first HB records");
  const uint32_t rb = region_base(bx);
  ulonglong2 w = M.lkw[rb + tid - LBASE];
  uint32_t nc = M.nchild[rb + tid] | (M.ninl[rb + tid] << 16), anc = M.lkey[rb + tid - LBASE].uid, wp = M.wpar[rb + tid];
  if (!hdl || !lim) return;  // (uniform over the block)
  // every region's compact base (exclusive prefix of the counts: region tid in e0, region tid + HB in e1), for
  // this block's records and their local parents' rows
  uint32_t e0 = a0, e1 = a1;
  e0 = wave_incscan32(e0);  // (HB = one wave)
  e1 = wave_incscan32(e1);
  e1 += rl32(e0, HB - 1);
  e0 -= a0;
  e1 -= a1;
  const uint32_t lb = bx < (uint32_t)HB ? __shfl(e0, (int)bx) : __shfl(e1, (int)(bx - HB));
  const uint32_t cnt = bx < (uint32_t)HB ? __shfl(a0, (int)bx) : __shfl(a1, (int)(bx - HB));
  if (bx == 0) {
    const uint32_t tot = wave_sum32(a0 + a1);
    if (tid == 0) {
      x1hdr(M.x1_send, 0)->L = tot < (uint32_t)XLCAP ? tot : (uint32_t)XLCAP;
      if (tot > (uint32_t)XLCAP) atomicOr(M.error, 64u);
    }
  }
  if (!cnt) return;
  X1Loc *xl = x1loc(M);
  uint64_t lts = 0;  // (the largest rel ts: the window's last dispatch time may be a local record's)
  for (uint32_t k0 = 0; k0 < cnt; k0 += HB) {  // (block-uniform: the parents' bases come by shuffles)
    const uint32_t k = k0 + tid;
    const bool in = k < cnt && lb + k < (uint32_t)XLCAP;
    const uint32_t rec = rb + (k < cnt ? k : tid);
    if (k0) {  // (past the region's first HB: loaded here)
      w = M.lkw[rec - LBASE];
      nc = M.nchild[rec] | (M.ninl[rec] << 16), anc = M.lkey[rec - LBASE].uid, wp = M.wpar[rec];
    }
    // the parent's accumulator row for k_dfin2 (a gen-0 slot, or WCAP + a local parent's compact index: its
    // region's base + its place in the region), with the child index of wpar.  (The shuffles run on every
    // lane: a lane shuffling from one that is off would read zero.)
    const uint32_t p = wp & 0xffffffu;
    const bool lpar = p >= (uint32_t)LBASE && p < (uint32_t)WTOT;
    const uint32_t off = lpar ? p - LBASE : 0u;
    const uint32_t r = off < (uint32_t)(NHB * LR) ? off / LR : NHB + (off - NHB * LR) / LRH;
    const uint32_t pe0 = __shfl(e0, (int)(r & (HB - 1))), pe1 = __shfl(e1, (int)(r & (HB - 1)));
    const uint32_t prow = lpar ? (uint32_t)WCAP + (r < (uint32_t)HB ? pe0 : pe1) + (p - region_base(r)) : p;
    if (in) {
      xl[lb + k] = X1Loc{w.x, w.y, nc, rec, anc, prow | (wp & 0xff000000u)};
      const uint64_t t = w.x & 0xffffffff00000000ull;
      lts = t > lts ? t : lts;
    }
  }
  lts = wave_max64(lts);
  if (tid == 0 && lts) atomicMax((unsigned long long *)&x1hdr(M.x1_send, 0)->lastkey, (unsigned long long)lts);
}

// XL: the partitioned wide engine's variant (k_gtile's accumulators zeroed; every region count written, for
// k_xlcompact): a separate instantiation, so that the single engine's kernel has none of that code.
template <bool WIDE, bool XL = false>
__global__ __launch_bounds__(HB) void k2_handle(const P2PDev M) {
  __shared__ uint64_t lds64[(WIDE ? K2_LDS_WORDS_W : K2_LDS_WORDS) / 2];
  uint32_t *lds = reinterpret_cast<uint32_t *>(lds64);
  PH_BEGIN();
  Ctl &C = *vec_ctl(M.C);
  BLK_T0();
#ifdef NSGPU_PHASE_PROF
  const uint64_t c_win = C.windows;
#endif
  // the run control and (holder blocks) the slot's record, all loaded at once
  const uint32_t c_done = C.done, c_mode = C.mode, W = C.W, c_wbase = C.wbase, c_fr = C.force_run, rt = C.rt,
                 c_nhub = C.nhub;
  const uint32_t c_drun = M.dist ? C.drun : 0u;  // a partitioned run's chunk: key order, hubs in slot order
  __shared__ int64_t s_look[2 * K_NKINDS];
  const HCtl hc{C.tmin, C.inline_lim, C.split_lo, C.split_hi, C.lim_rel, s_look};
  const uint32_t lt_ = threadIdx.x;  // (loaded now, stored in LDS just before the block's first barrier)
  const int64_t look_mine = lt_ < K_NKINDS ? M.lookahead[lt_] : (WIDE && lt_ < 2 * K_NKINDS ? M.lookw[lt_ - K_NKINDS] : 0);
  const uint64_t c_wn = C.windows;
  __shared__ uint32_t s_lcnt;  // local records this block made (its region's count, wide windows)
  if (threadIdx.x == 0) s_lcnt = 0;
  const uint64_t c_nfree = C.nfree, c_nF = C.nF, c_Pe = C.P_end;
  const uint32_t bx = blockIdx.x;
  SlotPre sp{1u, 0, 0, 0, 0};
  if (bx < (uint32_t)NHB) {
    const uint32_t i0 = bx * HB + threadIdx.x;
    sp = SlotPre{M.widx[i0], M.wctx[i0], M.wkind[i0], M.wa[i0], M.wkey[i0], M.wpkt[i0]};
  }
  if (M.dist && bx == 0 && threadIdx.x == 0) C.dtrim = 0;  // (k2_pa returned a trimmed run's rest to pending)
  // partitioned: every rank's X0 payload (window candidates, hub flag): a window some rank cannot hold
  // becomes a partitioned sorted run (the host's drun_sort, k_drun_first) before anything of it runs, on every rank
  bool ovf = false;
  if (M.dist) {  // (one lane per rank: HB = one wave)
    const uint32_t q = threadIdx.x;
    bool o = false;
    if (q < M.nranks) {
      const uint4 x = reinterpret_cast<const uint4 *>(M.x0_recv)[q];
      o = x.x > (uint32_t)WCAP || x.z != 0;
    }
    ovf = __ballot(o) != 0;
  }
  if (c_done || c_mode >= MODE_SORT || ovf) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      C.rk_go = 0;  // (k2_rank: nothing to rank or account)
      if (c_done == 1) C.done = 2;  // the final window is appended
      if (M.dist) {
        C.hdl = 0;  // (k_gtile / k_dfin2: nothing ran)
        if (!c_done && c_mode < MODE_SORT) C.mode = MODE_CUT;
      }
    }
    return;
  }
  if (M.dist && bx == 0 && threadIdx.x == 0) {  // the window k_dfin2 finishes and the next k2_pa appends
    C.hdl = 1;
    C.pK0 = C.K;
    C.puid0 = C.uid;
    C.ptmin = hc.tmin;
    C.pinline_lim = hc.inline_lim;
    C.pW = W;
    C.pvalid = 1;
    X1Hdr *h = x1hdr(M.x1_send, 0);
    h->W = W;
    h->needc = c_Pe > 65536 && C.live * 4 < c_Pe;  // this rank's pool wants a compaction
  }
  const bool run = c_mode == MODE_RUN;
  const uint32_t base = run ? c_wbase : 0;
  const bool handle = run || (W <= (uint32_t)WCAP && !c_fr);
  Red &R = M.dist ? x1hdr(M.x1_send, 0)->red : C.red[rt];
  if (WIDE && bx == 0 && threadIdx.x == 0) {  // what k2_rank ranks and accounts (its bookkeeping rewrites C.W ...)
    C.rk_W = W;
    C.rk_go = 2u | ((handle && !run) ? 1u : 0u) | (run ? 4u : 0u);  // 2: formed; 1: ranked; 4: a sorted run's chunk
    C.rk_win = c_wn;
    C.rk_lim = hc.lim;
  }
  PH_MARK(8);
  if (lt_ < 2 * K_NKINDS) s_look[lt_] = look_mine;
  __syncthreads();  // (s_lcnt, s_look)
  const bool helped = !WIDE && c_nhub != 0;  // (a window with hubs: the holder blocks help the hub blocks first)
  if (bx < (uint32_t)NHB) {
    if (handle) {
      if (helped) hub_help(M, C, bx * HB + threadIdx.x, W, base, hc, sp);
      handle_node2<WIDE>(M, C, bx * HB + threadIdx.x, W, base, R, lds, hc, sp, &s_lcnt);
    }
  } else if (bx < (uint32_t)(NHB + NHUB)) {
    if (handle) {
      const uint32_t hb = bx - NHB;
      const uint32_t nh = c_nhub < (uint32_t)MAXHUB ? c_nhub : (uint32_t)MAXHUB;
      for (uint32_t h = hb; h < nh; h += NHUB)
        hub_node<WIDE>(M, C, M.hub_list[h], W, base, run || c_drun != 0, R, hb, lds, hc, &s_lcnt, helped);
    }
  } else if (bx < (uint32_t)K2_GRID_W) {
    if constexpr (XL) {  // k_gtile's accumulators for this window (k_dfin2 read the last window's: local
      uint64_t *A = reinterpret_cast<uint64_t *>(M.gacc);  // records' uids take their parents' child prefixes)
      for (uint32_t i = (bx - (NHB + NHUB)) * HB + threadIdx.x; i < 2u * (uint32_t)NACC; i += NMB * HB) A[i] = 0;
    }
    maintain(M, C, bx - (NHB + NHUB), run, handle, W, c_nfree, c_nF, c_Pe);
  } else {
    if (!run && handle && !M.dist) rank_tile(M, C, bx - K2_GRID_W, wrank_of(M, c_wn));  // (keys known before the handlers run)
  }
  if (WIDE && (hc.lim || XL) && bx < (uint32_t)NLR) {  // this block's local region count (k2_rank / k2_scan /
    __syncthreads();                                       //  k_xlcompact read it; written even when 0: the
    const uint32_t cap = bx < (uint32_t)NHB ? (uint32_t)LR : (uint32_t)LRH;  // deferred pipeline keeps no reset)
    const uint32_t cnt = s_lcnt < cap ? s_lcnt : cap;
    if (threadIdx.x == 0) M.lcnt[bx] = cnt;
  }
  PH_MARK(9);
  BLK_REC(1, c_win);
}

// The local regions' prefix (NLR + 1 entries) into LDS from each thread's region count v (M.lcnt[thread],
// 0 past NLR); every thread of the block calls it.
template <int NT>
__device__ __forceinline__ void local_prefix(uint32_t v, uint32_t *pre) {
  static_assert(NT >= NLR && NLR <= 128, "one thread per region, two waves");
  __shared__ uint32_t s_w0;
  v = wave_incscan32(v);  // (inclusive wave scan)
  if (threadIdx.x == 63) s_w0 = v;
  __syncthreads();
  if (threadIdx.x >= 64) v += s_w0;
  if (threadIdx.x < (uint32_t)NLR) pre[threadIdx.x + 1] = v;
  if (threadIdx.x == 0) pre[0] = 0;
  __syncthreads();
}
// Record index -> dense index (gen-0 slot, or W + its region's prefix + its offset in the region).
__device__ __forceinline__ uint32_t dense_of(uint32_t rec, uint32_t W, const uint32_t *pre) {
  if (rec < LBASE) return rec;
  const uint32_t off = rec - LBASE;
  if (off < (uint32_t)(NHB * LR)) return W + pre[off / LR] + off % LR;
  const uint32_t o2 = off - (uint32_t)(NHB * LR);
  return W + pre[NHB + o2 / LRH] + o2 % LRH;
}
// ---- k2_rank (wide engines): every record's rank in the window's dispatch order, after the handlers ----
// All pairs of the window's records (gen-0 and local) by their chains (LKey): compare level by level —
// rel ts, then a gen-0 record before a local one, gen-0 ancestors by uid; chains that reach the same gen-0
// ancestor are ordered by the child index just below the first level where they part.
constexpr int RKT = 256;   // rows (threads) and columns per tile
constexpr int RK_GRID = 1024;
// a before b (distinct records)
__device__ __forceinline__ bool lk_before(const LKey &a, const LKey &b) {
#pragma unroll
  for (int t = 0; t < LKD; t++) {
    if (a.rel[t] != b.rel[t]) return a.rel[t] < b.rel[t];
    const bool ga = (uint32_t)t == a.depth, gb = (uint32_t)t == b.depth;
    if (ga != gb) return ga;
    if (ga) {
      if (a.uid != b.uid) return a.uid < b.uid;
      for (int u = t - 1; u >= 0; u--)
        if (a.j[u] != b.j[u]) return a.j[u] < b.j[u];
      return false;
    }
  }
  return false;  // (deeper chains are refused at create)
}
// The gen-0 records' ranks among themselves come from k2_handle's rank tiles (keys known before the
// handlers run); here, tiles of (all records x local records) add the local records before each record,
// and tiles of (local records x gen-0 records) the gen-0 records before each local one (rel ts only: at
// equal ts a gen-0 record comes first).  Each record's two order words are made once (local_record: lkw;
// a gen-0 row: its rel ts, with a zero low word, sorts before every local record of its ts), so a column
// costs one 16-B LDS load and two compares (64 columns a tile, unrolled: the loads pipeline); the exact
// chain compare runs after the tile, only for rows whose words tie with a distinct record's (chains of 3+
// levels with equal ts pairs).
constexpr int RKC = 64;  // columns per tile
// (diagnostic build: the tiles' phase marks only with NSGPU_TILE_MARKS — their atomics distort the per-block times)
#ifdef NSGPU_TILE_MARKS
#define TILE_MARK(i, win) BLK_MARK(i, win)
#else
#define TILE_MARK(i, win) (void)0
#endif
template <int NT>
__device__ void df_book(const P2PDev &M, Ctl &C, bool ranked, uint32_t W, uint32_t Lt, uint64_t wn);
// DF: the deferred pipeline's variant: it reads k2_handle's snapshot (rk_*), always runs for a formed window,
// copies the window's keys / contexts for the next k2_pa (pwkey / pwctx: k2_scan's job in the other
// pipeline), and its block 0 does the window's bookkeeping (df_book); the dispatch accounting (log, digest,
// uid resolution) is deferred to k2_sdef once the next k2_pa has staged the records in rank order.
template <int NT>
__device__ void df_sdef(const P2PDev &M, Ctl &C, uint32_t b, uint32_t nsb);
constexpr int RKT_DF = 1024;              // the deferred pipeline's k2_rank blocks: SUBS tiles at once
#ifndef NSDEF_N
#define NSDEF_N 4
#endif
#ifndef RK_GRID_DF_N
#define RK_GRID_DF_N 256
#endif
constexpr int NSDEF = NSDEF_N;            // blocks of the deferred accounting (df_sdef: each scans the whole
                                          // window, then resolves / logs / digests a quarter of its records)
static_assert(NSDEF == 1 || NSDEF == 2 || NSDEF == 4 || NSDEF == 8, "a thread's NMAX / NT records split evenly");
constexpr int RK_GRID_DF = RK_GRID_DF_N;    // one 1024-thread block per CU (~150 KB of LDS each): bookkeeping, accounting, tiles
template <bool DF>
__global__ __launch_bounds__(DF ? RKT_DF : RKT) void k2_rank(const P2PDev M) {
  constexpr int NT = DF ? RKT_DF : RKT, SUBS = NT / RKT;
  Ctl &C = *M.C;
  BLK_T0();
#ifdef NSGPU_PHASE_PROF
  const uint64_t c_win = DF ? C.rk_win : C.windows;  // (DF: block 0's bookkeeping advances C.windows)
  uint32_t n_tie = 0;
#endif
  // DF: blocks 1 .. NSDEF do the last window's dispatch accounting (k2_pa staged it) beside this window's
  // ranking
  if constexpr (DF) {
    if (blockIdx.x >= 1 && blockIdx.x <= (uint32_t)NSDEF) {
      if (M.sdef_fold) df_sdef<NT>(M, C, blockIdx.x - 1, NSDEF);
      BLK_REC(2, c_win);  // (diagnostic build: k2_scan's per-block slot, unused by the deferred pipeline)
      return;
    }
  }
  uint32_t c_done = 0, c_mode = 0, W, c_fr = 0, go = 3;
  uint64_t lim, wn;
  if (DF) {
    go = C.rk_go, W = C.rk_W, lim = C.rk_lim, wn = C.rk_win;
  } else {
    c_done = C.done, c_mode = C.mode, W = C.W, c_fr = C.force_run, lim = C.lim_rel, wn = C.windows;
  }
  const uint32_t lc = threadIdx.x < (uint32_t)NLR ? M.lcnt[threadIdx.x] : 0u;  // (its trip overlaps the control's)
  if (DF) {
    if (!(go & 2u)) return;  // (no window was formed: the run is over or paused)
    if (go & 4u) {  // (a sorted run's chunk: the host drives runs with the other pipeline — never here)
      if (blockIdx.x == 0 && threadIdx.x == 0) {
        atomicOr(M.error, 256u);
        C.done = 1;
      }
      return;
    }
  } else if (c_done || c_mode >= MODE_SORT || c_mode == MODE_RUN || W > (uint32_t)WCAP || c_fr || lim == 0) {
    return;
  }
  const bool ranked = (go & 1u) != 0;
  __shared__ uint32_t pre[NLR + 1];
  __shared__ ulonglong2 cws[SUBS][RKC];
  // the columns' rel ts alone (the gen-0-row and local-row x gen-0 tiles compare nothing else): 4 B a column, read
  // 4 at a time — the tiles are bound by their per-column LDS reads and 64-bit compares
  __shared__ __align__(16) uint32_t cwhs[SUBS][RKC];
  local_prefix<NT>((ranked && lim) ? lc : 0u, pre);
  const uint32_t Lt = pre[NLR], N = W + Lt;
  uint32_t *const wr = wrank_of(M, wn), *const lr = lrank_of(M, wn);
  uint32_t b0 = blockIdx.x, nb = gridDim.x;  // (DF: block 0 keeps the books, 1 .. NSDEF account, the others rank)
  if (DF) {
    if (blockIdx.x == 0) {
      df_book<NT>(M, C, ranked, W, Lt, wn);
      BLK_REC(2, c_win);
      return;
    }
    if (!ranked) return;
    b0 -= 1 + NSDEF, nb -= 1 + NSDEF;
    for (uint32_t i = b0 * NT + threadIdx.x; i < W; i += nb * NT) {  // (the next k2_pa rewrites wkey / wctx)
      M.pwkey[i] = M.wkey[i];
      M.pwctx[i] = M.wctx[i];
    }
  }
  if (Lt == 0 || N > (uint32_t)NMAX || Lt > (uint32_t)LMAX) return;  // (too many: the bookkeeping fails the run, error 64)
#ifdef NSGPU_PHASE_PROF
  if (c_win == g_blk_win && blockIdx.x == 0 && threadIdx.x == 0) {
    g_phase[57] = N;
    g_phase[58] = Lt;
  }
#endif
  TILE_MARK(48, c_win);
  const uint32_t nr = (N + RKT - 1) / RKT, ncl = (Lt + RKC - 1) / RKC;  // phase A: rows x local columns
  const uint32_t nl = (Lt + RKT - 1) / RKT, ncg = (W + RKC - 1) / RKC;  // phase B: local rows x gen-0 columns
  const uint32_t na = nr * ncl, ntile = na + nl * ncg;
  // SUBS tiles a block at once: sub-tile `sub` is RKT threads (whole waves) with its own column buffer
  const uint32_t sub = threadIdx.x / RKT, lt = threadIdx.x % RKT;
  ulonglong2 *const cw = cws[sub];
  uint32_t *const cwh = cwhs[sub];
  // a block's sub-tiles are spread over the tile space (sub-tile `sub` of block b0 takes tile base + sub x nb +
  // b0), so each block gets a mix of the costly tiles (rows with local records) and the cheap ones
  for (uint32_t t0 = 0; t0 < ntile; t0 += nb * SUBS) {  // (uniform over the block)
    const uint32_t t = t0 + sub * nb + b0;
    const bool tA = t < na, tB = !tA && t < ntile;
    uint32_t c = 0, slot = 0;  // slot: the row's accumulator (wrank[dense] for gen-0, LBASE + k for local k)
    uint32_t ix = 0, rx = 0, tj = 0;
    bool g0rows = false;  // (tA: every row is a gen-0 record)
    uint64_t wx = ~0ull, wx2 = ~0ull, relx = 0;
    if (tA) {  // rows: every record; columns: local records
      const uint32_t ti = t / ncl;
      tj = t % ncl;
      ix = ti * RKT + lt;
      g0rows = ti * RKT + RKT <= W;
      if (lt < (uint32_t)RKC) {
        const uint32_t cy = tj * RKC + lt;
        ulonglong2 w = make_ulonglong2(~0ull, ~0ull);  // (a padding column: after every row)
        if (cy < Lt) {
          const uint32_t r = dense_rec(W + cy, W, pre);
          w = M.lkw[r - LBASE];
          if (ti == 0) {  // the dense list k2_scan (ldat) and the next k2_pa (lrec) read; the local's context
            const uint32_t wp = M.wpar[r];
            M.ldat[cy] = make_uint4(r, M.nchild[r] | (M.ninl[r] << 16), (uint32_t)(w.x >> 32), wp);
            if (DF) M.ldpd[cy] = dense_of(wp & 0xffffffu, W, pre) | (wp & 0xff000000u);
            M.lrec[cy] = r;
            M.pwctx[r] = M.wctx[r];
          }
        }
        cw[lt] = w;
        cwh[lt] = (uint32_t)(w.x >> 32);  // (padding 0xffffffff: never below a row's rel ts)
      }
      if (ix < N) {
        rx = dense_rec(ix, W, pre);
        if (ix >= W) {
          const ulonglong2 w = M.lkw[rx - LBASE];
          wx = w.x;
          wx2 = w.y;
        } else {
          wx = (M.wkey[rx] >> 32) << 32;  // (a local record of smaller rel ts comes first)
          wx2 = 0;
        }
      }
    } else if (tB) {  // rows: local records; columns: gen-0 records (rel ts <= the row's)
      const uint32_t u = t - na, ti = u / ncg;
      tj = u % ncg;
      ix = ti * RKT + lt;
      if (lt < (uint32_t)RKC) {
        const uint32_t cy = tj * RKC + lt;
        cwh[lt] = cy < W ? (uint32_t)(M.wkey[cy] >> 32) : 0xffffffffu;  // (padding: counted out below)
      }
      if (ix < Lt) relx = M.wkey[dense_rec(W + ix, W, pre)] >> 32;
    }
    __syncthreads();
    TILE_MARK(50, c_win);
    const uint4 *const cwh4 = reinterpret_cast<const uint4 *>(cwh);
    if (tA && g0rows) {  // a local column precedes a gen-0 row iff its rel ts is smaller: one 32-bit compare
      const uint32_t tx = (uint32_t)(wx >> 32);
#pragma unroll 4
      for (int y4 = 0; y4 < RKC / 4; y4++) {
        const uint4 q = cwh4[y4];
        c += (uint32_t)(q.x < tx) + (uint32_t)(q.y < tx) + (uint32_t)(q.z < tx) + (uint32_t)(q.w < tx);
      }
      slot = rx;
    } else if (tA) {
      bool tie = false;
      const uint32_t self = ix - W - tj * RKC;  // (the row's own column, if it is one of this tile's)
#pragma unroll 16
      for (uint32_t y = 0; y < (uint32_t)RKC; y++) {
        const ulonglong2 w = cw[y];
        const bool eq = w.x == wx;
        c += (w.x < wx) | (eq & (w.y < wx2));
        tie |= eq & (w.y == wx2) & (y != self);
      }
      if (tie && ix < N) {  // (rare: deep chains)
        const LKey kx = M.lkey[rx - LBASE];
        for (uint32_t y = 0; y < (uint32_t)RKC; y++) {
          const ulonglong2 w = cw[y];
          const uint32_t cy = tj * RKC + y;
          if (w.x == wx && w.y == wx2 && y != self && cy < Lt) {
#ifdef NSGPU_PHASE_PROF
            n_tie++;
#endif
            c += lk_before(M.lkey[dense_rec(W + cy, W, pre) - LBASE], kx);
          }
        }
      }
      if (ix >= N) c = 0;
      slot = ix >= W ? ix - W + LBASE : rx;
    } else if (tB) {
      const uint32_t rx32 = (uint32_t)relx;  // (a rel ts: below 2^32)
#pragma unroll 4
      for (int y4 = 0; y4 < RKC / 4; y4++) {
        const uint4 q = cwh4[y4];
        c += (uint32_t)(q.x <= rx32) + (uint32_t)(q.y <= rx32) + (uint32_t)(q.z <= rx32) + (uint32_t)(q.w <= rx32);
      }
      const uint32_t nv = W - tj * RKC;  // (the last column tile's padding columns: 0xffffffff <= the row's rel ts
      if (nv < (uint32_t)RKC && rx32 == 0xffffffffu) c -= (uint32_t)RKC - nv;  //  only at that rel ts)
      if (ix >= Lt) c = 0;
      slot = ix + LBASE;
    }
    TILE_MARK(52, c_win);
    if (c) atomicAdd(slot >= LBASE ? &lr[slot - LBASE] : &wr[slot], c);
    __syncthreads();
    TILE_MARK(54, c_win);
  }
  BLK_REC(2, c_win);
#ifdef NSGPU_PHASE_PROF
  if (n_tie) atomicAdd((unsigned long long *)&g_phase[61], (unsigned long long)n_tie);  // (every window)
  if (c_win == g_blk_win) {
    if (n_tie) atomicAdd((unsigned long long *)&g_phase[56], (unsigned long long)n_tie);
    if (threadIdx.x == 0) atomicAdd((unsigned long long *)&g_phase[59], 1ull);
  }
#endif
}

// The deferred pipeline's window bookkeeping (k2_rank<true>'s block 0; NT threads): k2_scan's run
// bookkeeping without its scan — the child totals come from k2_handle (acc_tc / acc_tinl), the dispatch
// bases of the window go to winfo for k2_sdef, and the next k2_pa stages the window (pdf = 1).  The
// free-stack move and the hub resets are the block's; the rest is thread 0's.
template <int NT>
__device__ void df_book(const P2PDev &M, Ctl &C, bool ranked, uint32_t W, uint32_t Lt, uint64_t wn) {
  const int tid = threadIdx.x;
  // every run-control field the bookkeeping reads, loaded at once (one memory trip: a load issued after a
  // branch on another loaded value would wait for that value first)
  const uint64_t nF = C.nF, nfree = C.nfree, npush = C.npush;
  const uint32_t c_nhub = C.nhub;
  uint64_t tc = 0, tinl = 0, live = 0, P_end = 0, c_bound = 0, c_nbound = 0, K = 0, tmin = 0, ilim = 0, windows = 0,
           span_t = 0, hts = 0, max_window = 0, max_windows = 0, refits = 0;
  uint32_t uid = 0, rt = 0, stop_seen = 0, hcap = 0;
  if (tid == 0) {
    tc = C.acc_tc, tinl = C.acc_tinl, live = C.live, P_end = C.P_end, c_bound = C.bound, c_nbound = C.nbound;
    K = C.K, tmin = C.tmin, ilim = C.inline_lim, windows = C.windows, span_t = C.span_t, hts = C.hts;
    max_window = C.max_window, max_windows = C.max_windows, refits = C.refits;
    uid = C.uid, rt = C.rt, stop_seen = C.stop_seen, hcap = C.hcap;
  }
  const uint64_t consumed = nF < nfree ? nF : nfree;
  const uint64_t mv = consumed < npush ? consumed : npush;
  // the free stack loses the slots the fresh children took and gains the window's (disjoint ranges)
  for (uint64_t i = tid; i < mv; i += NT) M.fstack[nfree - consumed + i] = M.fstack[nfree + npush - mv + i];
  if (ranked) {
    const uint32_t nh = c_nhub < (uint32_t)MAXHUB ? c_nhub : (uint32_t)MAXHUB;
    for (uint32_t h = tid; h < nh; h += NT) M.node_tab[(uint64_t)M.hub_list[h] * NTAB] = 0;
  }
  if (tid != 0) return;
  C.acc_tc = 0;
  C.acc_tinl = 0;
  C.nfree = nfree - consumed + npush;
  const uint64_t P_end2 = P_end + (nF > nfree ? nF - nfree : 0);
  const uint64_t live2 = live - npush + nF;
  C.P_end = P_end2;
  C.live = live2;
  C.npush = 0;
  C.nF = 0;
  C.nhub = 0;
  C.force_run = 0;
  if (!ranked) {  // the window overflowed: a sorted run (host radix sort), nothing dispatched (k2_scan's branch)
    C.rW = W;
    C.r0 = 0;
    C.W = 0;
    C.pvalid = 0;
    C.refits = refits + 1;
    C.renarrow = c_nbound < c_bound ? 1u : 0u;
    if (c_nbound < c_bound) C.span_t = ((c_bound >> 32) >> 1) + 1;
    C.mode = MODE_SORT;
    return;
  }
  const uint32_t N = W + Lt;
  if (N > (uint32_t)NMAX || Lt > (uint32_t)LMAX) {  // (the adaptive span keeps windows well inside)
    atomicOr(M.error, 64u);
    C.done = 1;
    return;
  }
  C.winfo[wn & 3] = WInfo{K, tmin, ilim, uid, N, W, Lt};
  C.pK0 = K;
  C.puid0 = uid;
  C.ptmin = tmin;
  C.pinline_lim = ilim;
  C.pW = W;
  C.plt = Lt;
  C.pinl = (uint32_t)tinl;
  C.pvalid = 1;
  C.pdf = 1;
  C.K = K + N + tinl;
  C.uid = uid + (uint32_t)tc;
  const uint64_t pchild = tc - tinl - Lt;  // (the local records' uids were consumed, they ran in the window)
  C.pchild = pchild;
  bool done = stop_seen || (live2 + pchild == 0 && hts == ~0ull);
  if ((uint64_t)uid + tc >= (uint64_t)UID_DF_LIMIT) {  // (provisional uids must stay above every real one;
    atomicOr(M.error, 512u);                           //  unreachable: the pause below hands over first)
    done = true;
  }
  const uint64_t span = c_bound >> 32;  // wide windows: keep them inside the window capacity
  if (N > (uint32_t)(7 * NMAX / 8) || W > (uint32_t)(7 * WCAP / 8)) C.span_t = span - span / 4;
  else if (N < (uint32_t)(3 * NMAX / 4) && W < (uint32_t)(3 * WCAP / 4) && span_t < (1ull << 40))
    C.span_t = span_t + span_t / 8 + 1;
  C.red[rt ^ 1].tmin = C.red[rt ^ 1].wend = C.red[rt ^ 1].stopts = C.red[rt ^ 1].wendw = ~0ull;  // consumed
  C.rt = rt ^ 1;
  C.windows = windows + 1;
  if (N > max_window) C.max_window = N;
  C.W = 0;
  if (P_end2 > M.pool_cap) {
    atomicOr(M.error, 1u);
    done = true;
  }
  if (windows + 1 >= max_windows && !done) {
    atomicOr(M.error, 4u);
    done = true;
  }
  if (done) {
    C.done = 1;
  } else if (hcap) {  // the window was cut at the next host closure: pause
    C.hcap = 0;
    C.mode = MODE_HOST;
  } else if (P_end2 > 65536 && live2 * 4 < P_end2) {
    C.mode = MODE_COMPACT;
  } else if ((uint64_t)uid + tc >= (uint64_t)UID_DF_SOFT) {  // uids near the provisional range: the scanning
    C.mode = MODE_UIDX;                                        // pipeline takes over for the rest of the run
  }
}

// ---- k2_sdef: a deferred window's dispatch accounting (DF pipeline; one block) ----
// Window n's records, staged in rank order by the next k2_pa: exclusive scans of (children, inline children,
// same-ts group heads) give each record its dispatch rank (K0 + rank + the inline leaves of earlier ts groups)
// and child prefix; a local record's uid resolves through its parent's rank and this window's prefixes (k2_pa
// resolved the provisional ones at staging); the log and digest get every record and leaf; the child prefixes
// are kept (cpt) for the provisional uids of window n's children.  Afterwards the window's rank accumulators
// are cleared (their parity is window n + 2's).
// NSDEF blocks of NT threads (k2_rank<true>'s blocks 1 .. NSDEF, or the k2_sdef kernel): each scans the whole
// window and resolves / logs / digests its share (every NSDEF-th record of a thread).  Every record is loaded once, into
// registers (RPT consecutive ranks a thread), in the same memory trip as the run control; the scan's per-rank
// results go to LDS (child / inline prefixes, the group of each rank, group starts, and the rank of each dense
// index, through which a local record finds its parent's), so after the loads the kernel reads LDS only.
template <int NT>
__device__ void df_sdef(const P2PDev &M, Ctl &C, uint32_t b, uint32_t nsb) {
  const uint32_t sf = C.sflag;
  BLK_T0();
#ifdef NSGPU_PHASE_PROF
  const uint64_t c_win = C.rk_win - 1;  // (diagnostic build: marks 22..30 in the sampled window)
#endif
  static_assert(NT == (int)STG_NT, "k2_sdef's rank slices are the stage layout's");
  constexpr int RPT = NMAX / NT;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  WInfo wa[4];  // (all four: loaded with the flag, picked by it)
#pragma unroll
  for (int k = 0; k < 4; k++) wa[k] = C.winfo[k];
  // per record: key, counts, parent or first inline leaf (a local record's key has uid 0: gen-0 uids start
  // at 4) — one stage (the window k2_pa staged), loaded with the run control; record 8 tid + q is at
  // q * NT + tid (stg_pos), so each load of a wave reads consecutive entries
  uint64_t ek[RPT];
  uint32_t ec[RPT], ep[RPT];
  uint32_t prev_rel = 0;
  {
    const Stg *st = M.stage;
#pragma unroll
    for (int q = 0; q < RPT; q++) {  // (NMAX entries: in range, ignored past N)
      const Stg x = st[q * NT + tid];
      ek[q] = x.key;
      ec[q] = x.cnt;
      ep[q] = x.par;
    }
    if (tid > 0) prev_rel = (uint32_t)(st[(RPT - 1) * NT + tid - 1].key >> 32);
  }
  // (the window records in registers before the flag's test: otherwise the compiler sinks their loads past it,
  // a second trip)
#pragma unroll
  for (int k = 0; k < 4; k++)
    asm volatile("" ::"s"(wa[k].K0), "s"(wa[k].tmin), "s"(wa[k].uid0), "s"(wa[k].N), "s"(wa[k].W), "s"(wa[k].Lt));
  if (!(sf & 1u)) return;
  const uint32_t wi = (sf >> 1) & 3u, pn = wi & 1u;  // window n & 3, its parity (its child prefixes' buffer)
  WInfo w = wa[0];
#pragma unroll
  for (int k = 1; k < 4; k++)
    if ((uint32_t)k == wi) w = wa[k];
  const uint32_t N = w.N;
  __shared__ uint32_t s_cp[NMAX_PAD];   // child prefix by rank (lds_pad)
  __shared__ uint32_t s_ip[NMAX_PAD];   // inline prefix by rank
  __shared__ uint32_t s_grp[NMAX_PAD];  // same-ts group of each rank
  __shared__ uint32_t s_gs[NMAX_PAD];   // start rank of each group (by group: lds_pad)
  __shared__ uint16_t s_rk[NMAX];       // rank of each dense index (local records' parents)
  __shared__ uint64_t wsum[NT / 64];
  if ((uint32_t)(tid * RPT) > N) prev_rel = 0;
  uint64_t sum = 0;  // packed (children, inline children, group heads), 21 bits each
  {
    uint32_t pr = prev_rel;
#pragma unroll
    for (int q = 0; q < RPT; q++) {
      const uint32_t r = tid * RPT + q;
      if (r < N) {
        const uint32_t rel = (uint32_t)(ek[q] >> 32);
        const uint32_t hd = r == 0 || rel != pr;
        pr = rel;
        sum += (uint64_t)(ec[q] & 0x1ffu) | ((uint64_t)((ec[q] >> 9) & 0x1ffu) << 21) | ((uint64_t)hd << 42);
      }
    }
  }
  BLK_MARK(22, c_win);  // the records arrived
  uint64_t inc = sum;
  inc = wave_incscan64(inc);
  if (lane == 63) wsum[wid] = inc;
  __syncthreads();
  uint64_t off = 0, tot = 0;
  for (int k = 0; k < NT / 64; k++) {
    const uint64_t x = wsum[k];
    off += k < wid ? x : 0;
    tot += x;
  }
  const uint64_t ex = off + inc - sum;
  const uint32_t tinl = (uint32_t)((tot >> 21) & 0x1fffffu), ng = (uint32_t)(tot >> 42);
  BLK_MARK(24, c_win);  // block scan
  {
    uint32_t pr = prev_rel, bc = (uint32_t)(ex & 0x1fffffu), bi = (uint32_t)((ex >> 21) & 0x1fffffu),
             bh = (uint32_t)(ex >> 42);
#pragma unroll
    for (int q = 0; q < RPT; q++) {
      const uint32_t r = tid * RPT + q;
      if (r < N) {
        const uint32_t rel = (uint32_t)(ek[q] >> 32);
        const uint32_t hd = r == 0 || rel != pr;
        pr = rel;
        bh += hd;
        s_cp[lds_pad(r)] = bc;
        s_ip[lds_pad(r)] = bi;
        s_grp[lds_pad(r)] = bh - 1;
        if (hd) s_gs[lds_pad(bh - 1)] = r;
        s_rk[(ec[q] >> 18) % NMAX] = (uint16_t)r;
        if ((uint32_t)q % nsb == b) M.cpt[(uint64_t)pn * NMAX + q * NT + tid] = bc;  // (stg_pos(r): window n's children resolve through it)
        bc += ec[q] & 0x1ffu;
        bi += (ec[q] >> 9) & 0x1ffu;
      }
    }
  }
  __syncthreads();
  BLK_MARK(26, c_win);  // per-rank LDS arrays, prefixes stored
  uint64_t digest = 0;
#pragma unroll
  for (int q = 0; q < RPT; q++) {
    const uint32_t r = tid * RPT + q;
    if (r >= N || (uint32_t)q % nsb != b) continue;  // (this block's share of the records)
    const uint32_t rel = (uint32_t)(ek[q] >> 32);
    const uint64_t t = w.tmin + rel;
    uint32_t uid = (uint32_t)ek[q];
    if (uid == 0u) {  // a local record: its parent's child prefix + its child index
      uint32_t rp = s_rk[(ep[q] & 0xffffffu) % NMAX];
      if (rp >= N) {  // (cannot happen: the parent is a record of this window)
        atomicOr(M.error, 256u);
        rp = 0;
      }
      uid = w.uid0 + s_cp[lds_pad(rp)] + (ep[q] >> 24);
    } else if (uid & PROV) {  // (k2_pa resolves these at staging)
      atomicOr(M.error, 256u);
    }
    const uint32_t g = s_grp[lds_pad(r)];
    const uint32_t first = s_gs[lds_pad(g)];
    const uint32_t last = (g + 1 < ng ? s_gs[lds_pad(g + 1)] : N) - 1;
    const uint64_t rk = w.K0 + r + (tinl ? s_ip[lds_pad(first)] : 0u);
    digest += digest_term(rk, t, uid);
    if (rk < M.log_cap) {
      M.log_ts[rk] = t;
      M.log_uid[rk] = uid;
      M.log_ctx[rk] = M.stx[q * NT + tid];
    }
    const uint32_t ni = min((ec[q] >> 9) & 0x1ffu, M.maxc);  // (bounded: a staged record's leaves fit its row)
    const uint2 *lf = M.sleaf + (uint64_t)r * M.maxc;
    const uint32_t cpr = s_cp[lds_pad(r)], ipr = s_ip[lds_pad(r)];
    for (uint32_t k = 0; k < ni; k++) {  // its inline DoForwardUp leaves, in Schedule order
      const uint2 l = k ? lf[k] : make_uint2(ep[q] & 0xffffffu, ep[q] >> 24);
      const uint64_t lk = w.K0 + last + 1 + ipr + k;
      const uint32_t lu = w.uid0 + cpr + l.y;
      digest += digest_term(lk, t, lu);
      if (lk < M.log_cap) {
        M.log_ts[lk] = t;
        M.log_uid[lk] = lu;
        M.log_ctx[lk] = l.x;
      }
    }
    if (r == N - 1) C.last_ts = t;
  }
  digest = wave_sum64(digest);
  BLK_MARK(28, c_win);  // resolve, log, digest
  if (lane == 0 && digest) atomicAdd((unsigned long long *)&C.digest, (unsigned long long)digest);
  // the window's rank accumulators, cleared for window n + 2 (k2_pa read them; nothing here does)
  for (uint32_t i = b * NT + tid; i < w.W; i += nsb * NT) M.wrank[(uint64_t)pn * WTOT + i] = 0;
  for (uint32_t i = b * NT + tid; i < w.Lt; i += nsb * NT) M.lrank[(uint64_t)pn * LMAX + i] = 0;

  BLK_MARK(30, c_win);  // clears
}
__global__ __launch_bounds__(SCAN_THREADS) void k2_sdef(const P2PDev M) {
  df_sdef<SCAN_THREADS>(M, *M.C, blockIdx.x, gridDim.x);
}

// ---- k2_scan: rank order; child / inline prefixes, same-ts groups, run bookkeeping ----
// WIDE: the single engine's wide windows: the local records join the gen-0 ones (ranks from k2_rank), and
// a local record's uid is its parent's child prefix + its child index (DefaultSimulatorImpl gives uids in
// Schedule order).
// FL: the flush of a deferred window (host step, when the deferred pipeline paused after window n's
// bookkeeping): the same scan from the records, into sinfo / pwkey for the next k2_pa's appending, with
// window n's bases from winfo and its provisional uids resolved; no run bookkeeping (df_book did it).
template <bool WIDE, bool FL = false>
__global__ __launch_bounds__(SCAN_THREADS) void k2_scan(const P2PDev M) {
  static_assert(!FL || WIDE, "flushes are the deferred pipeline's");
  Ctl &C = *M.C;
  // one thread per RPT records (dense order: the W gen-0 slots, then the local records region by region);
  // the rank-ordered arrays hold NREC records (wide: 128 KB of LDS)
  constexpr int NREC = WIDE ? NMAX : WCAP;
  constexpr int RPT = NREC / SCAN_THREADS;
  constexpr int RPT0 = WCAP / SCAN_THREADS;  // (the gen-0 part, loaded speculatively at entry)
  constexpr int SBUF = 4 * NREC;
  __shared__ uint32_t sbuf[SBUF];
  uint32_t *l_slot = sbuf, *l_cnt = sbuf + NREC, *l_rel = sbuf + 2 * NREC, *gstart = sbuf + 3 * NREC;
  __shared__ uint32_t pre[NLR + 1];
  PH_BEGIN();
  BLK_T0();
#ifdef NSGPU_PHASE_PROF
  const uint64_t c_win = C.windows;
#endif
  const int tid = threadIdx.x;
  // the run control and the window's slots (speculatively at base 0), all loaded at once
  const uint64_t c_wn = C.windows;  // (FL: df_book counted window n already)
  const uint32_t c_done = C.done, c_mode = C.mode, W = FL ? C.pW : C.W, c_fr = FL ? 0u : C.force_run,
                 c_wbase = C.wbase;
  const uint32_t c_nhub = C.nhub, c_pvalid = C.pvalid, c_pdf = C.pdf;
  const WInfo wif = C.winfo[(c_wn + 3) & 3];  // (FL: window n = c_wn - 1)
  const uint32_t uid0 = FL ? wif.uid0 : C.uid;
  const uint64_t nF = C.nF, nfree = C.nfree, npush = C.npush, c_lim = C.lim_rel, c_bound = C.bound,
                 c_nbound = C.nbound, c_r0 = C.r0, c_rW = C.rW;
  const uint32_t c_rtrim = C.rtrim;
  const uint32_t c_lcnt = (WIDE && tid < NLR) ? M.lcnt[tid] : 0u;  // (the local regions' counts, at once)
  // the bookkeeping's run control as well (thread 0 writes it back at the end; loaded now, its trip
  // overlaps the slot loads instead of following the scan)
  struct Book {
    uint64_t K, tmin, inline_lim, live, P_end, r0, rW, windows, max_window, max_windows, hts, span_t;
    uint32_t uid, rt, stop_seen, hcap;
  } bk{};
  if (tid == 0)
    bk = Book{C.K, C.tmin, C.inline_lim, C.live, C.P_end, C.r0, C.rW, C.windows, C.max_window, C.max_windows, C.hts,
              C.span_t, C.uid, C.rt, C.stop_seen, C.hcap};
  // per record: rank, child counts, record index, rel ts; a local record's parent (wpar), later the
  // parent's rank | child index << 16
  // Slot q of a thread: q < RPT0 the gen-0 slot i = tid + q * SCAN_THREADS (dense index i), q >= RPT0 (wide)
  // the local record k = i - WCAP of k2_rank's dense list (dense index W + k); both loaded speculatively.
  uint32_t pr[RPT], pc[RPT], prec[RPT], prel[RPT], ppx[RPT], pr1[RPT];
  uint64_t gk[RPT0];
  uint32_t gctx[RPT0];
#pragma unroll
  for (int q = 0; q < RPT; q++) {
    const uint32_t i = tid + q * SCAN_THREADS;
    prec[q] = i;
    pr[q] = pc[q] = prel[q] = ppx[q] = pr1[q] = 0;
    if (q < RPT0) {  // (both parities' rank accumulators: the window's is picked once C.windows is back)
      pr[q] = M.wrank[i];
      pr1[q] = M.wrank[WTOT + i];
      pc[q] = M.nchild[i] | (M.ninl[i] << 16);
      gk[q] = M.wkey[i];
      gctx[q] = M.wctx[i];
    } else {
      const uint4 d = M.ldat[i - WCAP];
      prec[q] = d.x;
      pc[q] = d.y;
      prel[q] = d.z;
      ppx[q] = d.w;
      pr[q] = M.lrank[i - WCAP];
      pr1[q] = M.lrank[LMAX + i - WCAP];
    }
  }
  if (FL) {
    if (!(c_pvalid && c_pdf)) return;  // (the window was not handled: nothing to append)
  } else if (c_done || c_mode >= MODE_SORT) {
    return;
  }
  const uint64_t wn = FL ? c_wn - 1 : c_wn;  // the window scanned
  if (wn & 1) {
#pragma unroll
    for (int q = 0; q < RPT; q++) pr[q] = pr1[q];
  }
  if (FL) {  // a record that is a child of window n - 1 has a provisional uid: resolve it
    const uint32_t uq = C.winfo[(wn + 3) & 3].uid0;
    const uint32_t *cq = M.cpt + (uint64_t)((wn + 1) & 1) * NMAX;
#pragma unroll
    for (int q = 0; q < RPT0; q++) {
      const uint32_t u = (uint32_t)gk[q];
      const uint32_t i = tid + q * SCAN_THREADS;
      if (i < W && (u & PROV)) {
        if (((u >> 30) & 1u) != (uint32_t)((wn + 1) & 1)) atomicOr(M.error, 256u);
        gk[q] = (gk[q] & ~0xffffffffull) | (uint32_t)(uq + cq[stg_pos(((u & 0x3fffffffu) >> 8) % NMAX)] + (u & 0xffu));
      }
    }
  }
  const bool run = !FL && c_mode == MODE_RUN;
  const bool handled = run || (W <= (uint32_t)WCAP && !c_fr);
  const uint32_t base = run ? c_wbase : 0;
  // ---- pool bookkeeping: the free stack loses the slots the fresh children took and gains the
  // window's; its pushed part is moved down over the popped hole
  // (last in the kernel: a moving wave waits for its loads, and nothing here reads the stack)
  const uint64_t consumed = nF < nfree ? nF : nfree;
  const uint64_t mv = consumed < npush ? consumed : npush;
  auto stack_and_hubs = [&]() {
    if (FL) return;  // (df_book did it)
    for (uint64_t i = tid; i < mv; i += SCAN_THREADS) M.fstack[nfree - consumed + i] = M.fstack[nfree + npush - mv + i];
    if (handled) {
      const uint32_t nh = c_nhub < (uint32_t)MAXHUB ? c_nhub : (uint32_t)MAXHUB;
      for (uint32_t h = tid; h < nh; h += SCAN_THREADS) M.node_tab[(uint64_t)M.hub_list[h] * NTAB] = 0;
    }
  };
  if (!handled) {  // the window overflowed WCAP: it becomes a sorted run (host radix sort), nothing dispatched yet
    stack_and_hubs();
    __syncthreads();
    if (tid == 0) {
      C.acc_tc = 0;  // (k2_handle's totals: this pipeline scans its own)
      C.acc_tinl = 0;
      C.pdf = 0;
      C.nfree = nfree - consumed + npush;
      C.P_end += nF > nfree ? nF - nfree : 0;
      C.live = C.live - npush + nF;
      C.npush = 0;
      C.nF = 0;
      C.nhub = 0;
      C.rW = W;
      C.r0 = 0;
      C.W = 0;
      C.pvalid = 0;
      C.refits++;
      C.force_run = 0;
      // a widened window is trimmed back to its narrow bound before it runs (host step: the run's rule is
      // that every child sorts after every run event), and the next ones start narrower
      C.renarrow = c_nbound < c_bound ? 1u : 0u;
      if (c_nbound < c_bound) C.span_t = ((c_bound >> 32) >> 1) + 1;
      C.mode = MODE_SORT;
    }
    return;
  }
  // ---- the local records (wide windows): dense positions W .. N-1
  if constexpr (WIDE) local_prefix<SCAN_THREADS>(c_lim != 0 && !run ? c_lcnt : 0u, pre);
  const uint32_t Lt = (WIDE && !run) ? pre[NLR] : 0u;
  const uint32_t N = W + Lt;
  // dense index of slot q, and whether it holds a record of this window
  auto dense_q = [&](int q) -> uint32_t {
    const uint32_t i = tid + q * SCAN_THREADS;
    return q < RPT0 ? i : W + (i - (uint32_t)WCAP);
  };
  auto valid_q = [&](int q) -> bool {
    const uint32_t i = tid + q * SCAN_THREADS;
    return q < RPT0 ? i < W : i - (uint32_t)WCAP < Lt;
  };
  if (N > (uint32_t)NREC || Lt > (uint32_t)LMAX) {  // (the adaptive span keeps windows well inside; a run that got here fails loudly)
    if (tid == 0) {
      atomicOr(M.error, 64u);
      C.done = 1;
    }
    return;
  }
  // the keys / contexts the next k2_pa appends with (a local record's uid comes after the ranking)
#pragma unroll
  for (int q = 0; q < RPT0; q++) {
    const uint32_t i = tid + q * SCAN_THREADS;
    if (base != 0 && i < W) {
      gk[q] = M.wkey[base + i];
      gctx[q] = M.wctx[base + i];
    }
    if (run) pr[q] = i;
    if (i < W) {
      M.pwctx[i] = gctx[q];
      M.pwkey[i] = gk[q];
      prel[q] = (uint32_t)(gk[q] >> 32);
    }
  }
  if constexpr (WIDE) {
    if (Lt) {  // a local record's parent's rank (its uid below is the parent's child prefix + j)
      uint32_t *Fd = sbuf;  // [N] rank by dense index
#pragma unroll
      for (int q = 0; q < RPT; q++)
        if (valid_q(q)) Fd[dense_q(q)] = pr[q];
      __syncthreads();
#pragma unroll
      for (int q = RPT0; q < RPT; q++)
        if (valid_q(q)) ppx[q] = Fd[dense_of(ppx[q] & 0xffffffu, W, pre)] | ((ppx[q] >> 24) << 16);
      __syncthreads();  // (the buffer holds the rank-ordered arrays next)
    }
  }
  PH_MARK(16);
#pragma unroll
  for (int q = 0; q < RPT; q++) {  // record order -> rank order
    if (valid_q(q)) {
      const uint32_t r = pr[q];
      l_cnt[r] = pc[q];
      l_rel[r] = prel[q];
    }
  }
  __syncthreads();
  PH_MARK(17);
  // E consecutive ranks a thread (odd where it can be: a stride of E words is free of LDS bank conflicts)
  uint32_t E = (N + SCAN_THREADS - 1) / SCAN_THREADS;
  if (E % 2 == 0 && E < (uint32_t)RPT) E++;
  uint64_t sum = 0;  // packed (children, inline children, group heads), 21 bits each
  {
    uint32_t prev_rel = (tid * E < N && tid > 0) ? l_rel[tid * E - 1] : 0;
#pragma unroll
    for (int q = 0; q < RPT; q++) {
      const uint32_t r = tid * E + q;
      const bool in = (uint32_t)q < E && r < N;
      if (in) {
        const uint32_t c = l_cnt[r], rel = l_rel[r];
        const uint32_t hd = r == 0 || rel != prev_rel;
        prev_rel = rel;
        sum += (uint64_t)(c & 0xffffu) | ((uint64_t)(c >> 16) << 21) | ((uint64_t)hd << 42);
      }
    }
  }
  const int lane = tid & 63, wid = tid >> 6;
  uint64_t inc = sum;
  inc = wave_incscan64(inc);
  __shared__ uint64_t wsum64[SCAN_THREADS / 64];
  if (lane == 63) wsum64[wid] = inc;
  __syncthreads();
  uint64_t off = 0, tot = 0;
  for (int w = 0; w < SCAN_THREADS / 64; w++) {
    const uint64_t s = wsum64[w];
    off += w < wid ? s : 0;
    tot += s;
  }
  const uint64_t ex = off + inc - sum;
  const uint32_t tc = (uint32_t)(tot & 0x1fffffu), tinl = (uint32_t)((tot >> 21) & 0x1fffffu),
                 ng = (uint32_t)(tot >> 42);
  uint32_t bc = (uint32_t)(ex & 0x1fffffu), bi = (uint32_t)((ex >> 21) & 0x1fffffu), bh = (uint32_t)(ex >> 42);
  uint32_t g[RPT], ipr[RPT], cpr[RPT];
  {
    uint32_t prev_rel = (tid * E < N && tid > 0) ? l_rel[tid * E - 1] : 0;
#pragma unroll
    for (int q = 0; q < RPT; q++) {
      const uint32_t r = tid * E + q;
      const bool in = (uint32_t)q < E && r < N;
      uint32_t c = 0, hd = 0;
      if (in) {
        c = l_cnt[r];
        const uint32_t rel = l_rel[r];
        hd = r == 0 || rel != prev_rel;
        prev_rel = rel;
      }
      bh += hd;
      g[q] = bh - 1;
      cpr[q] = bc;
      ipr[q] = bi;
      if (in && hd) gstart[g[q]] = r;
      bc += c & 0xffffu;
      bi += c >> 16;
    }
  }
  const uint32_t last_rel = (tid == 0 && N) ? l_rel[N - 1] : 0u;  // (bookkeeping: the window's last ts)
  __syncthreads();
  PH_MARK(18);
  // per rank: inline prefix (l_cnt), group (l_rel: read above, free now), child prefix (l_slot); then each
  // thread writes its own records' sinfo (record order: coalesced for the gen-0 slots)
#pragma unroll
  for (int q = 0; q < RPT; q++) {
    const uint32_t r = tid * E + q;
    const bool in = (uint32_t)q < E && r < N;
    if (in) {
      l_cnt[r] = ipr[q];
      l_rel[r] = g[q];
      l_slot[r] = cpr[q];
    }
  }
  __syncthreads();
  // the keys / contexts the next k2_pa appends with: a local record's uid is its parent's child prefix +
  // its child index (DefaultSimulatorImpl::Schedule order); ranks cleared
#pragma unroll
  for (int q = 0; q < RPT; q++) {
    if (valid_q(q)) {
      const uint32_t r = pr[q], rc = prec[q];
      const uint32_t gg = l_rel[r];
      const uint32_t first = gstart[gg];
      const uint32_t last = (gg + 1 < ng ? gstart[gg + 1] : N) - 1;
      const uint32_t ip = l_cnt[r];
      M.sinfo[rc] = make_uint4(r + (tinl ? l_cnt[first] : 0), last + 1 + ip, l_slot[r], ip);
      if (WIDE && q >= RPT0) {  // (k2_rank wrote the dense list lrec)
        M.pwkey[rc] = ((uint64_t)prel[q] << 32) | (uint32_t)(uid0 + l_slot[ppx[q] & 0xffffu] + (ppx[q] >> 16));
        lrank_of(M, wn)[tid + q * SCAN_THREADS - WCAP] = 0;
      } else if (!run) {
        wrank_of(M, wn)[rc] = 0;
      }
    }
  }
  if (WIDE && Lt && tid < NLR) M.lcnt[tid] = 0;
  // the next chunk of a sorted run (a block search over the run's keys: every thread calls it)
  uint64_t rn1 = 0;
  bool rtrim = false;
  if (run && c_r0 + W < c_rW && !c_rtrim) run_chunk_end<SCAN_THREADS>(M, c_r0 + W, c_rW, rn1, rtrim);
  stack_and_hubs();
  PH_MARK(19);
  if (FL && tid == 0) {  // the next k2_pa appends window n from sinfo (df_book did the run bookkeeping)
    C.pK0 = wif.K0;
    C.puid0 = wif.uid0;
    C.pinl = tinl;
    C.pdf = 0;
    if (N) C.last_ts = wif.tmin + last_rel;
  }
  if (!FL && tid == 0) {
    C.acc_tc = 0;  // (k2_handle's totals: this pipeline scans its own)
    C.acc_tinl = 0;
    C.pdf = 0;
    C.pK0 = bk.K;
    C.puid0 = bk.uid;
    C.ptmin = bk.tmin;
    C.pinline_lim = bk.inline_lim;
    C.pW = W;
    C.plt = Lt;
    C.pinl = tinl;
    C.pvalid = 1;
    if (N) C.last_ts = bk.tmin + last_rel;
    C.K = bk.K + N + tinl;
    C.uid = bk.uid + tc;
    C.pchild = tc - tinl - Lt;  // (the local records' uids were consumed, they ran in the window)
    C.nfree = nfree - consumed + npush;
    const uint64_t P_end = bk.P_end + (nF > nfree ? nF - nfree : 0);
    const uint64_t live = bk.live - npush + nF;
    C.P_end = P_end;
    C.live = live;
    C.npush = 0;
    C.nF = 0;
    C.nhub = 0;
    C.force_run = 0;  // (a run chunk's slot tables may set it; it only matters for a normal window)
    uint32_t mode = c_mode;
    uint64_t r0 = bk.r0;
    bool flip = true;
    if (run) {
      r0 += W;
      C.r0 = r0;
      if (r0 >= bk.rW) {
        mode = MODE_NORMAL;
      } else if (c_rtrim) {  // the chunk ended a cut same-ts group: the run ends, k_trim returns the rest
        mode = MODE_TRIM;
      } else {
        flip = false;  // the run's chunks keep folding into the same reduction
        C.rnext = rn1;
        C.rtrim = rtrim ? 1u : 0u;
      }
    } else if (WIDE) {  // wide windows: keep them inside the window capacity (WCAP gen-0, NMAX records)
      const uint64_t span = c_bound >> 32;
      if (N > (uint32_t)(7 * NMAX / 8) || W > (uint32_t)(7 * WCAP / 8)) C.span_t = span - span / 4;
      else if (N < (uint32_t)(3 * NMAX / 4) && W < (uint32_t)(3 * WCAP / 4) && bk.span_t < (1ull << 40))
        C.span_t = bk.span_t + bk.span_t / 8 + 1;
    }
    if (flip) {
      const uint32_t rt = bk.rt;
      C.red[rt ^ 1].tmin = C.red[rt ^ 1].wend = C.red[rt ^ 1].stopts = C.red[rt ^ 1].wendw = ~0ull;  // consumed
      C.rt = rt ^ 1;
    }
    const uint64_t windows = bk.windows + 1;
    C.windows = windows;
    if (N > bk.max_window) C.max_window = N;
    C.W = 0;
    const uint64_t pending = live + (tc - tinl - Lt) + ((mode == MODE_RUN || mode == MODE_TRIM) ? bk.rW - r0 : 0);
    bool done = bk.stop_seen || (pending == 0 && bk.hts == ~0ull);
    if (P_end > M.pool_cap) {
      atomicOr(M.error, 1u);
      done = true;
    }
    if (windows >= bk.max_windows && !done) {
      atomicOr(M.error, 4u);
      done = true;
    }
    if ((uint64_t)bk.uid + tc > (uint64_t)UID_MAX_NEXT) {  // (fails before any child with a wrapped uid runs)
      atomicOr(M.error, 2048u);
      done = true;
    }
    if (done) {
      C.done = 1;
      if (mode == MODE_TRIM) mode = MODE_NORMAL;  // (the final window is appended by the next k2_pa)
    } else if (mode == MODE_NORMAL && bk.hcap) {  // the window was cut at the next host closure: pause
      C.hcap = 0;
      mode = MODE_HOST;
    } else if (mode == MODE_NORMAL && P_end > 65536 && live * 4 < P_end) {
      mode = MODE_COMPACT;
    }
    if (mode != c_mode) C.mode = mode;
  }
  PH_MARK(20);
  BLK_REC(2, c_win);
}

// ---- the deferred pipeline's flush, second part: every provisional uid still pending (children of window
// n - 1 in the pool, and in the window records when window n became a sorted run) resolves; afterwards the
// next k2_pa appends from sinfo (pdf = 0) and the other pipeline can take over.  (Grid-stride.)
__global__ __launch_bounds__(256) void k_xlate(const P2PDev M) {
  Ctl &C = *M.C;
  const uint64_t wn = C.windows;  // n + 1 (df_book counted window n), or n when window n became a sorted run
  const uint64_t P = C.P_end;
  const bool sorted = C.mode == MODE_SORT;
  const uint64_t nw = sorted ? C.rW : 0;
  const uint64_t wq = sorted ? wn + 3 : wn + 2;  // window n - 1 (mod 4: its parity, its winfo slot)
  const uint32_t uq = C.winfo[wq & 3].uid0;
  const uint32_t *cq = M.cpt + (uint64_t)(wq & 1) * NMAX;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < P; i += stride) {
    const uint32_t u = M.ev_uid[0][i];
    if (M.ev_ts[0][i] != TOMB && (u & PROV)) {
      if (((u >> 30) & 1u) != (uint32_t)(wq & 1)) atomicOr(M.error, 256u);
      M.ev_uid[0][i] = uq + cq[stg_pos(((u & 0x3fffffffu) >> 8) % NMAX)] + (u & 0xffu);
    }
  }
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nw; i += stride) {
    const uint64_t k = M.wkey[i];
    const uint32_t u = (uint32_t)k;
    if (u & PROV) {
      if (((u >> 30) & 1u) != (uint32_t)(wq & 1)) atomicOr(M.error, 256u);
      M.wkey[i] = (k & ~0xffffffffull) | (uint32_t)(uq + cq[stg_pos(((u & 0x3fffffffu) >> 8) % NMAX)] + (u & 0xffu));
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) C.pdf = 0;
}

// ---- local records' trace uids (traced wide engines): records made by this window's handlers carry
// their record index (flagged in pad_) until k2_scan has assigned the record's uid
__global__ __launch_bounds__(256) void k_tpatch(const P2PDev M) {
  const Ctl &C = *M.C;
  if (!M.trace || C.plt == 0) return;
  const uint64_t t0 = C.tn0, tn = *M.trace_n;
  const uint64_t t1 = tn < M.trace_cap ? tn : M.trace_cap;
  for (uint64_t i = t0 + (uint64_t)blockIdx.x * 256 + threadIdx.x; i < t1; i += (uint64_t)gridDim.x * 256) {
    if (M.trace[i].pad_) {  // a local record's: uid holds its record index
      M.trace[i].uid = (uint32_t)M.pwkey[M.trace[i].uid];
      M.trace[i].pad_ = 0;
    }
  }
}

// ================================ host-driven steps (rare) ================================
// ---- LSD radix sort of (key, slot) pairs: 8-bit digits, tiles of RS_TILE, stable ----
constexpr int RS_T = 256, RS_IPT = 16, RS_TILE = RS_T * RS_IPT;

// OR of the keys (-> the significant bits, i.e. the digit passes the sort needs).
__global__ __launch_bounds__(256) void k_rs_or(const uint64_t *__restrict__ keys, uint64_t n, unsigned long long *out) {
  uint64_t v = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) v |= keys[i];
  for (int o = 32; o > 0; o >>= 1) v |= __shfl_xor(v, o);
  if ((threadIdx.x & 63) == 0 && v) atomicOr(out, (unsigned long long)v);
}

__global__ __launch_bounds__(RS_T) void k_rs_hist(const uint64_t *__restrict__ keys, uint64_t n, int shift,
                                                  uint32_t *__restrict__ hist, uint32_t ntiles) {
  __shared__ uint32_t h[256];
  h[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t b0 = (uint64_t)blockIdx.x * RS_TILE;
#pragma unroll 4
  for (int k = 0; k < RS_IPT; k++) {
    const uint64_t i = b0 + (uint64_t)k * RS_T + threadIdx.x;
    if (i < n) atomicAdd(&h[(keys[i] >> shift) & 255u], 1u);
  }
  __syncthreads();
  hist[(uint64_t)threadIdx.x * ntiles + blockIdx.x] = h[threadIdx.x];
}

// Exclusive scan of m counts in place (digit-major: every tile's offset of every digit), one block.
__global__ __launch_bounds__(1024) void k_rs_scan(uint32_t *__restrict__ hist, uint64_t m) {
  __shared__ uint32_t wsum[16];
  __shared__ uint32_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (uint64_t c0 = 0; c0 < m; c0 += 4096) {
    uint32_t v[4], s = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const uint64_t i = c0 + threadIdx.x * 4 + q;
      v[q] = i < m ? hist[i] : 0u;
      s += v[q];
    }
    uint32_t tot;
    const uint32_t ex = block_exscan<1024>(s, wsum, &tot);
    uint32_t run = carry + ex;
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const uint64_t i = c0 + threadIdx.x * 4 + q;
      if (i < m) hist[i] = run;
      run += v[q];
    }
    __syncthreads();
    if (threadIdx.x == 0) carry += tot;
    __syncthreads();
  }
}

__global__ __launch_bounds__(RS_T) void k_rs_scatter(const uint64_t *__restrict__ kin, const uint32_t *__restrict__ vin,
                                                     uint64_t *__restrict__ kout, uint32_t *__restrict__ vout,
                                                     uint64_t n, int shift, const uint32_t *__restrict__ hist,
                                                     uint32_t ntiles) {
  __shared__ uint32_t off[256];
  __shared__ uint32_t wc[RS_T / 64][256];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  off[tid] = hist[(uint64_t)tid * ntiles + blockIdx.x];
  for (int w = 0; w < RS_T / 64; w++) wc[w][tid] = 0;
  __syncthreads();
  const uint64_t b0 = (uint64_t)blockIdx.x * RS_TILE;
  const uint64_t below = (1ull << lane) - 1ull;
  for (int k = 0; k < RS_IPT; k++) {
    const uint64_t i = b0 + (uint64_t)k * RS_T + tid;
    const bool valid = i < n;
    const uint64_t key = valid ? kin[i] : 0;
    const uint32_t v = valid ? (vin ? vin[i] : (uint32_t)i) : 0u;
    const uint32_t d = (uint32_t)(key >> shift) & 255u;
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int bt = 0; bt < 8; bt++) {
      const bool bit = (d >> bt) & 1u;
      const uint64_t bb = __ballot(bit);
      peers &= bit ? bb : ~bb;
    }
    const uint32_t rank = (uint32_t)__popcll(peers & below);
    if (valid && rank == 0) wc[wid][d] = (uint32_t)__popcll(peers);
    __syncthreads();
    if (valid) {
      uint32_t o = off[d] + rank;
      for (int w = 0; w < wid; w++) o += wc[w][d];
      kout[o] = key;
      vout[o] = v;
    }
    __syncthreads();
    uint32_t t = 0;
    for (int w = 0; w < RS_T / 64; w++) {
      t += wc[w][tid];
      wc[w][tid] = 0;
    }
    off[tid] += t;
    __syncthreads();
  }
}

template <class T>
__global__ __launch_bounds__(256) void k_rs_gather(const uint32_t *__restrict__ perm, const T *__restrict__ src,
                                                   T *__restrict__ dst, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) dst[i] = src[perm[i]];
}

// ---- pool compaction: live entries of [0, P_end) -> pool 1, dense (order is irrelevant) ----
__global__ __launch_bounds__(256) void k_cmp(const P2PDev M, uint64_t P) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t b0 = ((uint64_t)blockIdx.x * 256 + threadIdx.x) & ~63ull; b0 < P; b0 += stride) {
    const uint64_t i = b0 + (threadIdx.x & 63);
    const uint64_t ts = i < P ? M.ev_ts[0][i] : TOMB;
    const bool live = ts != TOMB;
    const uint64_t o = wave_alloc64(M.cmp_cnt, live);
    if (live) {
      M.ev_ts[1][o] = ts;
      M.ev_uid[1][o] = M.ev_uid[0][i];
      M.ev_ctx[1][o] = M.ev_ctx[0][i];
      M.ev_kind[1][o] = M.ev_kind[0][i];
      M.ev_a[1][o] = M.ev_a[0][i];
      M.ev_pkt[1][o] = M.ev_pkt[0][i];
    }
  }
}

// A widened window that overflowed (sorted by k_rs_*): the records past its narrow bound go back to the
// pool, so that the run is a narrow window (every child of a run event sorts after every run event); they
// fold into the pending reduction the run's chunks accumulate, and a host cut waits for a later window.
__global__ __launch_bounds__(1024) void k_renarrow(const P2PDev M) {
  Ctl &C = *M.C;
  const uint64_t n = C.rW, nb = C.nbound, tmin = C.tmin, P0 = C.P_end;
  __shared__ uint64_t s_cut;
  if (threadIdx.x == 0) {  // the first record past the narrow bound (the records are sorted by key)
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
      const uint64_t mid = (lo + hi) >> 1;
      if (M.wkey[mid] <= nb) lo = mid + 1;
      else hi = mid;
    }
    s_cut = lo;
  }
  __syncthreads();
  const uint64_t cut = s_cut, m = n - cut;
  if (P0 + m > M.pool_cap) {
    if (threadIdx.x == 0) atomicOr(M.error, 1u);
    return;
  }
  Red &R = C.red[C.rt];
  uint64_t tmn = ~0ull, wnd = ~0ull, wndw = ~0ull;
  for (uint64_t i = cut + threadIdx.x; i < n; i += 1024) {
    const uint64_t key = M.wkey[i];
    const uint64_t ts = tmin + (key >> 32);
    const uint32_t kind = M.wkind[i];
    const uint64_t d = P0 + (i - cut);
    M.ev_ts[0][d] = ts;
    M.ev_uid[0][d] = (uint32_t)key;
    M.ev_ctx[0][d] = M.wctx[i];
    M.ev_kind[0][d] = kind;
    M.ev_a[0][d] = M.wa[i];
    M.ev_pkt[0][d] = M.wpkt[i];
    tmn = ts < tmn ? ts : tmn;
    const uint64_t x = ts + (uint64_t)M.lookahead[kind & 0xffu], xw = ts + (uint64_t)M.lookw[kind & 0xffu];
    wnd = x < wnd ? x : wnd;
    wndw = xw < wndw ? xw : wndw;
    if ((kind & 0xffu) == K_STOP) {
      R.stopts = ts;
      R.stopuid = (uint32_t)key;
    }
  }
  publish_min<1024, true>(R, tmn, wnd, wndw);
  if (threadIdx.x == 0) {
    C.P_end = P0 + m;
    C.live += m;
    C.rW = cut;
    C.renarrow = 0;
    const uint64_t edge = nb >> 32;
    C.hrel = C.hrel < edge ? C.hrel : edge;
    if (m) C.hcap = 0;  // (the host event's key is past the trimmed run: a later window reaches it)
  }
}

// Mode transitions the host makes after a host-driven step.
__global__ __launch_bounds__(1024) void k_after_sort(const P2PDev M) {
  const uint64_t rW = M.C->rW;
  uint64_t r1 = 0;
  bool trim = false;
  if (rW) run_chunk_end<1024>(M, 0, rW, r1, trim);
  if (threadIdx.x != 0) return;
  M.C->mode = MODE_RUN;
  M.C->r0 = 0;
  M.C->rnext = r1;
  M.C->rtrim = trim ? 1u : 0u;
  M.C->lim_rel = 0;  // (a run has no local records)
}

// A run that ended after a cut same-ts group (run_chunk_end): its records [r0, rW) go back to the pool and
// fold into the reduction that bounds the next window (k2_scan flipped rt when it asked for the trim).
__global__ __launch_bounds__(1024) void k_trim(const P2PDev M) {
  Ctl &C = *M.C;
  const uint64_t cut = C.r0, n = C.rW, tmin = C.tmin, P0 = C.P_end, m = n - cut;
  if (P0 + m > M.pool_cap) {
    if (threadIdx.x == 0) atomicOr(M.error, 1u);
    return;
  }
  Red &R = C.red[C.rt ^ 1];
  uint64_t tmn = ~0ull, wnd = ~0ull, wndw = ~0ull;
  for (uint64_t i = cut + threadIdx.x; i < n; i += 1024) {
    const uint64_t key = M.wkey[i];
    const uint64_t ts = tmin + (key >> 32);
    const uint32_t kind = M.wkind[i];
    const uint64_t d = P0 + (i - cut);
    M.ev_ts[0][d] = ts;
    M.ev_uid[0][d] = (uint32_t)key;
    M.ev_ctx[0][d] = M.wctx[i];
    M.ev_kind[0][d] = kind;
    M.ev_a[0][d] = M.wa[i];
    M.ev_pkt[0][d] = M.wpkt[i];
    tmn = ts < tmn ? ts : tmn;
    const uint64_t x = ts + (uint64_t)M.lookahead[kind & 0xffu], xw = ts + (uint64_t)M.lookw[kind & 0xffu];
    wnd = x < wnd ? x : wnd;
    wndw = xw < wndw ? xw : wndw;
    if ((kind & 0xffu) == K_STOP) {
      R.stopts = ts;
      R.stopuid = (uint32_t)key;
    }
  }
  publish_min<1024, true>(R, tmn, wnd, wndw);
  if (threadIdx.x == 0) {
    C.P_end = P0 + m;
    C.live += m;
    C.rW = cut;
    C.rtrim = 0;
    if (m) C.hcap = 0;  // (the host event's key is past these: a later window reaches it)
    C.mode = MODE_NORMAL;
  }
}
__global__ void k_after_uidx(const P2PDev M) {
  if (M.C->mode == MODE_UIDX) M.C->mode = MODE_NORMAL;
}
__global__ void k_after_compact(const P2PDev M, uint64_t live) {
  M.C->P_end = live;
  M.C->live = live;
  M.C->nfree = 0;
  M.C->mode = MODE_NORMAL;
}

// ---- mixed host / device runs (nsgpu_p2p_advance, nsgpu_p2p_inject_send) ----
// Resume after a pause for the host: the next host key, and the uid / dispatch counters the host
// closures advanced (every host dispatch and Schedule call counts, as in DefaultSimulatorImpl).
__global__ void k_host_resume(const P2PDev M, uint64_t hts, uint32_t huid, uint32_t uid, uint64_t K) {
  Ctl &C = *M.C;
  C.hts = hts;
  C.huid = huid;
  C.uid = uid;
  C.K = K;
  if (C.mode == MODE_HOST) C.mode = MODE_NORMAL;
}

__global__ void k_set_uid(const P2PDev M, uint32_t uid) { M.C->uid = uid; }
// The run control copied into a pinned host snapshot by one wave on the engine's stream (drive's per-replay
// check without a copy-engine transfer between two graph replays; the event after it publishes the stores)
static_assert(sizeof(Ctl) % 4 == 0, "Ctl in words");
__global__ __launch_bounds__(64) void k_snap(const Ctl *__restrict__ c, Ctl *__restrict__ out) {
  const uint32_t *s = reinterpret_cast<const uint32_t *>(c);
  uint32_t *d = reinterpret_cast<uint32_t *>(out);
  for (uint32_t i = threadIdx.x; i < (uint32_t)(sizeof(Ctl) / 4); i += 64) d[i] = s[i];
}

// A host application's UdpSocket::Send of one datagram of application `a`'s flow, made by the host
// closure running now (uid `cur`): the same steps as OnOffApplication::SendPacket's send
// (onoff-application.cc:226-236 -> udp-socket-impl.cc DoSendTo -> Ipv4L3Protocol::Send -> the device),
// its Schedule calls taking uids from uid0.  The children become pending in place and fold into the
// reduction that bounds the next window.
// `room`: the uids left below UID_MAX_NEXT; a send whose Schedule calls would need more writes no child, sets the
// sticky uid error (2048) and reports out[2] = 1 (DefaultSimulatorImpl's m_uid would wrap there).
__global__ void k_inject(const P2PDev M, uint32_t a, uint64_t now, uint32_t cur, uint32_t ctx, uint32_t seq,
                         uint64_t room, uint32_t *out) {
  Ctl &C = *M.C;
  Emit E;
  E.now = now;
  E.ctx = ctx;  // the host closure's context: its Schedule calls inherit it
  E.slot0 = 0;
  E.n = 0;
  E.ch_ts = M.f_ts;  // (the fresh buffer is empty while the pipeline is paused)
  E.ch_ctx = M.f_ctx;
  E.ch_kind = M.f_kind;
  E.ch_a = M.f_a;
  E.ch_pkt = M.f_pkt;
  E.lookahead = M.lookahead;
  E.lookw = M.lookw;
  E.tmn = ~0ull;
  E.wnd = ~0ull;
  E.wndw = ~0ull;
  E.lim_abs = 0;  // (no window is forming: the children are pending)
  E.lj = -1;
  E.uid = cur, E.tloc = false;
  E.trseq = seq;
  E.demote = false;
  const uint32_t sz = M.app_pkt_size[a];
  Pkt p{a, 0, sz + 8 + 20, M.app_ttl[a]};
  M.appc[a].tx_packets++;
  M.appc[a].tx_bytes += sz;
  const uint32_t an = M.app_node[a];
  const uint32_t o = route_of(M, an, p);
  if (o == 0xffffffffu) {
    C.no_route++;
  } else {
    p.ipid = M.node_ipid[an]++;
    device_act(M, E, Act{ACT_SEND, o, p});
  }
  const uint32_t uid0 = C.uid;
  out[2] = 0;
  if ((uint64_t)E.n > room) {
    atomicOr(M.error, 2048u);
    out[0] = uid0;
    out[1] = E.trseq;
    out[2] = 1;
    return;
  }
  for (uint32_t j = 0; j < E.n; j++) {
    uint64_t dst;
    if (C.nfree) dst = M.fstack[--C.nfree];
    else dst = C.P_end++;
    if (dst >= M.pool_cap) {
      atomicOr(M.error, 1u);
      break;
    }
    M.ev_ts[0][dst] = M.f_ts[j];
    M.ev_uid[0][dst] = uid0 + j;
    M.ev_ctx[0][dst] = M.f_ctx[j];
    M.ev_kind[0][dst] = M.f_kind[j];
    M.ev_a[0][dst] = M.f_a[j];
    M.ev_pkt[0][dst] = M.f_pkt[j];
    C.live++;
  }
  Red &R = C.red[C.rt ^ 1];  // bounds the next window (k2_scan flipped rt)
  if (E.tmn < R.tmin) R.tmin = E.tmn;
  if (E.wnd < R.wend) R.wend = E.wnd;
  if (E.wndw < R.wendw) R.wendw = E.wndw;
  C.uid = uid0 + E.n;
  out[0] = C.uid;
  out[1] = E.trseq;
}
