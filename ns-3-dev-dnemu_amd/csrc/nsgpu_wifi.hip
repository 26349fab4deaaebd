// nsgpu_wifi.hip — the Wi-Fi PHY receive subset on the device (include/nsgpu.h: nsgpu_wifi_*).
//
// Replaces, for a transmission schedule fixed before Run (nsgpu_wifi_scenario, the wifi-test.cc:181-260
// harness shape): YansWifiPhy::SendPacket (yans-wifi-phy.cc:499-522) -> YansWifiChannel::Send
// (yans-wifi-channel.cc:77-115) -> YansWifiChannel::Receive (:117-122) -> YansWifiPhy::StartReceivePacket
// (yans-wifi-phy.cc:399-496) with InterferenceHelper::Add / AppendEvent / GetEnergyDuration
// (interference-helper.cc:129-212, 365-391), the WifiPhyStateHelper transitions
// (wifi-phy-state-helper.cc:122-183, 254-322, 391-423) and EndReceive's state part (yans-wifi-phy.cc:770-799).
//
// Decomposition.  A phy's receive state (NiChanges, m_firstPower, m_rxing, m_endTx/Rx/CcaBusy) is touched
// only by the events addressed to it: the Receive events of the other phys' transmissions, its own
// SendPacket calls and its own EndReceive events.  With the schedule fixed, each phy's event sequence is
// known up front, so lane j runs phy j's sequence in (ts, uid) order (k_wifi_phy).  Lane j computes the
// fan-out arithmetic of receiver j itself (distance, loss chain, delay: the 64-B fan-out record of
// nsgpu_fanout_yans never goes to HBM) while it consumes the transmission.
//
// Order inside one phy needs no global uid.  Uids are handed out in dispatch order, and every
// transmission's uid is a setup uid (below every run-time uid), so between two events of phy j at the
// same ts:
//   SendPacket before any Receive / EndReceive;
//   Receive(T1) before Receive(T2)       iff T1 precedes T2 in the schedule (their fan-outs' uid bases);
//   Receive(T) before EndReceive(R)      iff T was dispatched before the syncing Receive R: t_T <= ts_R;
//   EndReceive(R1) before EndReceive(R2) iff R1 precedes R2 (ts, then schedule order).
// A transmission's arrivals come at t_T + d with d > 0, so the next Receive of phy j is the smallest arrival
// among the transmissions t_T below it: a 64-transmission window after the first unconsumed one.
//
// The uids follow from counts (k_sync_hist, k_tx_base, k_sync_place, k_sync_rank): a Receive's syncing
// consumes one uid (the EndReceive), a transmission's fan-out consumes one per receiver.  With
// F(k) = fan-out uids of transmissions [0, k) and S(x) = syncs dispatched before x:
//   uid base of transmission k = uid_start + F(k) + #{syncs R: ts_R < t_k}
//   uid of EndReceive(R)       = uid_start + F(#{T: t_T <= ts_R}) + #{syncs before R in (ts, uid) order}.
// Syncs are bucketed by the number of transmissions before them; a bucket holds the syncs between two
// transmission times, so ranking inside it is a short scan.
//
// Roofline: latency-bound per phy (a serial chain of dependent list updates); per Receive event the
// algorithmic HBM traffic is the transmission descriptor read (broadcast, 48 B, cache-resident) plus the
// NiChange entries touched (2 x 16 B written, ~2 x 16 B read).  DESIGN.md §4.6 states the figures.
#include <algorithm>
#include <vector>
#include "nsgpu_device.h"
#include "nsgpu_internal.h"

namespace nsgpu {
namespace {

constexpr uint64_t INF = ~0ull;
constexpr uint32_t NONE = 0xffffffffu;
constexpr int PE_CAP = 8;  // pending EndReceive events of one phy: the live one + cancelled ones
// Diagnostic build only (-DNSGPU_PHASE_PROF, lib/libnsgpu_prof.so): lane 0 of each wave accumulates
// s_memtime deltas between the per-phy loop's sections (scripts/wifi_phases.py reads them).
#ifdef NSGPU_PHASE_PROF
__device__ unsigned long long g_wifi_ph[16];
#define WPH_T0() uint64_t wph_t = __builtin_amdgcn_s_memtime(); uint64_t wph[10] = {};
#define WPH(i)                                              \
  {                                                         \
    const uint64_t t_ = __builtin_amdgcn_s_memtime();       \
    wph[i] += t_ - wph_t;                                   \
    wph_t = t_;                                             \
  }
#define WPH_END()                                                                              \
  if ((threadIdx.x & 63) == 0) {                                                               \
    uint64_t w_ = 0;                                                                           \
    for (int q_ = 0; q_ < 10; q_++) {                                                          \
      atomicAdd(&g_wifi_ph[q_], (unsigned long long)wph[q_]);                                  \
      w_ += wph[q_];                                                                           \
    }                                                                                          \
    atomicMax(&g_wifi_ph[14], (unsigned long long)w_); /* the slowest wave */                  \
    atomicAdd(&g_wifi_ph[15], 1ull);                   /* waves */                             \
  }
#else
#define WPH_T0()
#define WPH(i)
#define WPH_END()
#endif
// (ERR_LDS: a SplitNi queue outgrew its LDS capacity — the run is repeated on the HBM ring store)
constexpr uint32_t ERR_WINDOW = 1, ERR_NICAP = 2, ERR_TX_IN_TX = 4, ERR_PENDING = 8, ERR_SYNCCAP = 16, ERR_LDS = 32;
enum Acc { A_DIGEST, A_DISPATCHED, A_RX, A_SYNC, A_DROP_RX, A_DROP_TX, A_DROP_ED, A_CCA_EVAL, A_CCA_SWITCH,
           A_END, A_END_CANCELLED, A_NI_INSERTS, A_NEAR, A_NI_MAX, A_LAST_TS, A_N };

struct NiEnt {  // InterferenceHelper::NiChange (interference-helper.cc:91-110)
  int64_t t;
  double d;
};

struct SyncRec {  // one syncing Receive, i.e. one EndReceive
  uint64_t ts;      // the Receive
  uint64_t end_ts;  // its EndReceive
  uint32_t tx, phy;
  uint32_t flags;   // NSGPU_WIFI_END_*
  uint32_t m;       // transmissions dispatched before the Receive (t_T <= ts)
  uint32_t uid;     // the Receive's uid
  uint32_t pad_;
};

struct TxDesc {  // one transmission, packed for the per-phy scan (64 B: four 16-B loads)
  double x, y, z;  // the sender's position
  double dbm;      // txPowerDbm
  uint64_t ts;
  int64_t dur;     // CalculateTxDuration
  uint32_t phy, chan;
  uint32_t pad_[2];
};

struct WifiDev {
  int64_t nphy;
  int64_t j0, nown;  // the receivers this engine runs: phys [j0, j0 + nown) (a partition; all of them alone)
  uint32_t ktx;  // dispatched transmissions: those with a key below the Stop event's
  uint32_t uid_start;
  const double *x, *y, *z;
  const uint32_t *chan, *chan_rank;
  nsgpu_loss_chain loss;
  double speed, rx_gain_db, edW, ccaW;
  uint64_t stop_ts;
  const uint64_t *tx_ts;
  const uint32_t *tx_phy, *tx_chan, *tx_uid;
  const int64_t *tx_dur;
  const double *tx_dbm, *tx_x, *tx_y, *tx_z;
  const TxDesc *txd;
  const uint64_t *fcum;  // [ktx + 1] fan-out uids of transmissions [0, k)
  const uint32_t *own_off, *own_idx;
  uint32_t ni_mask;
  NiEnt *ni;  // [nphy][ni_mask + 1] ring of each phy's NiChanges
  SyncRec *sync;
  unsigned long long *n_sync;
  uint64_t sync_cap;
  nsgpu_wifi_phy_counters *pc;
  nsgpu_wifi_rx_log *rx_log;  // nullable: [ktx][nphy]
  unsigned long long *acc;    // [A_N]
  uint32_t *err;
  uint32_t *hist, *off, *cur, *bucket, *base;
  nsgpu_wifi_end_record *ends;
  struct RxPre *pre;  // nullable: [nphy][ktx] receptions computed up front (k_wifi_rx)
  const struct TsDur *tsdur;  // [ktx] (ts, dur) of every transmission, packed for the per-phy scan
  struct RxS *srt;            // nullable: [nphy][ktx] each row of `pre` in (arrival, transmission) order
  const uint32_t *wlo, *whi;  // [ktx] the transmissions whose arrivals can interleave with k's (sorted rows)
};

// One (receiver, transmission) pair computed up front by k_wifi_rx: the Receive's arrival and its
// rxPowerW, or a marker (PRE_OWN: the receiver's own SendPacket, PRE_NONE: another channel, no Receive).
struct RxPre {
  uint64_t at;
  double w;
};
constexpr uint64_t PRE_NONE = ~0ull, PRE_OWN = ~0ull - 1;
struct TsDur {  // a TxDesc's (ts, dur) half-line
  uint64_t ts;
  int64_t dur;
};
static_assert(offsetof(TxDesc, dur) == offsetof(TxDesc, ts) + 8 && offsetof(TxDesc, ts) % 16 == 0, "TsDur view");
// One entry of a sorted reception row (k_wifi_rx_sort): a phy's Receives in their dispatch order — (arrival,
// then uid, i.e. transmission index) — with the markers of `pre` kept at their transmission's ts.
struct RxS {
  uint64_t at;   // arrival, or PRE_OWN / PRE_NONE
  double w;      // rxPowerW
  uint64_t tts;  // the transmission's ts
  uint32_t k;    // the transmission
  uint32_t dur;  // its duration (ns; < 2^32, checked at create)
};

// ConstantSpeedPropagationDelayModel::GetDelay + DefaultSimulatorImpl::ScheduleWithContext's m_currentTs +
__device__ __forceinline__ uint64_t arrival(const WifiDev &D, uint32_t k, double px, double py, double pz,
                                            double &dist) {
  dist = distance3(D.tx_x[k], D.tx_y[k], D.tx_z[k], px, py, pz);  // GetDistanceFrom (sender, receiver)
  return D.tx_ts[k] + (uint64_t)seconds_to_ts(dist / D.speed);
}

// InterferenceHelper::AddNiChangeEvent (interference-helper.cc:378-383): insert at upper_bound (time).
__device__ __forceinline__ void ni_insert(NiEnt *ring, uint32_t head, uint32_t &len, uint32_t m, int64_t t, double d) {
  uint32_t q = len;
  while (q > 0) {
    const NiEnt e = ring[(head + q - 1) & m];
    if (e.t <= t) break;
    ring[(head + q) & m] = e;
    q--;
  }
  ring[(head + q) & m] = NiEnt{t, d};
  len++;
}

__device__ __forceinline__ bool near_thr(double v, double thr) { return fabs(v - thr) <= 1e-9 * thr; }

__global__ void k_rx_log_init(nsgpu_wifi_rx_log *log, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    log[i] = nsgpu_wifi_rx_log{0, 0, NSGPU_WIFI_NOT_RUN, 0, 0, 0};
}

constexpr int NB = 8;  // ring entries loaded per batch (independent loads, one latency)

// Advances the prefix cursor over the ring entries [cur_n, len) with t < lim (fold: t <= lim).  The cursor
// caches m_firstPower + d_0 + ... + d_{cur_n - 1}, summed in list order exactly like the reference's loops
// (AppendEvent's fold, GetEnergyDuration's walk).  Entries under the cursor are in the past, so no
// insertion (always at upper_bound (t >= now)) lands before it.
template <bool LE>
__device__ __forceinline__ void cursor_advance(const NiEnt *ring, uint32_t head, uint32_t len, uint32_t m,
                                               int64_t lim, uint32_t &cur_n, double &cur_s) {
  while (cur_n < len) {
    NiEnt e[NB];
#pragma unroll
    for (int u = 0; u < NB; u++) e[u] = ring[(head + cur_n + u) & m];
#pragma unroll
    for (int u = 0; u < NB; u++) {
      if (cur_n >= len || (LE ? e[u].t > lim : e[u].t >= lim)) return;
      cur_s += e[u].d;
      cur_n++;
    }
  }
}

// ---- InterferenceHelper::m_niChanges stores (the list a phy's Receive events read and update) ----
// Both keep the reference list's order and its length (len: ni_cap, NiChange counts) and sum in list
// order; they differ in where the entries live.
//
// RingNi: the list as one time-sorted ring per phy in HBM, insertions shifting entries from the back
// (r02's kernel; the fallback when SplitNi's queues would not fit LDS).
struct RingNi {
  NiEnt *ring;
  uint32_t m, head, len, cur_n;  // cur_n: prefix cursor, entries [0, cur_n) summed into cur_s
  double cur_s;
  __device__ __forceinline__ uint32_t length() const { return len; }
  __device__ __forceinline__ bool room() const { return len + 2 <= m + 1; }
  __device__ __forceinline__ bool phys_room() const { return true; }
  __device__ __forceinline__ void on_receive(int64_t) {}
  // AppendEvent, not receiving (interference-helper.cc:192-212): fold the entries up to upper_bound (now)
  // into m_firstPower, drop them, the new entry first; returns m_firstPower
  __device__ __forceinline__ double fold_start(int64_t nw, double p) {
    cursor_advance<true>(ring, head, len, m, nw, cur_n, cur_s);
    head = (head + cur_n) & m;
    len -= cur_n;
    cur_n = 0;
    head = (head - 1) & m;
    ring[head] = NiEnt{nw, p};
    len++;
    return cur_s;
  }
  __device__ __forceinline__ void insert_start(int64_t nw, double p) { ni_insert(ring, head, len, m, nw, p); }
  __device__ __forceinline__ void insert_end(int64_t t, double d) { ni_insert(ring, head, len, m, t, d); }
  // GetEnergyDuration (interference-helper.cc:171-190): the entries before now only add up (the cursor
  // holds their sum); then noise += delta in list order until it drops below the threshold
  __device__ __forceinline__ int64_t energy_end(int64_t nw, double ccaW, uint32_t &flags) {
    cursor_advance<false>(ring, head, len, m, nw, cur_n, cur_s);
    double noise = cur_s;
    int64_t end = nw;
    for (uint32_t q = cur_n; q < len; q += NB) {
      NiEnt en[NB];
#pragma unroll
      for (int u = 0; u < NB; u++) en[u] = ring[(head + q + u) & m];
      bool stop = false;
#pragma unroll
      for (int u = 0; u < NB; u++) {
        if (q + u >= len) {
          stop = true;
          break;
        }
        noise += en[u].d;
        end = en[u].t;  // >= now: the cursor stopped at the first entry not before now
        if (near_thr(noise, ccaW)) flags |= NSGPU_WIFI_F_NEAR_CCA;
        if (noise < ccaW) {
          stop = true;
          break;
        }
      }
      if (stop) break;
    }
    return end;
  }
};

// SplitNi: the same list as two time-sorted queues in LDS — S, the start entries (+P at a Receive), and
// E, the end entries (-P at Receive + duration) — whose merge by time is the list: an end at t was
// inserted at t - duration < t, so before every start at t (upper_bound puts later insertions after
// equal times), and within S and within E insertion order is list order.  The cursor is eager: every
// Receive first sums the entries before now into cur_s and drops them from the queues (no insertion
// lands before the cursor, and the sums run in list order, so the values are the ring's).  Then
//   a start insertion is an append to S (every start is at or before now), not a shift over the ~100
//     pending ends a busy channel holds;
//   the live entries are only those at or after now: E holds at most the transmissions whose
//     [ts, ts + max delay + duration] interval covers one instant (host bound -> its LDS capacity), S the
//     starts at exactly now;
//   GetEnergyDuration walks E's entries at now, then S, then the rest of E, from LDS.
// `ndead` counts the summed entries the reference list still holds (until the next fold), so length()
// is the reference's list length.
struct SplitNi {
  int64_t *st, *et;  // this phy's S / E rings (LDS)
  double *sd, *ed;
  double *ec;        // E's running sums: ec[i] = cb + d[head] + ... + d[i] (summed in queue order)
  uint32_t scap, ecap, cap;  // queue capacities; cap = ni_cap (the reference list's limit)
  uint32_t hs, ns, he, ne, ndead;
  double cur_s;
  double cb;         // the running sum before E's head
  uint32_t nsum;     // terms summed into ec since its last rebase
  // the queues' heads in registers (INT64_MAX: empty), so that a cursor step is one LDS trip (the next
  // head's loads, issued together) instead of three dependent ones
  int64_t hte, hts;
  double hde, hce, hds;
  int64_t tte;  // E's tail: its time and running sum (valid while ne > 0): an append reads no LDS
  double tce;
  __device__ __forceinline__ void reload_e() {
    if (ne) {
      const uint32_t x = ex(0);
      hte = et[x];
      hde = ed[x];
      hce = ec[x];
    } else {
      hte = INT64_MAX;
    }
  }
  __device__ __forceinline__ void reload_s() {
    if (ns) {
      const uint32_t x = sx(0);
      hts = st[x];
      hds = sd[x];
    } else {
      hts = INT64_MAX;
    }
  }
  __device__ __forceinline__ uint32_t sx(uint32_t i) const {
    const uint32_t x = hs + i;
    return x < scap ? x : x - scap;
  }
  __device__ __forceinline__ uint32_t ex(uint32_t i) const {
    const uint32_t x = he + i;
    return x < ecap ? x : x - ecap;
  }
  __device__ __forceinline__ uint32_t length() const { return ndead + ns + ne; }
  __device__ __forceinline__ bool room() const { return length() + 2 <= cap; }
  __device__ __forceinline__ bool phys_room() const { return ns + 1 <= scap && ne + 1 <= ecap; }
  // sums the merged entries with t < lim (LE: t <= lim) into cur_s and drops them
  template <bool LE>
  __device__ __forceinline__ void advance(int64_t lim) {
    for (;;) {
      const bool e = hte <= hts;  // E first on equal times
      const int64_t t = e ? hte : hts;
      if (t == INT64_MAX || (LE ? t > lim : t >= lim)) return;
      if (e) {
        cur_s += hde;
        cb = hce;
        he = he + 1 == ecap ? 0 : he + 1;
        ne--;
        reload_e();
      } else {
        cur_s += hds;
        hs = hs + 1 == scap ? 0 : hs + 1;
        ns--;
        reload_s();
      }
      ndead++;
    }
  }
  __device__ __forceinline__ void on_receive(int64_t nw) { advance<false>(nw); }
  __device__ __forceinline__ double fold_start(int64_t nw, double p) {
    advance<true>(nw);  // (S is empty after it: every start is at or before now)
    ndead = 0;
    st[sx(0)] = nw;
    sd[sx(0)] = p;
    ns = 1;
    hts = nw;
    hds = p;
    return cur_s;
  }
  __device__ __forceinline__ void insert_start(int64_t nw, double p) {
    st[sx(ns)] = nw;
    sd[sx(ns)] = p;
    if (ns == 0) hts = nw, hds = p;
    ns++;
  }
  __device__ __forceinline__ void insert_end(int64_t t, double d) {  // upper_bound (t) from the back
    uint32_t q = ne;
    double c;
    if (ne == 0 || tte <= t) {  // an append (ends usually come in time order: equal durations)
      const uint32_t x = ex(ne);
      et[x] = t;
      ed[x] = d;
      c = (ne ? tce : cb) + d;
      ec[x] = c;
      if (ne == 0) hte = t, hde = d, hce = c;
      ne++;
      tte = t;
    } else {
      while (q > 0) {
        const int64_t x = et[ex(q - 1)];
        if (x <= t) break;
        et[ex(q)] = x;
        ed[ex(q)] = ed[ex(q - 1)];
        q--;
      }
      et[ex(q)] = t;
      ed[ex(q)] = d;
      ne++;
      c = q ? ec[ex(q - 1)] : cb;  // the running sums from the new entry on (the old tail stays last)
      for (uint32_t i = q; i < ne; i++) {
        c += ed[ex(i)];
        ec[ex(i)] = c;
        if (i == 0) hte = t, hde = d, hce = c;  // (a new head)
      }
    }
    tce = c;
    nsum += ne - q;
    // rebase before the sums grow far past the live part (their rounding error is relative to them)
    if (nsum > 4096 || fabs(c) > 16.0 * fabs(c - cb)) {
      cb = 0.0;
      c = 0.0;
      for (uint32_t i = 0; i < ne; i++) {
        c += ed[ex(i)];
        ec[ex(i)] = c;
        if (i == 0) hce = c;
      }
      tce = c;
      nsum = ne;
    }
  }
  // GetEnergyDuration's tail by bisection over E's running sums, certified: the walk's sum after entry i
  // is v_i = noise + d_ie + ... + d_i summed in order, a = noise + (ec[i] - ec[ie - 1]) approximates it
  // within far less than dl (both are within ~(n + 4096) ulps of the real sum, relative to the terms'
  // magnitudes, which `scale` bounds), and both fall with i.  The first i with a_i < ccaW - dl after
  // an a_{i-1} >= ccaW + dl is then exactly the walk's stop, and the near-threshold tests on v_{i-1}, v_i
  // are decided when a is further than dl from the band's edge.  Otherwise (a sum within ~1e-10 of the
  // threshold or the band's edge) the exact walk runs.  Returns false when undecided.
  __device__ __forceinline__ bool tail_bisect(uint32_t ie, double noise, double ccaW, int64_t &end,
                                              uint32_t &flags) const {
    const double base = ie ? ec[ex(ie - 1)] : cb;
    const double last = tce;  // (ec of E's tail)
    const double dl = 1e-10 * (noise + fabs(base) + fabs(last));
    uint32_t lo = ie, hi = ne;  // the first i with a_i < ccaW - dl (ne: none)
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (noise + (ec[ex(mid)] - base) < ccaW - dl) hi = mid;
      else lo = mid + 1;
    }
    const double nb = 1e-9 * ccaW;  // near_thr's band
    auto near_of = [&](double a, int &r) {  // 1 / 0 when decided, else r = -1
      const double x = fabs(a - ccaW);
      r = x > nb + dl ? 0 : (x < nb - dl ? 1 : -1);
    };
    int n0 = 0, n1 = 0;
    if (lo > ie) {  // v_{lo-1}: the last sum at or above the threshold
      const double a = noise + (ec[ex(lo - 1)] - base);
      if (!(a >= ccaW + dl)) return false;
      near_of(a, n0);
    }  // (lo == ie: it is `noise` itself, tested exactly by the walk's head)
    if (lo < ne) near_of(noise + (ec[ex(lo)] - base), n1);
    if (n0 < 0 || n1 < 0) return false;
    end = et[ex(lo < ne ? lo : ne - 1)];
    if (n0 | n1) flags |= NSGPU_WIFI_F_NEAR_CCA;
    return true;
  }
  __device__ __forceinline__ int64_t energy_end(int64_t nw, double ccaW, uint32_t &flags) {
    // (on_receive advanced the cursor to now: S holds starts at now only, E ends at or after now)
    double noise = cur_s;
    int64_t end = nw;
    bool stop = false;
    auto step = [&](int64_t t, double d) {
      noise += d;
      end = t;
      if (near_thr(noise, ccaW)) flags |= NSGPU_WIFI_F_NEAR_CCA;
      stop = noise < ccaW;
    };
    uint32_t ie = 0;
    while (!stop && ie < ne && (ie ? et[ex(ie)] : hte) == nw) {  // (the heads are in registers)
      step(nw, ie ? ed[ex(ie)] : hde);
      ie++;
    }
    for (uint32_t q = 0; !stop && q < ns; q++) step(q ? st[sx(q)] : hts, q ? sd[sx(q)] : hds);
    if (stop || ie >= ne) return end;
    if (tail_bisect(ie, noise, ccaW, end, flags)) return end;
    // The tail (undecided by the bisection): end entries after now, all deltas negative, so the sums only fall (round-to-nearest is
    // monotonic).  The walk stops at the first sum below the threshold; of the sums above it the last
    // is the nearest to it, so the near-threshold test needs only that one and the stopping one, and
    // the loop needs only the deltas (the stopping entry's time is read once at the end).
    double prev = noise;
    uint32_t i = ie, si = 0;
    for (; i < ne && !stop; i += NB) {
      double bd[NB];
#pragma unroll
      for (int u = 0; u < NB; u++) bd[u] = ed[ex(i + u < ne ? i + u : i)];
#pragma unroll
      for (int u = 0; u < NB; u++) {
        if (!stop && i + u < ne) {
          prev = noise;
          noise += bd[u];
          if (noise < ccaW) stop = true, si = i + u;
        }
      }
    }
    if (stop) {
      i = si;
    } else {  // every entry added: the walk ends at the last one
      i = ne - 1;
      prev = noise;  // (the last sum is the nearest of the ones at or above the threshold)
    }
    end = et[ex(i)];
    if (near_thr(prev, ccaW) || near_thr(noise, ccaW)) flags |= NSGPU_WIFI_F_NEAR_CCA;
    return end;
  }
};

// DbmToW (yans-wifi-phy.cc:727-732) of CalcRxPower (propagation-loss-model.cc:64-74) + RxGain
__device__ __forceinline__ double rx_power_w(const WifiDev &D, double tx_dbm, double dist) {
  const double rxPowerDbm = calc_rx_power(D.loss, tx_dbm, dist) + D.rx_gain_db;
  return pow(10.0, rxPowerDbm / 10.0) / 1000.0;
}

// The fan-out arithmetic of every (receiver j, transmission k) pair, all in parallel (the per-phy
// kernel's serial chain then reads 16 B per Receive instead of running the distance / delay / loss /
// DbmToW chain itself): YansWifiChannel::Send's receiver loop (yans-wifi-channel.cc:77-115).
__global__ __launch_bounds__(256) void k_wifi_rx(const WifiDev D) {
  const uint64_t K = D.ktx, n = (uint64_t)D.nown * K;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    const uint64_t jl = i / K, k = i - jl * K, j = D.j0 + jl;  // (rows: the engine's own receivers)
    const TxDesc t = D.txd[k];
    RxPre r{PRE_NONE, 0.0};
    if (t.phy == (uint32_t)j) {
      r.at = PRE_OWN;
    } else if (t.chan == D.chan[j]) {
      const double dist = distance3(t.x, t.y, t.z, D.x[j], D.y[j], D.z[j]);
      r.at = t.ts + (uint64_t)seconds_to_ts(dist / D.speed);
      r.w = rx_power_w(D, t.dbm, dist);
    }
    D.pre[i] = r;
  }
}

// Each reception row in dispatch order: entry (j, k) goes to position #{k' : (a', k') < (a, k)} of row j, where
// a is the arrival (a marker: its transmission's ts).  Every arrival lies in [ts, ts + dmax], so transmissions
// before wlo[k] (ts' + dmax < ts) all come first and those after whi[k] (ts' > ts + dmax) all come later: only
// the window [wlo[k], whi[k]] (at most WSORT_MAX, host-checked) is compared.
__global__ __launch_bounds__(256) void k_wifi_rx_sort(const WifiDev D) {
  const uint64_t K = D.ktx, n = (uint64_t)D.nown * K;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    const uint64_t j = i / K, k = i - j * K;
    const RxPre *row = D.pre + j * K;
    const RxPre r = row[k];
    const TsDur td = D.tsdur[k];
    const uint64_t a = r.at >= PRE_OWN ? td.ts : r.at;
    const uint32_t lo = D.wlo[k], hi = D.whi[k];
    uint32_t pos = lo;
    for (uint32_t q = lo; q <= hi; q++) {
      const uint64_t b = row[q].at;
      const uint64_t bq = b >= PRE_OWN ? D.tsdur[q].ts : b;
      pos += (bq < a || (bq == a && q < k)) ? 1u : 0u;
    }
    D.srt[j * K + pos] = RxS{r.at, r.w, td.ts, (uint32_t)k, (uint32_t)td.dur};
  }
}

// A phy's pending EndReceive events (the live one + cancelled ones), one record per lane in LDS.
struct PeSlots {
  uint64_t ts[PE_CAP], sts[PE_CAP];
  uint32_t tx[PE_CAP], slot[PE_CAP], can[PE_CAP];
};

// One lane = one phy: its SendPacket / Receive / EndReceive sequence in (ts, uid) order.  MODE 0: receptions
// computed here; 1: read from k_wifi_rx's table (each scan looks at the unconsumed transmissions in order);
// 2: read in order from the sorted row (k_wifi_rx_sort), the next entry prefetched while an event runs.
template <int MODE, class Ni>
__device__ __forceinline__ void phy_run(const WifiDev &D, const int64_t j, Ni &ni, PeSlots *pe) {
  const double px = D.x[j], py = D.y[j], pz = D.z[j];
  const uint32_t ch = D.chan[j];
  // InterferenceHelper (m_niChanges: `ni`, m_firstPower) and WifiPhyStateHelper; the two m_rxing flags
  // are set and cleared together (yans-wifi-phy.cc:466-468, :510-514, :776-797)
  uint32_t ni_max = 0;
  double firstPower = 0.0;
  bool rxing = false;
  int64_t endTx = 0, endRx = 0, endCca = 0;
  // pending EndReceive events (in LDS: a lane indexes them with its own per-lane index)
  uint64_t *pe_ts = pe->ts, *pe_sts = pe->sts;
  uint32_t *pe_tx = pe->tx, *pe_slot = pe->slot, *pe_can = pe->can;
  int npe = 0, live = -1;
  int e = -1;  // the first pending EndReceive (recomputed when the set changes)
  bool e_dirty = false;
  uint64_t e_ts = INF, e_sts = 0;
  // transmissions: [p, p + 64) is the window, bit i of `done` = transmission p + i consumed here
  uint32_t p = 0;
  uint64_t done = 0;
  uint32_t oc = D.own_off[j];
  const uint32_t oe = D.own_off[j + 1];
  uint32_t ok = oc < oe ? D.own_idx[oc] : NONE;
  uint64_t ok_ts = ok != NONE ? D.txd[ok].ts : INF;
  // MODE 2: sr = the row's next unconsumed entry, nx = that entry (loaded one event ahead)
  const RxS *srow = MODE == 2 ? D.srt + (uint64_t)(j - D.j0) * D.ktx : nullptr;
  uint32_t sr = 0;
  RxS nx{};
  if (MODE == 2 && D.ktx) nx = srow[0];
  bool have_c = false;
  uint64_t c_ts = INF, c_tts = 0;
  uint32_t c_k = NONE;
  double c_dist = 0.0, c_dbm = 0.0, c_w = 0.0;
  int64_t c_dur = 0;
  uint32_t err = 0;
  nsgpu_wifi_phy_counters c = {};
  uint64_t digest = 0, disp = 0, last_ts = 0, ni_ins = 0, cca_eval = 0, near = 0;
  WPH_T0();

  for (;;) {
    if (!have_c) {  // the next Receive: the smallest arrival of an unconsumed transmission
      c_ts = INF;
      c_k = NONE;
      uint32_t at = 64;  // where the scan stopped (64: it went through the whole window)
      if (MODE == 2) {
        for (;;) {
          if (sr >= D.ktx) break;
          const RxS r = nx;
          if (r.at >= PRE_OWN) {  // our own SendPacket (taken from the own list) / another channel: no Receive
            sr++;
            if (sr < D.ktx) nx = srow[sr];
            continue;
          }
          c_ts = r.at, c_k = r.k, c_w = r.w, c_tts = r.tts, c_dur = (int64_t)r.dur;
          if (sr + 1 < D.ktx) nx = srow[sr + 1];  // (in flight while this Receive runs)
          break;
        }
        at = 0;
      } else if (MODE == 1) {
        const RxPre *row = D.pre + (uint64_t)(j - D.j0) * D.ktx;
        for (uint32_t i0 = 0; i0 < 64 && at == 64; i0 += 2) {
          TsDur tp[2];  // two transmissions per memory trip (a scan usually reads the next two)
          RxPre rp[2];
#pragma unroll
          for (int u = 0; u < 2; u++) {
            const uint32_t k = p + i0 + u;
            if (k < D.ktx) {
              tp[u] = D.tsdur[k];
              rp[u] = row[k];
            } else {
              tp[u].ts = INF;
            }
          }
#pragma unroll
          for (int u = 0; u < 2; u++) {
            const uint32_t i = i0 + u, k = p + i;
            if (at != 64) break;
            if (k >= D.ktx || tp[u].ts >= c_ts) {
              at = i;
              break;
            }
            if ((done >> i) & 1ull) continue;
            if (rp[u].at == PRE_OWN) continue;
            if (rp[u].at == PRE_NONE) {
              done |= 1ull << i;
              continue;
            }
            if (rp[u].at < c_ts) c_ts = rp[u].at, c_k = k, c_w = rp[u].w, c_tts = tp[u].ts, c_dur = tp[u].dur;
          }
        }
      } else {
      for (uint32_t i0 = 0; i0 < 64 && at == 64; i0 += 2) {
        TxDesc tp[2];  // two descriptors per memory trip (a scan usually reads the next two)
#pragma unroll
        for (int u = 0; u < 2; u++) {
          const uint32_t k = p + i0 + u;
          if (k < D.ktx) tp[u] = D.txd[k];
          else tp[u].ts = INF;
        }
#pragma unroll
        for (int u = 0; u < 2; u++) {
          const uint32_t i = i0 + u, k = p + i;
          const TxDesc &t = tp[u];
          if (at != 64) break;
          if (k >= D.ktx || t.ts >= c_ts) {  // its arrival (and every later one) comes after c_ts
            at = i;
            break;
          }
          if ((done >> i) & 1ull) continue;
          if (t.phy == (uint32_t)j) continue;  // our own SendPacket: taken in order below
          if (t.chan != ch) {                  // not on our channel: no Receive (yans-wifi-channel.cc:88-91)
            done |= 1ull << i;
            continue;
          }
          // GetDistanceFrom (sender, receiver); ConstantSpeedPropagationDelayModel::GetDelay
          const double dist = distance3(t.x, t.y, t.z, px, py, pz);
          const uint64_t a = t.ts + (uint64_t)seconds_to_ts(dist / D.speed);
          if (a < c_ts) c_ts = a, c_k = k, c_dist = dist, c_tts = t.ts, c_dbm = t.dbm, c_dur = t.dur;
        }
      }
      }
      if (MODE != 2) {
        if (at == 64 && p + 64 < D.ktx && D.txd[p + 64].ts < c_ts) {
          err |= ERR_WINDOW;
          break;
        }
        while (done & 1ull) done >>= 1, p++;
      }
      have_c = true;
    }
    WPH(9);  // the scan for the next Receive (selection: the rest)
    if (e_dirty) {  // the first pending EndReceive (ts, then the syncing Receive's key), after a change
      e = -1;
      for (int q = 0; q < npe; q++)
        if (e < 0 || pe_ts[q] < pe_ts[e] ||
            (pe_ts[q] == pe_ts[e] && (pe_sts[q] < pe_sts[e] || (pe_sts[q] == pe_sts[e] && pe_tx[q] < pe_tx[e]))))
          e = q;
      e_ts = e >= 0 ? pe_ts[e] : INF;
      e_sts = e >= 0 ? pe_sts[e] : 0;
      e_dirty = false;
    }
    WPH(0);  // selection + pending EndReceive choice
    int kind = -1;
    uint64_t now = INF;
    if (ok != NONE) kind = 0, now = ok_ts;
    if (c_k != NONE && c_ts < now) kind = 1, now = c_ts;
    if (e >= 0 && (e_ts < now || (e_ts == now && kind == 1 && c_tts > e_sts))) kind = 2, now = e_ts;
    if (kind < 0) break;
    if (kind != 0 && now >= D.stop_ts) break;  // Stop (a setup uid) runs first; nothing after it does
    const int64_t nw = (int64_t)now;

    if (kind == 0) {  // YansWifiPhy::SendPacket (yans-wifi-phy.cc:499-522)
      if (endTx > nw) {  // SwitchToTx from TX: NS_FATAL_ERROR (wifi-phy-state-helper.cc:285-287)
        err |= ERR_TX_IN_TX;
        break;
      }
      if (rxing) {  // m_endRxEvent.Cancel (); NotifyRxEnd (); SwitchToTx's RX case (:263-268)
        pe_can[live] = true;
        live = -1;
        rxing = false;
        endRx = nw;
      }
      endTx = nw + D.txd[ok].dur;
      if (MODE != 2) {
        if (ok - p >= 64) {
          err |= ERR_WINDOW;
          break;
        }
        done |= 1ull << (ok - p);
        while (done & 1ull) done >>= 1, p++;
      }
      oc++;
      ok = oc < oe ? D.own_idx[oc] : NONE;
      ok_ts = ok != NONE ? D.txd[ok].ts : INF;
      last_ts = now;
      WPH(1);
      continue;
    }

    if (kind == 2) {  // YansWifiPhy::EndReceive (yans-wifi-phy.cc:770-799), its state part
      const bool can = pe_can[e];
      if (!can) rxing = false;  // NotifyRxEnd (); DoSwitchFromRx (wifi-phy-state-helper.cc:391-402)
      c.end++;
      c.end_cancelled += can ? 1u : 0u;
      SyncRec r;
      r.ts = pe_sts[e];
      r.end_ts = pe_ts[e];
      r.tx = pe_tx[e];
      r.phy = (uint32_t)j;
      r.flags = (can ? NSGPU_WIFI_END_CANCELLED : 0u) | NSGPU_WIFI_END_DISPATCHED;
      r.m = 0;
      r.uid = 0;
      r.pad_ = 0;
      D.sync[pe_slot[e]] = r;
      const int l = npe - 1;
      if (live == e) live = -1;
      if (e != l) {
        pe_ts[e] = pe_ts[l], pe_sts[e] = pe_sts[l], pe_tx[e] = pe_tx[l], pe_slot[e] = pe_slot[l], pe_can[e] = pe_can[l];
        if (live == l) live = e;
      }
      npe--;
      e_dirty = true;
      disp++;
      last_ts = now;
      WPH(1);
      continue;
    }

    // YansWifiChannel::Receive -> YansWifiPhy::StartReceivePacket (yans-wifi-phy.cc:399-496)
    const uint32_t k = c_k;
    const double rxPowerW = MODE != 0 ? c_w : rx_power_w(D, c_dbm, c_dist);
    const int64_t endNew = nw + c_dur;
    // InterferenceHelper::AppendEvent (interference-helper.cc:192-212)
    WPH(6);  // (kind decision, Receive operands)
    ni.on_receive(nw);
    WPH(7);  // the eager cursor
    if (!ni.room()) {
      err |= ERR_NICAP;
      break;
    }
    if (!ni.phys_room()) {
      err |= ERR_LDS;
      break;
    }
    if (!rxing) firstPower = ni.fold_start(nw, rxPowerW);  // fold up to upper_bound (now) into m_firstPower
    else ni.insert_start(nw, rxPowerW);
    WPH(8);  // fold / start entry
    ni.insert_end(endNew, -rxPowerW);
    ni_ins += 2;
    ni_max = ni.length() > ni_max ? ni.length() : ni_max;
    WPH(2);  // NiChanges: cursor, fold / insert, end entry
    // the state switch (WifiPhyStateHelper::GetState, wifi-phy-state-helper.cc:159-183)
    const int st = endTx > nw ? 2 : rxing ? 1 : endCca > nw ? 3 : 0;
    uint32_t outcome, flags = 0;
    bool maybe = false;
    if (st == 1 || st == 2) {  // drop; noise after the current Rx / Tx (:431-457)
      outcome = st == 1 ? NSGPU_WIFI_DROP_RX : NSGPU_WIFI_DROP_TX;
      int64_t until = (st == 1 ? endRx : endTx) - nw;  // GetDelayUntilIdle (:122-151)
      until = until > 0 ? until : 0;
      maybe = endNew > nw + until;
    } else {
      if (near_thr(rxPowerW, D.edW)) flags |= NSGPU_WIFI_F_NEAR_ED;
      if (rxPowerW > D.edW) {  // sync (:461-472): SwitchToRx, NotifyRxStart, Schedule (EndReceive)
        outcome = NSGPU_WIFI_SYNC;
        if (npe == PE_CAP) {
          err |= ERR_PENDING;
          break;
        }
        const unsigned long long slot = atomicAdd(D.n_sync, 1ull);
        if (slot >= D.sync_cap) {
          err |= ERR_SYNCCAP;
          break;
        }
        rxing = true;
        endRx = endNew;
        pe_ts[npe] = (uint64_t)endNew, pe_sts[npe] = now, pe_tx[npe] = k, pe_slot[npe] = (uint32_t)slot, pe_can[npe] = false;
        live = npe++;
        e_dirty = true;
        c.sync++;
      } else {
        outcome = NSGPU_WIFI_DROP_ED;
        maybe = true;
      }
    }
    WPH(3);  // state decision, sync
    int64_t cca = 0;
    if (maybe) {  // maybeCcaBusy (:482-495): InterferenceHelper::GetEnergyDuration (interference-helper.cc:171-190)
      flags |= NSGPU_WIFI_F_CCA_EVAL;
      const int64_t end = ni.energy_end(nw, D.ccaW, flags);
      cca = end > nw ? end - nw : 0;
      if (cca != 0) {  // SwitchMaybeToCcaBusy (wifi-phy-state-helper.cc:404-423)
        flags |= NSGPU_WIFI_F_CCA_SWITCH;
        endCca = endCca > nw + cca ? endCca : nw + cca;
        c.cca_switches++;
      }
      cca_eval++;
    }
    WPH(4);  // CCA (GetEnergyDuration)
    c.rx++;
    c.drop_rx += outcome == NSGPU_WIFI_DROP_RX;
    c.drop_tx += outcome == NSGPU_WIFI_DROP_TX;
    c.drop_ed += outcome == NSGPU_WIFI_DROP_ED;
    near += (flags & (NSGPU_WIFI_F_NEAR_ED | NSGPU_WIFI_F_NEAR_CCA)) ? 1 : 0;
    digest += nsgpu_wifi_term(1, now, k, (uint64_t)j, (uint64_t)outcome | (uint64_t)(flags & 3u) << 8 | (uint64_t)cca << 16);
    if (D.rx_log) {
      nsgpu_wifi_rx_log *l = D.rx_log + (uint64_t)k * D.nphy + j;
      l->outcome = (uint8_t)outcome;
      l->flags = (uint8_t)flags;
      l->cca_ns = cca;
    }
    if (MODE == 2) {
      sr++;
    } else {
      done |= 1ull << (k - p);
      while (done & 1ull) done >>= 1, p++;
    }
    have_c = false;
    disp++;
    last_ts = now;
    WPH(5);  // counters, digest, log
  }
  WPH_END();
  // EndReceive events left pending at the end: scheduled (uid consumed), never dispatched
  for (int q = 0; q < npe; q++) {
    SyncRec r;
    r.ts = pe_sts[q];
    r.end_ts = pe_ts[q];
    r.tx = pe_tx[q];
    r.phy = (uint32_t)j;
    r.flags = pe_can[q] ? NSGPU_WIFI_END_CANCELLED : 0u;
    r.m = 0;
    r.uid = 0;
    r.pad_ = 0;
    D.sync[pe_slot[q]] = r;
  }
  c.ni_len = ni.length();
  c.ni_max = ni_max;
  c.end_tx = endTx;
  c.end_rx = endRx;
  c.end_cca_busy = endCca;
  c.first_power = firstPower;
  c.rxing = rxing ? 1u : 0u;
  D.pc[j] = c;
  if (err) atomicOr(D.err, err);
  atomicAdd(&D.acc[A_DIGEST], (unsigned long long)digest);
  atomicAdd(&D.acc[A_DISPATCHED], (unsigned long long)disp);
  atomicAdd(&D.acc[A_RX], (unsigned long long)c.rx);
  atomicAdd(&D.acc[A_SYNC], (unsigned long long)c.sync);
  atomicAdd(&D.acc[A_DROP_RX], (unsigned long long)c.drop_rx);
  atomicAdd(&D.acc[A_DROP_TX], (unsigned long long)c.drop_tx);
  atomicAdd(&D.acc[A_DROP_ED], (unsigned long long)c.drop_ed);
  atomicAdd(&D.acc[A_CCA_EVAL], (unsigned long long)cca_eval);
  atomicAdd(&D.acc[A_CCA_SWITCH], (unsigned long long)c.cca_switches);
  atomicAdd(&D.acc[A_END], (unsigned long long)c.end);
  atomicAdd(&D.acc[A_END_CANCELLED], (unsigned long long)c.end_cancelled);
  atomicAdd(&D.acc[A_NI_INSERTS], (unsigned long long)ni_ins);
  atomicAdd(&D.acc[A_NEAR], (unsigned long long)near);
  atomicMax(&D.acc[A_NI_MAX], (unsigned long long)ni_max);
  atomicMax(&D.acc[A_LAST_TS], (unsigned long long)last_ts);
}

// HBM ring store: 64 phys per block.
template <int MODE>
__global__ __launch_bounds__(64) void k_wifi_phy(const WifiDev D) {
  const int64_t jl = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (jl >= D.nown) return;
  const int64_t j = D.j0 + jl;
  __shared__ PeSlots pes[64];
  RingNi ni{D.ni + (uint64_t)jl * (D.ni_mask + 1), D.ni_mask, 0, 0, 0, 0.0};
  phy_run<MODE>(D, j, ni, &pes[threadIdx.x]);
}

// LDS split store: blockDim.x phys per block, each with its S ring (scap entries), E ring (ecap) and
// pending EndReceive records in the block's dynamic LDS (wifi_lds_bytes).
__host__ __device__ constexpr size_t wifi_lds_per_phy(uint32_t scap, uint32_t ecap) {
  return (size_t)(scap + ecap) * 16 + (size_t)ecap * 8 + sizeof(PeSlots);
}
template <int MODE>
__global__ __launch_bounds__(64) void k_wifi_phy_lds(const WifiDev D, uint32_t scap, uint32_t ecap) {
  extern __shared__ uint64_t wlds[];
  const uint32_t P = blockDim.x, l = threadIdx.x;
  const int64_t jl = (int64_t)blockIdx.x * P + l;
  if (jl >= D.nown) return;
  const int64_t j = D.j0 + jl;
  const size_t w = 2 * scap + 3 * ecap;  // words per phy: E times, deltas, running sums; S times, deltas
  uint64_t *b = wlds + (size_t)l * w;
  PeSlots *pe = reinterpret_cast<PeSlots *>(wlds + (size_t)P * w) + l;
  SplitNi ni{reinterpret_cast<int64_t *>(b + 3 * ecap), reinterpret_cast<int64_t *>(b),
             reinterpret_cast<double *>(b + 3 * ecap + scap), reinterpret_cast<double *>(b + ecap),
             reinterpret_cast<double *>(b + 2 * ecap), scap, ecap, D.ni_mask + 1, 0, 0, 0, 0, 0, 0.0, 0.0, 0,
             INT64_MAX, INT64_MAX, 0.0, 0.0, 0.0, INT64_MIN, 0.0};
  phy_run<MODE>(D, j, ni, pe);
}

// Syncs per bucket m = #transmissions with t_T <= ts (binary search over the schedule).
__global__ __launch_bounds__(256) void k_sync_hist(const WifiDev D) {
  const uint64_t n = *D.n_sync < D.sync_cap ? *D.n_sync : D.sync_cap;
  for (uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x; s < n; s += (uint64_t)gridDim.x * 256) {
    const uint64_t ts = D.sync[s].ts;
    uint32_t lo = 0, hi = D.ktx;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (D.tx_ts[mid] <= ts) lo = mid + 1; else hi = mid;
    }
    D.sync[s].m = lo;
    atomicAdd(&D.hist[lo], 1u);
  }
}

// One block: off = exclusive scan of hist[0 .. ktx]; uid base of every transmission; their digest terms.
__global__ __launch_bounds__(1024) void k_tx_base(const WifiDev D) {
  __shared__ uint32_t wsum[16];
  __shared__ uint32_t carry;
  const uint32_t n = D.ktx + 1;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (uint32_t c0 = 0; c0 < n; c0 += 1024) {
    const uint32_t i = c0 + threadIdx.x;
    const uint32_t v = i < n ? D.hist[i] : 0u;
    uint32_t x = v;  // inclusive wave scan
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o);
      if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    uint32_t before = carry;
    for (int w = 0; w < wid; w++) before += wsum[w];
    if (i < n) D.off[i] = before + x - v;
    __syncthreads();
    if (threadIdx.x == 1023) carry = before + x;
    __syncthreads();
  }
  if (threadIdx.x == 0) D.off[n] = carry;
  __syncthreads();
  unsigned long long dg = 0;
  for (uint32_t k = threadIdx.x; k < D.ktx; k += 1024) {
    const uint32_t b = D.uid_start + (uint32_t)D.fcum[k] + D.off[k + 1];  // syncs with ts < t_k: buckets 0..k
    D.base[k] = b;
    dg += nsgpu_wifi_term(0, D.tx_ts[k], D.tx_uid[k], b, 0);
  }
  atomicAdd(&D.acc[A_DIGEST], dg);
}

__device__ __forceinline__ uint32_t rx_rank(const WifiDev &D, uint32_t j, uint32_t k) {
  const uint32_t s = D.tx_phy[k];
  return D.chan_rank[j] - (j > s ? 1u : 0u);  // ScheduleWithContext order of the receiver loop
}

__global__ __launch_bounds__(256) void k_sync_place(const WifiDev D) {
  const uint64_t n = *D.n_sync < D.sync_cap ? *D.n_sync : D.sync_cap;
  for (uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x; s < n; s += (uint64_t)gridDim.x * 256) {
    SyncRec &r = D.sync[s];
    r.uid = D.base[r.tx] + rx_rank(D, r.phy, r.tx);
    const uint32_t pos = D.off[r.m] + atomicAdd(&D.cur[r.m], 1u);
    D.bucket[pos] = (uint32_t)s;
  }
}

__global__ __launch_bounds__(256) void k_sync_rank(const WifiDev D) {
  const uint64_t n = *D.n_sync < D.sync_cap ? *D.n_sync : D.sync_cap;
  unsigned long long dg = 0;
  for (uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x; s < n; s += (uint64_t)gridDim.x * 256) {
    const SyncRec r = D.sync[s];
    const uint32_t lo = D.off[r.m], hi = D.off[r.m + 1];
    uint32_t before = 0;
    for (uint32_t q = lo; q < hi; q++) {
      const SyncRec o = D.sync[D.bucket[q]];
      before += (o.ts < r.ts || (o.ts == r.ts && o.uid < r.uid)) ? 1u : 0u;
    }
    const uint32_t uid = D.uid_start + (uint32_t)D.fcum[r.m] + lo + before;
    nsgpu_wifi_end_record e;
    e.ts = r.end_ts;
    e.sync_ts = r.ts;
    e.uid = uid;
    e.phy = r.phy;
    e.tx = r.tx;
    e.flags = r.flags;
    D.ends[s] = e;
    if (r.flags & NSGPU_WIFI_END_DISPATCHED)
      dg += nsgpu_wifi_term(2, r.end_ts, uid, r.phy, (r.flags & NSGPU_WIFI_END_CANCELLED) ? 1 : 0);
  }
  if (dg) atomicAdd(&D.acc[A_DIGEST], dg);
}

// Rx log: every scheduled Receive's key (the ones after the Stop included).
__global__ __launch_bounds__(256) void k_rx_log_keys(const WifiDev D) {
  const uint64_t n = (uint64_t)D.ktx * (uint64_t)D.nphy;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    const uint32_t k = (uint32_t)(i / (uint64_t)D.nphy), j = (uint32_t)(i % (uint64_t)D.nphy);
    if (j == D.tx_phy[k] || D.chan[j] != D.tx_chan[k]) continue;
    double dist;
    D.rx_log[i].ts = arrival(D, k, D.x[j], D.y[j], D.z[j], dist);
    D.rx_log[i].uid = D.base[k] + rx_rank(D, j, k);
  }
}

// WifiPhy::CalculateTxDuration — wifi-phy.cc:141-296 (preamble + PLCP header + payload, in us)
int64_t tx_duration_ns(uint32_t size, uint32_t mc, uint64_t rate, uint32_t bw, uint32_t preamble) {
  uint32_t pre, hdr, pay;
  if (mc == NSGPU_WIFI_OFDM || mc == NSGPU_WIFI_ERP_OFDM) {
    const uint32_t sym = bw == 10000000 ? 8 : bw == 5000000 ? 16 : 4;
    pre = mc == NSGPU_WIFI_ERP_OFDM ? 4 : sym * 4;                            // 16 / 32 / 64 (:196-214), ERP 4
    hdr = mc == NSGPU_WIFI_ERP_OFDM ? 16 : sym;                               // 4 / 8 / 16 (:148-166), ERP 16
    const double ndbps = (double)(rate * sym) / 1e6;                          // N_DBPS (:262)
    const uint32_t nsym = (uint32_t)lrint(ceil((16 + size * 8.0 + 6.0) / ndbps));  // (:265)
    pay = nsym * sym + (mc == NSGPU_WIFI_ERP_OFDM ? 6u : 0u);
  } else {  // DSSS (:173-183, :216-226, :281-283)
    pre = preamble == NSGPU_WIFI_PREAMBLE_SHORT ? 72 : 144;
    hdr = preamble == NSGPU_WIFI_PREAMBLE_SHORT ? 24 : 48;
    pay = (uint32_t)lrint(ceil((size * 8.0) / (rate / 1.0e6)));
  }
  return (int64_t)(pre + hdr + pay) * 1000;  // MicroSeconds (duration)
}

}  // namespace
}  // namespace nsgpu

using namespace nsgpu;

struct nsgpu_wifi {
  WifiDev D;
  int64_t n_tx;
  uint64_t stop_ts;
  uint32_t stop_uid;
  bool has_stop;
  std::vector<void *> allocs;
  hipStream_t last = nullptr;
  bool ran = false;
  // NiChanges store (nsgpu_wifi_set_store): the LDS split queues when their capacities fit, else the HBM
  // ring; lds_ok = the plan below exists, use_lds = the next run uses it
  int store = NSGPU_WIFI_STORE_AUTO;
  bool lds_ok = false, use_lds = false;
  uint32_t lds_P = 0, lds_pmax = 0, lds_scap = 0, lds_ecap = 0;
  size_t lds_bytes = 0;
  bool use_pre = false;  // the run reads its receptions from D.pre (allocated when the table fits HBM)
  bool use_sorted = false;  // ... in dispatch order from D.srt (allocated beside D.pre when the windows are short)
  // partitioned runs: this engine runs receivers [D.j0, D.j0 + D.nown); the partitions' results
  // are combined after the per-phy chains — RCCL (`comm`) or a loopback group on one device (`grouped`)
  nsgpu_comm *comm = nullptr;
  bool grouped = false;
  SyncRec *xsync = nullptr;  // the gathered sync records (nranks x sync_cap: padded to the largest rank's count)
  unsigned long long *x_acc = nullptr;  // [2][A_N]: the accumulators' sums and maxima over the partitions
  unsigned long long *x_cnt = nullptr;  // [nranks] sync counts
  uint32_t *x_err = nullptr;            // [nranks] error bits
};

constexpr uint32_t WSORT_MAX = 64;  // the longest interleaving window k_wifi_rx_sort compares

constexpr uint32_t SCAP_LDS = 8;  // S: starts at one instant (more: ERR_LDS, the run repeats on the ring)

extern "C" int nsgpu_wifi_tx_duration_ns(uint32_t size, uint32_t modclass, uint64_t rate_bps, uint32_t bw_hz,
                                         uint32_t preamble, int64_t *ns) {
  if (!ns || rate_bps == 0 || modclass > NSGPU_WIFI_ERP_OFDM) return set_error(NSGPU_EINVAL, "nsgpu_wifi_tx_duration_ns: bad mode");
  *ns = tx_duration_ns(size, modclass, rate_bps, bw_hz, preamble);
  return NSGPU_OK;
}

extern "C" int nsgpu_wifi_destroy(nsgpu_wifi *h) {
  if (!h) return NSGPU_OK;
  if (h->last) (void)hipStreamSynchronize(h->last);
  for (void *p : h->allocs) (void)hipFree(p);
  delete h;
  return NSGPU_OK;
}

template <class T>
static int dalloc(nsgpu_wifi *h, T **p, size_t n, const T *src = nullptr) {
  void *v = nullptr;
  NSGPU_HIP(hipMalloc(&v, std::max<size_t>(n, 1) * sizeof(T)));
  h->allocs.push_back(v);
  if (src && n) NSGPU_HIP(hipMemcpy(v, src, n * sizeof(T), hipMemcpyHostToDevice));
  *p = (T *)v;
  return NSGPU_OK;
}

// dist: a partition (nsgpu_wifi_create_dist) — it gets the exchange buffers, sized for comm's ranks (a
// loopback member, comm = NULL, combines through the host and needs one count / error slot).
static int wifi_create(const nsgpu_wifi_scenario *sc, int rx_log, int64_t j0, int64_t j1, nsgpu_comm *comm, bool dist,
                       nsgpu_wifi **out) {
  if (!sc || !out) return set_error(NSGPU_EINVAL, "nsgpu_wifi_create: null");
  *out = nullptr;
  const int64_t N = sc->n_phy, K = sc->n_tx;
  if (j1 < 0) j1 = N;
  if (j0 < 0 || j0 > j1 || j1 > N) return set_error(NSGPU_EINVAL, "nsgpu_wifi_create_dist: phys [%lld, %lld) of %lld", (long long)j0, (long long)j1, (long long)N);
  const int64_t NO = j1 - j0;  // the receivers this engine runs
  if (N < 1 || N > 0x7fffffff || K < 0 || K > 0x7fffffff) return set_error(NSGPU_EINVAL, "nsgpu_wifi_create: n_phy %lld n_tx %lld", (long long)N, (long long)K);
  if (!sc->x || !sc->y || !sc->z || !sc->channel || !sc->node) return set_error(NSGPU_EINVAL, "nsgpu_wifi_create: phy arrays");
  if (K && (!sc->tx_ts || !sc->tx_uid || !sc->tx_phy || !sc->tx_size || !sc->tx_dbm || !sc->tx_modclass ||
            !sc->tx_rate_bps || !sc->tx_bw_hz || !sc->tx_preamble))
    return set_error(NSGPU_EINVAL, "nsgpu_wifi_create: transmission arrays");
  if (!(sc->speed > 0)) return set_error(NSGPU_EINVAL, "nsgpu_wifi_create: speed must be > 0");
  if (sc->loss.n < 0 || sc->loss.n > NSGPU_MAX_LOSS_CHAIN) return set_error(NSGPU_EINVAL, "nsgpu_wifi_create: loss chain");
  const bool has_stop = sc->stop_ts != ~0ull;
  if (has_stop && sc->stop_uid >= sc->uid_start) return set_error(NSGPU_EINVAL, "nsgpu_wifi_create: the Stop uid must be a setup uid");
  // schedule: (ts, uid) order, setup uids, senders in range; dispatched = keys below the Stop event's
  uint32_t ktx = 0;
  for (int64_t k = 0; k < K; k++) {
    if (sc->tx_phy[k] >= (uint64_t)N) return set_error(NSGPU_EINVAL, "nsgpu_wifi_create: tx %lld sender", (long long)k);
    if (sc->tx_uid[k] >= sc->uid_start) return set_error(NSGPU_EINVAL, "nsgpu_wifi_create: tx %lld uid is not a setup uid", (long long)k);
    if (sc->tx_rate_bps[k] == 0 || sc->tx_modclass[k] > NSGPU_WIFI_ERP_OFDM) return set_error(NSGPU_EINVAL, "nsgpu_wifi_create: tx %lld mode", (long long)k);
    if (k && !key_less(sc->tx_ts[k - 1], sc->tx_uid[k - 1], sc->tx_ts[k], sc->tx_uid[k]))
      return set_error(NSGPU_EINVAL, "nsgpu_wifi_create: transmissions not in (ts, uid) order at %lld", (long long)k);
    if (!has_stop || key_less(sc->tx_ts[k], sc->tx_uid[k], sc->stop_ts, sc->stop_uid)) ktx = (uint32_t)k + 1;
  }
  uint32_t cap = 4;
  while (cap < sc->ni_cap && cap < (1u << 20)) cap <<= 1;
  // channel ranks (YansWifiChannel::Send's receiver order), fan-out sizes, own-transmission lists
  std::vector<uint32_t> rank((size_t)N), count_of;
  std::vector<uint32_t> chans(sc->channel, sc->channel + N);
  std::sort(chans.begin(), chans.end());
  chans.erase(std::unique(chans.begin(), chans.end()), chans.end());
  std::vector<uint32_t> seen(chans.size(), 0);
  for (int64_t j = 0; j < N; j++) {
    const size_t c = std::lower_bound(chans.begin(), chans.end(), sc->channel[j]) - chans.begin();
    rank[j] = seen[c]++;
  }
  std::vector<uint64_t> fcum((size_t)ktx + 1, 0);
  std::vector<uint32_t> tx_chan((size_t)std::max<int64_t>(K, 1)), own_off((size_t)N + 1, 0), own_idx;
  std::vector<double> tx_x((size_t)std::max<int64_t>(K, 1)), tx_y(tx_x.size()), tx_z(tx_x.size());
  std::vector<int64_t> tx_dur((size_t)std::max<int64_t>(K, 1));
  int64_t dur_min = INT64_MAX;
  for (int64_t k = 0; k < K; k++) {
    const uint32_t s = sc->tx_phy[k];
    tx_chan[k] = sc->channel[s];
    tx_x[k] = sc->x[s], tx_y[k] = sc->y[s], tx_z[k] = sc->z[s];
    tx_dur[k] = tx_duration_ns(sc->tx_size[k], sc->tx_modclass[k], sc->tx_rate_bps[k], sc->tx_bw_hz[k], sc->tx_preamble[k]);
    dur_min = std::min(dur_min, tx_dur[k]);
    if ((uint32_t)k < ktx) {
      const size_t c = std::lower_bound(chans.begin(), chans.end(), tx_chan[k]) - chans.begin();
      fcum[k + 1] = fcum[k] + (seen[c] - 1);
      own_off[s + 1]++;
    }
  }
  for (int64_t j = 0; j < N; j++) own_off[j + 1] += own_off[j];
  own_idx.resize(std::max<uint32_t>(own_off[N], 1));
  {
    std::vector<uint32_t> fill(own_off.begin(), own_off.end() - 1);
    for (uint32_t k = 0; k < ktx; k++) own_idx[fill[sc->tx_phy[k]]++] = k;
  }
  // syncs of one phy are at least one frame apart (a sync needs the phy out of RX and TX), and at most
  // one per transmission
  double xmin = 0, xmax = 0, ymin = 0, ymax = 0, zmin = 0, zmax = 0;
  for (int64_t j = 0; j < N; j++) {
    if (j == 0 || sc->x[j] < xmin) xmin = sc->x[j];
    if (j == 0 || sc->x[j] > xmax) xmax = sc->x[j];
    if (j == 0 || sc->y[j] < ymin) ymin = sc->y[j];
    if (j == 0 || sc->y[j] > ymax) ymax = sc->y[j];
    if (j == 0 || sc->z[j] < zmin) zmin = sc->z[j];
    if (j == 0 || sc->z[j] > zmax) zmax = sc->z[j];
  }
  uint64_t per_phy = ktx;
  const double diag = sqrt((xmax - xmin) * (xmax - xmin) + (ymax - ymin) * (ymax - ymin) + (zmax - zmin) * (zmax - zmin));
  // SplitNi's E queue: a phy's live end entries belong to receptions on the air at its current Receive,
  // i.e. to transmissions whose [ts, ts + max delay + duration] interval covers that instant: the largest
  // such overlap over the schedule bounds it (closed intervals; the sweep visits every start)
  uint32_t overlap = 0;
  // the interleaving windows of the sorted reception rows: wlo[k] = the first k' with ts' + dmax >= ts_k,
  // whi[k] = the last k' with ts' <= ts_k + dmax (arrivals lie in [ts, ts + dmax])
  std::vector<uint32_t> wlo(std::max<uint32_t>(ktx, 1)), whi(std::max<uint32_t>(ktx, 1));
  bool sortable = ktx > 0;
  if (ktx) {
    const int64_t dmax = (int64_t)ceil(diag / sc->speed * 1e9) + 2;
    for (uint32_t k = 0, lo = 0, hi = 0; k < ktx; k++) {
      while ((int64_t)sc->tx_ts[lo] + dmax < (int64_t)sc->tx_ts[k]) lo++;
      if (hi < k) hi = k;
      while (hi + 1 < ktx && (int64_t)sc->tx_ts[hi + 1] <= (int64_t)sc->tx_ts[k] + dmax) hi++;
      wlo[k] = lo, whi[k] = hi;
      if (hi - lo + 1 > WSORT_MAX || tx_dur[k] < 0 || tx_dur[k] > (int64_t)0xffffffffll) sortable = false;
    }
    std::vector<int64_t> ends(ktx);
    for (uint32_t k = 0; k < ktx; k++) ends[k] = (int64_t)sc->tx_ts[k] + dmax + tx_dur[k];
    std::sort(ends.begin(), ends.end());
    uint32_t gone = 0;  // intervals that ended before the current start
    for (uint32_t k = 0; k < ktx; k++) {
      while (gone < ktx && ends[gone] < (int64_t)sc->tx_ts[k]) gone++;
      overlap = std::max(overlap, k + 1 - gone);
    }
  }
  if (ktx) {
    const double span = (double)(sc->tx_ts[ktx - 1] - sc->tx_ts[0]) + diag / sc->speed * 1e9 + 2.0;
    per_phy = std::min<uint64_t>(ktx, (uint64_t)(span / (double)std::max<int64_t>(dur_min, 1)) + 2);
  }
  const uint64_t sync_cap = std::max<uint64_t>(per_phy * (uint64_t)N, 1);
  if ((uint64_t)sc->uid_start + fcum[ktx] + std::min<uint64_t>(sync_cap, fcum[ktx]) > 0xffffffffull)  // syncs <= receives
    return set_error(NSGPU_EINVAL, "nsgpu_wifi_create: the run would overflow the 32-bit uid counter");

  nsgpu_wifi *h = new nsgpu_wifi();
  h->n_tx = K;
  h->stop_ts = sc->stop_ts;
  h->stop_uid = sc->stop_uid;
  h->has_stop = has_stop;
  WifiDev &D = h->D;
  D.nphy = N;
  D.j0 = j0;
  D.nown = NO;
  D.ktx = ktx;
  D.uid_start = sc->uid_start;
  D.loss = sc->loss;
  D.speed = sc->speed;
  D.rx_gain_db = sc->rx_gain_db;
  D.edW = pow(10.0, sc->ed_threshold_dbm / 10.0) / 1000.0;    // SetEdThreshold (yans-wifi-phy.cc:228-232)
  D.ccaW = pow(10.0, sc->cca_threshold_dbm / 10.0) / 1000.0;  // SetCcaMode1Threshold (:234-238)
  D.stop_ts = has_stop ? sc->stop_ts : INF;
  D.ni_mask = cap - 1;
  D.sync_cap = sync_cap;
  {  // the LDS plan: P phys per block, each with SCAP_LDS + ecap entries of 16 B
    int dev = 0, lmax = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&lmax, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) == hipSuccess && lmax > 0) {
      const uint32_t ecap = std::max<uint32_t>(overlap + 2, 8);
      const size_t per = wifi_lds_per_phy(SCAP_LDS, ecap);
      const size_t pmax = std::min<size_t>(64, (size_t)lmax / per);
      // A lane's run is one serial chain of dependent steps, and a wave's step is the union of its lanes'
      // branches (event kinds, CCA walks of different lengths): spread the phys over every SIMD (one wave
      // each, 4 per CU) rather than packing 64 into a wave.
      int ncu = 0;
      if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu < 1) ncu = 256;
      size_t P = (size_t)((std::max<int64_t>(NO, 1) + 4 * (int64_t)ncu - 1) / (4 * (int64_t)ncu));
      if (const char *e = getenv("NSGPU_WIFI_PHYS_PER_BLOCK")) P = (size_t)atoi(e);  // (diagnostic sweeps)
      P = std::max<size_t>(1, std::min(P, pmax));
      if (pmax >= 1) {
        h->lds_ok = true;
        h->lds_P = (uint32_t)P;
        h->lds_scap = SCAP_LDS;
        h->lds_ecap = ecap;
        h->lds_bytes = P * per;
      }
      // auto: the split queues when LDS holds 8 phys' queues per block (longer queues: the HBM ring)
      h->lds_pmax = (uint32_t)pmax;
      h->use_lds = h->lds_ok && pmax >= 8;
    }
  }
  int rc = NSGPU_OK;
#define TRY(x)                    \
  do {                            \
    if ((rc = (x)) != NSGPU_OK) { \
      nsgpu_wifi_destroy(h);      \
      return rc;                  \
    }                             \
  } while (0)
  TRY(dalloc(h, (double **)&D.x, N, sc->x));
  TRY(dalloc(h, (double **)&D.y, N, sc->y));
  TRY(dalloc(h, (double **)&D.z, N, sc->z));
  TRY(dalloc(h, (uint32_t **)&D.chan, N, sc->channel));
  TRY(dalloc(h, (uint32_t **)&D.chan_rank, N, rank.data()));
  TRY(dalloc(h, (uint64_t **)&D.tx_ts, K, sc->tx_ts));
  TRY(dalloc(h, (uint32_t **)&D.tx_phy, K, sc->tx_phy));
  TRY(dalloc(h, (uint32_t **)&D.tx_uid, K, sc->tx_uid));
  TRY(dalloc(h, (uint32_t **)&D.tx_chan, K, tx_chan.data()));
  TRY(dalloc(h, (int64_t **)&D.tx_dur, K, tx_dur.data()));
  TRY(dalloc(h, (double **)&D.tx_dbm, K, sc->tx_dbm));
  TRY(dalloc(h, (double **)&D.tx_x, K, tx_x.data()));
  TRY(dalloc(h, (double **)&D.tx_y, K, tx_y.data()));
  TRY(dalloc(h, (double **)&D.tx_z, K, tx_z.data()));
  {
    std::vector<TxDesc> txd((size_t)std::max<int64_t>(K, 1));
    for (int64_t k = 0; k < K; k++)
      txd[k] = TxDesc{tx_x[k], tx_y[k], tx_z[k], sc->tx_dbm[k], sc->tx_ts[k], tx_dur[k], sc->tx_phy[k], tx_chan[k], {0, 0}};
    TRY(dalloc(h, (TxDesc **)&D.txd, K, txd.data()));
    std::vector<TsDur> td((size_t)std::max<int64_t>(K, 1));  // (ts, dur) alone: 8 transmissions a line
    for (int64_t k = 0; k < K; k++) td[k] = TsDur{sc->tx_ts[k], tx_dur[k]};
    TRY(dalloc(h, (TsDur **)&D.tsdur, K, td.data()));
  }
  TRY(dalloc(h, (uint64_t **)&D.fcum, fcum.size(), fcum.data()));
  TRY(dalloc(h, (uint32_t **)&D.own_off, own_off.size(), own_off.data()));
  TRY(dalloc(h, (uint32_t **)&D.own_idx, own_idx.size(), own_idx.data()));
  TRY(dalloc(h, (uint32_t **)&D.wlo, wlo.size(), wlo.data()));
  TRY(dalloc(h, (uint32_t **)&D.whi, whi.size(), whi.data()));
  TRY(dalloc(h, &D.ni, (size_t)std::max<int64_t>(NO, 1) * cap));
  TRY(dalloc(h, &D.sync, sync_cap));
  TRY(dalloc(h, &D.n_sync, 1));
  TRY(dalloc(h, &D.pc, N));
  NSGPU_HIP(hipMemset(D.pc, 0, (size_t)N * sizeof(*D.pc)));  // (a partition writes only its own phys')
  if (dist) {
    const int R = comm ? comm->nranks : 1;
    TRY(dalloc(h, &h->xsync, (uint64_t)R * sync_cap));  // (the padded gather: every rank's records up to sync_cap)
    TRY(dalloc(h, &h->x_acc, 2 * (size_t)A_N));
    TRY(dalloc(h, &h->x_cnt, (size_t)R));
    TRY(dalloc(h, &h->x_err, (size_t)R));
    h->comm = comm;
  }
  D.rx_log = nullptr;
  if (rx_log) TRY(dalloc(h, &D.rx_log, std::max<uint64_t>((uint64_t)ktx * (uint64_t)N, 1)));
  TRY(dalloc(h, &D.acc, A_N));
  TRY(dalloc(h, &D.err, 1));
  TRY(dalloc(h, &D.hist, (size_t)ktx + 1));
  TRY(dalloc(h, &D.off, (size_t)ktx + 2));
  TRY(dalloc(h, &D.cur, (size_t)ktx + 1));
  TRY(dalloc(h, &D.bucket, sync_cap));
  TRY(dalloc(h, &D.base, std::max<uint32_t>(ktx, 1)));
  TRY(dalloc(h, &D.ends, sync_cap));
  {  // the reception table (k_wifi_rx): n_phy x dispatched transmissions x 16 B, when half of free HBM holds it
    size_t fr = 0, tot = 0;
    const uint64_t bytes = (uint64_t)NO * ktx * sizeof(RxPre), sbytes = (uint64_t)NO * ktx * sizeof(RxS);
    D.pre = nullptr;
    D.srt = nullptr;
    if (ktx && NO && hipMemGetInfo(&fr, &tot) == hipSuccess && bytes <= fr / 2) {
      TRY(dalloc(h, &D.pre, (size_t)NO * ktx));
      h->use_pre = true;
      if (sortable && bytes + sbytes <= fr / 2) {  // and its rows in dispatch order
        TRY(dalloc(h, &D.srt, (size_t)NO * ktx));
        h->use_sorted = true;
      }
    }
  }
#undef TRY
  *out = h;
  return NSGPU_OK;
}

extern "C" int nsgpu_wifi_create(const nsgpu_wifi_scenario *sc, int rx_log, nsgpu_wifi **out) {
  return wifi_create(sc, rx_log, 0, -1, nullptr, false, out);
}

// A partition of the receivers (every partition knows the transmissions and runs its own
// receivers); comm = the RCCL communicator of one rank per GPU, or null for a loopback group member
// (nsgpu_wifi_group_run).
extern "C" int nsgpu_wifi_create_dist(const nsgpu_wifi_scenario *sc, int rx_log, int64_t phy_begin, int64_t phy_end,
                                      nsgpu_comm *comm, nsgpu_wifi **out) {
  if (!sc || phy_end < phy_begin) return set_error(NSGPU_EINVAL, "nsgpu_wifi_create_dist: bad arguments");
  int rc = wifi_create(sc, rx_log, phy_begin, phy_end, comm, true, out);
  if (rc == NSGPU_OK && !comm) (*out)->grouped = true;
  return rc;
}

// (k_wifi_rx: 0 ms when the run computes its receptions inline; k_wifi_phy: k_wifi_phy_lds with the LDS store)
static const char *const WIFI_KERNELS[] = {"k_wifi_rx", "k_wifi_phy", "k_sync_hist", "k_tx_base", "k_sync_place",
                                           "k_sync_rank"};
constexpr int WIFI_NK = 6;

// One whole run on `s`; with `ev` (WIFI_NK + 1 events) each kernel of the chain is bracketed.  The first part
// (wifi_launch_phys) runs the receivers' chains, the second (wifi_launch_uids) hands out the EndReceive uids
// from the syncs; a partitioned run combines the partitions' syncs and accumulators in between.
static int wifi_launch_phys(nsgpu_wifi *h, hipStream_t s, hipEvent_t *ev) {
  const WifiDev &D = h->D;
  NSGPU_HIP(hipMemsetAsync(D.n_sync, 0, sizeof(unsigned long long), s));
  NSGPU_HIP(hipMemsetAsync(D.acc, 0, A_N * sizeof(unsigned long long), s));
  NSGPU_HIP(hipMemsetAsync(D.err, 0, sizeof(uint32_t), s));
  NSGPU_HIP(hipMemsetAsync(D.hist, 0, ((size_t)D.ktx + 1) * sizeof(uint32_t), s));
  NSGPU_HIP(hipMemsetAsync(D.cur, 0, ((size_t)D.ktx + 1) * sizeof(uint32_t), s));
  const uint64_t nlog = (uint64_t)D.ktx * (uint64_t)D.nphy;
  if (D.rx_log && nlog) hipLaunchKernelGGL(k_rx_log_init, dim3(1024), dim3(256), 0, s, D.rx_log, nlog);
  if (ev) NSGPU_HIP(hipEventRecord(ev[0], s));
  WifiDev Dk = D;
  if (!h->use_pre) Dk.pre = nullptr;
  if (!h->use_pre || !h->use_sorted) Dk.srt = nullptr;
  const int mode = Dk.srt ? 2 : Dk.pre ? 1 : 0;
  if (Dk.pre) {
    const uint64_t n = (uint64_t)D.nown * D.ktx;
    const unsigned g = (unsigned)std::max<uint64_t>(std::min<uint64_t>((n + 255) / 256, 16384), 1);
    if (n) hipLaunchKernelGGL(k_wifi_rx, dim3(g), dim3(256), 0, s, Dk);
    if (n && Dk.srt) hipLaunchKernelGGL(k_wifi_rx_sort, dim3(g), dim3(256), 0, s, Dk);
  }
  if (ev) NSGPU_HIP(hipEventRecord(ev[1], s));
  if (h->use_lds) {
    const void *kf = mode == 2 ? (const void *)k_wifi_phy_lds<2> : mode == 1 ? (const void *)k_wifi_phy_lds<1>
                                                                             : (const void *)k_wifi_phy_lds<0>;
    if (h->lds_bytes > 65536)
      NSGPU_HIP(hipFuncSetAttribute(kf, hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->lds_bytes));
    const dim3 g((unsigned)std::max<int64_t>((D.nown + h->lds_P - 1) / h->lds_P, 1)), b(h->lds_P);
    if (mode == 2) hipLaunchKernelGGL(k_wifi_phy_lds<2>, g, b, h->lds_bytes, s, Dk, h->lds_scap, h->lds_ecap);
    else if (mode == 1) hipLaunchKernelGGL(k_wifi_phy_lds<1>, g, b, h->lds_bytes, s, Dk, h->lds_scap, h->lds_ecap);
    else hipLaunchKernelGGL(k_wifi_phy_lds<0>, g, b, h->lds_bytes, s, Dk, h->lds_scap, h->lds_ecap);
  } else {
    const dim3 g((unsigned)std::max<int64_t>((D.nown + 63) / 64, 1)), b(64);
    if (mode == 2) hipLaunchKernelGGL(k_wifi_phy<2>, g, b, 0, s, Dk);
    else if (mode == 1) hipLaunchKernelGGL(k_wifi_phy<1>, g, b, 0, s, Dk);
    else hipLaunchKernelGGL(k_wifi_phy<0>, g, b, 0, s, Dk);
  }
  if (ev) NSGPU_HIP(hipEventRecord(ev[2], s));
  NSGPU_HIP(hipGetLastError());
  h->last = s;
  return NSGPU_OK;
}
static int wifi_launch_uids(nsgpu_wifi *h, hipStream_t s, hipEvent_t *ev) {
  const WifiDev &D = h->D;
  const uint64_t nlog = (uint64_t)D.ktx * (uint64_t)D.nphy;
  hipLaunchKernelGGL(k_sync_hist, dim3(1024), dim3(256), 0, s, D);
  if (ev) NSGPU_HIP(hipEventRecord(ev[3], s));
  hipLaunchKernelGGL(k_tx_base, dim3(1), dim3(1024), 0, s, D);
  if (ev) NSGPU_HIP(hipEventRecord(ev[4], s));
  hipLaunchKernelGGL(k_sync_place, dim3(1024), dim3(256), 0, s, D);
  if (ev) NSGPU_HIP(hipEventRecord(ev[5], s));
  hipLaunchKernelGGL(k_sync_rank, dim3(1024), dim3(256), 0, s, D);
  if (ev) NSGPU_HIP(hipEventRecord(ev[6], s));
  if (D.rx_log && nlog) hipLaunchKernelGGL(k_rx_log_keys, dim3(1024), dim3(256), 0, s, D);
  NSGPU_HIP(hipGetLastError());
  h->last = s;
  h->ran = true;
  return NSGPU_OK;
}

// The partitions' results into every partition (after their chains): the accumulators summed (the two
// maxima maxed), the error bits or-ed, the sync records gathered in partition order (k_sync_rank ranks them
// by key, so any order gives the same uids).  `cnt[q]`, `err[q]`, `acc[q]` were read back from partition q.
static int wifi_combine_host(nsgpu_wifi *h, hipStream_t s, const std::vector<unsigned long long> &cnt,
                             const std::vector<uint32_t> &err, const std::vector<std::vector<unsigned long long>> &acc,
                             uint64_t *total) {
  unsigned long long a[A_N] = {};
  uint32_t e = 0;
  uint64_t tot = 0;
  for (size_t q = 0; q < cnt.size(); q++) {
    for (int i = 0; i < A_N; i++)
      a[i] = (i == A_NI_MAX || i == A_LAST_TS) ? std::max(a[i], acc[q][i]) : a[i] + acc[q][i];
    e |= err[q];
    tot += cnt[q];
  }
  if (tot > h->D.sync_cap) e |= ERR_SYNCCAP;
  if (e & ERR_SYNCCAP) tot = 0;  // (the run fails at its readers; the uid kernels see no records)
  NSGPU_HIP(hipMemcpyAsync(h->D.acc, a, sizeof(a), hipMemcpyHostToDevice, s));
  NSGPU_HIP(hipMemcpyAsync(h->D.err, &e, sizeof(e), hipMemcpyHostToDevice, s));
  const unsigned long long t = tot;
  NSGPU_HIP(hipMemcpyAsync(h->D.n_sync, &t, sizeof(t), hipMemcpyHostToDevice, s));
  NSGPU_HIP(hipStreamSynchronize(s));  // (the host sources above are on this stack frame)
  *total = tot;
  return NSGPU_OK;
}

// RCCL partition: counts, errors and accumulators gathered, then the sync records (padded to the largest
// partition's count) — one host synchronisation per run.
static int wifi_exchange_rccl(nsgpu_wifi *h, hipStream_t s, uint32_t *err_out) {
  const WifiDev &D = h->D;
  const int R = h->comm->nranks;
  ncclComm_t c = h->comm->comm;
  NCCL_TRY(ncclGroupStart());
  NCCL_TRY(ncclAllGather(D.n_sync, h->x_cnt, 1, ncclUint64, c, s));
  NCCL_TRY(ncclAllGather(D.err, h->x_err, 1, ncclUint32, c, s));
  NCCL_TRY(ncclAllReduce(D.acc, h->x_acc, A_N, ncclUint64, ncclSum, c, s));
  NCCL_TRY(ncclAllReduce(D.acc, h->x_acc + A_N, A_N, ncclUint64, ncclMax, c, s));
  NCCL_TRY(ncclGroupEnd());
  std::vector<unsigned long long> cnt(R), ac(2 * A_N);
  std::vector<uint32_t> er(R);
  NSGPU_HIP(hipMemcpyAsync(cnt.data(), h->x_cnt, R * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
  NSGPU_HIP(hipMemcpyAsync(er.data(), h->x_err, R * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  NSGPU_HIP(hipMemcpyAsync(ac.data(), h->x_acc, 2 * A_N * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
  NSGPU_HIP(hipStreamSynchronize(s));
  uint64_t maxc = 0;
  for (int q = 0; q < R; q++) maxc = std::max<uint64_t>(maxc, std::min<uint64_t>(cnt[q], D.sync_cap));
  std::vector<std::vector<unsigned long long>> acc(1, std::vector<unsigned long long>(A_N));
  for (int i = 0; i < A_N; i++) acc[0][i] = (i == A_NI_MAX || i == A_LAST_TS) ? ac[A_N + i] : ac[i];
  uint32_t e = 0;
  for (uint32_t x : er) e |= x;
  uint64_t tot = 0;
  for (int q = 0; q < R; q++) tot += cnt[q];
  if (maxc && tot <= D.sync_cap) {  // (xsync holds R x sync_cap records: the padding always fits)
    NCCL_TRY(ncclAllGather(D.sync, h->xsync, maxc * sizeof(SyncRec), ncclUint8, c, s));
    uint64_t off = 0;
    for (int q = 0; q < R; q++) {
      if (cnt[q]) NSGPU_HIP(hipMemcpyAsync(D.sync + off, h->xsync + (uint64_t)q * maxc, cnt[q] * sizeof(SyncRec), hipMemcpyDeviceToDevice, s));
      off += cnt[q];
    }
  } else if (maxc) {
    e |= ERR_SYNCCAP;  // (the run's syncs exceed the capacity a single engine would have)
  }
  uint64_t t2 = 0;
  int rc = wifi_combine_host(h, s, std::vector<unsigned long long>{tot}, std::vector<uint32_t>{e}, acc, &t2);
  *err_out = e;
  return rc;
}

// One run: the chains, the exchange of a partitioned (RCCL) run, the uids.  A partitioned run whose LDS
// start queue overflowed repeats its chains on the HBM ring before the uids (every rank sees the or-ed bits).
static int wifi_launch(nsgpu_wifi *h, hipStream_t s, hipEvent_t *ev) {
  int rc = wifi_launch_phys(h, s, ev);
  if (rc == NSGPU_OK && h->comm) {
    uint32_t e = 0;
    rc = wifi_exchange_rccl(h, s, &e);
    if (rc == NSGPU_OK && (e & ERR_LDS) && !(e & (ERR_TX_IN_TX | ERR_NICAP)) && h->use_lds) {
      h->use_lds = false;
      rc = wifi_launch_phys(h, s, ev);
      if (rc == NSGPU_OK) rc = wifi_exchange_rccl(h, s, &e);
    }
  }
  if (rc == NSGPU_OK) rc = wifi_launch_uids(h, s, ev);
  return rc;
}

// A loopback group (every partition on this device, in one process): the members' chains, their results
// combined through the host, then every member's uids — each member then reads like a partitioned rank.
extern "C" int nsgpu_wifi_group_run(nsgpu_wifi **m, int n, void *stream) {
  if (!m || n < 1) return set_error(NSGPU_EINVAL, "nsgpu_wifi_group_run: no members");
  for (int q = 0; q < n; q++)
    if (!m[q] || !m[q]->grouped) return set_error(NSGPU_EINVAL, "nsgpu_wifi_group_run: member %d is not a loopback partition", q);
  const hipStream_t s = (hipStream_t)stream;
  for (int attempt = 0; attempt < 2; attempt++) {
    for (int q = 0; q < n; q++) {
      int rc = wifi_launch_phys(m[q], s, nullptr);
      if (rc) return rc;
    }
    std::vector<unsigned long long> cnt(n);
    std::vector<uint32_t> er(n);
    std::vector<std::vector<unsigned long long>> acc(n, std::vector<unsigned long long>(A_N));
    for (int q = 0; q < n; q++) {
      NSGPU_HIP(hipMemcpyAsync(&cnt[q], m[q]->D.n_sync, sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
      NSGPU_HIP(hipMemcpyAsync(&er[q], m[q]->D.err, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
      NSGPU_HIP(hipMemcpyAsync(acc[q].data(), m[q]->D.acc, A_N * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    }
    NSGPU_HIP(hipStreamSynchronize(s));
    uint32_t e = 0;
    for (uint32_t x : er) e |= x;
    if ((e & ERR_LDS) && !(e & (ERR_TX_IN_TX | ERR_NICAP)) && attempt == 0) {
      for (int q = 0; q < n; q++) m[q]->use_lds = false;
      continue;
    }
    for (int q = 0; q < n; q++) cnt[q] = std::min<unsigned long long>(cnt[q], m[q]->D.sync_cap);
    for (int r = 0; r < n; r++) {  // every member's syncs into member r's gather buffer, in member order
      uint64_t off = 0;
      for (int q = 0; q < n; q++) {
        if (cnt[q] && off + cnt[q] <= m[r]->D.sync_cap)
          NSGPU_HIP(hipMemcpyAsync(m[r]->xsync + off, m[q]->D.sync, cnt[q] * sizeof(SyncRec), hipMemcpyDeviceToDevice, s));
        off += cnt[q];
      }
    }
    for (int r = 0; r < n; r++) {
      uint64_t tot = 0;
      int rc = wifi_combine_host(m[r], s, cnt, er, acc, &tot);
      if (rc) return rc;
      if (tot) NSGPU_HIP(hipMemcpyAsync(m[r]->D.sync, m[r]->xsync, tot * sizeof(SyncRec), hipMemcpyDeviceToDevice, s));
      rc = wifi_launch_uids(m[r], s, nullptr);
      if (rc) return rc;
    }
    return NSGPU_OK;
  }
  return NSGPU_OK;
}

extern "C" int nsgpu_wifi_set_store(nsgpu_wifi *h, int store) {
  if (!h) return set_error(NSGPU_EINVAL, "nsgpu_wifi_set_store: null");
  if (store & ~(NSGPU_WIFI_STORE_MASK | NSGPU_WIFI_INLINE_RX | NSGPU_WIFI_UNSORTED_RX))
    return set_error(NSGPU_EINVAL, "nsgpu_wifi_set_store: store %d", store);
  h->use_pre = h->D.pre != nullptr && !(store & NSGPU_WIFI_INLINE_RX);
  h->use_sorted = h->D.srt != nullptr && !(store & NSGPU_WIFI_UNSORTED_RX);
  store &= NSGPU_WIFI_STORE_MASK;
  switch (store) {
    case NSGPU_WIFI_STORE_AUTO:
      h->use_lds = h->lds_ok && h->lds_pmax >= 8;
      break;
    case NSGPU_WIFI_STORE_LDS:
      if (!h->lds_ok) return set_error(NSGPU_EINVAL, "nsgpu_wifi_set_store: the split queues do not fit LDS");
      h->use_lds = true;
      break;
    case NSGPU_WIFI_STORE_HBM:
      h->use_lds = false;
      break;
    default:
      return set_error(NSGPU_EINVAL, "nsgpu_wifi_set_store: store %d", store);
  }
  h->store = store;
  return NSGPU_OK;
}

extern "C" int nsgpu_wifi_get_store(nsgpu_wifi *h, int *store, uint32_t *phys_per_block, uint32_t *e_cap) {
  if (!h || !store) return set_error(NSGPU_EINVAL, "nsgpu_wifi_get_store: null");
  *store = (h->use_lds ? NSGPU_WIFI_STORE_LDS : NSGPU_WIFI_STORE_HBM) | (h->use_pre ? 0 : NSGPU_WIFI_INLINE_RX) |
           (h->use_pre && !h->use_sorted ? NSGPU_WIFI_UNSORTED_RX : 0);
  if (phys_per_block) *phys_per_block = h->use_lds ? h->lds_P : 64;
  if (e_cap) *e_cap = h->use_lds ? h->lds_ecap : h->D.ni_mask + 1;
  return NSGPU_OK;
}

extern "C" int nsgpu_wifi_run(nsgpu_wifi *h, void *stream) {
  if (!h) return set_error(NSGPU_EINVAL, "nsgpu_wifi_run: null");
  if (h->grouped) return set_error(NSGPU_ESTATE, "nsgpu_wifi_run: a loopback partition runs with its group (nsgpu_wifi_group_run)");
  return wifi_launch(h, (hipStream_t)stream, nullptr);
}

#ifdef NSGPU_PHASE_PROF
extern "C" int nsgpu_wifi_phase_read(unsigned long long *out, int reset) {  // (diagnostic build only)
  NSGPU_HIP(hipDeviceSynchronize());
  NSGPU_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wifi_ph), sizeof(unsigned long long) * 16));
  if (reset) {
    unsigned long long z[16] = {};
    NSGPU_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_wifi_ph), z, sizeof(z)));
  }
  return NSGPU_OK;
}
#endif

extern "C" int nsgpu_wifi_kernel_count(int *n) {
  *n = WIFI_NK;
  return NSGPU_OK;
}

extern "C" const char *nsgpu_wifi_kernel_name(int k) { return k >= 0 && k < WIFI_NK ? WIFI_KERNELS[k] : ""; }

// One run with every kernel of the chain bracketed by HIP events on `stream`: ms[k] = kernel k's time.
extern "C" int nsgpu_wifi_profile(nsgpu_wifi *h, void *stream, double *ms) {
  if (!h || !ms) return set_error(NSGPU_EINVAL, "nsgpu_wifi_profile: null");
  if (h->grouped) return set_error(NSGPU_ESTATE, "nsgpu_wifi_profile: a loopback partition runs with its group");
  hipEvent_t ev[WIFI_NK + 1] = {};
  int rc = NSGPU_OK;
  for (auto &e : ev)
    if (hipEventCreate(&e) != hipSuccess) rc = set_error(NSGPU_EHIP, "nsgpu_wifi_profile: hipEventCreate");
  if (rc == NSGPU_OK) rc = wifi_launch(h, (hipStream_t)stream, ev);
  if (rc == NSGPU_OK && hipEventSynchronize(ev[WIFI_NK]) != hipSuccess) rc = set_error(NSGPU_EHIP, "nsgpu_wifi_profile: sync");
  for (int k = 0; rc == NSGPU_OK && k < WIFI_NK; k++) {
    float f = 0;
    if (hipEventElapsedTime(&f, ev[k], ev[k + 1]) != hipSuccess) rc = set_error(NSGPU_EHIP, "nsgpu_wifi_profile: elapsed");
    ms[k] = f;
  }
  for (auto &e : ev)
    if (e) (void)hipEventDestroy(e);
  return rc;
}

static int wifi_check(nsgpu_wifi *h, uint64_t *n_sync) {
  if (!h || !h->ran) return set_error(NSGPU_ESTATE, "nsgpu_wifi: no run yet");
  NSGPU_HIP(hipStreamSynchronize(h->last));
  uint32_t err = 0;
  unsigned long long ns = 0;
  NSGPU_HIP(hipMemcpy(&err, h->D.err, sizeof(err), hipMemcpyDeviceToHost));
  NSGPU_HIP(hipMemcpy(&ns, h->D.n_sync, sizeof(ns), hipMemcpyDeviceToHost));
  if ((err & ERR_LDS) && !(err & (ERR_TX_IN_TX | ERR_NICAP)) && !h->comm && !h->grouped) {
    // an S queue outgrew its LDS capacity (more starts at one instant than SCAP_LDS): the same run on
    // the HBM ring, and every later run of this handle too
    h->use_lds = false;
    int rc = wifi_launch(h, h->last, nullptr);
    if (rc != NSGPU_OK) return rc;
    NSGPU_HIP(hipStreamSynchronize(h->last));
    NSGPU_HIP(hipMemcpy(&err, h->D.err, sizeof(err), hipMemcpyDeviceToHost));
    NSGPU_HIP(hipMemcpy(&ns, h->D.n_sync, sizeof(ns), hipMemcpyDeviceToHost));
  }
  if (err & ERR_TX_IN_TX) return set_error(NSGPU_ESTATE, "nsgpu_wifi: SendPacket while in TX (the reference's NS_FATAL_ERROR)");
  if (err & ERR_NICAP) return set_error(NSGPU_ENOMEM, "nsgpu_wifi: a NiChanges list outgrew ni_cap %u", h->D.ni_mask + 1);
  if (err & ERR_WINDOW) return set_error(NSGPU_ENOMEM, "nsgpu_wifi: more than 64 transmissions inside one arrival spread");
  if (err & ERR_PENDING) return set_error(NSGPU_ENOMEM, "nsgpu_wifi: more than %d pending EndReceive events on a phy", PE_CAP);
  if ((err & ERR_SYNCCAP) || ns > h->D.sync_cap) return set_error(NSGPU_ENOMEM, "nsgpu_wifi: sync capacity");
  if (n_sync) *n_sync = ns;
  return NSGPU_OK;
}

extern "C" int nsgpu_wifi_get_stats(nsgpu_wifi *h, nsgpu_wifi_stats *out) {
  uint64_t ns = 0;
  int rc = wifi_check(h, &ns);
  if (rc != NSGPU_OK) return rc;
  if (!out) return set_error(NSGPU_EINVAL, "nsgpu_wifi_get_stats: null");
  unsigned long long a[A_N];
  NSGPU_HIP(hipMemcpy(a, h->D.acc, sizeof(a), hipMemcpyDeviceToHost));
  const WifiDev &D = h->D;
  uint64_t fk = 0;
  NSGPU_HIP(hipMemcpy(&fk, D.fcum + D.ktx, sizeof(fk), hipMemcpyDeviceToHost));
  nsgpu_wifi_stats st = {};
  st.tx = D.ktx;
  st.rx = a[A_RX];
  st.sync = a[A_SYNC];
  st.drop_rx = a[A_DROP_RX];
  st.drop_tx = a[A_DROP_TX];
  st.drop_ed = a[A_DROP_ED];
  st.cca_evals = a[A_CCA_EVAL];
  st.cca_switches = a[A_CCA_SWITCH];
  st.end = a[A_END];
  st.end_cancelled = a[A_END_CANCELLED];
  st.ni_inserts = a[A_NI_INSERTS];
  st.near_threshold = a[A_NEAR];
  st.ni_max = (uint32_t)a[A_NI_MAX];
  st.dispatched = a[A_DISPATCHED] + D.ktx + (h->has_stop ? 1 : 0);
  st.digest = a[A_DIGEST] + (h->has_stop ? nsgpu_wifi_term(3, h->stop_ts, h->stop_uid, 0, 0) : 0);
  st.final_ts = h->has_stop ? h->stop_ts : a[A_LAST_TS];
  st.next_uid = (uint32_t)(D.uid_start + fk + ns);
  *out = st;
  return NSGPU_OK;
}

extern "C" int nsgpu_wifi_read_phys(nsgpu_wifi *h, nsgpu_wifi_phy_counters *out) {
  int rc = wifi_check(h, nullptr);
  if (rc != NSGPU_OK) return rc;
  NSGPU_HIP(hipMemcpy(out, h->D.pc, (size_t)h->D.nphy * sizeof(*out), hipMemcpyDeviceToHost));
  return NSGPU_OK;
}

extern "C" int nsgpu_wifi_read_tx_base(nsgpu_wifi *h, uint32_t *out) {
  int rc = wifi_check(h, nullptr);
  if (rc != NSGPU_OK) return rc;
  for (int64_t k = 0; k < h->n_tx; k++) out[k] = 0;
  if (h->D.ktx) NSGPU_HIP(hipMemcpy(out, h->D.base, (size_t)h->D.ktx * sizeof(uint32_t), hipMemcpyDeviceToHost));
  return NSGPU_OK;
}

extern "C" int nsgpu_wifi_read_ends(nsgpu_wifi *h, nsgpu_wifi_end_record *out, uint64_t cap, uint64_t *n) {
  uint64_t ns = 0;
  int rc = wifi_check(h, &ns);
  if (rc != NSGPU_OK) return rc;
  if (n) *n = ns;
  if (out && ns) {
    if (ns > cap) return set_error(NSGPU_EINVAL, "nsgpu_wifi_read_ends: %llu records, cap %llu", (unsigned long long)ns, (unsigned long long)cap);
    NSGPU_HIP(hipMemcpy(out, h->D.ends, ns * sizeof(*out), hipMemcpyDeviceToHost));
  }
  return NSGPU_OK;
}

extern "C" int nsgpu_wifi_read_rx_log(nsgpu_wifi *h, nsgpu_wifi_rx_log *out) {
  int rc = wifi_check(h, nullptr);
  if (rc != NSGPU_OK) return rc;
  if (!h->D.rx_log) return set_error(NSGPU_ESTATE, "nsgpu_wifi_read_rx_log: created without rx_log");
  const uint64_t nlog = (uint64_t)h->D.ktx * (uint64_t)h->D.nphy;
  if (nlog) NSGPU_HIP(hipMemcpy(out, h->D.rx_log, nlog * sizeof(*out), hipMemcpyDeviceToHost));
  for (uint64_t i = nlog; i < (uint64_t)h->n_tx * (uint64_t)h->D.nphy; i++)
    out[i] = nsgpu_wifi_rx_log{0, 0, NSGPU_WIFI_NOT_RUN, 0, 0, 0};
  return NSGPU_OK;
}
