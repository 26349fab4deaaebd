// nsgpu_wifil.hip — the closed-loop Wi-Fi PHY on the device (include/nsgpu.h: nsgpu_wifil_*, and
// nsgpu_sim_attach_wifi / nsgpu_sim_wifi_send / nsgpu_sim_wifi_state in nsgpu_simimpl.hip).
//
// Replaces, for transmissions that host closures start at run time (a MAC on the host):
// YansWifiPhy::SendPacket (yans-wifi-phy.cc:499-522) -> YansWifiChannel::Send (yans-wifi-channel.cc:77-115)
// -> YansWifiPhy::StartReceivePacket (yans-wifi-phy.cc:399-496) with InterferenceHelper::Add / AppendEvent /
// GetEnergyDuration (interference-helper.cc:129-212), the WifiPhyStateHelper transitions
// (wifi-phy-state-helper.cc:122-183, 254-322, 391-423), and YansWifiPhy::EndReceive (yans-wifi-phy.cc:770-799)
// with InterferenceHelper::CalculateSnrPer (interference-helper.cc:215-353) and the error-rate models
// (nist-error-rate-model.cc, yans-error-rate-model.cc, dsss-error-rate-model.cc).  EndReceive's m_random
// draw (:783) is the host's: each EndReceive's (snr, per) goes back to it (nsgpu_wifil_read_ends).
//
// Epochs.  The host runtime (nsgpu_sim) owns the uid counter and the dispatch order; before it runs a host
// closure with key (T, u) it advances the device to that key (nsgpu_wifil_advance): every phy's lane runs
// its pending Receive / EndReceive events with keys below (T, u), in (ts, uid) order, then the epoch's
// syncs get their EndReceive uids.  A host closure's SendPacket (nsgpu_wifil_send) applies the sender's
// state switch at once and queues one Receive per receiver, with the uids the runtime hands out.
// Order inside one phy needs no global rank: every Receive's uid is known when it is queued (the runtime's
// counter at the SendPacket), and an EndReceive scheduled in the running epoch has a uid above every uid
// handed out before the epoch — so it sorts after those at equal ts, and among themselves by their syncing
// Receives' keys (uids follow the dispatch order of the events that schedule them).
//
// State per phy lives in HBM between epochs: the InterferenceHelper list as a time-sorted ring (the r02
// RingNi layout of nsgpu_wifi.hip, with its eager prefix cursor), the state helper's end times, the pending
// Receive queue (sorted by (arrival, uid)) and up to LPE_CAP pending EndReceive records.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>
#include "nsgpu_device.h"
#include "nsgpu_internal.h"

namespace nsgpu {
namespace {

constexpr uint32_t NONE = 0xffffffffu;
constexpr int LPE_CAP = 8;  // pending EndReceive records of one phy (the live one + cancelled ones)
constexpr uint32_t END_STAGE = 128;  // EndReceive records an epoch returns with its counters (more: a second copy)
constexpr size_t STAT_HDR = 32;      // the status block: counters (5 x u32), the epoch flag (word 6), then the ends
static_assert(sizeof(nsgpu_wifil_end) % 8 == 0 && STAT_HDR % 8 == 0, "status block alignment");
constexpr uint32_t WE_TX_IN_TX = 1, WE_NICAP = 2, WE_RQCAP = 4, WE_PECAP = 8, WE_CAP = 16, WE_CKCAP = 32;
constexpr int NB = 8;  // ring entries loaded per batch

struct LNi {  // InterferenceHelper::NiChange (interference-helper.cc:91-110)
  int64_t t;
  double d;
};
struct LRx {  // a pending Receive: arrival, uid, transmission, rxPowerW (DbmToW of CalcRxPower + RxGain), and
  uint64_t at;  // the transmission's duration (so a Receive needs no second load)
  uint32_t uid, tx;
  double w;
  int64_t dur;
};
struct LPe {  // a pending EndReceive
  uint64_t ts, sts;          // its ts; the syncing Receive's ts
  uint32_t suid, euid;       // the syncing Receive's uid; its own uid (NONE: scheduled in the running epoch)
  uint32_t tx, can, sslot, used;
  double w;                  // rxPowerW
};
struct LTx {  // one SendPacket: duration and payload mode
  uint64_t ts;
  int64_t dur;
  uint64_t rate;
  uint32_t phy, mc, bw, preamble;
};
struct LPhy {  // a phy's state between epochs
  double firstPower, cur_s;      // InterferenceHelper::m_firstPower; the ring's prefix-cursor sum
  int64_t endTx, endRx, endCca;  // WifiPhyStateHelper m_endTx / m_endRx / m_endCcaBusy
  uint32_t rxing, head, len, cur_n;
  uint32_t rq_head, rq_len, live, ni_max;
  nsgpu_wifi_phy_counters c;
};
struct WMir {  // a phy's state helper fields in pinned host memory: GetState reads them with no device trip
  int64_t endTx, endRx, endCca;
  uint32_t rxing, pad;
};
struct LEv {  // one dispatched device event of the epoch
  uint64_t ts;
  uint32_t uid, ctx, sslot, pad;
};
struct LSync {  // one sync of the epoch (its EndReceive's uid comes from the sync order)
  uint64_t sts;
  uint32_t suid, euid;
  uint32_t loc, pad;  // its pending EndReceive record: pe[loc]
};
struct LCk {  // one chunk of an EndReceive's CalculatePer walk, evaluated by k_wl_mid: the noise before it,
  double noise;  // and (duration << 1) | (1: the PLCP header mode)
  int64_t dm;
};
struct LEck {  // an end record's chunks: ck[start, start + n) (n = NONE: its PER was computed inline)
  uint32_t start, n;
  double w;  // rxPowerW
};

struct WDev {
  int64_t nphy;
  const double *x, *y, *z;
  const uint32_t *chan, *chan_rank, *node;
  nsgpu_loss_chain loss;
  double speed, rx_gain_db, edW, ccaW, nf;  // nf: the noise figure as a ratio (DbToRatio)
  uint32_t model, ni_mask, rq_mask, pad;
  uint64_t inv_hi, inv_lo;  // int64x64_t::Invert (1e9): Time::GetSeconds at NS resolution
  LPhy *ps;
  LNi *ni;
  LRx *rq;
  LPe *pe;
  LTx *tx;
  LSync *sync;
  LEv *ev;
  nsgpu_wifil_end *ends;
  uint32_t *end_sslot;
  uint32_t *cnt;  // [0] events, [1] syncs, [2] ends, [3] error bits (sticky: a SendPacket's are seen at the
                  // next advance), [4] chunk slots claimed ([0..2], [4] zeroed by the order's
                  // k_wl_rank, for the epoch two on)
  LCk *ck;        // the epoch's deferred chunks (ck_cap; a walk that finds no room computes its PER inline)
  LEck *eck;      // per end record
  uint32_t *evc;             // the epoch's event-list stripes: EV_STRIPES counters, EV_STRIDE words apart
  LEv *evd;                  // the epoch's events in dense order, uids resolved (k_wl_gather; the host's copy)
  LEv *evp;                  // a phy's events of the epoch in its own EVB slots (k_wl_stepw, no claim); by parity
  uint32_t *evn;             // their counts (zeroed by k_wl_gather once read); by parity
  uint32_t *evt;             // their total, EV_STRIPES counters EV_STRIDE words apart (one would serialize 10^4
                             //   adds on one line); by parity, zeroed by k_wl_rank for the epoch two on
  uint32_t *gtot;            // k_wl_gather's claims (reset by k_wl_tsort)
  uint32_t *erank;           // the epoch's events: rank in its (ts, uid) order (k_wl_rank, when logging)
  ulonglong2 *evg;           // the epoch's keys (ts, uid << 32 | dense index), sorted by tiles (k_wl_tsort)
  uint32_t *ticket;          // k_wl_rank's blocks done (its last block: the digest sum, the counters' zeroing)
  uint32_t *mticket;         // k_wl_mid's blocks done (its last block closes the epoch: wl_fin)
  WMir *mir;                 // (mapped host memory) each phy's state fields: a lane whose phy changed writes them
  LRx *rxb;                  // the batched SendPackets' Receives, NSEND x nphy (k_wl_rx; at = ~0: none for that phy)
  unsigned long long *edig;  // every ordered epoch's digest terms, summed on the device (k_wl_rank)
  uint64_t sync_cap, ev_cap, end_cap, ck_cap;
  uint64_t ev_scap;  // events per stripe (stripe s holds ev[s * ev_scap, s * ev_scap + evc[s * EV_STRIDE]))
  const uint32_t *lis;  // the phys whose EndReceives the host takes back (nsgpu_wifil_listen), nlis of them
  uint32_t nlis, pad_lis;
  // a partition of the phys (nsgpu_wifil_create_dist / _group): this engine runs phys [j0, j0 + nown) — their
  // waves, Receives, pending records — while every array stays indexed by the global phy; a single engine has
  // j0 = 0, nown = nphy.  xsync: every partition's syncs of the epoch (xn of them) the sync order ranks this
  // partition's against (null: its own, the single engine).
  int64_t j0, nown;
  const LSync *xsync;
  uint32_t xn, pad_x;
};
// The epoch's dispatched events are appended to EV_STRIPES lists (phy j's to stripe j % EV_STRIPES): one
// counter a phy's event would serialize ~10^4 atomics an epoch on one line.
constexpr int EV_STRIPES = 64, EV_STRIDE = 32;

// ---- WifiMode attributes (the CreateWifiMode calls of wifi-phy.cc:355-840; phyRate: wifi-mode.cc:140-155) ----
struct Mode {
  uint32_t mc, bw, phy_rate, cons, code;  // code: 0 undefined, 1: 1/2, 2: 2/3, 3: 3/4
  uint64_t data_rate;
};
__host__ __device__ __forceinline__ Mode make_mode(uint32_t mc, uint64_t rate, uint32_t bw) {
  Mode m{mc, mc == NSGPU_WIFI_DSSS ? 22000000u : bw, (uint32_t)rate, rate == 1000000 ? 2u : 4u, 0u, rate};
  if (mc == NSGPU_WIFI_DSSS) return m;
  switch (rate * 20000000ull / m.bw) {  // the 20 MHz OFDM ladder; 10 / 5 MHz channels run at 1/2, 1/4 the rates
    case 6000000: m.cons = 2, m.code = 1; break;
    case 9000000: m.cons = 2, m.code = 3; break;
    case 12000000: m.cons = 4, m.code = 1; break;
    case 18000000: m.cons = 4, m.code = 3; break;
    case 24000000: m.cons = 16, m.code = 1; break;
    case 36000000: m.cons = 16, m.code = 3; break;
    case 48000000: m.cons = 64, m.code = 2; break;
    default: m.cons = 64, m.code = 3; break;
  }
  const uint32_t dr = (uint32_t)rate;
  m.phy_rate = m.code == 1 ? dr * 2 / 1 : m.code == 2 ? dr * 3 / 2 : dr * 4 / 3;
  return m;
}
// WifiPhy::GetPlcpHeaderMode — wifi-phy.cc:99-139
__device__ __forceinline__ Mode header_mode(const Mode &p, uint32_t preamble) {
  if (p.mc == NSGPU_WIFI_OFDM)
    return p.bw == 5000000 ? make_mode(NSGPU_WIFI_OFDM, 1500000, 5000000)
           : p.bw == 10000000 ? make_mode(NSGPU_WIFI_OFDM, 3000000, 10000000)
                              : make_mode(NSGPU_WIFI_OFDM, 6000000, 20000000);
  if (p.mc == NSGPU_WIFI_ERP_OFDM) return make_mode(NSGPU_WIFI_ERP_OFDM, 6000000, 20000000);
  return make_mode(NSGPU_WIFI_DSSS, preamble == NSGPU_WIFI_PREAMBLE_LONG ? 1000000 : 2000000, 22000000);
}
// WifiPhy::GetPlcpPreambleDurationMicroSeconds / GetPlcpHeaderDurationMicroSeconds — wifi-phy.cc:141-231
__device__ __forceinline__ uint32_t preamble_us(uint32_t mc, uint32_t bw, uint32_t preamble) {
  if (mc == NSGPU_WIFI_OFDM) return bw == 10000000 ? 32 : bw == 5000000 ? 64 : 16;
  if (mc == NSGPU_WIFI_ERP_OFDM) return 4;
  return preamble == NSGPU_WIFI_PREAMBLE_SHORT ? 72 : 144;
}
__device__ __forceinline__ uint32_t header_us(uint32_t mc, uint32_t bw, uint32_t preamble) {
  if (mc == NSGPU_WIFI_OFDM) return bw == 10000000 ? 8 : bw == 5000000 ? 16 : 4;
  if (mc == NSGPU_WIFI_ERP_OFDM) return 16;
  return preamble == NSGPU_WIFI_PREAMBLE_SHORT ? 24 : 48;
}

// ---- error-rate models ----
// DsssErrorRateModel — dsss-error-rate-model.cc:29-127, ENABLE_GSL unset (the CCK rates use the Matlab fits)
__device__ double dsss_success(uint64_t rate, double sinr, uint32_t nbits) {
  double ber;
  switch (rate) {
    case 1000000: {
      double EbN0 = sinr * 22000000.0 / 1000000.0;
      ber = 0.5 * exp(-EbN0);
      break;
    }
    case 2000000: {
      double x = sinr * 22000000.0 / 1000000.0 / 2.0;  // DqpskFunction (:29-35)
      ber = ((sqrt(2.0) + 1.0) / sqrt(8.0 * 3.1415926 * sqrt(2.0))) * (1.0 / sqrt(x)) * exp(-(2.0 - sqrt(2.0)) * x);
      break;
    }
    case 5500000:
      if (sinr > 10.0) ber = 0.0;
      else if (sinr < 0.1) ber = 0.5;
      else ber = 5.3681634344056195e-001 * exp(-(pow((sinr - 3.3092430025608586e-003) / 4.1654372361004000e-001,
                                                     1.0288981434358866e+000)));
      break;
    case 11000000:
      if (sinr > 10.0) ber = 0.0;
      else if (sinr < 0.1) ber = 0.5;
      else {
        const double a1 = 7.9056742265333456e-003, a2 = -1.8397449399176360e-001, a3 = 1.0740689468707241e+000,
                     a4 = 1.0523316904502553e+000, a5 = 3.0552298746496687e-001, a6 = 2.2032715128698435e+000;
        ber = (a1 * sinr * sinr + a2 * sinr + a3) / (sinr * sinr * sinr + a4 * sinr * sinr + a5 * sinr + a6);
      }
      break;
    default:
      return 0;
  }
  return pow((1.0 - ber), (double)nbits);
}
// NistErrorRateModel — nist-error-rate-model.cc:38-270 (YansWifiPhyHelper::Default's model)
__device__ double nist_pe(double p, uint32_t b) {  // CalculatePe
  const double D = sqrt(4.0 * p * (1.0 - p));
  if (b == 1)
    return 0.5 * (36.0 * pow(D, 10.0) + 211.0 * pow(D, 12.0) + 1404.0 * pow(D, 14.0) + 11633.0 * pow(D, 16.0) +
                  77433.0 * pow(D, 18.0) + 502690.0 * pow(D, 20.0) + 3322763.0 * pow(D, 22.0) +
                  21292910.0 * pow(D, 24.0) + 134365911.0 * pow(D, 26.0));
  if (b == 2)
    return 1.0 / (2.0 * b) *
           (3.0 * pow(D, 6.0) + 70.0 * pow(D, 7.0) + 285.0 * pow(D, 8.0) + 1276.0 * pow(D, 9.0) + 6160.0 * pow(D, 10.0) +
            27128.0 * pow(D, 11.0) + 117019.0 * pow(D, 12.0) + 498860.0 * pow(D, 13.0) + 2103891.0 * pow(D, 14.0) +
            8784123.0 * pow(D, 15.0));
  return 1.0 / (2.0 * b) *
         (42.0 * pow(D, 5.0) + 201.0 * pow(D, 6.0) + 1492.0 * pow(D, 7.0) + 10469.0 * pow(D, 8.0) + 62935.0 * pow(D, 9.0) +
          379644.0 * pow(D, 10.0) + 2253373.0 * pow(D, 11.0) + 13073811.0 * pow(D, 12.0) + 75152755.0 * pow(D, 13.0) +
          428005675.0 * pow(D, 14.0));
}
__device__ double nist_success(const Mode &m, double snr, uint32_t nbits) {
  if (m.mc == NSGPU_WIFI_DSSS) return dsss_success(m.data_rate, snr, nbits);
  const uint32_t b = m.cons == 64 ? (m.code == 2 ? 2u : 3u) : (m.code == 1 ? 1u : 3u);
  double ber;
  switch (m.cons) {
    case 2: ber = 0.5 * erfc(sqrt(snr)); break;                               // GetBpskBer
    case 4: ber = 0.5 * erfc(sqrt(snr / 2.0)); break;                         // GetQpskBer
    case 16: ber = 0.75 * 0.5 * erfc(sqrt(snr / (5.0 * 2.0))); break;         // Get16QamBer
    default: ber = 7.0 / 12.0 * 0.5 * erfc(sqrt(snr / (21.0 * 2.0))); break;  // Get64QamBer
  }
  if (ber == 0.0) return 1.0;  // GetFec*Ber
  double pe = nist_pe(ber, b);
  pe = pe < 1.0 ? pe : 1.0;
  return pow(1 - pe, (double)nbits);
}
// YansErrorRateModel — yans-error-rate-model.cc:45-300
__device__ uint32_t yans_factorial(uint32_t k) {
  uint32_t f = 1;
  while (k > 0) f *= k--;
  return f;
}
__device__ double yans_binomial(uint32_t k, double p, uint32_t n) {
  return yans_factorial(n) / (yans_factorial(k) * yans_factorial(n - k)) * pow(p, (double)k) * pow(1 - p, (double)(n - k));
}
__device__ double yans_pd(double ber, uint32_t d) {  // CalculatePd (Odd / Even)
  double pd = 0;
  if ((d % 2) == 0) {
    for (uint32_t i = d / 2 + 1; i < d; i++) pd += yans_binomial(i, ber, d);
    pd += 0.5 * yans_binomial(d / 2, ber, d);
  } else {
    for (uint32_t i = (d + 1) / 2; i < d; i++) pd += yans_binomial(i, ber, d);
  }
  return pd;
}
__device__ double yans_success(const Mode &m, double snr, uint32_t nbits) {
  if (m.mc == NSGPU_WIFI_DSSS) return dsss_success(m.data_rate, snr, nbits);
  const double EbNo = snr * m.bw / m.phy_rate;
  if (m.cons == 2) {  // GetFecBpskBer
    const double ber = 0.5 * erfc(sqrt(EbNo));
    const uint32_t dFree = m.code == 1 ? 10 : 5, adFree = m.code == 1 ? 11 : 8;
    if (ber == 0.0) return 1.0;
    double pmu = adFree * yans_pd(ber, dFree);
    pmu = pmu < 1.0 ? pmu : 1.0;
    return pow(1 - pmu, (double)nbits);
  }
  const unsigned int M = m.cons;  // GetQamBer + GetFecQamBer
  const double z = sqrt((1.5 * (log((double)M) / log(2.0)) * EbNo) / (M - 1.0));
  const double z1 = ((1.0 - 1.0 / sqrt((double)M)) * erfc(z));
  const double z2 = 1 - pow((1 - z1), 2.0);
  const double ber = z2 / (log((double)M) / log(2.0));
  uint32_t dFree, adFree, adFree1;
  if (M == 64) {
    if (m.code == 2) dFree = 6, adFree = 1, adFree1 = 16;
    else dFree = 5, adFree = 8, adFree1 = 31;
  } else {
    if (m.code == 1) dFree = 10, adFree = 11, adFree1 = 0;
    else dFree = 5, adFree = 8, adFree1 = 31;
  }
  if (ber == 0.0) return 1.0;
  double pmu = adFree * yans_pd(ber, dFree);
  pmu += adFree1 * yans_pd(ber, dFree + 1);
  pmu = pmu < 1.0 ? pmu : 1.0;
  return pow(1 - pmu, (double)nbits);
}

// Time::GetSeconds at NS resolution: To (S) = MulByInvert (Invert (1e9)) then GetDouble
// (nstime.h:398-431, int64x64-128.cc:94-118, int64x64-128.h:83-95).
__device__ __forceinline__ double get_seconds(const WDev &D, int64_t ts) {
  const bool neg = ts < 0;
  const u128 a = (u128)(neg ? -ts : ts) << 64;
  const u128 b = ((u128)D.inv_hi << 64) | D.inv_lo;
  const u128 ah = a >> 64, bh = b >> 64, al = a & (u128)~0ull, bl = b & (u128)~0ull;
  u128 mid = ah * bl + al * bh;
  mid >>= 64;
  const u128 r = ah * bh + mid;
  const uint64_t hi = (uint64_t)(r >> 64), lo = (uint64_t)r;
  double flo = (double)lo;
  flo /= 18446744073709551615.0;
  double v = (double)hi;
  v += flo;
  return neg ? -v : v;
}
// InterferenceHelper::CalculateChunkSuccessRate — interference-helper.cc:244-255
__device__ double chunk(const WDev &D, double snir, int64_t duration, const Mode &m) {
  if (duration == 0) return 1.0;
  const uint32_t rate = m.phy_rate;
  const uint64_t nbits = (uint64_t)(rate * get_seconds(D, duration));
  return D.model == NSGPU_WIFIL_YANS ? yans_success(m, snir, (uint32_t)nbits) : nist_success(m, snir, (uint32_t)nbits);
}
// InterferenceHelper::CalculateSnr — interference-helper.cc:215-227
__device__ __forceinline__ double snr_of(const WDev &D, double signal, double noiseInterference, const Mode &m) {
  const double Nt = 1.3803e-23 * 290.0 * m.bw;  // BOLTZMANN
  const double noiseFloor = D.nf * Nt;
  const double noise = noiseFloor + noiseInterference;
  return signal / noise;
}

// Cross-lane moves by DPP instead of ds_bpermute (an LDS round trip each): the previous lane's value (wave_shr:1;
// lane 0 gets 0) and an inclusive wave scan (row_shr 1 / 2 / 4 / 8, then row_bcast 15 / 31); every lane active.
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ uint32_t wdpp32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWS, 0xf, false);
}
__device__ __forceinline__ uint32_t prev_lane32(uint32_t v) { return wdpp32<0x138>(v); }
__device__ __forceinline__ uint64_t prev_lane64(uint64_t v) {
  return ((uint64_t)prev_lane32((uint32_t)(v >> 32)) << 32) | prev_lane32((uint32_t)v);
}
__device__ __forceinline__ uint32_t wave_incscan32(uint32_t v) {
  v += wdpp32<0x111>(v);
  v += wdpp32<0x112>(v);
  v += wdpp32<0x114>(v);
  v += wdpp32<0x118>(v);
  v += wdpp32<0x142, 0xa>(v);
  v += wdpp32<0x143, 0xc>(v);
  return v;
}

// One index of counter *ctr per calling lane: the wave's active lanes share one atomic (every phy's lane
// appending to the same epoch lists one atomic each serialized on the counter's line: ~11 ns apiece).
__device__ __forceinline__ uint32_t wave_alloc(uint32_t *ctr) {
  const uint64_t m = __ballot(1);
  const int lane = threadIdx.x & 63;
  const int first = __ffsll((unsigned long long)m) - 1;
  uint32_t base = 0;
  if (lane == first) base = atomicAdd(ctr, (uint32_t)__popcll(m));
  base = (uint32_t)__builtin_amdgcn_readlane((int)base, first);  // (first is uniform)
  return base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
}

// YansWifiChannel::Send's delivery of transmission t (index k, from the closure's uid base) to phy j (not the
// sender): its Receive — ConstantSpeed delay, the loss chain + RxGain, DbmToW, the receiver loop's uid.
__device__ __forceinline__ bool reception(const WDev &D, int64_t j, const LTx &t, uint32_t k, double dbm, uint32_t base,
                                          LRx &out) {
  const uint32_t s = t.phy;
  if (D.chan[j] != D.chan[s]) return false;  // other channels get nothing (yans-wifi-channel.cc:88-91)
  const double dist = distance3(D.x[s], D.y[s], D.z[s], D.x[j], D.y[j], D.z[j]);
  const uint64_t at = t.ts + (uint64_t)seconds_to_ts(dist / D.speed);  // ConstantSpeed delay (propagation-delay-model.cc:90-96)
  const double dBm = calc_rx_power(D.loss, dbm, dist) + D.rx_gain_db;      // StartReceivePacket: rxPowerDbm += RxGain
  const double w = pow(10.0, dBm / 10.0) / 1000.0;                         // DbmToW (yans-wifi-phy.cc:727-732)
  out = LRx{at, base + D.chan_rank[j] - (j > (int64_t)s ? 1u : 0u), k, w, t.dur};  // the receiver loop's Schedule order
  return true;
}
// The SendPackets one host closure made since the last epoch, applied by the next epoch launch (more than
// NSEND: the earlier ones by k_wl_send launches).
constexpr uint32_t NSEND = 8;
struct SendBatch {
  uint32_t n, k0;  // SendPackets; the first one's transmission index (they are k0 .. k0 + n - 1)
  LTx t[NSEND];
  double dbm[NSEND];
  uint32_t base[NSEND];
};

// ---- the NiChanges ring of one phy (RingNi of nsgpu_wifi.hip: time-sorted, eager prefix cursor) ----
__device__ __forceinline__ void ni_insert(LNi *ring, uint32_t head, uint32_t &len, uint32_t m, int64_t t, double d) {
  // AddNiChangeEvent (interference-helper.cc:378-383): at upper_bound (time).  The entries after it (a
  // start while receiving passes every pending end: ~100 of them) move up one place, read NB at a time
  // from the tail (one memory trip per NB, not per entry)
  uint32_t q = len;
  while (q > 0) {
    const uint32_t nb = q < (uint32_t)NB ? q : (uint32_t)NB;
    LNi e[NB];
#pragma unroll
    for (int u = 0; u < NB; u++) e[u] = ring[(head + q - 1 - u) & m];  // (past the head: masked, unused)
    uint32_t k = 0;  // the batch's entries after t: a run from the tail
#pragma unroll
    for (int u = 0; u < NB; u++)
      if ((uint32_t)u < nb && k == (uint32_t)u && e[u].t > t) k++;
#pragma unroll
    for (int u = 0; u < NB; u++)
      if ((uint32_t)u < k) ring[(head + q - u) & m] = e[u];
    q -= k;
    if (k < nb) break;
  }
  ring[(head + q) & m] = LNi{t, d};
  len++;
}
template <bool LE>
__device__ __forceinline__ void cursor_advance(const LNi *ring, uint32_t head, uint32_t len, uint32_t m, int64_t lim,
                                               uint32_t &cur_n, double &cur_s) {
  while (cur_n < len) {
    LNi e[NB];
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

// EndReceive's order key against another pending EndReceive of the same phy (ts, then uid; a uid of the
// running epoch is above every known one, and those order by their syncing Receives' keys).
__device__ __forceinline__ bool pe_before(const LPe &a, const LPe &b) {
  if (a.ts != b.ts) return a.ts < b.ts;
  const bool ka = a.euid != NONE, kb = b.euid != NONE;
  if (ka != kb) return ka;
  if (ka) return a.euid < b.euid;
  return a.sts != b.sts ? a.sts < b.sts : a.suid < b.suid;
}

__device__ __forceinline__ WMir mir_of(const LPhy &P) { return WMir{P.endTx, P.endRx, P.endCca, P.rxing, 0}; }
__device__ __forceinline__ void mir_put(const WDev &D, int64_t j, const WMir &m0, const LPhy &P) {
  if (P.endTx != m0.endTx || P.endRx != m0.endRx || P.endCca != m0.endCca || P.rxing != m0.rxing) D.mir[j] = mir_of(P);
}

// One phy's events of the epoch: every pending Receive / EndReceive with a key below (bts, buid).
#ifdef NSGPU_PHASE_PROF
// diagnostic build: [0] sum over epochs of the slowest lane's time, [1] sum of lane times, [2] lanes, [3] events,
// [4] sum over epochs of the most events one lane ran, [5] epochs, [6] max lane time, [7] its events
__device__ unsigned long long g_wl_ph[8];
__device__ unsigned long long g_wl_ep[2];  // the current epoch's slowest lane time / most events (reset by host)
// k_wl_stepw's waves, recorded without atomics for WREC_E epochs from epoch g_wtarget on (the epoch counter
// g_wepoch counts k_wl_prof_epoch launches): per wave (start, loads done, loop done, end) s_memtime stamps and
// its events
constexpr uint32_t WREC_E = 8, WREC_P = 16384;
__device__ unsigned long long g_wrec[WREC_E][WREC_P][5];
__device__ uint32_t g_wepoch, g_wtarget;
#endif
__global__ __launch_bounds__(64) void k_wl_step(const WDev D, uint64_t bts, uint32_t buid) {
  const int64_t j = D.j0 + (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (j >= D.j0 + D.nown) return;
#ifdef NSGPU_PHASE_PROF
  const uint64_t pt0 = __builtin_amdgcn_s_memrealtime();
  uint32_t pev = 0;
#endif
  LPhy P = D.ps[j];
  const WMir m0 = mir_of(P);
  LNi *ring = D.ni + (uint64_t)j * (D.ni_mask + 1);
  LRx *rq = D.rq + (uint64_t)j * (D.rq_mask + 1);
  LPe *pe = D.pe + (uint64_t)j * LPE_CAP;
  const uint32_t m = D.ni_mask, ctx = D.node[j];
  uint32_t err = 0;
  for (;;) {
    // the next pending EndReceive and the next Receive
    int e = -1;
    LPe eb{};
    for (int q = 0; q < LPE_CAP; q++) {
      const LPe c = pe[q];
      if (c.used && (e < 0 || pe_before(c, eb))) e = q, eb = c;
    }
    const bool hr = P.rq_len > 0;
    LRx r{};
    if (hr) r = rq[P.rq_head & D.rq_mask];
    bool take_r;
    if (hr && e >= 0) take_r = r.at < eb.ts || (r.at == eb.ts && (eb.euid == NONE || r.uid < eb.euid));
    else if (hr) take_r = true;
    else if (e >= 0) take_r = false;
    else break;
    if (take_r) {
      if (!(r.at < bts || (r.at == bts && r.uid < buid))) break;
    } else {
      if (!(eb.ts < bts || (eb.ts == bts && eb.euid != NONE && eb.euid < buid))) break;
    }
    if (!take_r) {  // ---- YansWifiPhy::EndReceive (yans-wifi-phy.cc:770-799)
      const int64_t nw = (int64_t)eb.ts;
      nsgpu_wifil_end rec{eb.ts, eb.euid, (uint32_t)j, 0.0, 0.0, eb.tx, eb.can ? (uint32_t)NSGPU_WIFI_END_CANCELLED : 0u,
                          eb.can ? 0.0 : eb.w};
      LEck eck{0, NONE, 0.0};
      P.c.end++;
      if (eb.can) {  // EventImpl::Invoke skips a cancelled event (event-impl.cc:40-46); still dispatched
        P.c.end_cancelled++;
      } else {
        // InterferenceHelper::CalculateSnrPer (interference-helper.cc:336-353): ni = (start, m_firstPower), the
        // list after the event's own start entry (the ring's head: no fold while receiving) up to its end
        // entry, (end, 0) — CalculateNoiseInterferenceW (:229-243) — then CalculatePer's walk (:257-334)
        const LTx t = D.tx[eb.tx];
        const Mode pm = make_mode(t.mc, t.rate, t.bw), hm = header_mode(pm, t.preamble);
        const double noise0 = P.firstPower;
        rec.snr = snr_of(D, eb.w, noise0, pm);
        const int64_t t0 = (int64_t)eb.sts;
        const int64_t hdrStart = t0 + (int64_t)preamble_us(t.mc, pm.bw, t.preamble) * 1000;
        const int64_t payStart = hdrStart + (int64_t)header_us(t.mc, pm.bw, t.preamble) * 1000;
        // The walk's sequential part (the noise sums, the chunk bounds) runs here; the chunks' error-rate
        // models (~10 pow / erfc calls each, ~100-200 chunks an EndReceive) run lane-parallel in k_wl_mid,
        // which multiplies them in this order.  A zero-length chunk is 1.0 (CalculateChunkSuccessRate) and
        // is not recorded.  Without room in the chunk pool the product is formed here.
        const uint32_t need = 2 * P.len + 2;
        const uint32_t cs = atomicAdd(&D.cnt[4], need);
        const bool defer = (uint64_t)cs + need <= D.ck_cap;
        uint32_t cn = 0;
        double psr = 1.0, noiseW = noise0;
        auto ck = [&](int64_t dur, bool hdr) {
          if (defer) {
            if (dur != 0) D.ck[cs + cn++] = LCk{noiseW, (int64_t)((uint64_t)dur << 1) | (hdr ? 1 : 0)};
          } else {
            psr *= hdr ? chunk(D, snr_of(D, eb.w, noiseW, hm), dur, hm) : chunk(D, snr_of(D, eb.w, noiseW, pm), dur, pm);
          }
        };
        int64_t previous = t0;
        uint32_t q = 1;
        LNi nb[NB];  // the ring read NB entries a trip (the walk itself stays one entry at a time)
        uint32_t nbq = q - (uint32_t)NB;  // (q - nbq >= NB: the first entry loads a batch)
        for (bool last = false; !last;) {
          int64_t current;
          double delta;
          if (q < P.len) {
            if (q - nbq >= (uint32_t)NB) {
              nbq = q;
#pragma unroll
              for (int u = 0; u < NB; u++) nb[u] = ring[(P.head + q + u) & m];
            }
            const LNi en = nb[q - nbq];
            if (en.t == nw && eb.w == -en.d) {
              current = nw, delta = 0.0, last = true;  // (the event's end entry: the closing (end, 0))
            } else {
              current = en.t, delta = en.d;
            }
            q++;
          } else {
            current = nw, delta = 0.0, last = true;
          }
          if (previous >= payStart) {
            ck(current - previous, false);
          } else if (previous >= hdrStart) {
            if (current >= payStart) {
              ck(payStart - previous, true);
              ck(current - payStart, false);
            } else {
              ck(current - previous, true);
            }
          } else {
            if (current >= payStart) {
              ck(payStart - hdrStart, true);
              ck(current - payStart, false);
            } else if (current >= hdrStart) {
              ck(current - hdrStart, true);
            }
          }
          noiseW += delta;
          previous = current;
        }
        eck = LEck{cs, defer ? cn : NONE, eb.w};
        rec.per = 1 - psr;  // (deferred: k_wl_mid overwrites it)
        P.rxing = 0;  // NotifyRxEnd (); SwitchFromRxEndOk / Error -> DoSwitchFromRx (wifi-phy-state-helper.cc:391-402)
      }
      const uint32_t sl = eb.euid == NONE ? eb.sslot : NONE;
      const uint32_t ei = wave_alloc(&D.cnt[2]);
      if (ei < D.end_cap) {
        D.ends[ei] = rec;
        D.end_sslot[ei] = sl;
        D.eck[ei] = eck;
      } else {
        err |= WE_CAP;
      }
      const uint32_t vi = wave_alloc(D.evc + (blockIdx.x % EV_STRIPES) * EV_STRIDE);
      if (vi < D.ev_scap) D.ev[(blockIdx.x % EV_STRIPES) * D.ev_scap + vi] = LEv{eb.ts, eb.euid, ctx, sl, 0};
      else err |= WE_CAP;
      pe[e].used = 0;
      if (P.live == (uint32_t)e) P.live = NONE;
#ifdef NSGPU_PHASE_PROF
      pev++;
#endif
      continue;
    }
    // ---- YansWifiChannel::Receive -> YansWifiPhy::StartReceivePacket (yans-wifi-phy.cc:399-496)
    P.rq_head++;
    P.rq_len--;
    const int64_t nw = (int64_t)r.at;
    const int64_t endNew = nw + D.tx[r.tx].dur;
    if (P.len + 2 > m + 1) {
      err |= WE_NICAP;
      break;
    }
    // InterferenceHelper::AppendEvent (interference-helper.cc:192-212)
    if (!P.rxing) {  // fold the entries up to upper_bound (now) into m_firstPower; the new entry first
      cursor_advance<true>(ring, P.head, P.len, m, nw, P.cur_n, P.cur_s);
      P.head = (P.head + P.cur_n) & m;
      P.len -= P.cur_n;
      P.cur_n = 0;
      P.head = (P.head - 1) & m;
      ring[P.head] = LNi{nw, r.w};
      P.len++;
      P.firstPower = P.cur_s;
    } else {
      ni_insert(ring, P.head, P.len, m, nw, r.w);
    }
    ni_insert(ring, P.head, P.len, m, endNew, -r.w);
    P.ni_max = P.len > P.ni_max ? P.len : P.ni_max;
    const int st = P.endTx > nw ? 2 : P.rxing ? 1 : P.endCca > nw ? 3 : 0;  // GetState (:159-183)
    bool maybe = false;
    P.c.rx++;
    if (st == 1 || st == 2) {  // drop; noise after the current Rx / Tx (:431-457)
      if (st == 1) P.c.drop_rx++;
      else P.c.drop_tx++;
      int64_t until = (st == 1 ? P.endRx : P.endTx) - nw;  // GetDelayUntilIdle (:122-151)
      until = until > 0 ? until : 0;
      maybe = endNew > nw + until;
    } else if (r.w > D.edW) {  // sync (:461-472): SwitchToRx, NotifyRxStart, Schedule (rxDuration, EndReceive)
      int q = -1;
      for (int k = 0; k < LPE_CAP; k++)
        if (!pe[k].used) {
          q = k;
          break;
        }
      const uint32_t sl = wave_alloc(&D.cnt[1]);
      if (q < 0 || sl >= D.sync_cap) {
        err |= q < 0 ? WE_PECAP : WE_CAP;
        break;
      }
      D.sync[sl] = LSync{r.at, r.uid, NONE, (uint32_t)(j * LPE_CAP + q), 0};
      pe[q] = LPe{(uint64_t)endNew, r.at, r.uid, NONE, r.tx, 0, sl, 1, r.w};
      P.live = (uint32_t)q;
      P.rxing = 1;
      P.endRx = endNew;
      P.c.sync++;
    } else {
      P.c.drop_ed++;
      maybe = true;
    }
    if (maybe) {  // maybeCcaBusy (:485-495): GetEnergyDuration (interference-helper.cc:171-190)
      cursor_advance<false>(ring, P.head, P.len, m, nw, P.cur_n, P.cur_s);
      double noise = P.cur_s;
      int64_t end = nw;
      for (uint32_t q0 = P.cur_n; q0 < P.len; q0 += NB) {  // (NB entries a trip; the sums one at a time)
        LNi en[NB];
#pragma unroll
        for (int u = 0; u < NB; u++) en[u] = ring[(P.head + q0 + u) & m];
        bool stop = false;
#pragma unroll
        for (int u = 0; u < NB; u++) {
          if (stop || q0 + u >= P.len) {
            stop = true;
            continue;
          }
          noise += en[u].d;
          end = en[u].t;
          if (noise < D.ccaW) stop = true;
        }
        if (stop) break;
      }
      const int64_t cca = end > nw ? end - nw : 0;
      if (cca != 0) {  // SwitchMaybeToCcaBusy (wifi-phy-state-helper.cc:404-423)
        P.endCca = P.endCca > nw + cca ? P.endCca : nw + cca;
        P.c.cca_switches++;
      }
    }
    const uint32_t vi = wave_alloc(D.evc + (blockIdx.x % EV_STRIPES) * EV_STRIDE);
    if (vi < D.ev_scap) D.ev[(blockIdx.x % EV_STRIPES) * D.ev_scap + vi] = LEv{r.at, r.uid, ctx, NONE, 0};
    else err |= WE_CAP;
#ifdef NSGPU_PHASE_PROF
    pev++;
#endif
  }
  D.ps[j] = P;
  mir_put(D, j, m0, P);
  if (err) atomicOr(&D.cnt[3], err);
#ifdef NSGPU_PHASE_PROF
  const uint64_t dt = __builtin_amdgcn_s_memrealtime() - pt0;
  atomicAdd(&g_wl_ph[1], (unsigned long long)dt);
  atomicAdd(&g_wl_ph[2], 1ull);
  atomicAdd(&g_wl_ph[3], (unsigned long long)pev);
  atomicMax(&g_wl_ep[0], (unsigned long long)dt);
  atomicMax(&g_wl_ep[1], (unsigned long long)pev);
  if (dt > g_wl_ph[6]) {
    g_wl_ph[6] = dt;
    g_wl_ph[7] = pev;
  }
#endif
}
// ---- the epoch with one wave per phy (the default; NSGPU_WIFIL_LANE=1: the lane-per-phy k_wl_step above) ----
// k_wl_step's lanes spend their time in the NiChanges ring: a start inserted while receiving shifts every
// pending end (100-300 entries at 10^4 phys), and the cursor and the CCA energy walk read the ring entry by
// entry, 8 a memory trip.  Here the 64 lanes of a wave serve ONE phy: the ring is read 64 entries a trip, an
// insertion shifts 64 entries a trip, and the sums whose order matters (the cursor's prefix, the energy
// walk, CalculatePer's walk) run over the loaded entries lane by lane with readlane — no memory trip.  The
// same operations in the same order as k_wl_step (bit-exact).  Every decision is wave-uniform; lane 0
// makes the stores of uniform values.
__device__ __forceinline__ uint32_t lead_run(uint64_t bm) { return ~bm ? (uint32_t)__builtin_ctzll(~bm) : 64u; }
__device__ __forceinline__ int64_t rl_i64(int64_t v, int u) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, u);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), u);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ double rl_d(double v, int u) { return __longlong_as_double(rl_i64(__double_as_longlong(v), u)); }
__device__ __forceinline__ uint32_t rl_u32(uint32_t v, int u) { return (uint32_t)__builtin_amdgcn_readlane((int)v, u); }

__device__ __forceinline__ LPe rl_pe(const LPe &a, int u) {
  LPe b;
  b.ts = (uint64_t)rl_i64((int64_t)a.ts, u);
  b.sts = (uint64_t)rl_i64((int64_t)a.sts, u);
  b.suid = rl_u32(a.suid, u);
  b.euid = rl_u32(a.euid, u);
  b.tx = rl_u32(a.tx, u);
  b.can = rl_u32(a.can, u);
  b.sslot = rl_u32(a.sslot, u);
  b.used = rl_u32(a.used, u);
  b.w = rl_d(a.w, u);
  return b;
}
template <bool LE>
__device__ __forceinline__ void w_cursor_advance(const LNi *ring, uint32_t head, uint32_t len, uint32_t m, int64_t lim,
                                                 uint32_t &cur_n, double &cur_s) {
  const uint32_t lane = threadIdx.x & 63;
  while (cur_n < len) {
    const uint32_t idx = cur_n + lane;
    LNi e{0, 0.0};
    bool in = false;
    if (idx < len) {
      e = ring[(head + idx) & m];
      in = LE ? e.t <= lim : e.t < lim;
    }
    const uint32_t k = lead_run(__ballot(in));  // (sorted: the entries up to lim are the chunk's head)
    for (uint32_t u = 0; u < k; u++) cur_s += rl_d(e.d, (int)u);
    cur_n += k;
    if (k < 64) return;
  }
}
// AddNiChangeEvent (interference-helper.cc:378-383) at upper_bound (t): the entries after it move up one
// place, 64 a trip from the tail.
__device__ __forceinline__ void w_ni_insert(LNi *ring, uint32_t head, uint32_t &len, uint32_t m, int64_t t, double d) {
  const uint32_t lane = threadIdx.x & 63;
  uint32_t q = len;
  while (q > 0) {
    const uint32_t c0 = q > 64 ? q - 64 : 0, n = q - c0;
    LNi e{0, 0.0};
    bool gt = false;
    if (lane < n) {
      e = ring[(head + c0 + lane) & m];
      gt = e.t > t;
    }
    const uint32_t k = (uint32_t)__popcll(__ballot(gt));  // (sorted: the entries after t are the chunk's tail)
    if (gt) ring[(head + c0 + lane + 1) & m] = e;
    q -= k;
    if (k < n) break;
  }
  if (lane == 0) ring[(head + q) & m] = LNi{t, d};
  len++;
}

// The epoch kernel's per-wave staging (r05): the ring of NiChanges in LDS (RL entries; a longer ring stays
// in HBM), the Receive queue in the wave's registers (64 entries; more: HBM, 64 a trip), and the epoch's
// appends — dispatched events, end records, syncs — staged in LDS and claimed with one atomic per list
// per wave (the r04 kernel waited one atomic round trip per event).  A staged sync's slot is LOCAL | index
// until the claim; the staged events, end records and pending records that name it are patched then.
constexpr uint32_t RL = 256;
constexpr uint32_t RSPEC = 32, QSPEC = 4;  // ring / queue entries loaded with the state (speculatively)
constexpr uint32_t EVB = 64, ENB = 8, SYB = 8;
constexpr uint32_t LOCAL = 0x80000000u;
struct LEnd {  // a staged end record
  nsgpu_wifil_end rec;
  LEck eck;
  uint32_t sl, pad;
};
__device__ __forceinline__ LRx rl_rx(const LRx &a, int u) {
  return LRx{(uint64_t)rl_i64((int64_t)a.at, u), rl_u32(a.uid, u), rl_u32(a.tx, u), rl_d(a.w, u), rl_i64(a.dur, u)};
}
__device__ __forceinline__ LRx shfl_up_rx(const LRx &a) {
  LRx b;
  b.at = prev_lane64(a.at);  // (lane 0's is not used)
  b.uid = prev_lane32(a.uid);
  b.tx = prev_lane32(a.tx);
  b.w = __longlong_as_double((long long)prev_lane64((uint64_t)__double_as_longlong(a.w)));
  b.dur = (int64_t)prev_lane64((uint64_t)a.dur);
  return b;
}

// One epoch of every phy, a wave each: first the SendPackets the last host closure made (nsgpu_wifil_send
// batches up to NSEND of them into this launch: the sender's switch and this phy's Receive of each, what
// k_wl_send does — they precede every event of the epoch), then every pending Receive / EndReceive with a
// key below (bts, buid), in (ts, uid) order.
__global__ __launch_bounds__(64) void k_wl_stepw(const WDev D, uint64_t bts, uint32_t buid,
                                                                                   const SendBatch sb) {
  const int64_t j = D.j0 + blockIdx.x;
  const uint32_t lane = threadIdx.x;
  if (j >= D.j0 + D.nown) return;
#ifdef NSGPU_PHASE_PROF
  const uint64_t pt0 = __builtin_amdgcn_s_memtime();
  uint64_t pt1 = pt0, pt2 = pt0;
  uint32_t pev = 0;
#endif
  __shared__ LNi s_ring[RL];
  __shared__ LEv s_ev[EVB];
  __shared__ LEnd s_end[ENB];
  __shared__ LSync s_sy[SYB];
  LPhy P = D.ps[j];
  // (issued with the state: the ring's first RSPEC entries and the queue's first QSPEC at their compact places
  // — a fast epoch leaves them there, head 0 — used when the state says they are the ones; the first trip moves
  // ~1 KB a wave, 10^4 waves at once)
  const LNi rg = lane < RSPEC && lane <= D.ni_mask ? D.ni[(uint64_t)j * (D.ni_mask + 1) + lane] : LNi{0, 0.0};
  const LRx q8 = lane < QSPEC && lane <= D.rq_mask ? D.rq[(uint64_t)j * (D.rq_mask + 1) + lane] : LRx{};
  const WMir m0 = mir_of(P);
  LNi *const gring = D.ni + (uint64_t)j * (D.ni_mask + 1);
  LRx *rq = D.rq + (uint64_t)j * (D.rq_mask + 1);
  LPe *pe = D.pe + (uint64_t)j * LPE_CAP;
  const uint32_t gm = D.ni_mask, ctx = D.node[j];
  uint32_t *const evc = D.evc + (uint32_t)(j % EV_STRIPES) * EV_STRIDE;
  LEv *const evs = D.ev + (uint64_t)(j % EV_STRIPES) * D.ev_scap;
  uint32_t err = 0;
  // the pending EndReceive records: lane q < LPE_CAP holds record q for the whole epoch (written back at the
  // end when changed)
  LPe mine{};
  if (lane < (uint32_t)LPE_CAP) mine = pe[lane];
  bool pe_dirty = false, changed = false;
  // ---- the batched SendPackets: lane i computes this phy's Receive of send i (YansWifiChannel::Send)
  LRx my{};
  bool ok = false;
  if (lane < sb.n) {  // (computed by k_wl_rx when the closure sent: off the epoch's critical path)
    my = D.rxb[(uint64_t)lane * D.nphy + j];
    ok = my.at != ~0ull;
  }
  const uint64_t okm = __ballot(ok);
  const uint32_t nins = (uint32_t)__popcll(okm);
#pragma unroll
  for (uint32_t i = 0; i < NSEND; i++) {  // the sender's switch (YansWifiPhy::SendPacket, yans-wifi-phy.cc:499-522)
    if (i >= sb.n) break;
    if (sb.t[i].phy != (uint32_t)j) continue;
    const LTx &t = sb.t[i];
    changed = true;
    if (P.endTx > (int64_t)t.ts) {  // NS_ASSERT (!IsStateTx ()); SwitchToTx from TX: NS_FATAL_ERROR (:285-287)
      err |= WE_TX_IN_TX;
      continue;
    }
    if (P.rxing) {  // m_endRxEvent.Cancel (); NotifyRxEnd (); SwitchToTx's RX case (:263-268)
      if (lane == P.live) mine.can = 1;
      pe_dirty = true;
      P.live = NONE;
      P.rxing = 0;
      P.endRx = (int64_t)t.ts;
    }
    P.endTx = (int64_t)t.ts + t.dur;
  }
  // ---- the Receive queue and the ring: registers and LDS when they fit
  const bool fast = P.rq_len + nins <= 64 && P.len + 2 * (P.rq_len + nins) + 2 <= RL;
  uint32_t rq0 = ~0u;  // (queue offset of the loaded chunk; ~0: none)
  LRx rqc{};
  uint32_t qn = 0;     // (fast: entries in rqc)
  if (nins) changed = true;
  if (fast) {
    rq0 = 0;
    qn = P.rq_len;
    const bool qc = (P.rq_head & D.rq_mask) == 0 && qn <= QSPEC, h0 = (P.head & gm) == 0;
    if (lane < qn) rqc = qc ? q8 : rq[(P.rq_head + lane) & D.rq_mask];
#pragma unroll
    for (uint32_t u = 0; u < RL / 64; u++) {
      const uint32_t i = u * 64 + lane;
      if (i < P.len) s_ring[(P.head + i) & (RL - 1)] = h0 && i < RSPEC ? rg : gring[(P.head + i) & gm];
    }
    for (uint32_t i = 0; i < sb.n; i++) {  // (sorted by (arrival, uid): an insertion in registers)
      if (!((okm >> i) & 1ull)) continue;
      if (qn > D.rq_mask) {  // (k_wl_send's capacity check)
        err |= WE_RQCAP;
        continue;
      }
      const LRx e = rl_rx(my, (int)i);
      const bool lt = lane < qn && (rqc.at < e.at || (rqc.at == e.at && rqc.uid < e.uid));
      const uint32_t pos = (uint32_t)__popcll(__ballot(lt));
      const LRx up = shfl_up_rx(rqc);
      if (lane > pos && lane <= qn) rqc = up;
      if (lane == pos) rqc = e;
      qn++;
    }
    P.rq_len = qn;
    __syncthreads();
  } else if (nins) {  // (k_wl_send's insertion into the HBM queue, in send order)
    for (uint32_t i = 0; i < sb.n; i++) {
      if (!((okm >> i) & 1ull)) continue;
      const LRx e = rl_rx(my, (int)i);
      if (P.rq_len > D.rq_mask) {
        err |= WE_RQCAP;
        continue;
      }
      if (lane == 0) {
        uint32_t q = P.rq_len;
        while (q > 0) {
          const LRx x = rq[(P.rq_head + q - 1) & D.rq_mask];
          if (x.at < e.at || (x.at == e.at && x.uid < e.uid)) break;
          rq[(P.rq_head + q) & D.rq_mask] = x;
          q--;
        }
        rq[(P.rq_head + q) & D.rq_mask] = e;
      }
      P.rq_len++;
    }
    __syncthreads();
  }
  LNi *const ring = fast ? s_ring : gring;
  const uint32_t m = fast ? RL - 1 : gm;
#ifdef NSGPU_PHASE_PROF
  pt1 = __builtin_amdgcn_s_memtime();
#endif
  // ---- staged appends
  uint32_t ns = 0, ne = 0, nv = 0;
  bool slotted = false;  // (the phy's own event slots are written: further events go to the stripes)
  auto flush = [&]() {  // claim the staged syncs, end records and events (one atomic each), patch, store
    __syncthreads();
    uint32_t bs = 0, be = 0, bv = 0;
    if (lane == 0) {
      if (ns) bs = atomicAdd(&D.cnt[1], ns);
      if (ne) be = atomicAdd(&D.cnt[2], ne);
      if (nv && slotted) bv = atomicAdd(evc, nv);
    }
    bs = rl_u32(bs, 0);
    be = rl_u32(be, 0);
    bv = rl_u32(bv, 0);
    const auto fix = [&](uint32_t sl) { return sl != NONE && (sl & LOCAL) ? bs + (sl & ~LOCAL) : sl; };
    if (ns) {
      if ((uint64_t)bs + ns > D.sync_cap) err |= WE_CAP;
      else if (lane < ns) D.sync[bs + lane] = s_sy[lane];
      if (lane < (uint32_t)LPE_CAP) mine.sslot = fix(mine.sslot);
    }
    if (ne) {
      if ((uint64_t)be + ne > D.end_cap) {
        err |= WE_CAP;
      } else if (lane < ne) {
        const LEnd x = s_end[lane];
        D.ends[be + lane] = x.rec;
        D.end_sslot[be + lane] = fix(x.sl);
        D.eck[be + lane] = x.eck;
      }
    }
    if (nv && !slotted) {  // the epoch's first EVB events: the phy's own slots (a count, no claim)
      if (lane < nv) {
        LEv v = s_ev[lane];
        v.sslot = fix(v.sslot);
        D.evp[(uint64_t)j * EVB + lane] = v;
      }
      if (lane == 0) {
        D.evn[j] = nv;
        atomicAdd(&D.evt[(uint32_t)(j % EV_STRIPES) * EV_STRIDE], nv);  // (its result unused: no wait)
      }
      slotted = true;
    } else if (nv) {  // (more: the stripes, claimed)
      if ((uint64_t)bv + nv > D.ev_scap) {
        err |= WE_CAP;
      } else if (lane < nv) {
        LEv v = s_ev[lane];
        v.sslot = fix(v.sslot);
        evs[bv + lane] = v;
      }
    }
    ns = ne = nv = 0;
    __syncthreads();
  };
  uint32_t rqn = 0;  // Receives taken this epoch
  bool ring_dirty = false;
  for (;;) {
    // the next pending EndReceive (the selection reads the records lane by lane)
    const uint64_t used = __ballot(lane < (uint32_t)LPE_CAP && mine.used);
    int e = -1;
    LPe eb{};
    for (int q = 0; q < LPE_CAP; q++) {
      if (!((used >> q) & 1ull)) continue;
      const LPe c = rl_pe(mine, q);
      if (e < 0 || pe_before(c, eb)) e = q, eb = c;
    }
    const bool hr = P.rq_len > 0;
    LRx r{};
    if (hr) {
      if (rq0 == ~0u || rqn - rq0 >= 64) {  // (HBM queue: the next 64 queued Receives, one trip)
        rq0 = rqn;
        rqc = lane < P.rq_len ? rq[(P.rq_head + lane) & D.rq_mask] : LRx{};
      }
      r = rl_rx(rqc, (int)(rqn - rq0));
    }
    bool take_r;
    if (hr && e >= 0) take_r = r.at < eb.ts || (r.at == eb.ts && (eb.euid == NONE || r.uid < eb.euid));
    else if (hr) take_r = true;
    else if (e >= 0) take_r = false;
    else break;
    if (take_r) {
      if (!(r.at < bts || (r.at == bts && r.uid < buid))) break;
    } else {
      if (!(eb.ts < bts || (eb.ts == bts && eb.euid != NONE && eb.euid < buid))) break;
    }
    changed = true;
#ifdef NSGPU_PHASE_PROF
    pev++;
#endif
    if (!take_r) {  // ---- YansWifiPhy::EndReceive (yans-wifi-phy.cc:770-799)
      const int64_t nw = (int64_t)eb.ts;
      nsgpu_wifil_end rec{eb.ts, eb.euid, (uint32_t)j, 0.0, 0.0, eb.tx, eb.can ? (uint32_t)NSGPU_WIFI_END_CANCELLED : 0u,
                          eb.can ? 0.0 : eb.w};
      LEck eck{0, NONE, 0.0};
      P.c.end++;
      if (eb.can) {  // EventImpl::Invoke skips a cancelled event (event-impl.cc:40-46); still dispatched
        P.c.end_cancelled++;
      } else {
        // InterferenceHelper::CalculateSnrPer (interference-helper.cc:336-353), as k_wl_step: the walk's
        // sequential part here (64 ring entries a trip, then lane by lane), the chunks' models in k_wl_mid
        const LTx t = D.tx[eb.tx];
        const Mode pm = make_mode(t.mc, t.rate, t.bw);
        const double noise0 = P.firstPower;
        rec.snr = snr_of(D, eb.w, noise0, pm);
        const int64_t t0 = (int64_t)eb.sts;
        const int64_t hdrStart = t0 + (int64_t)preamble_us(t.mc, pm.bw, t.preamble) * 1000;
        const int64_t payStart = hdrStart + (int64_t)header_us(t.mc, pm.bw, t.preamble) * 1000;
        const uint32_t need = 2 * P.len + 2;
        uint32_t cs = 0;
        if (lane == 0) cs = atomicAdd(&D.cnt[4], need);
        cs = rl_u32(cs, 0);
        const bool defer = (uint64_t)cs + need <= D.ck_cap;
        if (!defer) err |= WE_CKCAP;  // (the run fails: no inline fallback here)
        // the walk, 64 ring entries a batch, a lane per step: step k's (previous, current) interval gives its
        // chunks (CalculatePer's cases, interference-helper.cc:270-330); only the noise before each step — a
        // running double sum, whose order is the reference's — is formed lane by lane
        uint32_t cn = 0;
        double noiseW = noise0;
        int64_t previous = t0;
        for (uint32_t q0 = 1, last = 0; !last; q0 += 64) {
          const uint32_t q = q0 + lane;
          LNi c{0, 0.0};
          if (q < P.len) c = ring[(P.head + q) & m];
          const uint64_t em = __ballot(q < P.len && c.t == nw && eb.w == -c.d);  // (the event's end entry)
          const uint32_t nin = P.len > q0 ? (P.len - q0 < 64 ? P.len - q0 : 64) : 0;
          uint32_t nstep = 64, close = 64;  // steps of the batch; the lane of the closing (nw, 0) step
          if (em) {
            nstep = (uint32_t)__builtin_ctzll(em) + 1, close = nstep - 1, last = 1;
          } else if (nin < 64) {
            nstep = nin + 1, close = nin, last = 1;  // (the list ends: the closing step after it)
          }
          const int64_t cur = lane == close ? nw : c.t;
          const double dl = lane == close ? 0.0 : c.d;
          int64_t prv = (int64_t)prev_lane64((uint64_t)cur);
          if (lane == 0) prv = previous;
          double nz = 0.0;  // the noise before step `lane`
          double acc = noiseW;
          for (uint32_t k = 0; k < nstep; k++) {
            if (lane == k) nz = acc;
            acc += rl_d(dl, (int)k);
          }
          int64_t d1 = 0, d2 = 0;
          bool h1 = false;
          if (lane < nstep) {
            if (prv >= payStart) {
              d1 = cur - prv;
            } else if (prv >= hdrStart) {
              h1 = true;
              if (cur >= payStart) d1 = payStart - prv, d2 = cur - payStart;
              else d1 = cur - prv;
            } else if (cur >= payStart) {
              h1 = true;
              d1 = payStart - hdrStart, d2 = cur - payStart;
            } else if (cur >= hdrStart) {
              h1 = true;
              d1 = cur - hdrStart;
            }
          }
          // (a zero-length chunk is skipped: ck (dur != 0)); the chunks' places by a wave prefix count
          const uint32_t n1 = d1 != 0, n2 = d2 != 0, nc = n1 + n2;
          const uint32_t pre = wave_incscan32(nc);
          const uint32_t tot = rl_u32(pre, 63), at = cn + pre - nc;
          if (defer) {
            if (n1) D.ck[cs + at] = LCk{nz, (int64_t)((uint64_t)d1 << 1) | (h1 ? 1 : 0)};
            if (n2) D.ck[cs + at + n1] = LCk{nz, (int64_t)((uint64_t)d2 << 1)};
            cn += tot;
          }
          previous = rl_i64(cur, (int)(nstep - 1));
          noiseW = acc;
        }
        eck = LEck{cs, defer ? cn : NONE, eb.w};
        rec.per = 0.0;  // (k_wl_mid writes the product)
        P.rxing = 0;  // NotifyRxEnd (); SwitchFromRxEndOk / Error -> DoSwitchFromRx (wifi-phy-state-helper.cc:391-402)
      }
      if (ne == ENB || nv == EVB) flush();
      const uint32_t sl = eb.euid == NONE ? rl_u32(mine.sslot, e) : NONE;  // (after a flush: its patched slot)
      if (lane == 0) {
        s_end[ne] = LEnd{rec, eck, sl, 0};
        s_ev[nv] = LEv{eb.ts, eb.euid, ctx, sl, 0};
      }
      ne++;
      nv++;
      if (lane == (uint32_t)e) mine.used = 0;
      pe_dirty = true;
      if (P.live == (uint32_t)e) P.live = NONE;
      continue;
    }
    // ---- YansWifiChannel::Receive -> YansWifiPhy::StartReceivePacket (yans-wifi-phy.cc:399-496)
    P.rq_head++;
    P.rq_len--;
    rqn++;
    const int64_t nw = (int64_t)r.at;
    const int64_t endNew = nw + r.dur;
    if (P.len + 2 > gm + 1) {
      err |= WE_NICAP;
      break;
    }
    ring_dirty = true;
    // InterferenceHelper::AppendEvent (interference-helper.cc:192-212)
    if (!P.rxing) {  // fold the entries up to upper_bound (now) into m_firstPower; the new entry first
      w_cursor_advance<true>(ring, P.head, P.len, m, nw, P.cur_n, P.cur_s);
      P.head = (P.head + P.cur_n) & m;
      P.len -= P.cur_n;
      P.cur_n = 0;
      P.head = (P.head - 1) & m;
      if (lane == 0) ring[P.head] = LNi{nw, r.w};
      P.len++;
      P.firstPower = P.cur_s;
    } else {
      w_ni_insert(ring, P.head, P.len, m, nw, r.w);
    }
    w_ni_insert(ring, P.head, P.len, m, endNew, -r.w);
    P.ni_max = P.len > P.ni_max ? P.len : P.ni_max;
    const int st = P.endTx > nw ? 2 : P.rxing ? 1 : P.endCca > nw ? 3 : 0;  // GetState (:159-183)
    bool maybe = false;
    P.c.rx++;
    if (st == 1 || st == 2) {  // drop; noise after the current Rx / Tx (:431-457)
      if (st == 1) P.c.drop_rx++;
      else P.c.drop_tx++;
      int64_t until = (st == 1 ? P.endRx : P.endTx) - nw;  // GetDelayUntilIdle (:122-151)
      until = until > 0 ? until : 0;
      maybe = endNew > nw + until;
    } else if (r.w > D.edW) {  // sync (:461-472): SwitchToRx, NotifyRxStart, Schedule (rxDuration, EndReceive)
      const uint64_t fr = __ballot(lane < (uint32_t)LPE_CAP && !mine.used);  // (the first free record)
      const int q = fr ? __builtin_ctzll(fr) : -1;
      if (q < 0) {
        err |= WE_PECAP;
        break;
      }
      if (ns == SYB) flush();
      if (lane == 0) s_sy[ns] = LSync{r.at, r.uid, NONE, (uint32_t)(j * LPE_CAP + q), 0};
      const LPe np{(uint64_t)endNew, r.at, r.uid, NONE, r.tx, 0, LOCAL | ns, 1, r.w};
      ns++;
      if (lane == (uint32_t)q) mine = np;
      pe_dirty = true;
      P.live = (uint32_t)q;
      P.rxing = 1;
      P.endRx = endNew;
      P.c.sync++;
    } else {
      P.c.drop_ed++;
      maybe = true;
    }
    if (maybe) {  // maybeCcaBusy (:485-495): GetEnergyDuration (interference-helper.cc:171-190)
      w_cursor_advance<false>(ring, P.head, P.len, m, nw, P.cur_n, P.cur_s);
      double noise = P.cur_s;
      int64_t end = nw;
      bool stop = false;
      for (uint32_t q0 = P.cur_n; q0 < P.len && !stop; q0 += 64) {  // (64 entries a trip; the sums one at a time)
        const LNi en = q0 + lane < P.len ? ring[(P.head + q0 + lane) & m] : LNi{0, 0.0};
        const uint32_t n = P.len - q0 < 64 ? P.len - q0 : 64;
        for (uint32_t u = 0; u < n; u++) {
          noise += rl_d(en.d, (int)u);
          end = rl_i64(en.t, (int)u);
          if (noise < D.ccaW) {
            stop = true;
            break;
          }
        }
      }
      const int64_t cca = end > nw ? end - nw : 0;
      if (cca != 0) {  // SwitchMaybeToCcaBusy (wifi-phy-state-helper.cc:404-423)
        P.endCca = P.endCca > nw + cca ? P.endCca : nw + cca;
        P.c.cca_switches++;
      }
    }
    if (nv == EVB) flush();
    if (lane == 0) s_ev[nv] = LEv{r.at, r.uid, ctx, NONE, 0};
    nv++;
  }
#ifdef NSGPU_PHASE_PROF
  pt2 = __builtin_amdgcn_s_memtime();
#endif
  if (ns | ne | nv) flush();
  // ---- write-backs: the pending records, the queue's rest (fast, after insertions), the ring (fast), the state
  if (pe_dirty && lane < (uint32_t)LPE_CAP) pe[lane] = mine;
  if (fast && (nins || rqn)) {  // (the queue's rest at its compact place: head 0)
    if (lane >= rqn && lane < qn) rq[lane - rqn] = rqc;
    P.rq_head = 0;
  }
  if (fast && ring_dirty) {  // (the ring at its compact place: head 0)
#pragma unroll
    for (uint32_t u = 0; u < RL / 64; u++) {
      const uint32_t i = u * 64 + lane;
      if (i < P.len) gring[i] = s_ring[(P.head + i) & (RL - 1)];
    }
    P.head = 0;
  }
  if (lane == 0) {
    if (changed) D.ps[j] = P;
    mir_put(D, j, m0, P);
    if (err) atomicOr(&D.cnt[3], err);
  }
#ifdef NSGPU_PHASE_PROF
  const uint32_t we = g_wepoch - g_wtarget;
  if (lane == 0 && we < WREC_E && j < (int64_t)WREC_P) {
    unsigned long long *w = g_wrec[we][j];
    w[0] = pt0;
    w[1] = pt1;
    w[2] = pt2;
    w[3] = __builtin_amdgcn_s_memtime();
    w[4] = pev;
  }
#endif
}

#ifdef NSGPU_PHASE_PROF
__global__ void k_wl_prof_epoch() {  // (one thread: fold the epoch's maxima, reset them)
  g_wl_ph[0] += g_wl_ep[0];
  g_wl_ph[4] += g_wl_ep[1];
  g_wl_ph[5] += 1;
  g_wl_ep[0] = g_wl_ep[1] = 0;
  g_wepoch++;
}
#endif

// CalculatePer's chunk product for the epoch's deferred EndReceives (interference-helper.cc:257-334): one
// block per end record, a thread per chunk (CalculateChunkSuccessRate with the error-rate model, every
// chunk's model evaluated at once), then the product in walk order by one thread from LDS (its order is
// the reference's: a float product is not reassociated).
constexpr uint32_t PER_SEG = 4096;  // chunks a block holds in LDS at once (32 KB)
__device__ __forceinline__ void wl_per(const WDev &D, uint32_t bx, uint32_t nbx, double *s_c) {
  const uint32_t nend = D.cnt[2] < D.end_cap ? D.cnt[2] : (uint32_t)D.end_cap;
  for (uint32_t ei = bx; ei < nend; ei += nbx) {  // (block-uniform)
    const LEck k = D.eck[ei];
    if (k.n == NONE) continue;
    const LTx t = D.tx[D.ends[ei].tx];
    const Mode pm = make_mode(t.mc, t.rate, t.bw), hm = header_mode(pm, t.preamble);
    double psr = 1.0;
    for (uint32_t b = 0; b < k.n; b += PER_SEG) {
      const uint32_t mm = k.n - b < PER_SEG ? k.n - b : PER_SEG;
      for (uint32_t u = threadIdx.x; u < mm; u += 256) {
        const LCk x = D.ck[k.start + b + u];
        const int64_t dur = x.dm >> 1;
        s_c[u] = (x.dm & 1) ? chunk(D, snr_of(D, k.w, x.noise, hm), dur, hm) : chunk(D, snr_of(D, k.w, x.noise, pm), dur, pm);
      }
      __syncthreads();
      if (threadIdx.x == 0) {
#pragma unroll 16
        for (uint32_t i = 0; i < mm; i++) psr *= s_c[i];
      }
      __syncthreads();
    }
    if (threadIdx.x == 0) D.ends[ei].per = 1 - psr;
  }
}

// The epoch's syncs in dispatch order (ts, uid of the syncing Receive): EndReceive uid = uid0 + rank.  A
// partition ranks its own syncs among every partition's (D.xsync: keys are unique, so the order of the gather
// does not matter).
__device__ __forceinline__ void wl_sync_rank(const WDev &D, uint32_t uid0, uint32_t bx, uint32_t nbx) {
  const uint32_t n = D.cnt[1] < D.sync_cap ? D.cnt[1] : (uint32_t)D.sync_cap;
  const LSync *const X = D.xsync ? D.xsync : D.sync;
  const uint32_t nx = D.xsync ? D.xn : n;
  for (uint32_t i = bx * 256 + threadIdx.x; i < n; i += nbx * 256) {
    const LSync a = D.sync[i];
    uint32_t r = 0;
    for (uint32_t k = 0; k < nx; k++) {
      const LSync b = X[k];
      r += b.sts < a.sts || (b.sts == a.sts && b.suid < a.suid);
    }
    D.sync[i].euid = uid0 + r;
  }
}
// The epoch's first tail kernel: the deferred PER products (blocks 0 .. MID_PER-1) and the syncs' ranks
// (the rest) — independent, one launch.
constexpr uint32_t MID_PER = 128, MID_RANK = 64;

template <int CTRL>
__device__ __forceinline__ uint64_t wdpp64t(uint64_t v) {
  return ((uint64_t)wdpp32<CTRL>((uint32_t)(v >> 32)) << 32) | wdpp32<CTRL>((uint32_t)v);
}
__device__ __forceinline__ uint64_t wrl64(uint64_t v, int l) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
}
// (every lane active) quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror, then the four rows' sums
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
  v += wdpp64t<0xB1>(v);
  v += wdpp64t<0x4E>(v);
  v += wdpp64t<0x141>(v);
  v += wdpp64t<0x140>(v);
  return wrl64(v, 0) + wrl64(v, 16) + wrl64(v, 32) + wrl64(v, 48);
}
// The epoch's close, on the critical path: k_wl_mid's last block (wl_fin) — the EndReceive uids (the sync
// order's) into the epoch's end records and its syncs' pending records, the status block (counters, the
// first END_STAGE end records) straight into the host's mapped copy (no copy).
// The epoch's order, behind it on a second stream (nothing the PHY or the host closures do depends on it;
// only the digest and the log):
//   k_wl_gather: the events from the phys' own slots (and the stripes' overflow) into one dense array, the
//     EndReceive uids resolved;
//   k_wl_tsort: a block per tile of TS keys (ts, uid << 32 | dense index) sorts it in LDS (bitonic);
//   k_wl_rank: an event's rank = its place in its tile + its lower bound in every other tile (each tile read
//     once into LDS, the searches in LDS), then its digest term and (logging) its rank; the block that
//     finishes last writes the running digest sum into the host's mapped copy and zeroes the epoch's
//     counters for the epoch two on.
// The status blocks, event lists, syncs and counters are kept per epoch parity; an epoch's k_wl_stepw waits
// for the order of the epoch two back (their last reader), which had a whole epoch to finish.  Epochs above
// ERANK_MAX events are ordered by the host from the dense events.  (The r04 all-pairs count, k_wl_order, was
// quadratic — 384 us at 6.5 x 10^4 events — and on the critical path.)
constexpr uint32_t TS = 2048, TS_T = 1024;  // keys a tile; threads a block (two keys each)
constexpr uint32_t ERANK_MAX = 65536, NTILE = ERANK_MAX / TS;
__device__ __forceinline__ bool key_lt(const ulonglong2 &a, const ulonglong2 &b) {
  return a.x < b.x || (a.x == b.x && a.y < b.y);
}
struct StripeMap {  // dense index -> stripe slot (the stripes' prefix in LDS)
  uint32_t pre[EV_STRIPES + 1];
};
__device__ __forceinline__ uint32_t load_stripes(const WDev &D, StripeMap &sm) {
  if (threadIdx.x < (uint32_t)EV_STRIPES) {
    const uint32_t c = D.evc[threadIdx.x * EV_STRIDE];
    sm.pre[threadIdx.x + 1] = c < D.ev_scap ? c : (uint32_t)D.ev_scap;
  }
  if (threadIdx.x == 0) sm.pre[0] = 0;
  __syncthreads();
  if (threadIdx.x == 0)
    for (int k = 1; k <= EV_STRIPES; k++) sm.pre[k] += sm.pre[k - 1];  // (64 adds, LDS)
  __syncthreads();
  return sm.pre[EV_STRIPES];
}
__device__ __forceinline__ uint64_t stripe_slot(const WDev &D, const StripeMap &sm, uint32_t i) {
  uint32_t lo = 0, hi = EV_STRIPES;  // pre[lo] <= i < pre[hi]
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (sm.pre[mid] <= i) lo = mid;
    else hi = mid;
  }
  return (uint64_t)lo * D.ev_scap + (i - sm.pre[lo]);
}
__device__ __forceinline__ LEv resolved(const WDev &D, const StripeMap &sm, uint32_t k) {
  LEv e = D.ev[stripe_slot(D, sm, k)];
  if (e.sslot != NONE) e.uid = D.sync[e.sslot].euid;
  return e;
}
// The epoch's close (k_wl_mid's last block): the EndReceive uids (the sync order's) into the end records and
// the syncs' pending records, the status block straight into the host's mapped copy.
__device__ __forceinline__ void wl_fin(const WDev &D, uint8_t *hst, uint32_t seq) {
  __shared__ StripeMap sm;
  __shared__ uint32_t s_nt;
  const uint32_t tid = threadIdx.x;
  if (tid < 64) {  // the events in the phys' own slots (their striped total), then the stripes' overflow
    const uint32_t c = (uint32_t)wave_sum_u64(D.evt[tid * EV_STRIDE]);  // (wave 0, every lane)
    if (tid == 0) s_nt = c;
  }
  const uint32_t nev = load_stripes(D, sm) + s_nt;  // (load_stripes's barriers order s_nt)
  const uint32_t nend = D.cnt[2] < D.end_cap ? D.cnt[2] : (uint32_t)D.end_cap;
  const uint32_t nsync = D.cnt[1] < D.sync_cap ? D.cnt[1] : (uint32_t)D.sync_cap;
  for (uint32_t i = tid; i < nend; i += 256) {  // the end records' EndReceive uids
    const uint32_t sl = D.end_sslot[i];
    if (sl != NONE) D.ends[i].uid = D.sync[sl].euid;
  }
  for (uint32_t i = tid; i < nsync; i += 256) {  // (a record taken again this epoch: a later sync's)
    const LSync y = D.sync[i];
    LPe &p = D.pe[y.loc];
    if (p.used && p.euid == NONE && p.sslot == i) p.euid = y.euid;
  }
  __syncthreads();
  nsgpu_wifil_end *he = reinterpret_cast<nsgpu_wifil_end *>(hst + STAT_HDR);
  for (uint32_t i = tid; i < nend && i < END_STAGE; i += 256) he[i] = D.ends[i];
  uint32_t *hc = reinterpret_cast<uint32_t *>(hst);
  if (tid == 0) {
    hc[0] = nev;
    hc[1] = D.cnt[1];
    hc[2] = D.cnt[2];
    hc[3] = D.cnt[3];
    D.cnt[0] = nev;
  }
  __threadfence_system();  // (the block's writes to the host's copy land before the epoch's flag)
  __syncthreads();
  if (tid == 0) __hip_atomic_store(&hc[6], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
// The epoch's tail kernel: the deferred PER products (blocks 0 .. MID_PER-1), the syncs' ranks (the rest),
// then — the block that finishes last — the epoch's close (wl_fin).
__global__ __launch_bounds__(256) void k_wl_mid(const WDev D, uint32_t uid0, uint8_t *hst, uint32_t seq) {
  __shared__ double s_c[PER_SEG];
  __shared__ uint32_t s_last;
  if (blockIdx.x < MID_PER) wl_per(D, blockIdx.x, MID_PER, s_c);
  else wl_sync_rank(D, uid0, blockIdx.x - MID_PER, MID_RANK);
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    s_last = atomicAdd(D.mticket, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (!s_last) return;
  __threadfence();
  wl_fin(D, hst, seq);
  if (threadIdx.x == 0) atomicExch(D.mticket, 0u);
}
// The epoch's events into one dense array, uids resolved (off the critical path): a block of 256 phys claims
// its slots' events' places with one atomic (the dense order is the claims' order: the ranks do not depend
// on it — keys are unique — and erank / evd agree), block 0 also the stripes' overflow events.
__global__ __launch_bounds__(256) void k_wl_gather(const WDev D) {
  __shared__ StripeMap sm;
  __shared__ uint32_t s_wt[4], s_base, s_sbase;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint32_t nstr = blockIdx.x == 0 ? load_stripes(D, sm) : 0u;
  const uint64_t j = (uint64_t)D.j0 + (uint64_t)blockIdx.x * 256 + tid;
  const uint32_t n = j < (uint64_t)(D.j0 + D.nown) ? D.evn[j] : 0u;
  if (n) D.evn[j] = 0;  // (for the epoch two on, which reuses this parity)
  const uint32_t x = wave_incscan32(n);
  if (lane == 63) s_wt[wv] = x;
  __syncthreads();
  uint32_t off = x - n, tot = 0;
  for (uint32_t w = 0; w < 4; w++) {
    off += w < wv ? s_wt[w] : 0u;
    tot += s_wt[w];
  }
  if (tid == 0) {
    s_base = tot ? atomicAdd(D.gtot, tot) : 0u;
    s_sbase = nstr ? atomicAdd(D.gtot, nstr) : 0u;
  }
  __syncthreads();
  for (uint32_t u = 0; u < n; u++) {
    LEv e = D.evp[j * EVB + u];
    if (e.sslot != NONE) e.uid = D.sync[e.sslot].euid;
    D.evd[s_base + off + u] = e;
  }
  for (uint32_t k = tid; k < nstr; k += 256) D.evd[s_sbase + k] = resolved(D, sm, k);
}
__global__ __launch_bounds__(TS_T) void k_wl_tsort(const WDev D) {
  __shared__ ulonglong2 s_t[TS];
  const uint32_t tid = threadIdx.x;
  const uint32_t nev = D.cnt[0];
  if (blockIdx.x == 0 && tid == 0) *D.gtot = 0;  // (k_wl_gather is done with its claims)
  if (nev > ERANK_MAX) return;  // (the host orders it from the dense events)
  const uint32_t base = blockIdx.x * TS;
  if (base >= nev) return;  // (block-uniform)
  LEv e[2];
#pragma unroll
  for (uint32_t u = 0; u < 2; u++) {  // (both loads in flight)
    const uint32_t k = base + u * TS_T + tid;
    e[u] = k < nev ? D.evd[k] : LEv{~0ull, NONE, 0, NONE, 0};
  }
#pragma unroll
  for (uint32_t u = 0; u < 2; u++) {
    const uint32_t k = base + u * TS_T + tid;
    s_t[u * TS_T + tid] = k < nev ? make_ulonglong2(e[u].ts, (uint64_t)e[u].uid << 32 | k) : make_ulonglong2(~0ull, ~0ull);
  }
  __syncthreads();
  for (uint32_t kk = 2; kk <= TS; kk <<= 1) {  // bitonic: TS_T compare-exchanges a stage
    for (uint32_t j = kk >> 1; j > 0; j >>= 1) {
      const uint32_t i = 2 * j * (tid / j) + (tid % j), l = i + j;
      const ulonglong2 a = s_t[i], b = s_t[l];
      if (key_lt(b, a) == ((i & kk) == 0)) {
        s_t[i] = b;
        s_t[l] = a;
      }
      __syncthreads();
    }
  }
  const uint32_t n = nev - base < TS ? nev - base : TS;
  for (uint32_t i = tid; i < n; i += TS_T) D.evg[base + i] = s_t[i];
}
__global__ __launch_bounds__(TS_T) void k_wl_rank(const WDev D, uint64_t K0, int keep, unsigned long long *hdig) {
  __shared__ ulonglong2 s_o[TS];
  __shared__ unsigned long long s_dg[TS_T / 64];
  __shared__ uint32_t s_last;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint32_t nev = D.cnt[0];
  const uint32_t nt = (nev + TS - 1) / TS;
  uint64_t dg = 0;
  if (nev <= ERANK_MAX && blockIdx.x < nt) {  // (block-uniform)
    const uint32_t t = blockIdx.x, n = nev - t * TS < TS ? nev - t * TS : TS;
    ulonglong2 x[2];
    uint32_t r[2];
#pragma unroll
    for (uint32_t u = 0; u < 2; u++) {
      const uint32_t p = u * TS_T + tid;
      x[u] = p < n ? D.evg[t * TS + p] : make_ulonglong2(~0ull, ~0ull);
      r[u] = p;  // (its place in its own tile)
    }
    for (uint32_t t2 = 0; t2 < nt; t2++) {
      if (t2 == t) continue;
      const uint32_t n2 = nev - t2 * TS < TS ? nev - t2 * TS : TS;
#pragma unroll
      for (uint32_t u = 0; u < 2; u++) {
        const uint32_t p = u * TS_T + tid;
        if (p < n2) s_o[p] = D.evg[t2 * TS + p];
      }
      __syncthreads();
#pragma unroll
      for (uint32_t u = 0; u < 2; u++) {  // lower bound: the tile's keys below x
        uint32_t lo = 0, c = n2;
        while (c > 0) {
          const uint32_t h = c >> 1;
          if (key_lt(s_o[lo + h], x[u])) lo += h + 1, c -= h + 1;
          else c = h;
        }
        r[u] += lo;
      }
      __syncthreads();
    }
#pragma unroll
    for (uint32_t u = 0; u < 2; u++) {
      if (u * TS_T + tid >= n) break;
      dg += digest_term(K0 + r[u], x[u].x, (uint32_t)(x[u].y >> 32));
      if (keep) D.erank[(uint32_t)x[u].y] = r[u];
    }
  }
  dg = wave_sum_u64(dg);
  if (lane == 0) s_dg[wv] = dg;
  __syncthreads();
  if (tid == 0) {
    unsigned long long t = 0;
    for (uint32_t w = 0; w < TS_T / 64; w++) t += s_dg[w];
    if (t) atomicAdd(D.edig, t);
    __threadfence();
    s_last = atomicAdd(D.ticket, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (!s_last) return;
  // the last block: the running digest sum for the host; this parity's counters zeroed for the epoch two on
  // (the order is their last reader; that epoch's k_wl_stepw waits for this kernel)
  __threadfence();
  if (tid == 0) {
    *hdig = atomicAdd(D.edig, 0ull);
    atomicExch(D.ticket, 0u);
  }
  if (tid < 3 || tid == 4) D.cnt[tid] = 0;  // (events, syncs, ends; the chunk pool)
  if (tid < (uint32_t)EV_STRIPES) D.evc[tid * EV_STRIDE] = 0, D.evt[tid * EV_STRIDE] = 0;
}

// (diagnostic, NSGPU_WIFIL_NOORDER=1) what k_wl_rank's last block zeroes, without the order; and (partitions,
// whose epochs are ordered over every partition's gathered events) the partition's own lists once gathered
__global__ void k_wl_zero(const WDev D) {
  const uint32_t tid = threadIdx.x;
  if (tid < 3 || tid == 4) D.cnt[tid] = 0;
  if (tid < (uint32_t)EV_STRIPES) D.evc[tid * EV_STRIDE] = 0, D.evt[tid * EV_STRIDE] = 0;
  if (tid == 5 && D.gtot) *D.gtot = 0;
}
__global__ void k_wl_set(uint32_t *p, uint32_t v) { *p = v; }

// SendPacket of phy s at (ts): the sender's state switch (thread s) and one Receive per receiver.
__global__ __launch_bounds__(256) void k_wl_send(const WDev D, uint32_t k, LTx t, double dbm, uint32_t base) {
  const int64_t j = D.j0 + (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (blockIdx.x == 0 && threadIdx.x == 0) D.tx[k] = t;  // (every partition holds every transmission)
  if (j >= D.j0 + D.nown) return;
  const uint32_t s = t.phy;
  if ((uint32_t)j == s) {  // YansWifiPhy::SendPacket (yans-wifi-phy.cc:499-522)
    LPhy &P = D.ps[j];
    if (P.endTx > (int64_t)t.ts) {  // NS_ASSERT (!IsStateTx ()); SwitchToTx from TX: NS_FATAL_ERROR (:285-287)
      atomicOr(&D.cnt[3], WE_TX_IN_TX);
      return;
    }
    if (P.rxing) {  // m_endRxEvent.Cancel (); NotifyRxEnd (); SwitchToTx's RX case (:263-268)
      D.pe[(uint64_t)j * LPE_CAP + P.live].can = 1;
      P.live = NONE;
      P.rxing = 0;
      P.endRx = (int64_t)t.ts;
    }
    P.endTx = (int64_t)t.ts + t.dur;
    D.mir[j] = mir_of(P);  // (the host applied the same switch to its copy; a partition's mirror is gathered)
    return;
  }
  LRx e;
  if (!reception(D, j, t, k, dbm, base, e)) return;
  const uint64_t at = e.at;
  const uint32_t uid = e.uid;
  LPhy &P = D.ps[j];
  LRx *rq = D.rq + (uint64_t)j * (D.rq_mask + 1);
  if (P.rq_len > D.rq_mask) {
    atomicOr(&D.cnt[3], WE_RQCAP);
    return;
  }
  uint32_t q = P.rq_len;  // sorted by (arrival, uid)
  while (q > 0) {
    const LRx e = rq[(P.rq_head + q - 1) & D.rq_mask];
    if (e.at < at || (e.at == at && e.uid < uid)) break;
    rq[(P.rq_head + q) & D.rq_mask] = e;
    q--;
  }
  rq[(P.rq_head + q) & D.rq_mask] = e;
  P.rq_len++;
}

// The Receives of one SendPacket (YansWifiChannel::Send's loop), computed when the closure sends — while the
// host goes on — into the batch's row of D.rxb; the next epoch's k_wl_stepw queues them.  Thread 0 records
// the transmission.
__global__ __launch_bounds__(256) void k_wl_rx(const WDev D, LRx *row, LTx t, uint32_t k, double dbm, uint32_t base) {
  const int64_t j = D.j0 + (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (blockIdx.x == 0 && threadIdx.x == 0) D.tx[k] = t;
  if (j >= D.j0 + D.nown) return;
  LRx e{};
  if (j == (int64_t)t.phy || !reception(D, j, t, k, dbm, base, e)) e.at = ~0ull;
  row[j] = e;
}

// Pending device events and the smallest ts among them (Next / IsFinished).
__global__ __launch_bounds__(256) void k_wl_pending(const WDev D, unsigned long long *out) {
  const int64_t j = D.j0 + (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= D.j0 + D.nown) return;
  const LPhy P = D.ps[j];
  uint64_t n = P.rq_len, mt = P.rq_len ? D.rq[(uint64_t)j * (D.rq_mask + 1) + (P.rq_head & D.rq_mask)].at : ~0ull;
  for (int q = 0; q < LPE_CAP; q++) {
    const LPe &p = D.pe[(uint64_t)j * LPE_CAP + q];
    if (p.used) n++, mt = p.ts < mt ? p.ts : mt;
  }
  if (n) {
    atomicAdd(&out[0], (unsigned long long)n);
    atomicMin(&out[1], (unsigned long long)mt);
  }
}

// The EndReceive hand-back (nsgpu_wifil_next_end): over the listened phys, the smallest key of a pending EndReceive
// that is not cancelled (its uid assigned: every epoch's close gives the syncs theirs), and the earliest time at
// which one not yet scheduled could fall — a pending Receive (queued, or a staged SendPacket's) strong enough to
// sync (rxPowerW > the ED threshold, yans-wifi-phy.cc:461) ends its EndReceive at arrival + duration (:466-471).
// One block; out: [0] ts, [1] uid | phy << 32 (~0: none), [2] the potential ts (~0: none).
__global__ __launch_bounds__(256) void k_wl_nextend(const WDev D, uint32_t nsend, unsigned long long *out) {
  __shared__ uint64_t s_ts[256], s_tp[256];
  __shared__ uint32_t s_uid[256], s_phy[256];
  const uint32_t tid = threadIdx.x;
  uint64_t bts = ~0ull, tp = ~0ull;
  uint32_t buid = NONE, bphy = NONE;
  for (uint32_t i = tid; i < D.nlis; i += 256) {
    const uint32_t j = D.lis[i];
    for (int q = 0; q < LPE_CAP; q++) {
      const LPe &p = D.pe[(uint64_t)j * LPE_CAP + q];
      if (p.used && !p.can && p.euid != NONE && (p.ts < bts || (p.ts == bts && p.euid < buid))) {
        bts = p.ts;
        buid = p.euid;
        bphy = j;
      }
    }
    const LPhy P = D.ps[j];
    const LRx *rq = D.rq + (uint64_t)j * (D.rq_mask + 1);
    for (uint32_t k = 0; k < P.rq_len; k++) {
      const LRx r = rq[(P.rq_head + k) & D.rq_mask];
      if (r.w > D.edW && r.at + (uint64_t)r.dur < tp) tp = r.at + (uint64_t)r.dur;
    }
    for (uint32_t k = 0; k < nsend; k++) {
      const LRx r = D.rxb[(uint64_t)k * D.nphy + j];
      if (r.at != ~0ull && r.w > D.edW && r.at + (uint64_t)r.dur < tp) tp = r.at + (uint64_t)r.dur;
    }
  }
  s_ts[tid] = bts, s_uid[tid] = buid, s_phy[tid] = bphy, s_tp[tid] = tp;
  __syncthreads();
  for (uint32_t o = 128; o > 0; o >>= 1) {
    if (tid < o) {
      const uint32_t u = tid + o;
      if (s_ts[u] < s_ts[tid] || (s_ts[u] == s_ts[tid] && s_uid[u] < s_uid[tid]))
        s_ts[tid] = s_ts[u], s_uid[tid] = s_uid[u], s_phy[tid] = s_phy[u];
      if (s_tp[u] < s_tp[tid]) s_tp[tid] = s_tp[u];
    }
    __syncthreads();
  }
  if (tid == 0) {
    out[0] = s_ts[0];
    out[1] = s_uid[0] == NONE ? ~0ull : ((unsigned long long)s_phy[0] << 32) | s_uid[0];
    out[2] = s_tp[0];
  }
}

// int64x64_t::Invert (int64x64-128.cc:119-134) with Divu (:70-92) and MulByInvert (:94-118), on the host.
u128 umul_by_invert(u128 a, u128 b) {
  const u128 ah = a >> 64, bh = b >> 64, al = a & (u128)~0ull, bl = b & (u128)~0ull;
  u128 mid = ah * bl + al * bh;
  mid >>= 64;
  return ah * bh + mid;
}
u128 invert(uint64_t v) {
  const u128 a = (u128)1 << 64;
  u128 quo = a / v, rem = a % v;  // Divu (a, v)
  u128 result = quo << 64;
  u128 div;
  if ((rem >> 64) == 0) rem <<= 64, div = v;
  else div = (u128)v >> 64;
  result += rem / div;
  const u128 tmp = umul_by_invert((u128)v << 64, result);  // int64x64_t (v, false).MulByInvert (result)
  if ((uint64_t)(tmp >> 64) != 1) result += 1;             // GetHigh () != 1
  return result;
}

}  // namespace
}  // namespace nsgpu

using namespace nsgpu;

struct nsgpu_wifil {
  WDev D{};
  hipStream_t s = nullptr;
  std::vector<void *> allocs;
  std::vector<uint32_t> recv;  // fan-out uids of one SendPacket per phy
  uint64_t n_tx = 0, tx_cap = 0;
  SendBatch sb{};  // SendPackets not yet applied (the next epoch launch applies them; k_wl_send past NSEND)
  // mapped host memory: the epoch's status block — counters, digest sum, first END_STAGE end records (the
  // device's D.cnt / D.edig / D.ends are laid out the same way in one allocation) — k_wl_rank writes it
  uint8_t *h_stat = nullptr, *d_stat = nullptr;  // (mapped: k_wl_rank writes it; d_stat is its device address)
  uint8_t *stat[2] = {nullptr, nullptr};  // the device's status blocks, by epoch parity (the next one is zeroed
  uint32_t par = 0;                       //   by the running epoch's k_wl_tsort: no fills between epochs)
  uint32_t *evc[2] = {nullptr, nullptr};  // the event-list stripe counters, by epoch parity (likewise)
  uint32_t *h_cnt = nullptr;
  LEv *evb[2] = {nullptr, nullptr};      // the event lists, by epoch parity (the order reads them an epoch behind)
  LEv *evpb[2] = {nullptr, nullptr};     // the phys' own event slots, by epoch parity (likewise)
  uint32_t *evnb[2] = {nullptr, nullptr};
  uint32_t *evtb[2] = {nullptr, nullptr};  // their striped totals, by epoch parity
  LSync *syncb[2] = {nullptr, nullptr};  // the syncs, by epoch parity (likewise)
  hipStream_t s2 = nullptr;              // the epochs' order (k_wl_tsort / k_wl_rank)
  hipEvent_t ev_fin[2] = {nullptr, nullptr}, ev_ord[2] = {nullptr, nullptr};
  bool ord_pending[2] = {false, false};  // an order of this parity's epoch was launched and not yet waited for
  unsigned long long *h_digtot = nullptr, *d_digtot = nullptr;  // (mapped) the ordered epochs' digest sum
  uint64_t dig_added = 0;                // the part of it already added to a caller's digest
  uint32_t seq = 0;                      // epochs launched (the close's flag)
  // host-side timing (NSGPU_WIFIL_HOSTPROF=1, printed at destroy): launches, the wait, the rest of an advance,
  // and the time between advances (the host closure and the runtime), in ns summed over epochs
  bool hprof = false;
  uint64_t hp_n = 0, hp_launch = 0, hp_wait = 0, hp_post = 0, hp_out = 0;
  std::chrono::steady_clock::time_point hp_last{};
  nsgpu_wifil_end *h_ends = nullptr;
  WMir *h_mir = nullptr;                 // mapped host memory: every phy's state fields (D.mir; GetState)
  std::vector<uint32_t> erank;
  unsigned long long *d_pend = nullptr, *h_pend = nullptr;
  std::vector<LEv> ev;
  std::vector<nsgpu_wifil_end> ends, ends_epoch;
  // the EndReceive hand-back: listened phys (a flag each, and the list the device scans), each phy's node
  std::vector<uint8_t> lis_on;
  std::vector<uint32_t> lis_list, node_h;
  bool lis_dirty = false;
  uint32_t *d_lis = nullptr;
  unsigned long long *d_next = nullptr, *h_next = nullptr;
  // ---- a partitioned PHY (nsgpu_wifil_create_dist / nsgpu_wifil_create_group): this handle is the host side
  // every rank replicates (the MAC's closures, the uids, GetState, the ends); `mem` are the partitions it runs —
  // one (RCCL: `comm`, the others on other GPUs) or all of them (a loopback group on this device) — each an engine
  // over its phys [lo, hi) with every array indexed by the global phy, launched on this handle's stream.
  std::vector<nsgpu_wifil *> mem;
  nsgpu_comm *comm = nullptr;
  std::vector<int64_t> plo, phi;  // every partition's phys (RCCL: gathered at create)
  int64_t pmax = 0;               // the largest partition (the gathers' padding)
  WDev U{};                       // the order over every partition's events (k_wl_tsort / k_wl_rank)
  LSync *xsync = nullptr;         // every partition's syncs of the epoch
  LSync *xsr = nullptr;           // (RCCL) their gather, padded
  LEv *xev = nullptr;             // (RCCL) the events' gather, padded
  nsgpu_wifil_end *uend = nullptr, *xend = nullptr;  // every partition's end records; (RCCL) their gather, padded
  WMir *xmir = nullptr, *dmir = nullptr, *smir = nullptr;  // (RCCL) mirror: gather, the partition's, send staging
  uint8_t *xps = nullptr, *sps = nullptr;                  // (RCCL) phy states for read_phys: gather, staging
  unsigned long long *xsm = nullptr;                       // (RCCL) small per-rank words: gather
  unsigned long long *ssm = nullptr;                       // (RCCL) small per-rank words: send
  uint64_t u_evcap = 0, g_sync_cap = 0, g_end_cap = 0;
};

// Blocks of b threads over n phys (at least one: a partition with no phys still records a transmission, and
// its kernels return at once).
static unsigned wl_grid(int64_t n, int b) { return (unsigned)std::max<int64_t>((n + b - 1) / b, 1); }

// The epoch's status block (counters, digest, end records) is stat[b].
static void wl_use_stat(nsgpu_wifil *h, uint32_t b) {
  h->par = b;
  h->D.cnt = reinterpret_cast<uint32_t *>(h->stat[b]);
  h->D.ev = h->evb[b];
  h->D.evp = h->evpb[b];
  h->D.evn = h->evnb[b];
  h->D.evt = h->evtb[b];
  h->D.sync = h->syncb[b];
  h->D.ends = reinterpret_cast<nsgpu_wifil_end *>(h->stat[b] + STAT_HDR);
  h->D.evc = h->evc[b];
}

template <class T>
static int wl_alloc(nsgpu_wifil *h, T **p, size_t n, const T *src = nullptr) {
  void *v = nullptr;
  NSGPU_HIP(hipMalloc(&v, std::max<size_t>(n, 1) * sizeof(T)));
  h->allocs.push_back(v);
  if (src && n) NSGPU_HIP(hipMemcpy(v, src, n * sizeof(T), hipMemcpyHostToDevice));
  else NSGPU_HIP(hipMemset(v, 0, std::max<size_t>(n, 1) * sizeof(T)));
  *p = (T *)v;
  return NSGPU_OK;
}

extern "C" int nsgpu_wifil_destroy(nsgpu_wifil *h) {
  if (!h) return NSGPU_OK;
  if (h->s) (void)hipStreamSynchronize(h->s);
  for (nsgpu_wifil *m : h->mem) {  // (a partition runs on this handle's stream)
    m->s = nullptr;
    nsgpu_wifil_destroy(m);
  }
  h->mem.clear();
  if (h->hprof && h->hp_n)
    fprintf(stderr, "nsgpu_wifil host: %llu epochs, per epoch (us): launches %.2f, wait %.2f, rest of advance %.2f, "
            "between advances %.2f\n", (unsigned long long)h->hp_n, h->hp_launch / 1e3 / h->hp_n, h->hp_wait / 1e3 / h->hp_n,
            h->hp_post / 1e3 / h->hp_n, h->hp_out / 1e3 / (h->hp_n > 1 ? h->hp_n - 1 : 1));
  for (hipStream_t q : {h->s, h->s2})
    if (q) {
      (void)hipStreamSynchronize(q);
      (void)hipStreamDestroy(q);
    }
  for (int b = 0; b < 2; b++) {
    if (h->ev_fin[b]) (void)hipEventDestroy(h->ev_fin[b]);
    if (h->ev_ord[b]) (void)hipEventDestroy(h->ev_ord[b]);
  }
  if (h->h_digtot) (void)hipHostFree(h->h_digtot);
  for (void *p : h->allocs) (void)hipFree(p);
  if (h->h_stat) (void)hipHostFree(h->h_stat);
  if (h->h_mir) (void)hipHostFree(h->h_mir);
  if (h->h_pend) (void)hipHostFree(h->h_pend);
  if (h->h_next) (void)hipHostFree(h->h_next);
  delete h;
  return NSGPU_OK;
}

// (hipDeviceGetStreamPriorityRange: greatest = the most urgent, a smaller number)
static int wl_prio(bool high) {
  int least = 0, greatest = 0;
  if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) return 0;
  return high ? greatest : least;
}

// Each phy's place among the phys of its channel (YansWifiChannel::Send's receiver loop, m_phyList order) and the
// Receives one SendPacket of it schedules (the other phys of its channel).
static void wl_channel_ranks(const nsgpu_wifil_config *c, std::vector<uint32_t> &rank, std::vector<uint32_t> &recv) {
  const int64_t N = c->n_phy;
  rank.assign((size_t)N, 0);
  recv.assign((size_t)N, 0);
  std::vector<std::pair<uint32_t, uint32_t>> cnt;  // (channel, count so far)
  for (int64_t j = 0; j < N; j++) {
    auto it = std::find_if(cnt.begin(), cnt.end(), [&](const std::pair<uint32_t, uint32_t> &p) { return p.first == c->channel[j]; });
    if (it == cnt.end()) cnt.emplace_back(c->channel[j], 0), it = cnt.end() - 1;
    rank[j] = it->second++;
  }
  for (int64_t j = 0; j < N; j++)
    for (auto &p : cnt)
      if (p.first == c->channel[j]) recv[j] = p.second - 1;
}

// An engine over phys [j0, j0 + nown) of the config (the single engine: all of them); its epoch lists are sized
// for capn phys (a partition: the largest partition's, so that every rank's lists hold a gather's padding).
static int wl_create(const nsgpu_wifil_config *c, int64_t j0, int64_t nown, int64_t capn, nsgpu_wifil **out) {
  if (!c || !out || c->n_phy <= 0 || !c->x || !c->y || !c->z || !c->channel || !c->node)
    return set_error(NSGPU_EINVAL, "nsgpu_wifil_create: bad config");
  const auto pow2 = [](uint32_t v) { return v >= 2 && (v & (v - 1)) == 0; };
  if (!pow2(c->ni_cap) || !pow2(c->rxq_cap) || c->tx_cap == 0 || c->tx_cap >= 0xffffffffull || c->loss.n < 0 ||
      c->loss.n > NSGPU_MAX_LOSS_CHAIN || c->error_model > NSGPU_WIFIL_YANS)
    return set_error(NSGPU_EINVAL, "nsgpu_wifil_create: ni_cap / rxq_cap must be powers of two >= 2, tx_cap in (0, 2^32)");
  nsgpu_wifil *h = new nsgpu_wifil();
  {
    const char *e = getenv("NSGPU_WIFIL_HOSTPROF");
    h->hprof = e && e[0] == '1';
  }
  const int64_t N = c->n_phy;
  WDev &D = h->D;
  D.nphy = N;
  D.j0 = j0;
  D.nown = nown;
  D.loss = c->loss;
  D.speed = c->speed;
  D.rx_gain_db = c->rx_gain_db;
  D.edW = pow(10.0, c->ed_threshold_dbm / 10.0) / 1000.0;   // SetEdThreshold (yans-wifi-phy.cc:228-232)
  D.ccaW = pow(10.0, c->cca_threshold_dbm / 10.0) / 1000.0; // SetCcaMode1Threshold (:234-238)
  D.nf = pow(10.0, c->rx_noise_figure_db / 10.0);           // SetRxNoiseFigure: DbToRatio (:192-197)
  D.model = c->error_model;
  D.ni_mask = c->ni_cap - 1;
  D.rq_mask = c->rxq_cap - 1;
  const u128 inv = invert(1000000000ull);
  D.inv_hi = (uint64_t)(inv >> 64);
  D.inv_lo = (uint64_t)inv;
  // the receiver loop's order on each channel (m_phyList order)
  std::vector<uint32_t> rank;
  wl_channel_ranks(c, rank, h->recv);
  const uint64_t ev_cap = (uint64_t)capn * 64 + 4096, sync_cap = (uint64_t)capn * LPE_CAP + 1024;
  int rc;
#define WL_TRY(x)                \
  if ((rc = (x)) != NSGPU_OK) {  \
    nsgpu_wifil_destroy(h);      \
    return rc;                   \
  }
  WL_TRY(wl_alloc(h, (double **)&D.x, N, c->x));
  WL_TRY(wl_alloc(h, (double **)&D.y, N, c->y));
  WL_TRY(wl_alloc(h, (double **)&D.z, N, c->z));
  WL_TRY(wl_alloc(h, (uint32_t **)&D.chan, N, c->channel));
  WL_TRY(wl_alloc(h, (uint32_t **)&D.node, N, c->node));
  WL_TRY(wl_alloc(h, (uint32_t **)&D.chan_rank, N, rank.data()));
  std::vector<LPhy> ps((size_t)N);
  for (auto &p : ps) p.live = NONE;
  WL_TRY(wl_alloc(h, &D.ps, N, ps.data()));
  WL_TRY(wl_alloc(h, &D.ni, (size_t)N * c->ni_cap));
  WL_TRY(wl_alloc(h, &D.rq, (size_t)N * c->rxq_cap));
  WL_TRY(wl_alloc(h, &D.pe, (size_t)N * LPE_CAP));
  WL_TRY(wl_alloc(h, &D.tx, c->tx_cap));
  WL_TRY(wl_alloc(h, &D.edig, 1));
  for (int b = 0; b < 2; b++) {  // [cnt x 5 | pad | edig | ends x sync_cap], two of them (epoch parity)
    WL_TRY(wl_alloc(h, &h->stat[b], STAT_HDR + sync_cap * sizeof(nsgpu_wifil_end)));
    WL_TRY(wl_alloc(h, &h->evc[b], (size_t)EV_STRIPES * EV_STRIDE));
    WL_TRY(wl_alloc(h, &h->evb[b], ev_cap));
    WL_TRY(wl_alloc(h, &h->evpb[b], (size_t)N * EVB));
    WL_TRY(wl_alloc(h, &h->evnb[b], (size_t)N));
    WL_TRY(wl_alloc(h, &h->evtb[b], (size_t)EV_STRIPES * EV_STRIDE));
    WL_TRY(wl_alloc(h, &h->syncb[b], sync_cap));
  }
  WL_TRY(wl_alloc(h, &D.evd, (size_t)N * EVB + ev_cap));  // (the slots' events, then the stripes')
  D.ev_scap = ev_cap / EV_STRIPES;
  wl_use_stat(h, 0);
  WL_TRY(wl_alloc(h, &D.end_sslot, sync_cap));
  WL_TRY(wl_alloc(h, &D.eck, sync_cap));
  // deferred chunks an epoch (~100-600 an EndReceive): 64 MB, or 512 a phy (k_wl_stepw has no inline
  // fallback — its error-rate models would take ~130 more VGPRs and scratch from every lane: a full pool
  // fails the run, WE_CKCAP)
  D.ck_cap = std::max<uint64_t>(1ull << 22, (uint64_t)capn * 512);
  WL_TRY(wl_alloc(h, &D.ck, (size_t)D.ck_cap));
  WL_TRY(wl_alloc(h, &D.erank, std::min<uint64_t>(ev_cap, ERANK_MAX)));
  WL_TRY(wl_alloc(h, &D.ticket, 1));
  WL_TRY(wl_alloc(h, &D.mticket, 1));
  WL_TRY(wl_alloc(h, &D.gtot, 1));
  WL_TRY(wl_alloc(h, &D.rxb, (size_t)NSEND * N));
  WL_TRY(wl_alloc(h, &D.evg, std::min<uint64_t>(ev_cap, ERANK_MAX)));
  WL_TRY(wl_alloc(h, &h->d_pend, 2));
  WL_TRY(wl_alloc(h, &h->d_next, 4));
  WL_TRY(wl_alloc(h, &h->d_lis, (size_t)N));
  D.lis = h->d_lis;
  D.nlis = 0;
  h->lis_on.assign((size_t)N, 0);
  h->node_h.assign(c->node, c->node + N);
#undef WL_TRY
  D.sync_cap = sync_cap;
  D.ev_cap = ev_cap;
  D.end_cap = sync_cap;
  h->tx_cap = c->tx_cap;
  if (hipHostMalloc((void **)&h->h_stat, STAT_HDR + END_STAGE * sizeof(nsgpu_wifil_end),
                    hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer((void **)&h->d_stat, h->h_stat, 0) != hipSuccess ||
      hipHostMalloc((void **)&h->h_mir, (size_t)N * sizeof(WMir), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer((void **)&D.mir, h->h_mir, 0) != hipSuccess ||
      hipHostMalloc((void **)&h->h_pend, 2 * sizeof(unsigned long long), hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc((void **)&h->h_next, 4 * sizeof(unsigned long long), hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc((void **)&h->h_digtot, sizeof(unsigned long long), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer((void **)&h->d_digtot, h->h_digtot, 0) != hipSuccess ||
      // the PHY's epochs on a high-priority stream, the order behind them on a low-priority one: streams of
      // different priorities never share a hardware queue (with GPU_MAX_HW_QUEUES = 4 and other engines' streams
      // alive, two normal streams could land on one queue, and the order's ~55 us would then run in line with
      // the next epoch: 75 -> 112 us an epoch, VERDICT r05 item 2, scripts/wifil_interference.py)
      hipStreamCreateWithPriority(&h->s, hipStreamNonBlocking, wl_prio(true)) != hipSuccess ||
      hipStreamCreateWithPriority(&h->s2, hipStreamNonBlocking, wl_prio(false)) != hipSuccess ||
      hipEventCreateWithFlags(&h->ev_fin[0], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&h->ev_fin[1], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&h->ev_ord[0], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&h->ev_ord[1], hipEventDisableTiming) != hipSuccess) {
    nsgpu_wifil_destroy(h);
    return set_error(NSGPU_EHIP, "nsgpu_wifil_create: host buffers / stream");
  }
  h->h_cnt = reinterpret_cast<uint32_t *>(h->h_stat);
  h->h_ends = reinterpret_cast<nsgpu_wifil_end *>(h->h_stat + STAT_HDR);
  *h->h_digtot = 0;
  std::memset(h->h_mir, 0, (size_t)N * sizeof(WMir));  // (the phys' initial state: every end time 0, not receiving)
  *out = h;
  return NSGPU_OK;
}

extern "C" int nsgpu_wifil_create(const nsgpu_wifil_config *c, nsgpu_wifil **out) {
  if (!c || !out) return set_error(NSGPU_EINVAL, "nsgpu_wifil_create: bad config");
  return wl_create(c, 0, c->n_phy, c->n_phy, out);
}

extern "C" int nsgpu_wifil_receivers(nsgpu_wifil *h, uint32_t phy, uint32_t *n) {
  if (!h || !n || phy >= h->D.nphy) return set_error(NSGPU_EINVAL, "nsgpu_wifil_receivers: bad phy");
  *n = h->recv[phy];
  return NSGPU_OK;
}

// YansWifiChannel::Send's ScheduleWithContext calls for one SendPacket of `sender` (yans-wifi-channel.cc:77-115),
// on the host: every other phy of m_phyList on the sender's channel number, in list order, gets the Receive with
// uid uid_base + its place and the context of its device's node (0xffffffff: a phy without a device).  This is the
// uid-critical half of a binding's Send (nsgpu_sim_wifi_send hands out the same block); no device is touched.
extern "C" int nsgpu_wifil_send_plan(const nsgpu_wifil_config *c, uint32_t sender, uint32_t uid_base, uint32_t *rx_phy,
                                     uint32_t *rx_uid, uint32_t *rx_ctx, uint64_t cap, uint64_t *n) {
  if (!c || !n || !c->channel || !c->node || (int64_t)sender >= c->n_phy)
    return set_error(NSGPU_EINVAL, "nsgpu_wifil_send_plan: bad config / sender");
  uint64_t k = 0;
  for (int64_t j = 0; j < c->n_phy; j++) {
    if ((uint32_t)j == sender || c->channel[j] != c->channel[sender]) continue;  // (:86-91)
    if ((uint64_t)uid_base + k >= nsgpu::UID_NEXT_MAX) return nsgpu::uid_range_error("nsgpu_wifil_send_plan");
    if (k < cap) {
      if (rx_phy) rx_phy[k] = (uint32_t)j;
      if (rx_uid) rx_uid[k] = uid_base + (uint32_t)k;
      if (rx_ctx) rx_ctx[k] = c->node[j];  // dstNode (:101-110)
    }
    k++;
  }
  *n = k;
  return NSGPU_OK;
}

static int wl_check_bits(uint32_t e, const char *what) {
  if (!e) return NSGPU_OK;
  if (e & WE_TX_IN_TX)
    return set_error(NSGPU_ESTATE, "%s: SendPacket while transmitting (yans-wifi-phy.cc:508 NS_ASSERT)", what);
  return set_error(NSGPU_ENOMEM, "%s: capacity exceeded (bits %u: 2 NiChanges ring, 4 Receive queue, 8 pending "
                                 "EndReceive records, 16 epoch lists, 32 CalculatePer chunk pool)", what, e);
}
static int wl_check(nsgpu_wifil *h, const char *what) { return wl_check_bits(h->h_cnt[3], what); }

// The batched SendPackets as k_wl_send launches (before anything that reads the phys or moves one).
static int wl_flush_sends(nsgpu_wifil *h) {
  const unsigned g = wl_grid(h->D.nown, 256);
  for (uint32_t i = 0; i < h->sb.n; i++)
    hipLaunchKernelGGL(k_wl_send, dim3(g), dim3(256), 0, h->s, h->D, h->sb.k0 + i, h->sb.t[i], h->sb.dbm[i], h->sb.base[i]);
  h->sb.n = 0;
  NSGPU_HIP(hipGetLastError());
  return NSGPU_OK;
}

static int wl_queue_send(nsgpu_wifil *h, const LTx &t, double dbm, uint32_t uid_base);

// YansWifiPhy::SendPacket of `phy` from the host closure running at (now, closure uid); its fan-out takes
// the uids uid_base .. uid_base + receivers - 1 (nsgpu_wifil_receivers).
extern "C" int nsgpu_wifil_send(nsgpu_wifil *h, uint64_t now, uint32_t uid_base, uint32_t phy, uint32_t size, double dbm,
                                uint32_t modclass, uint64_t rate, uint32_t bw, uint32_t preamble) {
  if (!h || phy >= h->D.nphy) return set_error(NSGPU_EINVAL, "nsgpu_wifil_send: bad phy");
  if (h->n_tx >= h->tx_cap) return set_error(NSGPU_ENOMEM, "nsgpu_wifil_send: tx_cap SendPacket calls");
  uint32_t nrx = 0;
  int rc0 = nsgpu_wifil_receivers(h, phy, &nrx);
  if (rc0) return rc0;
  if ((uint64_t)uid_base + nrx > nsgpu::UID_NEXT_MAX) return nsgpu::uid_range_error("nsgpu_wifil_send");
  int64_t dur = 0;
  int rc = nsgpu_wifi_tx_duration_ns(size, modclass, rate, bw, preamble, &dur);  // CalculateTxDuration
  if (rc) return rc;
  const LTx t{now, dur, rate, phy, modclass, bw, preamble};
  WMir &mr = h->h_mir[phy];  // the sender's switch (k_wl_send's), in the host's copy of its state fields
  if (!(mr.endTx > (int64_t)now)) {
    if (mr.rxing) mr.rxing = 0, mr.endRx = (int64_t)now;
    mr.endTx = (int64_t)now + dur;
  }
  if (h->mem.empty()) return wl_queue_send(h, t, dbm, uid_base);
  h->n_tx++;
  for (nsgpu_wifil *m : h->mem)  // (every partition records the transmission; its receivers take their Receives)
    if (int rcm = wl_queue_send(m, t, dbm, uid_base)) return rcm;
  return NSGPU_OK;
}

// A SendPacket into the engine's batch (applied by its next epoch launch), its Receives computed now (k_wl_rx).
static int wl_queue_send(nsgpu_wifil *h, const LTx &t, double dbm, uint32_t uid_base) {
  if (h->sb.n == NSEND) {
    int rcf = wl_flush_sends(h);
    if (rcf) return rcf;
  }
  const uint32_t k = (uint32_t)h->n_tx++;
  if (h->sb.n == 0) h->sb.k0 = k;
  hipLaunchKernelGGL(k_wl_rx, dim3(wl_grid(h->D.nown, 256)), dim3(256), 0, h->s, h->D,
                     h->D.rxb + (uint64_t)h->sb.n * h->D.nphy, t, k, dbm, uid_base);
  NSGPU_HIP(hipGetLastError());
  h->sb.t[h->sb.n] = t;
  h->sb.dbm[h->sb.n] = dbm;
  h->sb.base[h->sb.n] = uid_base;
  h->sb.n++;
  return NSGPU_OK;  // (applied by the next epoch launch: its error bits, if any, fail that nsgpu_wifil_advance)
}

// The dispatch order of an epoch (gather, tile sort, rank) on the second stream behind the epoch's close; the
// event lets the epoch two on (same parity) wait for it.  Launched before the host waits for the close: the
// launches' API time overlaps the epoch's kernels.
static int wl_launch_order(nsgpu_wifil *h, const WDev &D, uint32_t b, uint64_t K0, int keep) {
  NSGPU_HIP(hipEventRecord(h->ev_fin[b], h->s));
  NSGPU_HIP(hipStreamWaitEvent(h->s2, h->ev_fin[b], 0));
  hipLaunchKernelGGL(k_wl_gather, dim3(wl_grid(D.nown, 256)), dim3(256), 0, h->s2, D);
  hipLaunchKernelGGL(k_wl_tsort, dim3(NTILE), dim3(TS_T), 0, h->s2, D);
  hipLaunchKernelGGL(k_wl_rank, dim3(NTILE), dim3(TS_T), 0, h->s2, D, K0, keep, h->d_digtot);
  NSGPU_HIP(hipGetLastError());
  NSGPU_HIP(hipEventRecord(h->ev_ord[b], h->s2));
  h->ord_pending[b] = true;
  return NSGPU_OK;
}

static int wlg_advance(nsgpu_wifil *G, uint64_t bts, uint32_t buid, uint32_t *uid, uint64_t *dispatched, uint64_t *digest,
                       uint64_t *log_ts, uint32_t *log_uid, uint32_t *log_ctx, uint64_t log_cap);
static int wlg_pending(nsgpu_wifil *G, uint64_t *n, uint64_t *next_ts);
static int wlg_next_end(nsgpu_wifil *G, nsgpu_wifil_next *out);

// Every device event with a key below (bound_ts, bound_uid) (~0: all of them): dispatched in (ts, uid) order
// from rank *dispatched on; the syncs' EndReceives take the uids from *uid on.  The dispatches are added to
// the caller's digest (nsgpu_dispatch_digest_term) and log (at their ranks, below log_cap).
extern "C" int nsgpu_wifil_advance(nsgpu_wifil *h, uint64_t bound_ts, uint32_t bound_uid, uint32_t *uid,
                                   uint64_t *dispatched, uint64_t *digest, uint64_t *log_ts, uint32_t *log_uid,
                                   uint32_t *log_ctx, uint64_t log_cap) {
  if (!h || !uid || !dispatched || !digest) return set_error(NSGPU_EINVAL, "nsgpu_wifil_advance: null");
  if (!h->mem.empty()) return wlg_advance(h, bound_ts, bound_uid, uid, dispatched, digest, log_ts, log_uid, log_ctx, log_cap);
  using clk = std::chrono::steady_clock;
  const clk::time_point hp0 = h->hprof ? clk::now() : clk::time_point{};
  if (h->hprof && h->hp_n) h->hp_out += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(hp0 - h->hp_last).count();
  const WDev D = h->D;  // (this epoch's parity: its status block, lists, syncs; zeroed by the order two epochs back)
  const uint32_t b = h->par;
  if (h->ord_pending[b]) {  // (that order is their last reader; it has had a whole epoch: usually done, then the
    const hipError_t q = hipEventQuery(h->ev_ord[b]);  //  stream needs no wait packet before this epoch's kernels)
    if (q == hipErrorNotReady) NSGPU_HIP(hipStreamWaitEvent(h->s, h->ev_ord[b], 0));
    else NSGPU_HIP(q);
    h->ord_pending[b] = false;
  }
  // epoch: the phys' waves, then the tail (PER products + sync ranks + the close), then the order behind it
  static const bool lane_step = [] {  // (NSGPU_WIFIL_LANE=1: the lane-per-phy step kernel)
    const char *e = getenv("NSGPU_WIFIL_LANE");
    return e && e[0] == '1';
  }();
  if (lane_step) {
    int rcf = wl_flush_sends(h);
    if (rcf) return rcf;
    hipLaunchKernelGGL(k_wl_step, dim3(wl_grid(D.nown, 64)), dim3(64), 0, h->s, D, bound_ts, bound_uid);
  } else {
    hipLaunchKernelGGL(k_wl_stepw, dim3(wl_grid(D.nown, 1)), dim3(64), 0, h->s, D, bound_ts, bound_uid, h->sb);
    h->sb.n = 0;
  }
#ifdef NSGPU_PHASE_PROF
  hipLaunchKernelGGL(k_wl_prof_epoch, dim3(1), dim3(1), 0, h->s);
#endif
  const uint32_t seq = ++h->seq;  // (the close writes it into the host's status block last: the epoch's flag)
  hipLaunchKernelGGL(k_wl_mid, dim3(MID_PER + MID_RANK), dim3(256), 0, h->s, D, *uid, h->d_stat, seq);
  NSGPU_HIP(hipGetLastError());
  const bool logging = log_ts && log_uid && log_ctx && *dispatched < log_cap;
  static const bool no_order = [] {  // (diagnostic: NSGPU_WIFIL_NOORDER=1 skips the order — digest and log wrong)
    const char *e = getenv("NSGPU_WIFIL_NOORDER");
    return e && e[0] == '1';
  }();
  if (no_order) {  // (the counters the order would zero for the epoch two on)
    hipLaunchKernelGGL(k_wl_zero, dim3(1), dim3(64), 0, h->s, D);
  } else if (int rco = wl_launch_order(h, D, b, *dispatched, logging ? 1 : 0)) {
    return rco;
  }
  const clk::time_point hp1 = h->hprof ? clk::now() : clk::time_point{};
  {  // the epoch's flag in the mapped status block (a spin: a stream synchronize's wake-up took microseconds);
     // the stream is queried now and then, so a failed kernel (no flag) ends the wait with its error
    volatile uint32_t *flag = reinterpret_cast<volatile uint32_t *>(h->h_stat) + 6;
    for (uint64_t n = 1; *flag != seq; n++) {
      if ((n & 1023) == 0) {
        const hipError_t q = hipStreamQuery(h->s);
        if (q == hipErrorNotReady) continue;
        NSGPU_HIP(q);
        if (*flag != seq) return set_error(NSGPU_EHIP, "nsgpu_wifil_advance: the epoch's kernels ended without its flag");
      }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
  }
  const clk::time_point hp2 = h->hprof ? clk::now() : clk::time_point{};
  wl_use_stat(h, b ^ 1);  // (the next epoch's block; SendPackets until then report their errors there)
  int rc = wl_check(h, "nsgpu_wifil_advance");
  if (rc) return rc;
  const uint32_t nev = h->h_cnt[0], nsync = h->h_cnt[1], nend = h->h_cnt[2];
  // (r05z4n: a diagnostic build that skipped the order also skipped its zeroing of the epoch counters, so nev
  // grew epoch by epoch past the dense array — a count beyond it is an engine fault, reported as one)
  if ((uint64_t)nev > (uint64_t)D.nphy * EVB + D.ev_cap || nend > D.end_cap || nsync > D.sync_cap)
    return set_error(NSGPU_ESTATE, "nsgpu_wifil_advance: epoch counts beyond the engine's arrays (events %u, syncs "
                                   "%u, ends %u): the epoch counters were not reset", nev, nsync, nend);
  //  the uid range before anything of the epoch is published (ends, dispatch count, digest): the
  // epoch's EndReceives are queued, none dispatched; the caller makes the error sticky (nsgpu_sim: uid_spent)
  if ((uint64_t)*uid + nsync > nsgpu::UID_NEXT_MAX) return nsgpu::uid_range_error("nsgpu_wifil_advance");
  h->ends_epoch.resize(nend);
  if (nend > END_STAGE) {
    NSGPU_HIP(hipMemcpyAsync(h->ends_epoch.data(), D.ends, nend * sizeof(nsgpu_wifil_end), hipMemcpyDeviceToHost, h->s));
  } else if (nend) {
    std::copy(h->h_ends, h->h_ends + nend, h->ends_epoch.begin());
  }
  if (nev > ERANK_MAX || (logging && nev)) NSGPU_HIP(hipStreamSynchronize(h->s2));  // (the dense events / ranks)
  if (nev > ERANK_MAX) {  // a large epoch: its order on the host
    h->ev.resize(nev);
    NSGPU_HIP(hipMemcpyAsync(h->ev.data(), D.evd, nev * sizeof(LEv), hipMemcpyDeviceToHost, h->s));
    NSGPU_HIP(hipStreamSynchronize(h->s));
    std::sort(h->ev.begin(), h->ev.end(), [](const LEv &a, const LEv &b) { return a.ts != b.ts ? a.ts < b.ts : a.uid < b.uid; });
    for (const LEv &e : h->ev) {
      const uint64_t rank = (*dispatched)++;
      *digest += nsgpu_dispatch_digest_term(rank, e.ts, e.uid);
      if (rank < log_cap && log_ts && log_uid && log_ctx) {
        log_ts[rank] = e.ts;
        log_uid[rank] = e.uid;
        log_ctx[rank] = e.ctx;
      }
    }
  } else {
    if (logging && nev) {  // the ranked events into the log (no host sort)
      h->ev.resize(nev);
      h->erank.resize(nev);
      NSGPU_HIP(hipMemcpyAsync(h->ev.data(), D.evd, nev * sizeof(LEv), hipMemcpyDeviceToHost, h->s));
      NSGPU_HIP(hipMemcpyAsync(h->erank.data(), D.erank, nev * sizeof(uint32_t), hipMemcpyDeviceToHost, h->s));
      NSGPU_HIP(hipStreamSynchronize(h->s));
      for (uint32_t i = 0; i < nev; i++) {
        const uint64_t rank = *dispatched + h->erank[i];
        if (rank < log_cap) {
          log_ts[rank] = h->ev[i].ts;
          log_uid[rank] = h->ev[i].uid;
          log_ctx[rank] = h->ev[i].ctx;
        }
      }
    }
    *dispatched += nev;
  }
  const uint64_t tot = *h->h_digtot;  // (the ordered epochs' terms so far: one aligned 8-byte store's value)
  *digest += tot - h->dig_added;
  h->dig_added = tot;
  if (h->hprof) {
    const clk::time_point hp3 = clk::now();
    const auto ns = [](clk::time_point a, clk::time_point b) {
      return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(b - a).count();
    };
    h->hp_launch += ns(hp0, hp1);
    h->hp_wait += ns(hp1, hp2);
    h->hp_post += ns(hp2, hp3);
    h->hp_n++;
    h->hp_last = hp3;
  }
  if (nend > END_STAGE) NSGPU_HIP(hipStreamSynchronize(h->s));
  std::sort(h->ends_epoch.begin(), h->ends_epoch.end(),
            [](const nsgpu_wifil_end &a, const nsgpu_wifil_end &b) { return a.ts != b.ts ? a.ts < b.ts : a.uid < b.uid; });
  h->ends.insert(h->ends.end(), h->ends_epoch.begin(), h->ends_epoch.end());
  *uid += nsync;
  return NSGPU_OK;
}

// Waits for the epochs' order behind the PHY (k_wl_tsort / k_wl_rank on the second stream) and adds the
// digest terms it summed since the last advance / flush.
extern "C" int nsgpu_wifil_flush(nsgpu_wifil *h, uint64_t *digest) {
  if (!h || !digest) return set_error(NSGPU_EINVAL, "nsgpu_wifil_flush: null");
  NSGPU_HIP(hipStreamSynchronize(h->mem.empty() ? h->s2 : h->s));  // (a partitioned PHY orders every epoch at once)
  const uint64_t tot = *h->h_digtot;
  *digest += tot - h->dig_added;
  h->dig_added = tot;
  return NSGPU_OK;
}

// MobilityModel::SetPosition of `phy`'s node (mobility-model.cc SetPosition -> DoSetPosition; e.g. a host closure
// at run time): YansWifiChannel::Send reads the positions at each send (yans-wifi-channel.cc:92-96), so the
// later sends' fan-outs see it; receptions already scheduled keep their delay and power.  In stream order with
// the sends.
extern "C" int nsgpu_wifil_set_position(nsgpu_wifil *h, uint32_t phy, double x, double y, double z) {
  if (!h || phy >= h->D.nphy) return set_error(NSGPU_EINVAL, "nsgpu_wifil_set_position: bad phy");
  if (!h->mem.empty()) {  // (every partition holds every position)
    for (nsgpu_wifil *m : h->mem)
      if (int rcm = nsgpu_wifil_set_position(m, phy, x, y, z)) return rcm;
    return NSGPU_OK;
  }
  if (int rcf = wl_flush_sends(h)) return rcf;  // (the sends so far see the positions they were made with)
  const double v[3] = {x, y, z};
  double *dst[3] = {const_cast<double *>(h->D.x), const_cast<double *>(h->D.y), const_cast<double *>(h->D.z)};
  for (int c = 0; c < 3; c++)
    NSGPU_HIP(hipMemcpyAsync(dst[c] + phy, &v[c], sizeof(double), hipMemcpyHostToDevice, h->s));
  NSGPU_HIP(hipStreamSynchronize(h->s));  // (v is on this stack)
  return NSGPU_OK;
}

// WifiPhyStateHelper::GetState / GetDelayUntilIdle of `phy` at `now` (wifi-phy-state-helper.cc:122-183).
extern "C" int nsgpu_wifil_get_state(nsgpu_wifil *h, uint32_t phy, uint64_t now, nsgpu_wifil_phy_state *out) {
  if (!h || !out || phy >= h->D.nphy) return set_error(NSGPU_EINVAL, "nsgpu_wifil_get_state: bad phy");
  // the state fields as the last epoch's kernels (their lanes write a changed phy's) and the host's SendPackets
  // left them: every event before `now` has run (the runtime advanced the device to the running closure)
  const WMir P = h->h_mir[phy];
  const int64_t nw = (int64_t)now;
  out->state = P.endTx > nw ? NSGPU_WIFIL_TX : P.rxing ? NSGPU_WIFIL_RX : P.endCca > nw ? NSGPU_WIFIL_CCA_BUSY : NSGPU_WIFIL_IDLE;
  out->rxing = P.rxing;
  out->end_tx = P.endTx;
  out->end_rx = P.endRx;
  out->end_cca_busy = P.endCca;
  int64_t r = 0;
  if (out->state == NSGPU_WIFIL_RX) r = P.endRx - nw;
  else if (out->state == NSGPU_WIFIL_TX) r = P.endTx - nw;
  else if (out->state == NSGPU_WIFIL_CCA_BUSY) r = P.endCca - nw;
  out->delay_until_idle = r > 0 ? r : 0;
  return NSGPU_OK;
}

// The EndReceive records dispatched since the last call, in dispatch order (cap 0: count only, kept).
extern "C" int nsgpu_wifil_read_ends(nsgpu_wifil *h, nsgpu_wifil_end *out, uint64_t cap, uint64_t *n) {
  if (!h || !n) return set_error(NSGPU_EINVAL, "nsgpu_wifil_read_ends: null");
  *n = h->ends.size();
  if (!out || cap == 0) return NSGPU_OK;
  const uint64_t k = std::min<uint64_t>(cap, h->ends.size());
  std::copy(h->ends.begin(), h->ends.begin() + (ptrdiff_t)k, out);
  h->ends.erase(h->ends.begin(), h->ends.begin() + (ptrdiff_t)k);
  *n = k;
  return NSGPU_OK;
}

static nsgpu_wifi_phy_counters wl_counters(const LPhy &p) {
  nsgpu_wifi_phy_counters c = p.c;
  c.ni_len = p.len;
  c.ni_max = p.ni_max;
  c.end_tx = p.endTx;
  c.end_rx = p.endRx;
  c.end_cca_busy = p.endCca;
  c.first_power = p.firstPower;
  c.rxing = p.rxing;
  return c;
}
static int wlg_read_phys(nsgpu_wifil *G, nsgpu_wifi_phy_counters *out);

extern "C" int nsgpu_wifil_read_phys(nsgpu_wifil *h, nsgpu_wifi_phy_counters *out) {
  if (!h || !out) return set_error(NSGPU_EINVAL, "nsgpu_wifil_read_phys: null");
  if (!h->mem.empty()) return wlg_read_phys(h, out);
  if (int rcf = wl_flush_sends(h)) return rcf;
  std::vector<LPhy> ps((size_t)h->D.nphy);
  NSGPU_HIP(hipMemcpyAsync(ps.data(), h->D.ps, ps.size() * sizeof(LPhy), hipMemcpyDeviceToHost, h->s));
  NSGPU_HIP(hipStreamSynchronize(h->s));
  for (size_t j = 0; j < ps.size(); j++) out[j] = wl_counters(ps[j]);
  return NSGPU_OK;
}

// The EndReceive hand-back: the host takes phy's EndReceives back (on = 1) or not.
extern "C" int nsgpu_wifil_listen(nsgpu_wifil *h, uint32_t phy, int on) {
  if (!h || phy >= h->D.nphy) return set_error(NSGPU_EINVAL, "nsgpu_wifil_listen: bad phy");
  const uint8_t v = on ? 1 : 0;
  if (h->lis_on[phy] != v) {
    h->lis_on[phy] = v;
    h->lis_dirty = true;
  }
  return NSGPU_OK;
}

// The next EndReceive of a listened phy (k_wl_nextend): a pending one (not cancelled) and the earliest time a
// sync not yet made could put one (see the kernel).  Valid between advances.
extern "C" int nsgpu_wifil_next_end(nsgpu_wifil *h, nsgpu_wifil_next *out) {
  if (!h || !out) return set_error(NSGPU_EINVAL, "nsgpu_wifil_next_end: null");
  if (!h->mem.empty()) return wlg_next_end(h, out);
  if (h->lis_dirty) {
    h->lis_list.clear();
    for (size_t j = 0; j < h->lis_on.size(); j++)
      if (h->lis_on[j]) h->lis_list.push_back((uint32_t)j);
    if (!h->lis_list.empty())
      NSGPU_HIP(hipMemcpyAsync(h->d_lis, h->lis_list.data(), h->lis_list.size() * sizeof(uint32_t),
                               hipMemcpyHostToDevice, h->s));
    h->D.nlis = (uint32_t)h->lis_list.size();
    h->lis_dirty = false;
  }
  memset(out, 0, sizeof(*out));
  out->ts = out->ts_potential = ~0ull;
  if (h->D.nlis == 0) return NSGPU_OK;
  hipLaunchKernelGGL(k_wl_nextend, dim3(1), dim3(256), 0, h->s, h->D, h->sb.n, h->d_next);
  NSGPU_HIP(hipGetLastError());
  NSGPU_HIP(hipMemcpyAsync(h->h_next, h->d_next, 3 * sizeof(unsigned long long), hipMemcpyDeviceToHost, h->s));
  NSGPU_HIP(hipStreamSynchronize(h->s));  // (lis_list stays alive until here)
  if (h->h_next[1] != ~0ull) {
    out->found = 1;
    out->ts = h->h_next[0];
    out->uid = (uint32_t)h->h_next[1];
    out->phy = (uint32_t)(h->h_next[1] >> 32);
  }
  out->ts_potential = h->h_next[2];
  return NSGPU_OK;
}

// (runtime) The last epoch's EndReceive with this uid, and a phy's node (the hand-back's context).
bool nsgpu::wifil_epoch_end(const nsgpu_wifil *h, uint32_t uid, nsgpu_wifil_end *out) {
  for (const nsgpu_wifil_end &e : h->ends_epoch)
    if (e.uid == uid) {
      *out = e;
      return true;
    }
  return false;
}
uint32_t nsgpu::wifil_node(const nsgpu_wifil *h, uint32_t phy) {
  return phy < h->node_h.size() ? h->node_h[phy] : 0xffffffffu;
}

// Pending Receive / EndReceive events and the smallest ts among them (~0: none).
extern "C" int nsgpu_wifil_pending(nsgpu_wifil *h, uint64_t *n, uint64_t *next_ts) {
  if (!h || !n || !next_ts) return set_error(NSGPU_EINVAL, "nsgpu_wifil_pending: null");
  if (!h->mem.empty()) return wlg_pending(h, n, next_ts);
  if (int rcf = wl_flush_sends(h)) return rcf;
  const unsigned long long init[2] = {0ull, ~0ull};
  NSGPU_HIP(hipMemcpyAsync(h->d_pend, init, sizeof(init), hipMemcpyHostToDevice, h->s));
  hipLaunchKernelGGL(k_wl_pending, dim3(wl_grid(h->D.nown, 256)), dim3(256), 0, h->s, h->D, h->d_pend);
  NSGPU_HIP(hipGetLastError());
  NSGPU_HIP(hipMemcpyAsync(h->h_pend, h->d_pend, 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost, h->s));
  NSGPU_HIP(hipStreamSynchronize(h->s));
  *n = h->h_pend[0];
  *next_ts = h->h_pend[1];
  return NSGPU_OK;
}

// ---------------- the partitioned PHY (SURVEY 8(e) for the closed loop: YansWifiChannel::Send's receivers
// split over GPUs) ----------------
// Every rank runs the same host program — the MAC's closures, the runtime's uids and order, GetState — over a
// replicated host handle (the one these functions take); the device work of a phy (its Receives,
// InterferenceHelper, state machine, EndReceive walks and PER chunks) runs on the partition that owns it.  A phy's
// chain needs no other phy's state, so the partitions exchange only per epoch: (1) the epoch's syncs — an
// EndReceive's uid is its sync's rank among every partition's syncs; (2) the counters, the end records (the
// host's m_random draws and hand-backs) and the phys' state fields (GetState, DcfManager's CCA queries); (3) the
// dispatched events, ordered over all partitions for the digest and the log.  The epochs run on one stream and
// the host waits for each exchange (no order behind the epoch: every partition's events are needed first).
// RCCL (nsgpu_wifil_create_dist): this rank's partition, the exchanges as all-gathers padded to the largest
// partition's count (every rank's lists are sized for the largest partition); loopback (nsgpu_wifil_create_group):
// every partition on this device, the exchanges as device copies.

// k words of every partition (partition order): loopback from each member, RCCL this rank's all-gathered.
template <class F>
static int wlg_words(nsgpu_wifil *G, int k, F fn, std::vector<unsigned long long> &out) {
  const int P = (int)G->plo.size();
  out.assign((size_t)P * k, 0ull);
  if (!G->comm) {
    for (int q = 0; q < P; q++)
      if (int rc = fn(G->mem[q], &out[(size_t)q * k])) return rc;
    return NSGPU_OK;
  }
  std::vector<unsigned long long> mine((size_t)k, 0ull);
  if (int rc = fn(G->mem[0], mine.data())) return rc;
  NSGPU_HIP(hipMemcpyAsync(G->ssm, mine.data(), (size_t)k * 8, hipMemcpyHostToDevice, G->s));
  NCCL_TRY(ncclAllGather(G->ssm, G->xsm, (size_t)k, ncclUint64, G->comm->comm, G->s));
  NSGPU_HIP(hipMemcpyAsync(out.data(), G->xsm, (size_t)P * k * 8, hipMemcpyDeviceToHost, G->s));
  NSGPU_HIP(hipStreamSynchronize(G->s));
  return NSGPU_OK;
}

// Every partition's first cnt[q] elements (esz bytes) of a device array, concatenated in partition order into
// dst: loopback from each member's array src(m), RCCL from this rank's, all-gathered padded to the largest count
// through xbuf (P x that count; every partition's array holds it: equal capacities).
template <class S>
static int wlg_cat(nsgpu_wifil *G, const std::vector<uint64_t> &cnt, size_t esz, S src, void *xbuf, void *dst) {
  const hipStream_t s = G->s;
  const int P = (int)cnt.size();
  uint64_t off = 0;
  if (!G->comm) {
    for (int q = 0; q < P; q++) {
      if (cnt[q])
        NSGPU_HIP(hipMemcpyAsync((uint8_t *)dst + off * esz, src(G->mem[q]), cnt[q] * esz, hipMemcpyDeviceToDevice, s));
      off += cnt[q];
    }
    return NSGPU_OK;
  }
  uint64_t maxc = 0;
  for (uint64_t c : cnt) maxc = std::max(maxc, c);
  if (!maxc) return NSGPU_OK;
  NCCL_TRY(ncclAllGather(src(G->mem[0]), xbuf, maxc * esz, ncclUint8, G->comm->comm, s));
  for (int q = 0; q < P; q++) {
    if (cnt[q])
      NSGPU_HIP(hipMemcpyAsync((uint8_t *)dst + off * esz, (const uint8_t *)xbuf + (uint64_t)q * maxc * esz, cnt[q] * esz,
                               hipMemcpyDeviceToDevice, s));
    off += cnt[q];
  }
  return NSGPU_OK;
}

// The phys' state fields of every partition into the host's copy (RCCL; a loopback group's partitions write the
// one mapped copy themselves).
static int wlg_mirror(nsgpu_wifil *G) {
  if (!G->comm) return NSGPU_OK;
  const hipStream_t s = G->s;
  const int P = (int)G->plo.size(), r = G->comm->rank;
  const int64_t lo = G->plo[r], n = G->phi[r] - G->plo[r];
  if (n) NSGPU_HIP(hipMemcpyAsync(G->smir, G->dmir + lo, (size_t)n * sizeof(WMir), hipMemcpyDeviceToDevice, s));
  NCCL_TRY(ncclAllGather(G->smir, G->xmir, (size_t)G->pmax * sizeof(WMir), ncclUint8, G->comm->comm, s));
  for (int q = 0; q < P; q++) {
    const int64_t nq = G->phi[q] - G->plo[q];
    if (nq)
      NSGPU_HIP(hipMemcpyAsync(G->h_mir + G->plo[q], G->xmir + (uint64_t)q * G->pmax, (size_t)nq * sizeof(WMir),
                               hipMemcpyDeviceToHost, s));
  }
  NSGPU_HIP(hipStreamSynchronize(s));
  return NSGPU_OK;
}

static int wlg_advance(nsgpu_wifil *G, uint64_t bts, uint32_t buid, uint32_t *uid, uint64_t *dispatched, uint64_t *digest,
                       uint64_t *log_ts, uint32_t *log_uid, uint32_t *log_ctx, uint64_t log_cap) {
  const hipStream_t s = G->s;
  const int P = (int)G->plo.size();
  // (1) every partition's epoch: the batched SendPackets, then its phys' events below the bound
  for (nsgpu_wifil *m : G->mem) {
    if (m->D.nown) hipLaunchKernelGGL(k_wl_stepw, dim3((unsigned)m->D.nown), dim3(64), 0, s, m->D, bts, buid, m->sb);
    m->sb.n = 0;
  }
  NSGPU_HIP(hipGetLastError());
  // (2) the syncs of every partition
  std::vector<unsigned long long> w;
  int rc = wlg_words(G, 1, [&](nsgpu_wifil *m, unsigned long long *o) -> int {
    uint32_t c = 0;
    NSGPU_HIP(hipMemcpyAsync(&c, m->D.cnt + 1, sizeof(c), hipMemcpyDeviceToHost, s));
    NSGPU_HIP(hipStreamSynchronize(s));
    o[0] = std::min<uint64_t>(c, m->D.sync_cap);
    return NSGPU_OK;
  }, w);
  if (rc) return rc;
  std::vector<uint64_t> cnt((size_t)P);
  uint64_t tsy = 0;
  for (int q = 0; q < P; q++) cnt[q] = w[q], tsy += w[q];
  uint32_t xerr = 0;
  if (tsy > G->g_sync_cap) {  // (the single engine's capacity: the run fails as it would there)
    xerr |= WE_CAP;
    tsy = 0;
  } else if ((rc = wlg_cat(G, cnt, sizeof(LSync), [](nsgpu_wifil *m) { return (const void *)m->D.sync; }, G->xsr, G->xsync))) {
    return rc;
  }
  // (3) each partition's tail: PER products, its syncs' EndReceive uids (ranks among all), the close
  for (nsgpu_wifil *m : G->mem) {
    WDev Dm = m->D;
    Dm.xsync = G->xsync;
    Dm.xn = (uint32_t)tsy;
    hipLaunchKernelGGL(k_wl_mid, dim3(MID_PER + MID_RANK), dim3(256), 0, s, Dm, *uid, m->d_stat, ++m->seq);
  }
  NSGPU_HIP(hipGetLastError());
  NSGPU_HIP(hipStreamSynchronize(s));
  // (4) every partition's counters (the close's status block), then the checks before anything is published
  if ((rc = wlg_words(G, 4, [&](nsgpu_wifil *m, unsigned long long *o) -> int {
         for (int i = 0; i < 4; i++) o[i] = m->h_cnt[i];
         return NSGPU_OK;
       }, w)))
    return rc;
  std::vector<uint64_t> nevq((size_t)P), nendq((size_t)P);
  uint64_t nev = 0, nend = 0, nsync = 0;
  uint32_t err = xerr;
  const nsgpu_wifil *m0 = G->mem[0];
  for (int q = 0; q < P; q++) {
    nevq[q] = w[(size_t)q * 4], nsync += w[(size_t)q * 4 + 1], nendq[q] = w[(size_t)q * 4 + 2];
    err |= (uint32_t)w[(size_t)q * 4 + 3];
    if (nevq[q] > (uint64_t)m0->D.nphy * EVB + m0->D.ev_cap || nendq[q] > m0->D.end_cap)
      return set_error(NSGPU_ESTATE, "nsgpu_wifil_advance: partition %d's epoch counts beyond its arrays (events %llu, "
                                     "ends %llu)", q, (unsigned long long)nevq[q], (unsigned long long)nendq[q]);
    nev += nevq[q], nend += nendq[q];
  }
  if ((rc = wl_check_bits(err, "nsgpu_wifil_advance"))) return rc;
  if (nsync != tsy) return set_error(NSGPU_ESTATE, "nsgpu_wifil_advance: sync counts changed in the close");
  if ((uint64_t)*uid + nsync > nsgpu::UID_NEXT_MAX) return nsgpu::uid_range_error("nsgpu_wifil_advance");
  // the end records (EndReceive uids patched by the closes) and the state fields
  if ((rc = wlg_cat(G, nendq, sizeof(nsgpu_wifil_end), [](nsgpu_wifil *m) { return (const void *)m->D.ends; }, G->xend,
                    G->uend)))
    return rc;
  G->ends_epoch.resize(nend);
  if (nend) NSGPU_HIP(hipMemcpyAsync(G->ends_epoch.data(), G->uend, nend * sizeof(nsgpu_wifil_end), hipMemcpyDeviceToHost, s));
  if ((rc = wlg_mirror(G))) return rc;
  // (5) the order over every partition's events: each gathers its own (uids resolved), the union is ranked once
  for (nsgpu_wifil *m : G->mem)
    if (m->D.nown) hipLaunchKernelGGL(k_wl_gather, dim3(wl_grid(m->D.nown, 256)), dim3(256), 0, s, m->D);
  if ((rc = wlg_cat(G, nevq, sizeof(LEv), [](nsgpu_wifil *m) { return (const void *)m->D.evd; }, G->xev, G->U.evd))) return rc;
  for (nsgpu_wifil *m : G->mem) hipLaunchKernelGGL(k_wl_zero, dim3(1), dim3(64), 0, s, m->D);
  const bool logging = log_ts && log_uid && log_ctx && *dispatched < log_cap;
  hipLaunchKernelGGL(k_wl_set, dim3(1), dim3(1), 0, s, G->U.cnt, (uint32_t)nev);
  hipLaunchKernelGGL(k_wl_tsort, dim3(NTILE), dim3(TS_T), 0, s, G->U);
  hipLaunchKernelGGL(k_wl_rank, dim3(NTILE), dim3(TS_T), 0, s, G->U, *dispatched, logging ? 1 : 0, G->d_digtot);
  NSGPU_HIP(hipGetLastError());
  NSGPU_HIP(hipStreamSynchronize(s));
  if (nev > ERANK_MAX || (logging && nev)) {
    G->ev.resize(nev);
    NSGPU_HIP(hipMemcpyAsync(G->ev.data(), G->U.evd, nev * sizeof(LEv), hipMemcpyDeviceToHost, s));
    if (nev <= ERANK_MAX) {
      G->erank.resize(nev);
      NSGPU_HIP(hipMemcpyAsync(G->erank.data(), G->U.erank, nev * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    }
    NSGPU_HIP(hipStreamSynchronize(s));
  }
  if (nev > ERANK_MAX) {  // a large epoch: its order on the host
    std::sort(G->ev.begin(), G->ev.end(), [](const LEv &a, const LEv &b) { return a.ts != b.ts ? a.ts < b.ts : a.uid < b.uid; });
    for (const LEv &e : G->ev) {
      const uint64_t rank = (*dispatched)++;
      *digest += nsgpu_dispatch_digest_term(rank, e.ts, e.uid);
      if (logging && rank < log_cap) log_ts[rank] = e.ts, log_uid[rank] = e.uid, log_ctx[rank] = e.ctx;
    }
  } else {
    if (logging)
      for (uint64_t i = 0; i < nev; i++) {
        const uint64_t rank = *dispatched + G->erank[i];
        if (rank < log_cap) log_ts[rank] = G->ev[i].ts, log_uid[rank] = G->ev[i].uid, log_ctx[rank] = G->ev[i].ctx;
      }
    *dispatched += nev;
  }
  const uint64_t tot = *G->h_digtot;
  *digest += tot - G->dig_added;
  G->dig_added = tot;
  std::sort(G->ends_epoch.begin(), G->ends_epoch.end(),
            [](const nsgpu_wifil_end &a, const nsgpu_wifil_end &b) { return a.ts != b.ts ? a.ts < b.ts : a.uid < b.uid; });
  G->ends.insert(G->ends.end(), G->ends_epoch.begin(), G->ends_epoch.end());
  *uid += (uint32_t)nsync;
  return NSGPU_OK;
}

static int wlg_pending(nsgpu_wifil *G, uint64_t *n, uint64_t *next_ts) {
  const hipStream_t s = G->s;
  std::vector<unsigned long long> w;
  int rc = wlg_words(G, 2, [&](nsgpu_wifil *m, unsigned long long *o) -> int {
    if (int rcf = wl_flush_sends(m)) return rcf;
    const unsigned long long init[2] = {0ull, ~0ull};
    NSGPU_HIP(hipMemcpyAsync(m->d_pend, init, sizeof(init), hipMemcpyHostToDevice, s));
    if (m->D.nown) hipLaunchKernelGGL(k_wl_pending, dim3(wl_grid(m->D.nown, 256)), dim3(256), 0, s, m->D, m->d_pend);
    NSGPU_HIP(hipGetLastError());
    NSGPU_HIP(hipMemcpyAsync(m->h_pend, m->d_pend, 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    NSGPU_HIP(hipStreamSynchronize(s));
    o[0] = m->h_pend[0], o[1] = m->h_pend[1];
    return NSGPU_OK;
  }, w);
  if (rc) return rc;
  *n = 0;
  *next_ts = ~0ull;
  for (size_t q = 0; q < w.size() / 2; q++) *n += w[2 * q], *next_ts = std::min<uint64_t>(*next_ts, w[2 * q + 1]);
  return NSGPU_OK;
}

static int wlg_next_end(nsgpu_wifil *G, nsgpu_wifil_next *out) {
  const hipStream_t s = G->s;
  if (G->lis_dirty) {  // (each partition scans its own listened phys)
    G->lis_list.clear();
    for (size_t j = 0; j < G->lis_on.size(); j++)
      if (G->lis_on[j]) G->lis_list.push_back((uint32_t)j);
    for (nsgpu_wifil *m : G->mem) {
      m->lis_list.clear();
      for (uint32_t j : G->lis_list)
        if ((int64_t)j >= m->D.j0 && (int64_t)j < m->D.j0 + m->D.nown) m->lis_list.push_back(j);
      if (!m->lis_list.empty())
        NSGPU_HIP(hipMemcpyAsync(m->d_lis, m->lis_list.data(), m->lis_list.size() * sizeof(uint32_t), hipMemcpyHostToDevice, s));
      m->D.nlis = (uint32_t)m->lis_list.size();
    }
    G->D.nlis = (uint32_t)G->lis_list.size();
    G->lis_dirty = false;
  }
  memset(out, 0, sizeof(*out));
  out->ts = out->ts_potential = ~0ull;
  if (G->D.nlis == 0) return NSGPU_OK;
  std::vector<unsigned long long> w;
  int rc = wlg_words(G, 3, [&](nsgpu_wifil *m, unsigned long long *o) -> int {
    hipLaunchKernelGGL(k_wl_nextend, dim3(1), dim3(256), 0, s, m->D, m->sb.n, m->d_next);
    NSGPU_HIP(hipGetLastError());
    NSGPU_HIP(hipMemcpyAsync(m->h_next, m->d_next, 3 * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    NSGPU_HIP(hipStreamSynchronize(s));
    for (int i = 0; i < 3; i++) o[i] = m->h_next[i];
    return NSGPU_OK;
  }, w);
  if (rc) return rc;
  uint64_t bts = ~0ull, bkey = ~0ull, tp = ~0ull;
  for (size_t q = 0; q < w.size() / 3; q++) {
    const uint64_t ts = w[3 * q], key = w[3 * q + 1];
    if (key != ~0ull && (ts < bts || (ts == bts && (uint32_t)key < (uint32_t)bkey))) bts = ts, bkey = key;
    tp = std::min<uint64_t>(tp, w[3 * q + 2]);
  }
  if (bkey != ~0ull) {
    out->found = 1;
    out->ts = bts;
    out->uid = (uint32_t)bkey;
    out->phy = (uint32_t)(bkey >> 32);
  }
  out->ts_potential = tp;
  return NSGPU_OK;
}

static int wlg_read_phys(nsgpu_wifil *G, nsgpu_wifi_phy_counters *out) {
  const hipStream_t s = G->s;
  for (nsgpu_wifil *m : G->mem)
    if (int rcf = wl_flush_sends(m)) return rcf;
  const int P = (int)G->plo.size();
  std::vector<LPhy> ps;
  if (!G->comm) {
    for (nsgpu_wifil *m : G->mem) {
      ps.resize((size_t)m->D.nown);
      if (m->D.nown)
        NSGPU_HIP(hipMemcpyAsync(ps.data(), m->D.ps + m->D.j0, ps.size() * sizeof(LPhy), hipMemcpyDeviceToHost, s));
      NSGPU_HIP(hipStreamSynchronize(s));
      for (int64_t i = 0; i < m->D.nown; i++) out[m->D.j0 + i] = wl_counters(ps[(size_t)i]);
    }
    return NSGPU_OK;
  }
  const nsgpu_wifil *m = G->mem[0];
  if (m->D.nown)
    NSGPU_HIP(hipMemcpyAsync(G->sps, m->D.ps + m->D.j0, (size_t)m->D.nown * sizeof(LPhy), hipMemcpyDeviceToDevice, s));
  NCCL_TRY(ncclAllGather(G->sps, G->xps, (size_t)G->pmax * sizeof(LPhy), ncclUint8, G->comm->comm, s));
  ps.resize((size_t)P * G->pmax);
  NSGPU_HIP(hipMemcpyAsync(ps.data(), G->xps, ps.size() * sizeof(LPhy), hipMemcpyDeviceToHost, s));
  NSGPU_HIP(hipStreamSynchronize(s));
  for (int q = 0; q < P; q++)
    for (int64_t i = 0; i < G->phi[q] - G->plo[q]; i++) out[G->plo[q] + i] = wl_counters(ps[(size_t)q * G->pmax + i]);
  return NSGPU_OK;
}

// The replicated host handle over partitions lo[q] .. hi[q] (contiguous, covering every phy): every partition on
// this device (comm null), or this rank's (comm).
static int wlg_make(const nsgpu_wifil_config *c, const std::vector<int64_t> &lo, const std::vector<int64_t> &hi,
                    nsgpu_comm *comm, nsgpu_wifil **out) {
  const int P = (int)lo.size();
  const int64_t N = c->n_phy;
  for (int q = 0; q < P; q++)
    if (lo[q] > hi[q] || (q == 0 ? lo[q] != 0 : lo[q] != hi[q - 1]) || (q == P - 1 && hi[q] != N))
      return set_error(NSGPU_EINVAL, "nsgpu_wifil partitions: [%lld, %lld) of partition %d does not continue the ones "
                                     "before it over [0, %lld)", (long long)lo[q], (long long)hi[q], q, (long long)N);
  nsgpu_wifil *G = new nsgpu_wifil();
  int rc;
#define WG_TRY(x)                \
  if ((rc = (x)) != NSGPU_OK) {  \
    nsgpu_wifil_destroy(G);      \
    return rc;                   \
  }
  G->comm = comm;
  G->plo = lo;
  G->phi = hi;
  for (int q = 0; q < P; q++) G->pmax = std::max<int64_t>(G->pmax, hi[q] - lo[q]);
  G->D.nphy = N;
  G->D.j0 = 0;
  G->D.nown = 0;  // (the handle runs no phy itself)
  std::vector<uint32_t> rank;
  wl_channel_ranks(c, rank, G->recv);
  G->node_h.assign(c->node, c->node + N);
  G->lis_on.assign((size_t)N, 0);
  G->tx_cap = c->tx_cap;
  if (hipStreamCreateWithPriority(&G->s, hipStreamNonBlocking, wl_prio(true)) != hipSuccess ||
      hipHostMalloc((void **)&G->h_mir, (size_t)N * sizeof(WMir), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostMalloc((void **)&G->h_digtot, sizeof(unsigned long long), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer((void **)&G->d_digtot, G->h_digtot, 0) != hipSuccess) {
    nsgpu_wifil_destroy(G);
    return set_error(NSGPU_EHIP, "nsgpu_wifil partitions: host buffers / stream");
  }
  std::memset(G->h_mir, 0, (size_t)N * sizeof(WMir));
  *G->h_digtot = 0;
  WMir *mir_dev = nullptr;  // (loopback: the partitions' lanes write the host's mapped copy)
  if (!comm && hipHostGetDevicePointer((void **)&mir_dev, G->h_mir, 0) != hipSuccess) {
    nsgpu_wifil_destroy(G);
    return set_error(NSGPU_EHIP, "nsgpu_wifil partitions: mapped mirror");
  }
  for (int q = 0; q < P; q++) {
    if (comm && q != comm->rank) continue;
    nsgpu_wifil *m = nullptr;
    WG_TRY(wl_create(c, lo[q], hi[q] - lo[q], G->pmax, &m));
    (void)hipStreamSynchronize(m->s);
    (void)hipStreamDestroy(m->s);
    m->s = G->s;  // (every partition's kernels and copies in one order)
    G->mem.push_back(m);
  }
  if (comm) {
    WG_TRY(wl_alloc(G, &G->dmir, (size_t)N));
    mir_dev = G->dmir;
  }
  for (nsgpu_wifil *m : G->mem) m->D.mir = mir_dev;
  const nsgpu_wifil *m0 = G->mem[0];
  G->g_sync_cap = (uint64_t)N * LPE_CAP + 1024;  // (the single engine's)
  const uint64_t ev_per = (uint64_t)m0->D.nphy * EVB + m0->D.ev_cap;  // (a partition's dense events at most)
  G->u_evcap = (uint64_t)P * ev_per;
  WG_TRY(wl_alloc(G, &G->xsync, (size_t)G->g_sync_cap));
  WG_TRY(wl_alloc(G, &G->uend, (size_t)P * m0->D.end_cap));
  WDev &U = G->U;
  WG_TRY(wl_alloc(G, &U.evd, (size_t)G->u_evcap));
  WG_TRY(wl_alloc(G, &U.evg, (size_t)std::min<uint64_t>(G->u_evcap, ERANK_MAX)));
  WG_TRY(wl_alloc(G, &U.erank, (size_t)std::min<uint64_t>(G->u_evcap, ERANK_MAX)));
  WG_TRY(wl_alloc(G, &U.cnt, 8));
  WG_TRY(wl_alloc(G, &U.ticket, 1));
  WG_TRY(wl_alloc(G, &U.edig, 1));
  WG_TRY(wl_alloc(G, &U.gtot, 1));
  WG_TRY(wl_alloc(G, &U.evc, (size_t)EV_STRIPES * EV_STRIDE));
  WG_TRY(wl_alloc(G, &U.evt, (size_t)EV_STRIPES * EV_STRIDE));
  if (comm) {
    WG_TRY(wl_alloc(G, &G->xsr, (size_t)P * m0->D.sync_cap));
    WG_TRY(wl_alloc(G, &G->xev, (size_t)P * ev_per));
    WG_TRY(wl_alloc(G, &G->xend, (size_t)P * m0->D.end_cap));
    WG_TRY(wl_alloc(G, &G->smir, (size_t)std::max<int64_t>(G->pmax, 1)));
    WG_TRY(wl_alloc(G, &G->xmir, (size_t)P * std::max<int64_t>(G->pmax, 1)));
    WG_TRY(wl_alloc(G, &G->sps, (size_t)std::max<int64_t>(G->pmax, 1) * sizeof(LPhy)));
    WG_TRY(wl_alloc(G, &G->xps, (size_t)P * std::max<int64_t>(G->pmax, 1) * sizeof(LPhy)));
    WG_TRY(wl_alloc(G, &G->ssm, 8));
    WG_TRY(wl_alloc(G, &G->xsm, (size_t)P * 8));
  }
#undef WG_TRY
  *out = G;
  return NSGPU_OK;
}

extern "C" int nsgpu_wifil_create_group(const nsgpu_wifil_config *c, const int64_t *bounds, int n, nsgpu_wifil **out) {
  if (!c || !out || !bounds || n < 1 || c->n_phy <= 0) return set_error(NSGPU_EINVAL, "nsgpu_wifil_create_group: bad arguments");
  std::vector<int64_t> lo((size_t)n), hi((size_t)n);
  for (int q = 0; q < n; q++) lo[q] = bounds[q], hi[q] = bounds[q + 1];
  return wlg_make(c, lo, hi, nullptr, out);
}

extern "C" int nsgpu_wifil_create_dist(const nsgpu_wifil_config *c, int64_t phy_begin, int64_t phy_end, nsgpu_comm *comm,
                                       nsgpu_wifil **out) {
  if (!c || !out || !comm || c->n_phy <= 0) return set_error(NSGPU_EINVAL, "nsgpu_wifil_create_dist: bad arguments");
  // every rank's partition, gathered (each rank checks the same list: all fail or none)
  const int R = comm->nranks;
  unsigned long long *d = nullptr;
  std::vector<unsigned long long> all((size_t)2 * R);
  const unsigned long long mine[2] = {(unsigned long long)phy_begin, (unsigned long long)phy_end};
  hipStream_t s = nullptr;
  NSGPU_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipError_t e = hipMalloc((void **)&d, (size_t)(2 + 2 * R) * sizeof(unsigned long long));
  if (e == hipSuccess) e = hipMemcpyAsync(d, mine, sizeof(mine), hipMemcpyHostToDevice, s);
  ncclResult_t nr = ncclSuccess;
  if (e == hipSuccess) nr = ncclAllGather(d, d + 2, 2, ncclUint64, comm->comm, s);
  if (e == hipSuccess && nr == ncclSuccess) e = hipMemcpyAsync(all.data(), d + 2, all.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (d) (void)hipFree(d);
  (void)hipStreamDestroy(s);
  if (e != hipSuccess) return set_error(NSGPU_EHIP, "nsgpu_wifil_create_dist: %s", hipGetErrorString(e));
  if (nr != ncclSuccess) return set_error(NSGPU_EHIP, "nsgpu_wifil_create_dist: %s", ncclGetErrorString(nr));
  std::vector<int64_t> lo((size_t)R), hi((size_t)R);
  for (int q = 0; q < R; q++) lo[q] = (int64_t)all[2 * q], hi[q] = (int64_t)all[2 * q + 1];
  return wlg_make(c, lo, hi, comm, out);
}

#ifdef NSGPU_PHASE_PROF
// (diagnostic build only) the k_wl_step counters above, reset after the read
extern "C" int nsgpu_wifil_prof_read(unsigned long long *out) {
  NSGPU_HIP(hipDeviceSynchronize());
  NSGPU_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wl_ph), sizeof(unsigned long long) * 8));
  unsigned long long z[8] = {};
  NSGPU_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_wl_ph), z, sizeof(z)));
  return NSGPU_OK;
}
// (diagnostic build only) k_wl_stepw's wave records: arm for WREC_E epochs from `target` on (out null), or read
// them (out: WREC_E x WREC_P x 5 words)
extern "C" int nsgpu_wifil_prof_waves(uint32_t target, unsigned long long *out) {
  NSGPU_HIP(hipDeviceSynchronize());
  if (!out) {
    const uint32_t z = 0;
    NSGPU_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_wepoch), &z, sizeof(z)));
    NSGPU_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_wtarget), &target, sizeof(target)));
    return NSGPU_OK;
  }
  NSGPU_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wrec), sizeof(unsigned long long) * WREC_E * WREC_P * 5));
  return NSGPU_OK;
}
#endif
