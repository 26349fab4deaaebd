// nsref_wifi.cc — CPU ORACLE (test infrastructure only; see nsref.h header).
// Sequential restatement of the Wi-Fi PHY receive subset (include/nsgpu_types.h, nsgpu_wifi_scenario):
// a DefaultSimulatorImpl-style loop over a (ts, uid)-ordered map, YansWifiPhy::SendPacket ->
// YansWifiChannel::Send -> YansWifiChannel::Receive -> YansWifiPhy::StartReceivePacket with its
// InterferenceHelper and WifiPhyStateHelper, and EndReceive's state part.  Built -O2 -ffp-contract=off.
#include "nsref.h"
#include <math.h>
#include <algorithm>
#include <map>
#include <utility>
#include <vector>

namespace {

// WifiPhy::GetPlcpPreambleDurationMicroSeconds — wifi-phy.cc:187-231
uint32_t plcp_preamble_us(uint32_t mc, uint32_t bw, uint32_t preamble) {
  switch (mc) {
    case NSGPU_WIFI_OFDM:
      return bw == 10000000 ? 32 : bw == 5000000 ? 64 : 16;
    case NSGPU_WIFI_ERP_OFDM:
      return 4;
    default:  // DSSS
      return preamble == NSGPU_WIFI_PREAMBLE_SHORT ? 72 : 144;
  }
}

// WifiPhy::GetPlcpHeaderDurationMicroSeconds — wifi-phy.cc:141-185
uint32_t plcp_header_us(uint32_t mc, uint32_t bw, uint32_t preamble) {
  switch (mc) {
    case NSGPU_WIFI_OFDM:
      return bw == 10000000 ? 8 : bw == 5000000 ? 16 : 4;
    case NSGPU_WIFI_ERP_OFDM:
      return 16;
    default:
      return preamble == NSGPU_WIFI_PREAMBLE_SHORT ? 24 : 48;
  }
}

// WifiPhy::GetPayloadDurationMicroSeconds — wifi-phy.cc:233-286
uint32_t payload_us(uint32_t size, uint32_t mc, uint64_t rate, uint32_t bw) {
  if (mc == NSGPU_WIFI_OFDM || mc == NSGPU_WIFI_ERP_OFDM) {
    uint32_t sym = bw == 10000000 ? 8 : bw == 5000000 ? 16 : 4;
    double ndbps = (double)(rate * sym) / 1e6;
    uint32_t nsym = (uint32_t)lrint(ceil((16 + size * 8.0 + 6.0) / ndbps));
    return mc == NSGPU_WIFI_ERP_OFDM ? nsym * sym + 6 : nsym * sym;
  }
  return (uint32_t)lrint(ceil((size * 8.0) / (rate / 1.0e6)));
}

struct NiChange {  // InterferenceHelper::NiChange — interference-helper.cc:91-110 (ordered by time only)
  int64_t t;
  double d;
};

struct Phy {
  // InterferenceHelper (interference-helper.cc:112-126)
  std::vector<NiChange> ni;
  double firstPower = 0.0;
  bool irxing = false;
  // WifiPhyStateHelper (wifi-phy-state-helper.cc:52-60)
  bool rxing = false;
  int64_t endTx = 0, endRx = 0, endCca = 0, startCca = 0, startRx = 0;
  // YansWifiPhy::m_endRxEvent: index into the EndReceive table, -1 = none
  int64_t endRxEvent = -1;
  nsgpu_wifi_phy_counters c{};
};

enum Kind { TX = 0, RX = 1, END = 2, STOP = 3 };
struct Ev {
  uint32_t kind, a, b;
  double rx_dbm;
};

struct Run {
  const nsgpu_wifi_scenario *sc;
  std::vector<Phy> phy;
  std::vector<int64_t> dur;
  std::map<std::pair<uint64_t, uint32_t>, Ev> q;  // the (ts, uid) order of scheduler.h:105-121
  uint32_t uid;
  uint64_t now = 0;
  double edW, ccaW;
  nsgpu_wifi_stats st{};
  std::vector<nsgpu_wifi_end_record> ends;
  nsgpu_wifi_rx_log *rx_log;
  uint32_t *tx_base;

  static double DbmToW(double dBm) {  // yans-wifi-phy.cc:727-732
    double mW = pow(10.0, dBm / 10.0);
    return mW / 1000.0;
  }
  static bool near(double v, double thr) { return fabs(v - thr) <= 1e-9 * thr; }

  // WifiPhyStateHelper::GetState — wifi-phy-state-helper.cc:159-183 (no SWITCHING: m_endSwitching = 0)
  int state(const Phy &p) const {
    if (p.endTx > (int64_t)now) return 2;  // TX
    if (p.rxing) return 1;                 // RX
    if (p.endCca > (int64_t)now) return 3; // CCA_BUSY
    return 0;                              // IDLE
  }
  // GetDelayUntilIdle — wifi-phy-state-helper.cc:122-151
  int64_t delay_until_idle(const Phy &p) const {
    int64_t r = 0;
    switch (state(p)) {
      case 1: r = p.endRx - (int64_t)now; break;
      case 2: r = p.endTx - (int64_t)now; break;
      case 3: r = p.endCca - (int64_t)now; break;
      default: r = 0;
    }
    return std::max<int64_t>(r, 0);
  }

  // InterferenceHelper::GetPosition / AddNiChangeEvent — interference-helper.cc:373-383
  void add_ni(Phy &p, NiChange c) {
    auto it = std::upper_bound(p.ni.begin(), p.ni.end(), c, [](const NiChange &a, const NiChange &b) { return a.t < b.t; });
    p.ni.insert(it, c);
  }
  // InterferenceHelper::AppendEvent — interference-helper.cc:192-212
  void append_event(Phy &p, int64_t start, int64_t end, double w) {
    if (!p.irxing) {
      auto nowIt = std::upper_bound(p.ni.begin(), p.ni.end(), NiChange{(int64_t)now, 0},
                                    [](const NiChange &a, const NiChange &b) { return a.t < b.t; });
      for (auto i = p.ni.begin(); i != nowIt; ++i) p.firstPower += i->d;
      p.ni.erase(p.ni.begin(), nowIt);
      p.ni.insert(p.ni.begin(), NiChange{start, w});
    } else {
      add_ni(p, NiChange{start, w});
    }
    add_ni(p, NiChange{end, -w});
    st.ni_inserts += 2;
    p.c.ni_max = std::max<uint32_t>(p.c.ni_max, (uint32_t)p.ni.size());
  }
  // InterferenceHelper::GetEnergyDuration — interference-helper.cc:171-190
  int64_t energy_duration(const Phy &p, double energyW, uint8_t &flags) const {
    double noiseInterferenceW = p.firstPower;
    int64_t end = (int64_t)now;
    for (const NiChange &i : p.ni) {
      noiseInterferenceW += i.d;
      end = i.t;
      if (end < (int64_t)now) continue;
      if (near(noiseInterferenceW, energyW)) flags |= NSGPU_WIFI_F_NEAR_CCA;
      if (noiseInterferenceW < energyW) break;
    }
    return end > (int64_t)now ? end - (int64_t)now : 0;
  }

  // YansWifiPhy::SendPacket — yans-wifi-phy.cc:499-522, then YansWifiChannel::Send — yans-wifi-channel.cc:77-115
  int send(uint32_t k) {
    const uint32_t s = sc->tx_phy[k];
    Phy &p = phy[s];
    if (state(p) == 2) return -1;  // NS_ASSERT (!IsStateTx ()); SwitchToTx from TX: NS_FATAL_ERROR (:285-287)
    if (state(p) == 1) {            // :510-514
      ends[p.endRxEvent].flags |= NSGPU_WIFI_END_CANCELLED;
      p.irxing = false;             // m_interference.NotifyRxEnd ()
    }
    // WifiPhyStateHelper::SwitchToTx — wifi-phy-state-helper.cc:254-290
    if (state(p) == 1) {
      p.rxing = false;
      p.endRx = (int64_t)now;
    }
    p.endTx = (int64_t)now + dur[k];
    st.tx++;
    if (tx_base) tx_base[k] = uid;
    st.digest += nsgpu_wifi_term(TX, now, sc->tx_uid[k], uid, 0);
    for (int64_t j = 0; j < sc->n_phy; j++) {
      if (j == (int64_t)s) continue;
      if (sc->channel[j] != sc->channel[s]) continue;
      double d = nsref_distance(sc->x[s], sc->y[s], sc->z[s], sc->x[j], sc->y[j], sc->z[j]);
      int64_t delay = nsref_const_speed_delay(d, sc->speed);
      double rx = nsref_calc_rx_power(sc->tx_dbm[k], d, &sc->loss);
      Ev e{RX, k, (uint32_t)j, rx};
      q.emplace(std::make_pair(now + (uint64_t)delay, uid), e);
      if (rx_log) {
        nsgpu_wifi_rx_log &l = rx_log[(uint64_t)k * sc->n_phy + j];
        l.ts = now + (uint64_t)delay;
        l.uid = uid;
      }
      uid++;
    }
    return 0;
  }

  // YansWifiPhy::StartReceivePacket — yans-wifi-phy.cc:399-496
  void start_receive(uint32_t k, uint32_t j, double rxPowerDbm) {
    Phy &p = phy[j];
    rxPowerDbm += sc->rx_gain_db;
    double rxPowerW = DbmToW(rxPowerDbm);
    int64_t rxDuration = dur[k];
    int64_t endRx = (int64_t)now + rxDuration;
    append_event(p, (int64_t)now, endRx, rxPowerW);  // m_interference.Add (:409-414)
    uint8_t outcome, flags = 0;
    bool maybeCca = false;
    switch (state(p)) {
      case 1:  // RX
        outcome = NSGPU_WIFI_DROP_RX;
        maybeCca = endRx > (int64_t)now + delay_until_idle(p);
        break;
      case 2:  // TX
        outcome = NSGPU_WIFI_DROP_TX;
        maybeCca = endRx > (int64_t)now + delay_until_idle(p);
        break;
      default:  // CCA_BUSY, IDLE
        if (near(rxPowerW, edW)) flags |= NSGPU_WIFI_F_NEAR_ED;
        if (rxPowerW > edW) {
          outcome = NSGPU_WIFI_SYNC;
          // WifiPhyStateHelper::SwitchToRx — wifi-phy-state-helper.cc:291-322
          p.rxing = true;
          p.startRx = (int64_t)now;
          p.endRx = (int64_t)now + rxDuration;
          p.irxing = true;  // m_interference.NotifyRxStart ()
          nsgpu_wifi_end_record r{};
          r.ts = (uint64_t)endRx;
          r.sync_ts = now;
          r.uid = uid;
          r.phy = j;
          r.tx = k;
          p.endRxEvent = (int64_t)ends.size();
          ends.push_back(r);
          q.emplace(std::make_pair((uint64_t)endRx, uid), Ev{END, (uint32_t)p.endRxEvent, 0, 0.0});
          uid++;
        } else {
          outcome = NSGPU_WIFI_DROP_ED;
          maybeCca = true;
        }
    }
    int64_t cca = 0;
    if (maybeCca) {
      flags |= NSGPU_WIFI_F_CCA_EVAL;
      cca = energy_duration(p, ccaW, flags);
      if (cca != 0) {  // WifiPhyStateHelper::SwitchMaybeToCcaBusy — wifi-phy-state-helper.cc:404-423
        flags |= NSGPU_WIFI_F_CCA_SWITCH;
        p.startCca = (int64_t)now;
        p.endCca = std::max<int64_t>(p.endCca, (int64_t)now + cca);
      }
    }
    st.rx++;
    p.c.rx++;
    switch (outcome) {
      case NSGPU_WIFI_SYNC: st.sync++; p.c.sync++; break;
      case NSGPU_WIFI_DROP_RX: st.drop_rx++; p.c.drop_rx++; break;
      case NSGPU_WIFI_DROP_TX: st.drop_tx++; p.c.drop_tx++; break;
      default: st.drop_ed++; p.c.drop_ed++;
    }
    if (flags & NSGPU_WIFI_F_CCA_EVAL) st.cca_evals++;
    if (flags & NSGPU_WIFI_F_CCA_SWITCH) { st.cca_switches++; p.c.cca_switches++; }
    if (flags & (NSGPU_WIFI_F_NEAR_ED | NSGPU_WIFI_F_NEAR_CCA)) st.near_threshold++;
    st.digest += nsgpu_wifi_term(RX, now, k, j, (uint64_t)outcome | (uint64_t)(flags & 3u) << 8 | (uint64_t)cca << 16);
    if (rx_log) {
      nsgpu_wifi_rx_log &l = rx_log[(uint64_t)k * sc->n_phy + j];
      l.outcome = outcome;
      l.flags = flags;
      l.cca_ns = cca;
    }
  }

  // YansWifiPhy::EndReceive — yans-wifi-phy.cc:770-799 (the PER draw is the host's; its state part here)
  void end_receive(uint32_t e) {
    nsgpu_wifi_end_record &r = ends[e];
    r.flags |= NSGPU_WIFI_END_DISPATCHED;
    Phy &p = phy[r.phy];
    st.end++;
    p.c.end++;
    if (r.flags & NSGPU_WIFI_END_CANCELLED) {  // EventImpl::Invoke skips a cancelled event (event-impl.cc:40-46)
      st.end_cancelled++;
      p.c.end_cancelled++;
    } else {
      p.irxing = false;  // m_interference.NotifyRxEnd ()
      p.rxing = false;   // WifiPhyStateHelper::DoSwitchFromRx — wifi-phy-state-helper.cc:391-402
    }
    st.digest += nsgpu_wifi_term(END, now, r.uid, r.phy, (r.flags & NSGPU_WIFI_END_CANCELLED) ? 1 : 0);
  }
};

}  // namespace

extern "C" {

int64_t nsref_wifi_tx_duration(uint32_t size, uint32_t modclass, uint64_t rate_bps, uint32_t bw_hz, uint32_t preamble) {
  // WifiPhy::CalculateTxDuration — wifi-phy.cc:288-296; MicroSeconds (duration) at NS resolution
  uint32_t us = plcp_preamble_us(modclass, bw_hz, preamble) + plcp_header_us(modclass, bw_hz, preamble) +
                payload_us(size, modclass, rate_bps, bw_hz);
  return (int64_t)us * 1000;
}

int nsref_wifi_run(const nsgpu_wifi_scenario *sc, nsgpu_wifi_stats *stats, nsgpu_wifi_phy_counters *phys,
                   uint32_t *tx_base, nsgpu_wifi_end_record *ends, uint64_t ends_cap, uint64_t *n_ends,
                   nsgpu_wifi_rx_log *rx_log) {
  Run r;
  r.sc = sc;
  r.phy.resize((size_t)sc->n_phy);
  r.dur.resize((size_t)sc->n_tx);
  r.uid = sc->uid_start;
  r.edW = Run::DbmToW(sc->ed_threshold_dbm);    // SetEdThreshold (:228-232)
  r.ccaW = Run::DbmToW(sc->cca_threshold_dbm);  // SetCcaMode1Threshold (:234-238)
  r.rx_log = rx_log;
  r.tx_base = tx_base;
  if (rx_log)
    for (int64_t i = 0; i < sc->n_tx * sc->n_phy; i++) rx_log[i] = nsgpu_wifi_rx_log{0, 0, NSGPU_WIFI_NOT_RUN, 0, 0, 0};
  if (tx_base)
    for (int64_t k = 0; k < sc->n_tx; k++) tx_base[k] = 0;
  for (int64_t k = 0; k < sc->n_tx; k++) {
    r.dur[k] = nsref_wifi_tx_duration(sc->tx_size[k], sc->tx_modclass[k], sc->tx_rate_bps[k], sc->tx_bw_hz[k],
                                      sc->tx_preamble[k]);
    r.q.emplace(std::make_pair(sc->tx_ts[k], sc->tx_uid[k]), Ev{TX, (uint32_t)k, 0, 0.0});
  }
  if (sc->stop_ts != ~0ull) r.q.emplace(std::make_pair(sc->stop_ts, sc->stop_uid), Ev{STOP, 0, 0, 0.0});
  // DefaultSimulatorImpl::Run — default-simulator-impl.cc:147-160
  while (!r.q.empty()) {
    auto it = r.q.begin();
    const Ev e = it->second;
    r.now = it->first.first;
    const uint32_t euid = it->first.second;
    r.q.erase(it);
    r.st.dispatched++;
    if (e.kind == STOP) {
      r.st.digest += nsgpu_wifi_term(STOP, r.now, euid, 0, 0);
      break;
    }
    if (e.kind == TX) {
      if (r.send(e.a) != 0) return -1;
    } else if (e.kind == RX) {
      r.start_receive(e.a, e.b, e.rx_dbm);
    } else {
      r.end_receive(e.a);
    }
  }
  r.st.final_ts = r.now;
  r.st.next_uid = r.uid;
  for (const Phy &p : r.phy) r.st.ni_max = std::max(r.st.ni_max, p.c.ni_max);
  if (stats) *stats = r.st;
  if (phys)
    for (int64_t j = 0; j < sc->n_phy; j++) {
      const Phy &p = r.phy[j];
      nsgpu_wifi_phy_counters c = p.c;
      c.ni_len = (uint32_t)p.ni.size();
      c.end_tx = p.endTx;
      c.end_rx = p.endRx;
      c.end_cca_busy = p.endCca;
      c.first_power = p.firstPower;
      c.rxing = p.rxing ? 1 : 0;
      phys[j] = c;
    }
  if (n_ends) *n_ends = r.ends.size();
  if (ends) {
    if (r.ends.size() > ends_cap) return -2;
    for (size_t i = 0; i < r.ends.size(); i++) ends[i] = r.ends[i];
  }
  return 0;
}

}  // extern "C"
