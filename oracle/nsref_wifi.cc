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


// ---- WifiMode attributes: the CreateWifiMode calls of wifi-phy.cc:355-840; phyRate per wifi-mode.cc:140-155 ----
struct Mode {
  uint32_t mc;
  uint64_t data_rate;
  uint32_t bw, phy_rate, cons;
  int code;  // 0 undefined, 1: 1/2, 2: 2/3, 3: 3/4
};
Mode make_mode(uint32_t mc, uint64_t rate, uint32_t bw) {
  Mode m{mc, rate, mc == NSGPU_WIFI_DSSS ? 22000000u : bw, (uint32_t)rate, rate == 1000000 ? 2u : 4u, 0};
  if (mc == NSGPU_WIFI_DSSS) return m;
  // the OFDM rate ladder of a 20 MHz channel, scaled by the channel width (10 / 5 MHz: half / quarter rates)
  switch (rate * 20000000ull / m.bw) {
    case 6000000: m.cons = 2, m.code = 1; break;
    case 9000000: m.cons = 2, m.code = 3; break;
    case 12000000: m.cons = 4, m.code = 1; break;
    case 18000000: m.cons = 4, m.code = 3; break;
    case 24000000: m.cons = 16, m.code = 1; break;
    case 36000000: m.cons = 16, m.code = 3; break;
    case 48000000: m.cons = 64, m.code = 2; break;
    default: m.cons = 64, m.code = 3; break;  // 54
  }
  const uint32_t dr = (uint32_t)rate;
  m.phy_rate = m.code == 1 ? dr * 2 / 1 : m.code == 2 ? dr * 3 / 2 : dr * 4 / 3;
  return m;
}
// WifiPhy::GetPlcpHeaderMode — wifi-phy.cc:99-139
Mode header_mode(const Mode &p, uint32_t preamble) {
  if (p.mc == NSGPU_WIFI_OFDM)
    return p.bw == 5000000 ? make_mode(NSGPU_WIFI_OFDM, 1500000, 5000000)
           : p.bw == 10000000 ? make_mode(NSGPU_WIFI_OFDM, 3000000, 10000000)
                              : make_mode(NSGPU_WIFI_OFDM, 6000000, 20000000);
  if (p.mc == NSGPU_WIFI_ERP_OFDM) return make_mode(NSGPU_WIFI_ERP_OFDM, 6000000, 20000000);
  return make_mode(NSGPU_WIFI_DSSS, preamble == NSGPU_WIFI_PREAMBLE_LONG ? 1000000 : 2000000, 22000000);
}

// DsssErrorRateModel — dsss-error-rate-model.cc:29-127 (ENABLE_GSL unset: the Matlab fits for CCK)
double dsss_dqpsk_function(double x) {
  return ((sqrt(2.0) + 1.0) / sqrt(8.0 * 3.1415926 * sqrt(2.0))) * (1.0 / sqrt(x)) * exp(-(2.0 - sqrt(2.0)) * x);
}
double dsss_success(uint64_t rate, double sinr, uint32_t nbits) {
  switch (rate) {
    case 1000000: {
      double EbN0 = sinr * 22000000.0 / 1000000.0;
      double ber = 0.5 * exp(-EbN0);
      return pow((1.0 - ber), nbits);
    }
    case 2000000: {
      double EbN0 = sinr * 22000000.0 / 1000000.0 / 2.0;
      double ber = dsss_dqpsk_function(EbN0);
      return pow((1.0 - ber), nbits);
    }
    case 5500000: {
      double ber;
      if (sinr > 10.0) ber = 0.0;        // WLAN_SIR_PERFECT
      else if (sinr < 0.1) ber = 0.5;    // WLAN_SIR_IMPOSSIBLE
      else {
        double a1 = 5.3681634344056195e-001, a2 = 3.3092430025608586e-003, a3 = 4.1654372361004000e-001,
               a4 = 1.0288981434358866e+000;
        ber = a1 * exp(-(pow((sinr - a2) / a3, a4)));
      }
      return pow((1.0 - ber), nbits);
    }
    case 11000000: {
      double ber;
      if (sinr > 10.0) ber = 0.0;
      else if (sinr < 0.1) ber = 0.5;
      else {
        double a1 = 7.9056742265333456e-003, a2 = -1.8397449399176360e-001, a3 = 1.0740689468707241e+000,
               a4 = 1.0523316904502553e+000, a5 = 3.0552298746496687e-001, a6 = 2.2032715128698435e+000;
        ber = (a1 * sinr * sinr + a2 * sinr + a3) / (sinr * sinr * sinr + a4 * sinr * sinr + a5 * sinr + a6);
      }
      return pow((1.0 - ber), nbits);
    }
  }
  return 0;
}

// NistErrorRateModel — nist-error-rate-model.cc:38-270
double nist_pe(double p, uint32_t bValue) {  // CalculatePe
  double D = sqrt(4.0 * p * (1.0 - p));
  double pe = 1.0;
  if (bValue == 1) {
    pe = 0.5 * (36.0 * pow(D, 10.0) + 211.0 * pow(D, 12.0) + 1404.0 * pow(D, 14.0) + 11633.0 * pow(D, 16.0) +
                77433.0 * pow(D, 18.0) + 502690.0 * pow(D, 20.0) + 3322763.0 * pow(D, 22.0) +
                21292910.0 * pow(D, 24.0) + 134365911.0 * pow(D, 26.0));
  } else if (bValue == 2) {
    pe = 1.0 / (2.0 * bValue) *
         (3.0 * pow(D, 6.0) + 70.0 * pow(D, 7.0) + 285.0 * pow(D, 8.0) + 1276.0 * pow(D, 9.0) + 6160.0 * pow(D, 10.0) +
          27128.0 * pow(D, 11.0) + 117019.0 * pow(D, 12.0) + 498860.0 * pow(D, 13.0) + 2103891.0 * pow(D, 14.0) +
          8784123.0 * pow(D, 15.0));
  } else if (bValue == 3) {
    pe = 1.0 / (2.0 * bValue) *
         (42.0 * pow(D, 5.0) + 201.0 * pow(D, 6.0) + 1492.0 * pow(D, 7.0) + 10469.0 * pow(D, 8.0) +
          62935.0 * pow(D, 9.0) + 379644.0 * pow(D, 10.0) + 2253373.0 * pow(D, 11.0) + 13073811.0 * pow(D, 12.0) +
          75152755.0 * pow(D, 13.0) + 428005675.0 * pow(D, 14.0));
  }
  return pe;
}
double nist_fec(double ber, double nbits, uint32_t bValue) {  // GetFec*Ber after the modulation's ber
  if (ber == 0.0) return 1.0;
  double pe = nist_pe(ber, bValue);
  pe = std::min(pe, 1.0);
  return pow(1 - pe, nbits);
}
double nist_success(const Mode &m, double snr, uint32_t nbits) {  // GetChunkSuccessRate
  if (m.mc == NSGPU_WIFI_DSSS) return dsss_success(m.data_rate, snr, nbits);
  const uint32_t b = m.cons == 64 ? (m.code == 2 ? 2u : 3u) : (m.code == 1 ? 1u : 3u);
  double ber;
  switch (m.cons) {
    case 2: ber = 0.5 * erfc(sqrt(snr)); break;                              // GetBpskBer
    case 4: ber = 0.5 * erfc(sqrt(snr / 2.0)); break;                        // GetQpskBer
    case 16: ber = 0.75 * 0.5 * erfc(sqrt(snr / (5.0 * 2.0))); break;        // Get16QamBer
    default: ber = 7.0 / 12.0 * 0.5 * erfc(sqrt(snr / (21.0 * 2.0))); break; // Get64QamBer
  }
  // GetFecBpskBer / GetFecQpskBer take nbits as double, the QAM ones as uint32_t (same value)
  return nist_fec(ber, (double)nbits, b);
}

// YansErrorRateModel — yans-error-rate-model.cc:45-300
uint32_t yans_factorial(uint32_t k) {
  uint32_t fact = 1;
  while (k > 0) fact *= k--;
  return fact;
}
double yans_binomial(uint32_t k, double p, uint32_t n) {
  return yans_factorial(n) / (yans_factorial(k) * yans_factorial(n - k)) * pow(p, k) * pow(1 - p, n - k);
}
double yans_pd(double ber, uint32_t d) {
  double pd = 0;
  if ((d % 2) == 0) {
    for (uint32_t i = d / 2 + 1; i < d; i++) pd += yans_binomial(i, ber, d);
    pd += 0.5 * yans_binomial(d / 2, ber, d);
  } else {
    for (uint32_t i = (d + 1) / 2; i < d; i++) pd += yans_binomial(i, ber, d);
  }
  return pd;
}
double yans_success(const Mode &m, double snr, uint32_t nbits) {
  if (m.mc == NSGPU_WIFI_DSSS) return dsss_success(m.data_rate, snr, nbits);
  const double EbNo = snr * m.bw / m.phy_rate;
  uint32_t dFree, adFree, adFree1 = 0;
  double ber;
  if (m.cons == 2) {  // GetFecBpskBer
    ber = 0.5 * erfc(sqrt(EbNo));
    if (m.code == 1) dFree = 10, adFree = 11;
    else dFree = 5, adFree = 8;
    if (ber == 0.0) return 1.0;
    double pmu = adFree * yans_pd(ber, dFree);
    pmu = std::min(pmu, 1.0);
    return pow(1 - pmu, (double)nbits);
  }
  // GetQamBer + GetFecQamBer
  const unsigned int M = m.cons;
  double z = sqrt((1.5 * (log(M) / log(2.0)) * EbNo) / (M - 1.0));
  double z1 = ((1.0 - 1.0 / sqrt(M)) * erfc(z));
  double z2 = 1 - pow((1 - z1), 2.0);
  ber = z2 / (log(M) / log(2.0));
  if (M == 4) {
    if (m.code == 1) dFree = 10, adFree = 11, adFree1 = 0;
    else dFree = 5, adFree = 8, adFree1 = 31;
  } else if (M == 16) {
    if (m.code == 1) dFree = 10, adFree = 11, adFree1 = 0;
    else dFree = 5, adFree = 8, adFree1 = 31;
  } else {
    if (m.code == 2) dFree = 6, adFree = 1, adFree1 = 16;
    else dFree = 5, adFree = 8, adFree1 = 31;
  }
  if (ber == 0.0) return 1.0;
  double pmu = adFree * yans_pd(ber, dFree);
  pmu += adFree1 * yans_pd(ber, dFree + 1);
  pmu = std::min(pmu, 1.0);
  return pow(1 - pmu, nbits);
}

double chunk_success(uint32_t model, const Mode &m, double snr, uint32_t nbits) {
  return model == NSGPU_WIFIL_YANS ? yans_success(m, snr, nbits) : nist_success(m, snr, nbits);
}

// ---- the closed loop: host closures (the MAC stand-in) + the PHY events, one (ts, uid) order ----
struct LoopTx {
  uint64_t ts;
  int64_t dur;
  uint32_t phy;
  Mode mode;
  uint32_t preamble;
  uint32_t uid;  // the SendPacket's closure (its sniffer record's place in the dispatch order)
};
struct LoopEnd {  // an EndReceive's event data
  uint32_t phy, tx, cancelled;
  uint64_t start;
  double w;
};
struct Loop {
  const nsgpu_wifil_config *cfg;
  const nsref_wifil_mac *mac;
  std::vector<Phy> phy;
  std::vector<LoopTx> txs;
  std::vector<LoopEnd> endv;
  enum { ATTEMPT = 0, RX = 1, END = 2, STOP = 3, SEND = 4, MOVE = 5, REPLY = 6 };
  // current positions (MobilityModel::SetPosition from a host closure moves a phy; YansWifiChannel::Send reads
  // them at each send, yans-wifi-channel.cc:92-96)
  std::vector<double> px, py, pz;
  void init_positions() {
    px.assign(cfg->x, cfg->x + cfg->n_phy);
    py.assign(cfg->y, cfg->y + cfg->n_phy);
    pz.assign(cfg->z, cfg->z + cfg->n_phy);
  }
  struct E {
    uint32_t kind, a, b, ctx;
    double rx_dbm;
  };
  std::map<std::pair<uint64_t, uint32_t>, E> q;
  uint32_t uid = 4, ctx = 0xffffffffu, cur_uid = 0;
  uint64_t now = 0, dispatched = 0, digest = 0, sends = 0, busy = 0;
  double edW, ccaW, noiseFigure;
  std::vector<nsgpu_wifil_end> ends;

  static double DbmToW(double dBm) { return pow(10.0, dBm / 10.0) / 1000.0; }
  int state(const Phy &p) const {
    if (p.endTx > (int64_t)now) return NSGPU_WIFIL_TX;
    if (p.rxing) return NSGPU_WIFIL_RX;
    if (p.endCca > (int64_t)now) return NSGPU_WIFIL_CCA_BUSY;
    return NSGPU_WIFIL_IDLE;
  }
  int64_t delay_until_idle(const Phy &p) const {
    int64_t r = 0;
    switch (state(p)) {
      case NSGPU_WIFIL_RX: r = p.endRx - (int64_t)now; break;
      case NSGPU_WIFIL_TX: r = p.endTx - (int64_t)now; break;
      case NSGPU_WIFIL_CCA_BUSY: r = p.endCca - (int64_t)now; break;
    }
    return std::max<int64_t>(r, 0);
  }
  void schedule(uint64_t ts, E e) { q.emplace(std::make_pair(ts, uid++), e); }
  void add_ni(Phy &p, NiChange c) {
    auto it = std::upper_bound(p.ni.begin(), p.ni.end(), c, [](const NiChange &a, const NiChange &b) { return a.t < b.t; });
    p.ni.insert(it, c);
  }
  void append_event(Phy &p, int64_t start, int64_t end, double w) {  // interference-helper.cc:192-212
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
    p.c.ni_max = std::max<uint32_t>(p.c.ni_max, (uint32_t)p.ni.size());
  }
  int64_t energy_duration(const Phy &p, double energyW) const {  // :171-190
    double noiseInterferenceW = p.firstPower;
    int64_t end = (int64_t)now;
    for (const NiChange &i : p.ni) {
      noiseInterferenceW += i.d;
      end = i.t;
      if (end < (int64_t)now) continue;
      if (noiseInterferenceW < energyW) break;
    }
    return end > (int64_t)now ? end - (int64_t)now : 0;
  }
  // CalculateSnr — interference-helper.cc:215-227
  double snr_of(double signal, double noiseInterference, const Mode &m) const {
    static const double BOLTZMANN = 1.3803e-23;
    double Nt = BOLTZMANN * 290.0 * m.bw;
    double noiseFloor = noiseFigure * Nt;
    double noise = noiseFloor + noiseInterference;
    return signal / noise;
  }
  // CalculateChunkSuccessRate — :244-255
  double chunk(double snir, int64_t duration, const Mode &m) const {
    if (duration == 0) return 1.0;
    uint32_t rate = m.phy_rate;
    uint64_t nbits = (uint64_t)(rate * nsref_get_seconds(duration));
    return chunk_success(cfg->error_model, m, snir, (uint32_t)nbits);
  }
  // CalculateSnrPer — :336-353 (CalculateNoiseInterferenceW :229-243, CalculatePer :257-334)
  void snr_per(const Phy &p, const LoopEnd &e, int64_t endTime, double &snr, double &per) const {
    const LoopTx &t = txs[e.tx];
    std::vector<NiChange> ni;
    double noiseInterference = p.firstPower;
    for (size_t i = 1; i < p.ni.size(); i++) {
      if (endTime == p.ni[i].t && e.w == -p.ni[i].d) break;
      ni.push_back(p.ni[i]);
    }
    ni.insert(ni.begin(), NiChange{(int64_t)e.start, noiseInterference});
    ni.push_back(NiChange{endTime, 0});
    snr = snr_of(e.w, noiseInterference, t.mode);
    double psr = 1.0;
    size_t j = 0;
    int64_t previous = ni[j].t;
    const Mode payloadMode = t.mode, headerMode = header_mode(t.mode, t.preamble);
    int64_t plcpHeaderStart = ni[j].t + (int64_t)plcp_preamble_us(t.mode.mc, t.mode.bw, t.preamble) * 1000;
    int64_t plcpPayloadStart = plcpHeaderStart + (int64_t)plcp_header_us(t.mode.mc, t.mode.bw, t.preamble) * 1000;
    double noiseInterferenceW = ni[j].d;
    double powerW = e.w;
    j++;
    while (j < ni.size()) {
      int64_t current = ni[j].t;
      if (previous >= plcpPayloadStart) {
        psr *= chunk(snr_of(powerW, noiseInterferenceW, payloadMode), current - previous, payloadMode);
      } else if (previous >= plcpHeaderStart) {
        if (current >= plcpPayloadStart) {
          psr *= chunk(snr_of(powerW, noiseInterferenceW, headerMode), plcpPayloadStart - previous, headerMode);
          psr *= chunk(snr_of(powerW, noiseInterferenceW, payloadMode), current - plcpPayloadStart, payloadMode);
        } else {
          psr *= chunk(snr_of(powerW, noiseInterferenceW, headerMode), current - previous, headerMode);
        }
      } else {
        if (current >= plcpPayloadStart) {
          psr *= chunk(snr_of(powerW, noiseInterferenceW, headerMode), plcpPayloadStart - plcpHeaderStart, headerMode);
          psr *= chunk(snr_of(powerW, noiseInterferenceW, payloadMode), current - plcpPayloadStart, payloadMode);
        } else if (current >= plcpHeaderStart) {
          psr *= chunk(snr_of(powerW, noiseInterferenceW, headerMode), current - plcpHeaderStart, headerMode);
        }
      }
      noiseInterferenceW += ni[j].d;
      previous = ni[j].t;
      j++;
    }
    per = 1 - psr;
  }

  // the MAC stand-in's attempt (see nsref.h); reply: the hand-back's reply (no retry, nothing rescheduled)
  int attempt(uint32_t i, bool reply = false) {
    Phy &p = phy[i];
    if (state(p) != NSGPU_WIFIL_IDLE) {
      busy++;
      if (!reply) schedule(now + mac->backoff[i], E{ATTEMPT, i, 0, ctx, 0.0});
      return 0;
    }
    // YansWifiPhy::SendPacket — yans-wifi-phy.cc:499-522 (IDLE: no reception to cancel)
    LoopTx t;
    t.ts = now;
    t.phy = i;
    t.mode = make_mode(mac->modclass, mac->rate, mac->bw);
    t.preamble = mac->preamble;
    t.uid = cur_uid;
    t.dur = nsref_wifi_tx_duration(mac->size, mac->modclass, mac->rate, mac->bw, mac->preamble);
    const uint32_t k = (uint32_t)txs.size();
    txs.push_back(t);
    p.endTx = (int64_t)now + t.dur;  // SwitchToTx (wifi-phy-state-helper.cc:254-290)
    sends++;
    // YansWifiChannel::Send — yans-wifi-channel.cc:77-115
    for (int64_t j = 0; j < cfg->n_phy; j++) {
      if (j == (int64_t)i || cfg->channel[j] != cfg->channel[i]) continue;
      double d = nsref_distance(px[i], py[i], pz[i], px[j], py[j], pz[j]);
      int64_t delay = nsref_const_speed_delay(d, cfg->speed);
      double rx = nsref_calc_rx_power(mac->dbm, d, &cfg->loss);
      schedule(now + (uint64_t)delay, E{RX, k, (uint32_t)j, cfg->node[j], rx});
    }
    if (!reply) schedule(now + mac->period, E{ATTEMPT, i, 0, ctx, 0.0});
    return 0;
  }
  // YansWifiPhy::SendPacket from a host closure whatever the state (a replayed transmission schedule):
  // yans-wifi-phy.cc:499-522 — a reception in progress is abandoned (m_endRxEvent.Cancel, NotifyRxEnd;
  // SwitchToTx's RX case, wifi-phy-state-helper.cc:263-268), then the channel's fan-out
  int send_packet(uint32_t i, uint32_t size, uint32_t modclass, uint64_t rate, uint32_t bw, uint32_t preamble,
                  double dbm) {
    Phy &p = phy[i];
    if (p.endTx > (int64_t)now) return -3;  // NS_ASSERT (!IsStateTx ())
    if (p.rxing) {
      endv[(size_t)p.endRxEvent].cancelled = 1;
      p.rxing = false;
      p.irxing = false;
      p.endRx = (int64_t)now;
    }
    LoopTx t;
    t.ts = now;
    t.phy = i;
    t.mode = make_mode(modclass, rate, bw);
    t.preamble = preamble;
    t.uid = cur_uid;
    t.dur = nsref_wifi_tx_duration(size, modclass, rate, bw, preamble);
    const uint32_t k = (uint32_t)txs.size();
    txs.push_back(t);
    p.endTx = (int64_t)now + t.dur;
    sends++;
    for (int64_t j = 0; j < cfg->n_phy; j++) {  // YansWifiChannel::Send — yans-wifi-channel.cc:77-115
      if (j == (int64_t)i || cfg->channel[j] != cfg->channel[i]) continue;
      double d = nsref_distance(px[i], py[i], pz[i], px[j], py[j], pz[j]);
      int64_t delay = nsref_const_speed_delay(d, cfg->speed);
      double rx = nsref_calc_rx_power(dbm, d, &cfg->loss);
      schedule(now + (uint64_t)delay, E{RX, k, (uint32_t)j, cfg->node[j], rx});
    }
    return 0;
  }
  // YansWifiPhy::StartReceivePacket — yans-wifi-phy.cc:399-496
  void start_receive(uint32_t k, uint32_t j, double rxPowerDbm) {
    Phy &p = phy[j];
    rxPowerDbm += cfg->rx_gain_db;
    double rxPowerW = DbmToW(rxPowerDbm);
    int64_t rxDuration = txs[k].dur;
    int64_t endRx = (int64_t)now + rxDuration;
    append_event(p, (int64_t)now, endRx, rxPowerW);
    bool maybeCca = false;
    p.c.rx++;
    switch (state(p)) {
      case NSGPU_WIFIL_RX:
        p.c.drop_rx++;
        maybeCca = endRx > (int64_t)now + delay_until_idle(p);
        break;
      case NSGPU_WIFIL_TX:
        p.c.drop_tx++;
        maybeCca = endRx > (int64_t)now + delay_until_idle(p);
        break;
      default:
        if (rxPowerW > edW) {
          p.c.sync++;
          p.rxing = true;
          p.endRx = (int64_t)now + rxDuration;
          p.irxing = true;
          p.endRxEvent = (int64_t)endv.size();
          endv.push_back(LoopEnd{j, k, 0, now, rxPowerW});
          schedule((uint64_t)endRx, E{END, (uint32_t)p.endRxEvent, 0, ctx, 0.0});
        } else {
          p.c.drop_ed++;
          maybeCca = true;
        }
    }
    if (maybeCca) {
      int64_t cca = energy_duration(p, ccaW);
      if (cca != 0) {
        p.c.cca_switches++;
        p.endCca = std::max<int64_t>(p.endCca, (int64_t)now + cca);
      }
    }
  }
  // YansWifiPhy::EndReceive — yans-wifi-phy.cc:770-799 (the m_random draw is the caller's)
  void end_receive(uint32_t e, uint32_t euid) {
    LoopEnd &r = endv[e];
    Phy &p = phy[r.phy];
    p.c.end++;
    nsgpu_wifil_end out{now, euid, r.phy, 0.0, 0.0, r.tx, 0u, r.cancelled ? 0.0 : r.w};
    if (r.cancelled) {
      p.c.end_cancelled++;
      out.flags = NSGPU_WIFI_END_CANCELLED;
    } else {
      snr_per(p, r, (int64_t)now, out.snr, out.per);
      p.irxing = false;
      p.rxing = false;
    }
    ends.push_back(out);
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


// A replayed transmission schedule: host closures scheduled at setup in send order (Schedule (ts_k, SendPacket
// of phy_k)), then Simulator::Stop (Time); the same PHY and run loop as nsref_wifil_run.
int nsref_wifil_replay(const nsgpu_wifil_config *cfg, const nsref_wifil_sends *sn, uint64_t *log_ts, uint32_t *log_uid,
                       uint32_t *log_ctx, uint64_t log_cap, nsgpu_wifil_end *ends, uint64_t ends_cap, uint64_t *n_ends,
                       nsgpu_wifi_phy_counters *phys, uint64_t out[6], uint64_t *tx_out, uint64_t tx_cap) {
  Loop L;
  L.cfg = cfg;
  L.mac = nullptr;
  L.phy.resize((size_t)cfg->n_phy);
  L.init_positions();
  L.edW = Loop::DbmToW(cfg->ed_threshold_dbm);
  L.ccaW = Loop::DbmToW(cfg->cca_threshold_dbm);
  L.noiseFigure = pow(10.0, cfg->rx_noise_figure_db / 10.0);
  for (uint64_t k = 0; k < sn->n; k++) {
    if (sn->phy[k] >= (uint64_t)cfg->n_phy) return -4;
    L.schedule(sn->ts[k], Loop::E{Loop::SEND, (uint32_t)k, 0, 0xffffffffu, 0.0});
  }
  for (uint64_t k = 0; k < sn->n_moves; k++) {  // Simulator::Schedule (t, &MobilityModel::SetPosition, ...)
    if (sn->move_phy[k] >= (uint64_t)cfg->n_phy) return -4;
    L.schedule(sn->move_ts[k], Loop::E{Loop::MOVE, (uint32_t)k, 0, 0xffffffffu, 0.0});
  }
  L.schedule(sn->stop_ts, Loop::E{Loop::STOP, 0, 0, 0xffffffffu, 0.0});
  while (!L.q.empty()) {
    auto it = L.q.begin();
    const Loop::E e = it->second;
    L.now = it->first.first;
    const uint32_t euid = it->first.second;
    L.q.erase(it);
    L.ctx = e.ctx;
    L.cur_uid = euid;
    const uint64_t rank = L.dispatched++;
    L.digest += nsgpu_dispatch_digest_term(rank, L.now, euid);
    if (rank < log_cap) {
      log_ts[rank] = L.now;
      log_uid[rank] = euid;
      log_ctx[rank] = e.ctx;
    }
    if (e.kind == Loop::STOP) break;
    if (e.kind == Loop::SEND) {
      const int rc = L.send_packet(sn->phy[e.a], sn->size[e.a], sn->modclass, sn->rate, sn->bw, sn->preamble, sn->dbm);
      if (rc) return rc;
    } else if (e.kind == Loop::MOVE) {
      const uint32_t j = sn->move_phy[e.a];
      L.px[j] = sn->move_xyz[3 * e.a], L.py[j] = sn->move_xyz[3 * e.a + 1], L.pz[j] = sn->move_xyz[3 * e.a + 2];
    } else if (e.kind == Loop::RX) {
      L.start_receive(e.a, e.b, e.rx_dbm);
    } else if (e.kind == Loop::END) {
      L.end_receive(e.a, euid);
    }
  }
  out[0] = L.dispatched;
  out[1] = L.digest;
  out[2] = L.uid;
  out[3] = L.now;
  out[4] = L.sends;
  out[5] = L.busy;
  if (tx_out)  // the SendPacket calls: (ts, closure uid, phy), in call order (= transmission index)
    for (size_t k = 0; k < L.txs.size() && k < tx_cap; k++) {
      tx_out[3 * k] = L.txs[k].ts;
      tx_out[3 * k + 1] = L.txs[k].uid;
      tx_out[3 * k + 2] = L.txs[k].phy;
    }
  if (n_ends) *n_ends = L.ends.size();
  if (ends) {
    if (L.ends.size() > ends_cap) return -2;
    for (size_t i = 0; i < L.ends.size(); i++) ends[i] = L.ends[i];
  }
  if (phys)
    for (int64_t j = 0; j < cfg->n_phy; j++) phys[j] = L.phy[(size_t)j].c;
  return 0;
}

double nsref_wifil_chunk_success(uint32_t model, uint32_t modclass, uint64_t rate, uint32_t bw, double snr, uint32_t nbits) {
  return chunk_success(model, make_mode(modclass, rate, bw), snr, nbits);
}

int nsref_wifil_run(const nsgpu_wifil_config *cfg, const nsref_wifil_mac *mac, uint64_t *log_ts, uint32_t *log_uid,
                    uint32_t *log_ctx, uint64_t log_cap, nsgpu_wifil_end *ends, uint64_t ends_cap, uint64_t *n_ends,
                    nsgpu_wifi_phy_counters *phys, uint64_t out[6], uint64_t *tx_out, uint64_t tx_cap) {
  Loop L;
  L.cfg = cfg;
  L.mac = mac;
  L.phy.resize((size_t)cfg->n_phy);
  L.init_positions();
  L.edW = Loop::DbmToW(cfg->ed_threshold_dbm);
  L.ccaW = Loop::DbmToW(cfg->cca_threshold_dbm);
  L.noiseFigure = pow(10.0, cfg->rx_noise_figure_db / 10.0);  // DbToRatio (SetRxNoiseFigure, yans-wifi-phy.cc:192-197)
  if (mac->uid_first) L.uid = mac->uid_first;  // (a uint32: it wraps after 0xffffffff as the reference's m_uid does)
  // setup: the attempts in phy order, then Stop (Time)
  for (int64_t i = 0; i < cfg->n_phy; i++) L.schedule(mac->first[i], Loop::E{Loop::ATTEMPT, (uint32_t)i, 0, 0xffffffffu, 0.0});
  L.schedule(mac->stop_ts, Loop::E{Loop::STOP, 0, 0, 0xffffffffu, 0.0});
  while (!L.q.empty()) {  // DefaultSimulatorImpl::Run / ProcessOneEvent (default-simulator-impl.cc:117-160)
    auto it = L.q.begin();
    const Loop::E e = it->second;
    L.now = it->first.first;
    const uint32_t euid = it->first.second;
    L.q.erase(it);
    L.ctx = e.ctx;
    L.cur_uid = euid;
    const uint64_t rank = L.dispatched++;
    L.digest += nsgpu_dispatch_digest_term(rank, L.now, euid);
    if (rank < log_cap) {
      log_ts[rank] = L.now;
      log_uid[rank] = euid;
      log_ctx[rank] = e.ctx;
    }
    if (e.kind == Loop::STOP) break;
    if (e.kind == Loop::ATTEMPT) L.attempt(e.a);
    else if (e.kind == Loop::REPLY) L.attempt(e.a, true);
    else if (e.kind == Loop::RX) L.start_receive(e.a, e.b, e.rx_dbm);
    else {
      L.end_receive(e.a, euid);
      const nsgpu_wifil_end &r = L.ends.back();  // the hand-back: the host's draw, then the MAC's callback
      if (mac->reply_on && !(r.flags & NSGPU_WIFI_END_CANCELLED) && 0.5 > r.per)
        L.schedule(L.now + mac->reply_delay, Loop::E{Loop::REPLY, r.phy, 0, L.ctx, 0.0});
    }
  }
  out[0] = L.dispatched;
  out[1] = L.digest;
  out[2] = L.uid;
  out[3] = L.now;
  out[4] = L.sends;
  out[5] = L.busy;
  if (tx_out)  // the SendPacket calls: (ts, closure uid, phy), in call order (= transmission index)
    for (size_t k = 0; k < L.txs.size() && k < tx_cap; k++) {
      tx_out[3 * k] = L.txs[k].ts;
      tx_out[3 * k + 1] = L.txs[k].uid;
      tx_out[3 * k + 2] = L.txs[k].phy;
    }
  if (n_ends) *n_ends = L.ends.size();
  if (ends) {
    if (L.ends.size() > ends_cap) return -2;
    for (size_t i = 0; i < L.ends.size(); i++) ends[i] = L.ends[i];
  }
  if (phys)
    for (int64_t j = 0; j < cfg->n_phy; j++) {
      const Phy &p = L.phy[j];
      nsgpu_wifi_phy_counters c = p.c;
      c.ni_len = (uint32_t)p.ni.size();
      c.end_tx = p.endTx;
      c.end_rx = p.endRx;
      c.end_cca_busy = p.endCca;
      c.first_power = p.firstPower;
      c.rxing = p.rxing ? 1 : 0;
      phys[j] = c;
    }
  return 0;
}

}  // extern "C"
