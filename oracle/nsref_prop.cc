// nsref_prop.cc — CPU ORACLE (test infrastructure only; see nsref.h header).
// Restatement of mobility distance, the propagation loss/delay models and the broadcast
// channel fan-out loops.  Built with -ffp-contract=off so that
// dx*dx+dy*dy+dz*dz rounds exactly like the reference's default -O2 x86-64 build.
#include "nsref.h"
#include <algorithm>
#include <vector>
#include <math.h>

static const double PI = 3.14159265358979323846;  // propagation-loss-model.cc:34

extern "C" {

// CalculateDistance (const Vector3D &a, const Vector3D &b) — src/core/model/vector.cc:63-70
double nsref_distance(double ax, double ay, double az, double bx, double by, double bz) {
  double dx = bx - ax;
  double dy = by - ay;
  double dz = bz - az;
  double distance = sqrt(dx * dx + dy * dy + dz * dz);
  return distance;
}

// One link's DoCalcRxPower.
static double do_calc_rx(const nsgpu_loss_model *m, double tx, double distance) {
  switch (m->kind) {
    case NSGPU_LOSS_LOG_DISTANCE: {  // propagation-loss-model.cc:464-491
      double exponent = m->p0, refd = m->p1, refloss = m->p2;
      if (distance <= refd) return tx;
      double pathLossDb = 10 * exponent * log10(distance / refd);
      double rxc = -refloss - pathLossDb;
      return tx + rxc;
    }
    case NSGPU_LOSS_FRIIS: {  // propagation-loss-model.cc:197-239
      double lambda = m->p0, sysloss = m->p1, mind = m->p2;
      if (distance <= mind) return tx;
      double numerator = lambda * lambda;
      double denominator = 16 * PI * PI * distance * distance * sysloss;
      double pr = 10 * log10(numerator / denominator);
      return tx + pr;
    }
    case NSGPU_LOSS_FIXED_RSS:  // propagation-loss-model.cc:718-723
      return m->p0;
    case NSGPU_LOSS_RANGE:  // propagation-loss-model.cc:822-834
      return distance <= m->p0 ? tx : -1000;
    default:
      return tx;
  }
}

// PropagationLossModel::CalcRxPower — propagation-loss-model.cc:64-74 (m_next chain).
double nsref_calc_rx_power(double tx_dbm, double distance, const nsgpu_loss_chain *chain) {
  double self = tx_dbm;
  for (int i = 0; i < chain->n; i++) self = do_calc_rx(&chain->m[i], self, distance);
  return self;
}

// ConstantSpeedPropagationDelayModel::GetDelay — propagation-delay-model.cc:90-96
int64_t nsref_const_speed_delay(double distance, double speed) {
  double seconds = distance / speed;
  return nsref_seconds(seconds);
}

// YansWifiChannel::Send — yans-wifi-channel.cc:77-115.
// senderMobility = a, receiverMobility = b; GetDistanceFrom (a, b) = CalculateDistance (a.pos, b.pos).
int64_t nsref_fanout_yans(const double *x, const double *y, const double *z,
                          const uint32_t *chan, const uint32_t *node, int64_t nphy,
                          int64_t sender, double tx_dbm, const nsgpu_loss_chain *loss, double speed,
                          uint64_t now_ts, uint32_t uid_base, nsgpu_rx_record *out) {
  int64_t k = 0;
  for (int64_t j = 0; j < nphy; j++) {
    if (j == sender) continue;
    if (chan[j] != chan[sender]) continue;
    double d = nsref_distance(x[sender], y[sender], z[sender], x[j], y[j], z[j]);
    int64_t delay = nsref_const_speed_delay(d, speed);
    double rx = nsref_calc_rx_power(tx_dbm, d, loss);
    nsgpu_rx_record r;
    r.ts = now_ts + (uint64_t)delay;  // DefaultSimulatorImpl::ScheduleWithContext: m_currentTs + GetTimeStep
    r.uid = uid_base + (uint32_t)k;
    r.context = node[j];
    r.phy = (uint32_t)j;
    r.pad_ = 0;
    r.rx_dbm = rx;
    out[k++] = r;
  }
  return k;
}

// SingleModelSpectrumChannel::StartTx — single-model-spectrum-channel.cc:106-183
int64_t nsref_fanout_spectrum(const double *x, const double *y, const double *z,
                              const uint32_t *node, int64_t nphy, int64_t sender,
                              const nsgpu_loss_chain *loss, double speed, double max_loss_db,
                              const double *psd_tx, int32_t nbands,
                              uint64_t now_ts, uint32_t uid_base,
                              nsgpu_rx_record *out, double *psd_out) {
  int64_t k = 0;
  for (int64_t j = 0; j < nphy; j++) {
    if (j == sender) continue;
    double d = nsref_distance(x[sender], y[sender], z[sender], x[j], y[j], z[j]);
    double gainDb = nsref_calc_rx_power(0, d, loss);
    if ((-gainDb) > max_loss_db) continue;  // beyond range: no uid consumed
    double gainLinear = pow(10.0, gainDb / 10.0);
    for (int32_t b = 0; b < nbands; b++) psd_out[k * nbands + b] = psd_tx[b] * gainLinear;  // SpectrumValue *=
    int64_t delay = speed > 0 ? nsref_const_speed_delay(d, speed) : 0;  // MicroSeconds (0) when no delay model
    nsgpu_rx_record r;
    r.ts = now_ts + (uint64_t)delay;
    r.uid = uid_base + (uint32_t)k;
    r.context = node[j];
    r.phy = (uint32_t)j;
    r.pad_ = 0;
    r.rx_dbm = gainDb;
    out[k++] = r;
  }
  return k;
}

// SpectrumConverter (spectrum-converter.cc): coefficient of input band `from` in output band `to`
static double converter_coeff(double ffl, double ffh, double tfl, double tfh) {  // GetCoefficient
  double coeff = std::min(ffh, tfh) - std::max(ffl, tfl);
  coeff = std::max(0.0, coeff);
  coeff = std::min(1.0, coeff / (tfh - tfl));
  return coeff;
}

// MultiModelSpectrumChannel::StartTx — multi-model-spectrum-channel.cc:226-331
int64_t nsref_fanout_spectrum_multi(const double *x, const double *y, const double *z, const uint32_t *node,
                                    const int32_t *rx_model, int64_t nphy, int64_t sender,
                                    int32_t n_models, const uint32_t *band_off, const double *fl, const double *fh,
                                    int32_t tx_model, const double *psd_tx,
                                    const nsgpu_loss_chain *loss, double speed, double max_loss_db,
                                    uint64_t now_ts, uint32_t uid_base,
                                    nsgpu_rx_record *out, double *psd_out, int32_t psd_stride,
                                    nsgpu_loss_trace *trace, int64_t *n_trace) {
  int64_t k = 0, nt = 0;
  std::vector<double> conv;
  const uint32_t t0 = band_off[tx_model], ntb = band_off[tx_model + 1] - t0;
  for (int32_t m = 0; m < n_models; m++) {  // for each rx SpectrumModel (:246-329)
    const uint32_t r0 = band_off[m], nrb = band_off[m + 1] - r0;
    bool any = false;
    for (int64_t j = 0; j < nphy && !any; j++) any = rx_model[j] == m;
    if (!any) continue;  // (only models some phy was added with are in the map)
    conv.assign(nrb, 0.0);
    if (m == tx_model) {  // no spectrum conversion needed (:254-258)
      for (uint32_t b = 0; b < nrb; b++) conv[b] = psd_tx[b];
    } else {  // SpectrumConverter::Convert: sum over input bands in order
      for (uint32_t b = 0; b < nrb; b++) {
        double sum = 0;
        for (uint32_t f = 0; f < ntb; f++)
          sum += psd_tx[f] * converter_coeff(fl[t0 + f], fh[t0 + f], fl[r0 + b], fh[r0 + b]);
        conv[b] = sum;
      }
    }
    for (int64_t j = 0; j < nphy; j++) {  // m_rxPhyList: AddRx order
      if (rx_model[j] != m || j == sender) continue;
      double d = nsref_distance(x[sender], y[sender], z[sender], x[j], y[j], z[j]);
      double gainDb = nsref_calc_rx_power(0, d, loss);
      if (trace) trace[nt] = nsgpu_loss_trace{(uint32_t)j, 0u, -gainDb};
      nt++;
      if ((-gainDb) > max_loss_db) continue;  // beyond range
      double gainLinear = pow(10.0, gainDb / 10.0);
      for (uint32_t b = 0; b < nrb; b++) psd_out[k * psd_stride + b] = conv[b] * gainLinear;
      int64_t delay = speed > 0 ? nsref_const_speed_delay(d, speed) : 0;
      nsgpu_rx_record r;
      r.ts = now_ts + (uint64_t)delay;
      r.uid = uid_base + (uint32_t)k;
      r.context = node[j];
      r.phy = (uint32_t)j;
      r.pad_ = 0;
      r.rx_dbm = gainDb;
      out[k++] = r;
    }
  }
  if (n_trace) *n_trace = nt;
  return k;
}

}  // extern "C"
