// nsgpu_fanout.hip — broadcast-channel fan-out kernels and the Seconds() conversion kernel.
//
// Yans (YansWifiChannel::Send, yans-wifi-channel.cc:77-115) and single-model spectrum
// (SingleModelSpectrumChannel::StartTx, single-model-spectrum-channel.cc:106-183) evaluate,
// for every other phy of the channel: distance (vector.cc:63-70), the loss chain
// (propagation-loss-model.cc:64-74) and the constant-speed delay (propagation-delay-model.cc:90-96),
// then ScheduleWithContext one event per surviving receiver, in phy-list order.  On the device
// each receiver is one lane; survivors are compacted with a two-pass block scan so that
// record k gets uid_base + k, the uid the reference's k-th ScheduleWithContext would take.
//
// Roofline (HBM): per receiver 32 B read (x, y, z, channel/node) + 32 B record written = 64 B
// (SURVEY §8(d)); spectrum adds 8 * nbands B of PSD written.  A batch of transmissions per
// launch (grid.y = n_tx) keeps the launch bandwidth-bound rather than launch-bound.
#include "nsgpu_device.h"
#include "nsgpu_internal.h"

namespace nsgpu {

constexpr int FAN_THREADS = 256;

enum FanKind { FAN_YANS = 0, FAN_SPECTRUM = 1 };

struct FanArgs {
  nsgpu_phy_soa phys;
  int64_t nphy;
  const nsgpu_tx_desc *tx;
  nsgpu_loss_chain loss;
  double speed;
  double max_loss_db;
  const double *psd_tx;
  int32_t nbands;
  nsgpu_rx_record *out;
  double *psd_out;
  uint32_t *count;
  uint32_t *block_counts;  // [n_tx][nblocks]
  int32_t nblocks;
};

// Survivor predicate and (for survivors) the per-receiver quantities.
template <int KIND>
__device__ __forceinline__ bool fan_eval(const FanArgs &a, const nsgpu_tx_desc &t, int64_t j, double &dist,
                                         double &rx) {
  if (j >= a.nphy || j == (int64_t)t.sender || (int64_t)t.sender >= a.nphy) return false;
  const double sx = a.phys.x[t.sender], sy = a.phys.y[t.sender], sz = a.phys.z[t.sender];
  if (KIND == FAN_YANS) {
    if (a.phys.channel[j] != a.phys.channel[t.sender]) return false;  // :88-91
    dist = distance3(sx, sy, sz, a.phys.x[j], a.phys.y[j], a.phys.z[j]);
    rx = calc_rx_power(a.loss, t.tx_dbm, dist);
    return true;
  } else {
    dist = distance3(sx, sy, sz, a.phys.x[j], a.phys.y[j], a.phys.z[j]);
    rx = calc_rx_power(a.loss, 0.0, dist);  // gainDb (:146)
    return !((-rx) > a.max_loss_db);        // :148-152 beyond range: skipped before Schedule
  }
}

// Pass 1: survivors per block.
template <int KIND>
__global__ __launch_bounds__(FAN_THREADS) void fan_count(FanArgs a) {
  const int64_t t = blockIdx.y;
  const nsgpu_tx_desc tx = a.tx[t];
  const int64_t j = (int64_t)blockIdx.x * FAN_THREADS + threadIdx.x;
  bool s;
  if (KIND == FAN_YANS) {  // every same-channel phy but the sender receives: no loss evaluation needed
    s = j < a.nphy && j != (int64_t)tx.sender && (int64_t)tx.sender < a.nphy &&
        a.phys.channel[j] == a.phys.channel[tx.sender];
  } else {
    double d, rx;
    s = fan_eval<KIND>(a, tx, j, d, rx);
  }
  const unsigned long long b = __ballot(s);
  __shared__ uint32_t wc[FAN_THREADS / 64];
  if ((threadIdx.x & 63) == 0) wc[threadIdx.x >> 6] = (uint32_t)__popcll(b);
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t c = 0;
    for (int w = 0; w < FAN_THREADS / 64; w++) c += wc[w];
    a.block_counts[t * a.nblocks + blockIdx.x] = c;
  }
}

// Pass 2: block offset from the preceding blocks' counts, local rank, write records.
// Yans with a channel-rank table (nsgpu_phy_soa.chan_rank): receiver j of transmission t is record
// chan_rank[j] - (j > sender) — the ScheduleWithContext order of the receiver loop — so one pass.
__global__ __launch_bounds__(FAN_THREADS) void fan_write_ranked(FanArgs a) {
  const int64_t t = blockIdx.y;
  const nsgpu_tx_desc tx = a.tx[t];
  const int64_t j = (int64_t)blockIdx.x * FAN_THREADS + threadIdx.x;
  if ((int64_t)tx.sender >= a.nphy) {  // not a phy of this channel: no receivers
    if (j == 0) a.count[t] = 0;
    return;
  }
  if (j >= a.nphy) return;
  if (j == (int64_t)tx.sender) {
    a.count[t] = a.phys.chan_count[j] - 1;
    return;
  }
  if (a.phys.channel[j] != a.phys.channel[tx.sender]) return;  // :88-91
  const double dist = distance3(a.phys.x[tx.sender], a.phys.y[tx.sender], a.phys.z[tx.sender], a.phys.x[j],
                                a.phys.y[j], a.phys.z[j]);
  const double rx = calc_rx_power(a.loss, tx.tx_dbm, dist);
  const uint32_t off = a.phys.chan_rank[j] - (j > (int64_t)tx.sender ? 1u : 0u);
  // the 32-B record as two 16-B non-temporal stores: written once, read back only by the host
  const uint64_t ts = tx.now_ts + (uint64_t)seconds_to_ts(dist / a.speed);
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  u32x4 *dst = reinterpret_cast<u32x4 *>(a.out + (t * (a.nphy - 1) + off));
  const uint64_t rxb = (uint64_t)__double_as_longlong(rx);
  const u32x4 w0 = {(uint32_t)ts, (uint32_t)(ts >> 32), tx.uid_base + off, a.phys.node[j]};
  const u32x4 w1 = {(uint32_t)j, 0u, (uint32_t)rxb, (uint32_t)(rxb >> 32)};
  __builtin_nontemporal_store(w0, dst);
  __builtin_nontemporal_store(w1, dst + 1);
}

template <int KIND>
__global__ __launch_bounds__(FAN_THREADS) void fan_write(FanArgs a) {
  const int64_t t = blockIdx.y;
  const nsgpu_tx_desc tx = a.tx[t];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __shared__ uint32_t s_off;
  __shared__ uint32_t wc[FAN_THREADS / 64];
  // block offset: sum of counts of blocks [0, blockIdx.x) — reduced by the first wave
  if (wid == 0) {
    uint32_t acc = 0;
    for (int b = lane; b < (int)blockIdx.x; b += 64) acc += a.block_counts[t * a.nblocks + b];
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if (lane == 0) s_off = acc;
  }
  const int64_t j = (int64_t)blockIdx.x * FAN_THREADS + threadIdx.x;
  double dist = 0, rx = 0;
  const bool s = fan_eval<KIND>(a, tx, j, dist, rx);
  const unsigned long long b = __ballot(s);
  if (lane == 0) wc[wid] = (uint32_t)__popcll(b);
  __syncthreads();
  uint32_t off = s_off;
  for (int w = 0; w < wid; w++) off += wc[w];
  off += (uint32_t)__popcll(b & ((1ull << lane) - 1));
  if (s) {
    int64_t delay = 0;
    if (KIND == FAN_YANS || a.speed > 0) delay = seconds_to_ts(dist / a.speed);  // Seconds (distance / m_speed)
    const int64_t slot = t * (a.nphy - 1) + off;
    nsgpu_rx_record r;
    r.ts = tx.now_ts + (uint64_t)delay;  // m_currentTs + time.GetTimeStep () (default-simulator-impl.cc:212)
    r.uid = tx.uid_base + off;
    r.context = a.phys.node[j];
    r.phy = (uint32_t)j;
    r.pad_ = 0;
    r.rx_dbm = rx;
    a.out[slot] = r;
    if (KIND == FAN_SPECTRUM) {
      const double gainLinear = pow(10.0, rx / 10.0);  // :153
      for (int q = 0; q < a.nbands; q++)
        a.psd_out[slot * a.nbands + q] = a.psd_tx[t * a.nbands + q] * gainLinear;
    }
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == FAN_THREADS - 1) {
    uint32_t total = s_off;
    for (int w = 0; w < FAN_THREADS / 64; w++) total += wc[w];
    a.count[t] = total;
  }
}

// ---- MultiModelSpectrumChannel::StartTx (multi-model-spectrum-channel.cc:226-331) ----
struct MultiArgs {
  nsgpu_phy_soa phys;
  const int32_t *rx_model;
  const uint32_t *iter, *iter_pos;  // receiver iteration order (model-grouped AddRx order) and its inverse
  int64_t nphy;
  nsgpu_spectrum_models models;
  const nsgpu_tx_desc *tx;
  const int32_t *tx_model;
  const double *psd_tx;  // [t][max_bands]
  nsgpu_loss_chain loss;
  double speed, max_loss_db;
  nsgpu_rx_record *out;
  double *psd_out;       // [(t * (nphy - 1) + k) * max_bands + b]
  nsgpu_loss_trace *trace;
  uint32_t *count;
  uint32_t *block_counts;  // [t][nblocks]
  double *conv;            // [t][n_models][max_bands]: the tx PSD in each rx model
  int32_t nblocks;
};

// SpectrumConverter::GetCoefficient (spectrum-converter.cc)
__device__ __forceinline__ double converter_coeff(double ffl, double ffh, double tfl, double tfh) {
  double c = fmin(ffh, tfh) - fmax(ffl, tfl);
  c = fmax(0.0, c);
  return fmin(1.0, c / (tfh - tfl));
}

// The transmission's PSD in every rx model: a copy for its own model (:254-258), else
// SpectrumConverter::Convert (sum over the input bands in order).  grid (n_models, n_tx).
__global__ __launch_bounds__(64) void fan_multi_convert(MultiArgs a) {
  const int m = blockIdx.x;
  const int64_t t = blockIdx.y;
  const int tm = a.tx_model[t];
  const uint32_t r0 = a.models.band_off[m], nrb = a.models.band_off[m + 1] - r0;
  const uint32_t t0 = a.models.band_off[tm], ntb = a.models.band_off[tm + 1] - t0;
  const double *p = a.psd_tx + t * a.models.max_bands;
  double *c = a.conv + (t * a.models.n_models + m) * a.models.max_bands;
  for (uint32_t b = threadIdx.x; b < nrb; b += 64) {
    double sum;
    if (m == tm) {
      sum = p[b];
    } else {
      sum = 0;
      const double tfl = a.models.fl[r0 + b], tfh = a.models.fh[r0 + b];
      for (uint32_t f = 0; f < ntb; f++) sum += p[f] * converter_coeff(a.models.fl[t0 + f], a.models.fh[t0 + f], tfl, tfh);
    }
    c[b] = sum;
  }
}

// Receiver at iteration position q: gain (and trace entry), survivor?
__device__ __forceinline__ bool multi_eval(const MultiArgs &a, const nsgpu_tx_desc &t, int64_t q, int64_t spos,
                                           int64_t &j, double &dist, double &gain) {
  if (q >= a.nphy || q == spos || spos >= a.nphy) return false;
  j = a.iter[q];
  dist = distance3(a.phys.x[t.sender], a.phys.y[t.sender], a.phys.z[t.sender], a.phys.x[j], a.phys.y[j], a.phys.z[j]);
  gain = calc_rx_power(a.loss, 0.0, dist);  // :290
  return !((-gain) > a.max_loss_db);        // :292-296
}

__global__ __launch_bounds__(FAN_THREADS) void fan_multi_count(MultiArgs a) {
  const int64_t t = blockIdx.y;
  const nsgpu_tx_desc tx = a.tx[t];
  const int64_t spos = (int64_t)tx.sender < a.nphy ? (int64_t)a.iter_pos[tx.sender] : a.nphy;
  const int64_t q = (int64_t)blockIdx.x * FAN_THREADS + threadIdx.x;
  int64_t j = 0;
  double d = 0, g = 0;
  const bool s = multi_eval(a, tx, q, spos, j, d, g);
  if (a.trace && q < a.nphy && q != spos && spos < a.nphy)  // m_propagationLossTrace, before the cut (:291)
    a.trace[t * (a.nphy - 1) + q - (q > spos ? 1 : 0)] = nsgpu_loss_trace{(uint32_t)j, 0u, -g};
  const unsigned long long b = __ballot(s);
  __shared__ uint32_t wc[FAN_THREADS / 64];
  if ((threadIdx.x & 63) == 0) wc[threadIdx.x >> 6] = (uint32_t)__popcll(b);
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t c = 0;
    for (int w = 0; w < FAN_THREADS / 64; w++) c += wc[w];
    a.block_counts[t * a.nblocks + blockIdx.x] = c;
  }
}

__global__ __launch_bounds__(FAN_THREADS) void fan_multi_write(MultiArgs a) {
  const int64_t t = blockIdx.y;
  const nsgpu_tx_desc tx = a.tx[t];
  const int64_t spos = (int64_t)tx.sender < a.nphy ? (int64_t)a.iter_pos[tx.sender] : a.nphy;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __shared__ uint32_t s_off;
  __shared__ uint32_t wc[FAN_THREADS / 64];
  if (wid == 0) {
    uint32_t acc = 0;
    for (int b = lane; b < (int)blockIdx.x; b += 64) acc += a.block_counts[t * a.nblocks + b];
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if (lane == 0) s_off = acc;
  }
  const int64_t q = (int64_t)blockIdx.x * FAN_THREADS + threadIdx.x;
  int64_t j = 0;
  double dist = 0, g = 0;
  const bool s = multi_eval(a, tx, q, spos, j, dist, g);
  const unsigned long long b = __ballot(s);
  if (lane == 0) wc[wid] = (uint32_t)__popcll(b);
  __syncthreads();
  uint32_t off = s_off;
  for (int w = 0; w < wid; w++) off += wc[w];
  off += (uint32_t)__popcll(b & ((1ull << lane) - 1));
  if (s) {
    const int64_t delay = a.speed > 0 ? seconds_to_ts(dist / a.speed) : 0;
    const int64_t slot = t * (a.nphy - 1) + off;
    nsgpu_rx_record r;
    r.ts = tx.now_ts + (uint64_t)delay;
    r.uid = tx.uid_base + off;
    r.context = a.phys.node[j];
    r.phy = (uint32_t)j;
    r.pad_ = 0;
    r.rx_dbm = g;
    a.out[slot] = r;
    const int m = a.rx_model[j];
    const uint32_t nrb = a.models.band_off[m + 1] - a.models.band_off[m];
    const double gainLinear = pow(10.0, g / 10.0);  // :297-298
    const double *c = a.conv + (t * a.models.n_models + m) * a.models.max_bands;
    for (uint32_t q2 = 0; q2 < nrb; q2++) a.psd_out[slot * a.models.max_bands + q2] = c[q2] * gainLinear;
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == FAN_THREADS - 1) {
    uint32_t total = s_off;
    for (int w = 0; w < FAN_THREADS / 64; w++) total += wc[w];
    a.count[t] = total;
  }
}

__global__ void seconds_kernel(const double *__restrict__ in, int64_t *__restrict__ out, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = seconds_to_ts(in[i]);
}

static int fan_launch(int kind, const nsgpu_phy_soa *phys, int64_t nphy, const nsgpu_tx_desc *d_tx, int64_t n_tx,
                      const nsgpu_loss_chain *loss, double speed, double max_loss_db, const double *d_psd_tx,
                      int32_t nbands, nsgpu_rx_record *d_out, double *d_psd_out, uint32_t *d_count,
                      void *d_workspace, void *stream) {
  if (!phys || !loss || !d_tx || !d_out || !d_count || !d_workspace)
    return set_error(NSGPU_EINVAL, "nsgpu_fanout: null pointer");
  if (nphy < 2 || n_tx < 1 || n_tx > 65535) return set_error(NSGPU_EINVAL, "nsgpu_fanout: nphy=%lld n_tx=%lld",
                                                              (long long)nphy, (long long)n_tx);
  if (loss->n < 0 || loss->n > NSGPU_MAX_LOSS_CHAIN) return set_error(NSGPU_EINVAL, "nsgpu_fanout: loss chain");
  if (kind == FAN_YANS && !(speed > 0)) return set_error(NSGPU_EINVAL, "nsgpu_fanout_yans: speed must be > 0");
  if (kind == FAN_SPECTRUM && nbands > 0 && (!d_psd_tx || !d_psd_out))
    return set_error(NSGPU_EINVAL, "nsgpu_fanout_spectrum: null psd");
  FanArgs a;
  a.phys = *phys;
  a.nphy = nphy;
  a.tx = d_tx;
  a.loss = *loss;
  a.speed = speed;
  a.max_loss_db = max_loss_db;
  a.psd_tx = d_psd_tx;
  a.nbands = nbands;
  a.out = d_out;
  a.psd_out = d_psd_out;
  a.count = d_count;
  a.block_counts = (uint32_t *)d_workspace;
  a.nblocks = (int32_t)((nphy + FAN_THREADS - 1) / FAN_THREADS);
  dim3 grid(a.nblocks, (unsigned)n_tx);
  hipStream_t s = (hipStream_t)stream;
  if ((phys->chan_rank == nullptr) != (phys->chan_count == nullptr))
    return set_error(NSGPU_EINVAL, "nsgpu_fanout: chan_rank and chan_count go together");
  if (kind == FAN_YANS && phys->chan_rank) {
    if (((uintptr_t)d_out & 15u) != 0)  // two 16-B stores per record
      return set_error(NSGPU_EINVAL, "nsgpu_fanout_yans: d_out must be 16-byte aligned with rank tables");
    hipLaunchKernelGGL(fan_write_ranked, grid, dim3(FAN_THREADS), 0, s, a);
  } else if (kind == FAN_YANS) {
    hipLaunchKernelGGL(fan_count<FAN_YANS>, grid, dim3(FAN_THREADS), 0, s, a);
    hipLaunchKernelGGL(fan_write<FAN_YANS>, grid, dim3(FAN_THREADS), 0, s, a);
  } else {
    hipLaunchKernelGGL(fan_count<FAN_SPECTRUM>, grid, dim3(FAN_THREADS), 0, s, a);
    hipLaunchKernelGGL(fan_write<FAN_SPECTRUM>, grid, dim3(FAN_THREADS), 0, s, a);
  }
  NSGPU_HIP(hipGetLastError());
  return NSGPU_OK;
}

}  // namespace nsgpu

using namespace nsgpu;

extern "C" int nsgpu_fanout_workspace_bytes(int64_t nphy, int64_t n_tx, uint64_t *bytes) {
  *bytes = (uint64_t)((nphy + FAN_THREADS - 1) / FAN_THREADS) * (uint64_t)n_tx * sizeof(uint32_t) + 256;
  return NSGPU_OK;
}

extern "C" int nsgpu_fanout_yans(const nsgpu_phy_soa *phys, int64_t nphy, const nsgpu_tx_desc *d_tx, int64_t n_tx,
                                 const nsgpu_loss_chain *loss, double speed, nsgpu_rx_record *d_out,
                                 uint32_t *d_count, void *d_workspace, void *stream) {
  return fan_launch(FAN_YANS, phys, nphy, d_tx, n_tx, loss, speed, 0.0, nullptr, 0, d_out, nullptr, d_count,
                    d_workspace, stream);
}

extern "C" int nsgpu_fanout_spectrum(const nsgpu_phy_soa *phys, int64_t nphy, const nsgpu_tx_desc *d_tx,
                                     int64_t n_tx, const nsgpu_loss_chain *loss, double speed, double max_loss_db,
                                     const double *d_psd_tx, int32_t nbands, nsgpu_rx_record *d_out,
                                     double *d_psd_out, uint32_t *d_count, void *d_workspace, void *stream) {
  return fan_launch(FAN_SPECTRUM, phys, nphy, d_tx, n_tx, loss, speed, max_loss_db, d_psd_tx, nbands, d_out,
                    d_psd_out, d_count, d_workspace, stream);
}

extern "C" int nsgpu_fanout_multi_workspace_bytes(int64_t nphy, int64_t n_tx, int32_t n_models, int32_t max_bands,
                                                  uint64_t *bytes) {
  const uint64_t counts = (uint64_t)((nphy + FAN_THREADS - 1) / FAN_THREADS) * (uint64_t)n_tx * sizeof(uint32_t);
  *bytes = ((counts + 255) & ~255ull) + (uint64_t)n_tx * n_models * max_bands * sizeof(double) + 256;
  return NSGPU_OK;
}

extern "C" int nsgpu_fanout_spectrum_multi(const nsgpu_phy_soa *phys, const int32_t *d_rx_model,
                                           const uint32_t *d_iter, const uint32_t *d_iter_pos, int64_t nphy,
                                           const nsgpu_spectrum_models *models, const nsgpu_tx_desc *d_tx,
                                           const int32_t *d_tx_model, const double *d_psd_tx, int64_t n_tx,
                                           const nsgpu_loss_chain *loss, double speed, double max_loss_db,
                                           nsgpu_rx_record *d_out, double *d_psd_out, nsgpu_loss_trace *d_trace,
                                           uint32_t *d_count, void *d_workspace, void *stream) {
  if (!phys || !d_rx_model || !d_iter || !d_iter_pos || !models || !d_tx || !d_tx_model || !d_psd_tx || !loss ||
      !d_out || !d_psd_out || !d_count || !d_workspace)
    return set_error(NSGPU_EINVAL, "nsgpu_fanout_spectrum_multi: null pointer");
  if (nphy < 2 || n_tx < 1 || n_tx > 65535 || models->n_models < 1 || models->n_models > 65535 ||
      models->max_bands < 1 || !models->band_off || !models->fl || !models->fh)
    return set_error(NSGPU_EINVAL, "nsgpu_fanout_spectrum_multi: nphy=%lld n_tx=%lld models=%d bands=%d",
                     (long long)nphy, (long long)n_tx, models->n_models, models->max_bands);
  if (loss->n < 0 || loss->n > NSGPU_MAX_LOSS_CHAIN) return set_error(NSGPU_EINVAL, "nsgpu_fanout: loss chain");
  MultiArgs a;
  a.phys = *phys;
  a.rx_model = d_rx_model;
  a.iter = d_iter;
  a.iter_pos = d_iter_pos;
  a.nphy = nphy;
  a.models = *models;
  a.tx = d_tx;
  a.tx_model = d_tx_model;
  a.psd_tx = d_psd_tx;
  a.loss = *loss;
  a.speed = speed;
  a.max_loss_db = max_loss_db;
  a.out = d_out;
  a.psd_out = d_psd_out;
  a.trace = d_trace;
  a.count = d_count;
  a.nblocks = (int32_t)((nphy + FAN_THREADS - 1) / FAN_THREADS);
  const uint64_t counts = (uint64_t)a.nblocks * (uint64_t)n_tx * sizeof(uint32_t);
  a.block_counts = (uint32_t *)d_workspace;
  a.conv = (double *)((char *)d_workspace + ((counts + 255) & ~255ull));
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(fan_multi_convert, dim3(models->n_models, (unsigned)n_tx), dim3(64), 0, s, a);
  hipLaunchKernelGGL(fan_multi_count, dim3(a.nblocks, (unsigned)n_tx), dim3(FAN_THREADS), 0, s, a);
  hipLaunchKernelGGL(fan_multi_write, dim3(a.nblocks, (unsigned)n_tx), dim3(FAN_THREADS), 0, s, a);
  NSGPU_HIP(hipGetLastError());
  return NSGPU_OK;
}

extern "C" int nsgpu_seconds_to_ts(const double *d_seconds, int64_t *d_out, int64_t n, void *stream) {
  if (n < 0 || (n > 0 && (!d_seconds || !d_out))) return set_error(NSGPU_EINVAL, "nsgpu_seconds_to_ts: bad args");
  if (n == 0) return NSGPU_OK;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(seconds_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, d_seconds, d_out, n);
  NSGPU_HIP(hipGetLastError());
  return NSGPU_OK;
}
