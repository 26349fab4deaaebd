/*
 * nsref.h — CPU ORACLE for the nsgpu hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * This is a plain-C++ restatement of the ns-3 (ybaddi/ns-3-dev-dnemu, ns-3.13-dev)
 * algorithms on the hot path.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it, and only as the checker / CPU baseline — never as
 * the thing measured or shipped.  The product path (libnsgpu.so) never links it.
 *
 * Parity pin: the reference tree cannot be built here
 * (its int64x64/Time headers include the waf-generated ns3/core-config.h and its
 * mpi module needs <mpi.h>), so there is no oracle/_ref.  This
 * restatement is pinned against every known-answer vector the reference's own
 * test suites hold for this path (the JSON files under tests/golden, each entry citing its
 * reference file:line), and against the survey-time reference run facts.
 *
 * Every function cites the reference file:line it restates.
 */
#ifndef NSREF_H
#define NSREF_H

#include <stdint.h>
#include "../include/nsgpu_types.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------- int64x64_t (src/core/model/int64x64-128.{h,cc}) ----------------
 * A 64.64 fixed-point value is passed as two little-endian 64-bit words of the
 * two's-complement int128: w[0] = low word, w[1] = high word. */
void     nsref_i64x64_from_double(double v, uint64_t out[2]);        /* int64x64-128.h:26-36 */
void     nsref_i64x64_from_int(int64_t v, uint64_t out[2]);          /* int64x64-128.h:37-66 */
void     nsref_i64x64_from_parts(int64_t hi, uint64_t lo, uint64_t out[2]); /* int64x64-128.h:67-74 */
void     nsref_i64x64_mul(const uint64_t a[2], const uint64_t b[2], uint64_t out[2]);  /* int64x64-128.cc:20-57 */
void     nsref_i64x64_div(const uint64_t a[2], const uint64_t b[2], uint64_t out[2]);  /* int64x64-128.cc:58-92 */
void     nsref_i64x64_invert(uint64_t v, uint64_t out[2]);                             /* int64x64-128.cc:119-134 */
void     nsref_i64x64_mul_by_invert(const uint64_t a[2], const uint64_t b[2], uint64_t out[2]); /* :94-118 */
int64_t  nsref_i64x64_get_high(const uint64_t a[2]);                 /* int64x64-128.h:98-105 */
uint64_t nsref_i64x64_get_low(const uint64_t a[2]);                  /* int64x64-128.h:106-113 */
double   nsref_i64x64_get_double(const uint64_t a[2]);               /* int64x64-128.h:85-97 */

/* ---------------- Time at NS resolution (src/core/model/nstime.h, time.cc) ---------------- */
int64_t  nsref_seconds(double s);                          /* Seconds(double).GetTimeStep(): nstime.h:388-391,403-418,586-589 */
void     nsref_seconds_batch(const double *s, int64_t *out, int64_t n);
double   nsref_get_seconds(int64_t ts);                    /* Time::GetSeconds(): nstime.h:398-401,419-431 */
int64_t  nsref_from_integer(int64_t v, int unit);          /* Time::FromInteger: nstime.h:344-361 (unit: 0=S..5=FS) */

/* ---------------- Mobility + propagation (src/propagation, src/mobility) ---------------- */
double nsref_distance(double ax, double ay, double az, double bx, double by, double bz);  /* vector.cc:63-70 */
double nsref_calc_rx_power(double tx_dbm, double distance, const nsgpu_loss_chain *chain); /* propagation-loss-model.cc:64-74 */
int64_t nsref_const_speed_delay(double distance, double speed);                           /* propagation-delay-model.cc:90-96 */

/* YansWifiChannel::Send (src/wifi/model/yans-wifi-channel.cc:77-115).
 * phys are in m_phyList order; returns the number of records written (= receivers scheduled). */
int64_t nsref_fanout_yans(const double *x, const double *y, const double *z,
                          const uint32_t *chan, const uint32_t *node, int64_t nphy,
                          int64_t sender, double tx_dbm, const nsgpu_loss_chain *loss, double speed,
                          uint64_t now_ts, uint32_t uid_base, nsgpu_rx_record *out);

/* SingleModelSpectrumChannel::StartTx (src/spectrum/model/single-model-spectrum-channel.cc:106-183):
 * loss computed with tx = 0 dBm, receivers with -gain > max_loss_db are skipped (no uid),
 * survivors get psd_out[k*nbands + b] = psd_tx[b] * 10^(gain/10). */
int64_t nsref_fanout_spectrum(const double *x, const double *y, const double *z,
                              const uint32_t *node, int64_t nphy, int64_t sender,
                              const nsgpu_loss_chain *loss, double speed, double max_loss_db,
                              const double *psd_tx, int32_t nbands,
                              uint64_t now_ts, uint32_t uid_base,
                              nsgpu_rx_record *out, double *psd_out);

/* MultiModelSpectrumChannel::StartTx (src/spectrum/model/multi-model-spectrum-channel.cc:226-331) with the
 * SpectrumConverter of spectrum-converter.cc: receivers grouped by rx SpectrumModel (ascending model index
 * = ascending SpectrumModelUid), AddRx order within a model; the tx PSD (model tx_model) converted once per
 * rx model, then scaled by each survivor's 10^(gain/10).  Models: n_models, band_off[n_models+1], fl/fh.
 * Records go to out[k], PSDs to psd_out[k * psd_stride + b]; every non-sender receiver (cut or not) gets a
 * PropagationLoss trace entry trace[i] (receiver iteration order); *n_trace = entries written. */
int64_t nsref_fanout_spectrum_multi(const double *x, const double *y, const double *z, const uint32_t *node,
                                    const int32_t *rx_model, int64_t nphy, int64_t sender,
                                    int32_t n_models, const uint32_t *band_off, const double *fl, const double *fh,
                                    int32_t tx_model, const double *psd_tx,
                                    const nsgpu_loss_chain *loss, double speed, double max_loss_db,
                                    uint64_t now_ts, uint32_t uid_base,
                                    nsgpu_rx_record *out, double *psd_out, int32_t psd_stride,
                                    nsgpu_loss_trace *trace, int64_t *n_trace);

/* ---------------- Sequential engine: DefaultSimulatorImpl + Map/Heap scheduler ----------------
 * (src/core/model/default-simulator-impl.cc:49-353, map-scheduler.cc:51-100, heap-scheduler.cc:44-217) */
enum { NSREF_SCHED_MAP = 0, NSREF_SCHED_HEAP = 1, NSREF_SCHED_LIST = 2, NSREF_SCHED_CALENDAR = 3 };

typedef void (*nsref_fn)(void *user, uint64_t arg);
typedef struct nsref_sim nsref_sim;

nsref_sim *nsref_sim_new(int scheduler);
void       nsref_sim_free(nsref_sim *s);
void       nsref_sim_set_uid(nsref_sim *s, uint32_t uid);  /* m_uid (a uint32: it wraps like the reference's) */
nsgpu_event_id nsref_sim_schedule(nsref_sim *s, int64_t delay, nsref_fn fn, void *user, uint64_t arg);
void       nsref_sim_schedule_with_context(nsref_sim *s, uint32_t ctx, int64_t delay, nsref_fn fn, void *user, uint64_t arg);
nsgpu_event_id nsref_sim_schedule_now(nsref_sim *s, nsref_fn fn, void *user, uint64_t arg);
nsgpu_event_id nsref_sim_schedule_destroy(nsref_sim *s, nsref_fn fn, void *user, uint64_t arg);
void       nsref_sim_remove(nsref_sim *s, const nsgpu_event_id *id);
void       nsref_sim_cancel(nsref_sim *s, const nsgpu_event_id *id);
int        nsref_sim_is_expired(nsref_sim *s, const nsgpu_event_id *id);
void       nsref_sim_run(nsref_sim *s);
void       nsref_sim_run_one(nsref_sim *s);       /* RunOneEvent (:167-170) */
int        nsref_sim_is_finished(nsref_sim *s);   /* IsFinished (:133-137) */
void       nsref_sim_stop(nsref_sim *s);
void       nsref_sim_stop_at(nsref_sim *s, int64_t delay);
void       nsref_sim_destroy(nsref_sim *s);
uint64_t   nsref_sim_now(nsref_sim *s);
uint32_t   nsref_sim_context(nsref_sim *s);
uint64_t   nsref_sim_delay_left(nsref_sim *s, const nsgpu_event_id *id);
uint64_t   nsref_sim_dispatched(nsref_sim *s);   /* RemoveNext count (cancelled included) */
uint32_t   nsref_sim_next_uid(nsref_sim *s);
/* Optional pop-order log of every dispatch: (ts, uid, ctx). */
void       nsref_sim_set_log(nsref_sim *s, uint64_t *ts, uint32_t *uid, uint32_t *ctx, uint64_t cap);

/* ---------------- utils/bench-simulator.cc (config 1) ----------------
 * Bench::RunBench/Cb (bench-simulator.cc:79-127) on the restated engine.
 * dist_ns: the distribution already converted by ReadDistribution (:59-76). */
typedef struct nsref_churn_result {
  uint64_t dispatched;   /* RemoveNext calls */
  uint64_t holds;        /* Bench::m_n */
  uint64_t final_ts;     /* ts of the last dispatched event */
  uint64_t digest;       /* sum_k nsgpu_dispatch_digest_term(k, ts_k, uid_k) */
  uint32_t next_uid;
  uint32_t pad_;
  double   run_seconds;  /* wall time of Simulator::Run only (bench-simulator.cc:94-97) */
  double   init_seconds; /* wall time of the initial inserts (:83-90) */
} nsref_churn_result;

/* Returns 0, or -3 when the CalendarScheduler reaches the reference's H3 crash (calendar-scheduler.cc:
 * 128,157,182-185: every pending event later than 2^32 ns); *out then describes the run up to it. */
int nsref_churn_run(const uint64_t *dist_ns, uint32_t n, uint32_t total, int scheduler,
                    uint64_t *log_ts, uint32_t *log_uid, uint64_t log_cap, nsref_churn_result *out);

/* ---------------- point-to-point subset (configs 2, 4, 5) ----------------
 * Sequential run of a nsgpu_p2p_scenario (see nsref_p2p.cc for the restated reference code).
 * devc/appc (optional) receive n_devices / n_apps counters; the optional log receives the pop order. */
int nsref_p2p_run(const nsgpu_p2p_scenario *sc, nsgpu_p2p_stats *stats, nsgpu_dev_counters *devc,
                  nsgpu_app_counters *appc, uint64_t *log_ts, uint32_t *log_uid, uint32_t *log_ctx,
                  uint64_t log_cap, double *run_seconds);
/* The same run, also recording every ascii trace sink call (nsgpu_trace_record, pop order) when
 * trace_n is non-NULL: *trace_n = records made, the first trace_cap of them copied to trace. */
/* Trace kinds the next nsref_p2p_run_trace / _probe runs record: bit k = nsgpu_trace_kind k (default 0xf). */
void nsref_p2p_set_trace_kinds(uint32_t mask);
int nsref_p2p_run_trace(const nsgpu_p2p_scenario *sc, nsgpu_p2p_stats *stats, nsgpu_dev_counters *devc,
                        nsgpu_app_counters *appc, uint64_t *log_ts, uint32_t *log_uid, uint32_t *log_ctx,
                        uint64_t log_cap, double *run_seconds, nsgpu_trace_record *trace, uint64_t trace_cap,
                        uint64_t *trace_n);

/* The same run with a host application interleaved (see nsref_p2p.cc): samples receives `count`
 * snapshots of application app_obs's counters. */
int nsref_p2p_run_probe(const nsgpu_p2p_scenario *sc, int64_t t0, int64_t period, uint32_t count, uint32_t app_send,
                        uint32_t app_obs, nsgpu_app_counters *samples, nsgpu_p2p_stats *stats,
                        nsgpu_dev_counters *devc, nsgpu_app_counters *appc, uint64_t *log_ts, uint32_t *log_uid,
                        uint32_t *log_ctx, uint64_t log_cap, nsgpu_trace_record *trace, uint64_t trace_cap,
                        uint64_t *trace_n);

/* The same run with host datagrams: after setup, Schedule (ts[k], UdpSocket::Send of one datagram of app[k]'s
 * flow) for k in order (a replay of a reference pcap's sends). */
int nsref_p2p_run_sends(const nsgpu_p2p_scenario *sc, uint64_t n, const int64_t *ts, const uint32_t *app,
                        nsgpu_p2p_stats *stats, nsgpu_dev_counters *devc, nsgpu_app_counters *appc, uint64_t *log_ts,
                        uint32_t *log_uid, uint32_t *log_ctx, uint64_t log_cap, nsgpu_trace_record *trace,
                        uint64_t trace_cap, uint64_t *trace_n);

/* bench-simulator ReadDistribution: (uint64_t)(data * 1000000000)  (bench-simulator.cc:66) */
uint64_t nsref_distribution_ns(double seconds);

/* ---------------- Wi-Fi PHY receive subset (nsref_wifi.cc) ----------------
 * WifiPhy::CalculateTxDuration (wifi-phy.cc:141-296) in ns, and a sequential run of a
 * nsgpu_wifi_scenario (SendPacket / YansWifiChannel::Send / StartReceivePacket / InterferenceHelper /
 * WifiPhyStateHelper / EndReceive's state part).  Any output pointer may be NULL.  rx_log has
 * n_tx * n_phy slots.  Returns 0, -1 (SendPacket while in TX: the reference's NS_FATAL_ERROR) or
 * -2 (more EndReceive records than ends_cap; *n_ends still holds the count). */
int64_t nsref_wifi_tx_duration(uint32_t size, uint32_t modclass, uint64_t rate_bps, uint32_t bw_hz, uint32_t preamble);
int nsref_wifi_run(const nsgpu_wifi_scenario *sc, nsgpu_wifi_stats *stats, nsgpu_wifi_phy_counters *phys,
                   uint32_t *tx_base, nsgpu_wifi_end_record *ends, uint64_t ends_cap, uint64_t *n_ends,
                   nsgpu_wifi_rx_log *rx_log);

/* Closed-loop Wi-Fi (the engine behind nsgpu_wifil_* / nsgpu_sim_attach_wifi): SendPacket from host
 * closures.  The host side is the tests' MAC stand-in (restated by the GPU tests on nsgpu_sim): setup
 * Schedule (first[i], attempt i) for every phy i in order, then Simulator::Stop (stop_ts); attempt i at
 * Now: if phy i's WifiPhyStateHelper state is IDLE, SendPacket (the packet below) and Schedule (period,
 * attempt i), else Schedule (backoff[i], attempt i).  EndReceive computes InterferenceHelper::
 * CalculateSnrPer (interference-helper.cc:216-367) with the configured error-rate model; the m_random draw
 * is the caller's (ends[], in dispatch order).  out[]: dispatched, digest (nsgpu_dispatch_digest_term),
 * next uid, final ts, SendPacket calls, attempts that found the phy busy. */
typedef struct nsref_wifil_mac {
  const uint64_t *first, *backoff;
  uint64_t period, stop_ts, rate;
  uint32_t size, modclass, bw, preamble;
  double dbm;
  uint32_t uid_first, pad_;  /* m_uid before the setup calls (0: 4) */
  /* the EndReceive hand-back (YansWifiPhy::EndReceive -> the MAC's receive callback, yans-wifi-phy.cc:783-791):
   * reply_on = 1: an EndReceive that is not cancelled and whose m_random draw (0.5 here) exceeds its per
   * Schedules (reply_delay, reply of its phy) in the EndReceive's context; the reply sends a frame when the phy is
   * IDLE (else counts as busy) and schedules nothing else */
  uint64_t reply_delay;
  uint32_t reply_on, pad2_;
} nsref_wifil_mac;
int nsref_wifil_run(const nsgpu_wifil_config *cfg, const nsref_wifil_mac *mac, uint64_t *log_ts, uint32_t *log_uid,
                    uint32_t *log_ctx, uint64_t log_cap, nsgpu_wifil_end *ends, uint64_t ends_cap, uint64_t *n_ends,
                    nsgpu_wifi_phy_counters *phys, uint64_t out[6], uint64_t *tx_out, uint64_t tx_cap);
/* (tx_out: 3 words per SendPacket call — ts, the closure's uid, phy — up to tx_cap calls; may be NULL)
 * A replayed transmission schedule (SendPacket of phy[k] with size[k] at ts[k], whatever the PHY state) on
 * the closed-loop PHY, then Simulator::Stop (stop_ts). */
typedef struct nsref_wifil_sends {
  uint64_t n;
  const uint64_t *ts;
  const uint32_t *phy, *size;
  uint32_t modclass, bw, preamble, pad_;
  uint64_t rate, stop_ts;
  double dbm;
  /* MobilityModel::SetPosition of move_phy[k] to move_xyz[3k..3k+2] at move_ts[k] (host closures scheduled after
   * the sends, before the Stop) */
  uint64_t n_moves;
  const uint64_t *move_ts;
  const uint32_t *move_phy;
  const double *move_xyz;
} nsref_wifil_sends;
int nsref_wifil_replay(const nsgpu_wifil_config *cfg, const nsref_wifil_sends *sn, uint64_t *log_ts, uint32_t *log_uid,
                       uint32_t *log_ctx, uint64_t log_cap, nsgpu_wifil_end *ends, uint64_t ends_cap, uint64_t *n_ends,
                       nsgpu_wifi_phy_counters *phys, uint64_t out[6], uint64_t *tx_out, uint64_t tx_cap);
/* InterferenceHelper::CalculateChunkSuccessRate's error-rate model call for one chunk (tests). */
double nsref_wifil_chunk_success(uint32_t model, uint32_t modclass, uint64_t rate, uint32_t bw, double snr, uint32_t nbits);

/* ---------------- Global routing (nsref_route.cc) ----------------
 * GlobalRouteManager::PopulateRoutingTables + Ipv4GlobalRouting::RouteInput/LookupGlobal over a
 * point-to-point topology: route_out[node * n_dst + k] = the device the node's first matching route
 * to dst_addr[k] leaves through, 0xfffffffe when the address is the node's own (local delivery),
 * 0xffffffff when no route matches.  dev_ifindex: the device's Ipv4 interface index (loopback is 0).
 * Returns 0, or -1 on an inconsistent interface numbering. */
int nsref_global_routes(uint32_t n_nodes, uint32_t n_devices, const uint32_t *dev_node, const uint32_t *dev_peer,
                        const uint32_t *dev_addr, const uint32_t *dev_mask, const uint32_t *dev_ifindex,
                        uint32_t n_dst, const uint32_t *dst_addr, uint32_t *route_out);

#ifdef __cplusplus
}
#endif
#endif
