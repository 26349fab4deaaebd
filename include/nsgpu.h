/*
 * nsgpu.h — C-ABI of libnsgpu.so, the MI355X (gfx950) discrete-event engine that sits behind
 * ns-3's SimulatorImpl / Scheduler plugin surface (ybaddi/ns-3-dev-dnemu, ns-3.13-dev).
 *
 * Every entry point is extern "C", takes plain pointers and sizes, and returns an int status
 * (NSGPU_OK = 0).  On failure nsgpu_last_error() describes it; the ns-3 side maps a non-zero
 * status to NS_FATAL_ERROR (SURVEY §8(b) error convention).  Pointers named d_* are device
 * (HBM) pointers; `stream` is a hipStream_t (NULL = the default stream).  Calls are made from
 * the single simulation thread (ns-3 is single-threaded w.r.t. the simulator).
 *
 * Which reference interface each group replaces is cited next to it; INTEGRATION.md shows
 * the ns-3 classes (ns3::HipBatchScheduler, ns3::HipSimulatorImpl) that bind them.
 */
#ifndef NSGPU_H
#define NSGPU_H

#include <stddef.h>
#include <stdint.h>
#include "nsgpu_types.h"

#ifdef __cplusplus
extern "C" {
#endif

enum {
  NSGPU_OK = 0,
  NSGPU_EINVAL = 1,   /* bad argument (shape, null pointer, capacity) */
  NSGPU_EHIP = 2,     /* HIP runtime error */
  NSGPU_ENOMEM = 3,   /* device allocation or fixed capacity exhausted */
  NSGPU_ESTATE = 4,   /* call not valid in the current state (e.g. empty queue) */
  NSGPU_ERANGE = 5    /* the uid counter would pass 0xfffffffe: DefaultSimulatorImpl's uint32 m_uid wraps to 0 after
                       * 0xffffffff (default-simulator-impl.cc:52-56,188-219), which no engine replicates;
                       * the run fails before an event with such a uid is dispatched */
};

/* ---------------- library / device plumbing ---------------- */
int         nsgpu_version(void);                 /* 100 * major + minor */
const char *nsgpu_last_error(void);
int         nsgpu_device_count(int *count);
int         nsgpu_set_device(int device);
int         nsgpu_malloc(void **d_ptr, size_t bytes);
int         nsgpu_free(void *d_ptr);
int         nsgpu_memcpy_htod(void *d_dst, const void *h_src, size_t bytes, void *stream);
int         nsgpu_memcpy_dtoh(void *h_dst, const void *d_src, size_t bytes, void *stream);
int         nsgpu_memset(void *d_dst, int value, size_t bytes, void *stream);
int         nsgpu_device_synchronize(void);
int         nsgpu_stream_create(void **stream);
int         nsgpu_stream_destroy(void *stream);
int         nsgpu_stream_sync(void *stream);
int         nsgpu_event_create(void **event);              /* hipEvent_t, for timing on a given stream */
int         nsgpu_event_destroy(void *event);
int         nsgpu_event_record(void *event, void *stream);
int         nsgpu_event_elapsed_ms(void *start, void *stop, float *ms);  /* synchronises `stop` */

/* ---------------- Time (src/core/model/nstime.h:388-439,586-589; int64x64-128.{h,cc}) ----------------
 * d_out[i] = Seconds (d_seconds[i]).GetTimeStep () at the default NS resolution, bit-exact
 * with the reference's 64.64 fixed point. */
int nsgpu_seconds_to_ts(const double *d_seconds, int64_t *d_out, int64_t n, void *stream);

/* ---------------- Broadcast-channel fan-out ----------------
 * Replaces the receiver loop of YansWifiChannel::Send (src/wifi/model/yans-wifi-channel.cc:77-115):
 * MobilityModel::GetDistanceFrom (mobility-model.cc:79-84), PropagationLossModel::CalcRxPower
 * (propagation-loss-model.cc:64-74) and ConstantSpeedPropagationDelayModel::GetDelay
 * (propagation-delay-model.cc:90-96) for every receiver in parallel.
 *
 * The phy list is SoA in HBM, in m_phyList (YansWifiChannel::Add) order.  One call handles
 * n_tx transmissions; transmission t writes its records at d_out + t * (nphy - 1) (survivors
 * first, in list order; the remaining slots of the stride are left untouched) and its survivor
 * count at d_count[t].  Record k of transmission t has uid = uid_base[t] + k — exactly the uids
 * ScheduleWithContext would hand out, since each survivor consumes one. */
typedef struct nsgpu_phy_soa {
  const double   *x, *y, *z;   /* positions (ConstantPositionMobilityModel), metres */
  const uint32_t *channel;     /* YansWifiPhy::GetChannelNumber () */
  const uint32_t *node;        /* NetDevice->GetNode ()->GetId (), 0xffffffff if none */
  /* Optional (both NULL: not given), built with the phy list by the caller: chan_rank[j] = how many
   * phys before j in m_phyList share j's channel, chan_count[j] = how many phys share it.  With them
   * nsgpu_fanout_yans places receiver records (and their uids) directly, without a counting pass; d_out
   * must then be 16-byte aligned.  The tables describe the channel numbers they were built from: rebuild
   * them whenever YansWifiChannel::Add changes m_phyList or a phy's channel number changes
   * (YansWifiPhy::SetChannelNumber, yans-wifi-phy.cc:328-358), or pass NULL (two-pass path) while stale. */
  const uint32_t *chan_rank;
  const uint32_t *chan_count;
} nsgpu_phy_soa;

typedef struct nsgpu_tx_desc {
  uint64_t now_ts;      /* Simulator::Now () of the Send call */
  double   tx_dbm;      /* txPowerDbm */
  uint32_t sender;      /* index of the sending phy in the list */
  uint32_t uid_base;    /* DefaultSimulatorImpl::m_uid at the Send call */
} nsgpu_tx_desc;

int nsgpu_fanout_yans(const nsgpu_phy_soa *phys, int64_t nphy, const nsgpu_tx_desc *d_tx, int64_t n_tx,
                      const nsgpu_loss_chain *loss, double speed,
                      nsgpu_rx_record *d_out, uint32_t *d_count, void *d_workspace, void *stream);

/* SingleModelSpectrumChannel::StartTx (src/spectrum/model/single-model-spectrum-channel.cc:106-183):
 * loss with tx = 0 dBm, receivers with -gain > max_loss_db are dropped before uid allocation
 * (compaction), survivors get d_psd_out[(t * (nphy-1) + k) * nbands + b] = psd_tx[t][b] * 10^(gain/10).
 * rx_dbm in the record holds the gain (dB).  speed <= 0 means no delay model (delay 0). */
int nsgpu_fanout_spectrum(const nsgpu_phy_soa *phys, int64_t nphy, const nsgpu_tx_desc *d_tx, int64_t n_tx,
                          const nsgpu_loss_chain *loss, double speed, double max_loss_db,
                          const double *d_psd_tx, int32_t nbands,
                          nsgpu_rx_record *d_out, double *d_psd_out, uint32_t *d_count,
                          void *d_workspace, void *stream);
int nsgpu_fanout_workspace_bytes(int64_t nphy, int64_t n_tx, uint64_t *bytes);

/* MultiModelSpectrumChannel::StartTx (src/spectrum/model/multi-model-spectrum-channel.cc:226-331) with
 * SpectrumConverter (spectrum-converter.cc).  The receivers are visited per rx SpectrumModel in ascending
 * model index (= SpectrumModelUid order of m_rxSpectrumModelInfoMap) and in AddRx order within a model:
 * d_iter[q] is the phy at visit position q, d_iter_pos its inverse (build both with the phy list, and again
 * whenever AddRx changes it).  d_rx_model[j]: phy j's rx model; d_tx_model[t] / d_psd_tx[t * max_bands + b]:
 * transmission t's PSD and its model.  The PSD is converted once per (transmission, rx model); each
 * survivor (-gain <= max_loss_db) gets a record as in nsgpu_fanout_spectrum (uid_base + rank in visit
 * order, rx_dbm = gain) and d_psd_out[(t * (nphy-1) + k) * max_bands + b] = converted[b] * 10^(gain/10)
 * for its model's bands.  d_trace (optional, [t * (nphy-1) + i]): the PropagationLoss trace call of every
 * non-sender receiver, in visit order, cut or not.  A single model with no conversion is
 * SingleModelSpectrumChannel::StartTx plus its trace.  Workspace: nsgpu_fanout_multi_workspace_bytes. */
int nsgpu_fanout_spectrum_multi(const nsgpu_phy_soa *phys, const int32_t *d_rx_model, const uint32_t *d_iter,
                                const uint32_t *d_iter_pos, int64_t nphy, const nsgpu_spectrum_models *models,
                                const nsgpu_tx_desc *d_tx, const int32_t *d_tx_model, const double *d_psd_tx,
                                int64_t n_tx, const nsgpu_loss_chain *loss, double speed, double max_loss_db,
                                nsgpu_rx_record *d_out, double *d_psd_out, nsgpu_loss_trace *d_trace,
                                uint32_t *d_count, void *d_workspace, void *stream);
int nsgpu_fanout_multi_workspace_bytes(int64_t nphy, int64_t n_tx, int32_t n_models, int32_t max_bands,
                                       uint64_t *bytes);

/* ---------------- Wi-Fi PHY receive subset (config 3) ----------------
 * Replaces, for a transmission schedule fixed before Run (nsgpu_wifi_scenario in nsgpu_types.h), the
 * event chain YansWifiPhy::SendPacket (src/wifi/model/yans-wifi-phy.cc:499-522) -> YansWifiChannel::Send
 * (yans-wifi-channel.cc:77-115) -> YansWifiChannel::Receive (:117-122) -> YansWifiPhy::StartReceivePacket
 * (yans-wifi-phy.cc:399-496) with InterferenceHelper (interference-helper.cc:129-212) and
 * WifiPhyStateHelper, and EndReceive's state part (yans-wifi-phy.cc:770-799).  The fan-out is fused into
 * the receive kernel.  Results equal a sequential DefaultSimulatorImpl run: uids, timestamps, decisions.
 *
 * nsgpu_wifi_create copies the scenario to HBM (host pointers; rx_log != 0 also keeps every Receive's
 * nsgpu_wifi_rx_log, n_tx * n_phy records).  nsgpu_wifi_run enqueues one whole run on `stream`
 * (asynchronous).  The readers synchronise with that stream and fail with NSGPU_ENOMEM / NSGPU_ESTATE
 * when the run hit a capacity (ni_cap, more than 64 transmissions within one arrival spread) or the
 * reference's fatal error (SendPacket while in TX). */
typedef struct nsgpu_wifi nsgpu_wifi;
int nsgpu_wifi_tx_duration_ns(uint32_t size, uint32_t modclass, uint64_t rate_bps, uint32_t bw_hz, uint32_t preamble,
                              int64_t *ns);  /* WifiPhy::CalculateTxDuration (wifi-phy.cc:141-296) */
int nsgpu_wifi_create(const nsgpu_wifi_scenario *sc, int rx_log, nsgpu_wifi **out);
int nsgpu_wifi_run(nsgpu_wifi *h, void *stream);
int nsgpu_wifi_get_stats(nsgpu_wifi *h, nsgpu_wifi_stats *out);
int nsgpu_wifi_read_phys(nsgpu_wifi *h, nsgpu_wifi_phy_counters *out);   /* n_phy */
int nsgpu_wifi_read_tx_base(nsgpu_wifi *h, uint32_t *out);               /* n_tx: uid base of each fan-out (0: after Stop) */
int nsgpu_wifi_read_ends(nsgpu_wifi *h, nsgpu_wifi_end_record *out, uint64_t cap, uint64_t *n);  /* unordered */
int nsgpu_wifi_read_rx_log(nsgpu_wifi *h, nsgpu_wifi_rx_log *out);        /* n_tx * n_phy */
int nsgpu_wifi_destroy(nsgpu_wifi *h);
/* Where a phy's InterferenceHelper::m_niChanges list lives (results are identical; the reference list's
 * order, length and ni_cap are kept either way):
 *   NSGPU_WIFI_STORE_LDS  two time-sorted queues per phy (start entries, end entries) in LDS, sized at
 *                         create from the schedule (the most transmissions on the air at one instant);
 *                         a run whose start queue overflows is repeated on the HBM ring by the readers;
 *   NSGPU_WIFI_STORE_HBM  one sorted ring per phy in HBM (ni_cap entries);
 *   NSGPU_WIFI_STORE_AUTO LDS when a block holds at least 8 phys' queues (the default).
 * Independently, the receptions (arrival, rxPowerW of every receiver x transmission pair: the fan-out
 * arithmetic) are computed up front into an HBM table by one parallel kernel when n_phy x transmissions
 * x 16 B fits half of the free HBM at create; | NSGPU_WIFI_INLINE_RX computes them inside the per-phy
 * kernel instead (same values: the same expressions).  When every transmission's arrivals can interleave
 * with at most 64 others' (arrivals lie within the grid's largest propagation delay of the send) and the
 * table fits twice more (32 B a pair), each phy's row is also put in dispatch order (arrival, uid) so the
 * per-phy chain reads its next Receive sequentially; | NSGPU_WIFI_UNSORTED_RX scans the unsorted row.
 * nsgpu_wifi_get_store reports the store the next run uses (| NSGPU_WIFI_INLINE_RX without the table,
 * | NSGPU_WIFI_UNSORTED_RX with the table but unsorted rows),
 * its phys per block and the end-queue (LDS) or ring (HBM) capacity. */
int nsgpu_wifi_set_store(nsgpu_wifi *h, int store);
/* Partitioned receive subset (the Wi-Fi split: every partition holds the transmissions — the
 * gathered Tx records — and runs its own receivers [phy_begin, phy_end); no all-to-all).  After the
 * receivers' chains the partitions' sync records are all-gathered and their counters and digest terms
 * all-reduced (RCCL on `comm`: nsgpu_wifi_run, one rank per GPU, synchronous), so every partition then hands
 * out the same EndReceive uids and reports the whole run's stats / ends / tx bases; nsgpu_wifi_read_phys and
 * the rx log hold the partition's own receivers.  comm = NULL makes a loopback member, run with the others of
 * its group on one device by nsgpu_wifi_group_run (tests).  Replaces no reference interface: the reference's
 * YansWifiChannel is not distributed (DistributedSimulatorImpl carries p2p links only). */
typedef struct nsgpu_comm nsgpu_comm;  /* RCCL communicator: nsgpu_comm_init below */
int nsgpu_wifi_create_dist(const nsgpu_wifi_scenario *sc, int rx_log, int64_t phy_begin, int64_t phy_end,
                           nsgpu_comm *comm, nsgpu_wifi **out);
int nsgpu_wifi_group_run(nsgpu_wifi **members, int n, void *stream);
int nsgpu_wifi_get_store(nsgpu_wifi *h, int *store, uint32_t *phys_per_block, uint32_t *e_cap);
/* Diagnostics: the kernels of one run and a run with each bracketed by HIP events (ms[k], k < count). */
int nsgpu_wifi_kernel_count(int *n);
const char *nsgpu_wifi_kernel_name(int k);
int nsgpu_wifi_profile(nsgpu_wifi *h, void *stream, double *ms);

/* ---------------- closed-loop Wi-Fi PHY (config 3 with the MAC on the host) ----------------
 * Replaces, for transmissions host closures start at run time (a MAC / DcfManager on the host that reads the
 * PHY state), YansWifiPhy::SendPacket (yans-wifi-phy.cc:499-522) -> YansWifiChannel::Send
 * (yans-wifi-channel.cc:77-115) -> StartReceivePacket (yans-wifi-phy.cc:399-496) -> EndReceive
 * (yans-wifi-phy.cc:770-799) with InterferenceHelper (interference-helper.cc:129-367: NiChanges, GetEnergyDuration,
 * CalculateSnrPer), the error-rate models (nist- / yans- / dsss-error-rate-model.cc) and WifiPhyStateHelper
 * (wifi-phy-state-helper.cc:122-183, 254-322, 391-423).  The device keeps every phy's state in HBM; the host
 * runtime (nsgpu_sim_attach_wifi) advances it to each host event's key.  Each EndReceive's (snr, per) comes
 * back for the host's m_random draw (yans-wifi-phy.cc:783; the PHY state does not depend on it). */
typedef struct nsgpu_wifil nsgpu_wifil;
int nsgpu_wifil_create(const nsgpu_wifil_config *cfg, nsgpu_wifil **out);
int nsgpu_wifil_destroy(nsgpu_wifil *h);
int nsgpu_wifil_receivers(nsgpu_wifil *h, uint32_t phy, uint32_t *n);  /* uids one SendPacket of phy takes */
/* SendPacket of phy from the closure running at `now`; its fan-out takes uids uid_base .. + receivers - 1 */
int nsgpu_wifil_send(nsgpu_wifil *h, uint64_t now, uint32_t uid_base, uint32_t phy, uint32_t size, double dbm,
                     uint32_t modclass, uint64_t rate, uint32_t bw, uint32_t preamble);
/* every device event with a key below (bound_ts, bound_uid) (~0: all): ranks from *dispatched, the syncs'
 * EndReceive uids from *uid, log entries (at their ranks, below log_cap) written.  The epoch's digest terms
 * are summed by kernels that run behind the next epochs (the order is not on the PHY's critical path): each
 * call adds to *digest the terms summed so far; nsgpu_wifil_flush adds the rest.  A direct caller MUST call
 * nsgpu_wifil_flush before reading the digest (until then it is partial, with no error); nsgpu_sim_run and
 * nsgpu_sim_host_stats flush by themselves.  NSGPU_ERANGE (the epoch's EndReceives would pass uid 0xfffffffe)
 * is returned before the epoch's ends, dispatch count or digest are published; the runtime makes it sticky. */
int nsgpu_wifil_advance(nsgpu_wifil *h, uint64_t bound_ts, uint32_t bound_uid, uint32_t *uid, uint64_t *dispatched,
                        uint64_t *digest, uint64_t *log_ts, uint32_t *log_uid, uint32_t *log_ctx, uint64_t log_cap);
int nsgpu_wifil_flush(nsgpu_wifil *h, uint64_t *digest);  /* waits for every epoch's order; adds its digest terms */
int nsgpu_wifil_get_state(nsgpu_wifil *h, uint32_t phy, uint64_t now, nsgpu_wifil_phy_state *out);
/* MobilityModel::SetPosition of phy's node (src/mobility/model/mobility-model.cc): the later SendPackets'
 * YansWifiChannel::Send fan-outs (yans-wifi-channel.cc:92-96) read the new position */
int nsgpu_wifil_set_position(nsgpu_wifil *h, uint32_t phy, double x, double y, double z);
int nsgpu_wifil_read_ends(nsgpu_wifil *h, nsgpu_wifil_end *out, uint64_t cap, uint64_t *n);  /* since last read */
int nsgpu_wifil_read_phys(nsgpu_wifil *h, nsgpu_wifi_phy_counters *out);                    /* n_phy */
int nsgpu_wifil_pending(nsgpu_wifil *h, uint64_t *n, uint64_t *next_ts);
/* The EndReceive hand-back (see nsgpu_sim_wifi_set_end_handler): phys whose EndReceives the host takes back, and
 * between advances the next one among them — a pending EndReceive that is not cancelled (found: its key and phy)
 * and ts_potential, the earliest time an EndReceive not yet scheduled could fall: a pending Receive strong enough
 * to sync (rxPowerW > the ED threshold, yans-wifi-phy.cc:461-471) ends at its arrival + duration (~0: none). */
typedef struct nsgpu_wifil_next {
  uint64_t ts;
  uint32_t uid, phy;
  int32_t found, pad_;
  uint64_t ts_potential;
} nsgpu_wifil_next;
int nsgpu_wifil_listen(nsgpu_wifil *h, uint32_t phy, int on);
/* YansWifiChannel::Send's ScheduleWithContext calls for one SendPacket of `sender` (yans-wifi-channel.cc:77-115),
 * host only: the receivers (every other phy on the sender's channel number, in m_phyList order), their Receive uids
 * (uid_base + place) and contexts (their device's node); *n = the count (entries past cap are not written). */
int nsgpu_wifil_send_plan(const nsgpu_wifil_config *cfg, uint32_t sender, uint32_t uid_base, uint32_t *rx_phy,
                          uint32_t *rx_uid, uint32_t *rx_ctx, uint64_t cap, uint64_t *n);
int nsgpu_wifil_next_end(nsgpu_wifil *h, nsgpu_wifil_next *out);
/* Partitioned closed-loop PHY (YansWifiChannel::Send, yans-wifi-channel.cc:77-115, fans a SendPacket out to
 * every receiver; the receivers are split over GPUs).  Every rank runs the same host program (MAC closures, uids,
 * GetState) over the returned handle, which takes every nsgpu_wifil_* call above; the device work of phys
 * [phy_begin, phy_end) — their Receives, InterferenceHelper, state machine, EndReceive — runs on this rank.  Per epoch
 * the ranks all-gather (RCCL on comm, one rank per GPU) the syncs (EndReceive uids = ranks among every rank's syncs),
 * the counters, end records and phy state fields, and the dispatched events (ordered once for digest and log): every
 * rank then returns what the single engine returns.  The ranks' ranges must tile [0, n_phy) in rank order.  A loopback
 * group (nsgpu_wifil_create_group: partitions [bounds[q], bounds[q+1]), q < n, all on this device, exchanging through
 * device copies) is the same split in one process (tests).  Replaces no reference interface: YansWifiChannel is not
 * distributed in the reference (DistributedSimulatorImpl carries p2p links only). */
int nsgpu_wifil_create_dist(const nsgpu_wifil_config *cfg, int64_t phy_begin, int64_t phy_end, nsgpu_comm *comm,
                            nsgpu_wifil **out);
int nsgpu_wifil_create_group(const nsgpu_wifil_config *cfg, const int64_t *bounds, int n, nsgpu_wifil **out);

/* ---------------- GPU-resident bench-simulator churn (config 1) ----------------
 * Runs utils/bench-simulator.cc's RunBench + Simulator::Run (bench-simulator.cc:79-127) over
 * MapScheduler order entirely on the device: n initial events Schedule (NanoSeconds (d[i])),
 * each dispatch k <= total schedules a child at now + d[k mod n].  Pop order is bit-exact;
 * it is reported as counters, an order-sensitive digest and (optionally) the full pop log. */
typedef struct nsgpu_hold_stats {
  uint64_t dispatched;   /* RemoveNext calls */
  uint64_t holds;        /* Bench::m_n */
  uint64_t final_ts;     /* ts of the last dispatched event */
  uint64_t digest;       /* sum_k nsgpu_dispatch_digest_term (k, ts_k, uid_k) */
  uint64_t rounds;       /* device rounds (parallel dispatch batches) */
  uint32_t max_batch;    /* largest batch dispatched in one round */
  uint32_t next_uid;     /* DefaultSimulatorImpl::m_uid after the run */
} nsgpu_hold_stats;

int nsgpu_hold_workspace_bytes(uint32_t n, uint64_t *bytes);
/* Diagnostic: when d_phase_cycles (7 x uint64, device) is non-NULL, later nsgpu_hold_run calls
 * record per-round-phase s_memtime cycle sums there (NULL turns it off). */
int nsgpu_hold_set_profile(uint64_t *d_phase_cycles);
int nsgpu_hold_run(const uint64_t *d_dist, uint32_t n, uint32_t total, nsgpu_hold_stats *d_stats,
                   uint64_t *d_log_ts, uint32_t *d_log_uid, uint64_t log_cap, void *d_workspace, void *stream);

/* ---------------- HipBatchScheduler (host closures) ----------------
 * The ns3::Scheduler interface (src/core/model/scheduler.h:75-97) — Insert, IsEmpty, PeekNext,
 * RemoveNext, Remove — with MapScheduler's (ts, uid) order (map-scheduler.cc:51-100).  Pending
 * events are kept sorted in HBM; staged inserts are sorted and merged on the device in bulk and
 * the next `batch` events are popped to the host in one copy.  `handle` is the caller's EventImpl*
 * (never dereferenced).  ns3::HipBatchScheduler forwards to these. */
typedef struct nsgpu_sched nsgpu_sched;
int nsgpu_sched_create(uint32_t batch, void *stream, nsgpu_sched **out);
int nsgpu_sched_destroy(nsgpu_sched *s);
int nsgpu_sched_insert(nsgpu_sched *s, const nsgpu_event *ev, uint64_t n);
int nsgpu_sched_is_empty(nsgpu_sched *s, int *empty);
int nsgpu_sched_size(nsgpu_sched *s, uint64_t *n);
int nsgpu_sched_peek_next(nsgpu_sched *s, nsgpu_event *out);
int nsgpu_sched_remove_next(nsgpu_sched *s, nsgpu_event *out);
int nsgpu_sched_remove(nsgpu_sched *s, const nsgpu_event *ev);
/* front machinery statistics: refills so far, current front size, running refill wall-time estimate */
int nsgpu_sched_stats(nsgpu_sched *s, uint64_t *refills, uint64_t *front, double *refill_us);

/* ---------------- HipSimulatorImpl host runtime (host closures) ----------------
 * Replaces DefaultSimulatorImpl's run loop (default-simulator-impl.cc:117-165) for events whose
 * closures stay on the host, keeping its semantics (:49-353: uid from 4, ScheduleDestroy consumes a
 * uid, IsExpired rule, cancelled events still dequeued, Stop/Stop (Time)).  Events live in the
 * HipBatchScheduler and are dispatched in WINDOWS (nsgpu_sim_pop_window, SURVEY 8(b)'s
 * nsgpu_pop_window): every pending event of the smallest timestamp, or — with a GPU-resident p2p engine
 * attached (nsgpu_sim_attach_p2p) — the next host event after the engine has dispatched every device
 * event before it, in one (ts, uid) order.  Two ways to use it:
 *   - C callbacks: nsgpu_sim_schedule* + nsgpu_sim_run;
 *   - raw handles (ns3::HipSimulatorImpl, the handle being an EventImpl*): nsgpu_sim_insert, then
 *     nsgpu_sim_pop_window / nsgpu_sim_begin per event (handles come back with bit 0 set).
 * INTEGRATION.md shows the ns-3 side. */
typedef void (*nsgpu_event_fn)(void *user, uint64_t arg);
typedef struct nsgpu_sim nsgpu_sim;
typedef struct nsgpu_p2p nsgpu_p2p;
int nsgpu_sim_create(uint32_t batch, void *stream, nsgpu_sim **out);
int nsgpu_sim_free(nsgpu_sim *s);
int nsgpu_sim_schedule(nsgpu_sim *s, int64_t delay, nsgpu_event_fn fn, void *user, uint64_t arg, nsgpu_event_id *id);
int nsgpu_sim_schedule_with_context(nsgpu_sim *s, uint32_t ctx, int64_t delay, nsgpu_event_fn fn, void *user,
                                    uint64_t arg);
int nsgpu_sim_schedule_now(nsgpu_sim *s, nsgpu_event_fn fn, void *user, uint64_t arg, nsgpu_event_id *id);
int nsgpu_sim_schedule_destroy(nsgpu_sim *s, nsgpu_event_fn fn, void *user, uint64_t arg, nsgpu_event_id *id);
int nsgpu_sim_is_expired(nsgpu_sim *s, const nsgpu_event_id *id, int *expired);
int nsgpu_sim_cancel(nsgpu_sim *s, const nsgpu_event_id *id);
int nsgpu_sim_remove(nsgpu_sim *s, const nsgpu_event_id *id);
int nsgpu_sim_run(nsgpu_sim *s);
int nsgpu_sim_stop(nsgpu_sim *s);
int nsgpu_sim_stop_at(nsgpu_sim *s, int64_t delay);
int nsgpu_sim_destroy(nsgpu_sim *s);
int nsgpu_sim_state(nsgpu_sim *s, uint64_t *now, uint32_t *context, uint64_t *dispatched, uint32_t *next_uid);
int nsgpu_sim_current_uid(nsgpu_sim *s, uint32_t *uid);
/* m_uid before anything is scheduled (default 4, default-simulator-impl.cc:52-56): the uids below it count as
 * consumed by Schedule calls this runtime did not see.  Every Schedule* / ScheduleDestroy that would take uid
 * 0xffffffff (or a wrapped one) fails with NSGPU_ERANGE, as do the attached engines' allocations. */
int nsgpu_sim_set_next_uid(nsgpu_sim *s, uint32_t uid);
int nsgpu_sim_next(nsgpu_sim *s, uint64_t *ts, int *empty);          /* Next (): host and device events */
int nsgpu_sim_is_finished(nsgpu_sim *s, int *finished);              /* IsFinished (): empty || stopped */
int nsgpu_sim_set_stop(nsgpu_sim *s, int stop);                      /* Stop (); Run clears it */
int nsgpu_sim_run_one(nsgpu_sim *s);                                 /* RunOneEvent () (callbacks) */
int nsgpu_sim_live_closures(nsgpu_sim *s, uint64_t *n);              /* callback closures still held */
int nsgpu_sim_drain(nsgpu_sim *s, nsgpu_event *out, uint32_t cap, uint32_t *n);  /* DoDispose */
/* windows: *n = 0 when nothing is left to dispatch or a Stop was dispatched */
int nsgpu_sim_pop_window(nsgpu_sim *s, nsgpu_event *out, uint32_t cap, uint32_t *n);
/* window event *e is dispatched next: *skip = 0 run it (Now/Context/uid set, dispatch counted), 1 a
 * closure of this window removed it, 2 a Stop was dispatched before it (it stays pending) */
int nsgpu_sim_begin(nsgpu_sim *s, const nsgpu_event *e, int *skip);
/* RunOneEvent (default-simulator-impl.cc:167-170): the next event as a one-event window, whatever
 * the stop flag says (*n = 0: nothing pending) */
int nsgpu_sim_pop_one(nsgpu_sim *s, nsgpu_event *out, uint32_t *n);
/* raw handles: handle must be even (an object pointer); *uid = the uid it got (ScheduleWithContext
 * order); remove_key: Scheduler::Remove of a pending event; key_expired: IsExpired's time rule */
int nsgpu_sim_insert(nsgpu_sim *s, uint64_t ts, uint32_t ctx, uint64_t handle, uint32_t *uid);
int nsgpu_sim_consume_uid(nsgpu_sim *s, uint32_t *uid);
int nsgpu_sim_remove_key(nsgpu_sim *s, uint64_t ts, uint32_t uid, uint32_t ctx, uint64_t handle);
int nsgpu_sim_key_expired(nsgpu_sim *s, uint64_t ts, uint32_t uid, int *expired);
/* the destroy list of raw handles (DefaultSimulatorImpl::m_destroyEvents, default-simulator-impl.cc
 * :79-92,235-242,256-268,306-322), kept by the runtime; the caller keeps the reference each entry
 * holds.  insert = ScheduleDestroy (consumes a uid; *ts = Now, the EventId's ts); pop = Destroy's
 * front + pop_front (*found = 0: the list is empty — call it until then, since a destroy closure may
 * schedule or remove destroy events); remove = Remove of a uid-2 EventId; pending = IsExpired's list
 * lookup. */
int nsgpu_sim_destroy_insert(nsgpu_sim *s, uint64_t handle, uint64_t *ts);
int nsgpu_sim_destroy_pop(nsgpu_sim *s, uint64_t *handle, int *found);
int nsgpu_sim_destroy_remove(nsgpu_sim *s, uint64_t handle, uint64_t ts, int *found);
int nsgpu_sim_destroy_pending(nsgpu_sim *s, uint64_t handle, uint64_t ts, int *pending);
/* dispatch accounting of the host events (the engine accounts for the device ones): count, cancelled
 * ones, digest (sum of nsgpu_dispatch_digest_term over their global ranks); optional log at global ranks */
int nsgpu_sim_host_stats(nsgpu_sim *s, uint64_t *host_dispatched, uint64_t *cancelled, uint64_t *digest);
/* the runtime's host-closure queue (a HipBatchScheduler): refills of its front batch, events served from
 * the front, time spent refilling (nsgpu_sched_stats) */
int nsgpu_sim_sched_stats(nsgpu_sim *s, uint64_t *refills, uint64_t *front, double *refill_us);
int nsgpu_sim_set_log(nsgpu_sim *s, uint64_t *ts, uint32_t *uid, uint32_t *ctx, uint64_t cap);
/* mixed host / device runs: the engine's events join this runtime's order (attach before scheduling;
 * the runtime continues from the engine's post-setup uid); a closure may make one of the engine's
 * OnOff applications send a datagram now (UdpSocket::Send from a host application) */
int nsgpu_sim_attach_p2p(nsgpu_sim *s, nsgpu_p2p *h);
/* the same after setup (ns3::HipSimulatorImpl::AdoptDeviceSubset): the program built its topology with the
 * stock helpers, whose setup-time Schedule calls took uids 4.. in this runtime; the engine was created with
 * a setup list mirroring them (NsgpuP2pScenario::FromNodeList) and the caller removed the host events the
 * engine now dispatches (nsgpu_sim_remove_key).  Host events that remain (the program's own) keep their
 * uids; nothing may have been dispatched yet, and the engine's post-setup uid must equal this runtime's. */
int nsgpu_sim_adopt_p2p(nsgpu_sim *s, nsgpu_p2p *h);
int nsgpu_sim_p2p_send(nsgpu_sim *s, uint32_t app);
/* the closed-loop Wi-Fi PHY: its events join this runtime's order (one host event per window after the
 * PHY's events before it); a closure's SendPacket (now, the runtime's next uids) and GetState (now) */
int nsgpu_sim_attach_wifi(nsgpu_sim *s, nsgpu_wifil *h);
int nsgpu_sim_wifi_send(nsgpu_sim *s, uint32_t phy, uint32_t size, double dbm, uint32_t modclass, uint64_t rate,
                        uint32_t bw, uint32_t preamble);
int nsgpu_sim_wifi_state(nsgpu_sim *s, uint32_t phy, nsgpu_wifil_phy_state *out);
/* a host closure's MobilityModel::SetPosition of phy's node (nsgpu_wifil_set_position on the attached PHY) */
int nsgpu_sim_wifi_set_position(nsgpu_sim *s, uint32_t phy, double x, double y, double z);
/* EndReceive hand-back (YansWifiPhy::EndReceive, yans-wifi-phy.cc:770-799): for every phy marked with
 * nsgpu_sim_wifi_listen, the runtime stops the device AT each of the phy's EndReceives (the event itself runs on
 * the device: CalculateSnrPer, the state switch) and calls fn (user, &end) right there in the (ts, uid) order,
 * with Now () = its time, the current uid = its uid and the context = the phy's node — where the reference makes
 * its m_random draw (:783) and calls the MAC (SwitchFromRxEndOk / Error -> the receive callbacks), so the
 * callback's Schedule / SendPacket calls take the uids and times the reference's would.  A cancelled EndReceive
 * (a SendPacket during RX, :504-508) is dispatched without a call, as the reference's cancelled EventImpl.  An
 * EndReceive scheduled inside an epoch is caught too: the runtime never advances past the earliest time a pending
 * Receive of a listened phy could end (nsgpu_wifil_next_end's ts_potential) before it knows whether it synced. */
typedef void (*nsgpu_wifi_end_fn)(void *user, const nsgpu_wifil_end *end);
int nsgpu_sim_wifi_set_end_handler(nsgpu_sim *s, nsgpu_wifi_end_fn fn, void *user);
int nsgpu_sim_wifi_listen(nsgpu_sim *s, uint32_t phy, int on);

/* ---------------- GPU-resident point-to-point subset (configs 2, 4) ----------------
 * Replaces, for a topology of PointToPointNetDevices, the handler chain
 *   PointToPointNetDevice::{Send,TransmitStart,TransmitComplete,Receive} (point-to-point-net-device.cc:206-346,462-518)
 *   PointToPointChannel::TransmitStart (point-to-point-channel.cc:82-103)
 *   Queue/DropTailQueue::{Enqueue,Dequeue,Drop} (queue.cc:61-200, drop-tail-queue.cc:83-132)
 *   Ipv4L3Protocol::{Receive,IpForward} with static next-hop routes (ipv4-l3-protocol.cc:434-537,815-841)
 *   UdpL4Protocol::Receive -> PacketSink, OnOffApplication (onoff-application.cc:132-252)
 * and the DefaultSimulatorImpl run loop over them, entirely on the device.  nsgpu_p2p_reset
 * loads the post-setup state; nsgpu_p2p_run runs Simulator::Run to the Stop event and returns when it
 * is done (graph replays of the window pipeline on an engine stream, ordered after `stream`). */
int nsgpu_p2p_create(const nsgpu_p2p_scenario *sc, uint64_t pool_cap, uint64_t log_cap, nsgpu_p2p **out);
int nsgpu_p2p_reset(nsgpu_p2p *h, void *stream);
int nsgpu_p2p_run(nsgpu_p2p *h, void *stream);
int nsgpu_p2p_results(nsgpu_p2p *h, nsgpu_p2p_stats *stats, nsgpu_dev_counters *devc, nsgpu_app_counters *appc,
                      uint64_t *log_ts, uint32_t *log_uid, uint32_t *log_ctx, uint64_t log_n, uint32_t *error,
                      void *stream);
int nsgpu_p2p_destroy(nsgpu_p2p *h);
/* GPU time (ms, HIP events on the engine stream) of the last nsgpu_p2p_run. */
int nsgpu_p2p_last_run_ms(nsgpu_p2p *h, double *gpu_ms);
/* 1: the engine runs wide windows — bounded by the cross-node lookahead (min over devices of the smallest
 * frame's tx time + channel delay), a same-node TransmitComplete before the window's end running inside
 * it.  Single engines whose nodes have at most 16 devices, unless NSGPU_P2P_NARROW=1 was
 * set when the engine was created. */
int nsgpu_p2p_get_wide(nsgpu_p2p *h, int *wide);
/* Launch mode of nsgpu_p2p_run: 0 = hipGraph replays (default), 1 = the same kernels launched one by
 * one (also selected by the environment variable NSGPU_P2P_EAGER; used under rocprofv3). */
int nsgpu_p2p_set_eager(nsgpu_p2p *h, int eager);
/* Ascii/pcap trace records (SURVEY 8(b) nsgpu_trace_drain; replaces the trace sinks that
 * PointToPointHelper::EnableAsciiAll / EnablePcapAll hook, point-to-point-helper.cc:81-219 and
 * trace-helper.cc:303-390): nsgpu_p2p_set_trace gives the engine a device buffer of `cap`
 * nsgpu_trace_record (call before the first run; a group member before nsgpu_p2p_group_create);
 * every run then records each Enqueue / Dequeue / Drop / MacRx sink call, unordered (trace order is
 * (ts, uid, seq)).  nsgpu_p2p_trace_read copies up to `cap` records of the last run and sets *n to
 * the number the run made (NSGPU_ENOMEM when that exceeds the buffer or `cap`). */
int nsgpu_p2p_set_trace(nsgpu_p2p *h, uint64_t cap);
/* The sinks recorded: bit k = nsgpu_trace_kind k.  Default 0xf (the device sinks above); 0x70 adds the
 * Ipv4L3Protocol Tx / Rx / Drop sinks InternetStackHelper::EnableAsciiIpv4All hooks
 * (internet-stack-helper.cc:593-730).  Call before nsgpu_p2p_run (a group member: before
 * nsgpu_p2p_group_create). */
int nsgpu_p2p_set_trace_kinds(nsgpu_p2p *h, uint32_t mask);
int nsgpu_p2p_trace_read(nsgpu_p2p *h, nsgpu_trace_record *out, uint64_t cap, uint64_t *n, void *stream);
/* The window pipeline's kernels: count and names (launch order). */
int nsgpu_p2p_kernel_count(int *n);
const char *nsgpu_p2p_kernel_name(int k);
/* Per-kernel device time of one full run (from the state nsgpu_p2p_reset loaded): in every
 * sample_every-th window each kernel is launched with start / stop HIP events that the command
 * processor records at the kernel's own start and end (hipExtLaunchKernel); kernel_ms[k] and
 * launches[k] (nsgpu_p2p_kernel_count entries) accumulate the bracketed time and launch count. */
int nsgpu_p2p_profile(nsgpu_p2p *h, void *stream, uint32_t sample_every, double *kernel_ms, uint64_t *launches);
/* The latency constants of the window pipeline's roofline (diagnostic, not a reference interface): a
 * kernel boundary (back-to-back launches of an empty 64-block kernel, graph-replayed: us per kernel) and
 * one dependent global-memory trip (a pointer chase with random jumps through a 128-MB table, every level a
 * line no L2 holds: us per level). */
int nsgpu_probe_latency(void *stream, double *boundary_us, double *trip_us);
/* Mixed host / device runs (driven by nsgpu_sim, see above): the uid the program's own Schedule calls
 * start from (after the setup-time ones); advance = dispatch every device event with a key below
 * (hts, huid) (hts = UINT64_MAX: all of them), with *uid / *dispatched the global uid counter and
 * dispatch count in and out; *ended = 1 when the run is over (Simulator::Stop reached, or nothing
 * pending on the device and no host key).  inject_send: while paused, application `app` (an OnOff
 * flow) sends one datagram at `now` on behalf of the host closure with uid cur_uid and context cur_ctx
 * (its Schedule calls inherit the context; its trace calls continue from *trace_seq).  counters: the device / application counters at this point. */
int nsgpu_p2p_setup_uid(nsgpu_p2p *h, uint32_t *uid);
int nsgpu_p2p_advance(nsgpu_p2p *h, uint64_t hts, uint32_t huid, uint32_t *uid, uint64_t *dispatched, int *ended,
                      void *stream);
int nsgpu_p2p_inject_send(nsgpu_p2p *h, uint32_t app, uint64_t now, uint32_t cur_uid, uint32_t cur_ctx,
                          uint32_t *uid, uint32_t *trace_seq, void *stream);
int nsgpu_p2p_counters(nsgpu_p2p *h, nsgpu_dev_counters *devc, nsgpu_app_counters *appc, void *stream);
/* the engine's pending device events between advances: count, smallest timestamp (UINT64_MAX: none),
 * and whether a device-dispatched Simulator::Stop ended its run */
int nsgpu_p2p_pending(nsgpu_p2p *h, uint64_t *n, uint64_t *next_ts, int *stopped, void *stream);
/* Diagnostic: in-kernel phase timers (s_memrealtime ticks, 100 MHz) of the pipeline kernels; only the
 * lib/libnsgpu_prof.so build (-DNSGPU_PHASE_PROF) records them, the product library returns ESTATE. */
int nsgpu_p2p_phase_read(uint64_t *out, int n, int reset);

/* ---------------- global routing ----------------
 * Replaces GlobalRouteManager::PopulateRoutingTables (SPFCalculate, global-route-manager-impl.cc:
 * 1327-1490) + Ipv4GlobalRouting::LookupGlobal (ipv4-global-routing.cc:136-242, RandomEcmpRouting off)
 * for point-to-point topologies with unit metrics: route_out[node * n_dst + k] (host memory) = the device
 * through which `node` forwards a datagram to any address of node dst_node[k]; 0xffffffff for the
 * destination itself and for unreachable nodes — except that a node with exactly one device always
 * forwards through it, reachable or not (GlobalRouter's stub-node default route, CheckForStubNode,
 * global-route-manager-impl.cc:1245-1290,1363-1366).  dev_addr / dev_ifindex: each device's IPv4 address and
 * interface index (both NULL: the lowest device wins ties).  One GPU BFS per destination. */
int nsgpu_route_global(uint32_t n_nodes, uint32_t n_devices, const uint32_t *dev_node, const uint32_t *dev_peer,
                       const uint32_t *dev_addr, const uint32_t *dev_ifindex, uint32_t n_dst, const uint32_t *dst_node,
                       uint32_t *route_out, void *stream);

/* ---------------- partitioned (multi-GPU) point-to-point runs ----------------
 * Replaces src/mpi's DistributedSimulatorImpl (distributed-simulator-impl.cc:146-326: LBTS by
 * MPI_Allgather of LbtsMessage) and MpiInterface::SendPacket / ReceiveMessages
 * (mpi-interface.cc:414-506: remote packets) for the GPU-resident p2p subset: one process per GPU,
 * node n simulated by rank node_owner[n] (Node::GetSystemId, node.cc:76-108).  Per window an RCCL
 * allgather of window bounds (X0), an allgather of window summaries — the LBTS and the global
 * dispatch order (X1) — and an all-to-all of remote events (X2), captured into the window graph.
 * The run reproduces the SEQUENTIAL DefaultSimulatorImpl pop order and uids (not the per-rank uids
 * of DistributedSimulatorImpl).  dispatched / final_ts / next_uid / windows in nsgpu_p2p_results are
 * run-global; digest and drop counters are this rank's share; counters are valid for owned nodes,
 * and the log holds the entries this rank dispatched (zeros elsewhere). */
int nsgpu_comm_unique_id(uint8_t *id);   /* 128 bytes, rank 0; share it with every rank */
int nsgpu_comm_init(const uint8_t *id, int nranks, int rank, nsgpu_comm **out);  /* on the rank's device */
int nsgpu_comm_destroy(nsgpu_comm *c);
/* comm == NULL: a loopback member (all partitions in one process on one device, see below). */
int nsgpu_p2p_create_dist(const nsgpu_p2p_scenario *sc, const uint32_t *node_owner, int rank, int nranks,
                          nsgpu_comm *comm, uint64_t pool_cap, uint64_t log_cap, nsgpu_p2p **out);
/* The constants a rank's partitioned engine is built from, computed on the host (no device, no communicator):
 * what nsgpu_p2p_create_dist derives from the scenario and the owner map (the same code: create_engine runs it
 * first).  Every field except n_init and pool_cap must be equal on every rank — the exchanges' sizes (X0 / X1 /
 * X2 bytes, X2 records per peer), the window capacities and the lookaheads that bound every window; ranks that
 * disagree would call collectives of different sizes, an RCCL hang no single process can see (the reference
 * sizes its LBTS messages and per-peer buffers the same way on every rank: distributed-simulator-impl.cc:146-216,
 * mpi-interface.cc:385-445).  node_owner == NULL: the single engine's plan (the exchange fields are 0). */
typedef struct nsgpu_p2p_plan {
  uint32_t wide;                /* wide windows (same-node TransmitCompletes inside the window) */
  uint32_t maxc;                /* children per event record */
  uint32_t wcap, xlcap;         /* gen-0 window records / local records of one rank's window */
  uint64_t x0_bytes;            /* X0 all-gather: bytes per rank */
  uint64_t x1_bytes;            /* X1 all-gather: bytes per rank */
  uint64_t x2_bytes;            /* X2 all-to-all: bytes per peer */
  uint32_t x2_records;          /* X2 event records per peer per window */
  uint32_t n_kinds;             /* entries of lookahead / lookw in use */
  int64_t lookahead[16];        /* narrow lookahead per event kind (ns) */
  int64_t lookw[16];            /* wide lookahead per event kind (ns; partitioned: capped below 3 tx_min) */
  int64_t tx_min, lx;           /* smallest transmission time; smallest cross-node delay (tx + channel) */
  uint64_t red0_tmin, red0_wend, red0_wendw;  /* window 0's bound: the whole setup's reduction */
  uint64_t stop_ts;             /* Simulator::Stop's time (~0: none) */
  uint32_t stop_uid, uid_init;  /* Stop's uid; m_uid after setup */
  uint32_t n_init, pad;         /* this rank's setup events (per rank) */
  uint64_t pool_cap;            /* this rank's pending pool (per rank: follows n_init unless given) */
} nsgpu_p2p_plan;
int nsgpu_p2p_dist_plan(const nsgpu_p2p_scenario *sc, const uint32_t *node_owner, int rank, int nranks,
                        uint64_t pool_cap, nsgpu_p2p_plan *out);
/* Loopback group: partitions 0..n-1 (created with comm == NULL) run on this device with the
 * collectives replaced by device-to-device copies — the partitioned algorithm on one GPU. */
typedef struct nsgpu_p2p_group nsgpu_p2p_group;
int nsgpu_p2p_group_create(nsgpu_p2p **members, int n, nsgpu_p2p_group **out);
int nsgpu_p2p_group_reset(nsgpu_p2p_group *g, void *stream);
int nsgpu_p2p_group_run(nsgpu_p2p_group *g, void *stream);
int nsgpu_p2p_group_destroy(nsgpu_p2p_group *g);

/* ---- setup journal -> setup list (NsgpuP2pScenario::FromNodeList's uid-critical part) ----
 * Every Schedule* / ScheduleDestroy / Stop (t) call a program makes before Run consumes one uid
 * (default-simulator-impl.cc:188-242), so the engine's setup list (nsgpu_p2p_scenario.setup_kind / setup_index)
 * must hold one entry per call, in call order.  HipSimulatorImpl journals each call, classified when it is
 * made: the stock start calls (NodeListPriv::Add -> Node::Start, src/network/model/node-list.cc:124-131;
 * Node::AddDevice -> NetDevice::Start and Node::AddApplication -> Application::Start, node.cc:111-145, each
 * with the index the object got on its node) are told apart from the program's own events by the closure's
 * type, so an application added before a later link, or a program's own ts-0 event with a node context, maps
 * to the right object.  This function checks the journal against the node list (each node started once
 * before its devices and applications, their indices in AddDevice / AddApplication order, every one started)
 * and returns the setup list, the journal entries the engine takes over, and which node-local device /
 * application each engine device / application is.  Anything inconsistent is NSGPU_EINVAL, never a shifted
 * uid. */
enum nsgpu_journal_kind {
  NSGPU_J_CALL = 0,          /* any other Schedule* (the program's own event): a consumed uid, kept on the host */
  NSGPU_J_DESTROY = 1,       /* ScheduleDestroy */
  NSGPU_J_STOP = 2,          /* Simulator::Stop (t): Schedule (t, &Simulator::Stop), simulator.cc:168-172 */
  NSGPU_J_NODE_START = 3,    /* ScheduleWithContext (k, 0, &Node::Start, node) */
  NSGPU_J_DEVICE_START = 4,  /* ScheduleWithContext (node, 0, &NetDevice::Start, device) */
  NSGPU_J_APP_START = 5      /* ScheduleWithContext (node, 0, &Application::Start, application) */
};
typedef struct nsgpu_journal_entry {
  uint64_t ts;       /* the event's timestamp (ns) */
  uint32_t context;  /* its context (0xffffffff: none) */
  uint32_t kind;     /* nsgpu_journal_kind */
  uint32_t local;    /* DEVICE_START: the node's GetNDevices () - 1 at the call; APP_START: GetNApplications () - 1 */
  uint32_t pad_;
} nsgpu_journal_entry;  /* 24 bytes */
enum nsgpu_node_device_kind { NSGPU_NDEV_P2P = 0, NSGPU_NDEV_LOOPBACK = 1, NSGPU_NDEV_OTHER = 2 };
typedef struct nsgpu_setup_map {
  /* caller-allocated outputs */
  uint32_t *setup_kind, *setup_index;  /* n (one per journal entry): the engine's setup list */
  uint32_t *owned;                     /* n: the journal entries the engine dispatches (the rest stay on the host) */
  uint32_t *dev_node, *dev_local;      /* node_dev_off[n_nodes]: engine device d is dev_node[d]'s device dev_local[d] */
  uint32_t *app_node, *app_local;      /* sum of node_n_apps: engine application a likewise */
  uint64_t n_owned;
  uint32_t n_devices, n_apps;          /* engine devices (point-to-point) and applications */
  int64_t stop_ns;                     /* Simulator::Stop's time, -1: none */
} nsgpu_setup_map;
/* node_dev_off[n_nodes + 1]: CSR of each node's devices in AddDevice order; node_dev_kind: their
 * nsgpu_node_device_kind (NSGPU_NDEV_OTHER fails: not in the GPU-resident subset); node_n_apps: each node's
 * GetNApplications () */
int nsgpu_setup_from_journal(const nsgpu_journal_entry *j, uint64_t n, uint32_t n_nodes, const uint64_t *node_dev_off,
                             const uint32_t *node_dev_kind, const uint32_t *node_n_apps, nsgpu_setup_map *out);

/* ---- trace codec (replaces the default sinks' formatting for GPU-resident events) ----
 * nsgpu_trace_record streams -> the bytes ns-3's default ascii / pcap sinks write:
 * AsciiTraceHelper::Default{Enqueue,Dequeue,Drop,Receive}SinkWithContext (src/network/helper/trace-helper.cc:
 * 303-390) through Packet::Print (src/network/model/packet.cc:427-476), InternetStackHelper's Ipv4 Tx / Rx /
 * Drop lines (src/internet/helper/internet-stack-helper.cc:650-730), and the PromiscSniffer pcap records
 * (src/point-to-point/helper/point-to-point-helper.cc:81-110 -> PcapFileWrapper::Write,
 * src/network/utils/pcap-file.cc:300-381).  ns3::HipSimulatorImpl hands nsgpu_trace_line's text to the
 * helper's OutputStreamWrapper and nsgpu_trace_packet's bytes to PcapFileWrapper::Write (Time, buffer,
 * length).  Output functions: out == NULL only sets *len (the size); otherwise cap must hold *len bytes. */
typedef struct nsgpu_trace_addressing {
  const uint32_t *dev_addr;         /* n_devices: the IPv4 address of the device's interface (0: none) */
  const uint32_t *dev_ip_ifindex;   /* n_devices: its Ipv4 interface index (loopback 0, then Assign order) */
  const uint32_t *app_remote_addr;  /* n_apps: the Remote address of a sender (0: the destination node's first
                                     * interface) */
  const uint32_t *app_remote_port;  /* n_apps: the Remote port of a sender */
} nsgpu_trace_addressing;
typedef struct nsgpu_trace_codec nsgpu_trace_codec;
int nsgpu_trace_codec_create(const nsgpu_p2p_scenario *sc, const nsgpu_trace_addressing *ad, nsgpu_trace_codec **out);
int nsgpu_trace_codec_free(nsgpu_trace_codec *c);
/* Time::GetSeconds () of ts ns (the ascii sinks' timestamp): int64x64_t MulByInvert (Invert (1e9)) then
 * GetDouble, src/core/model/nstime.h:419-431, int64x64-128.cc:94-134, int64x64-128.h:83-95 — not ts / 1e9 */
double nsgpu_time_get_seconds(int64_t ts);
/* trace order: the dispatching event's (ts, uid), then the call order inside it (seq) */
int nsgpu_trace_sort(nsgpu_trace_record *rec, uint64_t n);
int nsgpu_trace_line(const nsgpu_trace_codec *c, const nsgpu_trace_record *r, char *out, uint64_t cap, uint64_t *len);
int nsgpu_trace_packet(const nsgpu_trace_codec *c, const nsgpu_trace_record *r, uint8_t *out, uint64_t cap,
                       uint64_t *len);  /* the serialized packet the sniffer sees (PPP header included) */
int nsgpu_trace_ascii(const nsgpu_trace_codec *c, const nsgpu_trace_record *rec, uint64_t n, char *out, uint64_t cap,
                      uint64_t *len);   /* every record's line (EnableAsciiAll / EnableAsciiIpv4All on one stream) */
int nsgpu_trace_pcap(const nsgpu_trace_codec *c, const nsgpu_trace_record *rec, uint64_t n, uint32_t dev, uint8_t *out,
                     uint64_t cap, uint64_t *len);  /* device dev's pcap file (EnablePcapAll) */
/* ---- Wi-Fi sniffer records (YansWifiPhyHelper's sinks for the GPU-resident PHY) ----
 * YansWifiPhy calls MonitorSnifferTx in SendPacket (src/wifi/model/yans-wifi-phy.cc:516-519) and
 * MonitorSnifferRx after an EndReceive whose m_random draw passed (:783-790, signal / noise dBm from the
 * event's rxPowerW and the SNR); the State Tx / RxOk traces fire at the same instants.  The frame bytes
 * are the host MAC's (the device keeps sizes only): record tx's frame is frames[frame_off[tx] ..
 * frame_off[tx + 1]), its printed text (Packet::Print, for the ascii sinks) text[text_off[tx] ..). */
typedef struct nsgpu_wifi_sniff {
  uint64_t ts;           /* Now () of the call (ns) */
  uint32_t phy, tx;      /* the phy (YansWifiChannel index: its file / context) and the transmission */
  uint32_t kind;         /* 0: MonitorSnifferTx (+ State Tx), 1: MonitorSnifferRx (+ State RxOk) */
  uint32_t rate;         /* dataRate500KbpsUnits = the mode's GetDataRate () / 500000 */
  uint32_t freq_mhz;     /* GetChannelFrequencyMhz () */
  uint32_t short_preamble;
  double signal_dbm, noise_dbm;  /* Rx: RatioToDb (rxPowerW) + 30, RatioToDb (rxPowerW / snr) - RxNoiseFigure + 30 */
} nsgpu_wifi_sniff;
/* an Ok EndReceive's signal / noise dBm (yans-wifi-phy.cc:788-789) from its nsgpu_wifil_end */
int nsgpu_wifi_sniff_power(const nsgpu_wifil_end *e, double rx_noise_figure_db, double *signal_dbm, double *noise_dbm);
/* phy's pcap file (YansWifiPhyHelper::EnablePcapInternal, yans-wifi-helper.cc:415-445): dlt 105
 * (DLT_IEEE802_11: the frame as is) or 127 (DLT_IEEE802_11_RADIO: a RadiotapHeader first — TSFT = Now in us,
 * flags FCS included | short preamble, rate, channel frequency and CCK / OFDM / 2 / 5 GHz flags, and for Rx
 * the antenna signal / noise dBm; PcapSniffTxEvent / PcapSniffRxEvent, :244-392) */
int nsgpu_wifi_pcap(uint32_t dlt, const nsgpu_wifi_sniff *rec, uint64_t n, uint32_t phy, const uint64_t *frame_off,
                    const uint8_t *frames, uint8_t *out, uint64_t cap, uint64_t *len);
/* EnableAsciiAll (stream) lines (AsciiPhyTransmitSinkWithContext / AsciiPhyReceiveSinkWithContext,
 * yans-wifi-helper.cc:42-88, connected at /NodeList/<node>/DeviceList/<device>/$ns3::WifiNetDevice/Phy/State/
 * Tx and .../RxOk, :529-535): "t|r <Now ().GetSeconds ()> <context> <packet>" */
int nsgpu_wifi_ascii(const nsgpu_wifi_sniff *rec, uint64_t n, const uint32_t *phy_node, const uint32_t *phy_device,
                     const uint64_t *text_off, const char *text, char *out, uint64_t cap, uint64_t *len);
/* PcapFile::Init + Write (src/network/utils/pcap-file.cc:300-381) of arbitrary packets: record i is
 * data[off[i] .. off[i + 1]) with origLen orig_len[i] (inclLen = min (origLen, snaplen, its bytes)) */
int nsgpu_pcap_file(uint32_t linktype, uint32_t snaplen, uint64_t n, const uint32_t *sec, const uint32_t *usec,
                    const uint32_t *orig_len, const uint64_t *off, const uint8_t *data, uint8_t *out, uint64_t cap,
                    uint64_t *len);

#ifdef __cplusplus
}
#endif
#endif /* NSGPU_H */
