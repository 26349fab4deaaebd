"""Wi-Fi PHY scenarios for the device receive subset (include/nsgpu_types.h: nsgpu_wifi_scenario).

Host-side plumbing only: the phy list, positions and transmission schedule an ns-3 PHY harness would
build, and the C-ABI calls (nsgpu_wifi_*).  No simulation logic lives here.

The harness is the shape of src/wifi/test/wifi-test.cc:181-260 scaled up: YansWifiPhy objects on one
YansWifiChannel (YansWifiChannelHelper::Default: LogDistance exponent 3, reference loss 46.6777 dB at
1 m, ConstantSpeed 3e8 m/s — src/wifi/helper/yans-wifi-helper.cc:96-102), YansWifiPhy defaults
(RxGain 1 dB, TxGain 1 dB, TxPowerStart 16.0206 dBm, EnergyDetectionThreshold -96 dBm,
CcaMode1Threshold -99 dBm — src/wifi/model/yans-wifi-phy.cc:50-126), and every transmission a
Simulator::Schedule (t, &YansWifiPhy::SendPacket, phy, packet, mode, preamble, 0) made before Run,
in the order of the schedule builder below (that order fixes their setup uids).
"""
import ctypes as C

import numpy as np

import nsgpu

DSSS, OFDM, ERP_OFDM = 0, 1, 2
PREAMBLE_LONG, PREAMBLE_SHORT = 0, 1
STORE_AUTO, STORE_LDS, STORE_HBM = 0, 1, 2  # nsgpu_wifi_store: where each phy's NiChanges list lives
INLINE_RX = 4  # | store: receptions computed inside the per-phy kernel (no up-front reception table)
UNSORTED_RX = 8  # | store: the reception table's rows scanned unsorted (not put in dispatch order first)
SYNC, DROP_RX, DROP_TX, DROP_ED, NOT_RUN = 0, 1, 2, 3, 255
F_CCA_EVAL, F_CCA_SWITCH, F_NEAR_ED, F_NEAR_CCA = 1, 2, 4, 8
END_CANCELLED, END_DISPATCHED = 1, 2
NO_STOP = (1 << 64) - 1

# 802.11b DSSS 1 Mbps (WifiPhy::GetDsssRate1Mbps: 22 MHz, wifi-phy.cc:325-336)
DSSS_1M = (DSSS, 1000000, 22000000)
# a 1000-B UDP datagram as a broadcast data frame at the PHY: +8 UDP +20 IPv4 +8 LLC/SNAP +24 MAC header +4 FCS
FRAME_1000B = 1000 + 8 + 20 + 8 + 24 + 4


class WifiScenarioStruct(C.Structure):
    _fields_ = [
        ("n_phy", C.c_int64), ("x", C.c_void_p), ("y", C.c_void_p), ("z", C.c_void_p),
        ("channel", C.c_void_p), ("node", C.c_void_p), ("loss", nsgpu.LossChain), ("speed", C.c_double),
        ("rx_gain_db", C.c_double), ("ed_threshold_dbm", C.c_double), ("cca_threshold_dbm", C.c_double),
        ("n_tx", C.c_int64), ("tx_ts", C.c_void_p), ("tx_uid", C.c_void_p), ("tx_phy", C.c_void_p),
        ("tx_size", C.c_void_p), ("tx_dbm", C.c_void_p), ("tx_modclass", C.c_void_p), ("tx_rate_bps", C.c_void_p),
        ("tx_bw_hz", C.c_void_p), ("tx_preamble", C.c_void_p), ("uid_start", C.c_uint32), ("ni_cap", C.c_uint32),
        ("stop_ts", C.c_uint64), ("stop_uid", C.c_uint32), ("pad_", C.c_uint32),
    ]


class WifiStats(C.Structure):
    _fields_ = [(f, C.c_uint64) for f in ("dispatched", "tx", "rx", "sync", "drop_rx", "drop_tx", "drop_ed",
                                          "cca_evals", "cca_switches", "end", "end_cancelled", "ni_inserts",
                                          "near_threshold", "digest", "final_ts")] + \
               [("next_uid", C.c_uint32), ("ni_max", C.c_uint32)]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


RX_LOG_DTYPE = np.dtype([("ts", "<u8"), ("uid", "<u4"), ("outcome", "u1"), ("flags", "u1"), ("pad_", "<u2"),
                         ("cca_ns", "<i8")])
END_RECORD_DTYPE = np.dtype([("ts", "<u8"), ("sync_ts", "<u8"), ("uid", "<u4"), ("phy", "<u4"), ("tx", "<u4"),
                             ("flags", "<u4")])
PHY_COUNTERS_DTYPE = np.dtype([(f, "<u4") for f in ("rx", "sync", "drop_rx", "drop_tx", "drop_ed", "cca_switches",
                                                    "end", "end_cancelled", "ni_len", "ni_max")] +
                              [("end_tx", "<i8"), ("end_rx", "<i8"), ("end_cca_busy", "<i8"),
                               ("first_power", "<f8"), ("rxing", "<u4"), ("pad_", "<u4")])
TX_DTYPE = np.dtype([("ts", "<u8"), ("uid", "<u4"), ("phy", "<u4"), ("size", "<u4"), ("dbm", "<f8"),
                     ("modclass", "<u4"), ("rate", "<u8"), ("bw", "<u4"), ("preamble", "<u4")])


def tx_duration_ns(size, mode=DSSS_1M, preamble=PREAMBLE_LONG):
    """WifiPhy::CalculateTxDuration through the C-ABI (nsgpu_wifi_tx_duration_ns)."""
    out = C.c_int64()
    nsgpu.check(nsgpu.lib().nsgpu_wifi_tx_duration_ns(size, mode[0], mode[1], mode[2], preamble, C.byref(out)))
    return out.value


class Scenario:
    """Phys (m_phyList order) and a transmission schedule (TX_DTYPE, (ts, uid) order)."""

    def __init__(self, x, y, z, tx, channel=None, node=None, loss=((nsgpu.LOSS_LOG_DISTANCE, 3.0, 1.0, 46.6777),),
                 speed=300000000.0, rx_gain_db=1.0, ed_threshold_dbm=-96.0, cca_threshold_dbm=-99.0,
                 uid_start=None, stop_ts=None, stop_uid=None, ni_cap=256):
        n = len(x)
        self.x = np.ascontiguousarray(x, np.float64)
        self.y = np.ascontiguousarray(y, np.float64)
        self.z = np.ascontiguousarray(z, np.float64)
        self.channel = np.ascontiguousarray(np.ones(n, np.uint32) if channel is None else channel, np.uint32)
        self.node = np.ascontiguousarray(np.arange(n, dtype=np.uint32) if node is None else node, np.uint32)
        self.tx = np.ascontiguousarray(tx, TX_DTYPE)
        self.loss = loss
        self.speed, self.rx_gain_db = speed, rx_gain_db
        self.ed, self.cca = ed_threshold_dbm, cca_threshold_dbm
        self.uid_start = int(uid_start if uid_start is not None else (self.tx["uid"].max(initial=3) + 2))
        self.stop_ts = NO_STOP if stop_ts is None else int(stop_ts)
        self.stop_uid = 0 if stop_uid is None else int(stop_uid)
        self.ni_cap = ni_cap
        self._cols = {}

    @property
    def n_phy(self):
        return len(self.x)

    def c_struct(self):
        s = WifiScenarioStruct()
        s.n_phy = self.n_phy
        s.x, s.y, s.z = self.x.ctypes.data, self.y.ctypes.data, self.z.ctypes.data
        s.channel, s.node = self.channel.ctypes.data, self.node.ctypes.data
        s.loss = nsgpu.loss_chain(*self.loss)
        s.speed, s.rx_gain_db = self.speed, self.rx_gain_db
        s.ed_threshold_dbm, s.cca_threshold_dbm = self.ed, self.cca
        s.n_tx = len(self.tx)
        for f, col, dt in (("tx_ts", "ts", np.uint64), ("tx_uid", "uid", np.uint32), ("tx_phy", "phy", np.uint32),
                           ("tx_size", "size", np.uint32), ("tx_dbm", "dbm", np.float64),
                           ("tx_modclass", "modclass", np.uint32), ("tx_rate_bps", "rate", np.uint64),
                           ("tx_bw_hz", "bw", np.uint32), ("tx_preamble", "preamble", np.uint32)):
            a = np.ascontiguousarray(self.tx[col], dt)
            self._cols[f] = a  # keep alive with the struct
            setattr(s, f, a.ctypes.data)
        s.uid_start, s.ni_cap = self.uid_start, self.ni_cap
        s.stop_ts, s.stop_uid = self.stop_ts, self.stop_uid
        return s


def grid(n_side, spacing=100.0):
    """GridPositionAllocator, row first (grid-position-allocator: x = i % width, y = i / width), z = 0."""
    i = np.arange(n_side * n_side)
    return ((i % n_side) * spacing).astype(np.float64), ((i // n_side) * spacing).astype(np.float64), \
        np.zeros(n_side * n_side, np.float64)


def periodic_broadcast(n_phy, period_s=1.0, start_s=0.0, stop_s=2.0, size=FRAME_1000B, mode=DSSS_1M,
                       preamble=PREAMBLE_LONG, tx_dbm=16.0206 + 1.0, seed=1, senders=None, first_uid=4):
    """Every sender (default: every phy) transmits once per period from a seeded random phase
    (ns resolution).  The harness schedules them sender by sender, period by period, so the setup uids
    are first_uid, first_uid + 1, ... in that order; the schedule comes back in (ts, uid) order.
    Returns (tx, next free uid)."""
    rng = np.random.default_rng(seed)
    senders = np.arange(n_phy) if senders is None else np.asarray(senders)
    period = int(round(period_s * 1e9))
    phase = rng.integers(0, period, len(senders))
    rows = []
    for s, ph in zip(senders, phase):
        t = int(round(start_s * 1e9)) + int(ph)
        while t < int(round(stop_s * 1e9)):
            rows.append((t, int(s)))
            t += period
    tx = np.zeros(len(rows), TX_DTYPE)
    if rows:
        r = np.array(rows, dtype=np.int64)
        tx["ts"], tx["phy"] = r[:, 0], r[:, 1]
    tx["uid"] = first_uid + np.arange(len(rows))
    tx["size"], tx["dbm"] = size, tx_dbm
    tx["modclass"], tx["rate"], tx["bw"], tx["preamble"] = mode[0], mode[1], mode[2], preamble
    tx = np.sort(tx, order=["ts", "uid"])
    return tx, first_uid + len(rows)


def wifi_grid(n_side=100, spacing=100.0, period_s=1.0, stop_s=2.0, size=FRAME_1000B, seed=1, ni_cap=512):
    """Config 3's PHY workload: n_side x n_side phys, every phy broadcasting once per period, Stop at stop_s."""
    x, y, z = grid(n_side, spacing)
    tx, nxt = periodic_broadcast(len(x), period_s=period_s, stop_s=stop_s, size=size, seed=seed)
    return Scenario(x, y, z, tx, uid_start=nxt + 1, stop_ts=int(round(stop_s * 1e9)), stop_uid=nxt, ni_cap=ni_cap)


class Engine:
    """The device receive subset for one scenario (nsgpu_wifi_create / run / readers)."""

    def __init__(self, scenario, rx_log=False, stream=None, store=STORE_AUTO, phys=None, comm=None):
        """phys=(begin, end): a partition running those receivers (nsgpu_wifi_create_dist) — on the RCCL
        communicator `comm` (p2p.Comm), or, without one, a loopback member for group_run."""
        self.sc = scenario
        self.s = scenario.c_struct()
        self.stream = stream
        self.rx_log = rx_log
        self.phys_range = (0, scenario.n_phy) if phys is None else (int(phys[0]), int(phys[1]))
        self.comm = comm
        h = C.c_void_p()
        if phys is None and comm is None:
            nsgpu.check(nsgpu.lib().nsgpu_wifi_create(C.byref(self.s), int(rx_log), C.byref(h)))
        else:
            nsgpu.check(nsgpu.lib().nsgpu_wifi_create_dist(C.byref(self.s), int(rx_log), self.phys_range[0],
                                                           self.phys_range[1], comm.h if comm else None,
                                                           C.byref(h)))
        self.h = h.value
        nsgpu.check(nsgpu.lib().nsgpu_wifi_set_store(self.h, int(store)))

    def store(self):
        """(store the next run uses, phys per block, end-queue / ring capacity) — nsgpu_wifi_get_store."""
        st, p, e = C.c_int(), C.c_uint32(), C.c_uint32()
        nsgpu.check(nsgpu.lib().nsgpu_wifi_get_store(self.h, C.byref(st), C.byref(p), C.byref(e)))
        return st.value, p.value, e.value

    def launch(self):
        nsgpu.check(nsgpu.lib().nsgpu_wifi_run(self.h, self.stream))

    def run(self):
        self.launch()
        return self.stats()

    def profile(self):
        """One run with each kernel bracketed by HIP events (nsgpu_wifi_profile): {kernel: ms}."""
        n = C.c_int()
        nsgpu.check(nsgpu.lib().nsgpu_wifi_kernel_count(C.byref(n)))
        ms = np.zeros(n.value, np.float64)
        nsgpu.check(nsgpu.lib().nsgpu_wifi_profile(self.h, self.stream, ms.ctypes.data))
        return {nsgpu.lib().nsgpu_wifi_kernel_name(k).decode(): float(ms[k]) for k in range(n.value)}

    def stats(self):
        st = WifiStats()
        nsgpu.check(nsgpu.lib().nsgpu_wifi_get_stats(self.h, C.byref(st)))
        return st

    def phys(self):
        out = np.zeros(self.sc.n_phy, PHY_COUNTERS_DTYPE)
        nsgpu.check(nsgpu.lib().nsgpu_wifi_read_phys(self.h, out.ctypes.data))
        return out

    def tx_base(self):
        out = np.zeros(len(self.sc.tx), np.uint32)
        nsgpu.check(nsgpu.lib().nsgpu_wifi_read_tx_base(self.h, out.ctypes.data))
        return out

    def ends(self):
        """EndReceive records in uid order."""
        n = C.c_uint64()
        nsgpu.check(nsgpu.lib().nsgpu_wifi_read_ends(self.h, None, 0, C.byref(n)))
        out = np.zeros(n.value, END_RECORD_DTYPE)
        nsgpu.check(nsgpu.lib().nsgpu_wifi_read_ends(self.h, out.ctypes.data, n.value, C.byref(n)))
        return np.sort(out, order="uid")

    def rx_log_read(self):
        out = np.zeros(len(self.sc.tx) * self.sc.n_phy, RX_LOG_DTYPE)
        nsgpu.check(nsgpu.lib().nsgpu_wifi_read_rx_log(self.h, out.ctypes.data))
        return out

    def close(self):
        if getattr(self, "h", None):
            nsgpu.lib().nsgpu_wifi_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def partitions(n_phy, parts):
    """Contiguous receiver blocks [begin, end) of `parts` partitions (the row bands of a grid)."""
    return [(n_phy * p // parts, n_phy * (p + 1) // parts) for p in range(parts)]


def group_run(engines, stream=None):
    """One run of a loopback group (nsgpu_wifi_group_run): the partitions' chains, then their combined
    syncs and counters in every member."""
    arr = (C.c_void_p * len(engines))(*[e.h for e in engines])
    nsgpu.check(nsgpu.lib().nsgpu_wifi_group_run(arr, len(engines), stream))


# ---- closed-loop PHY (nsgpu_wifil_*: SendPacket from host closures on nsgpu_sim) ----
NIST, YANS = 0, 1  # nsgpu_wifil_error_model
IDLE, RX, TX, CCA_BUSY = 0, 1, 2, 3  # nsgpu_wifil_state
WIFIL_END_DTYPE = np.dtype([("ts", "<u8"), ("uid", "<u4"), ("phy", "<u4"), ("snr", "<f8"), ("per", "<f8"),
                            ("tx", "<u4"), ("flags", "<u4"), ("rx_w", "<f8")])


# ---- sniffer records (YansWifiPhyHelper's pcap / ascii sinks; the codec is in libnsgpu: nsgpu_wifi_*) ----
WIFI_SNIFF_DTYPE = np.dtype([("ts", "<u8"), ("phy", "<u4"), ("tx", "<u4"), ("kind", "<u4"), ("rate", "<u4"),
                             ("freq_mhz", "<u4"), ("short_preamble", "<u4"), ("signal_dbm", "<f8"),
                             ("noise_dbm", "<f8")])
DLT_IEEE802_11, DLT_IEEE802_11_RADIO = 105, 127


def sniff_power(end, noise_figure_db):
    """An Ok EndReceive's MonitorSnifferRx signal / noise dBm (yans-wifi-phy.cc:788-789), through the library."""
    e = np.ascontiguousarray(np.array([end], dtype=WIFIL_END_DTYPE))
    sig, noi = C.c_double(), C.c_double()
    nsgpu.check(nsgpu.lib().nsgpu_wifi_sniff_power(e.ctypes.data, noise_figure_db, C.byref(sig), C.byref(noi)))
    return sig.value, noi.value


def sniff_records(txs, ends, ok, mode, preamble, noise_figure_db, freq_mhz):
    """The sniffer calls of a closed-loop run in dispatch order: MonitorSnifferTx for every SendPacket (txs:
    (ts, closure uid, phy), transmission index = row) and MonitorSnifferRx for every EndReceive whose draw
    passed (ok[i] for ends[i]; cancelled ones never), keyed by the calling event's (ts, uid)."""
    rate = int(mode[1]) // 500000
    short = 1 if preamble == PREAMBLE_SHORT else 0
    rows, keys = [], []
    for k, (ts, uid, phy) in enumerate(np.asarray(txs, np.uint64).reshape(-1, 3)):
        rows.append((int(ts), int(phy), k, 0, rate, freq_mhz, short, 0.0, 0.0))
        keys.append((int(ts), int(uid)))
    for e, o in zip(ends, ok):
        if not o or (int(e["flags"]) & END_CANCELLED):
            continue
        sig, noi = sniff_power(e, noise_figure_db)
        rows.append((int(e["ts"]), int(e["phy"]), int(e["tx"]), 1, rate, freq_mhz, short, sig, noi))
        keys.append((int(e["ts"]), int(e["uid"])))
    order = sorted(range(len(rows)), key=lambda i: keys[i])
    return np.array([rows[i] for i in order], dtype=WIFI_SNIFF_DTYPE)


def _frames(frames):
    off = np.zeros(len(frames) + 1, np.uint64)
    off[1:] = np.cumsum([len(f) for f in frames]) if frames else []
    data = np.frombuffer(b"".join(bytes(f) for f in frames) or b"\0", np.uint8).copy()
    return off, data


def sniff_pcap(dlt, recs, phy, frames):
    """phy's pcap file (YansWifiPhyHelper::EnablePcap, DLT 105 or 127) from sniffer records; frames[tx] = the
    transmission's frame bytes (the host MAC's)."""
    import p2p
    recs = np.ascontiguousarray(recs, dtype=WIFI_SNIFF_DTYPE)
    off, data = _frames(frames)
    return p2p._out_bytes(lambda o, c, n: nsgpu.lib().nsgpu_wifi_pcap(dlt, recs.ctypes.data, len(recs), phy,
                                                                     off.ctypes.data, data.ctypes.data, o, c, n))


def sniff_ascii(recs, phy_node, phy_device, texts):
    """EnableAsciiAll (stream) lines of the sniffer records; texts[tx] = the frame's Packet::Print text."""
    import p2p
    recs = np.ascontiguousarray(recs, dtype=WIFI_SNIFF_DTYPE)
    off, data = _frames([t.encode() for t in texts])
    pn = np.ascontiguousarray(phy_node, np.uint32)
    pd = np.ascontiguousarray(phy_device, np.uint32)
    return p2p._out_bytes(lambda o, c, n: nsgpu.lib().nsgpu_wifi_ascii(recs.ctypes.data, len(recs), pn.ctypes.data,
                                                                      pd.ctypes.data, off.ctypes.data, data.ctypes.data,
                                                                      o, c, n)).decode()


class WifilConfigStruct(C.Structure):
    _fields_ = [
        ("n_phy", C.c_int64), ("x", C.c_void_p), ("y", C.c_void_p), ("z", C.c_void_p),
        ("channel", C.c_void_p), ("node", C.c_void_p), ("loss", nsgpu.LossChain), ("speed", C.c_double),
        ("rx_gain_db", C.c_double), ("ed_threshold_dbm", C.c_double), ("cca_threshold_dbm", C.c_double),
        ("rx_noise_figure_db", C.c_double), ("error_model", C.c_uint32), ("ni_cap", C.c_uint32),
        ("rxq_cap", C.c_uint32), ("pad_", C.c_uint32), ("tx_cap", C.c_uint64),
    ]


class WifilPhyState(C.Structure):
    _fields_ = [("state", C.c_uint32), ("rxing", C.c_uint32), ("end_tx", C.c_int64), ("end_rx", C.c_int64),
                ("end_cca_busy", C.c_int64), ("delay_until_idle", C.c_int64)]


class LoopPhys:
    """The phys of a closed-loop run (nsgpu_wifil_config): positions, channels, nodes and the PHY /
    channel attributes (defaults as Scenario above; RxNoiseFigure 7 dB, NistErrorRateModel as
    YansWifiPhyHelper::Default sets, yans-wifi-helper.cc:187)."""

    def __init__(self, x, y, z, channel=None, node=None, loss=((nsgpu.LOSS_LOG_DISTANCE, 3.0, 1.0, 46.6777),),
                 speed=300000000.0, rx_gain_db=1.0, ed_threshold_dbm=-96.0, cca_threshold_dbm=-99.0,
                 noise_figure_db=7.0, error_model=NIST, ni_cap=256, rxq_cap=256, tx_cap=1 << 16):
        n = len(x)
        self.x = np.ascontiguousarray(x, np.float64)
        self.y = np.ascontiguousarray(y, np.float64)
        self.z = np.ascontiguousarray(z, np.float64)
        self.channel = np.ascontiguousarray(np.ones(n, np.uint32) if channel is None else channel, np.uint32)
        self.node = np.ascontiguousarray(np.arange(n, dtype=np.uint32) if node is None else node, np.uint32)
        self.loss = loss
        self.speed, self.rx_gain_db, self.ed, self.cca = speed, rx_gain_db, ed_threshold_dbm, cca_threshold_dbm
        self.noise_figure_db, self.error_model = noise_figure_db, error_model
        self.ni_cap, self.rxq_cap, self.tx_cap = ni_cap, rxq_cap, tx_cap

    @property
    def n_phy(self):
        return len(self.x)

    def receivers(self, phy):
        """Fan-out uids one SendPacket of `phy` takes: the other phys on its channel."""
        return int(np.count_nonzero(self.channel == self.channel[phy])) - 1

    def send_plan(self, sender, uid_base):
        """nsgpu_wifil_send_plan (host only): YansWifiChannel::Send's Receive calls for one SendPacket of `sender` —
        (receiver phys, their uids, their contexts) in schedule order."""
        n = self.n_phy
        phy, uid, ctx = (np.zeros(max(n, 1), np.uint32) for _ in range(3))
        k = C.c_uint64()
        s = self.c_struct()
        nsgpu.check(nsgpu.lib().nsgpu_wifil_send_plan(C.byref(s), sender, uid_base, phy.ctypes.data, uid.ctypes.data,
                                                      ctx.ctypes.data, n, C.byref(k)))
        return phy[:k.value], uid[:k.value], ctx[:k.value]

    def c_struct(self):
        s = WifilConfigStruct()
        s.n_phy = self.n_phy
        s.x, s.y, s.z = self.x.ctypes.data, self.y.ctypes.data, self.z.ctypes.data
        s.channel, s.node = self.channel.ctypes.data, self.node.ctypes.data
        s.loss = nsgpu.loss_chain(*self.loss)
        s.speed, s.rx_gain_db = self.speed, self.rx_gain_db
        s.ed_threshold_dbm, s.cca_threshold_dbm = self.ed, self.cca
        s.rx_noise_figure_db, s.error_model = self.noise_figure_db, self.error_model
        s.ni_cap, s.rxq_cap, s.tx_cap = self.ni_cap, self.rxq_cap, self.tx_cap
        return s


class LoopPhy:
    """The closed-loop PHY on the device (nsgpu_wifil): attach it to a nsgpu.Sim, whose closures call
    Sim.wifi_send / Sim.wifi_state; EndReceive records (snr, per) come back through read_ends."""

    def __init__(self, phys, bounds=None, part=None, comm=None):
        """bounds=[0, b1, ..., n_phy]: a loopback group whose partitions [bounds[q], bounds[q+1]) run on this device
        (nsgpu_wifil_create_group); part=(begin, end) with comm (p2p.Comm): this rank's partition of an RCCL split
        (nsgpu_wifil_create_dist).  Either way the handle answers every call as the single engine would."""
        self.phys = phys
        self._cfg = phys.c_struct()
        h = C.c_void_p()
        if bounds is not None:
            self._bounds = np.ascontiguousarray(bounds, np.int64)
            nsgpu.check(nsgpu.lib().nsgpu_wifil_create_group(C.byref(self._cfg), self._bounds.ctypes.data,
                                                             len(self._bounds) - 1, C.byref(h)))
        elif part is not None:
            self._comm = comm
            nsgpu.check(nsgpu.lib().nsgpu_wifil_create_dist(C.byref(self._cfg), int(part[0]), int(part[1]),
                                                            comm.h, C.byref(h)))
        else:
            nsgpu.check(nsgpu.lib().nsgpu_wifil_create(C.byref(self._cfg), C.byref(h)))
        self.h = h.value

    def read_ends(self):
        n = C.c_uint64()
        nsgpu.check(nsgpu.lib().nsgpu_wifil_read_ends(self.h, None, 0, C.byref(n)))
        out = np.zeros(n.value, WIFIL_END_DTYPE)
        if n.value:
            nsgpu.check(nsgpu.lib().nsgpu_wifil_read_ends(self.h, out.ctypes.data, n.value, C.byref(n)))
        return out

    def read_phys(self):
        out = np.zeros(self.phys.n_phy, PHY_COUNTERS_DTYPE)
        nsgpu.check(nsgpu.lib().nsgpu_wifil_read_phys(self.h, out.ctypes.data))
        return out

    def pending(self):
        n, ts = C.c_uint64(), C.c_uint64()
        nsgpu.check(nsgpu.lib().nsgpu_wifil_pending(self.h, C.byref(n), C.byref(ts)))
        return n.value, ts.value

    def close(self):
        if self.h:
            nsgpu.lib().nsgpu_wifil_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
