"""ctypes binding of the CPU ORACLE (oracle/build/libnsref.so).  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module, and only as the checker / CPU baseline.  The product path never does.
See oracle/nsref.h for what is restated and where the reference code lives.
"""
import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libnsref.so")


class EventId(C.Structure):  # nsgpu_event_id (include/nsgpu_types.h)
    _fields_ = [("impl", C.c_uint64), ("ts", C.c_uint64), ("context", C.c_uint32), ("uid", C.c_uint32)]


class LossModel(C.Structure):
    _fields_ = [("kind", C.c_int32), ("pad_", C.c_int32), ("p0", C.c_double), ("p1", C.c_double), ("p2", C.c_double)]


class LossChain(C.Structure):
    _fields_ = [("n", C.c_int32), ("pad_", C.c_int32), ("m", LossModel * 4)]


RX_RECORD_DTYPE = np.dtype([("ts", "<u8"), ("uid", "<u4"), ("context", "<u4"), ("phy", "<u4"),
                            ("pad_", "<u4"), ("rx_dbm", "<f8")])


class ChurnResult(C.Structure):
    _fields_ = [("dispatched", C.c_uint64), ("holds", C.c_uint64), ("final_ts", C.c_uint64),
                ("digest", C.c_uint64), ("next_uid", C.c_uint32), ("pad_", C.c_uint32),
                ("run_seconds", C.c_double), ("init_seconds", C.c_double)]


LOSS_NONE, LOSS_LOG_DISTANCE, LOSS_FRIIS, LOSS_FIXED_RSS, LOSS_RANGE = 0, 1, 2, 3, 4
SCHED_MAP, SCHED_HEAP, SCHED_LIST, SCHED_CALENDAR = 0, 1, 2, 3

EVENT_FN = C.CFUNCTYPE(None, C.c_void_p, C.c_uint64)


def loss_chain(*models):
    """models: (kind, p0, p1, p2) tuples in m_next order."""
    ch = LossChain()
    ch.n = len(models)
    for i, (k, a, b, c) in enumerate(models):
        ch.m[i].kind, ch.m[i].p0, ch.m[i].p1, ch.m[i].p2 = k, a, b, c
    return ch


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        u64p = C.POINTER(C.c_uint64)
        L.nsref_i64x64_from_double.argtypes = [C.c_double, u64p]
        L.nsref_i64x64_from_int.argtypes = [C.c_int64, u64p]
        L.nsref_i64x64_from_parts.argtypes = [C.c_int64, C.c_uint64, u64p]
        for f in ("nsref_i64x64_mul", "nsref_i64x64_div", "nsref_i64x64_mul_by_invert"):
            getattr(L, f).argtypes = [u64p, u64p, u64p]
        L.nsref_i64x64_invert.argtypes = [C.c_uint64, u64p]
        L.nsref_i64x64_get_high.argtypes = [u64p]
        L.nsref_i64x64_get_high.restype = C.c_int64
        L.nsref_i64x64_get_low.argtypes = [u64p]
        L.nsref_i64x64_get_low.restype = C.c_uint64
        L.nsref_i64x64_get_double.argtypes = [u64p]
        L.nsref_i64x64_get_double.restype = C.c_double
        L.nsref_seconds.argtypes = [C.c_double]
        L.nsref_seconds.restype = C.c_int64
        L.nsref_seconds_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
        L.nsref_get_seconds.argtypes = [C.c_int64]
        L.nsref_get_seconds.restype = C.c_double
        L.nsref_from_integer.argtypes = [C.c_int64, C.c_int]
        L.nsref_from_integer.restype = C.c_int64
        L.nsref_distance.argtypes = [C.c_double] * 6
        L.nsref_distance.restype = C.c_double
        L.nsref_calc_rx_power.argtypes = [C.c_double, C.c_double, C.POINTER(LossChain)]
        L.nsref_calc_rx_power.restype = C.c_double
        L.nsref_const_speed_delay.argtypes = [C.c_double, C.c_double]
        L.nsref_const_speed_delay.restype = C.c_int64
        L.nsref_fanout_yans.argtypes = [C.c_void_p] * 5 + [C.c_int64, C.c_int64, C.c_double, C.POINTER(LossChain),
                                                           C.c_double, C.c_uint64, C.c_uint32, C.c_void_p]
        L.nsref_fanout_yans.restype = C.c_int64
        L.nsref_fanout_spectrum.argtypes = [C.c_void_p] * 4 + [C.c_int64, C.c_int64, C.POINTER(LossChain), C.c_double,
                                                               C.c_double, C.c_void_p, C.c_int32, C.c_uint64,
                                                               C.c_uint32, C.c_void_p, C.c_void_p]
        L.nsref_fanout_spectrum.restype = C.c_int64
        L.nsref_sim_new.argtypes = [C.c_int]
        L.nsref_sim_new.restype = C.c_void_p
        L.nsref_sim_free.argtypes = [C.c_void_p]
        L.nsref_sim_set_uid.argtypes = [C.c_void_p, C.c_uint32]
        L.nsref_sim_schedule.argtypes = [C.c_void_p, C.c_int64, EVENT_FN, C.c_void_p, C.c_uint64]
        L.nsref_sim_schedule.restype = EventId
        L.nsref_sim_schedule_with_context.argtypes = [C.c_void_p, C.c_uint32, C.c_int64, EVENT_FN, C.c_void_p,
                                                      C.c_uint64]
        L.nsref_sim_schedule_now.argtypes = [C.c_void_p, EVENT_FN, C.c_void_p, C.c_uint64]
        L.nsref_sim_schedule_now.restype = EventId
        L.nsref_sim_schedule_destroy.argtypes = [C.c_void_p, EVENT_FN, C.c_void_p, C.c_uint64]
        L.nsref_sim_schedule_destroy.restype = EventId
        for f in ("nsref_sim_remove", "nsref_sim_cancel"):
            getattr(L, f).argtypes = [C.c_void_p, C.POINTER(EventId)]
        L.nsref_sim_is_expired.argtypes = [C.c_void_p, C.POINTER(EventId)]
        L.nsref_sim_is_expired.restype = C.c_int
        for f in ("nsref_sim_run", "nsref_sim_stop", "nsref_sim_destroy", "nsref_sim_run_one"):
            getattr(L, f).argtypes = [C.c_void_p]
        L.nsref_sim_is_finished.argtypes = [C.c_void_p]
        L.nsref_sim_is_finished.restype = C.c_int
        L.nsref_sim_stop_at.argtypes = [C.c_void_p, C.c_int64]
        L.nsref_sim_now.argtypes = [C.c_void_p]
        L.nsref_sim_now.restype = C.c_uint64
        L.nsref_sim_context.argtypes = [C.c_void_p]
        L.nsref_sim_context.restype = C.c_uint32
        L.nsref_sim_delay_left.argtypes = [C.c_void_p, C.POINTER(EventId)]
        L.nsref_sim_delay_left.restype = C.c_uint64
        L.nsref_sim_dispatched.argtypes = [C.c_void_p]
        L.nsref_sim_dispatched.restype = C.c_uint64
        L.nsref_sim_next_uid.argtypes = [C.c_void_p]
        L.nsref_sim_next_uid.restype = C.c_uint32
        L.nsref_sim_set_log.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]
        L.nsref_churn_run.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_int, C.c_void_p, C.c_void_p,
                                      C.c_uint64, C.POINTER(ChurnResult)]
        L.nsref_churn_run.restype = C.c_int
        L.nsref_p2p_run.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                    C.c_void_p, C.c_uint64, C.c_void_p]
        L.nsref_p2p_run.restype = C.c_int
        L.nsref_p2p_run_trace.argtypes = [C.c_void_p] * 7 + [C.c_uint64, C.c_void_p, C.c_void_p, C.c_uint64,
                                                              C.c_void_p]
        L.nsref_p2p_run_probe.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_uint32, C.c_uint32, C.c_uint32] + \
            [C.c_void_p] * 7 + [C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p]
        L.nsref_p2p_run_trace.restype = C.c_int
        L.nsref_p2p_run_sends.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p] + [C.c_void_p] * 6 + \
            [C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p]
        L.nsref_p2p_set_trace_kinds.argtypes = [C.c_uint32]
        L.nsref_p2p_set_trace_kinds.restype = None
        L.nsref_distribution_ns.argtypes = [C.c_double]
        L.nsref_distribution_ns.restype = C.c_uint64
        _lib = L
    return _lib


# ---------------- convenience wrappers ----------------
def _w(x):
    return (C.c_uint64 * 2)(*x) if x is not None else (C.c_uint64 * 2)()


class I64x64:
    """int64x64_t restated (oracle)."""

    def __init__(self, words):
        self.w = (C.c_uint64 * 2)(*words)

    @classmethod
    def from_double(cls, v):
        o = _w(None)
        lib().nsref_i64x64_from_double(v, o)
        return cls(o)

    @classmethod
    def from_int(cls, v):
        o = _w(None)
        lib().nsref_i64x64_from_int(v, o)
        return cls(o)

    @classmethod
    def from_parts(cls, hi, lo):
        o = _w(None)
        lib().nsref_i64x64_from_parts(hi, lo, o)
        return cls(o)

    @classmethod
    def invert(cls, v):
        o = _w(None)
        lib().nsref_i64x64_invert(v, o)
        return cls(o)

    def _bin(self, f, other):
        o = _w(None)
        getattr(lib(), f)(self.w, other.w, o)
        return I64x64(o)

    def __mul__(self, o):
        return self._bin("nsref_i64x64_mul", o)

    def __truediv__(self, o):
        return self._bin("nsref_i64x64_div", o)

    def mul_by_invert(self, o):
        return self._bin("nsref_i64x64_mul_by_invert", o)

    def _int(self):
        v = self.w[0] | (self.w[1] << 64)
        return v - (1 << 128) if v >> 127 else v

    def __add__(self, o):
        v = (self._int() + o._int()) & ((1 << 128) - 1)
        return I64x64((v & ((1 << 64) - 1), v >> 64))

    def __sub__(self, o):
        v = (self._int() - o._int()) & ((1 << 128) - 1)
        return I64x64((v & ((1 << 64) - 1), v >> 64))

    def high(self):
        return lib().nsref_i64x64_get_high(self.w)

    def low(self):
        return lib().nsref_i64x64_get_low(self.w)

    def double(self):
        return lib().nsref_i64x64_get_double(self.w)


def seconds(s):
    return lib().nsref_seconds(float(s))


def seconds_batch(arr):
    arr = np.ascontiguousarray(arr, dtype=np.float64)
    out = np.empty(arr.shape, dtype=np.int64)
    lib().nsref_seconds_batch(arr.ctypes.data, out.ctypes.data, arr.size)
    return out


def get_seconds(ts):
    return lib().nsref_get_seconds(int(ts))


def fanout_yans(x, y, z, chan, node, sender, tx_dbm, chain, speed, now_ts, uid_base):
    n = len(x)
    out = np.zeros(n, dtype=RX_RECORD_DTYPE)
    arrs = [np.ascontiguousarray(a, dtype=t) for a, t in
            ((x, np.float64), (y, np.float64), (z, np.float64), (chan, np.uint32), (node, np.uint32))]
    k = lib().nsref_fanout_yans(*[a.ctypes.data for a in arrs], n, sender, tx_dbm, C.byref(chain), speed,
                                now_ts, uid_base, out.ctypes.data)
    return out[:k]


def fanout_spectrum(x, y, z, node, sender, chain, speed, max_loss_db, psd_tx, now_ts, uid_base):
    n = len(x)
    psd_tx = np.ascontiguousarray(psd_tx, dtype=np.float64)
    nb = psd_tx.size
    out = np.zeros(n, dtype=RX_RECORD_DTYPE)
    psd_out = np.zeros((n, nb), dtype=np.float64)
    arrs = [np.ascontiguousarray(a, dtype=t) for a, t in
            ((x, np.float64), (y, np.float64), (z, np.float64), (node, np.uint32))]
    k = lib().nsref_fanout_spectrum(*[a.ctypes.data for a in arrs], n, sender, C.byref(chain), speed, max_loss_db,
                                    psd_tx.ctypes.data, nb, now_ts, uid_base, out.ctypes.data, psd_out.ctypes.data)
    return out[:k], psd_out[:k]


def load_distribution(path):
    """bench-simulator ReadDistribution (bench-simulator.cc:59-76): doubles -> (uint64_t)(d*1e9)."""
    vals = []
    with open(path) as f:
        for tok in f.read().split():
            try:
                vals.append(float(tok))
            except ValueError:
                continue
    return np.array([lib().nsref_distribution_ns(v) for v in vals], dtype=np.uint64)


class CalendarCrash(RuntimeError):
    """The reference's CalendarScheduler crashes here; .result describes the run up to it."""

    def __init__(self, result):
        super().__init__(f"CalendarScheduler sentinel reached after {result.dispatched} dispatches (SURVEY H3)")
        self.result = result


def churn_run(dist_ns, total, scheduler=SCHED_MAP, log_cap=0):
    dist_ns = np.ascontiguousarray(dist_ns, dtype=np.uint64)
    res = ChurnResult()
    lts = np.zeros(log_cap, dtype=np.uint64) if log_cap else None
    luid = np.zeros(log_cap, dtype=np.uint32) if log_cap else None
    rc = lib().nsref_churn_run(dist_ns.ctypes.data, dist_ns.size, total, scheduler,
                               lts.ctypes.data if log_cap else None, luid.ctypes.data if log_cap else None, log_cap,
                               C.byref(res))
    if rc == -3:
        raise CalendarCrash(res)
    return res, lts, luid


class Sim:
    """Restated DefaultSimulatorImpl with Python closures (for semantics tests)."""

    def __init__(self, scheduler=SCHED_MAP):
        self.L = lib()
        self.h = self.L.nsref_sim_new(scheduler)
        self._keep = []

    def _fn(self, cb):
        f = EVENT_FN(lambda user, arg: cb())
        self._keep.append(f)
        return f

    def schedule(self, delay, cb):
        return self.L.nsref_sim_schedule(self.h, delay, self._fn(cb), None, 0)

    def schedule_with_context(self, ctx, delay, cb):
        self.L.nsref_sim_schedule_with_context(self.h, ctx, delay, self._fn(cb), None, 0)

    def schedule_now(self, cb):
        return self.L.nsref_sim_schedule_now(self.h, self._fn(cb), None, 0)

    def schedule_destroy(self, cb):
        return self.L.nsref_sim_schedule_destroy(self.h, self._fn(cb), None, 0)

    def remove(self, eid):
        self.L.nsref_sim_remove(self.h, C.byref(eid))

    def cancel(self, eid):
        self.L.nsref_sim_cancel(self.h, C.byref(eid))

    def is_expired(self, eid):
        return bool(self.L.nsref_sim_is_expired(self.h, C.byref(eid)))

    def run(self):
        self.L.nsref_sim_run(self.h)

    def run_one(self):
        self.L.nsref_sim_run_one(self.h)

    def is_finished(self):
        return bool(self.L.nsref_sim_is_finished(self.h))

    def stop(self, delay=None):
        if delay is None:
            self.L.nsref_sim_stop(self.h)
        else:
            self.L.nsref_sim_stop_at(self.h, delay)

    def destroy(self):
        self.L.nsref_sim_destroy(self.h)

    def now(self):
        return self.L.nsref_sim_now(self.h)

    def context(self):
        return self.L.nsref_sim_context(self.h)

    def dispatched(self):
        return self.L.nsref_sim_dispatched(self.h)

    def next_uid(self):
        return self.L.nsref_sim_next_uid(self.h)

    def set_next_uid(self, uid):
        self.L.nsref_sim_set_uid(self.h, uid)

    def close(self):
        if self.h:
            self.L.nsref_sim_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def p2p_run(scenario_struct, stats_struct, devc, appc, log_cap=0):
    """Sequential oracle run of a nsgpu_p2p_scenario (ctypes struct built by the caller).

    devc / appc: numpy structured arrays (n_devices / n_apps) filled in place.
    Returns (run_seconds, (log_ts, log_uid, log_ctx))."""
    secs = C.c_double()
    lts = np.zeros(log_cap, np.uint64)
    luid = np.zeros(log_cap, np.uint32)
    lctx = np.zeros(log_cap, np.uint32)
    lib().nsref_p2p_run(C.byref(scenario_struct), C.byref(stats_struct), devc.ctypes.data, appc.ctypes.data,
                        lts.ctypes.data if log_cap else None, luid.ctypes.data if log_cap else None,
                        lctx.ctypes.data if log_cap else None, log_cap, C.byref(secs))
    return secs.value, (lts, luid, lctx)


TRACE_RECORD_DTYPE = np.dtype([("ts", "<u8"), ("uid", "<u4"), ("seq", "<u2"), ("kind", "u1"), ("pad_", "u1"),
                               ("dev", "<u4"), ("app", "<u4"), ("ipid", "<u4"), ("size", "<u4"),
                               ("ttl", "<u4"), ("pad2_", "<u4")])  # nsgpu_trace_record


TRACE_DEVICE_KINDS, TRACE_IPV4_KINDS = 0x0F, 0x70  # nsgpu_trace_kind bits: the device sinks, Ipv4L3Protocol's


def p2p_run_trace(scenario_struct, stats_struct, devc, appc, log_cap=0, kinds=TRACE_DEVICE_KINDS):
    """p2p_run that also returns the ascii trace sink calls (TRACE_RECORD_DTYPE, pop order) of the
    nsgpu_trace_kind bits in `kinds`."""
    lib().nsref_p2p_set_trace_kinds(kinds)
    secs = C.c_double()
    lts = np.zeros(log_cap, np.uint64)
    luid = np.zeros(log_cap, np.uint32)
    lctx = np.zeros(log_cap, np.uint32)
    n = C.c_uint64()
    args = [C.byref(scenario_struct), C.byref(stats_struct), devc.ctypes.data, appc.ctypes.data,
            lts.ctypes.data if log_cap else None, luid.ctypes.data if log_cap else None,
            lctx.ctypes.data if log_cap else None, log_cap, C.byref(secs)]
    lib().nsref_p2p_run_trace(*args, None, 0, C.byref(n))  # count
    tr = np.zeros(n.value, TRACE_RECORD_DTYPE)
    lib().nsref_p2p_run_trace(*args, tr.ctypes.data, n.value, C.byref(n))
    lib().nsref_p2p_set_trace_kinds(TRACE_DEVICE_KINDS)
    return secs.value, (lts, luid, lctx), tr


APP_COUNTERS_DTYPE = np.dtype([("tx_packets", "<u4"), ("rx_packets", "<u4"), ("tx_bytes", "<u8"),
                               ("rx_bytes", "<u8")])  # nsgpu_app_counters


def p2p_run_probe(scenario_struct, stats_struct, devc, appc, t0, period, count, app_send, app_obs, log_cap=0,
                  kinds=TRACE_DEVICE_KINDS):
    """p2p run with the host probe application of nsref_p2p_run_probe; returns (log, trace, samples)."""
    lib().nsref_p2p_set_trace_kinds(kinds)
    from numpy import zeros
    lts = zeros(log_cap, np.uint64)
    luid = zeros(log_cap, np.uint32)
    lctx = zeros(log_cap, np.uint32)
    samples = zeros(count, APP_COUNTERS_DTYPE)
    n = C.c_uint64()
    args = [C.byref(scenario_struct), t0, period, count, app_send, app_obs, samples.ctypes.data, C.byref(stats_struct),
            devc.ctypes.data, appc.ctypes.data, lts.ctypes.data if log_cap else None,
            luid.ctypes.data if log_cap else None, lctx.ctypes.data if log_cap else None, log_cap]
    lib().nsref_p2p_run_probe(*args, None, 0, C.byref(n))
    tr = np.zeros(n.value, TRACE_RECORD_DTYPE)
    lib().nsref_p2p_run_probe(*args, tr.ctypes.data, n.value, C.byref(n))
    lib().nsref_p2p_set_trace_kinds(TRACE_DEVICE_KINDS)
    return (lts, luid, lctx), tr, samples


def p2p_run_sends(scenario_struct, stats_struct, devc, appc, ts, apps, log_cap=0, kinds=TRACE_DEVICE_KINDS):
    """p2p run with host datagrams (nsref_p2p_run_sends: Schedule (ts[k], send of app[k]) after setup); returns
    (log, trace)."""
    lib().nsref_p2p_set_trace_kinds(kinds)
    ts = np.ascontiguousarray(ts, np.int64)
    apps = np.ascontiguousarray(apps, np.uint32)
    lts = np.zeros(log_cap, np.uint64)
    luid = np.zeros(log_cap, np.uint32)
    lctx = np.zeros(log_cap, np.uint32)
    n = C.c_uint64()
    args = [C.byref(scenario_struct), len(ts), ts.ctypes.data, apps.ctypes.data, C.byref(stats_struct),
            devc.ctypes.data, appc.ctypes.data, lts.ctypes.data if log_cap else None,
            luid.ctypes.data if log_cap else None, lctx.ctypes.data if log_cap else None, log_cap]
    lib().nsref_p2p_run_sends(*args, None, 0, C.byref(n))
    tr = np.zeros(n.value, TRACE_RECORD_DTYPE)
    lib().nsref_p2p_run_sends(*args, tr.ctypes.data, n.value, C.byref(n))
    lib().nsref_p2p_set_trace_kinds(TRACE_DEVICE_KINDS)
    return (lts, luid, lctx), tr


def wifi_tx_duration(size, modclass, rate_bps, bw_hz, preamble):
    """WifiPhy::CalculateTxDuration restated (ns)."""
    f = lib().nsref_wifi_tx_duration
    f.restype = C.c_int64
    f.argtypes = [C.c_uint32, C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint32]
    return f(size, modclass, rate_bps, bw_hz, preamble)


def wifi_run(scenario_struct, stats_struct, phys, tx_base, end_dtype, rx_log=None):
    """Sequential oracle run of a nsgpu_wifi_scenario (ctypes struct built by the caller).

    phys (n_phy counters), tx_base (n_tx uint32) and rx_log (n_tx * n_phy, or None) are numpy arrays
    filled in place; returns (run_seconds, EndReceive records as `end_dtype`, in uid order)."""
    import time
    f = lib().nsref_wifi_run
    f.restype = C.c_int
    f.argtypes = [C.c_void_p] * 5 + [C.c_uint64, C.c_void_p, C.c_void_p]
    n = C.c_uint64()
    t0 = time.perf_counter()
    rc = f(C.byref(scenario_struct), C.byref(stats_struct), phys.ctypes.data, tx_base.ctypes.data, None, 0,
           C.byref(n), rx_log.ctypes.data if rx_log is not None else None)
    secs = time.perf_counter() - t0
    if rc != 0:
        raise RuntimeError(f"nsref_wifi_run: {rc}")
    ends = np.zeros(n.value, end_dtype)
    rc = f(C.byref(scenario_struct), C.byref(stats_struct), phys.ctypes.data, tx_base.ctypes.data,
           ends.ctypes.data, n.value, C.byref(n), rx_log.ctypes.data if rx_log is not None else None)
    if rc != 0:
        raise RuntimeError(f"nsref_wifi_run: {rc}")
    return secs, np.sort(ends, order="uid")


class WifilMacStruct(C.Structure):  # nsref_wifil_mac (nsref.h)
    _fields_ = [("first", C.c_void_p), ("backoff", C.c_void_p), ("period", C.c_uint64), ("stop_ts", C.c_uint64),
                ("rate", C.c_uint64), ("size", C.c_uint32), ("modclass", C.c_uint32), ("bw", C.c_uint32),
                ("preamble", C.c_uint32), ("dbm", C.c_double), ("uid_first", C.c_uint32), ("pad_", C.c_uint32),
                ("reply_delay", C.c_uint64), ("reply_on", C.c_uint32), ("pad2_", C.c_uint32)]


def wifil_run(cfg_struct, first, backoff, period, stop_ts, size, mode, preamble, dbm, n_phy, end_dtype,
              phys_dtype, log_cap=1 << 20, uid_first=0, reply_delay=None):
    """The closed-loop oracle run (nsref_wifil_run): the MAC stand-in of nsref.h over the PHY.  Returns
    (pop log (ts, uid, ctx), EndReceive records in dispatch order, per-phy counters, dict of totals).
    reply_delay (ns): the EndReceive hand-back's reply (nsref.h), None: off."""
    f = lib().nsref_wifil_run
    f.restype = C.c_int
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64,
                  C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]
    first = np.ascontiguousarray(first, np.uint64)
    backoff = np.ascontiguousarray(backoff, np.uint64)
    m = WifilMacStruct(first.ctypes.data, backoff.ctypes.data, period, stop_ts, mode[1], size, mode[0], mode[2],
                       preamble, dbm, uid_first, 0, reply_delay or 0, 0 if reply_delay is None else 1, 0)
    lts = np.zeros(log_cap, np.uint64)
    luid = np.zeros(log_cap, np.uint32)
    lctx = np.zeros(log_cap, np.uint32)
    phys = np.zeros(n_phy, phys_dtype)
    out = np.zeros(6, np.uint64)
    n = C.c_uint64()
    txo = np.zeros((1 << 20, 3), np.uint64)
    args = lambda ends, cap: (C.byref(cfg_struct), C.byref(m), lts.ctypes.data, luid.ctypes.data, lctx.ctypes.data,
                              log_cap, ends, cap, C.byref(n), phys.ctypes.data, out.ctypes.data, txo.ctypes.data,
                              txo.shape[0])
    rc = f(*args(None, 0))
    if rc != 0:
        raise RuntimeError(f"nsref_wifil_run: {rc}")
    ends = np.zeros(n.value, end_dtype)
    rc = f(*args(ends.ctypes.data, n.value))
    if rc != 0:
        raise RuntimeError(f"nsref_wifil_run: {rc}")
    tot = dict(zip(("dispatched", "digest", "next_uid", "final_ts", "sends", "busy"), (int(v) for v in out)))
    tot["txs"] = txo[:min(tot["sends"], txo.shape[0])].copy()  # (ts, closure uid, phy) per SendPacket
    k = min(tot["dispatched"], log_cap)
    return (lts[:k], luid[:k], lctx[:k]), ends, phys, tot


class WifilSendsStruct(C.Structure):  # nsref_wifil_sends (nsref.h)
    _fields_ = [("n", C.c_uint64), ("ts", C.c_void_p), ("phy", C.c_void_p), ("size", C.c_void_p),
                ("modclass", C.c_uint32), ("bw", C.c_uint32), ("preamble", C.c_uint32), ("pad_", C.c_uint32),
                ("rate", C.c_uint64), ("stop_ts", C.c_uint64), ("dbm", C.c_double), ("n_moves", C.c_uint64),
                ("move_ts", C.c_void_p), ("move_phy", C.c_void_p), ("move_xyz", C.c_void_p)]


def wifil_replay(cfg_struct, ts, phy, size, mode, preamble, dbm, stop_ts, n_phy, end_dtype, phys_dtype, log_cap=1 << 16,
                 moves=()):
    """moves: [(ts, phy, (x, y, z))] — MobilityModel::SetPosition host closures scheduled after the sends."""
    """A replayed transmission schedule on the closed-loop oracle PHY (nsref_wifil_replay): SendPacket of phy[k]
    (size[k] bytes) at ts[k], host closures scheduled at setup in send order, then Stop (stop_ts).  Returns as
    wifil_run."""
    f = lib().nsref_wifil_replay
    f.restype = C.c_int
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64,
                  C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]
    ts = np.ascontiguousarray(ts, np.uint64)
    phy = np.ascontiguousarray(phy, np.uint32)
    size = np.ascontiguousarray(size, np.uint32)
    mts = np.array([m[0] for m in moves] or [0], np.uint64)
    mph = np.array([m[1] for m in moves] or [0], np.uint32)
    mxyz = np.array([c for m in moves for c in m[2]] or [0.0], np.float64)
    sn = WifilSendsStruct(len(ts), ts.ctypes.data, phy.ctypes.data, size.ctypes.data, mode[0], mode[2], preamble, 0,
                          mode[1], stop_ts, dbm, len(moves), mts.ctypes.data, mph.ctypes.data, mxyz.ctypes.data)
    lts = np.zeros(log_cap, np.uint64)
    luid = np.zeros(log_cap, np.uint32)
    lctx = np.zeros(log_cap, np.uint32)
    phys = np.zeros(n_phy, phys_dtype)
    out = np.zeros(6, np.uint64)
    n = C.c_uint64()
    txo = np.zeros((len(ts) + 1, 3), np.uint64)
    args = lambda ends, cap: (C.byref(cfg_struct), C.byref(sn), lts.ctypes.data, luid.ctypes.data, lctx.ctypes.data,
                              log_cap, ends, cap, C.byref(n), phys.ctypes.data, out.ctypes.data, txo.ctypes.data,
                              txo.shape[0])
    rc = f(*args(None, 0))
    if rc != 0:
        raise RuntimeError(f"nsref_wifil_replay: {rc}")
    ends = np.zeros(n.value, end_dtype)
    rc = f(*args(ends.ctypes.data, n.value))
    if rc != 0:
        raise RuntimeError(f"nsref_wifil_replay: {rc}")
    tot = dict(zip(("dispatched", "digest", "next_uid", "final_ts", "sends", "busy"), (int(v) for v in out)))
    tot["txs"] = txo[:min(tot["sends"], txo.shape[0])].copy()  # (ts, closure uid, phy) per SendPacket
    k = min(tot["dispatched"], log_cap)
    return (lts[:k], luid[:k], lctx[:k]), ends, phys, tot


def wifil_chunk_success(model, mode, snr, nbits):
    f = lib().nsref_wifil_chunk_success
    f.restype = C.c_double
    f.argtypes = [C.c_uint32, C.c_uint32, C.c_uint64, C.c_uint32, C.c_double, C.c_uint32]
    return f(model, mode[0], mode[1], mode[2], snr, nbits)


def global_routes(dev_node, dev_peer, dev_addr, dev_mask, dev_ifindex, n_nodes, dst_addr):
    """GlobalRouteManager::PopulateRoutingTables + LookupGlobal restated (nsref_route.cc): uint32
    [n_nodes, n_dst] of output devices (0xfffffffe local delivery, 0xffffffff no route)."""
    f = lib().nsref_global_routes
    f.restype = C.c_int
    f.argtypes = [C.c_uint32, C.c_uint32] + [C.c_void_p] * 5 + [C.c_uint32, C.c_void_p, C.c_void_p]
    arrs = [np.ascontiguousarray(a, dtype=np.uint32) for a in (dev_node, dev_peer, dev_addr, dev_mask, dev_ifindex)]
    dst = np.ascontiguousarray(dst_addr, dtype=np.uint32)
    out = np.zeros((n_nodes, dst.size), np.uint32)
    rc = f(n_nodes, arrs[0].size, *[a.ctypes.data for a in arrs], dst.size, dst.ctypes.data, out.ctypes.data)
    if rc != 0:
        raise RuntimeError(f"nsref_global_routes: {rc}")
    return out


LOSS_TRACE_DTYPE = np.dtype([("rx_phy", "<u4"), ("pad_", "<u4"), ("loss_db", "<f8")])  # nsgpu_loss_trace


def fanout_spectrum_multi(x, y, z, node, rx_model, sender, models, tx_model, psd_tx, chain, speed, max_loss_db,
                          now_ts, uid_base):
    """MultiModelSpectrumChannel::StartTx restated; models: [(fl, fh), ...] in ascending SpectrumModelUid.
    Returns (records, [psd row per record], loss-trace entries)."""
    f = lib().nsref_fanout_spectrum_multi
    f.restype = C.c_int64
    f.argtypes = [C.c_void_p] * 5 + [C.c_int64, C.c_int64, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32,
                                     C.c_void_p, C.POINTER(LossChain), C.c_double, C.c_double, C.c_uint64,
                                     C.c_uint32, C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p]
    n = len(x)
    nb = [len(a) for a, _ in models]
    off = np.zeros(len(models) + 1, np.uint32)
    off[1:] = np.cumsum(nb)
    fl = np.concatenate([np.asarray(a, np.float64) for a, _ in models])
    fh = np.concatenate([np.asarray(b, np.float64) for _, b in models])
    stride = max(nb)
    arrs = [np.ascontiguousarray(a, dtype=t) for a, t in
            ((x, np.float64), (y, np.float64), (z, np.float64), (node, np.uint32), (rx_model, np.int32))]
    psd = np.ascontiguousarray(psd_tx, np.float64)
    out = np.zeros(n, RX_RECORD_DTYPE)
    psd_out = np.zeros((n, stride), np.float64)
    tr = np.zeros(n, LOSS_TRACE_DTYPE)
    nt = C.c_int64()
    k = f(*[a.ctypes.data for a in arrs], n, sender, len(models), off.ctypes.data, fl.ctypes.data, fh.ctypes.data,
          tx_model, psd.ctypes.data, C.byref(chain), speed, max_loss_db, now_ts, uid_base, out.ctypes.data,
          psd_out.ctypes.data, stride, tr.ctypes.data, C.byref(nt))
    rm = np.asarray(rx_model)
    rows = [psd_out[i, :nb[rm[out["phy"][i]]]] for i in range(k)]
    return out[:k], rows, tr[:nt.value]
