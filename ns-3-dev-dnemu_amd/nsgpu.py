"""Python binding of libnsgpu.so (include/nsgpu.h) — host plumbing for tests and bench.py.

This module only forwards to the C-ABI: every computation runs in the HIP kernels of
libnsgpu.so.  There is no CPU fallback: if the library (or a GPU) is missing, calls raise.
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# NSGPU_LIB selects another build of the same library (e.g. the phase-profiling diagnostic build)
LIB_PATH = os.environ.get("NSGPU_LIB") or os.path.join(_HERE, "lib", "libnsgpu.so")


class NsgpuError(RuntimeError):
    pass


class PhySoA(C.Structure):
    _fields_ = [("x", C.c_void_p), ("y", C.c_void_p), ("z", C.c_void_p), ("channel", C.c_void_p),
                ("node", C.c_void_p), ("chan_rank", C.c_void_p), ("chan_count", C.c_void_p)]


class SpectrumModels(C.Structure):  # nsgpu_spectrum_models
    _fields_ = [("n_models", C.c_int32), ("max_bands", C.c_int32), ("band_off", C.c_void_p), ("fl", C.c_void_p),
                ("fh", C.c_void_p)]


class LossModel(C.Structure):
    _fields_ = [("kind", C.c_int32), ("pad_", C.c_int32), ("p0", C.c_double), ("p1", C.c_double), ("p2", C.c_double)]


class LossChain(C.Structure):
    _fields_ = [("n", C.c_int32), ("pad_", C.c_int32), ("m", LossModel * 4)]


class HoldStats(C.Structure):
    _fields_ = [("dispatched", C.c_uint64), ("holds", C.c_uint64), ("final_ts", C.c_uint64),
                ("digest", C.c_uint64), ("rounds", C.c_uint64), ("max_batch", C.c_uint32),
                ("next_uid", C.c_uint32)]


LOSS_TRACE_DTYPE = np.dtype([("rx_phy", "<u4"), ("pad_", "<u4"), ("loss_db", "<f8")])  # nsgpu_loss_trace
TX_DESC_DTYPE = np.dtype([("now_ts", "<u8"), ("tx_dbm", "<f8"), ("sender", "<u4"), ("uid_base", "<u4")])
RX_RECORD_DTYPE = np.dtype([("ts", "<u8"), ("uid", "<u4"), ("context", "<u4"), ("phy", "<u4"),
                            ("pad_", "<u4"), ("rx_dbm", "<f8")])

LOSS_NONE, LOSS_LOG_DISTANCE, LOSS_FRIIS, LOSS_FIXED_RSS, LOSS_RANGE = 0, 1, 2, 3, 4

# symbol -> (restype, argtypes); the list is also what tests check the .so exports.
_vp, _i64, _u64, _u32, _i32, _d = C.c_void_p, C.c_int64, C.c_uint64, C.c_uint32, C.c_int32, C.c_double
SIGNATURES = {
    "nsgpu_version": (C.c_int, []),
    "nsgpu_last_error": (C.c_char_p, []),
    "nsgpu_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "nsgpu_set_device": (C.c_int, [C.c_int]),
    "nsgpu_malloc": (C.c_int, [C.POINTER(C.c_void_p), C.c_size_t]),
    "nsgpu_free": (C.c_int, [_vp]),
    "nsgpu_memcpy_htod": (C.c_int, [_vp, _vp, C.c_size_t, _vp]),
    "nsgpu_memcpy_dtoh": (C.c_int, [_vp, _vp, C.c_size_t, _vp]),
    "nsgpu_memset": (C.c_int, [_vp, C.c_int, C.c_size_t, _vp]),
    "nsgpu_device_synchronize": (C.c_int, []),
    "nsgpu_stream_create": (C.c_int, [C.POINTER(C.c_void_p)]),
    "nsgpu_stream_destroy": (C.c_int, [_vp]),
    "nsgpu_stream_sync": (C.c_int, [_vp]),
    "nsgpu_route_global": (C.c_int, [_u32, _u32, _vp, _vp, _vp, _vp, _u32, _vp, _vp, _vp]),
    "nsgpu_event_create": (C.c_int, [C.POINTER(C.c_void_p)]),
    "nsgpu_event_destroy": (C.c_int, [_vp]),
    "nsgpu_event_record": (C.c_int, [_vp, _vp]),
    "nsgpu_event_elapsed_ms": (C.c_int, [_vp, _vp, C.POINTER(C.c_float)]),
    "nsgpu_seconds_to_ts": (C.c_int, [_vp, _vp, _i64, _vp]),
    "nsgpu_fanout_yans": (C.c_int, [C.POINTER(PhySoA), _i64, _vp, _i64, C.POINTER(LossChain), _d, _vp, _vp, _vp,
                                    _vp]),
    "nsgpu_fanout_spectrum": (C.c_int, [C.POINTER(PhySoA), _i64, _vp, _i64, C.POINTER(LossChain), _d, _d, _vp,
                                        _i32, _vp, _vp, _vp, _vp, _vp]),
    "nsgpu_fanout_workspace_bytes": (C.c_int, [_i64, _i64, C.POINTER(C.c_uint64)]),
    "nsgpu_fanout_spectrum_multi": (C.c_int, [C.POINTER(PhySoA), _vp, _vp, _vp, _i64, C.POINTER(SpectrumModels), _vp,
                                              _vp, _vp, _i64, C.POINTER(LossChain), _d, _d, _vp, _vp, _vp, _vp, _vp,
                                              _vp]),
    "nsgpu_fanout_multi_workspace_bytes": (C.c_int, [_i64, _i64, _i32, _i32, C.POINTER(C.c_uint64)]),
    "nsgpu_hold_workspace_bytes": (C.c_int, [_u32, C.POINTER(C.c_uint64)]),
    "nsgpu_hold_set_profile": (C.c_int, [_vp]),
    "nsgpu_sched_create": (C.c_int, [_u32, _vp, C.POINTER(C.c_void_p)]),
    "nsgpu_sched_destroy": (C.c_int, [_vp]),
    "nsgpu_sched_insert": (C.c_int, [_vp, _vp, _u64]),
    "nsgpu_sched_is_empty": (C.c_int, [_vp, C.POINTER(C.c_int)]),
    "nsgpu_sched_size": (C.c_int, [_vp, C.POINTER(C.c_uint64)]),
    "nsgpu_sched_peek_next": (C.c_int, [_vp, _vp]),
    "nsgpu_sched_remove_next": (C.c_int, [_vp, _vp]),
    "nsgpu_sched_remove": (C.c_int, [_vp, _vp]),
    "nsgpu_sim_create": (C.c_int, [_u32, _vp, C.POINTER(C.c_void_p)]),
    "nsgpu_sim_free": (C.c_int, [_vp]),
    "nsgpu_sim_schedule": (C.c_int, [_vp, _i64, _vp, _vp, _u64, _vp]),
    "nsgpu_sim_schedule_with_context": (C.c_int, [_vp, _u32, _i64, _vp, _vp, _u64]),
    "nsgpu_sim_schedule_now": (C.c_int, [_vp, _vp, _vp, _u64, _vp]),
    "nsgpu_sim_schedule_destroy": (C.c_int, [_vp, _vp, _vp, _u64, _vp]),
    "nsgpu_sim_is_expired": (C.c_int, [_vp, _vp, C.POINTER(C.c_int)]),
    "nsgpu_sim_cancel": (C.c_int, [_vp, _vp]),
    "nsgpu_sim_remove": (C.c_int, [_vp, _vp]),
    "nsgpu_sim_run": (C.c_int, [_vp]),
    "nsgpu_sim_stop": (C.c_int, [_vp]),
    "nsgpu_sim_stop_at": (C.c_int, [_vp, _i64]),
    "nsgpu_sim_destroy": (C.c_int, [_vp]),
    "nsgpu_sim_state": (C.c_int, [_vp, _vp, _vp, _vp, _vp]),
    "nsgpu_sim_current_uid": (C.c_int, [_vp, _vp]),
    "nsgpu_sim_set_next_uid": (C.c_int, [_vp, _u32]),
    "nsgpu_sim_next": (C.c_int, [_vp, _vp, _vp]),
    "nsgpu_sim_set_stop": (C.c_int, [_vp, C.c_int]),
    "nsgpu_sim_drain": (C.c_int, [_vp, _vp, _u32, _vp]),
    "nsgpu_sim_pop_window": (C.c_int, [_vp, _vp, _u32, _vp]),
    "nsgpu_sim_begin": (C.c_int, [_vp, _vp, _vp]),
    "nsgpu_sim_insert": (C.c_int, [_vp, _u64, _u32, _u64, _vp]),
    "nsgpu_sim_consume_uid": (C.c_int, [_vp, _vp]),
    "nsgpu_sim_remove_key": (C.c_int, [_vp, _u64, _u32, _u32, _u64]),
    "nsgpu_sim_key_expired": (C.c_int, [_vp, _u64, _u32, _vp]),
    "nsgpu_sim_host_stats": (C.c_int, [_vp, _vp, _vp, _vp]),
    "nsgpu_sim_sched_stats": (C.c_int, [_vp, _vp, _vp, _vp]),
    "nsgpu_sim_set_log": (C.c_int, [_vp, _vp, _vp, _vp, _u64]),
    "nsgpu_sim_attach_p2p": (C.c_int, [_vp, _vp]),
    "nsgpu_sim_adopt_p2p": (C.c_int, [_vp, _vp]),
    "nsgpu_sim_p2p_send": (C.c_int, [_vp, _u32]),
    "nsgpu_sim_attach_wifi": (C.c_int, [_vp, _vp]),
    "nsgpu_sim_wifi_send": (C.c_int, [_vp, _u32, _u32, C.c_double, _u32, _u64, _u32, _u32]),
    "nsgpu_sim_wifi_state": (C.c_int, [_vp, _u32, _vp]),
    "nsgpu_sim_wifi_set_position": (C.c_int, [_vp, _u32, _d, _d, _d]),
    "nsgpu_wifil_set_position": (C.c_int, [_vp, _u32, _d, _d, _d]),
    "nsgpu_wifil_create": (C.c_int, [_vp, _vp]),
    "nsgpu_wifil_destroy": (C.c_int, [_vp]),
    "nsgpu_wifil_receivers": (C.c_int, [_vp, _u32, _vp]),
    "nsgpu_wifil_send": (C.c_int, [_vp, _u64, _u32, _u32, _u32, C.c_double, _u32, _u64, _u32, _u32]),
    "nsgpu_wifil_advance": (C.c_int, [_vp, _u64, _u32, _vp, _vp, _vp, _vp, _vp, _vp, _u64]),
    "nsgpu_wifil_flush": (C.c_int, [_vp, _vp]),
    "nsgpu_wifil_get_state": (C.c_int, [_vp, _u32, _u64, _vp]),
    "nsgpu_wifil_read_ends": (C.c_int, [_vp, _vp, _u64, _vp]),
    "nsgpu_wifil_read_phys": (C.c_int, [_vp, _vp]),
    "nsgpu_wifil_pending": (C.c_int, [_vp, _vp, _vp]),
    "nsgpu_sim_is_finished": (C.c_int, [_vp, _vp]),
    "nsgpu_sim_run_one": (C.c_int, [_vp]),
    "nsgpu_sim_pop_one": (C.c_int, [_vp, _vp, _vp]),
    "nsgpu_sim_live_closures": (C.c_int, [_vp, _vp]),
    "nsgpu_sim_destroy_insert": (C.c_int, [_vp, _u64, _vp]),
    "nsgpu_sim_destroy_pop": (C.c_int, [_vp, _vp, _vp]),
    "nsgpu_sim_destroy_remove": (C.c_int, [_vp, _u64, _u64, _vp]),
    "nsgpu_sim_destroy_pending": (C.c_int, [_vp, _u64, _u64, _vp]),
    "nsgpu_sched_stats": (C.c_int, [_vp, _vp, _vp, _vp]),
    "nsgpu_p2p_pending": (C.c_int, [_vp, _vp, _vp, _vp, _vp]),
    "nsgpu_p2p_get_wide": (C.c_int, [_vp, _vp]),
    "nsgpu_p2p_setup_uid": (C.c_int, [_vp, _vp]),
    "nsgpu_p2p_advance": (C.c_int, [_vp, _u64, _u32, _vp, _vp, _vp, _vp]),
    "nsgpu_p2p_inject_send": (C.c_int, [_vp, _u32, _u64, _u32, _u32, _vp, _vp, _vp]),
    "nsgpu_p2p_counters": (C.c_int, [_vp, _vp, _vp, _vp]),
    "nsgpu_p2p_create": (C.c_int, [_vp, _u64, _u64, C.POINTER(C.c_void_p)]),
    "nsgpu_p2p_reset": (C.c_int, [_vp, _vp]),
    "nsgpu_p2p_run": (C.c_int, [_vp, _vp]),
    "nsgpu_p2p_results": (C.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _u64, _vp, _vp]),
    "nsgpu_p2p_destroy": (C.c_int, [_vp]),
    "nsgpu_p2p_last_run_ms": (C.c_int, [_vp, C.POINTER(C.c_double)]),
    "nsgpu_p2p_set_eager": (C.c_int, [_vp, C.c_int]),
    "nsgpu_p2p_set_trace": (C.c_int, [_vp, _u64]),
    "nsgpu_p2p_set_trace_kinds": (C.c_int, [_vp, C.c_uint32]),
    "nsgpu_p2p_trace_read": (C.c_int, [_vp, _vp, _u64, C.POINTER(C.c_uint64), _vp]),
    "nsgpu_p2p_phase_read": (C.c_int, [_vp, C.c_int, C.c_int]),
    "nsgpu_p2p_kernel_count": (C.c_int, [C.POINTER(C.c_int)]),
    "nsgpu_p2p_kernel_name": (C.c_char_p, [C.c_int]),
    "nsgpu_probe_latency": (C.c_int, [_vp, _vp, _vp]),
    "nsgpu_p2p_profile": (C.c_int, [_vp, _vp, _u32, _vp, _vp]),
    "nsgpu_comm_unique_id": (C.c_int, [_vp]),
    "nsgpu_comm_init": (C.c_int, [_vp, C.c_int, C.c_int, C.POINTER(C.c_void_p)]),
    "nsgpu_comm_destroy": (C.c_int, [_vp]),
    "nsgpu_p2p_create_dist": (C.c_int, [_vp, _vp, C.c_int, C.c_int, _vp, _u64, _u64, C.POINTER(C.c_void_p)]),
    "nsgpu_p2p_dist_plan": (C.c_int, [_vp, _vp, C.c_int, C.c_int, _u64, _vp]),
    "nsgpu_wifil_listen": (C.c_int, [_vp, _u32, C.c_int]),
    "nsgpu_wifil_send_plan": (C.c_int, [_vp, _u32, _u32, _vp, _vp, _vp, _u64, C.POINTER(C.c_uint64)]),
    "nsgpu_wifil_next_end": (C.c_int, [_vp, _vp]),
    "nsgpu_wifil_create_dist": (C.c_int, [_vp, C.c_int64, C.c_int64, _vp, C.POINTER(C.c_void_p)]),
    "nsgpu_wifil_create_group": (C.c_int, [_vp, _vp, C.c_int, C.POINTER(C.c_void_p)]),
    "nsgpu_sim_wifi_set_end_handler": (C.c_int, [_vp, _vp, _vp]),
    "nsgpu_sim_wifi_listen": (C.c_int, [_vp, _u32, C.c_int]),
    "nsgpu_p2p_group_create": (C.c_int, [_vp, C.c_int, C.POINTER(C.c_void_p)]),
    "nsgpu_p2p_group_reset": (C.c_int, [_vp, _vp]),
    "nsgpu_p2p_group_run": (C.c_int, [_vp, _vp]),
    "nsgpu_p2p_group_destroy": (C.c_int, [_vp]),
    "nsgpu_hold_run": (C.c_int, [_vp, _u32, _u32, _vp, _vp, _vp, _u64, _vp, _vp]),
    "nsgpu_wifi_tx_duration_ns": (C.c_int, [_u32, _u32, _u64, _u32, _u32, _vp]),
    "nsgpu_wifi_create": (C.c_int, [_vp, C.c_int, C.POINTER(C.c_void_p)]),
    "nsgpu_wifi_create_dist": (C.c_int, [_vp, C.c_int, C.c_int64, C.c_int64, _vp, C.POINTER(C.c_void_p)]),
    "nsgpu_wifi_group_run": (C.c_int, [_vp, C.c_int, _vp]),
    "nsgpu_wifi_run": (C.c_int, [_vp, _vp]),
    "nsgpu_wifi_get_stats": (C.c_int, [_vp, _vp]),
    "nsgpu_wifi_read_phys": (C.c_int, [_vp, _vp]),
    "nsgpu_wifi_read_tx_base": (C.c_int, [_vp, _vp]),
    "nsgpu_wifi_read_ends": (C.c_int, [_vp, _vp, _u64, _vp]),
    "nsgpu_wifi_read_rx_log": (C.c_int, [_vp, _vp]),
    "nsgpu_wifi_destroy": (C.c_int, [_vp]),
    "nsgpu_wifi_set_store": (C.c_int, [_vp, C.c_int]),
    "nsgpu_wifi_get_store": (C.c_int, [_vp, _vp, _vp, _vp]),
    "nsgpu_wifi_kernel_count": (C.c_int, [C.POINTER(C.c_int)]),
    "nsgpu_wifi_kernel_name": (C.c_char_p, [C.c_int]),
    "nsgpu_wifi_profile": (C.c_int, [_vp, _vp, _vp]),
    # trace codec (host code in libnsgpu: nsgpu_trace.cc)
    "nsgpu_trace_codec_create": (C.c_int, [_vp, _vp, _vp]),
    "nsgpu_trace_codec_free": (C.c_int, [_vp]),
    "nsgpu_time_get_seconds": (C.c_double, [_i64]),
    "nsgpu_setup_from_journal": (C.c_int, [_vp, _u64, _u32, _vp, _vp, _vp, _vp]),
    "nsgpu_trace_sort": (C.c_int, [_vp, _u64]),
    "nsgpu_trace_line": (C.c_int, [_vp, _vp, _vp, _u64, _vp]),
    "nsgpu_trace_packet": (C.c_int, [_vp, _vp, _vp, _u64, _vp]),
    "nsgpu_trace_ascii": (C.c_int, [_vp, _vp, _u64, _vp, _u64, _vp]),
    "nsgpu_trace_pcap": (C.c_int, [_vp, _vp, _u64, _u32, _vp, _u64, _vp]),
    "nsgpu_pcap_file": (C.c_int, [_u32, _u32, _u64, _vp, _vp, _vp, _vp, _vp, _vp, _u64, _vp]),
    "nsgpu_wifi_sniff_power": (C.c_int, [_vp, C.c_double, _vp, _vp]),
    "nsgpu_wifi_pcap": (C.c_int, [_u32, _vp, _u64, _u32, _vp, _vp, _vp, _u64, _vp]),
    "nsgpu_wifi_ascii": (C.c_int, [_vp, _u64, _vp, _vp, _vp, _vp, _vp, _u64, _vp]),
}

_lib = None


def lib():
    """Load libnsgpu.so (fails loudly if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NsgpuError(f"{LIB_PATH} is missing: build it with `make -C ns-3-dev-dnemu_amd` "
                             "(or __graft_entry__.build()); there is no CPU fallback")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        _lib = L
    return _lib


def check(status):
    if status != 0:
        raise NsgpuError(f"nsgpu error {status}: {lib().nsgpu_last_error().decode()}")


def device_count():
    n = C.c_int(0)
    check(lib().nsgpu_device_count(C.byref(n)))
    return n.value


class DeviceBuffer:
    """A hipMalloc'd buffer (owned), with numpy upload/download."""

    def __init__(self, nbytes):
        self.nbytes = int(nbytes)
        p = C.c_void_p()
        check(lib().nsgpu_malloc(C.byref(p), max(self.nbytes, 1)))
        self.ptr = p.value

    @classmethod
    def from_array(cls, arr, stream=None):
        arr = np.ascontiguousarray(arr)
        b = cls(arr.nbytes)
        if arr.nbytes:
            check(lib().nsgpu_memcpy_htod(b.ptr, arr.ctypes.data, arr.nbytes, stream))
            check(lib().nsgpu_stream_sync(stream))
        return b

    def zero(self, stream=None):
        check(lib().nsgpu_memset(self.ptr, 0, self.nbytes, stream))

    def download(self, dtype, count=None, stream=None):
        dtype = np.dtype(dtype)
        count = self.nbytes // dtype.itemsize if count is None else count
        out = np.empty(count, dtype=dtype)
        if out.nbytes:
            check(lib().nsgpu_memcpy_dtoh(out.ctypes.data, self.ptr, out.nbytes, stream))
        return out

    def free(self):
        if self.ptr:
            lib().nsgpu_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def device_synchronize():
    check(lib().nsgpu_device_synchronize())


class Stream:
    def __init__(self):
        p = C.c_void_p()
        check(lib().nsgpu_stream_create(C.byref(p)))
        self.handle = p.value

    def sync(self):
        check(lib().nsgpu_stream_sync(self.handle))

    def __del__(self):
        try:
            lib().nsgpu_stream_destroy(self.handle)
        except Exception:
            pass


class Timer:
    """HIP events recorded on the stream the kernels are launched on."""

    def __init__(self):
        a, b = C.c_void_p(), C.c_void_p()
        check(lib().nsgpu_event_create(C.byref(a)))
        check(lib().nsgpu_event_create(C.byref(b)))
        self.a, self.b = a.value, b.value

    def start(self, stream):
        check(lib().nsgpu_event_record(self.a, stream))

    def stop(self, stream):
        check(lib().nsgpu_event_record(self.b, stream))

    def elapsed_ms(self):
        ms = C.c_float()
        check(lib().nsgpu_event_elapsed_ms(self.a, self.b, C.byref(ms)))
        return ms.value


def loss_chain(*models):
    ch = LossChain()
    ch.n = len(models)
    for i, (k, a, b, c) in enumerate(models):
        ch.m[i].kind, ch.m[i].p0, ch.m[i].p1, ch.m[i].p2 = k, a, b, c
    return ch


# ---------------- operations ----------------
def seconds_to_ts(values, stream=None):
    v = np.ascontiguousarray(values, dtype=np.float64)
    din = DeviceBuffer.from_array(v, stream)
    dout = DeviceBuffer(v.nbytes)
    check(lib().nsgpu_seconds_to_ts(din.ptr, dout.ptr, v.size, stream))
    return dout.download(np.int64, v.size, stream)


class PhyList:
    """m_phyList of a broadcast channel, resident in HBM as SoA."""

    def __init__(self, x, y, z, channel, node, stream=None):
        self.n = len(x)
        self.bufs = [DeviceBuffer.from_array(np.asarray(a, dtype=t), stream) for a, t in
                     ((x, np.float64), (y, np.float64), (z, np.float64), (channel, np.uint32), (node, np.uint32))]
        self.stream = stream
        self.channel = np.array(channel, dtype=np.uint32)
        self._rank_tables()

    def _rank_tables(self):
        # per-channel rank / size of every phy (m_phyList order): Yans records are placed without counting
        ch = self.channel
        order = np.argsort(ch, kind="stable")
        sch = ch[order]
        first = np.r_[True, sch[1:] != sch[:-1]] if ch.size else np.zeros(0, bool)
        start = np.maximum.accumulate(np.where(first, np.arange(ch.size), 0)) if ch.size else np.zeros(0, np.int64)
        rank = np.empty(ch.size, np.uint32)
        rank[order] = (np.arange(ch.size) - start).astype(np.uint32)
        _u, inv, cnt = np.unique(ch, return_inverse=True, return_counts=True)
        count = cnt[inv].astype(np.uint32)
        self.bufs[5:] = [DeviceBuffer.from_array(rank, self.stream), DeviceBuffer.from_array(count, self.stream)]
        self.soa = PhySoA(*[b.ptr for b in self.bufs])

    def set_channel(self, j, ch):
        """YansWifiPhy::SetChannelNumber (yans-wifi-phy.cc:328-358) on phy j: the channel array and the rank
        tables that depend on it are updated together (include/nsgpu.h, nsgpu_phy_soa)."""
        self.channel[j] = ch
        self.bufs[3] = DeviceBuffer.from_array(self.channel, self.stream)
        self._rank_tables()


class MultiModelFanout:
    """MultiModelSpectrumChannel::StartTx over a resident phy list (nsgpu_fanout_spectrum_multi).

    models: list of (fl, fh) band-edge arrays in ascending SpectrumModelUid order; rx_model[j]: phy j's
    model index.  The visit order (m_rxSpectrumModelInfoMap by model, AddRx order within) is built here."""

    def __init__(self, phys, rx_model, models, max_tx, stream=None):
        self.phys, self.max_tx, self.stream = phys, max_tx, stream
        self.rx_model = np.asarray(rx_model, np.int32)
        self.nb = np.array([len(fl) for fl, _ in models], np.int64)
        self.max_bands = int(self.nb.max())
        off = np.zeros(len(models) + 1, np.uint32)
        off[1:] = np.cumsum(self.nb)
        fl = np.concatenate([np.asarray(a, np.float64) for a, _ in models])
        fh = np.concatenate([np.asarray(b, np.float64) for _, b in models])
        it = np.argsort(self.rx_model, kind="stable").astype(np.uint32)
        pos = np.empty_like(it)
        pos[it] = np.arange(it.size, dtype=np.uint32)
        self.bufs = [DeviceBuffer.from_array(a, stream) for a in (self.rx_model, it, pos, off, fl, fh)]
        self.models = SpectrumModels(len(models), self.max_bands, self.bufs[3].ptr, self.bufs[4].ptr, self.bufs[5].ptr)
        n = phys.n
        ws = C.c_uint64()
        check(lib().nsgpu_fanout_multi_workspace_bytes(n, max_tx, len(models), self.max_bands, C.byref(ws)))
        self.ws = DeviceBuffer(ws.value)
        self.out = DeviceBuffer(max_tx * (n - 1) * RX_RECORD_DTYPE.itemsize)
        self.psd_out = DeviceBuffer(max_tx * (n - 1) * self.max_bands * 8)
        self.trace = DeviceBuffer(max_tx * (n - 1) * LOSS_TRACE_DTYPE.itemsize)
        self.count = DeviceBuffer(max_tx * 4)
        self.tx = DeviceBuffer(max_tx * TX_DESC_DTYPE.itemsize)
        self.tx_model = DeviceBuffer(max_tx * 4)
        self.psd_tx = DeviceBuffer(max_tx * self.max_bands * 8)

    def upload_tx(self, tx, tx_model, psd_tx):
        """psd_tx: [n_tx, max_bands] (each row's first nbands(tx_model) values used)."""
        tx = np.ascontiguousarray(tx, dtype=TX_DESC_DTYPE)
        assert len(tx) <= self.max_tx
        tm = np.ascontiguousarray(tx_model, np.int32)
        p = np.zeros((len(tx), self.max_bands), np.float64)
        for t, row in enumerate(psd_tx):
            p[t, :len(row)] = row
        for src, dst in ((tx, self.tx), (tm, self.tx_model), (p, self.psd_tx)):
            check(lib().nsgpu_memcpy_htod(dst.ptr, src.ctypes.data, src.nbytes, self.stream))
        return len(tx)

    def launch(self, n_tx, chain, speed, max_loss_db, trace=True):
        check(lib().nsgpu_fanout_spectrum_multi(C.byref(self.phys.soa), self.bufs[0].ptr, self.bufs[1].ptr,
                                                self.bufs[2].ptr, self.phys.n, C.byref(self.models), self.tx.ptr,
                                                self.tx_model.ptr, self.psd_tx.ptr, n_tx, C.byref(chain), speed,
                                                max_loss_db, self.out.ptr, self.psd_out.ptr,
                                                self.trace.ptr if trace else None, self.count.ptr, self.ws.ptr,
                                                self.stream))

    def results(self, n_tx):
        """Per transmission: (records, PSD rows trimmed to each receiver's model, loss-trace entries)."""
        n = self.phys.n
        counts = self.count.download(np.uint32, n_tx, self.stream)
        recs = self.out.download(RX_RECORD_DTYPE, n_tx * (n - 1), self.stream).reshape(n_tx, n - 1)
        psd = self.psd_out.download(np.float64, n_tx * (n - 1) * self.max_bands, self.stream)
        psd = psd.reshape(n_tx, n - 1, self.max_bands)
        tr = self.trace.download(LOSS_TRACE_DTYPE, n_tx * (n - 1), self.stream).reshape(n_tx, n - 1)
        out = []
        for t in range(n_tx):
            r = recs[t, :counts[t]]
            rows = [psd[t, k, :self.nb[self.rx_model[r["phy"][k]]]] for k in range(len(r))]
            out.append((r, rows, tr[t]))
        return out


class Fanout:
    """Batched broadcast fan-out (Yans / single-model spectrum) over a resident PhyList."""

    def __init__(self, phys, max_tx, nbands=0, stream=None):
        self.phys, self.max_tx, self.nbands, self.stream = phys, max_tx, nbands, stream
        ws = C.c_uint64()
        check(lib().nsgpu_fanout_workspace_bytes(phys.n, max_tx, C.byref(ws)))
        self.ws = DeviceBuffer(ws.value)
        self.out = DeviceBuffer(max_tx * (phys.n - 1) * RX_RECORD_DTYPE.itemsize)
        self.count = DeviceBuffer(max_tx * 4)
        self.tx = DeviceBuffer(max_tx * TX_DESC_DTYPE.itemsize)
        self.psd_out = DeviceBuffer(max_tx * (phys.n - 1) * max(nbands, 1) * 8) if nbands else None
        self.psd_tx = DeviceBuffer(max_tx * max(nbands, 1) * 8) if nbands else None

    def upload_tx(self, tx):
        tx = np.ascontiguousarray(tx, dtype=TX_DESC_DTYPE)
        assert len(tx) <= self.max_tx
        check(lib().nsgpu_memcpy_htod(self.tx.ptr, tx.ctypes.data, tx.nbytes, self.stream))
        return len(tx)

    def launch_yans(self, n_tx, chain, speed):
        check(lib().nsgpu_fanout_yans(C.byref(self.phys.soa), self.phys.n, self.tx.ptr, n_tx, C.byref(chain), speed,
                                      self.out.ptr, self.count.ptr, self.ws.ptr, self.stream))

    def launch_spectrum(self, n_tx, chain, speed, max_loss_db):
        check(lib().nsgpu_fanout_spectrum(C.byref(self.phys.soa), self.phys.n, self.tx.ptr, n_tx, C.byref(chain),
                                          speed, max_loss_db, self.psd_tx.ptr if self.psd_tx else None,
                                          self.nbands, self.out.ptr, self.psd_out.ptr if self.psd_out else None,
                                          self.count.ptr, self.ws.ptr, self.stream))

    def results(self, n_tx):
        counts = self.count.download(np.uint32, n_tx, self.stream)
        recs = self.out.download(RX_RECORD_DTYPE, n_tx * (self.phys.n - 1), self.stream)
        recs = recs.reshape(n_tx, self.phys.n - 1)
        out = [recs[t, :counts[t]] for t in range(n_tx)]
        psd = None
        if self.nbands:
            p = self.psd_out.download(np.float64, n_tx * (self.phys.n - 1) * self.nbands, self.stream)
            p = p.reshape(n_tx, self.phys.n - 1, self.nbands)
            psd = [p[t, :counts[t]] for t in range(n_tx)]
        return out, psd


class HoldRun:
    """GPU-resident utils/bench-simulator.cc run (config 1)."""

    def __init__(self, dist_ns, total, log_cap=0, stream=None):
        self.dist_ns = np.ascontiguousarray(dist_ns, dtype=np.uint64)
        self.n, self.total, self.log_cap, self.stream = self.dist_ns.size, int(total), int(log_cap), stream
        self.d_dist = DeviceBuffer.from_array(self.dist_ns, stream)
        ws = C.c_uint64()
        check(lib().nsgpu_hold_workspace_bytes(self.n, C.byref(ws)))
        self.ws = DeviceBuffer(ws.value)
        self.stats = DeviceBuffer(C.sizeof(HoldStats))
        self.log_ts = DeviceBuffer(max(log_cap, 1) * 8)
        self.log_uid = DeviceBuffer(max(log_cap, 1) * 4)

    def launch(self):
        check(lib().nsgpu_hold_run(self.d_dist.ptr, self.n, self.total, self.stats.ptr,
                                   self.log_ts.ptr if self.log_cap else None,
                                   self.log_uid.ptr if self.log_cap else None, self.log_cap, self.ws.ptr,
                                   self.stream))

    def result(self):
        raw = self.stats.download(np.uint8, C.sizeof(HoldStats), self.stream)
        st = HoldStats.from_buffer_copy(raw.tobytes())
        if self.log_cap:
            return st, self.log_ts.download(np.uint64, self.log_cap, self.stream), \
                self.log_uid.download(np.uint32, self.log_cap, self.stream)
        return st, None, None


# ---------------- HipBatchScheduler / HipSimulatorImpl host runtime ----------------
EVENT_DTYPE = np.dtype([("ts", "<u8"), ("uid", "<u4"), ("context", "<u4"), ("handle", "<u8")])


class EventId(C.Structure):  # nsgpu_event_id
    _fields_ = [("impl", C.c_uint64), ("ts", C.c_uint64), ("context", C.c_uint32), ("uid", C.c_uint32)]


EVENT_FN = C.CFUNCTYPE(None, C.c_void_p, C.c_uint64)
WIFI_END_FN = C.CFUNCTYPE(None, C.c_void_p, C.c_void_p)  # nsgpu_wifi_end_fn (user, const nsgpu_wifil_end *)


class Sched:
    """ns3::Scheduler interface over the HBM-resident batch scheduler (nsgpu_sched_*)."""

    def __init__(self, batch=4096, stream=None):
        h = C.c_void_p()
        check(lib().nsgpu_sched_create(batch, stream, C.byref(h)))
        self.h = h.value

    def insert(self, events):
        ev = np.ascontiguousarray(events, dtype=EVENT_DTYPE)
        check(lib().nsgpu_sched_insert(self.h, ev.ctypes.data, ev.size))

    def is_empty(self):
        e = C.c_int()
        check(lib().nsgpu_sched_is_empty(self.h, C.byref(e)))
        return bool(e.value)

    def size(self):
        n = C.c_uint64()
        check(lib().nsgpu_sched_size(self.h, C.byref(n)))
        return n.value

    def _one(self, f):
        out = np.zeros(1, EVENT_DTYPE)
        check(f(self.h, out.ctypes.data))
        return out[0]

    def peek_next(self):
        return self._one(lib().nsgpu_sched_peek_next)

    def remove_next(self):
        return self._one(lib().nsgpu_sched_remove_next)

    def remove(self, ev):
        e = np.array([tuple(ev)], dtype=EVENT_DTYPE)
        check(lib().nsgpu_sched_remove(self.h, e.ctypes.data))

    def __del__(self):
        try:
            lib().nsgpu_sched_destroy(self.h)
        except Exception:
            pass


class Sim:
    """HipSimulatorImpl host runtime with Python closures (the checker's Sim has the same interface)."""

    def __init__(self, batch=64, stream=None):
        h = C.c_void_p()
        check(lib().nsgpu_sim_create(batch, stream, C.byref(h)))
        self.h = h.value
        self._keep = []

    def _fn(self, cb):
        f = EVENT_FN(lambda user, arg: cb())
        self._keep.append(f)
        return f

    def schedule(self, delay, cb):
        i = EventId()
        check(lib().nsgpu_sim_schedule(self.h, delay, C.cast(self._fn(cb), C.c_void_p), None, 0, C.byref(i)))
        return i

    def schedule_with_context(self, ctx, delay, cb):
        check(lib().nsgpu_sim_schedule_with_context(self.h, ctx, delay, C.cast(self._fn(cb), C.c_void_p), None, 0))

    def schedule_now(self, cb):
        i = EventId()
        check(lib().nsgpu_sim_schedule_now(self.h, C.cast(self._fn(cb), C.c_void_p), None, 0, C.byref(i)))
        return i

    def schedule_destroy(self, cb):
        i = EventId()
        check(lib().nsgpu_sim_schedule_destroy(self.h, C.cast(self._fn(cb), C.c_void_p), None, 0, C.byref(i)))
        return i

    def remove(self, eid):
        check(lib().nsgpu_sim_remove(self.h, C.byref(eid)))

    def cancel(self, eid):
        check(lib().nsgpu_sim_cancel(self.h, C.byref(eid)))

    def is_expired(self, eid):
        e = C.c_int()
        check(lib().nsgpu_sim_is_expired(self.h, C.byref(eid), C.byref(e)))
        return bool(e.value)

    def run(self):
        check(lib().nsgpu_sim_run(self.h))

    def run_one(self):
        check(lib().nsgpu_sim_run_one(self.h))

    def is_finished(self):
        f = C.c_int()
        check(lib().nsgpu_sim_is_finished(self.h, C.byref(f)))
        return bool(f.value)

    def next(self):
        ts, empty = C.c_uint64(), C.c_int()
        check(lib().nsgpu_sim_next(self.h, C.byref(ts), C.byref(empty)))
        return None if empty.value else ts.value

    def live_closures(self):
        n = C.c_uint64()
        check(lib().nsgpu_sim_live_closures(self.h, C.byref(n)))
        return n.value

    def stop(self, delay=None):
        if delay is None:
            check(lib().nsgpu_sim_stop(self.h))
        else:
            check(lib().nsgpu_sim_stop_at(self.h, delay))

    def destroy(self):
        check(lib().nsgpu_sim_destroy(self.h))

    def _state(self):
        now, ctx, disp, uid = C.c_uint64(), C.c_uint32(), C.c_uint64(), C.c_uint32()
        check(lib().nsgpu_sim_state(self.h, C.byref(now), C.byref(ctx), C.byref(disp), C.byref(uid)))
        return now.value, ctx.value, disp.value, uid.value

    def now(self):
        return self._state()[0]

    def context(self):
        return self._state()[1]

    def dispatched(self):
        return self._state()[2]

    def next_uid(self):
        return self._state()[3]

    def current_uid(self):
        """The uid of the event being dispatched (the closure now running)."""
        u = C.c_uint32()
        check(lib().nsgpu_sim_current_uid(self.h, C.byref(u)))
        return u.value

    def set_next_uid(self, uid):
        """m_uid before anything is scheduled (the uids below it were consumed by calls this runtime did not see)."""
        check(lib().nsgpu_sim_set_next_uid(self.h, uid))

    # ---- windows (the pull interface ns3::HipSimulatorImpl uses) ----
    def insert_raw(self, ts, ctx, handle):
        u = C.c_uint32()
        check(lib().nsgpu_sim_insert(self.h, ts, ctx, handle, C.byref(u)))
        return u.value

    def pop_window(self, cap=1024):
        out = np.zeros(cap, EVENT_DTYPE)
        n = C.c_uint32()
        check(lib().nsgpu_sim_pop_window(self.h, out.ctypes.data, cap, C.byref(n)))
        return out[:n.value]

    def begin(self, ev):
        e = np.array([tuple(ev)], dtype=EVENT_DTYPE)
        skip = C.c_int()
        check(lib().nsgpu_sim_begin(self.h, e.ctypes.data, C.byref(skip)))
        return skip.value

    def remove_key(self, ts, uid, ctx=0, handle=0):
        check(lib().nsgpu_sim_remove_key(self.h, ts, uid, ctx, handle))

    def drain(self, cap=1024):
        out = np.zeros(cap, EVENT_DTYPE)
        n = C.c_uint32()
        check(lib().nsgpu_sim_drain(self.h, out.ctypes.data, cap, C.byref(n)))
        return out[:n.value]

    def pop_one(self):
        out = np.zeros(1, EVENT_DTYPE)
        n = C.c_uint32()
        check(lib().nsgpu_sim_pop_one(self.h, out.ctypes.data, C.byref(n)))
        return out[:n.value]

    def set_stop(self, stop):
        check(lib().nsgpu_sim_set_stop(self.h, int(stop)))

    def key_expired(self, ts, uid):
        e = C.c_int()
        check(lib().nsgpu_sim_key_expired(self.h, ts, uid, C.byref(e)))
        return bool(e.value)

    def destroy_insert(self, handle):
        ts = C.c_uint64()
        check(lib().nsgpu_sim_destroy_insert(self.h, handle, C.byref(ts)))
        return ts.value

    def destroy_pop(self):
        h, f = C.c_uint64(), C.c_int()
        check(lib().nsgpu_sim_destroy_pop(self.h, C.byref(h), C.byref(f)))
        return h.value if f.value else None

    def destroy_remove(self, handle, ts):
        f = C.c_int()
        check(lib().nsgpu_sim_destroy_remove(self.h, handle, ts, C.byref(f)))
        return bool(f.value)

    def destroy_pending(self, handle, ts):
        p = C.c_int()
        check(lib().nsgpu_sim_destroy_pending(self.h, handle, ts, C.byref(p)))
        return bool(p.value)

    # ---- mixed host / device runs ----
    def attach_p2p(self, engine):
        check(lib().nsgpu_sim_attach_p2p(self.h, engine.h))
        self._engine = engine

    def adopt_p2p(self, engine):
        """nsgpu_sim_adopt_p2p: the engine takes over after setup-time events were scheduled here."""
        check(lib().nsgpu_sim_adopt_p2p(self.h, engine.h))
        self._engine = engine

    def p2p_send(self, app):
        check(lib().nsgpu_sim_p2p_send(self.h, app))

    def attach_wifi(self, phy):
        """Attach a closed-loop Wi-Fi PHY (wifi.LoopPhy)."""
        check(lib().nsgpu_sim_attach_wifi(self.h, phy.h))
        self._engine = phy

    def wifi_set_position(self, phy, x, y, z):
        """MobilityModel::SetPosition of `phy`'s node from the running closure."""
        check(lib().nsgpu_sim_wifi_set_position(self.h, phy, x, y, z))

    def wifi_send(self, phy, size, dbm, mode, preamble):
        """YansWifiPhy::SendPacket of `phy` now (mode = (modclass, rate, bandwidth))."""
        check(lib().nsgpu_sim_wifi_send(self.h, phy, size, dbm, mode[0], mode[1], mode[2], preamble))

    def wifi_set_end_handler(self, fn):
        """EndReceive hand-back (nsgpu_sim_wifi_set_end_handler): fn(end) — a wifi.WIFIL_END_DTYPE record — runs at
        each EndReceive of a listened phy, in the order, as YansWifiPhy::EndReceive's host part (its m_random draw
        and the MAC callbacks); fn None: none."""
        import wifi
        if fn is None:
            check(lib().nsgpu_sim_wifi_set_end_handler(self.h, None, None))
            self._end_cb = None
            return
        size = wifi.WIFIL_END_DTYPE.itemsize

        def tramp(user, p):
            fn(np.frombuffer(C.string_at(p, size), wifi.WIFIL_END_DTYPE)[0])

        self._end_cb = WIFI_END_FN(tramp)
        check(lib().nsgpu_sim_wifi_set_end_handler(self.h, C.cast(self._end_cb, C.c_void_p), None))

    def wifi_listen(self, phy, on=True):
        """The hand-back for `phy`'s EndReceives on (or off)."""
        check(lib().nsgpu_sim_wifi_listen(self.h, phy, 1 if on else 0))

    def wifi_state(self, phy):
        """WifiPhyStateHelper::GetState of `phy` now: (state, delay until idle ns)."""
        import wifi
        st = wifi.WifilPhyState()
        check(lib().nsgpu_sim_wifi_state(self.h, phy, C.byref(st)))
        return st.state, st.delay_until_idle

    def set_log(self, cap):
        self.log = (np.zeros(cap, np.uint64), np.zeros(cap, np.uint32), np.zeros(cap, np.uint32))
        check(lib().nsgpu_sim_set_log(self.h, self.log[0].ctypes.data, self.log[1].ctypes.data,
                                      self.log[2].ctypes.data, cap))

    def host_stats(self):
        n, c, d = C.c_uint64(), C.c_uint64(), C.c_uint64()
        check(lib().nsgpu_sim_host_stats(self.h, C.byref(n), C.byref(c), C.byref(d)))
        return n.value, c.value, d.value

    def close(self):
        if self.h:
            lib().nsgpu_sim_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def route_global(dev_node, dev_peer, dev_addr, dev_ifindex, n_nodes, dst_node, stream=None):
    """nsgpu_route_global: uint32 [n_nodes, n_dst] next-hop devices (0xffffffff: none / local)."""
    arrs = [np.ascontiguousarray(a, dtype=np.uint32) for a in (dev_node, dev_peer, dev_addr, dev_ifindex)]
    dst = np.ascontiguousarray(dst_node, dtype=np.uint32)
    out = np.zeros((n_nodes, dst.size), np.uint32)
    check(lib().nsgpu_route_global(n_nodes, arrs[0].size, *[a.ctypes.data for a in arrs], dst.size, dst.ctypes.data,
                                   out.ctypes.data, stream))
    return out


def probe_latency(stream=None):
    """(kernel boundary us, dependent memory trip us) measured on the current device (nsgpu_probe_latency)."""
    b, t = C.c_double(), C.c_double()
    check(lib().nsgpu_probe_latency(stream, C.byref(b), C.byref(t)))
    return b.value, t.value
