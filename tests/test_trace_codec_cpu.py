"""The product library's trace codec (include/nsgpu.h nsgpu_trace_* / nsgpu_pcap_file, implemented in
ns-3-dev-dnemu_amd/csrc/nsgpu_trace.cc) — what ns3::HipSimulatorImpl hands to the helpers' OutputStreamWrapper
and PcapFileWrapper — pinned against the reference's own outputs and checked byte for byte against the
Python codec (trace.py) on every record set the oracle produces (no GPU):

  * src/network/test/known.pcap (tests/golden/known.pcap) rebuilt by PcapFile::Init + Write
    (pcap-file.cc:300-381), and DiffTestCase's file (pcap-file-test-suite.cc:1053-1101);
  * first.cc: the 19-event run's EnableAsciiAll file and both EnablePcapAll files against the md5s of
    the unmodified reference (tests/golden/survey_reference_runs.json);
  * congested grids (queue drops), ICMP errors (time exceeded / port unreachable, echo replies) and the
    Ipv4L3Protocol Tx / Rx / Drop records: equal to trace.py line for line and byte for byte."""
import hashlib
import json
import os

import numpy as np
import pytest

import nsref
import p2p
import trace

HERE = os.path.dirname(os.path.abspath(__file__))
KNOWN = open(os.path.join(HERE, "golden", "known.pcap"), "rb").read()
KAT = json.load(open(os.path.join(HERE, "golden", "pcap_known_kat.json")))


def oracle_records(sc, kinds=nsref.TRACE_DEVICE_KINDS):
    s = sc.c_struct()
    st = p2p.P2PStats()
    devc = np.zeros(s.n_devices, p2p.DEV_COUNTERS_DTYPE)
    appc = np.zeros(s.n_apps, p2p.APP_COUNTERS_DTYPE)
    _secs, _log, tr = nsref.p2p_run_trace(s, st, devc, appc, 0, kinds=kinds)
    return st, tr


def test_known_pcap_rebuilt_by_the_library():
    hdr, recs = trace.pcap_read(KNOWN)
    out = p2p.pcap_file(hdr[5], hdr[4], [(sec, usec, data, orig) for sec, usec, _i, orig, data in recs])
    assert out == KNOWN


def test_diff_test_case_file():
    import struct
    n = KAT["n_packet_bytes"]
    recs = [(ts, tu, struct.pack("<16H", *words), orig) for ts, tu, _i, orig, words in KAT["packets"]]
    out = p2p.pcap_file(1, n, recs)
    want = trace.pcap_file_header(snaplen=n, linktype=1)
    for ts, tu, data, orig in recs:
        want += trace.pcap_record(ts, tu, data, total_len=orig, snaplen=n)
    assert out == want
    d = trace.pcap_diff(KNOWN, out)
    e = KAT["diff_expected"]
    assert d == (e["file_vs_different"], e["sec"], e["usec"])


def test_first_cc_md5s_from_the_library():
    ref = json.load(open(os.path.join(HERE, "golden", "survey_reference_runs.json")))["first_cc"]
    sc = p2p.first_cc()
    st, tr = oracle_records(sc)
    assert st.dispatched == 19
    cc = p2p.TraceCodec(sc)
    tr = cc.sort(tr)
    assert np.array_equal(tr, trace.sort_records(tr))
    text = cc.ascii(tr)
    assert hashlib.md5(text.encode()).hexdigest() == ref["ascii_md5"]
    py = trace.Codec(sc)
    pc = cc.pcaps(tr, [py.ifindex[d] for d in range(len(sc.dev))])
    assert hashlib.md5(pc[(0, 0)]).hexdigest() == ref["node0_pcap_md5"]
    assert hashlib.md5(pc[(1, 0)]).hexdigest().startswith(ref["node1_pcap_md5_prefix"])
    # the per-record entry points (what the plugin's sinks call)
    assert "".join(cc.line(r) for r in tr) == text
    assert all(cc.packet(r) == py.packet_bytes(r) for r in tr)


def same_as_python(sc, tr):
    cc = p2p.TraceCodec(sc)
    py = trace.Codec(sc)
    tr = cc.sort(tr)
    assert cc.ascii(tr) == py.ascii(tr)
    want = py.pcaps(tr)
    got = cc.pcaps(tr, [py.ifindex[d] for d in range(len(sc.dev))])
    assert got == want
    return tr


def test_congested_grid_same_as_python():
    # 1 Mb/s links with 4 sources per destination column: DropTail overflows (test_gpu_p2p.py's grid)
    sc = p2p.grid(5, 5, bps=1_000_000, qmax=5, rate_bps=2_000_000, stop_ns=400_000_000, sim_stop_ns=500_000_000)
    _st, tr = oracle_records(sc)
    tr = same_as_python(sc, tr)
    assert (tr["kind"] == trace.TR_DROP).sum() > 0  # (the queue drops are in the record set)


@pytest.mark.parametrize("seed", range(3))
def test_icmp_and_ipv4_records_same_as_python(seed):
    sc = p2p.random_topology(30, 60, 10, seed, ttl=3, icmp=True, sink_window=(150_000_000, 600_000_000))
    st, tr = oracle_records(sc, kinds=0x7F)
    assert st.icmp_sent > 0
    tr = same_as_python(sc, tr)
    k = tr["kind"]
    assert ((tr["app"] & trace.PKT_ICMP) != 0).sum() > 0 and (k >= trace.TR_IP_TX).sum() > 0


def test_echo_reply_time_exceeded_same_as_python():
    """An echo reply whose TTL expires (the error's origin is the server's TTL-th hop back)."""
    sc = p2p.Scenario(70, icmp=True)
    links = [sc.link(i, i + 1, 5_000_000, 2_000_000) for i in range(69)]
    sc.install_stack()
    for i, (a, b) in enumerate(links):
        sc.assign_link(a, b, p2p.ip("10.1.%d.0" % (i + 1)))
    sc.add_echo_server(69, 1_000_000_000, 20_000_000_000)
    sc.add_echo_client(0, 69, 2_000_000_000, 10_000_000_000, count=1, ttl=255)
    sc.route_bfs()
    st, tr = oracle_records(sc, kinds=0x7F)
    assert st.icmp_sent == 1
    same_as_python(sc, tr)


def test_malformed_records_are_refused():
    sc = p2p.first_cc()
    cc = p2p.TraceCodec(sc)
    r = np.zeros(1, p2p.TRACE_RECORD_DTYPE)
    r["dev"] = 99
    r["size"] = 60
    import nsgpu
    with pytest.raises(nsgpu.NsgpuError):
        cc.ascii(r)


def halfway_timestamps(n, seed=7):
    """Timestamps whose GetSeconds () lies half-way between two 6-significant-digit decimals (where ts / 1e9
    and ns-3's int64x64 path can round apart): k * 10^(e-5) + 10^(e-5) / 2 ns for ts in [10^(e+3), 10^(e+4))
    ns, over 1 ms .. 100 s, plus the two values the round-4 review found by hand."""
    rng = np.random.default_rng(seed)
    out = [840_877_500, 236_789_500]
    per = n // 5
    for e in range(2, 7):  # ts in [10^(e+3), 10^(e+4)) ns: the 6th digit is 10^(e-2) ns, half of it 10^(e-2)/2
        step = 10 ** (e - 2)
        k = rng.integers(10 ** 5, 10 ** 6, per)
        out.extend((k * step + step // 2).tolist())
    return np.array(out, dtype=np.int64)


def test_ascii_seconds_are_ns3_get_seconds():
    """trace-helper.cc:306-390 print Simulator::Now ().GetSeconds () (int64x64 MulByInvert + GetDouble,
    nstime.h:419-431), not ts / 1e9: the product codec, the Python codec and the oracle's restatement
    (nsref_get_seconds) agree on 10^6 half-way timestamps, and ts / 1e9 would differ on some of them."""
    import nsgpu
    ts = halfway_timestamps(1_000_000)
    L = nsgpu.lib()
    prod = np.fromiter((L.nsgpu_time_get_seconds(int(t)) for t in ts), np.float64, len(ts))
    ref = np.fromiter((nsref.get_seconds(int(t)) for t in ts), np.float64, len(ts))
    assert np.array_equal(prod, ref)
    assert "%g" % prod[0] == "0.840877" and "%g" % prod[1] == "0.236789"
    sample = ts[::10]
    assert all(trace.get_seconds(int(t)) == r for t, r in zip(sample, ref[::10]))
    naive = ts / 1e9
    assert (naive != ref).sum() > 1000  # the cases the old ts / 1e9 printing got wrong exist in this set
    # the codec's ascii lines carry exactly those texts: one record per timestamp through nsgpu_trace_ascii
    sc = p2p.first_cc()
    _st, tr = oracle_records(sc)
    cc = p2p.TraceCodec(sc)
    recs = np.repeat(tr[:1], len(ts))
    recs["ts"] = ts.astype(np.uint64)
    for lo in range(0, len(ts), 250_000):
        lines = cc.ascii(recs[lo:lo + 250_000]).splitlines()
        got = [ln.split(" ", 2)[1] for ln in lines]
        assert got == ["%g" % x for x in ref[lo:lo + 250_000]]
    py = trace.Codec(sc)
    assert py.ascii(recs[:2000]) == cc.ascii(recs[:2000])


def test_halfway_run_codec_same_as_python():
    """The oracle's records of a run whose Receives land on half-way timestamps (test_gpu_trace.halfway_link):
    both codecs print ns-3's GetSeconds (), which differs from ts / 1e9 on some of its lines."""
    from test_gpu_trace import halfway_link
    sc = halfway_link()
    _st, tr = oracle_records(sc)
    tr = same_as_python(sc, tr)
    text = p2p.TraceCodec(sc).ascii(tr)
    got = [ln.split(" ", 2)[1] for ln in text.splitlines()]
    assert got == [trace.seconds_text(int(t)) for t in tr["ts"]]
    assert sum(g != "%g" % (int(t) / 1e9) for g, t in zip(got, tr["ts"])) > 100


def test_codec_create_refuses_missing_arrays():
    """nsgpu_trace_codec_create checks every array it reads (app_start_ns, setup_kind / setup_index included)."""
    import ctypes as C
    import nsgpu
    sc = p2p.first_cc()
    for field in ("app_start_ns", "setup_kind", "setup_index"):
        cc = p2p.TraceCodec(sc)  # the addressing arrays
        s = sc.c_struct()
        setattr(s, field, None)
        h = C.c_void_p()
        assert nsgpu.lib().nsgpu_trace_codec_create(C.byref(s), C.byref(cc._ad), C.byref(h)) != 0
