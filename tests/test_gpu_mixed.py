"""Mixed host / device runs: host closures (C callbacks, here Python ones through ctypes) interleaved
with the GPU-resident p2p engine's events in ONE (ts, uid) order (include/nsgpu.h: nsgpu_sim_attach_p2p,
nsgpu_sim_pop_window; the engine pauses its window pipeline at the next host event's key).

The host application (oracle: nsref_p2p_run_probe, oracle/nsref_p2p.cc) is scheduled right after
setup and, every `period`, reads a PacketSink's counters (a trace / stats callback reading device
state at its point of the order) and sends one datagram of an OnOff flow through its socket
(UdpSocket::Send from a host application: device events created by a host closure), then
re-schedules itself.  The full pop log (device and host dispatches), the trace records, every
counter, the samples, digest, dispatch count and next uid must equal the oracle's."""
import numpy as np
import pytest

import nsgpu
import nsref
import p2p
import trace
from test_gpu_trace import assert_same_trace

pytestmark = pytest.mark.gpu


def run_gpu(sc, t0, period, count, app_send, app_obs, log_cap, trace_cap):
    eng = p2p.Engine(sc, log_cap=log_cap)
    eng.set_trace(trace_cap)
    eng.reset()
    sim = nsgpu.Sim()
    sim.attach_p2p(eng)
    sim.set_log(log_cap)
    samples = []
    k = [0]

    def probe():
        samples.append(eng.counters()[1][app_obs].copy())
        sim.p2p_send(app_send)
        k[0] += 1
        if k[0] < count:
            sim.schedule(period, probe)

    if count:
        sim.schedule(t0, probe)
    sim.run()
    st, devc, appc, (lts, luid, lctx) = eng.results(log_n=log_cap)
    host_n, _host_c, host_d = sim.host_stats()
    m = sim.log[1] != 0  # the host dispatches' ranks
    lts, luid, lctx = lts.copy(), luid.copy(), lctx.copy()
    lts[m], luid[m], lctx[m] = sim.log[0][m], sim.log[1][m], sim.log[2][m]
    out = dict(dispatched=sim.dispatched(), digest=(int(st.digest) + host_d) & ((1 << 64) - 1),
               next_uid=sim.next_uid(), host=host_n)
    return out, devc, appc, (lts, luid, lctx), trace.sort_records(eng.trace()), np.array(samples)


def run_oracle(sc, t0, period, count, app_send, app_obs, log_cap):
    s = sc.c_struct()
    st = p2p.P2PStats()
    devc = np.zeros(s.n_devices, p2p.DEV_COUNTERS_DTYPE)
    appc = np.zeros(s.n_apps, p2p.APP_COUNTERS_DTYPE)
    log, tr, samples = nsref.p2p_run_probe(s, st, devc, appc, t0, period, count, app_send, app_obs, log_cap)
    return st, devc, appc, log, trace.sort_records(tr), samples


def check_same(sc, o, g):
    st, devc, appc, olog, otr, osamp = o
    gout, gdevc, gappc, glog, gtr, gsamp = g
    assert gout["dispatched"] == st.dispatched
    assert gout["digest"] == st.digest
    assert gout["next_uid"] == st.next_uid
    assert np.array_equal(gdevc, devc)
    assert np.array_equal(gappc, appc)
    n = int(min(st.dispatched, len(olog[0])))
    for a, b, name in zip(glog, olog, ("ts", "uid", "ctx")):
        assert np.array_equal(a[:n], b[:n]), name
    assert len(gsamp) == len(osamp)
    for f in ("tx_packets", "rx_packets", "tx_bytes", "rx_bytes"):
        assert np.array_equal(gsamp[f], osamp[f]), f
    assert_same_trace(sc, otr, gtr)


def flows_grid():
    g = p2p.grid(5, 5, qmax=6, rate_bps=2_000_000, stop_ns=300_000_000, sim_stop_ns=350_000_000,
                 flows=[(0, 24), (4, 20), (2, 22), (10, 14)])
    return g


@pytest.mark.parametrize("t0,period,count", [
    (150_000_000, 7_300_001, 20),     # between device events
    (100_000_000, 1_000_000, 60),     # the OnOff start time itself: ties with setup-scheduled events
    (0, 433_600, 40),                 # from time 0 (ties with the setup events), at the 542-B tx time
])
def test_host_probe_interleaved_with_device_events(t0, period, count):
    sc = flows_grid()
    app_send = [i for i, a in enumerate(sc.apps) if a["kind"] == p2p.APP_ONOFF][1]
    app_obs = [i for i, a in enumerate(sc.apps) if a["kind"] == p2p.APP_SINK][0]
    o = run_oracle(sc, t0, period, count, app_send, app_obs, 400000)
    g = run_gpu(sc, t0, period, count, app_send, app_obs, 400000, 400000)
    assert g[0]["host"] == count
    check_same(sc, o, g)


def test_host_probe_after_device_stop_is_not_run():
    """Simulator::Stop (a device event of the scenario) ends Run: host closures after it never run."""
    sc = flows_grid()
    app_send = [i for i, a in enumerate(sc.apps) if a["kind"] == p2p.APP_ONOFF][0]
    app_obs = [i for i, a in enumerate(sc.apps) if a["kind"] == p2p.APP_SINK][0]
    o = run_oracle(sc, 200_000_000, 20_000_000, 30, app_send, app_obs, 400000)
    g = run_gpu(sc, 200_000_000, 20_000_000, 30, app_send, app_obs, 400000, 400000)
    assert 0 < len(g[5]) < 30
    o = (o[0], o[1], o[2], o[3], o[4], o[5][:len(g[5])])  # (the oracle's sample buffer has `count` slots)
    check_same(sc, o, g)


def test_pull_windows_same_time_group_and_remove():
    """The raw-handle pull interface (what ns3::HipSimulatorImpl::Run uses): a window is every event of
    the smallest time; an event scheduled during the window sorts after it; a window event removed by
    an earlier one of the same window is skipped; dispatch order equals the (ts, uid) order."""
    s = nsgpu.Sim(batch=4)
    order = []
    uids = {}
    for h, ts in ((2, 50), (4, 10), (6, 10), (8, 10), (10, 30)):
        uids[h] = (ts, s.insert_raw(ts, 0, h))
    while True:
        w = s.pop_window()
        if len(w) == 0:
            break
        assert len(set(int(x) for x in w["ts"])) == 1
        for ev in w:
            if s.begin(ev) != 0:
                continue
            h = int(ev["handle"]) & ~1
            order.append(h)
            if h == 4:  # removes a later event of its own window and schedules one at the same time
                s.remove_key(*uids[8])
                uids[12] = (10, s.insert_raw(10, 0, 12))
    assert order == [4, 6, 12, 10, 2]


def test_run_after_device_stop_with_host_events_fails_loudly():
    """a device-dispatched Simulator::Stop ends the Run; a later Run (the pull interface that
    ns3::HipSimulatorImpl::Run uses) with host events still pending must fail, not return silently —
    the reference would resume them (default-simulator-impl.cc:153-165), this engine cannot."""
    sc = flows_grid()
    eng = p2p.Engine(sc, log_cap=0)
    eng.reset()
    sim = nsgpu.Sim()
    sim.attach_p2p(eng)
    ran = []
    sim.schedule(sc.stop_ns + 10_000_000, lambda: ran.append(1))  # after the device's Stop
    while len(sim.pop_window()):  # HipSimulatorImpl::Run: windows until an empty one
        pass
    assert ran == []
    with pytest.raises(nsgpu.NsgpuError, match="Simulator::Stop"):
        sim.pop_window()  # the next Run


def test_run_one_with_engine_attached_is_refused():
    """RunOneEvent dispatches ONE event (default-simulator-impl.cc:167-170); an attached engine
    advances in windows, so the one-event step is refused rather than running many device events."""
    sc = flows_grid()
    eng = p2p.Engine(sc, log_cap=0)
    eng.reset()
    sim = nsgpu.Sim()
    sim.attach_p2p(eng)
    sim.schedule(1000, lambda: None)
    with pytest.raises(nsgpu.NsgpuError, match="RunOneEvent"):
        sim.pop_one()


def test_send_after_engine_finished_is_refused():
    """once the attached engine has run out of device events (a Run with nothing pending on the
    host either ends there) it is not advanced again, so a UdpSocket::Send through it from a later Run's
    closure is refused with a clear error instead of queueing a datagram that would never be dispatched."""
    sc = p2p.grid(2, 2, stop_ns=120_000_000, flows=[(0, 3)])  # (OnOff 0.1-0.12 s)
    sc.setup = [x for x in sc.setup if x[0] != p2p.SETUP_STOP]  # no Simulator::Stop: the device drains
    sc.stop_ns = -1
    eng = p2p.Engine(sc, log_cap=0)
    eng.reset()
    sim = nsgpu.Sim()
    sim.attach_p2p(eng)
    app_send = [i for i, a in enumerate(sc.apps) if a["kind"] == p2p.APP_ONOFF][0]
    sim.run()  # the device drains; no host event: the Run ends and the engine is finished
    errs = []

    def late():
        try:
            sim.p2p_send(app_send)
        except nsgpu.NsgpuError as e:
            errs.append(str(e))

    sim.schedule(1_000_000_000, late)
    sim.run()
    assert errs and "finished" in errs[0]


def adopt_run(sc, own_event_ts=None):
    """ns3::HipSimulatorImpl + NsgpuP2pScenario::FromNodeList / AdoptInto, as the C++ module calls the C-ABI:
    the program's setup-time Schedule calls go to the host runtime first (the journal: Node::Start,
    NetDevice::Start, Application::Start, ScheduleDestroy, Simulator::Stop, in program order), then the
    engine built from the same scenario takes them over (nsgpu_sim_remove_key, nsgpu_sim_adopt_p2p) and Run
    pulls windows.  `own_event_ts`: one event of the program's own, scheduled between the setup calls, that
    stays on the host."""
    sim = nsgpu.Sim()
    owned = []
    handle = 2
    own = None
    for i, (kind, k) in enumerate(sc.setup):
        if own_event_ts is not None and i == len(sc.setup) // 2:
            handle += 2
            own = (own_event_ts, sim.insert_raw(own_event_ts, 0xFFFFFFFF, handle), handle)
        handle += 2
        if kind == p2p.SETUP_UID:
            sim.destroy_insert(handle)  # (NodeListPriv / ChannelListPriv's ScheduleDestroy)
            continue
        ts, ctx = 0, 0
        if kind in (p2p.SETUP_NODE, p2p.SETUP_NOOP):
            ctx = k
        elif kind == p2p.SETUP_DEVICE:
            ctx = sc.dev[k][0]
        elif kind == p2p.SETUP_APP:
            ctx = sc.apps[k]["node"]
        elif kind == p2p.SETUP_STOP:
            ts, ctx = sc.stop_ns, 0xFFFFFFFF
        owned.append((ts, sim.insert_raw(ts, ctx, handle), ctx, handle))
    if own is not None:  # the engine's setup list counts the program's own call as a consumed uid
        j = len(sc.setup) // 2
        sc.setup.insert(j, (p2p.SETUP_UID, 0))
    eng = p2p.Engine(sc, log_cap=200000)
    eng.reset()
    for ts, uid, ctx, h in owned:
        sim.remove_key(ts, uid, ctx, h)
    sim.adopt_p2p(eng)
    sim.set_log(200000)
    host = []
    while True:
        w = sim.pop_window()
        if len(w) == 0:
            break
        for ev in w:
            if sim.begin(ev) == 0:
                host.append(int(ev["handle"]) & ~1)
    return sim, eng, host, own


def test_adopt_after_setup_equals_attach_before():
    """The engine adopted after the stock helpers scheduled the setup events dispatches exactly the run the
    oracle (and the attach-before-setup path) makes: same pop log, digest, counters, next uid."""
    sc = flows_grid()
    o = run_oracle(sc, 0, 1, 0, 0, 0, 200000)
    sim, eng, host, _own = adopt_run(sc)
    assert host == []
    st, devc, appc, (lts, luid, lctx) = eng.results(log_n=200000)
    assert sim.dispatched() == o[0].dispatched and int(st.digest) == o[0].digest
    assert sim.next_uid() == o[0].next_uid
    assert np.array_equal(devc, o[1]) and np.array_equal(appc, o[2])
    n = int(o[0].dispatched)
    for a, b, name in zip((lts, luid, lctx), o[3], ("ts", "uid", "ctx")):
        assert np.array_equal(a[:n], b[:n]), name


def test_adopt_keeps_the_programs_own_setup_event():
    """A Schedule call of the program's own among the setup calls stays a host event (its uid is consumed in
    the engine's setup list): it runs at its time, between the device events."""
    sc = flows_grid()
    sim, eng, host, own = adopt_run(sc, own_event_ts=150_000_000)
    assert host == [own[2]]
    st = eng.results(log_n=0)[0]
    assert sim.dispatched() == int(st.dispatched)  # (the engine counts the run's dispatches, host ones included)
    # the device events keep their global ranks around the host event's: one rank of the engine's log is the
    # host event's (unwritten there), every other is in (ts, uid) order
    _, _, _, glog = eng.results(log_n=sim.dispatched())
    ts = glog[0][:sim.dispatched()].astype(np.int64)
    hole = np.flatnonzero(glog[1][:sim.dispatched()] == 0)  # (uids start at 4: an unwritten rank has uid 0)
    assert len(hole) == 1
    dev = np.delete(ts, hole)
    assert (np.diff(dev) >= 0).all() and dev[hole[0] - 1] <= own[0] <= dev[hole[0]]
