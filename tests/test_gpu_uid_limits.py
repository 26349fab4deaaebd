"""uid-space limits: DefaultSimulatorImpl's m_uid is a uint32 from 4 (default-simulator-impl.cc:52-56,
188-219) that wraps to 0 after 0xffffffff.  Each engine starts its counter just below a limit, against the oracle
started at the same uid (nsgpu_p2p_scenario.uid_first, nsgpu_sim_set_next_uid, nsref_wifil_mac.uid_first):

  * the deferred p2p pipeline's provisional-uid range (UID_DF_SOFT, nsgpu_p2p.hip): the run hands over to the
    scanning pipeline there and stays bit-exact past UID_DF_LIMIT;
  * the traced engine's old 2^31 limit (local records' trace uids are now flagged, not bit-31 tagged);
  * 2^32: a run whose last uid is 0xfffffffe is bit-exact; one more uid and the reference would hand out
    0xffffffff and then wrap to 0 — every engine fails with NSGPU_ERANGE instead (before such an event runs),
    while the oracle (a uint32 like the reference's) wraps."""
import numpy as np
import pytest

import nsgpu
import nsref
import p2p
import trace

pytestmark = pytest.mark.gpu

UID_DF_SOFT = 0x3FE00000 - (1 << 22)  # nsgpu_p2p.hip
U32 = 0xFFFFFFFF


def oracle_p2p(sc, log_cap=0):
    s = sc.c_struct()
    st = p2p.P2PStats()
    devc = np.zeros(s.n_devices, p2p.DEV_COUNTERS_DTYPE)
    appc = np.zeros(s.n_apps, p2p.APP_COUNTERS_DTYPE)
    _, log = nsref.p2p_run(s, st, devc, appc, log_cap)
    return st, devc, appc, log


def assert_same(o, g, log=True):
    from test_gpu_p2p import assert_same as same
    same(o, g, log)


def test_deferred_pipeline_hands_over_below_its_provisional_range_full_log():
    """16x16 grid (119,875 uids) started 40,000 uids below UID_DF_SOFT: full pop log = the oracle's."""
    sc = p2p.grid(16, 16)
    sc.uid_first = UID_DF_SOFT - 40_000
    o = oracle_p2p(sc, log_cap=130_000)
    eng = p2p.Engine(sc, log_cap=130_000)
    assert eng.wide()
    g = eng.run(log_n=130_000)
    assert o[0].next_uid > UID_DF_SOFT + 50_000
    assert_same(o, g)


def test_config4_past_the_deferred_limit():
    """The bench workload (128x128, 7.6 M uids) started 1 M uids below UID_DF_SOFT: it runs past UID_DF_LIMIT
    (0x3fe00000) on the scanning pipeline; every counter, the digest and next uid = the oracle's."""
    sc = p2p.grid(128, 128)
    sc.uid_first = UID_DF_SOFT - 1_000_000
    o = oracle_p2p(sc)
    assert o[0].next_uid > 0x3FE00000 + 1_000_000
    eng = p2p.Engine(sc)
    assert_same(o, eng.run(), log=False)


def uids_used(sc):
    st = oracle_p2p(sc)[0]
    return st.next_uid - 4


def test_p2p_last_uid_0xfffffffe_is_exact_and_one_more_fails():
    sc = p2p.grid(8, 8)
    n = uids_used(sc)
    sc.uid_first = U32 - n  # the run's last uid is 0xfffffffe, its counter ends at 0xffffffff
    o = oracle_p2p(sc, log_cap=40_000)
    assert o[0].next_uid == U32
    eng = p2p.Engine(sc, log_cap=40_000)
    assert_same(o, eng.run(log_n=40_000))
    sc.uid_first = U32 - n + 1  # the reference would hand out 0xffffffff, then wrap to 0
    assert oracle_p2p(sc)[0].next_uid == 0
    with pytest.raises(nsgpu.NsgpuError, match="error 5"):
        p2p.Engine(sc).run()


def test_partitioned_engine_uid_limit():
    sc = p2p.grid(6, 6)
    n = uids_used(sc)
    sc.uid_first = U32 - n
    o = oracle_p2p(sc)
    grp = p2p.LoopbackGroup(sc, 2)
    st = grp.run()[0]
    assert (st.dispatched, st.digest, st.next_uid) == (o[0].dispatched, o[0].digest, o[0].next_uid)
    sc.uid_first = U32 - n + 1
    with pytest.raises(nsgpu.NsgpuError, match="error 5"):
        p2p.LoopbackGroup(sc, 2).run()


def test_traced_engine_past_2_31():
    """A traced congested grid whose uids cross 2^31 (the old limit of the local records' trace uids)."""
    from test_gpu_trace import assert_same_trace, oracle_trace
    g = p2p.grid(4, 4, qmax=3, rate_bps=4_000_000, stop_ns=300_000_000, sim_stop_ns=400_000_000,
                 flows=[(0, 15), (1, 15), (4, 15), (5, 15)])
    g.uid_first = (1 << 31) - 3_000
    _ost, odevc, otr = oracle_trace(g)
    assert int(otr["uid"].max()) > (1 << 31)
    eng = p2p.Engine(g)
    eng.set_trace(len(otr) + 16)
    _st, gdevc, _appc, _log = eng.run()
    assert np.array_equal(gdevc, odevc)
    assert_same_trace(g, otr, trace.sort_records(eng.trace()))


# ---------------------------------------------------------------- the host-closure runtime (nsgpu_sim)
def test_sim_runtime_uid_limit():
    """Schedule calls near 2^32 on the runtime and on the restated DefaultSimulatorImpl: the same uids and
    dispatch order up to 0xfffffffe; the call that would take 0xffffffff fails (the oracle hands it out, then
    wraps to 0), and so does every Run after it (the closure's NS_FATAL_ERROR in ns-3)."""
    g, o = nsgpu.Sim(), nsref.Sim()
    g.set_next_uid(U32 - 3)
    o.set_next_uid(U32 - 3)
    order = {"g": [], "o": []}
    for k in range(3):
        ig = g.schedule(10 * (3 - k), lambda k=k: order["g"].append(k))
        io = o.schedule(10 * (3 - k), lambda k=k: order["o"].append(k))
        assert ig.uid == io.uid == U32 - 3 + k
    g.run()
    o.run()
    assert order["g"] == order["o"] == [2, 1, 0]
    assert g.next_uid() == o.next_uid() == U32
    with pytest.raises(nsgpu.NsgpuError, match="error 5"):
        g.schedule(5, lambda: None)
    with pytest.raises(nsgpu.NsgpuError, match="error 5"):
        g.schedule_destroy(lambda: None)
    with pytest.raises(nsgpu.NsgpuError, match="error 5"):
        g.run()
    o.schedule(5, lambda: None)
    assert o.next_uid() == 0  # (the reference's wrap)


# ---------------------------------------------------------------- the closed-loop Wi-Fi PHY (nsgpu_wifil)
def test_wifi_loop_uid_limit():
    """The 4x4 closed loop started so that its last uid is 0xfffffffe: bit-exact; one uid later the run fails
    with NSGPU_ERANGE (a SendPacket's receivers, an epoch's EndReceives or a host Schedule would take
    0xffffffff) while the oracle wraps."""
    from test_gpu_wifi_loop import check
    from wifi_loop_harness import run_gpu, run_oracle, scenario
    sc = scenario(stop_ns=60_000_000)
    n = run_oracle(sc)[3]["next_uid"] - 4
    first = U32 - n
    otot, _ends = check(sc, uid_first=first)
    assert otot["next_uid"] == U32
    assert run_oracle(sc, uid_first=first + 1)[3]["next_uid"] == 0
    with pytest.raises(nsgpu.NsgpuError, match="error 5"):
        run_gpu(sc, uid_first=first + 1)


# ---------------------------------------------------------------- a host closure's send on the attached p2p engine
def _probe_run(sc, t0, period, count, app_send):
    """Host closures every `period` from t0 sending one datagram of `app_send` (nsgpu_sim_p2p_send); returns each
    call's (uid counter before, after or the error) and how the run ended."""
    eng = p2p.Engine(sc)
    eng.reset()
    sim = nsgpu.Sim()
    sim.attach_p2p(eng)
    calls = []

    def probe():
        before = sim.next_uid()
        try:
            sim.p2p_send(app_send)
            calls.append((before, sim.next_uid()))
        except nsgpu.NsgpuError as e:
            calls.append((before, str(e)))
            return
        if len(calls) < count:
            sim.schedule(period, probe)

    sim.schedule(t0, probe)
    try:
        sim.run()
        ended = "ok"
    except nsgpu.NsgpuError as e:
        ended = str(e)
    return calls, ended


def test_p2p_inject_send_refused_at_the_uid_limit_before_any_child():
    """nsgpu_sim_p2p_send with fewer uids left than the send's Schedule calls need.  The send is
    refused on the device before any child is written (no wrapped uid enters the pool), the error is sticky
    (the engine's advance and the runtime's Run both fail with NSGPU_ERANGE), and a send with exactly enough
    room still succeeds (its last uid is 0xfffffffe)."""
    from test_gpu_mixed import flows_grid
    sc = flows_grid()
    app_send = [i for i, a in enumerate(sc.apps) if a["kind"] == p2p.APP_ONOFF][1]
    calls, ended = _probe_run(sc, 150_000_000, 7_300_001, 4, app_send)
    assert ended == "ok" and len(calls) == 4
    before, after = calls[2]
    need = after - before
    assert need >= 1
    base = sc.uid_first or 4  # (0: DefaultSimulatorImpl's start, 4)
    # exactly enough room at the third send: its children end at 0xfffffffe, the counter at 0xffffffff
    sc.uid_first = base + (U32 - need - before)
    calls, ended = _probe_run(sc, 150_000_000, 7_300_001, 3, app_send)
    assert all(isinstance(c[1], int) for c in calls[:2])  # (the run itself then ends at the limit)
    assert calls[2] == (U32 - need, U32)
    # one uid less: the third send is refused, and the run ends with the uid error
    sc.uid_first = base + (U32 - need - before) + 1
    calls, ended = _probe_run(sc, 150_000_000, 7_300_001, 3, app_send)
    assert calls[2][0] == U32 - need + 1 and "error 5" in calls[2][1]
    assert "error 5" in ended
