"""Closed-loop Wi-Fi (config 3 with the MAC on the host): host closures send only when the
device reports the phy IDLE, EndReceive's (snr, per) go back to the host for its draw.  GPU = oracle on the
full (ts, uid, context) pop log, the digest, the per-phy counters and state; SNR / PER within 1e-9
relative (device libm vs glibc; the state machine does not depend on them).  SNR / PER are parity
unpinned: the reference holds no CalculateSnrPer fixture (wifi-interference-test-suite.cc only compares
PERs of its own runs)."""
import numpy as np
import pytest

import wifi
from wifi_loop_harness import draws, run_gpu, run_oracle, scenario

pytestmark = pytest.mark.gpu

PHY_FIELDS = ("rx", "sync", "drop_rx", "drop_tx", "drop_ed", "cca_switches", "end", "end_cancelled", "ni_len",
              "end_tx", "end_rx", "end_cca_busy", "rxing")


def check(sc, log_cap=1 << 20, uid_first=0):
    olog, oends, ophys, otot = run_oracle(sc, log_cap, uid_first=uid_first)
    glog, gends, gphys, gtot, _keep = run_gpu(sc, log_cap, uid_first=uid_first)
    for f in ("dispatched", "digest", "next_uid", "final_ts", "sends", "busy"):
        assert gtot[f] == otot[f], (f, gtot[f], otot[f])
    for a, b in zip(glog, olog):
        assert np.array_equal(a, b)
    for f in PHY_FIELDS:
        assert np.array_equal(gphys[f], ophys[f]), f
    # m_firstPower: sums of +P / -P (DbmToW through the device's pow: within an ulp of glibc's, as in
    # test_gpu_wifi.py) — the residual of cancelled terms, compared absolutely
    np.testing.assert_allclose(gphys["first_power"], ophys["first_power"], rtol=1e-9, atol=1e-24)
    assert len(gends) == len(oends)
    for f in ("ts", "uid", "phy", "tx", "flags"):
        assert np.array_equal(gends[f], oends[f]), f
    np.testing.assert_allclose(gends["snr"], oends["snr"], rtol=1e-9, atol=0)
    np.testing.assert_allclose(gends["per"], oends["per"], rtol=1e-9, atol=1e-15)
    n = sc["phys"].n_phy
    assert np.array_equal(draws(gends, n), draws(oends, n))
    return otot, oends


def test_grid_4x4_dsss_nist():
    tot, ends = check(scenario())
    assert tot["sends"] > 50 and tot["busy"] > 10 and len(ends) > 100
    assert (ends["per"] > 0).any() and (ends["per"] < 1).all()


def test_grid_6x6_dense_collisions_cca_busy():
    """60 m spacing, 1 Mb/s 600-B frames every 12 ms: receptions overlap, CCA-busy phys back off."""
    tot, ends = check(scenario(n_side=6, spacing=60.0, seed=3, period=12_000_000, stop_ns=150_000_000, size=600))
    assert tot["busy"] > tot["sends"] // 4


@pytest.mark.parametrize("mode", [(wifi.OFDM, 6000000, 20000000), (wifi.OFDM, 54000000, 20000000),
                                  (wifi.ERP_OFDM, 24000000, 20000000), (wifi.DSSS, 11000000, 22000000)])
def test_modes_nist(mode):
    check(scenario(seed=5, mode=mode, size=400, stop_ns=120_000_000))


def test_yans_error_model_and_short_preamble():
    check(scenario(seed=7, mode=(wifi.DSSS, 2000000, 22000000), preamble=wifi.PREAMBLE_SHORT,
                   error_model=wifi.YANS, stop_ns=120_000_000))
    check(scenario(seed=8, mode=(wifi.OFDM, 36000000, 20000000), error_model=wifi.YANS, stop_ns=120_000_000))


def test_grid_100x100_short_stop_full_pop_log():
    """The bench's closed-loop workload (10,000 phys 100 m apart, 1000-B DSSS 1 Mb/s frames, period 1 s from
    seeded phases) cut at Stop 0.02 s (317 SendPackets, 3.17 M dispatches): every SendPacket fans out to
    9,999 receivers, so epochs hold ~10^4 events (k_wl_tail's sample sort, keys in LDS); the full pop log, digest, counters and end records equal the oracle's."""
    import numpy as np
    x, y, z = wifi.grid(100, 100.0)
    phys = wifi.LoopPhys(x, y, z, tx_cap=1 << 20, rxq_cap=1024, ni_cap=1024)
    rng = np.random.default_rng(11)
    n, period = phys.n_phy, 1_000_000_000
    sc = dict(phys=phys, first=rng.integers(0, period // 2, n).astype(np.uint64),
              backoff=(100_000 + 37_000 * np.arange(n)).astype(np.uint64), period=period, stop_ns=20_000_000,
              size=1000, mode=wifi.DSSS_1M, preamble=wifi.PREAMBLE_LONG, dbm=16.0206 + 1.0)
    tot, ends = check(sc, log_cap=1 << 22)
    assert tot["sends"] > 200 and tot["dispatched"] > 2_000_000 and len(ends) > 1000


@pytest.mark.parametrize("logged", [True, False])
def test_epoch_order_paths_lds_hbm_host(logged):
    """One SendPacket at 1 us, two at 1 ms, seven at 2 ms on the 100x100 grid (host closures scheduled in
    send order): the epochs that end at the next sends hold ~10^4 events (k_wl_tail's keys in LDS), ~2x10^4
    (more than LDS_EV: keys in HBM) and, in the last epoch, ~7x10^4 receptions plus every EndReceive (more
    than ERANK_MAX: the host orders it).  Pop log, digest, end records and counters = the oracle's replay.
    Unlogged (the bench's mode): the host-order epoch with no log, the order of the other
    epochs behind the PHY on the second stream; count, digest, next uid and end records = the oracle's."""
    import nsgpu
    import nsref
    x, y, z = wifi.grid(100, 100.0)
    ph = wifi.LoopPhys(x, y, z, tx_cap=64, rxq_cap=1024, ni_cap=1024)
    n = ph.n_phy
    sends = [(1_000, 5050), (1_000_000, 0), (1_000_000, 9999)] + [(2_000_000, p) for p in range(101, 808, 101)]
    ts = np.array([t for t, _p in sends], np.uint64)
    phy = np.array([p for _t, p in sends], np.uint32)
    size = np.full(len(sends), 1000, np.uint32)
    dbm, stop, cap = 16.0206 + 1.0, 30_000_000, 1 << 18
    olog, oends, ophys, otot = nsref.wifil_replay(ph.c_struct(), ts, phy, size, wifi.DSSS_1M, wifi.PREAMBLE_LONG, dbm,
                                                  stop, n, wifi.WIFIL_END_DTYPE, wifi.PHY_COUNTERS_DTYPE, log_cap=cap)
    assert otot["dispatched"] > 100_000
    sim = nsgpu.Sim()
    lp = wifi.LoopPhy(ph)
    sim.attach_wifi(lp)
    if logged:
        sim.set_log(cap)
    for t, p in sends:
        sim.schedule(t, (lambda p=p: lambda: sim.wifi_send(p, 1000, dbm, wifi.DSSS_1M, wifi.PREAMBLE_LONG))())
    sim.stop(stop)
    sim.run()
    assert sim.dispatched() == otot["dispatched"] and sim.next_uid() == otot["next_uid"]
    assert sim.host_stats()[2] == otot["digest"]
    if logged:
        k = min(sim.dispatched(), cap)
        for a, b in zip((sim.log[0][:k], sim.log[1][:k], sim.log[2][:k]), olog):
            assert np.array_equal(a, b)
    gends, gphys = lp.read_ends(), lp.read_phys()
    for f in ("ts", "uid", "phy", "tx", "flags"):
        assert np.array_equal(gends[f], oends[f]), f
    np.testing.assert_allclose(gends["per"], oends["per"], rtol=1e-9, atol=1e-15)
    for f in PHY_FIELDS[:8]:  # (the replay's oracle returns the counters only: nsref_wifil_replay)
        assert np.array_equal(gphys[f], ophys[f]), f
    lp.close()


def test_bench_native_mac_stand_in_equals_the_oracle():
    """bench.py's wifi-loop MAC stand-in as C callbacks (scripts/macstub.cc, lib/libnsgpu_macstub.so): on the
    6x6 dense grid its run's dispatch count, digest, next uid, sends and busy attempts equal the oracle's
    (nsref_wifil_run restates the same stand-in)."""
    import os
    import sys
    import types
    import nsgpu
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from wifi_loop_harness import run_oracle
    sc = scenario(n_side=6, spacing=60.0, seed=3, period=12_000_000, stop_ns=150_000_000, size=600)
    otot = run_oracle(sc)[3]
    w = bench.WifiLoop(types.SimpleNamespace(wifi_side=6, wifi_loop_stop=0.15, wifi_mac="native"), None)
    assert w.mac == "native"
    sim = nsgpu.Sim()
    lp = wifi.LoopPhy(sc["phys"])
    sim.attach_wifi(lp)
    disp, digest, info = w.run_native(sc, sim, lp)
    assert (disp, digest, info["next_uid"]) == (otot["dispatched"], otot["digest"], otot["next_uid"])
    assert (info["sends"], info["busy_attempts"]) == (otot["sends"], otot["busy"])
    assert otot["busy"] > 0


# ---------------------------------------------------------------- the EndReceive hand-back (nsgpu_sim_wifi_set_end_handler)
@pytest.mark.parametrize("reply_delay", [10_000, 0])
@pytest.mark.parametrize("dense", [False, True])
def test_end_handback_mac_replies_equal_the_oracle(reply_delay, dense):
    """YansWifiPhy::EndReceive's host part in the order (yans-wifi-phy.cc:770-799): every phy is handed back; at each
    EndReceive that is not cancelled and whose draw passes, the MAC stand-in schedules a reply (after a SIFS-like
    10 us, or Schedule (0): same time, a later uid) which sends if the phy is IDLE.  The replies' Schedule calls take
    their uids at the EndReceive's place (the runtime stops the device there, and never advances past a time where a
    pending Receive could still sync and end), so the full pop log, digest, end records, counters and sends equal
    the oracle's restatement with the same MAC (nsref_wifil_mac.reply_on)."""
    if dense:
        sc = scenario(n_side=6, spacing=60.0, seed=3, period=12_000_000, stop_ns=80_000_000, size=600)
    else:
        sc = scenario(stop_ns=120_000_000)
    sc["reply_delay"] = reply_delay
    olog, oends, ophys, otot = run_oracle(sc)
    glog, gends, gphys, gtot, _keep = run_gpu(sc)
    for f in ("dispatched", "digest", "next_uid", "final_ts", "sends", "busy"):
        assert gtot[f] == otot[f], (f, gtot[f], otot[f])
    for a, b in zip(glog, olog):
        assert np.array_equal(a, b)
    for f in PHY_FIELDS:
        assert np.array_equal(gphys[f], ophys[f]), f
    for f in ("ts", "uid", "phy", "tx", "flags"):
        assert np.array_equal(gends[f], oends[f]), f
    np.testing.assert_allclose(gends["per"], oends["per"], rtol=1e-9, atol=1e-15)
    live = int(np.count_nonzero((oends["flags"] & wifi.END_CANCELLED) == 0))
    assert gtot["handbacks"] == live > 20
    replies = int(np.count_nonzero(((oends["flags"] & wifi.END_CANCELLED) == 0) & (oends["per"] < 0.5)))
    assert replies > 10  # (the replies are part of the sends and busy counts compared above)


def test_end_handback_listening_alone_changes_nothing():
    """Every phy handed back to a handler that schedules nothing: the epochs the hand-back cuts (at every EndReceive,
    and before every time a pending Receive could end) leave the run identical to the plain one — the oracle's."""
    sc = scenario(n_side=6, spacing=60.0, seed=3, period=12_000_000, stop_ns=60_000_000, size=600)
    olog, oends, ophys, otot = run_oracle(sc)
    sc["reply_delay"] = 1 << 62  # (replies far past Stop: never dispatched; the handler still runs and schedules)
    glog, gends, _gphys, gtot, _keep = run_gpu(sc)
    # (the handler's Schedule calls take uids: compare against the oracle run with the same far replies)
    olog2, oends2, _ophys2, otot2 = run_oracle(sc)
    for f in ("dispatched", "digest", "next_uid", "sends", "busy"):
        assert gtot[f] == otot2[f], f
    for a, b in zip(glog, olog2):
        assert np.array_equal(a, b)
    # and before the first reply-uid the runs agree with the plain one: same events, same end records
    assert np.array_equal(gends["ts"], oends["ts"]) and np.array_equal(gends["phy"], oends["phy"])
    assert otot2["dispatched"] == otot["dispatched"] and gtot["handbacks"] > 20
