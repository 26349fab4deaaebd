"""CPU checks of the Wi-Fi PHY receive subset's oracle (oracle/nsref_wifi.cc) and host logic.

* WifiPhy::CalculateTxDuration against the reference's own known values (tests/golden/reference_kat.json
  "wifi_tx_duration", from src/wifi/test/tx-duration-test.cc:114-178), for the oracle and for the
  library's host-side restatement (nsgpu_wifi_tx_duration_ns: no GPU needed).
* Hand-worked micro scenarios whose outcome follows from the reference code by reading it.
* The oracle against a second, independent restatement (tests/wifi_pyref.py) on random small scenarios.
The receive state machine has no reference-held fixture (the reference's wifi tests drive it through
the MAC and only assert PER/throughput figures): beyond the KATs, its parity is pinned by these two
restatements agreeing."""
import json
import os

import numpy as np
import pytest

import nsref
import wifi
import wifi_pyref

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "reference_kat.json")


def kat():
    return json.load(open(GOLDEN))["wifi_tx_duration"]


def test_tx_duration_kats_oracle_and_library():
    k = kat()
    pre = {"long": wifi.PREAMBLE_LONG, "short": wifi.PREAMBLE_SHORT}
    n = 0
    for v in k["vectors"]:
        mc, rate, bw = k["modes"][v["mode"]]
        if v["what"] == "payload":  # CheckPayloadDuration: CalculateTxDuration minus the PLCP preamble + header
            got = nsref.wifi_tx_duration(v["size"], mc, rate, bw, wifi.PREAMBLE_LONG) - 192_000
            assert got == v["us"] * 1000, v
            continue
        want = v["us"] * 1000
        assert nsref.wifi_tx_duration(v["size"], mc, rate, bw, pre[v["preamble"]]) == want, v
        assert wifi.tx_duration_ns(v["size"], (mc, rate, bw), pre[v["preamble"]]) == want, v
        n += 1
    assert n == 42


def run_oracle(sc, rx_log=True):
    s = sc.c_struct()
    st = wifi.WifiStats()
    phys = np.zeros(sc.n_phy, wifi.PHY_COUNTERS_DTYPE)
    base = np.zeros(len(sc.tx), np.uint32)
    log = np.zeros(len(sc.tx) * sc.n_phy, wifi.RX_LOG_DTYPE) if rx_log else None
    _, ends = nsref.wifi_run(s, st, phys, base, wifi.END_RECORD_DTYPE, log)
    return st, phys, base, ends, log


def one_tx(ts, phy, uid, size=wifi.FRAME_1000B, mode=wifi.DSSS_1M):
    t = np.zeros(1, wifi.TX_DTYPE)
    t["ts"], t["phy"], t["uid"], t["size"], t["dbm"] = ts, phy, uid, size, 17.0206
    t["modclass"], t["rate"], t["bw"], t["preamble"] = mode[0], mode[1], mode[2], wifi.PREAMBLE_LONG
    return t


def line(xs):
    xs = np.asarray(xs, np.float64)
    return xs, np.zeros_like(xs), np.zeros_like(xs)


def test_single_link_syncs():
    """Phy 1 at 100 m: -88.66 dBm + RxGain > EnergyDetectionThreshold -96 dBm -> sync (yans-wifi-phy.cc:459-472);
    the fan-out takes uid 6, the EndReceive uid 7, at send + delay + CalculateTxDuration."""
    x, y, z = line([0.0, 100.0])
    sc = wifi.Scenario(x, y, z, one_tx(1000, 0, 4), uid_start=6, stop_ts=10 ** 9, stop_uid=5)
    st, phys, base, ends, log = run_oracle(sc)
    dur = wifi.tx_duration_ns(wifi.FRAME_1000B)
    assert dur == 8_704_000
    assert list(base) == [6]
    r = log[1]
    assert (r["ts"], r["uid"], r["outcome"], r["flags"]) == (1000 + 333, 6, wifi.SYNC, 0)
    assert len(ends) == 1 and ends[0]["uid"] == 7 and ends[0]["ts"] == 1333 + dur
    assert ends[0]["flags"] == wifi.END_DISPATCHED
    assert st.dispatched == 4 and st.next_uid == 8 and st.final_ts == 10 ** 9
    assert phys[1]["rxing"] == 0 and phys[1]["ni_len"] == 2 and phys[0]["end_tx"] == 1000 + dur


def test_second_signal_drops_and_extends_cca():
    """C (x=0) syncs to A (50 m), then B (100 m) arrives: drop (already in RX, :431-440); its end lies after
    A's, so maybeCcaBusy: the sum stays above CcaMode1Threshold until B ends -> CCA busy for B's duration."""
    x, y, z = line([0.0, 50.0, 100.0])
    tx = np.concatenate([one_tx(0, 1, 4), one_tx(0, 2, 5)])
    sc = wifi.Scenario(x, y, z, tx, uid_start=7, stop_ts=10 ** 9, stop_uid=6)
    st, phys, base, ends, log = run_oracle(sc)
    dur = wifi.tx_duration_ns(wifi.FRAME_1000B)
    a = log[0 * 3 + 0]
    b = log[1 * 3 + 0]
    assert a["outcome"] == wifi.SYNC
    assert b["outcome"] == wifi.DROP_RX and b["flags"] == wifi.F_CCA_EVAL | wifi.F_CCA_SWITCH
    assert b["cca_ns"] == dur
    # phy 1 (transmitting A) hears B while in TX: drop; phy 2 hears A while in TX
    assert log[1 * 3 + 1]["outcome"] == wifi.DROP_TX and log[0 * 3 + 2]["outcome"] == wifi.DROP_TX


def test_transmit_while_receiving_cancels_end_receive():
    """SendPacket while in RX cancels m_endRxEvent (yans-wifi-phy.cc:510-514): the EndReceive is still
    dispatched (counted) but does nothing; the phy is in TX."""
    x, y, z = line([0.0, 100.0])
    tx = np.concatenate([one_tx(0, 0, 4), one_tx(1_000_000, 1, 5)])
    sc = wifi.Scenario(x, y, z, tx, uid_start=7, stop_ts=10 ** 9, stop_uid=6)
    st, phys, base, ends, log = run_oracle(sc)
    assert log[1]["outcome"] == wifi.SYNC
    e = [r for r in ends if r["phy"] == 1][0]
    assert e["flags"] == wifi.END_CANCELLED | wifi.END_DISPATCHED
    assert st.end_cancelled == 1
    assert log[1 * 2 + 0]["outcome"] == wifi.DROP_TX  # phy 0 is still sending its own frame


def test_far_receiver_is_below_energy_detection():
    x, y, z = line([0.0, 1000.0])
    sc = wifi.Scenario(x, y, z, one_tx(0, 0, 4), uid_start=6, stop_ts=10 ** 9, stop_uid=5)
    st, phys, base, ends, log = run_oracle(sc)
    assert log[1]["outcome"] == wifi.DROP_ED and log[1]["flags"] == wifi.F_CCA_EVAL
    assert log[1]["cca_ns"] == 0 and len(ends) == 0


def random_scenario(seed, n=14, n_tx=60, span_ns=40_000_000, channels=(1,)):
    """Random phys and transmissions; no phy starts a frame while its previous one is still on the air
    (SendPacket in TX is the reference's NS_FATAL_ERROR)."""
    rng = np.random.default_rng(seed)
    x = rng.random(n) * 600.0
    y = rng.random(n) * 200.0
    z = rng.random(n) * 2.0
    chan = np.asarray(channels, np.uint32)[rng.integers(0, len(channels), n)]
    modes = [wifi.DSSS_1M, (wifi.DSSS, 11000000, 22000000), (wifi.OFDM, 6000000, 20000000)]
    rows, on_air = [], {}
    while len(rows) < n_tx:
        s, t = int(rng.integers(0, n)), int(rng.integers(0, span_ns))
        size = int(rng.choice([60, 300, wifi.FRAME_1000B]))
        m = modes[int(rng.integers(0, len(modes)))]
        d = wifi.tx_duration_ns(size, m)
        if any(t <= e and t + d >= b for b, e in on_air.get(s, [])):
            continue
        on_air.setdefault(s, []).append((t, t + d))
        rows.append((t, s, size, m))
    tx = np.zeros(len(rows), wifi.TX_DTYPE)
    for i, (t, s, size, m) in enumerate(sorted(rows, key=lambda r: (r[0], r[1]))):
        tx[i] = (t, 4 + i, s, size, 17.0206, m[0], m[1], m[2], wifi.PREAMBLE_LONG)
    return wifi.Scenario(x, y, z, tx, channel=chan, uid_start=5 + len(rows), stop_ts=span_ns + 3_000_000,
                         stop_uid=4 + len(rows), ni_cap=64)


def tie_scenario():
    """5x5 grid, 100 m: pairs of symmetric senders transmit at the same instant (equal-ts arrivals at the
    phys between them: Receive vs Receive ties), and later frames start exactly one frame duration after
    earlier ones (a Receive at the same ts as an EndReceive of the same phy)."""
    x, y, z = wifi.grid(5, 100.0)
    d = wifi.tx_duration_ns(1000)
    rows = [(0, 0), (0, 4), (d, 20), (d, 24), (2 * d, 2), (2 * d, 22), (3 * d, 10), (3 * d, 14), (3 * d + 1, 12),
            (4 * d, 0), (4 * d, 24), (5 * d, 4), (5 * d, 20)]
    tx = np.zeros(len(rows), wifi.TX_DTYPE)
    for i, (t, s_) in enumerate(sorted(rows)):
        tx[i] = (t, 4 + i, s_, 1000, 17.0206, wifi.DSSS, 1000000, 22000000, wifi.PREAMBLE_LONG)
    return wifi.Scenario(x, y, z, tx, uid_start=5 + len(rows), stop_ts=7 * d, stop_uid=4 + len(rows), ni_cap=64)


@pytest.mark.parametrize("seed,channels", [(1, (1,)), (2, (1,)), (3, (1, 6)), (4, (1, 6, 11)), (5, (1,)), ("ties", None)])
def test_oracle_matches_independent_restatement(seed, channels):
    sc = tie_scenario() if seed == "ties" else random_scenario(seed, channels=channels)
    st, phys, base, ends, log = run_oracle(sc)
    durs = [wifi.tx_duration_ns(int(t["size"]), (int(t["modclass"]), int(t["rate"]), int(t["bw"]))) for t in sc.tx]
    pst, plog, pends, pbase, pphy = wifi_pyref.run(sc, durs)
    for f in ("dispatched", "tx", "rx", "sync", "drop_rx", "drop_tx", "drop_ed", "cca_evals", "cca_switches",
              "end", "end_cancelled", "final_ts", "next_uid"):
        assert getattr(st, f) == pst[f], f
    assert list(base) == pbase
    assert len(ends) == len(pends)
    pe = sorted(pends, key=lambda e: e["uid"])
    for a, b in zip(ends, pe):
        assert (a["ts"], a["sync_ts"], a["uid"], a["phy"], a["tx"], a["flags"]) == \
            (b["ts"], b["sync_ts"], b["uid"], b["phy"], b["tx"], b["flags"])
    n = sc.n_phy
    for (k, j), (ts, uid, outcome, flags, cca) in plog.items():
        r = log[k * n + j]
        assert (r["ts"], r["uid"], r["outcome"], r["flags"] & 3, r["cca_ns"]) == (ts, uid, outcome, flags, cca), (k, j)
    assert int((log["outcome"] != wifi.NOT_RUN).sum()) == st.rx
    for j in range(n):
        for f in ("rx", "sync", "drop_rx", "drop_tx", "drop_ed", "cca_switches", "end", "end_cancelled", "ni_max"):
            assert phys[j][f] == pphy[j][f], (j, f)
        assert phys[j]["ni_len"] == len(pphy[j]["ni_t"])
        assert phys[j]["first_power"] == pphy[j]["first"]
    assert st.sync > 0 and st.drop_rx > 0 and st.cca_switches > 0


def test_schedule_validation_and_uid_overflow_guard():
    """The library rejects schedules the reference could not have produced (out of (ts, uid) order, a
    transmission uid that is not a setup uid) before touching the GPU."""
    import nsgpu
    x, y, z = line([0.0, 100.0])
    tx = np.concatenate([one_tx(10, 0, 5), one_tx(5, 1, 4)])
    sc = wifi.Scenario(x, y, z, tx, uid_start=7)
    with pytest.raises(nsgpu.NsgpuError, match="order"):
        wifi.Engine(sc)
    sc = wifi.Scenario(x, y, z, one_tx(0, 0, 9), uid_start=7)
    with pytest.raises(nsgpu.NsgpuError, match="setup uid"):
        wifi.Engine(sc)
