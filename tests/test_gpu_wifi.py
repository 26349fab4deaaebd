"""Wi-Fi PHY receive subset on the GPU (nsgpu_wifi_*) against the CPU oracle (oracle/nsref_wifi.cc).

Equal: every Receive's key (ts, uid), outcome (sync / drop in RX / drop in TX / below ED), CCA evaluation
and CCA-busy duration, every EndReceive's key and cancel flag, every fan-out's uid base, per-phy
counters and final state times, NiChange counts, and the run totals (dispatch count, digest, next uid).
Received power is computed with ROCm's pow/log10 (about 1 ulp from glibc: within 1e-9 relative,
north_star): m_firstPower is compared within that tolerance, and decisions within 1e-9 of a threshold
are flagged (near_threshold) — the tests require that none of them differ."""
import os

import numpy as np
import pytest

import nsgpu
import nsref
import wifi
from test_wifi_oracle import random_scenario, run_oracle, tie_scenario

pytestmark = pytest.mark.gpu

GOLDEN_SCHEDULE = os.path.join(os.path.dirname(__file__), "golden", "wifi_grid100_schedule.csv")


def grid100_committed():
    """10,000 phys on the 100 x 100 grid (100 m, YansWifiChannelHelper::Default's LogDistance) and the
    committed 300-frame schedule (scripts/make_wifi_schedule.py)."""
    rows = np.loadtxt(GOLDEN_SCHEDULE, delimiter=",", skiprows=1, dtype=np.int64)
    x, y, z = wifi.grid(100, 100.0)
    tx = np.zeros(len(rows), wifi.TX_DTYPE)
    tx["ts"], tx["phy"], tx["uid"] = rows[:, 0], rows[:, 1], 4 + np.arange(len(rows))
    tx["size"], tx["dbm"] = wifi.FRAME_1000B, 16.0206 + 1.0
    tx["modclass"], tx["rate"], tx["bw"], tx["preamble"] = wifi.DSSS, 1000000, 22000000, wifi.PREAMBLE_LONG
    n = len(rows)
    return wifi.Scenario(x, y, z, tx, uid_start=5 + n, stop_ts=80_000_000, stop_uid=4 + n, ni_cap=512)


def compare(sc, rx_log=True, store=wifi.STORE_AUTO):
    st, phys, base, ends, log = run_oracle(sc, rx_log=rx_log)
    eng = wifi.Engine(sc, rx_log=rx_log, store=store)
    g = eng.run()
    gd, od = g.as_dict(), st.as_dict()
    assert g.near_threshold == 0 and st.near_threshold == 0
    assert gd == od, {k: (gd[k], od[k]) for k in gd if gd[k] != od[k]}
    assert np.array_equal(eng.tx_base(), base)
    ge = eng.ends()
    assert len(ge) == len(ends)
    assert np.array_equal(ge, ends)
    gp = eng.phys()
    for f in wifi.PHY_COUNTERS_DTYPE.names:
        if f == "first_power":
            np.testing.assert_allclose(gp[f], phys[f], rtol=1e-9, atol=1e-24)
        else:
            assert np.array_equal(gp[f], phys[f]), f
    if rx_log:
        gl = eng.rx_log_read()
        for f in ("ts", "uid", "outcome", "flags", "cca_ns"):
            assert np.array_equal(gl[f], log[f]), (f, np.nonzero(gl[f] != log[f])[0][:10])
    eng.close()
    return st


def test_micro_scenarios():
    from test_wifi_oracle import line, one_tx
    x, y, z = line([0.0, 50.0, 100.0])
    tx = np.concatenate([one_tx(0, 1, 4), one_tx(0, 2, 5), one_tx(9_000_000, 0, 6)])
    compare(wifi.Scenario(x, y, z, tx, uid_start=8, stop_ts=10 ** 9, stop_uid=7))
    x, y, z = line([0.0, 100.0])
    tx = np.concatenate([one_tx(0, 0, 4), one_tx(1_000_000, 1, 5)])
    st = compare(wifi.Scenario(x, y, z, tx, uid_start=7, stop_ts=10 ** 9, stop_uid=6))
    assert st.end_cancelled == 1


STORES = [pytest.param(wifi.STORE_LDS, id="lds"), pytest.param(wifi.STORE_HBM, id="hbm"),
          pytest.param(wifi.STORE_LDS | wifi.INLINE_RX, id="lds-inline"),
          pytest.param(wifi.STORE_HBM | wifi.INLINE_RX, id="hbm-inline"),
          pytest.param(wifi.STORE_LDS | wifi.UNSORTED_RX, id="lds-unsorted"),
          pytest.param(wifi.STORE_HBM | wifi.UNSORTED_RX, id="hbm-unsorted")]


@pytest.mark.parametrize("store", STORES)
@pytest.mark.parametrize("seed,channels", [(1, (1,)), (2, (1,)), (3, (1, 6)), (4, (1, 6, 11)), (5, (1,)), ("ties", None)])
def test_small_scenarios_match_oracle(seed, channels, store):
    sc = tie_scenario() if seed == "ties" else random_scenario(seed, channels=channels)
    compare(sc, store=store)


def test_auto_store_is_lds_on_the_bench_grid():
    """The bench grid's end queues fit LDS (most transmissions on the air at once ~ 10 / ms x 8.5 ms)."""
    eng = wifi.Engine(wifi.wifi_grid(n_side=100, stop_s=0.15))
    store, per_block, ecap = eng.store()
    eng.close()
    assert store == wifi.STORE_LDS and 1 <= per_block <= 64 and ecap < 512, (store, per_block, ecap)
    eng = wifi.Engine(wifi.wifi_grid(n_side=100, stop_s=0.15), store=wifi.STORE_HBM | wifi.INLINE_RX)
    assert eng.store()[0] == wifi.STORE_HBM | wifi.INLINE_RX
    eng.close()
    eng = wifi.Engine(wifi.wifi_grid(n_side=100, stop_s=0.15), store=wifi.STORE_LDS | wifi.UNSORTED_RX)
    assert eng.store()[0] == wifi.STORE_LDS | wifi.UNSORTED_RX  # (the default store reads sorted rows)
    eng.close()


def test_start_queue_overflow_repeats_on_the_ring():
    """12 senders on a circle around phy 0 (integer (3, 4, 5) offsets: equal distances in floating point)
    transmitting at once: their 12 arrivals at phy 0 share one nanosecond, so its start queue holds
    more than SCAP_LDS (8) entries at one instant while it receives — the LDS run reports it and the
    readers repeat the run on the HBM ring; results equal the oracle's either way."""
    pts = [(0, 0)] + [(sx * a, sy * b) for a, b in ((3, 4), (4, 3)) for sx in (1, -1) for sy in (1, -1)] + \
          [(5, 0), (-5, 0), (0, 5), (0, -5)]
    x = np.array([p[0] * 20.0 for p in pts])
    y = np.array([p[1] * 20.0 for p in pts])
    z = np.zeros_like(x)
    from test_wifi_oracle import one_tx
    tx = np.concatenate([one_tx(1000, k, 4 + k) for k in range(1, len(pts))])
    n = len(pts) - 1
    sc = wifi.Scenario(x, y, z, tx, uid_start=5 + n, stop_ts=10 ** 9, stop_uid=4 + n)
    compare(sc, store=wifi.STORE_LDS)


def test_no_stop_event_and_empty_schedule():
    sc = random_scenario(7)
    sc.stop_ts = wifi.NO_STOP
    compare(sc)
    x, y, z = wifi.grid(3)
    compare(wifi.Scenario(x, y, z, np.zeros(0, wifi.TX_DTYPE), uid_start=4))


@pytest.mark.parametrize("store", STORES)
def test_grid_100x100_committed_schedule(store):
    """Config 3's grid (10,000 phys, LogDistance default) with the committed 300-frame schedule: 3 M
    Receive events, every one compared."""
    st = compare(grid100_committed(), store=store)
    assert st.rx == 300 * 9999
    assert st.sync > 1000 and st.drop_rx > 10000 and st.drop_tx > 1000 and st.cca_switches > 10000
    assert st.end_cancelled > 0


def test_wifi_grid_bench_config_prefix():
    """The bench workload (wifi.wifi_grid: every phy broadcasting once a second) cut at 0.15 s simulated:
    ~15 M events, totals / per-phy state / EndReceive records compared (no per-Receive log)."""
    sc = wifi.wifi_grid(n_side=100, stop_s=0.15)
    st = compare(sc, rx_log=False)
    assert st.dispatched > 10_000_000


@pytest.mark.parametrize("store", STORES)
def test_capacity_overflow_fails_loudly(store):
    sc = grid100_committed()
    sc.ni_cap = 8
    eng = wifi.Engine(sc, store=store)
    eng.launch()
    with pytest.raises(nsgpu.NsgpuError, match="ni_cap"):
        eng.stats()
    eng.close()


def test_send_while_transmitting_is_fatal_like_the_reference():
    from test_wifi_oracle import line, one_tx
    x, y, z = line([0.0, 100.0])
    tx = np.concatenate([one_tx(0, 0, 4), one_tx(1000, 0, 5)])
    sc = wifi.Scenario(x, y, z, tx, uid_start=7, stop_ts=10 ** 9, stop_uid=6)
    with pytest.raises(RuntimeError):
        run_oracle(sc)
    eng = wifi.Engine(sc)
    eng.launch()
    with pytest.raises(nsgpu.NsgpuError, match="TX"):
        eng.stats()
    eng.close()
