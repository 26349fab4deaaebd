"""The Wi-Fi receive subset partitioned by receiver (every partition holds the transmissions
and runs its own receivers; the syncs are all-gathered and the counters all-reduced after the chains):
loopback groups of 1-4 partitions on one device, and RCCL with one rank, against the CPU oracle
(oracle/nsref_wifi.cc) — the run totals, digest, every EndReceive, every fan-out's uid base, and each
partition's own receivers' counters and Receive log equal the sequential run's."""
import numpy as np
import pytest

import p2p
import wifi
from test_gpu_wifi import grid100_committed
from test_wifi_oracle import random_scenario, run_oracle, tie_scenario

pytestmark = pytest.mark.gpu


def check_partition(eng, st, phys, base, ends, log, sc):
    g = eng.stats()
    gd, od = g.as_dict(), st.as_dict()
    assert gd == od, {k: (gd[k], od[k]) for k in gd if gd[k] != od[k]}
    assert np.array_equal(eng.tx_base(), base)
    assert np.array_equal(eng.ends(), ends)
    b, e = eng.phys_range
    gp = eng.phys()
    for f in wifi.PHY_COUNTERS_DTYPE.names:
        if f == "first_power":
            np.testing.assert_allclose(gp[f][b:e], phys[f][b:e], rtol=1e-9, atol=1e-24)
        else:
            assert np.array_equal(gp[f][b:e], phys[f][b:e]), f
    if log is not None:
        gl = eng.rx_log_read().reshape(len(sc.tx), sc.n_phy)
        ol = log.reshape(len(sc.tx), sc.n_phy)
        for f in ("ts", "uid", "outcome", "flags", "cca_ns"):
            assert np.array_equal(gl[f][:, b:e], ol[f][:, b:e]), f


def run_group(sc, parts, rx_log=True, store=wifi.STORE_AUTO):
    st, phys, base, ends, log = run_oracle(sc, rx_log=rx_log)
    engs = [wifi.Engine(sc, rx_log=rx_log, store=store, phys=r) for r in wifi.partitions(sc.n_phy, parts)]
    wifi.group_run(engs)
    for eng in engs:
        check_partition(eng, st, phys, base, ends, log if rx_log else None, sc)
    for eng in engs:
        eng.close()


@pytest.mark.parametrize("parts", [1, 2, 3, 4])
@pytest.mark.parametrize("seed,channels", [(1, (1,)), (3, (1, 6)), (4, (1, 6, 11)), ("ties", None)])
def test_loopback_partitions_match_oracle(seed, channels, parts):
    sc = tie_scenario() if seed == "ties" else random_scenario(seed, channels=channels)
    run_group(sc, parts)


@pytest.mark.parametrize("store", [wifi.STORE_LDS, wifi.STORE_HBM | wifi.INLINE_RX, wifi.STORE_LDS | wifi.UNSORTED_RX])
def test_grid_100x100_four_partitions(store):
    """Config 3's grid with the committed 300-frame schedule in four row bands (3 M Receives)."""
    run_group(grid100_committed(), 4, store=store)


def test_more_partitions_than_receivers_and_start_overflow():
    """Empty partitions, and the LDS start-queue overflow repeated on the ring by the whole group."""
    from test_wifi_oracle import line, one_tx
    x, y, z = line([0.0, 50.0, 100.0])
    tx = np.concatenate([one_tx(0, 1, 4), one_tx(0, 2, 5), one_tx(9_000_000, 0, 6)])
    run_group(wifi.Scenario(x, y, z, tx, uid_start=8, stop_ts=10 ** 9, stop_uid=7), 5)
    pts = [(0, 0)] + [(sx * a, sy * b) for a, b in ((3, 4), (4, 3)) for sx in (1, -1) for sy in (1, -1)] + \
          [(5, 0), (-5, 0), (0, 5), (0, -5)]
    x = np.array([p[0] * 20.0 for p in pts])
    y = np.array([p[1] * 20.0 for p in pts])
    z = np.zeros_like(x)
    tx = np.concatenate([one_tx(1000, k, 4 + k) for k in range(1, len(pts))])
    n = len(pts) - 1
    run_group(wifi.Scenario(x, y, z, tx, uid_start=5 + n, stop_ts=10 ** 9, stop_uid=4 + n), 3, store=wifi.STORE_LDS)


def test_rccl_one_rank_matches_oracle():
    sc = random_scenario(2)
    st, phys, base, ends, log = run_oracle(sc, rx_log=True)
    comm = p2p.Comm(p2p.Comm.unique_id(), 1, 0)
    eng = wifi.Engine(sc, rx_log=True, phys=(0, sc.n_phy), comm=comm)
    eng.launch()
    check_partition(eng, st, phys, base, ends, log, sc)
    eng.close()


def test_group_member_cannot_run_alone():
    sc = random_scenario(1)
    eng = wifi.Engine(sc, phys=(0, sc.n_phy // 2))
    import nsgpu
    with pytest.raises(nsgpu.NsgpuError, match="group"):
        eng.launch()
    eng.close()
