"""The closed-loop Wi-Fi PHY split over GPUs by receiver (nsgpu_wifil_create_dist / _group,
DESIGN.md §5): every rank runs the same host program, each runs its own phys' Receives / InterferenceHelper /
state machine / EndReceive walks, and per epoch the syncs, counters, end records, state fields and dispatched
events are exchanged.  The handle must answer as the single engine does: full (ts, uid, context) pop log,
digest, next uid, per-phy counters and end records equal the oracle's (nsref_wifil_run: the single-process
restatement of yans-wifi-channel.cc:77-115 -> yans-wifi-phy.cc:399-522,770-799), through loopback groups of 1-4
partitions (empty ones included) on one device and through RCCL with one rank."""
import numpy as np
import pytest

import wifi
from wifi_loop_harness import draws, run_gpu, run_oracle, scenario

pytestmark = pytest.mark.gpu

PHY_FIELDS = ("rx", "sync", "drop_rx", "drop_tx", "drop_ed", "cca_switches", "end", "end_cancelled", "ni_len",
              "end_tx", "end_rx", "end_cca_busy", "rxing")


def check(sc, log_cap=1 << 20, oracle=None, **kw):
    olog, oends, ophys, otot = oracle if oracle is not None else run_oracle(sc, log_cap)
    glog, gends, gphys, gtot, _keep = run_gpu(sc, log_cap, **kw)
    for f in ("dispatched", "digest", "next_uid", "final_ts", "sends", "busy"):
        assert gtot[f] == otot[f], (f, gtot[f], otot[f])
    for a, b in zip(glog, olog):
        assert np.array_equal(a, b)
    for f in PHY_FIELDS:
        assert np.array_equal(gphys[f], ophys[f]), f
    np.testing.assert_allclose(gphys["first_power"], ophys["first_power"], rtol=1e-9, atol=1e-24)
    assert len(gends) == len(oends)
    for f in ("ts", "uid", "phy", "tx", "flags"):
        assert np.array_equal(gends[f], oends[f]), f
    np.testing.assert_allclose(gends["snr"], oends["snr"], rtol=1e-9, atol=0)
    np.testing.assert_allclose(gends["per"], oends["per"], rtol=1e-9, atol=1e-15)
    n = sc["phys"].n_phy
    assert np.array_equal(draws(gends, n), draws(oends, n))
    if "reply_delay" in sc:
        live = int(np.count_nonzero((oends["flags"] & wifi.END_CANCELLED) == 0))
        assert gtot["handbacks"] == live
    return otot, oends


@pytest.mark.parametrize("bounds", [[0, 16], [0, 8, 16], [0, 5, 5, 16], [0, 3, 7, 12, 16], [0, 0, 16, 16]])
def test_group_4x4_equals_the_oracle(bounds):
    """Partitions of the 4x4 grid (one, two, an empty middle one, four, empty first and last ones)."""
    sc = scenario()
    tot, ends = check(sc, bounds=bounds)
    assert tot["sends"] > 50 and len(ends) > 100


def test_group_6x6_dense_collisions_three_partitions():
    sc = scenario(n_side=6, spacing=60.0, seed=3, period=12_000_000, stop_ns=150_000_000, size=600)
    tot, _ends = check(sc, bounds=[0, 11, 23, 36])
    assert tot["busy"] > tot["sends"] // 4


@pytest.mark.parametrize("reply_delay", [10_000, 0])
def test_group_end_handback_replies(reply_delay):
    """The EndReceive hand-back across partitions: each scans its own listened phys, the next EndReceive is the
    smallest over all of them (replying MAC stand-in, as test_gpu_wifi_loop.py)."""
    sc = scenario(n_side=6, spacing=60.0, seed=3, period=12_000_000, stop_ns=80_000_000, size=600)
    sc["reply_delay"] = reply_delay
    check(sc, bounds=[0, 7, 7, 20, 36])


def test_group_modes_yans_short_preamble():
    check(scenario(seed=7, mode=(wifi.DSSS, 2000000, 22000000), preamble=wifi.PREAMBLE_SHORT,
                   error_model=wifi.YANS, stop_ns=120_000_000), bounds=[0, 6, 16])
    check(scenario(seed=5, mode=(wifi.OFDM, 54000000, 20000000), size=400, stop_ns=120_000_000), bounds=[0, 9, 16])


def _grid100(stop_ns=20_000_000):
    x, y, z = wifi.grid(100, 100.0)
    phys = wifi.LoopPhys(x, y, z, tx_cap=1 << 20, rxq_cap=1024, ni_cap=1024)
    rng = np.random.default_rng(11)
    n, period = phys.n_phy, 1_000_000_000
    return dict(phys=phys, first=rng.integers(0, period // 2, n).astype(np.uint64),
                backoff=(100_000 + 37_000 * np.arange(n)).astype(np.uint64), period=period, stop_ns=stop_ns,
                size=1000, mode=wifi.DSSS_1M, preamble=wifi.PREAMBLE_LONG, dbm=16.0206 + 1.0)


def test_grid_100x100_four_bands_and_one_rccl_rank():
    """The bench's closed loop (10,000 phys, every SendPacket fanned out to 9,999 receivers) cut at Stop 0.02 s:
    in four row bands of a loopback group, and as the one rank of an RCCL split — full pop log, digest, counters
    and end records equal the oracle's."""
    import p2p
    sc = _grid100()
    oracle = run_oracle(sc, 1 << 22)
    tot, ends = check(sc, 1 << 22, oracle=oracle, bounds=[0, 2500, 5000, 7500, 10000])
    assert tot["sends"] > 200 and tot["dispatched"] > 2_000_000 and len(ends) > 1000
    comm = p2p.Comm(p2p.Comm.unique_id(), 1, 0)
    check(sc, 1 << 22, oracle=oracle, part=(0, 10000), comm=comm)


def test_partitions_must_tile_the_phys():
    import nsgpu
    sc = scenario()
    for bad in ([0, 8], [1, 16], [0, 9, 8, 16], [0, 17]):
        with pytest.raises(nsgpu.NsgpuError):
            wifi.LoopPhy(sc["phys"], bounds=bad)
