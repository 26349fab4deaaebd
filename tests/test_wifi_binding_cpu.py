"""The uid-critical host half of an ns-3-side Wi-Fi binding (ns3-module/model/hip-yans-wifi-phy.cc), on CPU:

  * nsgpu_wifil_send_plan — YansWifiChannel::Send's ScheduleWithContext calls for one SendPacket
    (yans-wifi-channel.cc:77-115): which phys receive, in what order, with which uids and contexts.  Checked against
    the oracle's restated channel loop (nsref_fanout_yans, the loop its closed-loop run uses too) on grids with
    several channel numbers and phys that have no device (context 0xffffffff).
  * the EndReceive hand-back's MAC stand-in on the oracle (nsref_wifil_mac.reply_on): a reply per EndReceive that
    passes its draw, scheduled in the EndReceive's context — what tests/test_gpu_wifi_loop.py compares the device
    runtime (nsgpu_sim_wifi_set_end_handler) against."""
import numpy as np
import pytest

import nsref
import wifi
from wifi_loop_harness import run_oracle, scenario


@pytest.mark.parametrize("n_side,channels", [(4, 1), (6, 3), (10, 2)])
def test_send_plan_equals_the_channel_loop(n_side, channels):
    x, y, z = wifi.grid(n_side, 80.0)
    n = len(x)
    rng = np.random.default_rng(n_side)
    chan = rng.integers(1, channels + 1, n).astype(np.uint32)
    node = np.arange(n, dtype=np.uint32) * 3 + 7
    node[rng.random(n) < 0.1] = 0xFFFFFFFF  # (a phy without a device: dstNode 0xffffffff, :101-104)
    ph = wifi.LoopPhys(x, y, z, channel=chan, node=node)
    chain = nsref.loss_chain((nsref.LOSS_LOG_DISTANCE, 3.0, 1.0, 46.6777))
    for sender in (0, n // 2, n - 1):
        base = 1000 + 17 * sender
        phy, uid, ctx = ph.send_plan(sender, base)
        want = nsref.fanout_yans(x, y, z, chan, node, sender, 16.0, chain, 3e8, 5000, base)
        assert len(phy) == len(want) == ph.receivers(sender)
        assert np.array_equal(phy, want["phy"])
        assert np.array_equal(uid, want["uid"])
        assert np.array_equal(ctx, want["context"])
        assert np.array_equal(uid, base + np.arange(len(uid), dtype=np.uint32))


def test_send_plan_refuses_the_uid_limit():
    import nsgpu
    x, y, z = wifi.grid(3, 50.0)
    ph = wifi.LoopPhys(x, y, z)
    with pytest.raises(nsgpu.NsgpuError, match="error 5"):
        ph.send_plan(0, 0xFFFFFFFF - 3)  # (8 receivers: the last uids would pass 0xfffffffe)
    assert len(ph.send_plan(0, 0xFFFFFFFF - 8)[0]) == 8


def test_oracle_reply_mac():
    """The hand-back's MAC stand-in on the oracle: replies add sends (or busy attempts), each reply's send at an
    EndReceive's time + the delay, on that EndReceive's phy."""
    sc = scenario(stop_ns=100_000_000)
    _l0, ends0, _p0, t0 = run_oracle(sc)
    sc["reply_delay"] = 10_000
    _l1, ends1, _p1, t1 = run_oracle(sc)
    assert t1["sends"] + t1["busy"] > t0["sends"] + t0["busy"]
    ok = ends1[((ends1["flags"] & wifi.END_CANCELLED) == 0) & (ends1["per"] < 0.5)]
    keys = set(zip((ok["ts"] + 10_000).tolist(), ok["phy"].tolist()))
    reply_sends = [(int(ts), int(p)) for ts, _u, p in t1["txs"] if (int(ts), int(p)) in keys]
    assert len(reply_sends) > 10
