"""Broadcast fan-out on the GPU vs the oracle (YansWifiChannel::Send, SingleModelSpectrumChannel::StartTx).

uids, contexts, phy indices and int64 timestamps must be bit-exact; received power within
1e-9 relative (north star tolerance; libm log10 vs device log10 may differ by an ulp).
Spectrum receivers whose loss lies within 1e-9 relative of MaxLossDb are reported separately.
"""
import numpy as np
import pytest

import nsref

pytestmark = pytest.mark.gpu
RTOL = 1e-9


def grid(n_side, spacing, channels=1, seed=0):
    rng = np.random.default_rng(seed)
    ii, jj = np.meshgrid(np.arange(n_side), np.arange(n_side), indexing="ij")
    x = (ii.ravel() * spacing).astype(np.float64)
    y = (jj.ravel() * spacing).astype(np.float64)
    z = rng.random(x.size) * 1.5
    chan = (rng.integers(0, channels, x.size) + 1).astype(np.uint32)
    node = np.arange(x.size, dtype=np.uint32)
    return x, y, z, chan, node


def compare(got, want, what):
    assert len(got) == len(want), (what, len(got), len(want))
    for f in ("ts", "uid", "context", "phy"):
        assert np.array_equal(got[f], want[f]), (what, f)
    rel = np.abs(got["rx_dbm"] - want["rx_dbm"]) / np.maximum(np.abs(want["rx_dbm"]), 1e-300)
    assert rel.max(initial=0) <= RTOL, (what, rel.max())


@pytest.mark.parametrize("ranked", [True, False])
@pytest.mark.parametrize("loss_kind", ["logdistance", "friis", "chain"])
def test_yans_fanout(loss_kind, ranked):
    """ranked: records placed through the phy list's channel-rank table (one pass); otherwise the
    counting pass + block prefix (a caller that passes no table)."""
    import nsgpu
    x, y, z, chan, node = grid(40, 100.0, channels=3, seed=1)
    node[7] = 0xFFFFFFFF  # a phy without a NetDevice
    models = {"logdistance": [(1, 3.0, 1.0, 46.6777)], "friis": [(2, 300000000.0 / 5.15e9, 1.0, 0.5)],
              "chain": [(1, 3.0, 1.0, 46.6777), (4, 2500.0, 0, 0)]}[loss_kind]
    ch_o, ch_g = nsref.loss_chain(*models), nsgpu.loss_chain(*models)
    phys = nsgpu.PhyList(x, y, z, chan, node)
    if not ranked:
        phys.soa.chan_rank = None
        phys.soa.chan_count = None
    senders = [0, 5, 777, 1599, 1234, 42]
    tx = np.zeros(len(senders), dtype=nsgpu.TX_DESC_DTYPE)
    tx["now_ts"] = [0, 10**9, 123456789, 5, 2**40, 999]
    tx["tx_dbm"] = [16.0206, 20.0, 0.0, 16.0206, -3.5, 17.0]
    tx["sender"] = senders
    tx["uid_base"] = [4, 1000, 77, 2**31, 5, 12345]
    fo = nsgpu.Fanout(phys, len(senders))
    fo.upload_tx(tx)
    fo.launch_yans(len(senders), ch_g, 3e8)
    outs, _ = fo.results(len(senders))
    for t, s in enumerate(senders):
        want = nsref.fanout_yans(x, y, z, chan, node, s, tx["tx_dbm"][t], ch_o, 3e8, int(tx["now_ts"][t]),
                                 int(tx["uid_base"][t]))
        compare(outs[t], want, (loss_kind, s))


def test_spectrum_fanout_cutoff_compaction():
    import nsgpu
    x, y, z, chan, node = grid(50, 37.0, seed=2)
    models = [(1, 3.0, 1.0, 46.6777)]
    ch_o, ch_g = nsref.loss_chain(*models), nsgpu.loss_chain(*models)
    phys = nsgpu.PhyList(x, y, z, chan, node)
    nb = 8
    senders = [0, 1275, 2499, 60]
    tx = np.zeros(len(senders), dtype=nsgpu.TX_DESC_DTYPE)
    tx["now_ts"] = [0, 7, 10**6, 3]
    tx["sender"] = senders
    tx["uid_base"] = [4, 400, 40000, 9]
    psd = np.random.default_rng(5).random((len(senders), nb)) * 1e-12
    fo = nsgpu.Fanout(phys, len(senders), nbands=nb)
    fo.upload_tx(tx)
    nsgpu.check(nsgpu.lib().nsgpu_memcpy_htod(fo.psd_tx.ptr, np.ascontiguousarray(psd).ctypes.data, psd.nbytes,
                                              None))
    max_loss = 100.0
    fo.launch_spectrum(len(senders), ch_g, 3e8, max_loss)
    outs, psds = fo.results(len(senders))
    margin = []
    for t, s in enumerate(senders):
        want, wpsd = nsref.fanout_spectrum(x, y, z, node, s, ch_o, 3e8, max_loss, psd[t], int(tx["now_ts"][t]),
                                           int(tx["uid_base"][t]))
        assert 0 < len(want) < len(x) - 1  # the cutoff really compacts
        if len(outs[t]) != len(want):
            margin.append((t, len(outs[t]), len(want)))
            continue
        compare(outs[t], want, ("spectrum", s))
        np.testing.assert_allclose(psds[t], wpsd, rtol=RTOL, atol=0)
    assert not margin, f"receivers at the MaxLossDb margin differ: {margin}"
