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


def test_yans_channel_change_rebuilds_rank_tables():
    """YansWifiPhy::SetChannelNumber after the phy list was built: PhyList.set_channel updates the
    channel array and the rank tables together, so the one-pass placement stays the oracle's loop order."""
    import nsgpu
    x, y, z, chan, node = grid(30, 100.0, channels=2, seed=3)
    phys = nsgpu.PhyList(x, y, z, chan, node)
    for j, c in ((5, 2), (400, 1), (899, 3), (6, 2)):
        phys.set_channel(j, c)
        chan[j] = c
    ch_o, ch_g = nsref.loss_chain((1, 3.0, 1.0, 46.6777)), nsgpu.loss_chain((1, 3.0, 1.0, 46.6777))
    senders = [5, 400, 899, 0, 6]
    tx = np.zeros(len(senders), dtype=nsgpu.TX_DESC_DTYPE)
    tx["now_ts"], tx["tx_dbm"], tx["sender"], tx["uid_base"] = 1000, 16.0206, senders, 4
    fo = nsgpu.Fanout(phys, len(senders))
    fo.upload_tx(tx)
    fo.launch_yans(len(senders), ch_g, 3e8)
    outs, _ = fo.results(len(senders))
    for t, s in enumerate(senders):
        compare(outs[t], nsref.fanout_yans(x, y, z, chan, node, s, 16.0206, ch_o, 3e8, 1000, 4), ("chan", s))


def _models():
    from spectrum_util import bands_from_centers
    return [bands_from_centers(np.linspace(2.400e9, 2.480e9, 33)),   # uid 1
            bands_from_centers(np.linspace(2.405e9, 2.475e9, 8)),    # uid 2: coarser, offset
            bands_from_centers(np.linspace(2.390e9, 2.490e9, 51))]   # uid 3: wider, finer


def test_multimodel_spectrum_fanout():
    """MultiModelSpectrumChannel::StartTx: three rx SpectrumModels, receivers visited by model then AddRx
    order, tx PSDs in any model converted (SpectrumConverter) once per rx model, MaxLossDb compaction and the
    PropagationLoss trace of every receiver."""
    import nsgpu
    x, y, z, chan, node = grid(45, 41.0, seed=4)
    n = x.size
    rng = np.random.default_rng(9)
    rx_model = rng.integers(0, 3, n).astype(np.int32)
    models = _models()
    chain = [(1, 3.0, 1.0, 46.6777)]
    ch_o, ch_g = nsref.loss_chain(*chain), nsgpu.loss_chain(*chain)
    phys = nsgpu.PhyList(x, y, z, chan, node)
    senders = [0, 1012, n - 1, 77, 500, 1999]
    tx_model = [0, 1, 2, 1, 0, 2]
    tx = np.zeros(len(senders), dtype=nsgpu.TX_DESC_DTYPE)
    tx["now_ts"] = [0, 5, 10**9, 77, 3, 2**33]
    tx["sender"] = senders
    tx["uid_base"] = [4, 100, 2**31, 9, 77777, 5]
    psds = [rng.uniform(1e-14, 1e-12, len(models[m][0])) for m in tx_model]
    mf = nsgpu.MultiModelFanout(phys, rx_model, models, len(senders))
    mf.upload_tx(tx, tx_model, psds)
    max_loss = 105.0
    mf.launch(len(senders), ch_g, 3e8, max_loss)
    got = mf.results(len(senders))
    for t, s in enumerate(senders):
        want, wrows, wtr = nsref.fanout_spectrum_multi(x, y, z, node, rx_model, s, models, tx_model[t], psds[t], ch_o,
                                                       3e8, max_loss, int(tx["now_ts"][t]), int(tx["uid_base"][t]))
        recs, rows, tr = got[t]
        assert 0 < len(want) < n - 1
        compare(recs, want, ("multi", s))
        for a, b in zip(rows, wrows):
            np.testing.assert_allclose(a, b, rtol=RTOL, atol=0)
        assert np.array_equal(tr["rx_phy"], wtr["rx_phy"])
        np.testing.assert_allclose(tr["loss_db"], wtr["loss_db"], rtol=RTOL, atol=0)


def test_spectrum_converter_known_answers_on_gpu():
    """The reference's SpectrumConverterTestSuite (spectrum-value-test.cc:260-333) through the GPU channel."""
    import json
    import os
    import nsgpu
    from spectrum_util import bands_from_centers
    kat = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "spectrum_converter_kat.json")))
    names = sorted(kat["models"])
    models = [bands_from_centers(kat["models"][m]) for m in names]
    for case in kat["cases"]:
        x, y, z = np.array([0.0, 1.0]), np.zeros(2), np.zeros(2)
        phys = nsgpu.PhyList(x, y, z, np.ones(2, np.uint32), np.arange(2, dtype=np.uint32))
        rxm = [names.index(case["from"]), names.index(case["to"])]
        mf = nsgpu.MultiModelFanout(phys, rxm, models, 1)
        tx = np.zeros(1, dtype=nsgpu.TX_DESC_DTYPE)
        tx["uid_base"] = 4
        mf.upload_tx(tx, [rxm[0]], [case["input"]])
        mf.launch(1, nsgpu.loss_chain(), 0.0, 1e9)
        recs, rows, _ = mf.results(1)[0]
        assert len(recs) == 1
        assert np.max(np.abs(rows[0] - np.array(case["expected"]))) < kat["tolerance"]
