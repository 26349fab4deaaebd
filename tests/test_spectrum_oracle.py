"""MultiModelSpectrumChannel::StartTx / SpectrumConverter oracle (oracle/nsref_prop.cc) against the
reference's SpectrumConverterTestSuite known answers (src/spectrum/test/spectrum-value-test.cc:260-333,
tests/golden/spectrum_converter_kat.json) and against the single-model restatement."""
import json
import os

import numpy as np
import pytest

import nsref
from spectrum_util import bands_from_centers

HERE = os.path.dirname(os.path.abspath(__file__))
KAT = json.load(open(os.path.join(HERE, "golden", "spectrum_converter_kat.json")))


def convert_via_channel(frm, to, values):
    """A two-phy channel: phy 0 sends in model `frm`, phy 1 receives in model `to`, no loss model (gain 0 dB,
    the record's PSD is the converted PSD)."""
    names = sorted(KAT["models"])  # sof1 created first: smaller SpectrumModelUid
    models = [bands_from_centers(KAT["models"][n]) for n in names]
    rx_model = [names.index(frm), names.index(to)]
    chain = nsref.loss_chain()
    recs, rows, tr = nsref.fanout_spectrum_multi([0.0, 1.0], [0.0, 0.0], [0.0, 0.0], [0, 1], rx_model, 0, models,
                                                  names.index(frm), values, chain, 0.0, 1e9, 0, 4)
    assert len(recs) == 1 and recs[0]["phy"] == 1 and len(tr) == 1
    return rows[0]


@pytest.mark.parametrize("case", KAT["cases"], ids=lambda c: c["line"])
def test_converter_known_answers(case):
    got = convert_via_channel(case["from"], case["to"], case["input"])
    assert np.max(np.abs(got - np.array(case["expected"]))) < KAT["tolerance"]


def test_single_model_equals_single_model_channel():
    rng = np.random.default_rng(5)
    n = 300
    x, y = rng.uniform(0, 2000, n), rng.uniform(0, 2000, n)
    z = np.zeros(n)
    node = np.arange(n, dtype=np.uint32)
    fl, fh = bands_from_centers(np.linspace(2.4e9, 2.48e9, 17))
    psd = rng.uniform(1e-13, 1e-12, 17)
    chain = nsref.loss_chain((nsref.LOSS_LOG_DISTANCE, 3.0, 1.0, 46.6777))
    for sender in (0, 77, n - 1):
        a, pa = nsref.fanout_spectrum(x, y, z, node, sender, chain, 3e8, 110.0, psd, 1_000_000, 100)
        b, pb, tr = nsref.fanout_spectrum_multi(x, y, z, node, np.zeros(n, np.int32), sender, [(fl, fh)], 0, psd, chain,
                                                3e8, 110.0, 1_000_000, 100)
        assert np.array_equal(a, b) and np.array_equal(pa, np.array(pb))
        assert len(tr) == n - 1 and 0 < len(a) < n - 1  # the trace fires for receivers beyond MaxLossDb too
        assert np.array_equal(tr["rx_phy"], np.delete(np.arange(n), sender))


def test_receivers_visited_by_model_then_add_order():
    """m_rxSpectrumModelInfoMap is keyed by SpectrumModelUid: uids go to model 0's phys first."""
    n = 8
    rx_model = np.array([1, 0, 1, 0, 0, 1, 1, 0], np.int32)
    models = [bands_from_centers([1, 2, 3]), bands_from_centers([1.5, 2.5])]
    recs, rows, tr = nsref.fanout_spectrum_multi(np.arange(n) * 10.0, np.zeros(n), np.zeros(n), np.arange(n), rx_model,
                                                  2, models, 1, [1.0, 2.0], nsref.loss_chain(), 0.0, 1e9, 7, 50)
    want = [1, 3, 4, 7, 0, 5, 6]
    assert list(recs["phy"]) == want and list(recs["uid"]) == list(range(50, 57))
    assert list(tr["rx_phy"]) == want
    assert all(len(r) == (3 if rx_model[p] == 0 else 2) for r, p in zip(rows, recs["phy"]))
