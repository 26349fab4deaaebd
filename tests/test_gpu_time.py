"""Seconds(double) -> int64 ns on the GPU vs the oracle's int64x64 restatement: bit-exact."""
import numpy as np
import pytest

import nsref

pytestmark = pytest.mark.gpu


def test_seconds_bit_exact():
    import nsgpu
    rng = np.random.default_rng(3)
    vals = np.concatenate([
        rng.random(20000),                      # [0, 1) s
        rng.random(20000) * 1e-5,               # propagation delays (d/c ~ ns..us)
        rng.random(5000) * 1e4,                 # long simulations
        -rng.random(5000),                      # negative times
        np.array([0.0, 1.0, 0.5, 1e-9, 2.5e-9, 0.001, 1 / 3, 4.294967296, 333.3e-9, 1e-300, 9e9, -1e-9]),
        rng.uniform(0, 20000, 2000) / 3e8,      # distance / speed of light
    ])
    got = nsgpu.seconds_to_ts(vals)
    want = nsref.seconds_batch(vals)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, list(zip(vals[bad][:5], got[bad][:5], want[bad][:5]))
