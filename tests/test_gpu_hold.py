"""GPU-resident utils/bench-simulator.cc (config 1) vs the oracle (DefaultSimulatorImpl + MapScheduler).

Small runs compare the full pop log (ts, uid of every dispatch, in order); the full-size run
(10,000 pending, 5e6 holds — SURVEY §8(d)) compares counters, final time, next uid and the
order-sensitive digest of the whole pop order."""
import numpy as np
import pytest

import nsref

pytestmark = pytest.mark.gpu


def run_gpu(dist, total, log_cap=0):
    import nsgpu
    h = nsgpu.HoldRun(dist, total, log_cap=log_cap)
    h.launch()
    return h.result()


@pytest.mark.parametrize("n,total", [(1, 10), (7, 100), (200, 20000), (1000, 3000), (10000, 10)])
def test_hold_full_log(bench_dist, n, total):
    dist = bench_dist[:n]
    cap = n + total + 1
    res, lts, luid = nsref.churn_run(dist, total, log_cap=cap)
    st, gts, guid = run_gpu(dist, total, log_cap=cap)
    assert st.dispatched == res.dispatched == cap
    assert np.array_equal(gts, lts) and np.array_equal(guid, luid)
    assert st.digest == res.digest and st.final_ts == res.final_ts and st.next_uid == res.next_uid


def test_hold_ties_and_zero_delays():
    # equal timestamps (uid breaks ties) and zero delays (child at now, after every pending uid)
    dist = np.array([5, 5, 0, 3, 5, 0, 0, 1], dtype=np.uint64)
    total = 500
    cap = len(dist) + total + 1
    res, lts, luid = nsref.churn_run(dist, total, log_cap=cap)
    st, gts, guid = run_gpu(dist, total, log_cap=cap)
    assert np.array_equal(gts, lts) and np.array_equal(guid, luid)


def test_hold_full_size_digest(bench_dist):
    total = 5_000_000
    res, _, _ = nsref.churn_run(bench_dist, total)
    st, _, _ = run_gpu(bench_dist, total)
    assert (st.dispatched, st.holds, st.final_ts, st.next_uid, st.digest) == \
        (res.dispatched, res.holds, res.final_ts, res.next_uid, res.digest)


def test_hold_wide_delays():
    # utils/generate-distributions.pl draws U[0, 1e7) seconds: delays >= 2^31 ns take the wide kernel
    rng = np.random.default_rng(11)
    secs = rng.random(300) * 1e7
    dist = (secs * 1000000000).astype(np.uint64)
    total = 3000
    cap = len(dist) + total + 1
    res, lts, luid = nsref.churn_run(dist, total, log_cap=cap)
    st, gts, guid = run_gpu(dist, total, log_cap=cap)
    assert np.array_equal(gts, lts) and np.array_equal(guid, luid)
    assert st.digest == res.digest and st.next_uid == res.next_uid


def test_hold_mixed_boundary():
    # one delay exactly at the packed limit (2^31 - 1) and one just above it (wide path)
    for top in ((1 << 31) - 1, 1 << 31):
        dist = np.array([top, 1, 2, top, 0, 5], dtype=np.uint64)
        total = 200
        cap = len(dist) + total + 1
        res, lts, luid = nsref.churn_run(dist, total, log_cap=cap)
        st, gts, guid = run_gpu(dist, total, log_cap=cap)
        assert np.array_equal(gts, lts) and np.array_equal(guid, luid), top
