"""SimulatorEventsTestCase (src/core/test/simulator-test-suite.cc:111-168, run against
List/Map/Heap/Calendar at :463-482) on the restated oracle engine.  The GPU-backed runtime runs the
same script in tests/test_gpu_sched.py."""
import pytest

import nsref
from sim_scripts import simulator_events_script, random_script


@pytest.mark.parametrize("sched", [nsref.SCHED_MAP, nsref.SCHED_HEAP, nsref.SCHED_LIST, nsref.SCHED_CALENDAR])
def test_events_script_oracle(sched):
    s = nsref.Sim(sched)
    assert simulator_events_script(s) == []
    s.close()


def test_random_script_schedulers_agree():
    logs = []
    for sched in (nsref.SCHED_MAP, nsref.SCHED_LIST, nsref.SCHED_CALENDAR):
        s = nsref.Sim(sched)
        logs.append(random_script(s, seed=7))
        s.close()
    assert logs[0] == logs[1] == logs[2] and len(logs[0]) > 50


def test_calendar_churn_pop_order_equals_map(bench_dist):
    """bench-simulator with CalendarScheduler below the H3 limit (50k holds, ~3.7 s simulated):
    the same pop order as MapScheduler (full log), with resizes up to 16k buckets on the way."""
    n = 60001 + 1
    m, mts, muid = nsref.churn_run(bench_dist, 50_000, nsref.SCHED_MAP, log_cap=n)
    c, cts, cuid = nsref.churn_run(bench_dist, 50_000, nsref.SCHED_CALENDAR, log_cap=n)
    assert c.dispatched == m.dispatched == 60001 and c.digest == m.digest
    assert (cts == mts).all() and (cuid == muid).all()


def test_calendar_h3_crash_point(bench_dist):
    """SURVEY H3 (calendar-scheduler.cc:128,157,182-185): the probe saw `bench-simulator --calendar` abort once
    simulated time passes ~4.3 s (clean at 50k holds, abort at 90k).  The restated sentinel path is reached
    exactly when every pending event is later than 0xffffffff ns, and the order up to it is Map's."""
    with pytest.raises(nsref.CalendarCrash) as e:
        nsref.churn_run(bench_dist, 90_000, nsref.SCHED_CALENDAR)
    r = e.value.result
    m, mts, _ = nsref.churn_run(bench_dist, 90_000, nsref.SCHED_MAP, log_cap=100001)
    assert 0 < r.dispatched < m.dispatched
    # the next event Map dispatches is past 2^32 ns, and so is everything still pending
    assert mts[r.dispatched] > 0xFFFFFFFF and r.final_ts == mts[r.dispatched - 1]
