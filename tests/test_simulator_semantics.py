"""SimulatorEventsTestCase (src/core/test/simulator-test-suite.cc:111-168, run against
List/Map/Heap at :463-482) on the restated oracle engine.  The GPU-backed runtime runs the
same script in tests/test_gpu_sched.py."""
import pytest

import nsref
from sim_scripts import simulator_events_script, random_script


@pytest.mark.parametrize("sched", [nsref.SCHED_MAP, nsref.SCHED_HEAP, nsref.SCHED_LIST])
def test_events_script_oracle(sched):
    s = nsref.Sim(sched)
    assert simulator_events_script(s) == []
    s.close()


def test_random_script_schedulers_agree():
    logs = []
    for sched in (nsref.SCHED_MAP, nsref.SCHED_LIST):
        s = nsref.Sim(sched)
        logs.append(random_script(s, seed=7))
        s.close()
    assert logs[0] == logs[1] and len(logs[0]) > 50
