"""ns3::HipSimulatorImpl's call sequence (tests/plugin_sim.py, line for line the C++ plugin) through the
raw-handle C-ABI, against the oracle's restated DefaultSimulatorImpl (default-simulator-impl.cc).

Covers what the plugin owns beyond the window runtime: the destroy list kept in the runtime
(SimulatorEventsTestCase's destroy section, simulator-test-suite.cc:111-168, plus a destroy event
scheduled by a destroy closure and one removed by an earlier destroy closure — :79-92 pops the list
from the front until it is empty), IsFinished = empty || stopped (:133-137), RunOneEvent dispatching
whatever the stop flag says (:167-170), and the reference counts the runtime holds."""
import random

import pytest

import nsgpu
import nsref
from plugin_sim import PluginSim
from sim_scripts import random_script, simulator_events_script

pytestmark = pytest.mark.gpu

US = 1000


@pytest.fixture(scope="module", autouse=True)
def _device():
    nsgpu.check(nsgpu.lib().nsgpu_set_device(0))


@pytest.mark.parametrize("batch", [0, 1, 3])
def test_simulator_events_script_plugin(batch):
    p = PluginSim(batch=batch)
    assert simulator_events_script(p) == []
    p.dispose()
    assert p.held() == 0 and not p.unref_errors
    o = nsref.Sim()
    assert simulator_events_script(o) == []


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("batch", [0, 2, 16])
def test_random_script_plugin_matches_oracle(seed, batch):
    p = PluginSim(batch=batch)
    got = random_script(p, seed)
    want = random_script(nsref.Sim(nsref.SCHED_MAP), seed)
    assert got == want
    p.dispose()
    assert p.held() == 0 and not p.unref_errors


def destroy_script(sim):
    """Destroy-list semantics beyond SimulatorEventsTestCase: a destroy closure schedules a destroy
    event (it runs, after the rest of the list), removes a later one (it does not run), cancels one
    (it does not run), and sees a pending one as not expired.  Returns the run order and the
    IsExpired observations."""
    log = []
    ids = {}

    def d(name, action=None):
        def cb():
            log.append(name)
            if action:
                action()
        return cb

    def a_action():
        log.append(("B pending", not sim.is_expired(ids["B"])))
        sim.remove(ids["B"])
        log.append(("B after remove", sim.is_expired(ids["B"])))
        ids["E"] = sim.schedule_destroy(d("E", lambda: log.append(("E self", sim.is_expired(ids["E"])))))
        sim.cancel(ids["C"])

    sim.schedule(5 * US, lambda: log.append(("run", sim.now())))
    ids["A"] = sim.schedule_destroy(d("A", a_action))
    ids["B"] = sim.schedule_destroy(d("B"))
    ids["C"] = sim.schedule_destroy(d("C"))
    ids["D"] = sim.schedule_destroy(d("D", lambda: sim.schedule_destroy(d("F"))))
    sim.run()
    log.append(("A before destroy", sim.is_expired(ids["A"])))
    sim.destroy()
    log.append(("A after destroy", sim.is_expired(ids["A"])))
    log.append(("E after destroy", sim.is_expired(ids["E"])))
    return log


def test_destroy_list_semantics_match_oracle():
    p = PluginSim()
    got = destroy_script(p)
    want = destroy_script(nsref.Sim())
    assert got == want
    # what the reference does (default-simulator-impl.cc:79-92): E and F run after D, B and C never
    names = [x for x in got if isinstance(x, str)]
    assert names == ["A", "D", "E", "F"]
    p.dispose()
    assert p.held() == 0 and not p.unref_errors


def stop_script(sim):
    """Run / Stop / IsFinished / RunOneEvent interplay (:133-170)."""
    log = []
    for t, name in ((1, "a"), (2, "b"), (3, "c"), (4, "d"), (4, "e")):
        def cb(name=name):
            log.append((name, sim.now()))
            if name == "b":
                sim.stop()
        sim.schedule(t * US, cb)
    sim.run()
    log.append(("finished after stop", sim.is_finished()))
    sim.run_one()  # RunOneEvent ignores the stop flag
    log.append(("finished after run_one", sim.is_finished()))
    sim.run()  # Run clears the flag and continues
    log.append(("finished at end", sim.is_finished()))
    # the common loop, on a fresh batch of events
    for t in range(3):
        sim.schedule((10 + t) * US, lambda t=t: log.append(("loop", t, sim.now())))
    sim.schedule(11 * US, lambda: sim.stop(2 * US))  # Stop (Time) inside the loop: an event like any other
    while not sim.is_finished():
        sim.run_one()
    log.append(("loop done", sim.is_finished()))
    return log


def test_stop_isfinished_runoneevent_match_oracle():
    p = PluginSim()
    got = stop_script(p)
    want = stop_script(nsref.Sim())
    assert got == want
    assert ("finished after stop", True) in got
    p.dispose()
    assert p.held() == 0 and not p.unref_errors


def test_callback_runtime_releases_closures():
    """nsgpu_sim's C-callback closures are released at dispatch / removal: after a run only the
    pending ones are held (the round-2 runtime kept every closure until it was freed)."""
    s = nsgpu.Sim()
    rng = random.Random(7)
    ids = [s.schedule(rng.randrange(0, 1000) * US, lambda: None) for _ in range(2000)]
    for eid in ids[::7]:
        s.remove(eid)
    late = [s.schedule(10_000 * US + k, lambda: None) for k in range(5)]
    s.stop(5000 * US)
    s.run()
    assert s.live_closures() == len(late)
    assert all(not s.is_expired(e) for e in late)
    assert all(s.is_expired(e) for e in ids)
    # an id of a released (recycled) slot stays expired after the slot is reused
    again = [s.schedule(1, lambda: None) for _ in range(100)]
    assert all(s.is_expired(e) for e in ids) and not any(s.is_expired(e) for e in again)
    s.close()
