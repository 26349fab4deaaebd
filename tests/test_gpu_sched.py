"""HipBatchScheduler + HipSimulatorImpl host runtime on the GPU vs the oracle.

* SimulatorEventsTestCase (src/core/test/simulator-test-suite.cc:111-168) on the GPU-backed runtime;
* randomized Schedule/ScheduleWithContext/ScheduleNow/Cancel/Remove scripts: the dispatch log
  (now, context, tag) must equal the oracle's DefaultSimulatorImpl + MapScheduler log;
* the bare Scheduler interface under a random Insert/RemoveNext/Remove mix (small batches force
  many device flush/merge/pop cycles) pops in MapScheduler (ts, uid) order."""
import heapq

import numpy as np
import pytest

import nsref
from sim_scripts import simulator_events_script, random_script

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("batch", [1, 3, 64])
def test_events_script_gpu(batch):
    import nsgpu
    s = nsgpu.Sim(batch=batch)
    assert simulator_events_script(s) == []
    s.close()


@pytest.mark.parametrize("seed,batch", [(1, 2), (7, 5), (11, 64), (23, 4096)])
def test_random_script_matches_oracle(seed, batch):
    import nsgpu
    o = nsref.Sim(nsref.SCHED_MAP)
    want = random_script(o, seed=seed, n_ops=1500)
    g = nsgpu.Sim(batch=batch)
    got = random_script(g, seed=seed, n_ops=1500)
    assert got == want and len(want) > 30
    assert g.next_uid() == o.next_uid() and g.dispatched() == o.dispatched()


@pytest.mark.parametrize("batch", [1, 16, 1000])
def test_scheduler_interface_random(batch):
    import nsgpu
    rng = np.random.default_rng(batch)
    s = nsgpu.Sched(batch=batch)
    ref = []        # heap of (ts, uid)
    alive = {}      # uid -> (ts, uid, ctx, handle)
    uid = 4
    now = 0
    popped = []
    for step in range(4000):
        op = rng.random()
        if op < 0.5 or not alive:
            k = int(rng.integers(1, 40))
            evs = []
            for _ in range(k):
                ts = now + int(rng.integers(0, 5000))
                evs.append((ts, uid, int(rng.integers(0, 9)), uid * 8))
                heapq.heappush(ref, (ts, uid))
                alive[uid] = evs[-1]
                uid += 1
            s.insert(evs)
        elif op < 0.9:
            while ref and ref[0][1] not in alive:
                heapq.heappop(ref)
            e = s.remove_next()
            ts, u = heapq.heappop(ref)
            assert (int(e["ts"]), int(e["uid"])) == (ts, u)
            assert int(e["handle"]) == u * 8
            del alive[u]
            now = ts
            popped.append(u)
        else:
            u = list(alive)[int(rng.integers(0, len(alive)))]
            s.remove(alive.pop(u))
        assert s.size() == len(alive)
    # drain
    while alive:
        while ref and ref[0][1] not in alive:
            heapq.heappop(ref)
        e = s.remove_next()
        ts, u = heapq.heappop(ref)
        assert (int(e["ts"]), int(e["uid"])) == (ts, u)
        del alive[u]
    assert s.is_empty()
