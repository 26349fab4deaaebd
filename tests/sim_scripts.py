"""Backend-agnostic restatements of the reference's simulator event scripts.

`simulator_events_script` follows SimulatorEventsTestCase::DoRun
(src/core/test/simulator-test-suite.cc:111-168) step by step; `sim` is any object with the
Sim interface of oracle/nsref.py (schedule/remove/cancel/is_expired/run/destroy/now).
Returns the list of failed expectations (empty = pass).
"""

US = 1000  # MicroSeconds (1) at NS resolution


def simulator_events_script(sim):
    fails = []

    def expect(cond, msg):
        if not cond:
            fails.append(msg)

    st = {"a": True, "b": False, "c": True, "d": False, "destroy": False, "idC": None, "destroyId": None}

    def A():
        st["a"] = False

    def D():
        st["d"] = (sim.now() // US) == 11 + 10

    def B():
        st["b"] = (sim.now() // US) == 11
        sim.remove(st["idC"])
        sim.schedule(10 * US, D)

    def C():
        st["c"] = False

    def destroy():
        if sim.is_expired(st["destroyId"]):
            st["destroy"] = True

    a = sim.schedule(10 * US, A)
    sim.schedule(11 * US, B)
    st["idC"] = sim.schedule(12 * US, C)
    expect(not sim.is_expired(st["idC"]), "idC expired early")
    expect(not sim.is_expired(a), "a expired early")
    sim.cancel(a)
    expect(sim.is_expired(a), "a not expired after cancel")
    sim.run()
    expect(st["a"], "Event A did not run ?")
    expect(st["b"], "Event B did not run ?")
    expect(st["c"], "Event C did not run ?")
    expect(st["d"], "Event D did not run ?")

    an_id = sim.schedule_now(lambda: None)
    expect(not sim.is_expired(an_id), "Event should not have expired yet.")
    sim.remove(an_id)
    expect(sim.is_expired(an_id), "Event was removed: it is now expired")

    st["destroyId"] = sim.schedule_destroy(destroy)
    expect(not sim.is_expired(st["destroyId"]), "destroy 1 expired early")
    sim.cancel(st["destroyId"])
    expect(sim.is_expired(st["destroyId"]), "destroy 1 not expired after cancel")

    st["destroyId"] = sim.schedule_destroy(destroy)
    expect(not sim.is_expired(st["destroyId"]), "destroy 2 expired early")
    sim.remove(st["destroyId"])
    expect(sim.is_expired(st["destroyId"]), "destroy 2 not expired after remove")

    st["destroyId"] = sim.schedule_destroy(destroy)
    expect(not sim.is_expired(st["destroyId"]), "destroy 3 expired early")
    sim.run()
    expect(not sim.is_expired(st["destroyId"]), "destroy 3 expired after run")
    expect(not st["destroy"], "Event should not have run")
    sim.destroy()
    expect(sim.is_expired(st["destroyId"]), "Event should have expired now")
    expect(st["destroy"], "Event should have run")
    return fails


def random_script(sim, seed, n_ops=400):
    """Deterministic randomized Schedule/ScheduleWithContext/ScheduleNow/Cancel/Remove mix.

    Returns the dispatch log [(now, context, tag)] — identical for any backend that keeps
    DefaultSimulatorImpl semantics (uid order, (ts, uid) pop order, cancelled dispatch skipped).
    """
    import random
    rng = random.Random(seed)
    log = []
    ids = []
    counter = [0]

    def make(tag):
        def cb():
            log.append((sim.now(), sim.context(), tag))
            # handlers schedule more work, like model code does
            for _ in range(2 if rng.random() < 0.35 else 1):
                if counter[0] >= n_ops or rng.random() > 0.85:
                    break
                counter[0] += 1
                op = rng.random()
                t = counter[0]
                if op < 0.45:
                    ids.append(sim.schedule(rng.randrange(0, 50), make(t)))
                elif op < 0.75:
                    sim.schedule_with_context(rng.randrange(0, 8), rng.randrange(0, 50), make(t))
                elif op < 0.85:
                    ids.append(sim.schedule_now(make(t)))
                elif op < 0.93 and ids:
                    sim.cancel(ids[rng.randrange(len(ids))])
                elif ids:
                    sim.remove(ids[rng.randrange(len(ids))])
        return cb

    for i in range(20):
        counter[0] += 1
        ids.append(sim.schedule(rng.randrange(0, 30), make(-i - 1)))
    sim.run()
    return log
