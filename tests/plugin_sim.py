"""PluginSim: ns3::HipSimulatorImpl's call sequence, line for line, over the raw-handle C-ABI.

The C++ plugin (ns-3-dev-dnemu_amd/ns3-module/model/hip-simulator-impl.cc) needs an ns-3 build to run;
this mirror makes exactly its calls into libnsgpu (nsgpu_sim_insert / pop_window / pop_one / begin /
destroy_* / remove_key / key_expired / is_finished ...) with Python objects standing in for EventImpl
(a ref count held by the runtime, a cancel flag, Invoke skipping a cancelled closure), so the
parity tests drive the plugin's logic with the sim_scripts the oracle runs.  Handles are even
integers, as EventImpl* are even pointers.
"""
import nsgpu


class PyEventImpl:
    """ns3::EventImpl (event-impl.cc:34-53): Invoke runs the closure unless cancelled."""

    def __init__(self, fn):
        self.fn = fn
        self.cancelled = False
        self.runtime_refs = 0  # references the runtime's queue / destroy list hold (Ref/Unref balance)

    def invoke(self):
        if not self.cancelled:
            self.fn()


class PluginSim:
    def __init__(self, batch=0):
        self.rt = nsgpu.Sim(batch=batch)
        self.objs = {}
        self._next = 2
        self.unref_errors = []

    # ---- EventImpl bookkeeping ----
    def _new(self, cb):
        ev = PyEventImpl(cb)
        h = self._next
        self._next += 2
        self.objs[h] = ev
        return h, ev

    def _ref(self, h):
        self.objs[h].runtime_refs += 1

    def _unref(self, h):
        ev = self.objs[h]
        ev.runtime_refs -= 1
        if ev.runtime_refs < 0:
            self.unref_errors.append(h)

    def held(self):
        return sum(ev.runtime_refs for ev in self.objs.values())

    # ---- SimulatorImpl ----
    def now(self):
        return self.rt.now()

    def context(self):
        return self.rt.context()

    def schedule(self, delay, cb):  # HipSimulatorImpl::Schedule -> Enqueue
        assert delay >= 0
        ts = delay + self.rt.now()
        h, _ = self._new(cb)
        ctx = self.rt.context()
        uid = self.rt.insert_raw(ts, ctx, h)
        self._ref(h)  # Simulator::Schedule hands the queue one reference
        return (h, ts, ctx, uid)

    def schedule_with_context(self, ctx, delay, cb):
        h, _ = self._new(cb)
        self.rt.insert_raw(self.rt.now() + delay, ctx, h)
        self._ref(h)

    def schedule_now(self, cb):
        return self.schedule(0, cb)

    def schedule_destroy(self, cb):
        h, _ = self._new(cb)
        ts = self.rt.destroy_insert(h)
        self._ref(h)  # event->Ref () for the runtime's list entry
        return (h, ts, 0xFFFFFFFF, 2)

    def is_expired(self, eid):
        h, ts, _ctx, uid = eid
        ev = self.objs.get(h)
        if ev is None or ev.cancelled:
            return True
        if uid == 2:
            return not self.rt.destroy_pending(h, ts)
        return self.rt.key_expired(ts, uid)

    def remove(self, eid):
        h, ts, ctx, uid = eid
        if uid == 2:
            if self.rt.destroy_remove(h, ts):
                self._unref(h)
            return
        if self.is_expired(eid):
            return
        self.rt.remove_key(ts, uid, ctx, h)
        self.objs[h].cancelled = True
        self._unref(h)  # the queue's reference

    def cancel(self, eid):
        if not self.is_expired(eid):
            self.objs[eid[0]].cancelled = True

    def _dispatch(self, window):
        for e in window:
            if self.rt.begin(e) != 0:
                continue
            h = int(e["handle"]) & ~1
            self.objs[h].invoke()
            self._unref(h)

    def run(self):
        self.rt.set_stop(0)
        while True:
            w = self.rt.pop_window(4096)
            if len(w) == 0:
                return
            self._dispatch(w)

    def run_one(self):
        w = self.rt.pop_one()
        assert len(w) == 1, "RunOneEvent: no pending event"
        self._dispatch(w)

    def is_finished(self):
        return self.rt.is_finished()

    def stop(self, delay=None):
        if delay is None:
            self.rt.set_stop(1)
        else:  # Simulator::Schedule (time, &Simulator::Stop)
            self.schedule(delay, lambda: self.stop())

    def destroy(self):
        while True:
            h = self.rt.destroy_pop()
            if h is None:
                return
            ev = self.objs[h]
            if not ev.cancelled:
                ev.invoke()
            self._unref(h)

    def dispose(self):  # DoDispose: the pending events' and the destroy list's references
        while True:
            w = self.rt.drain()
            if len(w) == 0:
                break
            for e in w:
                self._unref(int(e["handle"]) & ~1)
        while True:
            h = self.rt.destroy_pop()
            if h is None:
                break
            self._unref(h)

    def close(self):
        self.rt.close()
