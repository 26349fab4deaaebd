"""CPU checks of the point-to-point oracle and the scenario builders (no GPU).

Conservation laws of the restated reference chain (queue.cc / drop-tail-queue.cc / p2p device):
every packet a device transmits is received by its peer unless the run stopped first, every
enqueued packet is dequeued or still queued, and without drops every sent packet reaches its sink."""
import numpy as np

import nsref
import p2p


def run_oracle(sc, log_cap=0):
    s = sc.c_struct()
    st = p2p.P2PStats()
    devc = np.zeros(s.n_devices, p2p.DEV_COUNTERS_DTYPE)
    appc = np.zeros(s.n_apps, p2p.APP_COUNTERS_DTYPE)
    secs, log = nsref.p2p_run(s, st, devc, appc, log_cap)
    return st, devc, appc, log


def test_grid_builder_mirrors_helper_order():
    g = p2p.grid(3, 4)
    # node (y, x) creation interleaved with its row link then column link (point-to-point-grid.cc:45-64)
    kinds = [k for k, _ in g.setup]
    # NodeListPriv singleton's ScheduleDestroy, node 0, node 1, its row link (2 devices), then the
    # ChannelListPriv singleton's ScheduleDestroy (channel created after both devices)
    assert kinds[:6] == [p2p.SETUP_UID, p2p.SETUP_NODE, p2p.SETUP_NODE, p2p.SETUP_DEVICE, p2p.SETUP_DEVICE,
                         p2p.SETUP_UID]
    assert kinds.count(p2p.SETUP_NOOP) == 12  # one LoopbackNetDevice per node
    assert len(g.dev) == 2 * (3 * 3 + 2 * 4)  # rows*(cols-1) + (rows-1)*cols links
    assert sum(1 for k in kinds if k == p2p.SETUP_NODE) == 12
    # every node routes to every destination, by XY
    for d, slot in g.dst_slot.items():
        col = g.route[:, slot]
        assert col[d] == p2p.NO_ROUTE and (np.delete(col, d) != p2p.NO_ROUTE).all()


def test_grid_no_drop_conservation():
    g = p2p.grid(6, 6, stop_ns=500_000_000, sim_stop_ns=600_000_000)
    st, devc, appc, _ = run_oracle(g)
    onoff = np.array([a["kind"] == p2p.APP_ONOFF for a in g.apps])
    assert devc["drop_packets"].sum() == 0
    assert appc["tx_packets"][onoff].sum() == appc["rx_packets"][~onoff].sum() > 0
    assert (devc["enq_packets"] == devc["deq_packets"]).all()
    assert st.cancelled >= 0 and st.ttl_drops == 0 and st.no_route_drops == 0


def test_random_topology_queue_conservation():
    for seed in range(5):
        sc = p2p.random_topology(15, 25, 8, seed)
        st, devc, appc, (lts, luid, lctx) = run_oracle(sc, log_cap=200000)
        assert st.dispatched > 100
        # a queue never holds more than MaxPackets, every enqueue is dequeued or still queued
        assert (devc["enq_packets"] >= devc["deq_packets"]).all()
        assert ((devc["enq_packets"] - devc["deq_packets"]) <= 20).all()
        # pop order is (ts, uid) ascending
        n = int(min(st.dispatched, 200000))
        key = lts[:n].astype(object) * (1 << 32) + luid[:n].astype(object)
        assert all(key[i] < key[i + 1] for i in range(n - 1))


def test_stop_application_before_start_leaves_the_flow_running():
    """Application::DoStart (src/network/model/application.cc:87-95) schedules StartApplication at StartTime and,
    when StopTime != 0, StopApplication at StopTime — with StopTime < StartTime the stop runs first (it cancels
    nothing yet) and the flow then runs until Simulator::Stop: the same packets as a flow that never stops.
    (Round 4's r04c GPU run used this scenario without a Simulator::Stop: unbounded in ns-3 as well.)"""
    def run(app_stop):
        sc = p2p.grid(2, 2, start_ns=100_000_000, stop_ns=app_stop, sim_stop_ns=1_000_000_000, flows=[(0, 3)])
        s = sc.c_struct()
        st = p2p.P2PStats()
        devc = np.zeros(s.n_devices, p2p.DEV_COUNTERS_DTYPE)
        appc = np.zeros(s.n_apps, p2p.APP_COUNTERS_DTYPE)
        nsref.p2p_run(s, st, devc, appc, 0)
        onoff = [i for i, a in enumerate(sc.apps) if a["kind"] == p2p.APP_ONOFF][0]
        return st, appc, onoff
    st_early, appc_early, a = run(20_000_000)
    st_never, appc_never, _ = run(0)
    assert appc_early["tx_packets"][a] == appc_never["tx_packets"][a] > 100  # (0.9 s / 8.192 ms)
    assert st_early.final_ts == 1_000_000_000
    # the stop event is one more dispatch (and one more uid) than the never-stopping flow's run
    assert st_early.dispatched == st_never.dispatched + 1
