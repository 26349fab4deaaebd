"""nsgpu_setup_from_journal (include/nsgpu.h, csrc/nsgpu_setup.cc): the uid-critical part of
NsgpuP2pScenario::FromNodeList, in the product library.  HipSimulatorImpl journals every setup-time Schedule
call, classified by what it starts (NodeListPriv::Add -> Node::Start, node-list.cc:124-131; Node::AddDevice /
AddApplication -> NetDevice::Start / Application::Start with the object's index on its node, node.cc:111-145);
the function turns the journal into the engine's setup list.  Checked against p2p.py's setup lists (the ones
every oracle / GPU test runs), with the program's own events interleaved, an application added before a later
link, and malformed journals (refused, never silently shifted).  No GPU."""
import numpy as np
import pytest

import nsgpu
import nsref
import p2p


def check_roundtrip(sc):
    j, devs, napp = p2p.scenario_journal(sc)
    setup, owned, dmap, amap, stop = p2p.setup_from_journal(j, devs, napp)
    assert setup == [(k, i if k != p2p.SETUP_UID else 0) for k, i in sc.setup]
    assert owned == [i for i, (k, _x) in enumerate(sc.setup) if k != p2p.SETUP_UID]
    assert stop == (sc.stop_ns if any(k == p2p.SETUP_STOP for k, _x in sc.setup) else -1)
    # engine device d is its node's device number (its position among the node's devices, loopback included)
    local = {}
    seen = [0] * sc.n_nodes
    for k, i in sc.setup:
        if k == p2p.SETUP_DEVICE:
            n = sc.dev[i][0]
            local[i] = (n, seen[n])
            seen[n] += 1
        elif k == p2p.SETUP_NOOP:
            seen[i] += 1
    assert dmap == [local[d] for d in range(len(sc.dev))]
    aseen = [0] * sc.n_nodes
    want = []
    for a in sc.apps:
        want.append((a["node"], aseen[a["node"]]))
        aseen[a["node"]] += 1
    assert amap == want
    return j, devs, napp


def test_first_cc():
    check_roundtrip(p2p.first_cc())


@pytest.mark.parametrize("shape", [(4, 4), (8, 8)])
def test_grid(shape):
    check_roundtrip(p2p.grid(*shape))


@pytest.mark.parametrize("seed", range(3))
def test_random_topology(seed):
    check_roundtrip(p2p.random_topology(20, 35, 6, seed))


def test_dumbbell():
    check_roundtrip(p2p.dumbbell(8))


def test_program_own_events_interleaved():
    """The program's own events (ts 0 with a node's context, later ones, context-free ones) between the helpers'
    start calls: each is a consumed uid at its place, the helpers' calls map as before."""
    sc = p2p.grid(3, 3)
    j, devs, napp = p2p.scenario_journal(sc)
    rng = np.random.default_rng(5)
    pos = sorted(rng.choice(np.arange(4, len(j)), 6, replace=False).tolist(), reverse=True)
    own = np.zeros(1, p2p.JOURNAL_DTYPE)
    rows = list(j)
    for n, p in enumerate(pos):
        e = own.copy()[0]
        e["kind"], e["context"], e["ts"] = p2p.J_CALL, [4, 0xFFFFFFFF, 8][n % 3], [0, 0, 7_000][n % 3]
        rows.insert(p, e)
    j2 = np.array(rows, dtype=p2p.JOURNAL_DTYPE)
    setup, owned, dmap, amap, _stop = p2p.setup_from_journal(j2, devs, napp)
    mine = [i for i, e in enumerate(j2) if e["kind"] == p2p.J_CALL]
    assert len(mine) == 6
    assert all(setup[i] == (p2p.SETUP_UID, 0) for i in mine)
    assert [s for i, s in enumerate(setup) if i not in mine] == [(k, i if k != p2p.SETUP_UID else 0) for k, i in sc.setup]
    assert not set(owned) & set(mine)
    assert len(dmap) == len(sc.dev) and len(amap) == len(sc.apps)


def app_before_link():
    """Node 0 gets a PacketSink before its second link (InternetStackHelper, an application, then one more
    PointToPointHelper::Install): node 0's journal has an Application::Start between two NetDevice::Starts."""
    sc = p2p.Scenario(3)
    a01, b01 = sc.link(0, 1, 5_000_000, 2_000_000)
    sc.install_stack()
    sc.add_sink(0, 0, 3_000_000_000)
    a02, b02 = sc.link(0, 2, 5_000_000, 2_000_000)
    sc.assign_link(a01, b01, p2p.ip("10.1.1.0"))
    sc.assign_link(a02, b02, p2p.ip("10.1.2.0"))
    sc.add_onoff(1, 0, 1_000_000_000, 1_500_000_000, on_s=1e9, off_s=0.0, remote_addr=sc.dev_addr[a01])
    sc.add_onoff(2, 0, 1_000_000_000, 1_500_000_000, on_s=1e9, off_s=0.0, remote_addr=sc.dev_addr[a02])
    sc.route_bfs()
    return sc


def test_application_added_before_a_device():
    sc = app_before_link()
    j, _devs, _napp = check_roundtrip(sc)
    k0 = [int(e["kind"]) for e in j if e["context"] == 0]
    assert k0.index(p2p.J_APP_START) < len(k0) - 1 - k0[::-1].index(p2p.J_DEVICE_START)
    # a positional mapping (Node::Start, then every device, then every application) would give node 0's
    # application start to its second point-to-point device: the classified journal does not
    s = sc.c_struct()
    st = p2p.P2PStats()
    devc = np.zeros(s.n_devices, p2p.DEV_COUNTERS_DTYPE)
    appc = np.zeros(s.n_apps, p2p.APP_COUNTERS_DTYPE)
    nsref.p2p_run(s, st, devc, appc, 0)
    assert appc["rx_packets"][0] > 0


def refused(j, devs, napp):
    with pytest.raises(nsgpu.NsgpuError):
        p2p.setup_from_journal(j, devs, napp)


def test_malformed_journals_are_refused():
    sc = p2p.grid(2, 2)
    j, devs, napp = p2p.scenario_journal(sc)
    first_dev = int(np.nonzero(j["kind"] == p2p.J_DEVICE_START)[0][0])
    # a device starting before its node
    b = j.copy()
    node = b[first_dev]["context"]
    nstart = int(np.nonzero((b["kind"] == p2p.J_NODE_START) & (b["context"] == node))[0][0])
    b[[nstart, first_dev]] = b[[first_dev, nstart]]
    refused(b, devs, napp)
    # a device index out of AddDevice order
    b = j.copy()
    b[first_dev]["local"] += 1
    refused(b, devs, napp)
    # a device that is not point-to-point
    d2 = [list(x) for x in devs]
    d2[int(j[first_dev]["context"])][0] = p2p.NDEV_OTHER
    refused(j, d2, napp)
    # a device the journal never starts (built before HipSimulatorImpl was selected)
    d2 = [list(x) for x in devs]
    d2[0].append(p2p.NDEV_P2P)
    refused(j, d2, napp)
    # an application count the journal does not match
    refused(j, devs, [x + (i == 1) for i, x in enumerate(napp)])
    # two Stop calls
    b = np.concatenate([j, j[-1:]])
    assert b[-1]["kind"] == p2p.J_STOP
    refused(b, devs, napp)
    # a start call at ts != 0 / for a node out of range
    b = j.copy()
    b[first_dev]["ts"] = 5
    refused(b, devs, napp)
    b = j.copy()
    b[first_dev]["context"] = 99
    refused(b, devs, napp)
    # a node started twice
    b = np.concatenate([j[:first_dev], j[nstart:nstart + 1], j[first_dev:]])
    refused(b, devs, napp)
