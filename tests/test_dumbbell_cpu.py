"""Config 5 scenario builder (simple-distributed.cc dumbbell) on the oracle: shape, system ids, and
the example's outcome (every left leaf's single 512-B datagram reaches its right leaf when the
router link is not congested)."""
import numpy as np

import nsref
import p2p


def run(sc):
    s = sc.c_struct()
    st = p2p.P2PStats()
    devc = np.zeros(s.n_devices, p2p.DEV_COUNTERS_DTYPE)
    appc = np.zeros(s.n_apps, p2p.APP_COUNTERS_DTYPE)
    nsref.p2p_run(s, st, devc, appc, 0)
    return st, devc, appc


def test_dumbbell_shape_and_owner():
    sc = p2p.dumbbell(4)
    assert sc.n_nodes == 10 and len(sc.dev) == 2 * 9 and sc.n_dst == 4
    own = p2p.dumbbell_owner(4)
    assert own.tolist() == [0] * 5 + [1] * 5
    own3 = p2p.dumbbell_owner(4, 3)
    assert own3.tolist() == [0] * 5 + [1] + [1, 1, 2, 2]


def test_dumbbell_example_outcome():
    st, devc, appc = run(p2p.dumbbell(4))
    sinks = appc[:4]
    assert sinks["rx_packets"].tolist() == [1] * 4 and sinks["rx_bytes"].tolist() == [512] * 4
    assert devc["drop_packets"].sum() == 0 and st.final_ts == 5_000_000_000


def test_dumbbell_router_congestion_drops():
    st, devc, appc = run(p2p.dumbbell(300))
    sc = p2p.dumbbell(300)
    ra = 0  # router 1's router-link device
    assert devc["drop_packets"][ra] > 0
    assert appc["rx_packets"][:300].sum() + devc["drop_packets"].sum() == 300
    assert sc.n_nodes == 602
