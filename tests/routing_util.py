"""Test helper: the oracle's global-routing table (oracle/nsref_route.cc) for a p2p.Scenario, in the
scenario's [node][destination slot] layout (NO_ROUTE for the destination itself)."""
import numpy as np

import nsref
import p2p


def oracle_table(sc, dst_addr=None):
    """dst_addr: {destination node: address used}; default: the destination's first device's address."""
    n = len(sc.dev)
    dnode = [r[0] for r in sc.dev]
    dpeer = [r[1] for r in sc.dev]
    dsts = sorted(sc.dst_slot, key=sc.dst_slot.get)
    addrs = []
    for d in dsts:
        if dst_addr and d in dst_addr:
            addrs.append(dst_addr[d])
        else:
            addrs.append(sc.dev_addr[next(i for i in range(n) if dnode[i] == d)])
    R = nsref.global_routes(dnode, dpeer, [sc.dev_addr[i] for i in range(n)], [sc.dev_mask[i] for i in range(n)],
                            [sc.dev_ifindex[i] for i in range(n)], sc.n_nodes, addrs).copy()
    for k, d in enumerate(dsts):
        assert R[d, k] == 0xFFFFFFFE  # RouteInput: local delivery
        R[d, k] = p2p.NO_ROUTE
    return R


def scenario_table(sc):
    if sc.route is not None:
        return sc.route
    R = np.zeros((sc.n_nodes, sc.n_dst), np.uint32)
    for n in range(sc.n_nodes):
        for k in range(sc.n_dst):
            R[n, k] = sc.next_hop(n, k)
    for d, k in sc.dst_slot.items():  # (a compressed table's default at the destination is never looked up)
        R[d, k] = p2p.NO_ROUTE
    return R
