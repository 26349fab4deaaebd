"""Global routing: the scenario builders' next-hop tables against the oracle's
restatement of GlobalRouteManagerImpl::SPFCalculate + Ipv4GlobalRouting::LookupGlobal
(oracle/nsref_route.cc; global-route-manager-impl.cc:601-733,1327-1490, ipv4-global-routing.cc:136-242).

The reference tree holds no routing-table golden file for these topologies ("parity unpinned" beyond the
restatement); the tie-break rule the tables use is derived from the restated code in
p2p.Scenario.route_bfs's docstring and checked here on topologies with equal-cost paths."""
import numpy as np
import pytest

import p2p
from routing_util import oracle_table, scenario_table


@pytest.mark.parametrize("n", [2, 3, 5, 8, 16])
def test_grid_xy_routes_are_global_routing(n):
    """PointToPointGridHelper assigns row links 10.x before column links 11.x, so LookupGlobal's first
    ECMP exit (smallest next-hop address) moves along the row first: the grid's XY tables."""
    g = p2p.grid(n, n)
    assert np.array_equal(scenario_table(g), oracle_table(g))


def test_grid_32x32_routes_are_global_routing():
    g = p2p.grid(32, 32)  # global-routing parity pinned at <= 32 x 32
    assert np.array_equal(scenario_table(g), oracle_table(g))


def test_grid_rectangular_and_many_flows():
    g = p2p.grid(6, 9, flows=[(0, 53), (53, 0), (8, 45), (30, 4), (12, 12 + 9 * 4)])
    assert np.array_equal(scenario_table(g), oracle_table(g))


@pytest.mark.parametrize("seed", range(8))
def test_random_topologies(seed):
    sc = p2p.random_topology(40, 90, 12, seed)
    assert np.array_equal(scenario_table(sc), oracle_table(sc))


def test_every_address_of_a_destination_routes_alike():
    sc = p2p.random_topology(30, 70, 6, 3)
    base = oracle_table(sc)
    for d in sc.dst_slot:
        for i, r in enumerate(sc.dev):
            if r[0] == d:
                assert np.array_equal(oracle_table(sc, {d: sc.dev_addr[i]})[:, sc.dst_slot[d]], base[:, sc.dst_slot[d]])


def test_dumbbell_incast_first_cc():
    for sc in (p2p.dumbbell(5), p2p.dumbbell(5, compressed=True), p2p.incast(12), p2p.first_cc()):
        assert np.array_equal(scenario_table(sc), oracle_table(sc))


def _diamond(addr_order):
    """0 -- 1 -- 3 and 0 -- 2 -- 3: two equal-cost paths from 0 to 3; the link networks are assigned in
    `addr_order`, which decides the exit (the smaller next-hop address)."""
    sc = p2p.Scenario(4)
    links = [sc.link(0, 1, 1_000_000, 1_000_000), sc.link(0, 2, 1_000_000, 1_000_000),
             sc.link(1, 3, 1_000_000, 1_000_000), sc.link(2, 3, 1_000_000, 1_000_000)]
    sc.install_stack()
    for k in addr_order:
        da, db = links[k]
        sc.assign_link(da, db, p2p.ip("10.0.0.0") + (addr_order.index(k) << 8))
    sc.add_sink(3, 0, 0)
    sc.add_onoff(0, 3, 0, 1_000_000, remote_addr=sc.dev_addr[links[2][1]])
    sc.stop(2_000_000)
    sc.route_bfs()
    return sc, links


def test_ecmp_tie_break_is_the_smallest_next_hop_address():
    sc, links = _diamond([0, 1, 2, 3])  # 0-1 network first: next hop 10.0.0.2 (node 1) < 10.0.1.2 (node 2)
    R = oracle_table(sc)
    assert R[0, 0] == links[0][0]
    assert np.array_equal(R, scenario_table(sc))
    sc, links = _diamond([1, 0, 2, 3])  # 0-2 network first: node 2 is the smaller next hop
    R = oracle_table(sc)
    assert R[0, 0] == links[1][0]
    assert np.array_equal(R, scenario_table(sc))


def test_parallel_links_pick_the_smaller_peer_address():
    sc = p2p.Scenario(3)
    l0 = sc.link(0, 1, 1_000_000, 1_000_000)
    l1 = sc.link(0, 1, 1_000_000, 1_000_000)
    sc.link(1, 2, 1_000_000, 1_000_000)
    sc.install_stack()
    sc.assign_link(*l1, p2p.ip("10.0.0.0"))
    sc.assign_link(*l0, p2p.ip("10.0.1.0"))
    sc.assign_link(2 * 2, 2 * 2 + 1, p2p.ip("10.0.2.0"))
    sc.add_sink(2, 0, 0)
    sc.add_onoff(0, 2, 0, 1_000_000, remote_addr=sc.dev_addr[5])
    sc.stop(2_000_000)
    sc.route_bfs()
    R = oracle_table(sc)
    assert R[0, 0] == l1[0]  # 10.0.0.2 < 10.0.1.2
    assert np.array_equal(R, scenario_table(sc))
