"""GPU global-routing tables (nsgpu_route_global, csrc/nsgpu_route.hip) against the oracle's restatement
of GlobalRouteManagerImpl::SPFCalculate + Ipv4GlobalRouting::LookupGlobal (oracle/nsref_route.cc) and,
at config 4's full size (128 x 128, where the reference's own SPF takes hours: SURVEY H9), against the
grid's XY tables that the oracle proves equal to global routing up to 32 x 32 (test_routing_oracle.py)."""
import time

import numpy as np
import pytest

import nsgpu
import p2p
from routing_util import oracle_table, scenario_table

pytestmark = pytest.mark.gpu


def gpu_table(sc):
    n = len(sc.dev)
    dsts = sorted(sc.dst_slot, key=sc.dst_slot.get)
    return nsgpu.route_global([r[0] for r in sc.dev], [r[1] for r in sc.dev], [sc.dev_addr[i] for i in range(n)],
                              [sc.dev_ifindex[i] for i in range(n)], sc.n_nodes, dsts)


@pytest.fixture(scope="module", autouse=True)
def _dev():
    nsgpu.check(nsgpu.lib().nsgpu_set_device(0))


@pytest.mark.parametrize("seed", range(6))
def test_random_topologies_match_oracle_spf(seed):
    sc = p2p.random_topology(60, 150, 16, seed)
    assert np.array_equal(gpu_table(sc), oracle_table(sc))


@pytest.mark.parametrize("n", [2, 5, 16, 32])
def test_grids_match_oracle_spf(n):
    g = p2p.grid(n, n, flows=[(0, n * n - 1), (n * n - 1, 0), (n - 1, n * (n - 1)), (n // 2, n * n - 1 - n // 2)])
    assert np.array_equal(gpu_table(g), oracle_table(g))


def test_dumbbell_and_incast_match_oracle_spf():
    for sc in (p2p.dumbbell(40), p2p.incast(30), p2p.first_cc()):
        assert np.array_equal(gpu_table(sc), oracle_table(sc))


def test_grid_128x128_config4_tables():
    g = p2p.grid(128, 128)
    t0 = time.perf_counter()
    R = gpu_table(g)
    secs = time.perf_counter() - t0
    assert np.array_equal(R, scenario_table(g))
    print(f"128x128, {g.n_dst} destinations: {secs:.3f} s")


def test_grid_all_pairs_64x64():
    """Every node a destination (4,096 BFS in batches of 1,024): the dense all-pairs table of a 64 x 64 grid
    equals XY routing everywhere."""
    n = 64
    g = p2p.grid(n, n)
    nd = len(g.dev)
    R = nsgpu.route_global([r[0] for r in g.dev], [r[1] for r in g.dev], [g.dev_addr[i] for i in range(nd)],
                           [g.dev_ifindex[i] for i in range(nd)], g.n_nodes, np.arange(g.n_nodes))
    g2 = p2p.grid(n, n, flows=[(0, d) for d in range(n * n)])
    want = scenario_table(g2)
    assert np.array_equal(R, want)
