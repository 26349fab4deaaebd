"""ICMP errors on the GPU p2p engine vs the oracle: the full (ts, uid, context) pop
order, every counter (icmp_sent included) and the trace records / ascii / pcap bytes of runs where TTL
expiries and unbound arrivals send time-exceeded and port-unreachable errors back to the senders."""
import numpy as np
import pytest

import nsref
import p2p
import trace
from test_gpu_trace import assert_same_run, assert_same_trace, gpu_full, oracle_full
from test_icmp_oracle import icmp_scenario, line

pytestmark = pytest.mark.gpu


def check(sc, log_cap=400000):
    o = oracle_full(sc, log_cap)
    g = gpu_full(sc, log_cap, len(o[4]) + 16)
    assert o[0].icmp_sent > 0
    assert g[0].icmp_sent == o[0].icmp_sent
    assert g[0].unreach_drops == o[0].unreach_drops
    assert_same_run(sc, o, g)
    return o


@pytest.mark.parametrize("case", ["ttl1", "unreach", "reply_unreach", "reply_ttl"])
def test_line_known_answers(case):
    sc = {"ttl1": lambda: line(3, client_ttl=1), "unreach": lambda: line(3),
          "reply_unreach": lambda: line(3, server=True, client_stop_ns=2_001_000_000),
          "reply_ttl": lambda: line(70, client_ttl=255, server=True)}[case]()
    check(sc, 4096)


@pytest.mark.parametrize("seed", [1, 2, 5, 6, 7])
def test_random_topologies_icmp(seed):
    o = check(icmp_scenario(seed))
    assert o[0].ttl_drops > 0 and o[0].unreach_drops > 0


def test_grid_ttl_expiry_with_congestion():
    """Column flows at 3 Mb/s through 8 rows of 2 Mb/s links with TTL 5 and 6-packet queues: DropTail drops at
    every first hop and the time-exceeded errors travel back up the columns against the data."""
    g = p2p.grid(8, 8, bps=2_000_000, qmax=6, rate_bps=3_000_000, ttl=5, icmp=True, stop_ns=300_000_000,
                 sim_stop_ns=400_000_000)
    o = check(g, 200000)
    assert o[1]["drop_packets"].sum() > 0


@pytest.mark.parametrize("nranks", [2, 3])
def test_partitioned_icmp_trace_union(nranks):
    g = p2p.grid(6, 6, qmax=4, rate_bps=2_000_000, ttl=3, icmp=True, stop_ns=300_000_000, sim_stop_ns=400_000_000)
    otr = oracle_full(g, 0)[4]
    assert ((otr["app"] & trace.PKT_ICMP) != 0).sum() > 0
    grp = p2p.LoopbackGroup(g, nranks, trace_cap=len(otr) + 16)
    grp.run()
    assert_same_trace(g, otr, trace.sort_records(grp.trace()))


def test_icmp_off_matches_plain_run():
    """icmp=False leaves the engine's behaviour unchanged: the same scenario's TTL drops are silent."""
    sc = icmp_scenario(1, icmp=False)
    o = oracle_full(sc, 100000)
    g = gpu_full(sc, 100000, len(o[4]) + 16)
    assert g[0].icmp_sent == 0 and g[0].ttl_drops == o[0].ttl_drops > 0
    assert_same_run(sc, o, g)
    assert np.array_equal(g[1], o[1])


def test_payload_needing_fragmentation_is_refused():
    """SendRealOut would fragment a 1473-byte payload (1501-byte IPv4 datagram > Mtu 1500): refused loudly."""
    import nsgpu
    ok = line(3)
    ok.apps[-1]["size"] = 1472
    p2p.Engine(ok).run()
    big = line(3)
    big.apps[-1]["size"] = 1473
    with pytest.raises(nsgpu.NsgpuError, match="fragmentation"):
        p2p.Engine(big)


# ---------------------------------------------------------------- Ipv4L3Protocol Tx / Rx / Drop records
ALL = nsref.TRACE_DEVICE_KINDS | nsref.TRACE_IPV4_KINDS


def check_ipv4(sc, log_cap=200000):
    """The run with the Ipv4 sinks recorded too: every record (seq included) equals the oracle's."""
    o = oracle_full(sc, log_cap, ALL)
    assert (o[4]["kind"] == trace.TR_IP_DROP).sum() > 0
    g = gpu_full(sc, log_cap, len(o[4]) + 16, ALL)
    assert_same_run(sc, o, g)
    return o


@pytest.mark.parametrize("case", ["ttl1", "reply_ttl", "seed1", "seed2", "icmp_off"])
def test_ipv4_records(case):
    sc = {"ttl1": lambda: line(3, client_ttl=1), "reply_ttl": lambda: line(70, client_ttl=255, server=True),
          "seed1": lambda: icmp_scenario(1), "seed2": lambda: icmp_scenario(2),
          "icmp_off": lambda: icmp_scenario(5, icmp=False)}[case]()
    check_ipv4(sc)


def test_ipv4_records_congested_grid():
    g = p2p.grid(8, 8, bps=2_000_000, qmax=6, rate_bps=3_000_000, ttl=5, icmp=True, stop_ns=300_000_000,
                 sim_stop_ns=400_000_000)
    check_ipv4(g)


@pytest.mark.parametrize("ttl,icmp", [(1, False), (2, False), (2, True)])
def test_ipv4_records_dumbbell_router_hubs(ttl, icmp):
    """TTL expiries at the dumbbell's routers, which the engine runs as hub blocks: with ICMP off through
    the stateless IpForward lanes, with ICMP on through the serial node pass, the time-exceeded errors'
    device steps and the Drop records after them."""
    sc = p2p.dumbbell(300)
    for a in sc.apps:
        a["ttl"] = ttl
    if icmp:
        sc.icmp = True
        sc.route_bfs()
    o = check_ipv4(sc)
    assert o[0].ttl_drops > 0 and (o[0].icmp_sent > 0) == icmp


@pytest.mark.parametrize("nranks", [2, 3])
def test_partitioned_ipv4_trace_union(nranks):
    g = p2p.grid(6, 6, qmax=4, rate_bps=2_000_000, ttl=3, icmp=True, stop_ns=300_000_000, sim_stop_ns=400_000_000)
    otr = oracle_full(g, 0, ALL)[4]
    assert (otr["kind"] == trace.TR_IP_DROP).sum() > 0
    grp = p2p.LoopbackGroup(g, nranks, trace_cap=len(otr) + 16, trace_kinds=ALL)
    grp.run()
    assert_same_trace(g, otr, trace.sort_records(grp.trace()))
