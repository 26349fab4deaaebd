"""Reference test fixtures on the GPU p2p engine (see tests/test_reference_fixtures_oracle.py): the
DropTailQueue sanity test and UdpClientServerTestCase's expected counts, plus the full trace against the
oracle's."""
import numpy as np
import pytest

import p2p
import trace
from reference_fixtures import (check_drop_tail_trace, check_udp_client_server, drop_tail_queue_scenario,
                                udp_client_server_scenario)
from test_reference_fixtures_oracle import run as oracle_run

pytestmark = pytest.mark.gpu
FIELDS = ("ts", "uid", "seq", "kind", "dev", "app", "ipid", "size", "ttl")


def same_trace(a, b):
    return len(a) == len(b) and all(np.array_equal(a[f], b[f]) for f in FIELDS)


def gpu_run(sc):
    eng = p2p.Engine(sc)
    eng.set_trace(4096)
    st, devc, appc, _log = eng.run()
    return st, devc, appc, trace.sort_records(eng.trace())


@pytest.mark.parametrize("n,q", [(5, 3), (9, 5)])
def test_drop_tail_queue_fixture_gpu(n, q):
    sc = drop_tail_queue_scenario(n_packets=n, qmax=q)
    st, devc, appc, tr = gpu_run(sc)
    check_drop_tail_trace(tr, devc, n_packets=n, qmax=q)
    ost, odevc, oappc, otr = oracle_run(sc)
    assert st.digest == ost.digest and np.array_equal(devc, odevc) and np.array_equal(appc, oappc)
    assert same_trace(tr, otr)


def test_udp_client_server_fixture_gpu():
    sc = udp_client_server_scenario()
    st, devc, appc, tr = gpu_run(sc)
    check_udp_client_server(appc)
    ost, odevc, oappc, otr = oracle_run(sc)
    assert st.digest == ost.digest and st.dispatched == ost.dispatched and np.array_equal(appc, oappc)
    assert same_trace(tr, otr)
