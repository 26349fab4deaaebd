"""Reference test fixtures restated as p2p scenarios, on the oracle (CPU): DropTailQueueTestCase
(src/network/test/drop-tail-queue-test-suite.cc:37-78) and UdpClientServerTestCase
(src/applications/test/udp-client-server-test.cc:59-108).  tests/test_gpu_reference_fixtures.py runs the
same scenarios on the GPU engine."""
import numpy as np

import nsref
import p2p
import trace
from reference_fixtures import (check_drop_tail_trace, check_udp_client_server, drop_tail_queue_scenario,
                                udp_client_server_scenario)


def run(sc):
    s = sc.c_struct()
    st = p2p.P2PStats()
    devc = np.zeros(s.n_devices, p2p.DEV_COUNTERS_DTYPE)
    appc = np.zeros(s.n_apps, p2p.APP_COUNTERS_DTYPE)
    _secs, _log, tr = nsref.p2p_run_trace(s, st, devc, appc, 0)
    return st, devc, appc, trace.sort_records(tr)


def test_drop_tail_queue_fixture():
    _st, devc, _appc, tr = run(drop_tail_queue_scenario())
    check_drop_tail_trace(tr, devc)


def test_drop_tail_queue_fixture_larger_queue():
    _st, devc, _appc, tr = run(drop_tail_queue_scenario(n_packets=9, qmax=5))
    check_drop_tail_trace(tr, devc, n_packets=9, qmax=5)


def test_udp_client_server_fixture():
    _st, _devc, appc, _tr = run(udp_client_server_scenario())
    check_udp_client_server(appc)
