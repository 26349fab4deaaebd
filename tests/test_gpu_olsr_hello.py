"""The reference's point-to-point HELLO pcaps replayed on the GPU-resident subset (tests/olsr_hello_replay.py):
the sends are host closures (nsgpu_sim_p2p_send) interleaved with the device's events; the pop log, trace
records and counters equal the oracle's, and every sniffer record's microsecond, length and order equal the
reference files' — which the library's pcap writer then rebuilds byte for byte."""
import numpy as np
import pytest

import olsr_hello_replay as hello

pytestmark = pytest.mark.gpu

FIELDS = ("ts", "uid", "seq", "kind", "dev", "app", "ipid", "size", "ttl")


def test_hello_pcaps_on_the_device():
    files, recs, _sends = hello.golden()
    sc, ost, odevc, oappc, olog, otr = hello.oracle_run()
    _sc, gtot, gdevc, gappc, glog, gtr, _keep = hello.gpu_run()
    assert gtot["dispatched"] == ost.dispatched and gtot["next_uid"] == ost.next_uid
    assert gtot["digest"] == ost.digest
    n = int(ost.dispatched)
    for a, b in zip(glog, olog):
        assert np.array_equal(a[:n], b[:n])
    assert np.array_equal(gdevc, odevc) and np.array_equal(gappc, oappc)
    assert len(gtr) == len(otr)
    for f in FIELDS:
        assert np.array_equal(gtr[f], otr[f]), f
    out = hello.rebuild(files, recs, hello.sniffer_records(sc, gtr))
    assert out[0] == files[0] and out[1] == files[1]
