"""The reference's Wi-Fi chain pcaps with a node moved mid-run (src/aodv/test/aodv-chain-regression-test-{0..4}-0.pcap,
bug-606-test-{0..2}-0.pcap; tests/aodv_replay.py) rebuilt by the closed-loop oracle from the replayed sends and
the MobilityModel::SetPosition at m_time / 3: every node's file byte for byte.  No GPU."""
import numpy as np
import pytest

import aodv_replay as aodv


@pytest.mark.parametrize("prefix", sorted(aodv.CASES))
def test_oracle_rebuilds_the_chain_pcaps(prefix):
    files, _recs, sends, rx = aodv.golden(prefix)
    n, m_time = aodv.CASES[prefix]
    _log, ends, _phys, tot = aodv.oracle_replay(prefix)
    assert len(ends) == len(rx)  # (every EndReceive of the replay is a reception some file holds)
    per = ends["per"]
    assert ((per < 0.5) | (per > 0.5)).all() and (per < 1e-3).all()  # the draws cannot change an outcome
    out = aodv.pcaps(prefix, ends, tot["txs"], [f for _t, _i, f in sends])
    for i in range(n):
        assert out[i] == files[i], i
    # after the move the central node neither hears nor is heard
    mv = aodv.move_ts(m_time) // 1000
    c = n // 2
    assert not [1 for (j, k, r) in rx if r > mv + 1000 and (j == c or sends[k][1] == c)]
    later = [1 for (_j, k, _r) in rx if sends[k][0] > mv]
    assert bool(later) == (n > 3)  # 5 nodes: the neighbour pairs on either side keep talking; 3: nobody hears anyone
