"""Wi-Fi sniffer traces of the GPU-resident closed-loop PHY (config 3's traces): the device's EndReceive
records feed the same codec as the oracle's (include/nsgpu.h nsgpu_wifi_*).

  * TcRegressionTest replayed on the device (tests/olsr_replay.py): the same receptions as the oracle,
    and the three reference pcaps rebuilt byte for byte from the device run;
  * the closed-loop grid of tests/wifi_loop_harness.py (6x6): every phy's pcap file (DLT_IEEE802_11 and the
    radiotap variant, whose signal / noise bytes come from the device's rxPowerW and SNR) and the ascii
    lines equal the oracle's."""
import numpy as np
import pytest

import olsr_replay as olsr
import wifi
from wifi_loop_harness import run_gpu, run_oracle, scenario

pytestmark = pytest.mark.gpu


def same_ends(g, o):
    for f in ("ts", "uid", "phy", "tx", "flags"):
        assert np.array_equal(g[f], o[f]), f
    np.testing.assert_allclose(g["snr"], o["snr"], rtol=1e-9, atol=0)
    np.testing.assert_allclose(g["per"], o["per"], rtol=1e-9, atol=1e-15)
    np.testing.assert_allclose(g["rx_w"], o["rx_w"], rtol=1e-9, atol=0)


def test_olsr_replay_on_the_device_rebuilds_the_reference_pcaps():
    files, _recs, _mac, sends, _rx = olsr.golden()
    olog, oends, _ophys, otot = olsr.oracle_replay()
    glog, gends, _gphys, gtot, _keep = olsr.gpu_replay()
    assert gtot["dispatched"] == otot["dispatched"] and gtot["next_uid"] == otot["next_uid"]
    for a, b in zip(glog, olog):
        assert np.array_equal(a, b)
    same_ends(gends, oends)
    assert np.array_equal(gtot["txs"], otot["txs"])
    out, _recs = olsr.pcaps(gends, gtot["txs"], [f for _t, _i, f in sends])
    for i in range(3):
        assert out[i] == files[i], i


def draw_ok(ends):
    """The harness's m_random stand-in (wifi_loop_harness.draws): phy j's k-th draw is a fixed value."""
    k = {}
    ok = []
    for e in ends:
        if e["flags"] & wifi.END_CANCELLED:
            ok.append(False)
            continue
        j = int(e["phy"])
        k[j] = k.get(j, 0) + 1
        u = (k[j] * 0.6180339887498949 + j * 0.1) % 1.0
        ok.append(u > float(e["per"]))
    return ok


def test_closed_loop_grid_sniffer_traces_equal_the_oracle():
    sc = scenario(n_side=6, spacing=60.0, seed=3, period=12_000_000, stop_ns=150_000_000, size=600)
    _olog, oends, _ophys, otot = run_oracle(sc)
    _glog, gends, _gphys, gtot, _keep = run_gpu(sc)
    same_ends(gends, oends)
    assert np.array_equal(gtot["txs"], otot["txs"])
    n = sc["phys"].n_phy
    freq = 2407 + 5 * 1  # 802.11b channel 1 (the harness's DSSS 1 Mb/s)
    orecs = wifi.sniff_records(otot["txs"], oends, draw_ok(oends), sc["mode"], sc["preamble"], 7.0, freq)
    grecs = wifi.sniff_records(gtot["txs"], gends, draw_ok(gends), sc["mode"], sc["preamble"], 7.0, freq)
    assert len(grecs) == len(orecs) and (grecs["kind"] == 1).sum() > 100
    # the host MAC's frames: synthetic bytes per transmission (the device keeps sizes only)
    frames = [bytes([(k * 7 + b) & 255 for b in range(sc["size"])]) for k in range(len(otot["txs"]))]
    for j in range(n):
        for dlt in (wifi.DLT_IEEE802_11, wifi.DLT_IEEE802_11_RADIO):
            assert wifi.sniff_pcap(dlt, grecs, j, frames) == wifi.sniff_pcap(dlt, orecs, j, frames), (j, dlt)
    texts = [f"ns3::WifiMacHeader (DATA, tx {k}) Payload (size={sc['size']})" for k in range(len(frames))]
    nodes, devs = np.arange(n), np.ones(n)
    assert wifi.sniff_ascii(grecs, nodes, devs, texts) == wifi.sniff_ascii(orecs, nodes, devs, texts)


@pytest.mark.parametrize("prefix", ["aodv-chain-regression-test", "bug-606-test"])
def test_aodv_chain_with_a_moving_node_on_the_device(prefix):
    """ChainRegressionTest's sends replayed on the device PHY with the central node moved by a host closure at
    m_time / 3 (nsgpu_sim_wifi_set_position): pop log, EndReceive records and the reference files byte for byte."""
    import aodv_replay as aodv
    files, _recs, sends, _rx = aodv.golden(prefix)
    olog, oends, _ophys, otot = aodv.oracle_replay(prefix)
    glog, gends, _gphys, gtot, _keep = aodv.gpu_replay(prefix)
    assert gtot["dispatched"] == otot["dispatched"] and gtot["next_uid"] == otot["next_uid"]
    for a, b in zip(glog, olog):
        assert np.array_equal(a, b)
    same_ends(gends, oends)
    assert np.array_equal(gtot["txs"], otot["txs"])
    out = aodv.pcaps(prefix, gends, gtot["txs"], [f for _t, _i, f in sends])
    for i in range(len(files)):
        assert out[i] == files[i], i
