"""Wi-Fi sniffer traces (config 3's traces; include/nsgpu.h nsgpu_wifi_*) pinned by the reference's own pcaps,
no GPU: the closed-loop oracle replays TcRegressionTest's transmissions and the library's codec rebuilds
the three golden files byte for byte (tests/olsr_replay.py); the radiotap variant and the ascii lines
against known answers restated from radiotap-header.cc:69-138,231-380 and yans-wifi-helper.cc:42-88."""
import math
import struct

import numpy as np

import olsr_replay as olsr
import wifi


def test_olsr_golden_structure():
    files, recs, mac, sends, rx = olsr.golden()
    assert [len(recs[i]) for i in range(3)] == [21, 31, 21]
    assert len(sends) == 31 and len(rx) == 42
    # the hidden pair: nodes 0 and 2 only ever hear node 1
    assert {src for (j, src, _t) in rx if j in (0, 2)} == {1}


def test_olsr_replay_receptions_match_the_reference():
    _files, _recs, _mac, sends, rx = olsr.golden()
    _log, ends, pc, tot = olsr.oracle_replay()
    assert tot["sends"] == 31
    phy_of = [i for _t, i, _f in sends]
    got = {(int(e["phy"]), phy_of[int(e["tx"])], int(e["ts"]) // 1000) for e in ends if not e["flags"]}
    assert got == rx
    assert float(ends["per"].max()) < 1.2e-5  # (the draw-independence the module doc relies on)
    # 0 and 2 receive each other's frames below the energy-detection threshold: no sync (drop_ed)
    assert int(pc["drop_ed"][0]) == sum(1 for _t, i, _f in sends if i == 2)
    assert int(pc["drop_ed"][2]) == sum(1 for _t, i, _f in sends if i == 0)


def test_olsr_pcaps_rebuilt_byte_for_byte():
    files, _recs, _mac, sends, _rx = olsr.golden()
    _log, ends, _pc, tot = olsr.oracle_replay()
    out, recs = olsr.pcaps(ends, tot["txs"], [f for _t, _i, f in sends])
    for i in range(3):
        assert out[i] == files[i], i


def test_radiotap_known_answer():
    """PcapSniffTxEvent / PcapSniffRxEvent with DLT_IEEE802_11_RADIO: RadiotapHeader (little-endian fields after
    the 8-byte header, in bit order) then the frame."""
    frame = bytes(range(20))
    recs = np.zeros(2, wifi.WIFI_SNIFF_DTYPE)
    recs[0] = (1_234_567_891, 0, 0, 0, 2, 2412, 0, 0.0, 0.0)         # Tx, 1 Mb/s DSSS at 2.412 GHz
    recs[1] = (2_000_000_500, 0, 0, 1, 12, 5180, 1, -61.5, -93.49)   # Rx, 6 Mb/s OFDM at 5.18 GHz, short preamble
    f = wifi.sniff_pcap(wifi.DLT_IEEE802_11_RADIO, recs, 0, [frame])
    assert struct.unpack_from("<IHHiIII", f, 0) == (0xa1b2c3d4, 2, 4, 0, 0, 65535, 127)
    off = 24
    sec, usec, incl, orig = struct.unpack_from("<IIII", f, off)
    assert (sec, usec, incl, orig) == (1, 234567, 22 + 20, 22 + 20)
    tx = f[off + 16:off + 16 + 22]
    assert tx == struct.pack("<BBHIQBBHH", 0, 0, 22, 0x0f, 1234567, 0x10, 2, 2412, 0x0020 | 0x0080)
    assert f[off + 16 + 22:off + 16 + 42] == frame
    off += 16 + 42
    sec, usec, incl, orig = struct.unpack_from("<IIII", f, off)
    assert (sec, usec, incl, orig) == (2, 0, 24 + 20, 24 + 20)
    rx = f[off + 16:off + 16 + 24]
    # signal floor (-61.5 + 0.5) = -61, noise floor (-93.49 + 0.5) = -93 (radiotap-header.cc:327-380)
    assert rx == struct.pack("<BBHIQBBHHbb", 0, 0, 24, 0x6f, 2000000, 0x10 | 0x02, 12, 5180, 0x0040 | 0x0100, -61, -93)


def test_sniff_power_formula():
    """signalDbm = RatioToDb (rxPowerW) + 30, noiseDbm = RatioToDb (rxPowerW / snr) - RxNoiseFigure + 30."""
    e = np.zeros(1, wifi.WIFIL_END_DTYPE)[0]
    e["rx_w"], e["snr"] = 7.9e-13, 3.25
    s, n = wifi.sniff_power(e, 7.0)
    assert s == 10.0 * math.log10(7.9e-13) + 30
    assert n == 10.0 * math.log10(7.9e-13 / 3.25) - 7.0 + 30


def test_ascii_lines():
    recs = np.zeros(2, wifi.WIFI_SNIFF_DTYPE)
    recs[0] = (1_500_000_000, 1, 0, 0, 2, 2412, 0, 0.0, 0.0)
    recs[1] = (1_500_900_000, 0, 0, 1, 2, 2412, 0, -80.0, -94.0)
    text = wifi.sniff_ascii(recs, [5, 6], [1, 1], ["ns3::WifiMacHeader (DATA) Payload (size=100)"])
    assert text == ("t 1.5 /NodeList/6/DeviceList/1/$ns3::WifiNetDevice/Phy/State/Tx ns3::WifiMacHeader (DATA) Payload (size=100)\n"
                    "r 1.5009 /NodeList/5/DeviceList/1/$ns3::WifiNetDevice/Phy/State/RxOk ns3::WifiMacHeader (DATA) Payload (size=100)\n")
