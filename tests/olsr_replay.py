"""The reference's own Wi-Fi pcaps as a PHY pin: src/olsr/test/olsr-tc-regression-test-{0,1,2}-1.pcap
(tests/golden/olsr/, data files of the reference's test suite), written by TcRegressionTest
(src/olsr/test/tc-regression-test.cc:71-115): three nodes in a 120-m chain, 802.11a OFDM 6 Mb/s
(ConstantRateWifiManager), YansWifiChannelHelper::Default (LogDistance n = 3, L0 46.6777 dB; ConstantSpeed
delay), YansWifiPhyHelper::Default with the YansErrorRateModel, AdhocWifiMac, and
wifiPhy.EnablePcapAll: DLT_IEEE802_11 files of MonitorSnifferTx (every SendPacket) and MonitorSnifferRx
(every EndReceive whose draw passed) per node.

The frames a node sent are the records whose transmitter address is its own; their times are the
SendPacket instants (us).  Replaying those SendPacket calls on the closed-loop PHY (host closures scheduled
at setup, YansWifiPhy::SendPacket of the node's phy with the recorded frame length) must give every node
exactly the receptions its file holds, at the recorded microseconds — the hidden pair (0 and 2, 240 m
apart: below the -96 dBm energy-detection threshold at each other) never syncs — and the sniffer codec
(nsgpu_wifi_pcap) must then rebuild each file byte for byte from the frames.

Sub-microsecond send times: a file stores microseconds only.  A reception ends at send + duration +
ConstantSpeed delay (Seconds (120 / 3e8) = 399 ns through int64x64), so a frame received one microsecond
late was sent at >= 601 ns past its microsecond; the replay sends at +601 ns then, at +0 ns otherwise (the
receptions' microseconds are checked, not assumed: the offset is chosen from one receiver and every other
receiver of the frame must agree).  The host's m_random draws: every EndReceive here has PER <= 1.2e-5, so
any draw above that (the replay uses 0.5) passes — the outcome does not depend on the RNG."""
import os

import numpy as np

import trace
import wifi

HERE = os.path.dirname(os.path.abspath(__file__))
OFDM6 = (wifi.OFDM, 6_000_000, 20_000_000)  # OfdmRate6Mbps
TX_DBM = 16.0206 + 1.0  # TxPowerStart + TxGain (yans-wifi-phy.cc:517-521)
FREQ_MHZ = 5000 + 5 * 36  # WIFI_PHY_STANDARD_80211a: channel 36 (GetChannelFrequencyMhz, yans-wifi-phy.cc:383-386)
STOP_NS = 30_000_000_000
N = 3


def golden():
    """{node: file bytes}, the parsed records, each node's MAC, the sends (us, node, frame) in time order and the
    receptions {(node, sender, us)}."""
    files = {i: open(os.path.join(HERE, "golden", "olsr", f"olsr-tc-regression-test-{i}-1.pcap"), "rb").read()
             for i in range(N)}
    recs = {i: trace.pcap_read(files[i])[1] for i in range(N)}
    ta = lambda d: d[10:16]  # noqa: E731  (the frame's address 2)
    heard = [set(ta(r[4]) for r in recs[i]) for i in range(N)]
    # the chain's ends cannot hear each other: a node's own address is in its file and its neighbours' only
    mac = [None] * N
    mac[0] = (heard[0] - heard[2]).pop()
    mac[2] = (heard[2] - heard[0]).pop()
    mac[1] = (heard[1] - {mac[0], mac[2]}).pop()
    sends = sorted((s * 10**6 + u, i, bytes(d)) for i in range(N) for (s, u, _incl, _orig, d) in recs[i]
                   if ta(d) == mac[i])
    rx = {(i, mac.index(ta(d)), s * 10**6 + u) for i in range(N) for (s, u, _incl, _orig, d) in recs[i]
          if ta(d) != mac[i]}
    return files, recs, mac, sends, rx


def schedule(sends, rx):
    """Send times (ns) with the sub-microsecond part each frame's receptions imply (see the module doc)."""
    import nsref
    out = []
    for t, i, frame in sends:
        dur_us = nsref.wifi_tx_duration(len(frame), *OFDM6, wifi.PREAMBLE_LONG) // 1000
        late = {r - t - dur_us for (_j, src, r) in rx if src == i and 0 <= r - t - dur_us <= 1}
        assert len(late) <= 1, (t, i, late)  # every receiver of the frame agrees
        out.append(t * 1000 + (601 if late == {1} else 0))
    return np.array(out, np.uint64)


def phys():
    x = np.array([0.0, 120.0, 240.0])  # GridPositionAllocator, DeltaX = m_step (tc-regression-test.cc:78-86)
    return wifi.LoopPhys(x, np.zeros(N), np.zeros(N), error_model=wifi.YANS)


def oracle_replay():
    import nsref
    _files, _recs, _mac, sends, rx = golden()
    ts = schedule(sends, rx)
    phy = np.array([i for _t, i, _f in sends], np.uint32)
    size = np.array([len(f) for _t, _i, f in sends], np.uint32)
    ph = phys()
    log, ends, pc, tot = nsref.wifil_replay(ph.c_struct(), ts, phy, size, OFDM6, wifi.PREAMBLE_LONG, TX_DBM, STOP_NS,
                                            N, wifi.WIFIL_END_DTYPE, wifi.PHY_COUNTERS_DTYPE)
    return log, ends, pc, tot


def gpu_replay():
    """The same schedule on the device PHY behind the host-closure runtime (nsgpu_sim_attach_wifi)."""
    import nsgpu
    _files, _recs, _mac, sends, rx = golden()
    ts = schedule(sends, rx)
    ph = phys()
    sim = nsgpu.Sim()
    lp = wifi.LoopPhy(ph)
    sim.attach_wifi(lp)
    sim.set_log(1 << 12)
    txs = []

    def send(i, size):
        txs.append((sim.now(), sim.current_uid(), i))
        sim.wifi_send(i, size, TX_DBM, OFDM6, wifi.PREAMBLE_LONG)

    for (t, i, frame), tn in zip(sends, ts):
        sim.schedule(int(tn), (lambda i=i, L=len(frame): lambda: send(i, L))())
    sim.stop(STOP_NS)
    sim.run()
    ends = lp.read_ends()
    k = min(sim.dispatched(), 1 << 12)
    log = (sim.log[0][:k].copy(), sim.log[1][:k].copy(), sim.log[2][:k].copy())
    tot = dict(dispatched=sim.dispatched(), next_uid=sim.next_uid(), txs=np.array(txs, np.uint64).reshape(-1, 3))
    return log, ends, lp.read_phys(), tot, (sim, lp)


def pcaps(ends, txs, frames):
    """Every node's DLT_IEEE802_11 file from a run's sniffer records (draw 0.5: see the module doc)."""
    ok = [float(e["per"]) < 0.5 for e in ends]
    recs = wifi.sniff_records(txs, ends, ok, OFDM6, wifi.PREAMBLE_LONG, 7.0, FREQ_MHZ)
    return {i: wifi.sniff_pcap(wifi.DLT_IEEE802_11, recs, i, frames) for i in range(N)}, recs
