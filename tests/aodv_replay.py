"""The reference's Wi-Fi chain pcaps with a moving node as a PHY pin: src/aodv/test/aodv-chain-regression-test-{0..4}-0.pcap
and bug-606-test-{0..2}-0.pcap (tests/golden/aodv/, data files of the reference's test suite), written by
ChainRegressionTest (src/aodv/test/aodv-regression.cc:90-170): m_size nodes 120 m apart in a row
(GridPositionAllocator, ConstantPositionMobilityModel), 802.11a OFDM 6 Mb/s (ConstantRateWifiManager, RTS/CTS
above 2200 B: never here), YansWifiChannelHelper::Default (LogDistance n = 3, L0 46.6777 dB; ConstantSpeed),
YansWifiPhyHelper::Default with the YansErrorRateModel, AdhocWifiMac, AODV routing, a V4Ping from node 0 to the
last node, EnablePcapAll (DLT_IEEE802_11 MonitorSnifferTx / Rx files) — and at Time (m_time / 3) the central
node is moved to (1e5, 1e5, 1e5) (MobilityModel::SetPosition from a host closure), out of everyone's range.

Which record is a send: a frame's MonitorSnifferTx is at its SendPacket instant in the sender's file, and every
MonitorSnifferRx of it is in a receiver's file one transmission time (+ the 400-ns delay, so +0 or +1 us) later
with the same bytes — the records with no earlier twin are the sends (ACKs carry no transmitter address, so the
timing, not the address, decides).  Replaying those SendPacket calls (host closures at the recorded instants,
the move as a host closure at m_time / 3) on the closed-loop PHY must give every node exactly its file's
receptions at the recorded microseconds: after the move the central node hears nothing and is heard by no one,
and the chain is cut.  The sniffer codec then rebuilds each file byte for byte from the frames.  Sub-microsecond
send times: the smallest offset inside the recorded microsecond that gives every recorded reception microsecond
(ConstantSpeed delay Seconds (d / 3e8) through int64x64).  The host's m_random draws (AODV's, the MAC's, the
PHY's EndReceive) stay on the host; every EndReceive that succeeded in these files has PER < 0.5 and
every one that failed has PER > 0.5, so the replay's draw of 0.5 gives the same outcomes (checked)."""
import os

import numpy as np

import trace
import wifi

HERE = os.path.dirname(os.path.abspath(__file__))
OFDM6 = (wifi.OFDM, 6_000_000, 20_000_000)  # OfdmRate6Mbps
TX_DBM = 16.0206 + 1.0  # TxPowerStart + TxGain
FREQ_MHZ = 5000 + 5 * 36  # 802.11a channel 36
STEP = 120.0
CASES = {"aodv-chain-regression-test": (5, 10_000_000_000), "bug-606-test": (3, 10_000_000_000)}


def move_ts(m_time):
    """Time (m_time / 3): int64x64 division, then GetHigh (the ns floor)."""
    return m_time // 3


def golden(prefix):
    """{node: file bytes}, {node: records}, the sends [(us, node, frame)] in time order, the receptions
    {(node, send index, us)}."""
    n, _t = CASES[prefix]
    files = {i: open(os.path.join(HERE, "golden", "aodv", f"{prefix}-{i}-0.pcap"), "rb").read() for i in range(n)}
    recs = {i: trace.pcap_read(files[i])[1] for i in range(n)}
    import nsref
    allr = sorted((s * 10**6 + u, i, bytes(d)) for i in range(n) for s, u, _inc, _orig, d in recs[i])
    dur_us = lambda L: nsref.wifi_tx_duration(L, *OFDM6, wifi.PREAMBLE_LONG) // 1000  # noqa: E731
    sends, rx, seen = [], set(), {}
    for t, i, d in allr:
        src = [k for k in seen.get(d, []) if sends[k][1] != i and 0 <= t - sends[k][0] - dur_us(len(d)) <= 1]
        if src:
            rx.add((i, src[-1], t))
        else:
            seen.setdefault(d, []).append(len(sends))
            sends.append((t, i, d))
    return files, recs, sends, rx


def positions(n):
    return np.arange(n) * STEP, np.zeros(n), np.zeros(n)


def schedule(prefix, sends, rx):
    """Send times (ns): the smallest offset in the recorded microsecond that gives every reception's microsecond."""
    import nsref
    n, m_time = CASES[prefix]
    x, y, z = positions(n)
    mv = move_ts(m_time)
    out = []
    for k, (t, i, d) in enumerate(sends):
        dur = nsref.wifi_tx_duration(len(d), *OFDM6, wifi.PREAMBLE_LONG)
        mine = [(j, r) for (j, kk, r) in rx if kk == k]
        ok = []
        for f in range(1000):
            ts = t * 1000 + f
            px = x.copy()
            if ts >= mv:
                px[n // 2] = 1e5
            good = True
            for j, r in mine:
                dist = np.sqrt((px[i] - px[j]) ** 2 + (y[i] - y[j]) ** 2 + (z[i] - z[j]) ** 2)
                delay = nsref.seconds(float(dist) / 3e8)
                good &= (ts + dur + delay) // 1000 == r
            if good:
                ok.append(f)
                break
        assert ok, (k, t, i, mine)
        out.append(t * 1000 + ok[0])
    return np.array(out, np.uint64)


def phys(n):
    x, y, z = positions(n)
    return wifi.LoopPhys(x, y, z, error_model=wifi.YANS)


def moves(prefix):
    n, m_time = CASES[prefix]
    return [(move_ts(m_time), n // 2, (1e5, 1e5, 1e5))]


def oracle_replay(prefix):
    import nsref
    n, m_time = CASES[prefix]
    _files, _recs, sends, rx = golden(prefix)
    ts = schedule(prefix, sends, rx)
    phy = np.array([i for _t, i, _f in sends], np.uint32)
    size = np.array([len(f) for _t, _i, f in sends], np.uint32)
    ph = phys(n)
    return nsref.wifil_replay(ph.c_struct(), ts, phy, size, OFDM6, wifi.PREAMBLE_LONG, TX_DBM, m_time, n,
                              wifi.WIFIL_END_DTYPE, wifi.PHY_COUNTERS_DTYPE, moves=moves(prefix))


def gpu_replay(prefix):
    """The same sends and move on the device PHY behind the host-closure runtime."""
    import nsgpu
    n, m_time = CASES[prefix]
    _files, _recs, sends, rx = golden(prefix)
    ts = schedule(prefix, sends, rx)
    ph = phys(n)
    sim = nsgpu.Sim()
    lp = wifi.LoopPhy(ph)
    sim.attach_wifi(lp)
    sim.set_log(1 << 13)
    txs = []

    def send(i, size):
        txs.append((sim.now(), sim.current_uid(), i))
        sim.wifi_send(i, size, TX_DBM, OFDM6, wifi.PREAMBLE_LONG)

    for (t, i, frame), tn in zip(sends, ts):
        sim.schedule(int(tn), (lambda i=i, L=len(frame): lambda: send(i, L))())
    for mt, j, (mx, my, mz) in moves(prefix):
        sim.schedule(int(mt), (lambda j=j, p=(mx, my, mz): lambda: sim.wifi_set_position(j, *p))())
    sim.stop(m_time)
    sim.run()
    ends = lp.read_ends()
    k = min(sim.dispatched(), 1 << 13)
    log = (sim.log[0][:k].copy(), sim.log[1][:k].copy(), sim.log[2][:k].copy())
    tot = dict(dispatched=sim.dispatched(), next_uid=sim.next_uid(), txs=np.array(txs, np.uint64).reshape(-1, 3))
    return log, ends, lp.read_phys(), tot, (sim, lp)


def pcaps(prefix, ends, txs, frames):
    """Every node's DLT_IEEE802_11 file from a run's sniffer records (draw 0.5: see the module doc)."""
    n, _t = CASES[prefix]
    ok = [float(e["per"]) < 0.5 for e in ends]
    recs = wifi.sniff_records(txs, ends, ok, OFDM6, wifi.PREAMBLE_LONG, 7.0, FREQ_MHZ)
    return {i: wifi.sniff_pcap(wifi.DLT_IEEE802_11, recs, i, frames) for i in range(n)}
