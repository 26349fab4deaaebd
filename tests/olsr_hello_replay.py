"""The reference's point-to-point pcaps as a device-timing pin: src/olsr/test/olsr-hello-regression-test-{0,1}-1.pcap
(tests/golden/olsr/, data files of the reference's test suite), written by HelloRegressionTest
(src/olsr/test/hello-regression-test.cc:66-87): two nodes, InternetStackHelper (OLSR routing: each node's
LoopbackNetDevice is its device 0), PointToPointHelper 5 Mb/s / 2 ms, 10.1.1.0/24, EnablePcapAll (the
PromiscSniffer: a device's Dequeue -> TransmitStart and its MacRx, point-to-point-helper.cc:81-110), Stop 5 s.

Each file holds the OLSR HELLOs (UDP broadcast, port 698) a node sent and received: 50- and 58-byte frames.
A node's sends are the records whose IPv4 source is its address; their instants are the send times (us).
Replaying those datagrams as host-closure UdpSocket::Sends on the GPU-resident point-to-point subset (one
OnOff flow per (node, payload size) that never starts by itself, a PacketSink on port 698 each side) must give
every device's sniffer exactly the file's records: the same microseconds (transmission time Seconds (bytes x 8 /
5e6) through int64x64, the 2 ms channel delay), lengths and order — the bytes then follow from the file.
OLSR itself (its timers' jitter draws, the HELLO contents) stays on the host; its events are not
modelled, so the run's uids are not the reference's (the pcap does not carry them).

Sub-microsecond send times: a receiver's microsecond is floor ((send + txTime + 2 ms) / 1 us); the replay sends
each datagram at the smallest nanosecond offset inside its recorded microsecond that gives the recorded reception
microsecond (a 58-byte frame's 92.8 us transmission makes it +200..999 ns or +0..199 ns)."""
import os

import numpy as np

import p2p
import trace

HERE = os.path.dirname(os.path.abspath(__file__))
BPS, DELAY_NS, PORT, STOP_NS = 5_000_000, 2_000_000, 698, 5_000_000_000
ADDR = (p2p.ip("10.1.1.1"), p2p.ip("10.1.1.2"))  # Ipv4AddressHelper::Assign: node 0's device first


def golden():
    """{node: file bytes}, {node: parsed records}, and the sends [(us, node, frame length)] in time order with
    each one's reception microsecond at the peer."""
    files = {i: open(os.path.join(HERE, "golden", "olsr", f"olsr-hello-regression-test-{i}-1.pcap"), "rb").read()
             for i in range(2)}
    recs = {i: trace.pcap_read(files[i])[1] for i in range(2)}
    src = lambda d: int.from_bytes(d[14:18], "big")  # noqa: E731  (PPP 2 + the IPv4 source at 12)
    sends = []
    for i in range(2):
        mine = [(s * 10**6 + u, orig, d) for s, u, _incl, orig, d in recs[i] if src(d) == ADDR[i]]
        theirs = [(s * 10**6 + u, orig, d) for s, u, _incl, orig, d in recs[1 - i] if src(d) == ADDR[i]]
        assert len(mine) == len(theirs)
        for (t, L, d), (r, L2, d2) in zip(mine, theirs):
            assert L == L2 and d == d2
            sends.append((t, i, L, r))
    return files, recs, sorted(sends)


def schedule(sends):
    """Send times (ns) with the sub-microsecond offset each reception implies (see the module doc)."""
    import nsref
    out = []
    for t, _i, L, r in sends:
        tx = nsref.seconds(L * 8 / BPS)  # PointToPointNetDevice::TransmitStart: Seconds (CalculateTxTime)
        f = [f for f in range(1000) if (t * 1000 + f + tx + DELAY_NS) // 1000 == r]
        assert f, (t, L, r)
        out.append(t * 1000 + f[0])
    return np.array(out, np.int64)


def scenario(sends):
    """The two nodes as HelloRegressionTest builds them, plus the datagrams' stand-in applications: returns
    (scenario, application of each send)."""
    sc = p2p.Scenario(2)
    sc.install_stack()  # internet.Install (c) before p2p.Install: the loopback is device 0
    da, db = sc.link(0, 1, BPS, DELAY_NS)
    sc.assign_link(da, db, p2p.ip("10.1.1.0"))
    for n in range(2):
        sc.add_sink(n, 0, 0, port=PORT)
    flows = {}
    apps = []
    for _t, i, L, _r in sends:
        key = (i, L)
        if key not in flows:  # (never started by itself: StartTime after the Stop)
            flows[key] = sc.add_onoff(i, 1 - i, STOP_NS + 1, 0, size=L - 2 - 28, remote_addr=ADDR[1 - i],
                                      remote_port=PORT)
        apps.append(flows[key])
    sc.stop(STOP_NS)
    sc.route_bfs()
    return sc, np.array(apps, np.uint32)


def oracle_run(log_cap=1024):
    import nsref
    _files, _recs, sends = golden()
    sc, apps = scenario(sends)
    s = sc.c_struct()
    st = p2p.P2PStats()
    devc = np.zeros(s.n_devices, p2p.DEV_COUNTERS_DTYPE)
    appc = np.zeros(s.n_apps, p2p.APP_COUNTERS_DTYPE)
    log, tr = nsref.p2p_run_sends(s, st, devc, appc, schedule(sends), apps, log_cap)
    return sc, st, devc, appc, log, trace.sort_records(tr)


def gpu_run(log_cap=1024):
    """The same sends as host closures on the runtime with the device subset attached (nsgpu_sim_p2p_send)."""
    import nsgpu
    _files, _recs, sends = golden()
    sc, apps = scenario(sends)
    eng = p2p.Engine(sc, log_cap=log_cap)
    eng.set_trace(1024)
    eng.reset()
    sim = nsgpu.Sim()
    sim.attach_p2p(eng)
    sim.set_log(log_cap)
    for t, a in zip(schedule(sends), apps):
        sim.schedule(int(t), (lambda a=int(a): lambda: sim.p2p_send(a))())
    sim.run()
    st, devc, appc, (lts, luid, lctx) = eng.results(log_n=log_cap)
    _host_n, _host_c, host_d = sim.host_stats()
    m = sim.log[1] != 0  # the host dispatches' ranks (the device's are in the engine's log)
    lts, luid, lctx = lts.copy(), luid.copy(), lctx.copy()
    lts[m], luid[m], lctx[m] = sim.log[0][m], sim.log[1][m], sim.log[2][m]
    tot = dict(dispatched=sim.dispatched(), next_uid=sim.next_uid(),
               digest=(int(st.digest) + host_d) & ((1 << 64) - 1))
    return sc, tot, devc, appc, (lts, luid, lctx), trace.sort_records(eng.trace()), (sim, eng)


def sniffer_records(sc, tr):
    """{node: [(us, length)]}: a device's PromiscSniffer calls (its Dequeues and MacRxs) in trace order."""
    out = {0: [], 1: []}
    for r in tr:
        if r["kind"] in (trace.TR_DEQUEUE, trace.TR_RX):
            n = sc.dev[int(r["dev"])][0]
            L = int(r["size"]) + (2 if r["kind"] == trace.TR_RX else 0)  # (MacRx's packet has no PPP header)
            out[n].append((int(r["ts"]) // 1000, L))
    return out


def rebuild(files, recs, sniff):
    """Each node's file from the run's sniffer records (time, length, order) and the file's own bytes (the
    OLSR payloads are the host's), written by the library's pcap writer (nsgpu_pcap_file)."""
    out = {}
    for n in range(2):
        assert [(s * 10**6 + u, orig) for s, u, _i, orig, _d in recs[n]] == sniff[n], n
        rows = [(us // 10**6, us % 10**6, d, L) for (us, L), (_s, _u, _i, _o, d) in zip(sniff[n], recs[n])]
        out[n] = p2p.pcap_file(trace.DLT_PPP, 65535, rows)
    return out
