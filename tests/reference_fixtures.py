"""Scenarios that restate reference test fixtures for the p2p engines (shared by the CPU oracle test and
the GPU test)."""
import p2p


def drop_tail_queue_scenario(n_packets=5, qmax=3):
    """src/network/test/drop-tail-queue-test-suite.cc:37-78 as a one-device scenario: a DropTailQueue with
    MaxPackets 3 behind a PointToPointNetDevice.  n_packets single-datagram OnOff flows (MaxBytes = one
    packet) on node 0 send at the same instant: the first goes straight to the idle transmitter
    (Enqueue + Dequeue, point-to-point-net-device.cc:494-509), the next three fill the queue (the test's p1..p3,
    NPackets 1, 2, 3), the fifth is dropped (its p4: NPackets stays 3), and the queue drains FIFO."""
    sc = p2p.Scenario(2)
    da, db = sc.link(0, 1, 10_000_000, 1_000_000, qmax=qmax)
    sc.install_stack()
    sc.assign_link(da, db, p2p.ip("10.1.1.0"))
    sc.add_sink(1, 0, 0)
    for _ in range(n_packets):
        sc.add_onoff(0, 1, 1_000_000_000, 2_000_000_000, rate_bps=1_000_000, size=100, on_s=1.0, off_s=0.0,
                     max_bytes=100, remote_addr=sc.dev_addr[db])
    sc.stop(3_000_000_000)
    sc.route_bfs()
    return sc


def check_drop_tail_trace(tr, devc, n_packets=5, qmax=3):
    """The queue calls of device 0 in trace order: what DropTailQueueTestCase asserts, as sink calls."""
    import trace
    calls = [(int(r["kind"]), int(r["app"])) for r in tr if int(r["dev"]) == 0]
    E, D, X = trace.TR_ENQUEUE, trace.TR_DEQUEUE, trace.TR_DROP
    first = 1  # app 0 is the PacketSink; the flows are apps 1..n
    want = [(E, first), (D, first)]                                   # straight to the transmitter
    want += [(E, first + i) for i in range(1, qmax + 1)]              # p1..p3: NPackets 1, 2, 3
    want += [(X, first + i) for i in range(qmax + 1, n_packets)]      # p4: dropped, NPackets still 3
    want += [(D, first + i) for i in range(1, qmax + 1)]              # Dequeue: p1, p2, p3 (FIFO)
    assert calls == want, calls
    assert devc[0]["enq_packets"] == qmax + 1 and devc[0]["drop_packets"] == n_packets - qmax - 1
    assert devc[0]["deq_packets"] == qmax + 1 and devc[1]["rx_packets"] == qmax + 1


def udp_client_server_scenario():
    """src/applications/test/udp-client-server-test.cc:59-108 (UdpClientServerTestCase) on the GPU-resident
    applications: two nodes, 10.1.1.0/24, a server on node 1 (port 4000, 1-10 s) and a client on node 0 (MaxPackets
    10, Interval 1 s, PacketSize 1024, 2-10 s).  The GPU subset has UdpEchoClient/UdpEchoServer, whose send schedule
    is UdpClient's (udp-client.cc: Send at Seconds (0) after start, then every Interval while m_sent < m_count;
    StopApplication cancels m_sendEvent); the link is a PointToPointNetDevice pair instead of SimpleNetDevice.
    The test's expected counts: the server receives 8 datagrams (2 s .. 9 s; Stop at 10 s precedes the 10 s Send)
    and loses none."""
    sc = p2p.Scenario(2)
    da, db = sc.link(0, 1, 5_000_000, 2_000_000)
    sc.install_stack()
    sc.assign_link(da, db, p2p.ip("10.1.1.0"))
    sc.add_echo_server(1, 1_000_000_000, 10_000_000_000, port=4000)
    sc.add_echo_client(0, 1, 2_000_000_000, 10_000_000_000, count=10, interval_ns=1_000_000_000, size=1024,
                       remote_addr=sc.dev_addr[db], remote_port=4000)
    sc.route_bfs()
    return sc


def check_udp_client_server(appc):
    server, client = appc[0], appc[1]
    assert server["rx_packets"] == 8  # GetReceived () == 8
    assert client["tx_packets"] == 8 and server["rx_packets"] == client["tx_packets"]  # GetLost () == 0
    assert client["rx_packets"] == 8  # every echo came back
