"""Point-to-point scenarios for the GPU-resident p2p subset (include/nsgpu_types.h: nsgpu_p2p_scenario).

Host-side plumbing only: builds the plain arrays ns-3's helpers would produce (creation order of
nodes, devices and applications, which fixes the setup-time uids) and drives the C-ABI
(nsgpu_p2p_*).  No simulation logic lives here.

Builders mirror the reference helpers:
  * grid(): PointToPointGridHelper (src/point-to-point-layout/model/point-to-point-grid.cc:33-72):
    node (y, x) is created row by row; after each node its row link (x-1 -> x) then its column link
    ((y-1, x) -> (y, x)) are installed with PointToPointHelper::Install (point-to-point-helper.cc:228-242),
    which adds device A then device B.
  * Routes are harness-computed static next-hop tables (global routing is infeasible at
    128x128 on the reference CPU): XY routing on grids, BFS shortest paths otherwise.
"""
import ctypes as C
from collections import deque

import numpy as np

import nsgpu

# nsgpu_trace_record (include/nsgpu_types.h): one ascii trace sink call
TRACE_DEVICE_KINDS, TRACE_IPV4_KINDS = 0x0F, 0x70  # nsgpu_trace_kind bits: the device sinks, Ipv4L3Protocol's
TRACE_RECORD_DTYPE = np.dtype([("ts", "<u8"), ("uid", "<u4"), ("seq", "<u2"), ("kind", "u1"), ("pad_", "u1"),
                               ("dev", "<u4"), ("app", "<u4"), ("ipid", "<u4"), ("size", "<u4"),
                               ("ttl", "<u4"), ("pad2_", "<u4")])

APP_ONOFF, APP_SINK, APP_ECHO_CLIENT, APP_ECHO_SERVER = 0, 1, 2, 3
SENDERS = (APP_ONOFF, APP_ECHO_CLIENT)  # applications that originate datagrams towards app["dst"]
SETUP_NODE, SETUP_DEVICE, SETUP_APP, SETUP_STOP, SETUP_UID, SETUP_NOOP = 0, 1, 2, 3, 4, 5
NO_ROUTE = 0xFFFFFFFF


class ScenarioStruct(C.Structure):
    _fields_ = [
        ("n_nodes", C.c_uint32), ("n_devices", C.c_uint32), ("n_apps", C.c_uint32), ("n_dst", C.c_uint32),
        ("dev_node", C.c_void_p), ("dev_peer", C.c_void_p), ("dev_bps", C.c_void_p), ("dev_ifg_ns", C.c_void_p),
        ("dev_delay_ns", C.c_void_p), ("dev_qmax", C.c_void_p), ("route", C.c_void_p),
        ("app_kind", C.c_void_p), ("app_node", C.c_void_p), ("app_start_ns", C.c_void_p),
        ("app_stop_ns", C.c_void_p), ("app_dst_node", C.c_void_p), ("app_dst_slot", C.c_void_p),
        ("app_rate_bps", C.c_void_p), ("app_pkt_size", C.c_void_p), ("app_on_s", C.c_void_p),
        ("app_off_s", C.c_void_p), ("app_max_bytes", C.c_void_p), ("app_ttl", C.c_void_p),
        ("stop_ns", C.c_int64), ("n_setup", C.c_uint32), ("icmp", C.c_uint32),
        ("setup_kind", C.c_void_p), ("setup_index", C.c_void_p),
        ("app_count", C.c_void_p), ("app_interval_ns", C.c_void_p), ("app_src_slot", C.c_void_p),
        ("route_default", C.c_void_p), ("route_exc_off", C.c_void_p), ("route_exc_slot", C.c_void_p),
        ("route_exc_dev", C.c_void_p), ("uid_first", C.c_uint32), ("pad_uid_", C.c_uint32),
    ]


class P2PStats(C.Structure):
    _fields_ = [("dispatched", C.c_uint64), ("cancelled", C.c_uint64), ("digest", C.c_uint64),
                ("final_ts", C.c_uint64), ("next_uid", C.c_uint32), ("windows", C.c_uint32),
                ("ttl_drops", C.c_uint64), ("no_route_drops", C.c_uint64), ("max_window", C.c_uint64),
                ("unreach_drops", C.c_uint64), ("refits", C.c_uint64), ("icmp_sent", C.c_uint64)]


DEV_COUNTERS_DTYPE = np.dtype([("enq_packets", "<u4"), ("enq_bytes", "<u4"), ("drop_packets", "<u4"),
                               ("drop_bytes", "<u4"), ("deq_packets", "<u4"), ("tx_packets", "<u4"),
                               ("rx_packets", "<u4"), ("pad_", "<u4")])
APP_COUNTERS_DTYPE = np.dtype([("tx_packets", "<u4"), ("rx_packets", "<u4"), ("tx_bytes", "<u8"),
                               ("rx_bytes", "<u8")])


class Scenario:
    """Arrays of a nsgpu_p2p_scenario plus the order of setup-time Schedule calls."""

    def __init__(self, n_nodes, icmp=False):
        self.icmp = icmp  # ICMP errors generated and routed back to senders (nsgpu_p2p_scenario.icmp)
        self.uid_first = 0  # m_uid before the first setup call (0: 4, DefaultSimulatorImpl's start)
        self.n_nodes = 0
        self.dev = []     # (node, peer, bps, ifg, delay, qmax)
        self.apps = []    # dicts
        self.setup = []   # (kind, index)
        self.stop_ns = -1
        self.route = None
        self.route_c = None  # compressed next hops: (default[n], exc_off[n+1], exc_slot, exc_dev)
        self.n_dst = 0
        self.dst_slot = {}
        # addressing (host side only: the trace codec prints it, the engines never read it)
        self.dev_addr = {}   # device -> IPv4 address (u32) of its interface
        self.dev_mask = {}   # device -> network mask (u32)
        self.dev_ifindex = {}  # device -> Ipv4 interface index (loopback 0, then Assign order per node)
        self._nif = {}
        for _ in range(n_nodes):
            self.add_node()

    def add_node(self):
        # the first Node creates the NodeListPriv singleton: ScheduleDestroy (&NodeListPriv::Delete)
        # consumes a uid (node-list.cc:80-90), then NodeListPriv::Add schedules Node::Start (:124-131)
        if self.n_nodes == 0:
            self.setup.append((SETUP_UID, 0))
        self.setup.append((SETUP_NODE, self.n_nodes))
        self.n_nodes += 1
        return self.n_nodes - 1

    def install_stack(self):
        # InternetStackHelper::Install: Ipv4L3Protocol::SetupLoopback adds a LoopbackNetDevice to each
        # node (ipv4-l3-protocol.cc:227-244) -> Node::AddDevice -> ScheduleWithContext (node, 0, Start)
        for n in range(self.n_nodes):
            self.setup.append((SETUP_NOOP, n))

    # PointToPointHelper::Install (a, b): device on a, then device on b, one channel
    def link(self, a, b, bps, delay_ns, qmax=100, ifg_ns=0):
        da, db = len(self.dev), len(self.dev) + 1
        self.dev.append([a, db, bps, ifg_ns, delay_ns, qmax])
        self.setup.append((SETUP_DEVICE, da))
        self.dev.append([b, da, bps, ifg_ns, delay_ns, qmax])
        self.setup.append((SETUP_DEVICE, db))
        if da == 0:  # the first channel creates the ChannelListPriv singleton: ScheduleDestroy (channel-list.cc:80-90)
            self.setup.append((SETUP_UID, 0))
        return da, db

    def _app(self, **kw):
        a = dict(dst=0, rate=0, size=0, on=0.0, off=0.0, maxb=0, ttl=64, count=0, interval=0, port=0,
                 remote_addr=None, remote_port=0)
        a.update(kw)
        self.apps.append(a)
        self.setup.append((SETUP_APP, len(self.apps) - 1))  # Node::AddApplication
        return len(self.apps) - 1

    def add_sink(self, node, start_ns, stop_ns, port=9):
        return self._app(kind=APP_SINK, node=node, start=start_ns, stop=stop_ns, port=port, ttl=0)

    def add_onoff(self, node, dst, start_ns, stop_ns, rate_bps=500000, size=512, on_s=1.0, off_s=1.0,
                  max_bytes=0, ttl=64, remote_addr=None, remote_port=9):
        return self._app(kind=APP_ONOFF, node=node, start=start_ns, stop=stop_ns, dst=dst, rate=rate_bps, size=size,
                         on=on_s, off=off_s, maxb=max_bytes, ttl=ttl, remote_addr=remote_addr, remote_port=remote_port)

    def add_echo_server(self, node, start_ns, stop_ns, port=9):  # UdpEchoServerHelper (port).Install
        return self._app(kind=APP_ECHO_SERVER, node=node, start=start_ns, stop=stop_ns, port=port, ttl=64)

    def add_echo_client(self, node, dst, start_ns, stop_ns, count=1, interval_ns=1_000_000_000, size=1024,
                        ttl=64, remote_addr=None, remote_port=9):  # UdpEchoClientHelper (address, port).Install
        return self._app(kind=APP_ECHO_CLIENT, node=node, start=start_ns, stop=stop_ns, dst=dst, size=size,
                         count=count, interval=interval_ns, ttl=ttl, remote_addr=remote_addr,
                         remote_port=remote_port)

    # Ipv4AddressHelper::Assign on the two devices of a link, then NewNetwork (ipv4-address-helper.cc)
    def assign_link(self, da, db, network, mask=0xFFFFFF00):
        for d, host in ((da, 1), (db, 2)):
            node = self.dev[d][0]
            self.dev_addr[d] = network + host
            self.dev_mask[d] = mask
            # Ipv4L3Protocol::AddInterface: the loopback is interface 0 (SetupLoopback at Install)
            self.dev_ifindex[d] = self._nif.get(node, 1)
            self._nif[node] = self.dev_ifindex[d] + 1

    def _slot_nodes(self):
        # route-table columns: every datagram destination (sender apps' dst), echo clients' own nodes, and
        # with ICMP every sender's node (an error goes back to the offending datagram's sender)
        return sorted({a["dst"] for a in self.apps if a["kind"] in SENDERS}
                      | {a["node"] for a in self.apps if a["kind"] == APP_ECHO_CLIENT or
                         (self.icmp and a["kind"] in SENDERS)})

    def stop(self, t_ns):  # Simulator::Stop (t)
        self.stop_ns = t_ns
        self.setup.append((SETUP_STOP, 0))

    # ---------------- routing ----------------
    def _neighbors(self):
        nb = [[] for _ in range(self.n_nodes)]
        for d, (node, peer, *_r) in enumerate(self.dev):
            nb[node].append((self.dev[peer][0], d))
        return nb

    def route_bfs(self):
        """Next-hop table towards every datagram destination with ns-3's global-routing choice.

        GlobalRouteManager::PopulateRoutingTables + Ipv4GlobalRouting::LookupGlobal (RandomEcmpRouting
        off) over point-to-point links with unit metrics pick, for a destination address of node D,
        the first host route SPFIntraAddRouter installed for D: D's first root exit direction.  An exit
        list only grows by SPFVertex::MergeRootExitDirections, which sorts it by (next-hop address,
        outgoing interface) (global-route-manager-impl.cc:314-326); it holds the first hops of every
        shortest path.  So node R forwards through the device d whose peer lies one hop closer to D and
        whose (peer address, interface index) is smallest.  CheckForStubNode (:1245-1323) gives a node
        with a single link a default route through it.  Without addresses (tests that assign none) the
        lowest device wins.  oracle/nsref_route.cc restates the SPF itself; tests/test_routing_oracle.py
        checks this table against it, tests/test_gpu_routing.py the GPU builder (nsgpu_route_global)."""
        dsts = self._slot_nodes()
        self.dst_slot = {d: i for i, d in enumerate(dsts)}
        self.n_dst = max(1, len(dsts))
        dev = np.array([r[:2] for r in self.dev], dtype=np.int64).reshape(-1, 2)
        dnode, dpeer = dev[:, 0], dev[:, 1]
        pnode = dnode[dpeer] if len(dev) else dnode
        nd = len(dev)
        has_addr = len(self.dev_addr) == nd and nd > 0
        if has_addr:
            tie = (np.array([self.dev_addr[int(p)] for p in dpeer], np.int64) << 32) | \
                np.array([self.dev_ifindex[d] for d in range(nd)], np.int64)
        else:
            tie = np.arange(nd, dtype=np.int64)
        # CSR of each node's devices (ascending device index)
        order = np.argsort(dnode, kind="stable")
        off = np.zeros(self.n_nodes + 1, np.int64)
        np.add.at(off, dnode + 1, 1)
        off = np.cumsum(off)
        ndev = np.diff(off)
        R = np.full((self.n_nodes, self.n_dst), NO_ROUTE, dtype=np.uint32)
        for dst, slot in self.dst_slot.items():
            dist = np.full(self.n_nodes, -1, dtype=np.int64)
            dist[dst] = 0
            front = np.array([dst], np.int64)
            lev = 0
            while front.size:  # level-synchronous BFS over the undirected links
                lev += 1
                cnt = ndev[front]
                idx = np.repeat(off[front], cnt) + (np.arange(cnt.sum()) - np.repeat(np.cumsum(cnt) - cnt, cnt))
                nb = np.unique(pnode[order[idx]])
                nb = nb[dist[nb] < 0]
                dist[nb] = lev
                front = nb
            ok = (dist[dnode] > 0) & (dist[pnode] == dist[dnode] - 1)
            cand = np.where(ok, tie, np.iinfo(np.int64).max)
            best = np.full(self.n_nodes, np.iinfo(np.int64).max, np.int64)
            np.minimum.at(best, dnode, cand)
            win = ok & (cand == best[dnode])
            R[dnode[win], slot] = np.nonzero(win)[0].astype(np.uint32)
            stub = (ndev == 1) & (np.arange(self.n_nodes) != dst)
            R[stub, slot] = order[off[:-1][stub]].astype(np.uint32)
        self.route = R

    def next_hop(self, n, slot):
        if self.route is not None:
            return int(self.route[n, slot])
        dflt, off, es, ed = self.route_c
        lo, hi = int(off[n]), int(off[n + 1])
        j = lo + int(np.searchsorted(es[lo:hi], slot))
        return int(ed[j]) if j < hi and es[j] == slot else int(dflt[n])

    # ---------------- C view ----------------
    def c_struct(self):
        dev = np.array(self.dev, dtype=np.int64).reshape(-1, 6) if self.dev else np.zeros((0, 6), np.int64)
        A = self.apps
        arrays = dict(
            dev_node=dev[:, 0].astype(np.uint32), dev_peer=dev[:, 1].astype(np.uint32),
            dev_bps=dev[:, 2].astype(np.uint64), dev_ifg_ns=dev[:, 3].astype(np.int64),
            dev_delay_ns=dev[:, 4].astype(np.int64), dev_qmax=dev[:, 5].astype(np.uint32),
            route=(np.ascontiguousarray(self.route, dtype=np.uint32) if self.route is not None
                   else np.zeros(0, np.uint32)),
            app_kind=np.array([a["kind"] for a in A], np.uint32),
            app_node=np.array([a["node"] for a in A], np.uint32),
            app_start_ns=np.array([a["start"] for a in A], np.int64),
            app_stop_ns=np.array([a["stop"] for a in A], np.int64),
            app_dst_node=np.array([a["dst"] for a in A], np.uint32),
            app_dst_slot=np.array([self.dst_slot.get(a["dst"], 0) if a["kind"] in SENDERS else 0 for a in A],
                                  np.uint32),
            app_count=np.array([a["count"] for a in A], np.uint32),
            app_interval_ns=np.array([a["interval"] for a in A], np.int64),
            app_src_slot=np.array([self.dst_slot.get(a["node"], NO_ROUTE) if a["kind"] in SENDERS else NO_ROUTE
                                   for a in A], np.uint32),
            app_rate_bps=np.array([a["rate"] for a in A], np.uint64),
            app_pkt_size=np.array([a["size"] for a in A], np.uint32),
            app_on_s=np.array([a["on"] for a in A], np.float64),
            app_off_s=np.array([a["off"] for a in A], np.float64),
            app_max_bytes=np.array([a["maxb"] for a in A], np.uint32),
            app_ttl=np.array([a["ttl"] for a in A], np.uint32),
            setup_kind=np.array([k for k, _ in self.setup], np.uint32),
            setup_index=np.array([i for _, i in self.setup], np.uint32),
        )
        if self.route is None:
            dflt, off, es, ed = self.route_c
            arrays.update(route_default=np.ascontiguousarray(dflt, np.uint32),
                          route_exc_off=np.ascontiguousarray(off, np.uint64),
                          route_exc_slot=np.ascontiguousarray(es, np.uint32),
                          route_exc_dev=np.ascontiguousarray(ed, np.uint32))
        s = ScenarioStruct()
        s.n_nodes, s.n_devices, s.n_apps, s.n_dst = self.n_nodes, len(self.dev), len(A), self.n_dst
        for k, v in arrays.items():
            setattr(s, k, v.ctypes.data if v.size else None)
        s.stop_ns = self.stop_ns
        s.n_setup = len(self.setup)
        s.icmp = 1 if self.icmp else 0
        s.uid_first = self.uid_first
        s._keep = arrays  # keep the arrays alive with the struct
        return s


def ip(dotted):
    a, b, c, d = (int(v) for v in dotted.split("."))
    return (a << 24) | (b << 16) | (c << 8) | d


def first_cc():
    """examples/tutorial/first.cc:27-69: two nodes, 5Mbps / 2ms point-to-point, 10.1.1.0/24,
    UdpEchoServer (port 9) on node 1 from 1 s to 10 s, UdpEchoClient on node 0 from 2 s to 10 s
    (MaxPackets 1, Interval 1 s, PacketSize 1024).  No Simulator::Stop: Run ends with an empty queue."""
    sc = Scenario(2)  # nodes.Create (2)
    da, db = sc.link(0, 1, 5_000_000, 2_000_000)  # pointToPoint.Install (nodes)
    sc.install_stack()  # stack.Install (nodes)
    sc.assign_link(da, db, ip("10.1.1.0"))  # address.Assign (devices)
    sc.add_echo_server(1, 1_000_000_000, 10_000_000_000, port=9)
    sc.add_echo_client(0, 1, 2_000_000_000, 10_000_000_000, count=1, interval_ns=1_000_000_000, size=1024,
                       remote_addr=sc.dev_addr[db], remote_port=9)
    sc.route_bfs()
    return sc


def dumbbell(n_leaves=4, leaf_bps=1_000_000, leaf_delay_ns=2_000_000, router_bps=5_000_000,
             router_delay_ns=5_000_000, qmax=100, rate_bps=1_000_000, size=512, max_bytes=512,
             start_ns=1_000_000_000, stop_ns=5_000_000_000, sim_stop_ns=5_000_000_000, compressed=None):
    """src/mpi/examples/simple-distributed.cc (config 5) with n_leaves leaves per side: left leaves
    (system id 0), router 1 (0), router 2 (1), right leaves (1); routers 5Mbps/5ms, leaves 1Mbps/2ms;
    PacketSinks (port 50000) on the right leaves and OnOff (OnTime 1, OffTime 0, 1Mbps, 512 B,
    MaxBytes 512) from left leaf i to right leaf i, all from 1 s to 5 s; Simulator::Stop (5 s).
    Routes: the dumbbell's unique shortest paths (what the example's global / nix-vector routing
    finds), written directly.  Returns the scenario; `dumbbell_owner` gives the example's system ids."""
    n = n_leaves
    sc = Scenario(0)
    for _ in range(n):  # leftLeafNodes.Create (n, 0)
        sc.add_node()
    r1, r2 = sc.add_node(), sc.add_node()  # CreateObject<Node> (0), CreateObject<Node> (1)
    for _ in range(n):  # rightLeafNodes.Create (n, 1)
        sc.add_node()
    left = lambda i: i  # noqa: E731
    right = lambda i: n + 2 + i  # noqa: E731
    ra, rb = sc.link(r1, r2, router_bps, router_delay_ns, qmax)  # routerLink.Install (routerNodes)
    lleaf, lrout, rleaf, rrout = [], [], [], []
    for i in range(n):
        da, db = sc.link(left(i), r1, leaf_bps, leaf_delay_ns, qmax)
        lleaf.append(da)
        lrout.append(db)
    for i in range(n):
        da, db = sc.link(right(i), r2, leaf_bps, leaf_delay_ns, qmax)
        rleaf.append(da)
        rrout.append(db)
    sc.install_stack()  # stack.InstallAll ()
    sc.assign_link(ra, rb, ip("10.2.1.0"))
    for i in range(n):  # leftAddress 10.1.1.0 + NewNetwork per leaf
        sc.assign_link(lleaf[i], lrout[i], ip("10.1.1.0") + (i << 8))
    for i in range(n):
        sc.assign_link(rleaf[i], rrout[i], ip("10.3.1.0") + (i << 8))
    for i in range(n):  # sinkHelper.Install (rightLeafNodes.Get (i)); Start (1 s), Stop (5 s)
        sc.add_sink(right(i), start_ns, stop_ns, port=50000)
    for i in range(n):
        sc.add_onoff(left(i), right(i), start_ns, stop_ns, rate_bps=rate_bps, size=size, on_s=1.0, off_s=0.0,
                     max_bytes=max_bytes, remote_addr=sc.dev_addr[rleaf[i]], remote_port=50000)
    sc.stop(sim_stop_ns)
    dsts = sc._slot_nodes()
    sc.dst_slot = {d: k for k, d in enumerate(dsts)}
    sc.n_dst = max(1, len(dsts))
    if compressed is None:
        compressed = sc.n_nodes * sc.n_dst > (1 << 24)
    if compressed:
        # every node has one way out except router 2 (one exception per right leaf = slot j) and the
        # right leaves (their own slot: local delivery, never looked up)
        dflt = np.full(sc.n_nodes, NO_ROUTE, np.uint32)
        dflt[:n] = lleaf
        dflt[r1] = ra
        dflt[n + 2:] = rleaf
        cnt = np.zeros(sc.n_nodes, np.uint64)
        cnt[r2] = n
        off = np.zeros(sc.n_nodes + 1, np.uint64)
        off[1:] = np.cumsum(cnt)
        sc.route_c = (dflt, off, np.arange(n, dtype=np.uint32), np.asarray(rrout, np.uint32))
        return sc
    R = np.full((sc.n_nodes, sc.n_dst), NO_ROUTE, dtype=np.uint32)
    for d, k in sc.dst_slot.items():
        j = d - (n + 2)
        R[:n, k] = lleaf            # left leaf -> its router
        R[r1, k] = ra               # router 1 -> router 2
        R[r2, k] = rrout[j]         # router 2 -> right leaf j
        R[n + 2:, k] = rleaf        # other right leaves -> router 2
        R[d, k] = NO_ROUTE          # (local delivery)
    sc.route = R
    return sc


def incast(n_src, bps=10_000_000, delay_ns=1_000_000, qmax=100, rate_bps=1_000_000, size=512, max_bytes=0,
           start_ns=1_000_000_000, stop_ns=1_050_000_000, sim_stop_ns=1_100_000_000):
    """Incast star: node 0 is a hub with a PacketSink, nodes 1..n_src each link to it (PointToPointHelper
    per leaf, creation order) and run an OnOff flow to it (OnTime 1, OffTime 0), all started at the
    same time — so every window holds n_src same-time Receives at one node that is also the sink
    (the hub node path with local deliveries, and with n_src > WCAP a sorted run whose chunks cut a
    same-time group of zero-delay DoForwardUp leaves)."""
    sc = Scenario(n_src + 1)
    for i in range(1, n_src + 1):
        da, db = sc.link(i, 0, bps, delay_ns, qmax)
    sc.install_stack()
    for i in range(n_src):
        sc.assign_link(2 * i, 2 * i + 1, ip("10.0.0.0") + (i << 8))
    sc.add_sink(0, 0, 0)
    for i in range(1, n_src + 1):
        sc.add_onoff(i, 0, start_ns, stop_ns, rate_bps=rate_bps, size=size, on_s=1.0, off_s=0.0, max_bytes=max_bytes,
                     remote_addr=sc.dev_addr[1])
    sc.stop(sim_stop_ns)
    sc.route_bfs()
    return sc


def dumbbell_owner(n_leaves, nranks=2):
    """Node (systemId) of simple-distributed.cc: left side + router 1 on 0, router 2 + right side on 1
    (nranks > 2: the right side's leaves spread over ranks 1..nranks-1 in contiguous blocks)."""
    n = n_leaves
    own = np.zeros(2 * n + 2, np.uint32)
    own[n + 1:] = 1
    if nranks > 2:
        blk = -(-n // (nranks - 1))
        own[n + 2:] = 1 + np.arange(n) // blk
    return own


def grid(rows, cols, bps=10_000_000, delay_ns=1_000_000, qmax=100, flows="columns", start_ns=100_000_000,
         stop_ns=2_000_000_000, sim_stop_ns=2_100_000_000, rate_bps=500_000, size=512, on_s=1e9, off_s=0.0,
         ttl=255, n_flows=None, icmp=False):
    """PointToPointGridHelper topology (point-to-point-grid.cc:33-72) with OnOff/PacketSink flows.

    flows="columns": one flow per column from row 0 to the last row;
    routes are XY (row first, then column) static next hops."""
    sc = Scenario(0, icmp=icmp)
    nid = lambda y, x: y * cols + x  # noqa: E731
    n = rows * cols
    # the device of each node towards its four grid neighbours (XY routing's next hops)
    right, left, down, up = (np.full(n, NO_ROUTE, np.uint32) for _ in range(4))
    row_links, col_links = [], []
    for y in range(rows):
        for x in range(cols):
            sc.add_node()  # rowNodes.Create (1)
            if x > 0:
                da, db = sc.link(nid(y, x - 1), nid(y, x), bps, delay_ns, qmax)
                right[nid(y, x - 1)], left[nid(y, x)] = da, db
                row_links.append((da, db))
            if y > 0:
                da, db = sc.link(nid(y - 1, x), nid(y, x), bps, delay_ns, qmax)
                down[nid(y - 1, x)], up[nid(y, x)] = da, db
                col_links.append((da, db))
    sc.install_stack()  # PointToPointGridHelper::InstallStack (point-to-point-grid.cc:79-89)
    # AssignIpv4Addresses (point-to-point-grid.cc:97-132): every row link, then every column link, one
    # /24 each (rowIp 10.0.0.0, colIp 11.0.0.0: disjoint at 128x128)
    for k, (da, db) in enumerate(row_links):
        sc.assign_link(da, db, ip("10.0.0.0") + (k << 8))
    for k, (da, db) in enumerate(col_links):
        sc.assign_link(da, db, ip("11.0.0.0") + (k << 8))
    fl = []
    if flows == "columns":
        ncol = cols if n_flows is None else min(cols, n_flows)
        fl = [(nid(0, x), nid(rows - 1, x)) for x in range(ncol)]
    else:
        fl = list(flows)
    # sinks first (PacketSinkHelper.Install), then the OnOff sources
    sinks = {}
    for _s, d in fl:
        if d not in sinks:
            sinks[d] = sc.add_sink(d, 0, 0)
    for s_, d in fl:
        # PointToPointGridHelper::GetIpv4Address (point-to-point-grid.cc:243-265): the node's left row
        # device, the right one in column 0
        yd, xd = divmod(d, cols)
        raddr = sc.dev_addr[int(right[d] if xd == 0 else left[d])] if cols > 1 else None
        sc.add_onoff(s_, d, start_ns, stop_ns, rate_bps=rate_bps, size=size, on_s=on_s, off_s=off_s, ttl=ttl,
                     remote_addr=raddr)
    sc.stop(sim_stop_ns)
    # XY routes towards each destination (with ICMP also towards every source): along the row first,
    # then along the column — global routing's choice on this helper's addressing (test_routing_oracle.py)
    dsts = sc._slot_nodes()
    sc.dst_slot = {d: i for i, d in enumerate(dsts)}
    sc.n_dst = max(1, len(dsts))
    R = np.full((n, sc.n_dst), NO_ROUTE, dtype=np.uint32)
    ys, xs = np.divmod(np.arange(n), cols)
    for d, slot in sc.dst_slot.items():
        yd, xd = divmod(d, cols)
        col = np.where(xs != xd, np.where(xd > xs, right, left), np.where(yd > ys, down, up))
        col[d] = NO_ROUTE
        R[:, slot] = col
    sc.route = R
    return sc


def random_topology(n_nodes, n_links, n_flows, seed, bps_choices=(1_000_000, 5_000_000, 10_000_000),
                    delay_choices=(100_000, 1_000_000, 2_000_000), qmax=20, stop_ns=1_000_000_000, ttl=64,
                    icmp=False, sink_window=None):
    """Connected random topology with OnOff flows (on/off cycling, max bytes) for parity tests.
    ttl: the flows' IP TTL (small values expire on long paths); sink_window: (start, stop) of every
    PacketSink (late starts / early stops leave datagrams without a bound endpoint)."""
    rng = np.random.default_rng(seed)
    sc = Scenario(n_nodes, icmp=icmp)
    edges = set()
    for n in range(1, n_nodes):  # spanning tree
        m = int(rng.integers(0, n))
        edges.add((m, n))
    while len(edges) < n_links:
        a, b = sorted(rng.choice(n_nodes, 2, replace=False).tolist())
        edges.add((a, b))
    links = [sc.link(a, b, int(rng.choice(bps_choices)), int(rng.choice(delay_choices)), qmax)
             for a, b in sorted(edges)]
    sc.install_stack()
    for k, (da, db) in enumerate(links):  # Ipv4AddressHelper ("10.1.0.0", "255.255.255.0"), NewNetwork per link
        sc.assign_link(da, db, ip("10.1.0.0") + (k << 8))
    flows = []
    for _ in range(n_flows):
        s_, d = rng.choice(n_nodes, 2, replace=False).tolist()
        flows.append((s_, d))
    sinks = {}
    for _s, d in flows:
        if d not in sinks:
            t0 = int(rng.integers(0, 50_000_000))
            sinks[d] = sc.add_sink(d, *(sink_window if sink_window else (t0, 0)))
    for s_, d in flows:
        st = int(rng.integers(50_000_000, 300_000_000))
        sc.add_onoff(s_, d, st, int(st + rng.integers(200_000_000, 600_000_000)),
                     rate_bps=int(rng.choice([200_000, 500_000, 2_000_000])), size=int(rng.choice([64, 512, 1000])),
                     on_s=float(rng.choice([0.05, 0.1, 1.0])), off_s=float(rng.choice([0.0, 0.02, 0.05])),
                     max_bytes=int(rng.choice([0, 0, 20000])), ttl=ttl)
    sc.stop(stop_ns)
    sc.route_bfs()
    return sc


class Engine:
    """The GPU engine for one scenario (nsgpu_p2p_create / reset / run / results)."""

    def __init__(self, scenario, log_cap=0, pool_cap=0, stream=None):
        self.s = scenario.c_struct()
        self.stream = stream
        self.log_cap = log_cap
        h = C.c_void_p()
        nsgpu.check(nsgpu.lib().nsgpu_p2p_create(C.byref(self.s), pool_cap, log_cap, C.byref(h)))
        self.h = h.value

    def reset(self):
        nsgpu.check(nsgpu.lib().nsgpu_p2p_reset(self.h, self.stream))

    def launch(self):
        nsgpu.check(nsgpu.lib().nsgpu_p2p_run(self.h, self.stream))

    def wide(self):
        """Whether this engine runs wide windows (nsgpu_p2p_get_wide)."""
        w = C.c_int()
        nsgpu.check(nsgpu.lib().nsgpu_p2p_get_wide(self.h, C.byref(w)))
        return bool(w.value)

    def set_eager(self, eager=True):
        nsgpu.check(nsgpu.lib().nsgpu_p2p_set_eager(self.h, int(eager)))

    def set_trace(self, cap, kinds=TRACE_DEVICE_KINDS):
        """Record the ascii/pcap trace sink calls of every run (nsgpu_p2p_set_trace), up to `cap`: the
        nsgpu_trace_kind bits in `kinds` (nsgpu_p2p_set_trace_kinds; TRACE_IPV4_KINDS adds the
        Ipv4L3Protocol Tx / Rx / Drop sinks)."""
        nsgpu.check(nsgpu.lib().nsgpu_p2p_set_trace(self.h, int(cap)))
        nsgpu.check(nsgpu.lib().nsgpu_p2p_set_trace_kinds(self.h, int(kinds)))
        self.trace_cap = int(cap)

    def trace(self):
        """The last run's trace records (trace.TRACE_RECORD_DTYPE), unordered."""
        n = C.c_uint64()
        out = np.zeros(self.trace_cap, TRACE_RECORD_DTYPE)
        nsgpu.check(nsgpu.lib().nsgpu_p2p_trace_read(self.h, out.ctypes.data, self.trace_cap, C.byref(n),
                                                     self.stream))
        return out[:n.value]

    def profile(self, sample_every=4):
        """One full run with per-kernel HIP-event brackets (nsgpu_p2p_profile); returns
        {kernel name: (average ms per launch, bracketed launches)}."""
        n = C.c_int()
        nsgpu.check(nsgpu.lib().nsgpu_p2p_kernel_count(C.byref(n)))
        ms = np.zeros(n.value, np.float64)
        cnt = np.zeros(n.value, np.uint64)
        self.reset()
        nsgpu.check(nsgpu.lib().nsgpu_p2p_profile(self.h, self.stream, sample_every, ms.ctypes.data,
                                                  cnt.ctypes.data))
        out = {}
        for k in range(n.value):
            name = nsgpu.lib().nsgpu_p2p_kernel_name(k).decode()
            out[name] = (float(ms[k] / cnt[k]) if cnt[k] else 0.0, int(cnt[k]))
        return out

    def counters(self):
        """Device / application counters now (nsgpu_p2p_counters: e.g. from a host closure)."""
        devc = np.zeros(self.s.n_devices, DEV_COUNTERS_DTYPE)
        appc = np.zeros(self.s.n_apps, APP_COUNTERS_DTYPE)
        nsgpu.check(nsgpu.lib().nsgpu_p2p_counters(self.h, devc.ctypes.data, appc.ctypes.data, self.stream))
        return devc, appc

    def results(self, log_n=0):
        st = P2PStats()
        devc = np.zeros(self.s.n_devices, DEV_COUNTERS_DTYPE)
        appc = np.zeros(self.s.n_apps, APP_COUNTERS_DTYPE)
        log_n = min(log_n, self.log_cap)
        lts = np.zeros(log_n, np.uint64)
        luid = np.zeros(log_n, np.uint32)
        lctx = np.zeros(log_n, np.uint32)
        err = C.c_uint32()
        nsgpu.check(nsgpu.lib().nsgpu_p2p_results(self.h, C.byref(st), devc.ctypes.data, appc.ctypes.data,
                                                  lts.ctypes.data if log_n else None,
                                                  luid.ctypes.data if log_n else None,
                                                  lctx.ctypes.data if log_n else None, log_n, C.byref(err),
                                                  self.stream))
        return st, devc, appc, (lts, luid, lctx)

    def run(self, log_n=0):
        self.reset()
        self.launch()
        return self.results(log_n)

    def close(self):
        if self.h:
            nsgpu.lib().nsgpu_p2p_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ---------------------------------------------------------------- partitioned runs
STAT_FIELDS = [f for f, _ in P2PStats._fields_]
RUN_GLOBAL_FIELDS = ("dispatched", "final_ts", "next_uid", "windows", "max_window")


def stats_to_dict(st):
    return {f: int(getattr(st, f)) for f in STAT_FIELDS}


def stats_from_dict(d):
    st = P2PStats()
    for k, v in d.items():
        setattr(st, k, v)
    return st


def owner_blocks(n_nodes, nranks):
    """Node -> rank map of contiguous, balanced node-id blocks, the way the reference's distributed
    examples give nodes their system id (Node (sid), node.cc:76-108; src/mpi/examples): a grid built
    row by row splits into row bands."""
    if nranks < 1:
        raise ValueError("nranks >= 1")
    return (np.arange(n_nodes, dtype=np.int64) * nranks // max(n_nodes, 1)).astype(np.uint32)


def merge_results(per_rank, owner, s):
    """One result from the per-rank results (stats, devc, appc, log) of a partitioned run: the
    run-global fields (dispatch count, final time, next uid, windows) from rank 0, per-rank tallies
    summed (the digest modulo 2^64), every device / application counter from the rank owning its
    node, and the dispatch log as the union of the entries each rank wrote (zeros elsewhere)."""
    owner = np.asarray(owner)
    out = {}
    for f in STAT_FIELDS:
        if f in RUN_GLOBAL_FIELDS:
            out[f] = int(getattr(per_rank[0][0], f))
        else:
            out[f] = sum(int(getattr(r[0], f)) for r in per_rank) & ((1 << 64) - 1)
    dev_node, app_node = s._keep["dev_node"], s._keep["app_node"]
    devc = per_rank[0][1].copy()
    appc = per_rank[0][2].copy()
    for r, (_st, dc, ac, _log) in enumerate(per_rank):
        m = owner[dev_node] == r
        devc[m] = dc[m]
        m = owner[app_node] == r
        appc[m] = ac[m]
    log = tuple(np.sum([rr[3][i] for rr in per_rank], axis=0, dtype=per_rank[0][3][i].dtype) for i in range(3))
    return stats_from_dict(out), devc, appc, log


class Comm:
    """RCCL communicator of a partitioned run (nsgpu_comm_*), one rank per GPU process; create it
    after selecting the rank's device."""

    @staticmethod
    def unique_id():
        buf = (C.c_uint8 * 128)()
        nsgpu.check(nsgpu.lib().nsgpu_comm_unique_id(buf))
        return bytes(buf)

    def __init__(self, uid, nranks, rank):
        buf = (C.c_uint8 * 128).from_buffer_copy(bytes(uid))
        h = C.c_void_p()
        nsgpu.check(nsgpu.lib().nsgpu_comm_init(buf, nranks, rank, C.byref(h)))
        self.h = h.value
        self.nranks, self.rank = nranks, rank

    def __del__(self):
        try:
            nsgpu.lib().nsgpu_comm_destroy(self.h)
        except Exception:
            pass


class Plan(C.Structure):
    """nsgpu_p2p_plan (include/nsgpu.h): the constants a rank's partitioned engine is built from."""
    _fields_ = [("wide", C.c_uint32), ("maxc", C.c_uint32), ("wcap", C.c_uint32), ("xlcap", C.c_uint32),
                ("x0_bytes", C.c_uint64), ("x1_bytes", C.c_uint64), ("x2_bytes", C.c_uint64),
                ("x2_records", C.c_uint32), ("n_kinds", C.c_uint32),
                ("lookahead", C.c_int64 * 16), ("lookw", C.c_int64 * 16), ("tx_min", C.c_int64), ("lx", C.c_int64),
                ("red0_tmin", C.c_uint64), ("red0_wend", C.c_uint64), ("red0_wendw", C.c_uint64),
                ("stop_ts", C.c_uint64), ("stop_uid", C.c_uint32), ("uid_init", C.c_uint32),
                ("n_init", C.c_uint32), ("pad", C.c_uint32), ("pool_cap", C.c_uint64)]


# the plan's fields that may differ between ranks (each rank's own setup events and pool)
PLAN_PER_RANK = ("n_init", "pool_cap", "pad")


def dist_plan(scenario, owner, rank, nranks, pool_cap=0):
    """nsgpu_p2p_dist_plan (host only, no device): the sizes and constants rank `rank`'s engine feeds its
    collectives — X0 / X1 / X2 bytes, X2 records per peer, window capacities, lookaheads, window 0's bound —
    as a dict (arrays as lists).  owner None: the single engine's plan."""
    s = scenario.c_struct()
    own = None
    if owner is not None:
        own = np.ascontiguousarray(owner, dtype=np.uint32)
        if len(own) != s.n_nodes:
            raise ValueError("owner: one rank per node")
    pl = Plan()
    nsgpu.check(nsgpu.lib().nsgpu_p2p_dist_plan(C.byref(s), own.ctypes.data if own is not None else None, rank,
                                                 nranks, pool_cap, C.byref(pl)))
    out = {}
    for f, _t in Plan._fields_:
        v = getattr(pl, f)
        out[f] = list(v)[:pl.n_kinds] if f in ("lookahead", "lookw") else int(v)
    return out


def plan_mismatch(plans):
    """The collective-shaping fields on which a list of per-rank plans disagree ({} when all agree)."""
    bad = {}
    for f in plans[0]:
        if f in PLAN_PER_RANK:
            continue
        vals = [p[f] for p in plans]
        if any(v != vals[0] for v in vals[1:]):
            bad[f] = vals
    return bad


class DistEngine(Engine):
    """Partition `rank` of `nranks` of a scenario (nsgpu_p2p_create_dist): the nodes with
    owner[n] == rank.  With a Comm it runs on its own (one process per GPU, RCCL collectives);
    without one it is a LoopbackGroup member."""

    def __init__(self, scenario, owner, rank, nranks, comm=None, log_cap=0, pool_cap=0, stream=None):
        self.s = scenario.c_struct()
        self.owner = np.ascontiguousarray(owner, dtype=np.uint32)
        if len(self.owner) != self.s.n_nodes:
            raise ValueError("owner: one rank per node")
        self.stream = stream
        self.log_cap = log_cap
        self.comm = comm
        h = C.c_void_p()
        nsgpu.check(nsgpu.lib().nsgpu_p2p_create_dist(C.byref(self.s), self.owner.ctypes.data, rank, nranks,
                                                       comm.h if comm is not None else None, pool_cap, log_cap,
                                                       C.byref(h)))
        self.h = h.value


class LoopbackGroup:
    """Every partition of one scenario on this GPU (nsgpu_p2p_group_*): the partitioned algorithm
    with device-to-device copies in place of the RCCL collectives — its parity harness on one device."""

    def __init__(self, scenario, nranks, owner=None, log_cap=0, pool_cap=0, stream=None, trace_cap=0,
                 trace_kinds=None):
        self.owner = owner_blocks(scenario.n_nodes, nranks) if owner is None else np.asarray(owner, np.uint32)
        self.members = [DistEngine(scenario, self.owner, r, nranks, None, log_cap, pool_cap, stream)
                        for r in range(nranks)]
        if trace_cap:
            for m in self.members:
                m.set_trace(trace_cap, TRACE_DEVICE_KINDS if trace_kinds is None else trace_kinds)
        self.stream = stream
        arr = (C.c_void_p * nranks)(*[m.h for m in self.members])
        h = C.c_void_p()
        nsgpu.check(nsgpu.lib().nsgpu_p2p_group_create(arr, nranks, C.byref(h)))
        self.h = h.value

    def reset(self):
        nsgpu.check(nsgpu.lib().nsgpu_p2p_group_reset(self.h, self.stream))

    def launch(self):
        nsgpu.check(nsgpu.lib().nsgpu_p2p_group_run(self.h, self.stream))

    def trace(self):
        """Every partition's trace records (each rank records the sink calls of its own nodes)."""
        return np.concatenate([m.trace() for m in self.members])

    def results(self, log_n=0):
        per = [m.results(log_n) for m in self.members]
        return merge_results(per, self.owner, self.members[0].s)

    def run(self, log_n=0):
        self.reset()
        self.launch()
        return self.results(log_n)

    def __del__(self):
        try:
            nsgpu.lib().nsgpu_p2p_group_destroy(self.h)
        except Exception:
            pass


class TraceAddressing(C.Structure):
    """nsgpu_trace_addressing (include/nsgpu.h)."""
    _fields_ = [("dev_addr", C.c_void_p), ("dev_ip_ifindex", C.c_void_p), ("app_remote_addr", C.c_void_p),
                ("app_remote_port", C.c_void_p)]


def _out_bytes(call):
    """Runs a size query, then the call into a buffer of that size (the codec's output convention)."""
    n = C.c_uint64(0)
    nsgpu.check(call(None, 0, C.byref(n)))
    buf = C.create_string_buffer(max(n.value, 1))
    nsgpu.check(call(buf, n.value, C.byref(n)))
    return buf.raw[:n.value]


class TraceCodec:
    """The product library's trace codec (nsgpu_trace_*, ns-3-dev-dnemu_amd/csrc/nsgpu_trace.cc) for a
    scenario: the ascii / pcap bytes of ns-3's default sinks from nsgpu_trace_record streams."""

    def __init__(self, sc):
        self.sc = sc
        self._s = sc.c_struct()
        nd, na = len(sc.dev), len(sc.apps)
        self._arrs = [np.array([sc.dev_addr.get(d, 0) for d in range(nd)], np.uint32),
                      np.array([sc.dev_ifindex.get(d, 0) for d in range(nd)], np.uint32),
                      np.array([a["remote_addr"] or 0 for a in sc.apps] or [0], np.uint32)[:max(na, 1)],
                      np.array([a["remote_port"] for a in sc.apps] or [0], np.uint32)]
        self._ad = TraceAddressing(*[a.ctypes.data for a in self._arrs])
        h = C.c_void_p()
        nsgpu.check(nsgpu.lib().nsgpu_trace_codec_create(C.byref(self._s), C.byref(self._ad), C.byref(h)))
        self.h = h

    def __del__(self):
        if getattr(self, "h", None):
            nsgpu.lib().nsgpu_trace_codec_free(self.h)
            self.h = None

    @staticmethod
    def sort(tr):
        tr = np.ascontiguousarray(np.array(tr, dtype=TRACE_RECORD_DTYPE))
        nsgpu.check(nsgpu.lib().nsgpu_trace_sort(tr.ctypes.data, len(tr)))
        return tr

    def ascii(self, tr):
        tr = np.ascontiguousarray(tr, dtype=TRACE_RECORD_DTYPE)
        return _out_bytes(lambda o, c, n: nsgpu.lib().nsgpu_trace_ascii(self.h, tr.ctypes.data, len(tr), o, c, n)).decode()

    def line(self, rec):
        r = np.ascontiguousarray(np.array([rec], dtype=TRACE_RECORD_DTYPE))
        return _out_bytes(lambda o, c, n: nsgpu.lib().nsgpu_trace_line(self.h, r.ctypes.data, o, c, n)).decode()

    def packet(self, rec):
        r = np.ascontiguousarray(np.array([rec], dtype=TRACE_RECORD_DTYPE))
        return _out_bytes(lambda o, c, n: nsgpu.lib().nsgpu_trace_packet(self.h, r.ctypes.data, o, c, n))

    def pcap(self, tr, dev):
        tr = np.ascontiguousarray(tr, dtype=TRACE_RECORD_DTYPE)
        return _out_bytes(lambda o, c, n: nsgpu.lib().nsgpu_trace_pcap(self.h, tr.ctypes.data, len(tr), dev, o, c, n))

    def pcaps(self, tr, ifindex):
        """{(node, ifindex): file bytes} for every point-to-point device (EnablePcapAll)."""
        return {(self.sc.dev[d][0], ifindex[d]): self.pcap(tr, d) for d in range(len(self.sc.dev))}


def pcap_file(linktype, snaplen, records):
    """PcapFile::Init + Write through the product library (nsgpu_pcap_file): records = [(sec, usec, data,
    orig_len)]."""
    n = len(records)
    sec = np.array([r[0] for r in records] or [0], np.uint32)
    usec = np.array([r[1] for r in records] or [0], np.uint32)
    orig = np.array([r[3] for r in records] or [0], np.uint32)
    off = np.zeros(n + 1, np.uint64)
    off[1:] = np.cumsum([len(r[2]) for r in records]) if n else []
    data = np.frombuffer(b"".join(bytes(r[2]) for r in records) or b"\0", np.uint8).copy()
    return _out_bytes(lambda o, c, k: nsgpu.lib().nsgpu_pcap_file(linktype, snaplen, n, sec.ctypes.data, usec.ctypes.data,
                                                                  orig.ctypes.data, off.ctypes.data, data.ctypes.data,
                                                                  o, c, k))


# ---------------- setup journal (HipSimulatorImpl's) -> setup list (nsgpu_setup_from_journal) ----------------
J_CALL, J_DESTROY, J_STOP, J_NODE_START, J_DEVICE_START, J_APP_START = 0, 1, 2, 3, 4, 5
NDEV_P2P, NDEV_LOOPBACK, NDEV_OTHER = 0, 1, 2
JOURNAL_DTYPE = np.dtype([("ts", "<u8"), ("context", "<u4"), ("kind", "<u4"), ("local", "<u4"), ("pad_", "<u4")])


class SetupMap(C.Structure):
    """nsgpu_setup_map (include/nsgpu.h)."""
    _fields_ = [("setup_kind", C.c_void_p), ("setup_index", C.c_void_p), ("owned", C.c_void_p),
                ("dev_node", C.c_void_p), ("dev_local", C.c_void_p), ("app_node", C.c_void_p),
                ("app_local", C.c_void_p), ("n_owned", C.c_uint64), ("n_devices", C.c_uint32),
                ("n_apps", C.c_uint32), ("stop_ns", C.c_int64)]


def scenario_journal(sc):
    """What HipSimulatorImpl journals while a program builds scenario `sc` with the stock helpers, and the node
    list it then sees: (journal entries, per-node device kinds in AddDevice order, per-node application counts).
    A setup UID entry is the singletons' ScheduleDestroy; NOOP the loopback device's start."""
    j = np.zeros(len(sc.setup), JOURNAL_DTYPE)
    devs = [[] for _ in range(sc.n_nodes)]
    napp = [0] * sc.n_nodes
    for i, (kind, k) in enumerate(sc.setup):
        e = j[i]
        e["context"] = 0xFFFFFFFF
        if kind == SETUP_UID:
            e["kind"] = J_DESTROY
        elif kind == SETUP_STOP:
            e["kind"], e["ts"] = J_STOP, sc.stop_ns
        elif kind == SETUP_NODE:
            e["kind"], e["context"] = J_NODE_START, k
        elif kind in (SETUP_DEVICE, SETUP_NOOP):
            n = sc.dev[k][0] if kind == SETUP_DEVICE else k
            e["kind"], e["context"], e["local"] = J_DEVICE_START, n, len(devs[n])
            devs[n].append(NDEV_P2P if kind == SETUP_DEVICE else NDEV_LOOPBACK)
        elif kind == SETUP_APP:
            n = sc.apps[k]["node"]
            e["kind"], e["context"], e["local"] = J_APP_START, n, napp[n]
            napp[n] += 1
    return j, devs, napp


def setup_from_journal(journal, node_devs, node_n_apps):
    """nsgpu_setup_from_journal: (setup list [(kind, index)], owned journal indices, engine device -> (node,
    local), engine application -> (node, local), stop_ns).  Raises NsgpuError on an inconsistent journal."""
    j = np.ascontiguousarray(journal, dtype=JOURNAL_DTYPE)
    n, nn = len(j), len(node_devs)
    off = np.zeros(nn + 1, np.uint64)
    off[1:] = np.cumsum([len(d) for d in node_devs]) if nn else []
    kinds = np.array([k for d in node_devs for k in d] or [0], np.uint32)
    napp = np.array(list(node_n_apps) or [0], np.uint32)
    nd, na = int(off[-1]), int(napp[:nn].sum()) if nn else 0
    sk, si, ow = (np.zeros(max(n, 1), np.uint32) for _ in range(3))
    dn, dl = np.zeros(max(nd, 1), np.uint32), np.zeros(max(nd, 1), np.uint32)
    an, al = np.zeros(max(na, 1), np.uint32), np.zeros(max(na, 1), np.uint32)
    m = SetupMap(sk.ctypes.data, si.ctypes.data, ow.ctypes.data, dn.ctypes.data, dl.ctypes.data, an.ctypes.data,
                 al.ctypes.data, 0, 0, 0, -1)
    nsgpu.check(nsgpu.lib().nsgpu_setup_from_journal(j.ctypes.data if n else None, n, nn, off.ctypes.data,
                                                     kinds.ctypes.data, napp.ctypes.data, C.byref(m)))
    setup = [(int(a), int(b)) for a, b in zip(sk[:n], si[:n])]
    return (setup, ow[:m.n_owned].tolist(), list(zip(dn[:m.n_devices].tolist(), dl[:m.n_devices].tolist())),
            list(zip(an[:m.n_apps].tolist(), al[:m.n_apps].tolist())), m.stop_ns)
