// nsref_route.cc — CPU ORACLE (test infrastructure only): ns-3.13 global routing over point-to-point
// links, restated from GlobalRouteManagerImpl / GlobalRouter / CandidateQueue / Ipv4GlobalRouting.
//
//   LSDB       GlobalRouter::DiscoverLSAs (global-router-interface.cc:588-704): one router-LSA per node,
//              link records in node device order; a p2p device gives a PointToPoint record {linkId =
//              the peer's router id, linkData = the local address} then a StubNetwork record {linkId =
//              the peer's address, linkData = the peer's mask} (:1021-1139); the loopback device that
//              InternetStackHelper adds after the links (ipv4-l3-protocol.cc:227-254) is a broadcast
//              link with no other router: a StubNetwork record {127.0.0.0, 255.0.0.0} (:751-811).
//              Router ids are allocated in node order (global-route-manager.cc:57-61).
//   SPF        GlobalRouteManagerImpl::SPFCalculate (global-route-manager-impl.cc:1327-1490), SPFNext
//              (:734-953), SPFNexthopCalculation (:966-1139), SPFGetNextLink (:1154-1226),
//              CheckForStubNode (:1245-1323), SPFIntraAddRouter (:1915-2055: host routes),
//              SPFProcessStubs / SPFIntraAddStub (:1654-1818: network routes), SPFVertex exit lists
//              (:271-349: Merge sorts and uniques), CandidateQueue (candidate-queue.cc:86-191: a list kept
//              sorted by distance, network before router on ties, upper_bound insertion).
//   Lookup     Ipv4GlobalRouting::LookupGlobal (ipv4-global-routing.cc:136-242): host routes in insertion
//              order, then network routes, then externals; RandomEcmpRouting off -> the first match.
//              RouteInput delivers locally first when the destination is one of the node's addresses.
//
// Every link metric is 1 (Ipv4Interface default).  Transit networks (CSMA) do not occur on this path.
#include <algorithm>
#include <cstdint>
#include <list>
#include <utility>
#include <vector>

#include "nsref.h"

namespace {

enum LinkType { P2P = 1, TRANSIT = 2, STUB = 3 };

struct LinkRecord {
  int type;
  uint32_t linkId, linkData;
  uint32_t metric;
};

struct Exit {  // SPFVertex::NodeExit_t: (next hop address, root's outgoing interface)
  uint32_t nextHop;
  int32_t outIf;
  bool operator<(const Exit &o) const { return nextHop != o.nextHop ? nextHop < o.nextHop : outIf < o.outIf; }
  bool operator==(const Exit &o) const { return nextHop == o.nextHop && outIf == o.outIf; }
};

struct HostRoute {
  uint32_t dest, gateway;
  int32_t iface;
};
struct NetRoute {
  uint32_t net, mask, gateway;
  int32_t iface;
};

enum Status { NOT_EXPLORED = 0, CANDIDATE = 1, IN_SPFTREE = 2 };

struct Topo {
  uint32_t n;
  std::vector<std::vector<LinkRecord>> lsa;          // router-LSA of each node (router id = node id)
  std::vector<std::vector<std::pair<uint32_t, uint32_t>>> ifaddr;  // per node: (ifindex -> (addr, mask))
  std::vector<std::vector<int32_t>> if_dev;          // per node: ifindex -> device (-1: loopback)
};

// One SPF vertex per router (p2p-only LSDBs have no network vertices).
struct Vertex {
  uint32_t dist = 0;
  std::list<Exit> exits;
  std::list<int> parents;
  std::list<int> children;
  bool processed = false;
};

struct Spf {
  const Topo &T;
  uint32_t root;
  std::vector<int> status;
  std::vector<Vertex> V;
  std::list<int> cand;  // CandidateQueue::m_candidates
  std::vector<HostRoute> host;
  std::vector<NetRoute> net;

  explicit Spf(const Topo &t, uint32_t r) : T(t), root(r), status(t.n, NOT_EXPLORED), V(t.n) {}

  // GlobalRouteManagerImpl::FindOutgoingInterfaceId -> Ipv4::GetInterfaceForPrefix (a, amask)
  int32_t find_if(uint32_t a, uint32_t amask = 0xffffffffu) const {
    const auto &ifs = T.ifaddr[root];
    for (uint32_t i = 0; i < ifs.size(); ++i)
      if ((ifs[i].first & amask) == (a & amask)) return (int32_t)i;
    return -1;
  }
  // CandidateQueue::Push: upper_bound by CompareSPFVertex (distance; network before router)
  void push(int w) {
    auto it = cand.begin();
    while (it != cand.end() && !(V[w].dist < V[*it].dist)) ++it;
    cand.insert(it, w);
  }
  // SPFGetNextLink (v, w, prev = 0): the first p2p record of v pointing at w
  const LinkRecord *link_to(int v, int w) const {
    for (const auto &l : T.lsa[v])
      if (l.linkId == (uint32_t)w) return &l;  // (the reference compares link ids only)
    return nullptr;
  }
  // SPFNexthopCalculation for router vertices (:966-1139)
  void nexthop(int v, Vertex &w, int wid, const LinkRecord *l, uint32_t distance) {
    if (v == (int)root) {
      const LinkRecord *remote = link_to(wid, v);  // SPFGetNextLink (w, v, 0)
      const uint32_t nextHop = remote->linkData;
      const int32_t outIf = find_if(l->linkData);
      w.exits.clear();  // SetRootExitDirection
      w.exits.push_back({nextHop, outIf});
    } else {
      w.exits = V[v].exits;  // InheritAllRootExitDirections
    }
    w.dist = distance;
    w.parents.clear();  // SetParent
    w.parents.push_back(v);
  }
  // SPFNext (:734-953)
  void next(int v) {
    for (const auto &l : T.lsa[v]) {
      if (l.type == STUB) continue;  // (a)
      const int w = (int)l.linkId;   // (b) m_lsdb->GetLSA (linkId)
      if (status[w] == IN_SPFTREE) continue;  // (c)
      const uint32_t distance = V[v].dist + l.metric;  // (d)
      if (status[w] == NOT_EXPLORED) {
        nexthop(v, V[w], w, &l, distance);
        status[w] = CANDIDATE;
        push(w);
      } else {  // CANDIDATE
        Vertex &cw = V[w];
        if (cw.dist < distance) continue;
        if (cw.dist == distance) {  // equal cost: merge exits and parents
          Vertex tmp;
          nexthop(v, tmp, w, &l, distance);
          for (const auto &e : tmp.exits) cw.exits.push_back(e);  // MergeRootExitDirections
          cw.exits.sort();
          cw.exits.unique();
          for (int p : tmp.parents) cw.parents.push_back(p);  // MergeParent
          cw.parents.sort();
          cw.parents.unique();
        } else {  // lower cost (not reachable with unit metrics in BFS order; restated anyway)
          nexthop(v, cw, w, &l, distance);
          cand.sort([&](int a, int b) { return V[a].dist < V[b].dist; });  // Reorder (stable)
        }
      }
    }
  }
  // SPFIntraAddRouter (:1915-2055): host routes to every p2p local address of v, one per exit
  void add_router(int v) {
    for (const auto &l : T.lsa[v]) {
      if (l.type != P2P) continue;
      for (const auto &e : V[v].exits)
        if (e.outIf >= 0) host.push_back({l.linkData, e.nextHop, e.outIf});
    }
  }
  // SPFProcessStubs / SPFIntraAddStub (:1654-1818)
  void stubs(int v) {
    if (v != (int)root) {
      for (const auto &l : T.lsa[v]) {
        if (l.type != STUB) continue;
        const uint32_t mask = l.linkData, netw = l.linkId & mask;
        for (const auto &e : V[v].exits)
          if (e.outIf >= 0) net.push_back({netw, mask, e.nextHop, e.outIf});
      }
    }
    for (int c : V[v].children) {
      if (!V[c].processed) {
        stubs(c);
        V[c].processed = true;
      }
    }
  }
  // CheckForStubNode (:1245-1323)
  bool stub_root() {
    int transits = 0;
    const LinkRecord *tl = nullptr;
    for (const auto &l : T.lsa[root])
      if (l.type == P2P || l.type == TRANSIT) {
        ++transits;
        tl = &l;
      }
    if (transits == 0) return true;
    if (transits == 1 && tl->type == P2P) {
      for (const auto &lr : T.lsa[tl->linkId]) {
        if (lr.type != P2P) continue;
        if (lr.linkId == root) {
          net.push_back({0u, 0u, lr.linkData, find_if(tl->linkData)});  // AddNetworkRouteTo (0.0.0.0/0)
          return true;
        }
      }
    }
    return false;
  }
  // SPFCalculate (:1327-1490)
  void run() {
    V[root].dist = 0;
    status[root] = IN_SPFTREE;
    if (stub_root()) return;
    int v = (int)root;
    for (;;) {
      next(v);
      if (cand.empty()) break;
      v = cand.front();
      cand.pop_front();
      status[v] = IN_SPFTREE;
      for (int p : V[v].parents) V[p].children.push_back(v);  // SPFVertexAddParent
      add_router(v);
    }
    stubs((int)root);
  }
  // Ipv4GlobalRouting::RouteInput local check + LookupGlobal (first match)
  int32_t lookup(uint32_t dest) const {
    for (const auto &a : T.ifaddr[root])
      if (a.first == dest) return -2;  // local delivery
    for (const auto &h : host)
      if (h.dest == dest) return h.iface;
    for (const auto &r : net)
      if ((dest & r.mask) == (r.net & r.mask)) return r.iface;
    return -1;
  }
};

}  // namespace

extern "C" int nsref_global_routes(uint32_t n_nodes, uint32_t n_devices, const uint32_t *dev_node,
                                   const uint32_t *dev_peer, const uint32_t *dev_addr, const uint32_t *dev_mask,
                                   const uint32_t *dev_ifindex, uint32_t n_dst, const uint32_t *dst_addr,
                                   uint32_t *route_out) {
  Topo T;
  T.n = n_nodes;
  T.lsa.resize(n_nodes);
  T.ifaddr.resize(n_nodes);
  T.if_dev.resize(n_nodes);
  // interfaces: loopback 0, then the p2p devices by their interface index (Ipv4AddressHelper::Assign order)
  std::vector<uint32_t> nif(n_nodes, 1);
  for (uint32_t d = 0; d < n_devices; ++d) nif[dev_node[d]] = std::max(nif[dev_node[d]], dev_ifindex[d] + 1);
  for (uint32_t n = 0; n < n_nodes; ++n) {
    T.ifaddr[n].assign(nif[n], {0u, 0u});
    T.if_dev[n].assign(nif[n], -1);
    T.ifaddr[n][0] = {0x7f000001u, 0xff000000u};
  }
  for (uint32_t d = 0; d < n_devices; ++d) {
    const uint32_t n = dev_node[d], i = dev_ifindex[d];
    if (i == 0 || i >= nif[n]) return -1;
    T.ifaddr[n][i] = {dev_addr[d], dev_mask[d]};
    T.if_dev[n][i] = (int32_t)d;
  }
  // router-LSAs: devices in node order (ascending device index = Node::AddDevice order), then loopback
  for (uint32_t d = 0; d < n_devices; ++d) {
    const uint32_t n = dev_node[d], p = dev_peer[d];
    T.lsa[n].push_back({P2P, dev_node[p], dev_addr[d], 1u});
    T.lsa[n].push_back({STUB, dev_addr[p], dev_mask[p], 1u});
  }
  for (uint32_t n = 0; n < n_nodes; ++n) T.lsa[n].push_back({STUB, 0x7f000000u, 0xff000000u, 1u});
  for (uint32_t r = 0; r < n_nodes; ++r) {
    Spf s(T, r);
    s.run();
    for (uint32_t k = 0; k < n_dst; ++k) {
      const int32_t i = s.lookup(dst_addr[k]);
      uint32_t out = 0xffffffffu;  // no route
      if (i == -2) out = 0xfffffffeu;  // local
      else if (i >= 0) out = T.if_dev[r][i] < 0 ? 0xffffffffu : (uint32_t)T.if_dev[r][i];
      route_out[(uint64_t)r * n_dst + k] = out;
    }
  }
  return 0;
}
