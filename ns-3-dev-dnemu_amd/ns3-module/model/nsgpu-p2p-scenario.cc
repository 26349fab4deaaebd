/* -*- Mode:C++; c-file-style:"gnu"; indent-tabs-mode:nil; -*- */
#include "nsgpu-p2p-scenario.h"
#include "ns3/fatal-error.h"
#include "ns3/node-list.h"
#include "ns3/node.h"
#include "ns3/application.h"
#include "ns3/point-to-point-net-device.h"
#include "ns3/point-to-point-channel.h"
#include "ns3/loopback-net-device.h"
#include "ns3/drop-tail-queue.h"
#include "ns3/ipv4.h"
#include "ns3/ipv4-l3-protocol.h"
#include "ns3/ipv4-list-routing.h"
#include "ns3/ipv4-static-routing.h"
#include "ns3/ipv4-global-routing.h"
#include "ns3/ipv4-routing-table-entry.h"
#include "ns3/onoff-application.h"
#include "ns3/packet-sink.h"
#include "ns3/udp-echo-client.h"
#include "ns3/udp-echo-server.h"
#include "ns3/inet-socket-address.h"
#include "ns3/address.h"
#include "ns3/uinteger.h"
#include "ns3/enum.h"
#include "ns3/data-rate.h"
#include "ns3/random-variable.h"
#include "ns3/output-stream-wrapper.h"
#include "ns3/pcap-file-wrapper.h"
#include "ns3/trace-helper.h"
#include <algorithm>
#include <cstdlib>
#include <map>
#include <sstream>

namespace ns3 {

#define NSGPU_TRY(call)                                                     \
  do {                                                                      \
      if ((call) != NSGPU_OK)                                               \
        {                                                                   \
          NS_FATAL_ERROR ("libnsgpu: " << nsgpu_last_error ());             \
        }                                                                   \
    } while (false)

NsgpuP2pScenario::NsgpuP2pScenario ()
  : m_nodes (0),
    m_nDst (0),
    m_icmp (true),
    m_stop (-1),
    m_firstLink (true),
    m_engine (0),
    m_codec (0)
{
}

NsgpuP2pScenario::~NsgpuP2pScenario ()
{
  if (m_codec != 0)
    {
      nsgpu_trace_codec_free (m_codec);
    }
  if (m_engine != 0)
    {
      nsgpu_p2p_destroy (m_engine);
    }
}

uint32_t
NsgpuP2pScenario::AddNode (void)
{
  if (m_nodes == 0)
    {
      m_setup.push_back (std::make_pair ((uint32_t) NSGPU_SETUP_UID, 0u));  // NodeListPriv's ScheduleDestroy
    }
  m_setup.push_back (std::make_pair ((uint32_t) NSGPU_SETUP_NODE, m_nodes));
  return m_nodes++;
}

std::pair<uint32_t, uint32_t>
NsgpuP2pScenario::Link (uint32_t a, uint32_t b, uint64_t bps, Time delay, uint32_t queueMaxPackets, Time interframeGap)
{
  const uint32_t da = m_dev.size (), db = da + 1;
  Dev x = {a, db, queueMaxPackets, bps, interframeGap.GetTimeStep (), delay.GetTimeStep ()};
  Dev y = {b, da, queueMaxPackets, bps, interframeGap.GetTimeStep (), delay.GetTimeStep ()};
  m_dev.push_back (x);
  m_setup.push_back (std::make_pair ((uint32_t) NSGPU_SETUP_DEVICE, da));
  m_dev.push_back (y);
  m_setup.push_back (std::make_pair ((uint32_t) NSGPU_SETUP_DEVICE, db));
  m_addr.resize (m_dev.size (), 0u);
  m_ifindex.resize (m_dev.size (), 0u);
  if (m_firstLink)
    {
      m_setup.push_back (std::make_pair ((uint32_t) NSGPU_SETUP_UID, 0u));  // ChannelListPriv's ScheduleDestroy
      m_firstLink = false;
    }
  return std::make_pair (da, db);
}

void
NsgpuP2pScenario::InstallStack (void)
{
  for (uint32_t n = 0; n < m_nodes; n++)
    {
      m_setup.push_back (std::make_pair ((uint32_t) NSGPU_SETUP_NOOP, n));  // LoopbackNetDevice
    }
}

uint32_t
NsgpuP2pScenario::AddApp (const App &a)
{
  m_app.push_back (a);
  m_setup.push_back (std::make_pair ((uint32_t) NSGPU_SETUP_APP, (uint32_t) (m_app.size () - 1)));
  return m_app.size () - 1;
}

uint32_t
NsgpuP2pScenario::AddPacketSink (uint32_t node, Time start, Time stop)
{
  App a = {NSGPU_APP_SINK, node, 0, 0, 0, 0, start.GetTimeStep (), stop.GetTimeStep (), 0, 0.0, 0.0, 0, 0, 0, 0};
  return AddApp (a);
}

uint32_t
NsgpuP2pScenario::AddOnOff (uint32_t node, uint32_t dstNode, Time start, Time stop, uint64_t rateBps,
                            uint32_t packetSize, double onSeconds, double offSeconds, uint32_t maxBytes, uint32_t ttl)
{
  App a = {NSGPU_APP_ONOFF, node, dstNode, packetSize, maxBytes, ttl, start.GetTimeStep (), stop.GetTimeStep (),
           rateBps, onSeconds, offSeconds, 0, 0, 0, 9};
  return AddApp (a);
}

void
NsgpuP2pScenario::Stop (Time at)
{
  m_stop = at.GetTimeStep ();
  m_setup.push_back (std::make_pair ((uint32_t) NSGPU_SETUP_STOP, 0u));
}

void
NsgpuP2pScenario::Assign (uint32_t da, uint32_t db, uint32_t network, uint32_t mask)
{
  m_nif.resize (m_nodes, 1u);
  const uint32_t d[2] = {da, db};
  for (int k = 0; k < 2; k++)
    {
      m_addr[d[k]] = (network & mask) + 1 + k;
      m_ifindex[d[k]] = m_nif[m_dev[d[k]].node]++;
    }
}

void
NsgpuP2pScenario::SetIcmp (bool on)
{
  m_icmp = on;
}

namespace {
/* ConstantVariable (v) prints as "Constant:v" (random-variable.cc:1931-1940); anything else draws from a
 * random stream, which the GPU-resident OnOff cannot */
double
ConstantSeconds (const RandomVariable &v, const char *what, uint32_t node)
{
  std::ostringstream os;
  os << v;
  const std::string s = os.str ();
  if (s.compare (0, 9, "Constant:") != 0)
    {
      NS_FATAL_ERROR ("NsgpuP2pScenario::FromNodeList: node " << node << ": OnOffApplication " << what << " is " << s
                      << ", not a ConstantVariable");
    }
  return std::strtod (s.c_str () + 9, 0);
}

Time
TimeAttribute (Ptr<Object> o, const char *name)
{
  TimeValue v;
  o->GetAttribute (name, v);
  return v.Get ();
}

uint32_t
UintAttribute (Ptr<Object> o, const char *name)
{
  UintegerValue v;
  o->GetAttribute (name, v);
  return (uint32_t) v.Get ();
}
/* The engine forwards along global routing's choices (PopulateRoutingTables + LookupGlobal, computed by
 * nsgpu_route_global): a node's Ipv4 must route through an Ipv4GlobalRouting in its Ipv4ListRouting (the
 * InternetStackHelper default, static priority 0 + global -10), with no static route of its own beyond the
 * interfaces' directly connected networks (Ipv4StaticRouting::NotifyInterfaceUp adds those; any other static
 * route would win over global routing) */
void
CheckGlobalRouting (Ptr<Ipv4> ip, uint32_t node)
{
  Ptr<Ipv4ListRouting> list = DynamicCast<Ipv4ListRouting> (ip->GetRoutingProtocol ());
  if (list == 0)
    {
      NS_FATAL_ERROR ("NsgpuP2pScenario::FromNodeList: node " << node << "'s Ipv4 routing is not an Ipv4ListRouting "
                      "(the engine models global routing)");
    }
  bool global = false;
  for (uint32_t i = 0; i < list->GetNRoutingProtocols (); i++)
    {
      int16_t priority;
      Ptr<Ipv4RoutingProtocol> rp = list->GetRoutingProtocol (i, priority);
      if (DynamicCast<Ipv4GlobalRouting> (rp) != 0)
        {
          global = true;
          continue;
        }
      Ptr<Ipv4StaticRouting> st = DynamicCast<Ipv4StaticRouting> (rp);
      if (st == 0)
        {
          NS_FATAL_ERROR ("NsgpuP2pScenario::FromNodeList: node " << node << " runs a routing protocol other than "
                          "static / global routing (not in the GPU-resident subset)");
        }
      for (uint32_t r = 0; r < st->GetNRoutes (); r++)
        {
          Ipv4RoutingTableEntry e = st->GetRoute (r);
          // the routes Ipv4StaticRouting adds by itself (ipv4-static-routing.cc NotifyInterfaceUp /
          // NotifyAddAddress): each interface address's own network on that interface, gateway-less.  Any other
          // route, gateway-less ones included (AddHostRouteTo (dst, if), AddNetworkRouteTo (net, mask, if)), is
          // consulted before global routing (priority 0 > -10) and would override the paths the engine models.
          bool own = false;
          if (e.GetGateway () == Ipv4Address::GetZero () && !e.IsDefault () && e.GetInterface () < ip->GetNInterfaces ())
            {
              for (uint32_t a = 0; a < ip->GetNAddresses (e.GetInterface ()) && !own; a++)
                {
                  Ipv4InterfaceAddress ia = ip->GetAddress (e.GetInterface (), a);
                  own = e.GetDestNetworkMask () == ia.GetMask ()
                        && e.GetDestNetwork () == ia.GetLocal ().CombineMask (ia.GetMask ());
                }
            }
          if (!own)
            {
              NS_FATAL_ERROR ("NsgpuP2pScenario::FromNodeList: node " << node << " holds the static route " << e
                              << " (the engine models global routing only)");
            }
        }
    }
  if (!global)
    {
      NS_FATAL_ERROR ("NsgpuP2pScenario::FromNodeList: node " << node << " has no Ipv4GlobalRouting");
    }
}
} // anonymous namespace

void
NsgpuP2pScenario::FromNodeList (Ptr<HipSimulatorImpl> impl)
{
  if (m_nodes != 0 || !m_setup.empty ())
    {
      NS_FATAL_ERROR ("NsgpuP2pScenario::FromNodeList: the scenario is not empty");
    }
  const uint32_t N = NodeList::GetNNodes ();
  m_nodes = N;
  // ---- the node list: each node's devices (in AddDevice order) and application count ----
  std::vector<uint64_t> devOff (N + 1, 0);
  std::vector<uint32_t> devKind, nApps (N, 0);
  for (uint32_t n = 0; n < N; n++)
    {
      Ptr<Node> node = NodeList::GetNode (n);
      for (uint32_t i = 0; i < node->GetNDevices (); i++)
        {
          Ptr<NetDevice> d = node->GetDevice (i);
          devKind.push_back (DynamicCast<PointToPointNetDevice> (d) != 0 ? (uint32_t) NSGPU_NDEV_P2P
                             : DynamicCast<LoopbackNetDevice> (d) != 0 ? (uint32_t) NSGPU_NDEV_LOOPBACK
                             : (uint32_t) NSGPU_NDEV_OTHER);
        }
      devOff[n + 1] = devKind.size ();
      nApps[n] = node->GetNApplications ();
    }
  // ---- the setup list from the journal (uid order; classified by HipSimulatorImpl when each call was made) ----
  const std::vector<HipSimulatorImpl::SetupCall> &J = impl->GetSetupJournal ();
  const size_t nj = J.size ();
  std::vector<nsgpu_journal_entry> journal (std::max (nj, (size_t) 1));
  for (size_t i = 0; i < nj; i++)
    {
      journal[i].ts = J[i].ts;
      journal[i].context = J[i].context;
      journal[i].kind = J[i].kind;
      journal[i].local = J[i].local;
      journal[i].pad_ = 0;
    }
  size_t nApp = 0;
  for (uint32_t n = 0; n < N; n++)
    {
      nApp += nApps[n];
    }
  std::vector<uint32_t> sk (journal.size ()), si (journal.size ()), owned (journal.size ());
  std::vector<uint32_t> dNode (std::max (devKind.size (), (size_t) 1)), dLocal (dNode.size ());
  std::vector<uint32_t> aNode (std::max (nApp, (size_t) 1)), aLocal (aNode.size ());
  nsgpu_setup_map map;
  map.setup_kind = &sk[0], map.setup_index = &si[0], map.owned = &owned[0];
  map.dev_node = &dNode[0], map.dev_local = &dLocal[0], map.app_node = &aNode[0], map.app_local = &aLocal[0];
  map.n_owned = 0, map.n_devices = 0, map.n_apps = 0, map.stop_ns = -1;
  NSGPU_TRY (nsgpu_setup_from_journal (&journal[0], nj, N, &devOff[0], devKind.empty () ? 0 : &devKind[0], N ? &nApps[0] : 0,
                                       &map));
  for (size_t i = 0; i < nj; i++)
    {
      m_setup.push_back (std::make_pair (sk[i], si[i]));
    }
  m_owned.assign (owned.begin (), owned.begin () + map.n_owned);
  m_stop = map.stop_ns;
  std::map<Ptr<NetDevice>, uint32_t> devIndex;
  std::vector<Ptr<NetDevice> > devs;    // engine device index -> object
  std::vector<Ptr<Application> > apps;  // engine application index -> object
  for (uint32_t d = 0; d < map.n_devices; d++)
    {
      devs.push_back (NodeList::GetNode (dNode[d])->GetDevice (dLocal[d]));
      devIndex[devs[d]] = d;
      m_devObj.push_back (devs[d]);
    }
  for (uint32_t a = 0; a < map.n_apps; a++)
    {
      apps.push_back (NodeList::GetNode (aNode[a])->GetApplication (aLocal[a]));
    }
  // ---- device parameters ----
  const uint32_t D = devs.size ();
  m_dev.resize (D);
  m_addr.assign (D, 0u);
  m_ifindex.assign (D, 0u);
  for (uint32_t d = 0; d < D; d++)
    {
      Ptr<PointToPointNetDevice> p = DynamicCast<PointToPointNetDevice> (devs[d]);
      Ptr<PointToPointChannel> ch = DynamicCast<PointToPointChannel> (p->GetChannel ());
      if (ch == 0 || ch->GetNDevices () != 2)
        {
          NS_FATAL_ERROR ("NsgpuP2pScenario::FromNodeList: device " << d << " has no point-to-point channel");
        }
      Ptr<NetDevice> other = ch->GetDevice (0) == devs[d] ? ch->GetDevice (1) : ch->GetDevice (0);
      if (devIndex.find (other) == devIndex.end ())
        {
          NS_FATAL_ERROR ("NsgpuP2pScenario::FromNodeList: device " << d << "'s peer is not in the subset");
        }
      Ptr<DropTailQueue> q = DynamicCast<DropTailQueue> (p->GetQueue ());
      if (q == 0)
        {
          NS_FATAL_ERROR ("NsgpuP2pScenario::FromNodeList: device " << d << "'s TxQueue is not a DropTailQueue");
        }
      EnumValue mode;
      q->GetAttribute ("Mode", mode);
      if (mode.Get () != DropTailQueue::PACKETS)
        {
          NS_FATAL_ERROR ("NsgpuP2pScenario::FromNodeList: device " << d << "'s DropTailQueue is not in PACKETS mode");
        }
      if (UintAttribute (p, "Mtu") != 1500)
        {
          // the engine forwards whole datagrams up to 1500 bytes (no Ipv4L3Protocol fragmentation, ipv4-l3-protocol.cc:722)
          NS_FATAL_ERROR ("NsgpuP2pScenario::FromNodeList: device " << d << "'s Mtu is " << UintAttribute (p, "Mtu")
                          << ", not 1500");
        }
      DataRateValue rate;
      p->GetAttribute ("DataRate", rate);
      Dev x = {devs[d]->GetNode ()->GetId (), devIndex[other], UintAttribute (q, "MaxPackets"), rate.Get ().GetBitRate (),
               TimeAttribute (p, "InterframeGap").GetTimeStep (), TimeAttribute (ch, "Delay").GetTimeStep ()};
      m_dev[d] = x;
    }
  // ---- Ipv4: interface addresses and indices, DefaultTtl ----
  std::vector<uint32_t> ttl (N, 64);
  std::map<uint32_t, uint32_t> nodeOfAddr;
  for (uint32_t n = 0; n < N; n++)
    {
      Ptr<Ipv4> ip = NodeList::GetNode (n)->GetObject<Ipv4> ();
      if (ip == 0)
        {
          continue;
        }
      for (uint32_t i = 0; i < ip->GetNInterfaces (); i++)
        {
          Ptr<NetDevice> nd = ip->GetNetDevice (i);
          if (ip->GetNAddresses (i) == 0 || devIndex.find (nd) == devIndex.end ())
            {
              continue;
            }
          const uint32_t a = ip->GetAddress (i, 0).GetLocal ().Get ();
          m_addr[devIndex[nd]] = a;
          m_ifindex[devIndex[nd]] = i;
          nodeOfAddr[a] = n;
        }
      CheckGlobalRouting (ip, n);
      Ptr<Ipv4L3Protocol> l3 = DynamicCast<Ipv4L3Protocol> (ip);
      if (l3 != 0)
        {
          ttl[n] = UintAttribute (l3, "DefaultTtl");
        }
    }
  // ---- applications ----
  for (uint32_t a = 0; a < apps.size (); a++)
    {
      Ptr<Application> o = apps[a];
      const uint32_t n = o->GetNode ()->GetId ();
      App x = {0, n, 0, 0, 0, ttl[n], TimeAttribute (o, "StartTime").GetTimeStep (),
               TimeAttribute (o, "StopTime").GetTimeStep (), 0, 0.0, 0.0, 0, 0, 0, 0};
      uint32_t remote = 0;
      if (DynamicCast<OnOffApplication> (o) != 0)
        {
          x.kind = NSGPU_APP_ONOFF;
          DataRateValue rate;
          o->GetAttribute ("DataRate", rate);
          x.rate = rate.Get ().GetBitRate ();
          x.size = UintAttribute (o, "PacketSize");
          x.maxBytes = UintAttribute (o, "MaxBytes");
          RandomVariableValue on, off;
          o->GetAttribute ("OnTime", on);
          o->GetAttribute ("OffTime", off);
          x.on = ConstantSeconds (on.Get (), "OnTime", n);
          x.off = ConstantSeconds (off.Get (), "OffTime", n);
          AddressValue peer;
          o->GetAttribute ("Remote", peer);
          if (!InetSocketAddress::IsMatchingType (peer.Get ()))
            {
              NS_FATAL_ERROR ("NsgpuP2pScenario::FromNodeList: OnOffApplication on node " << n << ": Remote is not "
                              "an InetSocketAddress");
            }
          const InetSocketAddress s = InetSocketAddress::ConvertFrom (peer.Get ());
          remote = s.GetIpv4 ().Get ();
          x.remotePort = s.GetPort ();
        }
      else if (DynamicCast<UdpEchoClient> (o) != 0)
        {
          x.kind = NSGPU_APP_ECHO_CLIENT;
          x.size = UintAttribute (o, "PacketSize");
          x.count = UintAttribute (o, "MaxPackets");
          x.interval = TimeAttribute (o, "Interval").GetTimeStep ();
          Ipv4AddressValue ra;
          o->GetAttribute ("RemoteAddress", ra);
          remote = ra.Get ().Get ();
          x.remotePort = UintAttribute (o, "RemotePort");
        }
      else if (DynamicCast<UdpEchoServer> (o) != 0)
        {
          x.kind = NSGPU_APP_ECHO_SERVER;
        }
      else if (DynamicCast<PacketSink> (o) != 0)
        {
          x.kind = NSGPU_APP_SINK;
        }
      else
        {
          NS_FATAL_ERROR ("NsgpuP2pScenario::FromNodeList: node " << n << " application " << a
                          << " is not OnOff / PacketSink / UdpEcho (not in the GPU-resident subset)");
        }
      if (x.kind == NSGPU_APP_ONOFF || x.kind == NSGPU_APP_ECHO_CLIENT)
        {
          if (nodeOfAddr.find (remote) == nodeOfAddr.end ())
            {
              NS_FATAL_ERROR ("NsgpuP2pScenario::FromNodeList: node " << n << " sends to an address no node has");
            }
          x.dst = nodeOfAddr[remote];
          x.remoteAddr = remote;
        }
      m_app.push_back (x);
    }
}

void
NsgpuP2pScenario::PopulateRoutingTables (void)
{
  m_dstSlot.assign (m_nodes, 0xffffffffu);
  m_nDst = 0;
  for (size_t i = 0; i < m_app.size (); i++)
    {
      if (m_app[i].kind == NSGPU_APP_ONOFF || m_app[i].kind == NSGPU_APP_ECHO_CLIENT)
        {
          m_dstSlot[m_app[i].dst] = 0;  // mark; numbered below in node order
          if (m_icmp || m_app[i].kind == NSGPU_APP_ECHO_CLIENT)
            {
              m_dstSlot[m_app[i].node] = 0;  // an ICMP error / an echo goes back to the sender
            }
        }
    }
  std::vector<uint32_t> dst;
  for (uint32_t n = 0; n < m_nodes; n++)
    {
      if (m_dstSlot[n] != 0xffffffffu)
        {
          m_dstSlot[n] = m_nDst++;
          dst.push_back (n);
        }
    }
  const size_t D = m_dev.size ();
  std::vector<uint32_t> devNode (D), devPeer (D);
  bool addressed = D > 0;
  for (size_t d = 0; d < D; d++)
    {
      devNode[d] = m_dev[d].node, devPeer[d] = m_dev[d].peer;
      addressed = addressed && m_addr[d] != 0;
    }
  m_route.assign ((size_t) m_nodes * std::max (m_nDst, 1u), 0xffffffffu);
  if (m_nDst > 0 && nsgpu_route_global (m_nodes, D, &devNode[0], &devPeer[0], addressed ? &m_addr[0] : 0,
                                        addressed ? &m_ifindex[0] : 0, m_nDst, &dst[0], &m_route[0], 0) != NSGPU_OK)
    {
      NS_FATAL_ERROR ("libnsgpu: " << nsgpu_last_error ());
    }
}

void
NsgpuP2pScenario::Fill (void)
{
  if (m_route.empty ())
    {
      RouteShortestPaths ();
    }
  const size_t D = m_dev.size (), A = m_app.size ();
  m_cDevNode.resize (D), m_cDevPeer.resize (D), m_cDevQmax.resize (D);
  m_cDevBps.resize (D), m_cDevIfg.resize (D), m_cDevDelay.resize (D);
  for (size_t d = 0; d < D; d++)
    {
      m_cDevNode[d] = m_dev[d].node, m_cDevPeer[d] = m_dev[d].peer, m_cDevQmax[d] = m_dev[d].qmax;
      m_cDevBps[d] = m_dev[d].bps, m_cDevIfg[d] = m_dev[d].ifg, m_cDevDelay[d] = m_dev[d].delay;
    }
  const size_t A1 = std::max (A, (size_t) 1);
  m_cKind.assign (A1, 0), m_cNode.assign (A1, 0), m_cDst.assign (A1, 0), m_cSlot.assign (A1, 0);
  m_cSrc.assign (A1, 0xffffffffu), m_cSize.assign (A1, 0), m_cMaxb.assign (A1, 0), m_cTtl.assign (A1, 0);
  m_cCount.assign (A1, 0), m_cRaddr.assign (A1, 0), m_cRport.assign (A1, 0);
  m_cStart.assign (A1, 0), m_cStop.assign (A1, 0), m_cIvl.assign (A1, 0), m_cRate.assign (A1, 0);
  m_cOn.assign (A1, 0.0), m_cOff.assign (A1, 0.0);
  for (size_t i = 0; i < A; i++)
    {
      const App &a = m_app[i];
      const bool sender = a.kind == NSGPU_APP_ONOFF || a.kind == NSGPU_APP_ECHO_CLIENT;
      m_cKind[i] = a.kind, m_cNode[i] = a.node, m_cDst[i] = a.dst, m_cSize[i] = a.size, m_cMaxb[i] = a.maxBytes;
      m_cTtl[i] = a.ttl, m_cCount[i] = a.count, m_cIvl[i] = a.interval, m_cRaddr[i] = a.remoteAddr;
      m_cRport[i] = a.remotePort;
      m_cSlot[i] = sender ? m_dstSlot[a.dst] : 0;
      m_cSrc[i] = sender ? m_dstSlot[a.node] : 0xffffffffu;
      m_cStart[i] = a.start, m_cStop[i] = a.stop, m_cRate[i] = a.rate, m_cOn[i] = a.on, m_cOff[i] = a.off;
    }
  m_cSk.resize (m_setup.size ()), m_cSi.resize (m_setup.size ());
  for (size_t i = 0; i < m_setup.size (); i++)
    {
      m_cSk[i] = m_setup[i].first, m_cSi[i] = m_setup[i].second;
    }
  nsgpu_p2p_scenario &sc = m_sc;
  sc = nsgpu_p2p_scenario ();
  sc.n_nodes = m_nodes;
  sc.n_devices = D;
  sc.n_apps = A;
  sc.n_dst = std::max (m_nDst, 1u);
  sc.dev_node = &m_cDevNode[0], sc.dev_peer = &m_cDevPeer[0], sc.dev_bps = &m_cDevBps[0];
  sc.dev_ifg_ns = &m_cDevIfg[0], sc.dev_delay_ns = &m_cDevDelay[0], sc.dev_qmax = &m_cDevQmax[0];
  sc.route = &m_route[0];
  sc.app_kind = &m_cKind[0], sc.app_node = &m_cNode[0], sc.app_start_ns = &m_cStart[0], sc.app_stop_ns = &m_cStop[0];
  sc.app_dst_node = &m_cDst[0], sc.app_dst_slot = &m_cSlot[0], sc.app_rate_bps = &m_cRate[0];
  sc.app_pkt_size = &m_cSize[0], sc.app_on_s = &m_cOn[0], sc.app_off_s = &m_cOff[0], sc.app_max_bytes = &m_cMaxb[0];
  sc.app_ttl = &m_cTtl[0], sc.app_count = &m_cCount[0], sc.app_interval_ns = &m_cIvl[0], sc.app_src_slot = &m_cSrc[0];
  sc.stop_ns = m_stop;
  sc.icmp = m_icmp ? 1u : 0u;
  sc.n_setup = m_setup.size ();
  sc.setup_kind = m_cSk.empty () ? 0 : &m_cSk[0];
  sc.setup_index = m_cSi.empty () ? 0 : &m_cSi[0];
}

nsgpu_p2p *
NsgpuP2pScenario::CreateEngine (uint64_t poolCap, uint64_t logCap)
{
  Fill ();
  if (nsgpu_p2p_create (&m_sc, poolCap, logCap, &m_engine) != NSGPU_OK ||
      nsgpu_p2p_reset (m_engine, 0) != NSGPU_OK)
    {
      NS_FATAL_ERROR ("libnsgpu: " << nsgpu_last_error ());
    }
  return m_engine;
}

void
NsgpuP2pScenario::AdoptInto (Ptr<HipSimulatorImpl> impl)
{
  if (m_engine == 0)
    {
      NS_FATAL_ERROR ("NsgpuP2pScenario::AdoptInto: CreateEngine first");
    }
  impl->AdoptDeviceSubset (m_engine, m_owned);
}

void
NsgpuP2pScenario::EnableTraceRecords (uint64_t capacity)
{
  if (m_engine == 0)
    {
      NS_FATAL_ERROR ("NsgpuP2pScenario::EnableTraceRecords: CreateEngine first");
    }
  NSGPU_TRY (nsgpu_p2p_set_trace (m_engine, capacity));
  NSGPU_TRY (nsgpu_p2p_reset (m_engine, 0));
}

void
NsgpuP2pScenario::WriteTraces (Ptr<OutputStreamWrapper> ascii, std::string pcapPrefix)
{
  if (m_engine == 0)
    {
      NS_FATAL_ERROR ("NsgpuP2pScenario::WriteTraces: CreateEngine first");
    }
  if (m_codec == 0)
    {
      nsgpu_trace_addressing ad;
      ad.dev_addr = m_addr.empty () ? 0 : &m_addr[0];
      ad.dev_ip_ifindex = m_ifindex.empty () ? 0 : &m_ifindex[0];
      ad.app_remote_addr = &m_cRaddr[0];
      ad.app_remote_port = &m_cRport[0];
      NSGPU_TRY (nsgpu_trace_codec_create (&m_sc, &ad, &m_codec));
    }
  uint64_t n = 0;
  NSGPU_TRY (nsgpu_p2p_trace_read (m_engine, 0, 0, &n, 0));
  std::vector<nsgpu_trace_record> rec (std::max (n, (uint64_t) 1));
  NSGPU_TRY (nsgpu_p2p_trace_read (m_engine, &rec[0], n, &n, 0));
  NSGPU_TRY (nsgpu_trace_sort (&rec[0], n));
  std::vector<char> line (512);
  std::vector<uint8_t> pkt (2048);
  if (ascii != 0)
    {
      std::ostream *os = ascii->GetStream ();
      for (uint64_t i = 0; i < n; i++)
        {
          uint64_t len = 0;
          NSGPU_TRY (nsgpu_trace_line (m_codec, &rec[i], 0, 0, &len));  // the size first (an ICMP line can exceed 512 B)
          if (len > line.size ())
            {
              line.resize (len);
            }
          NSGPU_TRY (nsgpu_trace_line (m_codec, &rec[i], &line[0], line.size (), &len));
          os->write (&line[0], (std::streamsize) len);
        }
    }
  if (!pcapPrefix.empty ())
    {
      // PointToPointHelper::EnablePcapInternal (point-to-point-helper.cc:81-110): one file per device,
      // PcapHelper::CreateFile (DLT_PPP), the PromiscSniffer's packets (after Dequeue, before MacRx)
      PcapHelper helper;
      // the device's NetDevice index on its node (Node::AddDevice order: the setup list's devices and loopbacks)
      std::vector<uint32_t> nxt (m_nodes, 0), devid (m_dev.size (), 0);
      for (size_t i = 0; i < m_setup.size (); i++)
        {
          if (m_setup[i].first == NSGPU_SETUP_DEVICE)
            {
              devid[m_setup[i].second] = nxt[m_dev[m_setup[i].second].node]++;
            }
          else if (m_setup[i].first == NSGPU_SETUP_NOOP)
            {
              nxt[m_setup[i].second]++;
            }
        }
      std::vector<Ptr<PcapFileWrapper> > files (m_dev.size ());
      for (uint32_t d = 0; d < m_dev.size (); d++)
        {
          // PcapHelper::GetFilenameFromDevice: <prefix>-<node id>-<device id>.pcap
          std::string fn;
          if (d < m_devObj.size () && m_devObj[d] != 0)
            {
              fn = helper.GetFilenameFromDevice (pcapPrefix, m_devObj[d]);
            }
          else
            {
              std::ostringstream name;
              name << pcapPrefix << "-" << m_dev[d].node << "-" << devid[d] << ".pcap";
              fn = name.str ();
            }
          files[d] = helper.CreateFile (fn, std::ios::out, PcapHelper::DLT_PPP);
        }
      for (uint64_t i = 0; i < n; i++)
        {
          if (rec[i].kind != NSGPU_TR_DEQUEUE && rec[i].kind != NSGPU_TR_RX)
            {
              continue;
            }
          uint64_t len = 0;
          NSGPU_TRY (nsgpu_trace_packet (m_codec, &rec[i], 0, 0, &len));
          if (len > pkt.size ())
            {
              pkt.resize (len);
            }
          NSGPU_TRY (nsgpu_trace_packet (m_codec, &rec[i], &pkt[0], pkt.size (), &len));
          files[rec[i].dev]->Write (TimeStep ((int64_t) rec[i].ts), &pkt[0], (uint32_t) len);
        }
    }
}

} // namespace ns3
