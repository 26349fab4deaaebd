/* -*- Mode:C++; c-file-style:"gnu"; indent-tabs-mode:nil; -*- */
#include "nsgpu-p2p-scenario.h"
#include "ns3/fatal-error.h"
#include <algorithm>

namespace ns3 {

NsgpuP2pScenario::NsgpuP2pScenario ()
  : m_nodes (0),
    m_nDst (0),
    m_icmp (true),
    m_stop (-1),
    m_firstLink (true),
    m_engine (0)
{
}

NsgpuP2pScenario::~NsgpuP2pScenario ()
{
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
  App a = {NSGPU_APP_SINK, node, 0, 0, 0, 0, start.GetTimeStep (), stop.GetTimeStep (), 0, 0.0, 0.0};
  return AddApp (a);
}

uint32_t
NsgpuP2pScenario::AddOnOff (uint32_t node, uint32_t dstNode, Time start, Time stop, uint64_t rateBps,
                            uint32_t packetSize, double onSeconds, double offSeconds, uint32_t maxBytes, uint32_t ttl)
{
  App a = {NSGPU_APP_ONOFF, node, dstNode, packetSize, maxBytes, ttl, start.GetTimeStep (), stop.GetTimeStep (),
           rateBps, onSeconds, offSeconds};
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

void
NsgpuP2pScenario::PopulateRoutingTables (void)
{
  m_dstSlot.assign (m_nodes, 0xffffffffu);
  m_nDst = 0;
  for (size_t i = 0; i < m_app.size (); i++)
    {
      if (m_app[i].kind == NSGPU_APP_ONOFF)
        {
          m_dstSlot[m_app[i].dst] = 0;  // mark; numbered below in node order
          if (m_icmp)
            {
              m_dstSlot[m_app[i].node] = 0;  // an ICMP error goes back to the sender
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

nsgpu_p2p *
NsgpuP2pScenario::CreateEngine (uint64_t poolCap, uint64_t logCap)
{
  if (m_route.empty ())
    {
      RouteShortestPaths ();
    }
  const size_t D = m_dev.size (), A = m_app.size ();
  std::vector<uint32_t> devNode (D), devPeer (D), devQmax (D);
  std::vector<uint64_t> devBps (D);
  std::vector<int64_t> devIfg (D), devDelay (D);
  for (size_t d = 0; d < D; d++)
    {
      devNode[d] = m_dev[d].node, devPeer[d] = m_dev[d].peer, devQmax[d] = m_dev[d].qmax;
      devBps[d] = m_dev[d].bps, devIfg[d] = m_dev[d].ifg, devDelay[d] = m_dev[d].delay;
    }
  std::vector<uint32_t> kind (A), node (A), dst (A), slot (A), src (A), size (A), maxb (A), ttl (A), zero (A, 0);
  std::vector<int64_t> start (A), stop (A), ivl (A, 0);
  std::vector<uint64_t> rate (A);
  std::vector<double> on (A), off (A);
  for (size_t i = 0; i < A; i++)
    {
      const App &a = m_app[i];
      kind[i] = a.kind, node[i] = a.node, dst[i] = a.dst, size[i] = a.size, maxb[i] = a.maxBytes, ttl[i] = a.ttl;
      slot[i] = a.kind == NSGPU_APP_ONOFF ? m_dstSlot[a.dst] : 0;
      src[i] = a.kind == NSGPU_APP_ONOFF ? m_dstSlot[a.node] : 0xffffffffu;
      start[i] = a.start, stop[i] = a.stop, rate[i] = a.rate, on[i] = a.on, off[i] = a.off;
    }
  std::vector<uint32_t> sk (m_setup.size ()), si (m_setup.size ());
  for (size_t i = 0; i < m_setup.size (); i++)
    {
      sk[i] = m_setup[i].first, si[i] = m_setup[i].second;
    }
  nsgpu_p2p_scenario sc = nsgpu_p2p_scenario ();
  sc.n_nodes = m_nodes;
  sc.n_devices = D;
  sc.n_apps = A;
  sc.n_dst = std::max (m_nDst, 1u);
  sc.dev_node = &devNode[0], sc.dev_peer = &devPeer[0], sc.dev_bps = &devBps[0];
  sc.dev_ifg_ns = &devIfg[0], sc.dev_delay_ns = &devDelay[0], sc.dev_qmax = &devQmax[0];
  sc.route = &m_route[0];
  sc.app_kind = &kind[0], sc.app_node = &node[0], sc.app_start_ns = &start[0], sc.app_stop_ns = &stop[0];
  sc.app_dst_node = &dst[0], sc.app_dst_slot = &slot[0], sc.app_rate_bps = &rate[0], sc.app_pkt_size = &size[0];
  sc.app_on_s = &on[0], sc.app_off_s = &off[0], sc.app_max_bytes = &maxb[0], sc.app_ttl = &ttl[0];
  sc.app_count = &zero[0], sc.app_interval_ns = &ivl[0], sc.app_src_slot = &src[0];
  sc.stop_ns = m_stop;
  sc.icmp = m_icmp ? 1u : 0u;
  sc.n_setup = m_setup.size ();
  sc.setup_kind = &sk[0];
  sc.setup_index = &si[0];
  if (nsgpu_p2p_create (&sc, poolCap, logCap, &m_engine) != NSGPU_OK ||
      nsgpu_p2p_reset (m_engine, 0) != NSGPU_OK)
    {
      NS_FATAL_ERROR ("libnsgpu: " << nsgpu_last_error ());
    }
  return m_engine;
}

} // namespace ns3
