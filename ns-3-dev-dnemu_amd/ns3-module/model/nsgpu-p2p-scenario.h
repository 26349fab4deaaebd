/* -*- Mode:C++; c-file-style:"gnu"; indent-tabs-mode:nil; -*- */
/*
 * ns3::NsgpuP2pScenario — the GPU-resident point-to-point subset of an ns-3 program (include/nsgpu.h,
 * nsgpu_p2p_create), in the order the program builds it, so that the setup-time Schedule calls — and
 * therefore every uid — come out as the reference's (node-list.cc:124-131, node.cc:111-145,
 * point-to-point-helper.cc:228-242, ipv4-l3-protocol.cc:227-244).  Two ways to fill it:
 *   - FromNodeList: the program built its topology with the stock helpers (NodeContainer::Create,
 *     PointToPointHelper::Install, InternetStackHelper::Install, Ipv4AddressHelper::Assign, OnOffHelper /
 *     PacketSinkHelper / UdpEcho*Helper::Install, Simulator::Stop) under HipSimulatorImpl; the scenario is
 *     read back from NodeList, the devices' / channels' / queues' / applications' attributes and the Ipv4
 *     interfaces, and its setup list from HipSimulatorImpl's setup journal.  AdoptInto then hands the
 *     program's setup events to the engine (HipSimulatorImpl::AdoptDeviceSubset);
 *   - by hand: AddNode / Link / InstallStack / Assign / AddPacketSink / AddOnOff / Stop, in program order,
 *     then HipSimulatorImpl::AttachDeviceSubset before anything is scheduled.
 * WriteTraces hands the engine's trace records to the helpers' own sinks: the ascii lines to an
 * OutputStreamWrapper (AsciiTraceHelper), the pcap records to one PcapFileWrapper per device, created
 * and named as PointToPointHelper::EnablePcapAll names them (PcapHelper::GetFilenameFromDevice, DLT_PPP).
 * tests/ use the Python twin of this class (ns-3-dev-dnemu_amd/p2p.py).
 */
#ifndef NSGPU_P2P_SCENARIO_H
#define NSGPU_P2P_SCENARIO_H

#include "ns3/nstime.h"
#include "ns3/ptr.h"
#include "nsgpu.h"
#include "hip-simulator-impl.h"
#include <stdint.h>
#include <string>
#include <vector>
#include <utility>

namespace ns3 {

class OutputStreamWrapper;
class NetDevice;

class NsgpuP2pScenario
{
public:
  NsgpuP2pScenario ();
  ~NsgpuP2pScenario ();

  uint32_t AddNode (void);
  /* PointToPointHelper::Install (a, b): device on a, then device on b; returns both device indices */
  std::pair<uint32_t, uint32_t> Link (uint32_t a, uint32_t b, uint64_t bps, Time delay, uint32_t queueMaxPackets,
                                      Time interframeGap);
  void InstallStack (void);
  uint32_t AddPacketSink (uint32_t node, Time start, Time stop);
  uint32_t AddOnOff (uint32_t node, uint32_t dstNode, Time start, Time stop, uint64_t rateBps, uint32_t packetSize,
                     double onSeconds, double offSeconds, uint32_t maxBytes, uint32_t ttl);
  void Stop (Time at);
  /* Ipv4AddressHelper (network, mask).Assign on the two devices of a link (host .1 on a, .2 on b) and
   * Ipv4L3Protocol::AddInterface's interface numbering (the loopback is interface 0) */
  void Assign (uint32_t da, uint32_t db, uint32_t network, uint32_t mask = 0xffffff00u);
  /* InternetStackHelper installs Icmpv4L4Protocol: TTL expiries and unbound arrivals send ICMP errors back
   * to the sender (icmpv4-l4-protocol.cc:131-165).  On by default, as in the reference. */
  void SetIcmp (bool on);
  /* Ipv4GlobalRoutingHelper::PopulateRoutingTables on the GPU (nsgpu_route_global): next hops towards every
   * flow destination and, with ICMP, every sender.  With every device addressed the ties are global
   * routing's (lowest peer address, then interface); an unaddressed topology takes the lowest device. */
  void PopulateRoutingTables (void);
  void RouteShortestPaths (void) { PopulateRoutingTables (); }

  /* The scenario of the program's own topology: NodeList (node-list.cc), each node's devices in
   * Node::AddDevice order — PointToPointNetDevice DataRate / InterframeGap / TxQueue (DropTailQueue in
   * PACKETS mode: MaxPackets), its PointToPointChannel's Delay and peer; the LoopbackNetDevice — its Ipv4
   * interfaces (address, interface index), DefaultTtl, and its applications in Node::AddApplication order
   * (OnOffApplication DataRate / PacketSize / Remote / OnTime / OffTime (ConstantVariable) / MaxBytes,
   * PacketSink, UdpEchoServer Port, UdpEchoClient RemoteAddress / RemotePort / MaxPackets / Interval /
   * PacketSize; StartTime / StopTime).  The setup list follows `impl`'s journal: per node, its first
   * zero-delay call is Node::Start, the next ones its devices' NetDevice::Start then its applications'
   * Application::Start (the helpers add devices before applications); the Stop event; every other call
   * keeps its uid on the host (NSGPU_SETUP_UID).  Anything outside the GPU-resident subset (another device
   * type, a random OnTime, a sink on a second port of a node, ...) is a fatal error. */
  void FromNodeList (Ptr<HipSimulatorImpl> impl);
  /* The journal entries the engine dispatches from now on (FromNodeList) */
  const std::vector<uint32_t> &GetOwnedSetupCalls (void) const { return m_owned; }

  /* The engine (owned by this object); `poolCap` / `logCap` as nsgpu_p2p_create's */
  nsgpu_p2p *CreateEngine (uint64_t poolCap, uint64_t logCap);
  /* FromNodeList's engine joins impl's order: its setup events leave the host queue */
  void AdoptInto (Ptr<HipSimulatorImpl> impl);

  /* Record the device sinks' calls during Run (nsgpu_p2p_set_trace; call before Run), then, after it,
   * write them through the helpers' sinks: the EnableAsciiAll (stream) lines to `ascii` (null: none) and
   * the EnablePcapAll (prefix) files `pcapPrefix`-<node>-<device>.pcap (empty: none).  Lines and records
   * are in the dispatch order of the events that made them ((ts, uid), then call order). */
  void EnableTraceRecords (uint64_t capacity);
  void WriteTraces (Ptr<OutputStreamWrapper> ascii, std::string pcapPrefix);

private:
  struct Dev
  {
    uint32_t node, peer, qmax;
    uint64_t bps;
    int64_t ifg, delay;
  };
  struct App
  {
    uint32_t kind, node, dst, size, maxBytes, ttl;
    int64_t start, stop;
    uint64_t rate;
    double on, off;
    uint32_t count;        // UdpEchoClient MaxPackets
    int64_t interval;      // UdpEchoClient Interval
    uint32_t remoteAddr;   // the sender's Remote address (0: its destination's first interface)
    uint32_t remotePort;
  };
  uint32_t AddApp (const App &a);
  /* the engine's view (kept alive for the trace codec) */
  void Fill (void);

  uint32_t m_nodes;
  std::vector<Dev> m_dev;
  std::vector<App> m_app;
  std::vector<std::pair<uint32_t, uint32_t> > m_setup;  // (nsgpu_setup_kind, index), program order
  std::vector<uint32_t> m_route;                        // [node][slot]
  std::vector<uint32_t> m_dstSlot;                      // node -> route slot (0xffffffff: none)
  std::vector<uint32_t> m_addr, m_ifindex;              // per device (address 0: unassigned)
  std::vector<uint32_t> m_nif;                          // next interface index per node
  std::vector<uint32_t> m_owned;                        // FromNodeList: the journal entries the engine owns
  std::vector<Ptr<NetDevice> > m_devObj;                // FromNodeList: the ns-3 device of each engine device
  uint32_t m_nDst;
  bool m_icmp;
  int64_t m_stop;
  bool m_firstLink;
  nsgpu_p2p *m_engine;
  nsgpu_trace_codec *m_codec;
  // the C view (Fill)
  nsgpu_p2p_scenario m_sc;
  std::vector<uint32_t> m_cDevNode, m_cDevPeer, m_cDevQmax, m_cKind, m_cNode, m_cDst, m_cSlot, m_cSrc, m_cSize,
    m_cMaxb, m_cTtl, m_cCount, m_cSk, m_cSi, m_cRaddr, m_cRport;
  std::vector<uint64_t> m_cDevBps, m_cRate;
  std::vector<int64_t> m_cDevIfg, m_cDevDelay, m_cStart, m_cStop, m_cIvl;
  std::vector<double> m_cOn, m_cOff;
};

} // namespace ns3

#endif /* NSGPU_P2P_SCENARIO_H */
