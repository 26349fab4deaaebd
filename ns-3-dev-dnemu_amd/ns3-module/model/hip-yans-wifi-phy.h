/* -*- Mode:C++; c-file-style:"gnu"; indent-tabs-mode:nil; -*- */
/*
 * The ns-3 side of the closed-loop Wi-Fi PHY on the device (libnsgpu nsgpu_wifil, include/nsgpu.h).
 *
 *  - ns3::HipYansWifiPhy : YansWifiPhy — the MAC-facing half of a YansWifiPhy whose receive path runs on the
 *    device: SendPacket (yans-wifi-phy.cc:499-522) hands the frame to nsgpu_sim_wifi_send (the device makes
 *    YansWifiChannel::Send's Receive events with the runtime's next uids, yans-wifi-channel.cc:77-115), the state
 *    queries (IsStateIdle / Rx / Tx / CcaBusy, GetDelayUntilIdle: wifi-phy-state-helper.cc:122-183) read the
 *    device's state through nsgpu_sim_wifi_state, and EndReceive (yans-wifi-phy.cc:770-799) comes back to the host
 *    at its place in the event order (nsgpu_sim_wifi_set_end_handler): the m_random draw, the Rx traces and the
 *    MAC's receive callbacks run here, so their Schedule calls take the uids the reference's would.
 *  - ns3::HipYansWifiPhyHelper : YansWifiPhyHelper — Create () makes HipYansWifiPhy objects (the stock helper's
 *    Create hard-codes ns3::YansWifiPhy, yans-wifi-helper.cc:232-241); everything else (pcap / ascii) is the
 *    stock helper's.
 *  - ns3::HipWifiBinding — after the topology is built: the channel's phys (m_phyList order), their positions,
 *    channel numbers, nodes and PHY attributes into a nsgpu_wifil_config, the engine created and attached to the
 *    HipSimulatorImpl's runtime, every phy bound to its index and handed back.
 *
 * Not delivered (documented in INTEGRATION.md §3.2): WifiPhyListener::NotifyRxStart / NotifyMaybeCcaBusyStart at the
 * device's syncs / CCA switches (NotifyTxStart and NotifyRxEndOk / Error are); a MAC that reads the state when it
 * needs it (GetState / IsStateIdle) is exact.
 */
#ifndef HIP_YANS_WIFI_PHY_H
#define HIP_YANS_WIFI_PHY_H

#include "ns3/yans-wifi-phy.h"
#include "ns3/yans-wifi-helper.h"
#include "ns3/yans-wifi-channel.h"
#include "ns3/random-variable.h"
#include "ns3/object-factory.h"
#include "ns3/packet.h"
#include "hip-simulator-impl.h"
#include "nsgpu.h"
#include <vector>

namespace ns3 {

class HipWifiBinding;

class HipYansWifiPhy : public YansWifiPhy
{
public:
  static TypeId GetTypeId (void);
  HipYansWifiPhy ();

  /* the runtime and this phy's index in the channel's m_phyList (HipWifiBinding::Attach) */
  void Bind (HipWifiBinding *binding, nsgpu_sim *runtime, uint32_t index);
  uint32_t GetIndex (void) const;

  virtual void SendPacket (Ptr<const Packet> packet, WifiMode mode, enum WifiPreamble preamble, uint8_t txPowerLevel);
  virtual void SetReceiveOkCallback (WifiPhy::RxOkCallback callback);
  virtual void SetReceiveErrorCallback (WifiPhy::RxErrorCallback callback);
  virtual void RegisterListener (WifiPhyListener *listener);
  virtual bool IsStateCcaBusy (void);
  virtual bool IsStateIdle (void);
  virtual bool IsStateBusy (void);
  virtual bool IsStateRx (void);
  virtual bool IsStateTx (void);
  virtual bool IsStateSwitching (void);
  virtual Time GetDelayUntilIdle (void);

  /* YansWifiPhy::EndReceive's host part, called by the runtime at the EndReceive's place (Now () = its time):
   * the m_random draw against the device's PER, then the traces and the MAC's callbacks (:783-798) */
  void EndReceiveHandBack (const nsgpu_wifil_end &end, Ptr<const Packet> packet, WifiMode mode,
                           enum WifiPreamble preamble);

private:
  nsgpu_wifil_phy_state State (void) const;
  /* YansWifiPhy::GetPowerDbm (:753-768, private there) from the public attributes */
  double PowerDbm (uint8_t level) const;

  HipWifiBinding *m_binding;
  nsgpu_sim *m_rt;
  uint32_t m_index;
  bool m_bound;
  UniformVariable m_random;  // YansWifiPhy::m_random (:783)
  WifiPhy::RxOkCallback m_rxOk;
  WifiPhy::RxErrorCallback m_rxError;
  std::vector<WifiPhyListener *> m_listeners;
};

class HipYansWifiPhyHelper : public YansWifiPhyHelper
{
public:
  /* YansWifiPhyHelper::Default (): NistErrorRateModel (yans-wifi-helper.cc:183-188) */
  static HipYansWifiPhyHelper Default (void);
  HipYansWifiPhyHelper ();
  void SetChannel (Ptr<YansWifiChannel> channel);
  void Set (std::string name, const AttributeValue &v);
  void SetErrorRateModel (std::string name,
                          std::string n0 = "", const AttributeValue &v0 = EmptyAttributeValue (),
                          std::string n1 = "", const AttributeValue &v1 = EmptyAttributeValue ());
  virtual Ptr<WifiPhy> Create (Ptr<Node> node, Ptr<WifiNetDevice> device) const;

private:
  ObjectFactory m_hipPhy;
  ObjectFactory m_hipErrorRateModel;
  Ptr<YansWifiChannel> m_hipChannel;
};

class HipWifiBinding : public Object
{
public:
  static TypeId GetTypeId (void);
  HipWifiBinding ();
  ~HipWifiBinding ();

  /* After the topology is built, before Run: the channel's phys (every one a HipYansWifiPhy) on the device,
   * attached to impl's runtime.  YansWifiChannel keeps its loss / delay models private: the chain and the
   * ConstantSpeed speed are passed (DefaultLoss () is YansWifiChannelHelper::Default's, yans-wifi-helper.cc:134-140). */
  void Attach (Ptr<HipSimulatorImpl> impl, Ptr<YansWifiChannel> channel, const nsgpu_loss_chain &loss,
               double speed = 299792458.0, uint64_t txCap = 1u << 20);
  static nsgpu_loss_chain DefaultLoss (void);

  /* a SendPacket of phy `index` (its transmission index on the device, in call order): the frame the receivers'
   * EndReceives hand back */
  void RecordTx (Ptr<const Packet> packet, WifiMode mode, enum WifiPreamble preamble);

private:
  virtual void DoDispose (void);
  static void EndHandBack (void *user, const nsgpu_wifil_end *end);

  struct Tx
  {
    Ptr<const Packet> packet;
    WifiMode mode;
    enum WifiPreamble preamble;
  };
  std::vector<Ptr<HipYansWifiPhy> > m_phys;
  std::vector<Tx> m_tx;
  nsgpu_wifil *m_engine;
  nsgpu_sim *m_rt;
};

} // namespace ns3

#endif /* HIP_YANS_WIFI_PHY_H */
