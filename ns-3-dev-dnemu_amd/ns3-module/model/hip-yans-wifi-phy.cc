/* -*- Mode:C++; c-file-style:"gnu"; indent-tabs-mode:nil; -*- */
/*
 * See hip-yans-wifi-phy.h.  The uid-critical work is library code, tested without ns-3:
 *  - which phys a SendPacket's YansWifiChannel::Send reaches, with which uids and contexts: nsgpu_sim_wifi_send /
 *    nsgpu_wifil_send_plan (tests/test_wifi_binding_cpu.py against the oracle's channel loop);
 *  - where the EndReceive's host part runs in the order: the runtime's hand-back (nsgpu_sim_wifi_set_end_handler,
 *    tests/test_gpu_wifi_loop.py: a MAC that replies at each EndReceive, full pop log = the oracle's).
 * This file only maps ns-3 objects onto those calls.
 */
#include "hip-yans-wifi-phy.h"
#include "ns3/log.h"
#include "ns3/simulator.h"
#include "ns3/mobility-model.h"
#include "ns3/wifi-net-device.h"
#include "ns3/node.h"
#include "ns3/nist-error-rate-model.h"
#include "ns3/yans-error-rate-model.h"
#include "ns3/uinteger.h"
#include <cmath>

NS_LOG_COMPONENT_DEFINE ("HipYansWifiPhy");

#define NSGPU_RT(call)                                                      \
  do {                                                                      \
      if ((call) != NSGPU_OK)                                               \
        {                                                                   \
          NS_FATAL_ERROR ("libnsgpu: " << nsgpu_last_error ());             \
        }                                                                   \
    } while (false)

namespace ns3 {

NS_OBJECT_ENSURE_REGISTERED (HipYansWifiPhy);
NS_OBJECT_ENSURE_REGISTERED (HipWifiBinding);

TypeId
HipYansWifiPhy::GetTypeId (void)
{
  static TypeId tid = TypeId ("ns3::HipYansWifiPhy")
    .SetParent<YansWifiPhy> ()
    .AddConstructor<HipYansWifiPhy> ()
  ;
  return tid;
}

HipYansWifiPhy::HipYansWifiPhy ()
  : m_binding (0),
    m_rt (0),
    m_index (0),
    m_bound (false),
    m_random (0.0, 1.0)
{
}

void
HipYansWifiPhy::Bind (HipWifiBinding *binding, nsgpu_sim *runtime, uint32_t index)
{
  m_binding = binding;
  m_rt = runtime;
  m_index = index;
  m_bound = true;
}

uint32_t
HipYansWifiPhy::GetIndex (void) const
{
  return m_index;
}

nsgpu_wifil_phy_state
HipYansWifiPhy::State (void) const
{
  if (!m_bound)
    {
      NS_FATAL_ERROR ("HipYansWifiPhy: not attached (HipWifiBinding::Attach before Run)");
    }
  nsgpu_wifil_phy_state st;
  NSGPU_RT (nsgpu_sim_wifi_state (m_rt, m_index, &st));  // (Now (): the runtime's, the device advanced to it)
  return st;
}

double
HipYansWifiPhy::PowerDbm (uint8_t level) const
{
  const double base = GetTxPowerStart (), end = GetTxPowerEnd ();
  const uint32_t n = GetNTxPower ();
  NS_ASSERT (base <= end);
  NS_ASSERT (n > 0);
  if (n > 1)
    {
      return base + level * (end - base) / (n - 1);
    }
  NS_ASSERT_MSG (base == end, "cannot have TxPowerEnd != TxPowerStart with TxPowerLevels == 1");
  return base;
}

// YansWifiPhy::SendPacket (yans-wifi-phy.cc:499-522): the traces and the listeners' NotifyTxStart here, the state
// switch (an RX abandoned: m_endRxEvent.Cancel) and YansWifiChannel::Send on the device
void
HipYansWifiPhy::SendPacket (Ptr<const Packet> packet, WifiMode txMode, enum WifiPreamble preamble, uint8_t txPower)
{
  NS_LOG_FUNCTION (this << packet << txMode << preamble << (uint32_t) txPower);
  NS_ASSERT (!IsStateTx ());
  const Time txDuration = CalculateTxDuration (packet->GetSize (), txMode, preamble);
  NotifyTxBegin (packet);
  const uint32_t rate500 = txMode.GetDataRate () / 500000;
  const bool shortPreamble = (WIFI_PREAMBLE_SHORT == preamble);
  NotifyMonitorSniffTx (packet, (uint16_t) GetChannelFrequencyMhz (), GetChannelNumber (), rate500, shortPreamble);
  for (std::vector<WifiPhyListener *>::const_iterator i = m_listeners.begin (); i != m_listeners.end (); ++i)
    {
      (*i)->NotifyTxStart (txDuration);  // (WifiPhyStateHelper::SwitchToTx, wifi-phy-state-helper.cc:254-290)
    }
  uint32_t modclass = NSGPU_WIFI_DSSS;
  switch (txMode.GetModulationClass ())
    {
    case WIFI_MOD_CLASS_DSSS: modclass = NSGPU_WIFI_DSSS; break;
    case WIFI_MOD_CLASS_OFDM: modclass = NSGPU_WIFI_OFDM; break;
    case WIFI_MOD_CLASS_ERP_OFDM: modclass = NSGPU_WIFI_ERP_OFDM; break;
    default: NS_FATAL_ERROR ("HipYansWifiPhy: modulation class " << txMode.GetModulationClass () << " is not on the device");
    }
  m_binding->RecordTx (packet, txMode, preamble);  // (the device's transmission index: SendPacket calls in order)
  NSGPU_RT (nsgpu_sim_wifi_send (m_rt, m_index, packet->GetSize (), PowerDbm (txPower) + GetTxGain (), modclass,
                                 txMode.GetDataRate (), txMode.GetBandwidth (),
                                 shortPreamble ? NSGPU_WIFI_PREAMBLE_SHORT : NSGPU_WIFI_PREAMBLE_LONG));
}

void
HipYansWifiPhy::SetReceiveOkCallback (WifiPhy::RxOkCallback callback)
{
  m_rxOk = callback;
  YansWifiPhy::SetReceiveOkCallback (callback);
}

void
HipYansWifiPhy::SetReceiveErrorCallback (WifiPhy::RxErrorCallback callback)
{
  m_rxError = callback;
  YansWifiPhy::SetReceiveErrorCallback (callback);
}

void
HipYansWifiPhy::RegisterListener (WifiPhyListener *listener)
{
  m_listeners.push_back (listener);
}

bool
HipYansWifiPhy::IsStateCcaBusy (void)
{
  return State ().state == NSGPU_WIFIL_CCA_BUSY;
}
bool
HipYansWifiPhy::IsStateIdle (void)
{
  return State ().state == NSGPU_WIFIL_IDLE;
}
bool
HipYansWifiPhy::IsStateBusy (void)
{
  return State ().state != NSGPU_WIFIL_IDLE;
}
bool
HipYansWifiPhy::IsStateRx (void)
{
  return State ().state == NSGPU_WIFIL_RX;
}
bool
HipYansWifiPhy::IsStateTx (void)
{
  return State ().state == NSGPU_WIFIL_TX;
}
bool
HipYansWifiPhy::IsStateSwitching (void)
{
  return false;  // (no channel switching on the device path)
}
Time
HipYansWifiPhy::GetDelayUntilIdle (void)
{
  return NanoSeconds (State ().delay_until_idle);
}

// YansWifiPhy::EndReceive (:770-799) after the device's CalculateSnrPer and state switch
void
HipYansWifiPhy::EndReceiveHandBack (const nsgpu_wifil_end &end, Ptr<const Packet> sent, WifiMode mode,
                                    enum WifiPreamble preamble)
{
  NS_ASSERT (Simulator::Now ().GetNanoSeconds () == (int64_t) end.ts);
  Ptr<Packet> packet = sent->Copy ();  // (YansWifiChannel::Send's copy per receiver, :97)
  if (m_random.GetValue () > end.per)
    {
      NotifyRxEnd (packet);
      const uint32_t rate500 = mode.GetDataRate () / 500000;
      const bool shortPreamble = (WIFI_PREAMBLE_SHORT == preamble);
      const double signalDbm = 10.0 * std::log10 (end.rx_w) + 30;
      const double noiseDbm = 10.0 * std::log10 (end.rx_w / end.snr) - GetRxNoiseFigure () + 30;
      NotifyMonitorSniffRx (packet, (uint16_t) GetChannelFrequencyMhz (), GetChannelNumber (), rate500, shortPreamble,
                            signalDbm, noiseDbm);
      for (std::vector<WifiPhyListener *>::const_iterator i = m_listeners.begin (); i != m_listeners.end (); ++i)
        {
          (*i)->NotifyRxEndOk ();  // (SwitchFromRxEndOk, wifi-phy-state-helper.cc:338-352)
        }
      if (!m_rxOk.IsNull ())
        {
          m_rxOk (packet, end.snr, mode, preamble);
        }
    }
  else
    {
      NotifyRxDrop (packet);
      for (std::vector<WifiPhyListener *>::const_iterator i = m_listeners.begin (); i != m_listeners.end (); ++i)
        {
          (*i)->NotifyRxEndError ();  // (SwitchFromRxEndError, :354-368)
        }
      if (!m_rxError.IsNull ())
        {
          m_rxError (packet, end.snr);
        }
    }
}

// ---- the helper ----
HipYansWifiPhyHelper
HipYansWifiPhyHelper::Default (void)
{
  HipYansWifiPhyHelper helper;
  helper.SetErrorRateModel ("ns3::NistErrorRateModel");
  return helper;
}

HipYansWifiPhyHelper::HipYansWifiPhyHelper ()
{
  m_hipPhy.SetTypeId ("ns3::HipYansWifiPhy");
}

void
HipYansWifiPhyHelper::SetChannel (Ptr<YansWifiChannel> channel)
{
  m_hipChannel = channel;
  YansWifiPhyHelper::SetChannel (channel);
}

void
HipYansWifiPhyHelper::Set (std::string name, const AttributeValue &v)
{
  m_hipPhy.Set (name, v);
  YansWifiPhyHelper::Set (name, v);
}

void
HipYansWifiPhyHelper::SetErrorRateModel (std::string name, std::string n0, const AttributeValue &v0,
                                         std::string n1, const AttributeValue &v1)
{
  m_hipErrorRateModel = ObjectFactory ();
  m_hipErrorRateModel.SetTypeId (name);
  m_hipErrorRateModel.Set (n0, v0);
  m_hipErrorRateModel.Set (n1, v1);
  YansWifiPhyHelper::SetErrorRateModel (name, n0, v0, n1, v1);
}

// YansWifiPhyHelper::Create (yans-wifi-helper.cc:232-241) with the device-backed phy
Ptr<WifiPhy>
HipYansWifiPhyHelper::Create (Ptr<Node> node, Ptr<WifiNetDevice> device) const
{
  Ptr<HipYansWifiPhy> phy = m_hipPhy.Create<HipYansWifiPhy> ();
  Ptr<ErrorRateModel> error = m_hipErrorRateModel.Create<ErrorRateModel> ();
  phy->SetErrorRateModel (error);
  phy->SetChannel (m_hipChannel);
  phy->SetMobility (node);
  phy->SetDevice (device);
  return phy;
}

// ---- the binding ----
TypeId
HipWifiBinding::GetTypeId (void)
{
  static TypeId tid = TypeId ("ns3::HipWifiBinding")
    .SetParent<Object> ()
    .AddConstructor<HipWifiBinding> ()
  ;
  return tid;
}

HipWifiBinding::HipWifiBinding ()
  : m_engine (0),
    m_rt (0)
{
}

HipWifiBinding::~HipWifiBinding ()
{
}

void
HipWifiBinding::DoDispose (void)
{
  if (m_rt)
    {
      nsgpu_sim_wifi_set_end_handler (m_rt, 0, 0);
    }
  m_phys.clear ();
  m_tx.clear ();
  if (m_engine)
    {
      nsgpu_wifil_destroy (m_engine);  // (after the runtime's last Run)
      m_engine = 0;
    }
  Object::DoDispose ();
}

nsgpu_loss_chain
HipWifiBinding::DefaultLoss (void)
{
  nsgpu_loss_chain c;
  c.n = 1;
  c.pad_ = 0;
  for (int i = 0; i < NSGPU_MAX_LOSS_CHAIN; i++)
    {
      c.m[i].kind = NSGPU_LOSS_NONE;
      c.m[i].pad_ = 0;
      c.m[i].p0 = c.m[i].p1 = c.m[i].p2 = 0;
    }
  c.m[0].kind = NSGPU_LOSS_LOG_DISTANCE;  // LogDistancePropagationLossModel's defaults (propagation-loss-model.cc:420-435)
  c.m[0].p0 = 3.0;
  c.m[0].p1 = 1.0;
  c.m[0].p2 = 46.6777;
  return c;
}

void
HipWifiBinding::RecordTx (Ptr<const Packet> packet, WifiMode mode, enum WifiPreamble preamble)
{
  Tx t;
  t.packet = packet;
  t.mode = mode;
  t.preamble = preamble;
  m_tx.push_back (t);
}

void
HipWifiBinding::EndHandBack (void *user, const nsgpu_wifil_end *end)
{
  HipWifiBinding *b = static_cast<HipWifiBinding *> (user);
  if (end->phy >= b->m_phys.size () || end->tx >= b->m_tx.size ())
    {
      NS_FATAL_ERROR ("HipWifiBinding: an EndReceive of an unknown phy / transmission");
    }
  const Tx &t = b->m_tx[end->tx];
  b->m_phys[end->phy]->EndReceiveHandBack (*end, t.packet, t.mode, t.preamble);
}

void
HipWifiBinding::Attach (Ptr<HipSimulatorImpl> impl, Ptr<YansWifiChannel> channel, const nsgpu_loss_chain &loss,
                        double speed, uint64_t txCap)
{
  NS_ASSERT (m_engine == 0);
  const uint32_t n = channel->GetNDevices ();
  std::vector<double> x (n), y (n), z (n);
  std::vector<uint32_t> chan (n), node (n);
  Ptr<HipYansWifiPhy> first;
  for (uint32_t i = 0; i < n; i++)  // (YansWifiChannel::m_phyList order = GetDevice (i)'s)
    {
      Ptr<WifiNetDevice> dev = DynamicCast<WifiNetDevice> (channel->GetDevice (i));
      Ptr<HipYansWifiPhy> phy = dev ? DynamicCast<HipYansWifiPhy> (dev->GetPhy ()) : 0;
      if (phy == 0)
        {
          NS_FATAL_ERROR ("HipWifiBinding: phy " << i << " of the channel is not a HipYansWifiPhy (HipYansWifiPhyHelper)");
        }
      Ptr<MobilityModel> mob = phy->GetMobility ()->GetObject<MobilityModel> ();
      const Vector p = mob->GetPosition ();
      x[i] = p.x;
      y[i] = p.y;
      z[i] = p.z;
      chan[i] = phy->GetChannelNumber ();
      node[i] = dev->GetNode () ? dev->GetNode ()->GetId () : 0xffffffffu;  // (yans-wifi-channel.cc:101-110)
      if (i == 0)
        {
          first = phy;
        }
      else if (phy->GetRxGain () != first->GetRxGain () || phy->GetEdThreshold () != first->GetEdThreshold ()
               || phy->GetCcaMode1Threshold () != first->GetCcaMode1Threshold ()
               || phy->GetRxNoiseFigure () != first->GetRxNoiseFigure ())
        {
          NS_FATAL_ERROR ("HipWifiBinding: the device path takes one set of PHY attributes per channel");
        }
      m_phys.push_back (phy);
    }
  if (n == 0)
    {
      return;
    }
  nsgpu_wifil_config cfg;
  cfg.n_phy = n;
  cfg.x = &x[0];
  cfg.y = &y[0];
  cfg.z = &z[0];
  cfg.channel = &chan[0];
  cfg.node = &node[0];
  cfg.loss = loss;
  cfg.speed = speed;
  cfg.rx_gain_db = first->GetRxGain ();
  cfg.ed_threshold_dbm = first->GetEdThreshold ();
  cfg.cca_threshold_dbm = first->GetCcaMode1Threshold ();
  cfg.rx_noise_figure_db = first->GetRxNoiseFigure ();
  Ptr<ErrorRateModel> erm = first->GetErrorRateModel ();
  if (DynamicCast<NistErrorRateModel> (erm) != 0)
    {
      cfg.error_model = NSGPU_WIFIL_NIST;
    }
  else if (DynamicCast<YansErrorRateModel> (erm) != 0)
    {
      cfg.error_model = NSGPU_WIFIL_YANS;
    }
  else
    {
      NS_FATAL_ERROR ("HipWifiBinding: error rate model " << erm->GetInstanceTypeId () << " is not on the device");
    }
  cfg.ni_cap = 1024;
  cfg.rxq_cap = 1024;
  cfg.pad_ = 0;
  cfg.tx_cap = txCap;
  NSGPU_RT (nsgpu_wifil_create (&cfg, &m_engine));
  m_rt = impl->GetRuntime ();
  NSGPU_RT (nsgpu_sim_attach_wifi (m_rt, m_engine));
  NSGPU_RT (nsgpu_sim_wifi_set_end_handler (m_rt, &HipWifiBinding::EndHandBack, this));
  for (uint32_t i = 0; i < n; i++)
    {
      m_phys[i]->Bind (this, m_rt, i);
      NSGPU_RT (nsgpu_sim_wifi_listen (m_rt, i, 1));  // (every phy's EndReceive runs its MAC callbacks)
    }
}

} // namespace ns3
