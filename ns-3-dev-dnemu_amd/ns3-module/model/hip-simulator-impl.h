/* -*- Mode:C++; c-file-style:"gnu"; indent-tabs-mode:nil; -*- */
/*
 * ns3::HipSimulatorImpl — a SimulatorImpl (src/core/model/simulator-impl.h:35-200) whose run loop is the
 * windowed runtime of libnsgpu (include/nsgpu.h, nsgpu_sim_*): the pending EventImpl* live in the
 * device-resident HipBatchScheduler, Run() pulls one WINDOW per call (every pending event of the
 * smallest timestamp; with a GPU-resident p2p subset attached, the engine first dispatches every device
 * event before the next host event) and invokes its closures here, on the host.  The uid counter,
 * Now/Context and the dispatch rank live in the runtime, so host closures and device events share one
 * (ts, uid) order.  Selected with
 *   NS_GLOBAL_VALUE="SimulatorImplementationType=ns3::HipSimulatorImpl"
 * (GlobalValue g_simTypeImpl, src/core/model/simulator.cc:44-48).
 */
#ifndef HIP_SIMULATOR_IMPL_H
#define HIP_SIMULATOR_IMPL_H

#include "ns3/simulator-impl.h"
#include "ns3/event-impl.h"
#include "ns3/event-id.h"
#include "ns3/ptr.h"
#include "nsgpu.h"
#include <vector>

namespace ns3 {

class HipSimulatorImpl : public SimulatorImpl
{
public:
  static TypeId GetTypeId (void);

  HipSimulatorImpl ();
  ~HipSimulatorImpl ();

  virtual void Destroy ();
  virtual bool IsFinished (void) const;
  virtual Time Next (void) const;
  virtual void Stop (void);
  virtual void Stop (Time const &time);
  virtual EventId Schedule (Time const &time, EventImpl *event);
  virtual void ScheduleWithContext (uint32_t context, Time const &time, EventImpl *event);
  virtual EventId ScheduleNow (EventImpl *event);
  virtual EventId ScheduleDestroy (EventImpl *event);
  virtual void Remove (const EventId &ev);
  virtual void Cancel (const EventId &ev);
  virtual bool IsExpired (const EventId &ev) const;
  virtual void Run (void);
  virtual void RunOneEvent (void);
  virtual Time Now (void) const;
  virtual Time GetDelayLeft (const EventId &id) const;
  virtual Time GetMaximumSimulationTime (void) const;
  virtual void SetScheduler (ObjectFactory schedulerFactory);
  virtual uint32_t GetSystemId (void) const;
  virtual uint32_t GetContext (void) const;

  /* A GPU-resident point-to-point subset (nsgpu_p2p, e.g. from NsgpuP2pScenario) joins this
   * simulator's event order; call before anything is scheduled on it. */
  void AttachDeviceSubset (nsgpu_p2p *engine);

  /* The setup journal: every Schedule* / ScheduleDestroy / Stop (Time) call made before the first Run, in
   * call order (= uid order, from 4), classified when it is made: the stock helpers' start calls
   * (NodeListPriv::Add's Node::Start, Node::AddDevice's NetDevice::Start, Node::AddApplication's
   * Application::Start, node-list.cc:124-131, node.cc:111-145) are told apart from the program's own events
   * by the closure's type (MakeEvent's class for (&Object::Start, Ptr<Node | NetDevice | Application>)), and
   * carry the index the device / application got on its node.  NsgpuP2pScenario::FromNodeList hands the
   * journal to nsgpu_setup_from_journal (include/nsgpu.h), which maps it to the engine's setup list. */
  enum SetupKind
  {
    SETUP_CALL = NSGPU_J_CALL,
    SETUP_DESTROY = NSGPU_J_DESTROY,
    SETUP_STOP = NSGPU_J_STOP,
    SETUP_NODE_START = NSGPU_J_NODE_START,
    SETUP_DEVICE_START = NSGPU_J_DEVICE_START,
    SETUP_APP_START = NSGPU_J_APP_START
  };
  struct SetupCall
  {
    uint32_t kind, context, uid;
    uint64_t ts;
    EventImpl *event;
    uint32_t local;  // SETUP_DEVICE_START / SETUP_APP_START: the object's index on its node
  };
  const std::vector<SetupCall> &GetSetupJournal (void) const;
  /* The engine built from this program's own topology (NsgpuP2pScenario::FromNodeList) takes over the
   * journal entries `owned`: their host events are removed (the engine dispatches them, with the same
   * uids) and the engine joins the event order; the program's other events stay on the host. */
  void AdoptDeviceSubset (nsgpu_p2p *engine, const std::vector<uint32_t> &owned);
  /* Dispatches so far (RemoveNext calls, cancelled events included: SURVEY H16), host and device. */
  uint64_t GetEventCount (void) const;
  /* The libnsgpu runtime behind this simulator (a device engine attaches to it: HipWifiBinding::Attach). */
  nsgpu_sim *GetRuntime (void) const;

private:
  virtual void DoDispose (void);
  /* Runs the first n events of m_window (a popped window) in order. */
  void Dispatch (uint32_t n);
  /* Unrefs the destroy list's references (the list itself lives in the runtime). */
  void ReleaseDestroyList (void);
  EventId Enqueue (uint64_t ts, uint32_t context, EventImpl *event);
  uint64_t NowTs (void) const;

  nsgpu_sim *m_rt;
  std::vector<nsgpu_event> m_window;
  std::vector<SetupCall> m_journal;
  bool m_running;    // Run was called (the journal is closed)
  bool m_nextStop;   // Stop (Time) is scheduling Simulator::Stop
};

} // namespace ns3

#endif /* HIP_SIMULATOR_IMPL_H */
