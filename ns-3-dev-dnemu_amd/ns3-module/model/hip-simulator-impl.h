/* -*- Mode:C++; c-file-style:"gnu"; indent-tabs-mode:nil; -*- */
/*
 * ns3::HipSimulatorImpl — SimulatorImpl (src/core/model/simulator-impl.h:35-200) whose event list is
 * the device-resident HipBatchScheduler and whose Run() can hand GPU-resident model subsets to
 * libnsgpu.so.  Selected with
 *   NS_GLOBAL_VALUE="SimulatorImplementationType=ns3::HipSimulatorImpl"
 * (GlobalValue g_simTypeImpl, src/core/model/simulator.cc:44-48).
 * Host-closure semantics equal DefaultSimulatorImpl's (default-simulator-impl.cc:49-353); the same
 * rules are implemented and tested in libnsgpu's nsgpu_sim_* runtime.
 */
#ifndef HIP_SIMULATOR_IMPL_H
#define HIP_SIMULATOR_IMPL_H

#include "ns3/simulator-impl.h"
#include "ns3/scheduler.h"
#include "ns3/event-impl.h"
#include "ns3/ptr.h"
#include <list>

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

  // number of RemoveNext dispatches (cancelled ones included)
  uint64_t GetEventCount (void) const;

private:
  virtual void DoDispose (void);
  void Dispatch (void);
  void Insert (uint64_t ts, uint32_t context, EventImpl *event);

  typedef std::list<EventId> DestroyList;
  DestroyList m_destroy;
  Ptr<Scheduler> m_events;
  bool m_stop;
  uint32_t m_nextUid;
  uint32_t m_uid;
  uint64_t m_ts;
  uint32_t m_context;
  int m_pending;
  uint64_t m_dispatched;
};

} // namespace ns3

#endif /* HIP_SIMULATOR_IMPL_H */
