/* -*- Mode:C++; c-file-style:"gnu"; indent-tabs-mode:nil; -*- */
#include "hip-simulator-impl.h"
#include "hip-batch-scheduler.h"
#include "ns3/simulator.h"
#include "ns3/assert.h"
#include "ns3/object-factory.h"

namespace ns3 {

NS_OBJECT_ENSURE_REGISTERED (HipSimulatorImpl);

TypeId
HipSimulatorImpl::GetTypeId (void)
{
  static TypeId tid = TypeId ("ns3::HipSimulatorImpl")
    .SetParent<SimulatorImpl> ()
    .AddConstructor<HipSimulatorImpl> ()
  ;
  return tid;
}

// uid 0 invalid, 1 "now", 2 "destroy": the first scheduled event gets 4 (as DefaultSimulatorImpl)
HipSimulatorImpl::HipSimulatorImpl ()
  : m_stop (false), m_nextUid (4), m_uid (0), m_ts (0), m_context (0xffffffff), m_pending (0), m_dispatched (0)
{
  m_events = CreateObject<HipBatchScheduler> ();
}

HipSimulatorImpl::~HipSimulatorImpl ()
{
}

void
HipSimulatorImpl::DoDispose (void)
{
  while (!m_events->IsEmpty ())
    {
      m_events->RemoveNext ().impl->Unref ();
    }
  m_events = 0;
  SimulatorImpl::DoDispose ();
}

void
HipSimulatorImpl::Destroy ()
{
  while (!m_destroy.empty ())
    {
      Ptr<EventImpl> ev = m_destroy.front ().PeekEventImpl ();
      m_destroy.pop_front ();
      if (!ev->IsCancelled ())
        {
          ev->Invoke ();
        }
    }
}

void
HipSimulatorImpl::SetScheduler (ObjectFactory schedulerFactory)
{
  // Simulator::GetImpl calls this after construction (simulator.cc:79-114): move pending events
  Ptr<Scheduler> s = schedulerFactory.Create<Scheduler> ();
  if (m_events != 0)
    {
      while (!m_events->IsEmpty ())
        {
          s->Insert (m_events->RemoveNext ());
        }
    }
  m_events = s;
}

uint32_t
HipSimulatorImpl::GetSystemId (void) const
{
  return 0;
}

void
HipSimulatorImpl::Insert (uint64_t ts, uint32_t context, EventImpl *event)
{
  Scheduler::Event ev;
  ev.impl = event;
  ev.key.m_ts = ts;
  ev.key.m_context = context;
  ev.key.m_uid = m_nextUid++;
  m_pending++;
  m_events->Insert (ev);
}

void
HipSimulatorImpl::Dispatch (void)
{
  Scheduler::Event next = m_events->RemoveNext ();
  NS_ASSERT (next.key.m_ts >= m_ts);
  m_pending--;
  m_ts = next.key.m_ts;           // Now / Context / Uid are updated before Invoke
  m_context = next.key.m_context;
  m_uid = next.key.m_uid;
  m_dispatched++;
  next.impl->Invoke ();           // a cancelled EventImpl is still dequeued, Invoke skips it
  next.impl->Unref ();
}

bool
HipSimulatorImpl::IsFinished (void) const
{
  return m_events->IsEmpty () || m_stop;
}

Time
HipSimulatorImpl::Next (void) const
{
  NS_ASSERT (!m_events->IsEmpty ());
  return TimeStep (m_events->PeekNext ().key.m_ts);
}

void
HipSimulatorImpl::Run (void)
{
  m_stop = false;
  while (!m_events->IsEmpty () && !m_stop)
    {
      Dispatch ();
    }
  NS_ASSERT (!m_events->IsEmpty () || m_pending == 0);
}

void
HipSimulatorImpl::RunOneEvent (void)
{
  Dispatch ();
}

void
HipSimulatorImpl::Stop (void)
{
  m_stop = true;
}

void
HipSimulatorImpl::Stop (Time const &time)
{
  Simulator::Schedule (time, &Simulator::Stop);
}

EventId
HipSimulatorImpl::Schedule (Time const &time, EventImpl *event)
{
  Time t = time + TimeStep (m_ts);
  NS_ASSERT (t.IsPositive () && t >= TimeStep (m_ts));
  uint32_t uid = m_nextUid;
  Insert ((uint64_t) t.GetTimeStep (), m_context, event);
  return EventId (event, (uint64_t) t.GetTimeStep (), m_context, uid);
}

void
HipSimulatorImpl::ScheduleWithContext (uint32_t context, Time const &time, EventImpl *event)
{
  Insert (m_ts + time.GetTimeStep (), context, event);
}

EventId
HipSimulatorImpl::ScheduleNow (EventImpl *event)
{
  uint32_t uid = m_nextUid;
  Insert (m_ts, m_context, event);
  return EventId (event, m_ts, m_context, uid);
}

EventId
HipSimulatorImpl::ScheduleDestroy (EventImpl *event)
{
  EventId id (Ptr<EventImpl> (event, false), m_ts, 0xffffffff, 2);
  m_destroy.push_back (id);
  m_nextUid++;                    // destroy events consume a uid too
  return id;
}

Time
HipSimulatorImpl::Now (void) const
{
  return TimeStep (m_ts);
}

Time
HipSimulatorImpl::GetDelayLeft (const EventId &id) const
{
  return IsExpired (id) ? TimeStep (0) : TimeStep (id.GetTs () - m_ts);
}

void
HipSimulatorImpl::Remove (const EventId &id)
{
  if (id.GetUid () == 2)
    {
      for (DestroyList::iterator i = m_destroy.begin (); i != m_destroy.end (); i++)
        {
          if (*i == id)
            {
              m_destroy.erase (i);
              break;
            }
        }
      return;
    }
  if (IsExpired (id))
    {
      return;
    }
  Scheduler::Event ev;
  ev.impl = id.PeekEventImpl ();
  ev.key.m_ts = id.GetTs ();
  ev.key.m_context = id.GetContext ();
  ev.key.m_uid = id.GetUid ();
  m_events->Remove (ev);
  ev.impl->Cancel ();
  ev.impl->Unref ();
  m_pending--;
}

void
HipSimulatorImpl::Cancel (const EventId &id)
{
  if (!IsExpired (id))
    {
      id.PeekEventImpl ()->Cancel ();
    }
}

bool
HipSimulatorImpl::IsExpired (const EventId &ev) const
{
  if (ev.GetUid () == 2)
    {
      if (ev.PeekEventImpl () == 0 || ev.PeekEventImpl ()->IsCancelled ())
        {
          return true;
        }
      for (DestroyList::const_iterator i = m_destroy.begin (); i != m_destroy.end (); i++)
        {
          if (*i == ev)
            {
              return false;
            }
        }
      return true;
    }
  return ev.PeekEventImpl () == 0 || ev.GetTs () < m_ts ||
         (ev.GetTs () == m_ts && ev.GetUid () <= m_uid) || ev.PeekEventImpl ()->IsCancelled ();
}

Time
HipSimulatorImpl::GetMaximumSimulationTime (void) const
{
  return TimeStep (0x7fffffffffffffffLL);
}

uint32_t
HipSimulatorImpl::GetContext (void) const
{
  return m_context;
}

uint64_t
HipSimulatorImpl::GetEventCount (void) const
{
  return m_dispatched;
}

} // namespace ns3
