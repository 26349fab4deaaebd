/* -*- Mode:C++; c-file-style:"gnu"; indent-tabs-mode:nil; -*- */
#include "hip-simulator-impl.h"
#include "ns3/simulator.h"
#include "ns3/fatal-error.h"
#include "ns3/object-factory.h"
#include <algorithm>

namespace ns3 {

NS_OBJECT_ENSURE_REGISTERED (HipSimulatorImpl);

#define NSGPU_RT(call)                                                      \
  do {                                                                      \
      if ((call) != NSGPU_OK)                                               \
        {                                                                   \
          NS_FATAL_ERROR ("libnsgpu: " << nsgpu_last_error ());             \
        }                                                                   \
    } while (false)

namespace {
/* the runtime hands raw handles back with bit 0 set (include/nsgpu.h, nsgpu_sim_insert) */
EventImpl *
HandleToEvent (uint64_t handle)
{
  return reinterpret_cast<EventImpl *> (static_cast<uintptr_t> (handle & ~static_cast<uint64_t> (1)));
}
} // anonymous namespace

TypeId
HipSimulatorImpl::GetTypeId (void)
{
  static TypeId tid = TypeId ("ns3::HipSimulatorImpl")
    .SetParent<SimulatorImpl> ()
    .AddConstructor<HipSimulatorImpl> ()
  ;
  return tid;
}

HipSimulatorImpl::HipSimulatorImpl ()
  : m_rt (0),
    m_window (4096)
{
  NSGPU_RT (nsgpu_sim_create (4096, 0, &m_rt));
}

HipSimulatorImpl::~HipSimulatorImpl ()
{
  nsgpu_sim_free (m_rt);
}

void
HipSimulatorImpl::AttachDeviceSubset (nsgpu_p2p *engine)
{
  NSGPU_RT (nsgpu_sim_attach_p2p (m_rt, engine));
}

uint64_t
HipSimulatorImpl::NowTs (void) const
{
  uint64_t now = 0;
  NSGPU_RT (nsgpu_sim_state (m_rt, &now, 0, 0, 0));
  return now;
}

uint64_t
HipSimulatorImpl::GetEventCount (void) const
{
  uint64_t n = 0;
  NSGPU_RT (nsgpu_sim_state (m_rt, 0, 0, &n, 0));
  return n;
}

void
HipSimulatorImpl::DoDispose (void)
{
  // pending closures were Ref'ed for the queue (Simulator::Schedule hands over one reference)
  uint32_t n = 0;
  do
    {
      NSGPU_RT (nsgpu_sim_drain (m_rt, &m_window[0], m_window.size (), &n));
      for (uint32_t i = 0; i < n; i++)
        {
          HandleToEvent (m_window[i].handle)->Unref ();
        }
    }
  while (n > 0);
  SimulatorImpl::DoDispose ();
}

void
HipSimulatorImpl::Destroy ()
{
  // ScheduleDestroy order; an event cancelled or removed meanwhile does not run
  std::vector<EventId> pending;
  pending.swap (m_atDestroy);
  for (std::vector<EventId>::iterator i = pending.begin (); i != pending.end (); ++i)
    {
      if (!i->PeekEventImpl ()->IsCancelled ())
        {
          i->PeekEventImpl ()->Invoke ();
        }
    }
}

void
HipSimulatorImpl::SetScheduler (ObjectFactory schedulerFactory)
{
  // Simulator::GetImpl hands over the SchedulerType factory (simulator.cc:79-114).  The runtime's
  // queue is the device-resident HipBatchScheduler whatever the factory: every ns-3 scheduler pops
  // in the same (ts, uid) order (scheduler.h:105-140), so the dispatch order does not change.
  (void) schedulerFactory;
}

uint32_t
HipSimulatorImpl::GetSystemId (void) const
{
  return 0;
}

EventId
HipSimulatorImpl::Enqueue (uint64_t ts, uint32_t context, EventImpl *event)
{
  uint32_t uid = 0;
  NSGPU_RT (nsgpu_sim_insert (m_rt, ts, context, reinterpret_cast<uintptr_t> (event), &uid));
  return EventId (event, ts, context, uid);
}

bool
HipSimulatorImpl::IsFinished (void) const
{
  uint64_t ts = 0;
  int empty = 1;
  NSGPU_RT (nsgpu_sim_next (m_rt, &ts, &empty));
  return empty != 0;
}

Time
HipSimulatorImpl::Next (void) const
{
  uint64_t ts = 0;
  int empty = 1;
  NSGPU_RT (nsgpu_sim_next (m_rt, &ts, &empty));
  if (empty)
    {
      NS_FATAL_ERROR ("HipSimulatorImpl::Next: no pending event");
    }
  return TimeStep (ts);
}

void
HipSimulatorImpl::RunWindows (uint32_t limit)
{
  uint32_t done = 0;
  while (done < limit)
    {
      uint32_t n = 0;
      const uint32_t cap = std::min<uint32_t> (limit - done, m_window.size ());
      NSGPU_RT (nsgpu_sim_pop_window (m_rt, &m_window[0], cap, &n));
      if (n == 0)
        {
          return;  // nothing pending (host or device), or a Stop was dispatched
        }
      for (uint32_t i = 0; i < n; i++)
        {
          int skip = 0;
          NSGPU_RT (nsgpu_sim_begin (m_rt, &m_window[i], &skip));
          if (skip != 0)
            {
              continue;  // removed by a closure of this window (released there), or after a Stop
            }
          EventImpl *ev = HandleToEvent (m_window[i].handle);
          ev->Invoke ();  // Invoke skips a cancelled closure; the dispatch still counts (H16)
          ev->Unref ();
          done++;
        }
    }
}

void
HipSimulatorImpl::Run (void)
{
  NSGPU_RT (nsgpu_sim_set_stop (m_rt, 0));
  RunWindows (0xffffffffu);
}

void
HipSimulatorImpl::RunOneEvent (void)
{
  RunWindows (1);
}

void
HipSimulatorImpl::Stop (void)
{
  NSGPU_RT (nsgpu_sim_set_stop (m_rt, 1));
}

void
HipSimulatorImpl::Stop (Time const &time)
{
  Simulator::Schedule (time, &Simulator::Stop);
}

EventId
HipSimulatorImpl::Schedule (Time const &time, EventImpl *event)
{
  const int64_t ts = time.GetTimeStep () + static_cast<int64_t> (NowTs ());
  if (time.IsStrictlyNegative () || ts < 0)
    {
      NS_FATAL_ERROR ("HipSimulatorImpl::Schedule: an event in the past");
    }
  return Enqueue (static_cast<uint64_t> (ts), GetContext (), event);
}

void
HipSimulatorImpl::ScheduleWithContext (uint32_t context, Time const &time, EventImpl *event)
{
  Enqueue (NowTs () + time.GetTimeStep (), context, event);
}

EventId
HipSimulatorImpl::ScheduleNow (EventImpl *event)
{
  return Enqueue (NowTs (), GetContext (), event);
}

EventId
HipSimulatorImpl::ScheduleDestroy (EventImpl *event)
{
  // uid 2 marks a destroy event; its own uid is consumed all the same
  NSGPU_RT (nsgpu_sim_consume_uid (m_rt, 0));
  EventId id (Ptr<EventImpl> (event, false), NowTs (), 0xffffffff, 2);
  m_atDestroy.push_back (id);
  return id;
}

Time
HipSimulatorImpl::Now (void) const
{
  return TimeStep (NowTs ());
}

Time
HipSimulatorImpl::GetDelayLeft (const EventId &id) const
{
  if (IsExpired (id))
    {
      return TimeStep (0);
    }
  return TimeStep (id.GetTs () - NowTs ());
}

void
HipSimulatorImpl::Remove (const EventId &id)
{
  if (id.GetUid () == 2)
    {
      std::vector<EventId>::iterator i = std::find (m_atDestroy.begin (), m_atDestroy.end (), id);
      if (i != m_atDestroy.end ())
        {
          m_atDestroy.erase (i);
        }
      return;
    }
  if (IsExpired (id))
    {
      return;
    }
  NSGPU_RT (nsgpu_sim_remove_key (m_rt, id.GetTs (), id.GetUid (), id.GetContext (),
                                  reinterpret_cast<uintptr_t> (id.PeekEventImpl ())));
  id.PeekEventImpl ()->Cancel ();
  id.PeekEventImpl ()->Unref ();  // the queue's reference
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
  EventImpl *impl = ev.PeekEventImpl ();
  if (impl == 0 || impl->IsCancelled ())
    {
      return true;
    }
  if (ev.GetUid () == 2)
    {
      return std::find (m_atDestroy.begin (), m_atDestroy.end (), ev) == m_atDestroy.end ();
    }
  int expired = 0;
  NSGPU_RT (nsgpu_sim_key_expired (m_rt, ev.GetTs (), ev.GetUid (), &expired));
  return expired != 0;
}

Time
HipSimulatorImpl::GetMaximumSimulationTime (void) const
{
  return TimeStep (0x7fffffffffffffffLL);  // the int64 ns horizon of Time
}

uint32_t
HipSimulatorImpl::GetContext (void) const
{
  uint32_t ctx = 0;
  NSGPU_RT (nsgpu_sim_state (m_rt, 0, &ctx, 0, 0));
  return ctx;
}

} // namespace ns3
