/* -*- Mode:C++; c-file-style:"gnu"; indent-tabs-mode:nil; -*- */
#include "hip-simulator-impl.h"
#include "ns3/simulator.h"
#include "ns3/fatal-error.h"
#include "ns3/object-factory.h"
#include "ns3/make-event.h"
#include "ns3/node-list.h"
#include "ns3/node.h"
#include "ns3/net-device.h"
#include "ns3/application.h"
#include <typeinfo>

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

/* The closure class MakeEvent instantiates for ScheduleWithContext (ctx, t, &T::Start, Ptr<T>) — the stock
 * start calls of NodeListPriv::Add (T = Node), Node::AddDevice (NetDevice) and Node::AddApplication
 * (Application) (node-list.cc:124-131, node.cc:111-145; &T::Start is &Object::Start, so the object's
 * pointer type is what tells them apart) */
template <typename T>
const std::type_info &
StartEventType (void)
{
  static const std::type_info *type = 0;
  if (type == 0)
    {
      EventImpl *e = MakeEvent (&T::Start, Ptr<T> ());
      type = &typeid (*e);
      e->Unref ();
    }
  return *type;
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
    m_window (4096),
    m_running (false),
    m_nextStop (false)
{
  // front size 0: adaptive (nsgpu_sched_host.h)
  NSGPU_RT (nsgpu_sim_create (0, 0, &m_rt));
}

HipSimulatorImpl::~HipSimulatorImpl ()
{
  ReleaseDestroyList ();
  nsgpu_sim_free (m_rt);
}

void
HipSimulatorImpl::ReleaseDestroyList (void)
{
  // the references the destroy list holds (m_destroyEvents' EventIds, default-simulator-impl.cc:235-242)
  uint64_t handle = 0;
  int found = 1;
  while (m_rt != 0 && found)
    {
      NSGPU_RT (nsgpu_sim_destroy_pop (m_rt, &handle, &found));
      if (found)
        {
          HandleToEvent (handle)->Unref ();
        }
    }
}

void
HipSimulatorImpl::AttachDeviceSubset (nsgpu_p2p *engine)
{
  NSGPU_RT (nsgpu_sim_attach_p2p (m_rt, engine));
}

const std::vector<HipSimulatorImpl::SetupCall> &
HipSimulatorImpl::GetSetupJournal (void) const
{
  return m_journal;
}

void
HipSimulatorImpl::AdoptDeviceSubset (nsgpu_p2p *engine, const std::vector<uint32_t> &owned)
{
  if (m_running)
    {
      NS_FATAL_ERROR ("HipSimulatorImpl::AdoptDeviceSubset: call it before Run");
    }
  for (size_t i = 0; i < owned.size (); i++)
    {
      if (owned[i] >= m_journal.size () || m_journal[owned[i]].kind == SETUP_DESTROY)
        {
          NS_FATAL_ERROR ("HipSimulatorImpl::AdoptDeviceSubset: journal entry " << owned[i] << " is not a pending event");
        }
      const SetupCall &c = m_journal[owned[i]];
      // the host closure leaves the queue (its uid stays consumed: the engine's copy of the event has it)
      NSGPU_RT (nsgpu_sim_remove_key (m_rt, c.ts, c.uid, c.context, reinterpret_cast<uintptr_t> (c.event)));
      c.event->Cancel ();
      c.event->Unref ();  // the queue's reference
    }
  NSGPU_RT (nsgpu_sim_adopt_p2p (m_rt, engine));
}

uint64_t
HipSimulatorImpl::NowTs (void) const
{
  uint64_t now = 0;
  NSGPU_RT (nsgpu_sim_state (m_rt, &now, 0, 0, 0));
  return now;
}

nsgpu_sim *
HipSimulatorImpl::GetRuntime (void) const
{
  return m_rt;
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
  ReleaseDestroyList ();
  SimulatorImpl::DoDispose ();
}

void
HipSimulatorImpl::Destroy ()
{
  // default-simulator-impl.cc:79-92: the front of the runtime's destroy list is popped before it runs,
  // until the list is empty, so a destroy event a destroy closure schedules runs too and one it
  // Removes does not
  uint64_t handle = 0;
  int found = 1;
  for (;;)
    {
      NSGPU_RT (nsgpu_sim_destroy_pop (m_rt, &handle, &found));
      if (!found)
        {
          break;
        }
      EventImpl *ev = HandleToEvent (handle);
      if (!ev->IsCancelled ())
        {
          ev->Invoke ();
        }
      ev->Unref ();  // the list's reference
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
  if (!m_running)
    {
      SetupCall c = {m_nextStop ? (uint32_t) SETUP_STOP : (uint32_t) SETUP_CALL, context, uid, ts, event, 0};
      if (!m_nextStop && context != 0xffffffffu)
        {
          const std::type_info &t = typeid (*event);
          if (t == StartEventType<Node> ())
            {
              c.kind = SETUP_NODE_START;
            }
          else if (t == StartEventType<NetDevice> () && context < NodeList::GetNNodes ())
            {
              // Node::AddDevice pushed the device before scheduling its start
              c.kind = SETUP_DEVICE_START;
              c.local = NodeList::GetNode (context)->GetNDevices () - 1;
            }
          else if (t == StartEventType<Application> () && context < NodeList::GetNNodes ())
            {
              c.kind = SETUP_APP_START;
              c.local = NodeList::GetNode (context)->GetNApplications () - 1;
            }
        }
      m_journal.push_back (c);
    }
  m_nextStop = false;
  return EventId (event, ts, context, uid);
}

bool
HipSimulatorImpl::IsFinished (void) const
{
  // default-simulator-impl.cc:133-137: nothing pending (host or device) or Stop was called
  int finished = 1;
  NSGPU_RT (nsgpu_sim_is_finished (m_rt, &finished));
  return finished != 0;
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
HipSimulatorImpl::Dispatch (uint32_t n)
{
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
    }
}

void
HipSimulatorImpl::Run (void)
{
  m_running = true;
  m_journal.clear ();
  NSGPU_RT (nsgpu_sim_set_stop (m_rt, 0));
  for (;;)
    {
      uint32_t n = 0;
      NSGPU_RT (nsgpu_sim_pop_window (m_rt, &m_window[0], m_window.size (), &n));
      if (n == 0)
        {
          return;  // nothing pending (host or device), or a Stop was dispatched
        }
      Dispatch (n);
    }
}

void
HipSimulatorImpl::RunOneEvent (void)
{
  // default-simulator-impl.cc:167-170: one event, whatever the stop flag says
  uint32_t n = 0;
  NSGPU_RT (nsgpu_sim_pop_one (m_rt, &m_window[0], &n));
  if (n == 0)
    {
      NS_FATAL_ERROR ("HipSimulatorImpl::RunOneEvent: no pending event");
    }
  Dispatch (n);
}

void
HipSimulatorImpl::Stop (void)
{
  NSGPU_RT (nsgpu_sim_set_stop (m_rt, 1));
}

void
HipSimulatorImpl::Stop (Time const &time)
{
  m_nextStop = true;  // (journaled as the Stop event: Simulator::Stop (Time) -> Schedule (time, &Simulator::Stop))
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
  // uid 2 marks a destroy event; its own uid is consumed all the same.  The EventId
  // adopts the caller's reference; the runtime's list entry holds one more (released by Destroy,
  // Remove or DoDispose).
  uint64_t ts = 0;
  NSGPU_RT (nsgpu_sim_destroy_insert (m_rt, reinterpret_cast<uintptr_t> (event), &ts));
  if (!m_running)
    {
      const SetupCall c = {(uint32_t) SETUP_DESTROY, 0xffffffffu, 2u, ts, event, 0};
      m_journal.push_back (c);
    }
  event->Ref ();
  return EventId (Ptr<EventImpl> (event, false), ts, 0xffffffff, 2);
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
      // the first list entry equal to id (default-simulator-impl.cc:256-268); its reference goes with it
      int found = 0;
      NSGPU_RT (nsgpu_sim_destroy_remove (m_rt, reinterpret_cast<uintptr_t> (id.PeekEventImpl ()), id.GetTs (),
                                          &found));
      if (found)
        {
          id.PeekEventImpl ()->Unref ();
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
      int pending = 0;
      NSGPU_RT (nsgpu_sim_destroy_pending (m_rt, reinterpret_cast<uintptr_t> (impl), ev.GetTs (), &pending));
      return pending == 0;
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
