/* -*- Mode:C++; c-file-style:"gnu"; indent-tabs-mode:nil; -*- */
#include "hip-batch-scheduler.h"
#include "ns3/event-impl.h"
#include "ns3/fatal-error.h"
#include "ns3/uinteger.h"

namespace ns3 {

NS_OBJECT_ENSURE_REGISTERED (HipBatchScheduler);

#define NSGPU_CHECK(call)                                                  \
  do {                                                                     \
      if ((call) != NSGPU_OK)                                              \
        {                                                                  \
          NS_FATAL_ERROR ("libnsgpu: " << nsgpu_last_error ());            \
        }                                                                  \
    } while (false)

TypeId
HipBatchScheduler::GetTypeId (void)
{
  static TypeId tid = TypeId ("ns3::HipBatchScheduler")
    .SetParent<Scheduler> ()
    .AddConstructor<HipBatchScheduler> ()
    .AddAttribute ("BatchSize",
                   "Events popped from the device-resident queue per host refill.",
                   UintegerValue (4096),
                   MakeUintegerAccessor (&HipBatchScheduler::SetBatch, &HipBatchScheduler::GetBatch),
                   MakeUintegerChecker<uint32_t> (1))
  ;
  return tid;
}

HipBatchScheduler::HipBatchScheduler ()
  : m_sched (0),
    m_batch (4096)
{
  NSGPU_CHECK (nsgpu_sched_create (m_batch, 0, &m_sched));
}

HipBatchScheduler::~HipBatchScheduler ()
{
  nsgpu_sched_destroy (m_sched);
}

void
HipBatchScheduler::SetBatch (uint32_t batch)
{
  // only meaningful before the first Insert: recreate the (empty) device queue
  uint64_t n = 0;
  NSGPU_CHECK (nsgpu_sched_size (m_sched, &n));
  if (n == 0)
    {
      nsgpu_sched_destroy (m_sched);
      m_batch = batch;
      NSGPU_CHECK (nsgpu_sched_create (m_batch, 0, &m_sched));
    }
}

uint32_t
HipBatchScheduler::GetBatch (void) const
{
  return m_batch;
}

// Scheduler::Event {EventImpl *impl; EventKey {m_ts, m_uid, m_context}} <-> nsgpu_event
static nsgpu_event
ToNsgpu (const Scheduler::Event &ev)
{
  nsgpu_event e;
  e.ts = ev.key.m_ts;
  e.uid = ev.key.m_uid;
  e.context = ev.key.m_context;
  e.handle = (uint64_t)(uintptr_t)ev.impl;
  return e;
}

static Scheduler::Event
FromNsgpu (const nsgpu_event &e)
{
  Scheduler::Event ev;
  ev.impl = (EventImpl *)(uintptr_t)e.handle;
  ev.key.m_ts = e.ts;
  ev.key.m_uid = e.uid;
  ev.key.m_context = e.context;
  return ev;
}

void
HipBatchScheduler::Insert (const Event &ev)
{
  nsgpu_event e = ToNsgpu (ev);
  NSGPU_CHECK (nsgpu_sched_insert (m_sched, &e, 1));
}

bool
HipBatchScheduler::IsEmpty (void) const
{
  int empty = 1;
  NSGPU_CHECK (nsgpu_sched_is_empty (m_sched, &empty));
  return empty != 0;
}

Scheduler::Event
HipBatchScheduler::PeekNext (void) const
{
  nsgpu_event e;
  NSGPU_CHECK (nsgpu_sched_peek_next (m_sched, &e));
  return FromNsgpu (e);
}

Scheduler::Event
HipBatchScheduler::RemoveNext (void)
{
  nsgpu_event e;
  NSGPU_CHECK (nsgpu_sched_remove_next (m_sched, &e));
  return FromNsgpu (e);
}

void
HipBatchScheduler::Remove (const Event &ev)
{
  nsgpu_event e = ToNsgpu (ev);
  NSGPU_CHECK (nsgpu_sched_remove (m_sched, &e));
}

} // namespace ns3
