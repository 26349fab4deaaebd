/* -*- Mode:C++; c-file-style:"gnu"; indent-tabs-mode:nil; -*- */
/*
 * ns3::HipBatchScheduler — the ns-3 side of the nsgpu HipBatchScheduler (include/nsgpu.h).
 * Drop this module into an ns-3 tree (src/nsgpu/) and select it with
 *   NS_GLOBAL_VALUE="SchedulerType=ns3::HipBatchScheduler"
 * (GlobalValue g_schedTypeImpl, src/core/model/simulator.cc:49-52).  It implements the five
 * Scheduler virtuals (src/core/model/scheduler.h:75-97) by forwarding to libnsgpu.so.
 */
#ifndef HIP_BATCH_SCHEDULER_H
#define HIP_BATCH_SCHEDULER_H

#include "ns3/scheduler.h"
#include "nsgpu.h"

namespace ns3 {

class HipBatchScheduler : public Scheduler
{
public:
  static TypeId GetTypeId (void);

  HipBatchScheduler ();
  virtual ~HipBatchScheduler ();

  virtual void Insert (const Event &ev);
  virtual bool IsEmpty (void) const;
  virtual Event PeekNext (void) const;
  virtual Event RemoveNext (void);
  virtual void Remove (const Event &ev);

private:
  void SetBatch (uint32_t batch);
  uint32_t GetBatch (void) const;
  nsgpu_sched *m_sched;
  uint32_t m_batch;
};

} // namespace ns3

#endif /* HIP_BATCH_SCHEDULER_H */
