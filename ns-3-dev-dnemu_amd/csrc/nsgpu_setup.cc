// nsgpu_setup.cc — the setup journal of a program built under HipSimulatorImpl -> the p2p engine's setup list
// (include/nsgpu.h nsgpu_setup_from_journal).  Host code.
//
// Every setup-time Schedule call consumes a uid (DefaultSimulatorImpl::m_uid, default-simulator-impl.cc:
// 188-219), so the engine's copy of the program's setup must list them in call order, each mapped to what it
// starts: NodeListPriv::Add's Node::Start (node-list.cc:124-131), Node::AddDevice's NetDevice::Start and
// Node::AddApplication's Application::Start (node.cc:111-145), Simulator::Stop (t)'s Stop event
// (simulator.cc:168-172), and everything else (ScheduleDestroy, the program's own events) as a consumed uid.
// The journal entries arrive classified by the ns-3 side (which start call each one is, and the node's device
// or application index it starts), so an application added before a later link, or a program's own ts-0 event
// with a node context, maps to the right object; anything inconsistent fails instead of shifting uids.
#include <cstdint>
#include <vector>

#include "nsgpu.h"

namespace nsgpu {
int set_error(int code, const char *fmt, ...);
}
using nsgpu::set_error;

extern "C" int nsgpu_setup_from_journal(const nsgpu_journal_entry *j, uint64_t n, uint32_t n_nodes,
                                        const uint64_t *node_dev_off, const uint32_t *node_dev_kind,
                                        const uint32_t *node_n_apps, nsgpu_setup_map *out) {
  if ((!j && n) || !node_dev_off || !node_n_apps || !out)
    return set_error(NSGPU_EINVAL, "nsgpu_setup_from_journal: null");
  if (!out->setup_kind || !out->setup_index || !out->owned || !out->dev_node || !out->dev_local || !out->app_node ||
      !out->app_local)
    return set_error(NSGPU_EINVAL, "nsgpu_setup_from_journal: null output array");
  if (node_dev_off[0] != 0) return set_error(NSGPU_EINVAL, "nsgpu_setup_from_journal: node_dev_off[0] != 0");
  for (uint32_t k = 0; k < n_nodes; k++)
    if (node_dev_off[k + 1] < node_dev_off[k])
      return set_error(NSGPU_EINVAL, "nsgpu_setup_from_journal: node_dev_off decreases at node %u", k);
  if (node_dev_off[n_nodes] && !node_dev_kind) return set_error(NSGPU_EINVAL, "nsgpu_setup_from_journal: null node_dev_kind");
  std::vector<uint8_t> started(n_nodes, 0);
  std::vector<uint32_t> ndev(n_nodes, 0), napp(n_nodes, 0);
  uint64_t n_owned = 0;
  uint32_t D = 0, A = 0;
  int64_t stop = -1;
  for (uint64_t i = 0; i < n; i++) {
    const nsgpu_journal_entry &e = j[i];
    uint32_t kind = NSGPU_SETUP_UID, index = 0;
    bool owned = false;
    const uint32_t c = e.context;
    switch (e.kind) {
      case NSGPU_J_CALL:
      case NSGPU_J_DESTROY:
        break;  // the program's own event / a ScheduleDestroy: its uid is consumed, the host keeps it
      case NSGPU_J_STOP:
        if (stop >= 0) return set_error(NSGPU_EINVAL, "nsgpu_setup_from_journal: entry %llu: a second Simulator::Stop", (unsigned long long)i);
        if ((int64_t)e.ts < 0) return set_error(NSGPU_EINVAL, "nsgpu_setup_from_journal: entry %llu: Stop at a negative time", (unsigned long long)i);
        stop = (int64_t)e.ts;
        kind = NSGPU_SETUP_STOP, owned = true;
        break;
      case NSGPU_J_NODE_START:
      case NSGPU_J_DEVICE_START:
      case NSGPU_J_APP_START: {
        if (c >= n_nodes)
          return set_error(NSGPU_EINVAL, "nsgpu_setup_from_journal: entry %llu: a start call for node %u of %u",
                           (unsigned long long)i, c, n_nodes);
        if (e.ts != 0)
          return set_error(NSGPU_EINVAL, "nsgpu_setup_from_journal: entry %llu: a start call for node %u at %llu ns "
                           "(the helpers' start calls are at 0)", (unsigned long long)i, c, (unsigned long long)e.ts);
        if (e.kind == NSGPU_J_NODE_START) {
          if (started[c]) return set_error(NSGPU_EINVAL, "nsgpu_setup_from_journal: entry %llu: node %u started twice", (unsigned long long)i, c);
          started[c] = 1;
          kind = NSGPU_SETUP_NODE, index = c, owned = true;
          break;
        }
        if (!started[c])
          return set_error(NSGPU_EINVAL, "nsgpu_setup_from_journal: entry %llu: node %u's %s starts before the node",
                           (unsigned long long)i, c, e.kind == NSGPU_J_DEVICE_START ? "device" : "application");
        if (e.kind == NSGPU_J_DEVICE_START) {
          const uint64_t nd = node_dev_off[c + 1] - node_dev_off[c];
          if (e.local != ndev[c] || e.local >= nd)
            return set_error(NSGPU_EINVAL, "nsgpu_setup_from_journal: entry %llu: node %u device %u starts as its "
                             "device %u (of %llu)", (unsigned long long)i, c, e.local, ndev[c], (unsigned long long)nd);
          ndev[c]++;
          const uint32_t dk = node_dev_kind[node_dev_off[c] + e.local];
          if (dk == NSGPU_NDEV_P2P) {
            out->dev_node[D] = c, out->dev_local[D] = e.local;
            kind = NSGPU_SETUP_DEVICE, index = D++;
          } else if (dk == NSGPU_NDEV_LOOPBACK) {
            kind = NSGPU_SETUP_NOOP, index = c;  // LoopbackNetDevice::Start does nothing the engine models
          } else {
            return set_error(NSGPU_EINVAL, "nsgpu_setup_from_journal: node %u device %u is not a PointToPointNetDevice "
                             "(not in the GPU-resident subset)", c, e.local);
          }
        } else {
          if (e.local != napp[c] || e.local >= node_n_apps[c])
            return set_error(NSGPU_EINVAL, "nsgpu_setup_from_journal: entry %llu: node %u application %u starts as its "
                             "application %u (of %u)", (unsigned long long)i, c, e.local, napp[c], node_n_apps[c]);
          napp[c]++;
          out->app_node[A] = c, out->app_local[A] = e.local;
          kind = NSGPU_SETUP_APP, index = A++;
        }
        owned = true;
        break;
      }
      default:
        return set_error(NSGPU_EINVAL, "nsgpu_setup_from_journal: entry %llu: kind %u", (unsigned long long)i, e.kind);
    }
    out->setup_kind[i] = kind, out->setup_index[i] = index;
    if (owned) out->owned[n_owned++] = (uint32_t)i;
  }
  for (uint32_t k = 0; k < n_nodes; k++) {
    const uint64_t nd = node_dev_off[k + 1] - node_dev_off[k];
    if (!started[k] || ndev[k] != nd || napp[k] != node_n_apps[k])
      return set_error(NSGPU_EINVAL, "nsgpu_setup_from_journal: node %u: %s, %u of %llu device starts, %u of %u "
                       "application starts in the journal (build the topology under HipSimulatorImpl, before Run)",
                       k, started[k] ? "started" : "never started", ndev[k], (unsigned long long)nd, napp[k], node_n_apps[k]);
  }
  out->n_owned = n_owned, out->n_devices = D, out->n_apps = A, out->stop_ns = stop;
  return NSGPU_OK;
}
