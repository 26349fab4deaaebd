// nsgpu_route.hip — global-routing next-hop tables on the device.
//
// Replaces, for point-to-point topologies with unit link metrics, what GlobalRouteManager::
// PopulateRoutingTables installs and Ipv4GlobalRouting::LookupGlobal picks (RandomEcmpRouting off):
//   * SPFCalculate (global-route-manager-impl.cc:1327-1490) gives every router vertex D the exits of
//     all shortest paths from the root; SPFVertex::MergeRootExitDirections keeps them sorted by
//     (next-hop address, outgoing interface) (:314-326), and SPFIntraAddRouter installs D's host routes
//     in that order (:1996-2049) — so LookupGlobal's first match for an address of D leaves through the
//     root's device whose peer is one hop closer to D with the smallest (peer address, interface index).
//   * CheckForStubNode (:1245-1323): a node with a single link gets a default route through it.
// One BFS per destination node: a workgroup walks the topology level by level from D (CSR of each
// node's devices), then every node picks its exit.  Distances and frontiers live in HBM scratch,
// destinations go in batches.  The oracle (oracle/nsref_route.cc) restates the SPF itself.
#include <vector>
#include "nsgpu_internal.h"

namespace nsgpu {

constexpr int RB = 1024;                    // threads per BFS workgroup
constexpr uint32_t UNSEEN = 0xffffffffu;
constexpr uint32_t NOROUTE = 0xffffffffu;

// BFS from dst_node[blockIdx.x] (level-synchronous; frontier counts in LDS).
__global__ __launch_bounds__(RB) void k_route_bfs(uint32_t n_nodes, const uint32_t *__restrict__ off,
                                                  const uint32_t *__restrict__ adj_node, const uint32_t *__restrict__ dst,
                                                  uint32_t *__restrict__ dist, uint32_t *__restrict__ queue) {
  __shared__ uint32_t s_cnt[2];
  const uint32_t D = dst[blockIdx.x];
  uint32_t *ds = dist + (uint64_t)blockIdx.x * n_nodes;
  uint32_t *q[2] = {queue + (uint64_t)blockIdx.x * 2 * n_nodes, queue + ((uint64_t)blockIdx.x * 2 + 1) * n_nodes};
  for (uint32_t i = threadIdx.x; i < n_nodes; i += RB) ds[i] = UNSEEN;
  if (threadIdx.x == 0) {
    s_cnt[0] = 1;
    s_cnt[1] = 0;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    ds[D] = 0;
    q[0][0] = D;
  }
  __syncthreads();
  uint32_t lev = 0, cur = 0;
  while (s_cnt[cur] != 0) {
    const uint32_t n = s_cnt[cur], nxt = cur ^ 1;
    ++lev;
    for (uint32_t i = threadIdx.x; i < n; i += RB) {
      const uint32_t u = q[cur][i];
      for (uint32_t e = off[u]; e < off[u + 1]; ++e) {
        const uint32_t v = adj_node[e];
        if (ds[v] == UNSEEN && atomicCAS(&ds[v], UNSEEN, lev) == UNSEEN) q[nxt][atomicAdd(&s_cnt[nxt], 1u)] = v;
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) s_cnt[cur] = 0;
    __syncthreads();
    cur = nxt;
  }
}

// Exit of every node towards each destination of the batch: out[k * n_nodes + node] (device id).
__global__ __launch_bounds__(256) void k_route_pick(uint32_t n_nodes, uint32_t nb, const uint32_t *__restrict__ off,
                                                    const uint32_t *__restrict__ adj_node,
                                                    const uint32_t *__restrict__ adj_dev,
                                                    const uint64_t *__restrict__ adj_tie, const uint32_t *__restrict__ dst,
                                                    const uint32_t *__restrict__ dist, uint32_t *__restrict__ out) {
  const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= (uint64_t)nb * n_nodes) return;
  const uint32_t k = (uint32_t)(t / n_nodes), R = (uint32_t)(t % n_nodes);
  const uint32_t *ds = dist + (uint64_t)k * n_nodes;
  const uint32_t e0 = off[R], e1 = off[R + 1];
  uint32_t best = NOROUTE;
  if (R != dst[k]) {
    if (e1 - e0 == 1) {
      best = adj_dev[e0];  // CheckForStubNode: default route through the single link
    } else {
      const uint32_t dR = ds[R];
      if (dR != UNSEEN) {
        uint64_t bt = ~0ull;
        for (uint32_t e = e0; e < e1; ++e) {
          if (ds[adj_node[e]] + 1u == dR && adj_tie[e] < bt) {
            bt = adj_tie[e];
            best = adj_dev[e];
          }
        }
      }
    }
  }
  out[t] = best;
}

}  // namespace nsgpu

using nsgpu::set_error;

extern "C" int nsgpu_route_global(uint32_t n_nodes, uint32_t n_devices, const uint32_t *dev_node,
                                  const uint32_t *dev_peer, const uint32_t *dev_addr, const uint32_t *dev_ifindex,
                                  uint32_t n_dst, const uint32_t *dst_node, uint32_t *route_out, void *stream) {
  if (!n_nodes || !dev_node || !dev_peer || !route_out || (n_dst && !dst_node))
    return set_error(NSGPU_EINVAL, "nsgpu_route_global: null argument");
  for (uint32_t d = 0; d < n_devices; ++d)
    if (dev_node[d] >= n_nodes || dev_peer[d] >= n_devices)
      return set_error(NSGPU_EINVAL, "nsgpu_route_global: device %u out of range", d);
  for (uint32_t k = 0; k < n_dst; ++k)
    if (dst_node[k] >= n_nodes) return set_error(NSGPU_EINVAL, "nsgpu_route_global: destination %u out of range", k);
  // CSR of each node's devices in device order; the tie key of an exit is (peer address, interface index)
  std::vector<uint32_t> off(n_nodes + 1, 0), adj_node(n_devices), adj_dev(n_devices);
  std::vector<uint64_t> adj_tie(n_devices);
  for (uint32_t d = 0; d < n_devices; ++d) ++off[dev_node[d] + 1];
  for (uint32_t n = 0; n < n_nodes; ++n) off[n + 1] += off[n];
  {
    std::vector<uint32_t> fill(off.begin(), off.end() - 1);
    for (uint32_t d = 0; d < n_devices; ++d) {
      const uint32_t e = fill[dev_node[d]]++;
      adj_node[e] = dev_node[dev_peer[d]];
      adj_dev[e] = d;
      adj_tie[e] = dev_addr && dev_ifindex ? ((uint64_t)dev_addr[dev_peer[d]] << 32) | dev_ifindex[d] : d;
    }
  }
  hipStream_t s = (hipStream_t)stream;
  // batch of destinations: dist (4 B) + two frontier queues (8 B) per node, <= 1 GiB of scratch
  const uint64_t per = 12ull * n_nodes;
  const uint32_t B = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>({(uint64_t)n_dst ? n_dst : 1, 1024,
                                                                       (1ull << 30) / per}));
  uint32_t *d_off = nullptr, *d_node = nullptr, *d_dev = nullptr, *d_dst = nullptr, *d_dist = nullptr,
           *d_q = nullptr, *d_out = nullptr;
  uint64_t *d_tie = nullptr;
  int rc = NSGPU_OK;
  auto fail = [&](hipError_t e, const char *what) {
    if (e != hipSuccess && rc == NSGPU_OK) rc = set_error(NSGPU_EHIP, "nsgpu_route_global: %s: %s", what, hipGetErrorString(e));
    return e != hipSuccess;
  };
  do {
    if (fail(hipMalloc(&d_off, 4ull * (n_nodes + 1)), "hipMalloc") || fail(hipMalloc(&d_node, 4ull * n_devices + 4), "hipMalloc") ||
        fail(hipMalloc(&d_dev, 4ull * n_devices + 4), "hipMalloc") || fail(hipMalloc(&d_tie, 8ull * n_devices + 8), "hipMalloc") ||
        fail(hipMalloc(&d_dst, 4ull * B), "hipMalloc") || fail(hipMalloc(&d_dist, 4ull * B * n_nodes), "hipMalloc") ||
        fail(hipMalloc(&d_q, 8ull * B * n_nodes), "hipMalloc") || fail(hipMalloc(&d_out, 4ull * B * n_nodes), "hipMalloc"))
      break;
    if (fail(hipMemcpyAsync(d_off, off.data(), 4ull * (n_nodes + 1), hipMemcpyHostToDevice, s), "copy") ||
        fail(hipMemcpyAsync(d_node, adj_node.data(), 4ull * n_devices, hipMemcpyHostToDevice, s), "copy") ||
        fail(hipMemcpyAsync(d_dev, adj_dev.data(), 4ull * n_devices, hipMemcpyHostToDevice, s), "copy") ||
        fail(hipMemcpyAsync(d_tie, adj_tie.data(), 8ull * n_devices, hipMemcpyHostToDevice, s), "copy"))
      break;
    std::vector<uint32_t> part((uint64_t)B * n_nodes);
    for (uint32_t k0 = 0; k0 < n_dst; k0 += B) {
      const uint32_t nb = std::min(B, n_dst - k0);
      if (fail(hipMemcpyAsync(d_dst, dst_node + k0, 4ull * nb, hipMemcpyHostToDevice, s), "copy")) break;
      hipLaunchKernelGGL(nsgpu::k_route_bfs, dim3(nb), dim3(nsgpu::RB), 0, s, n_nodes, d_off, d_node, d_dst, d_dist, d_q);
      if (fail(hipGetLastError(), "k_route_bfs")) break;
      const uint64_t tot = (uint64_t)nb * n_nodes;
      hipLaunchKernelGGL(nsgpu::k_route_pick, dim3((uint32_t)((tot + 255) / 256)), dim3(256), 0, s, n_nodes, nb, d_off,
                         d_node, d_dev, d_tie, d_dst, d_dist, d_out);
      if (fail(hipGetLastError(), "k_route_pick")) break;
      if (fail(hipMemcpyAsync(part.data(), d_out, 4ull * tot, hipMemcpyDeviceToHost, s), "copy") ||
          fail(hipStreamSynchronize(s), "sync"))
        break;
      for (uint32_t k = 0; k < nb; ++k)
        for (uint32_t n = 0; n < n_nodes; ++n) route_out[(uint64_t)n * n_dst + k0 + k] = part[(uint64_t)k * n_nodes + n];
    }
  } while (false);
  for (void *p : {(void *)d_off, (void *)d_node, (void *)d_dev, (void *)d_tie, (void *)d_dst, (void *)d_dist,
                  (void *)d_q, (void *)d_out})
    if (p) (void)hipFree(p);
  return rc;
}
