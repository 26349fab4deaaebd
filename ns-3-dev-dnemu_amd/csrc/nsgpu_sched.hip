// nsgpu_sched.hip — HipBatchScheduler: the ns3::Scheduler interface (scheduler.h:75-97) over an
// HBM-resident sorted event array, for events whose EventImpl closures stay on the host.
//
// Semantics are MapScheduler's (map-scheduler.cc:51-100): Insert, IsEmpty, PeekNext, RemoveNext,
// Remove, ordered by (ts, uid) (scheduler.h:105-121).  Design (batched, two-level):
//   * device: one sorted array D of 24-byte Scheduler::Event records {ts, uid, context, impl};
//   * host:   the "front" F — the next `batch` events popped from D in one copy — plus a small
//             binary heap H for inserts whose key is below the front bound (they must be popped
//             in order with F), and a staging vector S for every other insert;
//   * when F and H run dry, S is sorted on the device (LDS bitonic tiles + merge-path passes),
//     merged into D, and the next batch is copied out.  Removes are lazy: the uid is recorded and
//     the event is dropped when it surfaces (uids are unique, scheduler.h:58-63).
// The heavy part — keeping millions of pending keys ordered — is device work done in bulk;
// the per-event host cost is an array read.
#include <vector>
#include <algorithm>
#include <unordered_set>
#include "nsgpu_device.h"
#include "nsgpu_internal.h"

namespace nsgpu {

__host__ __device__ __forceinline__ bool ev_less(const nsgpu_event &a, const nsgpu_event &b) {
  return a.ts < b.ts || (a.ts == b.ts && a.uid < b.uid);
}

constexpr int TILE = 2048;       // elements per block-local sort tile
constexpr int TILE_THREADS = 1024;

// Block-local bitonic sort of TILE-element tiles (pads with +inf keys).
__global__ __launch_bounds__(TILE_THREADS) void sched_tile_sort(nsgpu_event *__restrict__ a, uint64_t n) {
  __shared__ nsgpu_event s[TILE];
  const uint64_t base = (uint64_t)blockIdx.x * TILE;
  for (int i = threadIdx.x; i < TILE; i += TILE_THREADS) {
    if (base + i < n) s[i] = a[base + i];
    else s[i] = nsgpu_event{~0ull, 0xffffffffu, 0, 0};
  }
  __syncthreads();
  for (int k = 2; k <= TILE; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < TILE; i += TILE_THREADS) {
        const int p = i ^ j;
        if (p > i) {
          const bool asc = (i & k) == 0;
          if (ev_less(s[p], s[i]) == asc) {
            nsgpu_event t = s[i];
            s[i] = s[p];
            s[p] = t;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int i = threadIdx.x; i < TILE; i += TILE_THREADS)
    if (base + i < n) a[base + i] = s[i];
}

// Merge-path merge of sorted runs: for every pair of runs [r, r+w) and [r+w, r+2w) of `in`
// (or of two separate arrays when `b` is given), each thread writes ITEMS consecutive outputs.
constexpr int ITEMS = 8;
__device__ __forceinline__ uint64_t merge_split(const nsgpu_event *A, uint64_t na, const nsgpu_event *B,
                                                uint64_t nb, uint64_t diag) {
  // number of elements taken from A among the first `diag` outputs (ties: A first — keys are unique)
  uint64_t lo = diag > nb ? diag - nb : 0, hi = diag < na ? diag : na;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (ev_less(B[diag - mid - 1], A[mid])) hi = mid;
    else lo = mid + 1;
  }
  return lo;
}

__global__ void sched_merge_pass(const nsgpu_event *__restrict__ in, nsgpu_event *__restrict__ out, uint64_t n,
                                 uint64_t w) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t o0 = t * ITEMS;
  if (o0 >= n) return;
  const uint64_t pair = o0 / (2 * w);
  const uint64_t a0 = pair * 2 * w;
  const uint64_t na = (a0 + w <= n) ? w : n - a0;
  const uint64_t b0 = a0 + na;
  const uint64_t nb = b0 >= n ? 0 : (b0 + w <= n ? w : n - b0);
  const nsgpu_event *A = in + a0, *B = in + b0;
  const uint64_t d0 = o0 - a0;
  uint64_t ia = merge_split(A, na, B, nb, d0), ib = d0 - ia;
  for (int q = 0; q < ITEMS && o0 + q < a0 + na + nb; q++) {
    const bool takeA = ib >= nb || (ia < na && !ev_less(B[ib], A[ia]));
    out[o0 + q] = takeA ? A[ia++] : B[ib++];
  }
}

__global__ void sched_merge_two(const nsgpu_event *__restrict__ A, uint64_t na, const nsgpu_event *__restrict__ B,
                                uint64_t nb, nsgpu_event *__restrict__ out) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t o0 = t * ITEMS;
  if (o0 >= na + nb) return;
  uint64_t ia = merge_split(A, na, B, nb, o0), ib = o0 - ia;
  for (int q = 0; q < ITEMS && o0 + q < na + nb; q++) {
    const bool takeA = ib >= nb || (ia < na && !ev_less(B[ib], A[ia]));
    out[o0 + q] = takeA ? A[ia++] : B[ib++];
  }
}

}  // namespace nsgpu

using namespace nsgpu;

struct nsgpu_sched {
  hipStream_t stream = nullptr;
  uint32_t batch = 4096;
  // device
  nsgpu_event *d_main = nullptr, *d_tmp = nullptr, *d_stage = nullptr, *d_stage2 = nullptr;
  uint64_t cap = 0, tmp_cap = 0, stage_cap = 0, stage2_cap = 0;
  uint64_t d_head = 0, d_n = 0;  // live device events are d_main[d_head, d_n)
  // host
  std::vector<nsgpu_event> front;  // popped batch, consumed from front_i
  size_t front_i = 0;
  bool front_bounded = false;      // true when d_main still holds events after the front
  nsgpu_event front_bound{};       // the largest key copied to the front
  std::vector<nsgpu_event> heap;   // inserts below the front bound (min-heap by key)
  std::vector<nsgpu_event> stage;  // inserts above the front bound, not yet on the device
  std::unordered_set<uint32_t> removed;
  uint64_t size = 0;
};

namespace {
struct HeapGreater {
  bool operator()(const nsgpu_event &a, const nsgpu_event &b) const { return ev_less(b, a); }
};

int grow(nsgpu_event **p, uint64_t *cap, uint64_t need) {
  if (need <= *cap) return NSGPU_OK;
  uint64_t nc = std::max<uint64_t>(need, *cap * 2 + 4096);
  nsgpu_event *q = nullptr;
  hipError_t e = hipMalloc(&q, nc * sizeof(nsgpu_event));
  if (e != hipSuccess) return set_error(NSGPU_ENOMEM, "nsgpu_sched: hipMalloc(%llu events)", (unsigned long long)nc);
  if (*p) (void)hipFree(*p);
  *p = q;
  *cap = nc;
  return NSGPU_OK;
}

// Sorts s->stage on the device and merges it into d_main[d_head, d_n).
int flush(nsgpu_sched *s) {
  const uint64_t ns = s->stage.size();
  if (ns == 0) return NSGPU_OK;
  const uint64_t live = s->d_n - s->d_head;
  int rc;
  if ((rc = grow(&s->d_stage, &s->stage_cap, ns))) return rc;
  if ((rc = grow(&s->d_stage2, &s->stage2_cap, ns))) return rc;
  NSGPU_HIP(hipMemcpyAsync(s->d_stage, s->stage.data(), ns * sizeof(nsgpu_event), hipMemcpyHostToDevice, s->stream));
  hipLaunchKernelGGL(sched_tile_sort, dim3((unsigned)((ns + TILE - 1) / TILE)), dim3(TILE_THREADS), 0, s->stream,
                     s->d_stage, ns);
  nsgpu_event *src = s->d_stage, *dst = s->d_stage2;
  for (uint64_t w = TILE; w < ns; w *= 2) {
    const uint64_t threads = (ns + ITEMS - 1) / ITEMS;
    hipLaunchKernelGGL(sched_merge_pass, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s->stream, src, dst,
                       ns, w);
    std::swap(src, dst);
  }
  // merge the sorted stage with the live device events into the spare array, then swap
  const uint64_t need = live + ns;
  if ((rc = grow(&s->d_tmp, &s->tmp_cap, need))) return rc;
  const uint64_t threads = (need + ITEMS - 1) / ITEMS;
  hipLaunchKernelGGL(sched_merge_two, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s->stream,
                     s->d_main + s->d_head, live, src, ns, s->d_tmp);
  NSGPU_HIP(hipGetLastError());
  std::swap(s->d_main, s->d_tmp);
  std::swap(s->cap, s->tmp_cap);
  s->d_head = 0;
  s->d_n = need;
  s->stage.clear();
  return NSGPU_OK;
}

// Refills the host front from the device (after flushing staged inserts).
int refill(nsgpu_sched *s) {
  int rc = flush(s);
  if (rc) return rc;
  const uint64_t live = s->d_n - s->d_head;
  const uint64_t take = std::min<uint64_t>(live, s->batch);
  s->front.resize(take);
  s->front_i = 0;
  if (take) {
    NSGPU_HIP(hipMemcpyAsync(s->front.data(), s->d_main + s->d_head, take * sizeof(nsgpu_event),
                             hipMemcpyDeviceToHost, s->stream));
    NSGPU_HIP(hipStreamSynchronize(s->stream));
  }
  s->d_head += take;
  s->front_bounded = s->d_n > s->d_head;
  if (take) s->front_bound = s->front.back();
  return NSGPU_OK;
}

// Pops (or peeks) the smallest live event.  Returns 1 if found.
int next_event(nsgpu_sched *s, nsgpu_event *out, bool pop, int *rc) {
  *rc = NSGPU_OK;
  for (;;) {
    const bool hf = s->front_i < s->front.size();
    const bool hh = !s->heap.empty();
    if (!hf && !hh) {
      if (s->stage.empty() && s->d_n == s->d_head) return 0;
      if ((*rc = refill(s))) return 0;
      continue;
    }
    bool from_front = hf && (!hh || ev_less(s->front[s->front_i], s->heap.front()));
    nsgpu_event e = from_front ? s->front[s->front_i] : s->heap.front();
    auto it = s->removed.find(e.uid);
    const bool dead = it != s->removed.end();
    if (dead || pop) {
      if (from_front) {
        s->front_i++;
      } else {
        std::pop_heap(s->heap.begin(), s->heap.end(), HeapGreater());
        s->heap.pop_back();
      }
    }
    if (dead) {
      s->removed.erase(it);
      continue;
    }
    *out = e;
    return 1;
  }
}
}  // namespace

extern "C" int nsgpu_sched_create(uint32_t batch, void *stream, nsgpu_sched **out) {
  if (!out) return set_error(NSGPU_EINVAL, "nsgpu_sched_create: null");
  nsgpu_sched *s = new nsgpu_sched();
  s->batch = batch ? batch : 4096;
  s->stream = (hipStream_t)stream;
  *out = s;
  return NSGPU_OK;
}

extern "C" int nsgpu_sched_destroy(nsgpu_sched *s) {
  if (!s) return NSGPU_OK;
  if (s->d_main) (void)hipFree(s->d_main);
  if (s->d_tmp) (void)hipFree(s->d_tmp);
  if (s->d_stage) (void)hipFree(s->d_stage);
  if (s->d_stage2) (void)hipFree(s->d_stage2);
  delete s;
  return NSGPU_OK;
}

// Scheduler::Insert (scheduler.h:75-78) for n events.
extern "C" int nsgpu_sched_insert(nsgpu_sched *s, const nsgpu_event *ev, uint64_t n) {
  if (!s || (n && !ev)) return set_error(NSGPU_EINVAL, "nsgpu_sched_insert: null");
  for (uint64_t i = 0; i < n; i++) {
    // an insert below the largest key already copied to the host front must pop in order with it
    const bool active = s->front_i < s->front.size() || !s->heap.empty();
    const bool in_front = active && ev_less(ev[i], s->front_bound);
    if (in_front) {
      s->heap.push_back(ev[i]);
      std::push_heap(s->heap.begin(), s->heap.end(), HeapGreater());
    } else {
      s->stage.push_back(ev[i]);
    }
  }
  s->size += n;
  return NSGPU_OK;
}

extern "C" int nsgpu_sched_is_empty(nsgpu_sched *s, int *empty) {
  if (!s || !empty) return set_error(NSGPU_EINVAL, "nsgpu_sched_is_empty: null");
  *empty = s->size == 0;
  return NSGPU_OK;
}

extern "C" int nsgpu_sched_size(nsgpu_sched *s, uint64_t *n) {
  if (!s || !n) return set_error(NSGPU_EINVAL, "nsgpu_sched_size: null");
  *n = s->size;
  return NSGPU_OK;
}

extern "C" int nsgpu_sched_peek_next(nsgpu_sched *s, nsgpu_event *out) {
  if (!s || !out) return set_error(NSGPU_EINVAL, "nsgpu_sched_peek_next: null");
  int rc;
  if (!next_event(s, out, false, &rc)) return rc ? rc : set_error(NSGPU_ESTATE, "PeekNext on an empty scheduler");
  return NSGPU_OK;
}

extern "C" int nsgpu_sched_remove_next(nsgpu_sched *s, nsgpu_event *out) {
  if (!s || !out) return set_error(NSGPU_EINVAL, "nsgpu_sched_remove_next: null");
  int rc;
  if (!next_event(s, out, true, &rc)) return rc ? rc : set_error(NSGPU_ESTATE, "RemoveNext on an empty scheduler");
  s->size--;
  return NSGPU_OK;
}

// Scheduler::Remove: the event must be pending (DefaultSimulatorImpl::Remove checks IsExpired first).
extern "C" int nsgpu_sched_remove(nsgpu_sched *s, const nsgpu_event *ev) {
  if (!s || !ev) return set_error(NSGPU_EINVAL, "nsgpu_sched_remove: null");
  if (s->size == 0) return set_error(NSGPU_ESTATE, "Remove on an empty scheduler");
  s->removed.insert(ev->uid);
  s->size--;
  return NSGPU_OK;
}
