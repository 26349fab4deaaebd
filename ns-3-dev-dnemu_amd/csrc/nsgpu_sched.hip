// nsgpu_sched.hip — HipBatchScheduler: the ns3::Scheduler interface (scheduler.h:75-97) over an
// HBM-resident sorted event array, for events whose EventImpl closures stay on the host.  The state
// and the per-event host paths are in nsgpu_sched_host.h (layout and cost model there); this file
// holds the refill — the one device round trip per front — and the C-ABI.
//
// A refill: (1) the stage ring (pinned host memory) is sorted in LDS tiles of 2048 by a kernel that
// reads it in place, (2) merge-path passes join the tiles, (3) one merge-path kernel joins the sorted
// stage with the live device array into the spare array AND writes the first B merged events into the
// pinned front, (4) one stream synchronisation.  No memcpy is enqueued on the way.
#include <chrono>
#include <cstring>
#include <cmath>
#include "nsgpu_device.h"
#include "nsgpu_sched_host.h"

namespace nsgpu {

constexpr int TILE = 2048;  // elements per block-local sort tile
constexpr int TILE_THREADS = 1024;

// Block-local bitonic sort of TILE-element tiles of `in` (pinned host memory) into `out` (pads with +inf).
__global__ __launch_bounds__(TILE_THREADS) void sched_tile_sort(const nsgpu_event *__restrict__ in,
                                                                nsgpu_event *__restrict__ out, uint64_t n) {
  __shared__ nsgpu_event s[TILE];
  const uint64_t base = (uint64_t)blockIdx.x * TILE;
  for (int i = threadIdx.x; i < TILE; i += TILE_THREADS) {
    if (base + i < n) s[i] = in[base + i];
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
    if (base + i < n) out[base + i] = s[i];
}

// Merge path: each thread writes ITEMS consecutive outputs of the merge of two sorted runs.
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

// One pass over pairs of runs [r, r + w) and [r + w, r + 2w) of `in`.
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

// The live device events A and the sorted stage B into `out`; outputs below `take` also go to the
// pinned host front (they are what the host dispatches next).
__global__ void sched_merge_front(const nsgpu_event *__restrict__ A, uint64_t na, const nsgpu_event *__restrict__ B,
                                  uint64_t nb, nsgpu_event *__restrict__ out, nsgpu_event *__restrict__ front,
                                  uint64_t take) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t o0 = t * ITEMS;
  if (o0 >= na + nb) return;
  uint64_t ia = merge_split(A, na, B, nb, o0), ib = o0 - ia;
  for (int q = 0; q < ITEMS && o0 + q < na + nb; q++) {
    const bool takeA = ib >= nb || (ia < na && !ev_less(B[ib], A[ia]));
    const nsgpu_event e = takeA ? A[ia++] : B[ib++];
    if (o0 + q < take) front[o0 + q] = e;
    else out[o0 + q] = e;
  }
}

namespace {
int grow_dev(nsgpu_event **p, uint64_t *cap, uint64_t need) {
  if (need <= *cap) return NSGPU_OK;
  const uint64_t nc = std::max<uint64_t>(need, *cap * 2 + 4096);
  nsgpu_event *q = nullptr;
  hipError_t e = hipMalloc(&q, nc * sizeof(nsgpu_event));
  if (e != hipSuccess) return set_error(NSGPU_ENOMEM, "nsgpu_sched: hipMalloc(%llu events)", (unsigned long long)nc);
  if (*p) (void)hipFree(*p);
  *p = q;
  *cap = nc;
  return NSGPU_OK;
}

// Pinned, device-visible host buffer of at least `need` events; `keep` events are carried over.
int grow_pinned(nsgpu_event **p, uint64_t *cap, uint64_t need, uint64_t keep) {
  if (need <= *cap) return NSGPU_OK;
  const uint64_t nc = std::max<uint64_t>(need, *cap * 2 + 1024);
  nsgpu_event *q = nullptr;
  hipError_t e = hipHostMalloc((void **)&q, nc * sizeof(nsgpu_event), hipHostMallocMapped);
  if (e != hipSuccess)
    return set_error(NSGPU_ENOMEM, "nsgpu_sched: hipHostMalloc(%llu events)", (unsigned long long)nc);
  if (*p) {
    if (keep) memcpy(q, *p, keep * sizeof(nsgpu_event));
    (void)hipHostFree(*p);
  }
  *p = q;
  *cap = nc;
  return NSGPU_OK;
}

template <class T>
T *dev_view(T *host) {  // the device address of a pinned host buffer
  void *d = nullptr;
  if (hipHostGetDevicePointer(&d, host, 0) != hipSuccess) return host;  // (unified addressing)
  return (T *)d;
}
}  // namespace

int sched_grow_stage(nsgpu_sched *s) { return grow_pinned(&s->h_stage, &s->stage_cap, s->stage_n + 1, s->stage_n); }

// The front size for the next refill (see nsgpu_sched_host.h): sqrt (R * P / c_heap), c_heap ~ 25 ns
// per heap push + pop at the heap sizes this produces.
static uint64_t front_size(const nsgpu_sched *s, uint64_t avail) {
  uint64_t b = s->batch_fixed;
  if (!b) {
    const double p = (double)std::max<uint64_t>(s->size, 1);
    b = (uint64_t)std::sqrt(s->refill_ns * p / 25.0);
    b = std::min<uint64_t>(std::max<uint64_t>(b, 256), 1u << 20);
  }
  return std::min<uint64_t>(b, avail);
}

int sched_refill(nsgpu_sched *s) {
  const auto t0 = std::chrono::steady_clock::now();
  const uint64_t ns = s->stage_n, live = s->d_n - s->d_head, need = live + ns;
  const uint64_t take = front_size(s, need);
  int rc;
  if ((rc = grow_pinned(&s->h_front, &s->front_cap, take, 0))) return rc;
  if (ns) {
    // sort the stage (read in place from pinned memory) into d_stage2 / d_tmp, merge with the live array
    if ((rc = grow_dev(&s->d_stage2, &s->stage2_cap, ns))) return rc;
    if ((rc = grow_dev(&s->d_tmp, &s->tmp_cap, need))) return rc;
    hipLaunchKernelGGL(sched_tile_sort, dim3((unsigned)((ns + TILE - 1) / TILE)), dim3(TILE_THREADS), 0, s->stream,
                       dev_view(s->h_stage), s->d_stage2, ns);
    // merge passes (stages larger than one tile) ping-pong between d_stage2 and d_stage3
    nsgpu_event *src = s->d_stage2, *dst = s->d_stage3;
    if (ns > (uint64_t)TILE && (rc = grow_dev(&s->d_stage3, &s->stage3_cap, ns))) return rc;
    dst = s->d_stage3;
    for (uint64_t w = TILE; w < ns; w *= 2) {
      const uint64_t threads = (ns + ITEMS - 1) / ITEMS;
      hipLaunchKernelGGL(sched_merge_pass, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s->stream, src, dst,
                         ns, w);
      std::swap(src, dst);
    }
    const uint64_t threads = (need + ITEMS - 1) / ITEMS;
    hipLaunchKernelGGL(sched_merge_front, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s->stream,
                       s->d_main + s->d_head, live, src, ns, s->d_tmp, dev_view(s->h_front), take);
    NSGPU_HIP(hipGetLastError());
    NSGPU_HIP(hipStreamSynchronize(s->stream));
    std::swap(s->d_main, s->d_tmp);
    std::swap(s->cap, s->tmp_cap);
    s->d_head = take;
    s->d_n = need;
    s->stage_n = 0;
  } else if (take) {
    NSGPU_HIP(hipMemcpyAsync(s->h_front, s->d_main + s->d_head, take * sizeof(nsgpu_event), hipMemcpyDeviceToHost,
                             s->stream));
    NSGPU_HIP(hipStreamSynchronize(s->stream));
    s->d_head += take;
  }
  s->front_n = take;
  s->front_i = 0;
  if (take) s->front_bound = s->h_front[take - 1];
  s->refills++;
  const double dt = std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - t0).count();
  s->refill_ns = 0.75 * s->refill_ns + 0.25 * dt;
  return NSGPU_OK;
}

}  // namespace nsgpu

using namespace nsgpu;

extern "C" int nsgpu_sched_create(uint32_t batch, void *stream, nsgpu_sched **out) {
  if (!out) return set_error(NSGPU_EINVAL, "nsgpu_sched_create: null");
  nsgpu_sched *s = new nsgpu_sched();
  s->batch_fixed = batch;
  s->stream = (hipStream_t)stream;
  const int rc = grow_pinned(&s->h_stage, &s->stage_cap, 4096, 0);
  if (rc) {
    delete s;
    return rc;
  }
  *out = s;
  return NSGPU_OK;
}

extern "C" int nsgpu_sched_destroy(nsgpu_sched *s) {
  if (!s) return NSGPU_OK;
  for (nsgpu_event *p : {s->d_main, s->d_tmp, s->d_stage2, s->d_stage3})
    if (p) (void)hipFree(p);
  for (nsgpu_event *p : {s->h_front, s->h_stage})
    if (p) (void)hipHostFree(p);
  delete s;
  return NSGPU_OK;
}

// Scheduler::Insert (scheduler.h:75-78) for n events.
extern "C" int nsgpu_sched_insert(nsgpu_sched *s, const nsgpu_event *ev, uint64_t n) {
  if (!s || (n && !ev)) return set_error(NSGPU_EINVAL, "nsgpu_sched_insert: null");
  for (uint64_t i = 0; i < n; i++) {
    const int rc = sched_insert1(s, ev[i]);
    if (rc) return rc;
  }
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
  if (!sched_next(s, out, false, &rc)) return rc ? rc : set_error(NSGPU_ESTATE, "PeekNext on an empty scheduler");
  return NSGPU_OK;
}

extern "C" int nsgpu_sched_remove_next(nsgpu_sched *s, nsgpu_event *out) {
  if (!s || !out) return set_error(NSGPU_EINVAL, "nsgpu_sched_remove_next: null");
  return sched_remove_next1(s, out);
}

// Scheduler::Remove: the event must be pending (DefaultSimulatorImpl::Remove checks IsExpired first).
extern "C" int nsgpu_sched_remove(nsgpu_sched *s, const nsgpu_event *ev) {
  if (!s || !ev) return set_error(NSGPU_EINVAL, "nsgpu_sched_remove: null");
  if (s->size == 0) return set_error(NSGPU_ESTATE, "Remove on an empty scheduler");
  s->removed.insert(ev->uid);
  s->size--;
  return NSGPU_OK;
}

// Statistics of the front machinery: refills so far, the current front size, the refill estimate.
extern "C" int nsgpu_sched_stats(nsgpu_sched *s, uint64_t *refills, uint64_t *front, double *refill_us) {
  if (!s) return set_error(NSGPU_EINVAL, "nsgpu_sched_stats: null");
  if (refills) *refills = s->refills;
  if (front) *front = s->front_n;
  if (refill_us) *refill_us = s->refill_ns / 1e3;
  return NSGPU_OK;
}
