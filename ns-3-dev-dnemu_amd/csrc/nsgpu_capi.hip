// nsgpu_capi.hip — library plumbing of the C-ABI (errors, device memory, streams).
#include <string.h>
#include "nsgpu_internal.h"

namespace nsgpu {
static thread_local char g_err[512] = "";

int set_error(int code, const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}
}  // namespace nsgpu

using nsgpu::set_error;

extern "C" {

int nsgpu_version(void) { return 1; }
const char *nsgpu_last_error(void) { return nsgpu::g_err; }

int nsgpu_device_count(int *count) {
  NSGPU_HIP(hipGetDeviceCount(count));
  return NSGPU_OK;
}
int nsgpu_set_device(int device) {
  NSGPU_HIP(hipSetDevice(device));
  return NSGPU_OK;
}
int nsgpu_malloc(void **d_ptr, size_t bytes) {
  if (!d_ptr) return set_error(NSGPU_EINVAL, "nsgpu_malloc: null");
  hipError_t e = hipMalloc(d_ptr, bytes ? bytes : 1);
  if (e != hipSuccess) return set_error(NSGPU_ENOMEM, "hipMalloc(%zu): %s", bytes, hipGetErrorString(e));
  return NSGPU_OK;
}
int nsgpu_free(void *d_ptr) {
  NSGPU_HIP(hipFree(d_ptr));
  return NSGPU_OK;
}
int nsgpu_memcpy_htod(void *d_dst, const void *h_src, size_t bytes, void *stream) {
  NSGPU_HIP(hipMemcpyAsync(d_dst, h_src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream));
  return NSGPU_OK;
}
int nsgpu_memcpy_dtoh(void *h_dst, const void *d_src, size_t bytes, void *stream) {
  NSGPU_HIP(hipMemcpyAsync(h_dst, d_src, bytes, hipMemcpyDeviceToHost, (hipStream_t)stream));
  NSGPU_HIP(hipStreamSynchronize((hipStream_t)stream));
  return NSGPU_OK;
}
int nsgpu_memset(void *d_dst, int value, size_t bytes, void *stream) {
  NSGPU_HIP(hipMemsetAsync(d_dst, value, bytes, (hipStream_t)stream));
  return NSGPU_OK;
}
int nsgpu_device_synchronize(void) {
  NSGPU_HIP(hipDeviceSynchronize());
  return NSGPU_OK;
}
int nsgpu_stream_create(void **stream) {
  hipStream_t s;
  NSGPU_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  *stream = (void *)s;
  return NSGPU_OK;
}
int nsgpu_stream_destroy(void *stream) {
  NSGPU_HIP(hipStreamDestroy((hipStream_t)stream));
  return NSGPU_OK;
}
int nsgpu_stream_sync(void *stream) {
  NSGPU_HIP(hipStreamSynchronize((hipStream_t)stream));
  return NSGPU_OK;
}

int nsgpu_event_create(void **event) {
  hipEvent_t e;
  NSGPU_HIP(hipEventCreate(&e));
  *event = (void *)e;
  return NSGPU_OK;
}
int nsgpu_event_destroy(void *event) {
  NSGPU_HIP(hipEventDestroy((hipEvent_t)event));
  return NSGPU_OK;
}
int nsgpu_event_record(void *event, void *stream) {
  NSGPU_HIP(hipEventRecord((hipEvent_t)event, (hipStream_t)stream));
  return NSGPU_OK;
}
int nsgpu_event_elapsed_ms(void *start, void *stop, float *ms) {
  NSGPU_HIP(hipEventSynchronize((hipEvent_t)stop));
  NSGPU_HIP(hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)stop));
  return NSGPU_OK;
}

}  // extern "C"
