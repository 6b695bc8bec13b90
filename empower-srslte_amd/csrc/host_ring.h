// Pinned host staging for per-call descriptor uploads. A call fills the next of N slots and uploads
// it on its stream; a slot is written again only once the upload that read it has run (its event).
// With one slot the host could prepare a call only after the GPU had reached the previous call's
// upload, i.e. the host ran in lockstep with the device; N slots let it run N calls ahead. The
// device-side copy can stay single: uploads and the kernels reading them are ordered on the stream.
#ifndef SRSGPU_HOST_RING_H
#define SRSGPU_HOST_RING_H
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>

namespace srsgpu {

// bytes from a device-visible view of pinned host memory into device memory, by a kernel on st
// (h2d.hip); falls back to hipMemcpyAsync for unaligned blocks
hipError_t launch_h2d(void *dst, const void *src_dev, size_t bytes, hipStream_t st);

struct HostRing {
  static constexpr int N = 4;
  void *h[N] = {};
  const char *dv[N] = {}; // each slot's device view (hipHostGetDevicePointer)
  hipEvent_t ev[N] = {};
  bool pending[N] = {};
  int cur = 0;
  size_t bytes = 0;
  // uploads by a kernel (launch_h2d) in the stream's order; SRSGPU_H2D=dma: hipMemcpyAsync (SDMA)
  bool kernel_h2d = true;

  hipError_t create(size_t b) {
    bytes = b;
    if (const char *e = getenv("SRSGPU_H2D")) kernel_h2d = strcmp(e, "dma") != 0;
    for (int i = 0; i < N; i++) {
      hipError_t e = hipHostMalloc(&h[i], b ? b : 1);
      if (e != hipSuccess) return e;
      void *d = nullptr;
      if (hipHostGetDevicePointer(&d, h[i], 0) != hipSuccess || !d) kernel_h2d = false;
      dv[i] = (const char *)d;
      e = hipEventCreateWithFlags(&ev[i], hipEventDisableTiming);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }
  // `bytes` at `src` (inside the current slot) to device memory `dst`, ordered on st
  hipError_t upload(void *dst, const void *src, size_t n, hipStream_t st) {
    const char *s = (const char *)src, *base = (const char *)h[cur];
    if (kernel_h2d && s >= base && s + n <= base + bytes) return launch_h2d(dst, dv[cur] + (s - base), n, st);
    return hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, st);
  }
  void destroy() {
    for (int i = 0; i < N; i++) {
      if (pending[i]) (void)hipEventSynchronize(ev[i]);
      if (h[i]) (void)hipHostFree(h[i]);
      if (ev[i]) (void)hipEventDestroy(ev[i]);
      h[i] = nullptr;
      ev[i] = nullptr;
      pending[i] = false;
    }
  }
  // the next slot, once its previous upload has run
  void *acquire(hipError_t *err) {
    cur = (cur + 1) % N;
    *err = pending[cur] ? hipEventSynchronize(ev[cur]) : hipSuccess;
    pending[cur] = false;
    return h[cur];
  }
  // after the upload of the current slot was enqueued on st
  hipError_t mark(hipStream_t st) {
    pending[cur] = true;
    return hipEventRecord(ev[cur], st);
  }
};

} // namespace srsgpu
#endif
