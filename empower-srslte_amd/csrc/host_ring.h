// Pinned host staging for per-call descriptor uploads. A call fills the next of N slots and uploads
// it on its stream; a slot is written again only once the upload that read it has run (its event).
// With one slot the host could prepare a call only after the GPU had reached the previous call's
// upload, i.e. the host ran in lockstep with the device; N slots let it run N calls ahead. The
// device-side copy can stay single: uploads and the kernels reading them are ordered on the stream.
#ifndef SRSGPU_HOST_RING_H
#define SRSGPU_HOST_RING_H
#include <hip/hip_runtime.h>
#include <stddef.h>

namespace srsgpu {

struct HostRing {
  static constexpr int N = 4;
  void *h[N] = {};
  hipEvent_t ev[N] = {};
  bool pending[N] = {};
  int cur = 0;
  size_t bytes = 0;

  hipError_t create(size_t b) {
    bytes = b;
    for (int i = 0; i < N; i++) {
      hipError_t e = hipHostMalloc(&h[i], b ? b : 1);
      if (e != hipSuccess) return e;
      e = hipEventCreateWithFlags(&ev[i], hipEventDisableTiming);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
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
