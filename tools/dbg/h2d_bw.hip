// Host-to-device copy bandwidth on the box, for the queue's ingest (rx_queue.hip stage()): one
// hipMemcpyAsync of `mb` MiB from pinned memory (hipHostMalloc), from malloc'd memory registered
// with hipHostRegister (as srsgpu_rxq_register does), and the same split over 2 and 4 streams.
// Prints GB/s per case (median of 5). Build:
//   hipcc --offload-arch=gfx950 -O3 -o tools/dbg/h2d_bw tools/dbg/h2d_bw.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#define CHK(x)                                                                                     \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) {                                                                        \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                                     \
      return 1;                                                                                    \
    }                                                                                              \
  } while (0)

static int run(const char *name, const char *src, char *dst, size_t bytes, int nstreams, hipStream_t *st,
               hipEvent_t e0, hipEvent_t e1) {
  std::vector<float> ms;
  for (int rep = 0; rep < 6; rep++) {
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0, st[0]));
    for (int k = 1; k < nstreams; k++) CHK(hipStreamWaitEvent(st[k], e0, 0));
    const size_t piece = bytes / nstreams;
    for (int k = 0; k < nstreams; k++)
      CHK(hipMemcpyAsync(dst + k * piece, src + k * piece, piece, hipMemcpyHostToDevice, st[k]));
    for (int k = 1; k < nstreams; k++) {
      hipEvent_t j;
      CHK(hipEventCreate(&j));
      CHK(hipEventRecord(j, st[k]));
      CHK(hipStreamWaitEvent(st[0], j, 0));
      CHK(hipEventDestroy(j));
    }
    CHK(hipEventRecord(e1, st[0]));
    CHK(hipEventSynchronize(e1));
    float t = 0;
    CHK(hipEventElapsedTime(&t, e0, e1));
    if (rep) ms.push_back(t);
  }
  std::sort(ms.begin(), ms.end());
  printf("%-28s %d stream(s): %7.2f GB/s (%.3f ms for %zu MB)\n", name, nstreams, bytes / (ms[2] * 1e-3) / 1e9,
         ms[2], bytes >> 20);
  return 0;
}

int main(int argc, char **argv) {
  const size_t bytes = (size_t)(argc > 1 ? atoi(argv[1]) : 128) << 20;
  char *pinned = nullptr, *dev = nullptr;
  CHK(hipHostMalloc(&pinned, bytes));
  memset(pinned, 1, bytes);
  char *reg = (char *)aligned_alloc(4096, bytes);
  memset(reg, 2, bytes);
  CHK(hipHostRegister(reg, bytes, hipHostRegisterMapped));
  CHK(hipMalloc(&dev, bytes));
  hipStream_t st[4];
  for (auto &s : st) CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  for (int ns : {1, 2, 4}) {
    if (run("hipHostMalloc", pinned, dev, bytes, ns, st, e0, e1)) return 1;
    if (run("hipHostRegister(malloc)", reg, dev, bytes, ns, st, e0, e1)) return 1;
  }
  CHK(hipHostUnregister(reg));
  free(reg);
  CHK(hipHostFree(pinned));
  CHK(hipFree(dev));
  return 0;
}
