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

// an HBM-streaming kernel on its own stream for `iters` passes over 1 GiB: the copies' competition
__global__ void k_busy(float4 *a, size_t n, int iters) {
  for (int it = 0; it < iters; it++)
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
      float4 v = a[i];
      v.x += 1.f;
      a[i] = v;
    }
}

static int run(const char *name, const char *src, char *dst, size_t bytes, int nstreams, hipStream_t *st,
               hipEvent_t e0, hipEvent_t e1) {
  std::vector<float> ms;
  for (int rep = 0; rep < 6; rep++) {
    for (int k = 0; k < nstreams; k++) CHK(hipStreamSynchronize(st[k])); // not the device: see k_busy
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
  // as the queue copies registered rows: runs of 20 rows of 122,880 bytes (SC16 20 MHz subframes) at
  // row offsets inside the registered region, one hipMemcpyAsync per run
  {
    const size_t row = 122880, rows = bytes / row, runl = 20;
    std::vector<float> ms;
    for (int rep = 0; rep < 4; rep++) {
      CHK(hipStreamSynchronize(st[0]));
      CHK(hipEventRecord(e0, st[0]));
      const double h0 = (double)clock() / CLOCKS_PER_SEC;
      for (size_t r = 1; r + runl <= rows; r += runl + 1)
        CHK(hipMemcpyAsync(dev + r * row, reg + r * row, runl * row, hipMemcpyHostToDevice, st[0]));
      const double h1 = (double)clock() / CLOCKS_PER_SEC;
      CHK(hipEventRecord(e1, st[0]));
      CHK(hipEventSynchronize(e1));
      float t = 0;
      CHK(hipEventElapsedTime(&t, e0, e1));
      if (rep) printf("registered runs of %zu rows at offsets: %.2f GB/s (%.3f ms), host %.3f ms to enqueue\n", runl,
                      (double)(rows / (runl + 1)) * runl * row / (t * 1e-3) / 1e9, t, (h1 - h0) * 1e3);
    }
  }
  // single rows (one 20 MHz SC16 subframe each) at every other row offset: one hipMemcpyAsync per row
  // against one hipMemcpyBatchAsync of the same copies (the per-copy overhead of the copy engine)
  for (size_t runl : {(size_t)1, (size_t)20}) {
    const size_t row = 122880, rows = bytes / row;
    std::vector<void *> ds, ss;
    std::vector<size_t> sz;
    for (size_t r = 1; r + runl <= rows; r += runl + 1) {
      ds.push_back(dev + r * row);
      ss.push_back(reg + r * row);
      sz.push_back(runl * row);
    }
    for (int mode = 0; mode < 2; mode++) {
      std::vector<float> ms;
      for (int rep = 0; rep < 4; rep++) {
        CHK(hipStreamSynchronize(st[0]));
        CHK(hipEventRecord(e0, st[0]));
        if (mode == 0) {
          for (size_t k = 0; k < ds.size(); k++)
            CHK(hipMemcpyAsync(ds[k], ss[k], sz[k], hipMemcpyHostToDevice, st[0]));
        } else {
          size_t fail = 0;
          CHK(hipMemcpyBatchAsync(ds.data(), ss.data(), sz.data(), ds.size(), nullptr, nullptr, 0, &fail, st[0]));
        }
        CHK(hipEventRecord(e1, st[0]));
        CHK(hipEventSynchronize(e1));
        float t = 0;
        CHK(hipEventElapsedTime(&t, e0, e1));
        if (rep) ms.push_back(t);
      }
      std::sort(ms.begin(), ms.end());
      printf("%zu copies of %zu row(s), %s: %.2f GB/s (%.3f ms, %.1f us per copy)\n", ds.size(), runl,
             mode ? "hipMemcpyBatchAsync" : "hipMemcpyAsync each", ds.size() * runl * row / (ms[1] * 1e-3) / 1e9,
             ms[1], ms[1] * 1e3 / ds.size());
    }
  }
  // the same with an HBM-bound kernel running beside the copy (as the queue's decode does)
  float4 *busy = nullptr;
  const size_t bn = ((size_t)1 << 30) / 16;
  CHK(hipMalloc(&busy, bn * 16));
  hipStream_t bs;
  CHK(hipStreamCreateWithFlags(&bs, hipStreamNonBlocking));
  hipLaunchKernelGGL(k_busy, dim3(2048), dim3(256), 0, bs, busy, bn, 200);
  if (run("pinned, HBM kernel beside", pinned, dev, bytes, 1, st, e0, e1)) return 1;
  if (run("registered, HBM kernel beside", reg, dev, bytes, 1, st, e0, e1)) return 1;
  CHK(hipStreamSynchronize(bs));
  CHK(hipFree(busy));
  CHK(hipHostUnregister(reg));
  free(reg);
  CHK(hipHostFree(pinned));
  CHK(hipFree(dev));
  return 0;
}
