// Descriptor uploads as a kernel (host_ring.h): the per-call descriptor blocks (a few KB to a few
// hundred KB of pinned host memory) are fetched by a small kernel that reads the device-visible view
// of the pinned slot over the fabric and writes the device copy, in the stream's own order. An SDMA
// copy between two kernels of a stream (hipMemcpyAsync host -> device) left the stream idle for
// 30-55 us per upload in the headline's kernel trace (profiles/r06_s5_kernel_stats_headline.csv:
// the ofdm -> chest, chest -> pdsch and reset -> de-RM gaps); a kernel in the same queue starts when
// the previous one ends.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "host_ring.h"

namespace srsgpu {

typedef uint32_t h2d_u4 __attribute__((ext_vector_type(4)));

// n16 16-byte vectors, then `tail` single bytes (all of an unaligned block); many loads in flight per
// thread (fabric latency). Either side may be a device view of pinned host memory.
__global__ __launch_bounds__(256) void k_h2d(const h2d_u4 *__restrict__ src, h2d_u4 *__restrict__ dst, size_t n16,
                                             const uint8_t *__restrict__ src_b, uint8_t *__restrict__ dst_b,
                                             size_t tail) {
  const size_t stride = (size_t)gridDim.x * 256;
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const h2d_u4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
    dst[i] = a;
    dst[i + stride] = b;
    dst[i + 2 * stride] = c;
    dst[i + 3 * stride] = d;
  }
  for (; i < n16; i += stride) dst[i] = src[i];
  for (size_t j = (size_t)blockIdx.x * 256 + threadIdx.x; j < tail; j += stride) dst_b[j] = src_b[j];
}

hipError_t launch_h2d(void *dst, const void *src_dev, size_t bytes, hipStream_t st) {
  if (!bytes) return hipSuccess;
  const bool aligned = ((uintptr_t)dst % 16) == 0 && ((uintptr_t)src_dev % 16) == 0;
  const size_t n16 = aligned ? bytes / 16 : 0;
  const size_t tail = bytes - n16 * 16;
  if (tail > 65536) return hipMemcpyAsync(dst, src_dev, bytes, hipMemcpyDefault, st); // large and unaligned: DMA
  const unsigned blocks = (unsigned)std::max<size_t>(1, std::min<size_t>(64, (n16 + tail / 16 + 1023) / 1024));
  hipLaunchKernelGGL(k_h2d, dim3(blocks), dim3(256), 0, st, (const h2d_u4 *)src_dev, (h2d_u4 *)dst, n16,
                     (const uint8_t *)src_dev + n16 * 16, (uint8_t *)dst + n16 * 16, tail);
  return hipGetLastError();
}

} // namespace srsgpu
