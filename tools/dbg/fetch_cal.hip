// FETCH_SIZE / WRITE_SIZE calibration for the access widths of the front-end kernels (the guide's x2
// correction is calibrated for 16-byte-per-lane streaming reads only). Each kernel streams a 1 GiB
// buffer once (past the 256 MiB Infinity Cache) with one access width per lane: reads of 4 / 8 /
// 16 bytes (one value per workgroup written), then writes of 2 / 4 / 8 / 16 bytes over 512 MiB.
// Run under rocprofv3 --pmc FETCH_SIZE (and separately WRITE_SIZE) --kernel-trace; the ratio of
// the counter to the bytes named in the kernel's name is the correction for that width.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/dbg/fetch_cal tools/dbg/fetch_cal.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <typename T> __global__ __launch_bounds__(256) void k_read(const T *__restrict__ p, size_t n, uint32_t *out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const T v = p[i];
    const uint32_t *w = (const uint32_t *)&v;
#pragma unroll
    for (int k = 0; k < (int)(sizeof(T) / 4); k++) acc ^= w[k];
  }
  if (acc == 0x12345678u) out[blockIdx.x] = acc; // never true for the zero buffer: keeps the loads
}

template <typename T> __global__ __launch_bounds__(256) void k_write(T *__restrict__ p, size_t n, T v) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) p[i] = v;
}

struct u16x1 {
  uint16_t a;
};

#define CHK(x)                                                                                     \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) {                                                                        \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                                     \
      return 1;                                                                                    \
    }                                                                                              \
  } while (0)

int main() {
  const size_t bytes = (size_t)1 << 30, wbytes = (size_t)1 << 29;
  void *buf = nullptr;
  uint32_t *out = nullptr;
  CHK(hipMalloc(&buf, bytes));
  CHK(hipMalloc(&out, 4 * 4096));
  CHK(hipMemset(buf, 0, bytes));
  CHK(hipDeviceSynchronize());
  const dim3 g(4096), b(256);
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(k_read<uint32_t>, g, b, 0, 0, (const uint32_t *)buf, bytes / 4, out);
    hipLaunchKernelGGL(k_read<uint2>, g, b, 0, 0, (const uint2 *)buf, bytes / 8, out);
    hipLaunchKernelGGL(k_read<uint4>, g, b, 0, 0, (const uint4 *)buf, bytes / 16, out);
    hipLaunchKernelGGL(k_write<uint16_t>, g, b, 0, 0, (uint16_t *)buf, wbytes / 2, (uint16_t)0);
    hipLaunchKernelGGL(k_write<uint32_t>, g, b, 0, 0, (uint32_t *)buf, wbytes / 4, 0u);
    hipLaunchKernelGGL(k_write<uint2>, g, b, 0, 0, (uint2 *)buf, wbytes / 8, make_uint2(0, 0));
    hipLaunchKernelGGL(k_write<uint4>, g, b, 0, 0, (uint4 *)buf, wbytes / 16, make_uint4(0, 0, 0, 0));
    CHK(hipGetLastError());
    CHK(hipDeviceSynchronize());
  }
  printf("read bytes per launch %zu, write bytes per launch %zu\n", bytes, wbytes);
  CHK(hipFree(buf));
  CHK(hipFree(out));
  return 0;
}
