// Address-space helper for kernels that read their buffer pointers from item descriptors.
#ifndef SRSGPU_GMEM_H
#define SRSGPU_GMEM_H
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace srsgpu {
// A pointer loaded from a descriptor is generic to the compiler, so every access through it is a
// flat instruction, which also counts against lgkmcnt: LDS waits then wait for global loads in
// flight. Descriptors only ever point at global memory; the round trip through an address-space-1
// pointer tells the address-space inference so, and the accesses become global_* instructions.
template <typename T> __device__ __forceinline__ T *gmem(T *p) {
  typedef __attribute__((address_space(1))) T gT;
  return (T *)(gT *)(__attribute__((address_space(1))) void *)(uintptr_t)p;
}
} // namespace srsgpu
#endif
