// Wave issue priority for latency-critical launches that run beside other streams' throughput
// kernels: s_setprio raises the wave's priority in its SIMD's instruction arbitration (0 = default).
#pragma once
#include <hip/hip_runtime.h>
#include <stdlib.h>

namespace srsgpu {
__device__ __forceinline__ void wave_prio(int prio) {
  switch (__builtin_amdgcn_readfirstlane(prio)) {
  case 1: __builtin_amdgcn_s_setprio(1); break;
  case 2: __builtin_amdgcn_s_setprio(2); break;
  case 3: __builtin_amdgcn_s_setprio(3); break;
  default: break;
  }
}
// the priority of a launch class from the environment (read per call, clamped to 0..3)
inline int env_prio(const char *name, int dflt) {
  const char *e = getenv(name);
  if (!e || !e[0]) return dflt;
  const int v = atoi(e);
  return v < 0 ? 0 : (v > 3 ? 3 : v);
}
} // namespace srsgpu
