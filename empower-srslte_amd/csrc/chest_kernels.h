// Internal launch interface of the CRS channel-estimation kernel (chest_kernels.hip).
#ifndef SRSGPU_CHEST_KERNELS_H
#define SRSGPU_CHEST_KERNELS_H
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace srsgpu {
// one (subframe, rx antenna, CRS port): grid and ce are 14 x 12*nof_prb complex planes
struct ChestItem {
  const float2 *grid;
  float2 *ce;
  float *noise; // noise estimate out (NULL: not computed)
  uint32_t sf_idx;
  uint32_t port; // 0 or 1: frequency shift v (refsignal_dl.c:40-57)
};
// crs: [10 subframes][4 CRS symbols][2*nof_prb] port-0/1 pilots; filt: flen taps (0: no smoothing)
hipError_t launch_chest(const ChestItem *d_items, int n, int nprb, int cell_id, const float2 *crs,
                        const float *filt, int flen, hipStream_t st);
// items[i].ce is the grid plane the port's CRS is written into
hipError_t launch_crs_put(const ChestItem *d_items, int n, int nprb, int cell_id, const float2 *crs,
                          hipStream_t st);
} // namespace srsgpu
#endif
