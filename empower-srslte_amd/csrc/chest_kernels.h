// Internal launch interface of the CRS channel-estimation kernel (chest_kernels.hip).
#ifndef SRSGPU_CHEST_KERNELS_H
#define SRSGPU_CHEST_KERNELS_H
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace srsgpu {
// one (subframe, rx antenna, CRS port): grid and ce are 14 (12 extended CP) x 12*nof_prb complex planes
struct ChestItem {
  const float2 *grid;
  float2 *ce;
  float *noise; // noise estimate in/out (NULL: not computed); see ChestCfg::noise_alg
  float *meas;  // [rsrp, rssi, rsrp_corr, cfo] out (NULL: not computed)
  uint32_t sf_idx;
  uint32_t port; // 0 or 1: frequency shift v (refsignal_dl.c:40-57)
  uint32_t cfo;  // CFO estimated for this grid (cfo_estimate_enable and the subframe mask)
  uint32_t pad;
};
// per-estimator configuration (the srslte_chest_dl_t fields chest_dl.c reads)
struct ChestCfg {
  int nprb, cell_id, nof_ports;
  int flen;           // smoothing taps (0: none; chest_dl.c:620 rule already applied by the host)
  int average;        // average_subframe
  int noise_alg;      // 0 REFS, 1 PSS, 2 EMPTY (srslte_chest_dl_noise_alg_t)
  int filt_auto;      // smooth_filter_auto: order-4 Gaussian from the noise estimate
  int rsrp_neighbour; // rsrp_corr computed
  float cfo_n, cfo_ng; // CFO formula: symbol size and normal-CP length of symbol 1
  int ns;             // OFDM symbols per slot: 7 normal CP, 6 extended CP (grid rows 2 ns)
  int rows;           // compact output: the CRS symbols' frequency-interpolated rows (4 x nsc, or
                      // the averaged row, 1 x nsc) instead of the 14 x nsc grid (srsgpu_chest_set_ce_rows)
};
// crs: [10 subframes][4 CRS symbols][2*nof_prb] port-0/1 pilots; filt: up to 64 taps; pss: the
// 62-element PSS of the cell's N_id_2
hipError_t launch_chest(const ChestItem *d_items, int n, const ChestCfg &cfg, const float2 *crs,
                        const float *filt, const float2 *pss, hipStream_t st);
// items[i].ce is the grid plane the port's CRS is written into
hipError_t launch_crs_put(const ChestItem *d_items, int n, int nprb, int cell_id, int ns, const float2 *crs,
                          hipStream_t st);
} // namespace srsgpu
#endif
