/*
 * srsgpu batched downlink channel estimator — C ABI of the MI355X (gfx950) CRS channel
 * estimation (reference: lib/src/phy/ch_estimation/chest_dl.c, srslte_chest_dl_estimate_port
 * :641-664 and the helpers it calls).
 *
 * Supported: CRS ports 0-3 (cell.nof_ports 1, 2 or 4; ports 2 / 3 carry their CRS in symbols 1 and
 * 8 only, refsignal_dl.c:76-122, and are interpolated in time as chest_dl.c:427-431 does), normal
 * cyclic prefix, non-MBSFN subframes,
 * every estimator setting srsUE's phch_worker uses (phch_worker.cc:149,553-565). Processing per grid:
 *   - least-squares pilot estimates; RSRP / RSSI / RSRP correlation / CFO measurements;
 *   - noise estimate: REFS (estimate_noise_pilots), PSS or EMPTY (subframes 0 and 5 only);
 *   - frequency smoothing (srslte_chest_dl_set_smooth_filter / _set_smooth_filter3_coeff, default
 *     [0.1, 0.8, 0.1]; or smooth_filter_auto's Gaussian from the noise estimate);
 *   - per-symbol interpolation in frequency then time, or with average_subframe (srsUE's default)
 *     the subframe average interpolated in frequency and copied to all 14 symbols.
 * Grid and estimate layout: 14 OFDM symbols x nof_prb*12 subcarriers of complex float per
 * (subframe, rx antenna), the layout srslte_ofdm_rx_sf produces.
 */
#ifndef SRSGPU_CHEST_BATCH_H
#define SRSGPU_CHEST_BATCH_H

#include <stddef.h>
#include <stdint.h>

#include "srsgpu/pdsch_batch.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct srsgpu_chest srsgpu_chest_t;

int srsgpu_chest_create(srsgpu_chest_t **q, const srsgpu_cell_t *cell, uint32_t max_grids);
void srsgpu_chest_destroy(srsgpu_chest_t *q);
void srsgpu_chest_set_stream(srsgpu_chest_t *q, void *hip_stream);
/* srslte_chest_dl_set_smooth_filter: filter_len 0 disables smoothing (at most 64 taps) */
int srsgpu_chest_set_smooth_filter(srsgpu_chest_t *q, const float *filter, uint32_t filter_len);
/* srslte_chest_dl_set_smooth_filter3_coeff: [w, 1-2w, w] */
void srsgpu_chest_set_smooth_filter3_coeff(srsgpu_chest_t *q, float w);
/* srslte_chest_dl_set_smooth_filter_gauss (chest_dl.c:475-494): order + 1 taps, the reference's float
 * arithmetic (srsUE: order 4, std dev 1.0, phch_worker.cc:553-556); -1 above 64 taps */
int srsgpu_chest_set_smooth_filter_gauss(srsgpu_chest_t *q, uint32_t order, float std_dev);

/* the srslte_chest_dl_t settings chest_dl.c reads (defaults as srslte_chest_dl_init leaves them:
 * all zero = per-symbol, REFS, fixed filter, no neighbour RSRP, no CFO) */
typedef struct {
  uint32_t average_subframe;   /* srslte_chest_dl_average_subframe */
  uint32_t noise_alg;          /* 0 REFS, 1 PSS, 2 EMPTY: srslte_chest_dl_noise_alg_t order */
  uint32_t smooth_filter_auto; /* srslte_chest_dl_set_smooth_filter_auto (needs d_noise) */
  uint32_t rsrp_neighbour;     /* srslte_chest_dl_set_rsrp_neighbour: meas[2] computed */
  uint32_t cfo_estimate_enable, cfo_estimate_sf_mask; /* srslte_chest_dl_cfo_estimate_enable */
  uint32_t symbol_sz;          /* FFT size for the CFO formula (srslte_symbol_sz(nof_prb)) */
} srsgpu_chest_cfg_t;
int srsgpu_chest_set_cfg(srsgpu_chest_t *q, const srsgpu_chest_cfg_t *cfg);
/* the current settings (as set_cfg left them) */
int srsgpu_chest_get_cfg(const srsgpu_chest_t *q, srsgpu_chest_cfg_t *cfg);

/* Estimate nof_grids grids: grid i (subframe index sf_idx[i], host array) at d_grid + i*stride
 * complex elements. For every CRS port p of the cell (srslte_chest_dl_estimate_multi order), the
 * estimate is written at d_ce + (i*nof_ports + p)*stride and the noise estimate at
 * d_noise[i*nof_ports + p] (d_noise may be NULL). Grids of one subframe's rx antennas are simply
 * separate grids, so a subframe's estimates come out as [rx antenna][port] planes. */
int srsgpu_chest_estimate_dev(srsgpu_chest_t *q, const uint32_t *sf_idx, uint32_t nof_grids,
                              const float *d_grid, size_t stride, float *d_ce, float *d_noise);
/* As above, plus measurements. d_noise is in/out: with PSS / EMPTY noise it is written only for
 * grids of subframes 0 and 5 and otherwise keeps (and, for smooth_filter_auto, supplies) the
 * caller's value, as q->noise_estimate does in the reference. d_meas (may be NULL) receives per
 * (grid, port) 4 floats [rsrp, rssi, rsrp_corr, cfo]: q->rsrp / q->rssi / q->rsrp_corr / q->cfo of
 * srslte_chest_dl_estimate_port; rsrp_corr only with rsrp_neighbour and cfo only where enabled
 * for the grid's subframe, else left untouched. */
int srsgpu_chest_estimate_meas_dev(srsgpu_chest_t *q, const uint32_t *sf_idx, uint32_t nof_grids,
                                   const float *d_grid, size_t stride, float *d_ce, float *d_noise,
                                   float *d_meas);

/* Compact estimates (default off) for a receiver whose PDSCH stage interpolates in time itself
 * (srsgpu_pdsch_set_ce_rows): each (grid, port) estimate plane then holds only the rows the
 * reference's time interpolation starts from, 4 x (12 nof_prb) complex values = the frequency-
 * interpolated estimates of CRS symbols 0 / 4 / 7 / 11 (chest_dl.c:397-408), or with
 * average_subframe the one averaged row (1 x 12 nof_prb) the reference copies to every symbol
 * (:410-414). The 14-symbol estimate follows from them by chest_dl.c:416-421 exactly; the
 * measurements and noise are unchanged. 3.5x (14x) fewer estimate bytes written and read. */
void srsgpu_chest_set_ce_rows(srsgpu_chest_t *q, int enable);

/* Transmit side (srslte_refsignal_cs_put_sf, refsignal_dl.c:380-402): the CRS of every port of
 * the cell into nof_grids grids; port p of grid i is the plane d_grid + (i*nof_ports + p)*stride.
 * Used to synthesise traffic on the device. */
int srsgpu_chest_put_crs_dev(srsgpu_chest_t *q, const uint32_t *sf_idx, uint32_t nof_grids,
                             float *d_grid, size_t stride);

#ifdef __cplusplus
}
#endif
#endif
