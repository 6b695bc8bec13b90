/*
 * srsgpu batched downlink channel estimator — C ABI of the MI355X (gfx950) CRS channel
 * estimation (reference: lib/src/phy/ch_estimation/chest_dl.c, srslte_chest_dl_estimate_port
 * :641-664 and the helpers it calls).
 *
 * Supported: CRS ports 0 and 1 (cell.nof_ports 1 or 2), normal cyclic prefix, per-symbol estimation
 * (average_subframe off), REFS noise estimation. Processing per grid:
 *   - least-squares pilot estimates;
 *   - optional frequency smoothing (srslte_chest_dl_set_smooth_filter /
 *     _set_smooth_filter3_coeff; default [0.1, 0.8, 0.1]);
 *   - linear interpolation in frequency, then in time;
 *   - noise estimate as estimate_noise_pilots computes it.
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
/* srslte_chest_dl_set_smooth_filter: filter_len 0 disables smoothing (max 16 taps, odd) */
int srsgpu_chest_set_smooth_filter(srsgpu_chest_t *q, const float *filter, uint32_t filter_len);
/* srslte_chest_dl_set_smooth_filter3_coeff: [w, 1-2w, w] */
void srsgpu_chest_set_smooth_filter3_coeff(srsgpu_chest_t *q, float w);

/* Estimate nof_grids grids: grid i (subframe index sf_idx[i], host array) at d_grid + i*stride
 * complex elements. For every CRS port p of the cell (srslte_chest_dl_estimate_multi order), the
 * estimate is written at d_ce + (i*nof_ports + p)*stride and the noise estimate at
 * d_noise[i*nof_ports + p] (d_noise may be NULL). Grids of one subframe's rx antennas are simply
 * separate grids, so a subframe's estimates come out as [rx antenna][port] planes. */
int srsgpu_chest_estimate_dev(srsgpu_chest_t *q, const uint32_t *sf_idx, uint32_t nof_grids,
                              const float *d_grid, size_t stride, float *d_ce, float *d_noise);

/* Transmit side (srslte_refsignal_cs_put_sf, refsignal_dl.c:380-402): the CRS of every port of
 * the cell into nof_grids grids; port p of grid i is the plane d_grid + (i*nof_ports + p)*stride.
 * Used to synthesise traffic on the device. */
int srsgpu_chest_put_crs_dev(srsgpu_chest_t *q, const uint32_t *sf_idx, uint32_t nof_grids,
                             float *d_grid, size_t stride);

#ifdef __cplusplus
}
#endif
#endif
