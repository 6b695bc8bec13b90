/*
 * srsgpu batched PCFICH decoder — C ABI of the MI355X (gfx950) CFI detection that precedes the
 * PDCCH search and the PDSCH grant on every subframe (reference: lib/src/phch/pcfich.c:178-241
 * srslte_pcfich_decode_multi, REG map regs.c:477-512). One wavefront per subframe: the 16 PCFICH
 * REs of OFDM symbol 0 are equalised (1 port: srslte_predecoding_single_multi with the noise
 * estimate; 2 ports: transmit diversity + layer demapping), QPSK soft-demapped, descrambled and
 * correlated with the three CFI codewords; bit-exact with the reference (tests/test_pcfich.py).
 *
 * Grid / estimate layout as srsgpu/pdsch_batch.h: plane a of the grid at d_grid + grid_offset +
 * a*ant_stride, plane (a, p) of the estimate at d_ce + ce_offset + (a*nof_ports + p)*ant_stride.
 */
#ifndef SRSGPU_PCFICH_BATCH_H
#define SRSGPU_PCFICH_BATCH_H

#include <stddef.h>
#include <stdint.h>

#include "srsgpu/pdsch_batch.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct srsgpu_pcfich srsgpu_pcfich_t;

typedef struct {
  uint64_t grid_offset; /* this subframe's [rx antenna] grid planes (complex elements) */
  uint64_t ce_offset;   /* this subframe's [rx antenna][port] estimate planes */
  uint32_t sf_idx;      /* subframe index 0..9 (scrambling, pcfich.c:96-101) */
  float noise_estimate; /* the noise_estimate argument of srslte_pcfich_decode_multi */
} srsgpu_pcfich_sf_t;

/* srslte_pcfich_init + srslte_pcfich_set_cell: RE map and the ten scrambling sequences. -1 on an
 * invalid cell (1 or 2 ports, 1 or 2 rx antennas, 6..110 PRB). */
int srsgpu_pcfich_create(srsgpu_pcfich_t **q, const srsgpu_cell_t *cell);
void srsgpu_pcfich_destroy(srsgpu_pcfich_t *q);
/* Take each subframe's noise estimate from device memory instead of sf[i].noise_estimate: subframe
 * i of a call uses d_noise[i] (e.g. the batch's srslte_chest_dl_get_noise_estimate values, left in
 * HBM by the estimator). NULL restores sf[i].noise_estimate. */
void srsgpu_pcfich_set_noise_dev(srsgpu_pcfich_t *q, const float *d_noise);
/* the 16 RE indices of symbol 0 (srslte_regs_pcfich_get order) */
int srsgpu_pcfich_re_map(const srsgpu_pcfich_t *q, uint32_t idx[16]);
/* srslte_pcfich_decode_multi for nof_sf subframes: d_cfi[i] = the detected CFI (1..3; 1 when no
 * correlation is positive, as the reference), d_corr[i] = the winning correlation (the
 * reference's corr_result). sf is a host array; d_* are device pointers; hip_stream may be NULL.
 * Returns 0, or -1 on invalid input. Asynchronous on the stream. */
int srsgpu_pcfich_decode_dev(srsgpu_pcfich_t *q, const srsgpu_pcfich_sf_t *sf, uint32_t nof_sf,
                             const float *d_grid, const float *d_ce, size_t ant_stride,
                             uint32_t *d_cfi, float *d_corr, void *hip_stream);

#ifdef __cplusplus
}
#endif
#endif
