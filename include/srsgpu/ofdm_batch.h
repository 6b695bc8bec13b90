/*
 * srsgpu batched OFDM receiver — C ABI of the MI355X (gfx950) FFT demodulation of downlink
 * subframes (reference: lib/src/phy/dft/ofdm.c, srslte_ofdm_rx_init/rx_sf/set_normalize
 * :47-136, 401-470; symbol sizes phy_common.c:227-275).
 *
 * Per subframe: 14 normal-CP OFDM symbols of symbol_sz samples. The first CP of each slot is
 * ceil(160 N/2048) samples, the others ceil(144 N/2048), 15 N samples in total. Each symbol gets
 * a forward DFT (unnormalised, as FFTW's forward plan; 1/sqrt(N) after
 * srsgpu_ofdm_rx_set_normalize(q, 1)). The grid row is bins [N - nre/2, N) followed by
 * [1, 1 + nre/2): the DC bin is skipped. Output: 14 x nof_prb*12 complex float per subframe, the
 * layout the channel estimator and PDSCH receiver take.
 * With srsgpu_ofdm_set_cp(q, 1) (SRSLTE_CP_EXT, ofdm.c:75-76): 12 symbols, every CP
 * ceil(512 N/2048) samples, still 15 N samples per subframe; the grid has 12 rows.
 * Non-MBSFN subframes; frequency shift (srslte_ofdm_set_freq_shift) is not supported.
 */
#ifndef SRSGPU_OFDM_BATCH_H
#define SRSGPU_OFDM_BATCH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct srsgpu_ofdm srsgpu_ofdm_t;

/* srslte_symbol_sz (standard_rates = 0) or srslte_symbol_sz_power2 (standard_rates = 1) */
int srsgpu_symbol_sz(uint32_t nof_prb, int standard_rates);

int srsgpu_ofdm_rx_create(srsgpu_ofdm_t **q, uint32_t nof_prb, uint32_t symbol_sz);
void srsgpu_ofdm_rx_destroy(srsgpu_ofdm_t *q);
void srsgpu_ofdm_rx_set_stream(srsgpu_ofdm_t *q, void *hip_stream);
void srsgpu_ofdm_rx_set_normalize(srsgpu_ofdm_t *q, int enable);
/* cyclic prefix of the handle, receive and transmit (srslte_cp_t: 0 normal, default; 1 extended) */
int srsgpu_ofdm_set_cp(srsgpu_ofdm_t *q, uint32_t cp);
/* nof_sf subframes: input i at d_in + i*in_stride complex samples (>= 15 symbol_sz), grid i at
 * d_out + i*out_stride complex elements (>= 14 * 12 * nof_prb, 12 * 12 * nof_prb for extended CP). Asynchronous on the stream. */
int srsgpu_ofdm_rx_sf_dev(srsgpu_ofdm_t *q, uint32_t nof_sf, const float *d_in, size_t in_stride,
                          float *d_out, size_t out_stride);

/* Transmit direction on the same handle (srslte_ofdm_tx_sf, ofdm.c:491-598; tx plans are
 * unnormalised by default, ofdm.c:276; srsgpu_ofdm_rx_set_normalize applies 1/sqrt(N) here too):
 * grid i at d_in + i*in_stride (14 x 12 nof_prb) -> 15 symbol_sz samples with CPs at
 * d_out + i*out_stride. Used to synthesise traffic on the device. */
int srsgpu_ofdm_tx_sf_dev(srsgpu_ofdm_t *q, uint32_t nof_sf, const float *d_in, size_t in_stride,
                          float *d_out, size_t out_stride);

#ifdef __cplusplus
}
#endif
#endif
