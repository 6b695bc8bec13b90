/*
 * srsgpu subframe batch queue — the caller side of the batched receive path for srsUE's PHY
 * workers.
 *
 * srsUE decodes one subframe per worker thread (srsue/src/phy/phch_worker.cc:548-806: OFDM,
 * channel estimation and srslte_pdsch_decode per subframe, up to nof_phy_threads workers,
 * srsue/src/phy/phy.cc:141-168). Called that way the GPU sees one subframe per launch. This queue
 * lets every worker hand its subframe over and block until its transport blocks are back, while
 * one dispatcher thread gathers the submissions into batches: it runs srsgpu_ofdm_rx_sf_dev,
 * srsgpu_chest_estimate_dev and srsgpu_pdsch_decode_dev once per batch (one host-to-device copy of
 * all time-domain samples, one device-to-host copy of all results) and wakes the submitters.
 * A batch closes when max_batch subframes are queued, when the oldest waited max_wait_us, or on
 * srsgpu_rxq_flush. All functions are thread-safe.
 */
#ifndef SRSGPU_RX_QUEUE_H
#define SRSGPU_RX_QUEUE_H

#include <stdint.h>

#include "srsgpu/pdsch_batch.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct srsgpu_rxq srsgpu_rxq_t;

typedef struct {
  /* in */
  const void *td[2];        /* host time-domain subframe per rx antenna: 15 * symbol_sz complex
                               float samples (srslte_ofdm_rx_sf's input, cyclic prefixes included) */
  srsgpu_pdsch_sf_t sf;     /* the grant; grid_offset / ce_offset / data_offset are the queue's */
  uint32_t reset_softbuffer[2]; /* new transport block: srslte_softbuffer_rx_reset first */
  uint8_t *data[2];         /* host output per TB: SRSGPU_DLSCH_DATA_LEN(tbs) bytes */
  /* out (valid once srsgpu_rxq_wait returned 0) */
  int32_t ret[2];           /* srslte_dlsch_decode2's result per TB: 0 ack, -1 CRC error, -2 invalid */
  uint32_t noi[2];          /* nof_iterations per TB */
  float noise;              /* srslte_chest_dl_get_noise_estimate of the subframe */
} srsgpu_rxq_item_t;

/* One cell (srsgpu_cell_t), FFT size symbol_sz (srsgpu_symbol_sz), nof_softbuffers HARQ
 * softbuffers of the cell's maximum code blocks, max_halfits (srslte_sch_set_max_noi). */
int srsgpu_rxq_create(srsgpu_rxq_t **q, const srsgpu_cell_t *cell, uint32_t symbol_sz,
                      uint32_t nof_softbuffers, uint32_t max_batch, uint32_t max_wait_us,
                      uint32_t max_halfits);
void srsgpu_rxq_destroy(srsgpu_rxq_t *q);
/* Queue one subframe; *ticket identifies it. The item, its input and output buffers must stay
 * valid until srsgpu_rxq_wait returns for the ticket. */
int srsgpu_rxq_submit(srsgpu_rxq_t *q, srsgpu_rxq_item_t *item, uint64_t *ticket);
/* Block until the ticket's results are written into its item: 0, or -1 if its batch failed. */
int srsgpu_rxq_wait(srsgpu_rxq_t *q, uint64_t ticket);
/* submit + wait: the synchronous call a PHY worker makes per subframe */
int srsgpu_rxq_decode(srsgpu_rxq_t *q, srsgpu_rxq_item_t *item);
/* close the current batch now */
void srsgpu_rxq_flush(srsgpu_rxq_t *q);
/* the queue's estimator and receiver, for their settings (srsgpu_chest_set_cfg / _set_smooth_filter,
 * srsgpu_pdsch_set_csi / _set_llr_8bit); change them only while nothing is queued */
struct srsgpu_chest;
struct srsgpu_chest *srsgpu_rxq_get_chest(srsgpu_rxq_t *q);
srsgpu_pdsch_t *srsgpu_rxq_get_pdsch(srsgpu_rxq_t *q);
/* batches run and subframes decoded so far */
void srsgpu_rxq_stats(srsgpu_rxq_t *q, uint64_t *batches, uint64_t *subframes);

#ifdef __cplusplus
}
#endif
#endif
