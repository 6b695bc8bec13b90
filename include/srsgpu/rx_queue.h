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

#include "srsgpu/dci.h"
#include "srsgpu/pdsch_batch.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct srsgpu_rxq srsgpu_rxq_t;

/* The estimator's per-subframe measurements as srsUE's PHY worker reads them after each subframe
 * (srslte_chest_dl_get_cfo / _get_snr / _get_rsrp / _get_rsrq / _get_rssi / _get_rsrp_neighbour,
 * chest_dl.c:737-846; phch_worker.cc:226-241, 301, 313, 1618-1628), linear values. Like the reference's
 * estimator object, the queue carries the CFO across subframes that do not estimate it
 * (srsgpu_chest_cfg_t.cfo_estimate_sf_mask) and the neighbour RSRP while rsrp_neighbour is off. */
typedef struct {
  float cfo, snr, rsrp, rsrq, rssi, rsrp_neighbour;
} srsgpu_rxq_meas_t;

typedef struct {
  /* in */
  const void *td[2];        /* host time-domain subframe per rx antenna: 15 * symbol_sz complex
                               float samples (srslte_ofdm_rx_sf's input, cyclic prefixes included;
                               int16 I/Q pairs with SRSGPU_RXQ_SC16) */
  srsgpu_pdsch_sf_t sf;     /* the grant; grid_offset / ce_offset / data_offset are the queue's */
  uint32_t reset_softbuffer[2]; /* new transport block: srslte_softbuffer_rx_reset first */
  uint8_t *data[2];         /* host output per TB: SRSGPU_DLSCH_DATA_LEN(tbs) bytes */
  /* out (valid once srsgpu_rxq_wait returned 0) */
  int32_t ret[2];           /* srslte_dlsch_decode2's result per TB: 0 ack, -1 CRC error, -2 invalid */
  uint32_t noi[2];          /* nof_iterations per TB */
  float noise;              /* srslte_chest_dl_get_noise_estimate of the subframe */
  srsgpu_rxq_meas_t meas;
} srsgpu_rxq_item_t;

/* srslte_ue_dl_decode_rnti (src/phy/ue/ue_dl.c:467-620) of one subframe, the call srsUE's PHY worker
 * makes when it has no grant yet (phch_worker.cc:548-806 -> ue_dl): FFT, channel estimation,
 * PCFICH (CFI), PDCCH LLRs and the DL DCI blind search for rnti, the DCI unpacked into the grant
 * (srslte_dci_msg_to_dl_grant), the redundancy version and softbuffer resets of ue_dl.c:503-534,
 * the MIMO type of the format (:536-566), then the PDSCH / DL-SCH decode of the grant. In a batch
 * the grids, estimates and LLRs stay in HBM; only the CFIs and the DCI search results (a few hundred
 * bytes per subframe) come back to the host between the stages, to build the next stage's
 * descriptors as the reference's host code does. */
typedef struct {
  /* in */
  const void *td[2];       /* time-domain subframe per rx antenna, as srsgpu_rxq_item_t */
  uint32_t tti;            /* sf_idx = tti % 10; the SI-RNTI redundancy version uses tti / 10 */
  uint16_t rnti;
  uint32_t tm;             /* the ue_dci_formats row (ue_dl.c:41-50): 0..7 for TM1..TM8 */
  int32_t rnti_type;       /* < 0: from the RNTI value (srslte_ue_dl_find_dl_dci); else the
                              srslte_rnti_type_t of srslte_ue_dl_find_dl_dci_type */
  uint32_t softbuffer[2];  /* q->softbuffers[0..1]: reset_tbs'd for every found grant */
  uint8_t *data[2];        /* host output per TB: SRSGPU_DLSCH_DATA_LEN(tbs) bytes */
  uint8_t acks[2];         /* in/out, as srslte_pdsch_decode's acks: a true ack skips the TB (its data,
                              noi and softbuffer are left as they are) */
  /* out (valid once srsgpu_rxq_wait returned 0) */
  int32_t ret;             /* srslte_ue_dl_decode_rnti's return: the grant's TB 0 size when a DCI
                              was found and the PDSCH decoded, 0 when no DCI was found, -1 on the
                              reference's error paths (DCI that does not unpack, a format the
                              reference does not decode, a PDSCH configuration error) */
  uint32_t cfi;            /* PCFICH result */
  float cfi_corr;
  int32_t found;           /* the search's result: 1 found, 0 not, -1 error (ue_dl.c:768-810) */
  uint32_t format;         /* SRSGPU_DCI_FORMAT* of the found DCI */
  uint32_t L, ncce;        /* its location */
  uint32_t mimo_type;      /* SRSGPU_MIMO_* the grant was decoded with */
  uint32_t rv[2];
  srsgpu_ra_dl_grant_t grant;
  uint32_t noi[2];
  float noise;             /* srslte_chest_dl_get_noise_estimate */
  /* the UL search that phch_worker runs on the same PDCCH after the DL one (phch_worker.cc:938-967):
   * srslte_ue_dl_find_ul_dci (ue_dl.c:811-838) and srslte_dci_msg_to_ul_grant of its result */
  uint16_t ul_rnti;        /* in: 0 = no UL search */
  uint32_t n_rb_ho;        /* in: PUSCH hopping offset (pusch_hopping.hopping_offset) */
  int32_t ul_found;        /* out: 1 found (a format 0 message), 0 not, -1 the search's error */
  uint32_t ul_L, ul_ncce, ul_nof_bits;
  uint8_t ul_data[128];    /* the message buffer (payload, 16 CRC bits) */
  int32_t ul_grant_ret;    /* srslte_dci_msg_to_ul_grant's return (-1 when nothing was found) */
  srsgpu_ra_ul_dci_t ul_dci;
  srsgpu_ra_ul_grant_t ul_grant;
  uint8_t acked_in[2];     /* internal: acks as submitted */
  /* out: the found DL DCI (srslte_dci_msg_t's nof_bits and message buffer: payload + 16 CRC bits) */
  uint32_t dci_nof_bits;
  uint8_t dci_data[128];
  srsgpu_rxq_meas_t meas;  /* out */
  /* in: the worker's TM3 / TM4 feedback for its UCI (phch_worker::compute_ri, phch_worker.cc:522-540):
   * SRSGPU_FEEDBACK_CN (srslte_ue_dl_ri_select) and / or SRSGPU_FEEDBACK_PMI
   * (srslte_ue_dl_ri_pmi_select) on this subframe's estimates (srsgpu_pdsch_feedback_dev) */
  uint32_t feedback;
  srsgpu_feedback_t fb;    /* out */
} srsgpu_rxq_ue_dl_t;

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
/* srslte_ue_dl_decode_rnti through the queue: submit (the item, its inputs and outputs stay valid
 * until the wait returns) and the synchronous form. Grant items (srsgpu_rxq_submit) and ue_dl items
 * share the queue and its batches. */
int srsgpu_rxq_submit_ue_dl(srsgpu_rxq_t *q, srsgpu_rxq_ue_dl_t *item, uint64_t *ticket);
int srsgpu_rxq_decode_rnti(srsgpu_rxq_t *q, srsgpu_rxq_ue_dl_t *item);
/* PHICH configuration of the cell (srslte_regs_init from the MIB: length 0 normal / 1 extended,
 * resources 0..3 = 1/6, 1/2, 1, 2): sets the PDCCH REG map of the ue_dl items. Default normal, 1.
 * Takes effect from the next batch the dispatcher starts (safe while batches are in flight). */
int srsgpu_rxq_set_phich(srsgpu_rxq_t *q, uint32_t phich_length, uint32_t phich_resources);
/* Zero-copy ingest: pin caller memory that holds time-domain subframes (hipHostRegister, mapped).
 * Submissions whose td buffers lie inside a registered region skip the host copy into the queue's
 * staging: the batch DMAs them straight from the caller's memory, one copy per span of td buffers
 * that are contiguous there or at most 512 KB apart in one region (the copy then also reads the
 * registered bytes between them, and discards them; SRSGPU_RXQ_INGEST=kernel: one kernel per batch
 * reads the td buffers over PCIe instead). Such a td buffer is read after srsgpu_rxq_submit returns: keep it unchanged until the
 * ticket is waited for (unregistered ones are copied before submit returns). td pointers must be
 * 16-byte aligned to be read in place (others are staged). The region must stay valid until
 * unregistered; unregister waits until nothing queued points into it. */
int srsgpu_rxq_register(srsgpu_rxq_t *q, void *host, size_t bytes);
int srsgpu_rxq_unregister(srsgpu_rxq_t *q, void *host);
/* Queue-owned device-visible host memory (hipHostMalloc, mapped): the recommended home of the
 * caller's sample rings and TB output buffers. A block from here is a zero-copy region of this queue
 * exactly as a registered one (td buffers DMA'd from it, TB bytes written into it by the decoder),
 * but its memory is never the caller's own: the caller never frees pinned pages itself, so no later
 * allocation of the caller's can land on pages the runtime still tracks as pinned. Returns the block
 * (16-byte aligned) or NULL. srsgpu_rxq_free_host waits until nothing queued points into it, then
 * frees it; blocks not freed are freed by srsgpu_rxq_destroy. */
void *srsgpu_rxq_alloc_host(srsgpu_rxq_t *q, size_t bytes);
int srsgpu_rxq_free_host(srsgpu_rxq_t *q, void *host);
/* Sample format of every td buffer: complex float (default; srslte_ofdm_rx_sf's input) or the radio's
 * int16 I/Q pairs (4 bytes per sample, half the PCIe bytes), converted on the GPU as value * scale
 * (0: 1 / 32768, UHD's sc16 -> fc32). Waits until nothing is queued. */
#define SRSGPU_RXQ_CF32 0
#define SRSGPU_RXQ_SC16 1
int srsgpu_rxq_set_input_format(srsgpu_rxq_t *q, uint32_t format, float scale);
/* antenna rows ingested so far: read from registered memory / staged by a host copy */
void srsgpu_rxq_ingest_stats(srsgpu_rxq_t *q, uint64_t *zero_copy_rows, uint64_t *staged_rows);
/* close the current batch now */
void srsgpu_rxq_flush(srsgpu_rxq_t *q);
/* the queue's estimator and receiver, for their settings (srsgpu_chest_set_cfg / _set_smooth_filter,
 * srsgpu_pdsch_set_csi / _set_llr_8bit); change them only while nothing is queued */
struct srsgpu_chest;
struct srsgpu_chest *srsgpu_rxq_get_chest(srsgpu_rxq_t *q);
srsgpu_pdsch_t *srsgpu_rxq_get_pdsch(srsgpu_rxq_t *q);
/* Seconds the queue's threads spent so far per stage (n <= 8 values): 0 front end enqueue (OFDM, channel
 * estimation, measurements), 1 control channel (PCFICH / PDCCH / DCI search round trips), 2 grants and
 * softbuffer resets, 3 PDSCH / DL-SCH enqueue, 4 waiting for the batch's results on the GPU, 5 result
 * copy-out into the items, 6 staging of the samples (closer thread). */
void srsgpu_rxq_timing(srsgpu_rxq_t *q, double *sec, uint32_t n);
/* batches run and subframes decoded so far */
void srsgpu_rxq_stats(srsgpu_rxq_t *q, uint64_t *batches, uint64_t *subframes);
/* Load generator for the queue (no reference counterpart; it stands in for srsUE's pool of PHY
 * worker threads, phch_worker.cc:548-806): `workers` native threads submit items[i] for
 * i = w, w + workers, ... and one collector thread waits for the tickets in index order. Item i
 * reuses the softbuffer / output slot of item i - reuse (0: no reuse), so its submission waits until
 * that item's results are in. Per item: t_sub / t_done (steady-clock seconds at submission and
 * after its wait returned) and status (the wait's result, -1 if it was never submitted). Flushes
 * after the last submission. Returns 0, or -1 if a submission was refused (the rest are skipped). */
int srsgpu_rxq_drive(srsgpu_rxq_t *q, srsgpu_rxq_item_t *const *items, uint32_t n, uint32_t workers,
                     uint32_t reuse, double *t_sub, double *t_done, int32_t *status);
/* Paced load (srsUE's real-time arrival, one subframe per stream per TTI): `streams` radio streams
 * each hand one subframe to the queue every period_us (1000: the LTE TTI). Submission i = t * streams
 * + s (tick t, stream s) uses items[(t % depth) * streams + s] (depth HARQ slots per stream: its
 * softbuffer / outputs) and is submitted at t0 + t * period_us by one of `workers` native producer
 * threads (stream s belongs to producer s mod workers); a slot is reused only once its previous
 * submission is collected. latency_ms[i] = results written - tick time (collected in submission
 * order, so an early finisher counts when every earlier one is in: an upper bound); status[i] as
 * srsgpu_rxq_wait (-1: not submitted). *acked: collected submissions whose TB 0 acked; *late_ms: the
 * furthest a submission went out behind its tick. Returns 0, or -1 if a submission was refused. */
int srsgpu_rxq_drive_paced(srsgpu_rxq_t *q, srsgpu_rxq_item_t *const *items, uint32_t streams, uint32_t depth,
                           uint32_t ticks, uint32_t period_us, uint32_t workers, float *latency_ms, int32_t *status,
                           uint32_t *acked, double *late_ms);
/* srsgpu_rxq_drive_paced with thread placement and a second latency: cpus[0..ncpus) (NULL / 0:
 * unpinned) take the collector (cpus[0]) and producer w (cpus[(1 + w) % ncpus]);
 * submit_latency_ms[i] (optional) = results written - the moment submission i actually went out,
 * i.e. the queue's own latency without the producer's lateness behind its tick (-1: not submitted). */
int srsgpu_rxq_drive_paced_ex(srsgpu_rxq_t *q, srsgpu_rxq_item_t *const *items, uint32_t streams, uint32_t depth,
                              uint32_t ticks, uint32_t period_us, uint32_t workers, const int32_t *cpus,
                              uint32_t ncpus, float *latency_ms, float *submit_latency_ms, int32_t *status,
                              uint32_t *acked, double *late_ms);
/* Pin the queue's own threads (closer, dispatcher, completer) to cpus[0], cpus[1 % n], cpus[2 % n]
 * (e.g. cores apart from the PHY workers that submit). 0, or -1 if a pin failed. */
int srsgpu_rxq_set_affinity(srsgpu_rxq_t *q, const int32_t *cpus, uint32_t n);

#ifdef __cplusplus
}
#endif
#endif
