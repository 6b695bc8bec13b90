/*
 * srsgpu batched UL-SCH transport-block decoder — C ABI of the MI355X (gfx950) path for the eNodeB's
 * PUSCH data.
 *
 * Replaces srslte_ulsch_decode (reference: lib/src/phy/phch/sch.c:883-889 -> srslte_ulsch_uci_decode
 * :944-985 with no UCI): per transport block, the UL-SCH channel deinterleaver of 36.212 5.2.2.8
 * (ulsch_deinterleave / ulsch_interleave_gen, sch.c:550-568,860-881: q bits read column by column
 * out of a rows x N_symb^PUSCH matrix of Qm-bit entries) into g bits, then the same decode_tb as the
 * DL-SCH (sch.c:437-498: segmentation, de-rate-matching with HARQ combining, turbo decoding with CRC
 * early stop, TB CRC). The decode runs on the DL-SCH object's softbuffers and decoder
 * (include/srsgpu/dlsch_batch.h), as the reference shares one srslte_sch_t.
 *
 * Not covered: UCI multiplexed on the PUSCH (ACK / RI / CQI, srslte_ulsch_uci_decode_ri_ack and
 * srslte_uci_decode_cqi_pusch); the data decode here is the uci_data = {0} case that
 * srslte_ulsch_decode runs.
 */
#ifndef SRSGPU_ULSCH_BATCH_H
#define SRSGPU_ULSCH_BATCH_H

#include <stdint.h>

#include "srsgpu/dlsch_batch.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  uint32_t tbs;         /* cfg->cb_segm.tbs */
  uint32_t rv;          /* cfg->rv */
  uint32_t Qm;          /* cfg->grant.Qm: 2, 4 or 6 */
  uint32_t nof_bits;    /* cfg->nbits.nof_bits = H'_total x Qm, the PUSCH's coded bits */
  uint32_t nof_symb;    /* cfg->nbits.nof_symb = N_symb^PUSCH, the interleaver's columns */
  uint32_t softbuffer;  /* softbuffer index of the DL-SCH object */
  uint64_t q_offset;    /* first int16 of this TB's q bits in d_q_bits, and of its g bits in d_g_bits */
  uint64_t data_offset; /* first output byte of this TB in d_data (SRSGPU_DLSCH_DATA_LEN(tbs) bytes) */
} srsgpu_ulsch_tb_t;

/* Device pointers, asynchronous on the DL-SCH handle's stream. d_g_bits is the caller's
 * deinterleaved-bits buffer (srslte_ulsch_decode's g_bits), same offsets as d_q_bits.
 * d_ret[i] / d_noi[i] as srsgpu_dlsch_decode_dev (sch.c's return values: 0 OK, -1 CRC error,
 * -2 invalid inputs). Returns -1 without launching anything if a TB's nof_bits is not a multiple
 * of Qm x nof_symb (the reference's deinterleaver table would then be partly unset). */
int srsgpu_ulsch_decode_dev(srsgpu_dlsch_t *q, const srsgpu_ulsch_tb_t *tb, uint32_t nof_tb,
                            const int16_t *d_q_bits, int16_t *d_g_bits, uint8_t *d_data,
                            uint32_t max_halfits, int32_t *d_ret, uint32_t *d_noi);
/* The channel deinterleaver alone (d_q -> d_g, same TB descriptors; tbs, rv, softbuffer and data_offset
 * unused): srslte_ulsch_decode of a PUSCH without data (tbs 0, sch.c:957-975) still writes g_bits. */
int srsgpu_ulsch_deinterleave_dev(srsgpu_dlsch_t *q, const srsgpu_ulsch_tb_t *tb, uint32_t nof_tb,
                                  const int16_t *d_q_bits, int16_t *d_g_bits);

#ifdef __cplusplus
}
#endif
#endif
