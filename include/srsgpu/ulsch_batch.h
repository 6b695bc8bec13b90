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
 * srsgpu_ulsch_decode_dev is the uci_data = {0} case that srslte_ulsch_decode runs;
 * srsgpu_ulsch_uci_decode_dev below adds the UCI multiplexed on the PUSCH (HARQ-ACK, RI, CQI).
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

/* UCI multiplexed on the PUSCH (srslte_pusch_decode, lib/src/phy/phch/pusch.c:626-657, with
 * srslte_ulsch_uci_decode_ri_ack / srslte_ulsch_uci_decode, sch.c:892-985, and uci.c): per TB
 *   - HARQ-ACK (1-2 bits) and RI from the STILL SCRAMBLED q bits and the PUSCH sequence c, with the
 *     reference's decoders (uci.c:746-790: Q' from the beta offsets, the bit positions of
 *     uci_ulsch_interleave_ack_gen / _ri_gen, decode_ri_ack_1bit / _2bits as they are); the ACK
 *     positions then count as zero;
 *   - descrambling, then the channel deinterleaver with the RI positions taken out (sch.c:550-568,
 *     860-881, the lut's write order included);
 *   - CQI (srslte_uci_decode_cqi_pusch, uci.c:428-464): the (32, O) block code by ML up to 11 bits,
 *     above that rate dematching, srslte_viterbi_decode_s and CRC8 (cqi_ack);
 *   - the data (decode_tb on the G = H' - Q'_ri - Q'_cqi symbols after the CQI) when tbs > 0.
 * q_bits are the scrambled soft bits (nof_bits per TB at q_offset, as srslte_pusch_decode holds them
 * before srslte_scrambling_s_offset); d_c holds each TB's scrambling sequence, one byte per bit
 * (srslte_sequence_t.c) at c_offset; d_g_bits receives the deinterleaved bits (CQI bits summed in
 * place as the reference's short-CQI decoder leaves them). d_uci[i] receives TB i's UCI. Returns -1
 * without launching anything on a reserved beta offset, an unsupported length, a matrix mismatch, or
 * HARQ-ACK / RI positions beyond the reference's array (Q' Qm > 3456, srslte_sch_t.ack_ri_bits, sch.h:70:
 * the reference writes past it). */
#define SRSGPU_UCI_MAX_CQI_BITS 183 /* O_cqi + 8 within the 191-bit Viterbi frame */
typedef struct {
  uint32_t O_ack, O_ri, O_cqi;                    /* uci_ack_len (0-2), uci_ri_len (0-2), uci_cqi_len */
  uint32_t I_offset_ack, I_offset_ri, I_offset_cqi; /* cfg->uci_cfg */
  uint32_t M_sc, M_sc_init;                       /* cfg->grant */
  uint64_t c_offset;                              /* the TB's scrambling sequence in d_c */
} srsgpu_uci_cfg_t;
typedef struct {
  uint8_t ack[2];  /* uci_ack, uci_ack_2 */
  uint8_t ri;      /* uci_ri */
  uint8_t cqi_ack; /* CRC8 of a CQI above 11 bits checked */
  uint8_t cqi[SRSGPU_UCI_MAX_CQI_BITS + 1]; /* uci_cqi, one bit per byte */
  uint32_t Q_ack, Q_ri, Q_cqi; /* Q' of each (the data starts at Q_cqi Qm in g) */
} srsgpu_uci_result_t;
int srsgpu_ulsch_uci_decode_dev(srsgpu_dlsch_t *q, const srsgpu_ulsch_tb_t *tb, const srsgpu_uci_cfg_t *uci,
                                uint32_t nof_tb, const int16_t *d_q_bits, const uint8_t *d_c, int16_t *d_g_bits,
                                uint8_t *d_data, uint32_t max_halfits, int32_t *d_ret, uint32_t *d_noi,
                                srsgpu_uci_result_t *d_uci);

#ifdef __cplusplus
}
#endif
#endif
