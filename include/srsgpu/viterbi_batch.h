/*
 * srsgpu batched Viterbi decoder — the convolutional decoder of the PDCCH blind search
 * (srslte_pdcch_decode_msg, lib/src/phy/phch/pdcch.c:330-345, decodes
 * every DCI candidate with srslte_viterbi_decode_f on a tail-biting K=7 r=1/3 decoder, pdcch.c:79).
 *
 * Many frames per launch, one wavefront per frame (its 64 lanes = the 64 trellis states). Same
 * result as the reference's srslte_viterbi_decode_f on an AVX2 build (lib/src/phy/fec/viterbi.c
 * with VITERBI_16: uint16 quantisation with gain 1000 / max|x|, decode37_avx2_16bit over three
 * copies of the frame, the middle third out; viterbi37_avx2_16bit.c arithmetic), bit for bit.
 */
#ifndef SRSGPU_VITERBI_BATCH_H
#define SRSGPU_VITERBI_BATCH_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SRSGPU_VITERBI_MAX_FRAME 192 /* bits per frame (DCI + 16 CRC bits are at most 73) */

typedef struct {
  uint64_t sym_offset;   /* first of the frame's 3 * frame_length float symbols in d_sym */
  uint64_t out_offset;   /* first of its frame_length output bytes (one bit per byte) in d_out */
  uint32_t frame_length; /* bits, 1 .. SRSGPU_VITERBI_MAX_FRAME */
  uint32_t pad;
} srsgpu_viterbi_frame_t;

/* srslte_viterbi_decode_f, tail-biting, polynomials {0x6D, 0x4F, 0x57} (srsLTE's PDCCH decoder),
 * for nof_frames frames described by the DEVICE array d_frames. Asynchronous on hip_stream (NULL:
 * the null stream). Returns -1 on invalid arguments. */
int srsgpu_viterbi37_tb_decode_f_dev(const srsgpu_viterbi_frame_t *d_frames, uint32_t nof_frames,
                                     const float *d_sym, uint8_t *d_out, void *hip_stream);

/* DCI candidates of the PDCCH blind search, decoded as srslte_pdcch_decode_msg does
 * (lib/src/phy/phch/pdcch.c:380-396, srslte_pdcch_dci_decode :322-360): skipped unless the mean
 * |llr| over the candidate's E bits exceeds 0.5; srslte_rm_conv_rx to 3 (nof_bits + 16) soft
 * bits; the Viterbi decoder above; the 16-bit CRC remainder (CRC16 0x11021 of the nof_bits
 * payload bits XOR the 16 received parity bits), which the caller compares with its RNTI. */
#define SRSGPU_DCI_MAX_BITS 128 /* SRSLTE_DCI_MAX_BITS */
#define SRSGPU_DCI_MAX_E 576    /* PDCCH_FORMAT_NOF_BITS(3): 8 CCEs x 72 bits */
typedef struct {
  uint64_t llr_offset; /* first of the candidate's E float LLRs (q->llr[ncce * 72 ..]) in d_llr */
  uint64_t out_offset; /* first of its nof_bits + 16 decoded bits (one per byte) in d_data */
  uint32_t E;          /* PDCCH_FORMAT_NOF_BITS(L) */
  uint32_t nof_bits;   /* srslte_dci_format_sizeof */
} srsgpu_dci_cand_t;
/* d_decoded[i] = 1 decoded (d_crc_rem[i] valid), 0 skipped by the mean check. Device arrays;
 * asynchronous on hip_stream. */
int srsgpu_dci_decode_dev(const srsgpu_dci_cand_t *d_cands, uint32_t nof_cands, const float *d_llr,
                          uint8_t *d_data, uint16_t *d_crc_rem, uint8_t *d_decoded, void *hip_stream);

#ifdef __cplusplus
}
#endif
#endif
