/*
 * srsgpu batched DL-SCH transport-block decoder — C ABI of the MI355X (gfx950) path from
 * descrambled int16 LLRs to transport blocks.
 *
 * One call decodes many transport blocks. That covers a subframe's TBs, or the TBs of many
 * subframes and cells. Each TB goes through the reference's receive chain
 * (reference: lib/src/phy/phch/sch.c:307-517, decode_tb / decode_tb_cb):
 *   - code block segmentation (cbsegm.c:58-140);
 *   - per code block, de-rate-matching with HARQ soft combining into the TB's softbuffer
 *     (srslte_rm_turbo_rx_lut, rm_turbo.c:378-430; sub-block layout for the windowed decoders);
 *   - turbo decoding with CRC early stop per half-iteration (CRC24B over K when C > 1, CRC24A over
 *     TBS+24 when C == 1) up to max_halfits half-iterations; blocks that passed in an earlier
 *     transmission are not decoded again but copied from the softbuffer;
 *   - TB assembly and the TB CRC24A check.
 * The results match srslte_dlsch_decode2 bit for bit: return code, data bytes, nof_iterations
 * and the softbuffer's cb_crc state.
 *
 * Softbuffers live in device memory, indexed 0 .. nof_softbuffers-1. Each holds max_cb rows of
 * SRSGPU_SOFTBUFFER_SIZE int16 (softbuffer.h SOFTBUFFER_SIZE), cb_crc flags and saved bytes. As in
 * the reference, the caller resets a softbuffer before a new transport block
 * (srslte_softbuffer_rx_reset).
 */
#ifndef SRSGPU_DLSCH_BATCH_H
#define SRSGPU_DLSCH_BATCH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SRSGPU_SOFTBUFFER_SIZE 18600

typedef struct srsgpu_dlsch srsgpu_dlsch_t;

typedef struct {
  uint32_t tbs;         /* transport block size in bits (cb_segm.tbs) */
  uint32_t rv;          /* redundancy version 0..3 */
  uint32_t Qm;          /* modulation order x layers factor, as srslte_dlsch_decode2 passes it */
  uint32_t nof_e_bits;  /* received coded bits of this TB */
  uint32_t softbuffer;  /* softbuffer index */
  uint64_t e_offset;    /* first LLR of this TB in the e-bits buffer (int16 elements) */
  uint64_t data_offset; /* first output byte of this TB in the data buffer */
} srsgpu_dlsch_tb_t;

/* Output bytes one TB needs: (tbs+24)/8 plus the last code block's 3 CRC bytes (C > 1). */
#define SRSGPU_DLSCH_DATA_LEN(tbs) ((tbs) / 8 + 6)

int srsgpu_dlsch_create(srsgpu_dlsch_t **q, uint32_t nof_softbuffers, uint32_t max_cb,
                        uint32_t max_cbs_per_call);
void srsgpu_dlsch_destroy(srsgpu_dlsch_t *q);
void srsgpu_dlsch_set_stream(srsgpu_dlsch_t *q, void *hip_stream);

/* srslte_softbuffer_rx_reset (softbuffer.c:125-150): zero the soft bits and the cb_crc flags. */
int srsgpu_dlsch_softbuffer_reset(srsgpu_dlsch_t *q, uint32_t softbuffer);
/* Reset softbuffers first .. first+count-1 in one pass (a batch of new transport blocks). */
int srsgpu_dlsch_softbuffer_reset_range(srsgpu_dlsch_t *q, uint32_t first, uint32_t count);
/* srslte_softbuffer_rx_reset_tbs: only the first (tbs+24)/6120+1 code blocks. */
int srsgpu_dlsch_softbuffer_reset_tbs(srsgpu_dlsch_t *q, uint32_t softbuffer, uint32_t tbs);
/* Many softbuffers in one launch: softbuffer slots[i] as srsgpu_dlsch_softbuffer_reset_tbs with its
 * first ncb[i] code blocks (NULL ncb: all, srslte_softbuffer_rx_reset). -1 on a slot out of range
 * (nothing reset). */
int srsgpu_dlsch_softbuffer_reset_list(srsgpu_dlsch_t *q, const uint32_t *slots, const uint32_t *ncb, uint32_t n);

/* Device pointers, asynchronous on the handle's stream. d_ret[i]: 0 TB decoded and CRC OK,
 * -1 CRC error, -2 invalid inputs (filler bits, too many CBs) — sch.c's return values.
 * d_noi[i]: srslte_sch_last_noi after TB i. The host array tb[] may be reused on return. */
int srsgpu_dlsch_decode_dev(srsgpu_dlsch_t *q, const srsgpu_dlsch_tb_t *tb, uint32_t nof_tb,
                            const int16_t *d_e_bits, uint8_t *d_data, uint32_t max_halfits,
                            int32_t *d_ret, uint32_t *d_noi);

/* As srsgpu_dlsch_decode_dev with each TB's output bytes at d_out[i] (data_offset ignored): device
 * memory, or host memory the device can address (registered / mapped), which the decoder then writes
 * over PCIe with no copy. */
int srsgpu_dlsch_decode_out_dev(srsgpu_dlsch_t *q, const srsgpu_dlsch_tb_t *tb, uint32_t nof_tb,
                                const int16_t *d_e_bits, uint8_t *const *d_out, uint32_t max_halfits,
                                int32_t *d_ret, uint32_t *d_noi);

/* Host pointers: e_bits[i] / data[i] per TB (offsets in tb[] ignored); synchronises. */
int srsgpu_dlsch_decode(srsgpu_dlsch_t *q, const srsgpu_dlsch_tb_t *tb, uint32_t nof_tb,
                        const int16_t *const *e_bits, uint8_t *const *data, uint32_t max_halfits,
                        int32_t *ret, uint32_t *noi);

/* Copy a softbuffer's state to the host (tests / debugging): rows [max_cb][SOFTBUFFER_SIZE]
 * int16 and cb_crc [max_cb]; either may be NULL. */
int srsgpu_dlsch_softbuffer_read(srsgpu_dlsch_t *q, uint32_t softbuffer, int16_t *rows,
                                 uint8_t *cb_crc);

/* Transmit side (srslte_dlsch_encode2, sch.c:540-; encode_tb_off :187-296), used to synthesise
 * traffic on the device: per TB, the TB CRC24A, code block segmentation with CRC24B, turbo
 * encoding (srslte_tcod_encode) and rate matching for tb[i].rv (as the reference produces it
 * after its rv 0 transmission filled the circular buffer). d_data + data_offset holds tbs/8 bytes;
 * the nof_e_bits coded bits are written unpacked (one 0/1 byte each) at d_e_bits + e_offset.
 * Returns -1 for TB sizes with filler bits (sch.c:203-206). */
int srsgpu_dlsch_encode_dev(srsgpu_dlsch_t *q, const srsgpu_dlsch_tb_t *tb, uint32_t nof_tb,
                            const uint8_t *d_data, uint8_t *d_e_bits);

/* De-rate-matching alone (srslte_rm_turbo_rx_lut_ semantics, rm_turbo.c:394-430) on device
 * buffers: d_out[t[i % (3K+12)]] += d_in[i] for i < in_len, with the sub-block table the AUTO
 * decoder expects when sb_layout != 0 (srslte_tdec_autoimp_get_subblocks(K) > 0). */
int srsgpu_rm_turbo_rx_dev(srsgpu_dlsch_t *q, const int16_t *d_in, int16_t *d_out, uint32_t in_len,
                           uint32_t K, uint32_t rv, int sb_layout);

/* 8-bit LLR chain (srslte_sch_t.llr_is_8bit; sch.c:344-364). Enabled, srsgpu_dlsch_decode(_dev)
 * takes int8 LLRs held in the int16 e-bits elements (values in [-128, 127]), de-rate-matches them
 * as srslte_rm_turbo_rx_lut_8bit (int8 sums wrapping at 8 bits, held sign-extended in the int16
 * softbuffer rows, the 8-bit decoder's sub-block table) and decodes with
 * srslte_tdec_iteration_8bit's decoders (SRSGPU_TDEC_AUTO_8BIT). A TB with a code block of
 * 400 < K <= 800 returns -2: the reference's 8-bit AUTO choice has no defined result there
 * (turbodecoder.c:439-459). Softbuffers must not change mode between transmissions of a TB. */
void srsgpu_dlsch_set_llr_8bit(srsgpu_dlsch_t *q, int enable);
/* CRC early stop between half-iterations (default on: sch.c:361-391, srsUE's decoder). Off is a
 * measurement mode with no reference counterpart: every code block runs max_halfits
 * half-iterations and its CRC is checked once after the last (the fixed-iteration processing rate
 * on real codewords; nof_iterations then reports max_halfits). */
void srsgpu_dlsch_set_early_stop(srsgpu_dlsch_t *q, int enable);
/* Tail stream (no reference counterpart; NULL = off, the default): under early stop, each decode
 * call's work after the first half-iteration and its CRC check (the few code blocks still running,
 * their bytes, the TB CRC and the epilogue of sch.c:393-491) goes to `hip_stream`, and the call's
 * results (TB bytes, d_ret, d_noi, softbuffers) are final when that stream reaches them. The engine's
 * own stream is free for the caller's next work meanwhile (e.g. the next batch's front end into
 * another engine); the next call into this engine makes its stream wait for the tail first.
 * The tail also READS the call's inputs: the e-bits LLRs (the rows of failed TBs are written from
 * them after the decode) stay unchanged until the tail stream has reached the end of the call. A
 * caller that rewrites its LLR buffer on the engine's stream before calling the engine again joins
 * the tail first (srsgpu_dlsch_join_tail). srsgpu_pdsch_* do so at every entry point that enqueues
 * work, so an engine taken from srsgpu_pdsch_get_dlsch() is safe with the PDSCH's own LLR buffer. */
int srsgpu_dlsch_set_tail_stream(srsgpu_dlsch_t *q, void *hip_stream);
/* Make the engine's stream wait for a pending tail (a no-op without one). 0, or -1 on a HIP error. */
int srsgpu_dlsch_join_tail(srsgpu_dlsch_t *q);
/* Half-iterations each code block of the last decode call ran (sch.c:361-391's cb_noi; every block
 * when early stop is off: max_halfits), in the decoder's block order: waits for the call, copies
 * min(n, blocks) values and returns the call's block count, or -1. A measurement aid (bench.py's
 * decoder work per batch). */
int srsgpu_dlsch_cb_halfits(srsgpu_dlsch_t *q, uint32_t *out, uint32_t n);
/* Direct de-rate-matching (default on). Code blocks of the window decoders (K > 400 under AUTO)
 * are de-rate-matched and HARQ-combined straight into the decoder's inputs, and their softbuffer
 * rows are written after the decode only when their TB failed (every block not decoded before
 * the call, exactly as srslte_rm_turbo_rx_lut leaves them). Decoded bytes, return codes,
 * nof_iterations and cb_crc are identical either way. The rows of an acked TB are left as they
 * were: the reference never reads them again (sch.c:323 skips blocks whose CRC passed, and the
 * next TB resets the softbuffer), so only srsgpu_dlsch_softbuffer_read can tell. Off: every row is
 * written before the decode (the reference's order). */
void srsgpu_dlsch_set_direct_derm(srsgpu_dlsch_t *q, int enable);
/* srslte_rm_turbo_rx_lut_8bit (rm_turbo.c:432-469) on device buffers, int8 values held in int16
 * elements: d_out[t[i % (3K+12)]] += d_in[i], wrapping at 8 bits, 8-bit decoder sub-block table. */
int srsgpu_rm_turbo_rx_8bit_dev(srsgpu_dlsch_t *q, const int16_t *d_in, int16_t *d_out,
                                uint32_t in_len, uint32_t K, uint32_t rv);

#ifdef __cplusplus
}
#endif
#endif
