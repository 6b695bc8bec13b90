/*
 * srsgpu batched turbo decoder — C ABI of the MI355X (gfx950) hot path.
 *
 * Additive batch extension of the srsLTE turbo-decoder API
 * (reference: lib/include/srslte/phy/fec/turbodecoder.h:102-140): one call decodes many code
 * blocks of the same size K on the GPU. The per-code-block srslte_tdec_* functions of
 * include/srslte/phy/fec/turbodecoder.h (this repo) forward to the same engine.
 *
 * Conventions (match the reference where it defines them):
 *   - impl: srslte_tdec_impl_type_t values; SRSLTE_TDEC_AUTO picks the decoder exactly like
 *     turbodecoder.c:364-390 (K<=400 SSE non-window, 400<K<=800 SSE16 window (8 sub-blocks),
 *     K>800 AVX16 window (16 sub-blocks)); GENERIC, SSE, SSE_WINDOW, AVX_WINDOW force one.
 *   - half-iterations: nof_halfits counts constituent-decoder runs, as srslte_tdec_run_all's
 *     nof_iterations does (turbodecoder.c:519-533).
 *   - input per CB: int16 LLRs, natural layout [s,p0,p1]*K + 12 tail values (3K+12), or, when
 *     sb_layout != 0 and the AUTO decoder is windowed, rm_turbo's sub-block layout
 *     (3*(K+32)+12; rm_turbo.c:239-264, turbodecoder_iter.h:301-308).
 *   - output per CB: K/8 bytes, MSB first (tdec_decision_byte).
 *   - return: 0 on success, -1 on error (message on stderr), like SRSLTE_SUCCESS/SRSLTE_ERROR.
 *   - *_dev entry points take device pointers (inputs resident in HBM) and are asynchronous on
 *     the batch's stream; the host-pointer entry points copy and synchronise.
 */
#ifndef SRSGPU_TDEC_BATCH_H
#define SRSGPU_TDEC_BATCH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct srsgpu_tdec_batch srsgpu_tdec_batch_t;

/* impl value for the reference's 8-bit path (srslte_tdec_iteration_8bit, turbodecoder.c:392-464):
 * int8 LLRs held in the int16 inputs (values in [-128, 127]); the SSE8 (16 sub-blocks) and AVX8
 * (32 sub-blocks) int8 window decoders where K allows them, otherwise the 16-bit AUTO decoder.
 * SRSLTE_TDEC_SSE8_WINDOW / _AVX8_WINDOW force one int8 decoder. Sub-block input layout
 * applies whenever an int8 decoder runs. */
#define SRSGPU_TDEC_AUTO_8BIT 16

/* Allocates device buffers for up to max_cbs code blocks of up to max_long_cb bits. */
int srsgpu_tdec_batch_create(srsgpu_tdec_batch_t **q, uint32_t max_cbs, uint32_t max_long_cb);
void srsgpu_tdec_batch_destroy(srsgpu_tdec_batch_t *q);
/* hip_stream: a hipStream_t (NULL = default stream). */
void srsgpu_tdec_batch_set_stream(srsgpu_tdec_batch_t *q, void *hip_stream);

/* Fixed number of half-iterations, no early stop (srslte_tdec_run_all semantics).
 * d_input: nof_cb rows of in_stride int16; d_output: nof_cb rows of out_stride bytes. */
int srsgpu_tdec_batch_run_dev(srsgpu_tdec_batch_t *q, int impl, int sb_layout,
                              const int16_t *d_input, size_t in_stride, uint32_t long_cb,
                              uint32_t nof_cb, uint32_t nof_halfits, uint8_t *d_output,
                              size_t out_stride);

/* CRC early stop per code block (sch.c:356-391 decode_tb_cb loop): after every half-iteration
 * the hard decision is CRC-checked over crc_len_bits bits with crc_poly (0x1800063 CRC24B for
 * C>1 with crc_len_bits = K, 0x1864CFB CRC24A for C==1 with TBS+24); a block stops when it
 * passes or after max_halfits. d_crc_ok[i] = 1 if passed; d_noi[i] = half-iterations run. */
int srsgpu_tdec_batch_decode_dev(srsgpu_tdec_batch_t *q, int impl, int sb_layout,
                                 const int16_t *d_input, size_t in_stride, uint32_t long_cb,
                                 uint32_t nof_cb, uint32_t max_halfits, uint32_t crc_poly,
                                 uint32_t crc_len_bits, uint8_t *d_output, size_t out_stride,
                                 uint8_t *d_crc_ok, uint32_t *d_noi);

/* Host-pointer versions (copy in, run, copy out, synchronise). input[i] / output[i] per CB. */
int srsgpu_tdec_batch_run(srsgpu_tdec_batch_t *q, int impl, int sb_layout,
                          const int16_t *const *input, uint32_t long_cb, uint32_t nof_cb,
                          uint32_t nof_halfits, uint8_t *const *output);
int srsgpu_tdec_batch_decode(srsgpu_tdec_batch_t *q, int impl, int sb_layout,
                             const int16_t *const *input, uint32_t long_cb, uint32_t nof_cb,
                             uint32_t max_halfits, uint32_t crc_poly, uint32_t crc_len_bits,
                             uint8_t *const *output, uint8_t *crc_ok, uint32_t *noi);

/* Decoder state of code block `cb` after the last half-iteration of the last job (run or
 * decode, the 16-bit decoders), as the reference holds it in srslte_tdec_t: app1 and ext1, K int16
 * each, in the decoder's own index space (sub-block order for the windowed decoders, natural for
 * SSE / generic), turbodecoder_iter.h:283-357. The device keeps A = app1 - ext1 and app2 =
 * interleave(ext1 ...); this reconstructs both arrays exactly (the subtractions wrap, so they
 * invert modulo 2^16). Synchronises the batch stream. Returns 0, or -1 if there is no such CB or
 * the last job ran an 8-bit decoder. */
int srsgpu_tdec_batch_read_state(srsgpu_tdec_batch_t *q, uint32_t cb, int16_t *app1, int16_t *ext1);

/* Input length (int16 elements) one CB needs for (impl, sb_layout, K). */
uint32_t srsgpu_tdec_input_len(int impl, int sb_layout, uint32_t long_cb);

/* Decoder launch schedule (process-wide; results are identical under every setting):
 *   fused      1: fixed-iteration jobs run all half-iterations in one launch per decoder kind;
 *              0: one launch per half-iteration (SRSGPU_TDEC_FUSED)
 *   es_fused   1: early-stop jobs check the CRC inside the decoder launches (k_win_bidir_es,
 *                 k_sse_es) and write the bytes in one k_es_bytes launch; 0: one decoder launch
 *                 and one k_decide launch per half-iteration; 2 (default): fused when every kind's
 *                 workgroups fit on the chip at once, the hybrid form when one does not (all kinds
 *                 fusable), else per decoder kind (SRSGPU_ES_FUSED); 3 (hybrid): the
 *                 first half-iteration per launch with k_decide, then the blocks still running
 *                 through the rest in one fused early-stop launch per kind
 *   es_chunk   half-iterations per fused early-stop launch, >= 1, default 8 (SRSGPU_ES_CHUNK)
 *   sse_bidir  1: the two-wave SSE decoder, 0: the one-wave one (SRSGPU_SSE_BIDIR; the fused early
 *                 stop of the SSE kind needs the two-wave one)
 * A negative argument keeps the current value; the defaults come from those environment variables.
 * Change it only while no decode is being issued. Returns 0, or -1 for es_chunk == 0 or es_fused > 3. */
int srsgpu_tdec_set_schedule(int fused, int es_fused, int es_chunk, int sse_bidir);
void srsgpu_tdec_get_schedule(int *fused, int *es_fused, int *es_chunk, int *sse_bidir);
/* Re-read the launch tuning knobs from the environment (SRSGPU_ES_PRIO, SRSGPU_TAIL_PRIO,
 * SRSGPU_DECIDE_PRIO, SRSGPU_H0_PRIO, SRSGPU_LLR_GENERIC, SRSGPU_LLR_NOXCD). They are read once, at
 * the first launch that needs them, and kept; a process that changes one of them afterwards calls
 * this (no launch reads the environment itself). */
void srsgpu_knobs_reload(void);

/* Live kernel timing with HIP events on the batch stream (for bench.py's roofline). */
void srsgpu_prof_enable(int on);
void srsgpu_prof_reset(void);
/* Sum of event-timed durations and launch count for kernels whose name contains `name`. */
int srsgpu_prof_get(const char *name, double *total_ms, uint64_t *count);

#ifdef __cplusplus
}
#endif
#endif
