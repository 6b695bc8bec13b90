/*
 * Drop-in turbo-decoder API served by the MI355X engine (libsrsgpu_phy.so).
 *
 * Replaces the reference header lib/include/srslte/phy/fec/turbodecoder.h (srsLTE 18.09):
 * same function names, argument meaning, return codes and call protocol
 * (init -> new_cb -> iteration... | run_all -> free), so callers such as
 * lib/src/phy/phch/sch.c:115,356-366 recompile unchanged against this include directory.
 * The struct keeps the reference's public bookkeeping fields (max_long_cb, dec_type,
 * force_not_sb, current_long_cb, current_cbidx, n_iter); the decoder state itself lives in
 * GPU memory behind `gpu`.
 *
 * The *_8bit entry points and the int8 SSE8 / AVX8 window decoders follow turbodecoder.c:392-563
 * bit-exactly. Differences, all documented in DESIGN.md: the input buffer is read once per code
 * block (at the first half-iteration) and never written (the reference copies tail values into
 * the caller's padding); where the reference's result is undefined (8-bit sub-block input at
 * 400 < K <= 800, 16-bit sub-block input to a manual int8 type) the call fails with a message;
 * the manual window types through the *_8bit entry points, which fault in the reference (no
 * interleaver selected, turbodecoder.c:451-453), decode with the type's own interleaver.
 */
#ifndef SRSLTE_TURBODECODER_H
#define SRSLTE_TURBODECODER_H

#include <stdbool.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SRSLTE_TCOD_RATE 3
#define SRSLTE_TCOD_TOTALTAIL 12
#define SRSLTE_TCOD_MAX_LEN_CB 6144
#define SRSLTE_TDEC_EXPECT_INPUT_SB 1

#ifndef SRSLTE_TURBODECODER_IMPL_H
#define SRSLTE_TURBODECODER_IMPL_H
/* reference: lib/include/srslte/phy/fec/turbodecoder_impl.h:33-42 */
typedef enum {
  SRSLTE_TDEC_AUTO = 0,
  SRSLTE_TDEC_GENERIC,
  SRSLTE_TDEC_SSE,
  SRSLTE_TDEC_SSE_WINDOW,
  SRSLTE_TDEC_AVX_WINDOW,
  SRSLTE_TDEC_SSE8_WINDOW,
  SRSLTE_TDEC_AVX8_WINDOW,
  SRSLTE_TDEC_NOF_IMP
} srslte_tdec_impl_type_t;
#endif

/* sizeof(srslte_tdec_t) in the reference (turbodecoder.h:68-100, LP64: 4 x 188 interleaver
 * structs plus pointers). srslte_sch_t embeds the decoder by value (sch.h:74), so objects built
 * against the reference's sch.h stay layout-compatible only if this struct has the same size and
 * alignment: the bookkeeping fields and the engine handle come first, the rest is padding.
 * tests/test_capi.py compares both sizes with the reference header. */
#define SRSLTE_TDEC_REF_SIZEOF 18264

typedef struct {
  uint32_t max_long_cb;
  srslte_tdec_impl_type_t dec_type;
  bool force_not_sb;
  uint32_t current_long_cb;
  int current_cbidx;
  int n_iter;
  void *gpu; /* engine state (device buffers, stream), owned by the library */
  uint8_t reserved[SRSLTE_TDEC_REF_SIZEOF - 4 * sizeof(uint32_t) - 2 * sizeof(int) - sizeof(void *)];
} srslte_tdec_t;

/* compile-time size check (C99 and C++): a negative array size if the layout drifts */
typedef char srslte_tdec_size_check_t[(sizeof(void *) != 8 || sizeof(srslte_tdec_t) == SRSLTE_TDEC_REF_SIZEOF) ? 1 : -1];

/* turbodecoder.h:102-107 */
int srslte_tdec_init(srslte_tdec_t *h, uint32_t max_long_cb);
int srslte_tdec_init_manual(srslte_tdec_t *h, uint32_t max_long_cb,
                            srslte_tdec_impl_type_t dec_type);
/* turbodecoder.h:109-116 */
void srslte_tdec_free(srslte_tdec_t *h);
void srslte_tdec_force_not_sb(srslte_tdec_t *h);
int srslte_tdec_new_cb(srslte_tdec_t *h, uint32_t long_cb);
int srslte_tdec_get_nof_iterations(srslte_tdec_t *h);
/* turbodecoder.h:118-120 */
uint32_t srslte_tdec_autoimp_get_subblocks(uint32_t long_cb);
uint32_t srslte_tdec_autoimp_get_subblocks_8bit(uint32_t long_cb);
/* turbodecoder.h:122-130: one half-iteration + hard decision / nof_iterations half-iterations */
void srslte_tdec_iteration(srslte_tdec_t *h, int16_t *input, uint8_t *output);
int srslte_tdec_run_all(srslte_tdec_t *h, int16_t *input, uint8_t *output,
                        uint32_t nof_iterations, uint32_t long_cb);
/* turbodecoder.h:132-140: the int8 decoders (turbodecoder.c:536-559), AUTO resolving to the
   8-bit AUTO choice (SSE8 / AVX8 windows, 16-bit fallbacks, turbodecoder.c:392-464) */
void srslte_tdec_iteration_8bit(srslte_tdec_t *h, int8_t *input, uint8_t *output);
int srslte_tdec_run_all_8bit(srslte_tdec_t *h, int8_t *input, uint8_t *output,
                             uint32_t nof_iterations, uint32_t long_cb);

#ifdef __cplusplus
}
#endif
#endif
