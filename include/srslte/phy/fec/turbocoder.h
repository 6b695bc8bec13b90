/*
 * Drop-in turbo encoder API (TX side, used for synthetic load generation).
 * Replaces the bit encoder of the reference header lib/include/srslte/phy/fec/turbocoder.h
 * (srsLTE 18.09): srslte_tcod_init / srslte_tcod_encode / srslte_tcod_free with the same
 * argument meaning and return codes. The byte/LUT encoder (srslte_tcod_encode_lut) belongs to
 * the TX rate-matching path and is not part of this library yet.
 */
#ifndef SRSLTE_TURBOCODER_H
#define SRSLTE_TURBOCODER_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SRSLTE_TCOD_MAX_LEN_CB_BYTES (6144 / 8)
#ifndef SRSLTE_TX_NULL
#define SRSLTE_TX_NULL 100
#endif

typedef struct {
  uint32_t max_long_cb;
  uint8_t *temp;
} srslte_tcod_t;

/* turbocoder.h:56-66 */
int srslte_tcod_init(srslte_tcod_t *h, uint32_t max_long_cb);
void srslte_tcod_free(srslte_tcod_t *h);
/* bits in (one per byte, SRSLTE_TX_NULL = filler), [s,p0,p1]*K + 12 tail bits out */
int srslte_tcod_encode(srslte_tcod_t *h, uint8_t *input, uint8_t *output, uint32_t long_cb);

#ifdef __cplusplus
}
#endif
#endif
