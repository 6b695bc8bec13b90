// Turbo encoder (TS 36.212 5.1.3.2): two 8-state RSC constituent encoders (g0 = 1+D^2+D^3,
// g1 = 1+D+D^3) around the QPP interleaver, trellis termination of each encoder in turn.
// Drop-in for srslte_tcod_encode (reference: lib/src/phy/fec/turbocoder.c:82-193), used to
// synthesise test and benchmark traffic on the host.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "srsgpu/qpp_table.h"
#include "srslte/phy/fec/turbocoder.h"

namespace {
struct Rsc {
  uint8_t s[3] = {0, 0, 0}; // shift register, s[0] newest
  // one step with input bit u; returns the parity bit (turbocoder.c:123-131)
  uint8_t step(uint8_t u) {
    uint8_t fb = u ^ s[2] ^ s[1];
    uint8_t par = s[2] ^ s[0] ^ fb;
    s[2] = s[1];
    s[1] = s[0];
    s[0] = fb;
    return par;
  }
  // termination input: the feedback value, which drives the register to zero (:160-177)
  uint8_t tail_bit() const { return s[2] ^ s[1]; }
};
} // namespace

extern "C" {

int srslte_tcod_init(srslte_tcod_t *h, uint32_t max_long_cb) {
  if (!h) return -1;
  h->max_long_cb = max_long_cb;
  h->temp = (uint8_t *)malloc(max_long_cb / 8 + 1);
  return h->temp ? 0 : -1;
}

void srslte_tcod_free(srslte_tcod_t *h) {
  if (!h) return;
  free(h->temp);
  h->temp = nullptr;
  h->max_long_cb = 0;
}

int srslte_tcod_encode(srslte_tcod_t *h, uint8_t *input, uint8_t *output, uint32_t long_cb) {
  if (!h || long_cb > h->max_long_cb) {
    fprintf(stderr, "Turbo coder initiated for max_long_cb=%d\n", h ? h->max_long_cb : 0);
    return -1;
  }
  int idx = -1;
  for (int i = 0; i < SRSGPU_NOF_CB_SIZES; i++)
    if (srsgpu_qpp_table[i][0] == long_cb) idx = i;
  if (idx < 0) {
    fprintf(stderr, "Invalid CB size %d\n", long_cb);
    return -1;
  }
  const uint64_t f1 = srsgpu_qpp_table[idx][1], f2 = srsgpu_qpp_table[idx][2];
  Rsc e1, e2;
  uint32_t k = 0;
  for (uint64_t i = 0; i < long_cb; i++) {
    const uint8_t in = input[i];
    const uint8_t u = in == SRSLTE_TX_NULL ? 0 : in;
    output[k++] = in;
    const uint8_t p1 = e1.step(u);
    output[k++] = in == SRSLTE_TX_NULL ? SRSLTE_TX_NULL : p1;
    const uint32_t pi = (uint32_t)((f1 * i + f2 * i * i) % long_cb);
    uint8_t u2 = input[pi];
    if (u2 == SRSLTE_TX_NULL) u2 = 0;
    output[k++] = e2.step(u2);
  }
  for (Rsc *e : {&e1, &e2}) {
    for (int j = 0; j < 3; j++) {
      uint8_t t = e->tail_bit();
      output[k++] = t;
      output[k++] = e->step(t);
    }
  }
  return 0;
}

} // extern "C"
