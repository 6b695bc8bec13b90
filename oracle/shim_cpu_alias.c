/*
 * TEST INFRASTRUCTURE (never shipped): the *_cpu names integration/srslte_gpu_shim.c calls for the
 * reference's own softbuffer work. In srsLTE the maintainer compiles softbuffer.c with its rx
 * functions renamed *_cpu; the check programs link softbuffer.c unchanged next to
 * the renamed shim, so these forward to it.
 */
#include "srslte/phy/fec/softbuffer.h"

int srslte_softbuffer_rx_init_cpu(srslte_softbuffer_rx_t *q, uint32_t nof_prb) {
  return srslte_softbuffer_rx_init(q, nof_prb);
}
void srslte_softbuffer_rx_free_cpu(srslte_softbuffer_rx_t *q) { srslte_softbuffer_rx_free(q); }
void srslte_softbuffer_rx_reset_cpu(srslte_softbuffer_rx_t *q) { srslte_softbuffer_rx_reset(q); }
void srslte_softbuffer_rx_reset_tbs_cpu(srslte_softbuffer_rx_t *q, uint32_t tbs) {
  srslte_softbuffer_rx_reset_tbs(q, tbs);
}
void srslte_softbuffer_rx_reset_cb_cpu(srslte_softbuffer_rx_t *q, uint32_t nof_cb) {
  srslte_softbuffer_rx_reset_cb(q, nof_cb);
}
