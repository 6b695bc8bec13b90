/* CPU ORACLE — TEST INFRASTRUCTURE ONLY (see dlsch_oracle.c). */
#ifndef SRSGPU_DLSCH_ORACLE_H
#define SRSGPU_DLSCH_ORACLE_H
#include <stdint.h>

#define ORC_CRC24A 0x1864CFB /* crc.h / sch.c:103 */
#define ORC_CRC24B 0x1800063
#define ORC_SOFTBUFFER_SIZE 18600 /* softbuffer.h */

typedef struct {
  uint32_t tbs, C, C1, K1, C2, K2, F;
} orc_cbsegm_t;

typedef struct {
  uint32_t max_cb;
  int16_t *buffer;  /* [max_cb][ORC_SOFTBUFFER_SIZE] soft bits (buffer_f) */
  uint8_t *data;    /* [max_cb][768] decoded bytes kept for retransmissions */
  uint8_t *cb_crc;  /* [max_cb] */
  uint8_t tb_crc;
} orc_softbuffer_t;

int orc_segm(uint32_t tbs, orc_cbsegm_t *s);
int orc_rm_turbo_rx_table(uint32_t K, uint32_t rv, uint32_t nsb, uint16_t *table);
int orc_rm_turbo_rx(const int16_t *in, int16_t *out, uint32_t in_len, uint32_t K, uint32_t rv,
                    uint32_t nsb);
int orc_rm_turbo_tx(const uint8_t *coded, uint32_t K, uint32_t rv, uint8_t *e, uint32_t E);
int orc_dlsch_encode(uint32_t tbs, uint32_t rv, uint32_t Qm, uint32_t nof_e_bits,
                     const uint8_t *data, uint8_t *e_bits);
int orc_softbuffer_init(orc_softbuffer_t *q, uint32_t max_cb);
void orc_softbuffer_reset(orc_softbuffer_t *q);
void orc_softbuffer_free(orc_softbuffer_t *q);
int orc_rm_turbo_rx_8bit(const int8_t *in, int8_t *out, uint32_t in_len, uint32_t K, uint32_t rv);
int orc_dlsch_decode8(orc_softbuffer_t *q, uint32_t tbs, uint32_t rv, uint32_t Qm,
                      uint32_t nof_e_bits, const int8_t *e_bits, uint8_t *data,
                      uint32_t max_halfits, uint32_t *nof_iterations);
int orc_dlsch_decode(orc_softbuffer_t *q, uint32_t tbs, uint32_t rv, uint32_t Qm,
                     uint32_t nof_e_bits, const int16_t *e_bits, uint8_t *data,
                     uint32_t max_halfits, uint32_t *nof_iterations);
/* UL-SCH (§8(f) rank 3): ulsch_deinterleave without RI bits (sch.c:550-568,860-881) and
 * srslte_ulsch_decode (sch.c:883-889 -> :944-985 with no UCI) */
int orc_ulsch_deinterleave(const int16_t *q_bits, uint32_t Qm, uint32_t nof_bits, uint32_t nof_symb,
                           int16_t *g_bits);
int orc_ulsch_decode(orc_softbuffer_t *q, uint32_t tbs, uint32_t rv, uint32_t Qm, uint32_t nof_bits,
                     uint32_t nof_symb, const int16_t *q_bits, uint8_t *data, uint32_t max_halfits,
                     uint32_t *nof_iterations);
#endif
