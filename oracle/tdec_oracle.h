/* CPU ORACLE — TEST INFRASTRUCTURE ONLY (see tdec_oracle.c). */
#ifndef SRSGPU_TDEC_ORACLE_H
#define SRSGPU_TDEC_ORACLE_H
#include <stdint.h>

/* values of srslte_tdec_impl_type_t (turbodecoder_impl.h:33-42) */
enum {
  ORC_TDEC_AUTO = 0,
  ORC_TDEC_GENERIC,
  ORC_TDEC_SSE,
  ORC_TDEC_SSE_WINDOW,
  ORC_TDEC_AVX_WINDOW,
  ORC_TDEC_SSE8_WINDOW,
  ORC_TDEC_AVX8_WINDOW
};

int orc_cbindex(uint32_t long_cb);
int orc_cbsize(uint32_t idx);
int orc_cbsegm(uint32_t tbs, uint32_t *C, uint32_t *C1, uint32_t *K1, uint32_t *C2, uint32_t *K2,
               uint32_t *F);
int orc_interl(uint32_t K, uint32_t nsb, uint16_t *fwd, uint16_t *rev);
uint32_t orc_autoimp_subblocks(uint32_t K);
int orc_tdec_input_len(int impl, int sb_layout, uint32_t K);
int orc_tdec_run(int impl, int sb_layout, const int16_t *input, uint32_t K, uint32_t nof_halfits,
                 uint8_t *decisions, int16_t *final_app1, int16_t *final_ext1);
int orc_tdec_decode_cb(int impl, int sb_layout, const int16_t *input, uint32_t K,
                       uint32_t max_halfits, uint32_t crc_poly, uint32_t crc_len_bits,
                       uint8_t *out_bytes, uint32_t *noi);
uint32_t orc_crc_checksum_byte(uint32_t poly, int order, const uint8_t *data, uint32_t len_bits);
/* 8-bit path (tdec8_oracle.c) */
uint32_t orc_autoimp_subblocks_8bit(uint32_t K);
int orc_tdec8_run(int impl, int sb_layout, const int8_t *input, uint32_t K, uint32_t nof_halfits,
                  uint8_t *decisions);
int orc_tdec8_run16(int impl, const int16_t *input, uint32_t K, uint32_t nof_halfits,
                    uint8_t *decisions);
int orc_tcod_encode(const uint8_t *in_bits, uint8_t *out_bits, uint32_t K);
#endif
