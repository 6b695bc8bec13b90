/* CPU ORACLE — TEST INFRASTRUCTURE ONLY (see pdsch_oracle.c). */
#ifndef SRSGPU_PDSCH_ORACLE_H
#define SRSGPU_PDSCH_ORACLE_H
#include <stdint.h>

int orc_pdsch_re_map(uint32_t nof_prb, uint32_t cell_id, uint32_t nof_ports, uint32_t lstart,
                     uint32_t sf_idx, const uint8_t *prb_mask, uint32_t *idx);
void orc_predecode_single(const float *y, const float *h, float *x, float *csi, int n,
                          float scaling, float noise);
int orc_predecode_multiplex(const float *y0, const float *y1, const float *h00, const float *h01,
                            const float *h10, const float *h11, float *x0, float *x1, float *csi0,
                            float *csi1, int n, float scaling, float noise, int codebook_idx,
                            int nof_layers);
void orc_predecode_ccd_2x2(const float *y0, const float *y1, const float *h00, const float *h01,
                           const float *h10, const float *h11, float *x0, float *x1, float *csi0,
                           float *csi1, int n, float scaling, float noise);
int orc_demod_s(int mod, const float *sym, int nsym, int16_t *llr);
int orc_sequence(uint32_t seed, uint32_t len, uint8_t *c);
uint32_t orc_pdsch_seed(uint16_t rnti, int q, uint32_t nslot, uint32_t cell_id);
int orc_scramble_s(uint32_t seed, int16_t *llr, uint32_t len);
int orc_csi_correction(int mod, const float *csi, int nsym, int16_t *e);
/* TM2 transmit diversity, 2 ports: predecoding + layer demapping -> d (interleaved complex) */
int orc_predecode_txdiv(const float *y0, const float *y1, const float *h00, const float *h01,
                        const float *h10, const float *h11, int nrx, int n, float scaling, float *d,
                        float *csi);
/* TM2 transmit diversity, 4 ports (n % 4 == 0): y [rx], h [port * 2 + rx] */
int orc_predecode_txdiv4(const float *const *y, const float *const *h, int nrx, int n, float scaling, float *d,
                         float *csi);
/* PDCCH Viterbi: srslte_viterbi_decode_f, tail-biting K=7 r=1/3, F bits out (one per byte) */
int orc_viterbi37_tb_decode_f(const float *sym, uint32_t F, uint8_t *out);
/* one DCI candidate as srslte_pdcch_decode_msg: 1 decoded (data: nof_bits + 16 bits), 0 skipped */
int orc_dci_decode(const float *e, uint32_t E, uint32_t nof_bits, uint8_t *data, uint16_t *crc_rem);
/* PCFICH: RE map (16 indices into symbol 0) and srslte_pcfich_decode_multi; y [rx], h [port*nrx+rx] */
int orc_pcfich_re_map(uint32_t nof_prb, uint32_t cell_id, uint32_t *idx);
int orc_pcfich_decode(uint32_t nof_prb, uint32_t cell_id, uint32_t nof_ports, uint32_t nrx,
                      const float *const *y, const float *const *h, float noise, uint32_t sf_idx,
                      uint32_t *cfi, float *corr);
/* UCI on the PUSCH: HARQ-ACK / RI / CQI and the deinterleaved g bits (see pdsch_oracle.c) */
int orc_viterbi37_tb_decode_s(const int16_t *sym, uint32_t F, uint8_t *out);
int orc_ulsch_uci(uint32_t tbs, uint32_t Qm, uint32_t nof_bits, uint32_t nsymb, uint32_t M_sc, uint32_t M_sc_init,
                  const uint32_t *I_off, const uint32_t *O, const int16_t *q_in, const uint8_t *c, uint8_t *out,
                  int16_t *g, uint32_t *qp);
/* 8-bit LLR chain (llr_is_8bit) */
int orc_demod_b(int mod, const float *sym, int nsym, int8_t *llr);
int orc_scramble_sb(uint32_t seed, int8_t *llr, uint32_t len);
int orc_csi_correction_b(int mod, const float *csi, int nsym, int8_t *e);
int orc_feedback(const float *h00, const float *h01, const float *h10, const float *h11, uint32_t nof_ce, float noise,
                 uint32_t flags, int nports, int nrx, float *out_cn, int32_t *out_i, float *sinr);
#endif
