/*
 * REFERENCE HARNESS — TEST INFRASTRUCTURE ONLY.
 *
 * Thin driver over the srsLTE reference FEC code compiled from its own sources in
 * /root/reference/lib (recipe: oracle/Makefile, target `ref`; output oracle/_ref/). It exposes
 * the same entry-point shapes as tdec_oracle.h so tests can check the restatement against the
 * real reference, and tests/golden/make_golden.py can record golden vectors from it.
 * Nothing here is product code and no reference source is copied into this repository.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "srslte/phy/fec/cbsegm.h"
#include "srslte/phy/fec/crc.h"
#include "srslte/phy/fec/tc_interl.h"
#include "srslte/phy/fec/turbocoder.h"
#include "srslte/phy/fec/turbodecoder.h"

/* Same call sequence as turbodecoder_test.c:200-266 / sch.c:356-366: init, (force_not_sb),
 * new_cb, then one srslte_tdec_iteration per half-iteration (each returns the decision). */
int ref_tdec_run(int impl, int sb_layout, const int16_t *input, uint32_t K, uint32_t nof_halfits,
                 uint8_t *decisions, int16_t *final_app1, int16_t *final_ext1) {
  srslte_tdec_t h;
  if (srslte_tdec_init_manual(&h, SRSLTE_TCOD_MAX_LEN_CB, (srslte_tdec_impl_type_t)impl)) return -1;
  if (!sb_layout) srslte_tdec_force_not_sb(&h);
  /* the reference writes tail copies into the input padding: give it a private copy */
  size_t n = 3 * (SRSLTE_TCOD_MAX_LEN_CB + 32) + 64;
  int16_t *buf = NULL;
  if (posix_memalign((void **)&buf, 64, n * sizeof(int16_t))) return -1;
  memset(buf, 0, n * sizeof(int16_t));
  int sb_eff = sb_layout && impl == SRSLTE_TDEC_AUTO && srslte_tdec_autoimp_get_subblocks(K) > 0;
  size_t in_len = sb_eff ? 3 * (K + 32) + 12 : 3 * K + 12;
  memcpy(buf, input, in_len * sizeof(int16_t));
  if (srslte_tdec_new_cb(&h, K)) {
    free(buf);
    srslte_tdec_free(&h);
    return -1;
  }
  uint8_t tmp[SRSLTE_TCOD_MAX_LEN_CB / 8];
  for (uint32_t i = 0; i < nof_halfits; i++) {
    srslte_tdec_iteration(&h, buf, decisions ? decisions + (size_t)i * (K / 8) : tmp);
  }
  if (final_app1) memcpy(final_app1, h.app1, K * sizeof(int16_t));
  if (final_ext1) memcpy(final_ext1, h.ext1, K * sizeof(int16_t));
  free(buf);
  srslte_tdec_free(&h);
  return 0;
}

/* srslte_tdec_run_all over many CBs with ONE decoder object (the CPU baseline loop of
 * BASELINE.md §3). inputs: n x stride int16, natural layout (force_not_sb), outputs n x K/8. */
int ref_tdec_run_all_many(int impl, const int16_t *inputs, size_t stride, uint32_t K, uint32_t n,
                          uint32_t nof_halfits, uint8_t *outputs) {
  srslte_tdec_t h;
  if (srslte_tdec_init_manual(&h, SRSLTE_TCOD_MAX_LEN_CB, (srslte_tdec_impl_type_t)impl)) return -1;
  srslte_tdec_force_not_sb(&h);
  int16_t *buf = NULL;
  size_t len = 3 * K + 12;
  if (posix_memalign((void **)&buf, 64, (len + 64) * sizeof(int16_t))) return -1;
  for (uint32_t c = 0; c < n; c++) {
    memcpy(buf, inputs + (size_t)c * stride, len * sizeof(int16_t));
    srslte_tdec_run_all(&h, buf, outputs + (size_t)c * (K / 8), nof_halfits, K);
  }
  free(buf);
  srslte_tdec_free(&h);
  return 0;
}

int ref_interl(uint32_t K, uint32_t nsb, uint16_t *fwd, uint16_t *rev) {
  srslte_tc_interl_t t;
  if (srslte_tc_interl_init(&t, SRSLTE_TCOD_MAX_LEN_CB)) return -1;
  int r = srslte_tc_interl_LTE_gen_interl(&t, K, nsb);
  if (!r) {
    memcpy(fwd, t.forward, K * sizeof(uint16_t));
    memcpy(rev, t.reverse, K * sizeof(uint16_t));
  }
  srslte_tc_interl_free(&t);
  return r;
}

int ref_tcod_encode(const uint8_t *in_bits, uint8_t *out_bits, uint32_t K) {
  srslte_tcod_t t;
  if (srslte_tcod_init(&t, SRSLTE_TCOD_MAX_LEN_CB)) return -1;
  uint8_t *in = malloc(K);
  memcpy(in, in_bits, K);
  int r = srslte_tcod_encode(&t, in, out_bits, K);
  free(in);
  /* srslte_tcod_free would tear down the shared static tables; keep them for reuse */
  free(t.temp);
  return r;
}

uint32_t ref_crc_checksum_byte(uint32_t poly, int order, const uint8_t *data, uint32_t len_bits) {
  srslte_crc_t c;
  if (srslte_crc_init(&c, poly, order)) return 0xffffffff;
  return srslte_crc_checksum_byte(&c, (uint8_t *)data, (int)len_bits);
}

int ref_cbsegm(uint32_t tbs, uint32_t *out6) {
  srslte_cbsegm_t s;
  int r = srslte_cbsegm(&s, tbs);
  out6[0] = s.C;
  out6[1] = s.C1;
  out6[2] = s.K1;
  out6[3] = s.C2;
  out6[4] = s.K2;
  out6[5] = s.F;
  return r;
}

uint32_t ref_autoimp_subblocks(uint32_t K) { return srslte_tdec_autoimp_get_subblocks(K); }

/* decode_tb_cb inner loop for one code block (sch.c:356-391): srslte_tdec_iteration then
 * srslte_crc_checksum_byte until the CRC passes or max_halfits half-iterations ran. */
int ref_tdec_decode_cb(int impl, int sb_layout, const int16_t *input, uint32_t K,
                       uint32_t max_halfits, uint32_t crc_poly, uint32_t crc_len_bits,
                       uint8_t *out_bytes, uint32_t *noi) {
  srslte_tdec_t h;
  srslte_crc_t crc;
  if (srslte_crc_init(&crc, crc_poly, 24)) return -1;
  if (srslte_tdec_init_manual(&h, SRSLTE_TCOD_MAX_LEN_CB, (srslte_tdec_impl_type_t)impl)) return -1;
  if (!sb_layout) srslte_tdec_force_not_sb(&h);
  size_t n = 3 * (SRSLTE_TCOD_MAX_LEN_CB + 32) + 64;
  int16_t *buf = NULL;
  if (posix_memalign((void **)&buf, 64, n * sizeof(int16_t))) return -1;
  memset(buf, 0, n * sizeof(int16_t));
  int sb_eff = sb_layout && impl == SRSLTE_TDEC_AUTO && srslte_tdec_autoimp_get_subblocks(K) > 0;
  memcpy(buf, input, (sb_eff ? 3 * (K + 32) + 12 : 3 * K + 12) * sizeof(int16_t));
  srslte_tdec_new_cb(&h, K);
  int ok = 0;
  uint32_t it = 0;
  do {
    srslte_tdec_iteration(&h, buf, out_bytes);
    it++;
    if (!srslte_crc_checksum_byte(&crc, out_bytes, (int)crc_len_bits)) ok = 1;
  } while (it < max_halfits && !ok);
  *noi = it;
  free(buf);
  srslte_tdec_free(&h);
  return ok;
}

/* ---------------------------------------------------------------- DL-SCH (sch.c) ---------- */
#include "srslte/phy/fec/rm_turbo.h"
#include "srslte/phy/fec/softbuffer.h"
#include "srslte/phy/phch/pdsch_cfg.h"
#include "srslte/phy/phch/sch.h"

/* srslte_rm_turbo_rx_lut_ (rm_turbo.c:394-430): out += de-rate-matched in; sb_layout selects the
 * sub-block table the decoder expects (enable_input_tdec). */
int ref_rm_turbo_rx(const int16_t *input, int16_t *output, uint32_t in_len, uint32_t K,
                    uint32_t rv, int sb_layout) {
  srslte_rm_turbo_gentables();
  int idx = srslte_cbsegm_cbindex(K);
  if (idx < 0) return -1;
  int16_t *in = NULL;
  if (posix_memalign((void **)&in, 64, (in_len + 32) * sizeof(int16_t))) return -1;
  memcpy(in, input, in_len * sizeof(int16_t));
  int r = srslte_rm_turbo_rx_lut_(in, output, in_len, (uint32_t)idx, rv, sb_layout != 0);
  free(in);
  return r;
}

static srslte_sch_t ref_sch;
static int ref_sch_ready = 0;

static int ref_sch_get(void) {
  if (!ref_sch_ready) {
    if (srslte_sch_init(&ref_sch)) return -1;
    ref_sch_ready = 1;
  }
  return 0;
}

static void ref_cfg(srslte_pdsch_cfg_t *cfg, uint32_t tbs, uint32_t rv, uint32_t Qm,
                    uint32_t nof_e_bits) {
  memset(cfg, 0, sizeof(*cfg));
  srslte_cbsegm(&cfg->cb_segm[0], tbs);
  cfg->grant.tb_en[0] = true;
  cfg->grant.Qm[0] = Qm;
  cfg->nbits[0].nof_bits = nof_e_bits;
  cfg->rv[0] = rv;
  cfg->nof_layers = 1;
}

/* srslte_dlsch_encode2 (sch.c:543-): data (tbs/8 bytes) -> packed e bits (nof_e_bits). */
int ref_dlsch_encode(uint32_t tbs, uint32_t rv, uint32_t Qm, uint32_t nof_e_bits,
                     const uint8_t *data, uint8_t *e_packed, uint32_t nof_prb) {
  if (ref_sch_get()) return -1;
  srslte_pdsch_cfg_t cfg;
  ref_cfg(&cfg, tbs, rv, Qm, nof_e_bits);
  srslte_softbuffer_tx_t sb;
  if (srslte_softbuffer_tx_init(&sb, nof_prb)) return -1;
  srslte_softbuffer_tx_reset(&sb);
  uint8_t *d = calloc(tbs / 8 + 16, 1);
  memcpy(d, data, tbs / 8);
  /* srslte_rm_turbo_tx_lut fills the circular buffer only at rv 0 (rm_turbo.c:332-343); a
   * retransmission reuses it, so encode rv 0 first as a HARQ process would */
  int r = 0;
  if (rv != 0) {
    srslte_pdsch_cfg_t cfg0;
    ref_cfg(&cfg0, tbs, 0, Qm, nof_e_bits);
    r = srslte_dlsch_encode2(&ref_sch, &cfg0, &sb, d, e_packed, 0);
  }
  if (!r) r = srslte_dlsch_encode2(&ref_sch, &cfg, &sb, d, e_packed, 0);
  free(d);
  srslte_softbuffer_tx_free(&sb);
  return r;
}

/* A persistent rx softbuffer per HARQ slot, as a UE keeps one per process. */
#define REF_NSLOT 8
static srslte_softbuffer_rx_t ref_sbrx[REF_NSLOT];
static int ref_sbrx_ready[REF_NSLOT];

int ref_softbuffer_reset(int slot, uint32_t nof_prb) {
  if (slot < 0 || slot >= REF_NSLOT) return -1;
  if (!ref_sbrx_ready[slot]) {
    if (srslte_softbuffer_rx_init(&ref_sbrx[slot], nof_prb)) return -1;
    ref_sbrx_ready[slot] = 1;
  }
  srslte_softbuffer_rx_reset(&ref_sbrx[slot]);
  return 0;
}

/* srslte_dlsch_decode2 (sch.c:500-512 -> decode_tb -> decode_tb_cb): int16 e bits -> data.
 * Returns the reference's return code; *noi = srslte_sch_last_noi; cb_crc[] copied out. */
int ref_dlsch_decode(int slot, uint32_t tbs, uint32_t rv, uint32_t Qm, uint32_t nof_e_bits,
                     const int16_t *e_bits, uint8_t *data, uint32_t max_halfits, uint32_t *noi,
                     uint8_t *cb_crc) {
  if (ref_sch_get()) return -100;
  if (slot < 0 || slot >= REF_NSLOT || !ref_sbrx_ready[slot]) return -100;
  srslte_pdsch_cfg_t cfg;
  ref_cfg(&cfg, tbs, rv, Qm, nof_e_bits);
  srslte_sch_set_max_noi(&ref_sch, max_halfits);
  int16_t *e = NULL;
  if (posix_memalign((void **)&e, 64, (nof_e_bits + 64) * sizeof(int16_t))) return -100;
  memcpy(e, e_bits, nof_e_bits * sizeof(int16_t));
  int r = srslte_dlsch_decode2(&ref_sch, &cfg, &ref_sbrx[slot], e, data, 0);
  free(e);
  *noi = srslte_sch_last_noi(&ref_sch);
  for (uint32_t i = 0; i < cfg.cb_segm[0].C && cb_crc; i++) cb_crc[i] = ref_sbrx[slot].cb_crc[i];
  return r;
}

/* ---------------------------------------------------------------- UL-SCH (§8(f) rank 3) ---- */
#include "srslte/phy/phch/pusch_cfg.h"

static void ref_ul_cfg(srslte_pusch_cfg_t *cfg, uint32_t tbs, uint32_t rv, uint32_t Qm,
                       uint32_t nof_bits, uint32_t nof_symb) {
  memset(cfg, 0, sizeof(*cfg));
  srslte_cbsegm(&cfg->cb_segm, tbs);
  cfg->grant.Qm = Qm;
  cfg->nbits.nof_bits = nof_bits;
  cfg->nbits.nof_symb = nof_symb;
  cfg->nbits.nof_re = nof_bits / Qm;
  cfg->rv = rv;
}

/* srslte_ulsch_encode (sch.c:987-1090, no UCI): data (tbs/8 bytes) -> packed q bits (nof_bits),
 * the rv 0 transmission first as a HARQ process makes it (rm_turbo.c:332-343) */
int ref_ulsch_encode(uint32_t tbs, uint32_t rv, uint32_t Qm, uint32_t nof_bits, uint32_t nof_symb,
                     const uint8_t *data, uint8_t *q_packed, uint32_t nof_prb) {
  if (ref_sch_get()) return -1;
  srslte_softbuffer_tx_t sb;
  if (srslte_softbuffer_tx_init(&sb, nof_prb)) return -1;
  srslte_softbuffer_tx_reset(&sb);
  uint8_t *d = calloc(tbs / 8 + 16, 1);
  uint8_t *g = calloc(nof_bits / 8 + 64, 1);
  memcpy(d, data, tbs / 8);
  int r = 0;
  for (uint32_t pass = (rv == 0); pass < 2 && !r; pass++) {
    srslte_pusch_cfg_t cfg;
    ref_ul_cfg(&cfg, tbs, pass ? rv : 0, Qm, nof_bits, nof_symb);
    memset(g, 0, nof_bits / 8 + 64);
    r = srslte_ulsch_encode(&ref_sch, &cfg, &sb, d, g, q_packed);
  }
  free(d);
  free(g);
  srslte_softbuffer_tx_free(&sb);
  return r;
}

/* srslte_ulsch_decode (sch.c:883-889): int16 q bits -> data, on the HARQ slot's softbuffer */
int ref_ulsch_decode(int slot, uint32_t tbs, uint32_t rv, uint32_t Qm, uint32_t nof_bits,
                     uint32_t nof_symb, const int16_t *q_bits, uint8_t *data, uint32_t max_halfits,
                     uint32_t *noi, uint8_t *cb_crc) {
  if (ref_sch_get()) return -100;
  if (slot < 0 || slot >= REF_NSLOT || !ref_sbrx_ready[slot]) return -100;
  srslte_pusch_cfg_t cfg;
  ref_ul_cfg(&cfg, tbs, rv, Qm, nof_bits, nof_symb);
  srslte_sch_set_max_noi(&ref_sch, max_halfits);
  int16_t *q = NULL, *g = NULL;
  if (posix_memalign((void **)&q, 64, (nof_bits + 64) * sizeof(int16_t))) return -100;
  if (posix_memalign((void **)&g, 64, (nof_bits + 64) * sizeof(int16_t))) return -100;
  memcpy(q, q_bits, nof_bits * sizeof(int16_t));
  memset(g, 0, (nof_bits + 64) * sizeof(int16_t));
  int r = srslte_ulsch_decode(&ref_sch, &cfg, &ref_sbrx[slot], q, g, data);
  free(q);
  free(g);
  *noi = srslte_sch_last_noi(&ref_sch);
  for (uint32_t i = 0; i < cfg.cb_segm.C && cb_crc; i++) cb_crc[i] = ref_sbrx[slot].cb_crc[i];
  return r;
}

/* ---------------------------------------------------------------- UCI on the PUSCH ---------- */
#include "srslte/phy/common/sequence.h"
#include "srslte/phy/phch/uci.h"
#include "srslte/phy/scrambling/scrambling.h"
/* the PUSCH configuration fields the UCI multiplexing reads (uci.c:270-290, 548-572): grant M_sc /
 * M_sc_init, the beta offset indices (36.213 Table 8.6.3-1..3), normal CP */
static void ref_uci_cfg(srslte_pusch_cfg_t *cfg, uint32_t M_sc, uint32_t M_sc_init, const uint32_t *I_off) {
  cfg->grant.M_sc = M_sc;
  cfg->grant.M_sc_init = M_sc_init;
  cfg->uci_cfg.I_offset_ack = I_off[0];
  cfg->uci_cfg.I_offset_ri = I_off[1];
  cfg->uci_cfg.I_offset_cqi = I_off[2];
  cfg->cp = SRSLTE_CP_NORM;
}

/* srslte_ulsch_uci_encode (sch.c:994-1090): data (tbs/8 bytes, tbs may be 0) with HARQ-ACK (O[0] bits
 * ack[]), RI (O[1] bits, ri) and CQI (O[2] bits cqi[], one per byte) -> packed q bits (nof_bits) */
int ref_ulsch_uci_encode(uint32_t tbs, uint32_t Qm, uint32_t nof_bits, uint32_t nof_symb, uint32_t M_sc,
                         uint32_t M_sc_init, const uint32_t *I_off, const uint32_t *O, const uint8_t *ack,
                         uint32_t ri, const uint8_t *cqi, const uint8_t *data, uint8_t *q_packed, uint32_t nof_prb) {
  if (ref_sch_get()) return -1;
  srslte_softbuffer_tx_t sb;
  if (srslte_softbuffer_tx_init(&sb, nof_prb)) return -1;
  srslte_softbuffer_tx_reset(&sb);
  uint8_t *d = calloc(tbs / 8 + 16, 1);
  uint8_t *g = calloc(nof_bits / 8 + 64, 1);
  if (tbs) memcpy(d, data, tbs / 8);
  srslte_pusch_cfg_t cfg;
  ref_ul_cfg(&cfg, tbs, 0, Qm, nof_bits, nof_symb);
  ref_uci_cfg(&cfg, M_sc, M_sc_init, I_off);
  srslte_uci_data_t u;
  memset(&u, 0, sizeof(u));
  u.uci_ack_len = O[0];
  u.uci_ack = ack[0];
  u.uci_ack_2 = ack[1];
  u.uci_ri_len = O[1];
  u.uci_ri = (uint8_t)ri;
  u.uci_cqi_len = O[2];
  for (uint32_t i = 0; i < O[2]; i++) u.uci_cqi[i] = cqi[i];
  const int r = srslte_ulsch_uci_encode(&ref_sch, &cfg, &sb, d, u, g, q_packed);
  free(d);
  free(g);
  srslte_softbuffer_tx_free(&sb);
  return r;
}

/* srslte_pusch_decode's UCI and data steps on received soft bits (pusch.c:626-657): HARQ-ACK and RI
 * from the still scrambled q bits with the sequence c (srslte_ulsch_uci_decode_ri_ack, sch.c:892-942),
 * descrambling (srslte_scrambling_s_offset), then srslte_ulsch_uci_decode (sch.c:944-985): the channel
 * deinterleaver without the RI positions, CQI (srslte_uci_decode_cqi_pusch) and the UL-SCH data on the
 * HARQ slot's softbuffer when tbs > 0. q: nof_bits int16 (scrambled), c: one byte per bit.
 * out: ack[0], ack[1], ri, cqi_ack, then the O[2] CQI bits; g_out: the deinterleaved g bits
 * (nof_bits). Returns srslte_ulsch_uci_decode's value (or the ri/ack step's error). */
int ref_ulsch_uci_decode(int slot, uint32_t tbs, uint32_t rv, uint32_t Qm, uint32_t nof_bits, uint32_t nof_symb,
                         uint32_t M_sc, uint32_t M_sc_init, const uint32_t *I_off, const uint32_t *O,
                         const int16_t *q_bits, const uint8_t *c, uint8_t *data, uint32_t max_halfits, uint32_t *noi,
                         uint8_t *cb_crc, uint8_t *out, int16_t *g_out) {
  if (ref_sch_get()) return -100;
  if (tbs && (slot < 0 || slot >= REF_NSLOT || !ref_sbrx_ready[slot])) return -100;
  srslte_pusch_cfg_t cfg;
  ref_ul_cfg(&cfg, tbs, rv, Qm, nof_bits, nof_symb);
  ref_uci_cfg(&cfg, M_sc, M_sc_init, I_off);
  srslte_sch_set_max_noi(&ref_sch, max_halfits);
  srslte_uci_data_t u;
  memset(&u, 0, sizeof(u));
  u.uci_ack_len = O[0];
  u.uci_ri_len = O[1];
  u.uci_cqi_len = O[2];
  int16_t *q = NULL, *g = NULL;
  short *cs = NULL;
  uint8_t *cc = NULL;
  if (posix_memalign((void **)&q, 64, (nof_bits + 64) * sizeof(int16_t))) return -100;
  if (posix_memalign((void **)&g, 64, (nof_bits + 64) * sizeof(int16_t))) return -100;
  if (posix_memalign((void **)&cs, 64, (nof_bits + 64) * sizeof(short))) return -100;
  if (posix_memalign((void **)&cc, 64, nof_bits + 64)) return -100;
  memcpy(q, q_bits, nof_bits * sizeof(int16_t));
  memset(g, 0, (nof_bits + 64) * sizeof(int16_t));
  memcpy(cc, c, nof_bits);
  for (uint32_t i = 0; i < nof_bits; i++) cs[i] = c[i] ? -1 : 1; /* sequence.c: c_short = 1 - 2c */
  srslte_sequence_t seq;
  memset(&seq, 0, sizeof(seq));
  seq.c = cc;
  seq.c_short = cs;
  seq.cur_len = seq.max_len = nof_bits;
  srslte_softbuffer_rx_t *sb = tbs ? &ref_sbrx[slot] : NULL;
  int r = srslte_ulsch_uci_decode_ri_ack(&ref_sch, &cfg, sb, q, cc, &u);
  if (!r) {
    srslte_scrambling_s_offset(&seq, q, 0, nof_bits);
    r = srslte_ulsch_uci_decode(&ref_sch, &cfg, sb, q, g, data, &u);
  }
  out[0] = u.uci_ack;
  out[1] = u.uci_ack_2;
  out[2] = u.uci_ri;
  out[3] = u.cqi_ack;
  for (uint32_t i = 0; i < O[2]; i++) out[4 + i] = u.uci_cqi[i];
  if (g_out) memcpy(g_out, g, nof_bits * sizeof(int16_t));
  *noi = tbs ? srslte_sch_last_noi(&ref_sch) : 0;
  for (uint32_t i = 0; tbs && i < cfg.cb_segm.C && cb_crc; i++) cb_crc[i] = ref_sbrx[slot].cb_crc[i];
  free(q);
  free(g);
  free(cs);
  free(cc);
  return r;
}

/* ---------------------------------------------------------------- PDSCH front-end ---------- */
#include "srslte/phy/mimo/precoding.h"
#include "srslte/phy/modem/demod_soft.h"
#include "srslte/phy/phch/pdsch.h"
#include "srslte/phy/common/sequence.h"
#include "srslte/phy/scrambling/scrambling.h"

/* srslte_demod_soft_demodulate_s (demod_soft.c:437-456): symbols interleaved re/im float32 */
int ref_demod_s(int mod, const float *sym, int nsym, int16_t *llr) {
  cf_t *s = NULL;
  int16_t *l = NULL;
  if (posix_memalign((void **)&s, 64, (nsym + 16) * sizeof(cf_t))) return -1;
  if (posix_memalign((void **)&l, 64, (6 * nsym + 64) * sizeof(int16_t))) return -1;
  memcpy(s, sym, nsym * sizeof(cf_t));
  int r = srslte_demod_soft_demodulate_s((srslte_mod_t)mod, s, l, nsym);
  const int bps = mod == SRSLTE_MOD_BPSK ? 1 : mod == SRSLTE_MOD_QPSK ? 2 : mod == SRSLTE_MOD_16QAM ? 4 : 6;
  memcpy(llr, l, (size_t)bps * nsym * sizeof(int16_t));
  free(s);
  free(l);
  return r;
}

/* srslte_sequence_pdsch (sequences.c:64-66) bits */
int ref_sequence_pdsch(uint16_t rnti, int q, uint32_t nslot, uint32_t cell_id, uint32_t len, uint8_t *c) {
  srslte_sequence_t seq;
  memset(&seq, 0, sizeof(seq));
  if (srslte_sequence_pdsch(&seq, rnti, q, nslot, cell_id, len)) return -1;
  memcpy(c, seq.c, len);
  srslte_sequence_free(&seq);
  return 0;
}

/* srslte_scrambling_s_offset (scrambling.c:48-51) with the PDSCH sequence */
int ref_scramble_pdsch_s(uint16_t rnti, int q, uint32_t nslot, uint32_t cell_id, int16_t *llr, uint32_t len) {
  srslte_sequence_t seq;
  memset(&seq, 0, sizeof(seq));
  if (srslte_sequence_pdsch(&seq, rnti, q, nslot, cell_id, len)) return -1;
  int16_t *l = NULL;
  if (posix_memalign((void **)&l, 64, (len + 32) * sizeof(int16_t))) return -1;
  memcpy(l, llr, len * sizeof(int16_t));
  srslte_scrambling_s_offset(&seq, l, 0, len);
  memcpy(llr, l, len * sizeof(int16_t));
  free(l);
  srslte_sequence_free(&seq);
  return 0;
}

/* srslte_predecoding_single_multi, one rx antenna (precoding.c:330-352); csi may be NULL */
int ref_predecode_single(const float *y, const float *h, float *x, float *csi, int n, float scaling, float noise) {
  cf_t *yy = NULL, *hh = NULL, *xx = NULL;
  float *cc = NULL;
  size_t sz = (n + 32) * sizeof(cf_t);
  if (posix_memalign((void **)&yy, 64, sz) || posix_memalign((void **)&hh, 64, sz) ||
      posix_memalign((void **)&xx, 64, sz) || posix_memalign((void **)&cc, 64, sz))
    return -1;
  memcpy(yy, y, n * sizeof(cf_t));
  memcpy(hh, h, n * sizeof(cf_t));
  cf_t *ya[SRSLTE_MAX_PORTS] = {yy}, *ha[SRSLTE_MAX_PORTS] = {hh};
  float *ca[SRSLTE_MAX_CODEWORDS] = {csi ? cc : NULL, NULL};
  int r = srslte_predecoding_single_multi(ya, ha, xx, ca, 1, n, scaling, noise);
  memcpy(x, xx, n * sizeof(cf_t));
  if (csi) memcpy(csi, cc, n * sizeof(float));
  free(yy);
  free(hh);
  free(xx);
  free(cc);
  return r;
}

/* precoding.c:1074 defines this without a declaration in precoding.h: declare it, or C99 would
 * call it through an implicit int() prototype and pass the floats as doubles */
int srslte_predecoding_ccd_mmse(cf_t *y[SRSLTE_MAX_PORTS], cf_t *h[SRSLTE_MAX_PORTS][SRSLTE_MAX_PORTS],
                                cf_t *x[SRSLTE_MAX_LAYERS], float *csi[SRSLTE_MAX_CODEWORDS],
                                int nof_rxant, int nof_ports, int nof_layers, int nof_symbols,
                                float scaling, float noise_estimate);

/* srslte_predecoding_ccd_mmse, 2 ports x 2 rx, 2 layers (precoding.c:1074-1097); h[port][rx];
 * csi0/csi1 may be NULL (non-CSI variant) */
int ref_predecode_ccd(const float *y0, const float *y1, const float *h00, const float *h01,
                      const float *h10, const float *h11, float *x0, float *x1, float *csi0,
                      float *csi1, int n, float scaling, float noise) {
  size_t sz = (n + 32) * sizeof(cf_t);
  cf_t *b[8] = {NULL};
  float *c[2] = {NULL};
  for (int i = 0; i < 8; i++)
    if (posix_memalign((void **)&b[i], 64, sz)) return -1;
  for (int i = 0; i < 2; i++)
    if (posix_memalign((void **)&c[i], 64, sz)) return -1;
  memcpy(b[0], y0, n * sizeof(cf_t));
  memcpy(b[1], y1, n * sizeof(cf_t));
  memcpy(b[2], h00, n * sizeof(cf_t));
  memcpy(b[3], h01, n * sizeof(cf_t));
  memcpy(b[4], h10, n * sizeof(cf_t));
  memcpy(b[5], h11, n * sizeof(cf_t));
  cf_t *ya[SRSLTE_MAX_PORTS] = {b[0], b[1]};
  cf_t *ha[SRSLTE_MAX_PORTS][SRSLTE_MAX_PORTS] = {{b[2], b[3]}, {b[4], b[5]}};
  cf_t *xa[SRSLTE_MAX_LAYERS] = {b[6], b[7]};
  float *ca[SRSLTE_MAX_CODEWORDS] = {csi0 ? c[0] : NULL, csi0 ? c[1] : NULL};
  int r = srslte_predecoding_ccd_mmse(ya, ha, xa, ca, 2, 2, 2, n, scaling, noise);
  memcpy(x0, b[6], n * sizeof(cf_t));
  memcpy(x1, b[7], n * sizeof(cf_t));
  if (csi0) {
    memcpy(csi0, c[0], n * sizeof(float));
    memcpy(csi1, c[1], n * sizeof(float));
  }
  for (int i = 0; i < 8; i++) free(b[i]);
  for (int i = 0; i < 2; i++) free(c[i]);
  return r;
}

/* srslte_predecoding_type(..., SRSLTE_MIMO_TYPE_SPATIAL_MULTIPLEX, ...) (precoding.c:1771-, :1715-1760):
 * 2 ports, 2 rx antennas, nof_layers 1 or 2; x1 / csi1 unused for one layer */
int ref_predecode_multiplex(const float *y0, const float *y1, const float *h00, const float *h01,
                            const float *h10, const float *h11, float *x0, float *x1, float *csi0,
                            float *csi1, int n, float scaling, float noise, int codebook_idx,
                            int nof_layers) {
  size_t sz = (n + 32) * sizeof(cf_t);
  cf_t *b[8] = {NULL};
  float *c[2] = {NULL};
  for (int i = 0; i < 8; i++)
    if (posix_memalign((void **)&b[i], 64, sz)) return -1;
  for (int i = 0; i < 2; i++)
    if (posix_memalign((void **)&c[i], 64, sz)) return -1;
  memcpy(b[0], y0, n * sizeof(cf_t));
  memcpy(b[1], y1, n * sizeof(cf_t));
  memcpy(b[2], h00, n * sizeof(cf_t));
  memcpy(b[3], h01, n * sizeof(cf_t));
  memcpy(b[4], h10, n * sizeof(cf_t));
  memcpy(b[5], h11, n * sizeof(cf_t));
  cf_t *ya[SRSLTE_MAX_PORTS] = {b[0], b[1]};
  cf_t *ha[SRSLTE_MAX_PORTS][SRSLTE_MAX_PORTS] = {{b[2], b[3]}, {b[4], b[5]}};
  cf_t *xa[SRSLTE_MAX_LAYERS] = {b[6], b[7]};
  float *ca[SRSLTE_MAX_CODEWORDS] = {csi0 ? c[0] : NULL, csi0 ? c[1] : NULL};
  int r = srslte_predecoding_type(ya, ha, xa, csi0 ? ca : NULL, 2, 2, nof_layers, codebook_idx, n,
                                  SRSLTE_MIMO_TYPE_SPATIAL_MULTIPLEX, scaling, noise);
  memcpy(x0, b[6], n * sizeof(cf_t));
  if (nof_layers == 2) memcpy(x1, b[7], n * sizeof(cf_t));
  if (csi0) {
    memcpy(csi0, c[0], n * sizeof(float));
    if (nof_layers == 2) memcpy(csi1, c[1], n * sizeof(float));
  }
  for (int i = 0; i < 8; i++) free(b[i]);
  for (int i = 0; i < 2; i++) free(c[i]);
  return r;
}

/* defined in pdsch.c:229 without a declaration in pdsch.h */
int srslte_pdsch_get(srslte_pdsch_t *q, cf_t *sf_symbols, cf_t *symbols, srslte_ra_dl_grant_t *grant,
                     uint32_t lstart, uint32_t subframe);

/* srslte_pdsch_get (pdsch.c:95-234, 250-255): RE extraction of one grant from a subframe grid
 * (nof_prb*12 x 14 cf32, 12 rows with extended CP); prb_mask[s*nof_prb + n] marks PRB n allocated in
 * slot s. nof_ports: the port count plus 256 for an extended-CP cell. */
int ref_pdsch_get(uint32_t nof_prb, uint32_t cell_id, uint32_t nof_ports, uint32_t lstart,
                  uint32_t sf_idx, const uint8_t *prb_mask, const float *grid, float *out) {
  srslte_pdsch_t q;
  memset(&q, 0, sizeof(q));
  q.cell.nof_prb = nof_prb;
  q.cell.id = cell_id;
  q.cell.nof_ports = nof_ports & 0xff;
  q.cell.cp = (nof_ports >> 8) & 1 ? SRSLTE_CP_EXT : SRSLTE_CP_NORM;
  srslte_ra_dl_grant_t g;
  memset(&g, 0, sizeof(g));
  for (uint32_t s = 0; s < 2; s++)
    for (uint32_t n = 0; n < nof_prb; n++) g.prb_idx[s][n] = prb_mask[s * nof_prb + n] != 0;
  return srslte_pdsch_get(&q, (cf_t *)grid, (cf_t *)out, &g, lstart, sf_idx);
}

/* ---------------------------------------------------------------- CRS (refsignal_dl.c) ---------- */
#include "srslte/phy/ch_estimation/refsignal_dl.h"

/* port 0/1 CRS of subframe sf_idx: 4 symbols x 2*nof_prb (refsignal_dl.c:265-318) */
int ref_crs_pilots(uint32_t nof_prb, uint32_t cell_id, uint32_t sf_idx, float *out) {
  srslte_refsignal_t q;
  memset(&q, 0, sizeof(q));
  if (srslte_refsignal_cs_init(&q, nof_prb)) return -1;
  srslte_cell_t cell;
  memset(&cell, 0, sizeof(cell));
  cell.nof_prb = nof_prb;
  cell.id = cell_id;
  cell.nof_ports = 1;
  cell.cp = SRSLTE_CP_NORM;
  if (srslte_refsignal_cs_set_cell(&q, cell)) return -1;
  memcpy(out, q.pilots[0][sf_idx], 4 * 2 * nof_prb * sizeof(cf_t));
  srslte_refsignal_free(&q);
  return 0;
}

/* the pilots of ports 2/3 (csr_refs.pilots[1]: symbol 1 of each slot, refsignal_dl.c:291-313) */
int ref_crs_pilots23(uint32_t nof_prb, uint32_t cell_id, uint32_t sf_idx, float *out) {
  srslte_refsignal_t q;
  memset(&q, 0, sizeof(q));
  if (srslte_refsignal_cs_init(&q, nof_prb)) return -1;
  srslte_cell_t cell;
  memset(&cell, 0, sizeof(cell));
  cell.nof_prb = nof_prb;
  cell.id = cell_id;
  cell.nof_ports = 4;
  cell.cp = SRSLTE_CP_NORM;
  if (srslte_refsignal_cs_set_cell(&q, cell)) return -1;
  memcpy(out, q.pilots[1][sf_idx], 2 * 2 * nof_prb * sizeof(cf_t));
  srslte_refsignal_free(&q);
  return 0;
}

/* the pilots of either CP (refsignal_dl.c:265-318): pair 0 (ports 0/1, 4 symbols) or 1 (ports 2/3,
 * 2 symbols) of subframe sf_idx, cp 0 normal / 1 extended */
int ref_crs_pilots_cp(uint32_t nof_prb, uint32_t cell_id, uint32_t cp, uint32_t pair, uint32_t sf_idx, float *out) {
  srslte_refsignal_t q;
  memset(&q, 0, sizeof(q));
  if (pair > 1 || srslte_refsignal_cs_init(&q, nof_prb)) return -1;
  srslte_cell_t cell;
  memset(&cell, 0, sizeof(cell));
  cell.nof_prb = nof_prb;
  cell.id = cell_id;
  cell.nof_ports = 4;
  cell.cp = cp ? SRSLTE_CP_EXT : SRSLTE_CP_NORM;
  if (srslte_refsignal_cs_set_cell(&q, cell)) return -1;
  memcpy(out, q.pilots[pair][sf_idx], (pair ? 2 : 4) * 2 * nof_prb * sizeof(cf_t));
  srslte_refsignal_free(&q);
  return 0;
}

/* srslte_refsignal_cs_get_sf (refsignal_dl.c:404-430) */
int ref_crs_get_sf(uint32_t nof_prb, uint32_t cell_id, uint32_t port, const float *grid, float *out) {
  srslte_cell_t cell;
  memset(&cell, 0, sizeof(cell));
  cell.nof_prb = nof_prb;
  cell.id = cell_id;
  cell.nof_ports = port < 2 ? 2 : 4;
  cell.cp = SRSLTE_CP_NORM;
  return srslte_refsignal_cs_get_sf(cell, port, (cf_t *)grid, (cf_t *)out);
}

#include "srslte/phy/phch/ra.h"
/* ra.c:697-731: MCS -> I_TBS (table 7.1.7.1-1) and modulation, then the TBS table 7.1.7.2.1-1.
 * Returns the TBS (or -1) and writes the srslte_mod_t value to *mod. */
int ref_mcs_tbs(uint32_t mcs, uint32_t nof_prb, uint32_t *mod) {
  int i = srslte_ra_tbs_idx_from_mcs(mcs);
  if (i < 0) return -1;
  *mod = (uint32_t)srslte_ra_mod_from_mcs(mcs);
  return srslte_ra_tbs_from_idx((uint32_t)i, nof_prb);
}

/* 8-bit path: init_manual(impl) [+ force_not_sb] + new_cb + nof_halfits x
 * srslte_tdec_iteration_8bit (turbodecoder.c:536-543), decisions after every half-iteration.
 * in_len int8 values are copied into a private, padded input (the reference writes tail copies
 * into it). */
int ref_tdec8_run(int impl, int sb_layout, const int8_t *input, size_t in_len, uint32_t K,
                  uint32_t nof_halfits, uint8_t *decisions) {
  srslte_tdec_t h;
  if (srslte_tdec_init_manual(&h, SRSLTE_TCOD_MAX_LEN_CB, (srslte_tdec_impl_type_t)impl)) return -1;
  if (!sb_layout) srslte_tdec_force_not_sb(&h);
  size_t n = 3 * (SRSLTE_TCOD_MAX_LEN_CB + 32) + 64;
  int8_t *buf = NULL;
  if (posix_memalign((void **)&buf, 64, n)) return -1;
  memset(buf, 0, n);
  memcpy(buf, input, in_len);
  if (srslte_tdec_new_cb(&h, K)) {
    free(buf);
    srslte_tdec_free(&h);
    return -1;
  }
  for (uint32_t i = 0; i < nof_halfits; i++) srslte_tdec_iteration_8bit(&h, buf, decisions + (size_t)i * (K / 8));
  free(buf);
  srslte_tdec_free(&h);
  return 0;
}

/* manual 8-bit window type through the 16-bit entry point (srslte_tdec_iteration), natural
 * input (force_not_sb) */
int ref_tdec8_run16(int impl, const int16_t *input, uint32_t K, uint32_t nof_halfits,
                    uint8_t *decisions) {
  srslte_tdec_t h;
  if (srslte_tdec_init_manual(&h, SRSLTE_TCOD_MAX_LEN_CB, (srslte_tdec_impl_type_t)impl)) return -1;
  srslte_tdec_force_not_sb(&h);
  size_t n = 3 * (SRSLTE_TCOD_MAX_LEN_CB + 32) + 64;
  int16_t *buf = NULL;
  if (posix_memalign((void **)&buf, 64, n * 2)) return -1;
  memset(buf, 0, n * 2);
  memcpy(buf, input, (3 * (size_t)K + 12) * 2);
  if (srslte_tdec_new_cb(&h, K)) {
    free(buf);
    srslte_tdec_free(&h);
    return -1;
  }
  for (uint32_t i = 0; i < nof_halfits; i++) srslte_tdec_iteration(&h, buf, decisions + (size_t)i * (K / 8));
  free(buf);
  srslte_tdec_free(&h);
  return 0;
}

/* ---------------------------------------------------------------- 8-bit LLR chain ---------- */
/* srslte_demod_soft_demodulate_b (demod_soft.c:458-477) */
int ref_demod_b(int mod, const float *sym, int nsym, int8_t *llr) {
  cf_t *s = NULL;
  int8_t *l = NULL;
  if (posix_memalign((void **)&s, 64, (nsym + 16) * sizeof(cf_t))) return -1;
  if (posix_memalign((void **)&l, 64, 6 * nsym + 64)) return -1;
  memcpy(s, sym, nsym * sizeof(cf_t));
  int r = srslte_demod_soft_demodulate_b((srslte_mod_t)mod, s, l, nsym);
  const int bps = mod == SRSLTE_MOD_BPSK ? 1 : mod == SRSLTE_MOD_QPSK ? 2 : mod == SRSLTE_MOD_16QAM ? 4 : 6;
  memcpy(llr, l, (size_t)bps * nsym);
  free(s);
  free(l);
  return r;
}

/* srslte_scrambling_sb_offset (scrambling.c:53-56) with the PDSCH sequence */
int ref_scramble_pdsch_sb(uint16_t rnti, int q, uint32_t nslot, uint32_t cell_id, int8_t *llr, uint32_t len) {
  srslte_sequence_t seq;
  memset(&seq, 0, sizeof(seq));
  if (srslte_sequence_pdsch(&seq, rnti, q, nslot, cell_id, len)) return -1;
  int8_t *l = NULL;
  if (posix_memalign((void **)&l, 64, len + 64)) return -1;
  memcpy(l, llr, len);
  srslte_scrambling_sb_offset(&seq, l, 0, len);
  memcpy(llr, l, len);
  free(l);
  srslte_sequence_free(&seq);
  return 0;
}

/* srslte_rm_turbo_rx_lut_8bit (rm_turbo.c:432-469): out += de-rate-matched in (int8) */
int ref_rm_turbo_rx_8bit(const int8_t *input, int8_t *output, uint32_t in_len, uint32_t K, uint32_t rv) {
  srslte_rm_turbo_gentables();
  int idx = srslte_cbsegm_cbindex(K);
  if (idx < 0) return -1;
  int8_t *in = NULL;
  if (posix_memalign((void **)&in, 64, in_len + 64)) return -1;
  memcpy(in, input, in_len);
  int r = srslte_rm_turbo_rx_lut_8bit(in, output, in_len, (uint32_t)idx, rv);
  free(in);
  return r;
}

/* srslte_dlsch_decode2 with llr_is_8bit (sch.c:344-364): int8 e bits -> data, on the same
 * persistent softbuffers as ref_dlsch_decode */
int ref_dlsch_decode8(int slot, uint32_t tbs, uint32_t rv, uint32_t Qm, uint32_t nof_e_bits,
                      const int8_t *e_bits, uint8_t *data, uint32_t max_halfits, uint32_t *noi,
                      uint8_t *cb_crc) {
  if (ref_sch_get()) return -100;
  if (slot < 0 || slot >= REF_NSLOT || !ref_sbrx_ready[slot]) return -100;
  srslte_pdsch_cfg_t cfg;
  ref_cfg(&cfg, tbs, rv, Qm, nof_e_bits);
  srslte_sch_set_max_noi(&ref_sch, max_halfits);
  int8_t *e = NULL;
  if (posix_memalign((void **)&e, 64, nof_e_bits + 64)) return -100;
  memcpy(e, e_bits, nof_e_bits);
  ref_sch.llr_is_8bit = true;
  int r = srslte_dlsch_decode2(&ref_sch, &cfg, &ref_sbrx[slot], e, data, 0);
  ref_sch.llr_is_8bit = false;
  free(e);
  *noi = srslte_sch_last_noi(&ref_sch);
  for (uint32_t i = 0; i < cfg.cb_segm[0].C && cb_crc; i++) cb_crc[i] = ref_sbrx[slot].cb_crc[i];
  return r;
}

/* ---------------------------------------------------------------- TM2 transmit diversity ---------- */
/* srslte_predecoding_type(..., SRSLTE_MIMO_TYPE_TX_DIVERSITY) (precoding.c:1811-1818) with 2 ports
 * and srslte_layerdemap_type (layermap.c:175-) -> d; csi may be NULL (CSI off) */
int ref_predecode_txdiv(const float *y0, const float *y1, const float *h00, const float *h01,
                        const float *h10, const float *h11, int nrx, int n, float scaling, float *d,
                        float *csi) {
  cf_t *y[SRSLTE_MAX_PORTS] = {NULL}, *h[SRSLTE_MAX_PORTS][SRSLTE_MAX_PORTS] = {{NULL}};
  cf_t *x[SRSLTE_MAX_LAYERS] = {NULL}, *dd = NULL;
  float *c[SRSLTE_MAX_CODEWORDS] = {NULL};
  const float *ys[2] = {y0, y1}, *hs[2][2] = {{h00, h01}, {h10, h11}};
  for (int a = 0; a < nrx; a++) {
    if (posix_memalign((void **)&y[a], 64, (n + 16) * sizeof(cf_t))) return -1;
    memcpy(y[a], ys[a], n * sizeof(cf_t));
    for (int p = 0; p < 2; p++) {
      if (posix_memalign((void **)&h[p][a], 64, (n + 16) * sizeof(cf_t))) return -1;
      memcpy(h[p][a], hs[p][a], n * sizeof(cf_t));
    }
  }
  for (int l = 0; l < 2; l++)
    if (posix_memalign((void **)&x[l], 64, (n + 16) * sizeof(cf_t))) return -1;
  if (posix_memalign((void **)&dd, 64, (n + 16) * sizeof(cf_t))) return -1;
  if (csi && posix_memalign((void **)&c[0], 64, (n + 16) * sizeof(float))) return -1;
  int r = srslte_predecoding_type(y, h, x, c, nrx, 2, 2, 0, n, SRSLTE_MIMO_TYPE_TX_DIVERSITY, scaling, 0.0f);
  int nsym[SRSLTE_MAX_CODEWORDS] = {0};
  cf_t *dp[SRSLTE_MAX_CODEWORDS] = {dd, NULL};
  if (r >= 0) r = srslte_layerdemap_type(x, dp, 2, 1, n / 2, nsym, SRSLTE_MIMO_TYPE_TX_DIVERSITY);
  memcpy(d, dd, n * sizeof(cf_t));
  if (csi) memcpy(csi, c[0], n * sizeof(float));
  for (int a = 0; a < nrx; a++) {
    free(y[a]);
    for (int p = 0; p < 2; p++) free(h[p][a]);
  }
  free(x[0]);
  free(x[1]);
  free(dd);
  free(c[0]);
  return r < 0 ? -1 : 0;
}

/* the same with 4 ports and 4 layers; y [rx], h [port * 2 + rx]; n % 4 == 0 */
int ref_predecode_txdiv4(const float *const *ys, const float *const *hs, int nrx, int n, float scaling, float *d,
                         float *csi) {
  cf_t *y[SRSLTE_MAX_PORTS] = {NULL}, *h[SRSLTE_MAX_PORTS][SRSLTE_MAX_PORTS] = {{NULL}};
  cf_t *x[SRSLTE_MAX_LAYERS] = {NULL}, *dd = NULL;
  float *c[SRSLTE_MAX_CODEWORDS] = {NULL};
  if (n % 4) return -1;
  for (int a = 0; a < nrx; a++) {
    if (posix_memalign((void **)&y[a], 64, (n + 16) * sizeof(cf_t))) return -1;
    memcpy(y[a], ys[a], n * sizeof(cf_t));
    for (int p = 0; p < 4; p++) {
      if (posix_memalign((void **)&h[p][a], 64, (n + 16) * sizeof(cf_t))) return -1;
      memcpy(h[p][a], hs[p * 2 + a], n * sizeof(cf_t));
    }
  }
  for (int l = 0; l < 4; l++)
    if (posix_memalign((void **)&x[l], 64, (n + 16) * sizeof(cf_t))) return -1;
  if (posix_memalign((void **)&dd, 64, (n + 16) * sizeof(cf_t))) return -1;
  if (csi && posix_memalign((void **)&c[0], 64, (n + 16) * sizeof(float))) return -1;
  int r = srslte_predecoding_type(y, h, x, c, nrx, 4, 4, 0, n, SRSLTE_MIMO_TYPE_TX_DIVERSITY, scaling, 0.0f);
  int nsym[SRSLTE_MAX_CODEWORDS] = {0};
  cf_t *dp[SRSLTE_MAX_CODEWORDS] = {dd, NULL};
  if (r >= 0) r = srslte_layerdemap_type(x, dp, 4, 1, n / 4, nsym, SRSLTE_MIMO_TYPE_TX_DIVERSITY);
  memcpy(d, dd, n * sizeof(cf_t));
  if (csi) memcpy(csi, c[0], n * sizeof(float));
  for (int a = 0; a < nrx; a++) {
    free(y[a]);
    for (int p = 0; p < 4; p++) free(h[p][a]);
  }
  for (int l = 0; l < 4; l++) free(x[l]);
  free(dd);
  free(c[0]);
  return r < 0 ? -1 : 0;
}

/* ---------------------------------------------------------------- Viterbi (PDCCH) ---------- */
#include "srslte/phy/fec/viterbi.h"
/* srslte_viterbi_decode_f on a tail-biting K=7 r=1/3 decoder (pdcch.c:79,341: poly {0x6D, 0x4F,
 * 0x57}, frame = DCI bits + 16): 3*F float symbols -> F bits (one per byte) */
int ref_viterbi37_tb_decode_f(const float *sym, uint32_t F, uint8_t *out) {
  int poly[3] = {0x6D, 0x4F, 0x57};
  srslte_viterbi_t v;
  if (srslte_viterbi_init(&v, SRSLTE_VITERBI_37, poly, F, true)) return -1;
  float *s = NULL;
  if (posix_memalign((void **)&s, 64, (3 * F + 64) * sizeof(float))) return -1;
  memcpy(s, sym, 3 * F * sizeof(float));
  int r = srslte_viterbi_decode_f(&v, s, out, F);
  free(s);
  srslte_viterbi_free(&v);
  return r < 0 ? -1 : 0;
}

/* srslte_pdcch_decode_msg's decode of one DCI candidate (pdcch.c:380-396 mean check, then
 * srslte_pdcch_dci_decode :322-360: srslte_rm_conv_rx, srslte_viterbi_decode_f, CRC16 remainder),
 * composed from the reference's own functions as pdcch.c calls them. Returns 1 when decoded, 0
 * when skipped (mean |llr| <= 0.5), -1 on error. */
#include <math.h>
#include <strings.h>
#include "srslte/phy/fec/rm_conv.h"
#include "srslte/phy/phch/dci.h"
#include "srslte/phy/utils/bit.h"
int ref_dci_decode(const float *e, uint32_t E, uint32_t nof_bits, uint8_t *data, uint16_t *crc_rem) {
  double mean = 0;
  for (uint32_t i = 0; i < E; i++) mean += fabsf(e[i]);
  mean /= E;
  if (!(mean > 0.5)) return 0;
  int poly[3] = {0x6D, 0x4F, 0x57};
  srslte_viterbi_t v;
  srslte_crc_t crc;
  if (srslte_viterbi_init(&v, SRSLTE_VITERBI_37, poly, SRSLTE_DCI_MAX_BITS + 16, true)) return -1;
  if (srslte_crc_init(&crc, SRSLTE_LTE_CRC16, 16)) return -1;
  float *rm = NULL, *in = NULL;
  if (posix_memalign((void **)&rm, 64, sizeof(float) * 3 * (SRSLTE_DCI_MAX_BITS + 16) + 64)) return -1;
  if (posix_memalign((void **)&in, 64, sizeof(float) * E + 64)) return -1;
  memcpy(in, e, sizeof(float) * E);
  bzero(rm, sizeof(float) * 3 * (SRSLTE_DCI_MAX_BITS + 16));
  const uint32_t coded_len = 3 * (nof_bits + 16);
  srslte_rm_conv_rx(in, E, rm, coded_len);
  srslte_viterbi_decode_f(&v, rm, data, nof_bits + 16);
  uint8_t *x = &data[nof_bits];
  const uint16_t p_bits = (uint16_t)srslte_bit_pack(&x, 16);
  const uint16_t crc_res = (uint16_t)(srslte_crc_checksum(&crc, data, nof_bits) & 0xffff);
  *crc_rem = p_bits ^ crc_res;
  srslte_viterbi_free(&v);
  free(rm);
  free(in);
  return 1;
}

/* ---------------------------------------------------------------- PCFICH ---------- */
#include "srslte/phy/phch/pcfich.h"
#include "srslte/phy/phch/regs.h"
#include "srslte/phy/utils/vector.h"
/* srslte_pcfich_decode_multi (pcfich.c:178-241) on one subframe: grids [nrx] and estimates
 * [port][rx] (14 x 12 nof_prb complex each), noise_estimate -> cfi, corr; and, with grids = NULL,
 * the 16 RE indices of srslte_regs_pcfich_get (index-valued grid) into idx */
int ref_pcfich(uint32_t nof_prb, uint32_t cell_id, uint32_t nof_ports, uint32_t nrx, const float *g0,
               const float *g1, const float *h00, const float *h01, const float *h10, const float *h11,
               float noise, uint32_t sf_idx, uint32_t *cfi, float *corr, uint32_t *idx) {
  srslte_cell_t cell = {nof_prb, nof_ports, cell_id, SRSLTE_CP_NORM, SRSLTE_PHICH_NORM, SRSLTE_PHICH_R_1};
  srslte_regs_t regs;
  srslte_pcfich_t q;
  if (srslte_regs_init(&regs, cell)) return -1;
  const uint32_t n = SRSLTE_SF_LEN_RE(nof_prb, SRSLTE_CP_NORM);
  if (!g0) {
    cf_t *g = srslte_vec_malloc(sizeof(cf_t) * n), out[REGS_PCFICH_NSYM];
    for (uint32_t i = 0; i < n; i++) g[i] = (float)i;
    const int r = srslte_regs_pcfich_get(&regs, g, out);
    for (int i = 0; i < r; i++) idx[i] = (uint32_t)crealf(out[i]);
    free(g);
    srslte_regs_free(&regs);
    return r;
  }
  if (srslte_pcfich_init(&q, nrx) || srslte_pcfich_set_cell(&q, &regs, cell)) return -1;
  cf_t *sf[SRSLTE_MAX_PORTS] = {NULL}, *ce[SRSLTE_MAX_PORTS][SRSLTE_MAX_PORTS] = {{NULL}};
  const float *gs[2] = {g0, g1}, *hs[2][2] = {{h00, h01}, {h10, h11}};
  for (uint32_t a = 0; a < nrx; a++) {
    sf[a] = srslte_vec_malloc(sizeof(cf_t) * n);
    memcpy(sf[a], gs[a], sizeof(cf_t) * n);
    for (uint32_t p = 0; p < nof_ports; p++) {
      ce[p][a] = srslte_vec_malloc(sizeof(cf_t) * n);
      memcpy(ce[p][a], hs[p][a], sizeof(cf_t) * n);
    }
  }
  const int r = srslte_pcfich_decode_multi(&q, sf, ce, noise, sf_idx, cfi, corr);
  for (uint32_t a = 0; a < nrx; a++) {
    free(sf[a]);
    for (uint32_t p = 0; p < nof_ports; p++) free(ce[p][a]);
  }
  srslte_pcfich_free(&q);
  srslte_regs_free(&regs);
  return r < 0 ? -1 : 0;
}

/* ---------------------------------------------------------------- PDCCH / DCI ---------- */
#include "srslte/phy/phch/pdcch.h"
#include "srslte/phy/phch/ra.h"

/* 36.213 tables as the reference's ra.c serves them */
int ref_tbs_from_idx(uint32_t idx, uint32_t nprb) { return srslte_ra_tbs_from_idx(idx, nprb); }
int ref_tbs_idx_from_mcs(uint32_t mcs) { return srslte_ra_tbs_idx_from_mcs(mcs); }
/* tbs_format1c_table[mcs] through srslte_ra_dl_dci_to_grant (ra.c:517-522) for an SI-RNTI 1C */
int ref_tbs_1c(uint32_t mcs) {
  srslte_ra_dl_dci_t d;
  srslte_ra_dl_grant_t g;
  memset(&d, 0, sizeof(d));
  d.alloc_type = SRSLTE_RA_ALLOC_TYPE2;
  d.type2_alloc.mode = SRSLTE_RA_TYPE2_LOC;
  d.type2_alloc.L_crb = 4;
  d.dci_is_1c = true;
  d.mcs_idx = mcs;
  d.tb_en[0] = true;
  if (srslte_ra_dl_dci_to_grant(&d, 25, SRSLTE_SIRNTI, &g)) return -1;
  return g.mcs[0].tbs;
}
uint32_t ref_dci_sizeof(uint32_t format, uint32_t nof_prb, uint32_t nof_ports) {
  return srslte_dci_format_sizeof((srslte_dci_format_t)format, nof_prb, nof_ports);
}

static int ref_regs_cell(srslte_regs_t *regs, srslte_cell_t *cell, uint32_t nof_prb, uint32_t cell_id,
                         uint32_t nof_ports, uint32_t phich_len, uint32_t phich_res) {
  /* nof_ports: the port count plus 256 for an extended-CP cell */
  srslte_cell_t c = {nof_prb, nof_ports & 0xff, cell_id, (nof_ports >> 8) & 1 ? SRSLTE_CP_EXT : SRSLTE_CP_NORM,
                     (srslte_phich_length_t)phich_len, (srslte_phich_resources_t)phich_res};
  *cell = c;
  return srslte_regs_init(regs, c);
}

/* srslte_regs_pdcch_get's symbol order for this cell and CFI as grid indices (an index-valued
 * grid), and NOF_CCE(cfi); returns the symbol count */
int ref_pdcch_map(uint32_t nof_prb, uint32_t cell_id, uint32_t nof_ports, uint32_t phich_len,
                  uint32_t phich_res, uint32_t cfi, uint32_t *idx, uint32_t *nof_cce) {
  srslte_regs_t regs;
  srslte_cell_t cell;
  srslte_pdcch_t q;
  if (ref_regs_cell(&regs, &cell, nof_prb, cell_id, nof_ports, phich_len, phich_res)) return -1;
  if (srslte_pdcch_init_ue(&q, SRSLTE_MAX_PRB, 1) || srslte_pdcch_set_cell(&q, &regs, cell)) return -1;
  const uint32_t n = SRSLTE_SF_LEN_RE(nof_prb, SRSLTE_CP_NORM);
  cf_t *g = srslte_vec_malloc(sizeof(cf_t) * n), *out = srslte_vec_malloc(sizeof(cf_t) * n);
  for (uint32_t i = 0; i < n; i++) g[i] = (float)i;
  const int r = srslte_regs_pdcch_get(&regs, cfi, g, out);
  for (int i = 0; i < r; i++) idx[i] = (uint32_t)crealf(out[i]);
  *nof_cce = q.nof_cce[cfi - 1];
  free(g);
  free(out);
  srslte_pdcch_free(&q);
  srslte_regs_free(&regs);
  return r;
}

/* srslte_pdcch_encode (pdcch.c:568-643) of n DCI messages (bits[i * 128 ..], nof_bits[i], at
 * aggregation level L[i] and first CCE ncce[i], CRC masked with rnti[i]) into the port grids
 * (14 x 12 nof_prb complex each, added to what they hold) */
int ref_pdcch_encode(uint32_t nof_prb, uint32_t cell_id, uint32_t nof_ports, uint32_t phich_len,
                     uint32_t phich_res, uint32_t cfi, uint32_t sf_idx, uint32_t n, const uint8_t *bits,
                     const uint32_t *nof_bits, const uint32_t *L, const uint32_t *ncce,
                     const uint16_t *rnti, float *grid0, float *grid1) {
  srslte_regs_t regs;
  srslte_cell_t cell;
  srslte_pdcch_t q;
  if (ref_regs_cell(&regs, &cell, nof_prb, cell_id, nof_ports, phich_len, phich_res)) return -1;
  if (srslte_pdcch_init_enb(&q, SRSLTE_MAX_PRB) || srslte_pdcch_set_cell(&q, &regs, cell)) return -1;
  cf_t *sf[SRSLTE_MAX_PORTS] = {(cf_t *)grid0, (cf_t *)grid1, NULL, NULL};
  int ret = 0;
  for (uint32_t i = 0; i < n && !ret; i++) {
    srslte_dci_msg_t msg;
    memset(&msg, 0, sizeof(msg));
    memcpy(msg.data, bits + 128 * i, nof_bits[i]);
    msg.nof_bits = nof_bits[i];
    srslte_dci_location_t loc = {L[i], ncce[i]};
    ret = srslte_pdcch_encode(&q, &msg, loc, rnti[i], sf, sf_idx, cfi) ? -1 : 0;
  }
  srslte_pdcch_free(&q);
  srslte_regs_free(&regs);
  return ret;
}

static int ref_pdcch_rx(srslte_regs_t *regs, srslte_pdcch_t *q, uint32_t nof_prb, uint32_t cell_id,
                        uint32_t nof_ports, uint32_t phich_len, uint32_t phich_res, uint32_t nrx) {
  srslte_cell_t cell;
  if (ref_regs_cell(regs, &cell, nof_prb, cell_id, nof_ports, phich_len, phich_res)) return -1;
  if (srslte_pdcch_init_ue(q, SRSLTE_MAX_PRB, nrx) || srslte_pdcch_set_cell(q, regs, cell)) return -1;
  return 0;
}

/* srslte_pdcch_extract_llr_multi (pdcch.c:424-506): grids [nrx], estimates [port][rx] -> the
 * 72 NOF_CCE(cfi) float LLRs of q->llr; returns that count */
int ref_pdcch_llr(uint32_t nof_prb, uint32_t cell_id, uint32_t nof_ports, uint32_t phich_len,
                  uint32_t phich_res, uint32_t nrx, uint32_t cfi, uint32_t sf_idx, float noise,
                  const float *g0, const float *g1, const float *h00, const float *h01, const float *h10,
                  const float *h11, float *llr) {
  srslte_regs_t regs;
  srslte_pdcch_t q;
  if (ref_pdcch_rx(&regs, &q, nof_prb, cell_id, nof_ports, phich_len, phich_res, nrx)) return -1;
  const uint32_t n = SRSLTE_SF_LEN_RE(nof_prb, SRSLTE_CP_NORM);
  cf_t *sf[SRSLTE_MAX_PORTS] = {NULL}, *ce[SRSLTE_MAX_PORTS][SRSLTE_MAX_PORTS] = {{NULL}};
  const float *gs[2] = {g0, g1}, *hs[2][2] = {{h00, h01}, {h10, h11}};
  for (uint32_t a = 0; a < nrx; a++) {
    sf[a] = srslte_vec_malloc(sizeof(cf_t) * n);
    memcpy(sf[a], gs[a], sizeof(cf_t) * n);
    for (uint32_t p = 0; p < nof_ports; p++) {
      ce[p][a] = srslte_vec_malloc(sizeof(cf_t) * n);
      memcpy(ce[p][a], hs[p][a], sizeof(cf_t) * n);
    }
  }
  int r = srslte_pdcch_extract_llr_multi(&q, sf, ce, noise, sf_idx, cfi);
  const int e = 72 * (int)q.nof_cce[cfi - 1];
  if (r == 0) memcpy(llr, q.llr, sizeof(float) * e);
  for (uint32_t a = 0; a < nrx; a++) {
    free(sf[a]);
    for (uint32_t p = 0; p < nof_ports; p++) free(ce[p][a]);
  }
  srslte_pdcch_free(&q);
  srslte_regs_free(&regs);
  return r ? -1 : e;
}

/* 4-port forms (any port count): grids / estimates as arrays, h[p * 2 + a] */
int ref_pdcch_encode_n(uint32_t nof_prb, uint32_t cell_id, uint32_t nof_ports, uint32_t phich_len, uint32_t phich_res,
                       uint32_t cfi, uint32_t sf_idx, uint32_t n, const uint8_t *bits, const uint32_t *nof_bits,
                       const uint32_t *L, const uint32_t *ncce, const uint16_t *rnti, float *const *grids) {
  srslte_regs_t regs;
  srslte_cell_t cell;
  srslte_pdcch_t q;
  if (ref_regs_cell(&regs, &cell, nof_prb, cell_id, nof_ports, phich_len, phich_res)) return -1;
  if (srslte_pdcch_init_enb(&q, SRSLTE_MAX_PRB) || srslte_pdcch_set_cell(&q, &regs, cell)) return -1;
  cf_t *sf[SRSLTE_MAX_PORTS] = {NULL};
  for (uint32_t p = 0; p < nof_ports; p++) sf[p] = (cf_t *)grids[p];
  int ret = 0;
  for (uint32_t i = 0; i < n && !ret; i++) {
    srslte_dci_msg_t msg;
    memset(&msg, 0, sizeof(msg));
    memcpy(msg.data, bits + 128 * i, nof_bits[i]);
    msg.nof_bits = nof_bits[i];
    srslte_dci_location_t loc = {L[i], ncce[i]};
    ret = srslte_pdcch_encode(&q, &msg, loc, rnti[i], sf, sf_idx, cfi) ? -1 : 0;
  }
  srslte_pdcch_free(&q);
  srslte_regs_free(&regs);
  return ret;
}

int ref_pdcch_llr_n(uint32_t nof_prb, uint32_t cell_id, uint32_t nof_ports, uint32_t phich_len, uint32_t phich_res,
                    uint32_t nrx, uint32_t cfi, uint32_t sf_idx, float noise, const float *const *gs,
                    const float *const *hs, float *llr) {
  srslte_regs_t regs;
  srslte_pdcch_t q;
  if (ref_pdcch_rx(&regs, &q, nof_prb, cell_id, nof_ports, phich_len, phich_res, nrx)) return -1;
  const uint32_t n = SRSLTE_SF_LEN_RE(nof_prb, SRSLTE_CP_NORM);
  cf_t *sf[SRSLTE_MAX_PORTS] = {NULL}, *ce[SRSLTE_MAX_PORTS][SRSLTE_MAX_PORTS] = {{NULL}};
  for (uint32_t a = 0; a < nrx; a++) {
    sf[a] = srslte_vec_malloc(sizeof(cf_t) * n);
    memcpy(sf[a], gs[a], sizeof(cf_t) * n);
    for (uint32_t p = 0; p < nof_ports; p++) {
      ce[p][a] = srslte_vec_malloc(sizeof(cf_t) * n);
      memcpy(ce[p][a], hs[p * 2 + a], sizeof(cf_t) * n);
    }
  }
  int r = srslte_pdcch_extract_llr_multi(&q, sf, ce, noise, sf_idx, cfi);
  const int e = 72 * (int)q.nof_cce[cfi - 1];
  if (r == 0) memcpy(llr, q.llr, sizeof(float) * e);
  for (uint32_t a = 0; a < nrx; a++) {
    free(sf[a]);
    for (uint32_t p = 0; p < nof_ports; p++) free(ce[p][a]);
  }
  srslte_pdcch_free(&q);
  srslte_regs_free(&regs);
  return r ? -1 : e;
}

int ref_pcfich_n(uint32_t nof_prb, uint32_t cell_id, uint32_t nof_ports, uint32_t nrx, const float *const *gs,
                 const float *const *hs, float noise, uint32_t sf_idx, uint32_t *cfi, float *corr) {
  srslte_cell_t cell = {nof_prb, nof_ports, cell_id, SRSLTE_CP_NORM, SRSLTE_PHICH_NORM, SRSLTE_PHICH_R_1};
  srslte_regs_t regs;
  srslte_pcfich_t q;
  if (srslte_regs_init(&regs, cell)) return -1;
  const uint32_t n = SRSLTE_SF_LEN_RE(nof_prb, SRSLTE_CP_NORM);
  if (srslte_pcfich_init(&q, nrx) || srslte_pcfich_set_cell(&q, &regs, cell)) return -1;
  cf_t *sf[SRSLTE_MAX_PORTS] = {NULL}, *ce[SRSLTE_MAX_PORTS][SRSLTE_MAX_PORTS] = {{NULL}};
  for (uint32_t a = 0; a < nrx; a++) {
    sf[a] = srslte_vec_malloc(sizeof(cf_t) * n);
    memcpy(sf[a], gs[a], sizeof(cf_t) * n);
    for (uint32_t p = 0; p < nof_ports; p++) {
      ce[p][a] = srslte_vec_malloc(sizeof(cf_t) * n);
      memcpy(ce[p][a], hs[p * 2 + a], sizeof(cf_t) * n);
    }
  }
  const int r = srslte_pcfich_decode_multi(&q, sf, ce, noise, sf_idx, cfi, corr);
  for (uint32_t a = 0; a < nrx; a++) {
    free(sf[a]);
    for (uint32_t p = 0; p < nof_ports; p++) free(ce[p][a]);
  }
  srslte_pcfich_free(&q);
  srslte_regs_free(&regs);
  return r < 0 ? -1 : 0;
}

/* The DL / UL DCI blind searches (ue_dl.c:768-932) run from the reference's own ue_dl.c in
 * oracle/ref_front.c (ue_dl.c reaches the DFT through ofdm.c, so it cannot be in this library). */

/* srslte_dci_msg_pack_pusch (dci.c:511-569, format 0) from 8 fields: freq_hop_fl (-1 disabled, 0..3),
 * L_crb, RB_start, mcs_idx, ndi, tpc_pusch, n_dmrs, cqi_request; returns nof_bits */
int ref_dci_pack_ul(uint32_t nof_prb, const int32_t *f, uint8_t *bits) {
  srslte_ra_ul_dci_t d;
  memset(&d, 0, sizeof(d));
  d.freq_hop_fl = f[0];
  d.type2_alloc.L_crb = (uint32_t)f[1];
  d.type2_alloc.RB_start = (uint32_t)f[2];
  d.mcs_idx = (uint32_t)f[3];
  d.ndi = f[4] != 0;
  d.tpc_pusch = (uint8_t)f[5];
  d.n_dmrs = (uint32_t)f[6];
  d.cqi_request = f[7] != 0;
  srslte_dci_msg_t msg;
  memset(&msg, 0, sizeof(msg));
  if (srslte_dci_msg_pack_pusch(&d, &msg, nof_prb)) return -1;
  memcpy(bits, msg.data, msg.nof_bits);
  return (int)msg.nof_bits;
}

/* srslte_dci_msg_to_ul_grant (dci.c:165-197): dci11 = freq_hop_fl riv L_crb RB_start mcs_idx rv_idx
 * n_dmrs ndi cqi_request tpc_pusch 0; grant10 = L_prb n_prb[0] n_prb[1] freq_hopping M_sc Qm mod tbs
 * mcs.idx ncs_dmrs (the order of ref_front.c) */
int ref_dci_to_ul_grant(const uint8_t *bits, uint32_t nof_bits, uint32_t nof_prb, uint32_t n_rb_ho,
                        int32_t *dci11, int32_t *grant10) {
  srslte_dci_msg_t msg;
  memset(&msg, 0, sizeof(msg));
  memcpy(msg.data, bits, SRSLTE_DCI_MAX_BITS);
  msg.nof_bits = nof_bits;
  msg.format = SRSLTE_DCI_FORMAT0;
  srslte_ra_ul_dci_t d;
  srslte_ra_ul_grant_t g;
  const int r = srslte_dci_msg_to_ul_grant(&msg, nof_prb, n_rb_ho, &d, &g, 0);
  const int32_t dv[11] = {(int32_t)d.freq_hop_fl, (int32_t)d.type2_alloc.riv, (int32_t)d.type2_alloc.L_crb,
                          (int32_t)d.type2_alloc.RB_start, (int32_t)d.mcs_idx, (int32_t)d.rv_idx, (int32_t)d.n_dmrs,
                          (int32_t)d.ndi, (int32_t)d.cqi_request, (int32_t)d.tpc_pusch, 0};
  const int32_t gv[10] = {(int32_t)g.L_prb, (int32_t)g.n_prb[0], (int32_t)g.n_prb[1], (int32_t)g.freq_hopping,
                          (int32_t)g.M_sc, (int32_t)g.Qm, (int32_t)g.mcs.mod, (int32_t)g.mcs.tbs,
                          (int32_t)g.mcs.idx, (int32_t)g.ncs_dmrs};
  memcpy(dci11, dv, sizeof(dv));
  memcpy(grant10, gv, sizeof(gv));
  return r;
}

/* bits: SRSLTE_DCI_MAX_BITS bytes as srslte_dci_msg_t.data holds them */
/* srslte_ra_dl_dci_t <-> 30 int32 fields (ref order of srsgpu_ra_dl_dci_t; the union's members
 * are read per allocation type) and srslte_ra_dl_grant_t -> 13 int32 fields + prb bytes */
static void ref_dci_out(const srslte_ra_dl_dci_t *d, int32_t *o) {
  memset(o, 0, sizeof(int32_t) * 30);
  o[0] = d->alloc_type;
  if (d->alloc_type == SRSLTE_RA_ALLOC_TYPE0) o[1] = d->type0_alloc.rbg_bitmask;
  if (d->alloc_type == SRSLTE_RA_ALLOC_TYPE1) {
    o[2] = d->type1_alloc.vrb_bitmask;
    o[3] = d->type1_alloc.rbg_subset;
    o[4] = d->type1_alloc.shift;
  }
  if (d->alloc_type == SRSLTE_RA_ALLOC_TYPE2) {
    o[5] = d->type2_alloc.riv;
    o[6] = d->type2_alloc.L_crb;
    o[7] = d->type2_alloc.RB_start;
    o[8] = d->type2_alloc.n_prb1a;
    o[9] = d->type2_alloc.n_gap;
    o[10] = d->type2_alloc.mode;
  }
  o[11] = d->harq_process; o[12] = d->mcs_idx; o[13] = d->rv_idx; o[14] = d->ndi;
  o[15] = d->mcs_idx_1; o[16] = d->rv_idx_1; o[17] = d->ndi_1; o[18] = d->tb_cw_swap;
  o[19] = d->sram_id; o[20] = d->pinfo; o[21] = d->pconf; o[22] = d->power_offset;
  o[23] = d->tb_en[0]; o[24] = d->tb_en[1]; o[25] = d->is_ra_order; o[26] = d->ra_preamble;
  o[27] = d->ra_mask_idx; o[28] = d->dci_is_1a; o[29] = d->dci_is_1c;
}
int ref_dci_to_dl_grant(const uint8_t *bits, uint32_t nof_bits, uint32_t format, uint16_t rnti,
                        uint32_t nof_prb, uint32_t nof_ports, int32_t *dci30, int32_t *grant13,
                        uint8_t *prb220) {
  srslte_dci_msg_t msg;
  memset(&msg, 0, sizeof(msg));
  memcpy(msg.data, bits, SRSLTE_DCI_MAX_BITS); /* the unpackers may read past nof_bits (1C, N_gap 2) */
  msg.nof_bits = nof_bits;
  msg.format = (srslte_dci_format_t)format;
  srslte_ra_dl_dci_t d;
  srslte_ra_dl_grant_t g;
  const int r = srslte_dci_msg_to_dl_grant(&msg, rnti, nof_prb, nof_ports, &d, &g);
  ref_dci_out(&d, dci30);
  grant13[0] = g.nof_prb; grant13[1] = g.Qm[0]; grant13[2] = g.Qm[1];
  grant13[3] = g.mcs[0].mod; grant13[4] = g.mcs[0].tbs; grant13[5] = g.mcs[0].idx;
  grant13[6] = g.mcs[1].mod; grant13[7] = g.mcs[1].tbs; grant13[8] = g.mcs[1].idx;
  grant13[9] = g.tb_en[0]; grant13[10] = g.tb_en[1]; grant13[11] = g.pinfo; grant13[12] = g.tb_cw_swap;
  for (int s = 0; s < 2; s++)
    for (int p = 0; p < 110; p++) prb220[s * 110 + p] = g.prb_idx[s][p];
  return r;
}
/* srslte_dci_msg_pack_pdsch (dci.c:1305) from 30 fields in the order above; returns nof_bits */
int ref_dci_pack_dl(uint32_t format, uint32_t nof_prb, uint32_t nof_ports, int crc_is_crnti,
                    const int32_t *f, uint8_t *bits) {
  srslte_ra_dl_dci_t d;
  memset(&d, 0, sizeof(d));
  d.alloc_type = (srslte_ra_type_t)f[0];
  if (f[0] == 0) d.type0_alloc.rbg_bitmask = f[1];
  if (f[0] == 1) {
    d.type1_alloc.vrb_bitmask = f[2];
    d.type1_alloc.rbg_subset = f[3];
    d.type1_alloc.shift = f[4];
  }
  if (f[0] == 2) {
    d.type2_alloc.riv = f[5];
    d.type2_alloc.L_crb = f[6];
    d.type2_alloc.RB_start = f[7];
    d.type2_alloc.n_prb1a = f[8];
    d.type2_alloc.n_gap = f[9];
    d.type2_alloc.mode = f[10];
  }
  d.harq_process = f[11]; d.mcs_idx = f[12]; d.rv_idx = f[13]; d.ndi = f[14];
  d.mcs_idx_1 = f[15]; d.rv_idx_1 = f[16]; d.ndi_1 = f[17]; d.tb_cw_swap = f[18];
  d.sram_id = f[19]; d.pinfo = f[20]; d.pconf = f[21]; d.power_offset = f[22];
  d.tb_en[0] = f[23]; d.tb_en[1] = f[24];
  srslte_dci_msg_t msg;
  memset(&msg, 0, sizeof(msg));
  if (srslte_dci_msg_pack_pdsch(&d, (srslte_dci_format_t)format, &msg, nof_prb, nof_ports, crc_is_crnti))
    return -1;
  memcpy(bits, msg.data, msg.nof_bits);
  return (int)msg.nof_bits;
}
/* srslte_pdcch_ue_locations_ncce / srslte_pdcch_common_locations_ncce (pdcch.c:227-300):
 * 2 uint32 (L, ncce) per candidate */
int ref_pdcch_locations(uint32_t nof_cce, uint32_t sf_idx, uint16_t rnti, int common, uint32_t *out) {
  srslte_dci_location_t c[64];
  const uint32_t n = common ? srslte_pdcch_common_locations_ncce(nof_cce, c, 64)
                            : srslte_pdcch_ue_locations_ncce(nof_cce, c, 64, sf_idx, rnti);
  for (uint32_t i = 0; i < n; i++) {
    out[2 * i] = c[i].L;
    out[2 * i + 1] = c[i].ncce;
  }
  return (int)n;
}

/* ---------------------------------------------------------------- PDSCH with MIMO ---------- */
/* the grant of a full-band allocation with tb_en / mcs per TB (ra.c's tables), CFI lstart */
static void ref_full_grant(srslte_ra_dl_grant_t *g, uint32_t nof_prb, uint32_t nof_tb, const uint32_t *mcs,
                           uint32_t tb_cw_swap) {
  memset(g, 0, sizeof(*g));
  g->nof_prb = nof_prb;
  for (int s = 0; s < 2; s++)
    for (uint32_t p = 0; p < nof_prb; p++) g->prb_idx[s][p] = true;
  for (uint32_t t = 0; t < nof_tb; t++) {
    g->tb_en[t] = true;
    g->mcs[t].idx = mcs[t];
    g->mcs[t].mod = srslte_ra_mod_from_mcs(mcs[t]);
    g->mcs[t].tbs = srslte_ra_tbs_from_idx(srslte_ra_tbs_idx_from_mcs(mcs[t]), nof_prb);
    g->Qm[t] = srslte_mod_bits_x_symbol(g->mcs[t].mod);
  }
  g->tb_cw_swap = tb_cw_swap != 0;
}

/* srslte_pdsch_encode (pdsch.c:1048-1131) of a full-band grant: mimo_type srslte_mimo_type_t, pmi as
 * srslte_pdsch_cfg_mimo takes it, data per TB; port p's grid (14 x 12 nof_prb cf32) written at
 * grids + p * 2 * SF_LEN_RE floats (REs outside the grant untouched). Returns the RE count or -1. */
int ref_pdsch_encode(uint32_t nof_prb, uint32_t cell_id, uint32_t nof_ports, uint32_t cfi, uint32_t sf_idx,
                     uint16_t rnti, uint32_t mimo_type, uint32_t pmi, uint32_t tb_cw_swap, uint32_t nof_tb,
                     const uint32_t *mcs, const uint32_t *rv, const uint8_t *data0, const uint8_t *data1,
                     float *grids) {
  srslte_cell_t cell;
  memset(&cell, 0, sizeof(cell));
  cell.nof_prb = nof_prb;
  cell.id = cell_id;
  cell.nof_ports = nof_ports;
  cell.cp = SRSLTE_CP_NORM;
  cell.phich_length = SRSLTE_PHICH_NORM;
  cell.phich_resources = SRSLTE_PHICH_R_1;
  srslte_pdsch_t q;
  if (srslte_pdsch_init_enb(&q, nof_prb) || srslte_pdsch_set_cell(&q, cell) || srslte_pdsch_set_rnti(&q, rnti))
    return -1;
  srslte_ra_dl_grant_t g;
  ref_full_grant(&g, nof_prb, nof_tb, mcs, tb_cw_swap);
  srslte_pdsch_cfg_t cfg;
  int rvs[SRSLTE_MAX_CODEWORDS] = {(int)rv[0], nof_tb > 1 ? (int)rv[1] : 0};
  if (srslte_pdsch_cfg_mimo(&cfg, cell, &g, cfi, sf_idx, rvs, (srslte_mimo_type_t)mimo_type, pmi)) return -1;
  srslte_softbuffer_tx_t sb[2], *sbp[SRSLTE_MAX_CODEWORDS] = {&sb[0], &sb[1]};
  for (int t = 0; t < 2; t++)
    if (srslte_softbuffer_tx_init(&sb[t], nof_prb)) return -1;
  uint8_t *data[SRSLTE_MAX_CODEWORDS] = {(uint8_t *)data0, (uint8_t *)data1};
  const uint32_t n = SRSLTE_SF_LEN_RE(nof_prb, SRSLTE_CP_NORM);
  cf_t *sf[SRSLTE_MAX_PORTS] = {NULL};
  for (uint32_t p = 0; p < nof_ports; p++) sf[p] = (cf_t *)grids + (size_t)p * n;
  const int r = srslte_pdsch_encode(&q, &cfg, sbp, data, rnti, sf);
  for (int t = 0; t < 2; t++) srslte_softbuffer_tx_free(&sb[t]);
  srslte_pdsch_free(&q);
  return r ? -1 : (int)cfg.nbits[0].nof_re;
}

/* srslte_pdsch_decode (pdsch.c:868-1007) of the same full-band grant: y [nrx] grids, h [port][rx]
 * estimates (each SF_LEN_RE cf32, y at ys + a n, h at hs + (p nrx + a) n), fresh softbuffers, max 8
 * half-iterations; data per TB (tbs / 8 + 3 bytes), ok[t] (1 acked), noi[t] (last_nof_iterations of the
 * TB's codeword). Returns srslte_pdsch_decode's value. */
int ref_pdsch_decode_mimo(uint32_t nof_prb, uint32_t cell_id, uint32_t nof_ports, uint32_t nrx, uint32_t cfi,
                          uint32_t sf_idx, uint16_t rnti, uint32_t mimo_type, uint32_t pmi, uint32_t tb_cw_swap,
                          uint32_t nof_tb, const uint32_t *mcs, const uint32_t *rv, float noise, const float *ys,
                          const float *hs, uint8_t *data0, uint8_t *data1, int32_t *ok, uint32_t *noi) {
  srslte_cell_t cell;
  memset(&cell, 0, sizeof(cell));
  cell.nof_prb = nof_prb;
  cell.id = cell_id;
  cell.nof_ports = nof_ports;
  cell.cp = SRSLTE_CP_NORM;
  cell.phich_length = SRSLTE_PHICH_NORM;
  cell.phich_resources = SRSLTE_PHICH_R_1;
  srslte_pdsch_t q;
  if (srslte_pdsch_init_ue(&q, nof_prb, nrx) || srslte_pdsch_set_cell(&q, cell) || srslte_pdsch_set_rnti(&q, rnti))
    return -1;
  srslte_pdsch_set_max_noi(&q, 8);
  srslte_ra_dl_grant_t g;
  ref_full_grant(&g, nof_prb, nof_tb, mcs, tb_cw_swap);
  srslte_pdsch_cfg_t cfg;
  int rvs[SRSLTE_MAX_CODEWORDS] = {(int)rv[0], nof_tb > 1 ? (int)rv[1] : 0};
  if (srslte_pdsch_cfg_mimo(&cfg, cell, &g, cfi, sf_idx, rvs, (srslte_mimo_type_t)mimo_type, pmi)) return -1;
  srslte_softbuffer_rx_t sb[2], *sbp[SRSLTE_MAX_CODEWORDS] = {&sb[0], &sb[1]};
  for (int t = 0; t < 2; t++) {
    if (srslte_softbuffer_rx_init(&sb[t], nof_prb)) return -1;
    srslte_softbuffer_rx_reset(&sb[t]);
  }
  const uint32_t n = SRSLTE_SF_LEN_RE(nof_prb, SRSLTE_CP_NORM);
  cf_t *y[SRSLTE_MAX_PORTS] = {NULL}, *h[SRSLTE_MAX_PORTS][SRSLTE_MAX_PORTS] = {{NULL}};
  for (uint32_t a = 0; a < nrx; a++) {
    y[a] = srslte_vec_malloc(sizeof(cf_t) * n);
    memcpy(y[a], ys + 2 * (size_t)a * n, sizeof(cf_t) * n);
    for (uint32_t p = 0; p < nof_ports; p++) {
      h[p][a] = srslte_vec_malloc(sizeof(cf_t) * n);
      memcpy(h[p][a], hs + 2 * (size_t)(p * nrx + a) * n, sizeof(cf_t) * n);
    }
  }
  uint8_t *data[SRSLTE_MAX_CODEWORDS] = {data0, data1};
  bool acks[SRSLTE_MAX_CODEWORDS] = {false, false};
  const int r = srslte_pdsch_decode(&q, &cfg, sbp, y, h, noise, rnti, data, acks);
  for (uint32_t t = 0; t < nof_tb; t++) {
    ok[t] = acks[t];
    noi[t] = srslte_pdsch_last_noi_cw(&q, nof_tb == 2 ? (t ^ (tb_cw_swap ? 1u : 0u)) : 0u);
  }
  for (uint32_t a = 0; a < nrx; a++) {
    free(y[a]);
    for (uint32_t p = 0; p < nof_ports; p++) free(h[p][a]);
  }
  for (int t = 0; t < 2; t++) srslte_softbuffer_rx_free(&sb[t]);
  srslte_pdsch_free(&q);
  return r;
}
