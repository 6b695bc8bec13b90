/*
 * CPU ORACLE — TEST INFRASTRUCTURE ONLY. Plain-C restatement of the srsLTE DL-SCH receive steps
 * around the turbo decoder (paths relative to /root/reference/lib):
 *   - turbo rate matching, 36.212 5.1.4.1 (src/phy/fec/rm_turbo.c): the receive de-interleaving
 *     table (srslte_rm_turbo_gentable_receive :163-228, sub-block variant interleave_table_sb
 *     :231-257), the scatter-add srslte_rm_turbo_rx_lut_ (:394-430) and, for test traffic, the
 *     transmit bit selection (srslte_rm_turbo_tx_lut :323-374);
 *   - transport-block encode / decode (src/phy/phch/sch.c): encode_tb_off (:187-296) and
 *     decode_tb / decode_tb_cb (:307-491) with the softbuffer of src/phy/fec/softbuffer.c.
 * The tables are built forward from the standard (circular buffer w of 3*Kp entries, <NULL>
 * dummies) rather than by the reference's inverse walk; tests/test_dlsch_oracle.py checks both
 * give identical tables and identical decode results against oracle/_ref.
 * Only tests/, __graft_entry__.smoke() and bench.py's CPU baseline may use this code.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "dlsch_oracle.h"
#include "tdec_oracle.h"

/* 36.212 Table 5.1.4-1 (rm_turbo.c:60-61): the 5-bit bit-reversal, an involution */
static const uint8_t PERM[32] = {0, 16, 8, 24, 4, 20, 12, 28, 2, 18, 10, 26, 6, 22, 14, 30,
                                 1, 17, 9, 25, 5, 21, 13, 29, 3, 19, 11, 27, 7, 23, 15, 31};

/* circular buffer w (36.212 5.1.4.1.2): entry = natural decoder-input index 3*k + stream of
 * d^(stream)_k (k < K+4; tails included, rm_turbo.c:213-228), or -1 for <NULL>. */
static int32_t *build_w(uint32_t K, uint32_t *R_out) {
  const uint32_t D = K + 4, R = (D + 31) / 32, Kp = 32 * R, ND = Kp - D;
  int32_t *w = malloc(sizeof(int32_t) * 3 * Kp);
  if (!w) return NULL;
  for (uint32_t k = 0; k < Kp; k++) {
    /* streams 0/1: column k/R of the column-permuted matrix, row k%R */
    const uint32_t y = (k % R) * 32 + PERM[k / R];
    const int32_t d0 = y < ND ? -1 : (int32_t)(3 * (y - ND) + 0);
    const int32_t d1 = y < ND ? -1 : (int32_t)(3 * (y - ND) + 1);
    /* stream 2: pi(k) = (P[k/R] + 32*(k%R) + 1) mod Kp */
    const uint32_t p = (PERM[k / R] + 32 * (k % R) + 1) % Kp;
    const int32_t d2 = p < ND ? -1 : (int32_t)(3 * (p - ND) + 2);
    w[k] = d0;
    w[Kp + 2 * k] = d1;
    w[Kp + 2 * k + 1] = d2;
  }
  *R_out = R;
  return w;
}

/* rm_turbo.c:236-256 inter(x, win) and the +32 stream alignment shared with the decoder */
static uint32_t to_sb(uint32_t idx, uint32_t K, uint32_t nsb) {
  if (idx < 3 * K) {
    const uint32_t x = idx / 3, L = K / nsb;
    return (idx % 3) * (K + 32) + (x % L) * nsb + x / L;
  }
  return idx - 3 * K + 3 * (K + 32);
}

int orc_rm_turbo_rx_table(uint32_t K, uint32_t rv, uint32_t nsb, uint16_t *table) {
  if (orc_cbindex(K) < 0 || orc_cbsize(orc_cbindex(K)) != (int)K || rv > 3) return -1;
  uint32_t R;
  int32_t *w = build_w(K, &R);
  if (!w) return -1;
  const uint32_t Ncb = 96 * R, N = 3 * K + 12;
  const uint32_t k0 = R * (24 * rv + 2); /* R*(2*ceil(Ncb/(8R))*rv + 2), Ncb/(8R) = 12 */
  uint32_t m = 0;
  for (uint32_t j = 0; m < N; j++) {
    const int32_t v = w[(k0 + j) % Ncb];
    if (v >= 0) table[m++] = (uint16_t)(nsb ? to_sb((uint32_t)v, K, nsb) : (uint32_t)v);
  }
  free(w);
  return 0;
}

int orc_rm_turbo_rx(const int16_t *in, int16_t *out, uint32_t in_len, uint32_t K, uint32_t rv,
                    uint32_t nsb) {
  const uint32_t N = 3 * K + 12;
  uint16_t *t = malloc(sizeof(uint16_t) * N);
  if (!t || orc_rm_turbo_rx_table(K, rv, nsb, t)) {
    free(t);
    return -1;
  }
  for (uint32_t i = 0; i < in_len; i++) {
    const uint32_t o = t[i % N];
    out[o] = (int16_t)(uint16_t)((uint32_t)(uint16_t)out[o] + (uint32_t)(uint16_t)in[i]);
  }
  free(t);
  return 0;
}

int orc_rm_turbo_tx(const uint8_t *coded, uint32_t K, uint32_t rv, uint8_t *e, uint32_t E) {
  uint32_t R;
  int32_t *w = build_w(K, &R);
  if (!w) return -1;
  const uint32_t Ncb = 96 * R, k0 = R * (24 * rv + 2);
  uint32_t m = 0;
  for (uint32_t j = 0; m < E; j++) {
    const int32_t v = w[(k0 + j) % Ncb];
    if (v >= 0) e[m++] = coded[v];
  }
  free(w);
  return 0;
}

static int get_bit(const uint8_t *bytes, uint32_t i) { return (bytes[i / 8] >> (7 - i % 8)) & 1; }

/* 24-bit CRC of a bit array (one bit per byte), same register as crc.c:144-155 */
static uint32_t crc_bits(uint32_t poly, const uint8_t *bits, uint32_t n) {
  uint32_t crc = 0;
  for (uint32_t i = 0; i < n; i++) {
    const uint32_t fb = ((crc >> 23) & 1) ^ bits[i];
    crc = (crc << 1) & 0xFFFFFF;
    if (fb) crc ^= poly & 0xFFFFFF;
  }
  return crc;
}

/* per-CB lengths of sch.c, receive side (decode_tb_cb :325-341): K1 blocks first */
static void rx_cb_params(const orc_cbsegm_t *s, uint32_t Qm, uint32_t nof_e_bits, uint32_t i,
                         uint32_t *K, uint32_t *rlen, uint32_t *rp, uint32_t *ne) {
  *K = i < s->C1 ? s->K1 : s->K2;
  *rlen = s->C == 1 ? *K : *K - 24;
  const uint32_t Gp = nof_e_bits / Qm;
  const uint32_t gamma = s->C > 0 ? Gp % s->C : Gp;
  const uint32_t n_e = Qm * (Gp / s->C);
  *rp = i * n_e;
  *ne = n_e;
  if (i > s->C - gamma) { /* sch.c:339: strictly greater (the encoder uses >=, :232) */
    *ne = n_e + Qm;
    *rp = (s->C - gamma) * n_e + (i - (s->C - gamma)) * *ne;
  }
}

int orc_segm(uint32_t tbs, orc_cbsegm_t *s) {
  memset(s, 0, sizeof(*s));
  s->tbs = tbs;
  if (tbs == 0) return 0;
  uint32_t F;
  if (orc_cbsegm(tbs, &s->C, &s->C1, &s->K1, &s->C2, &s->K2, &F)) return -1;
  s->F = F;
  return 0;
}

/* encode_tb_off (sch.c:187-296) + srslte_tcod_encode_lut's CRC placement: K2 blocks first,
 * TB CRC24A on the last CB, CB CRC24B when C > 1; e_bits unpacked (one bit per byte). */
int orc_dlsch_encode(uint32_t tbs, uint32_t rv, uint32_t Qm, uint32_t nof_e_bits,
                     const uint8_t *data, uint8_t *e_bits) {
  orc_cbsegm_t s;
  if (orc_segm(tbs, &s) || s.F || s.C == 0) return -1;
  uint8_t *a = malloc(tbs + 24);
  uint8_t *cb = malloc(6144 + 24);
  uint8_t *coded = malloc(3 * 6144 + 12);
  if (!a || !cb || !coded) return -1;
  for (uint32_t i = 0; i < tbs; i++) a[i] = (uint8_t)get_bit(data, i);
  const uint32_t tcrc = crc_bits(ORC_CRC24A, a, tbs);
  for (int b = 0; b < 24; b++) a[tbs + b] = (tcrc >> (23 - b)) & 1;
  const uint32_t Gp = nof_e_bits / Qm;
  const uint32_t gamma = Gp % s.C;
  uint32_t rp = 0, wp = 0;
  for (uint32_t i = 0; i < s.C; i++) {
    const uint32_t K = i < s.C2 ? s.K2 : s.K1;
    const uint32_t rlen = s.C > 1 ? K - 24 : K;
    const uint32_t n_e = i <= s.C - gamma - 1 ? Qm * (Gp / s.C) : Qm * ((Gp + s.C - 1) / s.C);
    memcpy(cb, a + rp, rlen);
    if (s.C > 1) {
      const uint32_t c = crc_bits(ORC_CRC24B, cb, rlen);
      for (int b = 0; b < 24; b++) cb[rlen + b] = (c >> (23 - b)) & 1;
    }
    orc_tcod_encode(cb, coded, K);
    orc_rm_turbo_tx(coded, K, rv, e_bits + wp, n_e);
    rp += rlen;
    wp += n_e;
  }
  free(a);
  free(cb);
  free(coded);
  return 0;
}

int orc_softbuffer_init(orc_softbuffer_t *q, uint32_t max_cb) {
  memset(q, 0, sizeof(*q));
  q->max_cb = max_cb;
  q->buffer = calloc((size_t)max_cb * ORC_SOFTBUFFER_SIZE, sizeof(int16_t));
  q->data = calloc((size_t)max_cb * 768, 1);
  q->cb_crc = calloc(max_cb, 1);
  return q->buffer && q->data && q->cb_crc ? 0 : -1;
}

void orc_softbuffer_reset(orc_softbuffer_t *q) { /* softbuffer.c:125-150 */
  memset(q->buffer, 0, (size_t)q->max_cb * ORC_SOFTBUFFER_SIZE * sizeof(int16_t));
  memset(q->cb_crc, 0, q->max_cb);
}

void orc_softbuffer_free(orc_softbuffer_t *q) {
  free(q->buffer);
  free(q->data);
  free(q->cb_crc);
  memset(q, 0, sizeof(*q));
}

/* decode_tb (sch.c:434-491) + decode_tb_cb (:307-421), AUTO decoder on the SB layout.
 * data needs room for the last CB's full K/8 bytes: tbs/8 + 3 (+ 3 when C > 1). */
int orc_dlsch_decode(orc_softbuffer_t *q, uint32_t tbs, uint32_t rv, uint32_t Qm,
                     uint32_t nof_e_bits, const int16_t *e_bits, uint8_t *data,
                     uint32_t max_halfits, uint32_t *nof_iterations) {
  orc_cbsegm_t s;
  if (orc_segm(tbs, &s)) return -1;
  if (s.tbs == 0 || s.C == 0) return 0;
  if (s.F) return -2;                   /* SRSLTE_ERROR_INVALID_INPUTS */
  if (s.C > q->max_cb) return -2;
  data[tbs / 8 + 0] = data[tbs / 8 + 1] = data[tbs / 8 + 2] = 0;
  uint32_t iters = 0;
  for (uint32_t i = 0; i < s.C; i++) {
    uint32_t K, rlen, rp, ne;
    rx_cb_params(&s, Qm, nof_e_bits, i, &K, &rlen, &rp, &ne);
    if (!q->cb_crc[i]) {
      int16_t *sb = q->buffer + (size_t)i * ORC_SOFTBUFFER_SIZE;
      if (orc_rm_turbo_rx(e_bits + rp, sb, ne, K, rv, orc_autoimp_subblocks(K))) return -1;
      const uint32_t poly = s.C > 1 ? ORC_CRC24B : ORC_CRC24A;
      const uint32_t len = s.C > 1 ? K : tbs + 24;
      uint32_t noi = 0;
      const int ok = orc_tdec_decode_cb(ORC_TDEC_AUTO, 1, sb, K, max_halfits, poly, len,
                                        data + i * rlen / 8, &noi);
      if (ok < 0) return -1;
      if (ok) q->cb_crc[i] = 1;
      iters += noi;
    } else {
      memcpy(data + i * rlen / 8, q->data + (size_t)i * 768, rlen / 8);
    }
  }
  q->tb_crc = 1;
  for (uint32_t i = 0; i < s.C && q->tb_crc; i++) q->tb_crc = q->cb_crc[i];
  if (!q->tb_crc) {
    for (uint32_t i = 0; i < s.C; i++) {
      uint32_t K, rlen, rp, ne;
      rx_cb_params(&s, Qm, nof_e_bits, i, &K, &rlen, &rp, &ne);
      if (q->cb_crc[i]) memcpy(q->data + (size_t)i * 768, data + i * rlen / 8, rlen / 8);
    }
  }
  *nof_iterations = iters / s.C;
  if (!q->tb_crc) return -1;
  const uint32_t par_rx = orc_crc_checksum_byte(ORC_CRC24A, 24, data, tbs);
  const uint32_t par_tx = ((uint32_t)data[tbs / 8] << 16) | ((uint32_t)data[tbs / 8 + 1] << 8) |
                          data[tbs / 8 + 2];
  return (par_rx == par_tx && par_rx) ? 0 : -1;
}

/* srslte_rm_turbo_rx_lut_8bit (rm_turbo.c:432-469 -> srslte_rm_turbo_rx_lut_sse_8bit :543-):
 * out[deinter[i % N]] += in[i] in int8 (wrapping; the order of the adds does not matter modulo
 * 256), with the sub-block table of the 8-bit decoder (srslte_tdec_autoimp_get_subblocks_8bit) */
int orc_rm_turbo_rx_8bit(const int8_t *in, int8_t *out, uint32_t in_len, uint32_t K, uint32_t rv) {
  const uint32_t N = 3 * K + 12;
  uint16_t *t = malloc(sizeof(uint16_t) * N);
  if (!t || orc_rm_turbo_rx_table(K, rv, orc_autoimp_subblocks_8bit(K), t)) {
    free(t);
    return -1;
  }
  for (uint32_t i = 0; i < in_len; i++) {
    const uint32_t o = t[i % N];
    out[o] = (int8_t)(uint8_t)((uint32_t)(uint8_t)out[o] + (uint32_t)(uint8_t)in[i]);
  }
  free(t);
  return 0;
}

/* decode_tb_cb with llr_is_8bit (sch.c:344-364): the softbuffer row holds int8 values
 * ((int8_t *) buffer_f) and srslte_tdec_iteration_8bit decodes it; early stop on the CB / TB CRC
 * after every half-iteration. The 8-bit AUTO choice at 400 < K <= 800 (8 sub-blocks) feeds the
 * SSE16 window 3K+12 converted values of a 3(K+32)+12 sub-block row, the remaining inputs being
 * whatever the decoder's conversion buffer last held (turbodecoder.c:439-459): no defined result,
 * so such a TB is refused (-2, as the GPU path). */
int orc_dlsch_decode8(orc_softbuffer_t *q, uint32_t tbs, uint32_t rv, uint32_t Qm,
                      uint32_t nof_e_bits, const int8_t *e_bits, uint8_t *data,
                      uint32_t max_halfits, uint32_t *nof_iterations) {
  orc_cbsegm_t s;
  if (orc_segm(tbs, &s)) return -1;
  if (s.tbs == 0 || s.C == 0) return 0;
  if (s.F) return -2;
  if (s.C > q->max_cb) return -2;
  for (uint32_t i = 0; i < s.C; i++) {
    const uint32_t K = i < s.C1 ? s.K1 : s.K2;
    if (orc_autoimp_subblocks_8bit(K) == 8) return -2;
  }
  data[tbs / 8 + 0] = data[tbs / 8 + 1] = data[tbs / 8 + 2] = 0;
  uint32_t iters = 0;
  uint8_t *dec = malloc((size_t)max_halfits * (6144 / 8) + 64);
  if (!dec) return -1;
  for (uint32_t i = 0; i < s.C; i++) {
    uint32_t K, rlen, rp, ne;
    rx_cb_params(&s, Qm, nof_e_bits, i, &K, &rlen, &rp, &ne);
    if (!q->cb_crc[i]) {
      int8_t *sb = (int8_t *)(q->buffer + (size_t)i * ORC_SOFTBUFFER_SIZE);
      if (orc_rm_turbo_rx_8bit(e_bits + rp, sb, ne, K, rv)) return -1;
      const uint32_t poly = s.C > 1 ? ORC_CRC24B : ORC_CRC24A;
      const uint32_t len = s.C > 1 ? K : tbs + 24;
      uint8_t *out = data + i * rlen / 8;
      /* decisions (packed bytes) after every half-iteration; the CRC decides where it stops */
      if (orc_tdec8_run(ORC_TDEC_AUTO, 1, sb, K, max_halfits, dec) < 0) return -1;
      uint32_t noi = 0;
      int ok = 0;
      while (noi < max_halfits && !ok) {
        memcpy(out, dec + (size_t)noi * (K / 8), K / 8);
        noi++;
        ok = orc_crc_checksum_byte(poly, 24, out, len) == 0;
      }
      if (ok) q->cb_crc[i] = 1;
      iters += noi;
    } else {
      memcpy(data + i * rlen / 8, q->data + (size_t)i * 768, rlen / 8);
    }
  }
  free(dec);
  q->tb_crc = 1;
  for (uint32_t i = 0; i < s.C && q->tb_crc; i++) q->tb_crc = q->cb_crc[i];
  if (!q->tb_crc) {
    for (uint32_t i = 0; i < s.C; i++) {
      uint32_t K, rlen, rp, ne;
      rx_cb_params(&s, Qm, nof_e_bits, i, &K, &rlen, &rp, &ne);
      if (q->cb_crc[i]) memcpy(q->data + (size_t)i * 768, data + i * rlen / 8, rlen / 8);
    }
  }
  *nof_iterations = iters / s.C;
  if (!q->tb_crc) return -1;
  const uint32_t par_rx = orc_crc_checksum_byte(ORC_CRC24A, 24, data, tbs);
  const uint32_t par_tx = ((uint32_t)data[tbs / 8] << 16) | ((uint32_t)data[tbs / 8 + 1] << 8) |
                          data[tbs / 8 + 2];
  return (par_rx == par_tx && par_rx) ? 0 : -1;
}

/* ---------------------------------------------------------------- UL-SCH ---------------------- */
/* ulsch_deinterleave (sch.c:860-881) with no RI bits: ulsch_interleave_gen (:550-568) numbers the
 * (row j, column i, bit k) entries of a rows x cols matrix of Qm-bit entries row by row and places
 * entry (j, i, k) at q index j Qm + i rows Qm + k; srslte_vec_lut_sis then sets g[lut[x]] = q[x].
 * rows = H' / cols with H' = nof_bits / Qm. -1 when nof_bits is not a whole matrix. */
int orc_ulsch_deinterleave(const int16_t *q_bits, uint32_t Qm, uint32_t nof_bits, uint32_t nof_symb,
                           int16_t *g_bits) {
  if (Qm == 0 || nof_symb == 0 || nof_bits % (Qm * nof_symb)) return -1;
  const uint32_t rows = nof_bits / Qm / nof_symb, cols = nof_symb;
  uint32_t idx = 0;
  for (uint32_t j = 0; j < rows; j++)
    for (uint32_t i = 0; i < cols; i++)
      for (uint32_t k = 0; k < Qm; k++) g_bits[idx++] = q_bits[j * Qm + i * rows * Qm + k];
  return 0;
}

/* srslte_ulsch_decode -> srslte_ulsch_uci_decode with uci_data = {0}: Q'_ri = Q'_cqi = 0, so
 * G Qm = nof_bits and decode_tb runs on the whole deinterleaved g (sch.c:956-983) */
int orc_ulsch_decode(orc_softbuffer_t *q, uint32_t tbs, uint32_t rv, uint32_t Qm, uint32_t nof_bits,
                     uint32_t nof_symb, const int16_t *q_bits, uint8_t *data, uint32_t max_halfits,
                     uint32_t *nof_iterations) {
  int16_t *g = malloc((size_t)(nof_bits + 1) * sizeof(int16_t));
  if (!g) return -1;
  int r = orc_ulsch_deinterleave(q_bits, Qm, nof_bits, nof_symb, g);
  if (!r) r = orc_dlsch_decode(q, tbs, rv, Qm, nof_bits, g, data, max_halfits, nof_iterations);
  free(g);
  return r;
}
