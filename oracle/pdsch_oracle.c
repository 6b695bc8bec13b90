/*
 * CPU ORACLE — TEST INFRASTRUCTURE ONLY. Plain-C restatement of the srsLTE PDSCH receive steps
 * between the channel estimate and the DL-SCH decoder (paths relative to /root/reference/lib):
 *   - RE extraction srslte_pdsch_get / srslte_pdsch_cp (src/phy/phch/pdsch.c:95-234) with the
 *     PRB copy helpers of src/phy/phch/prb_dl.c:51-97, returned as a gather index list;
 *   - SISO ZF/MMSE equalisation srslte_predecoding_single_multi (src/phy/mimo/precoding.c:
 *     243-352), plain and with CSI;
 *   - soft demapping srslte_demod_soft_demodulate_s (src/phy/modem/demod_soft.c:52-456): the
 *     SSE/AVX2 integer paths (round-to-nearest conversion, saturating pack, integer offsets) for
 *     whole SIMD blocks and the scalar C tail for the rest, exactly as the reference splits them;
 *   - the PDSCH scrambling sequence (src/phy/common/sequence.c:51-80, phch/sequences.c:64-66)
 *     and srslte_scrambling_s_offset (src/phy/scrambling/scrambling.c:48-51).
 * Only tests/, __graft_entry__.smoke() and bench.py's CPU baseline may use this code.
 */
#include <limits.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "dlsch_oracle.h"
#include "pdsch_oracle.h"

/* ---------------------------------------------------------------- RE extraction ---------- */
/* prb_dl.c:51-82 prb_cp_ref in read mode: skips one input RE before each interval */
static void cp_ref(uint32_t *in, uint32_t **out, int offset, int nof_refs, int nof_intervals) {
  const int ri = 12 / nof_refs - 1;
  for (int j = 0; j < offset; j++) *(*out)++ = (*in)++;
  for (int i = 0; i < nof_intervals - 1; i++) {
    (*in)++;
    for (int j = 0; j < ri; j++) *(*out)++ = (*in)++;
  }
  if (ri - offset > 0) {
    (*in)++;
    for (int j = 0; j < ri - offset; j++) *(*out)++ = (*in)++;
  }
}

static int has_ref(uint32_t l, uint32_t nof_ports, uint32_t nsymb) { /* SRSLTE_SYMBOL_HAS_REF, phy_common.h:132-134 */
  return (l == 1 && nof_ports == 4) || l == 0 || l == nsymb - 3;
}

/* nof_ports: the CRS port count, plus 256 for an extended-CP cell (SRSLTE_CP_NSYMB 6) */
int orc_pdsch_re_map(uint32_t nof_prb, uint32_t cell_id, uint32_t nof_ports, uint32_t lstart_grant,
                     uint32_t sf_idx, const uint8_t *prb_mask, uint32_t *idx) {
  const uint32_t nsymb = (nof_ports >> 8) & 1 ? 6 : 7;
  nof_ports &= 0xff;
  const uint32_t nof_refs = nof_ports == 1 ? 2 : 4;
  uint32_t *out = idx;
  uint32_t offset = 0;
  for (uint32_t s = 0; s < 2; s++) {
    for (uint32_t l = 0; l < nsymb; l++) {
      for (uint32_t n = 0; n < nof_prb; n++) {
        if (!prb_mask[s * nof_prb + n]) continue;
        uint32_t lstart = s == 0 ? lstart_grant : 0, lend = nsymb;
        int is_pbch = 0, is_sss = 0;
        const int centre = n >= nof_prb / 2 - 3 && n < nof_prb / 2 + 3 + (nof_prb % 2);
        if (s == 0 && (sf_idx == 0 || sf_idx == 5) && centre) {
          lend = nsymb - 2;
          is_sss = 1;
        }
        if (s == 1 && sf_idx == 0 && centre) {
          lstart = 4;
          is_pbch = 1;
        }
        const uint32_t lp = l + s * nsymb;
        uint32_t in = (lp * nof_prb + n) * 12;
        if (l >= lstart && l < lend) {
          if (has_ref(l, nof_ports, nsymb)) {
            offset = nof_refs == 2 ? (l == 0 ? cell_id % 6 : (cell_id + 3) % 6) : cell_id % 3;
            cp_ref(&in, &out, (int)offset, (int)nof_refs, (int)nof_refs);
          } else {
            for (int j = 0; j < 12; j++) *out++ = in++;
          }
        }
        if ((nof_prb % 2) && ((is_pbch && l < lstart) || (is_sss && l >= lend))) {
          if (n == nof_prb / 2 - 3) {
            if (has_ref(l, nof_ports, nsymb))
              cp_ref(&in, &out, (int)offset, (int)nof_refs, (int)nof_refs / 2);
            else
              for (int j = 0; j < 6; j++) *out++ = in++;
          } else if (n == nof_prb / 2 + 3) {
            in += 6;
            if (has_ref(l, nof_ports, nsymb))
              cp_ref(&in, &out, (int)offset, (int)nof_refs, (int)nof_refs / 2);
            else
              for (int j = 0; j < 6; j++) *out++ = in++;
          }
        }
      }
    }
  }
  return (int)(out - idx);
}

/* ---------------------------------------------------------------- equalisation ---------- */
void orc_predecode_single(const float *y, const float *h, float *x, float *csi, int n,
                          float scaling, float noise) {
  /* float operations in the order of srslte_predecoding_single_avx (:154-230): |h|^2 = hr*hr +
   * hi*hi, y*conj(h) via the addsub product, divide, then times 1/scaling; symbols past the last
   * whole 16 use the C path r / ((hh + n0) * scaling) (:231-240) whose conj() is the double
   * one. CSI mode (:256-296) uses an exact reciprocal where the reference's rcpps is
   * approximate (tests compare it with a tolerance). */
  const float inv = 1.0f / scaling;
  const int simd = n > 32 ? 16 * (n / 16) : 0; /* :330-338: the AVX kernel only above 32 */
  for (int i = 0; i < n; i++) {
    const float yr = y[2 * i], yi = y[2 * i + 1], hr = h[2 * i], hi = h[2 * i + 1];
    const float p1 = hr * hr, p2 = hi * hi;
    const float hh = p1 + p2;
    const float a1 = yr * hr, a2 = yi * -hi, b1 = yi * hr, b2 = yr * -hi;
    const float rr = a1 - a2, ri = b1 + b2;
    if (csi) {
      const float c = hh + noise;
      csi[i] = c;
      const float r = 1.0f / c;
      x[2 * i] = rr * inv * r;
      x[2 * i + 1] = ri * inv * r;
    } else if (i < simd) {
      const float d = noise > 0 ? hh + noise : hh;
      x[2 * i] = rr / d * inv;
      x[2 * i + 1] = ri / d * inv;
    } else {
      /* the C tail multiplies by conj() of double complex: products and sums in double, then
       * rounded to the float accumulators */
      const float hd = (float)((double)hr * hr + (double)hi * hi);
      const float rd = (float)((double)yr * hr - (double)yi * -(double)hi);
      const float id = (float)((double)yr * -(double)hi + (double)yi * hr);
      const float d = (hd + noise) * scaling;
      x[2 * i] = rd / d;
      x[2 * i + 1] = id / d;
    }
  }
}

/* ---------------------------------------------------------------- TM3: CDD 2x2 MMSE ---------- */
/* complex float arithmetic in the order gcc evaluates the reference's cf_t expressions (ISO C,
 * no contraction): (a+bi)(c+di) = (ac - bd) + (ad + bc)i */
typedef struct {
  float r, i;
} orc_cf;
static orc_cf cf_mul(orc_cf a, orc_cf b) { return (orc_cf){a.r * b.r - a.i * b.i, a.r * b.i + a.i * b.r}; }
static orc_cf cf_add(orc_cf a, orc_cf b) { return (orc_cf){a.r + b.r, a.i + b.i}; }
static orc_cf cf_sub(orc_cf a, orc_cf b) { return (orc_cf){a.r - b.r, a.i - b.i}; }
static orc_cf cf_conj(orc_cf a) { return (orc_cf){a.r, -a.i}; }
static orc_cf cf_neg(orc_cf a) { return (orc_cf){-a.r, -a.i}; }

/* srslte_mat_2x2_mmse_csi_gen (utils/mat.c:63-98) */
static void mmse_csi_gen(orc_cf y0, orc_cf y1, orc_cf h00, orc_cf h01, orc_cf h10, orc_cf h11,
                         orc_cf *x0, orc_cf *x1, float *csi0, float *csi1, float noise, float norm) {
  const orc_cf _h00 = cf_conj(h00), _h01 = cf_conj(h01), _h10 = cf_conj(h10), _h11 = cf_conj(h11);
  orc_cf a00 = cf_add(cf_mul(_h00, h00), cf_mul(_h10, h10));
  a00.r = a00.r + noise;
  const orc_cf a01 = cf_add(cf_mul(_h00, h01), cf_mul(_h10, h11));
  const orc_cf a10 = cf_add(cf_mul(_h01, h00), cf_mul(_h11, h10));
  orc_cf a11 = cf_add(cf_mul(_h01, h01), cf_mul(_h11, h11));
  a11.r = a11.r + noise;
  /* srslte_mat_cf_recip_gen(srslte_mat_2x2_det_gen(...)) (mat.c:35-42): conj(a) / |a|^2 */
  const orc_cf det = cf_sub(cf_mul(a00, a11), cf_mul(a01, a10));
  const float m2 = det.r * det.r + det.i * det.i;
  const orc_cf rcp = {det.r / m2, -det.i / m2};
  const orc_cf nrm = {norm * rcp.r, norm * rcp.i};
  const orc_cf b00 = cf_mul(a11, nrm), b01 = cf_mul(cf_neg(a01), nrm);
  const orc_cf b10 = cf_mul(cf_neg(a10), nrm), b11 = cf_mul(a00, nrm);
  const orc_cf w00 = cf_add(cf_mul(b00, _h00), cf_mul(b01, _h01));
  const orc_cf w01 = cf_add(cf_mul(b00, _h10), cf_mul(b01, _h11));
  const orc_cf w10 = cf_add(cf_mul(b10, _h00), cf_mul(b11, _h01));
  const orc_cf w11 = cf_add(cf_mul(b10, _h10), cf_mul(b11, _h11));
  *x0 = cf_add(cf_mul(y0, w00), cf_mul(y1, w01));
  *x1 = cf_add(cf_mul(y0, w10), cf_mul(y1, w11));
  *csi0 = 1.0f / b00.r;
  *csi1 = 1.0f / b11.r;
}

void orc_predecode_ccd_2x2(const float *y0, const float *y1, const float *h00, const float *h01,
                           const float *h10, const float *h11, float *x0, float *x1, float *csi0,
                           float *csi1, int n, float scaling, float noise) {
  /* srslte_predecoding_ccd_2x2_mmse(_csi) (mimo/precoding.c:930-1019, 1021-1072): h[port][rx]
   * (h01 = port 0 / rx 1, h10 = port 1 / rx 0), CDD precoder alternating per RE: even RE
   * H = [[h00 + h10, h00 - h10], [h01 + h11, h01 - h11]], odd RE the columns swap. Restated as
   * the reference's C loop (the exact tail); its AVX body uses rcpps, so the reference's first
   * 8*(n/8) REs agree with this only to the rcpps tolerance. */
  const float norm = 2.0f / scaling;
  for (int i = 0; i < n; i++) {
    const orc_cf p00 = {h00[2 * i], h00[2 * i + 1]}, p01 = {h01[2 * i], h01[2 * i + 1]};
    const orc_cf p10 = {h10[2 * i], h10[2 * i + 1]}, p11 = {h11[2 * i], h11[2 * i + 1]};
    orc_cf g00, g01, g10, g11;
    if (i % 2 == 0) {
      g00 = cf_add(p00, p10);
      g10 = cf_add(p01, p11);
      g01 = cf_sub(p00, p10);
      g11 = cf_sub(p01, p11);
    } else {
      g00 = cf_sub(p00, p10);
      g10 = cf_sub(p01, p11);
      g01 = cf_add(p00, p10);
      g11 = cf_add(p01, p11);
    }
    orc_cf a, b;
    float c0, c1;
    mmse_csi_gen((orc_cf){y0[2 * i], y0[2 * i + 1]}, (orc_cf){y1[2 * i], y1[2 * i + 1]}, g00, g01,
                 g10, g11, &a, &b, &c0, &c1, noise, norm);
    x0[2 * i] = a.r;
    x0[2 * i + 1] = a.i;
    x1[2 * i] = b.r;
    x1[2 * i + 1] = b.i;
    if (csi0) csi0[i] = c0;
    if (csi1) csi1[i] = c1;
  }
}

/* ---------------------------------------------------------------- TM4: spatial multiplexing ---- */
static orc_cf cf_mulj(orc_cf a) { return (orc_cf){-a.i, a.r}; } /* _Complex_I * a, exact */

/* srslte_predecoding_multiplex (mimo/precoding.c:1715-1760), 2 ports, 2 rx antennas, restated as
 * the reference's C loops (the exact tails; the AVX bodies use rcpps):
 *  - 2 layers: srslte_predecoding_multiplex_2x2_mmse(_csi) (:1331-1542): the codebook's precoder
 *    (0: [[h00, h10], [h01, h11]], 1: [[h00+h10, h00-h10], [h01+h11, h01-h11]], 2: with j h10 /
 *    j h11) into srslte_mat_2x2_mmse_csi_gen, norm (float) M_SQRT2 / scaling for codebook 0 else
 *    2 / scaling; h[port][rx] with h01 = port 0 / rx 1;
 *  - 1 layer: srslte_predecoding_multiplex_2x1_mrc(_csi) (:1546-1713): h0 / h1 the codebook's
 *    port combination at rx 0 / 1, hh = norm / (|h0|^2 + |h1|^2), x = (conj(h0) y0 + conj(h1) y1) hh,
 *    csi = (|h0|^2 + |h1|^2) / norm * (float) M_SQRT1_2.
 * Returns -1 on a codebook the reference refuses. */
int orc_predecode_multiplex(const float *y0, const float *y1, const float *h00, const float *h01,
                            const float *h10, const float *h11, float *x0, float *x1, float *csi0,
                            float *csi1, int n, float scaling, float noise, int codebook_idx,
                            int nof_layers) {
  if (codebook_idx < 0 || codebook_idx > (nof_layers == 2 ? 2 : 3)) return -1;
  for (int i = 0; i < n; i++) {
    const orc_cf p00 = {h00[2 * i], h00[2 * i + 1]}, p01 = {h01[2 * i], h01[2 * i + 1]};
    const orc_cf p10 = {h10[2 * i], h10[2 * i + 1]}, p11 = {h11[2 * i], h11[2 * i + 1]};
    const orc_cf ya = {y0[2 * i], y0[2 * i + 1]}, yb = {y1[2 * i], y1[2 * i + 1]};
    if (nof_layers == 2) {
      orc_cf g00, g01, g10, g11;
      float norm = 2.0f / scaling;
      if (codebook_idx == 0) {
        g00 = p00, g01 = p10, g10 = p01, g11 = p11;
        norm = 1.41421354f / scaling; /* (float) M_SQRT2 */
      } else if (codebook_idx == 1) {
        g00 = cf_add(p00, p10), g01 = cf_sub(p00, p10), g10 = cf_add(p01, p11), g11 = cf_sub(p01, p11);
      } else {
        g00 = cf_add(p00, cf_mulj(p10)), g01 = cf_sub(p00, cf_mulj(p10));
        g10 = cf_add(p01, cf_mulj(p11)), g11 = cf_sub(p01, cf_mulj(p11));
      }
      orc_cf a, b;
      float c0, c1;
      mmse_csi_gen(ya, yb, g00, g01, g10, g11, &a, &b, &c0, &c1, noise, norm);
      x0[2 * i] = a.r, x0[2 * i + 1] = a.i;
      x1[2 * i] = b.r, x1[2 * i + 1] = b.i;
      if (csi0) csi0[i] = c0;
      if (csi1) csi1[i] = c1;
    } else {
      orc_cf g0, g1;
      switch (codebook_idx) {
      case 0: g0 = cf_add(p00, p10), g1 = cf_add(p01, p11); break;
      case 1: g0 = cf_sub(p00, p10), g1 = cf_sub(p01, p11); break;
      case 2: g0 = cf_add(p00, cf_mulj(p10)), g1 = cf_add(p01, cf_mulj(p11)); break;
      default: g0 = cf_sub(p00, cf_mulj(p10)), g1 = cf_sub(p01, cf_mulj(p11)); break;
      }
      const float norm = 1.41421354f / scaling; /* (float) M_SQRT2 */
      const float s = g0.r * g0.r + g0.i * g0.i + g1.r * g1.r + g1.i * g1.i;
      const float hh = norm / s;
      const orc_cf x = cf_add(cf_mul(cf_conj(g0), ya), cf_mul(cf_conj(g1), yb));
      x0[2 * i] = x.r * hh, x0[2 * i + 1] = x.i * hh;
      if (csi0) csi0[i] = s / norm * 0.707106769f; /* (float) M_SQRT1_2 */
    }
  }
  return 0;
}

/* ---------------------------------------------------------------- soft demapping ---------- */
static int16_t sat16(int64_t v) { return (int16_t)(v > 32767 ? 32767 : v < -32768 ? -32768 : v); }
static int16_t wrap16(int32_t v) { return (int16_t)(uint16_t)(uint32_t)v; }

/* cvtps_epi32 (round to nearest even, MXCSR default) / cvttps_epi32 (truncate): out-of-range
 * and NaN give the "integer indefinite" 0x80000000 */
static int32_t cvt_rn(float v) {
  if (!(v >= -2147483648.0f && v < 2147483648.0f)) return INT32_MIN;
  return (int32_t)rintf(v);
}
static int32_t cvt_rz(float v) {
  if (!(v >= -2147483648.0f && v < 2147483648.0f)) return INT32_MIN;
  return (int32_t)v;
}
static int16_t abs16(int16_t v) { return wrap16(v < 0 ? -(int32_t)v : v); } /* _mm_abs_epi16 */

int orc_demod_s(int mod, const float *sym, int nsym, int16_t *llr) {
  switch (mod) {
  case 0: /* BPSK demod_bpsk_lte_s :56-60 */
    for (int i = 0; i < nsym; i++)
      llr[i] = (int16_t)(int32_t)(-100 * (sym[2 * i] + sym[2 * i + 1]) / sqrt(2));
    return 0;
  case 1: { /* QPSK: srslte_vec_convert_fi(x, -100*sqrt(2)) (vector_simd.c:394-429) */
    const float scale = (float)(-100 * sqrt(2));
    const int len = 2 * nsym, simd = 16 * (len / 16);
    for (int i = 0; i < simd; i++) llr[i] = sat16(cvt_rz(sym[i] * scale));
    for (int i = simd; i < len; i++) llr[i] = wrap16(cvt_rz(sym[i] * scale));
    return 0;
  }
  case 2: { /* 16QAM demod_16qam_lte_s_sse :96-155 */
    const int16_t off = (int16_t)(2 * 400 / sqrt(10));
    const int simd = 4 * (nsym / 4);
    for (int i = 0; i < simd; i++) {
      const int16_t re = sat16(cvt_rn(sym[2 * i] * -400.0f));
      const int16_t im = sat16(cvt_rn(sym[2 * i + 1] * -400.0f));
      llr[4 * i + 0] = re;
      llr[4 * i + 1] = im;
      llr[4 * i + 2] = wrap16(abs16(re) - off);
      llr[4 * i + 3] = wrap16(abs16(im) - off);
    }
    for (int i = simd; i < nsym; i++) {
      const int16_t yre = (int16_t)(int32_t)(400 * sym[2 * i]);
      const int16_t yim = (int16_t)(int32_t)(400 * sym[2 * i + 1]);
      llr[4 * i + 0] = (int16_t)-yre;
      llr[4 * i + 1] = (int16_t)-yim;
      llr[4 * i + 2] = (int16_t)(int32_t)(abs(yre) - 2 * 400 / sqrt(10));
      llr[4 * i + 3] = (int16_t)(int32_t)(abs(yim) - 2 * 400 / sqrt(10));
    }
    return 0;
  }
  case 3: { /* 64QAM demod_64qam_lte_s_sse :242-304 */
    const int16_t off1 = (int16_t)(4 * 700 / sqrt(42)), off2 = (int16_t)(2 * 700 / sqrt(42));
    const int simd = 4 * (nsym / 4);
    for (int i = 0; i < simd; i++) {
      const int16_t re = sat16(cvt_rn(sym[2 * i] * -700.0f));
      const int16_t im = sat16(cvt_rn(sym[2 * i + 1] * -700.0f));
      const int16_t a1r = wrap16(abs16(re) - off1), a1i = wrap16(abs16(im) - off1);
      llr[6 * i + 0] = re;
      llr[6 * i + 1] = im;
      llr[6 * i + 2] = a1r;
      llr[6 * i + 3] = a1i;
      llr[6 * i + 4] = wrap16(abs16(a1r) - off2);
      llr[6 * i + 5] = wrap16(abs16(a1i) - off2);
    }
    for (int i = simd; i < nsym; i++) {
      const float yre = (int16_t)(int32_t)(700 * sym[2 * i]);
      const float yim = (int16_t)(int32_t)(700 * sym[2 * i + 1]);
      llr[6 * i + 0] = (int16_t)(int32_t)-yre;
      llr[6 * i + 1] = (int16_t)(int32_t)-yim;
      llr[6 * i + 2] = (int16_t)(int32_t)(abs((int)yre) - 4 * 700 / sqrt(42));
      llr[6 * i + 3] = (int16_t)(int32_t)(abs((int)yim) - 4 * 700 / sqrt(42));
      llr[6 * i + 4] = (int16_t)(int32_t)(abs(llr[6 * i + 2]) - 2 * 700 / sqrt(42));
      llr[6 * i + 5] = (int16_t)(int32_t)(abs(llr[6 * i + 3]) - 2 * 700 / sqrt(42));
    }
    return 0;
  }
  default:
    return -1;
  }
}

/* ---------------------------------------------------------------- scrambling ---------- */
int orc_sequence(uint32_t seed, uint32_t len, uint8_t *c) { /* 36.211 7.2, Nc = 1600 */
  const uint32_t Nc = 1600, tot = Nc + len + 31;
  uint8_t *x1 = calloc(tot, 1), *x2 = calloc(tot, 1);
  if (!x1 || !x2) return -1;
  for (int n = 0; n < 31; n++) x2[n] = (seed >> n) & 1;
  x1[0] = 1;
  for (uint32_t n = 0; n < Nc + len; n++) {
    x1[n + 31] = (x1[n + 3] + x1[n]) & 1;
    x2[n + 31] = (x2[n + 3] + x2[n + 2] + x2[n + 1] + x2[n]) & 1;
  }
  for (uint32_t n = 0; n < len; n++) c[n] = (x1[n + Nc] + x2[n + Nc]) & 1;
  free(x1);
  free(x2);
  return 0;
}

uint32_t orc_pdsch_seed(uint16_t rnti, int q, uint32_t nslot, uint32_t cell_id) {
  return ((uint32_t)rnti << 14) + ((uint32_t)q << 13) + ((nslot / 2) << 9) + cell_id;
}

int orc_scramble_s(uint32_t seed, int16_t *llr, uint32_t len) {
  uint8_t *c = malloc(len + 1);
  if (!c || orc_sequence(seed, len, c)) return -1;
  for (uint32_t i = 0; i < len; i++)
    if (c[i]) llr[i] = wrap16(-(int32_t)llr[i]); /* _mm256_sign_epi16 with c_short = -1 */
  free(c);
  return 0;
}

/* ---------------------------------------------------------------- CSI weighting ---------- */
/* pdsch.c:676-776 csi_correction, 16-bit path: the SSE loop scales groups of 4 LLRs with
 * _mm_mulhi_pi16(e, cvtps_pi16(csi * (INT16_MAX / csi_max))) — QPSK and 64QAM blend the next
 * symbol's CSI into lanes 0-1 of the mixed groups (_mm_blend_ps(.., 3)) — and the C tail does
 * (int16)(e * (csi / csi_max)). csi_max = max over the codeword's symbols. */
int orc_csi_correction(int mod, const float *csi, int nsym, int16_t *e) {
  const int qm = mod == 0 ? 1 : mod == 1 ? 2 : mod == 2 ? 4 : 6;
  const int nbits = nsym * qm;
  float cmax = -INFINITY;
  for (int i = 0; i < nsym; i++)
    if (csi[i] > cmax) cmax = csi[i];
  if (nsym == 0) cmax = 1.0f;
  const float scale = 32767.0f / cmax;
  int i = 0;
#define MULHI(k, c) e[k] = (int16_t)(((int32_t)e[k] * (int32_t)sat16(cvt_rn((c) * scale))) >> 16)
  if (mod == 1) {
    for (; i < nbits - 3; i += 4) {
      const float c1 = csi[i / 2], c2 = csi[i / 2 + 1];
      MULHI(i, c2);
      MULHI(i + 1, c2);
      MULHI(i + 2, c1);
      MULHI(i + 3, c1);
    }
  } else if (mod == 2) {
    for (; i < nbits - 3; i += 4)
      for (int k = 0; k < 4; k++) MULHI(i + k, csi[i / 4]);
  } else if (mod == 3) {
    for (; i < nbits - 11; i += 12) {
      const float c1 = csi[i / 6], c3 = csi[i / 6 + 1];
      for (int k = 0; k < 4; k++) MULHI(i + k, c1);
      MULHI(i + 4, c3);
      MULHI(i + 5, c3);
      MULHI(i + 6, c1);
      MULHI(i + 7, c1);
      for (int k = 8; k < 12; k++) MULHI(i + k, c3);
    }
  }
#undef MULHI
  for (int sy = i / qm; sy < nsym; sy++) {
    const float c = csi[sy] / cmax;
    for (int k = 0; k < qm; k++) e[qm * sy + k] = wrap16(cvt_rz((float)e[qm * sy + k] * c));
  }
  return 0;
}

/* ---------------------------------------------------------------- 8-bit LLR chain ---------- */
/* The reference's llr_is_8bit receive path (pdsch.c:795-806, sch.c:344-364): int8 soft demapping,
 * int8 scrambling, the 8-bit CSI weighting and (dlsch_oracle.c) the 8-bit de-rate-matching. */
static int8_t sat8(int32_t v) { return (int8_t)(v > 127 ? 127 : v < -128 ? -128 : v); }
static int8_t wrap8(int32_t v) { return (int8_t)(uint8_t)(uint32_t)v; }
static int8_t abs8(int8_t v) { return wrap8(v < 0 ? -(int32_t)v : v); } /* _mm_abs_epi8 */

/* srslte_demod_soft_demodulate_b (demod_soft.c:458-477). SIMD blocks of 8 symbols (16 floats for
 * QPSK's srslte_vec_convert_fb, vector_simd.c:433-462: cvttps + packs_epi32 + packs_epi16, i.e.
 * truncate and saturate; the 16/64QAM SSE loops :153-178, :329-359: cvtps (nearest even), both
 * packs, abs_epi8 / sub_epi8 wrap with offsets (int8)(2*30/sqrt 10) = 18, (int8)(4*40/sqrt 42) =
 * 24, (int8)(2*40/sqrt 42) = 12). C tails: (int8_t) conversions (truncate, then the low byte), the
 * offsets subtracted in double. */
int orc_demod_b(int mod, const float *sym, int nsym, int8_t *llr) {
  switch (mod) {
  case 1: { /* demod_qpsk_lte_b :67-69 */
    const float scale = (float)(-20 * sqrt(2));
    const int len = 2 * nsym, simd = 16 * (len / 16);
    for (int i = 0; i < simd; i++) llr[i] = sat8(sat16(cvt_rz(sym[i] * scale)));
    for (int i = simd; i < len; i++) llr[i] = wrap8(cvt_rz(sym[i] * scale));
    return 0;
  }
  case 2: { /* demod_16qam_lte_b_sse */
    const int8_t off = (int8_t)(2 * 30 / sqrt(10));
    const int simd = 8 * (nsym / 8);
    for (int i = 0; i < simd; i++) {
      const int8_t re = sat8(sat16(cvt_rn(sym[2 * i] * -30.0f)));
      const int8_t im = sat8(sat16(cvt_rn(sym[2 * i + 1] * -30.0f)));
      llr[4 * i + 0] = re;
      llr[4 * i + 1] = im;
      llr[4 * i + 2] = wrap8(abs8(re) - off);
      llr[4 * i + 3] = wrap8(abs8(im) - off);
    }
    for (int i = simd; i < nsym; i++) { /* :180-191 */
      const int16_t yre = (int8_t)wrap8(cvt_rz(30 * sym[2 * i]));
      const int16_t yim = (int8_t)wrap8(cvt_rz(30 * sym[2 * i + 1]));
      llr[4 * i + 0] = wrap8(-yre);
      llr[4 * i + 1] = wrap8(-yim);
      llr[4 * i + 2] = wrap8((int32_t)(abs(yre) - 2 * 30 / sqrt(10)));
      llr[4 * i + 3] = wrap8((int32_t)(abs(yim) - 2 * 30 / sqrt(10)));
    }
    return 0;
  }
  case 3: { /* demod_64qam_lte_b_sse */
    const int8_t off1 = (int8_t)(4 * 40 / sqrt(42)), off2 = (int8_t)(2 * 40 / sqrt(42));
    const int simd = 8 * (nsym / 8);
    for (int i = 0; i < simd; i++) {
      const int8_t re = sat8(sat16(cvt_rn(sym[2 * i] * -40.0f)));
      const int8_t im = sat8(sat16(cvt_rn(sym[2 * i + 1] * -40.0f)));
      const int8_t a1r = wrap8(abs8(re) - off1), a1i = wrap8(abs8(im) - off1);
      llr[6 * i + 0] = re;
      llr[6 * i + 1] = im;
      llr[6 * i + 2] = a1r;
      llr[6 * i + 3] = a1i;
      llr[6 * i + 4] = wrap8(abs8(a1r) - off2);
      llr[6 * i + 5] = wrap8(abs8(a1i) - off2);
    }
    for (int i = simd; i < nsym; i++) { /* :360-371 */
      const float yre = (int8_t)wrap8(cvt_rz(40 * sym[2 * i]));
      const float yim = (int8_t)wrap8(cvt_rz(40 * sym[2 * i + 1]));
      llr[6 * i + 0] = wrap8((int32_t)-yre);
      llr[6 * i + 1] = wrap8((int32_t)-yim);
      llr[6 * i + 2] = wrap8((int32_t)(abs((int)yre) - 4 * 40 / sqrt(42)));
      llr[6 * i + 3] = wrap8((int32_t)(abs((int)yim) - 4 * 40 / sqrt(42)));
      llr[6 * i + 4] = wrap8((int32_t)(abs(llr[6 * i + 2]) - 2 * 40 / sqrt(42)));
      llr[6 * i + 5] = wrap8((int32_t)(abs(llr[6 * i + 3]) - 2 * 40 / sqrt(42)));
    }
    return 0;
  }
  default: /* BPSK is not a PDSCH modulation */
    return -1;
  }
}

/* srslte_scrambling_sb_offset (scrambling.c:53-56): srslte_vec_neg_bbb with c_char = 1 - 2c
 * (_mm256_sign_epi8 / the C tail y < 0 ? -x : x, both wrapping at -128) */
int orc_scramble_sb(uint32_t seed, int8_t *llr, uint32_t len) {
  uint8_t *c = malloc(len + 1);
  if (!c || orc_sequence(seed, len, c)) return -1;
  for (uint32_t i = 0; i < len; i++)
    if (c[i]) llr[i] = wrap8(-(int32_t)llr[i]);
  free(c);
  return 0;
}

/* csi_correction, 8-bit path (pdsch.c:707-713): e = (int8_t)((float)e * (csi / csi_max)) */
int orc_csi_correction_b(int mod, const float *csi, int nsym, int8_t *e) {
  const int qm = mod == 0 ? 1 : mod == 1 ? 2 : mod == 2 ? 4 : 6;
  float cmax = -INFINITY;
  for (int i = 0; i < nsym; i++)
    if (csi[i] > cmax) cmax = csi[i];
  if (nsym == 0) cmax = 1.0f;
  for (int sy = 0; sy < nsym; sy++) {
    const float c = csi[sy] / cmax;
    for (int k = 0; k < qm; k++) e[qm * sy + k] = wrap8(cvt_rz((float)e[qm * sy + k] * c));
  }
  return 0;
}

/* ---------------------------------------------------------------- TM2 transmit diversity ---------- */
/* srslte_predecoding_diversity_multi for 2 ports (precoding.c:670-685) + srslte_layerdemap_diversity
 * (layermap.c:143-151): d[2i] = x0[i], d[2i+1] = x1[i] for RE pairs (2i, 2i+1).
 * - CSI on: srslte_predecoding_diversity_csi (:569-602), generic arithmetic for every pair,
 *   csi[2i] = csi[2i+1] = hh before scaling;
 * - CSI off, n > 32: srslte_predecoding_diversity2_sse (:438-543) for the first 4*(n/4) REs, then
 *   the generic srslte_predecoding_diversity_gen_ (:356-428) from there;
 * - CSI off, n <= 32: generic for every pair.
 * Generic: float complex arithmetic as gcc evaluates it (no FMA), with the double conj() of
 * x1's terms (products and sums in double, rounded into the float accumulator) and the double
 * sqrt(2) factor; hh = 1e-4 when it is exactly 0. SSE: PROD = addsub(a*ldup(b), swap(a)*hdup(b)),
 * |h|^2 by hadd (re^2 + im^2, then h00 + h11), rx antennas added in order, x = x / hh * (sqrtf(2) /
 * scaling). y: [rx][2n floats], h: [port][rx][2n floats] (n REs of this grant, extraction order). */
typedef struct {
  float r, i;
} txd_cf;
static txd_cf txd_ld(const float *p, int k) { return (txd_cf){p[2 * k], p[2 * k + 1]}; }
static txd_cf txd_mul(txd_cf a, txd_cf b) { return (txd_cf){a.r * b.r - a.i * b.i, a.r * b.i + a.i * b.r}; }

static void txd_gen_pair(const float *const *y, const float *const h[2][2], int nrx, int i, float scaling,
                         float *d, float *csi) {
  float hh = 0;
  txd_cf x0 = {0, 0}, x1 = {0, 0};
  for (int p = 0; p < nrx; p++) {
    const txd_cf h00 = txd_ld(h[0][p], 2 * i), h01 = txd_ld(h[0][p], 2 * i + 1);
    const txd_cf h10 = txd_ld(h[1][p], 2 * i), h11 = txd_ld(h[1][p], 2 * i + 1);
    hh += h00.r * h00.r + h00.i * h00.i + h11.r * h11.r + h11.i * h11.i;
    const txd_cf r0 = txd_ld(y[p], 2 * i), r1 = txd_ld(y[p], 2 * i + 1);
    if (hh == 0) hh = 1e-4;
    const txd_cf a = txd_mul((txd_cf){h00.r, -h00.i}, r0), b = txd_mul(h11, (txd_cf){r1.r, -r1.i});
    x0.r = x0.r + (a.r + b.r);
    x0.i = x0.i + (a.i + b.i);
    /* -h10 * conj(r0) + conj(h01) * r1 in double complex */
    const double nr = -(double)h10.r, ni = -(double)h10.i, cr = r0.r, ci = -(double)r0.i;
    const double pr = nr * cr - ni * ci, pi = nr * ci + ni * cr;
    const double gr = h01.r, gi = -(double)h01.i, s1r = r1.r, s1i = r1.i;
    const double qr = gr * s1r - gi * s1i, qi = gr * s1i + gi * s1r;
    x1.r = (float)((double)x1.r + (pr + qr));
    x1.i = (float)((double)x1.i + (pi + qi));
  }
  if (csi) csi[2 * i] = csi[2 * i + 1] = hh;
  hh *= scaling;
  d[4 * i + 0] = (float)((double)(x0.r / hh) * sqrt(2));
  d[4 * i + 1] = (float)((double)(x0.i / hh) * sqrt(2));
  d[4 * i + 2] = (float)((double)(x1.r / hh) * sqrt(2));
  d[4 * i + 3] = (float)((double)(x1.i / hh) * sqrt(2));
}

static void txd_sse_pair(const float *const *y, const float *const h[2][2], int nrx, int i, float scaling,
                         float *d) {
  const float s2 = sqrtf(2) / scaling;
  float hh = 0;
  txd_cf x0 = {0, 0}, x1 = {0, 0};
  for (int p = 0; p < nrx; p++) {
    const txd_cf h00 = txd_ld(h[0][p], 2 * i), h01 = txd_ld(h[0][p], 2 * i + 1);
    const txd_cf h10 = txd_ld(h[1][p], 2 * i), h11 = txd_ld(h[1][p], 2 * i + 1);
    const txd_cf r0 = txd_ld(y[p], 2 * i), r1 = txd_ld(y[p], 2 * i + 1);
    const float g = (h00.r * h00.r + h00.i * h00.i) + (h11.r * h11.r + h11.i * h11.i);
    hh = p ? hh + g : g;
    const txd_cf a = txd_mul((txd_cf){h00.r, -h00.i}, r0), b = txd_mul(h11, (txd_cf){r1.r, -r1.i});
    const txd_cf c = txd_mul((txd_cf){h01.r, -h01.i}, r1), e = txd_mul(h10, (txd_cf){r0.r, -r0.i});
    const txd_cf u0 = {a.r + b.r, a.i + b.i}, u1 = {c.r - e.r, c.i - e.i};
    x0 = p ? (txd_cf){x0.r + u0.r, x0.i + u0.i} : u0;
    x1 = p ? (txd_cf){x1.r + u1.r, x1.i + u1.i} : u1;
  }
  d[4 * i + 0] = (x0.r / hh) * s2;
  d[4 * i + 1] = (x0.i / hh) * s2;
  d[4 * i + 2] = (x1.r / hh) * s2;
  d[4 * i + 3] = (x1.i / hh) * s2;
}

int orc_predecode_txdiv(const float *y0, const float *y1, const float *h00, const float *h01,
                        const float *h10, const float *h11, int nrx, int n, float scaling, float *d,
                        float *csi) {
  const float *y[2] = {y0, y1};
  const float *const h[2][2] = {{h00, h01}, {h10, h11}}; /* [port][rx] */
  int i0 = 0;
  if (!csi && n > 32) {
    for (; i0 < 2 * (n / 4); i0++) txd_sse_pair(y, h, nrx, i0, scaling, d);
  }
  for (int i = i0; i < n / 2; i++) txd_gen_pair(y, h, nrx, i, scaling, d, csi);
  return 0;
}

/* 4 ports (srslte_predecoding_diversity_multi with nof_ports == 4, precoding.c:670-685: no SSE form),
 * then srslte_layerdemap_diversity over 4 layers (layermap.c:143-151): d[4i+k] = x_k[i] for the RE
 * quadruplet 4i..4i+3, ports (0, 2) on REs 4i / 4i+1 and ports (1, 3) on 4i+2 / 4i+3 (the transmitter
 * of precoding.c:1863-1889).
 * - CSI off: srslte_predecoding_diversity_gen_ (:388-423): one channel per port pair read at the
 *   first RE of its pair (h0 = h[0][4i], h2 = h[2][4i], h1 = h[1][4i+2], h3 = h[3][4i+2]), gains
 *   hh02 / hh13 summed over rx antennas without the 1e-4 guard, float complex arithmetic,
 *   x / (hh * scaling) * sqrt(2) in double;
 * - CSI on: srslte_predecoding_diversity_csi (:604-662): per-RE gains a0..a3 (a0 from h[0][4i] and
 *   h[2][4i+1], a1 from h[0][4i+1] and h[2][4i], likewise a2 / a3 on ports 1 / 3 at 4i+2 / 4i+3),
 *   csi[4i+k] = a_k scaling / nof_rxant, x_k / (a_k scaling) * sqrtf(2) in float.
 * Layer symbols: m_ap = n / 4 (n % 4 == 2: (n - 2) / 4), and srslte_pdsch_decode demaps n / 4 per
 * layer, so d[4 (n / 4) ..] would be whatever the reference's buffer last held: n % 4 != 0 is refused.
 * y: [rx][2n floats], h: [port * 2 + rx][2n floats]. */
static txd_cf txd_conj(txd_cf a) { return (txd_cf){a.r, -a.i}; }
static txd_cf txd_add(txd_cf a, txd_cf b) { return (txd_cf){a.r + b.r, a.i + b.i}; }
static txd_cf txd_neg(txd_cf a) { return (txd_cf){-a.r, -a.i}; }
static float txd_pow(txd_cf a) { return a.r * a.r + a.i * a.i; }

int orc_predecode_txdiv4(const float *const *y, const float *const *h, int nrx, int n, float scaling, float *d,
                         float *csi) {
  if (n % 4 || nrx < 1 || nrx > 2) return -1;
  for (int i = 0; i < n / 4; i++) {
    txd_cf x[4] = {{0, 0}, {0, 0}, {0, 0}, {0, 0}};
    if (!csi) {
      float hh02 = 0, hh13 = 0;
      for (int p = 0; p < nrx; p++) {
        const txd_cf h0 = txd_ld(h[0 * 2 + p], 4 * i), h1 = txd_ld(h[1 * 2 + p], 4 * i + 2);
        const txd_cf h2 = txd_ld(h[2 * 2 + p], 4 * i), h3 = txd_ld(h[3 * 2 + p], 4 * i + 2);
        hh02 += h0.r * h0.r + h0.i * h0.i + h2.r * h2.r + h2.i * h2.i;
        hh13 += h1.r * h1.r + h1.i * h1.i + h3.r * h3.r + h3.i * h3.i;
        const txd_cf r0 = txd_ld(y[p], 4 * i), r1 = txd_ld(y[p], 4 * i + 1);
        const txd_cf r2 = txd_ld(y[p], 4 * i + 2), r3 = txd_ld(y[p], 4 * i + 3);
        x[0] = txd_add(x[0], txd_add(txd_mul(txd_conj(h0), r0), txd_mul(h2, txd_conj(r1))));
        x[1] = txd_add(x[1], txd_add(txd_mul(txd_neg(h2), txd_conj(r0)), txd_mul(txd_conj(h0), r1)));
        x[2] = txd_add(x[2], txd_add(txd_mul(txd_conj(h1), r2), txd_mul(h3, txd_conj(r3))));
        x[3] = txd_add(x[3], txd_add(txd_mul(txd_neg(h3), txd_conj(r2)), txd_mul(txd_conj(h1), r3)));
      }
      hh02 *= scaling;
      hh13 *= scaling;
      for (int k = 0; k < 4; k++) {
        const float g = k < 2 ? hh02 : hh13;
        d[8 * i + 2 * k] = (float)((double)(x[k].r / g) * sqrt(2));
        d[8 * i + 2 * k + 1] = (float)((double)(x[k].i / g) * sqrt(2));
      }
    } else {
      float a[4] = {0, 0, 0, 0};
      for (int p = 0; p < nrx; p++) {
        for (int q = 0; q < 2; q++) { /* q = 0: ports 0 / 2 on REs 4i, 4i+1; q = 1: ports 1 / 3 on 4i+2, 4i+3 */
          const int b = 4 * i + 2 * q;
          const txd_cf h00 = txd_ld(h[(q + 0) * 2 + p], b), h01 = txd_ld(h[(q + 2) * 2 + p], b);
          const txd_cf h10 = txd_ld(h[(q + 0) * 2 + p], b + 1), h11 = txd_ld(h[(q + 2) * 2 + p], b + 1);
          a[2 * q] += txd_pow(h00) + h11.r * h11.r + h11.i * h11.i;
          a[2 * q + 1] += txd_pow(h10) + h01.r * h01.r + h01.i * h01.i;
          const txd_cf r0 = txd_ld(y[p], b), r1 = txd_ld(y[p], b + 1);
          x[2 * q] = txd_add(x[2 * q], txd_add(txd_mul(txd_conj(h00), r0), txd_mul(h11, txd_conj(r1))));
          x[2 * q + 1] =
              txd_add(x[2 * q + 1], txd_add(txd_mul(txd_neg(h01), txd_conj(r0)), txd_mul(txd_conj(h10), r1)));
        }
      }
      for (int k = 0; k < 4; k++) {
        a[k] *= scaling;
        csi[4 * i + k] = a[k] / nrx;
        d[8 * i + 2 * k] = x[k].r / a[k] * sqrtf(2.0f);
        d[8 * i + 2 * k + 1] = x[k].i / a[k] * sqrtf(2.0f);
      }
    }
  }
  return 0;
}

/* ---------------------------------------------------------------- Viterbi (PDCCH) ---------- */
/* srslte_viterbi_decode_f with the tail-biting K=7 r=1/3 decoder srsLTE builds for the PDCCH
 * (pdcch.c:79,341). With AVX2 viterbi.c defines VITERBI_16 (:46-50), so decode_f quantises to
 * uint16 (gain 1000 / max|x|, srslte_vec_quant_fus offset 32767.5 clip 65535, vector.c:408-420)
 * and runs decode37_avx2_16bit (:133-160: TB_ITER = 3 copies of the frame, the middle third out)
 * over viterbi37_avx2_16bit.c: all 64 metrics start at 63, branch metric
 * avg(B2^s2, avg(B0^s0, B1^s1)) >> 3 with B = 0 / 65535, complement 8191 - metric, uint16
 * wrapping adds, "modulo" compare (signed 16-bit difference > 0), new state 2b / 2b+1 from old b
 * and b+32. The normalisation (:304-328) subtracts 0: its _mm256_srli_si256(v, 16) shifts each
 * 128-bit lane out entirely, so the minimum it takes is always 0 and the metrics just wrap. Best
 * end state = the last index of the minimum; chainback reads the decisions 6 positions past the
 * bit it decides (zero beyond the frame). */
static int orc_parity(int x) {
  x ^= x >> 16;
  x ^= x >> 8;
  x ^= x >> 4;
  x ^= x >> 2;
  x ^= x >> 1;
  return x & 1;
}

static int orc_vit_core(uint16_t *q, uint32_t F, uint8_t *out);
int orc_viterbi37_tb_decode_f(const float *sym, uint32_t F, uint8_t *out) {
  const uint32_t len = 3 * F;
  float mx = -9e9f;
  for (uint32_t i = 0; i < len; i++)
    if (fabs(sym[i]) > mx) mx = (float)fabs(sym[i]);
  const float gain = 1000.0f / mx;
  uint16_t *q = malloc(len * sizeof(uint16_t));
  if (!q) return -1;
  for (uint32_t i = 0; i < len; i++) {
    const float v = 32767.5f + gain * sym[i];
    long t = (v == v && v >= -9.2e18f && v < 9.2e18f) ? (long)v : LONG_MIN; /* cvttss2si 64 */
    if (t < 0) t = 0;
    if (t > 65535) t = 65535;
    q[i] = (uint16_t)t;
  }
  return orc_vit_core(q, F, out);
}

/* srslte_viterbi_decode_s on the same decoder (viterbi.c:558-584 with VITERBI_16): srslte_vec_quant_sus
 * (vector.c:450-460) with gain 1 and offset 32767, i.e. tmp = (int16_t)(32767 + (float)x) -- the float
 * converted as cvttss2si to 32 bits then truncated to 16 -- and 0 where that is negative: x <= 0 gives
 * 32767 + x (0 for x = -32768), x > 0 wraps negative and gives 0. Then decode37_avx2_16bit. */
int orc_viterbi37_tb_decode_s(const int16_t *sym, uint32_t F, uint8_t *out) {
  uint16_t *q = malloc(3 * F * sizeof(uint16_t));
  if (!q) return -1;
  for (uint32_t i = 0; i < 3 * F; i++) {
    const int16_t t = (int16_t)(int32_t)(32767.0f + (float)sym[i] * 1.0f);
    q[i] = (uint16_t)(t < 0 ? 0 : t);
  }
  return orc_vit_core(q, F, out);
}

/* the tail-biting trellis of decode37_avx2_16bit on quantised symbols q (3F, freed here) */
static int orc_vit_core(uint16_t *q, uint32_t F, uint8_t *out) {
  const int poly[3] = {0x6D, 0x4F, 0x57};
  const uint32_t nb = 3 * F;
  uint64_t *dec = calloc(nb + 6, sizeof(uint64_t));
  uint8_t *tmp = malloc(nb);
  if (!dec || !tmp) return -1;
  uint16_t B[3][32];
  for (int st = 0; st < 32; st++)
    for (int j = 0; j < 3; j++) B[j][st] = orc_parity((2 * st) & poly[j]) ? 65535 : 0;
  uint16_t old[64], nw[64];
  for (int st = 0; st < 64; st++) old[st] = 63;
  for (uint32_t t = 0; t < nb; t++) {
    const uint16_t *s = q + 3 * (t % F); /* the frame repeated TB_ITER times */
    uint64_t d = 0;
    for (int b = 0; b < 32; b++) {
      const uint32_t m0a = ((uint32_t)(B[0][b] ^ s[0]) + (uint32_t)(B[1][b] ^ s[1]) + 1) >> 1;
      const uint32_t metric = (((uint32_t)(B[2][b] ^ s[2]) + m0a + 1) >> 1) >> 3;
      const uint32_t mm = (uint16_t)(8191 - metric);
      const uint16_t m0 = (uint16_t)(old[b] + metric), m2 = (uint16_t)(old[b] + mm);
      const uint16_t m3 = (uint16_t)(old[b + 32] + metric), m1 = (uint16_t)(old[b + 32] + mm);
      const int d0 = (int16_t)(uint16_t)(m0 - m1) > 0, d1 = (int16_t)(uint16_t)(m2 - m3) > 0;
      nw[2 * b] = d0 ? m1 : m0;
      nw[2 * b + 1] = d1 ? m3 : m2;
      d |= (uint64_t)d0 << (2 * b) | (uint64_t)d1 << (2 * b + 1);
    }
    dec[t] = d;
    memcpy(old, nw, sizeof(old));
  }
  uint32_t best = 0;
  uint16_t mn = 65535;
  for (uint32_t st = 0; st < 64; st++)
    if (old[st] <= mn) {
      best = st;
      mn = old[st];
    }
  uint32_t es = (best % 64) << 2;
  for (int32_t b = (int32_t)nb - 1; b >= 0; b--) {
    const uint32_t k = (uint32_t)((dec[b + 6] >> (es >> 2)) & 1);
    es = (es >> 1) | (k << 7);
    tmp[b] = (uint8_t)k;
  }
  memcpy(out, tmp + F, F);
  free(q);
  free(dec);
  free(tmp);
  return 0;
}

/* DCI candidate decode as srslte_pdcch_decode_msg does it (pdcch.c:380-396: skipped unless the
 * mean |llr| over the E bits, summed in double, exceeds 0.5; then srslte_pdcch_dci_decode
 * :322-360): srslte_rm_conv_rx (rm_conv.c:99-157: 32-column sub-block interleaver over the three
 * streams, dummy positions skipped, repetitions soft-combined in input order with 10000 as the
 * empty marker, empty outputs 0), the Viterbi decoder above over nof_bits + 16 bits, and the CRC16
 * (0x11021, init 0) of the first nof_bits XOR the 16 received parity bits. Returns 1 decoded,
 * 0 skipped. */
static const uint8_t RM_PERM_CC[32] = {1, 17, 9, 25, 5, 21, 13, 29, 3, 19, 11, 27, 7, 23, 15, 31,
                                       0, 16, 8, 24, 4, 20, 12, 28, 2, 18, 10, 26, 6, 22, 14, 30};
static const uint8_t RM_PERM_CC_INV[32] = {16, 0, 24, 8, 20, 4, 28, 12, 18, 2, 26, 10, 22, 6, 30, 14,
                                           17, 1, 25, 9, 21, 5, 29, 13, 19, 3, 27, 11, 23, 7, 31, 15};
int orc_dci_decode(const float *e, uint32_t E, uint32_t nof_bits, uint8_t *data, uint16_t *crc_rem) {
  double mean = 0;
  for (uint32_t i = 0; i < E; i++) mean += fabsf(e[i]);
  mean /= E;
  if (!(mean > 0.5)) return 0;
  const uint32_t out_len = 3 * (nof_bits + 16);
  const int nrows = (int)((out_len / 3 - 1) / 32 + 1), K_p = nrows * 32;
  int ndummy = K_p - (int)(out_len / 3);
  if (ndummy < 0) ndummy = 0;
  float tmp[3 * 32 * 32], rm[3 * 144];
  for (int i = 0; i < 3 * K_p; i++) tmp[i] = 10000.0f;
  uint32_t k = 0;
  int j = 0;
  while (k < E) {
    const int d_i = (j % K_p) / nrows, d_j = (j % K_p) % nrows;
    if (d_j * 32 + RM_PERM_CC[d_i] >= ndummy) {
      if (tmp[j] == 10000.0f)
        tmp[j] = e[k];
      else if (e[k] != 10000.0f)
        tmp[j] += e[k];
      k++;
    }
    if (++j == 3 * K_p) j = 0;
  }
  for (uint32_t i = 0; i < out_len / 3; i++) {
    const int d_i = (int)(i + ndummy) / 32, d_j = (int)(i + ndummy) % 32;
    for (int s = 0; s < 3; s++) {
      const float o = tmp[K_p * s + RM_PERM_CC_INV[d_j] * nrows + d_i];
      rm[i * 3 + s] = o != 10000.0f ? o : 0;
    }
  }
  if (orc_viterbi37_tb_decode_f(rm, nof_bits + 16, data)) return -1;
  uint32_t crc = 0;
  for (uint32_t i = 0; i < nof_bits; i++) {
    const uint32_t fb = ((crc >> 15) & 1) ^ (data[i] & 1);
    crc = (crc << 1) & 0xFFFF;
    if (fb) crc ^= 0x1021;
  }
  uint32_t p = 0;
  for (int i = 0; i < 16; i++) p = (p << 1) | (data[nof_bits + i] & 1);
  *crc_rem = (uint16_t)(p ^ crc);
  return 1;
}

/* ---------------------------------------------------------------- PCFICH ---------- */
/* srslte_regs_pcfich_get's 16 REs (regs.c:477-512 regs_pcfich_init, :622-665 regs_reg_init):
 * REG i at k = (6 (N_ID mod 2 N_RB) + floor(i N_RB / 2) 6) mod 12 N_RB in OFDM symbol 0, its four
 * REs the six subcarriers k.. minus the reference signals at v_o = N_ID mod 3 and v_o + 3 */
int orc_pcfich_re_map(uint32_t nof_prb, uint32_t cell_id, uint32_t *idx) {
  const uint32_t k_hat = 6 * (cell_id % (2 * nof_prb)), vo = cell_id % 3;
  int n = 0;
  for (uint32_t i = 0; i < 4; i++) {
    const uint32_t k0 = (k_hat + (i * nof_prb / 2) * 6) % (nof_prb * 12);
    for (uint32_t s = 0; s < 6; s++)
      if (s != vo && s != vo + 3) idx[n++] = k0 + s;
  }
  return n;
}

/* srslte_pcfich_decode_multi (pcfich.c:178-241): the 16 REs, SISO predecoding with the noise
 * estimate (one port: the C path, 16 <= 32 symbols) or 2-port transmit diversity (generic path) +
 * layer demapping, QPSK soft demapping x (-sqrt 2) (demod_soft.c:71-73, vector product, exact),
 * scrambling by +-1 (sequences.c:42-44: c_init = (ns/2 + 1)(2 N_ID + 1) 2^9 + N_ID with ns =
 * 2 sf), and the sequential float correlation with the three codewords as +-1 (pcfich.c:129-147,
 * vector.c:359-366): cfi = 1 + the first index of the strict maximum over 0. y [rx][n], h
 * [port][rx][n] full subframe grids (complex float). */
int orc_pcfich_decode(uint32_t nof_prb, uint32_t cell_id, uint32_t nof_ports, uint32_t nrx,
                      const float *const *y, const float *const *h, float noise, uint32_t sf_idx,
                      uint32_t *cfi, float *corr) {
  static const uint8_t tab[3][32] = {
      {0, 1, 1, 0, 1, 1, 0, 1, 1, 0, 1, 1, 0, 1, 1, 0, 1, 1, 0, 1, 1, 0, 1, 1, 0, 1, 1, 0, 1, 1, 0, 1},
      {1, 0, 1, 1, 0, 1, 1, 0, 1, 1, 0, 1, 1, 0, 1, 1, 0, 1, 1, 0, 1, 1, 0, 1, 1, 0, 1, 1, 0, 1, 1, 0},
      {1, 1, 0, 1, 1, 0, 1, 1, 0, 1, 1, 0, 1, 1, 0, 1, 1, 0, 1, 1, 0, 1, 1, 0, 1, 1, 0, 1, 1, 0, 1, 1}};
  uint32_t idx[16];
  orc_pcfich_re_map(nof_prb, cell_id, idx);
  float ys[2][32], hs[4][2][32], d[32];
  for (uint32_t a = 0; a < nrx; a++)
    for (int i = 0; i < 16; i++) {
      ys[a][2 * i] = y[a][2 * idx[i]];
      ys[a][2 * i + 1] = y[a][2 * idx[i] + 1];
      for (uint32_t p = 0; p < nof_ports; p++) {
        hs[p][a][2 * i] = h[p * nrx + a][2 * idx[i]];
        hs[p][a][2 * i + 1] = h[p * nrx + a][2 * idx[i] + 1];
      }
    }
  if (nof_ports == 1) {
    /* srslte_predecoding_single_multi, C path (precoding.c:330-352 with n <= 32) */
    for (int i = 0; i < 16; i++) {
      float hh = 0, rr = 0, ri = 0;
      for (uint32_t a = 0; a < nrx; a++) {
        const double yr = ys[a][2 * i], yi = ys[a][2 * i + 1], hr = hs[0][a][2 * i], hi = hs[0][a][2 * i + 1];
        rr = (float)((double)rr + (yr * hr - yi * -hi));
        ri = (float)((double)ri + (yr * -hi + yi * hr));
        hh = (float)((double)hh + (hr * hr + hi * hi));
      }
      const float den = (hh + noise) * 1.0f;
      d[2 * i] = rr / den;
      d[2 * i + 1] = ri / den;
    }
  } else if (nof_ports == 4) { /* 4-port transmit diversity over the 4 REGs' quadruplets */
    const float *yy[2] = {ys[0], ys[1]};
    const float *h4[8];
    for (int p = 0; p < 4; p++)
      for (int a = 0; a < 2; a++) h4[2 * p + a] = hs[p][a];
    orc_predecode_txdiv4(yy, h4, (int)nrx, 16, 1.0f, d, NULL);
  } else {
    orc_predecode_txdiv(ys[0], nrx > 1 ? ys[1] : NULL, hs[0][0], nrx > 1 ? hs[0][1] : NULL, hs[1][0],
                        nrx > 1 ? hs[1][1] : NULL, (int)nrx, 16, 1.0f, d, NULL);
  }
  uint8_t c[32];
  orc_sequence(((2 * sf_idx) / 2 + 1) * (2 * cell_id + 1) * 512 + cell_id, 32, c);
  const float s2 = (float)(-sqrt(2));
  float l[32];
  for (int i = 0; i < 32; i++) {
    l[i] = d[i] * s2;
    if (c[i]) l[i] = -l[i];
  }
  float mx = 0;
  int index = 0;
  for (int k = 0; k < 3; k++) {
    float r = 0;
    for (int i = 0; i < 32; i++) r += (float)(2.0 * tab[k][i] - 1.0) * l[i];
    if (r > mx) {
      mx = r;
      index = k;
    }
  }
  *cfi = (uint32_t)index + 1;
  *corr = mx;
  return 0;
}

/* ---------------------------------------------------------------- UCI on the PUSCH ---------- */
/* srslte_pusch_decode's UCI steps (pusch.c:626-657) on a TB's q soft bits, still scrambled (q_in,
 * nof_bits int16) with the PUSCH sequence c (one byte per bit):
 *  1. HARQ-ACK (O[0] = 1 or 2 bits) and RI (O[1]) from the scrambled bits, srslte_uci_decode_ack_ri
 *     (uci.c:746-790): Q' = min(ceilf((float)O M_sc_init N_symb beta / K), 4 M_sc) (uci.c:548-572; K
 *     the TB's C1 K1 + C2 K2, or O_cqi (+8 above 11 bits) without data; beta / beta_cqi without data);
 *     bit group i at row H'/N - 1 - i/4, column {2,3,8,9} (ACK) or {1,4,7,10} (RI)[(3i) mod 4]
 *     (uci.c:499-546); one bit: the sum of -(q0 + q1) with q = c[p0] ? q : -q for BOTH positions
 *     (decode_ri_ack_1bit reads c at p0 twice, uint32 arithmetic); two bits: the groups in threes,
 *     each triple added when the loop reaches the next multiple of 3 (so a last, complete or partial,
 *     triple is never added); bit = sum > 0. The ACK positions are then zeroed (sch.c:921-924).
 *  2. descrambling, q = c ? -q : q (int16, srslte_scrambling_s_offset);
 *  3. the channel deinterleaver with the RI positions taken out (sch.c:550-568, 860-881): entries
 *     numbered row by row skipping RI, g[lut[x]] = q[x] in q order with the RI entries' lut = 0, so
 *     g[0] ends as the RI entry with the largest q index when there is one;
 *  4. CQI (O[2] bits, srslte_uci_decode_cqi_pusch uci.c:428-464): Q' = min(ceilf((float)(O + L)
 *     M_sc_init N_symb beta / K), M_sc N_symb - Q'_ri), L = 8 from 11 bits on (O < 11: 0), 999999 for
 *     K = 0; up to 11 bits the (32, O) block code by ML (uci.c:312-351): copies of 32 summed into
 *     g[0..32) (int16 wrap), then per word w the correlation with the +-1 code word over min(32, Q')
 *     as srslte_vec_dot_prod_sss computes it (16 int16 lanes of mullo + add with wrap, summed, then
 *     an int tail), the first maximum wins, bits MSB first; above 11 bits srslte_rm_conv_rx_s,
 *     srslte_viterbi_decode_s over O + 8 bits and CRC8 0x19B, the CQI taken only when it checks.
 * out: ack[0], ack[1], ri, cqi_ack, then the O[2] CQI bits; g: nof_bits deinterleaved bits;
 * qp: Q'_ack, Q'_ri, Q'_cqi (the data bits start at Q'_cqi Qm, G = nof_bits - (Q'_ri + Q'_cqi) Qm).
 * Returns -1 on a reserved beta index, a CQI longer than 183 bits, or HARQ-ACK / RI bits beyond the
 * reference's position array (srslte_sch_t.ack_ri_bits[12 * 288], sch.h:70: Q' Qm above 3456 writes past
 * it, so such a configuration has no defined result). */
#include "srsgpu/uci_tables.h"

static uint32_t uci_qp_ack_ri(uint32_t O, uint32_t O_cqi, float beta, uint32_t K, uint32_t M_sc,
                              uint32_t M_sc_init, uint32_t nsymb) {
  if (K == 0) K = O_cqi <= 11 ? O_cqi : O_cqi + 8;
  const uint32_t x = (uint32_t)ceilf((float)O * M_sc_init * nsymb * beta / K);
  return x < 4 * M_sc ? x : 4 * M_sc;
}

static uint32_t uci_pos(uint32_t i, uint32_t k, uint32_t Qm, uint32_t rows, int ri) {
  static const uint32_t ack_cols[4] = {2, 3, 8, 9}, ri_cols[4] = {1, 4, 7, 10};
  const uint32_t row = rows - 1 - i / 4, col = (ri ? ri_cols : ack_cols)[(3 * i) % 4];
  return row * Qm + rows * col * Qm + k;
}

static void uci_ack_ri(const int16_t *q, const uint8_t *c, uint32_t Qp, uint32_t O, uint32_t Qm, uint32_t rows,
                       int ri, uint8_t *data) {
  int32_t sum[3] = {0, 0, 0};
  for (uint32_t i = 0; i < Qp; i++) {
    if (O == 2 && i % 3 == 0 && i > 0) {
      int32_t v[6];
      for (int g = 0; g < 3; g++)
        for (int k = 0; k < 2; k++) {
          const uint32_t p = uci_pos(i - 3 + g, k, Qm, rows, ri);
          v[2 * g + k] = c[p] ? q[p] : -q[p];
        }
      sum[0] -= v[0] + v[3];
      sum[1] -= v[1] + v[4];
      sum[2] -= v[2] + v[5];
    } else if (O == 1) {
      const uint32_t p0 = uci_pos(i, 0, Qm, rows, ri), p1 = uci_pos(i, 1, Qm, rows, ri);
      const uint32_t q0 = c[p0] ? q[p0] : -q[p0], q1 = c[p0] ? q[p1] : -q[p1];
      sum[0] = (int32_t)((uint32_t)sum[0] + (uint32_t)(-(q0 + q1)));
    }
  }
  data[0] = sum[0] > 0;
  if (O == 2) data[1] = sum[1] > 0;
}

static uint32_t orc_crc8_bits(const uint8_t *b, uint32_t n) {
  uint32_t r = 0;
  for (uint32_t i = 0; i < n; i++) {
    const uint32_t fb = ((r >> 7) & 1) ^ (b[i] & 1);
    r = (r << 1) & 0xFF;
    if (fb) r ^= 0x9B;
  }
  return r;
}

int orc_ulsch_uci(uint32_t tbs, uint32_t Qm, uint32_t nof_bits, uint32_t nsymb, uint32_t M_sc, uint32_t M_sc_init,
                  const uint32_t *I_off, const uint32_t *O, const int16_t *q_in, const uint8_t *c, uint8_t *out,
                  int16_t *g, uint32_t *qp) {
  const uint32_t Hp = nof_bits / Qm, rows = Hp / nsymb, O_ack = O[0], O_ri = O[1], O_cqi = O[2];
  uint32_t K = 0;
  if (tbs) {
    orc_cbsegm_t sg;
    if (orc_segm(tbs, &sg)) return -1;
    K = sg.C1 * sg.K1 + sg.C2 * sg.K2;
  }
  if (O_cqi + 8 > 191 || O_ack > 2 || O_ri > 2) return -1;
  int16_t *q = malloc((nof_bits + 64) * sizeof(int16_t));
  uint8_t *ri_at = calloc(nof_bits + 64, 1);
  memcpy(q, q_in, nof_bits * sizeof(int16_t));
  memset(out, 0, 4 + O_cqi);
  uint32_t Q_ack = 0, Q_ri = 0, Q_cqi = 0;
  const float bcqi = SRSGPU_BETA_CQI[I_off[2] & 15];
  if (O_ack) {
    float beta = SRSGPU_BETA_ACK[I_off[0] & 15];
    if (!tbs) beta /= bcqi;
    if (beta < 0) return -1;
    Q_ack = uci_qp_ack_ri(O_ack, O_cqi, beta, K, M_sc, M_sc_init, nsymb);
    if (Q_ack * Qm > 12 * 288) return -1;
    uci_ack_ri(q, c, Q_ack, O_ack, Qm, rows, 0, out);
    for (uint32_t i = 0; i < Q_ack; i++)
      for (uint32_t k = 0; k < Qm; k++) q[uci_pos(i, k, Qm, rows, 0)] = 0;
  }
  if (O_ri) {
    float beta = SRSGPU_BETA_RI[I_off[1] & 15];
    if (!tbs) beta /= bcqi;
    if (beta < 0) return -1;
    Q_ri = uci_qp_ack_ri(O_ri, O_cqi, beta, K, M_sc, M_sc_init, nsymb);
    if (Q_ri * Qm > 12 * 288) return -1;
    uint8_t ri[2] = {0, 0};
    uci_ack_ri(q, c, Q_ri, O_ri, Qm, rows, 1, ri);
    out[2] = ri[0];
    for (uint32_t i = 0; i < Q_ri; i++)
      for (uint32_t k = 0; k < Qm; k++) ri_at[uci_pos(i, k, Qm, rows, 1)] = 1;
  }
  for (uint32_t x = 0; x < nof_bits; x++) q[x] = c[x] ? (int16_t)-q[x] : q[x];
  uint32_t idx = 0, x0 = 0, xr = 0;
  int any_ri = 0;
  for (uint32_t j = 0; j < rows; j++)
    for (uint32_t i = 0; i < nsymb; i++)
      for (uint32_t k = 0; k < Qm; k++) {
        const uint32_t x = j * Qm + i * rows * Qm + k;
        if (!ri_at[x]) {
          if (idx == 0) x0 = x;
          g[idx++] = q[x];
        } else {
          any_ri = 1;
          if (x > xr) xr = x;
        }
      }
  if (any_ri) g[0] = q[xr > x0 ? xr : x0]; /* the last of the writes to g[0], in q order */
  if (O_cqi) {
    if (bcqi < 0) return -1;
    const uint32_t L = O_cqi < 11 ? 0 : 8;
    uint32_t x = 999999;
    if (K > 0) x = (uint32_t)ceilf((float)(O_cqi + L) * M_sc_init * nsymb * bcqi / K);
    const uint32_t lim = M_sc * nsymb - Q_ri;
    Q_cqi = x < lim ? x : lim;
    const uint32_t Q = Q_cqi * Qm;
    if (O_cqi <= 11) {
      if (Q > 32) {
        uint32_t i = 1;
        for (; i < Q / 32; i++)
          for (int k = 0; k < 32; k++) g[k] = (int16_t)(g[k] + g[i * 32 + k]);
        for (uint32_t k = 0; k < Q % 32; k++) g[k] = (int16_t)(g[k] + g[i * 32 + k]);
      }
      const uint32_t len = Q < 32 ? Q : 32;
      uint32_t best = 0;
      int32_t bmax = INT32_MIN;
      for (uint32_t w = 0; w < (1u << O_cqi); w++) {
        int16_t cw[32];
        for (int i = 0; i < 32; i++) {
          uint32_t b = 0;
          for (uint32_t n = 0; n < O_cqi; n++) b ^= ((w >> (O_cqi - 1 - n)) & 1) & SRSGPU_CQI_BASIS[i][n];
          cw[i] = (int16_t)(2 * b - 1);
        }
        int16_t lane[16] = {0};
        uint32_t i = 0;
        for (; i + 16 <= len; i += 16)
          for (int k = 0; k < 16; k++) lane[k] = (int16_t)(lane[k] + (int16_t)(cw[i + k] * g[i + k]));
        int32_t corr = 0;
        for (int k = 0; k < 16; k++) corr += lane[k];
        for (; i < len; i++) corr += cw[i] * g[i];
        if (corr > bmax) {
          bmax = corr;
          best = w;
        }
      }
      for (uint32_t n = 0; n < O_cqi; n++) out[4 + n] = (uint8_t)((best >> (O_cqi - 1 - n)) & 1);
    } else {
      /* srslte_rm_conv_rx_s (rm_conv.c:166-223) to 3 (O + 8) soft bits */
      const uint32_t out_len = 3 * (O_cqi + 8);
      const int nrows = (int)((out_len / 3 - 1) / 32 + 1), K_p = nrows * 32;
      int ndummy = K_p - (int)(out_len / 3);
      if (ndummy < 0) ndummy = 0;
      int16_t tmp[3 * 32 * 32], rm[3 * 200];
      for (int i = 0; i < 3 * K_p; i++) tmp[i] = 10000;
      uint32_t k = 0;
      int j = 0;
      while (k < Q) {
        const int d_i = (j % K_p) / nrows, d_j = (j % K_p) % nrows;
        if (d_j * 32 + RM_PERM_CC[d_i] >= ndummy) {
          if (tmp[j] == 10000)
            tmp[j] = g[k];
          else if (g[k] != 10000)
            tmp[j] = (int16_t)(tmp[j] + g[k]);
          k++;
        }
        if (++j == 3 * K_p) j = 0;
      }
      for (uint32_t i = 0; i < out_len / 3; i++) {
        const int d_i = (int)(i + ndummy) / 32, d_j = (int)(i + ndummy) % 32;
        for (int s = 0; s < 3; s++) {
          const int16_t o = tmp[K_p * s + RM_PERM_CC_INV[d_j] * nrows + d_i];
          rm[i * 3 + s] = o != 10000 ? o : 0;
        }
      }
      uint8_t bits[200];
      if (orc_viterbi37_tb_decode_s(rm, O_cqi + 8, bits)) return -1;
      if (orc_crc8_bits(bits, O_cqi + 8) == 0) {
        out[3] = 1;
        memcpy(out + 4, bits, O_cqi);
      }
    }
  }
  qp[0] = Q_ack;
  qp[1] = Q_ri;
  qp[2] = Q_cqi;
  free(q);
  free(ri_at);
  return 0;
}

/* ---------------------------------------------------------------- TM3 / TM4 feedback ---------- */
/* srslte_precoding_pmi_select_1l_avx / _2l_avx (src/phy/mimo/precoding.c:2335-2450, 2699-2845) with
 * LV_HAVE_FMA: the complex products of simd.h:64-91 (PROD = fmaddsub(a, ldup(b), swap(a) * hdup(b)),
 * PROD_ADD / PROD_SUB with the inner fmaddsub / fmsubadd), four estimates every 96, 24 apart, summed in
 * the reference's order; _mm256_rcp_ps restated as an exact reciprocal (the reference's is approximate).
 * srslte_precoding_2x2_cn_gen + srslte_mat_2x2_cn (:2889-2912, utils/mat.c:107-127). The rank / PMI
 * choices of srslte_ue_dl_ri_select / srslte_ue_dl_ri_pmi_select (src/phy/ue/ue_dl.c:684-764). */
typedef struct {
  float r, i;
} ocf;
static ocf oc_ld(const float *p, uint32_t k) {
  ocf v = {0.f, 0.f};
  if (p) {
    v.r = p[2 * k];
    v.i = p[2 * k + 1];
  }
  return v;
}
static ocf oc_cj(ocf a) { return (ocf){a.r, -a.i}; }
static ocf oc_mulj(ocf a) { return (ocf){-a.i, a.r}; }
static ocf oc_add(ocf a, ocf b) { return (ocf){a.r + b.r, a.i + b.i}; }
static ocf oc_sub(ocf a, ocf b) { return (ocf){a.r - b.r, a.i - b.i}; }
static ocf oc_prod(ocf a, ocf b) { return (ocf){fmaf(a.r, b.r, -(a.i * b.i)), fmaf(a.i, b.r, a.r * b.i)}; }
static ocf oc_prod_add(ocf a, ocf b, ocf c) {
  const float ur = fmaf(a.i, b.i, -c.r), ui = fmaf(a.r, b.i, c.i);
  return (ocf){fmaf(a.r, b.r, -ur), fmaf(a.i, b.r, ui)};
}
static ocf oc_prod_sub(ocf a, ocf b, ocf c) {
  const float ur = fmaf(a.i, b.i, c.r), ui = fmaf(a.r, b.i, -c.i);
  return (ocf){fmaf(a.r, b.r, -ur), fmaf(a.i, b.r, ui)};
}

#define ORC_PMI_PREC 24

static float orc_pmi_1l(const float *const h[2][2], uint32_t nof_ce, float noise, int cb) {
  float s = 0.f;
  uint32_t count = 0;
  for (uint32_t j = 0; j < nof_ce - ORC_PMI_PREC * 4 + 1; j += ORC_PMI_PREC * 4) {
    float g[4];
    for (int k = 0; k < 4; k++) {
      const uint32_t p = j + ORC_PMI_PREC * k;
      const ocf h00 = oc_ld(h[0][0], p), h01 = oc_ld(h[1][0], p), h10 = oc_ld(h[0][1], p), h11 = oc_ld(h[1][1], p);
      ocf a0, a1, c;
      if (cb == 0) {
        a0 = oc_add(oc_cj(h00), oc_cj(h01));
        a1 = oc_add(oc_cj(h10), oc_cj(h11));
      } else if (cb == 1) {
        a0 = oc_sub(oc_cj(h00), oc_cj(h01));
        a1 = oc_sub(oc_cj(h10), oc_cj(h11));
      } else if (cb == 2) {
        a0 = oc_sub(oc_cj(h00), oc_mulj(oc_cj(h01)));
        a1 = oc_sub(oc_cj(h10), oc_mulj(oc_cj(h11)));
      } else {
        a0 = oc_add(oc_cj(h00), oc_mulj(oc_cj(h01)));
        a1 = oc_add(oc_cj(h10), oc_mulj(oc_cj(h11)));
      }
      const ocf b0 = oc_prod_add(a0, h00, oc_prod(a1, h10)), b1 = oc_prod_add(a0, h01, oc_prod(a1, h11));
      c = cb == 0 ? oc_add(b0, b1) : cb == 1 ? oc_sub(b0, b1) : cb == 2 ? oc_add(b0, oc_mulj(b1)) : oc_sub(b0, oc_mulj(b1));
      g[k] = c.r * 0.5f;
    }
    s += g[0] + g[1] + g[2] + g[3];
    count += 4;
  }
  return s / (noise * (float)count);
}

static float orc_pmi_2l(const float *const h[2][2], uint32_t nof_ce, float noise, int cb) {
  float s = 0.f;
  uint32_t count = 0;
  for (uint32_t j = 0; j < nof_ce - ORC_PMI_PREC * 4 + 1; j += ORC_PMI_PREC * 4) {
    float v[4];
    for (int k = 0; k < 4; k++) {
      const uint32_t p = j + ORC_PMI_PREC * k;
      const ocf h00 = oc_ld(h[0][0], p), h01 = oc_ld(h[1][0], p), h10 = oc_ld(h[0][1], p), h11 = oc_ld(h[1][1], p);
      ocf a00, a01, a10, a11, c00, c01, c10, c11;
      if (cb == 0) {
        a00 = oc_add(oc_cj(h00), oc_cj(h01));
        a01 = oc_add(oc_cj(h10), oc_cj(h11));
        a10 = oc_sub(oc_cj(h00), oc_cj(h01));
        a11 = oc_sub(oc_cj(h10), oc_cj(h11));
      } else {
        a00 = oc_sub(oc_cj(h00), oc_mulj(oc_cj(h01)));
        a01 = oc_sub(oc_cj(h10), oc_mulj(oc_cj(h11)));
        a10 = oc_add(oc_cj(h00), oc_mulj(oc_cj(h01)));
        a11 = oc_add(oc_cj(h10), oc_mulj(oc_cj(h11)));
      }
      const ocf b00 = oc_prod_add(a00, h00, oc_prod(a01, h10)), b01 = oc_prod_add(a00, h01, oc_prod(a01, h11));
      const ocf b10 = oc_prod_add(a10, h00, oc_prod(a11, h10)), b11 = oc_prod_add(a10, h01, oc_prod(a11, h11));
      if (cb == 0) {
        c00 = oc_add(b00, b01);
        c01 = oc_sub(b00, b01);
        c10 = oc_add(b10, b11);
        c11 = oc_sub(b10, b11);
      } else {
        c00 = oc_add(b00, oc_mulj(b01));
        c01 = oc_sub(b00, oc_mulj(b01));
        c10 = oc_add(b10, oc_mulj(b11));
        c11 = oc_sub(b10, oc_mulj(b11));
      }
      c00 = (ocf){c00.r * 0.25f + noise, c00.i * 0.25f + 0.f};
      c01 = (ocf){c01.r * 0.25f, c01.i * 0.25f};
      c10 = (ocf){c10.r * 0.25f, c10.i * 0.25f};
      c11 = (ocf){c11.r * 0.25f + noise, c11.i * 0.25f + 0.f};
      const ocf det = oc_prod_sub(c00, c11, oc_prod(c01, c10));
      const float rc = 1.0f / (det.i * det.i + det.r * det.r);
      const ocf inv = {noise * (rc * det.r), 0.f * (rc * -det.i)};
      const ocf den0 = oc_prod(c00, inv), den1 = oc_prod(c11, inv);
      v[k] = (1.0f / den0.r - 1.f) + (1.0f / den1.r - 1.f);
    }
    s += v[0] + v[1] + v[2] + v[3];
    count += 4;
  }
  return count ? s / (float)count : s;
}

static float orc_cn_2x2(const float *const h[2][2], uint32_t nof_ce) {
  float acc = 0.f;
  uint32_t count = 0;
  for (uint32_t i = 0; i < nof_ce; i += ORC_PMI_PREC) {
    const ocf h00 = oc_ld(h[0][0], i), h01 = oc_ld(h[1][0], i), h10 = oc_ld(h[0][1], i), h11 = oc_ld(h[1][1], i);
    const float a00 = h00.r * h00.r + h01.r * h01.r + h00.i * h00.i + h01.i * h01.i;
    const float a01r = (h00.r * h10.r - h00.i * -h10.i) + (h01.r * h11.r - h01.i * -h11.i);
    const float a01i = (h00.r * -h10.i + h00.i * h10.r) + (h01.r * -h11.i + h01.i * h11.r);
    const float a11 = h10.r * h10.r + h11.r * h11.r + h10.i * h10.i + h11.i * h11.i;
    const float b = a00 + a11, c = a00 * a11 - (a01r * a01r + a01i * a01i);
    const float sqr = sqrtf(b * b - 4.0f * c);
    acc += 10 * log10f((b + sqr) / (b - sqr));
    count++;
  }
  return count ? acc / (float)count : acc;
}

/* h[port][rx] estimate planes (complex float pairs; NULL = the zero plane of an absent rx antenna).
 * out_i: ri_tm3, ret_cn, ri, pmi, pmi_l0, pmi_l1, ret_pmi; sinr[2][4] */
int orc_feedback(const float *h00, const float *h01, const float *h10, const float *h11, uint32_t nof_ce, float noise,
                 uint32_t flags, int nports, int nrx, float *out_cn, int32_t *out_i, float *sinr) {
  const float *const h[2][2] = {{h00, h10}, {h01, h11}};
  const int do_pmi = (flags & 2u) && nports == 2, do_cn = (flags & 1u) && nports == 2 && nrx == 2;
  float cn = do_cn ? orc_cn_2x2(h, nof_ce) : 0.f;
  for (int c = 0; c < 4; c++) {
    sinr[c] = do_pmi ? orc_pmi_1l(h, nof_ce, noise, c) : 0.f;
    sinr[4 + c] = !do_pmi ? 0.f : nrx < 2 ? -INFINITY : c < 2 ? orc_pmi_2l(h, nof_ce, noise, c) : 0.f;
  }
  uint32_t pmi_l[2] = {0, 0};
  for (int L = 0; L < 2; L++) {
    float mx = 0.f;
    for (int c = 0; c < (L ? 2 : 4); c++)
      if (sinr[4 * L + c] > mx) {
        mx = sinr[4 * L + c];
        pmi_l[L] = (uint32_t)c;
      }
  }
  float best = -INFINITY;
  uint32_t best_ri = 0, best_pmi = 0;
  if (do_pmi)
    for (uint32_t L = 1; L <= 4; L++) {
      const float s = L <= 2 ? sinr[4 * (L - 1) + pmi_l[L - 1]] : -INFINITY;
      const float v = s * L * L;
      if (v > best + 0.1 || v > 1.0e+3) {
        best = v;
        best_pmi = L <= 2 ? pmi_l[L - 1] : 0;
        best_ri = L - 1;
      }
    }
  *out_cn = cn;
  out_i[0] = do_cn ? (cn < 17.0f ? 1 : 0) : 0;
  out_i[1] = do_cn ? 0 : -1;
  out_i[2] = (int32_t)best_ri;
  out_i[3] = (int32_t)best_pmi;
  out_i[4] = (int32_t)pmi_l[0];
  out_i[5] = (int32_t)pmi_l[1];
  out_i[6] = do_pmi ? 0 : -1;
  return 0;
}
