/*
 * CPU ORACLE — TEST INFRASTRUCTURE ONLY (see tdec_oracle.c for the rules).
 *
 * Scalar restatement of the srsLTE 18.09 8-bit turbo decoding path (paths relative to
 * /root/reference/lib):
 *   * srslte_tdec_iteration_8bit / srslte_tdec_run_all_8bit (src/phy/fec/turbodecoder.c:392-563):
 *     AUTO picks the 32-sub-block AVX8 window decoder for K % 32 == 0 && K > 2048, the
 *     16-sub-block SSE8 one for K % 16 == 0 && K > 800, and otherwise sign-extends the input to
 *     int16 and runs the 16-bit AUTO decoder (tdec_iteration_8, :439-464);
 *   * the int8 window decoders, WINIMP sse8 / avx8 of include/srslte/phy/fec/turbodecoder_win.h
 *     (:97-178 parameters): saturating int8 adds, "-INF" = 0 (so every unknown and every known
 *     start state is 0), normalisation by the maximum state every step (k != 0, :244-261), output
 *     (m1 - m0) shifted right by one (:565-567, simd_rb_shift), tail trellis with the scalar
 *     sadd of :196-203 (saturates upwards only, wraps downwards);
 *   * the half-iteration glue run_tdec_iteration_8bit (include/.../turbodecoder_iter.h:73-147
 *     with LLR_IS_8BIT): srslte_vec_sub_bbb is _mm256_subs_epi8 over the first K & ~31
 *     elements and a wrapping C subtraction for the rest (src/phy/utils/vector_simd.c:165-191,
 *     AVX2 build, 32-byte aligned buffers).
 * Pinned against the reference compiled from its own sources (tests/test_tdec8.py).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "tdec_oracle.h"

#define B_OVERLAP 40 /* turbodecoder_win.h: win_overlap_len of sse8 / avx8 */

static inline int8_t sat8(int v) { return (int8_t)(v > 127 ? 127 : (v < -128 ? -128 : v)); }
static inline int8_t adds8(int8_t a, int8_t b) { return sat8((int)a + b); }
static inline int8_t subs8(int8_t a, int8_t b) { return sat8((int)a - b); }
static inline int8_t max8(int8_t a, int8_t b) { return a > b ? a : b; }
/* turbodecoder_win.h:196-203 MAKE_FUNC(sadd) with use_saturated_add: z > 127 ? 127 : (int8_t) z */
static inline int8_t tail_add8(int8_t a, int8_t b) {
  int16_t z = (int16_t)((int16_t)a + b);
  return z > 127 ? 127 : (int8_t)z;
}

typedef struct {
  int8_t s[8];
} bst8;

/* :244-261 normalize with normalize_max, normalize_period 1 */
static void b_normalize(int k, bst8 *o) {
  if (k != 0) {
    int8_t m = o->s[0];
    for (int i = 1; i < 8; i++) m = max8(m, o->s[i]);
    for (int i = 0; i < 8; i++) o->s[i] = subs8(o->s[i], m);
  }
}

/* :395-418 with int8 saturating adds */
static void b_beta_step(bst8 *o, int8_t x, int8_t y) {
  const int8_t *b = o->s;
  int8_t xy = adds8(x, y);
  int8_t mb[8] = {adds8(b[4], xy), b[4], adds8(b[5], y), adds8(b[5], x),
                  adds8(b[6], x), adds8(b[6], y), b[7], adds8(b[7], xy)};
  int8_t nw[8] = {b[0], adds8(b[0], xy), adds8(b[1], x), adds8(b[1], y),
                  adds8(b[2], y), adds8(b[2], x), adds8(b[3], xy), b[3]};
  for (int i = 0; i < 8; i++) o->s[i] = max8(mb[i], nw[i]);
}

/* :521-539 */
static void b_alpha_branches(const bst8 *o, int8_t x, int8_t y, int8_t mb[8], int8_t nw[8]) {
  const int8_t *a = o->s;
  int8_t xy = adds8(x, y);
  mb[0] = a[0];
  mb[1] = adds8(a[3], y);
  mb[2] = adds8(a[4], y);
  mb[3] = a[7];
  mb[4] = a[1];
  mb[5] = adds8(a[2], y);
  mb[6] = adds8(a[5], y);
  mb[7] = a[6];
  nw[0] = adds8(a[1], xy);
  nw[1] = adds8(a[2], x);
  nw[2] = adds8(a[5], x);
  nw[3] = adds8(a[6], xy);
  nw[4] = adds8(a[0], xy);
  nw[5] = adds8(a[3], x);
  nw[6] = adds8(a[4], x);
  nw[7] = adds8(a[7], xy);
}

/* :263-307 beta_trellis: old = {0, -INF...} = all 0 (INF = 0), 3 tail steps, scalar sadd */
static void b_tail_trellis(const int8_t *xin, const int8_t *par, uint32_t K, bst8 *o) {
  memset(o->s, 0, 8);
  for (int k = (int)K + 2; k >= (int)K; k--) {
    int8_t x = xin[k], y = par[k], xy = tail_add8(x, y);
    const int8_t *b = o->s;
    int8_t mb[8] = {tail_add8(b[4], xy), b[4], tail_add8(b[5], y), tail_add8(b[5], x),
                    tail_add8(b[6], x), tail_add8(b[6], y), b[7], tail_add8(b[7], xy)};
    int8_t nw[8] = {b[0], tail_add8(b[0], xy), tail_add8(b[1], x), tail_add8(b[1], y),
                    tail_add8(b[2], y), tail_add8(b[2], x), tail_add8(b[3], xy), b[3]};
    for (int i = 0; i < 8; i++) o->s[i] = mb[i] > nw[i] ? mb[i] : nw[i];
  }
}

/* :614-622 dec = beta (:310-435) then alpha (:438-586), in SB index space (k*nb+d = step k of
 * sub-block d); xin / par carry the 3 tail values at [K..K+2]; beta_buf holds (L+1)*nb*8 */
static void b_win_dec(int nb, const int8_t *xin, const int8_t *app, const int8_t *par, int8_t *out,
                      uint32_t K, int8_t *beta_buf) {
  const int L = (int)(K / nb);
#define XIN(i) (app ? adds8(app[(i)], xin[(i)]) : xin[(i)])
  bst8 tail;
  b_tail_trellis(xin, par, K, &tail);
  for (int d = 0; d < nb; d++) {
    bst8 o;
    if (d == nb - 1) {
      o = tail;
    } else {
      memset(o.s, 0, 8); /* -INF = 0 */
      for (int k = B_OVERLAP - 1; k >= 0; k--) {
        int idx = k * nb + d + 1;
        b_beta_step(&o, XIN(idx), par[idx]);
        b_normalize(k, &o);
      }
    }
    memcpy(&beta_buf[((size_t)L * nb + d) * 8], o.s, 8);
    for (int k = L - 1; k >= 0; k--) {
      int idx = k * nb + d;
      b_beta_step(&o, XIN(idx), par[idx]);
      memcpy(&beta_buf[((size_t)k * nb + d) * 8], o.s, 8);
      b_normalize(k, &o);
    }
  }
  for (int d = 0; d < nb; d++) {
    bst8 o;
    memset(o.s, 0, 8); /* d == 0: state 0 known = 0, the others -INF = 0 */
    if (d > 0) {
      for (int k = 0; k < B_OVERLAP; k++) {
        int idx = (L - B_OVERLAP + k) * nb + d - 1;
        int8_t mb[8], nw[8];
        b_alpha_branches(&o, XIN(idx), par[idx], mb, nw);
        for (int i = 0; i < 8; i++) o.s[i] = max8(mb[i], nw[i]);
        b_normalize(k, &o);
      }
    }
    for (int k = 0; k < L; k++) {
      int idx = k * nb + d;
      int8_t mb[8], nw[8];
      b_alpha_branches(&o, XIN(idx), par[idx], mb, nw);
      const int8_t *be = &beta_buf[((size_t)(k + 1) * nb + d) * 8];
      int8_t m0 = adds8(be[0], mb[0]), m1 = adds8(be[0], nw[0]);
      for (int i = 1; i < 8; i++) {
        m0 = max8(m0, adds8(be[i], mb[i]));
        m1 = max8(m1, adds8(be[i], nw[i]));
      }
      out[idx] = (int8_t)(subs8(m1, m0) >> 1); /* simd_rb_shift(out, 1) */
      for (int i = 0; i < 8; i++) o.s[i] = max8(mb[i], nw[i]);
      b_normalize(k, &o);
    }
  }
#undef XIN
}

/* srslte_vec_sub_bbb (AVX2, aligned): saturating below K & ~31, wrapping above */
static void b_vec_sub(const int8_t *x, const int8_t *y, int8_t *z, uint32_t K) {
  const uint32_t K32 = K & ~31u;
  for (uint32_t i = 0; i < K; i++)
    z[i] = i < K32 ? subs8(x[i], y[i]) : (int8_t)(uint8_t)((int)x[i] - y[i]);
}

uint32_t orc_autoimp_subblocks_8bit(uint32_t K) {
  if (!(K % 32) && K > 2048) return 32;
  if (!(K % 16) && K > 800) return 16;
  if (!(K % 8) && K > 400) return 8;
  return 0;
}

/* one 8-bit window decoder run over a CB, nof_halfits half-iterations (turbodecoder_iter.h) */
static int b_run(int nb, int sb_input, const int8_t *in, uint32_t K, uint32_t nof_halfits,
                 uint8_t *decisions) {
  const uint32_t L = K / nb;
  size_t len = K + 16;
  int8_t *syst = calloc(len, 1), *par0 = calloc(len, 1), *par1 = calloc(len, 1);
  int8_t *app1 = calloc(len, 1), *app2 = calloc(len, 1), *ext1 = calloc(len, 1),
         *ext2 = calloc(len, 1);
  int8_t *beta = calloc((size_t)(L + 1) * nb * 8, 1);
  uint16_t *fwd = calloc(K, 2), *rev = calloc(K, 2);
  int ret = orc_interl(K, (uint32_t)nb, fwd, rev);
  if (ret == 0) {
    /* turbodecoder_iter.h:91-108 */
    if (sb_input) {
      for (uint32_t i = 0; i < K; i++) {
        syst[i] = in[i];
        par0[i] = in[(K + 32) + i];
        par1[i] = in[2 * (K + 32) + i];
      }
      for (uint32_t j = 0; j < 3; j++) {
        syst[K + j] = in[3 * (K + 32) + 2 * j];
        par0[K + j] = in[3 * (K + 32) + 2 * j + 1];
        app2[K + j] = in[3 * (K + 32) + 6 + 2 * j];
        par1[K + j] = in[3 * (K + 32) + 6 + 2 * j + 1];
      }
    } else { /* turbodecoder_win.h:634-674 */
      for (uint32_t p = 0; p < K; p++) {
        uint32_t idx = (p % L) * nb + p / L;
        syst[idx] = in[3 * p];
        par0[idx] = in[3 * p + 1];
        par1[idx] = in[3 * p + 2];
      }
      for (uint32_t j = 0; j < 3; j++) {
        syst[K + j] = in[3 * K + 2 * j];
        par0[K + j] = in[3 * K + 2 * j + 1];
        app2[K + j] = in[3 * K + 6 + 2 * j];
        par1[K + j] = in[3 * K + 6 + 2 * j + 1];
      }
    }
    for (uint32_t n = 0; n < nof_halfits; n++) {
      if ((n % 2) == 0) {
        if (n) b_vec_sub(app1, ext1, app1, K);
        b_win_dec(nb, syst, n ? app1 : NULL, par0, ext1, K, beta);
      } else {
        if (n > 1) b_vec_sub(ext1, app1, ext1, K);
        for (uint32_t i = 0; i < K; i++) app2[rev[i]] = ext1[i];
        b_win_dec(nb, app2, NULL, par1, ext2, K, beta);
        for (uint32_t i = 0; i < K; i++) app1[fwd[i]] = ext2[i];
      }
      if (decisions) { /* turbodecoder.c:353-360: ext1 after DEC1, app1 after DEC2 */
        const int8_t *v = (n % 2) ? app1 : ext1;
        uint8_t *ob = decisions + (size_t)n * (K / 8);
        for (uint32_t i = 0; i < K / 8; i++) {
          uint8_t byte = 0;
          for (uint32_t j = 0; j < 8; j++) {
            uint32_t p = 8 * i + j;
            if (v[(p % L) * nb + p / L] > 0) byte |= (uint8_t)(0x80 >> j);
          }
          ob[i] = byte;
        }
      }
    }
  }
  free(syst); free(par0); free(par1); free(app1); free(app2); free(ext1); free(ext2);
  free(beta); free(fwd); free(rev);
  return ret;
}

/* srslte_tdec_init_manual(impl) [+ force_not_sb when !sb_layout] + new_cb(K) + nof_halfits x
 * srslte_tdec_iteration_8bit; decisions after every half-iteration (nof_halfits * K/8 bytes).
 * Returns -2 where the reference has no defined result: AUTO with sub-block input at
 * 400 < K <= 800 (it converts only 3K+12 int8 values but reads the sub-block layout's
 * 3(K+32)+12, :459) and the manual window types, 8- and 16-bit (tdec_iteration_8 never sets
 * current_inter_idx outside AUTO, :451-453, so the reference dereferences the unset 1-sub-block
 * interleaver slot). */
int orc_tdec8_run(int impl, int sb_layout, const int8_t *input, uint32_t K, uint32_t nof_halfits,
                  uint8_t *decisions) {
  int idx = orc_cbindex(K);
  if (idx < 0) return -1;
  int nb8 = 0, conv16 = 0;
  if (impl == ORC_TDEC_AUTO) {
    uint32_t s = orc_autoimp_subblocks_8bit(K);
    if (s >= 16) {
      nb8 = (int)s;
    } else {
      if (s == 8 && sb_layout) return -2;
      conv16 = 1;
    }
  } else if (impl == ORC_TDEC_SSE8_WINDOW || impl == ORC_TDEC_AVX8_WINDOW ||
             impl == ORC_TDEC_SSE_WINDOW || impl == ORC_TDEC_AVX_WINDOW) {
    return -2; /* interleaver index left at 0 (1 sub-block): the reference faults */
  } else {
    conv16 = 1; /* manual 16-bit decoder: natural input (input_is_interleaved = current_dec > 0) */
    sb_layout = 0;
  }
  if (conv16) {
    size_t n = 3 * (size_t)K + 12;
    int16_t *w = malloc(n * 2);
    for (size_t i = 0; i < n; i++) w[i] = input[i]; /* convert_8_to_16, :425-430 */
    int r = orc_tdec_run(impl, sb_layout, w, K, nof_halfits, decisions, NULL, NULL);
    free(w);
    return r;
  }
  if (K % nb8 || K / nb8 <= B_OVERLAP) return -1;
  return b_run(nb8, sb_layout, input, K, nof_halfits, decisions);
}

/* the manual 8-bit window types driven through the 16-bit entry point (srslte_tdec_iteration,
 * tdec_iteration_16 :491-503): input truncated to int8 (convert_16_to_8), natural layout only
 * (with sub-block input the reference converts 3K+12 values of a 3(K+32)+12 layout) */
int orc_tdec8_run16(int impl, const int16_t *input, uint32_t K, uint32_t nof_halfits,
                    uint8_t *decisions) {
  const int nb = impl == ORC_TDEC_AVX8_WINDOW ? 32 : impl == ORC_TDEC_SSE8_WINDOW ? 16 : 0;
  if (!nb || orc_cbindex(K) < 0 || K % nb || K / nb <= B_OVERLAP) return -1;
  size_t n = 3 * (size_t)K + 12;
  int8_t *w = malloc(n);
  for (size_t i = 0; i < n; i++) w[i] = (int8_t)input[i];
  int r = b_run(nb, 0, w, K, nof_halfits, decisions);
  free(w);
  return r;
}
