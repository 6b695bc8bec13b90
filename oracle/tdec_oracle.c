/*
 * CPU ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Scalar C99 restatement of the srsLTE 18.09 turbo-decoder family and its helpers, written
 * from a reading of the reference (paths relative to /root/reference/lib). It is the parity
 * checker for the MI355X HIP path: only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it. The product library never links or calls it.
 *
 * Pinning: every function here is checked bit-exactly against the reference compiled from
 * its own sources (oracle/Makefile target `ref`, oracle/_ref/libsrsref.so) and against the
 * committed golden vectors in tests/golden/ (generated from that build by
 * tests/golden/make_golden.py).
 *
 * Arithmetic conventions (all on int16):
 *   sat_*  : saturating, like _mm*_adds_epi16/_subs_epi16 (windowed decoders)
 *   wrap_* : modulo 2^16, like _mm*_add_epi16 and plain C int16 stores (SSE/generic decoders)
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "srsgpu/qpp_table.h"
#include "tdec_oracle.h"

#define ORC_INF 10000 /* turbodecoder_win.h:63, turbodecoder_sse.c:51, turbodecoder_gen.c:41 */
#define ORC_WIN_OVERLAP 40 /* turbodecoder_win.h:59 win_overlap_len */

static inline int16_t sat16(int32_t v) {
  return (int16_t)(v > 32767 ? 32767 : (v < -32768 ? -32768 : v));
}
static inline int16_t sat_add(int16_t a, int16_t b) { return sat16((int32_t)a + b); }
static inline int16_t sat_sub(int16_t a, int16_t b) { return sat16((int32_t)a - b); }
static inline int16_t wrap16(int32_t v) { return (int16_t)(uint16_t)(uint32_t)v; }
static inline int16_t max16(int16_t a, int16_t b) { return a > b ? a : b; }

/* ---------------------------------------------------------------- code-block sizes ---- */

/* cbsegm.c:110-121 srslte_cbsegm_cbindex: smallest table index with K >= long_cb */
int orc_cbindex(uint32_t long_cb) {
  for (int j = 0; j < SRSGPU_NOF_CB_SIZES; j++) {
    if (srsgpu_qpp_table[j][0] >= long_cb) return j;
  }
  return -1;
}

int orc_cbsize(uint32_t idx) {
  return idx < SRSGPU_NOF_CB_SIZES ? (int)srsgpu_qpp_table[idx][0] : -1;
}

/* cbsegm.c:58-104 srslte_cbsegm (TS 36.212 5.1.2), F must be 0 for the DL-SCH decoder */
int orc_cbsegm(uint32_t tbs, uint32_t *C, uint32_t *C1, uint32_t *K1, uint32_t *C2,
               uint32_t *K2, uint32_t *F) {
  if (tbs == 0) {
    *C = *C1 = *K1 = *C2 = *K2 = *F = 0;
    return 0;
  }
  uint32_t B = tbs + 24, Bp, c;
  if (B <= 6144) {
    c = 1;
    Bp = B;
  } else {
    /* the reference uses ceilf((float)B/6120); B < 2^24 so the float quotient is exact enough */
    c = (B + 6120 - 1) / 6120;
    Bp = B + 24 * c;
  }
  int i1 = orc_cbindex((Bp - 1) / c + 1);
  if (i1 < 0) return -1;
  uint32_t k1 = srsgpu_qpp_table[i1][0];
  uint32_t k2 = i1 > 0 ? srsgpu_qpp_table[i1 - 1][0] : k1;
  *C = c;
  *K1 = k1;
  if (c == 1) {
    *K2 = 0;
    *C2 = 0;
    *C1 = 1;
  } else {
    *K2 = k2;
    *C2 = (c * k1 - Bp) / (k1 - k2);
    *C1 = c - *C2;
  }
  *F = *C1 * *K1 + *C2 * *K2 - Bp;
  return 0;
}

/* ---------------------------------------------------------------- QPP interleaver ---- */

/* tc_interl_lte.c:78-119: pi(i) = (f1*i + f2*i^2) mod K. With nsb > 1 the tables are
 * re-expressed in sub-block (SB) index space, where SB index k*nsb+d holds natural
 * position d*(K/nsb)+k. fwd[i] = pi, rev = pi^-1 (both in the chosen index space). */
int orc_interl(uint32_t K, uint32_t nsb, uint16_t *fwd, uint16_t *rev) {
  int idx = orc_cbindex(K);
  if (idx < 0 || srsgpu_qpp_table[idx][0] != K) return -1;
  uint64_t f1 = srsgpu_qpp_table[idx][1], f2 = srsgpu_qpp_table[idx][2];
  uint16_t *f = malloc(K * sizeof(uint16_t)), *r = malloc(K * sizeof(uint16_t));
  for (uint64_t i = 0; i < K; i++) {
    uint32_t j = (uint32_t)((f1 * i + f2 * i * i) % K);
    f[i] = (uint16_t)j;
    r[j] = (uint16_t)i;
  }
  if (nsb <= 1) {
    memcpy(fwd, f, K * 2);
    memcpy(rev, r, K * 2);
  } else {
    uint32_t L = K / nsb;
    for (uint32_t i = 0; i < K; i++) {
      uint32_t nat = (i % nsb) * L + i / nsb;   /* SB index -> natural position */
      uint32_t jf = f[nat], jr = r[nat];
      fwd[i] = (uint16_t)((jf % L) * nsb + jf / L); /* natural -> SB index */
      rev[i] = (uint16_t)((jr % L) * nsb + jr / L);
    }
  }
  free(f);
  free(r);
  return 0;
}

/* ---------------------------------------------------------------- windowed MAP ---- */
/* turbodecoder_win.h: WINIMP sse16 (nb=8, output >>1) and avx16 (nb=16). Lane d of the
 * reference SIMD register = sub-block d; here each sub-block is walked as a scalar chain. */

typedef struct {
  int16_t s[8];
} st8;

/* turbodecoder_win.h:244-261 normalize (16-bit: subtract state 0, every 2 steps, k != 0) */
static inline void win_normalize(int k, st8 *o) {
  if ((k % 2) == 0 && k != 0) {
    for (int i = 1; i < 8; i++) o->s[i] = sat_sub(o->s[i], o->s[0]);
    o->s[0] = 0;
  }
}

/* turbodecoder_win.h:397-417 one backward (beta) trellis step */
static inline void win_beta_step(st8 *o, int16_t x, int16_t y) {
  int16_t xy = sat_add(x, y);
  const int16_t *b = o->s;
  int16_t mb[8] = {sat_add(b[4], xy), b[4], sat_add(b[5], y), sat_add(b[5], x),
                   sat_add(b[6], x), sat_add(b[6], y), b[7], sat_add(b[7], xy)};
  int16_t nw[8] = {b[0], sat_add(b[0], xy), sat_add(b[1], x), sat_add(b[1], y),
                   sat_add(b[2], y), sat_add(b[2], x), sat_add(b[3], xy), b[3]};
  for (int i = 0; i < 8; i++) o->s[i] = max16(mb[i], nw[i]);
}

/* turbodecoder_win.h:521-539 forward (alpha) branch sums; m_b = input bit 0, nw = bit 1 */
static inline void win_alpha_branches(const st8 *o, int16_t x, int16_t y, int16_t mb[8],
                                      int16_t nw[8]) {
  int16_t xy = sat_add(x, y);
  const int16_t *a = o->s;
  mb[0] = a[0];
  mb[1] = sat_add(a[3], y);
  mb[2] = sat_add(a[4], y);
  mb[3] = a[7];
  mb[4] = a[1];
  mb[5] = sat_add(a[2], y);
  mb[6] = sat_add(a[5], y);
  mb[7] = a[6];
  nw[0] = sat_add(a[1], xy);
  nw[1] = sat_add(a[2], x);
  nw[2] = sat_add(a[5], x);
  nw[3] = sat_add(a[6], xy);
  nw[4] = sat_add(a[0], xy);
  nw[5] = sat_add(a[3], x);
  nw[6] = sat_add(a[4], x);
  nw[7] = sat_add(a[7], xy);
}

/* turbodecoder_win.h:263-307 beta_trellis: 3 tail steps, plain (wrapping) int16 adds */
static void win_tail_trellis(const int16_t *xin, const int16_t *par, uint32_t K, st8 *o) {
  o->s[0] = 0;
  for (int i = 1; i < 8; i++) o->s[i] = -ORC_INF;
  for (int k = (int)K + 2; k >= (int)K; k--) {
    int16_t x = xin[k], y = par[k], xy = wrap16(x + y);
    const int16_t *b = o->s;
    int16_t mb[8] = {wrap16(b[4] + xy), b[4], wrap16(b[5] + y), wrap16(b[5] + x),
                     wrap16(b[6] + x), wrap16(b[6] + y), b[7], wrap16(b[7] + xy)};
    int16_t nw[8] = {b[0], wrap16(b[0] + xy), wrap16(b[1] + x), wrap16(b[1] + y),
                     wrap16(b[2] + y), wrap16(b[2] + x), wrap16(b[3] + xy), b[3]};
    for (int i = 0; i < 8; i++) o->s[i] = max16(mb[i], nw[i]);
  }
}

/* turbodecoder_win.h:614-622 MAKE_FUNC(dec) = beta (:310-435) then alpha (:438-586).
 * Buffers are in SB index space: element k*nb+d = step k of sub-block d. xin/par carry the 3
 * tail values at [K..K+2]. app may be NULL. beta_buf holds (L+1)*nb*8 int16. */
static void win_dec(int nb, int div_out, const int16_t *xin, const int16_t *app,
                    const int16_t *par, int16_t *out, uint32_t K, int16_t *beta_buf) {
  const int L = (int)(K / nb);
#define XIN(i) (app ? sat_add(app[(i)], xin[(i)]) : xin[(i)])
  st8 tail;
  win_tail_trellis(xin, par, K, &tail);

  /* ---- beta ---- */
  for (int d = 0; d < nb; d++) {
    st8 o;
    if (d == nb - 1) {
      o = tail; /* :350-355 last sub-block starts from the tail trellis */
    } else {
      /* :376-384 + :386-433 with loop_len = 40: estimate the state at the start of
       * sub-block d+1 from its first 40 steps, entered from all-unknown states; :333-366
       * move_right hands it to sub-block d. */
      for (int i = 0; i < 8; i++) o.s[i] = -ORC_INF;
      for (int k = ORC_WIN_OVERLAP - 1; k >= 0; k--) {
        int idx = k * nb + (d + 1);
        win_beta_step(&o, XIN(idx), par[idx]);
        win_normalize(k, &o);
      }
    }
    int16_t *bp = &beta_buf[((size_t)L * nb + d) * 8]; /* :372-374 store beta[L] */
    memcpy(bp, o.s, 16);
    for (int k = L - 1; k >= 0; k--) {
      int idx = k * nb + d;
      win_beta_step(&o, XIN(idx), par[idx]);
      memcpy(&beta_buf[((size_t)k * nb + d) * 8], o.s, 16); /* :420-424 stored pre-normalise */
      win_normalize(k, &o);
    }
  }

  /* ---- alpha + LLR ---- */
  for (int d = 0; d < nb; d++) {
    st8 o;
    if (d == 0) {
      o.s[0] = 0; /* :496-500 first sub-block starts in state 0 */
      for (int i = 1; i < 8; i++) o.s[i] = -ORC_INF;
    } else {
      /* :501-506 + :512-584 with loop_len = 40 over the last 40 steps of sub-block d-1;
       * :469-495 move_left hands the estimate to sub-block d */
      for (int i = 0; i < 8; i++) o.s[i] = -ORC_INF;
      for (int k = 0; k < ORC_WIN_OVERLAP; k++) {
        int idx = (L - ORC_WIN_OVERLAP + k) * nb + (d - 1);
        int16_t mb[8], nw[8];
        win_alpha_branches(&o, XIN(idx), par[idx], mb, nw);
        for (int i = 0; i < 8; i++) o.s[i] = max16(mb[i], nw[i]);
        win_normalize(k, &o);
      }
    }
    for (int k = 0; k < L; k++) {
      int idx = k * nb + d;
      int16_t mb[8], nw[8];
      win_alpha_branches(&o, XIN(idx), par[idx], mb, nw);
      const int16_t *be = &beta_buf[((size_t)(k + 1) * nb + d) * 8]; /* :455 betaPtr += 8 */
      int16_t m0 = -32768, m1 = -32768;
      for (int i = 0; i < 8; i++) {
        m0 = max16(m0, sat_add(be[i], mb[i]));
        m1 = max16(m1, sat_add(be[i], nw[i]));
      }
      int16_t v = sat_sub(m1, m0);
      if (div_out) v = (int16_t)(v >> 1); /* :565-567 srai 1 (SSE16 window only) */
      out[idx] = v;
      for (int i = 0; i < 8; i++) o.s[i] = max16(mb[i], nw[i]);
      win_normalize(k, &o);
    }
  }
#undef XIN
}

/* ---------------------------------------------------------------- SSE non-window MAP ---- */
/* turbodecoder_sse.c:97-407. Branch metrics halved (srai 1) with wrapping adds, alpha stored
 * for the whole block, beta walked backwards producing the LLR. Natural index space.
 * scratch: branch 2*(K+3) + alpha 8*(K+1) int16. */
static void sse_dec(const int16_t *xin, const int16_t *app, const int16_t *par, int16_t *out,
                    uint32_t K, int16_t *scratch) {
  int16_t *g = scratch;               /* g[2i] = g0, g[2i+1] = g1 */
  int16_t *alpha = scratch + 2 * (K + 3);
  /* :300-353 tdec_sse_gamma */
  for (uint32_t i = 0; i < K; i++) {
    int16_t in = app ? wrap16(xin[i] + app[i]) : xin[i];
    g[2 * i + 1] = (int16_t)(wrap16(in + par[i]) >> 1);
    g[2 * i] = (int16_t)(wrap16(in - par[i]) >> 1);
  }
  for (uint32_t i = K; i < K + 3; i++) { /* :349-352 C division (truncation), no app */
    g[2 * i] = (int16_t)(((int32_t)xin[i] - par[i]) / 2);
    g[2 * i + 1] = (int16_t)(((int32_t)xin[i] + par[i]) / 2);
  }
  /* :211-297 tdec_sse_alpha: stored after each step, renormalised (register only) every 4 */
  int16_t a[8] = {0, -ORC_INF, -ORC_INF, -ORC_INF, -ORC_INF, -ORC_INF, -ORC_INF, -ORC_INF};
  memcpy(alpha, a, 16);
  for (uint32_t k = 0; k < K; k++) {
    int16_t g0 = g[2 * k], g1 = g[2 * k + 1], n[8];
    n[0] = max16(wrap16(a[1] + g1), wrap16(a[0] - g1));
    n[1] = max16(wrap16(a[2] + g0), wrap16(a[3] - g0));
    n[2] = max16(wrap16(a[5] + g0), wrap16(a[4] - g0));
    n[3] = max16(wrap16(a[6] + g1), wrap16(a[7] - g1));
    n[4] = max16(wrap16(a[0] + g1), wrap16(a[1] - g1));
    n[5] = max16(wrap16(a[3] + g0), wrap16(a[2] - g0));
    n[6] = max16(wrap16(a[4] + g0), wrap16(a[5] - g0));
    n[7] = max16(wrap16(a[7] + g1), wrap16(a[6] - g1));
    memcpy(a, n, 16);
    memcpy(&alpha[8 * (k + 1)], a, 16);
    if ((k % 4) == 3) { /* :286-295 subtract state 0 (wrapping) after every 4th step */
      int16_t a0 = a[0];
      for (int i = 0; i < 8; i++) a[i] = wrap16(a[i] - a0);
    }
  }
  /* :105-206 tdec_sse_beta */
  int16_t b[8] = {0, -ORC_INF, -ORC_INF, -ORC_INF, -ORC_INF, -ORC_INF, -ORC_INF, -ORC_INF};
  for (int k = (int)K + 2; k >= 0; k--) {
    int16_t g0 = g[2 * k], g1 = g[2 * k + 1];
    /* bp/bn after the shuffles of :156-160: index = source state of the transition */
    int16_t bp[8] = {wrap16(b[4] + g1), wrap16(b[0] + g1), wrap16(b[1] + g0), wrap16(b[5] + g0),
                     wrap16(b[6] + g0), wrap16(b[2] + g0), wrap16(b[3] + g1), wrap16(b[7] + g1)};
    int16_t bn[8] = {wrap16(b[0] - g1), wrap16(b[4] - g1), wrap16(b[5] - g0), wrap16(b[1] - g0),
                     wrap16(b[2] - g0), wrap16(b[6] - g0), wrap16(b[7] - g1), wrap16(b[3] - g1)};
    for (int i = 0; i < 8; i++) b[i] = max16(bp[i], bn[i]);
    if (k < (int)K) {
      /* :165-171 add the stored alpha, horizontal max via minpos(0x7FFF - v); the
       * difference hMax(bn) - hMax(bp) equals max(bp) - max(bn) modulo 2^16 */
      const int16_t *al = &alpha[8 * k];
      int16_t mp = -32768, mn = -32768;
      for (int i = 0; i < 8; i++) {
        mp = max16(mp, wrap16(bp[i] + al[i]));
        mn = max16(mn, wrap16(bn[i] + al[i]));
      }
      int16_t hp = wrap16(0x7FFF - mp), hn = wrap16(0x7FFF - mn);
      out[k] = wrap16(hn - hp);
      if ((k % 4) == 0) { /* :194-204 renormalise after every 4 steps */
        int16_t b0 = b[0];
        for (int i = 0; i < 8; i++) b[i] = wrap16(b[i] - b0);
      }
    }
  }
}

/* ---------------------------------------------------------------- generic MAP ---- */
/* turbodecoder_gen.c:59-236 (no halving, wrapping int16, normalise every 4 steps).
 * scratch: beta 8*(K+4). */
static void gen_dec(const int16_t *xin, const int16_t *app, const int16_t *par, int16_t *out,
                    uint32_t K, int16_t *beta) {
  const int end = (int)K + 3;
  beta[8 * end] = 0; /* :255-257 */
  for (int i = 1; i < 8; i++) beta[8 * end + i] = -ORC_INF;
  int16_t o[8];
  memcpy(o, &beta[8 * end], 16);
  for (int k = end - 1; k >= 0; k--) { /* :59-108 map_gen_beta */
    int16_t x = xin[k];
    if (app && k < (int)K) x = wrap16(x + app[k]);
    int16_t y = par[k], xy = wrap16(x + y);
    int16_t mb[8] = {wrap16(o[4] + xy), o[4], wrap16(o[5] + y), wrap16(o[5] + x),
                     wrap16(o[6] + x), wrap16(o[6] + y), o[7], wrap16(o[7] + xy)};
    int16_t nw[8] = {o[0], wrap16(o[0] + xy), wrap16(o[1] + x), wrap16(o[1] + y),
                     wrap16(o[2] + y), wrap16(o[2] + x), wrap16(o[3] + xy), o[3]};
    for (int i = 0; i < 8; i++) {
      o[i] = max16(mb[i], nw[i]);
      beta[8 * k + i] = o[i];
    }
    if ((k % 4) == 0 && k < (int)K) {
      for (int i = 1; i < 8; i++) o[i] = wrap16(o[i] - o[0]);
      o[0] = 0;
    }
  }
  int16_t a[8] = {0, -ORC_INF, -ORC_INF, -ORC_INF, -ORC_INF, -ORC_INF, -ORC_INF, -ORC_INF};
  for (int k = 1; k < (int)K + 1; k++) { /* :110-183 map_gen_alpha */
    int16_t x = xin[k - 1];
    if (app) x = wrap16(x + app[k - 1]);
    int16_t y = par[k - 1], xy = wrap16(x + y);
    int16_t mb[8] = {a[0], wrap16(a[3] + y), wrap16(a[4] + y), a[7],
                     a[1], wrap16(a[2] + y), wrap16(a[5] + y), a[6]};
    int16_t nw[8] = {wrap16(a[1] + xy), wrap16(a[2] + x), wrap16(a[5] + x), wrap16(a[6] + xy),
                     wrap16(a[0] + xy), wrap16(a[3] + x), wrap16(a[4] + x), wrap16(a[7] + xy)};
    int16_t m0 = wrap16(mb[0] + beta[8 * k]), m1 = wrap16(nw[0] + beta[8 * k]);
    for (int i = 1; i < 8; i++) {
      m0 = max16(m0, wrap16(mb[i] + beta[8 * k + i]));
      m1 = max16(m1, wrap16(nw[i] + beta[8 * k + i]));
    }
    for (int i = 0; i < 8; i++) a[i] = max16(mb[i], nw[i]);
    if ((k % 4) == 0) {
      for (int i = 1; i < 8; i++) a[i] = wrap16(a[i] - a[0]);
      a[0] = 0;
    }
    out[k - 1] = wrap16(m1 - m0);
  }
}

/* ---------------------------------------------------------------- driver ---- */

/* turbodecoder.c:364-376 srslte_tdec_autoimp_get_subblocks (AVX2 build) */
uint32_t orc_autoimp_subblocks(uint32_t K) {
  if (!(K % 16) && K > 800) return 16;
  if (!(K % 8) && K > 400) return 8;
  return 0;
}

/* Resolve the implementation actually run for (impl, K): turbodecoder.c:153-291,467-489 */
static int resolve_impl(int impl, uint32_t K) {
  if (impl == ORC_TDEC_AUTO) {
    uint32_t nsb = orc_autoimp_subblocks(K);
    return nsb == 16 ? ORC_TDEC_AVX_WINDOW : nsb == 8 ? ORC_TDEC_SSE_WINDOW : ORC_TDEC_SSE;
  }
  return impl;
}

static int impl_nsb(int r) {
  return r == ORC_TDEC_AVX_WINDOW ? 16 : r == ORC_TDEC_SSE_WINDOW ? 8 : 1;
}

int orc_tdec_input_len(int impl, int sb_layout, uint32_t K) {
  int r = resolve_impl(impl, K);
  int sb = sb_layout && impl == ORC_TDEC_AUTO && r != ORC_TDEC_SSE;
  return sb ? 3 * ((int)K + 32) + 12 : 3 * (int)K + 12;
}

/* One decoder object (srslte_tdec_t analogue) */
typedef struct {
  int impl_r, nsb;
  uint32_t K;
  int16_t *syst, *par0, *par1, *app1, *app2, *ext1, *ext2, *scratch;
  uint16_t *fwd, *rev;
  int n_iter;
} orc_tdec;

static void tdec_dec(orc_tdec *h, const int16_t *x, const int16_t *app, const int16_t *par,
                     int16_t *out) {
  switch (h->impl_r) {
    case ORC_TDEC_AVX_WINDOW: win_dec(16, 0, x, app, par, out, h->K, h->scratch); break;
    case ORC_TDEC_SSE_WINDOW: win_dec(8, 1, x, app, par, out, h->K, h->scratch); break;
    case ORC_TDEC_SSE: sse_dec(x, app, par, out, h->K, h->scratch); break;
    default: gen_dec(x, app, par, out, h->K, h->scratch); break;
  }
}

/* turbodecoder_iter.h:283-357 run_tdec_iteration_16bit: one half-iteration */
static void tdec_half_iteration(orc_tdec *h) {
  const uint32_t K = h->K;
  int n = h->n_iter;
  if ((n % 2) == 0) {
    if (n) {
      for (uint32_t i = 0; i < K; i++) h->app1[i] = wrap16(h->app1[i] - h->ext1[i]);
    }
    tdec_dec(h, h->syst, n ? h->app1 : NULL, h->par0, h->ext1);
  } else {
    if (n > 1) {
      for (uint32_t i = 0; i < K; i++) h->ext1[i] = wrap16(h->ext1[i] - h->app1[i]);
    }
    for (uint32_t i = 0; i < K; i++) h->app2[h->rev[i]] = h->ext1[i]; /* vec_lut scatter */
    tdec_dec(h, h->app2, NULL, h->par1, h->ext2);
    for (uint32_t i = 0; i < K; i++) h->app1[h->fwd[i]] = h->ext2[i];
  }
  h->n_iter++;
}

/* turbodecoder.c:353-360 + decision_byte: decide on app1 after DEC2, ext1 after DEC1;
 * bits MSB-first in natural order */
static void tdec_decision(const orc_tdec *h, uint8_t *outb) {
  const int16_t *v = (h->n_iter % 2) ? h->ext1 : h->app1;
  const uint32_t K = h->K, nsb = (uint32_t)h->nsb, L = K / nsb;
  for (uint32_t i = 0; i < K / 8; i++) {
    uint8_t byte = 0;
    for (uint32_t j = 0; j < 8; j++) {
      uint32_t p = 8 * i + j;
      uint32_t idx = nsb > 1 ? (p % L) * nsb + p / L : p;
      if (v[idx] > 0) byte |= (uint8_t)(0x80 >> j);
    }
    outb[i] = byte;
  }
}

/* extract_input variants: turbodecoder_iter.h:271-280 (SB input) and
 * turbodecoder_win.h:634-674 / turbodecoder_sse.c:412-493 / turbodecoder_gen.c:240-259
 * (natural [s,p0,p1] triplets + 12 tail values) */
static void tdec_extract(orc_tdec *h, const int16_t *in, int sb_input) {
  const uint32_t K = h->K, nsb = (uint32_t)h->nsb, L = K / nsb;
  if (sb_input) {
    for (uint32_t i = 0; i < K; i++) {
      h->syst[i] = in[i];
      h->par0[i] = in[(K + 32) + i];
      h->par1[i] = in[2 * (K + 32) + i];
    }
    for (uint32_t j = 0; j < 3; j++) {
      h->syst[K + j] = in[3 * (K + 32) + 2 * j];
      h->par0[K + j] = in[3 * (K + 32) + 2 * j + 1];
      h->app2[K + j] = in[3 * (K + 32) + 6 + 2 * j];
      h->par1[K + j] = in[3 * (K + 32) + 6 + 2 * j + 1];
    }
  } else {
    for (uint32_t p = 0; p < K; p++) {
      uint32_t idx = nsb > 1 ? (p % L) * nsb + p / L : p;
      h->syst[idx] = in[3 * p];
      h->par0[idx] = in[3 * p + 1];
      h->par1[idx] = in[3 * p + 2];
    }
    for (uint32_t j = 0; j < 3; j++) {
      h->syst[K + j] = in[3 * K + 2 * j];
      h->par0[K + j] = in[3 * K + 2 * j + 1];
      h->app2[K + j] = in[3 * K + 6 + 2 * j];
      h->par1[K + j] = in[3 * K + 6 + 2 * j + 1];
    }
  }
}

static int tdec_open(orc_tdec *h, int impl, uint32_t K) {
  memset(h, 0, sizeof(*h));
  int idx = orc_cbindex(K);
  if (idx < 0 || srsgpu_qpp_table[idx][0] != K) return -1;
  h->impl_r = resolve_impl(impl, K);
  h->nsb = impl_nsb(h->impl_r);
  h->K = K;
  size_t len = K + 16;
  h->syst = calloc(len, 2);
  h->par0 = calloc(len, 2);
  h->par1 = calloc(len, 2);
  h->app1 = calloc(len, 2);
  h->app2 = calloc(len, 2);
  h->ext1 = calloc(len, 2);
  h->ext2 = calloc(len, 2);
  h->scratch = calloc((size_t)(K + 16) * 8 * 2 + 64, 2);
  h->fwd = calloc(K, 2);
  h->rev = calloc(K, 2);
  return orc_interl(K, (uint32_t)h->nsb, h->fwd, h->rev);
}

static void tdec_close(orc_tdec *h) {
  free(h->syst); free(h->par0); free(h->par1); free(h->app1); free(h->app2);
  free(h->ext1); free(h->ext2); free(h->scratch); free(h->fwd); free(h->rev);
}

int orc_tdec_run(int impl, int sb_layout, const int16_t *input, uint32_t K,
                 uint32_t nof_halfits, uint8_t *decisions, int16_t *final_app1,
                 int16_t *final_ext1) {
  orc_tdec h;
  if (tdec_open(&h, impl, K)) return -1;
  int sb_input = sb_layout && impl == ORC_TDEC_AUTO && h.nsb > 1;
  tdec_extract(&h, input, sb_input);
  for (uint32_t n = 0; n < nof_halfits; n++) {
    tdec_half_iteration(&h);
    if (decisions) tdec_decision(&h, decisions + (size_t)n * (K / 8));
  }
  if (final_app1) memcpy(final_app1, h.app1, K * 2);
  if (final_ext1) memcpy(final_ext1, h.ext1, K * 2);
  tdec_close(&h);
  return 0;
}

/* ---------------------------------------------------------------- CRC ---- */
/* crc.c:34-48 gen_crc_table + crc.h:68-80 put_byte/get + crc.c:144-155 checksum_byte:
 * MSB-first table CRC, init 0, no final xor. */
uint32_t orc_crc_checksum_byte(uint32_t poly, int order, const uint8_t *data, uint32_t len_bits) {
  uint64_t table[256];
  const uint64_t mask = (((uint64_t)1 << (order - 1)) - 1) << 1 | 1;
  const uint64_t high = (uint64_t)1 << (order - 1);
  const int ord = order - 8;
  for (int i = 0; i < 256; i++) {
    uint64_t crc = ((uint64_t)i) << ord;
    for (int j = 0; j < 8; j++) {
      uint64_t bit = crc & high;
      crc <<= 1;
      if (bit) crc ^= poly;
    }
    table[i] = crc & mask;
  }
  uint64_t crc = 0;
  for (uint32_t i = 0; i < len_bits / 8; i++) {
    crc = (crc << 8) ^ table[((crc >> ord) & 0xff) ^ data[i]];
  }
  return (uint32_t)(crc & mask);
}

/* ---------------------------------------------------------------- code block decode loop ---- */
/* sch.c:356-391 decode_tb_cb inner loop for one code block: half-iterations with a CRC check
 * after each until it passes or max_halfits is reached. crc_len_bits = K (CRC24B, C>1) or
 * TBS+24 (CRC24A, C==1). Returns 1 if the CRC passed; *noi = half-iterations run. */
int orc_tdec_decode_cb(int impl, int sb_layout, const int16_t *input, uint32_t K,
                       uint32_t max_halfits, uint32_t crc_poly, uint32_t crc_len_bits,
                       uint8_t *out_bytes, uint32_t *noi) {
  orc_tdec h;
  if (tdec_open(&h, impl, K)) return -1;
  int sb_input = sb_layout && impl == ORC_TDEC_AUTO && h.nsb > 1;
  tdec_extract(&h, input, sb_input);
  int ok = 0;
  uint32_t n = 0;
  do {
    tdec_half_iteration(&h);
    tdec_decision(&h, out_bytes);
    n++;
    if (orc_crc_checksum_byte(crc_poly, 24, out_bytes, crc_len_bits) == 0) ok = 1;
  } while (n < max_halfits && !ok);
  *noi = n;
  tdec_close(&h);
  return ok;
}

/* ---------------------------------------------------------------- turbo encoder ---- */
/* turbocoder.c:82-193 srslte_tcod_encode (bits in, bits out, [s,p0,p1]*K + 12 tail) */
int orc_tcod_encode(const uint8_t *in_bits, uint8_t *out_bits, uint32_t K) {
  uint16_t *f = malloc(K * 2), *r = malloc(K * 2);
  if (orc_interl(K, 1, f, r)) {
    free(f);
    free(r);
    return -1;
  }
  uint8_t r1[3] = {0, 0, 0}, r2[3] = {0, 0, 0};
  uint32_t k = 0;
  for (uint32_t i = 0; i < K; i++) {
    uint8_t bit = in_bits[i] & 1;
    out_bits[k++] = in_bits[i];
    uint8_t in = bit ^ r1[2] ^ r1[1];
    uint8_t out = r1[2] ^ r1[0] ^ in;
    r1[2] = r1[1]; r1[1] = r1[0]; r1[0] = in;
    out_bits[k++] = out;
    bit = in_bits[f[i]] & 1;
    in = bit ^ r2[2] ^ r2[1];
    out = r2[2] ^ r2[0] ^ in;
    r2[2] = r2[1]; r2[1] = r2[0]; r2[0] = in;
    out_bits[k++] = out;
  }
  for (int enc = 0; enc < 2; enc++) {
    uint8_t *r = enc ? r2 : r1;
    for (int j = 0; j < 3; j++) {
      uint8_t bit = r[2] ^ r[1];
      out_bits[k++] = bit;
      uint8_t in = bit ^ r[2] ^ r[1];
      uint8_t out = r[2] ^ r[0] ^ in;
      r[2] = r[1]; r[1] = r[0]; r[0] = in;
      out_bits[k++] = out;
    }
  }
  free(f);
  free(r);
  return 0;
}
