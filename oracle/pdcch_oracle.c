/*
 * TEST INFRASTRUCTURE (never shipped): scalar C restatement of the srsLTE 18.09 PDCCH receive path
 * (paths relative to /root/reference/lib/src/phy), the checker for include/srsgpu/pdcch_batch.h.
 * Pinned by tests/golden/pdcch_golden.npz (recorded from the reference build) in
 * tests/test_pdcch_oracle.py.
 *
 *   orc_pdcch_map        srslte_regs_init (phch/regs.c:681-763) with regs_pcfich_init (:477-512),
 *                        regs_phich_init (:249-331) and regs_pdcch_init (:82-158); the symbol order
 *                        of srslte_regs_pdcch_get (:200-236); NOF_CCE (pdcch.c:183-186)
 *   orc_pdcch_llr        srslte_pdcch_extract_llr_multi (phch/pdcch.c:442-508)
 *   orc_pdcch_locations  srslte_pdcch_ue_locations_ncce / _common_locations_ncce (pdcch.c:227-300)
 *   orc_find_dci         srslte_ue_dl_find_dl_dci(_type) then srslte_ue_dl_find_ul_dci
 *                        (ue/ue_dl.c:768-932, the UL DCI a 1A search sets aside included) over
 *                        srslte_pdcch_decode_msg (pdcch.c:366-420) = orc_dci_decode; pinned to the
 *                        reference's ue_dl.c itself (oracle/_ref/ref_front)
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "pdsch_oracle.h"

/* ---------------------------------------------------------------- REG map ---------- */
typedef struct {
  uint32_t l, k0, k[4];
  int assigned;
} orc_reg_t;

/* the cell's REGs in the order srslte_regs_init sorts them (per PRB, round-robin over the control
 * symbols, symbol 0 with two REGs per PRB skipping the middle pass), PCFICH and PHICH REGs marked;
 * returns the count or -1 */
static int orc_regs(uint32_t nof_prb, uint32_t cell_id, uint32_t nof_ports, uint32_t phich_len,
                    uint32_t phich_res, orc_reg_t **out) {
  const uint32_t nctrl = nof_prb <= 10 ? 4 : 3, vo = cell_id % 3, ext = (nof_ports >> 8) & 1;
  nof_ports &= 0xff;
  uint32_t nper[4], total = 0;
  for (uint32_t l = 0; l < nctrl; l++) { /* regs_num_x_symbol (regs.c:587-616): symbol 3 has CRS with extended CP */
    nper[l] = l == 0 ? 2 : (l == 1 && nof_ports == 4) ? 2 : (l == 3 && ext) ? 2 : 3;
    total += nof_prb * nper[l];
  }
  orc_reg_t *r = calloc(total, sizeof(orc_reg_t));
  if (!r) return -1;
  uint32_t cnt[4] = {0, 0, 0, 0}, n = 0, l = 0, prb = 0, pass = 0;
  while (n < total) {
    if (nper[l] == 3 || pass != 1) { /* two-REG symbols take passes 0 and 2 */
      orc_reg_t *g = &r[n++];
      const uint32_t base = prb * 12;
      g->l = l;
      if (nper[l] == 2) { /* six subcarriers minus the reference signals at vo and vo + 3 */
        g->k0 = base + cnt[l] * 6;
        uint32_t m = 0;
        for (uint32_t s = 0; s < 6; s++)
          if (s != vo && s != vo + 3) g->k[m++] = g->k0 + s;
      } else {
        g->k0 = base + cnt[l] * 4;
        for (uint32_t s = 0; s < 4; s++) g->k[s] = g->k0 + s;
      }
      cnt[l]++;
    }
    if (++l == nctrl) {
      l = 0;
      if (++pass == 3) {
        pass = 0;
        prb++;
        memset(cnt, 0, sizeof(cnt));
      }
    }
  }
  /* PCFICH: 4 REGs of symbol 0 at k = 6 (N_ID mod 2 N_RB) + floor(i N_RB / 2) 6 */
  for (uint32_t i = 0; i < 4; i++) {
    const uint32_t k = (6 * (cell_id % (2 * nof_prb)) + (i * nof_prb / 2) * 6) % (nof_prb * 12);
    orc_reg_t *hit = NULL;
    for (uint32_t j = 0; j < total && !hit; j++)
      if (r[j].l == 0 && r[j].k0 == k) hit = &r[j];
    if (!hit || hit->assigned) {
      free(r);
      return -1;
    }
    hit->assigned = 1;
  }
  /* PHICH: ceil(Ng N_RB / 8) mapping units of 3 REGs (36.211 6.9.3 steps 2-8) */
  const float ng = phich_res == 0 ? (float)1 / 6 : phich_res == 1 ? (float)1 / 2 : phich_res == 2 ? 1.0f : 2.0f;
  const uint32_t units = (uint32_t)(int)ceilf(ng * ((float)nof_prb / 8));
  uint32_t nfree[3] = {0, 0, 0};
  orc_reg_t **fr[3];
  for (int s = 0; s < 3; s++) fr[s] = malloc(sizeof(orc_reg_t *) * (total + 1));
  for (uint32_t j = 0; j < total; j++)
    if (r[j].l < 3 && !r[j].assigned) fr[r[j].l][nfree[r[j].l]++] = &r[j];
  for (uint32_t mi = 0; mi < units; mi++)
    for (uint32_t i = 0; i < 3; i++) {
      const uint32_t li = phich_len ? i : 0;
      const uint32_t ni = ((cell_id * nfree[li] / nfree[0]) + mi + i * nfree[li] / 3) % nfree[li];
      fr[li][ni]->assigned = 1;
    }
  for (int s = 0; s < 3; s++) free(fr[s]);
  *out = r;
  return (int)total;
}

static const uint8_t ORC_PDCCH_PERM[32] = {1, 17, 9, 25, 5, 21, 13, 29, 3, 19, 11, 27, 7, 23, 15, 31,
                                           0, 16, 8, 24, 4, 20, 12, 28, 2, 18, 10, 26, 6, 22, 14, 30};

int orc_pdcch_map(uint32_t nof_prb, uint32_t cell_id, uint32_t nof_ports, uint32_t phich_len,
                  uint32_t phich_res, uint32_t cfi, uint32_t *idx, uint32_t *nof_cce) {
  if (cfi < 1 || cfi > 3) return -1;
  orc_reg_t *r;
  const int total = orc_regs(nof_prb, cell_id, nof_ports, phich_len, phich_res, &r);
  if (total < 0) return -1;
  const uint32_t nsym = nof_prb <= 10 ? cfi + 1 : cfi;
  orc_reg_t **avail = malloc(sizeof(orc_reg_t *) * total), **perm = malloc(sizeof(orc_reg_t *) * total);
  uint32_t m = 0;
  for (int j = 0; j < total; j++)
    if (r[j].l < nsym && !r[j].assigned) avail[m++] = &r[j];
  /* sub-block interleaver, 32 columns, column permutation, cyclic shift by N_ID (6.8.5) */
  const int rows = ((int)m - 1) / 32 + 1, nd = 32 * rows - (int)m > 0 ? 32 * rows - (int)m : 0;
  uint32_t k = 0;
  for (int c = 0; c < 32; c++)
    for (int row = 0; row < rows; row++) {
      const int pos = row * 32 + ORC_PDCCH_PERM[c];
      if (pos < nd) continue;
      const uint32_t src = k < cell_id ? (m + k - (cell_id % m)) % m : (k - cell_id) % m;
      perm[pos - nd] = avail[src];
      k++;
    }
  const uint32_t useful = (m / 9) * 9;
  for (uint32_t q = 0; q < useful; q++)
    for (int s = 0; s < 4; s++) idx[4 * q + s] = perm[q]->l * nof_prb * 12 + perm[q]->k[s];
  *nof_cce = useful / 9;
  free(avail);
  free(perm);
  free(r);
  return (int)(4 * useful);
}

/* ---------------------------------------------------------------- LLRs ---------- */
/* srslte_predecoding_single_multi without CSI (mimo/precoding.c:330-353): symbols below
 * 16 floor(n / 16) in the AVX kernel when n > 32 (:154-230: per-antenna |h|^2 = hadd of the
 * squares, antenna sums in order, + noise only when noise > 0, conj product by addsub, divide,
 * times 1/scaling), the rest in the C loop (:231-240, :243-254) whose conj() products accumulate in
 * double and round to the float accumulators */
static void orc_single_multi(const float *const *y, const float *const *h, uint32_t nrx, uint32_t n,
                             float noise, float *x) {
  const uint32_t simd = n > 32 ? 16 * (n / 16) : 0;
  for (uint32_t i = 0; i < n; i++) {
    if (i < simd) {
      float hh = 0, rr = 0, ri = 0;
      for (uint32_t a = 0; a < nrx; a++) {
        const float yr = y[a][2 * i], yi = y[a][2 * i + 1], hr = h[a][2 * i], hi = h[a][2 * i + 1];
        const float p = hr * hr + hi * hi;
        const float pr = yr * hr - yi * -hi, pi = yi * hr + yr * -hi;
        hh = a ? hh + p : p;
        rr = a ? rr + pr : pr;
        ri = a ? ri + pi : pi;
      }
      if (noise > 0) hh = hh + noise;
      x[2 * i] = rr / hh * 1.0f;
      x[2 * i + 1] = ri / hh * 1.0f;
    } else {
      float hh = 0, rr = 0, ri = 0;
      for (uint32_t a = 0; a < nrx; a++) {
        const double yr = y[a][2 * i], yi = y[a][2 * i + 1], hr = h[a][2 * i], hi = h[a][2 * i + 1];
        rr = (float)((double)rr + (yr * hr - yi * -hi));
        ri = (float)((double)ri + (yr * -hi + yi * hr));
        hh = (float)((double)hh + (hr * hr - -hi * hi));
      }
      const float den = (hh + noise) * 1.0f;
      x[2 * i] = rr / den;
      x[2 * i + 1] = ri / den;
    }
  }
}

static int orc_pdcch_llr4(uint32_t nof_prb, uint32_t cell_id, uint32_t phich_len, uint32_t phich_res, uint32_t nrx,
                          uint32_t cfi, uint32_t sf_idx, const float *const *gs, const float *const *hs, float *llr);
int orc_pdcch_llr(uint32_t nof_prb, uint32_t cell_id, uint32_t nof_ports, uint32_t phich_len,
                  uint32_t phich_res, uint32_t nrx, uint32_t cfi, uint32_t sf_idx, float noise,
                  const float *g0, const float *g1, const float *h00, const float *h01, const float *h10,
                  const float *h11, float *llr);

/* 4 ports as well: g [rx], h [port * 2 + rx] (4-port transmit diversity over the symbol quadruplets) */
int orc_pdcch_llr_n(uint32_t nof_prb, uint32_t cell_id, uint32_t nof_ports, uint32_t phich_len, uint32_t phich_res,
                    uint32_t nrx, uint32_t cfi, uint32_t sf_idx, float noise, const float *const *g,
                    const float *const *h, float *llr) {
  if (nof_ports == 4) return orc_pdcch_llr4(nof_prb, cell_id, phich_len, phich_res, nrx, cfi, sf_idx, g, h, llr);
  return orc_pdcch_llr(nof_prb, cell_id, nof_ports, phich_len, phich_res, nrx, cfi, sf_idx, noise, g[0], g[1], h[0],
                       h[1], h[2], h[3], llr);
}

int orc_pdcch_llr(uint32_t nof_prb, uint32_t cell_id, uint32_t nof_ports, uint32_t phich_len,
                  uint32_t phich_res, uint32_t nrx, uint32_t cfi, uint32_t sf_idx, float noise,
                  const float *g0, const float *g1, const float *h00, const float *h01, const float *h10,
                  const float *h11, float *llr) {
  uint32_t ncce;
  uint32_t *idx = malloc(sizeof(uint32_t) * 36 * 110 * 4);
  const int nsym = orc_pdcch_map(nof_prb, cell_id, nof_ports, phich_len, phich_res, cfi, idx, &ncce);
  if (nsym < 0) {
    free(idx);
    return -1;
  }
  const float *gs[2] = {g0, g1}, *hs[2][2] = {{h00, h01}, {h10, h11}}; /* [port][rx] */
  float *ys[2], *hh[2][2], *d = malloc(sizeof(float) * 2 * (nsym + 1));
  for (uint32_t a = 0; a < 2; a++) {
    ys[a] = calloc(2 * (nsym + 1), sizeof(float));
    for (uint32_t p = 0; p < 2; p++) hh[p][a] = calloc(2 * (nsym + 1), sizeof(float));
  }
  for (uint32_t a = 0; a < nrx; a++)
    for (int i = 0; i < nsym; i++) {
      memcpy(&ys[a][2 * i], &gs[a][2 * idx[i]], 8);
      for (uint32_t p = 0; p < nof_ports; p++) memcpy(&hh[p][a][2 * i], &hs[p][a][2 * idx[i]], 8);
    }
  if (nof_ports == 1) {
    const float *yy[2] = {ys[0], ys[1]}, *h0[2] = {hh[0][0], hh[0][1]};
    orc_single_multi(yy, h0, nrx, (uint32_t)nsym, noise / 2, d);
  } else { /* transmit diversity + layer demapping, no noise term (pdcch.c:495-496) */
    orc_predecode_txdiv(ys[0], nrx > 1 ? ys[1] : NULL, hh[0][0], nrx > 1 ? hh[0][1] : NULL, hh[1][0],
                        nrx > 1 ? hh[1][1] : NULL, (int)nrx, nsym, 1.0f, d, NULL);
  }
  /* QPSK soft demapping x (-sqrt 2) and the subframe's sequence, c_init = sf 2^9 + N_ID
   * (pdcch.c:197-205, sequences.c:57-59); its first 72 NOF_CCE(cfi) bits whatever its length */
  uint8_t *c = malloc(2 * (size_t)nsym + 64);
  orc_sequence(sf_idx * 512 + cell_id, 2 * (uint32_t)nsym, c);
  const float s2 = (float)(-sqrt(2));
  for (int i = 0; i < 2 * nsym; i++) {
    const float v = d[i] * s2;
    llr[i] = c[i] ? -v : v;
  }
  free(c);
  for (uint32_t a = 0; a < 2; a++) {
    free(ys[a]);
    for (uint32_t p = 0; p < 2; p++) free(hh[p][a]);
  }
  free(d);
  free(idx);
  return 2 * nsym;
}

static int orc_pdcch_llr4(uint32_t nof_prb, uint32_t cell_id, uint32_t phich_len, uint32_t phich_res, uint32_t nrx,
                          uint32_t cfi, uint32_t sf_idx, const float *const *gs, const float *const *hs, float *llr) {
  uint32_t ncce;
  uint32_t *idx = malloc(sizeof(uint32_t) * 36 * 110 * 4);
  const int nsym = orc_pdcch_map(nof_prb, cell_id, 4, phich_len, phich_res, cfi, idx, &ncce);
  if (nsym < 0 || nsym % 4) {
    free(idx);
    return -1;
  }
  float *ys[2], *hh[8], *d = malloc(sizeof(float) * 2 * (nsym + 1));
  for (uint32_t a = 0; a < 2; a++) ys[a] = calloc(2 * (nsym + 1), sizeof(float));
  for (int p = 0; p < 8; p++) hh[p] = calloc(2 * (nsym + 1), sizeof(float));
  for (uint32_t a = 0; a < nrx; a++)
    for (int i = 0; i < nsym; i++) {
      memcpy(&ys[a][2 * i], &gs[a][2 * idx[i]], 8);
      for (uint32_t p = 0; p < 4; p++) memcpy(&hh[p * 2 + a][2 * i], &hs[p * 2 + a][2 * idx[i]], 8);
    }
  const float *yy[2] = {ys[0], ys[1]}, *h4[8];
  for (int p = 0; p < 8; p++) h4[p] = hh[p];
  orc_predecode_txdiv4(yy, h4, (int)nrx, nsym, 1.0f, d, NULL); /* pdcch.c:495-496, no noise term */
  uint8_t *c = malloc(2 * (size_t)nsym + 64);
  orc_sequence(sf_idx * 512 + cell_id, 2 * (uint32_t)nsym, c);
  const float s2 = (float)(-sqrt(2));
  for (int i = 0; i < 2 * nsym; i++) {
    const float v = d[i] * s2;
    llr[i] = c[i] ? -v : v;
  }
  free(c);
  for (uint32_t a = 0; a < 2; a++) free(ys[a]);
  for (int p = 0; p < 8; p++) free(hh[p]);
  free(d);
  free(idx);
  return 2 * nsym;
}

/* ---------------------------------------------------------------- blind search ---------- */
int orc_pdcch_locations(uint32_t nof_cce, uint32_t sf_idx, uint16_t rnti, int common, uint32_t *out) {
  uint32_t n = 0;
  if (common) { /* L = 8 and 4 over the first min(16, nof_cce) CCEs */
    for (uint32_t l = 3; l > 1; l--) {
      const uint32_t L = 1u << l, lim = nof_cce < 16 ? nof_cce : 16;
      for (uint32_t i = 0; i < lim / L; i++) {
        const uint32_t c = L * (i % (nof_cce / L));
        if (n < 64 && c + L <= nof_cce) {
          out[2 * n] = l;
          out[2 * n + 1] = c;
          n++;
        }
      }
    }
    return (int)n;
  }
  /* 36.213 9.1.1: Y_k = 39827 Y_{k-1} mod 65537, Y_-1 = RNTI; 6, 6, 2, 2 candidates at L = 1, 2, 4, 8
   * taken from L = 8 down */
  uint32_t Y = rnti;
  for (uint32_t m = 0; m <= sf_idx; m++) Y = (39827 * Y) % 65537;
  static const uint32_t cand[4] = {6, 6, 2, 2};
  for (int l = 3; l >= 0; l--) {
    const uint32_t L = 1u << l;
    if (nof_cce < L) continue;
    for (uint32_t i = 0; i < cand[l]; i++) {
      const uint32_t c = L * ((Y + i) % (nof_cce / L));
      if (n < 64 && c + L <= nof_cce) {
        out[2 * n] = (uint32_t)l;
        out[2 * n + 1] = c;
        n++;
      }
    }
  }
  return (int)n;
}

/* srslte_dci_format_sizeof (dci.c:223-360) for the DL formats the search uses */
static uint32_t orc_riv_nbits(uint32_t n) { return (uint32_t)ceilf(log2f((float)n * ((float)n + 1) / 2)); }
static int orc_ambiguous(uint32_t s) {
  static const uint32_t a[10] = {12, 14, 16, 20, 24, 26, 32, 40, 44, 56};
  for (int i = 0; i < 10; i++)
    if (a[i] == s) return 1;
  return 0;
}
static uint32_t orc_P(uint32_t n) { return n <= 10 ? 1 : n <= 26 ? 2 : n <= 63 ? 3 : 4; }
static uint32_t orc_1a_size(uint32_t n) {
  const uint32_t f0 = 1 + 1 + orc_riv_nbits(n) + 5 + 1 + 2 + 3 + 1;
  uint32_t s = 1 + 1 + orc_riv_nbits(n) + 5 + 3 + 1 + 2 + 2;
  while (s < f0) s++;
  if (orc_ambiguous(s)) s++;
  return s;
}
static uint32_t orc_ngap1(uint32_t n) {
  return n <= 10 ? n / 2 : n == 11 ? 4 : n <= 19 ? 8 : n <= 26 ? 12 : n <= 44 ? 18 : n <= 49 ? 27
         : n <= 63 ? 27 : n <= 79 ? 32 : 48;
}
uint32_t orc_dci_sizeof(uint32_t format, uint32_t n, uint32_t nports) {
  const uint32_t P = orc_P(n), rbg = (uint32_t)ceilf((float)n / P);
  uint32_t s = 0;
  switch (format) {
  case 0: { /* format 0, padded to 1A's size */
    s = 1 + 1 + orc_riv_nbits(n) + 5 + 1 + 2 + 3 + 1;
    while (s < orc_1a_size(n)) s++;
    return s;
  }
  case 1: /* format 1: never the size of 0 or 1A, nor an ambiguous one */
    s = rbg + 5 + 3 + 1 + 2 + 2 + (n > 10 ? 1 : 0);
    while (s == orc_dci_sizeof(0, n, nports) || s == orc_1a_size(n) || orc_ambiguous(s)) s++;
    return s;
  case 2: return orc_1a_size(n);
  case 3: { /* 1C */
    const uint32_t g = orc_ngap1(n), nvrb = 2 * (g < n - g ? g : n - g), step = n < 50 ? 2 : 4;
    return orc_riv_nbits(nvrb / step) + 5 + (n >= 50 ? 1 : 0);
  }
  case 4:
  case 5: /* 1B, 1D */
    s = orc_1a_size(n) - 1 + (nports <= 2 ? 2 : 4) + 1;
    while (orc_ambiguous(s)) s++;
    return s;
  case 6:
  case 7:
  case 8: { /* 2, 2A, 2B */
    const uint32_t pb = format == 6 ? (nports <= 2 ? 3 : 6) : format == 7 ? (nports <= 2 ? 0 : 2) : 0;
    s = rbg + 2 + 3 + 1 + 2 * (5 + 1 + 2) + pb + (n > 10 ? 1 : 0);
    while (orc_ambiguous(s)) s++;
    return s;
  }
  default: return 0;
  }
}

static const uint32_t ORC_UE_FORMATS[8][2] = {{2, 1}, {2, 1}, {2, 7}, {2, 6}, {2, 5}, {2, 4}, {2, 1}, {2, 8}};

/* the UL DCI a DL search set aside (ue_dl.c:785-792: format 0 found while searching 1A, first one) */
typedef struct {
  int set;
  uint16_t rnti;
  int32_t out5[5];
  uint8_t data[128];
} orc_pending_t;

/* dci_blind_search (ue_dl.c:768-810) over one format and a candidate list: 1 found, 0 not, -1 the
 * reference's SRSLTE_ERROR (decode_msg refuses a location past nCCE 87) */
static int orc_blind(const float *llr, const uint32_t *loc, uint32_t nloc, uint32_t format, uint32_t nbits,
                     uint16_t rnti, int32_t *out5, uint8_t *data, orc_pending_t *pend) {
  uint8_t buf[160];
  for (uint32_t i = 0; i < nloc; i++) {
    const uint32_t L = loc[2 * i], c = loc[2 * i + 1];
    if (c > 87) return -1;
    uint16_t rem = 0;
    if (orc_dci_decode(llr + 72 * c, 72u << L, nbits, buf, &rem) != 1 || rem != rnti) continue;
    const uint32_t got = (format == 0 || format == 2) ? (buf[0] ? 2u : 0u) : format;
    if (got == 0 && format == 2) { /* the UL DCI, kept for srslte_ue_dl_find_ul_dci */
      if (pend && !pend->set) {
        pend->set = 1;
        pend->rnti = rem;
        pend->out5[0] = 1;
        pend->out5[1] = 0;
        pend->out5[2] = (int32_t)L;
        pend->out5[3] = (int32_t)c;
        pend->out5[4] = (int32_t)nbits;
        memset(pend->data, 0, 128);
        memcpy(pend->data, buf, nbits + 16);
      }
      continue;
    }
    if (got != format) continue;
    out5[0] = 1;
    out5[1] = (int32_t)format;
    out5[2] = (int32_t)L;
    out5[3] = (int32_t)c;
    out5[4] = (int32_t)nbits;
    memset(data, 0, 128);
    memcpy(data, buf, nbits + 16);
    return 1;
  }
  return 0;
}

static void orc_none(int32_t *out5, int r) {
  out5[0] = r < 0 ? -1 : 0;
  out5[1] = -1;
  out5[2] = out5[3] = out5[4] = 0;
}

/* srslte_ue_dl_find_dl_dci(_type) (rnti != 0) and then srslte_ue_dl_find_ul_dci (ul_rnti != 0,
 * ue_dl.c:811-838) on one subframe's LLRs, in phch_worker's order (phch_worker.cc:548-806, 938-967) on a
 * ue_dl object with no UL DCI pending from an earlier subframe. rnti 0: no DL search (out5 reports the
 * reference's "RNTI not specified" error, -1). */
int orc_find_dci(uint32_t nof_prb, uint32_t cell_id, uint32_t nof_ports, uint32_t phich_len, uint32_t phich_res,
                 uint32_t cfi, uint32_t sf_idx, const float *llr, uint16_t rnti, uint32_t tm, int rnti_type,
                 uint16_t ul_rnti, int32_t *out5, uint8_t *data, int32_t *ul5, uint8_t *uldata) {
  uint32_t ncce, *idx = malloc(sizeof(uint32_t) * 36 * 110 * 4);
  if (orc_pdcch_map(nof_prb, cell_id, nof_ports, phich_len, phich_res, cfi, idx, &ncce) < 0 || tm > 7) {
    free(idx);
    return -1;
  }
  free(idx);
  orc_none(out5, 0);
  if (ul5) orc_none(ul5, 0);
  orc_pending_t pend;
  memset(&pend, 0, sizeof(pend));
  uint32_t ue[128], com[128];
  const uint32_t ncom = (uint32_t)orc_pdcch_locations(ncce, sf_idx, rnti, 1, com);
  if (rnti) {
    const int common = rnti_type < 0 ? (rnti == 0xFFFF || rnti == 0xFFFE || rnti <= 0x000A)
                                     : (rnti_type == 1 || rnti_type == 2 || rnti_type == 5);
    int r = 0;
    if (common) {
      const uint32_t f[2] = {2, 3}; /* 1A, 1C */
      for (int i = 0; i < 2 && ncom && !r; i++)
        r = orc_blind(llr, com, ncom, f[i], orc_dci_sizeof(f[i], nof_prb, nof_ports), rnti, out5, data, &pend);
    } else {
      const uint32_t nue = (uint32_t)orc_pdcch_locations(ncce, sf_idx, rnti, 0, ue);
      for (int i = 0; i < 2 && !r; i++) {
        const uint32_t f = ORC_UE_FORMATS[tm][i];
        r = orc_blind(llr, ue, nue, f, orc_dci_sizeof(f, nof_prb, nof_ports), rnti, out5, data, &pend);
      }
      if (!r && ncom) r = orc_blind(llr, com, ncom, 2, orc_dci_sizeof(2, nof_prb, nof_ports), rnti, out5, data, &pend);
    }
    if (r < 0) orc_none(out5, -1);
  } else {
    orc_none(out5, -1); /* dci_blind_search: "RNTI not specified" (ue_dl.c:805-807) */
  }
  if (ul5 && ul_rnti && cfi >= 1 && cfi <= 3) {
    if (pend.set && pend.rnti == ul_rnti) { /* ue_dl.c:815-819 */
      memcpy(ul5, pend.out5, sizeof(pend.out5));
      memcpy(uldata, pend.data, 128);
    } else {
      const uint32_t nue = (uint32_t)orc_pdcch_locations(ncce, sf_idx, ul_rnti, 0, ue);
      const int r = orc_blind(llr, ue, nue, 0, orc_dci_sizeof(0, nof_prb, nof_ports), ul_rnti, ul5, uldata, NULL);
      if (r < 0) orc_none(ul5, -1);
    }
  }
  return 0;
}

int orc_find_dl_dci(uint32_t nof_prb, uint32_t cell_id, uint32_t nof_ports, uint32_t phich_len,
                    uint32_t phich_res, uint32_t cfi, uint32_t sf_idx, const float *llr, uint16_t rnti,
                    uint32_t tm, int rnti_type, int32_t *out5, uint8_t *data) {
  return orc_find_dci(nof_prb, cell_id, nof_ports, phich_len, phich_res, cfi, sf_idx, llr, rnti, tm, rnti_type, 0,
                      out5, data, NULL, NULL);
}
