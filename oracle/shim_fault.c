/*
 * TEST INFRASTRUCTURE (never shipped): error paths and HARQ state of integration/srslte_gpu_shim.c.
 *
 * 1. Fault injection. The program is linked with -Wl,--wrap=hipMalloc, so every device allocation
 *    the shim itself makes goes through __wrap_hipMalloc below (the library's own allocations do
 *    not). For each drop-in (srslte_pdsch_decode, srslte_dlsch_decode2, srslte_pcfich_decode_multi,
 *    srslte_rm_turbo_rx_lut) and each k, the k-th shim allocation of a fresh object is made to
 *    fail: the call must return SRSLTE_ERROR, and the next call, with allocations working again,
 *    must succeed (the object's GPU state was released, not left half built).
 * 2. HARQ growth. One srslte_sch_t decodes two HARQ processes with different grant sizes: process A
 *    on a small allocation, then process B on a much larger one (more e-bits and a larger TB than
 *    the object has seen), then A's retransmissions. Each transmission goes through the reference
 *    srslte_dlsch_decode2 (sch.c:506) and the shim's on the same LLRs, each with its own
 *    srslte_sch_t and softbuffers: return value, bytes, nof_iterations, cb_crc and tb_crc must agree
 *    (the shim must not drop A's combined soft bits when B's grant arrives).
 * Prints "fault_cases=<n> fault_failures=<n> harq_tx=<n> harq_mismatches=<n>"; exit 0 iff both
 * failure counts are 0. Built by `make -C oracle shim` into oracle/_ref/shim_fault.
 */
#include <complex.h>
#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "srslte/phy/fec/cbsegm.h"
#include "srslte/phy/fec/softbuffer.h"
#include "srslte/phy/phch/pcfich.h"
#include "srslte/phy/phch/pdsch.h"
#include "srslte/phy/phch/ra.h"
#include "srslte/phy/phch/sch.h"
#include "srslte/phy/utils/vector.h"

int srsgpu_shim_pdsch_decode(srslte_pdsch_t *q, srslte_pdsch_cfg_t *cfg,
                             srslte_softbuffer_rx_t *softbuffers[SRSLTE_MAX_CODEWORDS],
                             cf_t *sf_symbols[SRSLTE_MAX_PORTS],
                             cf_t *ce[SRSLTE_MAX_PORTS][SRSLTE_MAX_PORTS], float noise_estimate,
                             uint16_t rnti, uint8_t *data[SRSLTE_MAX_CODEWORDS],
                             bool acks[SRSLTE_MAX_CODEWORDS]);
int srsgpu_shim_dlsch_decode2(srslte_sch_t *q, srslte_pdsch_cfg_t *cfg, srslte_softbuffer_rx_t *softbuffer,
                              int16_t *e_bits, uint8_t *data, int tb_idx);
int srsgpu_shim_rm_turbo_rx_lut(int16_t *input, int16_t *output, uint32_t in_len, uint32_t cb_idx,
                                uint32_t rv_idx);
int srsgpu_shim_softbuffer_rx_init(srslte_softbuffer_rx_t *q, uint32_t nof_prb);
void srsgpu_shim_softbuffer_rx_reset(srslte_softbuffer_rx_t *q);
void srsgpu_shim_softbuffer_rx_free(srslte_softbuffer_rx_t *q);
int srsgpu_shim_pcfich_decode_multi(srslte_pcfich_t *q, cf_t *sf_symbols[SRSLTE_MAX_PORTS],
                                    cf_t *ce[SRSLTE_MAX_PORTS][SRSLTE_MAX_PORTS], float noise_estimate,
                                    uint32_t nsubframe, uint32_t *cfi, float *corr_result);
int srsgpu_shim_release(const void *owner);

/* ---- allocation fault injection ---- */
int __real_hipMalloc(void **p, size_t n);
static int alloc_count = 0, alloc_fail_at = -1;
int __wrap_hipMalloc(void **p, size_t n) {
  if (alloc_count++ == alloc_fail_at) {
    *p = NULL;
    return 2; /* hipErrorOutOfMemory */
  }
  return __real_hipMalloc(p, n);
}

/* srslte_dlsch_encode2 writes the e-bits packed, MSB first (sch.c:281 with a bit offset) */
static int ebit(const uint8_t *packed, uint32_t i) { return (packed[i / 8] >> (7 - i % 8)) & 1; }

static uint64_t rng = 12345;
static double urand(void) {
  rng = rng * 6364136223846793005ULL + 1442695040888963407ULL;
  return ((rng >> 11) + 0.5) / 9007199254740992.0;
}
static float gauss(void) { return (float)(sqrt(-2.0 * log(urand())) * cos(2.0 * M_PI * urand())); }

typedef int (*call_fn)(void *ctx);
static uint32_t ncases = 0, nfail = 0;
/* fail the k-th shim allocation of call(ctx) for k = 0, 1, ... until a call makes fewer
 * allocations than k + 1; each failing call must return SRSLTE_ERROR and the retry succeed */
static void fault_sweep(const char *name, call_fn call, void *ctx, const void *owner) {
  for (int k = 0; k < 16; k++) {
    if (owner) srsgpu_shim_release(owner);
    alloc_count = 0;
    alloc_fail_at = k;
    const int r1 = call(ctx);
    const int injected = alloc_count > k;
    alloc_fail_at = -1;
    if (!injected) {
      if (r1 < 0) {
        fprintf(stderr, "%s: fails without an injected fault (%d)\n", name, r1);
        nfail++;
      }
      break;
    }
    ncases++;
    const int r2 = call(ctx);
    if (r1 != SRSLTE_ERROR || r2 < 0) {
      fprintf(stderr, "%s: allocation %d failed -> %d, retry -> %d\n", name, k, r1, r2);
      nfail++;
    }
  }
}

/* ---- the drop-ins under test ---- */
typedef struct {
  srslte_pdsch_t *rx;
  srslte_pdsch_cfg_t *cfg;
  srslte_softbuffer_rx_t **sb;
  cf_t **y;
  cf_t *(*h)[SRSLTE_MAX_PORTS];
  uint8_t **data;
} pdsch_ctx_t;
static int call_pdsch(void *p) {
  pdsch_ctx_t *c = p;
  bool acks[SRSLTE_MAX_CODEWORDS] = {false, false};
  srsgpu_shim_softbuffer_rx_reset(c->sb[0]);
  return srsgpu_shim_pdsch_decode(c->rx, c->cfg, c->sb, c->y, c->h, 0.1f, 0x1234, c->data, acks);
}
typedef struct {
  srslte_sch_t *sch;
  srslte_pdsch_cfg_t *cfg;
  srslte_softbuffer_rx_t *sb;
  int16_t *e;
  uint8_t *data;
} dlsch_ctx_t;
static int call_dlsch(void *p) { /* a clean codeword: 0, or SRSLTE_ERROR on a GPU failure */
  dlsch_ctx_t *c = p;
  srsgpu_shim_softbuffer_rx_reset(c->sb);
  return srsgpu_shim_dlsch_decode2(c->sch, c->cfg, c->sb, c->e, c->data, 0);
}
typedef struct {
  srslte_pcfich_t *q;
  cf_t **y;
  cf_t *(*h)[SRSLTE_MAX_PORTS];
} pcfich_ctx_t;
static int call_pcfich(void *p) {
  pcfich_ctx_t *c = p;
  uint32_t cfi = 0;
  float corr = 0;
  const int r = srsgpu_shim_pcfich_decode_multi(c->q, c->y, c->h, 0.0f, 1, &cfi, &corr);
  return r == 1 ? 0 : r;
}
/* srslte_rm_turbo_rx_lut keeps a context per calling thread: each call runs in a new thread */
static void *rm_thread(void *p) {
  static int16_t in[3 * 6200], out[3 * 6200 + 100];
  for (int i = 0; i < 3 * 6200; i++) in[i] = (int16_t)(i % 61 - 30);
  memset(out, 0, sizeof(out));
  *(int *)p = srsgpu_shim_rm_turbo_rx_lut(in, out, 3 * 6144, 187, 0);
  return NULL;
}
static int call_rm(void *p) {
  (void)p;
  int r = -100;
  pthread_t t;
  if (pthread_create(&t, NULL, rm_thread, &r)) return -100;
  pthread_join(t, NULL);
  return r;
}

int main(void) {
  const uint32_t nof_prb = 50;
  srslte_cell_t cell = {nof_prb, 1, 7, SRSLTE_CP_NORM, SRSLTE_PHICH_NORM, SRSLTE_PHICH_R_1};
  const uint32_t n = SRSLTE_SF_LEN_RE(nof_prb, SRSLTE_CP_NORM);
  cf_t *y[SRSLTE_MAX_PORTS] = {NULL}, *h[SRSLTE_MAX_PORTS][SRSLTE_MAX_PORTS] = {{NULL}};
  y[0] = srslte_vec_malloc(sizeof(cf_t) * n);
  h[0][0] = srslte_vec_malloc(sizeof(cf_t) * n);
  for (uint32_t i = 0; i < n; i++) {
    y[0][i] = gauss() + gauss() * _Complex_I;
    h[0][0][i] = 1.0f + 0.1f * gauss();
  }
  srslte_ra_dl_grant_t grant;
  memset(&grant, 0, sizeof(grant));
  grant.nof_prb = nof_prb;
  for (uint32_t s = 0; s < 2; s++)
    for (uint32_t p = 0; p < nof_prb; p++) grant.prb_idx[s][p] = true;
  grant.tb_en[0] = true;
  grant.mcs[0].idx = 9;
  grant.mcs[0].mod = srslte_ra_mod_from_mcs(9);
  grant.mcs[0].tbs = srslte_ra_tbs_from_idx(srslte_ra_tbs_idx_from_mcs(9), nof_prb);
  grant.Qm[0] = srslte_mod_bits_x_symbol(grant.mcs[0].mod);
  srslte_pdsch_cfg_t cfg;
  memset(&cfg, 0, sizeof(cfg));
  if (srslte_pdsch_cfg(&cfg, cell, &grant, 2, 1, 0)) return 2;

  /* 1. fault injection */
  srslte_pdsch_t rx;
  if (srslte_pdsch_init_ue(&rx, nof_prb, 1) || srslte_pdsch_set_cell(&rx, cell) || srslte_pdsch_set_rnti(&rx, 0x1234))
    return 2;
  srslte_softbuffer_rx_t sb0, sb1;
  if (srsgpu_shim_softbuffer_rx_init(&sb0, nof_prb) || srsgpu_shim_softbuffer_rx_init(&sb1, nof_prb)) return 2;
  srslte_softbuffer_rx_t *sbp[SRSLTE_MAX_CODEWORDS] = {&sb0, NULL};
  uint8_t *data[SRSLTE_MAX_CODEWORDS] = {calloc(grant.mcs[0].tbs / 8 + 16, 1), NULL};
  pdsch_ctx_t pc = {&rx, &cfg, sbp, y, h, data};
  fault_sweep("srslte_pdsch_decode", call_pdsch, &pc, &rx);

  /* a clean codeword from the reference encoder, so the DL-SCH decode succeeds (returns 0) */
  srslte_sch_t sch, enc;
  srslte_softbuffer_tx_t stx0;
  if (srslte_sch_init(&sch) || srslte_sch_init(&enc) || srslte_softbuffer_tx_init(&stx0, nof_prb)) return 2;
  uint8_t *bits = calloc(cfg.nbits[0].nof_bits + 16, 1), *tb = calloc(grant.mcs[0].tbs / 8 + 16, 1);
  for (int i = 0; i < grant.mcs[0].tbs / 8; i++) tb[i] = (uint8_t)(urand() * 256);
  srslte_softbuffer_tx_reset(&stx0);
  if (srslte_dlsch_encode2(&enc, &cfg, &stx0, tb, bits, 0)) return 2;
  {
    /* check the codeword on the reference decoder first */
    srslte_sch_t chk;
    srslte_softbuffer_rx_t sbc;
    int16_t *l = calloc(cfg.nbits[0].nof_bits + 16, sizeof(int16_t));
    uint8_t *o = calloc(grant.mcs[0].tbs / 8 + 16, 1);
    for (uint32_t i = 0; i < cfg.nbits[0].nof_bits; i++) l[i] = ebit(bits, i) ? 100 : -100;
    if (srslte_sch_init(&chk) || srslte_softbuffer_rx_init(&sbc, nof_prb)) return 2;
    srslte_softbuffer_rx_reset(&sbc);
    const int rc = srslte_dlsch_decode2(&chk, &cfg, &sbc, l, o, 0);
    if (rc != 0 || memcmp(o, tb, grant.mcs[0].tbs / 8)) {
      fprintf(stderr, "reference decode of the clean codeword: %d\n", rc);
      return 2;
    }
    srslte_softbuffer_rx_free(&sbc);
    srslte_sch_free(&chk);
    free(l);
    free(o);
  }
  int16_t *e = calloc(cfg.nbits[0].nof_bits + 16, sizeof(int16_t));
  for (uint32_t i = 0; i < cfg.nbits[0].nof_bits; i++) e[i] = ebit(bits, i) ? 100 : -100;
  dlsch_ctx_t dc = {&sch, &cfg, &sb1, e, data[0]};
  fault_sweep("srslte_dlsch_decode2", call_dlsch, &dc, &sch);

  srslte_regs_t regs;
  static srslte_pcfich_t pq;
  if (srslte_regs_init(&regs, cell) || srslte_pcfich_init(&pq, 1) || srslte_pcfich_set_cell(&pq, &regs, cell))
    return 2;
  pcfich_ctx_t fc = {&pq, y, h};
  fault_sweep("srslte_pcfich_decode_multi", call_pcfich, &fc, &pq);
  fault_sweep("srslte_rm_turbo_rx_lut", call_rm, NULL, NULL);
  srsgpu_shim_release(&rx);
  srsgpu_shim_release(&sch);
  srsgpu_shim_release(&pq);

  /* 2. HARQ growth: process A on 6 PRB, process B on 100 PRB, then A's retransmissions */
  srslte_cell_t big = {100, 1, 3, SRSLTE_CP_NORM, SRSLTE_PHICH_NORM, SRSLTE_PHICH_R_1};
  srslte_sch_t stx, sa, sbs;
  if (srslte_sch_init(&stx) || srslte_sch_init(&sa) || srslte_sch_init(&sbs)) return 2;
  srslte_softbuffer_tx_t tA, tB;
  srslte_softbuffer_rx_t rA, rB, gA, gB; /* reference (r*) and shim (g*) receive softbuffers */
  if (srslte_softbuffer_tx_init(&tA, 100) || srslte_softbuffer_tx_init(&tB, 100) ||
      srslte_softbuffer_rx_init(&rA, 100) || srslte_softbuffer_rx_init(&rB, 100) ||
      srsgpu_shim_softbuffer_rx_init(&gA, 100) || srsgpu_shim_softbuffer_rx_init(&gB, 100))
    return 2;
  uint32_t ntx = 0, nbad = 0;
  uint8_t *ebits = malloc(100 * 12 * 14 * 8);
  int16_t *llr = malloc(sizeof(int16_t) * 100 * 12 * 14 * 8), *llr2 = malloc(sizeof(int16_t) * 100 * 12 * 14 * 8);
  uint8_t *dtA = calloc(10000, 1), *dtB = calloc(10000, 1), *da = calloc(10000, 1), *db = calloc(10000, 1);
  for (uint32_t round = 0; round < 6; round++) {
    srslte_ra_dl_grant_t gsA, gsB;
    memset(&gsA, 0, sizeof(gsA));
    memset(&gsB, 0, sizeof(gsB));
    gsA.nof_prb = 6;
    for (uint32_t s = 0; s < 2; s++)
      for (uint32_t p = 10; p < 16; p++) gsA.prb_idx[s][p] = true;
    gsB.nof_prb = 100;
    for (uint32_t s = 0; s < 2; s++)
      for (uint32_t p = 0; p < 100; p++) gsB.prb_idx[s][p] = true;
    const uint32_t mA = 20 + round, mB = 16;
    gsA.tb_en[0] = gsB.tb_en[0] = true;
    gsA.mcs[0].idx = mA;
    gsA.mcs[0].mod = srslte_ra_mod_from_mcs(mA);
    gsA.mcs[0].tbs = srslte_ra_tbs_from_idx(srslte_ra_tbs_idx_from_mcs(mA), 6);
    gsA.Qm[0] = srslte_mod_bits_x_symbol(gsA.mcs[0].mod);
    gsB.mcs[0].idx = mB;
    gsB.mcs[0].mod = srslte_ra_mod_from_mcs(mB);
    gsB.mcs[0].tbs = srslte_ra_tbs_from_idx(srslte_ra_tbs_idx_from_mcs(mB), 100);
    gsB.Qm[0] = srslte_mod_bits_x_symbol(gsB.mcs[0].mod);
    for (int i = 0; i < gsA.mcs[0].tbs / 8; i++) dtA[i] = (uint8_t)(urand() * 256);
    for (int i = 0; i < gsB.mcs[0].tbs / 8; i++) dtB[i] = (uint8_t)(urand() * 256);
    srslte_softbuffer_tx_reset(&tA);
    srslte_softbuffer_tx_reset(&tB);
    srslte_softbuffer_rx_reset(&rA);
    srslte_softbuffer_rx_reset(&rB);
    srsgpu_shim_softbuffer_rx_reset(&gA);
    srsgpu_shim_softbuffer_rx_reset(&gB);
    /* A rv 0, B rv 0, A rv 2, B rv 2, A rv 3, A rv 1 */
    const struct { int a; uint32_t rv; } seq[6] = {{1, 0}, {0, 0}, {1, 2}, {0, 2}, {1, 3}, {1, 1}};
    for (uint32_t s = 0; s < 6; s++) {
      const int isA = seq[s].a;
      srslte_pdsch_cfg_t c;
      memset(&c, 0, sizeof(c));
      if (srslte_pdsch_cfg(&c, big, isA ? &gsA : &gsB, 1, 2, (int)seq[s].rv))
        return 2;
      if (srslte_dlsch_encode2(&stx, &c, isA ? &tA : &tB, isA ? dtA : dtB, ebits, 0)) return 2;
      const uint32_t ne = c.nbits[0].nof_bits;
      /* weak first transmissions: LLRs of amplitude 6 in noise of deviation 12 */
      for (uint32_t i = 0; i < ne; i++) llr[i] = (int16_t)((ebit(ebits, i) ? 6 : -6) + 12.0f * gauss());
      memcpy(llr2, llr, sizeof(int16_t) * ne);
      memset(da, 0, 10000);
      memset(db, 0, 10000);
      const int r1 = srslte_dlsch_decode2(&sa, &c, isA ? &rA : &rB, llr, da, 0);
      const int r2 = srsgpu_shim_dlsch_decode2(&sbs, &c, isA ? &gA : &gB, llr2, db, 0);
      srslte_softbuffer_rx_t *ra = isA ? &rA : &rB, *ga = isA ? &gA : &gB;
      int bad = r1 != r2 || sa.nof_iterations != sbs.nof_iterations || ra->tb_crc != ga->tb_crc ||
                memcmp(da, db, c.cb_segm[0].tbs / 8 + 3);
      for (uint32_t i = 0; i < c.cb_segm[0].C; i++) bad |= ra->cb_crc[i] != ga->cb_crc[i];
      if (bad)
        fprintf(stderr, "harq mismatch round %u step %u (%s rv %u): ret %d/%d noi %u/%u\n", round, s,
                isA ? "A" : "B", seq[s].rv, r1, r2, sa.nof_iterations, sbs.nof_iterations);
      nbad += bad;
      ntx++;
    }
  }
  printf("fault_cases=%u fault_failures=%u harq_tx=%u harq_mismatches=%u\n", ncases, nfail, ntx, nbad);
  return nfail || nbad ? 1 : 0;
}
