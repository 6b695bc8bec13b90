/*
 * TEST INFRASTRUCTURE (never shipped): time-domain drop-in check of integration/srslte_gpu_shim.c's
 * front end — srslte_ofdm_rx_sf, srslte_chest_dl_estimate_multi and srslte_pdsch_decode in one
 * receive chain, the way srsUE's ue_dl.c calls them (ue_dl.c:379-433).
 *
 * Per subframe: the reference encoder (srslte_pdsch_encode, pdsch.c:1048) fills the PDSCH REs, the
 * reference CRS (srslte_refsignal_cs_put_sf, refsignal_dl.c:380) is added, each rx antenna sees
 * its own channel (gain, phase, frequency slope) and noise, and a float64 inverse DFT with cyclic
 * prefixes (the inverse of ofdm.c:401-470, as oracle/ofdm_oracle.py:tx_sf with 1/N) makes the time
 * signal. Then on the GPU through the shim: OFDM demodulation (compared with the frequency grid),
 * channel estimation (the estimate compared with the true channel; noise_estimate, rsrp, rssi,
 * cfo written back into the reference object), and the PDSCH decode, compared bit for bit with
 * the reference CPU srslte_pdsch_decode fed the same GPU grids and estimates.
 *
 * ofdm.c and chest_dl.c need FFTW and cannot be compiled here, so the srslte_ofdm_t /
 * srslte_chest_dl_t objects are filled field by field as srslte_ofdm_rx_init (ofdm.c:47-104) and
 * srslte_chest_dl_init / _set_cell (chest_dl.c:150-160, 229-266) leave them, with srsUE's settings.
 *
 * Phases: (A) srsUE's default estimator (average_subframe, Gaussian filter order 4 / std dev 1,
 * REFS noise, neighbour RSRP, CFO on every subframe); then the cell changes (other PRB count and
 * cell id, so every GPU handle must be recreated), (B) per-symbol estimation with EMPTY noise,
 * whose value may change only in subframes 0 and 5 (chest_dl.c:628-637). Finally every object is
 * released (srsgpu_shim_release) and the registry must be empty.
 *
 * Built by `make -C oracle shim`; tests/test_integration.py runs it on the GPU.
 * Usage: shim_front nof_prb_a nof_prb_b cell_id mcs nof_rx nof_sf snr_db seed
 * Prints "sf=<n> acks=<n> mismatches=<n> ofdm_err=<max> ce_err=<max> recreated=<0|1> live=<n>".
 */
#include <complex.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "srslte/phy/ch_estimation/chest_dl.h"
#include "srslte/phy/ch_estimation/refsignal_dl.h"
#include "srslte/phy/dft/ofdm.h"
#include "srslte/phy/fec/softbuffer.h"
#include "srslte/phy/phch/pdsch.h"
#include "srslte/phy/phch/ra.h"
#include "srslte/phy/utils/vector.h"

int srsgpu_shim_pdsch_decode(srslte_pdsch_t *q, srslte_pdsch_cfg_t *cfg,
                             srslte_softbuffer_rx_t *softbuffers[SRSLTE_MAX_CODEWORDS],
                             cf_t *sf_symbols[SRSLTE_MAX_PORTS],
                             cf_t *ce[SRSLTE_MAX_PORTS][SRSLTE_MAX_PORTS], float noise_estimate,
                             uint16_t rnti, uint8_t *data[SRSLTE_MAX_CODEWORDS],
                             bool acks[SRSLTE_MAX_CODEWORDS]);
int srsgpu_shim_chest_dl_estimate_multi(srslte_chest_dl_t *q, cf_t *input[SRSLTE_MAX_PORTS],
                                        cf_t *ce[SRSLTE_MAX_PORTS][SRSLTE_MAX_PORTS], uint32_t sf_idx,
                                        uint32_t nof_rx_antennas);
void srsgpu_shim_ofdm_rx_sf(srslte_ofdm_t *q);
int srsgpu_shim_release(const void *owner);
int srsgpu_shim_softbuffer_rx_init(srslte_softbuffer_rx_t *q, uint32_t nof_prb);
void srsgpu_shim_softbuffer_rx_reset(srslte_softbuffer_rx_t *q);
void srsgpu_shim_softbuffer_rx_free(srslte_softbuffer_rx_t *q);
int srsgpu_shim_live(void);

static uint64_t rng = 1;
static double urand(void) {
  rng = rng * 6364136223846793005ULL + 1442695040888963407ULL;
  return ((rng >> 11) + 0.5) / 9007199254740992.0;
}
static double gauss(void) { return sqrt(-2.0 * log(urand())) * cos(2.0 * M_PI * urand()); }

/* the fields srslte_ofdm_rx_init sets (ofdm.c:50-64), normal CP, not MBSFN, unnormalised */
static void ofdm_fields(srslte_ofdm_t *q, uint32_t nof_prb, cf_t *in, cf_t *out) {
  memset(q, 0, sizeof(*q));
  q->symbol_sz = (uint32_t)srslte_symbol_sz(nof_prb);
  q->nof_symbols = SRSLTE_CP_NSYMB(SRSLTE_CP_NORM);
  q->cp = SRSLTE_CP_NORM;
  q->nof_re = nof_prb * SRSLTE_NRE;
  q->nof_guards = (q->symbol_sz - q->nof_re) / 2;
  q->slot_sz = SRSLTE_SLOT_LEN(q->symbol_sz);
  q->sf_sz = SRSLTE_SF_LEN(q->symbol_sz);
  q->in_buffer = in;
  q->out_buffer = out;
}

/* float64 inverse of the receive mapping: bins [N - nre/2, N) <- grid[0, nre/2), bins [1, 1 + nre/2)
 * <- grid[nre/2, nre), x = IDFT / N with the CP copied from the symbol tail */
static void tx_time(const cf_t *grid, uint32_t nof_prb, uint32_t N, cf_t *x) {
  const uint32_t nre = nof_prb * SRSLTE_NRE, h = nre / 2;
  const uint32_t cp0 = (uint32_t)ceil(160.0 * N / 2048), cp = (uint32_t)ceil(144.0 * N / 2048);
  double complex *X = calloc(N, sizeof(double complex)), *t = calloc(N, sizeof(double complex));
  double complex *tw = malloc(N * sizeof(double complex));
  for (uint32_t n = 0; n < N; n++) tw[n] = cexp(I * 2.0 * M_PI * (double)n / (double)N);
  uint32_t pos = 0;
  for (uint32_t s = 0; s < 14; s++) {
    memset(X, 0, N * sizeof(double complex));
    for (uint32_t i = 0; i < h; i++) {
      X[N - h + i] = grid[s * nre + i];
      X[1 + i] = grid[s * nre + h + i];
    }
    for (uint32_t n = 0; n < N; n++) {
      double complex acc = 0;
      for (uint32_t k = 0; k < N; k++)
        if (X[k] != 0) acc += X[k] * tw[((uint64_t)k * n) % N];
      t[n] = acc / (double)N;
    }
    const uint32_t c = (s % 7 == 0) ? cp0 : cp;
    for (uint32_t i = 0; i < c; i++) x[pos + i] = (cf_t)t[N - c + i];
    for (uint32_t i = 0; i < N; i++) x[pos + c + i] = (cf_t)t[i];
    pos += c + N;
  }
  free(X);
  free(t);
  free(tw);
}

/* srslte_chest_dl_set_smooth_filter_gauss (chest_dl.c:471-490) */
static void chest_gauss(srslte_chest_dl_t *q, uint32_t order, float std_dev) {
  const int len = (int)order + 1, center = (len - 1) / 2;
  float norm = 0.0f;
  for (int i = 0; i < len; i++) {
    q->smooth_filter[i] = expf(-powf(i - center, 2) / (2.0f * powf(std_dev, 2)));
    norm += q->smooth_filter[i];
  }
  for (int i = 0; i < len; i++) q->smooth_filter[i] *= 1.0f / norm;
  q->smooth_filter_len = (uint32_t)len;
}

/* srslte_chest_dl_get_noise_estimate (chest_dl.c:741-751) */
static float chest_noise(const srslte_chest_dl_t *q) {
  float n = 0;
  for (int i = 0; i < q->last_nof_antennas; i++) {
    float a = 0;
    for (uint32_t p = 0; p < q->cell.nof_ports; p++) a += q->noise_estimate[i][p];
    n += a / q->cell.nof_ports;
  }
  return q->last_nof_antennas ? n / q->last_nof_antennas : n;
}

int main(int argc, char **argv) {
  if (argc != 9) {
    fprintf(stderr, "usage: %s nof_prb_a nof_prb_b cell_id mcs nof_rx nof_sf snr_db seed\n", argv[0]);
    return 2;
  }
  const uint32_t prbs[2] = {(uint32_t)atoi(argv[1]), (uint32_t)atoi(argv[2])};
  const uint32_t cell_id0 = atoi(argv[3]), mcs = atoi(argv[4]), nof_rx = atoi(argv[5]);
  const uint32_t nof_sf = atoi(argv[6]);
  const float snr_db = (float)atof(argv[7]);
  rng = (uint64_t)atoll(argv[8]) * 2654435761ULL + 11;
  const uint16_t rnti = 0x4601;
  const uint32_t max_prb = 100;

  srslte_pdsch_t tx, rx;
  if (srslte_pdsch_init_enb(&tx, max_prb) || srslte_pdsch_init_ue(&rx, max_prb, nof_rx)) return 2;
  srslte_refsignal_t csr;
  if (srslte_refsignal_cs_init(&csr, max_prb)) return 2;
  const uint32_t nmax = SRSLTE_SF_LEN_RE(max_prb, SRSLTE_CP_NORM), tmax = SRSLTE_SF_LEN(2048);
  cf_t *txg = srslte_vec_malloc(sizeof(cf_t) * nmax);
  cf_t *ytrue[2], *grid[SRSLTE_MAX_PORTS] = {NULL}, *xt[2];
  cf_t *ce[SRSLTE_MAX_PORTS][SRSLTE_MAX_PORTS] = {{NULL}};
  srslte_ofdm_t ofdm[2];
  for (uint32_t a = 0; a < nof_rx; a++) {
    ytrue[a] = srslte_vec_malloc(sizeof(cf_t) * nmax);
    grid[a] = srslte_vec_malloc(sizeof(cf_t) * nmax);
    xt[a] = srslte_vec_malloc(sizeof(cf_t) * tmax);
    ce[0][a] = srslte_vec_malloc(sizeof(cf_t) * nmax);
  }
  srslte_chest_dl_t chest;
  memset(&chest, 0, sizeof(chest));
  srslte_softbuffer_tx_t sbt;
  srslte_softbuffer_rx_t sra, srb;
  if (srslte_softbuffer_tx_init(&sbt, max_prb) || srslte_softbuffer_rx_init(&sra, max_prb) ||
      srsgpu_shim_softbuffer_rx_init(&srb, max_prb))
    return 2;
  srslte_softbuffer_tx_t *sbt_p[SRSLTE_MAX_CODEWORDS] = {&sbt};
  srslte_softbuffer_rx_t *sra_p[SRSLTE_MAX_CODEWORDS] = {&sra}, *srb_p[SRSLTE_MAX_CODEWORDS] = {&srb};
  const size_t dl = 75376 / 8 + 16;
  uint8_t *dtx = calloc(dl, 1), *da = calloc(dl, 1), *db = calloc(dl, 1);
  uint8_t *dtx_p[SRSLTE_MAX_CODEWORDS] = {dtx}, *da_p[SRSLTE_MAX_CODEWORDS] = {da}, *db_p[SRSLTE_MAX_CODEWORDS] = {db};

  uint32_t nsf = 0, nacks = 0, nbad = 0, recreated = 1;
  double ofdm_err = 0, ce_err = 0;
  int live_a = -1;
  for (int phase = 0; phase < 2; phase++) {
    const uint32_t nof_prb = prbs[phase], cell_id = cell_id0 + phase;
    srslte_cell_t cell = {nof_prb, 1, cell_id, SRSLTE_CP_NORM, SRSLTE_PHICH_NORM, SRSLTE_PHICH_R_1};
    if (srslte_pdsch_set_cell(&tx, cell) || srslte_pdsch_set_cell(&rx, cell) ||
        srslte_pdsch_set_rnti(&tx, rnti) || srslte_pdsch_set_rnti(&rx, rnti) ||
        srslte_refsignal_cs_set_cell(&csr, cell))
      return 2;
    for (uint32_t a = 0; a < nof_rx; a++) ofdm_fields(&ofdm[a], nof_prb, xt[a], grid[a]);
    /* the chest object as srslte_chest_dl_init + _set_cell leave it, then srsUE's settings */
    chest.cell = cell;
    chest.noise_alg = phase == 0 ? SRSLTE_NOISE_ALG_REFS : SRSLTE_NOISE_ALG_EMPTY;
    chest.average_subframe = phase == 0;
    chest.rsrp_neighbour = true;
    chest.cfo_estimate_enable = phase == 0;
    chest.cfo_estimate_sf_mask = 1023;
    chest.smooth_filter_auto = false;
    chest_gauss(&chest, 4, 1.0f);
    for (uint32_t a = 0; a < nof_rx; a++) chest.noise_estimate[a][0] = -1.0f;

    srslte_ra_dl_grant_t grant;
    memset(&grant, 0, sizeof(grant));
    grant.nof_prb = nof_prb;
    for (uint32_t s = 0; s < 2; s++)
      for (uint32_t p = 0; p < nof_prb; p++) grant.prb_idx[s][p] = true;
    grant.tb_en[0] = true;
    grant.mcs[0].idx = mcs;
    grant.mcs[0].mod = srslte_ra_mod_from_mcs(mcs);
    grant.mcs[0].tbs = srslte_ra_tbs_from_idx(srslte_ra_tbs_idx_from_mcs(mcs), nof_prb);
    grant.Qm[0] = srslte_mod_bits_x_symbol(grant.mcs[0].mod);
    const uint32_t tbs = (uint32_t)grant.mcs[0].tbs, n = SRSLTE_SF_LEN_RE(nof_prb, SRSLTE_CP_NORM);
    const uint32_t N = ofdm[0].symbol_sz, nsc = nof_prb * SRSLTE_NRE;
    const float sigma2 = powf(10.0f, -snr_db / 10.0f);
    float noise_prev[2] = {-1.0f, -1.0f};

    for (uint32_t k = 0; k < nof_sf; k++, nsf++) {
      const uint32_t sf_idx = (k * 3 + phase) % 10;
      for (uint32_t i = 0; i < tbs / 8; i++) dtx[i] = (uint8_t)(urand() * 256);
      srslte_softbuffer_tx_reset(&sbt);
      srslte_softbuffer_rx_reset(&sra);
      srsgpu_shim_softbuffer_rx_reset(&srb);
      srslte_pdsch_cfg_t cfg;
      memset(&cfg, 0, sizeof(cfg));
      int rv[SRSLTE_MAX_CODEWORDS] = {0, 0};
      if (srslte_pdsch_cfg_mimo(&cfg, cell, &grant, 2, sf_idx, rv, SRSLTE_MIMO_TYPE_SINGLE_ANTENNA, 0)) return 2;
      memset(txg, 0, sizeof(cf_t) * n);
      cf_t *txp[SRSLTE_MAX_PORTS] = {txg};
      if (srslte_pdsch_encode(&tx, &cfg, sbt_p, dtx_p, rnti, txp)) return 2;
      srslte_refsignal_cs_put_sf(cell, 0, csr.pilots[0][sf_idx], txg);
      for (uint32_t a = 0; a < nof_rx; a++) {
        const double amp = 0.6 + 0.8 * urand(), ph = 2 * M_PI * urand(), slope = 0.01 * (urand() - 0.5);
        for (uint32_t i = 0; i < n; i++) {
          const uint32_t sc = i % nsc;
          const double complex h = amp * cexp(I * (ph + slope * sc));
          ytrue[a][i] = (cf_t)(h * txg[i] + sqrt(sigma2 / 2) * (gauss() + I * gauss()));
        }
        tx_time(ytrue[a], nof_prb, N, xt[a]);
        /* ---- shim OFDM ---- */
        srsgpu_shim_ofdm_rx_sf(&ofdm[a]);
        double emax = 0, ymax = 0;
        for (uint32_t i = 0; i < n; i++) {
          emax = fmax(emax, cabs(grid[a][i] - ytrue[a][i]));
          ymax = fmax(ymax, cabs(ytrue[a][i]));
        }
        ofdm_err = fmax(ofdm_err, emax / ymax);
        /* true channel kept for the estimate check */
        for (uint32_t i = 0; i < n; i++) ytrue[a][i] = (cf_t)(amp * cexp(I * (ph + slope * (i % nsc))));
      }
      /* ---- shim channel estimation ---- */
      if (srsgpu_shim_chest_dl_estimate_multi(&chest, grid, ce, sf_idx, nof_rx)) return 3;
      for (uint32_t a = 0; a < nof_rx; a++) {
        double e = 0, hp = 0;
        for (uint32_t i = 0; i < n; i++) {
          e += pow(cabs(ce[0][a][i] - ytrue[a][i]), 2);
          hp += pow(cabs(ytrue[a][i]), 2);
        }
        ce_err = fmax(ce_err, sqrt(e / hp));
        const float nz = chest.noise_estimate[a][0];
        int bad = !(isfinite(nz) && chest.rsrp[a][0] > 0 && chest.rssi[a][0] > 0 && chest.rsrp_corr[a][0] > 0);
        if (phase == 0) /* REFS: written every subframe */
          bad |= !(nz > 0);
        else if (sf_idx == 0 || sf_idx == 5) /* EMPTY: written in subframes 0 / 5 */
          bad |= !(nz >= 0) || nz == -1.0f;
        else
          bad |= nz != noise_prev[a];
        if (bad) fprintf(stderr, "sf %u rx %u: noise %g (before %g) rsrp %g\n", sf_idx, a, nz, noise_prev[a],
                         chest.rsrp[a][0]);
        nbad += bad;
        noise_prev[a] = nz;
      }
      if (phase == 0 && !isfinite(chest.cfo)) nbad++;
      /* ---- PDSCH: reference CPU vs shim GPU on the same grids / estimates ---- */
      const float noise_est = chest_noise(&chest) > 0 ? chest_noise(&chest) : sigma2;
      bool acka[SRSLTE_MAX_CODEWORDS] = {false, false}, ackb[SRSLTE_MAX_CODEWORDS] = {false, false};
      memset(da, 0, dl);
      memset(db, 0, dl);
      const int ra = srslte_pdsch_decode(&rx, &cfg, sra_p, grid, ce, noise_est, rnti, da_p, acka);
      const uint32_t noia = rx.last_nof_iterations[0];
      const int rb = srsgpu_shim_pdsch_decode(&rx, &cfg, srb_p, grid, ce, noise_est, rnti, db_p, ackb);
      const uint32_t noib = rx.last_nof_iterations[0];
      const int bad = ra != rb || acka[0] != ackb[0] || noia != noib || memcmp(da, db, tbs / 8) ||
                      sra.tb_crc != srb.tb_crc;
      if (bad)
        fprintf(stderr, "mismatch phase %d sf %u: ret %d/%d ack %d/%d noi %u/%u\n", phase, sf_idx, ra, rb,
                acka[0], ackb[0], noia, noib);
      if (acka[0] && memcmp(da, dtx, tbs / 8)) {
        fprintf(stderr, "phase %d sf %u: reference acked wrong data\n", phase, sf_idx);
        nbad++;
      }
      nbad += bad;
      nacks += acka[0];
    }
    const int live = srsgpu_shim_live();
    if (phase == 0) live_a = live;
    else recreated = live == live_a; /* same objects, new handles: no entry leaked */
  }
  int released = 0;
  for (uint32_t a = 0; a < nof_rx; a++) released += srsgpu_shim_release(&ofdm[a]);
  released += srsgpu_shim_release(&chest);
  released += srsgpu_shim_release(&rx);
  srsgpu_shim_softbuffer_rx_free(&srb);
  const int live = srsgpu_shim_live();
  if (released != (int)nof_rx + 2 || live != 0 || srsgpu_shim_release(&chest) != 0) nbad++;
  printf("sf=%u acks=%u mismatches=%u ofdm_err=%.3g ce_err=%.3g recreated=%d live=%d\n", nsf, nacks, nbad,
         ofdm_err, ce_err, recreated, live);
  return nbad || !recreated || ofdm_err > 1e-4 ? 1 : 0;
}
