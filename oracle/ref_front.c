/* TEST INFRASTRUCTURE ONLY (never linked into the product library).
 *
 * Reference runner for the parts of the receive path whose source files reach the FFTW-backed DFT:
 * the reference's own ch_estimation/chest_dl.c (with sync/pss.c, utils/convolution.c,
 * resampling/interp.c, utils/filter.c) and ue/ue_dl.c (with phch/phich.c, phch/pmch.c, dft/ofdm.c),
 * compiled where they lie by `make -C oracle ref` and linked into this executable with the seven
 * srslte_dft_* symbols left unresolved (-Wl,--unresolved-symbols=ignore-in-object-files, lazy
 * binding). No stand-in is linked for them: the linker leaves them at address 0, and the
 * estimation and DCI-search paths below never call a DFT (a call would fault at once).
 * Paths relative to /root/reference/lib/src/phy.
 *
 *   ref_front chest IN OUT   srslte_chest_dl_init / set_cell / the srsUE setters, then
 *                            srslte_chest_dl_estimate_port over (rx antenna, port) in
 *                            srslte_chest_dl_estimate_multi's order (chest_dl.c:683-694) for a
 *                            sequence of subframes on ONE estimator object (so the PSS / EMPTY noise
 *                            state carries between subframes as in srsUE), recording CE grids, noise,
 *                            RSRP, RSSI, RSRP correlation, CFO and the getters after every subframe.
 *   ref_front dci IN OUT     srslte_pdcch_extract_llr_multi on given grids / estimates, then
 *                            srslte_ue_dl_find_dl_dci(_type) and srslte_ue_dl_find_ul_dci
 *                            (ue_dl.c:768-932) in phch_worker's order (DL search, then the UL search,
 *                            phch_worker.cc:548-806, 938-967) on ONE srslte_ue_dl_t, and
 *                            srslte_dci_msg_to_ul_grant (dci.c:165-197) of a found UL DCI.
 *   ref_front ue_dl IN OUT   srslte_ue_dl_decode_rnti's steps after the FFT (chest, PCFICH, PDCCH, DCI
 *                            search, grant, PDSCH) on given grids: the recorded-signal fixtures.
 *   ref_front pdsch_bench IN OUT   the CPU baseline of BASELINE configs[2] (bench.py): per pthread,
 *                            pinned to its own CPU, one srslte_chest_dl_t + srslte_pdsch_t +
 *                            softbuffer, running what srslte_ue_dl_decode_rnti runs after the FFT
 *                            (ue_dl.c:408-433, 580: srslte_chest_dl_estimate, the noise estimate,
 *                            srslte_pdsch_cfg, srslte_pdsch_decode with CRC early stop) over given
 *                            resource grids; prints one JSON line (wall time, subframes, acks,
 *                            code blocks that passed their CRC).
 *
 * Formats of IN / OUT: see the readers below (little-endian 32-bit words, complex float pairs);
 * tests/srsgpu_testlib.py (ref_front_chest / ref_front_dci) writes and reads them.
 */
#define _GNU_SOURCE
#include <complex.h>
#include <pthread.h>
#include <sched.h>
#include <time.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "srslte/phy/ch_estimation/chest_dl.h"
#include "srslte/phy/phch/dci.h"
#include "srslte/phy/phch/pdsch.h"
#include "srslte/phy/phch/ra.h"
#include "srslte/phy/phch/pdcch.h"
#include "srslte/phy/phch/ra.h"
#include "srslte/phy/phch/regs.h"
#include "srslte/phy/ue/ue_dl.h"
#include "srslte/phy/utils/vector.h"

static FILE *fin, *fout;

static uint32_t rd_u32(void) {
  uint32_t v;
  if (fread(&v, 4, 1, fin) != 1) {
    fprintf(stderr, "ref_front: short input\n");
    exit(2);
  }
  return v;
}
static float rd_f32(void) {
  float v;
  if (fread(&v, 4, 1, fin) != 1) {
    fprintf(stderr, "ref_front: short input\n");
    exit(2);
  }
  return v;
}
static void rd_buf(void *p, size_t bytes) {
  if (fread(p, 1, bytes, fin) != bytes) {
    fprintf(stderr, "ref_front: short input\n");
    exit(2);
  }
}
static void wr(const void *p, size_t bytes) {
  if (fwrite(p, 1, bytes, fout) != bytes) exit(3);
}
static void wr_f32(float v) { wr(&v, 4); }
static void wr_i32(int32_t v) { wr(&v, 4); }

/* IN: nof_prb id nof_ports nrx nsf | filt_mode(0 list, 1 gauss) flen filt[32] g_order g_std |
 *     smooth_auto average noise_alg rsrp_neighbour cfo_enable cfo_mask | noise_init |
 *     nsf x { sf_idx, grid[nrx][14*12*nof_prb] cf32 (12 rows with extended CP) }
 * OUT per subframe: noise_before[nrx][nports] | ce[rx][port] grids | noise rsrp rssi rsrp_corr cfo
 *     [rx][port] (cfo: q->cfo right after that (rx, port) estimate) | get_noise_estimate get_snr
 *     get_rssi get_rsrq get_rsrp get_rsrp_neighbour get_cfo */
static int run_chest(void) {
  srslte_cell_t cell;
  memset(&cell, 0, sizeof(cell));
  cell.nof_prb = rd_u32();
  cell.id = rd_u32();
  cell.nof_ports = rd_u32(); /* plus 256 for an extended-CP cell */
  cell.cp = (cell.nof_ports >> 8) & 1 ? SRSLTE_CP_EXT : SRSLTE_CP_NORM;
  cell.nof_ports &= 0xff;
  cell.phich_length = SRSLTE_PHICH_NORM;
  cell.phich_resources = SRSLTE_PHICH_R_1;
  const uint32_t nrx = rd_u32(), nsf = rd_u32();
  const uint32_t filt_mode = rd_u32(), flen = rd_u32();
  float filt[32];
  for (int i = 0; i < 32; i++) filt[i] = rd_f32();
  const uint32_t g_order = rd_u32();
  const float g_std = rd_f32();
  const uint32_t smooth_auto = rd_u32(), average = rd_u32(), noise_alg = rd_u32(), rsrp_nb = rd_u32(),
                 cfo_en = rd_u32(), cfo_mask = rd_u32();
  const float noise_init = rd_f32();

  srslte_chest_dl_t q;
  if (srslte_chest_dl_init(&q, cell.nof_prb) || srslte_chest_dl_set_cell(&q, cell)) return -1;
  if (filt_mode == 1)
    srslte_chest_dl_set_smooth_filter_gauss(&q, g_order, g_std);
  else
    srslte_chest_dl_set_smooth_filter(&q, flen ? filt : NULL, flen);
  srslte_chest_dl_set_smooth_filter_auto(&q, smooth_auto != 0);
  srslte_chest_dl_average_subframe(&q, average != 0);
  srslte_chest_dl_set_noise_alg(&q, (srslte_chest_dl_noise_alg_t)noise_alg);
  srslte_chest_dl_set_rsrp_neighbour(&q, rsrp_nb != 0);
  srslte_chest_dl_cfo_estimate_enable(&q, cfo_en != 0, cfo_mask);
  for (uint32_t a = 0; a < nrx; a++)
    for (uint32_t p = 0; p < cell.nof_ports; p++) q.noise_estimate[a][p] = noise_init;

  const uint32_t n = SRSLTE_SF_LEN_RE(cell.nof_prb, cell.cp);
  cf_t *in[SRSLTE_MAX_PORTS] = {NULL}, *ce[SRSLTE_MAX_PORTS][SRSLTE_MAX_PORTS] = {{NULL}};
  for (uint32_t a = 0; a < nrx; a++) {
    in[a] = srslte_vec_malloc(sizeof(cf_t) * n);
    for (uint32_t p = 0; p < cell.nof_ports; p++) ce[p][a] = srslte_vec_malloc(sizeof(cf_t) * n);
  }
  for (uint32_t s = 0; s < nsf; s++) {
    const uint32_t sf_idx = rd_u32();
    for (uint32_t a = 0; a < nrx; a++) rd_buf(in[a], sizeof(cf_t) * n);
    for (uint32_t a = 0; a < nrx; a++)
      for (uint32_t p = 0; p < cell.nof_ports; p++) wr_f32(q.noise_estimate[a][p]);
    float cfo[SRSLTE_MAX_PORTS][SRSLTE_MAX_PORTS];
    /* srslte_chest_dl_estimate_multi (chest_dl.c:683-694), one port estimate at a time so that the
     * CFO (a single q->cfo, overwritten by each) is seen per (antenna, port) */
    for (uint32_t a = 0; a < nrx; a++)
      for (uint32_t p = 0; p < cell.nof_ports; p++) {
        if (srslte_chest_dl_estimate_port(&q, in[a], ce[p][a], sf_idx, p, a)) return -1;
        cfo[a][p] = q.cfo;
      }
    q.last_nof_antennas = nrx;
    for (uint32_t a = 0; a < nrx; a++)
      for (uint32_t p = 0; p < cell.nof_ports; p++) wr(ce[p][a], sizeof(cf_t) * n);
    for (uint32_t a = 0; a < nrx; a++)
      for (uint32_t p = 0; p < cell.nof_ports; p++) {
        wr_f32(q.noise_estimate[a][p]);
        wr_f32(q.rsrp[a][p]);
        wr_f32(q.rssi[a][p]);
        wr_f32(q.rsrp_corr[a][p]);
        wr_f32(cfo[a][p]);
      }
    wr_f32(srslte_chest_dl_get_noise_estimate(&q));
    wr_f32(srslte_chest_dl_get_snr(&q));
    wr_f32(srslte_chest_dl_get_rssi(&q));
    wr_f32(srslte_chest_dl_get_rsrq(&q));
    wr_f32(srslte_chest_dl_get_rsrp(&q));
    wr_f32(srslte_chest_dl_get_rsrp_neighbour(&q));
    wr_f32(srslte_chest_dl_get_cfo(&q));
  }
  for (uint32_t a = 0; a < nrx; a++) {
    free(in[a]);
    for (uint32_t p = 0; p < cell.nof_ports; p++) free(ce[p][a]);
  }
  srslte_chest_dl_free(&q);
  return 0;
}

static void wr_msg(int ret, const srslte_dci_msg_t *m, const srslte_dci_location_t *loc) {
  wr_i32(ret);
  wr_i32(ret == 1 ? (int32_t)m->format : -1);
  wr_i32(ret == 1 ? (int32_t)loc->L : 0);
  wr_i32(ret == 1 ? (int32_t)loc->ncce : 0);
  wr_i32(ret == 1 ? (int32_t)m->nof_bits : 0);
  uint8_t data[SRSLTE_DCI_MAX_BITS];
  memset(data, 0, sizeof(data));
  if (ret == 1) memcpy(data, m->data, SRSLTE_DCI_MAX_BITS);
  wr(data, sizeof(data));
}

/* IN: nof_prb id nof_ports nrx phich_len phich_res nsf |
 *     nsf x { sf_idx cfi noise(f32) dl_rnti tm rnti_type(i32) ul_rnti n_rb_ho
 *             y[nrx][n] cf32, h[port][rx][n] cf32 }   (n = 14*12*nof_prb)
 * OUT per subframe: nllr, llr[nllr] | DL: ret format L ncce nof_bits data[128] |
 *     UL (ul_rnti != 0): same | UL grant: ret, 11 ra_ul_dci fields, 10 ra_ul_grant fields |
 *     pending_ul_dci_rnti left in q */
static int run_dci(void) {
  srslte_cell_t cell;
  memset(&cell, 0, sizeof(cell));
  cell.nof_prb = rd_u32();
  cell.id = rd_u32();
  cell.nof_ports = rd_u32(); /* plus 256 for an extended-CP cell */
  cell.cp = (cell.nof_ports >> 8) & 1 ? SRSLTE_CP_EXT : SRSLTE_CP_NORM;
  cell.nof_ports &= 0xff;
  const uint32_t nrx = rd_u32();
  cell.phich_length = rd_u32() ? SRSLTE_PHICH_EXT : SRSLTE_PHICH_NORM;
  cell.phich_resources = (srslte_phich_resources_t)rd_u32();
  const uint32_t nsf = rd_u32();

  /* the parts of srslte_ue_dl_init / _set_cell the searches use (ue_dl.c:58-230): the REG map and
   * the PDCCH receiver; the FFT, estimator, PDSCH and PHICH objects are not created (the OFDM
   * object needs the DFT) and the searches never touch them */
  srslte_ue_dl_t *q = calloc(1, sizeof(srslte_ue_dl_t));
  q->cell = cell;
  if (srslte_regs_init(&q->regs, cell) || srslte_pdcch_init_ue(&q->pdcch, SRSLTE_MAX_PRB, nrx) /* as srsUE: ue_dl_init with SRSLTE_MAX_PRB */ ||
      srslte_pdcch_set_cell(&q->pdcch, &q->regs, cell))
    return -1;

  const uint32_t n = SRSLTE_SF_LEN_RE(cell.nof_prb, cell.cp);
  cf_t *y[SRSLTE_MAX_PORTS] = {NULL}, *h[SRSLTE_MAX_PORTS][SRSLTE_MAX_PORTS] = {{NULL}};
  for (uint32_t a = 0; a < nrx; a++) {
    y[a] = srslte_vec_malloc(sizeof(cf_t) * n);
    for (uint32_t p = 0; p < cell.nof_ports; p++) h[p][a] = srslte_vec_malloc(sizeof(cf_t) * n);
  }
  for (uint32_t s = 0; s < nsf; s++) {
    const uint32_t sf_idx = rd_u32(), cfi = rd_u32();
    const float noise = rd_f32();
    const uint16_t dl_rnti = (uint16_t)rd_u32();
    const uint32_t tm = rd_u32();
    const int32_t rnti_type = (int32_t)rd_u32();
    const uint16_t ul_rnti = (uint16_t)rd_u32();
    const uint32_t n_rb_ho = rd_u32();
    for (uint32_t a = 0; a < nrx; a++) rd_buf(y[a], sizeof(cf_t) * n);
    for (uint32_t p = 0; p < cell.nof_ports; p++)
      for (uint32_t a = 0; a < nrx; a++) rd_buf(h[p][a], sizeof(cf_t) * n);
    if (srslte_pdcch_extract_llr_multi(&q->pdcch, y, h, noise, sf_idx, cfi)) return -1;
    const uint32_t nllr = 72 * q->pdcch.nof_cce[cfi - 1];
    wr_i32((int32_t)nllr);
    wr(q->pdcch.llr, sizeof(float) * nllr);

    srslte_dci_msg_t msg;
    memset(&msg, 0, sizeof(msg));
    memset(&q->last_location, 0, sizeof(q->last_location));
    memset(&q->last_location_ul, 0, sizeof(q->last_location_ul)); /* a pending UL DCI sets it */
    int r = rnti_type < 0 ? srslte_ue_dl_find_dl_dci(q, tm, cfi, sf_idx, dl_rnti, &msg)
                          : srslte_ue_dl_find_dl_dci_type(q, tm, cfi, sf_idx, dl_rnti,
                                                          (srslte_rnti_type_t)rnti_type, &msg);
    wr_msg(r, &msg, &q->last_location);

    srslte_dci_msg_t ul;
    memset(&ul, 0, sizeof(ul));
    int ru = 0;
    if (ul_rnti) ru = srslte_ue_dl_find_ul_dci(q, cfi, sf_idx, ul_rnti, &ul);
    wr_msg(ru, &ul, &q->last_location_ul);
    srslte_ra_ul_dci_t d;
    srslte_ra_ul_grant_t g;
    memset(&d, 0, sizeof(d));
    memset(&g, 0, sizeof(g));
    int rg = -100;
    if (ru == 1) rg = srslte_dci_msg_to_ul_grant(&ul, cell.nof_prb, n_rb_ho, &d, &g, 0);
    wr_i32(rg);
    wr_i32((int32_t)d.freq_hop_fl);
    wr_i32((int32_t)d.type2_alloc.riv);
    wr_i32((int32_t)d.type2_alloc.L_crb);
    wr_i32((int32_t)d.type2_alloc.RB_start);
    wr_i32((int32_t)d.mcs_idx);
    wr_i32((int32_t)d.rv_idx);
    wr_i32((int32_t)d.n_dmrs);
    wr_i32((int32_t)d.ndi);
    wr_i32((int32_t)d.cqi_request);
    wr_i32((int32_t)d.tpc_pusch);
    wr_i32(0);
    wr_i32((int32_t)g.L_prb);
    wr_i32((int32_t)g.n_prb[0]);
    wr_i32((int32_t)g.n_prb[1]);
    wr_i32((int32_t)g.freq_hopping);
    wr_i32((int32_t)g.M_sc);
    wr_i32((int32_t)g.Qm);
    wr_i32((int32_t)g.mcs.mod);
    wr_i32((int32_t)g.mcs.tbs);
    wr_i32((int32_t)g.mcs.idx);
    wr_i32((int32_t)g.ncs_dmrs);
    wr_i32((int32_t)q->pending_ul_dci_rnti); /* a UL DCI no UL search took */
    /* every request starts from a ue_dl with no UL DCI pending, as after a subframe whose UL search took
     * it (phch_worker searches UL for the C-RNTI it searched DL for); the GPU search keeps no state
     * between subframes */
    q->pending_ul_dci_rnti = 0;
  }
  for (uint32_t a = 0; a < nrx; a++) {
    free(y[a]);
    for (uint32_t p = 0; p < cell.nof_ports; p++) free(h[p][a]);
  }
  srslte_pdcch_free(&q->pdcch);
  srslte_regs_free(&q->regs);
  free(q);
  return 0;
}

/* ---------------------------------------------------------------- recorded signals ---- */
/* srslte_ue_dl_decode_rnti (ue_dl.c:467-620) after its FFT, on given resource grids: the reference's
 * recorded-signal tests run srslte_ofdm_rx_sf on a capture (FFTW, absent here), so the grids come from
 * the numpy OFDM oracle and everything after the FFT is the reference's own code, called in
 * decode_rnti's order on ONE ue_dl-shaped object (built as srslte_ue_dl_init / _set_cell /
 * _set_rnti build it, minus the FFT objects): srslte_chest_dl_estimate_multi and
 * srslte_pcfich_decode_multi (the body of srslte_ue_dl_decode_estimate_mbsfn, :409-433, here with the
 * correlation kept), the noise estimate, srslte_pdcch_extract_llr_multi, srslte_ue_dl_find_dl_dci,
 * srslte_dci_msg_to_dl_grant, the redundancy versions and softbuffer resets (:498-534), the MIMO type
 * of the format (:536-566), srslte_ue_dl_cfg_grant and srslte_pdsch_decode (:580-584).
 * After the decode, phch_worker's per-subframe reads of the estimator (srslte_chest_dl_get_*,
 * phch_worker.cc:226-241, 301, 313, 1618-1628) and its TM3 / TM4 feedback (compute_ri, :522-540:
 * srslte_ue_dl_ri_select with 2 ports and 2 rx antennas, srslte_ue_dl_ri_pmi_select with 2 ports;
 * q->pmi is cleared before each subframe so that a subframe's PMI does not depend on the previous one).
 * IN: nof_prb id nof_ports nrx phich_len phich_res max_prb rnti tm nsf | filt_mode(0 list, 1 gauss, 2 the
 *     init default) flen filt[32] g_order g_std average noise_alg rsrp_neighbour cfo_enable cfo_mask |
 *     nsf x { tti, grid[nrx][n] cf32 }
 * OUT per subframe: cfi corr(f32) noise(f32) | DL search (wr_msg) | ret(i32) tbs(i32) rv(i32) mod(i32)
 *     ack(i32) noi(i32) nof_re(i32) | data[12000] | ce[port][rx] grids cf32 | getters: noise snr rssi rsrq
 *     rsrp rsrp_neighbour cfo (f32) | feedback: cn(f32) ri_tm3 ret_cn ri pmi pmi_l[2] ret_pmi (i32)
 *     sinr[2][4] (f32) */
static int run_ue_dl(void) {
  srslte_cell_t cell;
  memset(&cell, 0, sizeof(cell));
  cell.nof_prb = rd_u32();
  cell.id = rd_u32();
  cell.nof_ports = rd_u32();
  cell.cp = SRSLTE_CP_NORM;
  const uint32_t nrx = rd_u32();
  cell.phich_length = rd_u32() ? SRSLTE_PHICH_EXT : SRSLTE_PHICH_NORM;
  cell.phich_resources = (srslte_phich_resources_t)rd_u32();
  const uint32_t max_prb = rd_u32();
  const uint16_t rnti = (uint16_t)rd_u32();
  const uint32_t tm = rd_u32(), nsf = rd_u32();
  const uint32_t filt_mode = rd_u32(), flen = rd_u32();
  float filt[32];
  for (int i = 0; i < 32; i++) filt[i] = rd_f32();
  const uint32_t g_order = rd_u32();
  const float g_std = rd_f32();
  const uint32_t average = rd_u32(), noise_alg = rd_u32(), rsrp_nb = rd_u32(), cfo_en = rd_u32(),
                 cfo_mask = rd_u32();
  if (!nrx || nrx > 2 || max_prb < cell.nof_prb) return -1;

  srslte_ue_dl_t *q = calloc(1, sizeof(srslte_ue_dl_t));
  q->nof_rx_antennas = nrx;
  const uint32_t n = SRSLTE_SF_LEN_RE(cell.nof_prb, cell.cp), nmax = SRSLTE_SF_LEN_RE(max_prb, cell.cp);
  for (int j = 0; j < SRSLTE_MAX_PORTS; j++) {
    q->sf_symbols_m[j] = srslte_vec_malloc(nmax * sizeof(cf_t));
    for (int i = 0; i < SRSLTE_MAX_PORTS; i++) {
      q->ce_m[i][j] = srslte_vec_malloc(nmax * sizeof(cf_t));
      bzero(q->ce_m[i][j], nmax * sizeof(cf_t));
    }
  }
  for (int i = 0; i < SRSLTE_MAX_TB; i++) {
    q->softbuffers[i] = srslte_vec_malloc(sizeof(srslte_softbuffer_rx_t));
    if (srslte_softbuffer_rx_init(q->softbuffers[i], max_prb)) return -1;
  }
  q->cell = cell;
  if (srslte_chest_dl_init(&q->chest, max_prb) || srslte_pcfich_init(&q->pcfich, nrx) ||
      srslte_pdcch_init_ue(&q->pdcch, max_prb, nrx) || srslte_pdsch_init_ue(&q->pdsch, max_prb, nrx) ||
      srslte_regs_init(&q->regs, cell) || srslte_chest_dl_set_cell(&q->chest, cell) ||
      srslte_pcfich_set_cell(&q->pcfich, &q->regs, cell) || srslte_pdcch_set_cell(&q->pdcch, &q->regs, cell) ||
      srslte_pdsch_set_cell(&q->pdsch, cell))
    return -1;
  srslte_ue_dl_set_rnti(q, rnti);
  if (filt_mode == 1)
    srslte_chest_dl_set_smooth_filter_gauss(&q->chest, g_order, g_std);
  else if (filt_mode == 0)
    srslte_chest_dl_set_smooth_filter(&q->chest, flen ? filt : NULL, flen);
  srslte_chest_dl_average_subframe(&q->chest, average != 0);
  srslte_chest_dl_set_noise_alg(&q->chest, (srslte_chest_dl_noise_alg_t)noise_alg);
  srslte_chest_dl_set_rsrp_neighbour(&q->chest, rsrp_nb != 0);
  srslte_chest_dl_cfo_estimate_enable(&q->chest, cfo_en != 0, cfo_mask);
  uint8_t *data[SRSLTE_MAX_CODEWORDS] = {calloc(1, 100000), calloc(1, 100000)};
  for (uint32_t s = 0; s < nsf; s++) {
    const uint32_t tti = rd_u32(), sf_idx = tti % 10;
    for (uint32_t a = 0; a < nrx; a++) rd_buf(q->sf_symbols_m[a], sizeof(cf_t) * n);
    uint32_t cfi = 0;
    float corr = 0.f;
    srslte_chest_dl_estimate_multi(&q->chest, q->sf_symbols_m, q->ce_m, sf_idx, nrx);
    if (srslte_pcfich_decode_multi(&q->pcfich, q->sf_symbols_m, q->ce_m, srslte_chest_dl_get_noise_estimate(&q->chest),
                                   sf_idx, &cfi, &corr) < 0)
      return -1;
    const float noise = srslte_chest_dl_get_noise_estimate(&q->chest);
    wr_i32((int32_t)cfi);
    wr_f32(corr);
    wr_f32(noise);
    int32_t ret = 0, tbs = 0, rv = 0, mod = 0, ack = 0, noi = 0, nre = 0;
    srslte_dci_msg_t msg;
    memset(&msg, 0, sizeof(msg));
    memset(&q->last_location, 0, sizeof(q->last_location));
    int found = 0;
    if (cfi >= 1 && cfi <= 3) {
      if (srslte_pdcch_extract_llr_multi(&q->pdcch, q->sf_symbols_m, q->ce_m, noise, sf_idx, cfi)) return -1;
      found = srslte_ue_dl_find_dl_dci(q, tm, cfi, sf_idx, rnti, &msg);
    }
    wr_msg(found, &msg, &q->last_location);
    memset(data[0], 0, 100000);
    if (found == 1) {
      srslte_ra_dl_dci_t dci;
      srslte_ra_dl_grant_t grant;
      bool acks[SRSLTE_MAX_CODEWORDS] = {false, false};
      if (srslte_dci_msg_to_dl_grant(&msg, rnti, cell.nof_prb, cell.nof_ports, &dci, &grant)) return -1;
      int rvidx[SRSLTE_MAX_CODEWORDS] = {1};
      for (int i = 0; i < SRSLTE_MAX_CODEWORDS; i++) {
        if (!grant.tb_en[i]) continue;
        if (dci.rv_idx < 0) {
          const uint32_t k = (tti / 10 / 2) % 4;
          rvidx[i] = ((uint32_t)ceilf((float)1.5 * k)) % 4;
        } else {
          rvidx[i] = (uint32_t)(i == 0 ? dci.rv_idx : dci.rv_idx_1);
        }
        srslte_softbuffer_rx_reset_tbs(q->softbuffers[i], (uint32_t)grant.mcs[i].tbs);
      }
      srslte_mimo_type_t mimo = cell.nof_ports == 1 ? SRSLTE_MIMO_TYPE_SINGLE_ANTENNA : SRSLTE_MIMO_TYPE_TX_DIVERSITY;
      if (msg.format != SRSLTE_DCI_FORMAT1 && msg.format != SRSLTE_DCI_FORMAT1A && msg.format != SRSLTE_DCI_FORMAT1C)
        return -1; /* the recordings carry 1A / 1C only */
      if (srslte_ue_dl_cfg_grant(q, &grant, cfi, sf_idx, rvidx, mimo)) return -1;
      tbs = q->pdsch_cfg.grant.mcs[0].tbs;
      rv = rvidx[0];
      mod = (int32_t)q->pdsch_cfg.grant.mcs[0].mod;
      nre = (int32_t)q->pdsch_cfg.nbits[0].nof_re;
      if (q->pdsch_cfg.grant.mcs[0].mod > 0 && q->pdsch_cfg.grant.mcs[0].tbs >= 0) {
        const int r = srslte_pdsch_decode(&q->pdsch, &q->pdsch_cfg, q->softbuffers, q->sf_symbols_m, q->ce_m, noise,
                                          rnti, data, acks);
        ack = acks[0];
        noi = (int32_t)srslte_pdsch_last_noi_cw(&q->pdsch, 0);
        ret = r == SRSLTE_SUCCESS ? tbs : 0; /* ue_dl.c:612-616 */
      }
    }
    wr_i32(ret);
    wr_i32(tbs);
    wr_i32(rv);
    wr_i32(mod);
    wr_i32(ack);
    wr_i32(noi);
    wr_i32(nre);
    wr(data[0], 12000);
    for (uint32_t p = 0; p < cell.nof_ports; p++)
      for (uint32_t a = 0; a < nrx; a++) wr(q->ce_m[p][a], sizeof(cf_t) * n);
    wr_f32(srslte_chest_dl_get_noise_estimate(&q->chest));
    wr_f32(srslte_chest_dl_get_snr(&q->chest));
    wr_f32(srslte_chest_dl_get_rssi(&q->chest));
    wr_f32(srslte_chest_dl_get_rsrq(&q->chest));
    wr_f32(srslte_chest_dl_get_rsrp(&q->chest));
    wr_f32(srslte_chest_dl_get_rsrp_neighbour(&q->chest));
    wr_f32(srslte_chest_dl_get_cfo(&q->chest));
    float cn = 0.f;
    uint8_t ri3 = 0, ri4 = 0, pmi4 = 0;
    int ret_cn = -1, ret_pmi = -1;
    for (int l = 0; l < SRSLTE_MAX_LAYERS; l++) {
      q->pmi[l] = 0;
      for (int c = 0; c < SRSLTE_MAX_CODEBOOKS; c++) q->sinr[l][c] = 0.f;
    }
    if (cell.nof_ports == 2 && nrx == 2) ret_cn = srslte_ue_dl_ri_select(q, &ri3, &cn);
    if (cell.nof_ports == 2) ret_pmi = srslte_ue_dl_ri_pmi_select(q, &ri4, &pmi4, NULL);
    wr_f32(cn);
    wr_i32(ri3);
    wr_i32(ret_cn);
    wr_i32(ri4);
    wr_i32(pmi4);
    wr_i32((int32_t)q->pmi[0]);
    wr_i32((int32_t)q->pmi[1]);
    wr_i32(ret_pmi);
    for (int l = 0; l < 2; l++)
      for (int c = 0; c < 4; c++) wr_f32(q->sinr[l][c]);
  }
  return 0;
}

/* ---------------------------------------------------------------- CPU baseline ---- */
/* One worker's objects. They are built one after the other on the main thread: srslte_tcod_init /
 * srslte_tcod_free share unguarded static tables (turbocoder.c:48-79: the first init builds them, any
 * free releases them), so concurrent set-up races and a second free double-frees; the objects are
 * never freed (the process exits after the run). */
typedef struct {
  srslte_cell_t cell;
  uint32_t cfi, rnti, mcs, max_noi, nsf, nthreads, reps, cpu;
  int tid;
  const uint32_t *sf_idx;
  const cf_t *grids; /* nsf x SF_LEN_RE */
  pthread_barrier_t *bar;
  srslte_chest_dl_t chest;
  srslte_pdsch_t pdsch;
  srslte_softbuffer_rx_t sb;
  uint64_t decoded, acked, cb_ok, cb_bits_ok, noi_sum;
  int err;
} bench_arg_t;

static int bench_setup(bench_arg_t *a) {
  if (srslte_chest_dl_init(&a->chest, a->cell.nof_prb) || srslte_chest_dl_set_cell(&a->chest, a->cell) ||
      srslte_pdsch_init_ue(&a->pdsch, a->cell.nof_prb, 1) || srslte_pdsch_set_cell(&a->pdsch, a->cell) ||
      srslte_pdsch_set_rnti(&a->pdsch, (uint16_t)a->rnti) || srslte_softbuffer_rx_init(&a->sb, a->cell.nof_prb))
    return -1;
  srslte_pdsch_set_max_noi(&a->pdsch, a->max_noi);
  return 0;
}

static void *bench_thread(void *p) {
  bench_arg_t *a = (bench_arg_t *)p;
  cpu_set_t set;
  CPU_ZERO(&set);
  CPU_SET(a->cpu, &set);
  (void)pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
  const uint32_t n = SRSLTE_SF_LEN_RE(a->cell.nof_prb, a->cell.cp);
  srslte_chest_dl_t *chest = &a->chest;
  srslte_pdsch_t *pdsch = &a->pdsch;
  srslte_softbuffer_rx_t *sb = &a->sb;
  cf_t *sf = srslte_vec_malloc(sizeof(cf_t) * n), *ce[SRSLTE_MAX_PORTS] = {NULL};
  ce[0] = srslte_vec_malloc(sizeof(cf_t) * n);
  cf_t *sf_m[SRSLTE_MAX_PORTS] = {sf, NULL, NULL, NULL};
  cf_t *ce_m[SRSLTE_MAX_PORTS][SRSLTE_MAX_PORTS] = {{ce[0], NULL}, {NULL}};
  uint8_t *data[SRSLTE_MAX_CODEWORDS] = {srslte_vec_malloc(128 * 1024) /* >= TBS / 8 of any grant */, NULL};
  srslte_softbuffer_rx_t *sbs[SRSLTE_MAX_CODEWORDS] = {sb, NULL};
  srslte_ra_dl_grant_t grant;
  memset(&grant, 0, sizeof(grant));
  grant.nof_prb = a->cell.nof_prb;
  for (int sl = 0; sl < 2; sl++)
    for (uint32_t q = 0; q < a->cell.nof_prb; q++) grant.prb_idx[sl][q] = true;
  grant.tb_en[0] = true;
  grant.mcs[0].idx = a->mcs;
  grant.mcs[0].mod = srslte_ra_mod_from_mcs(a->mcs);
  grant.mcs[0].tbs = srslte_ra_tbs_from_idx(srslte_ra_tbs_idx_from_mcs(a->mcs), a->cell.nof_prb);
  grant.Qm[0] = srslte_mod_bits_x_symbol(grant.mcs[0].mod);
  pthread_barrier_wait(a->bar);
  for (uint32_t r = 0; r < a->reps && !a->err; r++) {
    for (uint32_t i = (uint32_t)a->tid; i < a->nsf; i += a->nthreads) {
      /* srslte_ue_dl_decode_estimate after the FFT (ue_dl.c:408-433), then ue_dl.c:580 */
      memcpy(sf, a->grids + (size_t)i * n, sizeof(cf_t) * n);
      if (srslte_chest_dl_estimate(chest, sf, ce, a->sf_idx[i])) {
        a->err = 2;
        break;
      }
      const float noise = srslte_chest_dl_get_noise_estimate(chest);
      srslte_pdsch_cfg_t cfg;
      if (srslte_pdsch_cfg(&cfg, a->cell, &grant, a->cfi, a->sf_idx[i], 0)) {
        a->err = 3;
        break;
      }
      srslte_softbuffer_rx_reset(sb); /* a new transport block every subframe */
      bool acks[SRSLTE_MAX_CODEWORDS] = {false, false};
      if (srslte_pdsch_decode(pdsch, &cfg, sbs, sf_m, ce_m, noise, (uint16_t)a->rnti, data, acks)) {
        a->err = 4;
        break;
      }
      a->decoded++;
      a->acked += acks[0];
      a->noi_sum += srslte_pdsch_last_noi_cw(pdsch, 0);
      for (uint32_t c = 0; c < cfg.cb_segm[0].C; c++)
        if (sb->cb_crc[c]) {
          a->cb_ok++;
          a->cb_bits_ok += c < cfg.cb_segm[0].C2 ? cfg.cb_segm[0].K2 : cfg.cb_segm[0].K1;
        }
    }
  }
  free(sf);
  free(ce[0]);
  free(data[0]);
  return NULL;
}

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

/* IN: nof_prb id cfi rnti mcs max_noi nthreads reps nsf ncpu cpus[ncpu] | nsf x {sf_idx, grid cf32}
 * (one rx antenna, one port: BASELINE configs[2]). OUT (text): one JSON object */
static int run_pdsch_bench(void) {
  srslte_cell_t cell;
  memset(&cell, 0, sizeof(cell));
  cell.nof_prb = rd_u32();
  cell.id = rd_u32();
  cell.nof_ports = 1;
  cell.cp = SRSLTE_CP_NORM;
  cell.phich_length = SRSLTE_PHICH_NORM;
  cell.phich_resources = SRSLTE_PHICH_R_1;
  const uint32_t cfi = rd_u32(), rnti = rd_u32(), mcs = rd_u32(), max_noi = rd_u32(), nthreads = rd_u32(),
                 reps = rd_u32(), nsf = rd_u32(), ncpu = rd_u32();
  if (!nthreads || !nsf || !ncpu || ncpu > 4096) return -1;
  uint32_t *cpus = malloc(sizeof(uint32_t) * ncpu), *sfi = malloc(sizeof(uint32_t) * nsf);
  for (uint32_t i = 0; i < ncpu; i++) cpus[i] = rd_u32();
  const uint32_t n = SRSLTE_SF_LEN_RE(cell.nof_prb, cell.cp);
  cf_t *grids = srslte_vec_malloc(sizeof(cf_t) * n * nsf);
  for (uint32_t i = 0; i < nsf; i++) {
    sfi[i] = rd_u32();
    rd_buf(grids + (size_t)i * n, sizeof(cf_t) * n);
  }
  pthread_barrier_t bar;
  pthread_barrier_init(&bar, NULL, nthreads + 1);
  bench_arg_t *args = calloc(nthreads, sizeof(bench_arg_t));
  pthread_t *th = malloc(sizeof(pthread_t) * nthreads);
  for (uint32_t t = 0; t < nthreads; t++) {
    bench_arg_t *a = &args[t];
    a->cell = cell;
    a->cfi = cfi;
    a->rnti = rnti;
    a->mcs = mcs;
    a->max_noi = max_noi;
    a->nsf = nsf;
    a->nthreads = nthreads;
    a->reps = reps;
    a->cpu = cpus[t % ncpu];
    a->tid = (int)t;
    a->sf_idx = sfi;
    a->grids = grids;
    a->bar = &bar;
    if (bench_setup(a)) return -1;
  }
  for (uint32_t t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, bench_thread, &args[t]);
  pthread_barrier_wait(&bar); /* every thread has built its objects */
  const double t0 = now_s();
  for (uint32_t t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  const double wall = now_s() - t0;
  uint64_t dec = 0, ack = 0, cbok = 0, bits = 0, noi = 0;
  int err = 0;
  for (uint32_t t = 0; t < nthreads; t++) {
    dec += args[t].decoded;
    ack += args[t].acked;
    cbok += args[t].cb_ok;
    bits += args[t].cb_bits_ok;
    noi += args[t].noi_sum;
    err |= args[t].err;
  }
  fprintf(fout,
          "{\"wall_s\": %.6f, \"subframes\": %llu, \"acked\": %llu, \"cb_ok\": %llu, \"cb_bits_ok\": %llu, "
          "\"noi_mean\": %.4f, \"threads\": %u, \"error\": %d}\n",
          wall, (unsigned long long)dec, (unsigned long long)ack, (unsigned long long)cbok, (unsigned long long)bits,
          dec ? (double)noi / (double)dec : 0.0, nthreads, err);
  free(args);
  free(th);
  free(grids);
  free(cpus);
  free(sfi);
  return err ? -1 : 0;
}

int main(int argc, char **argv) {
  if (argc != 4) {
    fprintf(stderr, "usage: ref_front chest|dci|ue_dl|pdsch_bench IN OUT\n");
    return 2;
  }
  fin = fopen(argv[2], "rb");
  fout = fopen(argv[3], "wb");
  if (!fin || !fout) return 2;
  int r = !strcmp(argv[1], "chest")         ? run_chest()
          : !strcmp(argv[1], "dci")         ? run_dci()
          : !strcmp(argv[1], "ue_dl")       ? run_ue_dl()
          : !strcmp(argv[1], "pdsch_bench") ? run_pdsch_bench()
                                            : -1;
  fclose(fin);
  fclose(fout);
  return r ? 1 : 0;
}
