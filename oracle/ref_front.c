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
 *
 * Formats of IN / OUT: see the readers below (little-endian 32-bit words, complex float pairs);
 * tests/srsgpu_testlib.py (ref_front_chest / ref_front_dci) writes and reads them.
 */
#include <complex.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "srslte/phy/ch_estimation/chest_dl.h"
#include "srslte/phy/phch/dci.h"
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
 *     nsf x { sf_idx, grid[nrx][14*12*nof_prb] cf32 }
 * OUT per subframe: noise_before[nrx][nports] | ce[rx][port] grids | noise rsrp rssi rsrp_corr cfo
 *     [rx][port] (cfo: q->cfo right after that (rx, port) estimate) | get_noise_estimate get_snr
 *     get_rssi get_rsrq get_rsrp get_rsrp_neighbour get_cfo */
static int run_chest(void) {
  srslte_cell_t cell;
  memset(&cell, 0, sizeof(cell));
  cell.nof_prb = rd_u32();
  cell.id = rd_u32();
  cell.nof_ports = rd_u32();
  cell.cp = SRSLTE_CP_NORM;
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
  cell.nof_ports = rd_u32();
  cell.cp = SRSLTE_CP_NORM;
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

int main(int argc, char **argv) {
  if (argc != 4) {
    fprintf(stderr, "usage: ref_front chest|dci IN OUT\n");
    return 2;
  }
  fin = fopen(argv[2], "rb");
  fout = fopen(argv[3], "wb");
  if (!fin || !fout) return 2;
  int r = !strcmp(argv[1], "chest") ? run_chest() : !strcmp(argv[1], "dci") ? run_dci() : -1;
  fclose(fin);
  fclose(fout);
  return r ? 1 : 0;
}
