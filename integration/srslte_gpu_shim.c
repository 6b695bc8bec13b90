/*
 * Reference-side binding: routes the srsLTE receive API onto libsrsgpu_phy.so.
 *
 * A maintainer adds this file to srsLTE's srslte_phy library (lib/src/phy/CMakeLists.txt) and
 * compiles it against srsLTE's own headers. It is not part of this repository's product library.
 * The GPU side is reached only through this repository's C ABI (include/srsgpu/ headers). The file
 * defines the receive entry points that srsLTE's ue_dl.c / pdsch_test.c call:
 *
 *   srslte_ofdm_rx_sf(q)                 (replaces dft/ofdm.c:460-470 for normal-CP subframes)
 *   srslte_chest_dl_estimate(_multi)(q, in, ce, sf_idx[, nof_rx])  (chest_dl.c:681-715, ports 0-1,
 *                                        every estimator setting of srsUE's phch_worker)
 *   srslte_pdsch_decode(q, cfg, sb, sf_symbols, ce, noise, rnti, data, acks)
 *                                        (pdsch.c:868-1007, TM1 single antenna port, TM2 transmit
 *                                        diversity, TM3 CDD, TM4 spatial multiplexing)
 *   srslte_dlsch_decode2(q, cfg, sb, e_bits, data, tb_idx)  (sch.c:506-517, 16- or 8-bit LLRs)
 *   srslte_ulsch_decode(q, cfg, sb, q_bits, g_bits, data)   (sch.c:883-889, no UCI: enb_ul.c's
 *                                        PUSCH data decode)
 *   srslte_rm_turbo_rx_lut(in, out, in_len, cb_idx, rv)      (rm_turbo.c:378-381)
 *   srslte_pcfich_decode_multi(q, sf, ce, noise, sf_idx, cfi, corr)  (pcfich.c:178-241)
 *   srslte_pdcch_extract_llr_multi(q, sf, ce, noise, sf_idx, cfi)      (pdcch.c:442-508)
 *   srslte_pdcch_decode_msg(q, msg, location, format, cfi, crc_rem)    (pdcch.c:366-420)
 *   srslte_softbuffer_rx_init / _free / _reset / _reset_tbs / _reset_cb  (softbuffer.c:46-153):
 *                                        the reference's host work, plus the GPU softbuffer state
 *   srsgpu_shim_release(q)               called from srslte_ofdm_rx_free / srslte_chest_dl_free /
 *                                        srslte_pdsch_free / srslte_sch_free / srslte_pcfich_free /
 *                                        srslte_pdcch_free
 *                                        (one added line each)
 *
 * Build it with -DSRSGPU_SHIM and drop the replaced functions from their reference translation
 * units. The reference objects keep their own state. This file keeps one GPU handle per object in
 * a small registry keyed by the object's address, because the reference structs have no spare
 * field. The registry is shared by srsUE's PHY worker threads (phch_worker.cc, one ue_dl per
 * worker): lookups and claims hold a mutex; a registered object is only used by the thread that
 * owns the object, as in the reference. Calls that are out of the GPU path's scope (MBSFN, frequency
 * shift, 3 ports, 4-port CDD / spatial multiplexing) return SRSLTE_ERROR and print a message. Normal
 * and extended CP and 1, 2 or 4 CRS ports run on the GPU. There is no
 * hidden CPU path behind them. Every device allocation and copy is checked: a failure returns
 * SRSLTE_ERROR (srslte_ofdm_rx_sf, void in the reference, prints and returns) and leaves the
 * object's GPU state released, so the next call starts afresh.
 * Each call moves one subframe host -> device -> host, as the reference API is per subframe.
 * Batch users call include/srsgpu/ headers directly and keep the data in HBM.
 */
#include <math.h>
#include <pthread.h>
#include <stdbool.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "srslte/phy/ch_estimation/chest_dl.h"
#include "srslte/phy/dft/ofdm.h"
#include "srslte/phy/fec/cbsegm.h"
#include "srslte/phy/fec/rm_turbo.h"
#include "srslte/phy/fec/softbuffer.h"
#include "srslte/phy/phch/pcfich.h"
#include "srslte/phy/phch/pdcch.h"
#include "srslte/phy/phch/pdsch.h"
#include "srslte/phy/phch/sch.h"

#include "srsgpu/chest_batch.h"
#include "srsgpu/dlsch_batch.h"
#include "srsgpu/ofdm_batch.h"
#include "srsgpu/pcfich_batch.h"
#include "srsgpu/pdcch_batch.h"
#include "srsgpu/pdsch_batch.h"
#include "srsgpu/ulsch_batch.h"
#include "srsgpu/viterbi_batch.h"

/* ---- HIP runtime entry points used for the host <-> device staging (libamdhip64) ---- */
typedef int hipError_t;
typedef void *hipStream_t;
extern hipError_t hipMalloc(void **ptr, size_t size);
extern hipError_t hipFree(void *ptr);
extern hipError_t hipMemcpy(void *dst, const void *src, size_t n, int kind);
extern hipError_t hipMemcpyAsync(void *dst, const void *src, size_t n, int kind, hipStream_t st);
extern hipError_t hipStreamCreate(hipStream_t *st);
extern hipError_t hipStreamDestroy(hipStream_t st);
extern hipError_t hipStreamSynchronize(hipStream_t st);
#define H2D 1
#define D2H 2

/* checked device allocation and copies: a failure prints and returns nonzero */
static int shim_alloc(void *p, size_t n) {
  void **pp = (void **)p;
  if (hipMalloc(pp, n ? n : 1) != 0) {
    *pp = NULL;
    fprintf(stderr, "srsgpu shim: hipMalloc of %zu bytes failed\n", n);
    return -1;
  }
  return 0;
}
static int shim_copy(void *dst, const void *src, size_t n, int kind) {
  if (n && hipMemcpy(dst, src, n, kind) != 0) {
    fprintf(stderr, "srsgpu shim: hipMemcpy of %zu bytes failed\n", n);
    return -1;
  }
  return 0;
}

/* ---- object registry ---- */
#define SHIM_MAX 64
typedef enum { SHIM_NONE = 0, SHIM_OFDM, SHIM_CHEST, SHIM_PDSCH, SHIM_SCH, SHIM_PCFICH, SHIM_PDCCH } shim_kind_t;
typedef struct {
  const void *owner;
  shim_kind_t kind;
  void *gpu;          /* srsgpu_ofdm_t / srsgpu_chest_t / srsgpu_pdsch_t */
  float *d_a, *d_b, *d_c, *d_d;
  uint32_t nof_prb, cell_id, aux; /* aux: FFT size (OFDM), CRS port count (chest, PDSCH), or
                                     e-bits capacity (SCH) */
  const void *sb[SHIM_MAX]; /* pdsch / sch: softbuffer object -> GPU softbuffer index */
} shim_entry_t;
static shim_entry_t shim[SHIM_MAX];
static pthread_mutex_t shim_mutex = PTHREAD_MUTEX_INITIALIZER;

static void shim_reset(shim_entry_t *e);

/* the entry of `owner`, claiming a free one if there is none */
static shim_entry_t *shim_get(const void *owner, shim_kind_t kind) {
  shim_entry_t *e = NULL;
  pthread_mutex_lock(&shim_mutex);
  for (int i = 0; i < SHIM_MAX && !e; i++)
    if (shim[i].owner == owner) e = &shim[i];
  if (e && e->kind != kind) {
    /* a freed object of another type whose free function has no release hook, and a new one at
     * the same address: drop the old type's GPU state with the old type's destructor */
    shim_reset(e);
    e->kind = kind;
  }
  for (int i = 0; i < SHIM_MAX && !e; i++)
    if (!shim[i].owner) {
      memset(&shim[i], 0, sizeof(shim[i]));
      shim[i].owner = owner;
      shim[i].kind = kind;
      e = &shim[i];
    }
  pthread_mutex_unlock(&shim_mutex);
  if (!e) fprintf(stderr, "srsgpu shim: more than %d live objects\n", SHIM_MAX);
  return e;
}

/* frees the entry's GPU handle and staging buffers; the entry stays claimed by its owner */
static void shim_reset(shim_entry_t *e) {
  if (e->gpu) {
    if (e->kind == SHIM_OFDM) srsgpu_ofdm_rx_destroy((srsgpu_ofdm_t *)e->gpu);
    if (e->kind == SHIM_CHEST) srsgpu_chest_destroy((srsgpu_chest_t *)e->gpu);
    if (e->kind == SHIM_PDSCH) srsgpu_pdsch_destroy((srsgpu_pdsch_t *)e->gpu);
    if (e->kind == SHIM_SCH) srsgpu_dlsch_destroy((srsgpu_dlsch_t *)e->gpu);
    if (e->kind == SHIM_PCFICH) srsgpu_pcfich_destroy((srsgpu_pcfich_t *)e->gpu);
    if (e->kind == SHIM_PDCCH) srsgpu_pdcch_destroy((srsgpu_pdcch_t *)e->gpu);
  }
  if (e->d_a) hipFree(e->d_a);
  if (e->d_b) hipFree(e->d_b);
  if (e->d_c) hipFree(e->d_c);
  if (e->d_d) hipFree(e->d_d);
  const void *owner = e->owner;
  const shim_kind_t kind = e->kind;
  memset(e, 0, sizeof(*e));
  e->owner = owner;
  e->kind = kind;
}

/* Releases the GPU state of a reference object: srslte_ofdm_rx_free (ofdm.c:356),
 * srslte_chest_dl_free (chest_dl.c:173), srslte_pdsch_free (pdsch.c:344) and srslte_sch_free
 * (sch.c:156) call it before they clear the object. Returns 1 if the object had GPU state. */
int srsgpu_shim_release(const void *owner) {
  shim_entry_t *e = NULL;
  pthread_mutex_lock(&shim_mutex);
  for (int i = 0; i < SHIM_MAX && !e; i++)
    if (owner && shim[i].owner == owner) e = &shim[i];
  if (e) {
    shim_reset(e);
    memset(e, 0, sizeof(*e)); /* free for the next object */
  }
  pthread_mutex_unlock(&shim_mutex);
  return e != NULL;
}

/* number of objects with GPU state (for tests) */
int srsgpu_shim_live(void) {
  int n = 0;
  pthread_mutex_lock(&shim_mutex);
  for (int i = 0; i < SHIM_MAX; i++) n += shim[i].owner != NULL;
  pthread_mutex_unlock(&shim_mutex);
  return n;
}

/* ------------------------------------------------------------------ OFDM ---- */
void srslte_ofdm_rx_sf(srslte_ofdm_t *q) {
  if (q->mbsfn_subframe || q->freq_shift) {
    fprintf(stderr, "srsgpu shim: only non-MBSFN, unshifted OFDM runs on the GPU\n");
    return;
  }
  const uint32_t nof_prb = q->nof_re / SRSLTE_NRE;
  shim_entry_t *e = shim_get(q, SHIM_OFDM);
  if (!e) return;
  const size_t nout = SRSLTE_SF_LEN_RE(nof_prb, q->cp);
  const uint32_t ext = q->cp == SRSLTE_CP_EXT;
  if (e->aux != 2 * q->symbol_sz + ext || e->nof_prb != nof_prb || !e->gpu) {
    shim_reset(e);
    if (srsgpu_ofdm_rx_create((srsgpu_ofdm_t **)&e->gpu, nof_prb, q->symbol_sz) ||
        srsgpu_ofdm_set_cp((srsgpu_ofdm_t *)e->gpu, ext) ||
        shim_alloc(&e->d_a, sizeof(cf_t) * q->sf_sz) || shim_alloc(&e->d_b, sizeof(cf_t) * nout)) {
      shim_reset(e);
      fprintf(stderr, "srsgpu shim: srslte_ofdm_rx_sf: GPU setup failed\n");
      return;
    }
    e->aux = 2 * q->symbol_sz + ext;
    e->nof_prb = nof_prb;
  }
  srsgpu_ofdm_rx_set_normalize((srsgpu_ofdm_t *)e->gpu, q->fft_plan.norm);
  if (shim_copy(e->d_a, q->in_buffer, sizeof(cf_t) * q->sf_sz, H2D) ||
      srsgpu_ofdm_rx_sf_dev((srsgpu_ofdm_t *)e->gpu, 1, e->d_a, q->sf_sz, e->d_b, nout) ||
      shim_copy(q->out_buffer, e->d_b, sizeof(cf_t) * nout, D2H))
    fprintf(stderr, "srsgpu shim: srslte_ofdm_rx_sf failed\n");
}

/* ------------------------------------------------------------------ PCFICH ---- */
/* srslte_pcfich_decode_multi (pcfich.c:178-241): *cfi and *corr_result from the GPU
 * (srsgpu_pcfich_decode_dev), bit-exact; returns 1 as the reference. Only OFDM symbol 0 of the grids
 * is staged. The reference's scratch buffers in q (symbols, ce, d, data_f) are not filled. */
int srslte_pcfich_decode_multi(srslte_pcfich_t *q, cf_t *sf_symbols[SRSLTE_MAX_PORTS],
                               cf_t *ce[SRSLTE_MAX_PORTS][SRSLTE_MAX_PORTS], float noise_estimate,
                               uint32_t nsubframe, uint32_t *cfi, float *corr_result) {
  if (!q || !sf_symbols || nsubframe >= SRSLTE_NSUBFRAMES_X_FRAME) return SRSLTE_ERROR_INVALID_INPUTS;
  if (q->cell.nof_ports == 3 || q->cell.nof_ports > 4 || q->nof_rx_antennas > 2 || !ce) {
    fprintf(stderr, "srsgpu shim: GPU PCFICH covers 1, 2 or 4 ports, 1-2 rx antennas\n");
    return SRSLTE_ERROR;
  }
  shim_entry_t *e = shim_get(q, SHIM_PCFICH);
  if (!e) return SRSLTE_ERROR;
  const uint32_t np = q->cell.nof_ports, nrx = q->nof_rx_antennas, n = q->cell.nof_prb * SRSLTE_NRE;
  const uint32_t key = (np * 4 + nrx) * 2 + (q->cell.cp == SRSLTE_CP_EXT);
  if (e->nof_prb != q->cell.nof_prb || e->cell_id != q->cell.id || e->aux != key || !e->gpu) {
    shim_reset(e);
    srsgpu_cell_t c = {q->cell.nof_prb, q->cell.id, np, nrx, q->cell.cp == SRSLTE_CP_EXT};
    if (srsgpu_pcfich_create((srsgpu_pcfich_t **)&e->gpu, &c) || shim_alloc(&e->d_a, sizeof(cf_t) * n * 2) ||
        shim_alloc(&e->d_b, sizeof(cf_t) * n * 8) || shim_alloc(&e->d_c, sizeof(float) * 2)) { /* cfi, corr */
      shim_reset(e);
      return SRSLTE_ERROR;
    }
    e->nof_prb = q->cell.nof_prb;
    e->cell_id = q->cell.id;
    e->aux = key;
  }
  for (uint32_t a = 0; a < nrx; a++) {
    if (shim_copy(e->d_a + 2 * (size_t)a * n, sf_symbols[a], sizeof(cf_t) * n, H2D)) return SRSLTE_ERROR;
    for (uint32_t p = 0; p < np; p++) /* reference ce[port][rx]; GPU planes [rx][port] */
      if (shim_copy(e->d_b + 2 * (size_t)(a * np + p) * n, ce[p][a], sizeof(cf_t) * n, H2D)) return SRSLTE_ERROR;
  }
  const srsgpu_pcfich_sf_t sf = {0, 0, nsubframe, noise_estimate};
  if (srsgpu_pcfich_decode_dev((srsgpu_pcfich_t *)e->gpu, &sf, 1, e->d_a, e->d_b, n,
                               (uint32_t *)e->d_c, e->d_c + 1, NULL))
    return SRSLTE_ERROR;
  uint32_t out[2];
  if (shim_copy(out, e->d_c, sizeof(out), D2H)) return SRSLTE_ERROR;
  if (cfi) *cfi = out[0];
  if (corr_result) memcpy(corr_result, &out[1], sizeof(float));
  return 1;
}

/* ------------------------------------------------------------------ PDCCH ---- */
/* srslte_pdcch_extract_llr_multi (pdcch.c:442-508): the control symbols of the grids and estimates go
 * to the GPU (srsgpu_pdcch_extract_llr_dev); the 72 NOF_CCE(cfi) LLRs come back into q->llr, the rest
 * of q->llr zeroed as the reference does, bit-exact. The reference's scratch buffers (symbols, ce, x,
 * d) are not filled. */
#define SHIM_PDCCH_LLR_CAP (72 * 128)
int srslte_pdcch_extract_llr_multi(srslte_pdcch_t *q, cf_t *sf_symbols[SRSLTE_MAX_PORTS],
                                   cf_t *ce[SRSLTE_MAX_PORTS][SRSLTE_MAX_PORTS], float noise_estimate,
                                   uint32_t nsubframe, uint32_t cfi) {
  if (!q || nsubframe >= SRSLTE_NSUBFRAMES_X_FRAME || cfi < 1 || cfi > 3) return SRSLTE_ERROR_INVALID_INPUTS;
  if (q->cell.nof_ports == 3 || q->cell.nof_ports > 4 || q->nof_rx_antennas < 1 || q->nof_rx_antennas > 2 ||
      !sf_symbols || !ce) {
    fprintf(stderr, "srsgpu shim: GPU PDCCH covers 1, 2 or 4 ports, 1-2 rx antennas\n");
    return SRSLTE_ERROR;
  }
  shim_entry_t *e = shim_get(q, SHIM_PDCCH);
  if (!e) return SRSLTE_ERROR;
  const uint32_t np = q->cell.nof_ports, nrx = q->nof_rx_antennas, nprb = q->cell.nof_prb;
  const uint32_t ext = q->cell.cp == SRSLTE_CP_EXT;
  const uint32_t key = (((q->cell.phich_length * 4u + q->cell.phich_resources) * 8u + np) * 4u + nrx) * 2u + ext;
  const size_t n = SRSLTE_SF_LEN_RE(nprb, q->cell.cp);
  if (e->nof_prb != nprb || e->cell_id != q->cell.id || e->aux != key || !e->gpu) {
    shim_reset(e);
    srsgpu_cell_t c = {nprb, q->cell.id, np, nrx, ext};
    if (srsgpu_pdcch_create((srsgpu_pdcch_t **)&e->gpu, &c, q->cell.phich_length, q->cell.phich_resources) ||
        shim_alloc(&e->d_a, sizeof(cf_t) * n * nrx) || shim_alloc(&e->d_b, sizeof(cf_t) * n * nrx * np) ||
        shim_alloc(&e->d_c, sizeof(float) * SHIM_PDCCH_LLR_CAP)) {
      shim_reset(e);
      fprintf(stderr, "srsgpu shim: srslte_pdcch_extract_llr_multi: GPU setup failed\n");
      return SRSLTE_ERROR;
    }
    e->nof_prb = nprb;
    e->cell_id = q->cell.id;
    e->aux = key;
  }
  const uint32_t e_bits = 72 * srsgpu_pdcch_nof_cce((srsgpu_pdcch_t *)e->gpu, cfi);
  if (e_bits != 72 * q->nof_cce[cfi - 1] || e_bits > SHIM_PDCCH_LLR_CAP || e_bits > q->max_bits) {
    fprintf(stderr, "srsgpu shim: PDCCH REG map differs from the object's (%u / %u CCEs)\n", e_bits / 72,
            q->nof_cce[cfi - 1]);
    return SRSLTE_ERROR;
  }
  /* only the control region is read: cfi symbols (cfi + 1 below 11 PRB) */
  const size_t nctrl = (size_t)(nprb <= 10 ? cfi + 1 : cfi) * nprb * SRSLTE_NRE;
  for (uint32_t a = 0; a < nrx; a++) {
    if (!sf_symbols[a] || shim_copy(e->d_a + 2 * (size_t)a * n, sf_symbols[a], sizeof(cf_t) * nctrl, H2D))
      return SRSLTE_ERROR;
    for (uint32_t p = 0; p < np; p++) /* reference ce[port][rx]; GPU planes [rx][port] */
      if (!ce[p][a] || shim_copy(e->d_b + 2 * (size_t)(a * np + p) * n, ce[p][a], sizeof(cf_t) * nctrl, H2D))
        return SRSLTE_ERROR;
  }
  const srsgpu_pdcch_sf_t sf = {0, 0, 0, nsubframe, cfi, noise_estimate, 0};
  if (srsgpu_pdcch_extract_llr_dev((srsgpu_pdcch_t *)e->gpu, &sf, 1, e->d_a, e->d_b, n, e->d_c, NULL))
    return SRSLTE_ERROR;
  bzero(q->llr, sizeof(float) * q->max_bits);
  if (shim_copy(q->llr, e->d_c, sizeof(float) * e_bits, D2H)) return SRSLTE_ERROR;
  return SRSLTE_SUCCESS;
}

/* srslte_pdcch_decode_msg (pdcch.c:366-420): the candidate's LLRs from q->llr through the GPU DCI
 * decoder (srsgpu_dci_decode_dev: the mean |llr| > 0.5 check, rate recovery, tail-biting Viterbi,
 * CRC remainder). msg->data receives nof_bits + 16 bits and *crc_rem the remainder as in the
 * reference; a candidate under the mean threshold leaves msg and *crc_rem untouched. */
#define SHIM_DCI_LLR_OFF 16                                  /* floats: after the descriptor */
#define SHIM_DCI_OUT_OFF (4 * (SHIM_DCI_LLR_OFF + SRSGPU_DCI_MAX_E)) /* bytes */
int srslte_pdcch_decode_msg(srslte_pdcch_t *q, srslte_dci_msg_t *msg, srslte_dci_location_t *location,
                            srslte_dci_format_t format, uint32_t cfi, uint16_t *crc_rem) {
  if (!q || !msg || !location || !srslte_dci_location_isvalid(location)) {
    if (location) fprintf(stderr, "Invalid parameters, location=%d,%d\n", location->ncce, location->L);
    return SRSLTE_ERROR_INVALID_INPUTS;
  }
  const uint32_t nof_cce = (cfi > 0 && cfi < 4) ? q->nof_cce[cfi - 1] : 0;
  const uint32_t E = 72u << location->L;
  if (location->ncce * 72 + E > nof_cce * 72) {
    fprintf(stderr, "Invalid location: nCCE: %d, L: %d, NofCCE: %d\n", location->ncce, location->L, nof_cce);
    return SRSLTE_ERROR_INVALID_INPUTS;
  }
  const uint32_t nof_bits = srslte_dci_format_sizeof(format, q->cell.nof_prb, q->cell.nof_ports);
  if (nof_bits > SRSGPU_DCI_MAX_BITS - 16) return SRSLTE_ERROR; /* the reference's buffers end there */
  shim_entry_t *e = shim_get(q, SHIM_PDCCH);
  if (!e) return SRSLTE_ERROR;
  if (!e->d_d && shim_alloc(&e->d_d, SHIM_DCI_OUT_OFF + SRSGPU_DCI_MAX_BITS + 16 + 4)) return SRSLTE_ERROR;
  /* one upload: the candidate descriptor, then its E LLRs */
  float stage[SHIM_DCI_LLR_OFF + SRSGPU_DCI_MAX_E];
  const srsgpu_dci_cand_t cand = {SHIM_DCI_LLR_OFF, SHIM_DCI_OUT_OFF, E, nof_bits};
  memcpy(stage, &cand, sizeof(cand));
  memcpy(stage + SHIM_DCI_LLR_OFF, &q->llr[location->ncce * 72], sizeof(float) * E);
  uint8_t *d = (uint8_t *)e->d_d;
  const size_t crc_off = SHIM_DCI_OUT_OFF + SRSGPU_DCI_MAX_BITS + 16; /* 2-byte aligned */
  if (shim_copy(d, stage, sizeof(float) * (SHIM_DCI_LLR_OFF + E), H2D) ||
      srsgpu_dci_decode_dev((const srsgpu_dci_cand_t *)d, 1, (const float *)d, d, (uint16_t *)(d + crc_off),
                            d + crc_off + 2, NULL))
    return SRSLTE_ERROR;
  uint8_t out[SRSGPU_DCI_MAX_BITS + 16 + 4];
  if (shim_copy(out, d + SHIM_DCI_OUT_OFF, sizeof(out), D2H)) return SRSLTE_ERROR;
  if (!out[SRSGPU_DCI_MAX_BITS + 16 + 2]) return SRSLTE_SUCCESS; /* mean |llr| <= 0.5: skipped */
  memcpy(msg->data, out, nof_bits + 16);
  if (crc_rem) memcpy(crc_rem, out + SRSGPU_DCI_MAX_BITS + 16, sizeof(uint16_t));
  msg->nof_bits = nof_bits;
  if (format == SRSLTE_DCI_FORMAT0 || format == SRSLTE_DCI_FORMAT1A)
    msg->format = msg->data[0] == 0 ? SRSLTE_DCI_FORMAT0 : SRSLTE_DCI_FORMAT1A; /* pdcch.c:398-403 */
  else
    msg->format = format;
  return SRSLTE_SUCCESS;
}

/* ------------------------------------------------------------------ channel estimation ---- */
/* srslte_chest_dl_set_smooth_filter_gauss (chest_dl.c:471-490): what smooth_filter_auto leaves in q */
static void shim_gauss(srslte_chest_dl_t *q, uint32_t order, float std_dev) {
  const uint32_t len = order + 1;
  const int center = (int)(len - 1) / 2;
  float norm = 0.0f;
  for (int i = 0; i < (int)len; i++) {
    q->smooth_filter[i] = expf(-powf(i - center, 2) / (2.0f * powf(std_dev, 2)));
    norm += q->smooth_filter[i];
  }
  for (uint32_t i = 0; i < len; i++) q->smooth_filter[i] *= 1.0f / norm;
  q->smooth_filter_len = len;
}

/* srslte_chest_dl_estimate_multi (chest_dl.c:681-694): every rx antenna x every CRS port, with
 * the reference object's settings (average_subframe, noise algorithm, smoothing filter or
 * smooth_filter_auto, neighbour RSRP, CFO mask); writes back what the reference writes into q:
 * noise_estimate, rsrp, rssi, rsrp_corr, cfo, last_nof_antennas (and the auto filter) */
int srslte_chest_dl_estimate_multi(srslte_chest_dl_t *q, cf_t *input[SRSLTE_MAX_PORTS],
                                   cf_t *ce[SRSLTE_MAX_PORTS][SRSLTE_MAX_PORTS], uint32_t sf_idx,
                                   uint32_t nof_rx_antennas) {
  if (q->cell.nof_ports == 3 || q->cell.nof_ports > 4 || nof_rx_antennas > 2) {
    fprintf(stderr, "srsgpu shim: GPU channel estimation covers 1, 2 or 4 CRS ports, 1-2 rx\n");
    return SRSLTE_ERROR;
  }
  shim_entry_t *e = shim_get(q, SHIM_CHEST);
  if (!e) return SRSLTE_ERROR;
  const uint32_t n = SRSLTE_SF_LEN_RE(q->cell.nof_prb, q->cell.cp), np = q->cell.nof_ports;
  const uint32_t key = np * 2 + (q->cell.cp == SRSLTE_CP_EXT);
  if (e->nof_prb != q->cell.nof_prb || e->cell_id != q->cell.id || e->aux != key || !e->gpu) {
    shim_reset(e);
    srsgpu_cell_t c = {q->cell.nof_prb, q->cell.id, np, 1, q->cell.cp == SRSLTE_CP_EXT};
    if (srsgpu_chest_create((srsgpu_chest_t **)&e->gpu, &c, 2) || shim_alloc(&e->d_a, sizeof(cf_t) * n * 2) ||
        shim_alloc(&e->d_b, sizeof(cf_t) * n * 8) ||
        shim_alloc(&e->d_c, sizeof(float) * 8 * 5)) { /* noise [8] + measurements [8][4] */
      shim_reset(e);
      return SRSLTE_ERROR;
    }
    e->nof_prb = q->cell.nof_prb;
    e->cell_id = q->cell.id;
    e->aux = key;
  }
  srsgpu_chest_t *g = (srsgpu_chest_t *)e->gpu;
  const srsgpu_chest_cfg_t cfg = {q->average_subframe, (uint32_t)q->noise_alg, q->smooth_filter_auto,
                                  q->rsrp_neighbour, q->cfo_estimate_enable, q->cfo_estimate_sf_mask,
                                  (uint32_t)srslte_symbol_sz(q->cell.nof_prb)};
  if (srsgpu_chest_set_cfg(g, &cfg) ||
      srsgpu_chest_set_smooth_filter(g, q->smooth_filter, q->smooth_filter_len))
    return SRSLTE_ERROR;
  /* in/out state: the noise estimate (kept by PSS / EMPTY outside subframes 0 and 5) and the
   * measurements left untouched when disabled */
  float st[8 + 32];
  for (uint32_t a = 0; a < nof_rx_antennas; a++)
    for (uint32_t p = 0; p < np; p++) {
      float *m = &st[8 + 4 * (a * np + p)];
      st[a * np + p] = q->noise_estimate[a][p];
      m[0] = q->rsrp[a][p];
      m[1] = q->rssi[a][p];
      m[2] = q->rsrp_corr[a][p];
      m[3] = q->cfo;
    }
  if (shim_copy(e->d_c, st, sizeof(st), H2D)) return SRSLTE_ERROR;
  uint32_t sfs[2] = {sf_idx, sf_idx};
  for (uint32_t a = 0; a < nof_rx_antennas; a++)
    if (shim_copy(e->d_a + 2 * (size_t)a * n, input[a], sizeof(cf_t) * n, H2D)) return SRSLTE_ERROR;
  if (srsgpu_chest_estimate_meas_dev(g, sfs, nof_rx_antennas, e->d_a, n, e->d_b, e->d_c, e->d_c + 8))
    return SRSLTE_ERROR;
  if (shim_copy(st, e->d_c, sizeof(st), D2H)) return SRSLTE_ERROR;
  for (uint32_t a = 0; a < nof_rx_antennas; a++)
    for (uint32_t p = 0; p < np; p++) /* GPU order [rx][port]; reference ce[port][rx] */
      if (shim_copy(ce[p][a], e->d_b + 2 * (size_t)(a * np + p) * n, sizeof(cf_t) * n, D2H))
        return SRSLTE_ERROR;
  for (uint32_t a = 0; a < nof_rx_antennas; a++)
    for (uint32_t p = 0; p < np; p++) {
      const float *m = &st[8 + 4 * (a * np + p)];
      q->noise_estimate[a][p] = st[a * np + p];
      q->rsrp[a][p] = m[0];
      q->rssi[a][p] = m[1];
      q->rsrp_corr[a][p] = m[2];
      q->cfo = m[3]; /* the reference overwrites it per (rx, port): the last one stays */
      if (q->smooth_filter_auto) shim_gauss(q, 4, q->noise_estimate[a][p] * 200.0f);
    }
  q->last_nof_antennas = (int)nof_rx_antennas;
  return SRSLTE_SUCCESS;
}

/* srslte_chest_dl_estimate (chest_dl.c:696-715): one rx antenna */
int srslte_chest_dl_estimate(srslte_chest_dl_t *q, cf_t *input, cf_t *ce[SRSLTE_MAX_PORTS],
                             uint32_t sf_idx) {
  cf_t *in[SRSLTE_MAX_PORTS] = {input};
  cf_t *ce2[SRSLTE_MAX_PORTS][SRSLTE_MAX_PORTS];
  memset(ce2, 0, sizeof(ce2));
  for (uint32_t p = 0; p < q->cell.nof_ports && p < SRSLTE_MAX_PORTS; p++) ce2[p][0] = ce[p];
  return srslte_chest_dl_estimate_multi(q, in, ce2, sf_idx, 1);
}

/* ------------------------------------------------------------------ PDSCH ---- */
/* ------------------------------------------------------------------ softbuffers ---- */
/* The soft bits of a reference softbuffer live in HBM, in a slot of the decoding object's GPU
 * softbuffer pool. The srslte_softbuffer_rx_* drop-ins below do the reference's host work
 * (SHIM_CPU: softbuffer.c compiled with its rx functions renamed *_cpu) and record
 * how many leading code-block rows the caller reset; the next decode applies that to the slot. */
#ifndef SHIM_CPU
#define SHIM_CPU(f) f##_cpu
#endif
int SHIM_CPU(srslte_softbuffer_rx_init)(srslte_softbuffer_rx_t *q, uint32_t nof_prb);
void SHIM_CPU(srslte_softbuffer_rx_free)(srslte_softbuffer_rx_t *q);
void SHIM_CPU(srslte_softbuffer_rx_reset)(srslte_softbuffer_rx_t *q);
void SHIM_CPU(srslte_softbuffer_rx_reset_tbs)(srslte_softbuffer_rx_t *q, uint32_t tbs);
void SHIM_CPU(srslte_softbuffer_rx_reset_cb)(srslte_softbuffer_rx_t *q, uint32_t nof_cb);

#define SHIM_SB_MAX 1024
static struct {
  const void *sb;
  uint32_t reset_cb; /* leading rows reset since the last decode */
} shim_sbs[SHIM_SB_MAX];

static void shim_sb_mark(const srslte_softbuffer_rx_t *sb, uint32_t nof_cb) {
  pthread_mutex_lock(&shim_mutex);
  int slot = -1;
  for (int i = 0; i < SHIM_SB_MAX && slot < 0; i++)
    if (shim_sbs[i].sb == sb) slot = i;
  for (int i = 0; i < SHIM_SB_MAX && slot < 0; i++)
    if (!shim_sbs[i].sb) {
      shim_sbs[i].sb = sb;
      shim_sbs[i].reset_cb = 0;
      slot = i;
    }
  if (slot >= 0 && nof_cb > shim_sbs[slot].reset_cb) shim_sbs[slot].reset_cb = nof_cb;
  pthread_mutex_unlock(&shim_mutex);
  if (slot < 0) fprintf(stderr, "srsgpu shim: more than %d live softbuffers\n", SHIM_SB_MAX);
}

int srslte_softbuffer_rx_init(srslte_softbuffer_rx_t *q, uint32_t nof_prb) {
  const int ret = SHIM_CPU(srslte_softbuffer_rx_init)(q, nof_prb);
  if (ret == SRSLTE_SUCCESS) shim_sb_mark(q, q->max_cb);
  return ret;
}

void srslte_softbuffer_rx_free(srslte_softbuffer_rx_t *q) {
  pthread_mutex_lock(&shim_mutex);
  for (int i = 0; i < SHIM_SB_MAX; i++)
    if (shim_sbs[i].sb == q) shim_sbs[i].sb = NULL;
  for (int i = 0; i < SHIM_MAX; i++) /* its slots in every decoding object become free */
    for (int j = 0; j < SHIM_MAX; j++)
      if (shim[i].sb[j] == q) shim[i].sb[j] = NULL;
  pthread_mutex_unlock(&shim_mutex);
  SHIM_CPU(srslte_softbuffer_rx_free)(q);
}

void srslte_softbuffer_rx_reset(srslte_softbuffer_rx_t *q) {
  SHIM_CPU(srslte_softbuffer_rx_reset)(q);
  shim_sb_mark(q, q->max_cb);
}

void srslte_softbuffer_rx_reset_tbs(srslte_softbuffer_rx_t *q, uint32_t tbs) {
  SHIM_CPU(srslte_softbuffer_rx_reset_tbs)(q, tbs);
  shim_sb_mark(q, (tbs + 24) / (SRSLTE_TCOD_MAX_LEN_CB - 24) + 1); /* softbuffer.c:120-121 */
}

void srslte_softbuffer_rx_reset_cb(srslte_softbuffer_rx_t *q, uint32_t nof_cb) {
  SHIM_CPU(srslte_softbuffer_rx_reset_cb)(q, nof_cb);
  shim_sb_mark(q, nof_cb);
}

/* GPU softbuffer index of a reference softbuffer in the object's pool, with the resets recorded
 * since its last decode applied */
static int shim_softbuffer(shim_entry_t *e, srsgpu_dlsch_t *dl, srslte_softbuffer_rx_t *sb) {
  int slot = -1, fresh = 0;
  uint32_t nreset = 0;
  pthread_mutex_lock(&shim_mutex);
  for (int i = 0; i < SHIM_MAX && slot < 0; i++)
    if (e->sb[i] == sb) slot = i;
  for (int i = 0; i < SHIM_MAX && slot < 0; i++)
    if (!e->sb[i]) {
      e->sb[i] = sb;
      slot = i;
      fresh = 1;
    }
  for (int i = 0; i < SHIM_SB_MAX; i++)
    if (shim_sbs[i].sb == sb) {
      nreset = shim_sbs[i].reset_cb;
      shim_sbs[i].reset_cb = 0;
    }
  pthread_mutex_unlock(&shim_mutex);
  if (slot < 0) return -1;
  if (fresh || nreset >= sb->max_cb) /* a new slot starts reset (softbuffer_rx_init) */
    srsgpu_dlsch_softbuffer_reset(dl, (uint32_t)slot);
  else if (nreset > 0) /* softbuffer.c:127-150 zero the first nreset rows and every cb_crc flag */
    srsgpu_dlsch_softbuffer_reset_tbs(dl, (uint32_t)slot, (nreset - 1) * (SRSLTE_TCOD_MAX_LEN_CB - 24));
  return slot;
}

/* the code block CRC flags and tb_crc the reference leaves in the softbuffer (sch.c:404-408) */
static void shim_mirror_crc(srsgpu_dlsch_t *dl, uint32_t slot, srslte_softbuffer_rx_t *sb, uint32_t C) {
  uint8_t crc[SHIM_MAX];
  if (srsgpu_dlsch_softbuffer_read(dl, slot, NULL, crc) == 0) {
    for (uint32_t i = 0; i < sb->max_cb && i < SHIM_MAX; i++) sb->cb_crc[i] = crc[i] != 0;
    sb->tb_crc = true;
    for (uint32_t i = 0; i < C && sb->tb_crc; i++) sb->tb_crc = sb->cb_crc[i];
  }
}

/* ------------------------------------------------------------------ DL-SCH ---- */
/* The GPU DL-SCH object of a srslte_sch_t is created once, with a softbuffer pool sized for the
 * largest cell (every softbuffer's max_cb fits: softbuffer.c:56 sizes it from the cell's PRBs), so
 * the soft bits of every HARQ process survive any grant. Only the staging buffers grow. */
static uint32_t shim_sch_max_cb(void) {
  return (uint32_t)srslte_ra_tbs_from_idx(26, SRSLTE_MAX_PRB) / (SRSLTE_TCOD_MAX_LEN_CB - 24) + 1;
}

/* The GPU DL-SCH object of `q` with staging for nof_e LLR elements (d_a) and a TB of tbs bits
 * (d_b), and the GPU softbuffer index of `softbuffer`; NULL on failure */
static shim_entry_t *shim_sch_stage(srslte_sch_t *q, srslte_softbuffer_rx_t *softbuffer, uint32_t nof_e,
                                    uint32_t tbs, int *slot) {
  shim_entry_t *e = shim_get(q, SHIM_SCH);
  if (!e) return NULL;
  if (!e->gpu) {
    const uint32_t max_cb = shim_sch_max_cb();
    if (srsgpu_dlsch_create((srsgpu_dlsch_t **)&e->gpu, SHIM_MAX, max_cb, max_cb) ||
        shim_alloc(&e->d_c, 2 * sizeof(int32_t))) {
      shim_reset(e);
      return NULL;
    }
    e->nof_prb = max_cb; /* SCH entries: the pool's code blocks per softbuffer */
  }
  if (softbuffer->max_cb > e->nof_prb) {
    fprintf(stderr, "srsgpu shim: softbuffer with %u code blocks, the GPU pool holds %u\n",
            softbuffer->max_cb, e->nof_prb);
    return NULL;
  }
  /* staging: e-bits (d_a, capacity aux) and TB bytes (d_b, capacity cell_id) grow on demand */
  if (e->aux < nof_e || !e->d_a) {
    if (e->d_a) hipFree(e->d_a);
    e->d_a = NULL;
    e->aux = 0;
    if (shim_alloc(&e->d_a, sizeof(int16_t) * nof_e)) return NULL;
    e->aux = nof_e;
  }
  const uint32_t dlen = SRSGPU_DLSCH_DATA_LEN(tbs) + 16;
  if (e->cell_id < dlen || !e->d_b) {
    if (e->d_b) hipFree(e->d_b);
    e->d_b = NULL;
    e->cell_id = 0;
    if (shim_alloc(&e->d_b, dlen)) return NULL;
    e->cell_id = dlen;
  }
  *slot = shim_softbuffer(e, (srsgpu_dlsch_t *)e->gpu, softbuffer);
  return *slot < 0 ? NULL : e;
}

/* srslte_dlsch_decode2 (sch.c:506-517 -> decode_tb :430-497): one transport block from host
 * LLRs; sets q->nof_iterations (srslte_sch_last_noi) and the softbuffer's cb_crc / tb_crc */
int srslte_dlsch_decode2(srslte_sch_t *q, srslte_pdsch_cfg_t *cfg, srslte_softbuffer_rx_t *softbuffer,
                         int16_t *e_bits, uint8_t *data, int tb_idx) {
  if (!q || !cfg || !softbuffer || !e_bits || !data || tb_idx < 0 || tb_idx >= SRSLTE_MAX_CODEWORDS)
    return SRSLTE_ERROR_INVALID_INPUTS;
  const uint32_t Nl = cfg->nof_layers != (uint32_t)SRSLTE_RA_DL_GRANT_NOF_TB(&cfg->grant) ? 2 : 1;
  const uint32_t tbs = cfg->cb_segm[tb_idx].tbs, nof_e = cfg->nbits[tb_idx].nof_bits;
  int slot = -1;
  shim_entry_t *e = shim_sch_stage(q, softbuffer, nof_e, tbs, &slot);
  if (!e) return SRSLTE_ERROR;
  srsgpu_dlsch_t *dl = (srsgpu_dlsch_t *)e->gpu;
  srsgpu_dlsch_tb_t tb = {tbs, cfg->rv[tb_idx], cfg->grant.Qm[tb_idx] * Nl, nof_e, (uint32_t)slot, 0, 0};
  /* llr_is_8bit (sch.c:344-364): e_bits holds int8 LLRs; the GPU takes them as int16 elements */
  srsgpu_dlsch_set_llr_8bit(dl, q->llr_is_8bit);
  if (q->llr_is_8bit) {
    int16_t *w = malloc(sizeof(int16_t) * (nof_e ? nof_e : 1));
    if (!w) return SRSLTE_ERROR;
    for (uint32_t i = 0; i < nof_e; i++) w[i] = ((const int8_t *)e_bits)[i];
    const int r = shim_copy(e->d_a, w, sizeof(int16_t) * nof_e, H2D);
    free(w);
    if (r) return SRSLTE_ERROR;
  } else if (shim_copy(e->d_a, e_bits, sizeof(int16_t) * nof_e, H2D)) {
    return SRSLTE_ERROR;
  }
  int32_t *d_ret = (int32_t *)e->d_c;
  uint32_t *d_noi = (uint32_t *)e->d_c + 1;
  if (srsgpu_dlsch_decode_dev(dl, &tb, 1, (const int16_t *)e->d_a, (uint8_t *)e->d_b, q->max_iterations,
                              d_ret, d_noi))
    return SRSLTE_ERROR;
  int32_t rn[2];
  if (shim_copy(rn, e->d_c, sizeof(rn), D2H)) return SRSLTE_ERROR;
  if (rn[0] != SRSLTE_ERROR_INVALID_INPUTS) {
    /* the TB and its CRC bytes (sch.c:466-468) */
    if (shim_copy(data, e->d_b, tbs / 8 + 3, D2H)) return SRSLTE_ERROR;
    q->nof_iterations = (uint32_t)rn[1];
    shim_mirror_crc(dl, (uint32_t)slot, softbuffer, cfg->cb_segm[tb_idx].C);
  }
  return rn[0];
}

/* ------------------------------------------------------------------ UL-SCH ---- */
/* srslte_ulsch_decode (sch.c:883-889 -> srslte_ulsch_uci_decode :944-985 without UCI): the channel
 * deinterleaver into g_bits and decode_tb on the GPU (srsgpu_ulsch_decode_dev), on the same GPU
 * softbuffer pool as the object's DL-SCH calls. Writes data, g_bits (the deinterleaved LLRs, as
 * the reference leaves them), q->nof_iterations and the softbuffer's cb_crc / tb_crc. RI / ACK bits
 * left on the object by srslte_ulsch_uci_decode_ri_ack (q->nof_ri_ack_bits) are out of scope. */
int srslte_ulsch_decode(srslte_sch_t *q, srslte_pusch_cfg_t *cfg, srslte_softbuffer_rx_t *softbuffer,
                        int16_t *q_bits, int16_t *g_bits, uint8_t *data) {
  if (!q || !cfg || !softbuffer || !q_bits || !g_bits || !data) return SRSLTE_ERROR_INVALID_INPUTS;
  if (q->nof_ri_ack_bits) {
    fprintf(stderr, "srsgpu shim: UL-SCH with RI / ACK bits is not on the GPU path\n");
    return SRSLTE_ERROR;
  }
  const uint32_t tbs = cfg->cb_segm.tbs, nb = cfg->nbits.nof_bits;
  int slot = -1;
  /* d_a holds the q bits in its first half and the g bits in its second */
  shim_entry_t *e = shim_sch_stage(q, softbuffer, 2 * nb, tbs, &slot);
  if (!e) return SRSLTE_ERROR;
  srsgpu_dlsch_t *dl = (srsgpu_dlsch_t *)e->gpu;
  const uint32_t Qm = cfg->grant.Qm, ns = cfg->nbits.nof_symb;
  if (!Qm || !ns || nb % (Qm * ns)) {
    fprintf(stderr, "srsgpu shim: UL-SCH with %u bits is not a %u x %u-column matrix\n", nb, Qm, ns);
    return SRSLTE_ERROR;
  }
  srsgpu_ulsch_tb_t tb = {tbs, cfg->rv, Qm, nb, ns, (uint32_t)slot, 0, 0};
  srsgpu_dlsch_set_llr_8bit(dl, 0);
  int16_t *d_q = (int16_t *)e->d_a, *d_g = (int16_t *)e->d_a + nb;
  if (shim_copy(d_q, q_bits, sizeof(int16_t) * nb, H2D)) return SRSLTE_ERROR;
  int32_t *d_ret = (int32_t *)e->d_c;
  uint32_t *d_noi = (uint32_t *)e->d_c + 1;
  if (tbs == 0) { /* sch.c:957-975: deinterleaved into g_bits, then nothing to decode */
    if (srsgpu_ulsch_deinterleave_dev(dl, &tb, 1, d_q, d_g) || shim_copy(g_bits, d_g, sizeof(int16_t) * nb, D2H))
      return SRSLTE_ERROR;
    return SRSLTE_SUCCESS;
  }
  if (srsgpu_ulsch_decode_dev(dl, &tb, 1, d_q, d_g, (uint8_t *)e->d_b, q->max_iterations, d_ret, d_noi))
    return SRSLTE_ERROR;
  int32_t rn[2];
  if (shim_copy(rn, e->d_c, sizeof(rn), D2H) || shim_copy(g_bits, d_g, sizeof(int16_t) * nb, D2H))
    return SRSLTE_ERROR;
  if (rn[0] != SRSLTE_ERROR_INVALID_INPUTS) {
    if (shim_copy(data, e->d_b, tbs / 8 + 3, D2H)) return SRSLTE_ERROR;
    q->nof_iterations = (uint32_t)rn[1];
    shim_mirror_crc(dl, (uint32_t)slot, softbuffer, cfg->cb_segm.C);
  }
  return rn[0];
}

/* srslte_rm_turbo_rx_lut (rm_turbo.c:378-381, :394-430): output[deinter[i % (3K+12)]] += input[i]
 * on host buffers, with the sub-block layout the AUTO decoder expects. Latency-bound by nature
 * (one code block per call). Every calling thread (srsUE's PHY workers) has a context of its own:
 * a GPU DL-SCH object, staging buffers and a stream, so workers do not serialise on one another;
 * the context is freed when the thread exits. */
typedef struct {
  srsgpu_dlsch_t *dl;
  int16_t *d_in, *d_out;
  uint32_t cap;
  hipStream_t st;
} shim_rm_t;
static pthread_key_t shim_rm_key;
static pthread_once_t shim_rm_once = PTHREAD_ONCE_INIT;
static void shim_rm_free(void *p) {
  shim_rm_t *c = (shim_rm_t *)p;
  if (!c) return;
  if (c->dl) srsgpu_dlsch_destroy(c->dl);
  if (c->d_in) hipFree(c->d_in);
  if (c->d_out) hipFree(c->d_out);
  if (c->st) hipStreamDestroy(c->st);
  free(c);
}
static void shim_rm_key_init(void) { (void)pthread_key_create(&shim_rm_key, shim_rm_free); }

/* this thread's context with room for in_len input elements, or NULL */
static shim_rm_t *shim_rm_ctx(uint32_t in_len) {
  (void)pthread_once(&shim_rm_once, shim_rm_key_init);
  shim_rm_t *c = (shim_rm_t *)pthread_getspecific(shim_rm_key);
  if (!c) {
    c = (shim_rm_t *)calloc(1, sizeof(*c));
    if (!c) return NULL;
    if (hipStreamCreate(&c->st) != 0 || srsgpu_dlsch_create(&c->dl, 1, 1, 1) ||
        shim_alloc(&c->d_out, sizeof(int16_t) * (3 * (SRSLTE_TCOD_MAX_LEN_CB + 32) + 12)) ||
        pthread_setspecific(shim_rm_key, c) != 0) {
      shim_rm_free(c);
      fprintf(stderr, "srsgpu shim: rate-dematching context setup failed\n");
      return NULL;
    }
    srsgpu_dlsch_set_stream(c->dl, c->st);
  }
  if (in_len > c->cap) {
    if (c->d_in) hipFree(c->d_in);
    c->d_in = NULL;
    c->cap = 0;
    if (shim_alloc(&c->d_in, sizeof(int16_t) * in_len)) return NULL;
    c->cap = in_len;
  }
  return c;
}
static int shim_copy_on(shim_rm_t *c, void *dst, const void *src, size_t n, int kind) {
  if (n && hipMemcpyAsync(dst, src, n, kind, c->st) != 0) {
    fprintf(stderr, "srsgpu shim: hipMemcpyAsync of %zu bytes failed\n", n);
    return -1;
  }
  return 0;
}

int srslte_rm_turbo_rx_lut(int16_t *input, int16_t *output, uint32_t in_len, uint32_t cb_idx, uint32_t rv_idx) {
  if (rv_idx >= 4 || cb_idx >= SRSLTE_NOF_TC_CB_SIZES || !input || !output) {
    printf("Invalid inputs rv_idx=%d, cb_idx=%d\n", rv_idx, cb_idx);
    return SRSLTE_ERROR_INVALID_INPUTS;
  }
  const uint32_t K = (uint32_t)srslte_cbsegm_cbsize(cb_idx), out_len = 3 * K + 12;
  shim_rm_t *c = shim_rm_ctx(in_len);
  if (!c || shim_copy_on(c, c->d_in, input, sizeof(int16_t) * in_len, H2D) ||
      shim_copy_on(c, c->d_out, output, sizeof(int16_t) * out_len, H2D) ||
      srsgpu_rm_turbo_rx_dev(c->dl, c->d_in, c->d_out, in_len, K, rv_idx, 1) ||
      shim_copy_on(c, output, c->d_out, sizeof(int16_t) * out_len, D2H) || hipStreamSynchronize(c->st) != 0)
    return SRSLTE_ERROR;
  return SRSLTE_SUCCESS;
}

/* srslte_rm_turbo_rx_lut_8bit (rm_turbo.c:432-469): the same on int8 buffers (sums wrapping at 8
 * bits, the 8-bit decoder's sub-block table), through int16 device elements */
int srslte_rm_turbo_rx_lut_8bit(int8_t *input, int8_t *output, uint32_t in_len, uint32_t cb_idx,
                                uint32_t rv_idx) {
  if (rv_idx >= 4 || cb_idx >= SRSLTE_NOF_TC_CB_SIZES || !input || !output) {
    printf("Invalid inputs rv_idx=%d, cb_idx=%d\n", rv_idx, cb_idx);
    return SRSLTE_ERROR_INVALID_INPUTS;
  }
  const uint32_t K = (uint32_t)srslte_cbsegm_cbsize(cb_idx), out_len = 3 * (K + 32) + 12;
  shim_rm_t *c = shim_rm_ctx(in_len);
  if (!c) return SRSLTE_ERROR;
  int16_t *w = malloc(sizeof(int16_t) * (in_len + out_len));
  if (!w) return SRSLTE_ERROR;
  int16_t *wo = w + in_len;
  for (uint32_t i = 0; i < in_len; i++) w[i] = input[i];
  for (uint32_t i = 0; i < out_len; i++) wo[i] = output[i];
  int ret = SRSLTE_ERROR;
  if (!shim_copy_on(c, c->d_in, w, sizeof(int16_t) * in_len, H2D) &&
      !shim_copy_on(c, c->d_out, wo, sizeof(int16_t) * out_len, H2D) &&
      !srsgpu_rm_turbo_rx_8bit_dev(c->dl, c->d_in, c->d_out, in_len, K, rv_idx) &&
      !shim_copy_on(c, wo, c->d_out, sizeof(int16_t) * out_len, D2H) && hipStreamSynchronize(c->st) == 0) {
    for (uint32_t i = 0; i < out_len; i++) output[i] = (int8_t)wo[i];
    ret = SRSLTE_SUCCESS;
  }
  free(w);
  return ret;
}

int srslte_pdsch_decode(srslte_pdsch_t *q, srslte_pdsch_cfg_t *cfg,
                        srslte_softbuffer_rx_t *softbuffers[SRSLTE_MAX_CODEWORDS],
                        cf_t *sf_symbols[SRSLTE_MAX_PORTS], cf_t *ce[SRSLTE_MAX_PORTS][SRSLTE_MAX_PORTS],
                        float noise_estimate, uint16_t rnti, uint8_t *data[SRSLTE_MAX_CODEWORDS],
                        bool acks[SRSLTE_MAX_CODEWORDS]) {
  if (!q || !cfg || !sf_symbols || !data) return SRSLTE_ERROR_INVALID_INPUTS;
  const uint32_t nof_tb = SRSLTE_RA_DL_GRANT_NOF_TB(&cfg->grant);
  const bool siso = cfg->mimo_type == SRSLTE_MIMO_TYPE_SINGLE_ANTENNA && q->cell.nof_ports == 1 &&
                    nof_tb == 1 && cfg->grant.tb_en[0] && q->nof_rx_antennas <= 2;
  const bool cdd = cfg->mimo_type == SRSLTE_MIMO_TYPE_CDD && q->cell.nof_ports == 2 && nof_tb == 2 &&
                   cfg->nof_layers == 2 && q->nof_rx_antennas == 2;
  /* TM2 / DCI 1A on a 2- or 4-port cell: SFBC (SFBC-FSTD) transmit diversity, one TB (precoding.c:1811-1818) */
  const bool txdiv = cfg->mimo_type == SRSLTE_MIMO_TYPE_TX_DIVERSITY && (q->cell.nof_ports == 2 || q->cell.nof_ports == 4) &&
                     nof_tb == 1 && cfg->grant.tb_en[0] && q->nof_rx_antennas <= 2;
  /* TM4 closed-loop spatial multiplexing (precoding.c:1715-1760): 2 TBs on 2 layers (2x2 MMSE) or
   * TB 0 on 1 layer (2x1 MRC), 2 ports, 2 rx */
  const bool sm = cfg->mimo_type == SRSLTE_MIMO_TYPE_SPATIAL_MULTIPLEX && q->cell.nof_ports == 2 &&
                  q->nof_rx_antennas == 2 &&
                  ((nof_tb == 2 && cfg->nof_layers == 2) || (nof_tb == 1 && cfg->nof_layers == 1 && cfg->grant.tb_en[0]));
  if ((!siso && !cdd && !txdiv && !sm) || q->llr_is_8bit != q->dl_sch.llr_is_8bit) {
    fprintf(stderr, "srsgpu shim: GPU PDSCH covers TM1 (1 port), TM2 transmit diversity (2 or 4 ports, 1-2 "
                    "rx), TM3 CDD (2 ports, 2 layers, 2 rx) and TM4 spatial multiplexing (2 ports, 2 rx, "
                    "1-2 layers), normal or extended CP, 16-bit or 8-bit LLRs (the same in the PDSCH and its "
                    "DL-SCH)\n");
    return SRSLTE_ERROR;
  }
  if (nof_tb == 1 && acks[0]) return SRSLTE_SUCCESS; /* pdsch.c:963-965 */
  if (nof_tb == 2 && acks[0] && acks[1]) return SRSLTE_SUCCESS;
  shim_entry_t *e = shim_get(q, SHIM_PDSCH);
  if (!e) return SRSLTE_ERROR;
  const uint32_t n = SRSLTE_SF_LEN_RE(q->cell.nof_prb, q->cell.cp), np = q->cell.nof_ports;
  const uint32_t max_tbs = (uint32_t)srslte_ra_tbs_from_idx(26, q->cell.nof_prb);
  const size_t dlen = SRSGPU_DLSCH_DATA_LEN(max_tbs) + 16;
  const uint32_t key = (np * 4 + q->nof_rx_antennas) * 2 + (q->cell.cp == SRSLTE_CP_EXT);
  if (e->nof_prb != q->cell.nof_prb || e->cell_id != q->cell.id || e->aux != key || !e->gpu) {
    shim_reset(e);
    srsgpu_cell_t c = {q->cell.nof_prb, q->cell.id, np, q->nof_rx_antennas, q->cell.cp == SRSLTE_CP_EXT};
    const uint32_t max_cb = max_tbs / (SRSLTE_TCOD_MAX_LEN_CB - 24) + 1; /* softbuffer.c:56 */
    if (srsgpu_pdsch_create((srsgpu_pdsch_t **)&e->gpu, &c, SHIM_MAX, max_cb, 1) ||
        shim_alloc(&e->d_a, sizeof(cf_t) * n * 2) || shim_alloc(&e->d_b, sizeof(cf_t) * n * 8) ||
        shim_alloc(&e->d_c, 2 * dlen) || shim_alloc(&e->d_d, 4 * sizeof(int32_t))) {
      shim_reset(e);
      return SRSLTE_ERROR;
    }
    e->nof_prb = q->cell.nof_prb;
    e->cell_id = q->cell.id;
    e->aux = key;
  }
  srsgpu_pdsch_t *g = (srsgpu_pdsch_t *)e->gpu;
  srsgpu_dlsch_t *dl = srsgpu_pdsch_get_dlsch(g);

  srsgpu_pdsch_sf_t sf;
  memset(&sf, 0, sizeof(sf));
  sf.sf_idx = cfg->sf_idx;
  sf.lstart = cfg->nbits[0].lstart;
  for (int s = 0; s < 2; s++)
    for (uint32_t p = 0; p < q->cell.nof_prb; p++) sf.prb_idx[s][p] = cfg->grant.prb_idx[s][p];
  sf.nof_re = cfg->nbits[0].nof_re;
  sf.rnti = rnti;
  sf.noise_estimate = noise_estimate;
  sf.scaling = q->rho_a != 0.0f ? q->rho_a : 1.0f; /* pdsch.c:924-927 */
  sf.mimo_type = cdd     ? SRSGPU_MIMO_CDD
                 : sm    ? SRSGPU_MIMO_SPATIAL_MULTIPLEX
                 : txdiv ? SRSGPU_MIMO_TX_DIVERSITY
                         : SRSGPU_MIMO_SINGLE_ANTENNA;
  sf.codebook_idx = sm ? cfg->codebook_idx : 0;
  sf.tb_cw_swap = cfg->tb_cw_swap ? 1 : 0;
  sf.grid_offset = 0;
  sf.ce_offset = 0;
  for (uint32_t t = 0; t < nof_tb; t++) {
    /* an acked TB is skipped as srslte_pdsch_decode skips it (pdsch.c:946-947): no decode */
    const int slot = acks[t] ? 0 : shim_softbuffer(e, dl, softbuffers[t]);
    if (slot < 0) return SRSLTE_ERROR;
    if (acks[t]) sf.skip_tb |= 1u << t;
    sf.mod[t] = (uint32_t)cfg->grant.mcs[t].mod;
    sf.tbs[t] = (uint32_t)cfg->grant.mcs[t].tbs;
    sf.rv[t] = cfg->rv[t];
    sf.softbuffer[t] = (uint32_t)slot;
    sf.data_offset[t] = t * dlen;
  }
  for (uint32_t a = 0; a < q->nof_rx_antennas; a++) {
    if (shim_copy(e->d_a + 2 * (size_t)a * n, sf_symbols[a], sizeof(cf_t) * n, H2D)) return SRSLTE_ERROR;
    for (uint32_t p = 0; p < np; p++) /* reference ce[port][rx] -> GPU [rx][port] planes */
      if (shim_copy(e->d_b + 2 * (size_t)(a * np + p) * n, ce[p][a], sizeof(cf_t) * n, H2D))
        return SRSLTE_ERROR;
  }
  srsgpu_pdsch_set_csi(g, q->csi_enabled);
  srsgpu_pdsch_set_llr_8bit(g, q->llr_is_8bit); /* pdsch.c:795-806 */
  int32_t *d_ret = (int32_t *)e->d_d;
  uint32_t *d_noi = (uint32_t *)e->d_d + 2;
  if (srsgpu_pdsch_decode_dev(g, &sf, 1, e->d_a, e->d_b, (size_t)n, (uint8_t *)e->d_c,
                              q->dl_sch.max_iterations, d_ret, d_noi))
    return SRSLTE_ERROR; /* RE count mismatch: pdsch.c:886-890 */
  int32_t ret[2] = {-1, -1};
  uint32_t noi[2] = {0, 0};
  if (shim_copy(ret, d_ret, sizeof(int32_t) * nof_tb, D2H) || shim_copy(noi, d_noi, sizeof(uint32_t) * nof_tb, D2H))
    return SRSLTE_ERROR;
  for (uint32_t t = 0; t < nof_tb; t++) {
    if (acks[t]) continue; /* already acked: the reference does not touch it */
    srslte_softbuffer_rx_t *sb = softbuffers[t];
    if (shim_copy(data[t], (uint8_t *)e->d_c + t * dlen, (size_t)sf.tbs[t] / 8, D2H)) return SRSLTE_ERROR;
    /* last_nof_iterations is indexed by codeword (pdsch.c:815) */
    const uint32_t cw = nof_tb == 2 ? (t ^ sf.tb_cw_swap) : 0;
    q->last_nof_iterations[cw] = noi[t];
    /* srslte_pdsch_codeword_decode (pdsch.c:811-822): ack on a good TB CRC; srslte_pdsch_decode
     * returns SRSLTE_SUCCESS whatever the codeword result (pdsch.c:966-985) */
    acks[t] = ret[t] == SRSLTE_SUCCESS;
    if (ret[t] != SRSLTE_ERROR_INVALID_INPUTS) shim_mirror_crc(dl, sf.softbuffer[t], sb, cfg->cb_segm[t].C);
  }
  return SRSLTE_SUCCESS;
}
