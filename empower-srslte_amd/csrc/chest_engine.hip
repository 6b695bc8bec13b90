// Host side of the MI355X CRS channel estimator (include/srsgpu/chest_batch.h): cell-specific
// reference-signal table and per-call descriptors.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdio.h>
#include <string.h>
#include <vector>

#include "chest_kernels.h"
#include "host_ring.h"
#include "srsgpu/chest_batch.h"
#include "tdec_engine.h"

namespace srsgpu {

// CRS (refsignal_dl.c:265-318, 36.211 6.10.1.1): for slot ns and OFDM symbol lp in {0, 4} (ports
// 0/1; {0, 3} with extended CP) or {1} (ports 2/3), c_init = 2^10 (7(ns+1) + lp + 1)(2 N_ID + 1) +
// 2 N_ID + N_cp (N_cp 1 normal, 0 extended CP) and r(m) = ((1 - 2c(2m')) + j(1 - 2c(2m'+1))) /
// sqrt(2), m' = m + 110 - nof_prb.
// Layout: [10 subframes][4 symbols][2 nof_prb] of ports 0/1, then [10][2][2 nof_prb] of ports 2/3.
static void crs_table(uint32_t nprb, uint32_t id, bool ext, std::vector<float> &t) {
  const uint32_t np = 2 * nprb, len = 4 * 110, Nc = 1600;
  t.assign((size_t)10 * 6 * np * 2, 0.f);
  std::vector<uint8_t> x1(Nc + len + 31), x2(Nc + len + 31);
  for (uint32_t ns = 0; ns < 20; ns++)
    for (uint32_t l = 0; l < 3; l++) {
      const uint32_t lp = l == 0 ? 0 : l == 1 ? (ext ? 3 : 4) : 1;
      const uint32_t cinit = 1024 * (7 * (ns + 1) + lp + 1) * (2 * id + 1) + 2 * id + (ext ? 0 : 1);
      std::fill(x1.begin(), x1.end(), 0);
      std::fill(x2.begin(), x2.end(), 0);
      x1[0] = 1;
      for (int n = 0; n < 31; n++) x2[n] = (cinit >> n) & 1;
      for (uint32_t n = 0; n < Nc + len; n++) {
        x1[n + 31] = (x1[n + 3] + x1[n]) & 1;
        x2[n + 31] = (x2[n + 3] + x2[n + 2] + x2[n + 1] + x2[n]) & 1;
      }
      const uint32_t sf = ns / 2;
      const size_t row = l < 2 ? (size_t)sf * 4 + (ns % 2) * 2 + l : 40 + (size_t)sf * 2 + ns % 2;
      for (uint32_t m = 0; m < np; m++) {
        const uint32_t mp = m + 110 - nprb;
        const uint8_t c0 = (x1[2 * mp + Nc] + x2[2 * mp + Nc]) & 1;
        const uint8_t c1 = (x1[2 * mp + 1 + Nc] + x2[2 * mp + 1 + Nc]) & 1;
        const size_t o = (row * np + m) * 2;
        t[o] = (float)((1 - 2 * (float)c0) / sqrt(2));
        t[o + 1] = (float)((1 - 2 * (float)c1) / sqrt(2));
      }
    }
}

struct ChestEngine {
  hipStream_t st = nullptr;
  srsgpu_cell_t cell{};
  uint32_t cap = 0;
  float2 *d_crs = nullptr, *d_pss = nullptr;
  float *d_filt = nullptr;
  srsgpu_chest_cfg_t cfg{};
  int flen = 3;
  float filt[64] = {0.1f, 1 - 2 * 0.1f, 0.1f};
  bool filt_dirty = true;
  bool ce_rows = false; // srsgpu_chest_set_ce_rows
  ChestItem *d_items = nullptr;
  HostRing ring; // pinned item staging (host_ring.h)

  int create(const srsgpu_cell_t &c, uint32_t n) {
    if (c.nof_prb < 6 || c.nof_prb > 110 || c.id > 503 || !n || (c.nof_ports != 1 && c.nof_ports != 2 && c.nof_ports != 4) ||
        c.cp > 1) {
      fprintf(stderr, "srsgpu: invalid cell for channel estimation (1, 2 or 4 CRS ports, normal or extended CP)\n");
      return -1;
    }
    cell = c;
    cap = n;
    n *= c.nof_ports; // one work item per (grid, port)
    std::vector<float> t;
    crs_table(c.nof_prb, c.id, c.cp == 1, t);
    HIPCHK(hipMalloc(&d_crs, t.size() * 4));
    HIPCHK(hipMemcpy(d_crs, t.data(), t.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMalloc(&d_filt, 64 * 4));
    // PSS of N_id_2 = id % 3 for the PSS noise estimate (sync/pss.c:354-382)
    float pss[2 * 62];
    const float root[3] = {25.0f, 29.0f, 34.0f};
    for (int i = 0; i < 62; i++) { // the argument in double precision, rounded to float (pss.c:370-377)
      const float fi = (float)i;
      const float arg = i < 31 ? (float)((float)-1 * M_PI * root[c.id % 3] * (fi * (fi + 1.0)) / 63.0)
                               : (float)((float)-1 * M_PI * root[c.id % 3] * ((fi + 2.0) * (fi + 1.0)) / 63.0);
      pss[2 * i] = cosf(arg);
      pss[2 * i + 1] = sinf(arg);
    }
    HIPCHK(hipMalloc(&d_pss, sizeof(pss)));
    HIPCHK(hipMemcpy(d_pss, pss, sizeof(pss), hipMemcpyHostToDevice));
    cfg.symbol_sz = c.nof_prb <= 6 ? 128 : c.nof_prb <= 15 ? 256 : c.nof_prb <= 25 ? 384
                  : c.nof_prb <= 50 ? 768 : c.nof_prb <= 75 ? 1024 : 1536;
    HIPCHK(ring.create(sizeof(ChestItem) * n));
    HIPCHK(hipMalloc(&d_items, sizeof(ChestItem) * n));
    return 0;
  }

  void destroy() {
    if (st) (void)hipStreamSynchronize(st);
    for (void *p : {(void *)d_crs, (void *)d_pss, (void *)d_filt, (void *)d_items})
      if (p) (void)hipFree(p);
    ring.destroy();
  }

  int estimate(const uint32_t *sf_idx, uint32_t n, const float *d_grid, size_t stride, float *d_ce,
               float *d_noise, float *d_meas) {
    if (n > cap) {
      fprintf(stderr, "srsgpu: %u grids exceed the capacity %u\n", n, cap);
      return -1;
    }
    if (ce_rows && (cell.nof_ports > 2 || (cell.cp == 1 && !cfg.average_subframe))) {
      // the 4 compact rows are the normal-CP ports 0/1 layout; the averaged row fits any CP
      fprintf(stderr, "srsgpu: compact estimate rows need a 1- or 2-port cell, and average_subframe with extended CP\n");
      return -1;
    }
    hipError_t re;
    ChestItem *h_items = (ChestItem *)ring.acquire(&re);
    HIPCHK(re);
    if (filt_dirty) {
      HIPCHK(hipMemcpy(d_filt, filt, sizeof(filt), hipMemcpyHostToDevice));
      filt_dirty = false;
    }
    const uint32_t np = cell.nof_ports;
    for (uint32_t i = 0; i < n; i++) {
      if (sf_idx[i] > 9) return -1;
      for (uint32_t p = 0; p < np; p++) { // srslte_chest_dl_estimate_multi: every port per rx
        ChestItem &t = h_items[i * np + p];
        t.grid = (const float2 *)d_grid + i * stride;
        t.ce = (float2 *)d_ce + (i * np + p) * stride;
        t.noise = d_noise ? d_noise + i * np + p : nullptr;
        t.meas = d_meas ? d_meas + (size_t)(i * np + p) * 4 : nullptr;
        t.sf_idx = sf_idx[i];
        t.port = p;
        t.cfo = cfg.cfo_estimate_enable && ((1u << sf_idx[i]) & cfg.cfo_estimate_sf_mask); // chest_dl.c:607
        t.pad = 0;
      }
    }
    HIPCHK(ring.upload(d_items, h_items, sizeof(ChestItem) * n * np, st));
    HIPCHK(ring.mark(st));
    // chest_dl.c:620-621: no smoothing for an empty filter or a 3-tap one with w == 0
    ChestCfg kc;
    kc.nprb = (int)cell.nof_prb;
    kc.cell_id = (int)cell.id;
    kc.nof_ports = (int)np;
    kc.flen = (flen == 3 && filt[0] == 0.f) ? 0 : flen;
    kc.average = cfg.average_subframe ? 1 : 0;
    kc.noise_alg = (int)cfg.noise_alg;
    kc.filt_auto = cfg.smooth_filter_auto ? 1 : 0;
    kc.rsrp_neighbour = cfg.rsrp_neighbour ? 1 : 0;
    kc.cfo_n = (float)cfg.symbol_sz;
    kc.cfo_ng = ceilf((144.0f * (float)cfg.symbol_sz) / 2048.0f); // SRSLTE_CP_LEN_NORM(1, n)
    kc.rows = ce_rows ? 1 : 0;
    kc.ns = cell.cp == 1 ? 6 : 7;
    ProfScope ps("k_chest", st);
    HIPCHK(launch_chest(d_items, (int)(n * np), kc, d_crs, d_filt, d_pss, st));
    return 0;
  }

  int put_crs(const uint32_t *sf_idx, uint32_t n, float *d_grid, size_t stride) {
    if (n > cap) {
      fprintf(stderr, "srsgpu: %u grids exceed the capacity %u\n", n, cap);
      return -1;
    }
    hipError_t re;
    ChestItem *h_items = (ChestItem *)ring.acquire(&re);
    HIPCHK(re);
    const uint32_t np = cell.nof_ports;
    for (uint32_t i = 0; i < n; i++) {
      if (sf_idx[i] > 9) return -1;
      for (uint32_t p = 0; p < np; p++) {
        ChestItem &t = h_items[i * np + p];
        t.grid = nullptr;
        t.ce = (float2 *)d_grid + (i * np + p) * stride;
        t.noise = nullptr;
        t.meas = nullptr;
        t.cfo = 0;
        t.sf_idx = sf_idx[i];
        t.port = p;
      }
    }
    HIPCHK(ring.upload(d_items, h_items, sizeof(ChestItem) * n * np, st));
    HIPCHK(ring.mark(st));
    HIPCHK(launch_crs_put(d_items, (int)(n * np), (int)cell.nof_prb, (int)cell.id, cell.cp == 1 ? 6 : 7, d_crs, st));
    return 0;
  }
};

} // namespace srsgpu

struct srsgpu_chest {
  srsgpu::ChestEngine e;
};

extern "C" {

int srsgpu_chest_create(srsgpu_chest_t **q, const srsgpu_cell_t *cell, uint32_t n) {
  if (!q || !cell) return -1;
  auto *c = new srsgpu_chest();
  if (c->e.create(*cell, n)) {
    c->e.destroy();
    delete c;
    *q = nullptr;
    return -1;
  }
  *q = c;
  return 0;
}

void srsgpu_chest_destroy(srsgpu_chest_t *q) {
  if (!q) return;
  q->e.destroy();
  delete q;
}

void srsgpu_chest_set_stream(srsgpu_chest_t *q, void *s) {
  if (q) q->e.st = (hipStream_t)s;
}

int srsgpu_chest_set_smooth_filter(srsgpu_chest_t *q, const float *f, uint32_t len) {
  if (!q || len >= 65 || (len && !f)) { // chest_dl.c:427: below SRSLTE_CHEST_MAX_SMOOTH_FIL_LEN
    fprintf(stderr, "srsgpu: smoothing filter must be shorter than 65 taps\n");
    return -1;
  }
  q->e.flen = (int)len;
  for (uint32_t i = 0; i < len; i++) q->e.filt[i] = f[i];
  q->e.filt_dirty = true;
  return 0;
}

void srsgpu_chest_set_smooth_filter3_coeff(srsgpu_chest_t *q, float w) { // chest_dl.c:464-469
  if (!q) return;
  q->e.flen = 3;
  q->e.filt[0] = w;
  q->e.filt[2] = w;
  q->e.filt[1] = 1 - 2 * w;
  q->e.filt_dirty = true;
}

int srsgpu_chest_set_smooth_filter_gauss(srsgpu_chest_t *q, uint32_t order, float std_dev) {
  // chest_dl.c:475-494 in the reference's float arithmetic: exp(-(i - c)^2 / (2 std^2)) normalised
  // by its sum (accumulated in order); order 0 leaves the filter as it is
  if (!q || order + 1 >= 65) return -1;
  const uint32_t len = order + 1;
  const int c = (int)(len - 1) / 2;
  float f[64];
  for (uint32_t i = 0; i < len; i++) f[i] = expf(-powf((float)((int)i - c), 2) / (2.0f * powf(std_dev, 2)));
  float norm = 0.f;
  for (uint32_t i = 0; i < len; i++) norm += f[i];
  const float inv = 1.0f / norm;
  for (uint32_t i = 0; i < len; i++) f[i] *= inv;
  return srsgpu_chest_set_smooth_filter(q, f, len);
}

void srsgpu_chest_set_ce_rows(srsgpu_chest_t *q, int enable) {
  if (q) q->e.ce_rows = enable != 0;
}

int srsgpu_chest_set_cfg(srsgpu_chest_t *q, const srsgpu_chest_cfg_t *cfg) {
  if (!q || !cfg || cfg->noise_alg > 2 || !cfg->symbol_sz) return -1;
  q->e.cfg = *cfg;
  return 0;
}

int srsgpu_chest_get_cfg(const srsgpu_chest_t *q, srsgpu_chest_cfg_t *cfg) {
  if (!q || !cfg) return -1;
  *cfg = q->e.cfg;
  return 0;
}

int srsgpu_chest_estimate_meas_dev(srsgpu_chest_t *q, const uint32_t *sf_idx, uint32_t n, const float *d_grid,
                                   size_t stride, float *d_ce, float *d_noise, float *d_meas) {
  if (!q || (!sf_idx && n) || !d_grid || !d_ce) return -1;
  if (q->e.cfg.smooth_filter_auto && !d_noise) {
    fprintf(stderr, "srsgpu: smooth_filter_auto needs the noise estimate array\n");
    return -1;
  }
  return q->e.estimate(sf_idx, n, d_grid, stride, d_ce, d_noise, d_meas);
}

int srsgpu_chest_estimate_dev(srsgpu_chest_t *q, const uint32_t *sf_idx, uint32_t n, const float *d_grid,
                              size_t stride, float *d_ce, float *d_noise) {
  return srsgpu_chest_estimate_meas_dev(q, sf_idx, n, d_grid, stride, d_ce, d_noise, nullptr);
}

int srsgpu_chest_put_crs_dev(srsgpu_chest_t *q, const uint32_t *sf_idx, uint32_t n, float *d_grid,
                             size_t stride) {
  if (!q || (!sf_idx && n) || !d_grid) return -1;
  return q->e.put_crs(sf_idx, n, d_grid, stride);
}

} // extern "C"
