// Host side of the MI355X OFDM receiver (include/srsgpu/ofdm_batch.h): FFT plan (radix split and
// twiddle table) per symbol size.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdio.h>
#include <vector>

#include "ofdm_kernels.h"
#include "srsgpu/ofdm_batch.h"
#include "tdec_engine.h"

struct srsgpu_ofdm {
  hipStream_t st = nullptr;
  uint32_t nof_prb = 0, N = 0;
  float2 *d_tw = nullptr;
  uint32_t radices = 0;
  int nstages = 0;
  bool normalize = false;
  bool ext_cp = false; // srslte_cp_t SRSLTE_CP_EXT: 12 symbols per subframe
};

extern "C" {

// phy_common.c:227-275 srslte_symbol_sz (non-standard rates) / _power2 (standard rates)
int srsgpu_symbol_sz(uint32_t nof_prb, int standard_rates) {
  if (nof_prb == 0 || nof_prb > 110) return -1;
  if (nof_prb <= 6) return 128;
  if (nof_prb <= 15) return 256;
  if (nof_prb <= 25) return standard_rates ? 512 : 384;
  if (nof_prb <= 50) return standard_rates ? 1024 : 768;
  if (nof_prb <= 75) return standard_rates ? 1536 : 1024;
  return standard_rates ? 2048 : 1536;
}

int srsgpu_ofdm_rx_create(srsgpu_ofdm_t **q, uint32_t nof_prb, uint32_t symbol_sz) {
  if (!q) return -1;
  *q = nullptr;
  if (nof_prb < 6 || nof_prb > 110 || symbol_sz < 12 * nof_prb || symbol_sz > 2048) {
    fprintf(stderr, "srsgpu: invalid OFDM size (nof_prb=%u symbol_sz=%u)\n", nof_prb, symbol_sz);
    return -1;
  }
  // radix split: 4s first, then a 2, then 3s (N = 2^a 3^b)
  uint32_t n = symbol_sz, rad = 0;
  int ns = 0;
  std::vector<int> rs;
  while (n % 4 == 0) rs.push_back(4), n /= 4;
  while (n % 2 == 0) rs.push_back(2), n /= 2;
  while (n % 3 == 0) rs.push_back(3), n /= 3;
  if (n != 1 || rs.size() > 8) {
    fprintf(stderr, "srsgpu: symbol size %u is not 2^a 3^b\n", symbol_sz);
    return -1;
  }
  for (int r : rs) rad |= (uint32_t)r << (4 * ns++);
  auto *o = new srsgpu_ofdm();
  o->nof_prb = nof_prb;
  o->N = symbol_sz;
  o->radices = rad;
  o->nstages = ns;
  std::vector<float2> tw(symbol_sz);
  for (uint32_t k = 0; k < symbol_sz; k++) {
    const double a = -2.0 * M_PI * (double)k / (double)symbol_sz;
    tw[k] = make_float2((float)cos(a), (float)sin(a));
  }
  if (hipMalloc(&o->d_tw, symbol_sz * sizeof(float2)) != hipSuccess ||
      hipMemcpy(o->d_tw, tw.data(), symbol_sz * sizeof(float2), hipMemcpyHostToDevice) != hipSuccess) {
    if (o->d_tw) (void)hipFree(o->d_tw);
    delete o;
    return -1;
  }
  *q = o;
  return 0;
}

void srsgpu_ofdm_rx_destroy(srsgpu_ofdm_t *q) {
  if (!q) return;
  if (q->st) (void)hipStreamSynchronize(q->st);
  if (q->d_tw) (void)hipFree(q->d_tw);
  delete q;
}

void srsgpu_ofdm_rx_set_stream(srsgpu_ofdm_t *q, void *s) {
  if (q) q->st = (hipStream_t)s;
}

void srsgpu_ofdm_rx_set_normalize(srsgpu_ofdm_t *q, int enable) {
  if (q) q->normalize = enable != 0;
}

int srsgpu_ofdm_set_cp(srsgpu_ofdm_t *q, uint32_t cp) {
  if (!q || cp > 1) return -1;
  q->ext_cp = cp == 1;
  return 0;
}

int srsgpu_ofdm_rx_sf_dev(srsgpu_ofdm_t *q, uint32_t nof_sf, const float *d_in, size_t in_stride,
                          float *d_out, size_t out_stride) {
  if (!q || !d_in || !d_out) return -1;
  const size_t nsym = q->ext_cp ? 12 : 14;
  if (in_stride < 15 * (size_t)q->N || out_stride < nsym * 12 * q->nof_prb) return -1;
  const float scale = q->normalize ? 1.0f / sqrtf((float)q->N) : 1.0f;
  srsgpu::ProfScope ps("k_ofdm_rx", q->st);
  HIPCHK(srsgpu::launch_ofdm_rx((const float2 *)d_in, in_stride, (float2 *)d_out, out_stride, (int)nof_sf,
                                (int)q->N, (int)(12 * q->nof_prb), q->d_tw, q->radices, q->nstages, scale,
                                q->ext_cp, q->st));
  return 0;
}

int srsgpu_ofdm_tx_sf_dev(srsgpu_ofdm_t *q, uint32_t nof_sf, const float *d_in, size_t in_stride,
                          float *d_out, size_t out_stride) {
  if (!q || !d_in || !d_out) return -1;
  const size_t nsym = q->ext_cp ? 12 : 14;
  if (out_stride < 15 * (size_t)q->N || in_stride < nsym * 12 * q->nof_prb) return -1;
  const float scale = q->normalize ? 1.0f / sqrtf((float)q->N) : 1.0f;
  srsgpu::ProfScope ps("k_ofdm_tx", q->st);
  HIPCHK(srsgpu::launch_ofdm_tx((const float2 *)d_in, in_stride, (float2 *)d_out, out_stride, (int)nof_sf,
                                (int)q->N, (int)(12 * q->nof_prb), q->d_tw, q->radices, q->nstages, scale,
                                q->ext_cp, q->st));
  return 0;
}

} // extern "C"
