// srsgpu PCFICH engine: host-side RE map (regs.c:477-512, :622-665) and scrambling sequences
// (pcfich.c:96-101, sequences.c:42-44), per-call descriptors; the kernel is k_pcfich in
// pdsch_kernels.hip.
#include <hip/hip_runtime.h>

#include <cstring>
#include <vector>

#include "pdsch_kernels.h"
#include "srsgpu/pcfich_batch.h"

struct srsgpu_pcfich {
  srsgpu_cell_t cell;
  uint32_t idx[16];
  uint32_t *d_idx = nullptr, *d_seq = nullptr;
  srsgpu::PcfichItem *h_it = nullptr, *d_it = nullptr;
  uint32_t cap = 0;
  hipEvent_t copied = nullptr; // the last descriptor upload out of h_it has finished
  bool recorded = false;
  hipStream_t last = nullptr; // stream of the last call (its kernel may still read d_it)
  const float *d_noise = nullptr; // srsgpu_pcfich_set_noise_dev
};

// 36.211 7.2 Gold sequence, first 32 bits packed LSB first: x1 starts at 1, x2 at c_init, N_c = 1600
static uint32_t gold32(uint32_t c_init) {
  std::vector<uint8_t> x1(1600 + 32 + 31, 0), x2(1600 + 32 + 31, 0);
  x1[0] = 1;
  for (int i = 0; i < 31; i++) x2[i] = (c_init >> i) & 1;
  for (int n = 0; n < 1600 + 32; n++) {
    x1[n + 31] = x1[n + 3] ^ x1[n];
    x2[n + 31] = x2[n + 3] ^ x2[n + 2] ^ x2[n + 1] ^ x2[n];
  }
  uint32_t w = 0;
  for (int n = 0; n < 32; n++) w |= (uint32_t)(x1[n + 1600] ^ x2[n + 1600]) << n;
  return w;
}

extern "C" {

int srsgpu_pcfich_create(srsgpu_pcfich_t **q, const srsgpu_cell_t *cell) {
  if (!q || !cell || cell->nof_prb < 6 || cell->nof_prb > 110 || cell->id > 503 ||
      (cell->nof_ports != 1 && cell->nof_ports != 2 && cell->nof_ports != 4) || cell->nof_rx_ant < 1 || cell->nof_rx_ant > 2 ||
      cell->cp > 1) // the PCFICH REGs lie in symbol 0, the same for both CPs (regs.c:477-512)
    return -1;
  srsgpu_pcfich *p = new srsgpu_pcfich;
  p->cell = *cell;
  if (hipEventCreateWithFlags(&p->copied, hipEventDisableTiming)) {
    p->copied = nullptr;
    srsgpu_pcfich_destroy(p);
    return -1;
  }
  const uint32_t N = cell->nof_prb, k_hat = 6 * (cell->id % (2 * N)), vo = cell->id % 3;
  int n = 0;
  for (uint32_t i = 0; i < 4; i++) { // REG i, its subcarriers minus the CRS at vo, vo + 3
    const uint32_t k0 = (k_hat + (i * N / 2) * 6) % (N * 12);
    for (uint32_t s = 0; s < 6; s++)
      if (s != vo && s != vo + 3) p->idx[n++] = k0 + s;
  }
  uint32_t seq[10];
  for (uint32_t sf = 0; sf < 10; sf++) seq[sf] = gold32((sf + 1) * (2 * cell->id + 1) * 512 + cell->id);
  if (hipMalloc(&p->d_idx, sizeof(p->idx)) || hipMalloc(&p->d_seq, sizeof(seq)) ||
      hipMemcpy(p->d_idx, p->idx, sizeof(p->idx), hipMemcpyHostToDevice) ||
      hipMemcpy(p->d_seq, seq, sizeof(seq), hipMemcpyHostToDevice)) {
    srsgpu_pcfich_destroy(p);
    return -1;
  }
  *q = p;
  return 0;
}

void srsgpu_pcfich_destroy(srsgpu_pcfich_t *q) {
  if (!q) return;
  (void)hipFree(q->d_idx);
  (void)hipFree(q->d_seq);
  (void)hipFree(q->d_it);
  (void)hipHostFree(q->h_it);
  if (q->copied) (void)hipEventDestroy(q->copied);
  delete q;
}

void srsgpu_pcfich_set_noise_dev(srsgpu_pcfich_t *q, const float *d_noise) {
  if (q) q->d_noise = d_noise;
}

int srsgpu_pcfich_re_map(const srsgpu_pcfich_t *q, uint32_t idx[16]) {
  if (!q || !idx) return -1;
  memcpy(idx, q->idx, sizeof(q->idx));
  return 16;
}

int srsgpu_pcfich_decode_dev(srsgpu_pcfich_t *q, const srsgpu_pcfich_sf_t *sf, uint32_t nof_sf,
                             const float *d_grid, const float *d_ce, size_t ant_stride,
                             uint32_t *d_cfi, float *d_corr, void *hip_stream) {
  if (!q || (nof_sf && (!sf || !d_grid || !d_ce || !d_cfi || !d_corr))) return -1;
  if (nof_sf == 0) return 0;
  if (ant_stride < (size_t)q->cell.nof_prb * 12) return -1;
  hipStream_t st = (hipStream_t)hip_stream;
  // h_it is reused: wait until the previous call's upload out of it is done (not its kernel); on
  // the same stream the previous kernel's reads of d_it are ordered before the next upload, on
  // another stream wait for them
  if (q->recorded && (st == q->last ? hipEventSynchronize(q->copied) : hipStreamSynchronize(q->last)))
    return -1;
  if (nof_sf > q->cap) {
    if (q->recorded && hipStreamSynchronize(q->last)) return -1; // the last kernel reads d_it
    (void)hipFree(q->d_it);
    (void)hipHostFree(q->h_it);
    q->d_it = nullptr;
    q->h_it = nullptr;
    q->cap = 0;
    if (hipHostMalloc(&q->h_it, sizeof(srsgpu::PcfichItem) * nof_sf) ||
        hipMalloc(&q->d_it, sizeof(srsgpu::PcfichItem) * nof_sf))
      return -1;
    q->cap = nof_sf;
  }
  for (uint32_t i = 0; i < nof_sf; i++) {
    if (sf[i].sf_idx > 9) return -1;
    q->h_it[i] = {sf[i].grid_offset, sf[i].ce_offset, sf[i].sf_idx, sf[i].noise_estimate,
                  q->d_noise ? q->d_noise + i : nullptr};
  }
  if (hipMemcpyAsync(q->d_it, q->h_it, sizeof(srsgpu::PcfichItem) * nof_sf, hipMemcpyHostToDevice, st) ||
      hipEventRecord(q->copied, st))
    return -1;
  q->recorded = true;
  q->last = st;
  return srsgpu::launch_pcfich(q->d_it, (int)nof_sf, (const float2 *)d_grid, (const float2 *)d_ce,
                               ant_stride, (int)q->cell.nof_prb, (int)q->cell.nof_ports,
                               (int)q->cell.nof_rx_ant, q->d_idx, q->d_seq, d_cfi, d_corr, st)
             ? -1
             : 0;
}

} // extern "C"
