// Subframe batch queue (include/srsgpu/rx_queue.h): PHY-worker threads submit single subframes,
// batches of them run through OFDM -> channel estimation -> [PCFICH -> PDCCH search -> grant] ->
// PDSCH / DL-SCH (the GPU counterpart of srsUE's per-subframe worker pool,
// srsue/src/phy/phy.cc:141-168, phch_worker.cc:548-806, and of srslte_ue_dl_decode_rnti,
// lib/src/phy/ue/ue_dl.c:467-620).
//
// Two batches in flight. Submissions fill one of two staging slots: the submitting worker copies
// its time-domain samples into the slot's pinned buffer itself (the copies of many workers run in
// parallel). A closer thread closes the filling slot (max_batch subframes, the oldest waited
// max_wait_us, or a flush), switches the workers to the other slot as soon as that one is free,
// waits for the closed slot's copies and starts its host-to-device transfer on a copy stream. The
// dispatcher thread runs the closed batches in order on the compute stream, each after its
// transfer's event. So the staging (host copies + DMA) of batch k+1 overlaps the decode of batch k.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <pthread.h>
#include <sched.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <set>
#include <thread>
#include <vector>

#include "srsgpu/chest_batch.h"
#include "srsgpu/dci.h"
#include "srsgpu/dlsch_batch.h"
#include "srsgpu/ofdm_batch.h"
#include "srsgpu/pcfich_batch.h"
#include "srsgpu/pdcch_batch.h"
#include "srsgpu/pdsch_batch.h"
#include "srsgpu/rx_queue.h"
#include "host_ring.h"

namespace {

#define RXQ_CHK(x)                                                                                 \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) {                                                                        \
      fprintf(stderr, "srsgpu rxq: %s failed: %s\n", #x, hipGetErrorString(e_));                   \
      return -1;                                                                                   \
    }                                                                                              \
  } while (0)

// one queued subframe: a grant item or a ue_dl item
struct Pending {
  srsgpu_rxq_item_t *it;
  srsgpu_rxq_ue_dl_t *ue;
  uint64_t ticket;
  std::chrono::steady_clock::time_point t;
  const void *td(int a) const { return it ? it->td[a] : ue->td[a]; }
  uint32_t sf_idx() const { return it ? it->sf.sf_idx : ue->tti % 10; }
};

// PSS / EMPTY noise (chest_dl.c:628-637): only subframes 0 and 5 estimate the noise; every other
// subframe keeps the estimate the object holds, i.e. the latest one of an earlier subframe. One
// thread per (rx antenna, port) column walks the batch in submission order from the value the
// previous batch left (last[c]).
__global__ void k_noise_carry(float *__restrict__ noise, const uint8_t *__restrict__ est, int n, int cols,
                              float *__restrict__ last) {
  const int c = threadIdx.x;
  if (c >= cols) return;
  float v = last[c];
  for (int i = 0; i < n; i++) {
    if (est[i])
      v = noise[i * cols + c];
    else
      noise[i * cols + c] = v;
  }
  last[c] = v;
}

// srslte_chest_dl_get_noise_estimate (chest_dl.c:741-750) of the listed subframes, in the
// reference's float order: per antenna the sum over ports / nports, summed over antennas, / nrx
__global__ void k_sf_noise(const float *__restrict__ noise, const uint32_t *__restrict__ sel, int n, int nrx,
                           int nports, float *__restrict__ out) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const float *v = noise + (size_t)sel[j] * nrx * nports;
  float s = 0.f;
  for (int a = 0; a < nrx; a++) {
    float acc = 0.f;
    for (int p = 0; p < nports; p++) acc += v[a * nports + p];
    s += acc / (float)nports;
  }
  out[j] = nrx ? s / (float)nrx : s;
}

// noise rows (nrx * nports values) of the listed subframes, packed in list order: the PDSCH call of
// a batch where some subframes carry no PDSCH reads its noise by call position
__global__ void k_noise_gather(const float *__restrict__ noise, const uint32_t *__restrict__ sel, int n, int cols,
                               float *__restrict__ out) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n * cols) return;
  out[j] = noise[(size_t)sel[j / cols] * cols + j % cols];
}

// Ingest of one batch's time-domain samples into the slot's device buffer (dst: [item][antenna] rows of
// `row` complex floats). src[r] is a device-visible pointer to row r's samples: host memory the caller
// registered (srsgpu_rxq_register, read over PCIe by the GPU: no host copy, no per-item DMA call) or the
// slot's raw staging buffer. sc16: int16 I/Q pairs scaled by `scale` (the radio's native format, half the
// PCIe bytes), else complex floats. Rows with a null src were staged by the DMA already.
__global__ __launch_bounds__(256) void k_ingest(const void *const *__restrict__ src, int nrows, size_t row,
                                                int sc16, float scale, float2 *__restrict__ dst) {
  const int r = blockIdx.y;
  if (r >= nrows || !src[r]) return;
  float2 *d = dst + (size_t)r * row;
  if (sc16) {
    const uint4 *s4 = (const uint4 *)src[r]; // 4 samples per 16 B
    const size_t n4 = row / 4;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
      const uint4 v = s4[i];
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
      float4 *o = (float4 *)(d + 4 * i);
#pragma unroll
      for (int k = 0; k < 2; k++) {
        const uint32_t a = w[2 * k], b = w[2 * k + 1];
        o[k] = make_float4((float)(int16_t)(a & 0xffff) * scale, (float)(int16_t)(a >> 16) * scale,
                           (float)(int16_t)(b & 0xffff) * scale, (float)(int16_t)(b >> 16) * scale);
      }
    }
  } else {
    const float4 *s4 = (const float4 *)src[r]; // 2 samples per 16 B
    float4 *o = (float4 *)d;
    const size_t n2 = row / 2;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n2; i += (size_t)gridDim.x * 256)
      o[i] = s4[i];
  }
}

// srslte_chest_dl_get_* (chest_dl.c:737-846) of every subframe of a batch, in the reference's float
// order, one thread per subframe: out[i] = {cfo, snr, rsrp, rsrq, rssi, rsrp_neighbour}. meas holds
// the estimator's [subframe][rx][port] {rsrp, rssi, rsrp_corr, cfo} (srsgpu_chest_estimate_meas_dev),
// noise the per-(rx, port) noise after the PSS / EMPTY carry. The reference's q->cfo is the last
// (rx, port) estimate of the latest subframe that estimated it: cfo_src[i] (-1: the carried value in
// last), and q->rsrp_corr is only rewritten with rsrp_neighbour on.
__global__ void k_getters(const float *__restrict__ noise, const float *__restrict__ meas,
                          const int32_t *__restrict__ cfo_src, int rsrp_nb, const float *__restrict__ last, int n,
                          int nrx, int np, int nof_prb, float *__restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int cols = nrx * np;
  const float *m = meas + (size_t)i * cols * 4;
  const float *nb = rsrp_nb ? m : last;
  float nn = 0.f; // srslte_chest_dl_get_noise_estimate
  for (int a = 0; a < nrx; a++) {
    float acc = 0.f;
    for (int p = 0; p < np; p++) acc += noise[(size_t)i * cols + a * np + p];
    nn += acc / (float)np;
  }
  nn /= (float)nrx;
  float rs = 0.f; // srslte_chest_dl_get_snr's sum
  for (int a = 0; a < nrx; a++)
    for (int p = 0; p < np; p++) rs += m[(a * np + p) * 4] / (float)np;
  float rssi = 0.f, rsrq = 0.f, rsrp = -1e9f, nbr = -1e9f;
  for (int a = 0; a < nrx; a++) {
    rssi += 4.f * m[(a * np) * 4 + 1] / (float)nof_prb / 12.f;
    rsrq += (float)nof_prb * m[(a * np) * 4] / m[(a * np) * 4 + 1];
    float v = 0.f, w = 0.f;
    for (int p = 0; p < np; p++) {
      v += m[(a * np + p) * 4];
      w += nb[(a * np + p) * 4 + 2];
    }
    v /= (float)np;
    w /= (float)np;
    if (v > rsrp) rsrp = v;
    if (w > nbr) nbr = w;
  }
  const int lc = (nrx - 1) * np + np - 1;
  float *o = out + (size_t)i * 6;
  o[0] = cfo_src[i] >= 0 ? meas[((size_t)cfo_src[i] * cols + lc) * 4 + 3] : last[lc * 4 + 3];
  o[1] = rs / nn;
  o[2] = rsrp;
  o[3] = rsrq / (float)nrx;
  o[4] = rssi / (float)nrx;
  o[5] = nbr;
}

// the estimator state the next batch starts from: the CFO of the last subframe that estimated it, and
// the neighbour RSRP of the batch's last subframe when it was computed
__global__ void k_meas_last(const float *__restrict__ meas, int cfo_from, int nb_from, int cols, float *__restrict__ last) {
  const int c = threadIdx.x;
  if (c >= cols) return;
  if (cfo_from >= 0) last[c * 4 + 3] = meas[((size_t)cfo_from * cols + c) * 4 + 3];
  if (nb_from >= 0) last[c * 4 + 2] = meas[((size_t)nb_from * cols + c) * 4 + 2];
}

// transport blocks of a PDSCH subframe (srsgpu/pdsch_batch.h)
uint32_t sf_ntb(const srsgpu_pdsch_sf_t &s) {
  return s.mimo_type == SRSGPU_MIMO_CDD || (s.mimo_type == SRSGPU_MIMO_SPATIAL_MULTIPLEX && s.tbs[1] > 0) ? 2 : 1;
}

} // namespace

struct srsgpu_rxq {
  srsgpu_cell_t cell{};
  uint32_t N = 0, max_batch = 0, max_wait_us = 0, max_halfits = 8, nports = 1, nrx = 1;
  uint32_t phich_len = 0, phich_res = 2;
  bool phich_dirty = false; // srsgpu_rxq_set_phich: the dispatcher rebuilds pdcch before its next use
  size_t td_len = 0, gsz = 0, dlen = 0; // complex samples per antenna / grid elements / TB bytes
  hipStream_t st = nullptr, cst = nullptr; // compute / copy streams
  srsgpu_ofdm_t *ofdm = nullptr;
  srsgpu_chest_t *chest = nullptr;
  srsgpu_pdsch_t *pdsch = nullptr;
  srsgpu_pcfich_t *pcfich = nullptr;
  srsgpu_pdcch_t *pdcch = nullptr; // created with the PHICH configuration on the first ue_dl batch
  // device working buffers: one batch's kernels use them after the previous batch's, in stream order
  float *d_grid = nullptr, *d_ce = nullptr, *d_noise = nullptr;
  float *d_noise_last = nullptr; // PSS / EMPTY: the estimate carried between batches
  float *d_meas = nullptr;       // [subframe][rx][port] {rsrp, rssi, rsrp_corr, cfo}
  float *d_meas_last = nullptr;  // [rx][port] x 4: q->cfo / q->rsrp_corr carried between batches
  int32_t *d_cfo_src = nullptr;
  float *d_getters = nullptr;    // [subframe] x 6 (srsgpu_rxq_meas_t)
  srsgpu_feedback_t *d_fb = nullptr; // the ue_dl items' TM3 / TM4 feedback
  std::vector<srsgpu_feedback_sf_t> fb_sf;
  uint8_t *d_est = nullptr;      // per subframe: 1 if it estimates the noise
  uint8_t *d_data = nullptr;     // TB bytes of outputs the device cannot address (then copied back)
  int32_t *d_ret = nullptr;
  uint32_t *d_noi = nullptr;
  // control channel of the ue_dl items (consumed by the dispatcher within the batch)
  uint32_t *d_sel = nullptr;   // their subframe indices in the batch
  float *d_uenoise = nullptr;  // their noise estimates
  uint32_t *d_who = nullptr;   // subframes of the PDSCH call
  float *d_pnoise = nullptr;   // their noise rows
  uint32_t *d_cfi = nullptr, *h_cfi = nullptr;
  float *d_corr = nullptr, *h_corr = nullptr;
  float *d_llr = nullptr;
  size_t llr_stride = 0;
  srsgpu_dci_result_t *d_res = nullptr, *h_res = nullptr;
  srsgpu_dci_result_t *d_res_ul = nullptr, *h_res_ul = nullptr;

  // Batch slots. A slot takes submissions (FILLING), is closed and its samples staged (CLOSED ->
  // STAGED, closer thread), dispatched (RUNNING: the dispatcher enqueues the whole batch on the GPU
  // and moves on to the next slot) and completed (the completer waits for the batch's results and
  // writes them into the items) before it takes submissions again. Three slots: one filling, one on
  // the GPU, one completing; the GPU gets the next batch while the host finishes the last.
  enum { FILLING = 0, CLOSED = 1, STAGED = 2, RUNNING = 3 };
  static constexpr int NSLOT = 4;
  int nslot = 3; // slots in use (SRSGPU_RXQ_SLOTS, 3 or 4)
  struct Slot {
    float *h_td = nullptr, *d_td = nullptr; // pinned staging (raw format) / device samples (cf32)
    float *d_raw = nullptr;                  // SC16: the staged raw samples before conversion
    const void **h_src = nullptr, **d_src = nullptr; // per row: registered host source (device view) or null
    std::vector<const void *> h_host;                // per row: the registered host pointer itself
    std::vector<const char *> h_rgn;                 // per row: the start of its registered region
    void *d_reg = nullptr;                           // registered rows' DMA target (ingest_dma)
    hipEvent_t staged = nullptr;
    std::vector<Pending> items;
    int state = FILLING;
    int copying = 0; // submitters still copying their samples in
    uint32_t nstaged = 0; // items whose samples went through the staging buffer
    int sc16 = 0;          // the input format of this slot's items (set with its first item)
    float sc16_scale = 1.0f / 32768.0f;
    // the batch's pinned host inputs of H2D copies and its results (per slot: the next batch is
    // prepared while this one's copies may still be in flight)
    uint8_t *h_est = nullptr;
    int32_t *h_cfo_src = nullptr;
    uint32_t *h_sel = nullptr, *h_who = nullptr;
    float *h_noise = nullptr, *h_getters = nullptr;
    int32_t *h_ret = nullptr;
    uint32_t *h_noi = nullptr;
    uint8_t *h_data = nullptr;
    srsgpu_feedback_t *h_fb = nullptr;
    hipEvent_t done = nullptr;
    // what the completer needs: the PDSCH subframes (batch index, TB count, TB sizes), each TB's
    // staging offset in h_data (-1: written by the device into the caller's registered buffer), the
    // ue_dl items' states
    int r = 0;
    bool fb_any = false;
    std::vector<uint32_t> who, ntb_of;
    std::vector<uint32_t> tbs_of;   // per TB of the call
    std::vector<int64_t> stage_off; // per TB of the call
    std::vector<int> ue_state;      // per item: ue_dl 1 decoded, 0 no PDSCH call, -1 error
    size_t staged_bytes = 0;
  } slot[NSLOT];
  // input format (srsgpu_rxq_set_input_format) and caller memory the GPU reads directly
  int sc16 = 0; // guarded by m; a change waits until nothing is queued and holds new submissions
  float sc16_scale = 1.0f / 32768.0f;
  bool fmt_busy = false;
  struct Region {
    const char *h;
    size_t bytes;
    const char *d; // device view of the same memory
    bool owned;    // srsgpu_rxq_alloc_host (hipHostMalloc'd here), else the caller's (hipHostRegister'd)
  };
  std::vector<Region> regions; // guarded by m
  uint64_t zero_copy_rows = 0, staged_rows = 0, zero_copy_tbs = 0, staged_tbs = 0, dma_copies = 0;
  // registered rows: true (default) DMA them (one copy per run of address-contiguous rows) and convert
  // on the device; false (SRSGPU_RXQ_INGEST=kernel) the ingest kernel reads them over the bus
  bool ingest_dma = true;
  bool wake_all = false; // SRSGPU_RXQ_WAKE_ALL=1: every submission wakes the closer (diagnosis)
  // The queue's waits on the GPU (a batch's results, the control channel's round trips) block on the
  // completion interrupt instead of spinning a core (hipEventBlockingSync): a PHY host shares its cores
  // with the radio and the stack, and a container's CPU quota counts a spinning waiter in full (the GPU
  // box: 16 CPUs of quota over 256 visible cores). SRSGPU_RXQ_SPIN=1 spins (A/B).
  bool spin_wait = false;
  hipEvent_t ev_ctl = nullptr; // control(): the CFI / DCI results are on the host
  std::vector<std::pair<const char *, uint32_t>> reg; // stage(): registered rows by host address
  static constexpr size_t kMaxGap = 512 * 1024;        // stage(): bytes between rows one span may bridge
  // device view of a registered host pointer holding `bytes`, or null (caller holds m); aligned16: the
  // ingest kernel reads 16 B vectors (else the samples are staged)
  const void *device_view(const void *p, size_t bytes, bool aligned16 = true, const char **rgn = nullptr) const {
    const char *c = (const char *)p;
    for (const Region &r : regions)
      if (c >= r.h && c + bytes <= r.h + r.bytes) {
        const char *d = r.d + (c - r.h);
        if (aligned16 && ((uintptr_t)d & 15)) return nullptr;
        if (rgn) *rgn = r.h;
        return d;
      }
    return nullptr;
  }
  int fill = 0; // the slot submissions go to

  std::mutex m;
  std::condition_variable cv_close, cv_ready, cv_done, cv_slot, cv_comp;
  std::deque<int> ready;      // staged slots, in batch order
  std::deque<int> completing; // dispatched slots, in batch order
  uint64_t next_ticket = 1, done_upto = 0; // tickets are completed in order
  std::set<uint64_t> failed;               // tickets whose batch failed, until waited for
  bool stop = false, flush = false, comp_stop = false;
  uint64_t nbatches = 0, nsf = 0;
  uint32_t nsb = 0; // softbuffers of the caller
  // time per stage, seconds (srsgpu_rxq_timing): 0 front end enqueue (OFDM, chest, getters), 1 control
  // channel (PCFICH / PDCCH round trips), 2 grants and softbuffer resets, 3 PDSCH / DL-SCH enqueue, 4 the
  // completer waiting for a batch's results, 5 result copy-out, 6 staging (closer thread)
  double tm[8] = {};
  std::vector<uint32_t> rs_slot, rs_ncb; // the batch's softbuffer resets, one launch
  std::thread closer, worker, completer;

  int setup(const srsgpu_cell_t *c, uint32_t symbol_sz, uint32_t nsb_in, uint32_t mb, uint32_t wait_us,
            uint32_t maxh) {
    cell = *c;
    N = symbol_sz;
    max_batch = mb;
    max_wait_us = wait_us;
    max_halfits = maxh;
    nsb = nsb_in;
    nports = cell.nof_ports;
    nrx = cell.nof_rx_ant;
    td_len = (size_t)15 * N;
    gsz = (size_t)(cell.cp == 1 ? 12 : 14) * 12 * cell.nof_prb; // grid rows: OFDM symbols per subframe
    dlen = SRSGPU_DLSCH_DATA_LEN(75376) + 16;
    // 72 NOF_CCE(cfi) floats per subframe at most: the largest CCE count of the cell, which the
    // smallest PHICH allocation (normal length, Ng = 1/6) leaves (110 PRB: 96 CCEs)
    uint32_t max_cce = 0;
    for (uint32_t cfi = 1; cfi <= 3; cfi++) {
      uint32_t nc = 0;
      if (srsgpu_pdcch_cell_map(&cell, 0, 0, cfi, nullptr, 0, &nc) < 0) return -1;
      if (nc > max_cce) max_cce = nc;
    }
    llr_stride = 72 * (size_t)max_cce;
    const uint32_t max_cb = 13;
    RXQ_CHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    RXQ_CHK(hipStreamCreateWithFlags(&cst, hipStreamNonBlocking));
    if (srsgpu_ofdm_rx_create(&ofdm, cell.nof_prb, N) || srsgpu_chest_create(&chest, &cell, mb * nrx) ||
        srsgpu_pdsch_create(&pdsch, &cell, nsb_in, max_cb, mb) || srsgpu_pcfich_create(&pcfich, &cell))
      return -1;
    srsgpu_ofdm_rx_set_stream(ofdm, st);
    if (srsgpu_ofdm_set_cp(ofdm, cell.cp)) return -1;
    srsgpu_chest_set_stream(chest, st);
    srsgpu_pdsch_set_stream(pdsch, st);
    if (const char *e = getenv("SRSGPU_RXQ_SLOTS")) nslot = std::min(std::max(atoi(e), 3), NSLOT);
    if (const char *e = getenv("SRSGPU_RXQ_SPIN")) spin_wait = e[0] == '1';
    RXQ_CHK(hipEventCreateWithFlags(&ev_ctl, hipEventDisableTiming | (spin_wait ? 0u : hipEventBlockingSync)));
    for (int k = 0; k < nslot; k++) {
      Slot &s = slot[k];
      RXQ_CHK(hipMalloc(&s.d_td, sizeof(float) * 2 * td_len * mb * nrx));
      RXQ_CHK(hipMalloc(&s.d_raw, sizeof(float) * td_len * mb * nrx)); // SC16 rows: 4 B per sample
      RXQ_CHK(hipHostMalloc(&s.h_td, sizeof(float) * 2 * td_len * mb * nrx));
      RXQ_CHK(hipHostMalloc(&s.h_src, sizeof(void *) * mb * nrx));
      RXQ_CHK(hipMalloc(&s.d_src, sizeof(void *) * mb * nrx));
      s.h_host.assign((size_t)mb * nrx, nullptr);
      s.h_rgn.assign((size_t)mb * nrx, nullptr);
      RXQ_CHK(hipMalloc(&s.d_reg, sizeof(float) * 2 * td_len * mb * nrx));
      RXQ_CHK(hipEventCreateWithFlags(&s.staged, hipEventDisableTiming));
      RXQ_CHK(hipEventCreateWithFlags(&s.done, hipEventDisableTiming | (spin_wait ? 0u : hipEventBlockingSync)));
      RXQ_CHK(hipHostMalloc(&s.h_est, mb));
      RXQ_CHK(hipHostMalloc(&s.h_cfo_src, sizeof(int32_t) * mb));
      RXQ_CHK(hipHostMalloc(&s.h_sel, sizeof(uint32_t) * mb));
      RXQ_CHK(hipHostMalloc(&s.h_who, sizeof(uint32_t) * mb));
      RXQ_CHK(hipHostMalloc(&s.h_noise, sizeof(float) * mb * nrx * nports));
      RXQ_CHK(hipHostMalloc(&s.h_getters, sizeof(float) * 6 * mb));
      RXQ_CHK(hipHostMalloc(&s.h_ret, sizeof(int32_t) * 2 * mb));
      RXQ_CHK(hipHostMalloc(&s.h_noi, sizeof(uint32_t) * 2 * mb));
      RXQ_CHK(hipHostMalloc(&s.h_data, dlen * 2 * mb));
      RXQ_CHK(hipHostMalloc(&s.h_fb, sizeof(srsgpu_feedback_t) * mb));
    }
    RXQ_CHK(hipMalloc(&d_grid, sizeof(float) * 2 * gsz * mb * nrx));
    RXQ_CHK(hipMalloc(&d_ce, sizeof(float) * 2 * gsz * mb * nrx * nports));
    RXQ_CHK(hipMalloc(&d_noise, sizeof(float) * mb * nrx * nports));
    RXQ_CHK(hipMalloc(&d_data, dlen * 2 * mb));
    RXQ_CHK(hipMalloc(&d_ret, sizeof(int32_t) * 2 * mb));
    RXQ_CHK(hipMalloc(&d_noi, sizeof(uint32_t) * 2 * mb));
    RXQ_CHK(hipMalloc(&d_noise_last, sizeof(float) * nrx * nports));
    RXQ_CHK(hipMemset(d_noise_last, 0, sizeof(float) * nrx * nports)); // srslte_chest_dl_init: 0
    RXQ_CHK(hipMalloc(&d_meas, sizeof(float) * 4 * mb * nrx * nports));
    RXQ_CHK(hipMalloc(&d_meas_last, sizeof(float) * 4 * nrx * nports));
    RXQ_CHK(hipMemset(d_meas_last, 0, sizeof(float) * 4 * nrx * nports)); // bzero'd estimator
    RXQ_CHK(hipMalloc(&d_cfo_src, sizeof(int32_t) * mb));
    RXQ_CHK(hipMalloc(&d_getters, sizeof(float) * 6 * mb));
    RXQ_CHK(hipMalloc(&d_fb, sizeof(srsgpu_feedback_t) * mb));
    RXQ_CHK(hipMalloc(&d_est, mb));
    RXQ_CHK(hipMalloc(&d_sel, sizeof(uint32_t) * mb));
    RXQ_CHK(hipMalloc(&d_uenoise, sizeof(float) * mb));
    RXQ_CHK(hipMalloc(&d_who, sizeof(uint32_t) * mb));
    RXQ_CHK(hipMalloc(&d_pnoise, sizeof(float) * mb * nrx * nports));
    RXQ_CHK(hipMalloc(&d_cfi, sizeof(uint32_t) * mb));
    RXQ_CHK(hipHostMalloc(&h_cfi, sizeof(uint32_t) * mb));
    RXQ_CHK(hipMalloc(&d_corr, sizeof(float) * mb));
    RXQ_CHK(hipHostMalloc(&h_corr, sizeof(float) * mb));
    RXQ_CHK(hipMalloc(&d_llr, sizeof(float) * llr_stride * mb));
    RXQ_CHK(hipMalloc(&d_res, sizeof(srsgpu_dci_result_t) * mb));
    RXQ_CHK(hipHostMalloc(&h_res, sizeof(srsgpu_dci_result_t) * mb));
    RXQ_CHK(hipMalloc(&d_res_ul, sizeof(srsgpu_dci_result_t) * mb));
    RXQ_CHK(hipHostMalloc(&h_res_ul, sizeof(srsgpu_dci_result_t) * mb));
    srsgpu_pcfich_set_noise_dev(pcfich, d_uenoise);
    if (const char *e = getenv("SRSGPU_RXQ_INGEST")) ingest_dma = strcmp(e, "kernel") != 0;
    if (const char *e = getenv("SRSGPU_RXQ_WAKE_ALL")) wake_all = e[0] == '1';
    closer = std::thread([this] { close_loop(); });
    worker = std::thread([this] { run_loop(); });
    completer = std::thread([this] { comp_loop(); });
    return 0;
  }

  void teardown() {
    {
      std::lock_guard<std::mutex> l(m);
      stop = true;
    }
    cv_close.notify_all();
    cv_ready.notify_all();
    cv_slot.notify_all();
    if (closer.joinable()) closer.join();
    if (worker.joinable()) worker.join();
    {
      std::lock_guard<std::mutex> l(m);
      comp_stop = true; // the dispatcher is gone: the completer finishes what it was handed, then leaves
    }
    cv_comp.notify_all();
    if (completer.joinable()) completer.join();
    // a fault of the queue's last work shows here rather than in the caller's next HIP call
    for (hipStream_t x : {st, cst})
      if (x) {
        const hipError_t e = hipStreamSynchronize(x);
        if (e != hipSuccess) fprintf(stderr, "srsgpu rxq: teardown sync: %s\n", hipGetErrorString(e));
      }
    if (ofdm) srsgpu_ofdm_rx_destroy(ofdm);
    if (chest) srsgpu_chest_destroy(chest);
    if (pdsch) srsgpu_pdsch_destroy(pdsch);
    if (pcfich) srsgpu_pcfich_destroy(pcfich);
    if (pdcch) srsgpu_pdcch_destroy(pdcch);
    for (Slot &s : slot) {
      for (void *p : {(void *)s.d_td, (void *)s.d_raw, (void *)s.d_src, (void *)s.d_reg})
        if (p) (void)hipFree(p);
      for (void *p : {(void *)s.h_td, (void *)s.h_src, (void *)s.h_est, (void *)s.h_cfo_src, (void *)s.h_sel,
                      (void *)s.h_who, (void *)s.h_noise, (void *)s.h_getters, (void *)s.h_ret, (void *)s.h_noi,
                      (void *)s.h_data, (void *)s.h_fb})
        if (p) (void)hipHostFree(p);
      if (s.staged) (void)hipEventDestroy(s.staged);
      if (s.done) (void)hipEventDestroy(s.done);
    }
    for (const Region &r : regions) (void)(r.owned ? hipHostFree((void *)r.h) : hipHostUnregister((void *)r.h));
    regions.clear();
    for (void *p : {(void *)d_grid, (void *)d_ce, (void *)d_noise, (void *)d_data, (void *)d_ret,
                    (void *)d_noi, (void *)d_noise_last, (void *)d_est, (void *)d_sel, (void *)d_uenoise,
                    (void *)d_cfi, (void *)d_corr, (void *)d_llr, (void *)d_res, (void *)d_who,
                    (void *)d_pnoise, (void *)d_res_ul, (void *)d_meas, (void *)d_meas_last, (void *)d_cfo_src,
                    (void *)d_getters, (void *)d_fb})
      if (p) (void)hipFree(p);
    for (void *p : {(void *)h_cfi, (void *)h_corr, (void *)h_res, (void *)h_res_ul})
      if (p) (void)hipHostFree(p);
    if (ev_ctl) (void)hipEventDestroy(ev_ctl);
    if (st) (void)hipStreamDestroy(st);
    if (cst) (void)hipStreamDestroy(cst);
  }

  // ---------------------------------------------------------------- submission ----
  int submit(srsgpu_rxq_item_t *it, srsgpu_rxq_ue_dl_t *ue, uint64_t *ticket) {
    const void *td[2] = {it ? it->td[0] : ue->td[0], it ? it->td[1] : ue->td[1]};
    if (!td[0] || (nrx > 1 && !td[1])) return -1;
    size_t row_bytes;
    int s, idx;
    const void *dv[2] = {nullptr, nullptr};
    bool need_copy = false, wake = false;
    {
      std::unique_lock<std::mutex> l(m);
      // the filling slot has room (else wait for the closer to switch to the other slot), and no
      // input format change is under way
      cv_slot.wait(l, [&] {
        return stop || (!fmt_busy && slot[fill].state == FILLING && slot[fill].items.size() < max_batch);
      });
      if (stop) return -1;
      s = fill;
      idx = (int)slot[s].items.size();
      if (idx == 0) { // the slot's format: every item of it is submitted under the same one
        slot[s].sc16 = sc16;
        slot[s].sc16_scale = sc16_scale;
      }
      row_bytes = (slot[s].sc16 ? 4 : 8) * td_len;
      *ticket = next_ticket++;
      slot[s].items.push_back({it, ue, *ticket, std::chrono::steady_clock::now()});
      for (uint32_t a = 0; a < nrx; a++) {
        const char *rgn = nullptr;
        dv[a] = device_view(td[a], row_bytes, true, &rgn);
        slot[s].h_src[(size_t)idx * nrx + a] = dv[a]; // null: staged by the host copy below
        slot[s].h_host[(size_t)idx * nrx + a] = dv[a] ? td[a] : nullptr;
        slot[s].h_rgn[(size_t)idx * nrx + a] = rgn; // the region stays registered while the row is queued
        need_copy = need_copy || !dv[a];
      }
      if (need_copy) slot[s].copying++;
      // the closer waits for a first item, then for a full slot (or its deadline): only those wake it
      // (a wake per submission had the closer contend for the lock with every worker)
      wake = wake_all || idx == 0 || slot[s].items.size() >= max_batch;
    }
    if (wake) cv_close.notify_one();
    if (!need_copy) return 0;
    // the worker stages its own unregistered samples (outside the lock: many workers copy at once)
    for (uint32_t a = 0; a < nrx; a++)
      if (!dv[a]) memcpy((char *)slot[s].h_td + ((size_t)idx * nrx + a) * row_bytes, td[a], row_bytes);
    {
      std::lock_guard<std::mutex> l(m);
      // the closer, having closed the slot, waits for the last copy to finish
      wake = --slot[s].copying == 0 && (wake_all || slot[s].state == CLOSED);
    }
    if (wake) cv_close.notify_one();
    return 0;
  }

  // the closed slot's samples to the device: one DMA of the staged rows' region (up to the last staged
  // row); registered rows either by DMA straight from the caller's memory into d_reg, one copy per run
  // of rows contiguous there (ingest_dma), or read over the bus by the ingest kernel; the ingest kernel
  // then converts SC16 rows and moves registered rows into place. The staged DMA may cover registered
  // rows' places with stale staging bytes: the ingest kernel writes them after it on the same stream.
  bool stage(Slot &sl, size_t n) {
    const int sc16 = sl.sc16;
    const size_t rows = n * nrx, row_bytes = (sc16 ? 4 : 8) * td_len;
    size_t last = 0, nst = 0;
    for (size_t r = 0; r < rows; r++)
      if (!sl.h_src[r]) {
        last = r + 1;
        nst++;
      }
    sl.nstaged = (uint32_t)nst;
    char *dst_raw = sc16 ? (char *)sl.d_raw : (char *)sl.d_td;
    if (last && hipMemcpyAsync(dst_raw, sl.h_td, last * row_bytes, hipMemcpyHostToDevice, cst) != hipSuccess)
      return false;
    if (ingest_dma) {
      // registered rows in host address order, one DMA per span of the caller's memory into d_reg: rows
      // that touch or overlap share a span (a row handed over twice is copied once), and so do rows a
      // short gap apart in one registered region: the gap's bytes cost less than a copy's own overhead
      // (~12 us per hipMemcpyAsync on the copy engine, r05_s37), as long as d_reg has room for them.
      // The ingest kernel then reads every row from its place in d_reg.
      reg.clear();
      for (size_t r = 0; r < rows; r++)
        if (sl.h_src[r]) reg.push_back({(const char *)sl.h_host[r], (uint32_t)r});
      std::sort(reg.begin(), reg.end());
      const size_t cap = sizeof(float) * 2 * td_len * max_batch * nrx; // d_reg's bytes
      const char *sp0 = nullptr, *sp1 = nullptr, *rg = nullptr;           // the open span, its region
      size_t dpos = 0, d0 = 0; // bytes of d_reg used; the open span's place there
      auto flush_span = [&]() {
        if (!sp0) return true;
        dma_copies++;
        const bool ok = hipMemcpyAsync((char *)sl.d_reg + d0, sp0, (size_t)(sp1 - sp0), hipMemcpyHostToDevice,
                                       cst) == hipSuccess;
        dpos = d0 + (size_t)(sp1 - sp0);
        sp0 = nullptr;
        return ok;
      };
      for (size_t i = 0; i < reg.size(); i++) {
        const char *h = reg[i].first, *rgn = sl.h_rgn[reg[i].second];
        const size_t later = (reg.size() - 1 - i) * row_bytes; // what the rows after this one may need
        const bool joins = sp0 && rgn == rg && h <= sp1 + kMaxGap &&
                           d0 + (size_t)(std::max(sp1, h + row_bytes) - sp0) + later <= cap;
        if (!joins) {
          if (!flush_span()) return false;
          sp0 = h;
          sp1 = h;
          rg = rgn;
          d0 = dpos;
        }
        sp1 = std::max(sp1, h + row_bytes);
        sl.h_src[reg[i].second] = (const char *)sl.d_reg + d0 + (size_t)(h - sp0);
      }
      if (!flush_span()) return false;
    }
    const bool kernel = sc16 || nst < rows;
    if (kernel) {
      // staged rows: SC16 converts from the raw copy, cf32 is in place
      for (size_t r = 0; r < rows; r++)
        if (!sl.h_src[r]) sl.h_src[r] = sc16 ? (const void *)(dst_raw + r * row_bytes) : nullptr;
      if (xfer(sl.d_src, sl.h_src, sizeof(void *) * rows, hipMemcpyHostToDevice, cst) != hipSuccess)
        return false;
      const unsigned gx = (unsigned)std::min<size_t>(64, (td_len / 2 + 255) / 256);
      hipLaunchKernelGGL(k_ingest, dim3(gx, (unsigned)rows), dim3(256), 0, cst, (const void *const *)sl.d_src,
                         (int)rows, td_len, sc16, sl.sc16_scale, (float2 *)sl.d_td);
      if (hipGetLastError() != hipSuccess) return false;
    }
    zero_copy_rows += rows - nst;
    staged_rows += nst;
    return hipEventRecord(sl.staged, cst) == hipSuccess;
  }

  // closer thread: close the filling slot, switch the workers to the next one once it is free, wait
  // for the closed slot's copies, start its transfer and hand it to the dispatcher
  void close_loop() {
    std::unique_lock<std::mutex> l(m);
    for (;;) {
      cv_close.wait(l, [this] { return stop || !slot[fill].items.empty(); });
      if (stop) return;
      const int s = fill;
      const auto deadline = slot[s].items.front().t + std::chrono::microseconds(max_wait_us);
      cv_close.wait_until(l, deadline, [&] { return stop || flush || slot[s].items.size() >= max_batch; });
      if (stop) return;
      flush = false;
      slot[s].state = CLOSED;
      // the closed slot's transfer starts at once (its buffers are its own), overlapping the batches
      // ahead of it; only then does the closer wait for the next slot to be free for submissions
      // (waiting first held every transfer back until the batch two ahead had completed)
      cv_close.wait(l, [&] { return stop || slot[s].copying == 0; });
      if (stop) return;
      const size_t n = slot[s].items.size();
      l.unlock();
      const double ts = now_s(), cs = trace ? cpu_s() : 0.0;
      const uint64_t dc0 = dma_copies;
      const bool ok = stage(slot[s], n);
      const double te = now_s();
      if (trace)
        fprintf(stderr, "rxq trace: n %zu stage wall %.3f ms cpu %.3f ms, %llu copies\n", n, (te - ts) * 1e3,
                (cpu_s() - cs) * 1e3, (unsigned long long)(dma_copies - dc0));
      l.lock();
      tm[6] += te - ts;
      if (!ok) fprintf(stderr, "srsgpu rxq: staging copy failed: %s\n", hipGetErrorString(hipGetLastError()));
      slot[s].state = STAGED;
      ready.push_back(ok ? s : -1 - s);
      cv_ready.notify_one();
      // the next slot takes submissions once its batch has been completed
      const int nx = (s + 1) % nslot;
      cv_slot.wait(l, [&] { return stop || slot[nx].state == FILLING; });
      if (stop) return;
      fill = nx;
      cv_slot.notify_all();
    }
  }

  // dispatcher thread: enqueue the staged batches in order, each on the GPU as a whole, and hand them
  // to the completer
  void run_loop() {
    std::unique_lock<std::mutex> l(m);
    for (;;) {
      cv_ready.wait(l, [this] { return stop || !ready.empty(); });
      if (ready.empty() && stop) return;
      const int tag = ready.front();
      ready.pop_front();
      const int s = tag < 0 ? -1 - tag : tag;
      Slot &sl = slot[s];
      sl.state = RUNNING;
      std::vector<Pending> b = sl.items;
      l.unlock();
      int r = tag < 0 ? -1 : 0;
      if (!r) r = hipStreamWaitEvent(st, sl.staged, 0) == hipSuccess ? 0 : -1;
      if (!r) r = enqueue(sl, b, sl.d_td);
      if (!r) r = hipEventRecord(sl.done, st) == hipSuccess ? 0 : -1;
      // a failed batch may have left work in flight that reads its buffers: drain before reuse
      if (r && tag >= 0) fprintf(stderr, "srsgpu rxq: dispatch failed: %s\n", hipGetErrorString(hipGetLastError()));
      if (r) {
        (void)hipStreamSynchronize(st);
        (void)hipStreamSynchronize(cst);
      }
      sl.r = r;
      l.lock();
      for (int k = 0; k < 4; k++) tm[k] += run_tm[k];
      completing.push_back(s);
      cv_comp.notify_one();
    }
  }

  // completer thread: wait for each dispatched batch's results, write them into its items, free the slot
  void comp_loop() {
    std::unique_lock<std::mutex> l(m);
    for (;;) {
      cv_comp.wait(l, [this] { return comp_stop || !completing.empty(); });
      if (completing.empty()) return;
      const int s = completing.front();
      completing.pop_front();
      Slot &sl = slot[s];
      l.unlock();
      double w = 0, c = 0;
      if (!sl.r) {
        const double t0 = now_s();
        const hipError_t e = hipEventSynchronize(sl.done);
        if (e != hipSuccess) {
          sl.r = -1;
          fprintf(stderr, "srsgpu rxq: batch wait: %s\n", hipGetErrorString(e));
        }
        const double t1 = now_s();
        if (!sl.r) complete(sl);
        w = t1 - t0;
        c = now_s() - t1;
      }
      l.lock();
      tm[4] += w;
      tm[5] += c;
      if (sl.r) {
        fprintf(stderr, "srsgpu rxq: batch of %zu subframes failed\n", sl.items.size());
        for (const Pending &p : sl.items) failed.insert(p.ticket);
      }
      done_upto = sl.items.back().ticket;
      nbatches++;
      nsf += sl.items.size();
      sl.items.clear();
      sl.state = FILLING;
      cv_done.notify_all();
      cv_slot.notify_all();
    }
  }

  // ---------------------------------------------------------------- one batch ----
  // the control channel of the batch's ue_dl items (ue_dl.c:408-433, :484-497): PCFICH on their
  // grids with the estimator's noise, CFI back to the host, PDCCH LLRs and the DL DCI search,
  // results back to the host
  int control(Slot &sl, const std::vector<Pending> &b, const std::vector<uint32_t> &ue) {
    const uint32_t nu = (uint32_t)ue.size();
    for (uint32_t j = 0; j < nu; j++) sl.h_sel[j] = ue[j];
    RXQ_CHK(xfer(d_sel, sl.h_sel, sizeof(uint32_t) * nu, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_sf_noise, dim3((nu + 63) / 64), dim3(64), 0, st, d_noise, d_sel, (int)nu, (int)nrx,
                       (int)nports, d_uenoise);
    RXQ_CHK(hipGetLastError());
    std::vector<srsgpu_pcfich_sf_t> pc(nu);
    for (uint32_t j = 0; j < nu; j++)
      pc[j] = {(uint64_t)ue[j] * nrx * gsz, (uint64_t)ue[j] * nrx * nports * gsz, b[ue[j]].sf_idx(), 0.f};
    if (srsgpu_pcfich_decode_dev(pcfich, pc.data(), nu, d_grid, d_ce, gsz, d_cfi, d_corr, st)) return -1;
    RXQ_CHK(xfer(h_cfi, d_cfi, sizeof(uint32_t) * nu, hipMemcpyDeviceToHost, st));
    RXQ_CHK(xfer(h_corr, d_corr, sizeof(float) * nu, hipMemcpyDeviceToHost, st));
    RXQ_CHK(hipEventRecord(ev_ctl, st));
    RXQ_CHK(hipEventSynchronize(ev_ctl));
    uint32_t plen, pres;
    bool rebuild;
    {
      std::lock_guard<std::mutex> l(m);
      plen = phich_len;
      pres = phich_res;
      rebuild = phich_dirty;
      phich_dirty = false;
    }
    if (pdcch && rebuild) { // only this thread uses pdcch, and its previous batch has finished
      srsgpu_pdcch_destroy(pdcch);
      pdcch = nullptr;
    }
    if (!pdcch) {
      if (srsgpu_pdcch_create(&pdcch, &cell, plen, pres)) return -1;
      srsgpu_pdcch_set_noise_dev(pdcch, d_uenoise);
    }
    std::vector<srsgpu_pdcch_sf_t> ps(nu);
    std::vector<srsgpu_dci_search_t> se(nu);
    for (uint32_t j = 0; j < nu; j++) {
      const srsgpu_rxq_ue_dl_t *u = b[ue[j]].ue;
      ps[j] = {(uint64_t)ue[j] * nrx * gsz, (uint64_t)ue[j] * nrx * nports * gsz, (uint64_t)j * llr_stride,
               u->tti % 10, h_cfi[j], 0.f, 0};
      se[j] = {(uint64_t)j * llr_stride, u->tti % 10, h_cfi[j], u->rnti, u->tm, u->rnti_type, u->ul_rnti};
    }
    if (srsgpu_pdcch_extract_llr_dev(pdcch, ps.data(), nu, d_grid, d_ce, gsz, d_llr, st) ||
        srsgpu_pdcch_find_dci_dev(pdcch, se.data(), nu, d_llr, d_res, d_res_ul, st))
      return -1;
    RXQ_CHK(xfer(h_res, d_res, sizeof(srsgpu_dci_result_t) * nu, hipMemcpyDeviceToHost, st));
    RXQ_CHK(xfer(h_res_ul, d_res_ul, sizeof(srsgpu_dci_result_t) * nu, hipMemcpyDeviceToHost, st));
    RXQ_CHK(hipEventRecord(ev_ctl, st));
    RXQ_CHK(hipEventSynchronize(ev_ctl));
    // the workers' TM3 / TM4 feedback on the same estimates (phch_worker.cc:522-540); its results come
    // back with the batch's other results
    bool any = false;
    fb_sf.resize(nu);
    for (uint32_t j = 0; j < nu; j++) {
      fb_sf[j] = {(uint64_t)ue[j] * nrx * nports * gsz, 0.f, b[ue[j]].ue->feedback};
      any = any || b[ue[j]].ue->feedback;
    }
    if (any && srsgpu_pdsch_feedback_dev(pdsch, fb_sf.data(), nu, d_ce, gsz, d_uenoise, d_fb)) return -1;
    sl.fb_any = any;
    return 0;
  }

  // the grant of a found DCI as srslte_ue_dl_decode_rnti configures it (ue_dl.c:498-574): unpack,
  // redundancy versions, softbuffer resets, MIMO type of the format, srslte_pdsch_cfg_mimo's
  // lstart / RE count. Returns 1 with sf filled (decode it), 0 (no PDSCH call), -1 (error).
  int grant_of(srsgpu_rxq_ue_dl_t *u, const srsgpu_dci_result_t &res, uint32_t cfi, srsgpu_dlsch_t *dl,
               srsgpu_pdsch_sf_t &sf) {
    srsgpu_ra_dl_dci_t dci;
    memset(&dci, 0, sizeof(dci));
    memset(&u->grant, 0, sizeof(u->grant));
    if (srsgpu_dci_msg_to_dl_grant(res.data, res.nof_bits, res.format, u->rnti, cell.nof_prb, cell.nof_ports, &dci,
                                   &u->grant))
      return -1;
    const srsgpu_ra_dl_grant_t &g = u->grant;
    const uint32_t ntb = (g.tb_en[0] ? 1 : 0) + (g.tb_en[1] ? 1 : 0);
    uint32_t rv[2] = {1, 0}; // int rvidx[SRSLTE_MAX_CODEWORDS] = {1}
    for (int i = 0; i < 2; i++) {
      if (!g.tb_en[i]) continue;
      if (dci.rv_idx < 0) { // 36.321 5.3.1 SI redundancy version (ue_dl.c:503-509)
        const uint32_t k = (u->tti / 10 / 2) % 4;
        rv[i] = ((uint32_t)ceilf(1.5f * (float)k)) % 4;
      } else {
        rv[i] = (uint32_t)(i == 0 ? dci.rv_idx : dci.rv_idx_1);
      }
      if (u->softbuffer[i] >= nsb) return -1; // srsgpu_dlsch_softbuffer_reset_tbs's check
      rs_slot.push_back(u->softbuffer[i]); // reset_tbs: (tbs + 24) / 6120 + 1 blocks (softbuffer.c:113-116)
      rs_ncb.push_back(((uint32_t)g.tbs[i] + 24) / 6120 + 1);
    }
    u->rv[0] = rv[0];
    u->rv[1] = rv[1];
    uint32_t mimo;
    switch (res.format) {
    case SRSGPU_DCI_FORMAT1:
    case SRSGPU_DCI_FORMAT1A:
    case SRSGPU_DCI_FORMAT1C:
      mimo = cell.nof_ports == 1 ? SRSGPU_MIMO_SINGLE_ANTENNA : SRSGPU_MIMO_TX_DIVERSITY;
      break;
    case SRSGPU_DCI_FORMAT2A:
      mimo = (ntb == 1 && dci.pinfo == 0) ? SRSGPU_MIMO_TX_DIVERSITY : SRSGPU_MIMO_CDD;
      break;
    case SRSGPU_DCI_FORMAT2: // spatial multiplexing unless one TB with pinfo 0
      mimo = (ntb == 1 && dci.pinfo == 0) ? SRSGPU_MIMO_TX_DIVERSITY : SRSGPU_MIMO_SPATIAL_MULTIPLEX;
      break;
    default: // formats the reference does not decode (ue_dl.c:560-566)
      return -1;
    }
    u->mimo_type = mimo;
    // q->pdsch_cfg.grant.mcs[0].mod > 0 && tbs >= 0 (ue_dl.c:581)
    if (!(g.mod[0] > 0 && g.tbs[0] >= 0)) return 0;
    if (!g.tb_en[0] || ((mimo == SRSGPU_MIMO_CDD || (mimo == SRSGPU_MIMO_SPATIAL_MULTIPLEX && ntb == 2)) &&
                        !g.tb_en[1])) {
      fprintf(stderr, "srsgpu rxq: grant without transport block 0 / CDD with one TB is not on the GPU path\n");
      return -1;
    }
    memset(&sf, 0, sizeof(sf));
    sf.sf_idx = u->tti % 10;
    sf.lstart = cell.nof_prb < 10 ? cfi + 1 : cfi; // srslte_ra_dl_grant_to_nbits (ra.c:570)
    memcpy(sf.prb_idx, g.prb_idx, sizeof(sf.prb_idx));
    sf.rnti = u->rnti;
    sf.scaling = 1.0f;
    sf.mimo_type = mimo;
    sf.tb_cw_swap = g.tb_cw_swap;
    if (mimo == SRSGPU_MIMO_SPATIAL_MULTIPLEX) {
      // srslte_ue_dl_cfg_grant's pinfo -> pmi (ue_dl.c:438-456, 36.212 Table 5.3.3.1.5-4) and
      // srslte_pdsch_cfg_mimo's codebook (pdsch.c:586-596): pmi with one TB, pmi + 1 with two
      const uint32_t pmi = ntb == 1 ? (g.pinfo > 0 && g.pinfo < 5 ? g.pinfo - 1 : g.pinfo % 4) : g.pinfo % 2;
      sf.codebook_idx = ntb == 1 ? pmi : pmi + 1;
    }
    for (int i = 0; i < 2; i++) {
      sf.mod[i] = g.mod[i];
      sf.tbs[i] = g.tb_en[i] ? (uint32_t)g.tbs[i] : 0;
      sf.rv[i] = rv[i];
      // a TB the caller already acked is skipped by srslte_pdsch_decode (pdsch.c:946-947): no decode,
      // the caller's softbuffer and data stay as they are
      sf.softbuffer[i] = u->softbuffer[i];
      if (u->acks[i]) sf.skip_tb |= 1u << i;
    }
    const int nre = srsgpu_pdsch_nof_re(&cell, &sf);
    if (nre <= 0) return -1;
    sf.nof_re = (uint32_t)nre;
    return 1;
  }

  static double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
  }
  static double cpu_s() { // this thread's CPU time (SRSGPU_RXQ_TRACE: busy or waiting)
    timespec ts;
    clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
  }
  const bool trace = getenv("SRSGPU_RXQ_TRACE") != nullptr;
  // The batch's small copies between device buffers and the slot's pinned host buffers: hipMemcpyAsync
  // (DMA), or with SRSGPU_RXQ_COPY=kernel copy kernels through the pinned buffer's device view
  // (launch_h2d), as the engines' host rings do. A/B r06_s7: the kernel copies lost 25-30 % of the
  // saturated rate at batch 256 (99-105 K against 129-147 K subframes/s; a batch makes 10-15 of them,
  // each a launch on the dispatcher thread) and 1-4 % at batch 1024, so DMA stays the default here.
  const bool kcopy = [] {
    const char *e = getenv("SRSGPU_RXQ_COPY");
    return e && strcmp(e, "kernel") == 0;
  }();
  hipError_t xfer(void *dst, const void *src, size_t n, hipMemcpyKind k, hipStream_t s) {
    if (!n) return hipSuccess;
    if (kcopy) {
      void *v = nullptr;
      void *host = k == hipMemcpyHostToDevice ? const_cast<void *>(src) : dst;
      if (hipHostGetDevicePointer(&v, host, 0) == hipSuccess && v)
        return k == hipMemcpyHostToDevice ? srsgpu::launch_h2d(dst, v, n, s) : srsgpu::launch_h2d(v, src, n, s);
    }
    return hipMemcpyAsync(dst, src, n, k, s);
  }
  double run_tm[8] = {}; // the dispatcher's stage times of its last batch, added to tm under the lock

  // one batch, enqueued as a whole: OFDM of the staged samples, channel estimation and measurements,
  // the ue_dl items' control channel (its host round trips) and grants, the softbuffer resets, the
  // PDSCH / DL-SCH of every subframe with a grant (TB bytes straight into registered caller buffers,
  // the others into d_data), and the copies of the results into the slot's pinned buffers
  int enqueue(Slot &sl, std::vector<Pending> &b, const float *d_td) {
    const uint32_t n = (uint32_t)b.size();
    for (double &v : run_tm) v = 0;
    double t0 = now_s(), t1;
    auto lap = [&](int k) {
      t1 = now_s();
      run_tm[k] += t1 - t0;
      t0 = t1;
    };
    rs_slot.clear();
    rs_ncb.clear();
    if (srsgpu_ofdm_rx_sf_dev(ofdm, n * nrx, d_td, td_len, d_grid, gsz)) return -1;
    std::vector<uint32_t> sfi(n * nrx);
    for (uint32_t i = 0; i < n; i++)
      for (uint32_t a = 0; a < nrx; a++) sfi[i * nrx + a] = b[i].sf_idx();
    srsgpu_chest_cfg_t ccfg;
    if (srsgpu_chest_get_cfg(chest, &ccfg)) return -1;
    if (ccfg.noise_alg != 0 && ccfg.smooth_filter_auto) {
      // each subframe's filter would come from the previous subframe's noise: no batch order
      fprintf(stderr, "srsgpu rxq: smooth_filter_auto with PSS / EMPTY noise is not batched\n");
      return -1;
    }
    if (srsgpu_chest_estimate_meas_dev(chest, sfi.data(), n * nrx, d_grid, gsz, d_ce, d_noise, d_meas)) return -1;
    if (ccfg.noise_alg != 0) { // PSS / EMPTY: carry the estimate across subframes in order
      for (uint32_t i = 0; i < n; i++) sl.h_est[i] = (uint8_t)(b[i].sf_idx() == 0 || b[i].sf_idx() == 5);
      RXQ_CHK(xfer(d_est, sl.h_est, n, hipMemcpyHostToDevice, st));
      // grids of one subframe's rx antennas are consecutive: n rows of nrx * nports columns
      hipLaunchKernelGGL(k_noise_carry, dim3(1), dim3(64), 0, st, d_noise, d_est, (int)n, (int)(nrx * nports),
                         d_noise_last);
      RXQ_CHK(hipGetLastError());
    }
    { // the estimator getters of every subframe (srsgpu_rxq_meas_t)
      int32_t src = -1;
      for (uint32_t i = 0; i < n; i++) {
        if (ccfg.cfo_estimate_enable && ((ccfg.cfo_estimate_sf_mask >> b[i].sf_idx()) & 1u)) src = (int32_t)i;
        sl.h_cfo_src[i] = src;
      }
      const int cols = (int)(nrx * nports);
      RXQ_CHK(xfer(d_cfo_src, sl.h_cfo_src, sizeof(int32_t) * n, hipMemcpyHostToDevice, st));
      hipLaunchKernelGGL(k_getters, dim3((n + 63) / 64), dim3(64), 0, st, d_noise, d_meas, d_cfo_src,
                         (int)ccfg.rsrp_neighbour, d_meas_last, (int)n, (int)nrx, (int)nports, (int)cell.nof_prb,
                         d_getters);
      RXQ_CHK(hipGetLastError());
      hipLaunchKernelGGL(k_meas_last, dim3(1), dim3(64), 0, st, d_meas, src, ccfg.rsrp_neighbour ? (int)n - 1 : -1,
                         cols, d_meas_last);
      RXQ_CHK(hipGetLastError());
      RXQ_CHK(xfer(sl.h_getters, d_getters, sizeof(float) * 6 * n, hipMemcpyDeviceToHost, st));
    }
    srsgpu_dlsch_t *dl = srsgpu_pdsch_get_dlsch(pdsch);
    std::vector<uint32_t> ue;
    for (uint32_t i = 0; i < n; i++)
      if (b[i].ue) ue.push_back(i);
    sl.fb_any = false;
    lap(0);
    if (!ue.empty() && control(sl, b, ue)) return -1;
    lap(1);
    if (sl.fb_any)
      RXQ_CHK(xfer(sl.h_fb, d_fb, sizeof(srsgpu_feedback_t) * ue.size(), hipMemcpyDeviceToHost, st));
    // grants: the grant items' own, the ue_dl items' from their DCI
    std::vector<srsgpu_pdsch_sf_t> sfs;
    sl.who.clear();
    sl.ue_state.assign(n, 1);
    for (uint32_t i = 0, j = 0; i < n; i++) {
      srsgpu_pdsch_sf_t s;
      if (b[i].ue) {
        srsgpu_rxq_ue_dl_t *u = b[i].ue;
        const srsgpu_dci_result_t &res = h_res[j];
        u->cfi = h_cfi[j];
        u->cfi_corr = h_corr[j];
        u->found = res.found;
        u->format = res.format;
        u->L = res.L;
        u->ncce = res.ncce;
        u->dci_nof_bits = res.found == 1 ? res.nof_bits : 0;
        memset(u->dci_data, 0, sizeof(u->dci_data));
        if (res.found == 1) memcpy(u->dci_data, res.data, std::min(sizeof(u->dci_data), sizeof(res.data)));
        // srslte_ue_dl_find_ul_dci + srslte_dci_msg_to_ul_grant (phch_worker.cc:938-967)
        const srsgpu_dci_result_t &ur = h_res_ul[j];
        u->ul_found = u->ul_rnti ? ur.found : 0;
        u->ul_L = ur.L;
        u->ul_ncce = ur.ncce;
        u->ul_nof_bits = ur.nof_bits;
        memcpy(u->ul_data, ur.data, sizeof(u->ul_data));
        memset(&u->ul_dci, 0, sizeof(u->ul_dci));
        memset(&u->ul_grant, 0, sizeof(u->ul_grant));
        u->ul_grant_ret = u->ul_found == 1 ? srsgpu_dci_msg_to_ul_grant(ur.data, ur.nof_bits, cell.nof_prb, u->n_rb_ho,
                                                                         &u->ul_dci, &u->ul_grant)
                                           : -1;
        u->acked_in[0] = u->acks[0];
        u->acked_in[1] = u->acks[1];
        for (int t = 0; t < 2; t++)
          if (!u->acks[t]) u->noi[t] = 0; // an acked TB keeps what it had (the reference's last noi)
        j++;
        if (res.found != 1) { // no DCI, or the search's error: srslte_ue_dl_decode_rnti returns 0
          sl.ue_state[i] = 0;
          continue;
        }
        sl.ue_state[i] = grant_of(u, res, u->cfi, dl, s);
        if (sl.ue_state[i] != 1) continue;
      } else {
        s = b[i].it->sf;
        const uint32_t ntb = sf_ntb(s);
        for (uint32_t t = 0; t < ntb; t++)
          if (b[i].it->reset_softbuffer[t]) {
            if (s.softbuffer[t] >= nsb) return -1;
            rs_slot.push_back(s.softbuffer[t]);
            rs_ncb.push_back(UINT32_MAX); // srslte_softbuffer_rx_reset: every block
          }
      }
      s.grid_offset = (uint64_t)i * nrx * gsz;
      s.ce_offset = (uint64_t)i * nrx * nports * gsz;
      sfs.push_back(s);
      sl.who.push_back(i);
    }
    const uint32_t np = (uint32_t)sfs.size();
    if (!rs_slot.empty() && srsgpu_dlsch_softbuffer_reset_list(dl, rs_slot.data(), rs_ncb.data(), (uint32_t)rs_slot.size()))
      return -1;
    // each TB's output: the caller's buffer itself when it lies in registered memory (the decoder writes
    // it over PCIe), else the next free bytes of d_data, copied back in one transfer and then into place
    std::vector<uint8_t *> outp;
    sl.ntb_of.clear();
    sl.tbs_of.clear();
    sl.stage_off.clear();
    sl.staged_bytes = 0;
    {
      std::lock_guard<std::mutex> lk(m); // regions
      for (uint32_t k = 0; k < np; k++) {
        const Pending &p = b[sl.who[k]];
        const uint32_t ntb = sf_ntb(sfs[k]);
        sl.ntb_of.push_back(ntb);
        for (uint32_t t = 0; t < ntb; t++) {
          uint8_t *out = p.it ? p.it->data[t] : p.ue->data[t];
          const size_t len = SRSGPU_DLSCH_DATA_LEN(sfs[k].tbs[t]);
          const bool skip = (sfs[k].skip_tb >> t) & 1u;
          const void *dv = (out && !skip) ? device_view(out, len, false) : nullptr;
          sl.tbs_of.push_back(sfs[k].tbs[t]);
          if (dv) {
            outp.push_back((uint8_t *)dv);
            sl.stage_off.push_back(-1);
            zero_copy_tbs++;
          } else {
            outp.push_back(d_data + sl.staged_bytes);
            sl.stage_off.push_back(skip || !out ? -2 : (int64_t)sl.staged_bytes);
            if (!skip && out) {
              sl.staged_bytes += (len + 15) & ~(size_t)15;
              staged_tbs++;
            }
          }
        }
      }
    }
    lap(2);
    if (np) {
      srsgpu_pdsch_set_noise_dev(pdsch, d_noise);
      // the PDSCH's per-subframe noise comes from d_noise at the subframe's position in the call:
      // compact the noise rows of the decoded subframes when some subframes have no PDSCH
      if (np != n) {
        for (uint32_t k = 0; k < np; k++) sl.h_who[k] = sl.who[k];
        const int cols = (int)(nrx * nports);
        RXQ_CHK(xfer(d_who, sl.h_who, sizeof(uint32_t) * np, hipMemcpyHostToDevice, st));
        hipLaunchKernelGGL(k_noise_gather, dim3((np * cols + 255) / 256), dim3(256), 0, st, d_noise, d_who,
                           (int)np, cols, d_pnoise);
        RXQ_CHK(hipGetLastError());
        srsgpu_pdsch_set_noise_dev(pdsch, d_pnoise);
      }
      // TB results come back in call order: (subframe, tb), CDD subframes holding two
      const double pw = now_s(), pc = cpu_s();
      if (srsgpu_pdsch_decode_out_dev(pdsch, sfs.data(), np, d_grid, d_ce, gsz, outp.data(), max_halfits, d_ret, d_noi))
        return -1;
      if (trace)
        fprintf(stderr, "rxq trace: n %u pdsch_decode wall %.3f ms cpu %.3f ms\n", n, (now_s() - pw) * 1e3,
                (cpu_s() - pc) * 1e3);
      const size_t ntbs = outp.size();
      if (sl.staged_bytes)
        RXQ_CHK(xfer(sl.h_data, d_data, sl.staged_bytes, hipMemcpyDeviceToHost, st));
      RXQ_CHK(xfer(sl.h_ret, d_ret, sizeof(int32_t) * ntbs, hipMemcpyDeviceToHost, st));
      RXQ_CHK(xfer(sl.h_noi, d_noi, sizeof(uint32_t) * ntbs, hipMemcpyDeviceToHost, st));
    }
    RXQ_CHK(xfer(sl.h_noise, d_noise, sizeof(float) * n * nrx * nports, hipMemcpyDeviceToHost, st));
    lap(3);
    if (trace)
      fprintf(stderr, "rxq trace: n %u front %.3f control %.3f grants %.3f pdsch %.3f ms\n", n, run_tm[0] * 1e3,
              run_tm[1] * 1e3, run_tm[2] * 1e3, run_tm[3] * 1e3);
    return 0;
  }

  // the results of a finished batch into its items (completer thread)
  void complete(Slot &sl) {
    const std::vector<Pending> &b = sl.items;
    const uint32_t n = (uint32_t)b.size();
    for (uint32_t k = 0, t0 = 0; k < (uint32_t)sl.who.size(); k++) {
      const Pending &p = b[sl.who[k]];
      for (uint32_t t = 0; t < sl.ntb_of[k]; t++, t0++) {
        uint8_t *out = p.it ? p.it->data[t] : p.ue->data[t];
        if (p.it) {
          p.it->ret[t] = sl.h_ret[t0];
          p.it->noi[t] = sl.h_noi[t0];
        } else {
          if (p.ue->acked_in[t]) continue; // skipped as srslte_pdsch_decode skips it: nothing written
          p.ue->noi[t] = sl.h_noi[t0];
          p.ue->acks[t] = sl.h_ret[t0] == 0;
        }
        if (out && sl.stage_off[t0] >= 0) memcpy(out, sl.h_data + sl.stage_off[t0], SRSGPU_DLSCH_DATA_LEN(sl.tbs_of[t0]));
      }
    }
    for (uint32_t i = 0, jf = 0; i < n; i++) {
      // srslte_chest_dl_get_noise_estimate (chest_dl.c:741-750): mean over ports, then antennas
      float nn = 0.f;
      for (uint32_t a = 0; a < nrx; a++) {
        float acc = 0.f;
        for (uint32_t p = 0; p < nports; p++) acc += sl.h_noise[(i * nrx + a) * nports + p];
        nn += acc / (float)nports;
      }
      nn /= (float)nrx;
      const float *g = sl.h_getters + (size_t)i * 6;
      const srsgpu_rxq_meas_t meas = {g[0], g[1], g[2], g[3], g[4], g[5]};
      if (b[i].it) {
        b[i].it->noise = nn;
        b[i].it->meas = meas;
      } else {
        srsgpu_rxq_ue_dl_t *u = b[i].ue;
        u->noise = nn;
        u->meas = meas;
        // ue_dl.c:612-616: TB 0's size when a DCI was found and the PDSCH call succeeded
        u->ret = sl.ue_state[i] < 0 ? -1 : (u->found == 1 ? u->grant.tbs[0] : 0);
        if (u->feedback && sl.fb_any) {
          u->fb = sl.h_fb[jf];
        } else {
          memset(&u->fb, 0, sizeof(u->fb));
          u->fb.ret_cn = u->fb.ret_pmi = -1;
        }
        jf++;
      }
    }
  }
};

extern "C" {

int srsgpu_rxq_create(srsgpu_rxq_t **q, const srsgpu_cell_t *cell, uint32_t symbol_sz,
                      uint32_t nof_softbuffers, uint32_t max_batch, uint32_t max_wait_us,
                      uint32_t max_halfits) {
  if (!q || !cell || !symbol_sz || !max_batch || !max_halfits || cell->nof_rx_ant < 1 ||
      cell->nof_rx_ant > 2 || (cell->nof_ports != 1 && cell->nof_ports != 2 && cell->nof_ports != 4))
    return -1;
  auto *r = new srsgpu_rxq();
  if (r->setup(cell, symbol_sz, nof_softbuffers, max_batch, max_wait_us, max_halfits)) {
    r->teardown();
    delete r;
    *q = nullptr;
    return -1;
  }
  *q = r;
  return 0;
}

void srsgpu_rxq_destroy(srsgpu_rxq_t *q) {
  if (!q) return;
  q->teardown();
  delete q;
}

int srsgpu_rxq_submit(srsgpu_rxq_t *q, srsgpu_rxq_item_t *it, uint64_t *ticket) {
  if (!q || !it || !ticket) return -1;
  return q->submit(it, nullptr, ticket);
}

int srsgpu_rxq_submit_ue_dl(srsgpu_rxq_t *q, srsgpu_rxq_ue_dl_t *u, uint64_t *ticket) {
  if (!q || !u || !ticket || u->tm > 7) return -1;
  return q->submit(nullptr, u, ticket);
}

int srsgpu_rxq_wait(srsgpu_rxq_t *q, uint64_t ticket) {
  if (!q || ticket == 0) return -1;
  std::unique_lock<std::mutex> l(q->m);
  if (ticket >= q->next_ticket) return -1;
  q->cv_done.wait(l, [&] { return q->done_upto >= ticket; });
  // a failure is reported once, to the ticket's waiter, and then forgotten
  return q->failed.erase(ticket) ? -1 : 0;
}

int srsgpu_rxq_decode(srsgpu_rxq_t *q, srsgpu_rxq_item_t *it) {
  uint64_t t = 0;
  if (srsgpu_rxq_submit(q, it, &t)) return -1;
  return srsgpu_rxq_wait(q, t);
}

int srsgpu_rxq_decode_rnti(srsgpu_rxq_t *q, srsgpu_rxq_ue_dl_t *u) {
  uint64_t t = 0;
  if (srsgpu_rxq_submit_ue_dl(q, u, &t)) return -1;
  return srsgpu_rxq_wait(q, t);
}

int srsgpu_rxq_set_phich(srsgpu_rxq_t *q, uint32_t phich_length, uint32_t phich_resources) {
  if (!q || phich_length > 1 || phich_resources > 3) return -1;
  std::lock_guard<std::mutex> l(q->m);
  q->phich_len = phich_length;
  q->phich_res = phich_resources;
  q->phich_dirty = true; // the dispatcher rebuilds the map before its next ue_dl batch
  return 0;
}

void srsgpu_rxq_flush(srsgpu_rxq_t *q) {
  if (!q) return;
  {
    std::lock_guard<std::mutex> l(q->m);
    if (q->slot[q->fill].items.empty()) return; // nothing to close: the next submission waits as usual
    q->flush = true;
  }
  q->cv_close.notify_one();
}

int srsgpu_rxq_register(srsgpu_rxq_t *q, void *host, size_t bytes) {
  if (!q || !host || !bytes) return -1;
  if (hipHostRegister(host, bytes, hipHostRegisterMapped) != hipSuccess) {
    fprintf(stderr, "srsgpu rxq: hipHostRegister of %zu bytes failed\n", bytes);
    return -1;
  }
  void *d = nullptr;
  if (hipHostGetDevicePointer(&d, host, 0) != hipSuccess || !d) {
    (void)hipHostUnregister(host);
    return -1;
  }
  std::lock_guard<std::mutex> l(q->m);
  q->regions.push_back({(const char *)host, bytes, (const char *)d, false});
  return 0;
}

// remove a region of the given kind once nothing queued or in flight points into it: 0, -1 if there
// is no such region, -2 if it is of the other kind (then kept)
static int rxq_drop_region(srsgpu_rxq_t *q, void *host, bool owned) {
  std::unique_lock<std::mutex> l(q->m);
  q->cv_done.wait(l, [&] { return q->done_upto + 1 >= q->next_ticket; });
  auto it = std::find_if(q->regions.begin(), q->regions.end(), [&](const srsgpu_rxq::Region &r) { return r.h == host; });
  if (it == q->regions.end()) return -1;
  if (it->owned != owned) {
    fprintf(stderr, owned ? "srsgpu rxq: free_host of a registered region (use srsgpu_rxq_unregister)\n"
                          : "srsgpu rxq: unregister of a queue-owned block (use srsgpu_rxq_free_host)\n");
    return -2;
  }
  q->regions.erase(it);
  return 0;
}

int srsgpu_rxq_unregister(srsgpu_rxq_t *q, void *host) {
  if (!q || !host) return -1;
  // every batch that read or wrote the region has completed (its done event synchronised), and the
  // copy stream's spans from it with them: no device view of it outlives this call
  if (rxq_drop_region(q, host, false)) return -1;
  return hipHostUnregister(host) == hipSuccess ? 0 : -1;
}

void *srsgpu_rxq_alloc_host(srsgpu_rxq_t *q, size_t bytes) {
  if (!q || !bytes) return nullptr;
  void *h = nullptr, *d = nullptr;
  if (hipHostMalloc(&h, bytes, hipHostMallocMapped) != hipSuccess || !h) {
    fprintf(stderr, "srsgpu rxq: hipHostMalloc of %zu bytes failed\n", bytes);
    return nullptr;
  }
  if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess || !d) {
    (void)hipHostFree(h);
    return nullptr;
  }
  std::lock_guard<std::mutex> l(q->m);
  q->regions.push_back({(const char *)h, bytes, (const char *)d, true});
  return h;
}

int srsgpu_rxq_free_host(srsgpu_rxq_t *q, void *host) {
  if (!q || !host) return -1;
  if (rxq_drop_region(q, host, true)) return -1;
  return hipHostFree(host) == hipSuccess ? 0 : -1;
}

int srsgpu_rxq_set_input_format(srsgpu_rxq_t *q, uint32_t format, float scale) {
  if (!q || format > SRSGPU_RXQ_SC16) return -1;
  {
    std::unique_lock<std::mutex> l(q->m);
    q->cv_done.wait(l, [&] { return !q->fmt_busy; });
    q->fmt_busy = true; // new submissions wait; the queued ones drain under the old format
    q->cv_done.wait(l, [&] { return q->done_upto + 1 >= q->next_ticket; });
    q->sc16 = format == SRSGPU_RXQ_SC16;
    q->sc16_scale = scale != 0.f ? scale : 1.0f / 32768.0f;
    q->fmt_busy = false;
  }
  q->cv_slot.notify_all();
  q->cv_done.notify_all();
  return 0;
}

void srsgpu_rxq_ingest_stats(srsgpu_rxq_t *q, uint64_t *zero_copy_rows, uint64_t *staged_rows) {
  if (!q) return;
  std::lock_guard<std::mutex> l(q->m);
  if (zero_copy_rows) *zero_copy_rows = q->zero_copy_rows;
  if (staged_rows) *staged_rows = q->staged_rows;
}

void srsgpu_rxq_timing(srsgpu_rxq_t *q, double *sec, uint32_t n) {
  if (!q || !sec) return;
  std::lock_guard<std::mutex> l(q->m);
  for (uint32_t i = 0; i < n && i < 8; i++) sec[i] = q->tm[i];
}

struct srsgpu_chest *srsgpu_rxq_get_chest(srsgpu_rxq_t *q) { return q ? q->chest : nullptr; }
srsgpu_pdsch_t *srsgpu_rxq_get_pdsch(srsgpu_rxq_t *q) { return q ? q->pdsch : nullptr; }

void srsgpu_rxq_stats(srsgpu_rxq_t *q, uint64_t *batches, uint64_t *subframes) {
  if (!q) return;
  std::lock_guard<std::mutex> l(q->m);
  if (batches) *batches = q->nbatches;
  if (subframes) *subframes = q->nsf;
}

int srsgpu_rxq_drive(srsgpu_rxq_t *q, srsgpu_rxq_item_t *const *items, uint32_t n, uint32_t workers,
                     uint32_t reuse, double *t_sub, double *t_done, int32_t *status) {
  if (!q || !items || !workers || workers > 256 || !t_sub || !t_done || !status) return -1;
  std::mutex m;
  // the collector waits for submissions, producers for collected items: each side wakes only the other
  std::condition_variable cv_col, cv_prod;
  std::vector<uint64_t> tickets(n, 0);
  std::vector<uint8_t> state(n, 0); // 1 submitted, 2 refused
  uint32_t ndone = 0, producing = workers;
  int err = 0;
  auto now = [] {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
  };
  auto produce = [&](uint32_t w) {
    for (uint32_t i = w; i < n; i += workers) {
      if (reuse && i >= reuse) { // the item's softbuffer / output slot: wait for its last user
        std::unique_lock<std::mutex> l(m);
        cv_prod.wait(l, [&] { return ndone > i - reuse || err; });
      }
      {
        std::lock_guard<std::mutex> l(m);
        if (err) break;
      }
      t_sub[i] = now();
      uint64_t t = 0;
      const int r = srsgpu_rxq_submit(q, items[i], &t);
      {
        std::lock_guard<std::mutex> l(m);
        tickets[i] = t;
        state[i] = r ? 2 : 1;
        if (r && !err) err = r;
      }
      cv_col.notify_one();
      if (r) cv_prod.notify_all();
    }
    {
      std::lock_guard<std::mutex> l(m);
      producing--;
    }
    cv_col.notify_one();
  };
  std::thread collector([&] {
    for (uint32_t i = 0; i < n; i++) {
      uint8_t s;
      uint64_t t;
      {
        std::unique_lock<std::mutex> l(m);
        cv_col.wait(l, [&] { return state[i] != 0 || producing == 0; });
        s = state[i];
        t = tickets[i];
      }
      status[i] = s == 1 ? srsgpu_rxq_wait(q, t) : -1;
      t_done[i] = now();
      {
        std::lock_guard<std::mutex> l(m);
        ndone = i + 1;
      }
      cv_prod.notify_all();
    }
  });
  std::vector<std::thread> pool;
  for (uint32_t w = 0; w < workers; w++) pool.emplace_back(produce, w);
  for (auto &t : pool) t.join();
  srsgpu_rxq_flush(q); // the last, partial batch
  collector.join();
  return err ? -1 : 0;
}

// pin a std::thread to one CPU (no-op for cpu < 0); 0 or the pthread error
static int pin_thread(std::thread &t, int cpu) {
  if (cpu < 0) return 0;
  cpu_set_t set;
  CPU_ZERO(&set);
  CPU_SET(cpu, &set);
  return pthread_setaffinity_np(t.native_handle(), sizeof(set), &set);
}

int srsgpu_rxq_set_affinity(srsgpu_rxq_t *q, const int32_t *cpus, uint32_t n) {
  if (!q || (!cpus && n)) return -1;
  std::thread *th[3] = {&q->closer, &q->worker, &q->completer};
  int r = 0;
  for (int k = 0; k < 3; k++)
    if (n && pin_thread(*th[k], cpus[k % n])) r = -1;
  return r;
}

int srsgpu_rxq_drive_paced(srsgpu_rxq_t *q, srsgpu_rxq_item_t *const *items, uint32_t streams, uint32_t depth,
                           uint32_t ticks, uint32_t period_us, uint32_t workers, float *latency_ms, int32_t *status,
                           uint32_t *acked, double *late_ms) {
  return srsgpu_rxq_drive_paced_ex(q, items, streams, depth, ticks, period_us, workers, nullptr, 0, latency_ms,
                                   nullptr, status, acked, late_ms);
}

int srsgpu_rxq_drive_paced_ex(srsgpu_rxq_t *q, srsgpu_rxq_item_t *const *items, uint32_t streams, uint32_t depth,
                              uint32_t ticks, uint32_t period_us, uint32_t workers, const int32_t *cpus,
                              uint32_t ncpus, float *latency_ms, float *submit_latency_ms, int32_t *status,
                              uint32_t *acked, double *late_ms) {
  if (!q || !items || !streams || !depth || !ticks || !period_us || !workers || workers > 256 || !latency_ms ||
      !status || (!cpus && ncpus))
    return -1;
  using clk = std::chrono::steady_clock;
  const uint64_t n = (uint64_t)streams * ticks;
  std::mutex m;
  // the collector waits for submissions, producers for collected items: each side wakes only the other
  std::condition_variable cv_col, cv_prod;
  std::vector<uint64_t> tickets(n, 0);
  std::vector<uint8_t> state(n, 0); // 1 submitted, 2 refused / skipped
  std::vector<clk::time_point> t_sub(n);
  uint64_t ndone = 0;
  uint32_t producing = std::min(workers, streams), nack = 0;
  int err = 0;
  double worst_late = 0; // how far behind its tick a submission went out (a producer that falls behind)
  const clk::time_point t0 = clk::now() + std::chrono::milliseconds(2);
  auto tick_time = [&](uint64_t t) { return t0 + std::chrono::microseconds((uint64_t)period_us * t); };
  // producer w owns streams w, w + W, ...: at each tick it submits their subframes
  auto produce = [&](uint32_t w) {
    for (uint64_t t = 0; t < ticks; t++) {
      std::this_thread::sleep_until(tick_time(t));
      for (uint32_t st = w; st < streams; st += producing) {
        const uint64_t i = t * streams + st;
        if (t >= depth) { // the item's softbuffer / output slot: its use depth ticks ago is collected
          std::unique_lock<std::mutex> l(m);
          cv_prod.wait(l, [&] { return ndone > i - (uint64_t)depth * streams || err; });
        }
        int r = -1;
        uint64_t tk = 0;
        bool skip;
        {
          std::lock_guard<std::mutex> l(m);
          skip = err != 0;
        }
        if (!skip) {
          const clk::time_point ts = clk::now();
          const double late = std::chrono::duration<double, std::milli>(ts - tick_time(t)).count();
          r = srsgpu_rxq_submit(q, items[(t % depth) * streams + st], &tk);
          std::lock_guard<std::mutex> l(m);
          t_sub[i] = ts;
          if (late > worst_late) worst_late = late;
        }
        {
          std::lock_guard<std::mutex> l(m);
          tickets[i] = tk;
          state[i] = r ? 2 : 1;
          if (r && !err) err = -1;
        }
        cv_col.notify_one();
        if (r) cv_prod.notify_all();
      }
    }
  };
  std::thread collector([&] {
    for (uint64_t i = 0; i < n; i++) {
      uint8_t s;
      uint64_t tk;
      clk::time_point ts;
      {
        std::unique_lock<std::mutex> l(m);
        cv_col.wait(l, [&] { return state[i] != 0; });
        s = state[i];
        tk = tickets[i];
        ts = t_sub[i];
      }
      const int r = s == 1 ? srsgpu_rxq_wait(q, tk) : -1;
      const clk::time_point done = clk::now();
      status[i] = r;
      latency_ms[i] = (float)std::chrono::duration<double, std::milli>(done - tick_time(i / streams)).count();
      if (submit_latency_ms)
        submit_latency_ms[i] = s == 1 ? (float)std::chrono::duration<double, std::milli>(done - ts).count() : -1.f;
      const srsgpu_rxq_item_t *it = items[((i / streams) % depth) * streams + i % streams];
      {
        std::lock_guard<std::mutex> l(m);
        if (!r && it->ret[0] == 0) nack++;
        ndone = i + 1;
      }
      cv_prod.notify_all();
    }
  });
  // CPUs: the collector on cpus[0], producer w on cpus[(1 + w) % ncpus]
  if (ncpus) (void)pin_thread(collector, cpus[0]);
  std::vector<std::thread> pool;
  for (uint32_t w = 0; w < producing; w++) {
    pool.emplace_back(produce, w);
    if (ncpus) (void)pin_thread(pool.back(), cpus[(1 + w) % ncpus]);
  }
  for (auto &t : pool) t.join();
  srsgpu_rxq_flush(q);
  collector.join();
  if (acked) *acked = nack;
  if (late_ms) *late_ms = worst_late;
  return err ? -1 : 0;
}

} // extern "C"
