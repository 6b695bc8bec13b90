// Subframe batch queue (include/srsgpu/rx_queue.h): PHY-worker threads submit single subframes,
// one dispatcher thread runs them through OFDM -> channel estimation -> PDSCH / DL-SCH in batches
// (the GPU counterpart of srsUE's per-subframe worker pool, srsue/src/phy/phy.cc:141-168,
// phch_worker.cc:548-806).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <set>
#include <thread>
#include <vector>

#include "srsgpu/chest_batch.h"
#include "srsgpu/dlsch_batch.h"
#include "srsgpu/ofdm_batch.h"
#include "srsgpu/pdsch_batch.h"
#include "srsgpu/rx_queue.h"

namespace {

#define RXQ_CHK(x)                                                                                 \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) {                                                                        \
      fprintf(stderr, "srsgpu rxq: %s failed: %s\n", #x, hipGetErrorString(e_));                   \
      return -1;                                                                                   \
    }                                                                                              \
  } while (0)

struct Pending {
  srsgpu_rxq_item_t *it;
  uint64_t ticket;
  std::chrono::steady_clock::time_point t;
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

} // namespace

struct srsgpu_rxq {
  srsgpu_cell_t cell{};
  uint32_t N = 0, max_batch = 0, max_wait_us = 0, max_halfits = 8, nports = 1, nrx = 1;
  size_t td_len = 0, gsz = 0, dlen = 0; // complex samples per antenna / grid elements / TB bytes
  hipStream_t st = nullptr;
  srsgpu_ofdm_t *ofdm = nullptr;
  srsgpu_chest_t *chest = nullptr;
  srsgpu_pdsch_t *pdsch = nullptr;
  float *d_td = nullptr, *d_grid = nullptr, *d_ce = nullptr, *d_noise = nullptr;
  float *d_noise_last = nullptr; // PSS / EMPTY: the estimate carried between batches
  uint8_t *d_est = nullptr, *h_est = nullptr; // per subframe: 1 if it estimates the noise
  uint8_t *d_data = nullptr;
  int32_t *d_ret = nullptr;
  uint32_t *d_noi = nullptr;
  float *h_td = nullptr, *h_noise = nullptr; // pinned staging
  uint8_t *h_data = nullptr;
  int32_t *h_ret = nullptr;
  uint32_t *h_noi = nullptr;

  std::mutex m;
  std::condition_variable cv_work, cv_done;
  std::deque<Pending> queue;
  uint64_t next_ticket = 1, done_upto = 0; // tickets are completed in order
  std::set<uint64_t> failed;               // tickets whose batch failed, until waited for
  bool stop = false, flush = false;
  uint64_t nbatches = 0, nsf = 0;
  std::thread worker;

  int setup(const srsgpu_cell_t *c, uint32_t symbol_sz, uint32_t nsb, uint32_t mb, uint32_t wait_us,
            uint32_t maxh) {
    cell = *c;
    N = symbol_sz;
    max_batch = mb;
    max_wait_us = wait_us;
    max_halfits = maxh;
    nports = cell.nof_ports;
    nrx = cell.nof_rx_ant;
    td_len = (size_t)15 * N;
    gsz = (size_t)14 * 12 * cell.nof_prb;
    dlen = SRSGPU_DLSCH_DATA_LEN(75376) + 16;
    const uint32_t max_cb = 13;
    RXQ_CHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    if (srsgpu_ofdm_rx_create(&ofdm, cell.nof_prb, N) ||
        srsgpu_chest_create(&chest, &cell, mb * nrx) ||
        srsgpu_pdsch_create(&pdsch, &cell, nsb, max_cb, mb))
      return -1;
    srsgpu_ofdm_rx_set_stream(ofdm, st);
    srsgpu_chest_set_stream(chest, st);
    srsgpu_pdsch_set_stream(pdsch, st);
    RXQ_CHK(hipMalloc(&d_td, sizeof(float) * 2 * td_len * mb * nrx));
    RXQ_CHK(hipMalloc(&d_grid, sizeof(float) * 2 * gsz * mb * nrx));
    RXQ_CHK(hipMalloc(&d_ce, sizeof(float) * 2 * gsz * mb * nrx * nports));
    RXQ_CHK(hipMalloc(&d_noise, sizeof(float) * mb * nrx * nports));
    RXQ_CHK(hipMalloc(&d_data, dlen * 2 * mb));
    RXQ_CHK(hipMalloc(&d_ret, sizeof(int32_t) * 2 * mb));
    RXQ_CHK(hipMalloc(&d_noi, sizeof(uint32_t) * 2 * mb));
    RXQ_CHK(hipMalloc(&d_noise_last, sizeof(float) * nrx * nports));
    RXQ_CHK(hipMemset(d_noise_last, 0, sizeof(float) * nrx * nports)); // srslte_chest_dl_init: 0
    RXQ_CHK(hipMalloc(&d_est, mb));
    RXQ_CHK(hipHostMalloc(&h_est, mb));
    RXQ_CHK(hipHostMalloc(&h_td, sizeof(float) * 2 * td_len * mb * nrx));
    RXQ_CHK(hipHostMalloc(&h_noise, sizeof(float) * mb * nrx * nports));
    RXQ_CHK(hipHostMalloc(&h_data, dlen * 2 * mb));
    RXQ_CHK(hipHostMalloc(&h_ret, sizeof(int32_t) * 2 * mb));
    RXQ_CHK(hipHostMalloc(&h_noi, sizeof(uint32_t) * 2 * mb));
    worker = std::thread([this] { loop(); });
    return 0;
  }

  void teardown() {
    {
      std::lock_guard<std::mutex> l(m);
      stop = true;
    }
    cv_work.notify_all();
    if (worker.joinable()) worker.join();
    if (ofdm) srsgpu_ofdm_rx_destroy(ofdm);
    if (chest) srsgpu_chest_destroy(chest);
    if (pdsch) srsgpu_pdsch_destroy(pdsch);
    for (void *p : {(void *)d_td, (void *)d_grid, (void *)d_ce, (void *)d_noise, (void *)d_data,
                    (void *)d_ret, (void *)d_noi, (void *)d_noise_last, (void *)d_est})
      if (p) (void)hipFree(p);
    for (void *p : {(void *)h_td, (void *)h_noise, (void *)h_data, (void *)h_ret, (void *)h_noi, (void *)h_est})
      if (p) (void)hipHostFree(p);
    if (st) (void)hipStreamDestroy(st);
  }

  // one batch: inputs staged and copied in one transfer, three pipeline calls, one copy back
  int run(std::vector<Pending> &b) {
    const uint32_t n = (uint32_t)b.size();
    const size_t sfc = 2 * td_len; // floats per antenna plane
    for (uint32_t i = 0; i < n; i++)
      for (uint32_t a = 0; a < nrx; a++)
        memcpy(h_td + (i * nrx + a) * sfc, b[i].it->td[a], sizeof(float) * sfc);
    RXQ_CHK(hipMemcpyAsync(d_td, h_td, sizeof(float) * sfc * n * nrx, hipMemcpyHostToDevice, st));
    if (srsgpu_ofdm_rx_sf_dev(ofdm, n * nrx, d_td, td_len, d_grid, gsz)) return -1;
    std::vector<uint32_t> sfi(n * nrx);
    for (uint32_t i = 0; i < n; i++)
      for (uint32_t a = 0; a < nrx; a++) sfi[i * nrx + a] = b[i].it->sf.sf_idx;
    srsgpu_chest_cfg_t ccfg;
    if (srsgpu_chest_get_cfg(chest, &ccfg)) return -1;
    if (ccfg.noise_alg != 0 && ccfg.smooth_filter_auto) {
      // each subframe's filter would come from the previous subframe's noise: no batch order
      fprintf(stderr, "srsgpu rxq: smooth_filter_auto with PSS / EMPTY noise is not batched\n");
      return -1;
    }
    if (srsgpu_chest_estimate_dev(chest, sfi.data(), n * nrx, d_grid, gsz, d_ce, d_noise)) return -1;
    if (ccfg.noise_alg != 0) { // PSS / EMPTY: carry the estimate across subframes in order
      for (uint32_t i = 0; i < n; i++) h_est[i] = (uint8_t)(b[i].it->sf.sf_idx == 0 || b[i].it->sf.sf_idx == 5);
      RXQ_CHK(hipMemcpyAsync(d_est, h_est, n, hipMemcpyHostToDevice, st));
      // grids of one subframe's rx antennas are consecutive: n rows of nrx * nports columns
      hipLaunchKernelGGL(k_noise_carry, dim3(1), dim3(64), 0, st, d_noise, d_est, (int)n, (int)(nrx * nports),
                         d_noise_last);
      RXQ_CHK(hipGetLastError());
    }
    srsgpu_pdsch_set_noise_dev(pdsch, d_noise);
    srsgpu_dlsch_t *dl = srsgpu_pdsch_get_dlsch(pdsch);
    std::vector<srsgpu_pdsch_sf_t> sfs(n);
    for (uint32_t i = 0; i < n; i++) {
      srsgpu_pdsch_sf_t &s = sfs[i];
      s = b[i].it->sf;
      s.grid_offset = (uint64_t)i * nrx * gsz;
      s.ce_offset = (uint64_t)i * nrx * nports * gsz;
      s.data_offset[0] = (uint64_t)(2 * i) * dlen;
      s.data_offset[1] = (uint64_t)(2 * i + 1) * dlen;
      const uint32_t ntb = s.mimo_type == SRSGPU_MIMO_CDD ? 2 : 1;
      for (uint32_t t = 0; t < ntb; t++)
        if (b[i].it->reset_softbuffer[t] && srsgpu_dlsch_softbuffer_reset(dl, s.softbuffer[t]))
          return -1;
    }
    // TB results come back in call order: (subframe, tb), CDD subframes holding two
    if (srsgpu_pdsch_decode_dev(pdsch, sfs.data(), n, d_grid, d_ce, gsz, d_data, max_halfits, d_ret,
                                d_noi))
      return -1;
    uint32_t ntbs = 0;
    for (uint32_t i = 0; i < n; i++) ntbs += sfs[i].mimo_type == SRSGPU_MIMO_CDD ? 2 : 1;
    RXQ_CHK(hipMemcpyAsync(h_data, d_data, dlen * 2 * n, hipMemcpyDeviceToHost, st));
    RXQ_CHK(hipMemcpyAsync(h_ret, d_ret, sizeof(int32_t) * ntbs, hipMemcpyDeviceToHost, st));
    RXQ_CHK(hipMemcpyAsync(h_noi, d_noi, sizeof(uint32_t) * ntbs, hipMemcpyDeviceToHost, st));
    RXQ_CHK(hipMemcpyAsync(h_noise, d_noise, sizeof(float) * n * nrx * nports, hipMemcpyDeviceToHost, st));
    RXQ_CHK(hipStreamSynchronize(st));
    uint32_t k = 0;
    for (uint32_t i = 0; i < n; i++) {
      srsgpu_rxq_item_t *it = b[i].it;
      const uint32_t ntb = sfs[i].mimo_type == SRSGPU_MIMO_CDD ? 2 : 1;
      for (uint32_t t = 0; t < ntb; t++, k++) {
        it->ret[t] = h_ret[k];
        it->noi[t] = h_noi[k];
        if (it->data[t])
          memcpy(it->data[t], h_data + (2 * i + t) * dlen, SRSGPU_DLSCH_DATA_LEN(sfs[i].tbs[t]));
      }
      // srslte_chest_dl_get_noise_estimate (chest_dl.c:741-750): mean over ports, then antennas
      float nn = 0.f;
      for (uint32_t a = 0; a < nrx; a++) {
        float acc = 0.f;
        for (uint32_t p = 0; p < nports; p++) acc += h_noise[(i * nrx + a) * nports + p];
        nn += acc / (float)nports;
      }
      it->noise = nn / (float)nrx;
    }
    return 0;
  }

  void loop() {
    std::unique_lock<std::mutex> l(m);
    for (;;) {
      cv_work.wait(l, [this] { return stop || !queue.empty(); });
      if (queue.empty() && stop) return;
      // let the batch fill: up to max_batch, or until the oldest waited max_wait_us
      const auto deadline = queue.front().t + std::chrono::microseconds(max_wait_us);
      cv_work.wait_until(l, deadline, [this] { return stop || flush || queue.size() >= max_batch; });
      flush = false;
      std::vector<Pending> b;
      while (!queue.empty() && b.size() < max_batch) {
        b.push_back(queue.front());
        queue.pop_front();
      }
      l.unlock();
      const int r = run(b);
      // a failed batch may have left copies in flight that still read the pinned staging
      // buffers: drain the stream before they are reused
      if (r) (void)hipStreamSynchronize(st);
      l.lock();
      if (r) {
        fprintf(stderr, "srsgpu rxq: batch of %zu subframes failed\n", b.size());
        for (const Pending &p : b) failed.insert(p.ticket);
      }
      done_upto = b.back().ticket;
      nbatches++;
      nsf += b.size();
      cv_done.notify_all();
    }
  }
};

extern "C" {

int srsgpu_rxq_create(srsgpu_rxq_t **q, const srsgpu_cell_t *cell, uint32_t symbol_sz,
                      uint32_t nof_softbuffers, uint32_t max_batch, uint32_t max_wait_us,
                      uint32_t max_halfits) {
  if (!q || !cell || !symbol_sz || !max_batch || !max_halfits || cell->nof_rx_ant < 1 ||
      cell->nof_rx_ant > 2 || cell->nof_ports < 1 || cell->nof_ports > 2)
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
  if (!q || !it || !ticket || !it->td[0] || (q->nrx > 1 && !it->td[1])) return -1;
  {
    std::lock_guard<std::mutex> l(q->m);
    if (q->stop) return -1;
    *ticket = q->next_ticket++;
    q->queue.push_back({it, *ticket, std::chrono::steady_clock::now()});
  }
  q->cv_work.notify_one();
  return 0;
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

void srsgpu_rxq_flush(srsgpu_rxq_t *q) {
  if (!q) return;
  {
    std::lock_guard<std::mutex> l(q->m);
    if (q->queue.empty()) return; // nothing to close: the next submission waits as usual
    q->flush = true;
  }
  q->cv_work.notify_one();
}

struct srsgpu_chest *srsgpu_rxq_get_chest(srsgpu_rxq_t *q) { return q ? q->chest : nullptr; }
srsgpu_pdsch_t *srsgpu_rxq_get_pdsch(srsgpu_rxq_t *q) { return q ? q->pdsch : nullptr; }

void srsgpu_rxq_stats(srsgpu_rxq_t *q, uint64_t *batches, uint64_t *subframes) {
  if (!q) return;
  std::lock_guard<std::mutex> l(q->m);
  if (batches) *batches = q->nbatches;
  if (subframes) *subframes = q->nsf;
}

} // extern "C"
