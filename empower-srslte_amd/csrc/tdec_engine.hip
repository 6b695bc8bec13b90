// Host side of the MI355X turbo decoder: device-buffer engine, half-iteration schedule and the
// C ABI (include/srsgpu/tdec_batch.h + the drop-in include/srslte/phy/fec/turbodecoder.h).
//
// Schedule per code-block batch (all CBs share K; mirrors turbodecoder_iter.h:283-357):
//   load          user layout -> pair-interleaved syst/par0 (SP0), par1 (P1 plane of XP1), tails
//   halfit(n)     one constituent decoder run: DEC1 for even n, DEC2 for odd n, with the
//                 interleave / subtract glue fused into its output stage (tdec_kernels.hip)
//   decide(n)     hard decision after half-iteration n (+ CRC and early-stop flags when asked,
//                 sch.c:361-391)
#include <hip/hip_runtime.h>
#include <chrono>

#include <map>
#include <mutex>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <string>
#include <utility>
#include <vector>

#include "srsgpu/qpp_table.h"
#include "srsgpu/tdec_batch.h"
#include "srslte/phy/fec/turbodecoder.h"
#include "tdec_engine.h"

namespace srsgpu {

// ------------------------------------------------------------------ profiling ----
struct ProfRec {
  std::string name;
  hipEvent_t a, b;
};
struct Prof {
  std::mutex mu;
  bool on = false;
  std::vector<ProfRec> pending;
  std::vector<hipEvent_t> pool; // drained events, reused (hipEventCreate is not free)
  std::map<std::string, std::pair<double, uint64_t>> acc;
  void drain() {
    for (auto &r : pending) {
      float ms = 0;
      if (hipEventSynchronize(r.b) == hipSuccess && hipEventElapsedTime(&ms, r.a, r.b) == hipSuccess) {
        auto &e = acc[r.name];
        e.first += ms;
        e.second += 1;
      }
      pool.push_back(r.a);
      pool.push_back(r.b);
    }
    pending.clear();
  }
} g_prof;

bool prof_on() { return g_prof.on; }
hipEvent_t prof_event() {
  {
    std::lock_guard<std::mutex> g(g_prof.mu);
    if (!g_prof.pool.empty()) {
      hipEvent_t e = g_prof.pool.back();
      g_prof.pool.pop_back();
      return e;
    }
  }
  hipEvent_t e = nullptr;
  return hipEventCreate(&e) == hipSuccess ? e : nullptr;
}
void prof_push(const char *name, hipEvent_t a, hipEvent_t b) {
  std::lock_guard<std::mutex> g(g_prof.mu);
  g_prof.pending.push_back({name, a, b});
}

// ------------------------------------------------------------------ tables ----
int cb_index(uint32_t K) {
  for (int i = 0; i < SRSGPU_NOF_CB_SIZES; i++)
    if (srsgpu_qpp_table[i][0] == K) return i;
  return -1;
}

// turbodecoder.c:364-376 (AVX2 build)
uint32_t auto_subblocks(uint32_t K) {
  if (!(K % 16) && K > 800) return 16;
  if (!(K % 8) && K > 400) return 8;
  return 0;
}

// impl actually run for (impl, K): turbodecoder.c:153-291, 467-489
// turbodecoder.c:392-423 (AVX2 build): the int8 window decoders where K allows them, else the
// 16-bit AUTO choice on the sign-extended input (tdec_iteration_8, :439-464)
uint32_t auto_subblocks_8bit(uint32_t K) {
  if (!(K % 32) && K > 2048) return 32;
  if (!(K % 16) && K > 800) return 16;
  if (!(K % 8) && K > 400) return 8;
  return 0;
}

int resolve_impl(int impl, uint32_t K) {
  if (impl == SRSGPU_TDEC_AUTO_8BIT) {
    const uint32_t s = auto_subblocks_8bit(K);
    if (s == 32) return SRSLTE_TDEC_AVX8_WINDOW;
    if (s == 16) return SRSLTE_TDEC_SSE8_WINDOW;
    impl = SRSLTE_TDEC_AUTO;
  }
  if (impl == SRSLTE_TDEC_AUTO) {
    uint32_t nsb = auto_subblocks(K);
    return nsb == 16 ? SRSLTE_TDEC_AVX_WINDOW : nsb == 8 ? SRSLTE_TDEC_SSE_WINDOW : SRSLTE_TDEC_SSE;
  }
  return impl;
}
int impl_nb(int r) {
  switch (r) {
  case SRSLTE_TDEC_AVX8_WINDOW: return 32;
  case SRSLTE_TDEC_AVX_WINDOW:
  case SRSLTE_TDEC_SSE8_WINDOW: return 16;
  case SRSLTE_TDEC_SSE_WINDOW: return 8;
  default: return 1;
  }
}

// turbodecoder_iter.h:31-47,91-108: the 16-bit decoders read sub-block input only when chosen by
// AUTO (input_is_interleaved = current_dec > 0); the int8 ones always (input_is_interleaved 1)
bool sb_input_for(int impl, int r) {
  if (impl_nb(r) <= 1) return false;
  return impl == SRSLTE_TDEC_AUTO || impl == SRSGPU_TDEC_AUTO_8BIT || r == SRSLTE_TDEC_SSE8_WINDOW ||
         r == SRSLTE_TDEC_AVX8_WINDOW;
}

// QPP interleaver (TS 36.212 5.1.3.2.3) in the decoder's index space: natural for nb == 1, the
// sub-block index k*nb+d <-> natural d*(K/nb)+k otherwise (tc_interl_lte.c:78-119).
void gen_interleaver(uint32_t K, uint32_t nb, std::vector<uint16_t> &fwd, std::vector<uint16_t> &rev) {
  int idx = cb_index(K);
  uint64_t f1 = srsgpu_qpp_table[idx][1], f2 = srsgpu_qpp_table[idx][2];
  std::vector<uint32_t> pi(K);
  for (uint64_t i = 0; i < K; i++) pi[i] = (uint32_t)((f1 * i + f2 * i * i) % K);
  fwd.assign(K, 0);
  rev.assign(K, 0);
  const uint32_t L = nb > 1 ? K / nb : K;
  auto to_idx = [&](uint32_t p) { return nb > 1 ? (p % L) * nb + p / L : p; };
  for (uint32_t p = 0; p < K; p++) {
    uint32_t i = to_idx(p), j = to_idx(pi[p]);
    fwd[i] = (uint16_t)j; // app2[i] = ext1[fwd[i]]
    rev[j] = (uint16_t)i; // app1[j] = ext2[rev[j]]
  }
}

} // namespace srsgpu

using srsgpu::TdecEngine;
using srsgpu::g_prof;
using srsgpu::auto_subblocks;
using srsgpu::cb_index;
using srsgpu::impl_nb;
using srsgpu::resolve_impl;
using srsgpu::sb_input_for;
typedef TdecEngine Engine;

struct srsgpu_tdec_batch {
  Engine e;
};

extern "C" {

void srsgpu_knobs_reload(void) { srsgpu::knobs_slot().store(srsgpu::knobs_from_env(), std::memory_order_release); }

uint32_t srsgpu_tdec_input_len(int impl, int sb_layout, uint32_t K) {
  const int sb = sb_layout && sb_input_for(impl, resolve_impl(impl, K));
  return sb ? 3 * (K + 32) + 12 : 3 * K + 12;
}

int srsgpu_tdec_batch_create(srsgpu_tdec_batch_t **q, uint32_t max_cbs, uint32_t max_long_cb) {
  if (!q) return -1;
  auto *b = new srsgpu_tdec_batch();
  if (b->e.create(max_cbs, max_long_cb)) {
    b->e.destroy();
    delete b;
    *q = nullptr;
    return -1;
  }
  *q = b;
  return 0;
}

void srsgpu_tdec_batch_destroy(srsgpu_tdec_batch_t *q) {
  if (!q) return;
  (void)hipStreamSynchronize(q->e.st);
  q->e.destroy();
  delete q;
}

void srsgpu_tdec_batch_set_stream(srsgpu_tdec_batch_t *q, void *s) {
  if (q) q->e.st = (hipStream_t)s;
}

int srsgpu_tdec_batch_run_dev(srsgpu_tdec_batch_t *q, int impl, int sb_layout, const int16_t *d_in,
                              size_t in_stride, uint32_t K, uint32_t n, uint32_t nhalf, uint8_t *d_out,
                              size_t out_stride) {
  if (!q || !d_in || !d_out) return -1;
  if (out_stride < K / 8) return -1;
  return q->e.run(impl, sb_layout, d_in, in_stride, K, n, nhalf, d_out, out_stride);
}

int srsgpu_tdec_batch_decode_dev(srsgpu_tdec_batch_t *q, int impl, int sb_layout, const int16_t *d_in,
                                 size_t in_stride, uint32_t K, uint32_t n, uint32_t maxh, uint32_t poly,
                                 uint32_t crc_len, uint8_t *d_out, size_t out_stride, uint8_t *d_ok,
                                 uint32_t *d_noi) {
  if (!q || !d_in || !d_out) return -1;
  if (out_stride < K / 8) return -1;
  return q->e.decode(impl, sb_layout, d_in, in_stride, K, n, maxh, poly, crc_len, d_out, out_stride, d_ok,
                     d_noi);
}

int srsgpu_tdec_batch_read_state(srsgpu_tdec_batch_t *q, uint32_t cb, int16_t *app1, int16_t *ext1) {
  if (!q || !app1 || !ext1) return -1;
  return q->e.read_state(cb, app1, ext1);
}

static int host_stage_in(Engine &e, int impl, int sb_layout, const int16_t *const *input, uint32_t K,
                         uint32_t n, size_t *stride) {
  if (n > e.cap_cbs || K > e.cap_K || cb_index(K) < 0) {
    fprintf(stderr, "srsgpu: batch of %u x K=%u exceeds capacity or invalid K\n", n, K);
    return -1;
  }
  const size_t len = srsgpu_tdec_input_len(impl, sb_layout, K);
  *stride = 3 * (e.cap_K + 32) + 12;
  if (e.stage(n, K, len)) return -1;
  for (uint32_t i = 0; i < n; i++) {
    if (!input[i]) return -1;
    HIPCHK(hipMemcpyAsync(e.in_stage + i * *stride, input[i], len * 2, hipMemcpyHostToDevice, e.st));
  }
  return 0;
}

int srsgpu_tdec_batch_run(srsgpu_tdec_batch_t *q, int impl, int sb_layout, const int16_t *const *input,
                          uint32_t K, uint32_t n, uint32_t nhalf, uint8_t *const *output) {
  if (!q || !input || !output) return -1;
  Engine &e = q->e;
  size_t stride;
  if (host_stage_in(e, impl, sb_layout, input, K, n, &stride)) return -1;
  if (e.run(impl, sb_layout, e.in_stage, stride, K, n, nhalf, e.out_stage, K / 8)) return -1;
  for (uint32_t i = 0; i < n; i++)
    HIPCHK(hipMemcpyAsync(output[i], e.out_stage + (size_t)i * (K / 8), K / 8, hipMemcpyDeviceToHost, e.st));
  HIPCHK(hipStreamSynchronize(e.st));
  return 0;
}

int srsgpu_tdec_batch_decode(srsgpu_tdec_batch_t *q, int impl, int sb_layout, const int16_t *const *input,
                             uint32_t K, uint32_t n, uint32_t maxh, uint32_t poly, uint32_t crc_len,
                             uint8_t *const *output, uint8_t *crc_ok, uint32_t *noi) {
  if (!q || !input || !output) return -1;
  Engine &e = q->e;
  size_t stride;
  if (host_stage_in(e, impl, sb_layout, input, K, n, &stride)) return -1;
  if (e.decode(impl, sb_layout, e.in_stage, stride, K, n, maxh, poly, crc_len, e.out_stage, K / 8, nullptr,
               nullptr))
    return -1;
  for (uint32_t i = 0; i < n; i++)
    HIPCHK(hipMemcpyAsync(output[i], e.out_stage + (size_t)i * (K / 8), K / 8, hipMemcpyDeviceToHost, e.st));
  if (crc_ok) HIPCHK(hipMemcpyAsync(crc_ok, e.cb_ok, n, hipMemcpyDeviceToHost, e.st));
  if (noi) HIPCHK(hipMemcpyAsync(noi, e.noi, (size_t)n * 4, hipMemcpyDeviceToHost, e.st));
  HIPCHK(hipStreamSynchronize(e.st));
  return 0;
}

int srsgpu_tdec_set_schedule(int fused, int es_fused, int es_chunk, int sse_bidir) {
  if (es_chunk == 0 || es_fused > 3) return -1;
  srsgpu::TdSched &t = srsgpu::td_sched();
  if (fused >= 0) t.fused = fused != 0;
  if (es_fused >= 0) t.es_fused = es_fused;
  if (es_chunk > 0) t.es_chunk = es_chunk;
  if (sse_bidir >= 0) t.sse_bidir = sse_bidir != 0;
  return 0;
}

void srsgpu_tdec_get_schedule(int *fused, int *es_fused, int *es_chunk, int *sse_bidir) {
  const srsgpu::TdSched &t = srsgpu::td_sched();
  if (fused) *fused = t.fused;
  if (es_fused) *es_fused = t.es_fused;
  if (es_chunk) *es_chunk = t.es_chunk;
  if (sse_bidir) *sse_bidir = t.sse_bidir;
}

void srsgpu_prof_enable(int on) {
  std::lock_guard<std::mutex> g(g_prof.mu);
  g_prof.on = on != 0;
}

void srsgpu_prof_reset(void) {
  std::lock_guard<std::mutex> g(g_prof.mu);
  g_prof.drain();
  g_prof.acc.clear();
}

int srsgpu_prof_get(const char *name, double *total_ms, uint64_t *count) {
  std::lock_guard<std::mutex> g(g_prof.mu);
  g_prof.drain();
  double t = 0;
  uint64_t c = 0;
  for (auto &kv : g_prof.acc) {
    if (!name || kv.first.find(name) != std::string::npos) {
      t += kv.second.first;
      c += kv.second.second;
    }
  }
  if (total_ms) *total_ms = t;
  if (count) *count = c;
  return 0;
}

// ------------------------------------------------------------------ drop-in srslte_tdec_* ----
// Reference: lib/src/phy/fec/turbodecoder.c:133-564. One engine (capacity one CB) per object;
// srslte_tdec_iteration keeps the one-half-iteration-per-call protocol.

struct TdecGpu {
  Engine e;
  std::vector<int16_t> conv; // int8 <-> int16 input conversion (the 8-bit entry points)
  int16_t *d_in = nullptr;
  uint8_t *d_out = nullptr;
  size_t in_len = 0;
  // decision bytes written by the half-iteration's own launch (k_win_spread) into mapped, coherent
  // host memory: no k_decide launch and no copy per srslte_tdec_iteration call (null: not available)
  uint8_t *h_out = nullptr, *dh_out = nullptr;
  size_t flag_off = 0; // the launch's completion word in the same buffer (polled, SRSGPU_SPREAD_POLL)
  uint32_t seq = 0;
};

int srslte_tdec_init(srslte_tdec_t *h, uint32_t max_long_cb) {
  return srslte_tdec_init_manual(h, max_long_cb, SRSLTE_TDEC_AUTO);
}

int srslte_tdec_init_manual(srslte_tdec_t *h, uint32_t max_long_cb, srslte_tdec_impl_type_t dec_type) {
  if (!h) return -1;
  memset(h, 0, sizeof(*h));
  if (dec_type > SRSLTE_TDEC_AVX8_WINDOW) {
    fprintf(stderr, "Error decoder %d not supported\n", (int)dec_type);
    return -1;
  }
  auto *g = new TdecGpu();
  if (g->e.create(1, max_long_cb ? max_long_cb : 1)) {
    g->e.destroy();
    delete g;
    return -1;
  }
  // a stream of its own (non-blocking): null-stream launches carry HIP's implicit cross-stream
  // synchronisation
  if (hipMalloc(&g->d_in, (3 * (max_long_cb + 32) + 12) * 2) != hipSuccess ||
      hipMalloc(&g->d_out, max_long_cb / 8 + 1) != hipSuccess ||
      hipStreamCreateWithFlags(&g->e.st, hipStreamNonBlocking) != hipSuccess) {
    fprintf(stderr, "srsgpu: device allocation failed\n");
    if (g->d_in) (void)hipFree(g->d_in);
    if (g->d_out) (void)hipFree(g->d_out);
    g->e.st = nullptr;
    g->e.destroy();
    delete g;
    return -1;
  }
  g->flag_off = (max_long_cb / 8 + 15) & ~(size_t)15;
  if (hipHostMalloc((void **)&g->h_out, g->flag_off + 16, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer((void **)&g->dh_out, g->h_out, 0) != hipSuccess) {
    if (g->h_out) (void)hipHostFree(g->h_out);
    g->h_out = g->dh_out = nullptr; // the k_decide + copy path
  }
  h->gpu = g;
  h->max_long_cb = max_long_cb;
  h->dec_type = dec_type;
  h->current_cbidx = -1;
  return 0;
}

void srslte_tdec_free(srslte_tdec_t *h) {
  if (!h) return;
  auto *g = (TdecGpu *)h->gpu;
  if (g) {
    (void)hipStreamSynchronize(g->e.st);
    if (g->d_in) (void)hipFree(g->d_in);
    if (g->d_out) (void)hipFree(g->d_out);
    if (g->h_out) (void)hipHostFree(g->h_out);
    g->e.destroy();
    if (g->e.st) (void)hipStreamDestroy(g->e.st);
    delete g;
  }
  memset(h, 0, sizeof(*h));
}

void srslte_tdec_force_not_sb(srslte_tdec_t *h) {
  if (h) h->force_not_sb = true;
}

int srslte_tdec_new_cb(srslte_tdec_t *h, uint32_t long_cb) {
  if (long_cb > h->max_long_cb) {
    fprintf(stderr, "TDEC was initialized for max_long_cb=%d\n", h->max_long_cb);
    return -1;
  }
  h->n_iter = 0;
  h->current_long_cb = long_cb;
  h->current_cbidx = cb_index(long_cb);
  if (h->current_cbidx < 0) {
    fprintf(stderr, "Invalid CB length %d\n", long_cb);
    return -1;
  }
  return 0;
}

int srslte_tdec_get_nof_iterations(srslte_tdec_t *h) { return h->n_iter; }

uint32_t srslte_tdec_autoimp_get_subblocks(uint32_t long_cb) { return auto_subblocks(long_cb); }

// turbodecoder.c:392-406 (AVX2 build)
uint32_t srslte_tdec_autoimp_get_subblocks_8bit(uint32_t long_cb) { return srsgpu::auto_subblocks_8bit(long_cb); }

// at the first half-iteration of a code block the (int16) input of decoder `impl` is uploaded and loaded
static int tdec_gpu_upload(srslte_tdec_t *h, const int16_t *input, int impl) {
  auto *g = (TdecGpu *)h->gpu;
  Engine &e = g->e;
  const uint32_t K = h->current_long_cb;
  const int sb = !h->force_not_sb;
  if (h->n_iter == 0) {
    const size_t len = srsgpu_tdec_input_len(impl, sb, K);
    HIPCHK(hipMemcpyAsync(g->d_in, input, len * 2, hipMemcpyHostToDevice, e.st));
    if (e.load(impl, sb, g->d_in, len, K, 1)) return -1;
  }
  return 0;
}

// one half-iteration
static int tdec_gpu_halfit(srslte_tdec_t *h, const int16_t *input, int impl) {
  if (tdec_gpu_upload(h, input, impl)) return -1;
  if (((TdecGpu *)h->gpu)->e.halfit(h->n_iter, false)) return -1;
  h->n_iter++;
  return 0;
}

static int tdec_gpu_decide(srslte_tdec_t *h, uint8_t *output) {
  auto *g = (TdecGpu *)h->gpu;
  Engine &e = g->e;
  const uint32_t K = h->current_long_cb;
  if (e.decide(h->n_iter - 1, g->d_out, K / 8, false)) return -1;
  HIPCHK(hipMemcpyAsync(output, g->d_out, K / 8, hipMemcpyDeviceToHost, e.st));
  HIPCHK(hipStreamSynchronize(e.st));
  return 0;
}

// one half-iteration and its decision bytes (the srslte_tdec_iteration protocol): one k_win_spread
// launch that also writes the bytes into the handle's mapped host buffer when the block allows it
// (windowed kind, K / nb a multiple of 16), else the half-iteration, k_decide and a copy
static int tdec_gpu_step(srslte_tdec_t *h, const int16_t *input, int impl, uint8_t *output) {
  auto *g = (TdecGpu *)h->gpu;
  Engine &e = g->e;
  const uint32_t K = h->current_long_cb;
  if (tdec_gpu_upload(h, input, impl)) return -1;
  const bool poll = srsgpu::knobs().spread_poll;
  const uint32_t seq = ++g->seq ? g->seq : ++g->seq; // never 0
  volatile uint32_t *hflag = (volatile uint32_t *)(g->h_out + g->flag_off);
  const int r = g->dh_out ? e.halfit_bytes(h->n_iter, g->dh_out, K / 8,
                                           poll ? (uint32_t *)(g->dh_out + g->flag_off) : nullptr, seq)
                          : 1;
  if (r < 0) return -1;
  if (r == 1) {
    if (e.halfit(h->n_iter, false)) return -1;
    h->n_iter++;
    return tdec_gpu_decide(h, output);
  }
  h->n_iter++;
  bool seen = false;
  if (poll) { // the launch stores seq after the bytes (system-scope release); bounded spin, then the stream
    const auto t0 = std::chrono::steady_clock::now();
    while (!(seen = __atomic_load_n(hflag, __ATOMIC_ACQUIRE) == seq) &&
           std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(20)) {
    }
  }
  if (!seen) HIPCHK(hipStreamSynchronize(e.st));
  memcpy(output, g->h_out, K / 8);
  return 0;
}

static bool is_int8_type(int t) { return t == SRSLTE_TDEC_SSE8_WINDOW || t == SRSLTE_TDEC_AVX8_WINDOW; }

// 16-bit entry with a manual int8 window type (tdec_iteration_16, turbodecoder.c:491-503): the
// input is truncated to int8 (convert_16_to_8); natural layout only — with sub-block input the
// reference converts 3K+12 values of a 3(K+32)+12 layout
static const int16_t *tdec_input16(srslte_tdec_t *h, int16_t *input) {
  if (!is_int8_type(h->dec_type)) return input;
  auto *g = (TdecGpu *)h->gpu;
  if (!h->force_not_sb) {
    fprintf(stderr, "srsgpu: int8 decoder type %d with 16-bit sub-block input is not defined by the "
                    "reference (use srslte_tdec_force_not_sb)\n", (int)h->dec_type);
    return nullptr;
  }
  const size_t n = 3 * (size_t)h->current_long_cb + 12;
  g->conv.resize(n);
  for (size_t i = 0; i < n; i++) g->conv[i] = (int8_t)input[i];
  return g->conv.data();
}

// 8-bit entry (tdec_iteration_8, turbodecoder.c:439-464): int8 values sign-extended into the
// engine's int16 lanes; AUTO becomes the 8-bit AUTO choice
// Converted once per code block, like the reference (turbodecoder.c:458): the input is only
// uploaded by the first half-iteration, later calls just resolve the implementation.
static const int16_t *tdec_input8(srslte_tdec_t *h, const int8_t *input, int *impl) {
  auto *g = (TdecGpu *)h->gpu;
  *impl = h->dec_type == SRSLTE_TDEC_AUTO ? SRSGPU_TDEC_AUTO_8BIT : (int)h->dec_type;
  if (h->n_iter != 0) return g->conv.data();
  const size_t n = srsgpu_tdec_input_len(*impl, !h->force_not_sb, h->current_long_cb);
  g->conv.resize(n);
  for (size_t i = 0; i < n; i++) g->conv[i] = input[i];
  return g->conv.data();
}

void srslte_tdec_iteration(srslte_tdec_t *h, int16_t *input, uint8_t *output) {
  if (h && h->gpu && h->current_cbidx >= 0) {
    const int16_t *in = h->n_iter == 0 ? tdec_input16(h, input) : input;
    if (!in) return;
    (void)tdec_gpu_step(h, in, h->dec_type, output);
  }
}

int srslte_tdec_run_all(srslte_tdec_t *h, int16_t *input, uint8_t *output, uint32_t nof_iterations,
                        uint32_t long_cb) {
  if (!h || !h->gpu) return -1;
  if (srslte_tdec_new_cb(h, long_cb)) return -1;
  const int16_t *in = tdec_input16(h, input);
  if (!in) return -1;
  do {
    if (tdec_gpu_halfit(h, in, h->dec_type)) return -1;
  } while (h->n_iter < (int)nof_iterations);
  return tdec_gpu_decide(h, output);
}

void srslte_tdec_iteration_8bit(srslte_tdec_t *h, int8_t *input, uint8_t *output) {
  if (h && h->gpu && h->current_cbidx >= 0) {
    int impl = 0;
    const int16_t *in = tdec_input8(h, input, &impl);
    (void)tdec_gpu_step(h, in, impl, output);
  }
}

int srslte_tdec_run_all_8bit(srslte_tdec_t *h, int8_t *input, uint8_t *output, uint32_t nof_iterations,
                             uint32_t long_cb) {
  if (!h || !h->gpu) return -1;
  if (srslte_tdec_new_cb(h, long_cb)) return -1;
  int impl = 0;
  const int16_t *in = tdec_input8(h, input, &impl);
  do {
    if (tdec_gpu_halfit(h, in, impl)) return -1;
  } while (h->n_iter < (int)nof_iterations);
  return tdec_gpu_decide(h, output);
}

} // extern "C"
