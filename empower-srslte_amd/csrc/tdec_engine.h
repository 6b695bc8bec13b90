// Turbo-decoder engine shared by the batch C ABI (tdec_engine.hip) and the DL-SCH engine
// (dlsch_engine.hip): device buffers, half-iteration schedule, early stop.
#ifndef SRSGPU_TDEC_ENGINE_H
#define SRSGPU_TDEC_ENGINE_H
#include <hip/hip_runtime.h>

#include <algorithm>
#include <map>
#include <tuple>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <utility>
#include <vector>

#include "srsgpu/qpp_table.h"
#include "wave_prio.h"
#include "srsgpu/tdec_batch.h"
#include "srslte/phy/fec/turbodecoder.h"
#include "tdec_kernels.h"
#include "host_ring.h"
#include "dlsch_kernels.h"

#define HIPCHK(x)                                                                               \
  do {                                                                                            \
    hipError_t e_ = (x);                                                                          \
    if (e_ != hipSuccess) {                                                                       \
      fprintf(stderr, "srsgpu: %s failed: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__,      \
              __LINE__);                                                                          \
      return -1;                                                                                  \
    }                                                                                             \
  } while (0)

namespace srsgpu {

// live kernel timing (srsgpu_prof_*)
bool prof_on();
hipEvent_t prof_event(); // from a pool of drained events
void prof_push(const char *name, hipEvent_t a, hipEvent_t b);
struct ProfScope {
  hipEvent_t a = nullptr, b = nullptr;
  const char *name;
  hipStream_t st;
  ProfScope(const char *n, hipStream_t s) : name(n), st(s) {
    if (prof_on()) {
      a = prof_event();
      b = prof_event();
      if (a && b) (void)hipEventRecord(a, st);
    }
  }
  ~ProfScope() {
    if (a && b) {
      (void)hipEventRecord(b, st);
      prof_push(name, a, b);
    }
  }
};

int cb_index(uint32_t K);
uint32_t auto_subblocks(uint32_t K);
uint32_t auto_subblocks_8bit(uint32_t K);
int resolve_impl(int impl, uint32_t K);
int impl_nb(int r);
bool sb_input_for(int impl, int r); // does the decoder read rm_turbo's sub-block layout
void gen_interleaver(uint32_t K, uint32_t nb, std::vector<uint16_t> &fwd, std::vector<uint16_t> &rev);

// ------------------------------------------------------------------ engine ----
// A job = code blocks of one or many sizes. TdSpec lists them in the caller's numbering: spec i
// holds n code blocks of size K numbered cb0 .. cb0+n-1 (input rows, outputs and per-CB flags use
// that number) and the CRC its early stop checks. The engine turns the specs into device groups
// (tdec_kernels.h), ordered by decoder variant, and runs every half-iteration as one launch per
// variant plus one decide launch, whatever the number of distinct sizes.
struct TdSpec {
  uint32_t K, n, poly, crc_len, cb0;
};

struct TdecEngine {
  hipStream_t st = nullptr;
  uint32_t cap_cbs = 0, cap_K = 0;
  size_t cap_pairs = 0, cap_elems = 0, cap_dw = 0, cap_sc = 0;
  // concatenated per-group arrays: SP0 short4; XP1 = X2, P1 short2 planes of cap_elems; A short2;
  // T short2 [pairs][12]; D packed decisions; scratch (sequential decoders)
  void *SP0 = nullptr, *XP1 = nullptr, *A = nullptr, *T = nullptr, *D = nullptr, *scratch = nullptr;
  uint32_t *Dfz = nullptr; // frozen decision words of the fused early stop (TdEs::dfz)
  uint8_t *cb_end = nullptr; // TdEs::cb_end, zero between jobs
  // the hybrid schedule's list of pairs still running after the first half-iteration (TdEs::run_list;
  // run_cnt per group at its pair0, zeroed by k_pair_done). SRSGPU_ES_COMPACT=0: every pair (A/B)
  uint32_t *run_list = nullptr, *run_cnt = nullptr;
  uint32_t *spread_cnt = nullptr; // k_win_spread's per-pair workgroup arrival counters (zero between launches)
  uint8_t *cb_done = nullptr, *pair_done = nullptr, *cb_ok = nullptr;
  uint32_t *noi = nullptr;
  int16_t *in_stage = nullptr; // host-pointer API staging
  uint8_t *out_stage = nullptr;
  struct Interl {
    uint16_t *fwd, *rev, *dmap;
  };
  std::map<std::pair<uint32_t, uint32_t>, Interl> interl;
  std::map<uint32_t, uint32_t *> crc_tables; // poly -> x^(d+24) mod P, d < 6144 (k_decide)
  // (K, nb, poly, crc_len) -> chain-major CRC weights after DEC1 and DEC2 (TdGroup::wc)
  std::map<std::tuple<uint32_t, uint32_t, uint32_t, uint32_t>, std::pair<uint32_t *, uint32_t *>> wc_tables;
  // current job (one pass)
  std::vector<TdGroup> groups; // kind order
  TdGroup *d_groups = nullptr;
  // pinned staging of the group table: a ring, so a call does not wait for the previous call's upload
  // (which sits on the stream behind that call's earlier kernels: the host would run in lockstep with
  // the device); last_up is what d_groups holds after the last upload
  HostRing gring;
  std::vector<TdGroup> last_up;
  size_t groups_cap = 0, uploaded = 0;
  // second stream of the fused early stop: the SSE kind beside the window kinds
  hipStream_t aux = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  // tail stream (srsgpu_dlsch_set_tail_stream): under the hybrid early-stop schedule, everything after
  // the first half-iteration moves to split_st (st is switched for the rest of the call)
  hipStream_t split_st = nullptr;
  hipEvent_t ev_split = nullptr;
  // defer_bytes (the DL-SCH engine's request): the natural-order bytes of the blocks a fused early-stop
  // launch ended are left in Dfz / cb_end for the caller's epilogue (k_tb_finish, FzSrc) instead of a
  // k_es_bytes launch; only for a job decoded in one pass (the group table and Dfz stay as they are).
  // bytes_deferred tells the caller, after decode_multi, that it did so.
  bool defer_bytes = false, defer_now = false, bytes_deferred = false;
  int kind_g0[TD_NKIND + 1] = {0};
  int kind_blocks[TD_NKIND] = {0};
  size_t kind_lds[TD_NKIND] = {0};
  int total_pairs = 0;
  static int num_cus() {
    static const int n = [] {
      int dev = 0, v = 0;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
        return 256;
      return v;
    }();
    return n;
  }
  // K and interleaver of the last single-size job (the drop-in srslte_tdec_* path)
  uint32_t K = 0;
  const uint16_t *fwd = nullptr, *rev = nullptr, *dmap = nullptr;

  static constexpr size_t EXTRA_PAIRS = 256; // odd groups each add half a pair

  int create(uint32_t max_cbs, uint32_t max_K) {
    if (max_cbs == 0 || max_K == 0 || max_K > SRSLTE_TCOD_MAX_LEN_CB) {
      fprintf(stderr, "srsgpu: invalid batch capacity %u x %u\n", max_cbs, max_K);
      return -1;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
      fprintf(stderr, "srsgpu: no HIP device available\n");
      return -1;
    }
    cap_cbs = max_cbs;
    cap_K = max_K;
    cap_pairs = (max_cbs + 1) / 2 + EXTRA_PAIRS;
    // T4 regions pad a pair's K elements by at most 3 * 32 (t4_pair_elems)
    cap_elems = (size_t)((max_cbs + 1) / 2) * (max_K + 96) + EXTRA_PAIRS * (std::min<uint32_t>(max_K, 1024) + 96);
    cap_dw = cap_elems / 16 + cap_pairs * 16;
    cap_sc = (cap_elems + 4 * cap_pairs) * 8;
    HIPCHK(hipMalloc(&SP0, cap_elems * 8));
    HIPCHK(hipMalloc(&XP1, cap_elems * 8));
    HIPCHK(hipMalloc(&A, cap_elems * 4));
    HIPCHK(hipMalloc(&D, cap_dw * 4));
    HIPCHK(hipMalloc(&T, cap_pairs * 12 * 4));
    HIPCHK(hipMalloc(&scratch, cap_sc * 4));
    HIPCHK(hipMalloc(&cb_done, cap_cbs));
    HIPCHK(hipMalloc(&cb_ok, cap_cbs));
    HIPCHK(hipMalloc(&pair_done, cap_pairs));
    HIPCHK(hipMalloc(&noi, (size_t)cap_cbs * 4));
    HIPCHK(hipMalloc(&Dfz, cap_dw * 4));
    HIPCHK(hipMalloc(&cb_end, cap_cbs));
    HIPCHK(hipMemset(cb_end, 0, cap_cbs));
    HIPCHK(hipMalloc(&run_list, cap_pairs * 4));
    HIPCHK(hipMalloc(&run_cnt, cap_pairs * 4));
    HIPCHK(hipMemset(run_cnt, 0, cap_pairs * 4));
    HIPCHK(hipMalloc(&spread_cnt, (size_t)spread_max_pairs() * 4));
    HIPCHK(hipMemset(spread_cnt, 0, (size_t)spread_max_pairs() * 4));
    return 0;
  }

  void destroy() {
    gring.destroy();
    for (void *p : {SP0, XP1, A, D, T, scratch, (void *)d_groups})
      if (p) (void)hipFree(p);
    for (void *p : {(void *)cb_done, (void *)cb_ok, (void *)pair_done, (void *)noi, (void *)in_stage,
                    (void *)out_stage, (void *)Dfz, (void *)cb_end, (void *)run_list, (void *)run_cnt,
                    (void *)spread_cnt})
      if (p) (void)hipFree(p);
    if (aux) (void)hipStreamSynchronize(aux);
    for (hipEvent_t e : {ev_fork, ev_join, ev_split})
      if (e) (void)hipEventDestroy(e);
    if (aux) (void)hipStreamDestroy(aux);
    for (auto &kv : crc_tables) (void)hipFree(kv.second);
    crc_tables.clear();
    for (auto &kv : wc_tables) {
      (void)hipFree(kv.second.first);
      (void)hipFree(kv.second.second);
    }
    wc_tables.clear();
    for (auto &kv : interl)
      for (uint16_t *p : {kv.second.fwd, kv.second.rev, kv.second.dmap}) (void)hipFree(p);
    interl.clear();
  }

  TdArrays arrays() const { return TdArrays{SP0, XP1, A, D, T, scratch, cap_elems}; }

  const Interl *get_interleaver(uint32_t Kv, uint32_t nbv) {
    auto key = std::make_pair(Kv, nbv);
    auto it = interl.find(key);
    if (it == interl.end()) {
      std::vector<uint16_t> f, r, m(Kv);
      gen_interleaver(Kv, nbv, f, r);
      // dmap[p]: natural position p -> SB index j -> interleaved index i = rev[j], which DEC2
      // decodes as step i / NB of chain i % NB: chain-major decision index (k_decide)
      const uint32_t L = Kv / nbv, G16 = (L + 15) / 16;
      for (uint32_t p = 0; p < Kv; p++) {
        const uint32_t j = nbv > 1 ? (p % L) * nbv + p / L : p;
        const uint32_t i = r[j];
        m[p] = (uint16_t)((i % nbv) * 16 * G16 + i / nbv);
      }
      // device scatter tables: T16 layout, sub-block-index valued (tdec_kernels.h)
      const uint32_t nt = (uint32_t)t16_table_elems((int)Kv, (int)nbv);
      std::vector<uint16_t> f16(nt, 0), r16(nt, 0);
      for (uint32_t d = 0; d < nbv; d++)
        for (uint32_t k = 0; k < L; k++) {
          const uint32_t e = ((k / 16) * nbv + d) * 16 + k % 16, i = k * nbv + d;
          f16[e] = f[i];
          r16[e] = r[i];
        }
      Interl t{};
      if (hipMalloc(&t.fwd, nt * 2) != hipSuccess || hipMalloc(&t.rev, nt * 2) != hipSuccess ||
          hipMalloc(&t.dmap, Kv * 2) != hipSuccess)
        return nullptr;
      if (hipMemcpy(t.fwd, f16.data(), nt * 2, hipMemcpyHostToDevice) != hipSuccess ||
          hipMemcpy(t.rev, r16.data(), nt * 2, hipMemcpyHostToDevice) != hipSuccess ||
          hipMemcpy(t.dmap, m.data(), Kv * 2, hipMemcpyHostToDevice) != hipSuccess)
        return nullptr;
      it = interl.emplace(key, t).first;
    }
    return &it->second;
  }

  const uint32_t *crc_table(uint32_t poly) {
    auto it = crc_tables.find(poly);
    if (it != crc_tables.end()) return it->second;
    std::vector<uint32_t> t(6144);
    uint32_t r = 1u << 23; // x^23; one shift below gives x^24 mod P
    for (int d = 0; d < 6144; d++) {
      const uint32_t top = r & 0x800000u;
      r = (r << 1) & 0xFFFFFFu;
      if (top) r ^= poly & 0xFFFFFFu;
      t[d] = r; // x^(d + 24) mod P
    }
    uint32_t *dt = nullptr;
    if (hipMalloc(&dt, t.size() * 4) != hipSuccess) return nullptr;
    if (hipMemcpy(dt, t.data(), t.size() * 4, hipMemcpyHostToDevice) != hipSuccess) return nullptr;
    crc_tables.emplace(poly, dt);
    return dt;
  }

  // CRC weight per decision bit in chain-major order (k_decide folds the CRC over the decoder's
  // decision words directly): after DEC1 natural position p = d L + k sits at d*16*G16 + k; after
  // DEC2 at dmap[p]
  int wc_table(uint32_t Kv, uint32_t nbv, uint32_t poly, uint32_t crc_len, const Interl *il,
               const uint32_t *w[2]) {
    const auto key = std::make_tuple(Kv, nbv, poly, crc_len);
    auto it = wc_tables.find(key);
    if (it == wc_tables.end()) {
      std::vector<uint32_t> pw(6144);
      uint32_t r = 1u << 23;
      for (int d = 0; d < 6144; d++) {
        const uint32_t top = r & 0x800000u;
        r = (r << 1) & 0xFFFFFFu;
        if (top) r ^= poly & 0xFFFFFFu;
        pw[d] = r;
      }
      const uint32_t L = Kv / nbv, G16 = (L + 15) / 16, n = nbv * G16 * 16;
      std::vector<uint16_t> dm(Kv);
      if (hipMemcpy(dm.data(), il->dmap, Kv * 2, hipMemcpyDeviceToHost) != hipSuccess) return -1;
      std::vector<uint32_t> w1(n, 0), w2(n, 0);
      for (uint32_t p = 0; p < Kv && p < crc_len; p++) {
        const uint32_t v = pw[crc_len - 1 - p];
        w1[(p / L) * 16 * G16 + p % L] = v;
        w2[dm[p]] = v;
      }
      uint32_t *d1 = nullptr, *d2 = nullptr;
      if (hipMalloc(&d1, n * 4) != hipSuccess || hipMalloc(&d2, n * 4) != hipSuccess) return -1;
      if (hipMemcpy(d1, w1.data(), n * 4, hipMemcpyHostToDevice) != hipSuccess ||
          hipMemcpy(d2, w2.data(), n * 4, hipMemcpyHostToDevice) != hipSuccess)
        return -1;
      it = wc_tables.emplace(key, std::make_pair(d1, d2)).first;
    }
    w[0] = it->second.first;
    w[1] = it->second.second;
    return 0;
  }

  static int kind_of(int r) {
    if (r == SRSLTE_TDEC_SSE8_WINDOW) return TD_KIND_B16;
    if (r == SRSLTE_TDEC_AVX8_WINDOW) return TD_KIND_B32;
    const int nbv = impl_nb(r);
    return nbv == 16 ? TD_KIND_W16 : nbv == 8 ? TD_KIND_W8 : r == SRSLTE_TDEC_SSE ? TD_KIND_SSE : TD_KIND_GEN;
  }

  int check_spec(int impl, uint32_t Kv, uint32_t n) {
    if (cb_index(Kv) < 0) {
      fprintf(stderr, "srsgpu: invalid code block size K=%u\n", Kv);
      return -1;
    }
    if (Kv > cap_K || n > cap_cbs || n == 0) {
      fprintf(stderr, "srsgpu: batch of %u x K=%u exceeds capacity %u x %u\n", n, Kv, cap_cbs, cap_K);
      return -1;
    }
    if ((impl < SRSLTE_TDEC_AUTO || impl > SRSLTE_TDEC_AVX8_WINDOW) && impl != SRSGPU_TDEC_AUTO_8BIT) {
      fprintf(stderr, "srsgpu: decoder type %d not supported\n", impl);
      return -1;
    }
    const int nbv = impl_nb(resolve_impl(impl, Kv));
    if (nbv > 1 && (Kv % nbv || Kv / nbv <= 40)) {
      // the reference windowed decoders need K/nb > win_overlap_len (turbodecoder_win.h:59);
      // at K/nb == 40 its estimation pass doubles as the final pass (:331, :469) — a manual-
      // mode-only corner (AUTO never selects it) that is rejected here
      fprintf(stderr, "srsgpu: K=%u not supported by the %d-sub-block window decoder\n", Kv, nbv);
      return -1;
    }
    return 0;
  }

  // Lay out specs[0..ns) as device groups. Returns 1 (nothing launched) if they do not fit.
  int plan(int impl, int sb_layout, const TdSpec *specs, size_t ns) {
    std::vector<size_t> order(ns);
    for (size_t i = 0; i < ns; i++) order[i] = i;
    std::vector<int> kind(ns);
    for (size_t i = 0; i < ns; i++) kind[i] = kind_of(resolve_impl(impl, specs[i].K));
    std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) {
      return std::make_pair(kind[a], specs[a].K) < std::make_pair(kind[b], specs[b].K);
    });
    groups.assign(ns, TdGroup{});
    size_t elems = 0, dw = 0, sc = 0;
    int pairs = 0;
    for (int k = 0; k <= TD_NKIND; k++) kind_g0[k] = (int)ns;
    for (int k = 0; k < TD_NKIND; k++) {
      kind_blocks[k] = 0;
      kind_lds[k] = 0;
    }
    for (size_t gi = 0; gi < ns; gi++) {
      const TdSpec &sp = specs[order[gi]];
      const int r = resolve_impl(impl, sp.K);
      const int nbv = impl_nb(r), kd = kind[order[gi]];
      if (kind_g0[kd] == (int)ns) kind_g0[kd] = (int)gi;
      TdGroup &g = groups[gi];
      g.K = (int)sp.K;
      g.nb = nbv;
      g.ncb = (int)sp.n;
      g.npairs = (int)((sp.n + 1) / 2);
      g.cb0 = (int)sp.cb0;
      g.pair0 = pairs;
      g.elem0 = (int64_t)elems;
      g.dw0 = (int64_t)dw;
      g.sc0 = (int64_t)sc;
      g.sb_input = sb_layout && sb_input_for(impl, r);
      if (sb_layout && impl == SRSGPU_TDEC_AUTO_8BIT && r == SRSLTE_TDEC_SSE_WINDOW) {
        // turbodecoder.c:457-460 converts 3K+12 int8 values but the SSE16 window decoder then
        // reads the sub-block layout's 3(K+32)+12: undefined in the reference
        fprintf(stderr, "srsgpu: 8-bit input in sub-block layout at K=%u (400 < K <= 800) is not "
                        "defined by the reference\n", sp.K);
        return -1;
      }
      g.blk_half = kind_blocks[kd];
      kind_blocks[kd] += halfit_blocks(nbv, g.npairs);
      if (nbv > 1) kind_lds[kd] = std::max(kind_lds[kd], bidir_lds_bytes(g.K, nbv));
      const Interl *it = get_interleaver(sp.K, (uint32_t)nbv);
      if (!it) return -1;
      g.fwd = it->fwd;
      g.rev = it->rev;
      g.dmap = it->dmap;
      g.crc_bytes = (int)(sp.crc_len / 8);
      g.crc_pw = nullptr;
      g.wc[0] = g.wc[1] = nullptr;
      if (g.crc_bytes) {
        g.crc_pw = crc_table(sp.poly);
        if (!g.crc_pw || wc_table(sp.K, (uint32_t)nbv, sp.poly, sp.crc_len, it, g.wc)) return -1;
      }
      pairs += g.npairs;
      elems += (size_t)g.npairs * t4_pair_elems(g.K, nbv);
      dw += (size_t)g.npairs * dec_words_host(g.K, nbv);
      if (nbv == 1) sc += seq_scratch_elems(g.K, g.npairs);
    }
    for (int k = TD_NKIND - 1; k >= 0; k--) kind_g0[k] = std::min(kind_g0[k], kind_g0[k + 1]);
    if ((size_t)pairs > cap_pairs || elems > cap_elems || dw > cap_dw || sc > cap_sc) return 1;
    total_pairs = pairs;
    return 0;
  }

  int upload_groups() {
    const size_t ng = groups.size();
    if (ng > groups_cap) {
      gring.destroy(); // waits for the uploads still reading it
      if (d_groups) {
        HIPCHK(hipStreamSynchronize(st)); // kernels of earlier calls may still read the old table
        HIPCHK(hipFree(d_groups));
      }
      groups_cap = std::max<size_t>(ng, 64);
      HIPCHK(hipMalloc(&d_groups, groups_cap * sizeof(TdGroup)));
      HIPCHK(gring.create(groups_cap * sizeof(TdGroup)));
      uploaded = 0;
    }
    if (uploaded == ng && memcmp(last_up.data(), groups.data(), ng * sizeof(TdGroup)) == 0) return 0;
    hipError_t re;
    TdGroup *h = (TdGroup *)gring.acquire(&re);
    HIPCHK(re);
    memcpy(h, groups.data(), ng * sizeof(TdGroup));
    HIPCHK(gring.upload(d_groups, h, ng * sizeof(TdGroup), st));
    HIPCHK(gring.mark(st));
    last_up.assign(groups.begin(), groups.end());
    uploaded = ng;
    return 0;
  }

  // load the inputs of the planned groups; first: reset the per-CB flags of the whole job
  // (total_cbs code blocks; init_done seeds cb_done: blocks already decoded are skipped, noi 0).
  // flags = false: a fixed-half-iteration job, which never reads the early-stop flags
  // derm: the DL-SCH's de-rate-matching items by decoder position; groups whose loader would be
  // k_load_sbt (16-byte aligned sub-block rows, nb a multiple of 8) are loaded by k_load_derm
  // from the items' LLRs instead of from their rows (the items are marked `direct` by the caller)
  uint32_t derm_max_ne = 0; // the largest E among the direct items of the next job (set by the caller)
  static bool derm_direct(const TdGroup &g, int rows_aligned) {
    return g.sb_input && rows_aligned >= 16 && g.nb % 8 == 0;
  }
  // P1 deferral (defer_p1, the hybrid early-stop schedule with packed stragglers): the first
  // half-iteration (DEC1) does not read P1, so k_load_derm leaves it out and the pairs k_decide lists
  // as still running get theirs just before the early-stop launch (at 20 dB 3 % of them): a quarter
  // of the loader's writes. p1_runs / p1_dc: the direct loads of this pass, for that late launch.
  struct P1Run {
    size_t g0, g1;
    int blocks;
  };
  std::vector<P1Run> p1_runs;
  DermCall p1_dc{};
  bool p1_deferred = false;
  int load_planned(const int16_t *d_in, size_t in_stride, const int16_t *const *rows,
                   int rows_aligned, const uint8_t *init_done, bool first, uint32_t total_cbs,
                   bool flags = true, const DermCall *derm = nullptr, bool defer_p1 = false) {
    // load launches: runs of groups with the same loader (nb, sb_input); rows_aligned is the
    // byte alignment every row is guaranteed to have (0: none)
    const size_t ng = groups.size();
    struct Run {
      size_t g0, g1;
      int blocks;
      bool vec, direct;
    };
    std::vector<Run> runs;
    for (size_t g0 = 0; g0 < ng;) {
      const TdGroup &f = groups[g0];
      bool vec = f.sb_input ? (rows ? rows_aligned >= 16
                                    : ((uintptr_t)d_in % 16 == 0 && (in_stride * 2) % 16 == 0))
                            : (rows ? rows_aligned >= 8 : ((uintptr_t)d_in % 8 == 0 && in_stride % 4 == 0));
      const bool direct = derm && rows && derm_direct(f, rows_aligned);
      size_t g1 = g0;
      while (g1 < ng && groups[g1].nb == f.nb && groups[g1].sb_input == f.sb_input) {
        if (!f.sb_input) vec = vec && (groups[g1].K / groups[g1].nb) % 4 == 0;
        g1++;
      }
      int blocks = 0;
      for (size_t g = g0; g < g1; g++) {
        groups[g].blk_load = blocks;
        blocks += direct ? groups[g].npairs
                         : load_blocks(groups[g].K, groups[g].nb, groups[g].npairs, groups[g].sb_input,
                                       f.sb_input && vec);
      }
      runs.push_back(Run{g0, g1, blocks, vec, direct});
      g0 = g1;
    }
    if (upload_groups()) return -1;
    const TdArrays a = arrays();
    p1_runs.clear();
    p1_deferred = false;
    for (const Run &r : runs) {
      const TdGroup &f = groups[r.g0];
      if (r.direct) {
        ProfScope ps("k_ldderm", st); // k_load_derm (a name no other scope contains: srsgpu_prof_get matches substrings)
        HIPCHK(launch_load_derm(d_groups + r.g0, (int)(r.g1 - r.g0), r.blocks, *derm, a, derm_max_ne, st,
                                defer_p1 ? 1 : 0));
        if (defer_p1) {
          p1_runs.push_back(P1Run{r.g0, r.g1, r.blocks});
          p1_dc = *derm;
          p1_deferred = true;
        }
        continue;
      }
      ProfScope ps("k_load", st);
      HIPCHK(launch_load(d_groups + r.g0, (int)(r.g1 - r.g0), r.blocks, f.nb, f.sb_input, r.vec, d_in,
                         in_stride, rows, a, st));
    }
    if (!flags) return 0;
    // every code block of this pass: done = init_done, ok = noi = 0, and the pair flags (a job in
    // several passes seeds each pass's blocks before its decode)
    (void)first;
    (void)total_cbs;
    HIPCHK(launch_pair_done(d_groups, (int)ng, total_pairs, init_done, cb_done, cb_ok, noi, pair_done, st, run_cnt));
    return 0;
  }

  // single-size job (batch API and the drop-in srslte_tdec_* path)
  int load(int impl, int sb_layout, const int16_t *d_in, size_t in_stride, uint32_t Kv, uint32_t n,
           const int16_t *const *rows = nullptr, int rows_aligned = 0,
           const uint8_t *init_done = nullptr, uint32_t poly = 0, uint32_t crc_len = 0,
           bool early_flags = false) {
    if (check_spec(impl, Kv, n)) return -1;
    if (!rows && in_stride < srsgpu_tdec_input_len(impl, sb_layout, Kv)) {
      fprintf(stderr, "srsgpu: input stride %zu too small\n", in_stride);
      return -1;
    }
    const TdSpec sp{Kv, n, poly, crc_len, 0};
    const int r = plan(impl, sb_layout, &sp, 1);
    if (r) {
      if (r > 0) fprintf(stderr, "srsgpu: batch of %u x K=%u exceeds capacity\n", n, Kv);
      return -1;
    }
    K = Kv;
    fwd = groups[0].fwd;
    rev = groups[0].rev;
    dmap = groups[0].dmap;
    return load_planned(d_in, in_stride, rows, rows_aligned, init_done, true, n, early_flags);
  }

  // dec: leave hard decisions in D (needed by the decide() that follows this half-iteration)
  int last_n = -1; // the last half-iteration launched (read_state)

  // kind k of the planned job is one group of a few pairs that k_win_spread can take (latency form)
  bool use_spread(int k) const {
    const int g0 = kind_g0[k], g1 = kind_g0[k + 1];
    if (g1 - g0 != 1 || !knobs().spread) return false;
    const TdGroup &f = groups[g0];
    return f.npairs <= spread_max_pairs() && spread_ok(k, f.K, f.nb);
  }

  // half-iteration n of a one-group job that k_win_spread takes, with the decision bytes of its
  // blocks written to outb by the same launch (the drop-in's one launch per call); 1: not this job
  // flag (optional, host-mapped): seq stored there by the launch once the bytes are written
  int halfit_bytes(int n, uint8_t *outb, size_t out_stride, uint32_t *flag = nullptr, uint32_t seq = 0) {
    if (groups.size() != 1) return 1;
    int k = 0;
    while (k < TD_NKIND && kind_g0[k + 1] - kind_g0[k] != 1) k++;
    if (k == TD_NKIND || !use_spread(k)) return 1;
    last_n = n;
    const TdGroup &f = groups[0];
    ProfScope ps("k_win_spread", st);
    SpreadOut so;
    so.cnt = spread_cnt;
    so.flag = flag;
    so.seq = seq;
    HIPCHK(launch_halfit_spread(n, k, d_groups, f.npairs, f.K, f.nb, true, arrays(), nullptr, st, outb, out_stride, so));
    return 0;
  }

  int halfit(int n, bool early, bool dec = true) {
    last_n = n;
    const uint8_t *pd = early ? pair_done : nullptr;
    const TdArrays a = arrays();
    for (int k = 0; k < TD_NKIND; k++) {
      const int g0 = kind_g0[k], g1 = kind_g0[k + 1];
      if (g1 <= g0) continue;
      static const char *const names[TD_NKIND] = {"k_win_bidir", "k_win_bidir", "k_sse_halfit",
                                                   "k_gen_halfit", "k_win8_bidir", "k_win8_bidir"};
      if (use_spread(k)) {
        ProfScope ps("k_win_spread", st);
        const TdGroup &f = groups[g0];
        HIPCHK(launch_halfit_spread(n, k, d_groups + g0, f.npairs, f.K, f.nb, dec, a, pd, st));
        continue;
      }
      ProfScope ps(names[k], st);
      HIPCHK(launch_halfit(n, k, d_groups + g0, g1 - g0, kind_blocks[k], kind_lds[k], dec, a, pd, st));
    }
    return 0;
  }

  // app1 / ext1 of caller CB `cb` as the reference holds them after half-iteration last_n
  // (turbodecoder_iter.h:283-357): after DEC1 app1 = A and ext1 = DEC1's LLR = E' + A, with
  // E'[j] = X2[rev[j]]; after DEC2 ext1 = X2[rev[j]] (the subtracted ext1 that was interleaved)
  // and app1 = A + ext1. All int16 wrapping.
  int read_state(uint32_t cb, int16_t *app1, int16_t *ext1) {
    if (last_n < 0) return -1;
    const TdGroup *g = nullptr;
    for (const TdGroup &x : groups)
      if (cb >= (uint32_t)x.cb0 && cb < (uint32_t)(x.cb0 + x.ncb)) g = &x;
    // groups are in kind order: from kind_g0[TD_KIND_B16] on, the int8 decoders (scaled values)
    if (!g || (int)(g - groups.data()) >= kind_g0[TD_KIND_B16]) return -1;
    const uint32_t K = (uint32_t)g->K, nb = (uint32_t)g->nb, c = cb - (uint32_t)g->cb0;
    const size_t base = (size_t)g->elem0 + (size_t)(c / 2) * t4_pair_elems((int)K, (int)nb);
    std::vector<uint32_t> a(K), x(K);
    HIPCHK(hipStreamSynchronize(st));
    HIPCHK(hipMemcpy(a.data(), (uint32_t *)A + base, K * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(x.data(), (uint32_t *)XP1 + base, K * 4, hipMemcpyDeviceToHost));
    std::vector<uint16_t> f, r;
    gen_interleaver(K, nb, f, r);
    const int sh = (c & 1) ? 16 : 0;
    for (uint32_t j = 0; j < K; j++) {
      // the first DEC1 runs without a priori (app1 still all zero, turbodecoder_iter.h:318-323)
      // and leaves A unwritten
      const uint16_t av = last_n == 0 ? 0 : (uint16_t)(a[j] >> sh), ev = (uint16_t)(x[r[j]] >> sh);
      if (last_n & 1) {
        ext1[j] = (int16_t)ev;
        app1[j] = (int16_t)(uint16_t)(av + ev);
      } else {
        app1[j] = (int16_t)av;
        ext1[j] = (int16_t)(uint16_t)(ev + av);
      }
    }
    return 0;
  }

  int decide(int n, uint8_t *d_out, size_t out_stride, bool early, uint32_t maxh = 0, bool list = false) {
    ProfScope ps("k_decide", st);
    HIPCHK(launch_decide(n, d_groups, (int)groups.size(), total_pairs, arrays(), d_out, out_stride,
                         early, cb_done, cb_ok, noi, (int)maxh, pair_done, st, list ? run_list : nullptr,
                         list ? run_cnt : nullptr));
    return 0;
  }

  int run(int impl, int sb_layout, const int16_t *d_in, size_t in_stride, uint32_t Kv, uint32_t n,
          uint32_t nhalf, uint8_t *d_out, size_t out_stride) {
    if (nhalf == 0) {
      fprintf(stderr, "srsgpu: nof_halfits must be > 0\n");
      return -1;
    }
    if (load(impl, sb_layout, d_in, in_stride, Kv, n)) return -1;
    if (halfits_fixed((int)nhalf)) return -1;
    return decide((int)nhalf - 1, d_out, out_stride, false);
  }

  // all nh half-iterations of a fixed-iteration job, decisions after the last: windowed kinds in
  // one launch each (k_win_bidir_run), the sequential decoders one launch per half-iteration.
  // SRSGPU_TDEC_FUSED=0 selects the per-half-iteration launches everywhere (A/B measurements).
  int halfits_fixed(int nh) {
    const bool fused = td_sched().fused != 0;
    if (!fused || nh < 2) {
      for (int h = 0; h < nh; h++)
        if (halfit(h, false, h + 1 == nh)) return -1;
      return 0;
    }
    last_n = nh - 1;
    const TdArrays a = arrays();
    for (int k = 0; k < TD_NKIND; k++) {
      const int g0 = kind_g0[k], g1 = kind_g0[k + 1];
      if (g1 <= g0) continue;
      if (use_spread(k)) { // a few pairs: per-half-iteration latency launches beat one long one
        const TdGroup &f = groups[g0];
        for (int h = 0; h < nh; h++) {
          ProfScope ps("k_win_spread", st);
          HIPCHK(launch_halfit_spread(h, k, d_groups + g0, f.npairs, f.K, f.nb, h + 1 == nh, a, nullptr, st));
        }
      } else if (halfits_fusable(k)) {
        ProfScope ps("k_win_bidir_run", st);
        HIPCHK(launch_halfits(0, nh, k, d_groups + g0, g1 - g0, kind_blocks[k], kind_lds[k], true, a, st));
      } else {
        for (int h = 0; h < nh; h++) {
          ProfScope ps(k == TD_KIND_SSE ? "k_sse_halfit" : "k_gen_halfit", st);
          HIPCHK(launch_halfit(h, k, d_groups + g0, g1 - g0, kind_blocks[k], kind_lds[k], h + 1 == nh,
                               a, nullptr, st));
        }
      }
    }
    return 0;
  }

  // early-stop decoding of one pass (planned groups) — maxh half-iterations at most. The windowed
  // kinds and the SSE decoder (K <= 400 under AUTO) run every half-iteration with its CRC check in
  // one launch each (k_win_bidir_es, k_sse_es); GENERIC one launch per half-iteration plus a decide
  // launch, which skips the pairs the fused launches finished.
  // SRSGPU_TDEC_FUSED=0 selects the per-half-iteration launches everywhere (A/B measurements).
  // the hybrid early-stop schedule (decode_planned): es_fused 3, or 2 when a kind's workgroups do not
  // fit on the chip at once; every kind fusable. A plan() must have run.
  bool hybrid_planned(uint32_t maxh) const {
    const int es_mode = td_sched().es_fused;
    if (!((es_mode == 3 || es_mode == 2) && maxh > 1)) return false;
    bool all_es = true, any_big = false;
    for (int k = 0; k < TD_NKIND; k++)
      if (kind_g0[k + 1] > kind_g0[k]) {
        if (!halfits_es_fusable(k)) all_es = false;
        const size_t per_cu = std::max<size_t>(1, std::min<size_t>(8, 160 * 1024 / (kind_lds[k] + 2048)));
        if ((size_t)kind_blocks[k] > (size_t)num_cus() * per_cu) any_big = true;
      }
    return all_es && (es_mode == 3 || any_big);
  }
  int decode_planned(uint32_t maxh, uint8_t *d_out, size_t out_stride) {
    // td_sched().es_chunk: half-iterations per early-stop launch. One launch per half-iteration
    // (with the CRC check inside, no decide launch) lets the kernels of other streams in between;
    // longer launches save launches but hold every CU until they end
    const int es_mode = td_sched().es_fused;
    // es_fused 2 (auto): a kind runs fused when its workgroups fit on the chip at once (small,
    // launch-bound jobs such as C5's); a larger job keeps one launch per half-iteration, whose
    // kernel boundaries let the front end of other streams in and bound the tail of the last
    // round of workgroups to one half-iteration
    auto es_on = [&](int k) {
      if (!halfits_es_fusable(k) || es_mode == 0) return false;
      if (es_mode == 1 || es_mode == 3) return true;
      const size_t per_cu = std::max<size_t>(1, std::min<size_t>(8, 160 * 1024 / (kind_lds[k] + 2048)));
      return (size_t)kind_blocks[k] <= (size_t)num_cus() * per_cu;
    };
    const int chunk = td_sched().es_chunk;
    bool seq = false, es_any = false;
    const TdArrays a = arrays();
    // the early-stop launches' wave priority, 0..3 (SRSGPU_ES_PRIO from the knob snapshot, wave_prio.h;
    // default 3): the few workgroups still running after the heavy pass win their SIMDs' issue
    // arbitration against other streams' throughput kernels (headline 0.871 -> 0.858 ms, r05_s34 / s35)
    TdEs es{d_out, out_stride, cb_done, cb_ok, noi, (int)maxh, 0, 0, Dfz, cb_end, knobs().es_prio};
    // es_fused 3 (hybrid): the first half-iteration of every kind as one launch per kind plus one
    // k_decide (the whole batch's heavy pass, with kernel boundaries that let other streams in), then
    // the blocks still running (a few at high SNR) through the remaining half-iterations in ONE
    // early-stop launch per kind, where they loop without a launch and a k_decide per half-iteration
    // es_fused 2 (auto) takes this form too when a kind's workgroups do not fit on the chip at once
    // (a fused launch would leave its last round of workgroups to run every half-iteration alone)
    if (p1_deferred && !hybrid_planned(maxh)) {
      fprintf(stderr, "srsgpu: internal: P1 deferred without the hybrid schedule\n");
      return -1;
    }
    {
      if (hybrid_planned(maxh)) {
        // "_h0": the first half-iteration's own scope name (a subset of "k_win_bidir" for
        // srsgpu_prof_get, which matches substrings)
        static const char *const names0[TD_NKIND] = {"k_win_bidir_h0", "k_win_bidir_h0", "k_sse_halfit",
                                                      "k_gen_halfit", "k_win8_bidir", "k_win8_bidir"};
        // windowed kinds: the pairs still running are listed after the first half-iteration and packed
        // by the early-stop launch (TdEs::run_list); the SSE kind keeps its own mapping
        const bool compact = knobs().es_compact || p1_deferred;
        // only 16-bit window kinds: the first half-iteration as an early-stop launch of one half-iteration
        // per kind, whose workgroups check their own blocks' CRC, write the bytes of those that end and
        // list the pairs still running (no k_decide launch, no decision-word round trip)
        bool h0_fused = knobs().h0_decide;
        for (int k = 0; k < TD_NKIND; k++)
          if (kind_g0[k + 1] > kind_g0[k] && k != TD_KIND_W16 && k != TD_KIND_W8) h0_fused = false;
        for (int k = 0; k < TD_NKIND; k++) {
          const int g0 = kind_g0[k], g1 = kind_g0[k + 1];
          if (g1 <= g0) continue;
          ProfScope ps(names0[k], st);
          if (h0_fused) {
            TdEs e0 = es;
            e0.n0 = 0;
            e0.n1 = 1;
            e0.prio = knobs().h0_prio;
            e0.bytes_direct = 1;
            if (compact) {
              e0.list_out = run_list;
              e0.cnt_out = run_cnt;
            }
            HIPCHK(launch_halfits_es(k, d_groups + g0, g1 - g0, kind_blocks[k], kind_lds[k], a, e0, st));
          } else {
            HIPCHK(launch_halfit(0, k, d_groups + g0, g1 - g0, kind_blocks[k], kind_lds[k], true, a, pair_done, st));
          }
        }
        auto split = [&]() -> int {
          if (split_st && split_st != st) {
            // the few blocks still running, their bytes and the caller's epilogue on the tail stream:
            // the caller's stream goes on with its next work meanwhile
            if (!ev_split) HIPCHK(hipEventCreateWithFlags(&ev_split, hipEventDisableTiming));
            HIPCHK(hipEventRecord(ev_split, st));
            HIPCHK(hipStreamWaitEvent(split_st, ev_split, 0));
            st = split_st;
          }
          return 0;
        };
        // the tail stream takes over right after the first half-iteration (the first check and the P1
        // loads too), so the caller's stream moves on to its next work two launches earlier
        // (SRSGPU_SPLIT_EARLY=0: after them)
        if (knobs().split_early && split()) return -1;
        if (!h0_fused && decide(0, d_out, out_stride, true, maxh, compact)) return -1;
        if (p1_deferred) { // P1 of the pairs still running (k_load_derm mode 2), before their DEC2
          const TdArrays a1 = arrays();
          for (const P1Run &r : p1_runs) {
            ProfScope ps("k_ldderm", st);
            HIPCHK(launch_load_derm(d_groups + r.g0, (int)(r.g1 - r.g0), r.blocks, p1_dc, a1, derm_max_ne, st, 2,
                                    run_list, run_cnt));
          }
        }
        if (split()) return -1;
        es.n0 = 1;
        es.n1 = (int)maxh;
        for (int k = 0; k < TD_NKIND; k++) {
          const int g0 = kind_g0[k], g1 = kind_g0[k + 1];
          if (g1 <= g0) continue;
          TdEs ek = es;
          if (compact && k != TD_KIND_SSE) {
            ek.run_list = run_list;
            ek.run_cnt = run_cnt;
          }
          ProfScope ps(k == TD_KIND_SSE ? "k_sse_es" : "k_win_bidir_es", st);
          HIPCHK(launch_halfits_es(k, d_groups + g0, g1 - g0, kind_blocks[k], kind_lds[k], a, ek, st));
        }
        if (defer_now) {
          bytes_deferred = true;
        } else {
          ProfScope ps("k_es_bytes", st);
          HIPCHK(launch_es_bytes(d_groups, (int)groups.size(), total_pairs, es, st));
        }
        last_n = (int)maxh - 1;
        return 0;
      }
    }
    // The SSE kind (K <= 400: a few workgroups, each a long serial chain) runs fused on a second
    // stream beside the fused window kinds: the kinds are disjoint groups (their own arrays,
    // flags and Dfz ranges), so the launch's critical path is the longer of the two, not the sum.
    int n_es = 0;
    for (int k = 0; k < TD_NKIND; k++)
      if (kind_g0[k + 1] > kind_g0[k] && es_on(k)) n_es++;
    const bool fork = n_es > 1 && kind_g0[TD_KIND_SSE + 1] > kind_g0[TD_KIND_SSE] && es_on(TD_KIND_SSE);
    if (fork) {
      if (!aux) {
        HIPCHK(hipStreamCreateWithFlags(&aux, hipStreamNonBlocking));
        HIPCHK(hipEventCreateWithFlags(&ev_fork, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&ev_join, hipEventDisableTiming));
      }
      HIPCHK(hipEventRecord(ev_fork, st));
      HIPCHK(hipStreamWaitEvent(aux, ev_fork, 0));
    }
    for (int k = 0; k < TD_NKIND; k++) {
      const int g0 = kind_g0[k], g1 = kind_g0[k + 1];
      if (g1 <= g0) continue;
      if (es_on(k)) {
        es_any = true;
        hipStream_t ks = fork && k == TD_KIND_SSE ? aux : st;
        for (int n0 = 0; n0 < (int)maxh; n0 += chunk) {
          es.n0 = n0;
          es.n1 = std::min(n0 + chunk, (int)maxh);
          ProfScope ps(k == TD_KIND_SSE ? "k_sse_es" : "k_win_bidir_es", ks);
          HIPCHK(launch_halfits_es(k, d_groups + g0, g1 - g0, kind_blocks[k], kind_lds[k], a, es, ks));
        }
      } else {
        seq = true;
      }
    }
    if (fork) {
      HIPCHK(hipEventRecord(ev_join, aux));
      HIPCHK(hipStreamWaitEvent(st, ev_join, 0));
    }
    if (es_any && defer_now) {
      bytes_deferred = true;
    } else if (es_any) {
      ProfScope ps("k_es_bytes", st);
      HIPCHK(launch_es_bytes(d_groups, (int)groups.size(), total_pairs, es, st));
    }
    last_n = (int)maxh - 1;
    if (!seq) return 0;
    for (uint32_t h = 0; h < maxh; h++) {
      last_n = (int)h;
      for (int k = 0; k < TD_NKIND; k++) {
        const int g0 = kind_g0[k], g1 = kind_g0[k + 1];
        if (g1 <= g0 || es_on(k)) continue;
        static const char *const names[TD_NKIND] = {"k_win_bidir", "k_win_bidir", "k_sse_halfit",
                                                     "k_gen_halfit", "k_win8_bidir", "k_win8_bidir"};
        ProfScope ps(names[k], st);
        HIPCHK(launch_halfit((int)h, k, d_groups + g0, g1 - g0, kind_blocks[k], kind_lds[k], true, a,
                             pair_done, st));
      }
      if (decide((int)h, d_out, out_stride, true, maxh)) return -1;
    }
    return 0;
  }

  // Mixed sizes: specs in any order (cb0 ranges disjoint, < total_cbs); CB c's input at rows[c]
  // (or d_in + c * in_stride), its decision bytes at d_out + c * out_stride. Specs that do not fit
  // the arrays together are decoded in several passes.
  int decode_multi(int impl, int sb_layout, const std::vector<TdSpec> &specs, uint32_t total_cbs,
                   const int16_t *d_in, size_t in_stride, const int16_t *const *rows, int rows_aligned,
                   const uint8_t *init_done, uint32_t maxh, uint8_t *d_out, size_t out_stride,
                   uint8_t *d_ok, uint32_t *d_noi, bool fixed = false, const DermCall *derm = nullptr) {
    if (maxh == 0 || total_cbs > cap_cbs) {
      fprintf(stderr, "srsgpu: invalid early-stop job (max_halfits=%u, %u code blocks)\n", maxh, total_cbs);
      return -1;
    }
    for (const TdSpec &sp : specs) {
      if (check_spec(impl, sp.K, sp.n)) return -1;
      if (sp.crc_len == 0 || sp.crc_len % 8 || sp.crc_len > sp.K || sp.cb0 + sp.n > total_cbs) {
        fprintf(stderr, "srsgpu: invalid early-stop parameters (crc_len=%u K=%u)\n", sp.crc_len, sp.K);
        return -1;
      }
      if (!rows && in_stride < srsgpu_tdec_input_len(impl, sb_layout, sp.K)) {
        fprintf(stderr, "srsgpu: input stride %zu too small\n", in_stride);
        return -1;
      }
    }
    // the caller's ok / noi arrays (total_cbs entries) take the place of the engine's own for this
    // job, so the flags land there without a copy; restored on every return
    struct Swap {
      TdecEngine &e;
      uint8_t *ok;
      uint32_t *ni;
      ~Swap() {
        e.cb_ok = ok;
        e.noi = ni;
      }
    } swap{*this, cb_ok, noi};
    if (d_ok) cb_ok = d_ok;
    if (d_noi) noi = d_noi;
    bytes_deferred = false;
    bool first = true;
    for (size_t s0 = 0; s0 < specs.size();) {
      size_t s1 = specs.size();
      int r;
      while ((r = plan(impl, sb_layout, specs.data() + s0, s1 - s0)) == 1 && s1 - s0 > 1)
        s1 = s0 + (s1 - s0 + 1) / 2;
      if (r) {
        if (r > 0) fprintf(stderr, "srsgpu: code block group exceeds the decoder capacity\n");
        return -1;
      }
      // P1 deferral needs the hybrid schedule's k_decide list (and the early stop)
      const bool defer_p1 = derm && !fixed && knobs().defer_p1 && hybrid_planned(maxh);
      if (load_planned(d_in, in_stride, rows, rows_aligned, init_done, first, total_cbs, true, derm, defer_p1))
        return -1;
      defer_now = defer_bytes && s0 == 0 && s1 == specs.size(); // one pass: Dfz / groups stay for the caller
      if (fixed) { // all maxh half-iterations, then one CRC check (no early stop: measurement mode)
        if (halfits_fixed((int)maxh) || decide((int)maxh - 1, d_out, out_stride, true, maxh)) return -1;
      } else if (decode_planned(maxh, d_out, out_stride)) {
        return -1;
      }
      first = false;
      s0 = s1;
    }
    return 0;
  }

  int decode(int impl, int sb_layout, const int16_t *d_in, size_t in_stride, uint32_t Kv, uint32_t n,
             uint32_t maxh, uint32_t poly, uint32_t crc_len, uint8_t *d_out, size_t out_stride,
             uint8_t *d_ok, uint32_t *d_noi, const int16_t *const *rows = nullptr,
             int rows_aligned = 0, const uint8_t *init_done = nullptr) {
    const std::vector<TdSpec> sp{TdSpec{Kv, n, poly, crc_len, 0}};
    return decode_multi(impl, sb_layout, sp, n, d_in, in_stride, rows, rows_aligned, init_done, maxh,
                        d_out, out_stride, d_ok, d_noi);
  }

  int stage(uint32_t n, uint32_t Kv, size_t in_len) {
    if (!in_stage) {
      HIPCHK(hipMalloc(&in_stage, (size_t)cap_cbs * (3 * (cap_K + 32) + 12) * 2));
      HIPCHK(hipMalloc(&out_stage, (size_t)cap_cbs * (cap_K / 8)));
    }
    (void)n;
    (void)Kv;
    (void)in_len;
    return 0;
  }
};

} // namespace srsgpu
#endif
