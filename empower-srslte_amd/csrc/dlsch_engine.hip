// Host side of the MI355X DL-SCH transport-block decoder (include/srsgpu/dlsch_batch.h).
//
// One call = many transport blocks:
//   host      code block segmentation and the per-CB receive parameters of decode_tb_cb
//             (sch.c:325-341), grouping of the CBs by (K, CRC) for the turbo decoder
//   k_derm    de-rate-matching + HARQ combining of every CB into its softbuffer row
//   decoder   ONE TdecEngine job over all (K, CRC) groups (one launch per decoder variant and
//             half-iteration, however many sizes) on the softbuffer rows themselves (row pointer
//             table, SB layout), CRC early stop per half-iteration, CBs that passed in an earlier
//             transmission start out "done"
//   k_tb_finish  TB bytes, cb_crc / saved bytes, nof_iterations, TB CRC
#include <hip/hip_runtime.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <string.h>
#include <tuple>
#include <vector>

#include "dlsch_kernels.h"
#include "host_ring.h"
#include "srsgpu/dlsch_batch.h"
#include "srsgpu/uci_tables.h"
#include "srsgpu/ulsch_batch.h"
#include "tdec_engine.h"

namespace srsgpu {

// ------------------------------------------------------------------ segmentation ----
struct Segm {
  uint32_t tbs = 0, C = 0, C1 = 0, K1 = 0, C2 = 0, K2 = 0, F = 0;
};

// srslte_cbsegm (cbsegm.c:58-112): C = ceil(B / 6120) (B > 6144), K1 = smallest table size
// >= ceil(B'/C), K2 = the next smaller one, C2 = (C*K1 - B') / (K1 - K2)
static int segm(uint32_t tbs, Segm &s) {
  s = Segm();
  s.tbs = tbs;
  if (tbs == 0) return 0;
  const uint32_t B = tbs + 24;
  uint32_t Bp;
  if (B <= 6144) {
    s.C = 1;
    Bp = B;
  } else {
    s.C = (B + 6119) / 6120;
    Bp = B + 24 * s.C;
  }
  const uint32_t target = (Bp - 1) / s.C + 1;
  int idx = -1;
  for (int i = 0; i < SRSGPU_NOF_CB_SIZES; i++)
    if (srsgpu_qpp_table[i][0] >= target) {
      idx = i;
      break;
    }
  if (idx < 0) return -1;
  s.K1 = srsgpu_qpp_table[idx][0];
  if (s.C == 1) {
    s.K2 = 0;
    s.C2 = 0;
    s.C1 = 1;
  } else {
    s.K2 = idx > 0 ? srsgpu_qpp_table[idx - 1][0] : s.K1;
    s.C2 = s.K1 > s.K2 ? (s.C * s.K1 - Bp) / (s.K1 - s.K2) : 0;
    s.C1 = s.C - s.C2;
  }
  s.F = s.C1 * s.K1 + s.C2 * s.K2 - Bp;
  return 0;
}

// ------------------------------------------------------------------ rate-matching table ----
// Receive table of 36.212 5.1.4.1 for (K, rv): entry m = decoder-input index of the m-th
// non-<NULL> bit of the circular buffer read from k0 (rm_turbo.c:163-228). Built forward: the
// buffer holds v0 (systematic), then v1/v2 interleaved, each the column-permuted R x 32 matrix
// with ND leading dummies; v2 uses pi(k) = (P[k/R] + 32(k%R) + 1) mod Kp. Decoder index of
// stream s, position k: 3k+s (natural) or, for the windowed decoders, the sub-block layout
// s*(K+32) + (k % (K/nsb))*nsb + k/(K/nsb), tails at 3*(K+32) (rm_turbo.c:231-257).
static const uint8_t RM_PERM[32] = {0, 16, 8, 24, 4, 20, 12, 28, 2, 18, 10, 26, 6, 22, 14, 30,
                                    1, 17, 9, 25, 5, 21, 13, 29, 3, 19, 11, 27, 7, 23, 15, 31};

static void rm_rx_table(uint32_t K, uint32_t rv, uint32_t nsb, std::vector<uint16_t> &t) {
  const uint32_t D = K + 4, R = (D + 31) / 32, Kp = 32 * R, ND = Kp - D, Ncb = 3 * Kp;
  auto dec_index = [&](uint32_t d) -> uint32_t { // d = 3k + s, natural index
    if (!nsb) return d;
    if (d >= 3 * K) return d - 3 * K + 3 * (K + 32);
    const uint32_t k = d / 3, s = d % 3, L = K / nsb;
    return s * (K + 32) + (k % L) * nsb + k / L;
  };
  auto entry = [&](uint32_t w) -> int64_t { // circular-buffer position -> d or -1 (<NULL>)
    if (w < Kp) {
      const uint32_t y = (w % R) * 32 + RM_PERM[w / R];
      return y < ND ? -1 : (int64_t)(3 * (y - ND));
    }
    const uint32_t k = (w - Kp) / 2;
    if (((w - Kp) & 1) == 0) {
      const uint32_t y = (k % R) * 32 + RM_PERM[k / R];
      return y < ND ? -1 : (int64_t)(3 * (y - ND) + 1);
    }
    const uint32_t p = (RM_PERM[k / R] + 32 * (k % R) + 1) % Kp;
    return p < ND ? -1 : (int64_t)(3 * (p - ND) + 2);
  };
  const uint32_t N = 3 * K + 12, k0 = R * (24 * rv + 2);
  t.resize(N);
  uint32_t m = 0;
  for (uint32_t j = 0; m < N; j++) {
    const int64_t v = entry((k0 + j) % Ncb);
    if (v >= 0) t[m++] = (uint16_t)dec_index((uint32_t)v);
  }
}

// ------------------------------------------------------------------ engine ----
struct DlschEngine {
  hipStream_t st = nullptr;
  uint32_t nslots = 0, max_cb = 0, cap = 0;
  int16_t *soft = nullptr;   // [nslots * max_cb][SOFTBUFFER_SIZE]
  uint8_t *saved = nullptr;  // [nslots * max_cb][768]
  uint8_t *cbcrc = nullptr;  // [nslots * max_cb]
  uint8_t *fresh = nullptr;  // [nslots * max_cb]: row reset since last use (counts as zero)
  // per-call device arrays (capacity cap CBs / cap TBs)
  DermItem *d_items = nullptr;
  TbItem *d_tbs = nullptr;
  const int16_t **d_rows = nullptr;
  uint32_t *d_cbmap = nullptr;
  uint8_t *d_init = nullptr, *d_dec = nullptr, *d_ok = nullptr;
  uint32_t *d_noi = nullptr;
  uint32_t *d_late = nullptr; // [1 + cap]: count, then the decoder positions of the deferred rows
  int32_t *d_ret_stage = nullptr;
  uint32_t *d_noi_stage = nullptr;
  // pinned staging for the per-call descriptors, reused once the previous copies completed
  DermItem *h_items = nullptr; // rm_rx_dev's single item
  TbItem *h_tbs = nullptr;
  const int16_t **h_rows = nullptr;
  uint32_t *h_cbmap = nullptr;
  // a decode call's descriptors packed into one block (records, row pointers, CB map, TBs), one
  // upload per call
  uint8_t *h_blk = nullptr, *d_blk = nullptr; // h_blk: the current slot of blk_ring
  HostRing blk_ring;                           // pinned staging of the blocks (host_ring.h)
  std::vector<DermRec> rec_tb; // records in TB order while the call is planned
  // table sets per (K, rv, layout): index into d_tabs (device, append-only)
  std::map<std::tuple<uint32_t, uint32_t, uint32_t>, uint16_t> tab_index;
  DermTabs *d_tabs = nullptr;
  static constexpr uint32_t TABS_CAP = 4096;
  hipEvent_t staged = nullptr;
  bool staged_pending = false;
  bool llr8 = false; // srslte_sch_t.llr_is_8bit: int8 LLRs, 8-bit de-RM and decoders
  bool fixed = false; // srsgpu_dlsch_set_early_stop(0): every CB runs max_halfits, one CRC check
  // srsgpu_dlsch_set_direct_derm: window-decoder code blocks are de-rate-matched straight into the
  // decoder inputs (k_load_derm) and their softbuffer rows written after the decode, only for TBs
  // that failed (the only rows the reference reads again)
  bool direct_derm = true;
  // the epilogue (k_tb_finish) also makes the bytes of the blocks the fused early stop ended and the
  // rows of failed TBs: two launches fewer per call (SRSGPU_EPILOGUE=split: the separate k_es_bytes
  // and k_derm_late, for A/B; read at create)
  bool fused_epilogue = true;
  std::map<std::tuple<uint32_t, uint32_t, uint32_t>, uint16_t *> tables, inv_tables, inv_t4_tables;
  TdecEngine tdec;
  // transmit side: per-CB encode descriptors (lazily allocated) and the long CRC24A table
  EncItem *h_enc = nullptr, *d_enc = nullptr;
  uint32_t *d_crc_a = nullptr;
  // UL-SCH deinterleaver descriptors (lazily allocated)
  UlItem *h_ul = nullptr, *d_ul = nullptr;
  int32_t *d_uci_ret = nullptr; // [2 cap]: ret / noi of the data TBs of a UCI call (lazily allocated)
  // host-pointer API staging
  int16_t *e_stage = nullptr;
  uint8_t *data_stage = nullptr;
  size_t e_stage_len = 0, data_stage_len = 0;

  int create(uint32_t slots, uint32_t mcb, uint32_t cap_cbs) {
    if (!slots || !mcb || !cap_cbs) return -1;
    nslots = slots;
    max_cb = mcb;
    cap = cap_cbs;
    if (const char *e = getenv("SRSGPU_EPILOGUE")) fused_epilogue = strcmp(e, "split") != 0;
    const size_t rows = (size_t)slots * mcb;
    HIPCHK(hipMalloc(&soft, rows * SRSGPU_SOFTBUFFER_SIZE * 2));
    HIPCHK(hipMemset(soft, 0, rows * SRSGPU_SOFTBUFFER_SIZE * 2));
    HIPCHK(hipMalloc(&saved, rows * 768));
    HIPCHK(hipMemset(saved, 0, rows * 768));
    HIPCHK(hipMalloc(&cbcrc, rows));
    HIPCHK(hipMemset(cbcrc, 0, rows));
    HIPCHK(hipMalloc(&fresh, rows));
    HIPCHK(hipMemset(fresh, 1, rows));
    HIPCHK(hipMalloc(&d_items, sizeof(DermItem) * cap));
    HIPCHK(hipMalloc(&d_tbs, sizeof(TbItem) * cap));
    HIPCHK(hipMalloc(&d_rows, sizeof(int16_t *) * cap));
    HIPCHK(hipMalloc(&d_cbmap, sizeof(uint32_t) * cap));
    HIPCHK(hipMalloc(&d_init, cap));
    HIPCHK(hipMalloc(&d_dec, (size_t)cap * 768));
    HIPCHK(hipMalloc(&d_ok, cap));
    HIPCHK(hipMalloc(&d_noi, sizeof(uint32_t) * cap));
    HIPCHK(hipMalloc(&d_late, sizeof(uint32_t) * (cap + 1)));
    HIPCHK(hipMalloc(&d_ret_stage, sizeof(int32_t) * cap));
    HIPCHK(hipMalloc(&d_noi_stage, sizeof(uint32_t) * cap));
    HIPCHK(hipHostMalloc(&h_items, sizeof(DermItem) * cap));
    HIPCHK(blk_ring.create(blk_bytes(cap, cap)));
    HIPCHK(hipMalloc(&d_blk, blk_bytes(cap, cap)));
    HIPCHK(hipMalloc(&d_tabs, sizeof(DermTabs) * TABS_CAP));
    HIPCHK(hipHostMalloc(&h_tbs, sizeof(TbItem) * cap));
    HIPCHK(hipHostMalloc(&h_rows, sizeof(int16_t *) * cap));
    HIPCHK(hipHostMalloc(&h_cbmap, sizeof(uint32_t) * cap));
    HIPCHK(hipEventCreateWithFlags(&staged, hipEventDisableTiming));
    if (tdec.create(cap, 6144)) return -1;
    // x^(d+24) mod 0x1864CFB for every bit distance d of a TB: the TB CRC24A as a parallel XOR
    // fold (k_tb_finish, k_dlsch_encode)
    std::vector<uint32_t> t(CRC_A_LEN);
    uint32_t r = 1u << 23;
    for (uint32_t d = 0; d < CRC_A_LEN; d++) {
      const uint32_t top = r & 0x800000u;
      r = (r << 1) & 0xFFFFFFu;
      if (top) r ^= 0x864CFBu;
      t[d] = r;
    }
    HIPCHK(hipMalloc(&d_crc_a, CRC_A_LEN * 4));
    HIPCHK(hipMemcpy(d_crc_a, t.data(), CRC_A_LEN * 4, hipMemcpyHostToDevice));
    return 0;
  }

  void destroy() {
    if (tail_st) (void)hipStreamSynchronize(tail_st);
    if (st) (void)hipStreamSynchronize(st);
    if (ev_tail) (void)hipEventDestroy(ev_tail);
    for (void *p : {(void *)soft, (void *)saved, (void *)cbcrc, (void *)fresh, (void *)d_items, (void *)d_tbs,
                    (void *)d_rows, (void *)d_cbmap, (void *)d_init, (void *)d_dec, (void *)d_ok,
                    (void *)d_noi, (void *)d_late, (void *)d_ret_stage, (void *)d_noi_stage, (void *)e_stage,
                    (void *)data_stage, (void *)d_enc, (void *)d_crc_a, (void *)d_ul, (void *)d_uci_ret})
      if (p) (void)hipFree(p);
    blk_ring.destroy();
    list_ring.destroy();
    if (d_list) (void)hipFree(d_list);
    for (void *p : {(void *)h_items, (void *)h_tbs, (void *)h_rows, (void *)h_cbmap, (void *)h_enc,
                    (void *)h_ul})
      if (p) (void)hipHostFree(p);
    for (void *p : {(void *)d_blk, (void *)d_tabs})
      if (p) (void)hipFree(p);
    for (auto &kv : tables) (void)hipFree(kv.second);
    tables.clear();
    for (auto &kv : inv_tables) (void)hipFree(kv.second);
    inv_tables.clear();
    for (auto &kv : inv_t4_tables) (void)hipFree(kv.second);
    inv_t4_tables.clear();
    if (staged) (void)hipEventDestroy(staged);
    tdec.destroy();
  }

  // inverse of the receive table: decoder-input position -> table entry (0xFFFF: none), over the
  // row length rounded up to 8 (k_derm gathers 8 entries per 16-byte access)
  const uint16_t *inv_table(uint32_t K, uint32_t rv, uint32_t nsb) {
    auto key = std::make_tuple(K, rv, nsb);
    auto it = inv_tables.find(key);
    if (it != inv_tables.end()) return it->second;
    std::vector<uint16_t> t;
    rm_rx_table(K, rv, nsb, t);
    const uint32_t rowlen = nsb ? 3 * (K + 32) + 12 : 3 * K + 12;
    std::vector<uint16_t> inv((rowlen + 7) / 8 * 8, 0xFFFF);
    for (uint32_t m = 0; m < t.size(); m++) inv[t[m]] = (uint16_t)m;
    uint16_t *d = nullptr;
    if (hipMalloc(&d, inv.size() * 2) != hipSuccess) return nullptr;
    if (hipMemcpy(d, inv.data(), inv.size() * 2, hipMemcpyHostToDevice) != hipSuccess) return nullptr;
    inv_tables.emplace(key, d);
    return d;
  }

  // the inverse table in the window decoders' T4 order (k_load_derm): entry st * ne + el is the
  // table entry m that lands on stream st (sys, p0, p1) of T4 element el of a pair region (step
  // k = 4 (el / 4nb) + el % 4 of chain d = el / 4 % nb; padded steps k >= L repeat step L - 1, as
  // k_load_sbt fills them), then the 12 tail positions; ne = nsb * 4 * ceil(K / nsb / 4)
  const uint16_t *inv_t4_table(uint32_t K, uint32_t rv, uint32_t nsb) {
    auto key = std::make_tuple(K, rv, nsb);
    auto it = inv_t4_tables.find(key);
    if (it != inv_t4_tables.end()) return it->second;
    std::vector<uint16_t> t;
    rm_rx_table(K, rv, nsb, t);
    std::vector<uint16_t> inv(3 * (K + 32) + 16, 0xFFFF);
    for (uint32_t m = 0; m < t.size(); m++) inv[t[m]] = (uint16_t)m;
    const uint32_t L = K / nsb, G4 = (L + 3) / 4, ne = nsb * 4 * G4;
    std::vector<uint16_t> t4(3 * ne + 16, 0xFFFF);
    for (uint32_t st = 0; st < 3; st++)
      for (uint32_t el = 0; el < ne; el++) {
        const uint32_t k = std::min(4 * (el / (4 * nsb)) + el % 4, L - 1), d = el / 4 % nsb;
        t4[st * ne + el] = inv[st * (K + 32) + k * nsb + d];
      }
    for (uint32_t i = 0; i < 12; i++) t4[3 * ne + i] = inv[3 * (K + 32) + i];
    uint16_t *d = nullptr;
    if (hipMalloc(&d, t4.size() * 2) != hipSuccess) return nullptr;
    if (hipMemcpy(d, t4.data(), t4.size() * 2, hipMemcpyHostToDevice) != hipSuccess) return nullptr;
    inv_t4_tables.emplace(key, d);
    return d;
  }

  // the packed block of a call: records, row pointers, CB map, TBs (256-byte aligned regions)
  static size_t al(size_t n) { return (n + 255) & ~(size_t)255; }
  static size_t blk_bytes(uint32_t ncb, uint32_t ntb) {
    return al(sizeof(DermRec) * ncb) + al(sizeof(int16_t *) * ncb) + al(4 * (size_t)ncb) + al(sizeof(TbItem) * ntb);
  }

  // index of the table set of (K, rv, layout) in d_tabs (created and uploaded on first use)
  int tab_of(uint32_t K, uint32_t rv, uint32_t nsb) {
    const auto key = std::make_tuple(K, rv, nsb);
    auto it = tab_index.find(key);
    if (it != tab_index.end()) return it->second;
    if (tab_index.size() >= TABS_CAP) return -1;
    DermTabs t{table(K, rv, nsb), inv_table(K, rv, nsb), nsb && nsb % 8 == 0 ? inv_t4_table(K, rv, nsb) : nullptr};
    if (!t.table || !t.inv || (nsb && nsb % 8 == 0 && !t.inv_t4)) return -1;
    const uint16_t idx = (uint16_t)tab_index.size();
    if (hipMemcpy(d_tabs + idx, &t, sizeof(t), hipMemcpyHostToDevice) != hipSuccess) return -1;
    tab_index.emplace(key, idx);
    return idx;
  }

  const uint16_t *table(uint32_t K, uint32_t rv, uint32_t nsb) {
    auto key = std::make_tuple(K, rv, nsb);
    auto it = tables.find(key);
    if (it != tables.end()) return it->second;
    std::vector<uint16_t> t;
    rm_rx_table(K, rv, nsb, t);
    uint16_t *d = nullptr;
    if (hipMalloc(&d, t.size() * 2) != hipSuccess) return nullptr;
    if (hipMemcpy(d, t.data(), t.size() * 2, hipMemcpyHostToDevice) != hipSuccess) return nullptr;
    tables.emplace(key, d);
    return d;
  }

  // encode_tb_off (sch.c:187-296) for a batch of TBs: CB i < C2 has K2 (the encoder's order),
  // E per CB by sch.c:237-241, e bits unpacked (one per byte) at e_offset
  static constexpr uint32_t CRC_A_LEN = 400000; // > 24 + the largest TBS (391656, 36.213)
  int encode(const srsgpu_dlsch_tb_t *tb, uint32_t ntb, const uint8_t *d_data, uint8_t *d_e) {
    if (!h_enc) {
      HIPCHK(hipHostMalloc(&h_enc, sizeof(EncItem) * cap));
      HIPCHK(hipMalloc(&d_enc, sizeof(EncItem) * cap));
    }
    const uint32_t *crc_b = tdec.crc_table(0x1800063);
    if (!crc_b) return -1;
    if (staged_pending) HIPCHK(hipEventSynchronize(staged));
    uint32_t n = 0;
    for (uint32_t b = 0; b < ntb; b++) {
      const srsgpu_dlsch_tb_t &x = tb[b];
      Segm sg;
      if (x.tbs == 0) continue;
      if (segm(x.tbs, sg) || sg.F || x.tbs + 24 > CRC_A_LEN || x.rv > 3 || !x.Qm) {
        fprintf(stderr, "Error filler bits are not supported. Use standard TBS\n"); // sch.c:203-206
        return -1;
      }
      if (n + sg.C > cap) {
        fprintf(stderr, "srsgpu: %u code blocks exceed the capacity %u\n", n + sg.C, cap);
        return -1;
      }
      const uint32_t Gp = x.nof_e_bits / x.Qm, gamma = Gp % sg.C;
      uint32_t rp = 0, wp = 0;
      for (uint32_t i = 0; i < sg.C; i++, n++) {
        const uint32_t K = i < sg.C2 ? sg.K2 : sg.K1;
        EncItem &e = h_enc[n];
        e.data = d_data + x.data_offset;
        e.tbs = x.tbs;
        e.K = K;
        e.rlen = sg.C > 1 ? K - 24 : K;
        e.rp = rp;
        e.ne = i <= sg.C - gamma - 1 ? x.Qm * (Gp / sg.C) : x.Qm * ((Gp + sg.C - 1) / sg.C);
        e.N = 3 * K + 12;
        e.table = table(K, x.rv, 0);
        const TdecEngine::Interl *il = e.table ? tdec.get_interleaver(K, 1) : nullptr;
        if (!il) return -1;
        e.pi = il->fwd;
        e.last = i == sg.C - 1;
        e.crc_cb = sg.C > 1;
        e.e = d_e + x.e_offset + wp;
        rp += e.rlen;
        wp += e.ne;
      }
    }
    HIPCHK(hipMemcpyAsync(d_enc, h_enc, sizeof(EncItem) * n, hipMemcpyHostToDevice, st));
    HIPCHK(hipEventRecord(staged, st));
    staged_pending = true;
    ProfScope ps("k_dlsch_encode", st);
    HIPCHK(launch_dlsch_encode(d_enc, (int)n, d_crc_a, crc_b, st));
    return 0;
  }

  int16_t *row(uint32_t slot, uint32_t cb) {
    return soft + ((size_t)slot * max_cb + cb) * SRSGPU_SOFTBUFFER_SIZE;
  }

  // srslte_softbuffer_rx_reset(_cb): cb_crc cleared now; the soft bits are zeroed lazily (the
  // next de-rate-matching pass treats a fresh softbuffer's rows as zero and rewrites them whole)
  // srsgpu_dlsch_softbuffer_reset_list: one upload (ring-staged) and one launch for n softbuffers
  HostRing list_ring;
  uint32_t *d_list = nullptr;
  static constexpr uint32_t LIST_CAP = 4096;
  int reset_list(const uint32_t *slots, const uint32_t *ncb, uint32_t n) {
    for (uint32_t i = 0; i < n; i++)
      if (slots[i] >= nslots) return -1;
    if (!d_list) {
      HIPCHK(list_ring.create(sizeof(uint32_t) * 2 * LIST_CAP));
      HIPCHK(hipMalloc(&d_list, sizeof(uint32_t) * 2 * LIST_CAP));
    }
    for (uint32_t i0 = 0; i0 < n; i0 += LIST_CAP) {
      const uint32_t m = std::min(LIST_CAP, n - i0);
      hipError_t re;
      uint32_t *h = (uint32_t *)list_ring.acquire(&re);
      HIPCHK(re);
      for (uint32_t i = 0; i < m; i++) {
        h[2 * i] = slots[i0 + i];
        h[2 * i + 1] = ncb ? std::min(ncb[i0 + i], max_cb) : max_cb;
      }
      HIPCHK(list_ring.upload(d_list, h, sizeof(uint32_t) * 2 * m, st));
      HIPCHK(list_ring.mark(st));
      HIPCHK(launch_sb_reset_list(fresh, cbcrc, d_list, m, max_cb, st));
    }
    return 0;
  }

  int reset(uint32_t slot, uint32_t count, uint32_t ncb) {
    if (slot + count > nslots) return -1;
    // one launch: fresh = 1 for the first ncb rows of each slot (reset_tbs), cb_crc = 0 for all
    HIPCHK(launch_sb_reset(fresh + (size_t)slot * max_cb, cbcrc + (size_t)slot * max_cb, count, max_cb,
                           std::min(ncb, max_cb), st));
    return 0;
  }

  // The previous call's inputs and what the host derived from them: a repeat of the same TBs, LLR /
  // data / result pointers and settings (a traffic loop's steady state) skips the per-code-block
  // host work and reuses the descriptor block already on the device (its content would be equal).
  struct Memo {
    std::vector<uint8_t> key;
    bool valid = false;
    uint32_t ncb = 0, ndirect = 0, derm_max_ne = 0, norder = 0;
    size_t o_rows = 0, o_map = 0, o_tbs = 0;
    const int16_t *e_base = nullptr;
    std::vector<TdSpec> specs;
  } memo;
  std::vector<uint8_t> memo_scratch;
  std::vector<uint32_t> cb_key, key_start;                // per code block of a call: its group key
  std::vector<std::pair<uint32_t, uint32_t>> key_list;    // distinct keys, code blocks per key
  // a decoder group's key, ordered as (K, poly, crc length): K < 2^13, the CRC polynomial 24B (0) or
  // 24A (1), the CRC length K (24B) or tbs + 24 <= 6144 (24A, C = 1)
  static uint32_t group_key(uint32_t K, uint32_t poly, uint32_t crclen) {
    return (K << 14) | ((poly == 0x1864CFBu ? 1u : 0u) << 13) | crclen;
  }
  static void group_unkey(uint32_t key, uint32_t &K, uint32_t &poly, uint32_t &crclen) {
    K = key >> 14;
    poly = ((key >> 13) & 1u) ? 0x1864CFBu : 0x1800063u;
    crclen = key & 0x1FFFu;
  }

  void memo_key(std::vector<uint8_t> &k, const srsgpu_dlsch_tb_t *tb, uint32_t ntb, const int16_t *const *e_ptr,
                uint8_t *const *data_ptr, uint32_t maxh, const int32_t *d_ret, const uint32_t *d_noi_out) const {
    const size_t n1 = sizeof(srsgpu_dlsch_tb_t) * ntb, n2 = sizeof(void *) * ntb;
    const uintptr_t tail[8] = {(uintptr_t)d_ret, (uintptr_t)d_noi_out, maxh, llr8, direct_derm, fixed,
                               (uintptr_t)d_blk, ntb};
    k.resize(n1 + 2 * n2 + sizeof(tail));
    memcpy(k.data(), tb, n1);
    memcpy(k.data() + n1, e_ptr, n2);
    memcpy(k.data() + n1 + n2, data_ptr, n2);
    memcpy(k.data() + n1 + 2 * n2, tail, sizeof(tail));
  }

  // srsgpu_dlsch_set_tail_stream: the early-stop tail of a decode call runs on tail_st; the engine's
  // next work on st waits for it (join_tail, at every entry point that enqueues work)
  uint32_t last_ncb = 0; // code blocks of the last decode call (d_noi holds their half-iterations)
  hipStream_t tail_st = nullptr;
  hipEvent_t ev_tail = nullptr;
  bool tail_pending = false;
  int join_tail() {
    if (tail_pending) {
      HIPCHK(hipStreamWaitEvent(st, ev_tail, 0));
      tail_pending = false;
    }
    return 0;
  }

  int decode(const srsgpu_dlsch_tb_t *tb, uint32_t ntb, const int16_t *const *e_ptr,
             uint8_t *const *data_ptr, uint32_t maxh, int32_t *d_ret, uint32_t *d_noi_out) {
    if (ntb > cap) {
      fprintf(stderr, "srsgpu: %u transport blocks exceed the capacity %u\n", ntb, cap);
      return -1;
    }
    if (maxh == 0) {
      fprintf(stderr, "srsgpu: max_halfits must be > 0\n");
      return -1;
    }
    if (join_tail()) return -1;
    tdec.st = st;
    tdec.split_st = tail_st;
    memo_key(memo_scratch, tb, ntb, e_ptr, data_ptr, maxh, d_ret, d_noi_out);
    if (memo.valid && memo_scratch == memo.key)
      return launch_decode(memo.ncb, memo.ndirect, memo.norder, memo.o_rows, memo.o_map, memo.o_tbs, memo.e_base,
                           memo.specs, ntb, maxh, d_ret, memo.derm_max_ne);
    memo.valid = false;
    {
      hipError_t re;
      h_blk = (uint8_t *)blk_ring.acquire(&re);
      HIPCHK(re);
    }
    // ---- host: segmentation, CB list in TB order, groups by (K, CRC) ----
    uint32_t ncb = 0, max_n = 0;
    rec_tb.resize(cap);
    cb_key.resize(cap);
    const int16_t *e_base = nullptr; // the records' LLR offsets are relative to the lowest TB pointer
    for (uint32_t b = 0; b < ntb; b++)
      if (e_ptr[b] && (!e_base || e_ptr[b] < e_base)) e_base = e_ptr[b];
    for (uint32_t b = 0; b < ntb; b++) {
      const srsgpu_dlsch_tb_t &t = tb[b];
      TbItem &ti = h_tbs[b];
      memset(&ti, 0, sizeof(ti));
      ti.data = data_ptr[b];
      ti.ret = d_ret + b;
      ti.noi = d_noi_out + b;
      Segm s;
      if (t.softbuffer >= nslots || t.rv > 3 || t.Qm == 0 || segm(t.tbs, s)) {
        fprintf(stderr, "srsgpu: invalid transport block %u (tbs=%u rv=%u Qm=%u softbuffer=%u)\n", b,
                t.tbs, t.rv, t.Qm, t.softbuffer);
        return -1;
      }
      if (s.tbs == 0 || s.C == 0) { // sch.c:451-453
        ti.preset_ret = 0;
        continue;
      }
      if (s.F || s.C > max_cb) { // sch.c:455-463
        fprintf(stderr, s.F ? "Error filler bits are not supported. Use standard TBS\n"
                            : "Error number of CB (%d) exceeds soft buffer size (%d CBs)\n",
                s.C, max_cb);
        ti.preset_ret = -2;
        continue;
      }
      if (ncb + s.C > cap) {
        fprintf(stderr, "srsgpu: code blocks of this call exceed the capacity %u\n", cap);
        return -1;
      }
      if (llr8 && (auto_subblocks_8bit(s.K1) == 8 || (s.C2 && auto_subblocks_8bit(s.K2) == 8))) {
        // 400 < K <= 800: the reference's 8-bit AUTO choice feeds a 16-bit window 3K+12 converted
        // values of a 3(K+32)+12 sub-block row (turbodecoder.c:439-459), the rest being whatever
        // its conversion buffer last held: no defined result to reproduce
        fprintf(stderr, "srsgpu: 8-bit LLRs with code block size %u have no defined decode "
                        "(turbodecoder.c:439-459)\n", auto_subblocks_8bit(s.K1) == 8 ? s.K1 : s.K2);
        ti.preset_ret = -2;
        continue;
      }
      ti.tbs = s.tbs;
      ti.C = s.C;
      ti.C1 = s.C1;
      ti.K1 = s.K1;
      ti.K2 = s.K2;
      ti.first = ncb;
      ti.cb_crc = cbcrc + (size_t)t.softbuffer * max_cb;
      ti.saved = saved + (size_t)t.softbuffer * max_cb * 768;
      const uint32_t Gp = t.nof_e_bits / t.Qm;
      const uint32_t gamma = Gp % s.C;
      const uint32_t n_e = t.Qm * (Gp / s.C);
      // per distinct block size of the TB (K1, K2): de-RM table, row length, loader kind, group key
      struct PerK {
        uint32_t K, nsb;
        int tab;
        bool direct;
        uint32_t key;
      } pk[2];
      for (int w = 0; w < 2; w++) {
        const uint32_t K = w == 0 ? s.K1 : (s.C2 ? s.K2 : s.K1);
        PerK &q = pk[w];
        q.K = K;
        q.nsb = llr8 ? auto_subblocks_8bit(K) : auto_subblocks(K);
        q.tab = tab_of(K, t.rv, q.nsb);
        if (q.tab < 0) return -1;
        // the loader the decoder job will pick for this block (TdecEngine::derm_direct)
        const int r = resolve_impl(llr8 ? SRSGPU_TDEC_AUTO_8BIT : SRSLTE_TDEC_AUTO, K);
        q.direct = direct_derm && sb_input_for(llr8 ? SRSGPU_TDEC_AUTO_8BIT : SRSLTE_TDEC_AUTO, r) && impl_nb(r) % 8 == 0;
        q.key = group_key(K, s.C > 1 ? 0x1800063u : 0x1864CFBu, s.C > 1 ? K : s.tbs + 24);
      }
      const ptrdiff_t eo0 = e_ptr[b] - e_base;
      if (eo0 < 0 || eo0 + (ptrdiff_t)t.nof_e_bits > (ptrdiff_t)UINT32_MAX) {
        fprintf(stderr, "srsgpu: the LLRs of a call must lie within 2^32 elements of each other\n");
        return -1;
      }
      for (uint32_t i = 0; i < s.C; i++, ncb++) {
        const PerK &q = pk[i < s.C1 ? 0 : 1];
        const uint32_t K = q.K;
        uint32_t rp = i * n_e, ne = n_e;
        if (i > s.C - gamma) { // sch.c:339-342
          ne = n_e + t.Qm;
          rp = (s.C - gamma) * n_e + (i - (s.C - gamma)) * ne;
        }
        DermRec &it = rec_tb[ncb];
        it.e_off = (uint32_t)(eo0 + rp);
        it.ne = ne;
        it.N = (uint16_t)(3 * K + 12);
        it.tab = (uint16_t)q.tab;
        it.row = t.softbuffer * max_cb + i;
        it.rowlen = (uint16_t)(q.nsb ? 3 * (K + 32) + 12 : 3 * K + 12);
        it.w8 = llr8;
        it.tb = b;
        it.direct = q.direct;
        max_n = std::max(max_n, std::min(ne, 3 * K + 12));
        cb_key[ncb] = q.key;
      }
    }
    // code blocks grouped by (K, CRC) in key order, stable within a group (a counting sort: a call
    // holds thousands of blocks and a handful of keys)
    std::vector<uint32_t> order(ncb);
    {
      key_list.clear();
      for (uint32_t u = 0; u < ncb; u++) {
        const uint32_t k = cb_key[u];
        if (key_list.empty() || key_list.back().first != k) {
          auto f = std::find_if(key_list.begin(), key_list.end(), [&](const std::pair<uint32_t, uint32_t> &e) { return e.first == k; });
          if (f == key_list.end()) {
            key_list.push_back({k, 1});
            continue;
          }
          std::iter_swap(f, key_list.end() - 1); // the list's order does not matter until sorted below
        }
        key_list.back().second++;
      }
      std::sort(key_list.begin(), key_list.end());
      std::vector<uint32_t> &start = key_start;
      start.assign(key_list.size(), 0);
      for (size_t g = 1; g < key_list.size(); g++) start[g] = start[g - 1] + key_list[g - 1].second;
      for (uint32_t u = 0; u < ncb; u++) {
        const size_t g = std::lower_bound(key_list.begin(), key_list.end(), std::make_pair(cb_key[u], 0u)) - key_list.begin();
        order[start[g]++] = u;
      }
    }
    // records in decoder order (k_load_derm reads them by decoder position), packed with the row
    // pointers, the CB map and the TBs into one block: one upload
    const size_t o_rows = al(sizeof(DermRec) * ncb), o_map = o_rows + al(sizeof(int16_t *) * ncb),
                 o_tbs = o_map + al(4 * (size_t)ncb), o_end = o_tbs + sizeof(TbItem) * ntb;
    DermRec *b_rec = reinterpret_cast<DermRec *>(h_blk);
    const int16_t **b_rows = reinterpret_cast<const int16_t **>(h_blk + o_rows);
    uint32_t *b_map = reinterpret_cast<uint32_t *>(h_blk + o_map);
    uint32_t ndirect = 0;
    tdec.derm_max_ne = 0;
    for (uint32_t p = 0; p < order.size(); p++) {
      const uint32_t u = order[p];
      b_map[u] = p;
      b_rec[p] = rec_tb[u];
      b_rec[p].pos = p;
      b_rows[p] = soft + (size_t)b_rec[p].row * SRSGPU_SOFTBUFFER_SIZE;
      if (b_rec[p].direct) {
        ndirect++;
        tdec.derm_max_ne = std::max(tdec.derm_max_ne, b_rec[p].ne);
      }
    }
    memcpy(h_blk + o_tbs, h_tbs, sizeof(TbItem) * ntb);
    // ---- device ----
    HIPCHK(blk_ring.upload(d_blk, h_blk, o_end, st));
    HIPCHK(blk_ring.mark(st));
    // one decoder job over all (K, CRC) groups: one launch per decoder variant and half-iteration
    std::vector<TdSpec> specs;
    for (uint32_t g = 0, p0 = 0; g < key_list.size(); g++) {
      uint32_t K, poly, crclen;
      group_unkey(key_list[g].first, K, poly, crclen);
      specs.push_back(TdSpec{K, key_list[g].second, poly, crclen, p0});
      p0 += key_list[g].second;
    }
    const int r = launch_decode(ncb, ndirect, (uint32_t)order.size(), o_rows, o_map, o_tbs, e_base, specs, ntb, maxh,
                                d_ret, tdec.derm_max_ne);
    if (!r) {
      memo.key.swap(memo_scratch);
      memo.ncb = ncb;
      memo.ndirect = ndirect;
      memo.norder = (uint32_t)order.size();
      memo.o_rows = o_rows;
      memo.o_map = o_map;
      memo.o_tbs = o_tbs;
      memo.e_base = e_base;
      memo.specs = specs;
      memo.derm_max_ne = tdec.derm_max_ne;
      memo.valid = true;
    }
    return r;
  }

  // the device part of decode() on the descriptor block in d_blk
  int launch_decode(uint32_t ncb, uint32_t ndirect, uint32_t norder, size_t o_rows, size_t o_map, size_t o_tbs,
                    const int16_t *e_base, const std::vector<TdSpec> &specs, uint32_t ntb, uint32_t maxh,
                    int32_t *d_ret, uint32_t derm_max_ne) {
    tdec.derm_max_ne = derm_max_ne;
    last_ncb = ncb;
    const TbItem *d_tbs_c = reinterpret_cast<const TbItem *>(d_blk + o_tbs);
    const uint32_t *d_map_c = reinterpret_cast<const uint32_t *>(d_blk + o_map);
    const int16_t *const *d_rows_c = reinterpret_cast<const int16_t *const *>(d_blk + o_rows);
    const DermCall dc{reinterpret_cast<const DermRec *>(d_blk), d_tabs, e_base, soft, cbcrc, fresh, d_ret};
    if (ndirect) HIPCHK(launch_derm_flags(dc, (int)ncb, d_init, d_late, st));
    if (ndirect < ncb) {
      ProfScope ps("k_derm", st);
      HIPCHK(launch_derm(dc, (int)ncb, d_init, st));
    }
    // the epilogue makes the bytes of the blocks the fused early stop ended (no k_es_bytes) and the
    // rows of failed TBs (no k_derm_late) itself, unless SRSGPU_EPILOGUE=split (A/B) or a TB may hold
    // more blocks than it has LDS slots for
    tdec.defer_bytes = fused_epilogue && max_cb <= 32;
    tdec.bytes_deferred = false;
    if (!specs.empty() &&
        tdec.decode_multi(llr8 ? SRSGPU_TDEC_AUTO_8BIT : SRSLTE_TDEC_AUTO, 1, specs, norder, nullptr, 0,
                          d_rows_c, 16, d_init, maxh, d_dec, 768, d_ok, d_noi, fixed, ndirect ? &dc : nullptr))
      return -1;
    // the epilogue on the stream the decoder job ended on (the tail stream when it split)
    const hipStream_t es = tdec.st;
    tdec.st = st;
    FzSrc fz;
    if (tdec.bytes_deferred) fz = FzSrc{tdec.d_groups, (int)tdec.groups.size(), tdec.Dfz, tdec.cb_end};
    const bool inline_rows = ndirect && fused_epilogue;
    {
      ProfScope ps("k_tb_finish", es);
      HIPCHK(launch_tb_finish(d_tbs_c, (int)ntb, d_map_c, d_dec, 768, d_ok, d_init, d_noi, d_crc_a, es,
                              ndirect ? dc : DermCall{}, ndirect && !inline_rows ? d_late : nullptr, fz, inline_rows));
    }
    if (ndirect && !inline_rows) { // rows of the direct blocks of failed TBs, for the retransmission
      ProfScope ps("k_rows_late", es); // k_derm_late
      HIPCHK(launch_derm_late(dc, (int)ncb, d_late, es));
    }
    if (es != st) {
      if (!ev_tail) HIPCHK(hipEventCreateWithFlags(&ev_tail, hipEventDisableTiming));
      HIPCHK(hipEventRecord(ev_tail, es));
      tail_pending = true;
    }
    return 0;
  }
};

} // namespace srsgpu

using srsgpu::DlschEngine;
using srsgpu::ProfScope;
using srsgpu::UlItem;
using srsgpu::launch_uci_ack_ri;
using srsgpu::launch_uci_cqi;
using srsgpu::launch_ulsch_deinterleave;

struct srsgpu_dlsch {
  DlschEngine e;
};

extern "C" {

int srsgpu_dlsch_create(srsgpu_dlsch_t **q, uint32_t nslots, uint32_t max_cb, uint32_t cap) {
  if (!q) return -1;
  auto *d = new srsgpu_dlsch();
  if (d->e.create(nslots, max_cb, cap)) {
    d->e.destroy();
    delete d;
    *q = nullptr;
    return -1;
  }
  *q = d;
  return 0;
}

void srsgpu_dlsch_destroy(srsgpu_dlsch_t *q) {
  if (!q) return;
  q->e.destroy();
  delete q;
}

void srsgpu_dlsch_set_stream(srsgpu_dlsch_t *q, void *s) {
  if (!q) return;
  q->e.st = (hipStream_t)s;
  (void)q->e.join_tail(); // a pending tail: the new stream waits for it
}

int srsgpu_dlsch_set_tail_stream(srsgpu_dlsch_t *q, void *s) {
  if (!q || q->e.join_tail()) return -1;
  q->e.tail_st = (hipStream_t)s;
  return 0;
}

int srsgpu_dlsch_join_tail(srsgpu_dlsch_t *q) { return q ? q->e.join_tail() : -1; }

int srsgpu_dlsch_cb_halfits(srsgpu_dlsch_t *q, uint32_t *out, uint32_t n) {
  if (!q || (!out && n) || q->e.join_tail()) return -1;
  const uint32_t m = std::min(n, q->e.last_ncb);
  if (m && (hipMemcpyAsync(out, q->e.d_noi, sizeof(uint32_t) * m, hipMemcpyDeviceToHost, q->e.st) != hipSuccess ||
            hipStreamSynchronize(q->e.st) != hipSuccess))
    return -1;
  return (int)q->e.last_ncb;
}

int srsgpu_dlsch_softbuffer_reset(srsgpu_dlsch_t *q, uint32_t slot) {
  return q && !q->e.join_tail() ? q->e.reset(slot, 1, q->e.max_cb) : -1;
}

int srsgpu_dlsch_softbuffer_reset_range(srsgpu_dlsch_t *q, uint32_t first, uint32_t count) {
  return q && !q->e.join_tail() ? q->e.reset(first, count, q->e.max_cb) : -1;
}

int srsgpu_dlsch_softbuffer_reset_list(srsgpu_dlsch_t *q, const uint32_t *slots, const uint32_t *ncb, uint32_t n) {
  if (!q || (!slots && n) || q->e.join_tail()) return -1;
  return q->e.reset_list(slots, ncb, n);
}

int srsgpu_dlsch_softbuffer_reset_tbs(srsgpu_dlsch_t *q, uint32_t slot, uint32_t tbs) {
  if (!q || q->e.join_tail()) return -1;
  const uint32_t n = (tbs + 24) / 6120 + 1; // softbuffer.c:113-116
  return q->e.reset(slot, 1, n < q->e.max_cb ? n : q->e.max_cb);
}

int srsgpu_dlsch_decode_dev(srsgpu_dlsch_t *q, const srsgpu_dlsch_tb_t *tb, uint32_t ntb,
                            const int16_t *d_e, uint8_t *d_data, uint32_t maxh, int32_t *d_ret,
                            uint32_t *d_noi) {
  if (!q || (!tb && ntb) || !d_e || !d_data || !d_ret || !d_noi) return -1;
  if (ntb == 0) return 0;
  std::vector<const int16_t *> e(ntb);
  std::vector<uint8_t *> d(ntb);
  for (uint32_t i = 0; i < ntb; i++) {
    e[i] = d_e + tb[i].e_offset;
    d[i] = d_data + tb[i].data_offset;
  }
  return q->e.decode(tb, ntb, e.data(), d.data(), maxh, d_ret, d_noi);
}

int srsgpu_dlsch_decode_out_dev(srsgpu_dlsch_t *q, const srsgpu_dlsch_tb_t *tb, uint32_t ntb, const int16_t *d_e,
                                uint8_t *const *d_out, uint32_t maxh, int32_t *d_ret, uint32_t *d_noi) {
  if (!q || (!tb && ntb) || !d_e || (!d_out && ntb) || !d_ret || !d_noi) return -1;
  if (ntb == 0) return 0;
  std::vector<const int16_t *> e(ntb);
  for (uint32_t i = 0; i < ntb; i++) {
    if (!d_out[i]) return -1;
    e[i] = d_e + tb[i].e_offset;
  }
  return q->e.decode(tb, ntb, e.data(), d_out, maxh, d_ret, d_noi);
}

// srslte_ulsch_decode (sch.c:883-889 -> srslte_ulsch_uci_decode :944-985 without UCI): the channel
// deinterleaver of every TB (ulsch_deinterleave, :860-881) into the caller's g bits, then decode_tb
// on them through the DL-SCH path (the reference's decode_tb is the same function for both links)
// the channel deinterleaver launch of ntb UL-SCH TBs (q -> g, sch.c:550-568, 860-881)
static int ulsch_deinterleave(srsgpu_dlsch_t *q, const srsgpu_ulsch_tb_t *tb, uint32_t ntb, const int16_t *d_q,
                              int16_t *d_g) {
  DlschEngine &E = q->e;
  if (ntb > E.cap || E.join_tail()) return -1;
  for (uint32_t i = 0; i < ntb; i++) {
    const uint32_t Qm = tb[i].Qm, ns = tb[i].nof_symb;
    if ((Qm != 2 && Qm != 4 && Qm != 6) || ns == 0 || tb[i].nof_bits % (Qm * ns)) {
      fprintf(stderr, "srsgpu: UL-SCH TB %u: %u coded bits are not a %u x %u-column matrix\n", i,
              tb[i].nof_bits, Qm, ns);
      return -1;
    }
  }
  if (!E.h_ul) {
    HIPCHK(hipHostMalloc(&E.h_ul, sizeof(UlItem) * E.cap));
    HIPCHK(hipMalloc(&E.d_ul, sizeof(UlItem) * E.cap));
  }
  if (E.staged_pending) HIPCHK(hipEventSynchronize(E.staged));
  uint32_t max_bits = 0;
  for (uint32_t i = 0; i < ntb; i++) {
    const uint32_t Qm = tb[i].Qm, cols = tb[i].nof_symb;
    E.h_ul[i] = UlItem{tb[i].q_offset, tb[i].nof_bits / Qm / cols, cols, Qm};
    max_bits = std::max(max_bits, tb[i].nof_bits);
  }
  HIPCHK(hipMemcpyAsync(E.d_ul, E.h_ul, sizeof(UlItem) * ntb, hipMemcpyHostToDevice, E.st));
  {
    ProfScope ps("k_ulsch_deinterleave", E.st);
    HIPCHK(launch_ulsch_deinterleave(E.d_ul, (int)ntb, max_bits, d_q, d_g, E.st));
  }
  // the next staging of E.h_ul (here or in decode()) waits for this copy
  HIPCHK(hipEventRecord(E.staged, E.st));
  E.staged_pending = true;
  return 0;
}

int srsgpu_ulsch_deinterleave_dev(srsgpu_dlsch_t *q, const srsgpu_ulsch_tb_t *tb, uint32_t ntb, const int16_t *d_q,
                                  int16_t *d_g) {
  if (!q || (!tb && ntb) || !d_q || !d_g) return -1;
  if (ntb == 0) return 0;
  return ulsch_deinterleave(q, tb, ntb, d_q, d_g);
}

int srsgpu_ulsch_decode_dev(srsgpu_dlsch_t *q, const srsgpu_ulsch_tb_t *tb, uint32_t ntb,
                            const int16_t *d_q, int16_t *d_g, uint8_t *d_data, uint32_t maxh,
                            int32_t *d_ret, uint32_t *d_noi) {
  if (!q || (!tb && ntb) || !d_q || !d_g || !d_data || !d_ret || !d_noi) return -1;
  if (ntb == 0) return 0;
  if (ulsch_deinterleave(q, tb, ntb, d_q, d_g)) return -1;
  std::vector<srsgpu_dlsch_tb_t> dl(ntb);
  std::vector<const int16_t *> e(ntb);
  std::vector<uint8_t *> d(ntb);
  for (uint32_t i = 0; i < ntb; i++) {
    // G = nb_q / Qm - Q'_ri - Q'_cqi with no UCI: every coded bit is data (sch.c:976-979)
    dl[i] = srsgpu_dlsch_tb_t{tb[i].tbs, tb[i].rv, tb[i].Qm, tb[i].nof_bits, tb[i].softbuffer,
                              tb[i].q_offset, tb[i].data_offset};
    e[i] = d_g + tb[i].q_offset;
    d[i] = d_data + tb[i].data_offset;
  }
  return q->e.decode(dl.data(), ntb, e.data(), d.data(), maxh, d_ret, d_noi);
}

// srsgpu_ulsch_uci_decode_dev: Q' of each UCI kind on the host (uci.c:270-290, 548-572, in the
// reference's float order), then k_uci_ack_ri on the scrambled q bits, the deinterleaver in its UCI
// mode, k_uci_cqi (g[0], CQI, ret / noi of TBs without data) and decode_tb of the data part.
static uint32_t uci_qp_ack_ri(uint32_t O, uint32_t O_cqi, float beta, uint32_t K, uint32_t M_sc, uint32_t M_sc_init,
                              uint32_t nsymb) {
  if (K == 0) K = O_cqi <= 11 ? O_cqi : O_cqi + 8;
  const uint32_t x = (uint32_t)ceilf((float)O * M_sc_init * nsymb * beta / K);
  return std::min(x, 4 * M_sc);
}

int srsgpu_ulsch_uci_decode_dev(srsgpu_dlsch_t *q, const srsgpu_ulsch_tb_t *tb, const srsgpu_uci_cfg_t *uci,
                                uint32_t ntb, const int16_t *d_q, const uint8_t *d_c, int16_t *d_g, uint8_t *d_data,
                                uint32_t maxh, int32_t *d_ret, uint32_t *d_noi, srsgpu_uci_result_t *d_uci) {
  if (!q || (!tb && ntb) || (!uci && ntb) || !d_q || !d_c || !d_g || !d_data || !d_ret || !d_noi || !d_uci) return -1;
  if (ntb == 0) return 0;
  DlschEngine &E = q->e;
  if (ntb > E.cap || E.join_tail()) return -1;
  std::vector<srsgpu::UlItem> it(ntb);
  uint32_t max_bits = 0;
  for (uint32_t i = 0; i < ntb; i++) {
    const srsgpu_ulsch_tb_t &t = tb[i];
    const srsgpu_uci_cfg_t &u = uci[i];
    const uint32_t Qm = t.Qm, ns = t.nof_symb;
    if ((Qm != 2 && Qm != 4 && Qm != 6) || ns < 11 || t.nof_bits % (Qm * ns) || u.O_ack > 2 || u.O_ri > 2 ||
        u.O_cqi > SRSGPU_UCI_MAX_CQI_BITS || u.I_offset_ack > 15 || u.I_offset_ri > 15 || u.I_offset_cqi > 15 ||
        !u.M_sc || t.nof_bits / Qm != u.M_sc * ns) {
      fprintf(stderr, "srsgpu: invalid UCI PUSCH configuration for TB %u\n", i);
      return -1;
    }
    srsgpu::Segm sg;
    if (srsgpu::segm(t.tbs, sg)) return -1;
    const uint32_t K = sg.C1 * sg.K1 + sg.C2 * sg.K2;
    const float bcqi = SRSGPU_BETA_CQI[u.I_offset_cqi];
    srsgpu::UlItem &x = it[i];
    x = srsgpu::UlItem{t.q_offset, t.nof_bits / Qm / ns, ns, Qm};
    x.uci = 1;
    x.O_ack = u.O_ack;
    x.O_ri = u.O_ri;
    x.O_cqi = u.O_cqi;
    x.tbs = t.tbs;
    x.c_offset = u.c_offset;
    if (u.O_ack) { // sch.c:906-910: beta / beta_cqi without data
      float beta = SRSGPU_BETA_ACK[u.I_offset_ack];
      if (t.tbs == 0) beta /= bcqi;
      if (beta < 0) {
        fprintf(stderr, "Error beta is reserved\n");
        return -1;
      }
      x.Q_ack = uci_qp_ack_ri(u.O_ack, u.O_cqi, beta, K, u.M_sc, u.M_sc_init, ns);
    }
    if (u.O_ri) {
      float beta = SRSGPU_BETA_RI[u.I_offset_ri];
      if (t.tbs == 0) beta /= bcqi;
      if (beta < 0) {
        fprintf(stderr, "Error beta is reserved\n");
        return -1;
      }
      x.Q_ri = uci_qp_ack_ri(u.O_ri, u.O_cqi, beta, K, u.M_sc, u.M_sc_init, ns);
    }
    if (u.O_cqi) { // uci.c:270-290
      if (bcqi < 0) {
        fprintf(stderr, "Error beta is reserved\n");
        return -1;
      }
      const uint32_t L = u.O_cqi < 11 ? 0 : 8;
      uint32_t v = 999999;
      if (K > 0) v = (uint32_t)ceilf((float)(u.O_cqi + L) * u.M_sc_init * ns * bcqi / K);
      x.Q_cqi = std::min(v, u.M_sc * ns - x.Q_ri);
    }
    if (x.Q_ack * Qm > 12 * 288 || x.Q_ri * Qm > 12 * 288) { // srslte_sch_t.ack_ri_bits[12 * 288] (sch.h:70)
      fprintf(stderr, "srsgpu: HARQ-ACK / RI of TB %u exceed the reference's 3456 positions\n", i);
      return -1;
    }
    if (x.Q_ri + x.Q_cqi >= t.nof_bits / Qm && t.tbs) {
      fprintf(stderr, "srsgpu: UCI leaves no data symbols in TB %u\n", i);
      return -1;
    }
    max_bits = std::max(max_bits, t.nof_bits);
  }
  if (!E.h_ul) {
    HIPCHK(hipHostMalloc(&E.h_ul, sizeof(UlItem) * E.cap));
    HIPCHK(hipMalloc(&E.d_ul, sizeof(UlItem) * E.cap));
  }
  if (E.staged_pending) HIPCHK(hipEventSynchronize(E.staged));
  memcpy(E.h_ul, it.data(), sizeof(srsgpu::UlItem) * ntb);
  HIPCHK(hipMemcpyAsync(E.d_ul, E.h_ul, sizeof(srsgpu::UlItem) * ntb, hipMemcpyHostToDevice, E.st));
  HIPCHK(hipEventRecord(E.staged, E.st));
  E.staged_pending = true;
  {
    ProfScope ps("k_uci", E.st);
    HIPCHK(launch_uci_ack_ri(E.d_ul, (int)ntb, d_q, d_c, d_uci, E.st));
    HIPCHK(launch_ulsch_deinterleave(E.d_ul, (int)ntb, max_bits, d_q, d_g, E.st, d_c));
    HIPCHK(launch_uci_cqi(E.d_ul, (int)ntb, d_q, d_c, d_g, d_uci, d_ret, d_noi, E.st));
  }
  // decode_tb of the data: G = H' - Q'_ri - Q'_cqi symbols after the CQI (sch.c:972-983)
  std::vector<srsgpu_dlsch_tb_t> dl;
  std::vector<const int16_t *> e;
  std::vector<uint8_t *> d;
  std::vector<uint32_t> idx;
  for (uint32_t i = 0; i < ntb; i++) {
    if (!tb[i].tbs) continue;
    const uint32_t Qm = tb[i].Qm, G = tb[i].nof_bits / Qm - it[i].Q_ri - it[i].Q_cqi;
    dl.push_back(srsgpu_dlsch_tb_t{tb[i].tbs, tb[i].rv, Qm, G * Qm, tb[i].softbuffer, 0, 0});
    e.push_back(d_g + tb[i].q_offset + (size_t)it[i].Q_cqi * Qm);
    d.push_back(d_data + tb[i].data_offset);
    idx.push_back(i);
  }
  if (dl.empty()) return 0;
  // the data TBs' results land at their own indices: decode into a contiguous run, then scatter
  // only when some TB carries no data
  if (dl.size() == ntb) return q->e.decode(dl.data(), (uint32_t)dl.size(), e.data(), d.data(), maxh, d_ret, d_noi);
  if (!E.d_uci_ret) HIPCHK(hipMalloc(&E.d_uci_ret, sizeof(int32_t) * 2 * E.cap));
  int32_t *r_tmp = E.d_uci_ret;
  uint32_t *n_tmp = (uint32_t *)(r_tmp + E.cap);
  if (q->e.decode(dl.data(), (uint32_t)dl.size(), e.data(), d.data(), maxh, r_tmp, n_tmp) || E.join_tail())
    return -1; // (the scatter below reads what the tail wrote)
  for (size_t k = 0; k < dl.size(); k++) {
    HIPCHK(hipMemcpyAsync(d_ret + idx[k], r_tmp + k, 4, hipMemcpyDeviceToDevice, E.st));
    HIPCHK(hipMemcpyAsync(d_noi + idx[k], n_tmp + k, 4, hipMemcpyDeviceToDevice, E.st));
  }
  return 0;
}

int srsgpu_dlsch_decode(srsgpu_dlsch_t *q, const srsgpu_dlsch_tb_t *tb, uint32_t ntb,
                        const int16_t *const *e_bits, uint8_t *const *data, uint32_t maxh,
                        int32_t *ret, uint32_t *noi) {
  if (!q || (!tb && ntb) || !e_bits || !data || !ret || !noi) return -1;
  if (ntb == 0) return 0;
  DlschEngine &E = q->e;
  if (ntb > E.cap || E.join_tail()) return -1;
  size_t elen = 0, dlen = 0;
  for (uint32_t i = 0; i < ntb; i++) {
    elen += tb[i].nof_e_bits;
    dlen += SRSGPU_DLSCH_DATA_LEN(tb[i].tbs);
  }
  if (elen > E.e_stage_len) {
    if (E.e_stage) (void)hipFree(E.e_stage);
    E.e_stage = nullptr;
    HIPCHK(hipMalloc(&E.e_stage, elen * 2 + 64));
    E.e_stage_len = elen;
  }
  if (dlen > E.data_stage_len) {
    if (E.data_stage) (void)hipFree(E.data_stage);
    E.data_stage = nullptr;
    HIPCHK(hipMalloc(&E.data_stage, dlen + 64));
    E.data_stage_len = dlen;
  }
  std::vector<srsgpu_dlsch_tb_t> t(tb, tb + ntb);
  size_t eo = 0, dof = 0;
  for (uint32_t i = 0; i < ntb; i++) {
    t[i].e_offset = eo;
    t[i].data_offset = dof;
    if (tb[i].nof_e_bits)
      HIPCHK(hipMemcpyAsync(E.e_stage + eo, e_bits[i], (size_t)tb[i].nof_e_bits * 2,
                            hipMemcpyHostToDevice, E.st));
    eo += tb[i].nof_e_bits;
    dof += SRSGPU_DLSCH_DATA_LEN(tb[i].tbs);
  }
  HIPCHK(hipMemsetAsync(E.data_stage, 0, dlen, E.st));
  if (srsgpu_dlsch_decode_dev(q, t.data(), ntb, E.e_stage, E.data_stage, maxh, E.d_ret_stage,
                              E.d_noi_stage) ||
      E.join_tail()) // the copies below read what the tail wrote
    return -1;
  for (uint32_t i = 0; i < ntb; i++)
    HIPCHK(hipMemcpyAsync(data[i], E.data_stage + t[i].data_offset, SRSGPU_DLSCH_DATA_LEN(tb[i].tbs),
                          hipMemcpyDeviceToHost, E.st));
  HIPCHK(hipMemcpyAsync(ret, E.d_ret_stage, sizeof(int32_t) * ntb, hipMemcpyDeviceToHost, E.st));
  HIPCHK(hipMemcpyAsync(noi, E.d_noi_stage, sizeof(uint32_t) * ntb, hipMemcpyDeviceToHost, E.st));
  HIPCHK(hipStreamSynchronize(E.st));
  return 0;
}

int srsgpu_dlsch_softbuffer_read(srsgpu_dlsch_t *q, uint32_t slot, int16_t *rows, uint8_t *cb_crc) {
  if (!q || slot >= q->e.nslots) return -1;
  DlschEngine &E = q->e;
  if (E.join_tail()) return -1;
  std::vector<uint8_t> fr(E.max_cb);
  HIPCHK(hipMemcpyAsync(fr.data(), E.fresh + (size_t)slot * E.max_cb, E.max_cb, hipMemcpyDeviceToHost, E.st));
  if (rows)
    HIPCHK(hipMemcpyAsync(rows, E.row(slot, 0), (size_t)E.max_cb * SRSGPU_SOFTBUFFER_SIZE * 2,
                          hipMemcpyDeviceToHost, E.st));
  HIPCHK(hipStreamSynchronize(E.st));
  for (uint32_t i = 0; rows && i < E.max_cb; i++) // lazily reset rows read as zero
    if (fr[i]) memset(rows + (size_t)i * SRSGPU_SOFTBUFFER_SIZE, 0, SRSGPU_SOFTBUFFER_SIZE * 2);
  if (cb_crc)
    HIPCHK(hipMemcpyAsync(cb_crc, E.cbcrc + (size_t)slot * E.max_cb, E.max_cb, hipMemcpyDeviceToHost,
                          E.st));
  HIPCHK(hipStreamSynchronize(E.st));
  return 0;
}

int srsgpu_dlsch_encode_dev(srsgpu_dlsch_t *q, const srsgpu_dlsch_tb_t *tb, uint32_t nof_tb,
                            const uint8_t *d_data, uint8_t *d_e_bits) {
  if (!q || (!tb && nof_tb) || !d_data || !d_e_bits || q->e.join_tail()) return -1;
  return q->e.encode(tb, nof_tb, d_data, d_e_bits);
}

static int rm_rx_dev(srsgpu_dlsch_t *q, const int16_t *d_in, int16_t *d_out, uint32_t in_len,
                     uint32_t K, uint32_t rv, uint32_t nsb, bool w8) {
  if (!q || !d_in || !d_out || rv > 3 || srsgpu::cb_index(K) < 0) return -1;
  DlschEngine &E = q->e;
  if (E.staged_pending) HIPCHK(hipEventSynchronize(E.staged));
  const uint16_t *tab = E.table(K, rv, nsb);
  if (!tab) return -1;
  srsgpu::DermItem &it = E.h_items[0];
  it.e = d_in;
  it.ne = in_len;
  it.N = 3 * K + 12;
  it.table = tab;
  it.inv = nullptr;
  it.row = d_out;
  it.cb_crc = nullptr;
  it.pos = 0;
  it.fresh = nullptr;
  it.w8 = w8;
  HIPCHK(hipMemcpyAsync(E.d_items, E.h_items, sizeof(srsgpu::DermItem), hipMemcpyHostToDevice, E.st));
  HIPCHK(hipEventRecord(E.staged, E.st));
  E.staged_pending = true;
  HIPCHK(srsgpu::launch_derm_rmw(E.d_items, std::min(in_len, 3 * K + 12), E.st));
  return 0;
}

int srsgpu_rm_turbo_rx_dev(srsgpu_dlsch_t *q, const int16_t *d_in, int16_t *d_out, uint32_t in_len,
                           uint32_t K, uint32_t rv, int sb_layout) {
  return rm_rx_dev(q, d_in, d_out, in_len, K, rv, sb_layout ? srsgpu::auto_subblocks(K) : 0, false);
}

int srsgpu_rm_turbo_rx_8bit_dev(srsgpu_dlsch_t *q, const int16_t *d_in, int16_t *d_out,
                                uint32_t in_len, uint32_t K, uint32_t rv) {
  return rm_rx_dev(q, d_in, d_out, in_len, K, rv, srsgpu::auto_subblocks_8bit(K), true);
}

void srsgpu_dlsch_set_early_stop(srsgpu_dlsch_t *q, int enable) {
  if (q) q->e.fixed = enable == 0;
}

void srsgpu_dlsch_set_llr_8bit(srsgpu_dlsch_t *q, int enable) {
  if (q) q->e.llr8 = enable != 0;
}

void srsgpu_dlsch_set_direct_derm(srsgpu_dlsch_t *q, int enable) {
  if (q) q->e.direct_derm = enable != 0;
}

} // extern "C"
