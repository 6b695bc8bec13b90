// Host side of the MI355X PDSCH receiver (include/srsgpu/pdsch_batch.h): RE maps, scrambling
// sequence tables, per-call descriptors; the compute is pdsch_kernels.hip + the DL-SCH engine.
#include <hip/hip_runtime.h>

#include <map>
#include <unordered_map>
#include <stdio.h>
#include <string.h>
#include <string>
#include <vector>

#include "feedback_kernels.h"
#include "host_ring.h"
#include "pdsch_kernels.h"
#include "srsgpu/pdsch_batch.h"
#include "tdec_engine.h"

namespace srsgpu {

// ------------------------------------------------------------------ RE map ----
// Gather order of srslte_pdsch_cp in read mode (pdsch.c:95-234): slots, OFDM symbols (7 per slot,
// 6 with extended CP), allocated PRBs; PSS/SSS (subframes 0/5, slot 0, last two symbols) and PBCH (subframe 0, slot 1, first 4
// symbols) cut the 6 (or, for odd nof_prb, 7) central PRBs; in symbols carrying CRS the
// reference REs are skipped with prb_cp_ref's interval walk (prb_dl.c:51-82).
static void re_map(const srsgpu_cell_t &c, uint32_t lstart_grant, uint32_t sf_idx,
                   const uint8_t prb[2][110], std::vector<uint32_t> &m) {
  const uint32_t N = c.nof_prb, ns = c.cp == 1 ? 6 : 7, nref = c.nof_ports == 1 ? 2 : 4;
  m.clear();
  auto refsym = [&](uint32_t l) { return (l == 1 && c.nof_ports == 4) || l == 0 || l == ns - 3; };
  // prb_cp_ref: 'offset' REs, then (intervals-1) x [skip 1, take ri], then [skip 1, take ri-offset]
  auto take_ref = [&](uint32_t &in, int offset, int intervals) {
    const int ri = 12 / (int)nref - 1;
    for (int j = 0; j < offset; j++) m.push_back(in++);
    for (int i = 0; i < intervals - 1; i++) {
      in++;
      for (int j = 0; j < ri; j++) m.push_back(in++);
    }
    if (ri - offset > 0) {
      in++;
      for (int j = 0; j < ri - offset; j++) m.push_back(in++);
    }
  };
  uint32_t offset = 0;
  for (uint32_t s = 0; s < 2; s++)
    for (uint32_t l = 0; l < ns; l++)
      for (uint32_t n = 0; n < N; n++) {
        if (!prb[s][n]) continue;
        uint32_t lst = s == 0 ? lstart_grant : 0, lend = ns;
        const bool centre = n >= N / 2 - 3 && n < N / 2 + 3 + (N % 2);
        const bool sss = s == 0 && (sf_idx == 0 || sf_idx == 5) && centre;
        const bool pbch = s == 1 && sf_idx == 0 && centre;
        if (sss) lend = ns - 2;
        if (pbch) lst = 4;
        uint32_t in = ((l + s * ns) * N + n) * 12;
        if (l >= lst && l < lend) {
          if (refsym(l)) {
            offset = nref == 2 ? (l == 0 ? c.id % 6 : (c.id + 3) % 6) : c.id % 3;
            take_ref(in, (int)offset, (int)nref);
          } else {
            for (int j = 0; j < 12; j++) m.push_back(in++);
          }
        }
        if ((N % 2) && ((pbch && l < lst) || (sss && l >= lend))) {
          if (n == N / 2 - 3 || n == N / 2 + 3) {
            if (n == N / 2 + 3) in += 6;
            if (refsym(l))
              take_ref(in, (int)offset, (int)nref / 2);
            else
              for (int j = 0; j < 6; j++) m.push_back(in++);
          }
        }
      }
}

static const int kQm[4] = {1, 2, 4, 6};
// The Qm srslte_dlsch_encode2 / srslte_dlsch_decode2 hand to encode_tb / decode_tb (sch.c:506-545):
// the modulation order times Nl = 2 when the layers outnumber the TBs (transmit diversity over 2 or 4
// layers), which changes how the codeword's E bits split over the code blocks (36.212 5.1.4.1.2)
static uint32_t dlsch_qm(const srsgpu_pdsch_sf_t &s, uint32_t tb) {
  return (uint32_t)kQm[s.mod[tb]] * (s.mimo_type == SRSGPU_MIMO_TX_DIVERSITY ? 2u : 1u);
}

// ------------------------------------------------------------------ engine ----
struct PdschEngine {
  hipStream_t st = nullptr;
  srsgpu_cell_t cell{};
  uint32_t max_sf = 0;
  bool csi = false;
  bool llr8 = false; // srslte_pdsch_t.llr_is_8bit
  int ce_rows = 0;   // srsgpu_pdsch_set_ce_rows: 0 full estimate planes, 4 / 1 the chest's compact rows
  const float *noise_dev = nullptr; // per-subframe chest noise estimates (nof_rx_ant each)
  srsgpu_dlsch_t *dl = nullptr;
  // Gold tables: x1 and the 31 x2 basis sequences, bits 0 .. 32*words-1
  uint32_t gold_words = 0;
  uint32_t *d_x1 = nullptr, *d_x2b = nullptr;
  std::map<std::string, std::pair<uint32_t *, uint32_t>> maps; // device RE maps
  // per-call buffers
  GoldItem *h_gold = nullptr, *d_gold = nullptr;
  LlrItem *h_llr = nullptr, *d_llr = nullptr;
  srsgpu_dlsch_tb_t *h_tb = nullptr;
  uint32_t *d_c = nullptr;   // [max_sf][cwords]
  float *d_csi = nullptr;    // [max_sf][max_re]
  uint32_t *d_csimax = nullptr;
  int16_t *d_e = nullptr;    // [max_sf][max_bits]
  uint32_t max_re = 0, max_bits = 0, cwords = 0;
  // one scrambling sequence per distinct seed of a call (a UE's TBs use at most 10 subframe seeds per
  // codeword): the TBs that share a seed read the same words
  std::unordered_map<uint32_t, uint32_t> gold_slot;
  uint32_t ngold = 0, nper = 0;
  // Sequences kept across calls: a receiver sees a handful of seeds (RNTI x codeword x subframe; the
  // reference pre-generates them per user, pdsch.c:436-440), so the first GCACHE distinct seeds get a
  // full-length sequence generated once and reused by every later call (no k_gold launch and no item
  // upload when a call's seeds are all known). A seed first met in a call is generated by that call's
  // k_gold and becomes usable by later calls once the launch is enqueued (gold_commit); the cache is
  // cleared when the stream changes (the entries were made in another stream's order).
  static constexpr uint32_t GCACHE = 64;
  uint32_t *d_gcache = nullptr;
  std::unordered_map<uint32_t, uint32_t> gcache; // seed -> slot of d_gcache
  std::vector<std::pair<uint32_t, uint32_t>> gcache_new; // this call's additions (seed, slot)
  const uint32_t *gold(uint32_t seed, uint32_t len) {
    auto hit = gcache.find(seed);
    if (hit != gcache.end()) return d_gcache + (size_t)hit->second * cwords;
    auto it = gold_slot.find(seed);
    if (it == gold_slot.end()) {
      GoldItem &g = h_gold[ngold];
      g.seed = seed;
      const uint32_t slot = (uint32_t)(gcache.size() + gcache_new.size());
      if (d_gcache && slot < GCACHE) {
        g.len = max_bits;
        g.c = d_gcache + (size_t)slot * cwords;
        gcache_new.push_back({seed, slot});
      } else {
        g.len = len;
        g.c = d_c + (size_t)nper++ * cwords;
      }
      it = gold_slot.emplace(seed, ngold++).first;
    } else if (h_gold[it->second].len < len) {
      h_gold[it->second].len = len; // the sequence's prefix does not depend on its length
    }
    return h_gold[it->second].c;
  }
  void gold_reset() {
    gold_slot.clear();
    gcache_new.clear();
    ngold = nper = 0;
  }
  // after the call's k_gold is enqueued: its new full-length sequences serve later calls
  void gold_commit() {
    for (const auto &kv : gcache_new) gcache.emplace(kv.first, kv.second);
    gcache_new.clear();
  }
  // the call's generation (only sequences not already on the device)
  int gold_launch() {
    if (!ngold) return 0;
    HIPCHK(ring.upload(d_gold, h_gold, sizeof(GoldItem) * ngold, st));
    {
      ProfScope ps("k_gold", st);
      HIPCHK(launch_gold(d_gold, (int)ngold, gold_bits(), d_x1, d_x2b, gold_words, st));
    }
    gold_commit();
    return 0;
  }
  uint32_t gold_bits() const {
    uint32_t m = 0;
    for (uint32_t i = 0; i < ngold; i++) m = std::max(m, h_gold[i].len);
    return m;
  }
  // pinned per-call staging, one ring slot = [GoldItem x 2 max_sf][LlrItem x 2 max_sf][TxItem x max_sf];
  // h_gold / h_llr / h_tx point into the slot of the current call (host_ring.h)
  HostRing ring;
  int ring_take() {
    hipError_t e;
    uint8_t *b = (uint8_t *)ring.acquire(&e);
    if (e != hipSuccess) return -1;
    const uint32_t mtb = 2 * max_sf;
    h_gold = (GoldItem *)b;
    h_llr = (LlrItem *)(b + sizeof(GoldItem) * mtb);
    h_tx = (TxItem *)(b + (sizeof(GoldItem) + sizeof(LlrItem)) * mtb);
    return 0;
  }
  // TM3 / TM4 feedback items (lazily allocated; the host array is reused once its upload is done)
  FbItem *h_fb = nullptr, *d_fb = nullptr;
  hipEvent_t fb_staged = nullptr;
  bool fb_pending = false;
  // transmit side (lazily allocated)
  TxItem *h_tx = nullptr, *d_tx = nullptr;
  uint8_t *d_ebits = nullptr; // [2 max_sf][max_bits] coded bits
  float2 *d_mod = nullptr;    // constellation tables

  int create(const srsgpu_cell_t &c, uint32_t nsb, uint32_t max_cb, uint32_t msf) {
    if (c.nof_prb < 6 || c.nof_prb > 110 || c.id > 503 || !msf ||
        (c.nof_ports != 1 && c.nof_ports != 2 && c.nof_ports != 4) || c.nof_rx_ant < 1 ||
        c.nof_rx_ant > 2 || c.cp > 1) {
      fprintf(stderr, "srsgpu: invalid cell (nof_prb=%u id=%u ports=%u rx=%u)\n", c.nof_prb, c.id,
              c.nof_ports, c.nof_rx_ant);
      return -1;
    }
    cell = c;
    max_sf = msf;
    max_re = c.nof_prb * 12 * 14;
    max_bits = max_re * 6;
    cwords = (max_bits + 31) / 32 + 2;
    if (srsgpu_dlsch_create(&dl, nsb, max_cb, 2 * msf * max_cb)) return -1;
    // Gold tables (36.211 7.2): x1(n+31) = x1(n+3) + x1(n), x1 = 1,0,0..; x2 basis i: seed 1 << i
    gold_words = (1600 + max_bits + 64) / 32 + 2;
    const uint32_t nbits = gold_words * 32;
    std::vector<uint8_t> a(nbits + 31);
    std::vector<uint32_t> x1w(gold_words, 0), x2w((size_t)31 * gold_words, 0);
    a.assign(nbits + 31, 0);
    a[0] = 1;
    for (uint32_t n = 0; n < nbits; n++) a[n + 31] = (a[n + 3] + a[n]) & 1;
    for (uint32_t n = 0; n < nbits; n++) x1w[n / 32] |= (uint32_t)a[n] << (n % 32);
    for (int i = 0; i < 31; i++) {
      a.assign(nbits + 31, 0);
      a[i] = 1;
      for (uint32_t n = 0; n < nbits; n++) a[n + 31] = (a[n + 3] + a[n + 2] + a[n + 1] + a[n]) & 1;
      for (uint32_t n = 0; n < nbits; n++) x2w[(size_t)i * gold_words + n / 32] |= (uint32_t)a[n] << (n % 32);
    }
    HIPCHK(hipMalloc(&d_x1, x1w.size() * 4));
    HIPCHK(hipMalloc(&d_x2b, x2w.size() * 4));
    HIPCHK(hipMemcpy(d_x1, x1w.data(), x1w.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(d_x2b, x2w.data(), x2w.size() * 4, hipMemcpyHostToDevice));
    const uint32_t mtb = 2 * msf; // up to 2 TBs per subframe (CDD)
    HIPCHK(ring.create((sizeof(GoldItem) + sizeof(LlrItem)) * mtb + sizeof(TxItem) * max_sf));
    HIPCHK(hipHostMalloc(&h_tb, sizeof(srsgpu_dlsch_tb_t) * mtb));
    HIPCHK(hipMalloc(&d_gold, sizeof(GoldItem) * mtb));
    HIPCHK(hipMalloc(&d_llr, sizeof(LlrItem) * mtb));
    HIPCHK(hipMalloc(&d_c, (size_t)mtb * cwords * 4));
    HIPCHK(hipMalloc(&d_csi, (size_t)mtb * max_re * 4));
    HIPCHK(hipMalloc(&d_csimax, (size_t)mtb * 4));
    HIPCHK(hipMalloc(&d_e, (size_t)mtb * max_bits * 2));
    HIPCHK(hipMalloc(&d_gcache, (size_t)GCACHE * cwords * 4));
    return 0;
  }

  void destroy() {
    if (st) (void)hipStreamSynchronize(st);
    for (void *p : {(void *)d_x1, (void *)d_x2b, (void *)d_gold, (void *)d_llr, (void *)d_c,
                    (void *)d_csi, (void *)d_csimax, (void *)d_e, (void *)d_tx, (void *)d_ebits,
                    (void *)d_mod, (void *)d_fb, (void *)d_gcache})
      if (p) (void)hipFree(p);
    ring.destroy();
    for (void *p : {(void *)h_tb, (void *)h_fb})
      if (p) (void)hipHostFree(p);
    if (fb_staged) (void)hipEventDestroy(fb_staged);
    for (auto &kv : maps) (void)hipFree(kv.second.first);
    maps.clear();
    if (dl) srsgpu_dlsch_destroy(dl);
    dl = nullptr;
  }

  // device RE map of a grant, cached; returns its RE count
  // the previous lookup's key: consecutive subframes of a call mostly share their allocation class
  uint8_t last_prb[2 * 110];
  uint32_t last_cls = ~0u, last_lstart = ~0u, last_nre = 0;
  const uint32_t *last_map = nullptr;
  const uint32_t *map(const srsgpu_pdsch_sf_t &s, uint32_t *nre) {
    const uint32_t cls = s.sf_idx == 0 ? 0 : s.sf_idx == 5 ? 5 : 1;
    if (last_map && cls == last_cls && s.lstart == last_lstart && !memcmp(last_prb, s.prb_idx, sizeof(last_prb))) {
      *nre = last_nre;
      return last_map;
    }
    const uint32_t *m = map_lookup(s, cls, nre);
    if (m) {
      memcpy(last_prb, s.prb_idx, sizeof(last_prb));
      last_cls = cls;
      last_lstart = s.lstart;
      last_nre = *nre;
      last_map = m;
    }
    return m;
  }
  const uint32_t *map_lookup(const srsgpu_pdsch_sf_t &s, uint32_t cls, uint32_t *nre) {
    std::string key((const char *)s.prb_idx, 2 * 110);
    key += (char)cls;
    key += (char)s.lstart;
    auto it = maps.find(key);
    if (it == maps.end()) {
      std::vector<uint32_t> m;
      re_map(cell, s.lstart, cls, s.prb_idx, m);
      uint32_t *d = nullptr;
      if (hipMalloc(&d, std::max<size_t>(m.size(), 1) * 4) != hipSuccess) return nullptr;
      if (!m.empty() && hipMemcpy(d, m.data(), m.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
        return nullptr;
      it = maps.emplace(key, std::make_pair(d, (uint32_t)m.size())).first;
    }
    *nre = it->second.second;
    return it->second.first;
  }

  // TBs of a call in order: (subframe, tb); tb t of a CDD subframe sits on codeword
  // cw = t ^ tb_cw_swap (pdsch.c:959-995)
  static uint32_t nof_tb(const srsgpu_pdsch_sf_t &s) {
    return s.mimo_type == SRSGPU_MIMO_CDD || (s.mimo_type == SRSGPU_MIMO_SPATIAL_MULTIPLEX && s.tbs[1] > 0) ? 2 : 1;
  }

  // 4-port transmit diversity demaps 4 floor(n / 4) symbols (srslte_pdsch_decode's n / nof_layers,
  // pdsch.c:908, and m_ap of precoding.c:391 / :605); the reference would read any remaining symbol
  // from whatever its layer buffer last held. Normal-CP grants of a 4-port cell always hold whole
  // quadruplets (tests/test_txdiv.py); extended-CP grants of subframe 0 that hold only one of the
  // half PRBs beside the PBCH of an odd-sized cell do not (4 + 4 + 6 + 4 REs in slot 1's symbols
  // 0-3), and are refused here since the reference's result is undefined for them.
  int txdiv4_ragged(const srsgpu_pdsch_sf_t &s, uint32_t nre) const {
    if (s.mimo_type != SRSGPU_MIMO_TX_DIVERSITY || cell.nof_ports != 4 || nre % 4 == 0) return 0;
    fprintf(stderr, "srsgpu: 4-port transmit diversity needs a multiple of 4 REs (grant has %u)\n", nre);
    return -1;
  }

  int check(const srsgpu_pdsch_sf_t &s, uint32_t i) {
    const uint32_t nt = nof_tb(s);
    bool ok = s.sf_idx <= 9 && s.lstart <= 4;
    for (uint32_t t = 0; t < nt; t++) ok = ok && s.mod[t] <= 3;
    if (!ok) {
      fprintf(stderr, "srsgpu: invalid subframe %u (mod=%u sf_idx=%u lstart=%u)\n", i, s.mod[0], s.sf_idx,
              s.lstart);
      return -1;
    }
    if (s.mimo_type == SRSGPU_MIMO_SINGLE_ANTENNA) {
      if (cell.nof_ports != 1) {
        fprintf(stderr, "srsgpu: single-antenna PDSCH needs a 1-port cell\n");
        return -1;
      }
    } else if (s.mimo_type == SRSGPU_MIMO_TX_DIVERSITY) { // precoding.c:1811-1818, 2 or 4 ports
      if (cell.nof_ports != 2 && cell.nof_ports != 4) {
        fprintf(stderr, "Number of ports must be 2 or 4 for transmit diversity (nof_ports=%d)\n", cell.nof_ports);
        return -1;
      }
    } else if (s.mimo_type == SRSGPU_MIMO_CDD) { // precoding.c:1085-1097
      if (cell.nof_ports != 2 || cell.nof_rx_ant != 2) {
        fprintf(stderr, "Error predecoding CCD: Invalid combination of ports %u and rx antennax %u\n",
                cell.nof_ports, cell.nof_rx_ant);
        return -1;
      }
    } else if (s.mimo_type == SRSGPU_MIMO_SPATIAL_MULTIPLEX) { // precoding.c:1715-1760
      // the 2x2 MMSE and 2x1 MRC equalisers read both rx antennas
      if (cell.nof_ports != 2 || cell.nof_rx_ant != 2) {
        fprintf(stderr, "srsgpu: spatial multiplexing on the GPU needs 2 ports and 2 rx antennas\n");
        return -1;
      }
      if (s.codebook_idx > (nof_tb(s) == 2 ? 2u : 3u)) { // precoding.c:1350-1352, :1581-1583
        fprintf(stderr, "Wrong codebook_idx=%u\n", s.codebook_idx);
        return -1;
      }
    } else {
      fprintf(stderr, "srsgpu: MIMO type %u is not supported on the GPU\n", s.mimo_type);
      return -1;
    }
    return 0;
  }

  // The previous llr() call's inputs: a repeat (same subframes, pointers and settings) launches on
  // the LLR items and scrambling sequences already on the device. The sequences depend only on the
  // (RNTI, codeword, subframe, cell) seeds, as the reference's per-user pre-generated ones do
  // (pdsch.c:436-440). encode() reuses those buffers and clears the memo.
  std::vector<uint8_t> memo_key, memo_scratch;
  bool memo_valid = false;
  uint32_t memo_k = 0, memo_mre = 0;
  int memo_ndual = 0;
  int memo_p0 = 0; // nof_rx_ant when every item equalises port 0 alone (k_pdsch_llr_p0), else 0

  int llr(const srsgpu_pdsch_sf_t *sf, uint32_t n, const float *d_grid, const float *d_ce,
          size_t ant_stride, int16_t *const *e_ptr) {
    if (n > max_sf) {
      fprintf(stderr, "srsgpu: %u subframes exceed the capacity %u\n", n, max_sf);
      return -1;
    }
    {
      const uint32_t nt = count_tb(sf, n);
      const size_t n1 = sizeof(srsgpu_pdsch_sf_t) * n, n2 = sizeof(void *) * nt;
      const uintptr_t tail[9] = {(uintptr_t)d_grid, (uintptr_t)d_ce, ant_stride, csi, llr8, (uintptr_t)ce_rows,
                                 (uintptr_t)noise_dev, n, nt};
      memo_scratch.resize(n1 + n2 + sizeof(tail));
      memcpy(memo_scratch.data(), sf, n1);
      memcpy(memo_scratch.data() + n1, e_ptr, n2);
      memcpy(memo_scratch.data() + n1 + n2, tail, sizeof(tail));
      if (memo_valid && memo_scratch == memo_key) {
        if (csi) HIPCHK(hipMemsetAsync(d_csimax, 0, (size_t)memo_k * 4, st));
        ProfScope ps("k_pdsch_llr", st);
        HIPCHK(launch_pdsch_llr(d_llr, (int)memo_k, memo_mre, csi, st, memo_ndual, memo_p0));
        return 0;
      }
      memo_valid = false;
    }
    if (ring_take()) return -1;
    uint32_t mre = 0, k = 0;
    int n_dual = 0;
    bool p0 = true;
    gold_reset();
    for (uint32_t i = 0; i < n; i++) {
      const srsgpu_pdsch_sf_t &s = sf[i];
      if (check(s, i)) return -1;
      uint32_t nre = 0;
      const uint32_t *m = map(s, &nre);
      if (!m) return -1;
      if (nre != s.nof_re) { // pdsch.c:886-890
        fprintf(stderr, "Error expecting %d symbols but got %d\n", s.nof_re, nre);
        return -1;
      }
      if (txdiv4_ragged(s, nre)) return -1;
      const uint32_t nt = nof_tb(s);
      for (uint32_t tb = 0; tb < nt; tb++, k++) {
        const uint32_t cw = nt == 2 ? (tb ^ (s.tb_cw_swap ? 1u : 0u)) : 0u;
        const int q = kQm[s.mod[tb]];
        // sequences.c:64-66: rnti 2^14 + q 2^13 + (ns/2) 2^9 + N_ID
        const uint32_t *gc = gold(((uint32_t)s.rnti << 14) + (cw << 13) + ((2 * s.sf_idx / 2) << 9) + cell.id,
                                  nre * q);
        LlrItem &t = h_llr[k];
        memset(&t, 0, sizeof(t));
        for (uint32_t a = 0; a < cell.nof_rx_ant; a++) {
          t.y[a] = (const float2 *)d_grid + s.grid_offset + a * ant_stride;
          for (uint32_t p = 0; p < cell.nof_ports; p++)
            t.h[p][a] = (const float2 *)d_ce + s.ce_offset + (a * cell.nof_ports + p) * ant_stride;
        }
        t.map = m;
        t.c = gc;
        t.e = e_ptr[k];
        t.csi = d_csi + (size_t)k * max_re;
        t.csi_max = d_csimax + k;
        t.nof_re = nre;
        t.qm = q;
        t.mod = (int)s.mod[tb];
        t.nrx = (int)cell.nof_rx_ant;
        t.nports = (int)cell.nof_ports;
        t.cdd = s.mimo_type == SRSGPU_MIMO_CDD;
        if (s.mimo_type == SRSGPU_MIMO_SPATIAL_MULTIPLEX)
          t.mux = nt == 2 ? 1 + (int)s.codebook_idx : -(1 + (int)s.codebook_idx);
        t.txdiv = s.mimo_type == SRSGPU_MIMO_TX_DIVERSITY ? (int)cell.nof_ports : 0;
        t.layer = (int)cw;
        p0 = p0 && !t.cdd && !t.mux && !t.txdiv;
        t.csi_mode = csi ? 1 : 0;
        t.llr8 = llr8 ? 1 : 0;
        t.ce_rows = ce_rows;
        t.nsc = 12 * cell.nof_prb;
        t.inv_nsc = 1.0f / (float)t.nsc;
        t.aligned = ((uintptr_t)t.e % 4) == 0;
        t.noise = s.noise_estimate;
        t.noise_dev = noise_dev ? noise_dev + (size_t)i * cell.nof_rx_ant * cell.nof_ports : nullptr;
        t.scaling = s.scaling != 0.f ? s.scaling : 1.0f;
        t.inv_scaling = 1.0f / t.scaling;
        // the two TBs of a 2-layer MMSE with one modulation: one 2x2 solve per RE for both
        if (tb == 1 && (t.cdd || t.mux > 0) && s.mod[0] == s.mod[1]) {
          h_llr[k - 1].dual = 1;
          t.dual = 2;
          n_dual++;
        }
        mre = std::max(mre, nre);
      }
    }
    if (gold_launch()) return -1;
    HIPCHK(ring.upload(d_llr, h_llr, sizeof(LlrItem) * k, st));
    HIPCHK(ring.mark(st));
    if (csi) HIPCHK(hipMemsetAsync(d_csimax, 0, (size_t)k * 4, st));
    ProfScope ps("k_pdsch_llr", st);
    HIPCHK(launch_pdsch_llr(d_llr, (int)k, mre, csi, st, n_dual, p0 && cell.nof_rx_ant <= 2 ? (int)cell.nof_rx_ant : 0));
    memo_key.swap(memo_scratch);
    memo_k = k;
    memo_mre = mre;
    memo_ndual = n_dual;
    memo_p0 = p0 && cell.nof_rx_ant <= 2 ? (int)cell.nof_rx_ant : 0;
    memo_valid = true;
    return 0;
  }

  // srslte_pdsch_encode (pdsch.c:1048-1131): DL-SCH encoding of each TB (codeword cw = tb ^ tb_cw_swap
  // with two TBs, pdsch.c:1083-1089), then per RE the codewords' scrambled symbols, layer mapping and
  // precoding of the MIMO type, mapped into every port's grid (port p at grid_offset + p port_stride;
  // other REs untouched). Single antenna, transmit diversity (2 ports), CDD (2 ports, 2 TBs) and
  // spatial multiplexing (2 ports, 1 TB on 1 layer or 2 TBs on 2 layers, codebook_idx).
  int encode(const srsgpu_pdsch_sf_t *sf, uint32_t n, const uint8_t *d_data, float *d_grid, uint64_t port_stride) {
    if (n > max_sf) {
      fprintf(stderr, "srsgpu: %u subframes exceed the capacity %u\n", n, max_sf);
      return -1;
    }
    if (!d_tx) {
      HIPCHK(hipMalloc(&d_tx, sizeof(TxItem) * max_sf));
      HIPCHK(hipMalloc(&d_ebits, (size_t)2 * max_sf * max_bits + 64));
      // modem/lte_tables.c: levels k / sqrt(N) in double, stored as float; 36.211 7.1 bit order
      std::vector<float2> t;
      const float b = (float)(1 / sqrt(2.0));
      t.push_back(make_float2(b, b));
      t.push_back(make_float2(-b, -b));
      for (int i = 0; i < 4; i++) t.push_back(make_float2(i & 2 ? -b : b, i & 1 ? -b : b));
      const float l16[2] = {(float)(1 / sqrt(10.0)), (float)(3 / sqrt(10.0))};
      for (int i = 0; i < 16; i++) { // b0 b1 signs, b2 b3 levels
        const float re = l16[(i >> 1) & 1], im = l16[i & 1];
        t.push_back(make_float2(i & 8 ? -re : re, i & 4 ? -im : im));
      }
      const float l64[4] = {(float)(3 / sqrt(42.0)), (float)(1 / sqrt(42.0)), (float)(5 / sqrt(42.0)),
                            (float)(7 / sqrt(42.0))}; // (b2 b4) / (b3 b5) = 00 01 10 11
      for (int i = 0; i < 64; i++) {
        const int bi = ((i >> 3) & 1) << 1 | ((i >> 1) & 1), bq = ((i >> 2) & 1) << 1 | (i & 1);
        t.push_back(make_float2(i & 32 ? -l64[bi] : l64[bi], i & 16 ? -l64[bq] : l64[bq]));
      }
      HIPCHK(hipMalloc(&d_mod, t.size() * sizeof(float2)));
      HIPCHK(hipMemcpy(d_mod, t.data(), t.size() * sizeof(float2), hipMemcpyHostToDevice));
    }
    if (ring_take()) return -1;
    memo_valid = false; // the sequences and items below overwrite the ones llr() keeps
    uint32_t mre = 0, k = 0;
    gold_reset();
    for (uint32_t i = 0; i < n; i++) {
      const srsgpu_pdsch_sf_t &s = sf[i];
      if (check(s, i)) return -1;
      if (s.mimo_type != SRSGPU_MIMO_SINGLE_ANTENNA && port_stride < (uint64_t)(cell.cp == 1 ? 12 : 14) * 12 * cell.nof_prb) {
        fprintf(stderr, "srsgpu: a %u-port transmission needs a port stride of at least one grid\n", cell.nof_ports);
        return -1;
      }
      if (s.mimo_type == SRSGPU_MIMO_SPATIAL_MULTIPLEX && s.codebook_idx > (s.tbs[1] > 0 ? 2u : 3u)) {
        fprintf(stderr, "Invalid multiplex combination: codebook_idx=%u\n", s.codebook_idx); // precoding.c:2009
        return -1;
      }
      uint32_t nre = 0;
      const uint32_t *m = map(s, &nre);
      if (!m) return -1;
      if (nre != s.nof_re) {
        fprintf(stderr, "Error expecting %d symbols but got %d\n", s.nof_re, nre);
        return -1;
      }
      if (txdiv4_ragged(s, nre)) return -1;
      const uint32_t ntb = nof_tb(s);
      const float sc = s.scaling != 0.f ? s.scaling : 1.0f;
      TxItem &x = h_tx[i];
      memset(&x, 0, sizeof(x));
      for (uint32_t tb = 0; tb < ntb; tb++, k++) {
        const uint32_t cw = ntb == 2 ? (tb ^ (s.tb_cw_swap ? 1u : 0u)) : 0u;
        const int q = kQm[s.mod[tb]];
        srsgpu_dlsch_tb_t &t = h_tb[k];
        t.tbs = s.tbs[tb];
        t.rv = s.rv[tb];
        t.Qm = dlsch_qm(s, tb);
        t.nof_e_bits = nre * q;
        t.softbuffer = 0;
        t.e_offset = (uint64_t)k * max_bits;
        t.data_offset = s.data_offset[tb];
        // sequences.c:64-66: rnti 2^14 + q 2^13 + (ns/2) 2^9 + N_ID, q = codeword
        const uint32_t *gc = gold(((uint32_t)s.rnti << 14) + (cw << 13) + ((2 * s.sf_idx / 2) << 9) + cell.id,
                                  nre * q);
        x.e[cw] = d_ebits + (size_t)k * max_bits;
        x.c[cw] = gc;
        x.qm[cw] = q;
      }
      x.map = m;
      x.grid = (float2 *)d_grid + s.grid_offset;
      x.port_stride = port_stride;
      x.nof_re = nre;
      x.mimo = (int)s.mimo_type;
      x.nlayers = s.mimo_type == SRSGPU_MIMO_SPATIAL_MULTIPLEX ? (int)ntb : (int)cell.nof_ports;
      x.codebook = (int)s.codebook_idx;
      switch (s.mimo_type) {
      case SRSGPU_MIMO_TX_DIVERSITY: x.scaling = sc / sqrtf(2.0f); break;
      case SRSGPU_MIMO_CDD: x.scaling = 0.5f * sc; break;
      case SRSGPU_MIMO_SPATIAL_MULTIPLEX:
        x.scaling = (ntb == 1 || s.codebook_idx == 0) ? sc / sqrtf(2.0f) : sc / 2.0f;
        break;
      default: x.scaling = sc;
      }
      mre = std::max(mre, nre);
    }
    if (srsgpu_dlsch_encode_dev(dl, h_tb, k, d_data, d_ebits)) return -1;
    if (gold_launch()) return -1;
    HIPCHK(ring.upload(d_tx, h_tx, sizeof(TxItem) * n, st));
    HIPCHK(ring.mark(st));
    ProfScope ps("k_pdsch_tx", st);
    HIPCHK(launch_pdsch_tx(d_tx, (int)n, mre, d_mod, st));
    return 0;
  }

  // srsgpu_pdsch_feedback_dev: one FbItem per subframe, one launch
  int feedback(const srsgpu_feedback_sf_t *sf, uint32_t n, const float *d_ce, size_t ant_stride, const float *d_noise,
               srsgpu_feedback_t *out) {
    if (n > max_sf) {
      fprintf(stderr, "srsgpu: %u subframes exceed the capacity %u\n", n, max_sf);
      return -1;
    }
    if (!h_fb) {
      HIPCHK(hipHostMalloc(&h_fb, sizeof(FbItem) * max_sf));
      HIPCHK(hipMalloc(&d_fb, sizeof(FbItem) * max_sf));
      HIPCHK(hipEventCreateWithFlags(&fb_staged, hipEventDisableTiming));
    }
    if (fb_pending) HIPCHK(hipEventSynchronize(fb_staged));
    const uint32_t nof_ce = (cell.cp == 1 ? 12u : 14u) * 12u * cell.nof_prb; // SRSLTE_SF_LEN_RE
    if (ant_stride < nof_ce) {
      fprintf(stderr, "srsgpu: feedback needs full estimate planes (stride %zu < %u)\n", ant_stride, nof_ce);
      return -1;
    }
    const uint32_t P = cell.nof_ports, R = cell.nof_rx_ant;
    for (uint32_t i = 0; i < n; i++) {
      FbItem &t = h_fb[i];
      memset(&t, 0, sizeof(t));
      const float2 *base = (const float2 *)d_ce + sf[i].ce_offset;
      for (uint32_t p = 0; p < 2 && p < P; p++)
        for (uint32_t a = 0; a < R; a++) t.h[p][a] = base + (size_t)(a * P + p) * ant_stride; // [rx][port] planes
      t.noise = sf[i].noise_estimate;
      t.noise_dev = d_noise ? d_noise + i : nullptr;
      t.flags = sf[i].flags;
      t.nof_ce = nof_ce;
      t.nrx = (int)R;
      t.nports = (int)P;
      t.out = out + i;
    }
    HIPCHK(hipMemcpyAsync(d_fb, h_fb, sizeof(FbItem) * n, hipMemcpyHostToDevice, st));
    HIPCHK(hipEventRecord(fb_staged, st));
    fb_pending = true;
    ProfScope ps("k_feedback", st);
    HIPCHK(launch_feedback(d_fb, (int)n, st));
    return 0;
  }

  uint32_t count_tb(const srsgpu_pdsch_sf_t *sf, uint32_t n) const {
    uint32_t k = 0;
    for (uint32_t i = 0; i < n; i++) k += nof_tb(sf[i]);
    return k;
  }
};

} // namespace srsgpu

using srsgpu::PdschEngine;

struct srsgpu_pdsch {
  PdschEngine e;
};

extern "C" {

int srsgpu_pdsch_create(srsgpu_pdsch_t **q, const srsgpu_cell_t *cell, uint32_t nsb, uint32_t max_cb,
                        uint32_t max_sf) {
  if (!q || !cell) return -1;
  auto *p = new srsgpu_pdsch();
  if (p->e.create(*cell, nsb, max_cb, max_sf)) {
    p->e.destroy();
    delete p;
    *q = nullptr;
    return -1;
  }
  *q = p;
  return 0;
}

void srsgpu_pdsch_destroy(srsgpu_pdsch_t *q) {
  if (!q) return;
  q->e.destroy();
  delete q;
}

void srsgpu_pdsch_set_stream(srsgpu_pdsch_t *q, void *s) {
  if (!q) return;
  if (q->e.st != (hipStream_t)s) q->e.gcache.clear(); // kept sequences were made in the old stream's order
  q->e.st = (hipStream_t)s;
  srsgpu_dlsch_set_stream(q->e.dl, s);
}

void srsgpu_pdsch_set_noise_dev(srsgpu_pdsch_t *q, const float *d_noise) {
  if (q) q->e.noise_dev = d_noise;
}

void srsgpu_pdsch_set_csi(srsgpu_pdsch_t *q, int enable) {
  if (q) q->e.csi = enable != 0;
}

int srsgpu_pdsch_set_ce_rows(srsgpu_pdsch_t *q, int rows) {
  if (!q || (rows != 0 && rows != 1 && rows != 4)) return -1;
  if (rows == 4 && q->e.cell.cp == 1) return -1; // 4 rows: the normal-CP CRS symbols 0 / 4 / 7 / 11
  if (rows == 4 && q->e.cell.nof_ports > 2) return -1; // the estimator writes compact rows for <= 2 ports
  q->e.ce_rows = rows;
  return 0;
}

void srsgpu_pdsch_set_llr_8bit(srsgpu_pdsch_t *q, int enable) {
  if (!q) return;
  q->e.llr8 = enable != 0;
  srsgpu_dlsch_set_llr_8bit(q->e.dl, enable);
}

srsgpu_dlsch_t *srsgpu_pdsch_get_dlsch(srsgpu_pdsch_t *q) { return q ? q->e.dl : nullptr; }

int srsgpu_pdsch_nof_re(const srsgpu_cell_t *cell, const srsgpu_pdsch_sf_t *sf) {
  if (!cell || !sf) return -1;
  std::vector<uint32_t> m;
  srsgpu::re_map(*cell, sf->lstart, sf->sf_idx, sf->prb_idx, m);
  return (int)m.size();
}

int srsgpu_pdsch_llr_dev(srsgpu_pdsch_t *q, const srsgpu_pdsch_sf_t *sf, uint32_t n, const float *d_grid,
                         const float *d_ce, size_t ant_stride, int16_t *d_e, const uint64_t *e_offset) {
  if (!q || (!sf && n) || !d_grid || !d_ce || !d_e || !e_offset) return -1;
  if (srsgpu_dlsch_join_tail(q->e.dl)) return -1; // the previous call's tail may read its LLRs
  const uint32_t k = q->e.count_tb(sf, n);
  std::vector<int16_t *> e(k);
  for (uint32_t i = 0; i < k; i++) e[i] = d_e + e_offset[i];
  return q->e.llr(sf, n, d_grid, d_ce, ant_stride, e.data());
}

int srsgpu_pdsch_encode_dev(srsgpu_pdsch_t *q, const srsgpu_pdsch_sf_t *sf, uint32_t n,
                            const uint8_t *d_data, float *d_grid) {
  if (!q || (!sf && n) || !d_data || !d_grid || srsgpu_dlsch_join_tail(q->e.dl)) return -1;
  return q->e.encode(sf, n, d_data, d_grid, 0);
}

int srsgpu_pdsch_encode_ports_dev(srsgpu_pdsch_t *q, const srsgpu_pdsch_sf_t *sf, uint32_t n, const uint8_t *d_data,
                                  float *d_grid, size_t port_stride) {
  if (!q || (!sf && n) || !d_data || !d_grid || srsgpu_dlsch_join_tail(q->e.dl)) return -1;
  return q->e.encode(sf, n, d_data, d_grid, (uint64_t)port_stride);
}

int srsgpu_pdsch_feedback_dev(srsgpu_pdsch_t *q, const srsgpu_feedback_sf_t *sf, uint32_t n, const float *d_ce,
                              size_t ant_stride, const float *d_noise, srsgpu_feedback_t *d_out) {
  if (!q || (!sf && n) || !d_ce || !d_out || srsgpu_dlsch_join_tail(q->e.dl)) return -1;
  return q->e.feedback(sf, n, d_ce, ant_stride, d_noise, d_out);
}

static int pdsch_decode(srsgpu_pdsch_t *q, const srsgpu_pdsch_sf_t *sf, uint32_t n, const float *d_grid,
                        const float *d_ce, size_t ant_stride, uint8_t *d_data, uint8_t *const *d_out, uint32_t maxh,
                        int32_t *d_ret, uint32_t *d_noi);

int srsgpu_pdsch_decode_dev(srsgpu_pdsch_t *q, const srsgpu_pdsch_sf_t *sf, uint32_t n, const float *d_grid,
                            const float *d_ce, size_t ant_stride, uint8_t *d_data, uint32_t maxh,
                            int32_t *d_ret, uint32_t *d_noi) {
  if (!d_data) return -1;
  return pdsch_decode(q, sf, n, d_grid, d_ce, ant_stride, d_data, nullptr, maxh, d_ret, d_noi);
}

int srsgpu_pdsch_decode_out_dev(srsgpu_pdsch_t *q, const srsgpu_pdsch_sf_t *sf, uint32_t n, const float *d_grid,
                                const float *d_ce, size_t ant_stride, uint8_t *const *d_out, uint32_t maxh,
                                int32_t *d_ret, uint32_t *d_noi) {
  if (!d_out) return -1;
  return pdsch_decode(q, sf, n, d_grid, d_ce, ant_stride, nullptr, d_out, maxh, d_ret, d_noi);
}

static int pdsch_decode(srsgpu_pdsch_t *q, const srsgpu_pdsch_sf_t *sf, uint32_t n, const float *d_grid,
                        const float *d_ce, size_t ant_stride, uint8_t *d_data, uint8_t *const *d_out, uint32_t maxh,
                        int32_t *d_ret, uint32_t *d_noi) {
  if (!q || (!sf && n) || !d_grid || !d_ce || !d_ret || !d_noi) return -1;
  PdschEngine &E = q->e;
  // a tail of the previous call (srsgpu_dlsch_set_tail_stream on srsgpu_pdsch_get_dlsch) still reads
  // E.d_e, which llr() rewrites on st: the stream waits for it first
  if (srsgpu_dlsch_join_tail(E.dl)) return -1;
  const uint32_t k = E.count_tb(sf, n);
  std::vector<int16_t *> e(k);
  for (uint32_t i = 0; i < k; i++) e[i] = E.d_e + (size_t)i * E.max_bits;
  if (E.llr(sf, n, d_grid, d_ce, ant_stride, e.data())) return -1;
  uint32_t j = 0;
  for (uint32_t i = 0; i < n; i++)
    for (uint32_t tb = 0; tb < PdschEngine::nof_tb(sf[i]); tb++, j++) {
      srsgpu_dlsch_tb_t &t = E.h_tb[j];
      const bool skip = (sf[i].skip_tb >> tb) & 1u; // acked earlier: no decode (pdsch.c:946-947)
      t.tbs = skip ? 0 : sf[i].tbs[tb];
      t.rv = sf[i].rv[tb];
      t.Qm = srsgpu::dlsch_qm(sf[i], tb);
      t.nof_e_bits = sf[i].nof_re * srsgpu::kQm[sf[i].mod[tb]];
      t.softbuffer = skip ? 0 : sf[i].softbuffer[tb];
      t.e_offset = (uint64_t)j * E.max_bits;
      t.data_offset = sf[i].data_offset[tb];
    }
  if (d_out) return srsgpu_dlsch_decode_out_dev(E.dl, E.h_tb, k, E.d_e, d_out, maxh, d_ret, d_noi);
  return srsgpu_dlsch_decode_dev(E.dl, E.h_tb, k, E.d_e, d_data, maxh, d_ret, d_noi);
}

} // extern "C"
