// srsgpu PDCCH engine (include/srsgpu/pdcch_batch.h): the cell's REG grid and PDCCH REG order
// restated from the reference's regs.c on the host, per-subframe scrambling sequences, the LLR
// extraction launch (k_pdcch_llr in pdsch_kernels.hip) and the DL blind search (candidate lists on
// the host, candidate decoding by srsgpu_dci_decode_dev, first RNTI match per search by
// k_dci_select). Paths relative to /root/reference/lib.
#include <hip/hip_runtime.h>
#include <math.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

#include "pdsch_kernels.h"
#include "srsgpu/dci.h"
#include "srsgpu/pdcch_batch.h"
#include "srsgpu/viterbi_batch.h"

namespace {

struct Reg {
  uint32_t l, k0, k[4];
  bool assigned;
};

// regs.c:587-616 regs_num_x_symbol: symbol 3 (control regions of 4 symbols, nof_prb <= 10) carries
// CRS with extended CP
int regs_num_x_symbol(uint32_t symbol, uint32_t nof_ports, bool ext_cp) {
  switch (symbol) {
  case 0: return 2;
  case 1: return nof_ports == 4 ? 2 : 3;
  case 3: return ext_cp ? 2 : 3;
  default: return 3;
  }
}

// regs.c:612-651 regs_reg_init: a REG of symbol l, the nreg-th of its PRB; with 2 REGs per PRB the
// reference signal subcarriers vo and vo + 3 are skipped
Reg reg_init(uint32_t symbol, uint32_t nreg, uint32_t k0, uint32_t maxreg, uint32_t vo) {
  Reg r{};
  r.l = symbol;
  if (maxreg == 2) {
    r.k0 = k0 + nreg * 6;
    uint32_t j = 0;
    for (uint32_t i = 0; i < vo; i++) r.k[j++] = k0 + nreg * 6 + i;
    for (uint32_t i = 0; i < 2; i++) r.k[j++] = k0 + nreg * 6 + i + vo + 1;
    const uint32_t z = j;
    for (uint32_t i = 0; i < 4 - z; i++) r.k[j++] = k0 + nreg * 6 + vo + 3 + i + 1;
  } else {
    r.k0 = k0 + nreg * 4;
    for (uint32_t i = 0; i < 4; i++) r.k[i] = k0 + nreg * 4 + i;
  }
  return r;
}

// 36.211 7.2 Gold sequence c(0..len-1) for c_init, packed LSB first (sequence.c:51-80)
std::vector<uint32_t> gold(uint32_t c_init, uint32_t len) {
  const uint32_t nc = 1600, n = nc + len + 31;
  std::vector<uint8_t> x1(n, 0), x2(n, 0);
  x1[0] = 1;
  for (int i = 0; i < 31; i++) x2[i] = (c_init >> i) & 1;
  for (uint32_t i = 0; i + 31 < n; i++) {
    x1[i + 31] = x1[i + 3] ^ x1[i];
    x2[i + 31] = x2[i + 3] ^ x2[i + 2] ^ x2[i + 1] ^ x2[i];
  }
  std::vector<uint32_t> w((len + 31) / 32, 0);
  for (uint32_t i = 0; i < len; i++) w[i / 32] |= (uint32_t)(x1[i + nc] ^ x2[i + nc]) << (i % 32);
  return w;
}

const uint8_t kPdcchPerm[32] = {1, 17, 9, 25, 5, 21, 13, 29, 3, 19, 11, 27, 7, 23, 15, 31,
                                0, 16, 8, 24, 4, 20, 12, 28, 2, 18, 10, 26, 6, 22, 14, 30}; // regs.c:75-77

// k_dci_select: the first candidate of each search whose CRC remainder equals the RNTI and whose
// format is the searched one (ue_dl.c:768-810 dci_blind_search, over the concatenated searches of
// find_dl_dci_type_crnti / _siprarnti). A candidate the reference's decode_msg refuses before that ends
// the search with found = -1, as the reference's search then returns SRSLTE_ERROR. Format 0 found while
// searching 1A is the UL DCI: the first one is set aside (ue_dl.c:785-792) and, when the UL search that
// follows (srslte_ue_dl_find_ul_dci, ue_dl.c:811-838) is for the same RNTI, is its result; otherwise the
// UL search scans its own list (the UE-specific locations of its RNTI, format 0).
struct SelCand {
  uint32_t format, L, ncce, nof_bits;
  uint64_t out_offset;
  uint32_t refused, pad; // srslte_dci_location_isvalid fails (ncce > 87, dci.c:215-221)
};
struct SelSearch {
  uint32_t c0, nc, rnti, ul_rnti; // rnti 0: no DL search (the reference's "RNTI not specified")
  uint32_t ul_c0, ul_nc, pad0, pad1;
};
__device__ inline uint32_t dci_format_of(const SelCand &c, const uint8_t *bits) {
  // pdcch.c:386-391: 0 / 1A share a size, the first bit tells them apart
  return (c.format == SRSGPU_DCI_FORMAT0 || c.format == SRSGPU_DCI_FORMAT1A)
             ? (bits[0] == 0 ? (uint32_t)SRSGPU_DCI_FORMAT0 : (uint32_t)SRSGPU_DCI_FORMAT1A)
             : c.format;
}
__device__ inline void dci_take(srsgpu_dci_result_t &r, const SelCand &c, uint32_t f, const uint8_t *bits) {
  r.found = 1;
  r.format = f;
  r.L = c.L;
  r.ncce = c.ncce;
  r.nof_bits = c.nof_bits;
  for (uint32_t b = 0; b < c.nof_bits + 16 && b < SRSGPU_DCI_MAX_BITS; b++) r.data[b] = bits[b];
}
__device__ inline void dci_none(srsgpu_dci_result_t &r, int32_t found) {
  r.found = found;
  r.format = 0xFFFFFFFFu;
  r.L = r.ncce = r.nof_bits = 0;
  for (int b = 0; b < SRSGPU_DCI_MAX_BITS; b++) r.data[b] = 0;
}
__global__ void k_dci_select(const SelSearch *__restrict__ ss, int n, const SelCand *__restrict__ cand,
                             const uint8_t *__restrict__ data, const uint16_t *__restrict__ crc_rem,
                             const uint8_t *__restrict__ decoded, srsgpu_dci_result_t *__restrict__ res,
                             srsgpu_dci_result_t *__restrict__ res_ul) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  const SelSearch q = ss[s];
  srsgpu_dci_result_t r;
  dci_none(r, q.rnti ? 0 : -1);
  int pend = -1; // the UL DCI set aside by the DL search
  for (uint32_t i = q.c0; q.rnti && i < q.c0 + q.nc; i++) {
    if (cand[i].refused) { // srslte_pdcch_decode_msg fails, the search returns SRSLTE_ERROR (ue_dl.c:785-788)
      r.found = -1;
      break;
    }
    if (!decoded[i] || crc_rem[i] != (uint16_t)q.rnti) continue;
    const SelCand c = cand[i];
    const uint8_t *bits = data + c.out_offset;
    const uint32_t f = dci_format_of(c, bits);
    if (f == SRSGPU_DCI_FORMAT0 && c.format == SRSGPU_DCI_FORMAT1A) {
      if (pend < 0) pend = (int)i;
      continue;
    }
    if (f != c.format) continue;
    dci_take(r, c, f, bits);
    break;
  }
  res[s] = r;
  if (!res_ul) return;
  srsgpu_dci_result_t u;
  dci_none(u, 0);
  if (q.ul_rnti) {
    if (pend >= 0 && q.ul_rnti == q.rnti) { // ue_dl.c:815-819
      dci_take(u, cand[pend], SRSGPU_DCI_FORMAT0, data + cand[pend].out_offset);
    } else {
      for (uint32_t i = q.ul_c0; i < q.ul_c0 + q.ul_nc; i++) {
        if (cand[i].refused) {
          u.found = -1;
          break;
        }
        if (!decoded[i] || crc_rem[i] != (uint16_t)q.ul_rnti) continue;
        const SelCand c = cand[i];
        const uint8_t *bits = data + c.out_offset;
        if (bits[0] != 0) continue; // a format 1A message: not what the UL search looks for
        dci_take(u, c, SRSGPU_DCI_FORMAT0, bits);
        break;
      }
    }
  }
  res_ul[s] = u;
}

// ue_dl.c:41-50
const uint32_t kUeFormats[8][2] = {{SRSGPU_DCI_FORMAT1A, SRSGPU_DCI_FORMAT1},  {SRSGPU_DCI_FORMAT1A, SRSGPU_DCI_FORMAT1},
                                   {SRSGPU_DCI_FORMAT1A, SRSGPU_DCI_FORMAT2A}, {SRSGPU_DCI_FORMAT1A, SRSGPU_DCI_FORMAT2},
                                   {SRSGPU_DCI_FORMAT1A, SRSGPU_DCI_FORMAT1D}, {SRSGPU_DCI_FORMAT1A, SRSGPU_DCI_FORMAT1B},
                                   {SRSGPU_DCI_FORMAT1A, SRSGPU_DCI_FORMAT1},  {SRSGPU_DCI_FORMAT1A, SRSGPU_DCI_FORMAT2B}};

// one upload slot (host pinned + device), reused once its last launch has finished
struct Slot {
  void *h = nullptr, *d = nullptr;
  size_t cap = 0;
  hipEvent_t done = nullptr;
  bool pending = false;
  int reserve(size_t bytes) {
    if (pending && hipEventSynchronize(done) != hipSuccess) return -1;
    pending = false;
    if (bytes <= cap) return 0;
    (void)hipFree(d);
    (void)hipHostFree(h);
    d = h = nullptr;
    cap = 0;
    if (hipHostMalloc(&h, bytes) != hipSuccess || hipMalloc(&d, bytes) != hipSuccess) return -1;
    cap = bytes;
    return 0;
  }
  int mark(hipStream_t st) {
    if (hipEventRecord(done, st) != hipSuccess) return -1;
    pending = true;
    return 0;
  }
  void release() {
    if (pending) (void)hipEventSynchronize(done);
    (void)hipFree(d);
    (void)hipHostFree(h);
    if (done) (void)hipEventDestroy(done);
  }
};

// srslte_regs_init + srslte_pdcch_set_cell on the host: the PDCCH symbol order (grid indices) and
// NOF_CCE for each CFI
int build_maps(const srsgpu_cell_t &cell, uint32_t phich_length, uint32_t phich_resources,
               std::vector<uint32_t> maps[3], uint32_t nof_cce[3]) {
  const uint32_t nprb = cell.nof_prb, id = cell.id, np = cell.nof_ports;
  // srslte_regs_init (regs.c:681-763): REGs sorted by PRB, then symbol, then position
  const uint32_t max_ctrl = nprb <= 10 ? 4 : 3, vo = id % 3;
  uint32_t n[4] = {0, 0, 0, 0}, nof_regs = 0;
  for (uint32_t i = 0; i < max_ctrl; i++) {
    n[i] = (uint32_t)regs_num_x_symbol(i, np, cell.cp == 1);
    nof_regs += nprb * n[i];
  }
  std::vector<Reg> regs(nof_regs);
  {
    uint32_t j[4] = {0, 0, 0, 0}, k = 0, i = 0, prb = 0, jmax = 0;
    while (k < nof_regs) {
      if (n[i] == 3 || (n[i] == 2 && jmax != 1)) {
        regs[k] = reg_init(i, j[i], prb * 12, n[i], vo);
        j[i]++;
        k++;
      }
      i++;
      if (i == max_ctrl) {
        i = 0;
        jmax++;
      }
      if (jmax == 3) {
        prb++;
        memset(j, 0, sizeof(j));
        jmax = 0;
      }
    }
  }
  // regs_pcfich_init (regs.c:477-512)
  const uint32_t k_hat = 6 * (id % (2 * nprb));
  for (uint32_t i = 0; i < 4; i++) {
    const uint32_t k = (k_hat + (i * nprb / 2) * 6) % (nprb * 12);
    bool ok = false;
    for (Reg &r : regs)
      if (r.l == 0 && r.k0 == k && !r.assigned) {
        r.assigned = ok = true;
        break;
      }
    if (!ok) return -1;
  }
  // regs_phich_init (regs.c:249-331)
  {
    const float ng = phich_resources == 0 ? (float)1 / 6 : phich_resources == 1 ? (float)1 / 2
                     : phich_resources == 2 ? 1.0f : 2.0f;
    const uint32_t ngroups = (uint32_t)(int)ceilf(ng * ((float)nprb / 8));
    std::vector<Reg *> ph[3];
    for (Reg &r : regs)
      if (r.l < 3 && !r.assigned) ph[r.l].push_back(&r);
    const uint32_t cnt[3] = {(uint32_t)ph[0].size(), (uint32_t)ph[1].size(), (uint32_t)ph[2].size()};
    for (uint32_t mi = 0; mi < ngroups; mi++)
      for (uint32_t i = 0; i < 3; i++) {
        const uint32_t li = phich_length ? i : 0;
        if (cnt[li] == 0 || cnt[0] == 0) return -1;
        const uint32_t ni = ((id * cnt[li] / cnt[0]) + mi + i * cnt[li] / 3) % cnt[li];
        ph[li][ni]->assigned = true;
      }
  }
  // regs_pdcch_init (regs.c:82-158): interleaving of the free REGs of the CFI's control symbols
  // (sub-block interleaver of 32 columns with the column permutation) and the cyclic shift by the
  // cell id; the REG count rounded down to whole CCEs afterwards
  for (uint32_t cfi = 0; cfi < 3; cfi++) {
    const uint32_t nctrl = nprb <= 10 ? cfi + 2 : cfi + 1;
    std::vector<const Reg *> tmp;
    for (const Reg &r : regs)
      if (r.l < nctrl && !r.assigned) tmp.push_back(&r);
    const uint32_t m = (uint32_t)tmp.size();
    std::vector<const Reg *> order(m, nullptr);
    const int nrows = ((int)m - 1) / 32 + 1;
    int ndummy = 32 * nrows - (int)m;
    if (ndummy < 0) ndummy = 0;
    uint32_t k = 0;
    for (int jj = 0; jj < 32; jj++)
      for (int ii = 0; ii < nrows; ii++)
        if (ii * 32 + kPdcchPerm[jj] >= ndummy) {
          const uint32_t mm = (uint32_t)(ii * 32 + kPdcchPerm[jj] - ndummy);
          const uint32_t kp = k < id ? (m + k - (id % m)) % m : (k - id) % m;
          order[mm] = tmp[kp];
          k++;
        }
    const uint32_t nregs = (m / 9) * 9;
    nof_cce[cfi] = nregs / 9;
    maps[cfi].resize(4 * (size_t)nregs);
    for (uint32_t r = 0; r < nregs; r++)
      for (uint32_t i = 0; i < 4; i++) maps[cfi][4 * r + i] = order[r]->k[i] + order[r]->l * nprb * 12;
  }
  return 0;
}

} // namespace

struct srsgpu_pdcch {
  srsgpu_cell_t cell{};
  uint32_t nof_cce[3] = {0, 0, 0};
  std::vector<uint32_t> map[3];        // per CFI: 36 nof_cce grid indices
  uint32_t *d_map = nullptr;           // the three maps concatenated
  uint32_t map_off[3] = {0, 0, 0};
  uint32_t *d_seq = nullptr;           // [10][seq_words] scrambling bits
  uint32_t seq_words = 0;
  Slot items[2], search[2];            // double-buffered uploads
  int it_turn = 0, se_turn = 0;
  // search scratch (device): candidates' decoded bits, CRC remainders, decoded flags
  uint8_t *d_bits = nullptr, *d_dec = nullptr;
  uint16_t *d_crc = nullptr;
  size_t cand_cap = 0;
  hipEvent_t search_done = nullptr;
  bool search_pending = false;
  const float *d_noise = nullptr; // srsgpu_pdcch_set_noise_dev
};

extern "C" {

int srsgpu_pdcch_create(srsgpu_pdcch_t **q, const srsgpu_cell_t *cell, uint32_t phich_length,
                        uint32_t phich_resources) {
  if (!q || !cell || cell->nof_prb < 6 || cell->nof_prb > 110 || cell->id > 503 || (cell->nof_ports != 1 &&
      cell->nof_ports != 2 && cell->nof_ports != 4) || cell->nof_rx_ant < 1 || cell->nof_rx_ant > 2 || phich_length > 1 ||
      phich_resources > 3 || cell->cp > 1)
    return -1;
  srsgpu_pdcch *p = new srsgpu_pdcch;
  p->cell = *cell;
  if (build_maps(*cell, phich_length, phich_resources, p->map, p->nof_cce)) {
    srsgpu_pdcch_destroy(p);
    return -1;
  }
  const uint32_t id = cell->id;
  // srslte_pdcch_set_cell (pdcch.c:197-205): c_init = subframe * 512 + cell id, 8 nregs(3) bits
  const uint32_t seq_len = 8 * 9 * p->nof_cce[2];
  p->seq_words = (seq_len + 31) / 32;
  std::vector<uint32_t> seq((size_t)10 * p->seq_words);
  for (uint32_t sf = 0; sf < 10; sf++) {
    const std::vector<uint32_t> w = gold(sf * 512 + id, seq_len);
    memcpy(&seq[(size_t)sf * p->seq_words], w.data(), w.size() * 4);
  }
  size_t total = 0;
  for (int c = 0; c < 3; c++) {
    p->map_off[c] = (uint32_t)total;
    total += p->map[c].size();
  }
  std::vector<uint32_t> all(total);
  for (int c = 0; c < 3; c++) memcpy(all.data() + p->map_off[c], p->map[c].data(), p->map[c].size() * 4);
  bool bad = hipMalloc(&p->d_map, total * 4 + 4) || hipMalloc(&p->d_seq, seq.size() * 4 + 4) ||
             hipMemcpy(p->d_map, all.data(), total * 4, hipMemcpyHostToDevice) ||
             hipMemcpy(p->d_seq, seq.data(), seq.size() * 4, hipMemcpyHostToDevice) ||
             hipEventCreateWithFlags(&p->search_done, hipEventDisableTiming);
  for (int i = 0; i < 2 && !bad; i++)
    bad = hipEventCreateWithFlags(&p->items[i].done, hipEventDisableTiming) ||
          hipEventCreateWithFlags(&p->search[i].done, hipEventDisableTiming);
  if (bad) {
    srsgpu_pdcch_destroy(p);
    return -1;
  }
  *q = p;
  return 0;
}

void srsgpu_pdcch_destroy(srsgpu_pdcch_t *q) {
  if (!q) return;
  for (int i = 0; i < 2; i++) {
    q->items[i].release();
    q->search[i].release();
  }
  if (q->search_pending) (void)hipEventSynchronize(q->search_done);
  if (q->search_done) (void)hipEventDestroy(q->search_done);
  for (void *p : {(void *)q->d_map, (void *)q->d_seq, (void *)q->d_bits, (void *)q->d_dec, (void *)q->d_crc})
    (void)hipFree(p);
  delete q;
}

int srsgpu_pdcch_cell_map(const srsgpu_cell_t *cell, uint32_t phich_length, uint32_t phich_resources,
                          uint32_t cfi, uint32_t *idx, uint32_t max, uint32_t *nof_cce) {
  if (!cell || cell->nof_prb < 6 || cell->nof_prb > 110 || cell->id > 503 || (cell->nof_ports != 1 &&
      cell->nof_ports != 2 && cell->nof_ports != 4) || phich_length > 1 || phich_resources > 3 || cfi < 1 || cfi > 3 ||
      cell->cp > 1)
    return -1;
  std::vector<uint32_t> maps[3];
  uint32_t ncce[3];
  if (build_maps(*cell, phich_length, phich_resources, maps, ncce)) return -1;
  if (nof_cce) *nof_cce = ncce[cfi - 1];
  if (!idx) return (int)maps[cfi - 1].size();
  if (maps[cfi - 1].size() > max) return -1;
  memcpy(idx, maps[cfi - 1].data(), maps[cfi - 1].size() * 4);
  return (int)maps[cfi - 1].size();
}

uint32_t srsgpu_pdcch_nof_cce(const srsgpu_pdcch_t *q, uint32_t cfi) {
  return q && cfi >= 1 && cfi <= 3 ? q->nof_cce[cfi - 1] : 0;
}

void srsgpu_pdcch_set_noise_dev(srsgpu_pdcch_t *q, const float *d_noise) {
  if (q) q->d_noise = d_noise;
}

int srsgpu_pdcch_re_map(const srsgpu_pdcch_t *q, uint32_t cfi, uint32_t *idx, uint32_t max) {
  if (!q || cfi < 1 || cfi > 3 || !idx) return -1;
  const std::vector<uint32_t> &m = q->map[cfi - 1];
  if (m.size() > max) return -1;
  memcpy(idx, m.data(), m.size() * 4);
  return (int)m.size();
}

int srsgpu_pdcch_extract_llr_dev(srsgpu_pdcch_t *q, const srsgpu_pdcch_sf_t *sf, uint32_t nof_sf,
                                 const float *d_grid, const float *d_ce, size_t ant_stride,
                                 float *d_llr, void *hip_stream) {
  if (!q || (nof_sf && (!sf || !d_grid || !d_ce || !d_llr))) return -1;
  if (nof_sf == 0) return 0;
  if (ant_stride < (size_t)14 * 12 * q->cell.nof_prb) return -1;
  hipStream_t st = (hipStream_t)hip_stream;
  Slot &s = q->items[q->it_turn];
  q->it_turn ^= 1;
  if (s.reserve(sizeof(srsgpu::PdcchItem) * nof_sf)) return -1;
  srsgpu::PdcchItem *h = (srsgpu::PdcchItem *)s.h;
  uint32_t max_sym = 0;
  for (uint32_t i = 0; i < nof_sf; i++) {
    const uint32_t cfi = sf[i].cfi;
    if (sf[i].sf_idx > 9 || cfi < 1 || cfi > 3 || (sf[i].llr_offset & 1)) return -1;
    const uint32_t nsym = 36 * q->nof_cce[cfi - 1];
    h[i] = {sf[i].grid_offset, sf[i].ce_offset, sf[i].llr_offset, q->d_map + q->map_off[cfi - 1],
            q->d_seq + (size_t)sf[i].sf_idx * q->seq_words, nsym, sf[i].noise_estimate,
            q->d_noise ? q->d_noise + i : nullptr};
    if (nsym > max_sym) max_sym = nsym;
  }
  { // every subframe's 72 NOF_CCE(cfi) LLRs in a region of its own: overlapping ones would be written twice
    std::vector<std::pair<uint64_t, uint64_t>> reg(nof_sf);
    for (uint32_t i = 0; i < nof_sf; i++) reg[i] = {sf[i].llr_offset, 2 * (uint64_t)h[i].nof_symbols};
    std::sort(reg.begin(), reg.end());
    for (uint32_t i = 1; i < nof_sf; i++)
      if (reg[i - 1].first + reg[i - 1].second > reg[i].first) {
        fprintf(stderr, "srsgpu pdcch: LLR regions of two subframes overlap (llr_offset spacing below 72 NOF_CCE)\n");
        return -1;
      }
  }
  if (hipMemcpyAsync(s.d, s.h, sizeof(srsgpu::PdcchItem) * nof_sf, hipMemcpyHostToDevice, st) ||
      srsgpu::launch_pdcch_llr((const srsgpu::PdcchItem *)s.d, (int)nof_sf, max_sym, (const float2 *)d_grid,
                               (const float2 *)d_ce, ant_stride, (int)q->cell.nof_ports,
                               (int)q->cell.nof_rx_ant, d_llr, st) ||
      s.mark(st))
    return -1;
  return 0;
}

uint32_t srsgpu_pdcch_ue_locations(uint32_t nof_cce, uint32_t sf_idx, uint16_t rnti, srsgpu_dci_location_t *c,
                                   uint32_t max) {
  // pdcch.c:227-266 (36.213 9.1.1): Y_k = (39827 Y_{k-1}) mod 65537 from Y_-1 = rnti
  static const uint32_t ncand[4] = {6, 6, 2, 2};
  uint32_t Yk = rnti;
  for (uint32_t m = 0; m < sf_idx + 1; m++) Yk = (39827 * Yk) % 65537;
  uint32_t k = 0;
  for (int l = 3; l >= 0; l--) {
    const uint32_t L = 1u << l;
    for (uint32_t i = 0; i < ncand[l]; i++)
      if (nof_cce >= L) {
        const uint32_t ncce = L * ((Yk + i) % (nof_cce / L));
        if (k < max && ncce + L <= nof_cce) {
          if (c) c[k] = {(uint32_t)l, ncce};
          k++;
        }
      }
  }
  return k;
}

uint32_t srsgpu_pdcch_common_locations(uint32_t nof_cce, srsgpu_dci_location_t *c, uint32_t max) {
  // pdcch.c:274-300
  uint32_t k = 0;
  for (uint32_t l = 3; l > 1; l--) {
    const uint32_t L = 1u << l;
    for (uint32_t i = 0; i < (nof_cce < 16 ? nof_cce : 16) / L; i++) {
      const uint32_t ncce = L * (i % (nof_cce / L));
      if (k < max && ncce + L <= nof_cce) {
        if (c) c[k] = {l, ncce};
        k++;
      }
    }
  }
  return k;
}

int srsgpu_pdcch_find_dci_dev(srsgpu_pdcch_t *q, const srsgpu_dci_search_t *s, uint32_t nof_search,
                              const float *d_llr, srsgpu_dci_result_t *d_res, srsgpu_dci_result_t *d_res_ul,
                              void *hip_stream) {
  if (!q || (nof_search && (!s || !d_llr || !d_res))) return -1;
  if (nof_search == 0) return 0;
  hipStream_t st = (hipStream_t)hip_stream;
  // candidate lists in the reference's search order
  std::vector<SelSearch> ss(nof_search);
  std::vector<SelCand> cand;
  std::vector<srsgpu_dci_cand_t> dc;
  const uint32_t nprb = q->cell.nof_prb, np = q->cell.nof_ports;
  for (uint32_t i = 0; i < nof_search; i++) {
    const srsgpu_dci_search_t &x = s[i];
    const uint32_t ul_rnti = d_res_ul ? x.ul_rnti : 0;
    if (x.cfi < 1 || x.cfi > 3 || x.sf_idx > 9 || x.rnti > 0xFFFF || ul_rnti > 0xFFFF || x.tm > 7 ||
        x.rnti_type > 6 || (x.rnti == 0 && ul_rnti == 0))
      return -1;
    const uint32_t ncce = q->nof_cce[x.cfi - 1];
    ss[i] = {(uint32_t)cand.size(), 0, x.rnti, ul_rnti, 0, 0, 0, 0};
    srsgpu_dci_location_t ue[64], com[64];
    const uint32_t ncom = srsgpu_pdcch_common_locations(ncce, com, 64);
    auto add = [&](const srsgpu_dci_location_t *loc, uint32_t nl, uint32_t format) {
      const uint32_t nb = srsgpu_dci_format_sizeof(format, nprb, np);
      for (uint32_t j = 0; j < nl; j++) {
        const uint64_t off = (uint64_t)cand.size() * (SRSGPU_DCI_MAX_BITS + 16);
        cand.push_back({format, loc[j].L, loc[j].ncce, nb, off, loc[j].ncce > 87 ? 1u : 0u, 0u});
        dc.push_back({x.llr_offset + 72 * (uint64_t)loc[j].ncce, off, 72u << loc[j].L, nb});
      }
    };
    bool ul_shared = false;
    if (x.rnti) {
      // ue_dl.c:840-852: the RNTI type from the value (SI-RNTI, P-RNTI, RA-RNTI range) unless given
      const bool common = x.rnti_type < 0 ? (x.rnti == 0xFFFF || x.rnti == 0xFFFE || x.rnti <= 0x000A)
                                          : (x.rnti_type == 1 || x.rnti_type == 2 || x.rnti_type == 5);
      if (common) { // find_dl_dci_type_siprarnti (ue_dl.c:855-874)
        add(com, ncom, SRSGPU_DCI_FORMAT1A);
        add(com, ncom, SRSGPU_DCI_FORMAT1C);
      } else { // find_dl_dci_type_crnti (ue_dl.c:877-913)
        const uint32_t nue = srsgpu_pdcch_ue_locations(ncce, x.sf_idx, (uint16_t)x.rnti, ue, 64);
        add(ue, nue, kUeFormats[x.tm][0]); // 1A: the UL search's candidates too when the RNTIs agree
        add(ue, nue, kUeFormats[x.tm][1]);
        add(com, ncom, SRSGPU_DCI_FORMAT1A);
        if (ul_rnti == x.rnti) {
          ss[i].ul_c0 = ss[i].c0;
          ss[i].ul_nc = nue;
          ul_shared = true;
        }
      }
      ss[i].nc = (uint32_t)cand.size() - ss[i].c0;
    }
    if (ul_rnti && !ul_shared) { // srslte_ue_dl_find_ul_dci's own list (ue_dl.c:825-832)
      const uint32_t nue = srsgpu_pdcch_ue_locations(ncce, x.sf_idx, (uint16_t)ul_rnti, ue, 64);
      ss[i].ul_c0 = (uint32_t)cand.size();
      add(ue, nue, SRSGPU_DCI_FORMAT0);
      ss[i].ul_nc = nue;
    }
  }
  const size_t nc = cand.size();
  // scratch for the candidate decodes (reused once the previous search has finished with it)
  if (q->search_pending && hipEventSynchronize(q->search_done)) return -1;
  q->search_pending = false;
  if (nc > q->cand_cap) {
    (void)hipFree(q->d_bits);
    (void)hipFree(q->d_dec);
    (void)hipFree(q->d_crc);
    q->d_bits = q->d_dec = nullptr;
    q->d_crc = nullptr;
    q->cand_cap = 0;
    if (hipMalloc(&q->d_bits, nc * (SRSGPU_DCI_MAX_BITS + 16)) || hipMalloc(&q->d_dec, nc) ||
        hipMalloc(&q->d_crc, nc * 2))
      return -1;
    q->cand_cap = nc;
  }
  const size_t b_dc = nc * sizeof(srsgpu_dci_cand_t), b_sel = nc * sizeof(SelCand),
               b_ss = nof_search * sizeof(SelSearch);
  Slot &sl = q->search[q->se_turn];
  q->se_turn ^= 1;
  if (sl.reserve(b_dc + b_sel + b_ss + 64)) return -1;
  char *h = (char *)sl.h, *d = (char *)sl.d;
  memcpy(h, dc.data(), b_dc);
  memcpy(h + b_dc, cand.data(), b_sel);
  memcpy(h + b_dc + b_sel, ss.data(), b_ss);
  if (hipMemcpyAsync(d, h, b_dc + b_sel + b_ss, hipMemcpyHostToDevice, st)) return -1;
  if (nc && srsgpu_dci_decode_dev((const srsgpu_dci_cand_t *)d, (uint32_t)nc, d_llr, q->d_bits, q->d_crc, q->d_dec,
                                  st))
    return -1;
  hipLaunchKernelGGL(k_dci_select, dim3((nof_search + 63) / 64), dim3(64), 0, st, (const SelSearch *)(d + b_dc + b_sel),
                     (int)nof_search, (const SelCand *)(d + b_dc), q->d_bits, q->d_crc, q->d_dec, d_res, d_res_ul);
  if (hipGetLastError() != hipSuccess || sl.mark(st) || hipEventRecord(q->search_done, st)) return -1;
  q->search_pending = true;
  return 0;
}

int srsgpu_pdcch_find_dl_dci_dev(srsgpu_pdcch_t *q, const srsgpu_dci_search_t *s, uint32_t nof_search,
                                 const float *d_llr, srsgpu_dci_result_t *d_res, void *hip_stream) {
  if (!q || (nof_search && !s)) return -1;
  for (uint32_t i = 0; i < nof_search; i++)
    if (s[i].rnti == 0) return -1; // a DL search needs its RNTI
  return srsgpu_pdcch_find_dci_dev(q, s, nof_search, d_llr, d_res, nullptr, hip_stream);
}

} // extern "C"
