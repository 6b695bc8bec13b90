// MI355X DL-SCH kernels around the turbo decoder (paths relative to /root/reference/lib):
//   k_derm        srslte_rm_turbo_rx_lut (src/phy/fec/rm_turbo.c:394-430): soft-combine a code
//                 block's E received LLRs into its HARQ softbuffer row, out[t[i % N]] += in[i]
//                 (int16 wrap). Written as a gather over the N = 3K+12 table entries: entry m
//                 sums in[m], in[m+N], ... (repetition) and adds once, so every row element is
//                 owned by one thread (the table is a bijection) and no atomics are needed.
//   k_tb_finish   decode_tb / decode_tb_cb epilogue (src/phy/phch/sch.c:393-491): TB bytes from
//                 the per-CB decisions (or from the softbuffer's saved bytes for CBs that passed
//                 in an earlier transmission), cb_crc / saved-data update, nof_iterations and
//                 the TB CRC24A check.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "dlsch_kernels.h"
#include "uci_dev.h"
#include "wave_prio.h"
#include "srsgpu/dlsch_batch.h"

#include <algorithm>

namespace srsgpu {

// Pointers read from an item descriptor are generic to the compiler, and accesses through them
// become flat instructions, which count against lgkmcnt too (the LDS waits then wait for global
// loads in flight). The descriptors only ever point at global memory: say so.
template <typename T> using gp_t = T __attribute__((address_space(1))) *;
template <typename T> __device__ __forceinline__ gp_t<T> glob(T *p) {
  return (gp_t<T>)(__attribute__((address_space(1))) void *)(uintptr_t)p;
}
typedef uint32_t u4v __attribute__((ext_vector_type(4))); // HIP's uint4 class has no AS-1 methods
// generic pointer known to be global (the address-space inference turns its accesses into global_*)
template <typename T> __device__ __forceinline__ T *glob_g(T *p) { return (T *)glob(p); }
// one softbuffer entry: int16 wrap, or (w8) int8 wrap sign-extended into the int16 entry
__device__ __forceinline__ uint32_t derm_fold(uint32_t v, bool w8) {
  return w8 ? (uint32_t)(uint16_t)(int16_t)(int8_t)(uint8_t)v : v & 0xFFFFu;
}

// One workgroup per code block, gathering by row position: entry o of the softbuffer row becomes
// old[o] (or 0 when the row was reset since its last use: lazy reset, no memset pass) plus the
// sum of the E received LLRs e[i] with i = m (mod N), m = inv[o] the circular-buffer entry that
// lands on o. Eight consecutive entries per thread: one 16-byte inverse-table load, one 16-byte
// row load (unless fresh) and one 16-byte row store; the LLRs (≈14 KB per block) are gathered
// from L1/L2. Wrapping int16 sums, as rm_turbo.c:394-430's `output[j] += input[i]`, so the order
// of the additions does not matter.
#define DERM_LDS 12288 // LLRs staged per code block (24 KB of LDS)
// The E LLRs of one code block into LDS words (two per word) by a 256-thread workgroup: 16-byte
// loads for the aligned middle, 4-byte loads for the head and tail words (E is even for every Qm,
// so the block's LLRs start 4-byte aligned; an odd tail is read alone), 2-byte pairs otherwise.
__device__ __forceinline__ void stage_llrs(uint32_t *es, const int16_t *ep, uint32_t ne) {
  const gp_t<const uint16_t> e = glob(reinterpret_cast<const uint16_t *>(ep));
  if (((uintptr_t)ep & 3) == 0) {
    const gp_t<const uint32_t> e32 = glob(reinterpret_cast<const uint32_t *>(ep));
    const uint32_t nw2 = ne / 2;
    const uint32_t head = (uint32_t)((16 - ((uintptr_t)ep & 15)) & 15) / 4; // words to alignment
    const uint32_t h = head < nw2 ? head : nw2;
    const uint32_t nq = (nw2 - h) / 4;
    const gp_t<const u4v> e4 = glob(reinterpret_cast<const u4v *>(ep + 2 * h));
#pragma unroll 4
    for (uint32_t q = threadIdx.x; q < nq; q += blockDim.x) {
      const u4v v = e4[q];
      es[h + 4 * q] = v.x;
      es[h + 4 * q + 1] = v.y;
      es[h + 4 * q + 2] = v.z;
      es[h + 4 * q + 3] = v.w;
    }
    const uint32_t t0 = h + 4 * nq; // tail words t0 .. nw2-1 (at most 3) and the head words
    if (threadIdx.x < h) es[threadIdx.x] = e32[threadIdx.x];
    if (threadIdx.x >= 64 && threadIdx.x - 64 < nw2 - t0) es[t0 + threadIdx.x - 64] = e32[t0 + threadIdx.x - 64];
    if ((ne & 1) && threadIdx.x == 128) es[ne / 2] = e[ne - 1];
  } else {
    const uint32_t nw = (ne + 1) / 2;
    for (uint32_t w = threadIdx.x; w < nw; w += blockDim.x)
      es[w] = (uint32_t)e[2 * w] | (2 * w + 1 < ne ? (uint32_t)e[2 * w + 1] << 16 : 0u);
  }
}

// the full descriptor of record i of a call
__device__ __forceinline__ DermItem derm_get(const DermCall &c, uint32_t i) {
  const DermRec r = c.rec[i];
  const DermTabs t = c.tabs[r.tab];
  DermItem it;
  it.e = c.e + r.e_off;
  it.ne = r.ne;
  it.N = r.N;
  it.table = t.table;
  it.inv = t.inv;
  it.inv_t4 = t.inv_t4;
  it.row = c.soft + (size_t)r.row * SRSGPU_SOFTBUFFER_SIZE;
  it.cb_crc = c.cbcrc + r.row;
  it.fresh = c.fresh + r.row;
  it.pos = r.pos;
  it.rowlen = r.rowlen;
  it.w8 = r.w8;
  it.direct = r.direct;
  it.tb_ret = c.ret + r.tb;
  return it;
}

// phase 0: before the decode, every item not `direct`; phase 1: after k_tb_finish, the direct
// items of failed TBs that were not decoded before this call (their rows as the reference leaves
// them; an acked TB's rows are never read again: sch.c:323 skips blocks whose CRC passed, and the
// next TB resets the softbuffer)
// one code block into its row by the whole workgroup (es: DERM_LDS / 2 words of LDS)
__device__ __forceinline__ void derm_item(const DermItem &it, uint32_t *es) {
  const bool fresh = it.fresh && *glob(it.fresh);
  const bool w8 = it.w8 != 0;
  const uint32_t N = it.N, ne = it.ne, len = it.rowlen;
  const gp_t<const uint16_t> e = glob(reinterpret_cast<const uint16_t *>(it.e));
  auto add = [&](uint32_t old, uint32_t m) -> uint32_t { // one entry, wrapping
    uint32_t acc = old;
    for (uint32_t i = m; i < ne; i += N) acc += e[i];
    return derm_fold(acc, w8);
  };
  const uint32_t nv = (len + 7) / 8; // the inverse table is padded: entries past len are 0xFFFF
  const gp_t<const u4v> inv = glob(reinterpret_cast<const u4v *>(it.inv));
  const gp_t<u4v> row = glob(reinterpret_cast<u4v *>(it.row));
  // rows hold SOFTBUFFER_SIZE entries, so the padded tail of the last vector stays inside the
  // row; entries past len keep their value (or become 0 on a fresh row)
  if (ne <= N && ne <= DERM_LDS) {
    // each circular-buffer entry received at most once (the usual case): the E LLRs are staged
    // in LDS with 16-byte loads and gathered from there (scattered 2-byte global gathers cost
    // one address-unit slot per lane)
    stage_llrs(es, it.e, ne);
    __syncthreads();
    const uint16_t *el = reinterpret_cast<const uint16_t *>(es);
#pragma unroll 4
    for (uint32_t v = threadIdx.x; v < nv; v += blockDim.x) {
      const u4v iv = inv[v];
      const u4v ov = fresh ? u4v{0, 0, 0, 0} : row[v];
      const uint32_t im[4] = {iv.x, iv.y, iv.z, iv.w}, om[4] = {ov.x, ov.y, ov.z, ov.w};
      uint32_t r[4];
#pragma unroll
      for (int h = 0; h < 4; h++) {
        const uint32_t m0 = im[h] & 0xFFFFu, m1 = im[h] >> 16;
        const uint32_t e0 = m0 < ne ? el[m0] : 0u, e1 = m1 < ne ? el[m1] : 0u; // 0xFFFF >= ne
        if (w8)
          r[h] = derm_fold(om[h] + e0, true) | (derm_fold((om[h] >> 16) + e1, true) << 16);
        else
          r[h] = ((om[h] + e0) & 0xFFFFu) | (((om[h] >> 16) + e1) << 16);
      }
      row[v] = u4v{r[0], r[1], r[2], r[3]};
    }
  } else {
    for (uint32_t v = threadIdx.x; v < nv; v += blockDim.x) {
      const u4v iv = inv[v];
      const u4v ov = fresh ? u4v{0, 0, 0, 0} : row[v];
      const uint32_t im[4] = {iv.x, iv.y, iv.z, iv.w}, om[4] = {ov.x, ov.y, ov.z, ov.w};
      uint32_t r[4];
#pragma unroll
      for (int h = 0; h < 4; h++) {
        const uint32_t m0 = im[h] & 0xFFFFu, m1 = im[h] >> 16;
        const uint32_t lo = m0 == 0xFFFFu ? om[h] & 0xFFFFu : add(om[h] & 0xFFFFu, m0);
        const uint32_t hi = m1 == 0xFFFFu ? om[h] >> 16 : add(om[h] >> 16, m1);
        r[h] = lo | (hi << 16);
      }
      row[v] = u4v{r[0], r[1], r[2], r[3]};
    }
  }
  __syncthreads();
  if (fresh && threadIdx.x == 0) *glob(it.fresh) = 0; // the row now holds real soft bits
}

__global__ __launch_bounds__(256) void k_derm(DermCall dc, int nitems, uint8_t *__restrict__ init_done) {
  __shared__ uint32_t es[DERM_LDS / 2];
  const int g = blockIdx.x;
  if (g >= nitems) return;
  const DermItem it = derm_get(dc, g);
  const uint8_t skip = it.cb_crc ? *glob(it.cb_crc) : 0;
  if (threadIdx.x == 0) init_done[it.pos] = skip;
  if (skip || it.direct) return; // sch.c:323: blocks whose CRC passed before are not combined again
  derm_item(it, es);
}

// the deferred rows: the direct blocks k_tb_finish listed (late[0] of them at late[1..], decoder
// positions: blocks of failed TBs not decoded before the call), a few workgroups looping over the
// list, so an all-acked batch costs one short launch
__global__ __launch_bounds__(256) void k_derm_late(DermCall dc, const uint32_t *__restrict__ late) {
  __shared__ uint32_t es[DERM_LDS / 2];
  const uint32_t n = late[0];
  for (uint32_t q = blockIdx.x; q < n; q += gridDim.x) {
    const DermItem it = derm_get(dc, late[1 + q]);
    derm_item(it, es);
    __syncthreads(); // es is reused by the next block
  }
}

// srsgpu_rm_turbo_rx_dev: arbitrary output buffers, read-modify-write in place (one block)
__global__ __launch_bounds__(256) void k_derm_rmw(const DermItem *__restrict__ items) {
  const DermItem it = items[0];
  const uint32_t N = it.N;
  const uint32_t lim = it.ne < N ? it.ne : N;
  for (uint32_t m = blockIdx.x * 256 + threadIdx.x; m < lim; m += gridDim.x * 256) {
    uint32_t acc = 0;
    for (uint32_t i = m; i < it.ne; i += N) acc += (uint16_t)it.e[i];
    const uint32_t o = it.table[m];
    it.row[o] = (int16_t)(uint16_t)derm_fold((uint16_t)it.row[o] + acc, it.w8 != 0);
  }
}

__global__ __launch_bounds__(256) void k_derm_flags(DermCall dc, int n, uint8_t *__restrict__ init_done,
                                                    uint32_t *__restrict__ late) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i == 0 && late) late[0] = 0;
  if (i >= n) return;
  const DermRec r = dc.rec[i];
  init_done[r.pos] = dc.cbcrc[r.row];
}

// ------------------------------------------------------------------ direct de-RM ----
// k_derm followed by k_load_sbt (tdec_kernels.hip) in one pass, for the window decoders' groups:
// the decoder input at softbuffer-row position o of code block c is what k_derm would store
// there, (fresh ? 0 : row[o]) + the LLRs e[i] with i = inv[o] (mod N). The inverse table comes in
// the decoder's own T4 order (DermItem::inv_t4, built per (K, rv) on the host), so every output is
// computed where it is stored: one workgroup per code-block pair stages both blocks' LLRs in LDS
// (dynamic, `stage` per block), then each thread forms whole 16-byte SP0 / P1 vectors from
// coalesced table loads and LDS gathers, consecutive lanes storing consecutive vectors. Reused
// rows (HARQ retransmissions, not fresh) add their old entries, read at their row positions. HBM
// traffic per code block: its E LLRs in and the 12 B per info bit of SP0 / P1 out (the separate
// passes also wrote and re-read the 3(K+32)+12 row entries).
#define LDR_THREADS 256
// mode 0: SP0, P1 and T of every pair; 1: SP0 and T only (P1 deferred: the first half-iteration does
// not read it, and at high SNR few blocks reach the second); 2: P1 only, for the pairs k_decide listed
// as still running after the first half-iteration (TdEs::run_list / run_cnt per group at pair0:
// workgroup j of a group takes its list entry j)
struct LdrBlk {
  const int16_t *e, *row;
  const uint16_t *t4;
  uint32_t ne, N;
  bool fresh, staged;
};
__device__ __forceinline__ LdrBlk ldr_blk(const DermCall &dc, int c, uint32_t stage) {
  const DermItem it = derm_get(dc, c);
  return LdrBlk{it.e, it.row, it.inv_t4, it.ne, it.N, it.fresh && *glob(it.fresh), it.ne <= it.N && it.ne <= stage};
}
// the usual first transmission: both rows fresh, both blocks' LLRs staged, one table (same K and rv),
// 16-bit: an output element is the staged LLR its table entry m names (0 past E), the same m for both
// blocks — two table words per 16-byte SP0 vector, no per-element branches
__device__ __forceinline__ bool ldr_fast_ok(const LdrBlk &a, const LdrBlk &b, bool w8) {
  return a.fresh && b.fresh && a.staged && b.staged && a.t4 == b.t4 && !w8;
}
// tw: the table's stream-0/1 words (entries 2v, 2v+1 of stream st at word st ne/2 + v), in LDS or HBM
template <typename TW>
__device__ __forceinline__ void ldr_fast(TW tw, const LdrBlk &ba, const LdrBlk &bb, const uint16_t *l0,
                                         const uint16_t *l1, int ne, int mode, gp_t<u4v> SP0, gp_t<u4v> P1,
                                         uint32_t *T12) {
  const uint32_t na = ba.ne, nbk = bb.ne;
  auto pk = [&](uint32_t m) -> uint32_t {
    return (m < na ? (uint32_t)l0[m] : 0u) | ((m < nbk ? (uint32_t)l1[m] : 0u) << 16);
  };
#pragma unroll 4
  for (int v = threadIdx.x; v < (mode == 2 ? 0 : ne / 2); v += LDR_THREADS) {
    const uint32_t sa = tw[v], pa = tw[ne / 2 + v];
    SP0[v] = u4v{pk(sa & 0xFFFFu), pk(pa & 0xFFFFu), pk(sa >> 16), pk(pa >> 16)};
  }
  typedef uint32_t u2f __attribute__((ext_vector_type(2)));
  const gp_t<const u2f> qa = glob(reinterpret_cast<const u2f *>(ba.t4 + 2 * ne));
#pragma unroll 4
  for (int v = threadIdx.x; v < (mode == 1 ? 0 : ne / 4); v += LDR_THREADS) {
    const u2f ma = qa[v];
    P1[v] = u4v{pk(ma.x & 0xFFFFu), pk(ma.x >> 16), pk(ma.y & 0xFFFFu), pk(ma.y >> 16)};
  }
  if (threadIdx.x < 12 && mode != 2) glob(T12)[threadIdx.x] = pk(glob(ba.t4)[3 * ne + threadIdx.x]);
}
// every other case (HARQ combining with the row's old entries, unstaged LLRs, two tables, 8-bit)
__device__ __forceinline__ void ldr_generic(const LdrBlk &ba, const LdrBlk &bb, const uint16_t *l0, const uint16_t *l1,
                                            bool w8, int K, int nb, int ne, int mode, gp_t<u4v> SP0, gp_t<u4v> P1,
                                            uint32_t *T12) {
  const int L = K / nb;
  // value of T4 element el of stream st of block b, given its table entry m
  auto value = [&](const LdrBlk &b, const uint16_t *lds, int st, int el, uint32_t m) -> uint32_t {
    uint32_t acc = 0;
    if (!b.fresh) { // the row's old entry at its row position (padded steps: step L - 1's)
      const int k = min(4 * (el / (4 * nb)) + (el & 3), L - 1), d = (el >> 2) % nb;
      acc = (uint16_t)glob(b.row)[st * (K + 32) + k * nb + d];
    }
    if (b.staged) {
      acc += m < b.ne ? (uint32_t)lds[m] : 0u; // 0xFFFF >= ne
    } else if (m != 0xFFFFu) {
      const gp_t<const uint16_t> e = glob(reinterpret_cast<const uint16_t *>(b.e));
      for (uint32_t i = m; i < b.ne; i += b.N) acc += e[i];
    }
    return derm_fold(acc, w8) & 0xFFFFu;
  };
  const gp_t<const uint32_t> ta = glob(reinterpret_cast<const uint32_t *>(ba.t4));
  const gp_t<const uint32_t> tb = glob(reinterpret_cast<const uint32_t *>(bb.t4));
  // SP0: vector v holds T4 elements 2v, 2v + 1 as (sys a, sys b, p0 a, p0 b) each
#pragma unroll 4
  for (int v = threadIdx.x; v < (mode == 2 ? 0 : ne / 2); v += LDR_THREADS) {
    const uint32_t sa = ta[v], pa = ta[ne / 2 + v], sb = tb[v], pb = tb[ne / 2 + v];
    const int el = 2 * v;
    SP0[v] = u4v{value(ba, l0, 0, el, sa & 0xFFFFu) | (value(bb, l1, 0, el, sb & 0xFFFFu) << 16),
                 value(ba, l0, 1, el, pa & 0xFFFFu) | (value(bb, l1, 1, el, pb & 0xFFFFu) << 16),
                 value(ba, l0, 0, el + 1, sa >> 16) | (value(bb, l1, 0, el + 1, sb >> 16) << 16),
                 value(ba, l0, 1, el + 1, pa >> 16) | (value(bb, l1, 1, el + 1, pb >> 16) << 16)};
  }
  // P1: vector v holds T4 elements 4v .. 4v + 3 as (p1 a, p1 b) each
  typedef uint32_t u2v __attribute__((ext_vector_type(2)));
  const gp_t<const u2v> qa = glob(reinterpret_cast<const u2v *>(ba.t4 + 2 * ne));
  const gp_t<const u2v> qb = glob(reinterpret_cast<const u2v *>(bb.t4 + 2 * ne));
#pragma unroll 4
  for (int v = threadIdx.x; v < (mode == 1 ? 0 : ne / 4); v += LDR_THREADS) {
    const u2v ma = qa[v], mb = qb[v];
    const int el = 4 * v;
    P1[v] = u4v{value(ba, l0, 2, el, ma.x & 0xFFFFu) | (value(bb, l1, 2, el, mb.x & 0xFFFFu) << 16),
                value(ba, l0, 2, el + 1, ma.x >> 16) | (value(bb, l1, 2, el + 1, mb.x >> 16) << 16),
                value(ba, l0, 2, el + 2, ma.y & 0xFFFFu) | (value(bb, l1, 2, el + 2, mb.y & 0xFFFFu) << 16),
                value(ba, l0, 2, el + 3, ma.y >> 16) | (value(bb, l1, 2, el + 3, mb.y >> 16) << 16)};
  }
  if (threadIdx.x < 12 && mode != 2) { // the tails: row positions 3(K+32) .. +11, table entries 3 ne + t
    const int t = threadIdx.x;
    auto tail = [&](const LdrBlk &b, const uint16_t *lds) -> uint32_t {
      const uint32_t m = glob(b.t4)[3 * ne + t];
      uint32_t acc = b.fresh ? 0u : (uint16_t)glob(b.row)[3 * (K + 32) + t];
      if (b.staged) {
        acc += m < b.ne ? (uint32_t)lds[m] : 0u;
      } else if (m != 0xFFFFu) {
        const gp_t<const uint16_t> e = glob(reinterpret_cast<const uint16_t *>(b.e));
        for (uint32_t i = m; i < b.ne; i += b.N) acc += e[i];
      }
      return derm_fold(acc, w8) & 0xFFFFu;
    };
    const uint32_t va = tail(ba, l0), vb = tail(bb, l1);
    glob(T12)[t] = va | (vb << 16);
  }
}

// the last group whose first load workgroup is <= w
__device__ __forceinline__ int ldr_group(const TdGroup *__restrict__ groups, int ngroups, int w) {
  int lo = 0, hi = ngroups - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (groups[mid].blk_load <= w)
      lo = mid;
    else
      hi = mid - 1;
  }
  return lo;
}

__global__ __launch_bounds__(LDR_THREADS) void k_load_derm(const TdGroup *__restrict__ groups, int ngroups,
                                                           DermCall dc, TdArrays arr, uint32_t stage, int mode,
                                                           const uint32_t *__restrict__ list,
                                                           const uint32_t *__restrict__ cnt, int fast) {
  extern __shared__ __attribute__((aligned(16))) uint32_t ldr_lds[];
  uint32_t *llr0 = ldr_lds, *llr1 = ldr_lds + stage / 2;
  const TdGroup &G = groups[ldr_group(groups, ngroups, (int)blockIdx.x)];
  const int K = G.K, ncb = G.ncb, npairs = G.npairs, nb = G.nb;
  int pair = blockIdx.x - G.blk_load;
  if (pair >= npairs) return;
  if (mode == 2) {
    if (pair >= (int)cnt[G.pair0]) return;
    pair = (int)list[G.pair0 + pair];
  }
  const int L = K / nb, G4 = (L + 3) >> 2, ne = nb * 4 * G4;
  const int c0 = G.cb0 + 2 * pair, c1 = 2 * pair + 1 < ncb ? c0 + 1 : c0;
  const LdrBlk ba = ldr_blk(dc, c0, stage), bb = ldr_blk(dc, c1, stage);
  const bool w8 = dc.rec[c0].w8 != 0; // one LLR width per call
  if (ba.staged) stage_llrs(llr0, ba.e, ba.ne);
  if (bb.staged) stage_llrs(llr1, bb.e, bb.ne);
  __syncthreads();
  const uint16_t *l0 = reinterpret_cast<const uint16_t *>(llr0), *l1 = reinterpret_cast<const uint16_t *>(llr1);
  const size_t pbase = (size_t)G.elem0 + (size_t)pair * t4_pair_elems(K, nb);
  const gp_t<u4v> SP0 = glob(reinterpret_cast<u4v *>((int16_t *)arr.SP0 + 4 * pbase));
  const gp_t<u4v> P1 = glob(reinterpret_cast<u4v *>((int16_t *)arr.XP1 + 2 * (arr.plane + pbase)));
  uint32_t *T12 = reinterpret_cast<uint32_t *>(arr.T) + (size_t)(G.pair0 + pair) * 12;
  if (fast && ldr_fast_ok(ba, bb, w8))
    ldr_fast(glob(reinterpret_cast<const uint32_t *>(ba.t4)), ba, bb, l0, l1, ne, mode, SP0, P1, T12);
  else
    ldr_generic(ba, bb, l0, l1, w8, K, nb, ne, mode, SP0, P1, T12);
}

// The previous form of k_load_derm, kept for A/B measurements (SRSGPU_LDERM=tile): row-order
// inverse tables, six (stream, block) chunks of 2048 row positions formed in LDS per tile and
// written out in the T4 layout through an LDS transposition, 512 threads per pair.
#define LDT_THREADS 512
#define LDT_TILE 2048                      // row positions per (stream, block) chunk of a tile
#define LDT_PIECES (6 * LDT_TILE / 8)      // 16-byte pieces of a tile
#define LDT_PPT (LDT_PIECES / LDT_THREADS) // pieces per thread
__global__ __launch_bounds__(LDT_THREADS) void k_load_derm_tile(const TdGroup *__restrict__ groups, int ngroups,
                                                           DermCall dc, TdArrays arr, uint32_t stage) {
  extern __shared__ __attribute__((aligned(16))) uint32_t ldt_lds[];
  uint16_t(*tile)[LDT_TILE] = reinterpret_cast<uint16_t(*)[LDT_TILE]>(ldt_lds); // [6][LDT_TILE]
  uint32_t *llr0 = ldt_lds + 6 * LDT_TILE / 2, *llr1 = llr0 + stage / 2;
  int gi = 0;
  { // the last group whose first workgroup is <= blockIdx.x
    int lo = 0, hi = ngroups - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (groups[mid].blk_load <= (int)blockIdx.x)
        lo = mid;
      else
        hi = mid - 1;
    }
    gi = lo;
  }
  const TdGroup &G = groups[gi];
  const int K = G.K, ncb = G.ncb, npairs = G.npairs, nb = G.nb;
  const int pair = blockIdx.x - G.blk_load;
  if (pair >= npairs) return;
  const int L = K / nb, G4 = (L + 3) >> 2, S = LDT_TILE / nb;
  const int c0 = G.cb0 + 2 * pair, c1 = 2 * pair + 1 < ncb ? c0 + 1 : c0;
  // the two blocks' fields (selected by h, which is wave-uniform: no indexed private arrays)
  struct Blk {
    const int16_t *e, *row;
    const uint16_t *inv;
    uint32_t ne, N;
    bool fresh, staged;
  };
  auto blk = [&](int c) {
    const DermItem it = derm_get(dc, c);
    return Blk{it.e, it.row, it.inv, it.ne, it.N, it.fresh && *glob(it.fresh),
               it.ne <= it.N && it.ne <= stage};
  };
  const Blk ba = blk(c0), bb = blk(c1);
  const bool w8 = dc.rec[c0].w8 != 0; // one LLR width per call
  // tile pieces: chunk c = (stream, block), 8 row positions from sub-block index e
  auto piece_at = [&](int q, int k0, int &c, int &pc, uint32_t &o8) {
    const int idx = threadIdx.x + LDT_THREADS * q;
    c = idx / (LDT_TILE / 8);
    pc = idx - c * (LDT_TILE / 8);
    const int st = c >> 1;
    int e = k0 * nb + pc * 8; // past the last step: its copy (values unused)
    if (e >= L * nb) e = (L - 1) * nb + (e & (nb - 1));
    o8 = (uint32_t)(st * (K + 32) + e) / 8;
  };
  u4v iv[LDT_PPT], ov[LDT_PPT];
  auto fetch = [&](int k0) {
#pragma unroll
    for (int q = 0; q < LDT_PPT; q++) {
      int c, pc;
      uint32_t o8;
      piece_at(q, k0, c, pc, o8);
      const Blk &b = (c & 1) ? bb : ba;
      iv[q] = glob(reinterpret_cast<const u4v *>(b.inv))[o8];
      ov[q] = b.fresh ? u4v{0, 0, 0, 0} : glob(reinterpret_cast<const u4v *>(b.row))[o8];
    }
  };
  fetch(0); // the first tile's table loads fly while the LLRs are staged
  if (ba.staged) stage_llrs(llr0, ba.e, ba.ne);
  if (bb.staged) stage_llrs(llr1, bb.e, bb.ne);
  __syncthreads();
  // value of a row position of block b given its inverse-table entry m and the row's old value
  auto value = [&](const Blk &b, const uint16_t *lds, uint32_t m, uint32_t old) -> uint32_t {
    uint32_t acc = b.fresh ? 0u : old;
    if (b.staged) {
      acc += m < b.ne ? (uint32_t)lds[m] : 0u; // 0xFFFF >= ne
    } else if (m != 0xFFFFu) {
      const gp_t<const uint16_t> e = glob(reinterpret_cast<const uint16_t *>(b.e));
      for (uint32_t i = m; i < b.ne; i += b.N) acc += e[i];
    }
    return derm_fold(acc, w8);
  };
  const size_t pbase = (size_t)G.elem0 + (size_t)pair * t4_pair_elems(K, nb);
  const gp_t<u4v> SP0 = glob(reinterpret_cast<u4v *>((int16_t *)arr.SP0 + 4 * pbase));
  const gp_t<u4v> P1 = glob(reinterpret_cast<u4v *>((int16_t *)arr.XP1 + 2 * (arr.plane + pbase)));
  for (int k0 = 0; k0 < 4 * G4; k0 += S) {
#pragma unroll
    for (int q = 0; q < LDT_PPT; q++) {
      int c, pc;
      uint32_t o8;
      piece_at(q, k0, c, pc, o8);
      const bool h = c & 1;
      const Blk &b = h ? bb : ba;
      const uint16_t *lds = reinterpret_cast<const uint16_t *>(h ? llr1 : llr0);
      const uint32_t im[4] = {iv[q].x, iv[q].y, iv[q].z, iv[q].w}, om[4] = {ov[q].x, ov[q].y, ov[q].z, ov[q].w};
      uint32_t r[4];
#pragma unroll
      for (int u = 0; u < 4; u++)
        r[u] = (value(b, lds, im[u] & 0xFFFFu, om[u] & 0xFFFFu) & 0xFFFFu) |
               (value(b, lds, im[u] >> 16, om[u] >> 16) << 16);
      *reinterpret_cast<u4v *>(&tile[c][pc * 8]) = u4v{r[0], r[1], r[2], r[3]};
    }
    __syncthreads();
    if (k0 + S < 4 * G4) fetch(k0 + S);
    // the tile's steps as T4 elements: el -> step (el / 4 / nb) * 4 + el % 4, chain el / 4 % nb
    const int nel = min(S, 4 * G4 - k0) * nb;
    auto at = [&](int c, int el) -> uint32_t {
      const int g4l = el / (4 * nb), d = (el >> 2) % nb, u = el & 3;
      return tile[c][(4 * g4l + u) * nb + d];
    };
    const size_t e0 = (size_t)k0 * nb; // T4 element of the tile's first step
#pragma unroll
    for (int q = 0; q < LDT_TILE / 2 / LDT_THREADS; q++) {
      const int v = threadIdx.x + LDT_THREADS * q; // SP0 elements 2v, 2v + 1
      if (2 * v < nel) {
        const int ea = 2 * v, eb = 2 * v + 1;
        SP0[e0 / 2 + v] = u4v{at(0, ea) | (at(1, ea) << 16), at(2, ea) | (at(3, ea) << 16),
                              at(0, eb) | (at(1, eb) << 16), at(2, eb) | (at(3, eb) << 16)};
      }
    }
    if (4 * (int)threadIdx.x < nel) {
      const int e = 4 * threadIdx.x;
      P1[e0 / 4 + threadIdx.x] = u4v{at(4, e) | (at(5, e) << 16), at(4, e + 1) | (at(5, e + 1) << 16),
                                     at(4, e + 2) | (at(5, e + 2) << 16), at(4, e + 3) | (at(5, e + 3) << 16)};
    }
    __syncthreads();
  }
  if (threadIdx.x < 12) { // the tails: row positions 3(K+32) .. +11
    const int t = threadIdx.x;
    const uint32_t o = 3u * (K + 32) + t;
    auto tail = [&](const Blk &b, const uint32_t *l) -> uint32_t {
      const uint32_t m = glob(b.inv)[o];
      const uint32_t old = b.fresh ? 0u : (uint16_t)glob(b.row)[o];
      return value(b, reinterpret_cast<const uint16_t *>(l), m, old) & 0xFFFFu;
    };
    const uint32_t va = tail(ba, llr0), vb = tail(bb, llr1);
    glob(reinterpret_cast<uint32_t *>(arr.T))[(size_t)(G.pair0 + pair) * 12 + t] = va | (vb << 16);
  }
}

// XOR-reduce one value per thread over the workgroup
__device__ __forceinline__ uint32_t wg_xor(uint32_t v, uint32_t *red) {
  for (int o = 32; o > 0; o >>= 1) v ^= __shfl_xor(v, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  uint32_t r = 0;
  for (int w = 0; w < (int)(blockDim.x >> 6); w++) r ^= red[w];
  __syncthreads();
  return r;
}

// One workgroup per TB. The per-CB bookkeeping is gathered first (thread i: CB i's index,
// init_done, sizes; the cb_crc / noi update), then every byte is moved by all threads at once and
// the CRC weights are fetched eight bytes per thread and round: the TB's dependent loads are a few
// round trips, not one chain per CB (the CB-serial form spent ~60 us per 512-TB launch waiting).
#define TBF_MAXC 64 // > SRSLTE_MAX_CODEBLOCKS (phy_common.h:57)
#define TBF_FZ 32   // code blocks of one TB whose bytes the workgroup makes from decision words (FzSrc)

// Natural-order bytes of decoder block g from its frozen decision words (es_check / sse_es_check:
// Dfz, cb_end = 1 + parity of the half-iteration that ended it), exactly as k_es_bytes writes them
// (turbodecoder.c:353-360 + decision_byte, MSB first), into `out` (LDS) by the whole workgroup.
__device__ void fz_bytes(const FzSrc &fz, int gi, int g, int end, uint32_t *dw, uint8_t *out) {
  const TdGroup &G = fz.groups[gi];
  const int K = G.K, NB = G.nb, c = g - G.cb0, pair = c >> 1, h = c & 1;
  const int L = K / NB, G16 = (L + 15) / 16, nw = NB * G16;
  const gp_t<const uint32_t> src = glob(fz.dfz + G.dw0 + (size_t)pair * nw);
  for (int q = threadIdx.x; q < nw; q += blockDim.x) dw[q] = src[q];
  __syncthreads();
  const gp_t<const uint16_t> dmap = glob(G.dmap);
  const bool dec2 = end == 2;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const float invL = 1.0f / (float)L;
  const int gap = 16 * G16 - L;
  constexpr int PMAX = 6144 / 256;
  int ci[PMAX];
#pragma unroll
  for (int u = 0; u < PMAX; u++) { // every map load issued before the first use
    const int p = wv * 64 + u * 256 + lane;
    int cc = 0;
    if (p < K) {
      if (dec2) {
        cc = (int)dmap[p];
      } else {
        const int d = (int)(((float)p + 0.5f) * invL); // exact: see k_decide
        cc = p + d * gap;
      }
    }
    ci[u] = cc;
  }
#pragma unroll
  for (int u = 0; u < PMAX; u++) {
    const int p0 = wv * 64 + u * 256;
    if (p0 >= K) break;
    const int p = p0 + lane;
    const uint32_t bit = p < K ? (dw[ci[u] >> 4] >> ((ci[u] & 15) + 16 * h)) & 1u : 0u;
    const uint64_t m = __ballot(bit);
    if (lane < 8 && p0 + 8 * lane < K)
      out[(p0 >> 3) + lane] = (uint8_t)(__builtin_bitreverse32((uint32_t)((m >> (8 * lane)) & 0xffu)) >> 24);
  }
  __syncthreads(); // dw is reused by the next block
}

__global__ __launch_bounds__(256) void k_tb_finish(const TbItem *__restrict__ tbs_, int ntb,
                                                   const uint32_t *__restrict__ cbmap,
                                                   const uint8_t *__restrict__ dec, size_t dec_stride,
                                                   const uint8_t *__restrict__ cb_ok_in,
                                                   const uint8_t *__restrict__ init_done,
                                                   const uint32_t *__restrict__ noi_in,
                                                   const uint32_t *__restrict__ crc_a, DermCall dc,
                                                   uint32_t *__restrict__ late, int prio, FzSrc fz,
                                                   int inline_rows) {
  __shared__ uint32_t red[4];
  __shared__ uint32_t crc_tab[256];
  __shared__ uint32_t c_ck0[TBF_MAXC + 1];
  __shared__ uint32_t c_g[TBF_MAXC], c_dst[TBF_MAXC], c_nb[TBF_MAXC], c_rb[TBF_MAXC];
  __shared__ uint8_t c_init[TBF_MAXC], c_ok[TBF_MAXC];
  __shared__ int8_t c_fz[TBF_MAXC];    // slot of the block's bytes in fzb, -1: in dec / saved
  __shared__ uint8_t c_end[TBF_MAXC];  // cb_end of the block (FzSrc)
  __shared__ int16_t c_grp[TBF_MAXC];  // its decoder group
  __shared__ uint32_t fz_dw[6144 / 16 + 16];
  // the bytes made here (TBF_FZ blocks x 768), later the LLR staging of the inline rows (DERM_LDS)
  __shared__ __attribute__((aligned(16))) uint32_t fz_lds[(TBF_FZ * 768 > DERM_LDS * 2 ? TBF_FZ * 768 : DERM_LDS * 2) / 4];
  uint8_t *fzb = reinterpret_cast<uint8_t *>(fz_lds);
  __shared__ int all_ok;
  __shared__ uint32_t noi_sum;
  wave_prio(prio);
  const int b = blockIdx.x;
  if (b >= ntb) return;
  TbItem t = tbs_[b];
  t.data = glob_g(t.data);
  t.cb_crc = glob_g(t.cb_crc);
  t.saved = glob_g(t.saved);
  t.ret = glob_g(t.ret);
  t.noi = glob_g(t.noi);
  if (t.C == 0 || t.C > TBF_MAXC) { // tbs == 0 (sch.c:451-453) or invalid inputs: result set on the host
    if (threadIdx.x == 0) {
      *t.ret = t.C ? -1 : t.preset_ret;
      *t.noi = 0;
    }
    return;
  }
  const uint32_t C = t.C;
  // 1. per CB i (thread i): its global index, where its bytes go (CB i owns [i*rlen/8, ...); the last
  //    CB also writes its 3 CRC bytes, as its full K/8-byte decision lands last in the reference,
  //    sch.c:363-366), init_done, and the cb_crc / nof_iterations update of sch.c:394-419
  if (threadIdx.x < 64) {
    const uint32_t i = threadIdx.x;
    uint32_t s = 0;
    int ok = 1;
    if (i < C) {
      const uint32_t K = i < t.C1 ? t.K1 : t.K2;
      const uint32_t rlen = C == 1 ? K : K - 24;
      const uint32_t g = cbmap[t.first + i];
      const uint8_t ini = init_done[g];
      c_g[i] = g;
      c_dst[i] = i * (rlen / 8);
      c_rb[i] = rlen / 8;
      c_nb[i] = ini ? rlen / 8 : (i == C - 1 ? K / 8 : rlen / 8);
      c_init[i] = ini;
      uint8_t crc_i = t.cb_crc[i];
      if (!ini) {
        s = noi_in[g];
        if (cb_ok_in[g]) {
          crc_i = 1;
          t.cb_crc[i] = 1;
        }
      }
      c_ok[i] = crc_i;
      ok = crc_i != 0;
    }
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    ok = __all(ok);
    if (i == 0) {
      all_ok = ok;
      noi_sum = s;
    }
    // blocks a fused early-stop launch ended: their bytes are made here from the decision words
    c_fz[i] = -1;
    if (fz.groups && i < C && !c_init[i]) {
      const int g = (int)c_g[i];
      const uint8_t end = glob(fz.cb_end)[g];
      c_end[i] = end;
      if (end) {
        int gi = 0;
        while (gi + 1 < fz.ngroups && !(fz.groups[gi].cb0 <= g && g < fz.groups[gi].cb0 + fz.groups[gi].ncb)) gi++;
        c_grp[i] = (int16_t)gi;
      }
    } else if (i < C) {
      c_end[i] = 0;
    }
  }
  __syncthreads();
  if (fz.groups) {
    int slot = 0;
    for (uint32_t i = 0; i < C; i++) {
      if (!c_end[i]) continue;
      if (slot < TBF_FZ) {
        fz_bytes(fz, c_grp[i], (int)c_g[i], c_end[i], fz_dw, fzb + 768 * slot);
        if (threadIdx.x == 0) {
          c_fz[i] = (int8_t)slot;
          glob(fz.cb_end)[c_g[i]] = 0;
        }
        slot++;
      }
    }
    __syncthreads();
  }
  // where CB i's bytes are: made here (LDS), saved from an earlier transmission, or its decision row
  auto cb_src = [&](uint32_t i) -> const uint8_t * {
    if (c_fz[i] >= 0) return fzb + 768 * c_fz[i];
    return c_init[i] ? t.saved + (size_t)i * 768 : glob_g(dec) + (size_t)c_g[i] * dec_stride;
  };
  // 2. TB bytes, CBs in order (a later CB's bytes win where the regions meet, as the reference's
  //    sequential copies): the (CB, byte) pairs of the TB spread over all threads
  //    Eight CBs at a time: their bytes (at most 768 = 3 x 256 per CB) are all loaded before any
  //    is stored, so the loads are not ordered behind the stores of earlier CBs.
  for (uint32_t i0 = 0; i0 < C; i0 += 8) {
    uint8_t v[8][3];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const uint32_t i = i0 + u;
      if (i >= C) break;
      const uint8_t *src = cb_src(i);
#pragma unroll
      for (int r = 0; r < 3; r++) {
        const uint32_t j = threadIdx.x + r * 256;
        v[u][r] = j < c_nb[i] ? src[j] : 0;
      }
    }
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const uint32_t i = i0 + u;
      if (i >= C) break;
      uint8_t *dst = t.data + c_dst[i];
#pragma unroll
      for (int r = 0; r < 3; r++) {
        const uint32_t j = threadIdx.x + r * 256;
        if (j < c_nb[i]) dst[j] = v[u][r];
      }
      if (i + 1 < C && c_dst[i] + c_nb[i] > c_dst[i + 1]) __syncthreads(); // overlaps keep their order
    }
  }
  __syncthreads();
  const int ok_all = all_ok;
  if (!ok_all) {
    // the direct blocks of this failed TB that were not decoded before: their rows are due
    if (late && threadIdx.x < C && !c_init[threadIdx.x] && dc.rec[c_g[threadIdx.x]].direct)
      late[1 + atomicAdd(late, 1u)] = c_g[threadIdx.x];
    // keep the bytes of the blocks that passed for the retransmission (sch.c:407-416)
    for (uint32_t i = 0; i < C; i++) {
      if (!c_ok[i]) continue;
      const uint8_t *src = t.data + c_dst[i];
      uint8_t *dst = t.saved + (size_t)i * 768;
      for (uint32_t j = threadIdx.x; j < c_rb[i]; j += blockDim.x) dst[j] = src[j];
    }
    if (inline_rows && dc.rec) {
      // the rows themselves (k_derm_late's work): the bytes in fzb are consumed, its LDS stages the LLRs
      __syncthreads();
      for (uint32_t i = 0; i < C; i++)
        if (!c_init[i] && dc.rec[c_g[i]].direct) derm_item(derm_get(dc, c_g[i]), fz_lds);
    }
  }
  // 3. TB CRC24A over tbs bits vs the 24 bits that follow (sch.c:475-491). crc.c:144-155 (MSB
  //    first, zero init) is linear: the checksum is M(x) x^24 mod P, the XOR over any cut of the
  //    message into pieces of each piece's byte-table CRC shifted by x^(8 bytes after it) mod P
  //    (crc_a[n - 24], or x^n itself below 24 bits; a carry-less multiply mod P). The pieces are
  //    32-byte chunks of each code block's bytes, read straight from its decision row (or its
  //    saved bytes) with 16-byte loads, so the CRC does not wait for the TB bytes of step 2.
  uint32_t crc = 0;
  if (ok_all) {
    if (threadIdx.x < 256) { // byte table: T[i] = i x^24 mod P, i.e. i << 16 through 8 shift steps
      uint32_t r = threadIdx.x << 16;
#pragma unroll
      for (int k = 0; k < 8; k++) r = ((r << 1) ^ ((r & 0x800000u) ? 0x864CFBu : 0u)) & 0xFFFFFFu;
      crc_tab[threadIdx.x] = r;
    }
    const uint32_t nbytes = t.tbs / 8;
    if (threadIdx.x == 0) { // chunks per code block: its bytes within [0, nbytes), 32 per chunk
      uint32_t q = 0;
      for (uint32_t i = 0; i < C; i++) {
        c_ck0[i] = q;
        const uint32_t len = c_dst[i] < nbytes ? min(c_rb[i], nbytes - c_dst[i]) : 0u;
        q += (len + 31) / 32;
      }
      c_ck0[C] = q;
    }
    __syncthreads();
    const uint32_t nck = c_ck0[C];
    uint32_t acc = 0;
    for (uint32_t q = threadIdx.x; q < nck; q += blockDim.x) {
      uint32_t i = 0;
      while (c_ck0[i + 1] <= q) i++;
      const uint32_t off = 32 * (q - c_ck0[i]);
      const uint32_t len = min(c_rb[i], nbytes - c_dst[i]), n = min(32u, len - off);
      u4v w0, w1;
      if (c_fz[i] >= 0) {
        const u4v *src = reinterpret_cast<const u4v *>(fzb + 768 * c_fz[i] + off);
        w0 = src[0];
        w1 = src[1];
      } else {
        const uint8_t *src = (c_init[i] ? t.saved + (size_t)i * 768 : glob_g(dec) + (size_t)c_g[i] * dec_stride) + off;
        w0 = *glob(reinterpret_cast<const u4v *>(src));
        w1 = *glob(reinterpret_cast<const u4v *>(src + 16));
      }
      const uint32_t wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
      const uint32_t after = nbytes - (c_dst[i] + off + n); // bytes after the chunk
      const uint32_t shift = after == 0 ? 1u : 8 * after < 24 ? (1u << (8 * after)) : crc_a[8 * after - 24];
      uint32_t r = 0;
#pragma unroll
      for (uint32_t k = 0; k < 32; k++)
        if (k < n) r = ((r << 8) & 0xFFFFFFu) ^ crc_tab[((r >> 16) ^ (wv[k >> 2] >> (8 * (k & 3)))) & 0xFFu];
      if (after) { // r x^(8 after) mod P
        uint64_t m = 0;
        for (int b = 0; b < 24; b++)
          if ((shift >> b) & 1u) m ^= (uint64_t)r << b;
        for (int bit = 46; bit >= 24; bit--)
          if ((m >> bit) & 1u) m ^= (uint64_t)0x1864CFBu << (bit - 24);
        r = (uint32_t)m & 0xFFFFFFu;
      }
      acc ^= r;
    }
    crc = wg_xor(acc, red);
  }
  if (threadIdx.x == 0) {
    *t.noi = noi_sum / C;
    int ret = -1;
    if (ok_all) {
      const uint32_t nbytes = t.tbs / 8;
      const uint32_t tx = ((uint32_t)t.data[nbytes] << 16) | ((uint32_t)t.data[nbytes + 1] << 8) |
                          t.data[nbytes + 2];
      ret = (crc == tx && crc) ? 0 : -1;
    }
    *t.ret = ret;
  }
}

static inline unsigned cdiv(size_t n, unsigned b) { return (unsigned)((n + b - 1) / b); }

// srslte_softbuffer_rx_reset(_tbs) of count consecutive softbuffers: cb_crc cleared, the first ncb
// rows marked fresh (their soft bits count as zero until rewritten)
__global__ __launch_bounds__(256) void k_sb_reset(uint8_t *__restrict__ fresh, uint8_t *__restrict__ cbcrc,
                                                  uint32_t n, uint32_t max_cb, uint32_t ncb) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  cbcrc[i] = 0;
  if (i % max_cb < ncb) fresh[i] = 1;
}

hipError_t launch_sb_reset(uint8_t *fresh, uint8_t *cbcrc, uint32_t count, uint32_t max_cb, uint32_t ncb,
                           hipStream_t st) {
  const size_t n = (size_t)count * max_cb;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_sb_reset, dim3(cdiv(n, 256)), dim3(256), 0, st, fresh, cbcrc, (uint32_t)n, max_cb, ncb);
  return hipGetLastError();
}

// many softbuffers at once: list[2 k] = slot, list[2 k + 1] = rows of it marked fresh (reset_tbs' count)
__global__ __launch_bounds__(256) void k_sb_reset_list(uint8_t *__restrict__ fresh, uint8_t *__restrict__ cbcrc,
                                                       const uint32_t *__restrict__ list, uint32_t n, uint32_t max_cb) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n * max_cb) return;
  const uint32_t k = i / max_cb, c = i - k * max_cb;
  const size_t r = (size_t)list[2 * k] * max_cb + c;
  cbcrc[r] = 0;
  if (c < list[2 * k + 1]) fresh[r] = 1;
}

hipError_t launch_sb_reset_list(uint8_t *fresh, uint8_t *cbcrc, const uint32_t *d_list, uint32_t n, uint32_t max_cb,
                                hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_sb_reset_list, dim3(cdiv((size_t)n * max_cb, 256)), dim3(256), 0, st, fresh, cbcrc, d_list, n,
                     max_cb);
  return hipGetLastError();
}

hipError_t launch_derm(const DermCall &c, int nitems, uint8_t *init_done, hipStream_t st) {
  if (nitems <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_derm, dim3((unsigned)nitems), dim3(256), 0, st, c, nitems, init_done);
  return hipGetLastError();
}

hipError_t launch_derm_late(const DermCall &c, int nitems, const uint32_t *late, hipStream_t st) {
  if (nitems <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_derm_late, dim3((unsigned)std::min(nitems, 512)), dim3(256), 0, st, c, late);
  return hipGetLastError();
}

hipError_t launch_derm_flags(const DermCall &c, int nitems, uint8_t *init_done, uint32_t *late,
                             hipStream_t st) {
  if (nitems <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_derm_flags, dim3(cdiv((size_t)nitems, 256)), dim3(256), 0, st, c, nitems,
                     init_done, late);
  return hipGetLastError();
}

hipError_t launch_load_derm(const TdGroup *dg, int ng, int nblocks, const DermCall &c,
                            const TdArrays &a, uint32_t max_ne, hipStream_t st, int mode,
                            const uint32_t *list, const uint32_t *cnt) {
  if (ng <= 0 || nblocks <= 0) return hipSuccess;
  // LLRs staged per block: the largest E of the call, rounded to 8, at most 8192 (16 KB); blocks
  // with more (or with repetition, E > 3K+12) gather theirs from HBM
  const uint32_t stage = std::min<uint32_t>(8192, (max_ne + 7) / 8 * 8);
  const size_t lds = 4 * (size_t)stage;
  static const bool tile = [] {
    const char *e = getenv("SRSGPU_LDERM");
    return e && e[0] == 't';
  }();
  if (tile && mode == 0) {
    hipLaunchKernelGGL(k_load_derm_tile, dim3((unsigned)nblocks), dim3(LDT_THREADS), lds + 6 * LDT_TILE * 2, st, dg,
                       ng, c, a, stage);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_load_derm, dim3((unsigned)nblocks), dim3(LDR_THREADS), lds, st, dg, ng, c, a, stage, mode,
                     list, cnt, knobs().ldderm_fast ? 1 : 0);
  return hipGetLastError();
}

hipError_t launch_derm_rmw(const DermItem *d_item, uint32_t n, hipStream_t st) {
  const unsigned gx = std::min(cdiv(n, 256), 64u);
  hipLaunchKernelGGL(k_derm_rmw, dim3(gx ? gx : 1), dim3(256), 0, st, d_item);
  return hipGetLastError();
}

hipError_t launch_tb_finish(const TbItem *d_tbs, int ntb, const uint32_t *cbmap, const uint8_t *dec,
                            size_t dec_stride, const uint8_t *cb_ok, const uint8_t *init_done,
                            const uint32_t *noi, const uint32_t *crc_a, hipStream_t st,
                            const DermCall &dc, uint32_t *late, const FzSrc &fz, bool inline_rows) {
  if (ntb <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_tb_finish, dim3((unsigned)ntb), dim3(256), 0, st, d_tbs, ntb, cbmap, dec,
                     dec_stride, cb_ok, init_done, noi, crc_a, dc, late, knobs().tail_prio, fz,
                     inline_rows ? 1 : 0);
  return hipGetLastError();
}

// ------------------------------------------------------------------ UL-SCH ----
// ulsch_deinterleave (sch.c:860-881) without RI bits: ulsch_interleave_gen numbers the entries
// (row j, column i, bit k) row by row, entry (j, i, k) sits at q index (i rows + j) Qm + k, and
// srslte_vec_lut_sis writes g[lut[x]] = q[x]. One thread per g element (coalesced stores, the
// gathered reads are rows x Qm apart).
// With UCI (srsgpu_ulsch_uci_decode_dev, sch.c:860-881 with RI bits): q is still scrambled; the RI
// entries are left out of g (the g index drops by Qm per RI group before the entry in row-major
// order), HARQ-ACK entries read as 0 (sch.c:921-924) and every value is descrambled on the way
// (srslte_scrambling_s_offset, c ? -q : q). The lut's extra writes to g[0] are k_uci_cqi's.
__global__ __launch_bounds__(256) void k_ulsch_deinterleave(const UlItem *__restrict__ items,
                                                            const int16_t *__restrict__ q,
                                                            int16_t *__restrict__ g,
                                                            const uint8_t *__restrict__ c) {
  const UlItem it = items[blockIdx.y];
  const uint32_t n = it.rows * it.cols * it.Qm;
  const uint32_t x = blockIdx.x * 256 + threadIdx.x;
  if (x >= n) return;
  const uint32_t rowlen = it.cols * it.Qm;
  const uint32_t j = x / rowlen, r = x - j * rowlen;
  const uint32_t i = r / it.Qm, k = r - i * it.Qm;
  const size_t src = (size_t)(i * it.rows + j) * it.Qm + k;
  if (!it.uci) {
    g[it.q_offset + x] = q[it.q_offset + src];
    return;
  }
  if (uci_group(j, i, it.rows, true) < it.Q_ri) return; // an RI entry
  int16_t v = uci_group(j, i, it.rows, false) < it.Q_ack ? (int16_t)0 : q[it.q_offset + src];
  if (c[it.c_offset + src]) v = (int16_t)(-(int32_t)v);
  g[it.q_offset + x - (size_t)uci_ri_before(j, i, it.rows, it.Q_ri) * it.Qm] = v;
}

hipError_t launch_ulsch_deinterleave(const UlItem *d_items, int n, uint32_t max_bits, const int16_t *q,
                                     int16_t *g, hipStream_t st, const uint8_t *c) {
  if (n <= 0 || max_bits == 0) return hipSuccess;
  hipLaunchKernelGGL(k_ulsch_deinterleave, dim3((max_bits + 255) / 256, (unsigned)n), dim3(256), 0, st,
                     d_items, q, g, c);
  return hipGetLastError();
}

// ------------------------------------------------------------------ transmit ----
// encode_tb_off (sch.c:187-296) for one code block per workgroup: the code block's bits are
// assembled in LDS (TB bits, the TB CRC24A on the last block, the CB CRC24B when C > 1; both
// CRCs as XOR folds of x^(d+24) mod P over the set bits, crc.c:144-155 being linear), the two
// RSC encoders of srslte_tcod_encode (turbocoder.c:82-193) run in one lane each over LDS, and
// rate matching reads the circular buffer through the receive table: e[m] = coded[table[m mod N]]
// (rm_turbo.c:332-376 is the inverse of the receive mapping).
__global__ __launch_bounds__(256) void k_dlsch_encode(const EncItem *__restrict__ items, int nitems,
                                                      const uint32_t *__restrict__ crc_a,
                                                      const uint32_t *__restrict__ crc_b) {
  __shared__ uint8_t bits[6144];
  __shared__ uint8_t coded[3 * 6144 + 12];
  __shared__ uint32_t red[4];
  const int it = blockIdx.x;
  if (it >= nitems) return;
  const EncItem t = items[it];
  auto data_bit = [&](uint32_t p) -> uint32_t { return (t.data[p >> 3] >> (7 - (p & 7))) & 1u; };
  uint32_t tcrc = 0;
  if (t.last) { // TB CRC24A over tbs bits
    uint32_t acc = 0;
    for (uint32_t p = threadIdx.x; p < t.tbs; p += blockDim.x)
      if (data_bit(p)) acc ^= crc_a[t.tbs - 1 - p];
    tcrc = wg_xor(acc, red);
  }
  for (uint32_t j = threadIdx.x; j < t.rlen; j += blockDim.x) {
    const uint32_t p = t.rp + j;
    bits[j] = (uint8_t)(p < t.tbs ? data_bit(p) : (tcrc >> (23 - (p - t.tbs))) & 1u);
  }
  __syncthreads();
  if (t.crc_cb) { // CB CRC24B over the rlen bits
    uint32_t acc = 0;
    for (uint32_t j = threadIdx.x; j < t.rlen; j += blockDim.x)
      if (bits[j]) acc ^= crc_b[t.rlen - 1 - j];
    const uint32_t c = wg_xor(acc, red);
    if (threadIdx.x < 24) bits[t.rlen + threadIdx.x] = (uint8_t)((c >> (23 - threadIdx.x)) & 1u);
    __syncthreads();
  }
  // turbocoder.c:123-131: fb = u ^ s2 ^ s1, parity = s2 ^ s0 ^ fb; tails :160-177
  if (threadIdx.x == 0 || threadIdx.x == 64) {
    const bool second = threadIdx.x == 64;
    uint32_t s0 = 0, s1 = 0, s2 = 0;
    for (uint32_t i = 0; i < t.K; i++) {
      const uint32_t u = second ? bits[t.pi[i]] : bits[i];
      const uint32_t fb = u ^ s2 ^ s1;
      const uint32_t par = s2 ^ s0 ^ fb;
      s2 = s1;
      s1 = s0;
      s0 = fb;
      if (second) {
        coded[3 * i + 2] = (uint8_t)par;
      } else {
        coded[3 * i] = (uint8_t)u;
        coded[3 * i + 1] = (uint8_t)par;
      }
    }
    const uint32_t o = 3 * t.K + (second ? 6 : 0);
    for (int j = 0; j < 3; j++) {
      const uint32_t u = s2 ^ s1; // drives the register to zero
      const uint32_t fb = u ^ s2 ^ s1;
      const uint32_t par = s2 ^ s0 ^ fb;
      s2 = s1;
      s1 = s0;
      s0 = fb;
      coded[o + 2 * j] = (uint8_t)u;
      coded[o + 2 * j + 1] = (uint8_t)par;
    }
  }
  __syncthreads();
  for (uint32_t m = threadIdx.x; m < t.ne; m += blockDim.x) t.e[m] = coded[t.table[m % t.N]];
}

hipError_t launch_dlsch_encode(const EncItem *d_items, int n, const uint32_t *crc_a,
                               const uint32_t *crc_b, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_dlsch_encode, dim3((unsigned)n), dim3(256), 0, st, d_items, n, crc_a, crc_b);
  return hipGetLastError();
}

} // namespace srsgpu
