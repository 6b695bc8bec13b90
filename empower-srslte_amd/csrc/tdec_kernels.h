// Internal launch interface of the turbo-decoder kernels (tdec_kernels.hip).
//
// A decoder job is a list of GROUPS: code blocks of one size K and one decoder variant (AUTO
// picks the variant from K, turbodecoder.c:364-422), plus the CRC the early stop checks. Mixed
// sizes (many cells, many TBs) decode together: one launch per variant and half-iteration covers
// every group of that variant; a workgroup finds its group by binary search over the groups'
// first-workgroup numbers (wave-uniform scalar loads), so launch count does not grow with the
// number of distinct K.
#ifndef SRSGPU_TDEC_KERNELS_H
#define SRSGPU_TDEC_KERNELS_H
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace srsgpu {

// decoder variants, in the order groups are laid out in a job (B16 / B32: the int8 window
// decoders of srslte_tdec_iteration_8bit, 16 / 32 sub-blocks)
enum {
  TD_KIND_W16 = 0,
  TD_KIND_W8 = 1,
  TD_KIND_SSE = 2,
  TD_KIND_GEN = 3,
  TD_KIND_B16 = 4,
  TD_KIND_B32 = 5,
  TD_NKIND = 6
};

struct TdGroup {
  int32_t K, nb, ncb, npairs; // nb: 16 / 8 windowed sub-blocks, 1 sequential
  int32_t cb0;                // first code block of the group in the caller's numbering (rows,
                              // outputs, cb_done / cb_ok / noi)
  int32_t pair0;              // first pair (T, pair_done; monotonic over the group list)
  int32_t blk_load, blk_half; // first workgroup of the group in its load / half-iteration launch
  int64_t elem0;              // first element of the group's per-pair T4 regions (SP0, X2, P1, A)
  int64_t dw0;                // first packed decision word (D)
  int64_t sc0;                // first short2 of the sequential decoders' scratch
  const uint16_t *fwd, *rev, *dmap;
  const uint32_t *crc_pw;     // x^(d+24) mod P of the group's CRC (early stop)
  const uint32_t *wc[2];      // CRC weight of each decision bit in the decoder's chain-major order
                              // after DEC1 / DEC2: crc_pw[crc_bits - 1 - p] for the natural
                              // position p the bit carries, 0 for padding and p >= crc_bits
  int32_t crc_bytes;          // CRC-checked prefix in bytes (0: no CRC)
  int32_t sb_input;           // input rows in rm_turbo's sub-block layout
};

// Decoder inputs SP0 and P1 (written by the loaders, read by every half-iteration) use the T4
// layout: within a pair's region, step k of sub-block chain d sits at
// ((k >> 2) * nb + d) * 4 + (k & 3). A chain's steps come in runs of 4 (16 bytes of short2, 32 of
// short4), so one 16-byte load per lane covers 4 trellis steps. X2 and A, the targets of the
// interleaver scatter, stay in sub-block order k * nb + d: one step's scatter from the nb chains
// of a pair then lands on nb consecutive elements (QPP interleavers are contention-free), a
// 64-byte store. For nb = 1 (sequential decoders) both are the natural index. Region size of a
// pair (every array):
__host__ __device__ inline int t4_pair_elems(int K, int nb) { return nb * 4 * ((K / nb + 3) / 4); }
__host__ __device__ inline int t4_pos(int k, int d, int nb) { return ((k >> 2) * nb + d) * 4 + (k & 3); }
// Interleaver tables (TdGroup::fwd / rev) are in T16 layout: entry (q * nb + d) * 16 + j holds,
// for step k = 16 q + j of chain d (k < K / nb; padding 0), the sub-block index of its scatter
// target; nb * 16 * ceil(K / nb / 16) entries.
__host__ __device__ inline int t16_table_elems(int K, int nb) { return nb * 16 * ((K / nb + 15) / 16); }

struct TdArrays {
  void *SP0, *XP1, *A, *D, *T, *scratch;
  size_t plane; // elements of the X2 plane: P1 starts at XP1 + plane
};

// user input -> SP0 / P1 / T for groups [0, ng) of dg (all with the same nb and sb_input).
// rows != NULL: code block c's input starts at rows[c], else at in + c * in_stride.
// vec: natural rows may be read as 8-byte words; sub-block rows as 16-byte vectors.
hipError_t launch_load(const TdGroup *dg, int ng, int nblocks, int nb, int sb_input, bool vec,
                       const int16_t *in, size_t in_stride, const int16_t *const *rows,
                       const TdArrays &a, hipStream_t st);
// workgroups a group needs in the load / half-iteration launch of its kind
// vec16: sub-block rows that are 16-byte aligned (8 elements per thread)
int load_blocks(int K, int nb, int npairs, int sb_input, bool vec16);
int halfit_blocks(int nb, int npairs);
size_t seq_scratch_elems(int K, int npairs); // short2 elements
size_t bidir_lds_bytes(int K, int nb);
int dec_words_host(int K, int nb);
// one half-iteration n (DEC1 for even n, DEC2 for odd n) of every group of one kind
hipError_t launch_halfit(int n, int kind, const TdGroup *dg, int ng, int nblocks, size_t lds,
                         bool dec, const TdArrays &a, const uint8_t *pair_done, hipStream_t st);
// the same for ONE group of at most spread_max_pairs() pairs as k_win_spread (latency form), when
// spread_ok(kind, K, nb): a windowed kind with K / nb a multiple of 16 and at least 48
int spread_max_pairs();
bool spread_ok(int kind, int K, int nb);
// outb (dec only): the decision bytes of every block of the group also written by the same launch,
// row cb0 + c at outb + (cb0 + c) * out_stride (k_decide's fixed-iteration output)
// cnt: per-pair arrival counters of the pair's workgroups (zeroed, left zeroed; needed with outb);
// flag (optional, host-mapped): seq is stored there once the bytes are written
struct SpreadOut {
  uint32_t *cnt = nullptr, *flag = nullptr;
  uint32_t seq = 0;
};
hipError_t launch_halfit_spread(int n, int kind, const TdGroup *dg, int npairs, int K, int nb, bool dec,
                                const TdArrays &a, const uint8_t *pair_done, hipStream_t st,
                                uint8_t *outb = nullptr, size_t out_stride = 0, const SpreadOut &so = SpreadOut{});
// half-iterations n0 .. n0+nh-1 of every group of one windowed kind in one launch (fixed-iteration
// jobs: no early stop in between); dec: decisions after the last one
bool halfits_fusable(int kind);
// the process-wide launch schedule (srsgpu_tdec_set_schedule)
struct TdSched {
  int fused, es_fused, es_chunk, sse_bidir;
};
TdSched &td_sched();
bool halfits_es_fusable(int kind);
hipError_t launch_halfits(int n0, int nh, int kind, const TdGroup *dg, int ng, int nblocks,
                          size_t lds, bool dec, const TdArrays &a, hipStream_t st);
// Early-stop state of k_win_bidir_es (sch.c:361-391 per code block): natural-order decision
// bytes, done / ok flags and the half-iteration count of every CB in the caller's numbering.
struct TdEs {
  uint8_t *outb;
  size_t out_stride;
  uint8_t *cb_done, *cb_ok;
  uint32_t *noi;
  int max_halfits;
  int n0, n1; // this launch runs half-iterations n0 .. n1-1 (0 <= n0 < n1 <= max_halfits)
  uint32_t *dfz;  // decision words of the blocks that ended (layout of D), for k_es_bytes
  uint8_t *cb_end; // per CB: 0, or 1 + parity of the half-iteration that ended it (kept zero between jobs)
  int prio;        // 0..3: the early-stop waves' issue priority on their SIMD (s_setprio; 0 = default)
  // windowed kinds after a k_decide that listed the pairs still running (hybrid schedule): per group,
  // run_cnt[pair0] of them at run_list[pair0 ..] (group-local pair numbers, any order); null: every pair
  const uint32_t *run_list = nullptr, *run_cnt = nullptr;
  // bytes_direct with n0 = 0, n1 = 1: the hybrid schedule's first half-iteration with the decide of its
  // own blocks fused in (k_win_bidir_h0c): the blocks that pass get their natural-order bytes written at
  // once, and with list_out / cnt_out the pairs still running are appended to their group's list there
  // (the run_list / run_cnt of the early-stop launch that follows; cnt_out zeroed by launch_pair_done)
  int bytes_direct = 0;
  uint32_t *list_out = nullptr, *cnt_out = nullptr;
};
// the natural-order bytes of the blocks the fused launches ended (after the last of them)
hipError_t launch_es_bytes(const TdGroup *dg, int ng, int npairs, const TdEs &es, hipStream_t st);
// half-iterations es.n0 .. es.n1-1 of an early-stop job for the groups of one kind in one launch:
// the CRC after each half-iteration, done / ok / noi and the decision bytes of finished blocks
// as launch_decide with early = true does, workgroups leave when all their blocks are done
hipError_t launch_halfits_es(int kind, const TdGroup *dg, int ng, int nblocks, size_t lds,
                             const TdArrays &a, const TdEs &es, hipStream_t st);
// hard decision after half-iteration n for every pair of the job (npairs in total); early: also
// the CRC, cb_done / cb_ok / noi and pair_done (turbodecoder.c:353-360, sch.c:361-391)
// run_list / run_cnt (early, optional): every pair not done after half-iteration n is appended to its
// group's list (TdEs::run_list; run_cnt zeroed by launch_pair_done)
hipError_t launch_decide(int n, const TdGroup *dg, int ng, int npairs, const TdArrays &a,
                         uint8_t *outb, size_t out_stride, bool early, uint8_t *cb_done,
                         uint8_t *cb_ok, uint32_t *noi, int max_halfits, uint8_t *pair_done,
                         hipStream_t st, uint32_t *run_list = nullptr, uint32_t *run_cnt = nullptr);
// the early-stop flags of the job's code blocks: cb_done = init_done (0 without), cb_ok = noi = 0,
// pair_done[p] = both code blocks of pair p done
hipError_t launch_pair_done(const TdGroup *dg, int ng, int npairs, const uint8_t *init_done, uint8_t *cb_done,
                            uint8_t *cb_ok, uint32_t *noi, uint8_t *pair_done, hipStream_t st,
                            uint32_t *run_cnt = nullptr);
} // namespace srsgpu
#endif
