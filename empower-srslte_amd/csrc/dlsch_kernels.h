// Internal launch interface of the DL-SCH kernels (dlsch_kernels.hip).
#ifndef SRSGPU_DLSCH_KERNELS_H
#define SRSGPU_DLSCH_KERNELS_H
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "tdec_kernels.h"

namespace srsgpu {

// one code block to de-rate-match into its softbuffer row
struct DermItem {
  const int16_t *e;       // its E received LLRs (sch.c:330-341 rp / n_e2)
  uint32_t ne;            // E
  uint32_t N;             // 3K + 12 (table length)
  const uint16_t *table;  // receive table for (K, rv), decoder layout
  const uint16_t *inv;    // its inverse: row position -> table entry m, 0xFFFF if none (rowlen,
                          // padded with 0xFFFF to a multiple of 8)
  int16_t *row;           // softbuffer row (SOFTBUFFER_SIZE int16)
  const uint8_t *cb_crc;  // softbuffer cb_crc[i]: already decoded -> skipped
  uint32_t pos;           // position in the decoder's (K-grouped) CB order
  uint32_t rowlen;        // decoder-input length of the row: 3(K+32)+12 (SB) or 3K+12
  uint8_t *fresh;         // row reset since its last use: content counts as zero (cleared here)
  uint32_t w8;            // 8-bit LLR chain (llr_is_8bit, rm_turbo.c:432-469): int8 values held
                          // sign-extended in the int16 row, sums wrapping at 8 bits
  uint32_t direct;        // de-rate-matched straight into the decoder inputs (k_load_derm); the
                          // row itself is written after the decode, only if the TB failed
  const int32_t *tb_ret;  // its TB's return code (k_tb_finish), read by the deferred row pass
  const uint16_t *inv_t4; // direct: the inverse table in the decoder's T4 order, [3][ne] + 12 tails
};

// The per-call form of the DermItems of a decode: 32 bytes per code block uploaded per call (the
// full DermItem, 104 bytes of pointers and sizes, made the descriptor upload the largest copy of a
// 512-subframe batch); the pointers come from the call (DermCall) and a table set per (K, rv,
// layout) that stays on the device (DermTabs). derm_get() expands a record.
struct DermRec {
  uint32_t e_off;  // its LLRs: DermCall::e + e_off
  uint32_t ne;     // E
  uint32_t row;    // softbuffer row index (slot * max_cb + cb): the row, its cb_crc and fresh flags
  uint32_t pos;    // position in the decoder's order
  uint32_t tb;     // its TB in the call: DermCall::ret + tb
  uint16_t N, rowlen;
  uint16_t tab;    // its table set in DermCall::tabs
  uint8_t w8, direct;
};
struct DermTabs {
  const uint16_t *table, *inv, *inv_t4;
};
struct DermCall {
  const DermRec *rec;     // by decoder position
  const DermTabs *tabs;
  const int16_t *e;       // LLR base of the call
  int16_t *soft;          // softbuffer rows (SRSGPU_SOFTBUFFER_SIZE int16 each)
  uint8_t *cbcrc, *fresh; // per row
  const int32_t *ret;     // per TB
};

// one transport block's epilogue
struct TbItem {
  uint8_t *data;      // output bytes
  uint8_t *cb_crc;    // softbuffer cb_crc[0..C)
  uint8_t *saved;     // softbuffer saved bytes [C][768]
  int32_t *ret;       // SRSLTE_SUCCESS / SRSLTE_ERROR
  uint32_t *noi;      // nof_iterations (sum over decoded CBs / C)
  uint32_t tbs, C, C1, K1, K2;
  uint32_t first;     // index of CB 0 in the call's CB list
  int32_t preset_ret; // result when C == 0 (tbs == 0 or invalid inputs)
};

// one code block to encode and rate-match (transmit side)
struct EncItem {
  const uint8_t *data;     // TB bytes (MSB first)
  uint8_t *e;              // ne output bits, one per byte
  const uint16_t *table;   // receive table (K, rv), natural layout, N entries
  const uint16_t *pi;      // QPP interleaver pi(i)
  uint32_t tbs, K, rlen, rp, ne, N;
  uint32_t last;           // carries the TB CRC
  uint32_t crc_cb;         // C > 1: CB CRC24B
};

// rows of the items that are not `direct` (before the decode), init_done of every item
hipError_t launch_derm(const DermCall &c, int nitems, uint8_t *init_done, hipStream_t st);
// after k_tb_finish: rows of the direct items it listed in late (late[0] of them at late[1..]:
// blocks of failed TBs not decoded before this call)
hipError_t launch_derm_late(const DermCall &c, int nitems, const uint32_t *late, hipStream_t st);
// init_done[pos] = cb_crc before this call, for every item; late[0] = 0 (late may be null)
hipError_t launch_derm_flags(const DermCall &c, int nitems, uint8_t *init_done, uint32_t *late,
                             hipStream_t st);
hipError_t launch_derm_rmw(const DermItem *d_item, uint32_t n, hipStream_t st);
// softbuffer reset of count slots of max_cb rows from fresh / cbcrc: cb_crc = 0, the first ncb
// rows of each slot fresh
hipError_t launch_sb_reset_list(uint8_t *fresh, uint8_t *cbcrc, const uint32_t *d_list, uint32_t n, uint32_t max_cb,
                                hipStream_t st);
hipError_t launch_sb_reset(uint8_t *fresh, uint8_t *cbcrc, uint32_t count, uint32_t max_cb, uint32_t ncb,
                           hipStream_t st);
// dec / cb_ok / init_done / noi are in decoder order; cbmap[first + i] is CB i's position there
// crc_a[d] = x^(d+24) mod P_24A for d < the largest TBS + 24
// dc.rec / late (both or neither): a failed TB appends its direct blocks not decoded before the
// call to late (launch_derm_late)
// The decision words of the blocks a fused early-stop launch ended (the decoder job's Dfz / cb_end and
// its group table, tdec_kernels.h TdEs): with groups set, k_tb_finish turns those blocks' words into
// their natural-order bytes itself (k_es_bytes' work, no launch of its own) and clears cb_end.
struct FzSrc {
  const TdGroup *groups = nullptr;
  int ngroups = 0;
  const uint32_t *dfz = nullptr;
  uint8_t *cb_end = nullptr;
};
// inline_rows (with dc.rec, late null): a failed TB's workgroup writes the rows of its direct blocks
// not decoded before the call itself (k_derm_late's work, no launch of its own)
hipError_t launch_tb_finish(const TbItem *d_tbs, int ntb, const uint32_t *cbmap, const uint8_t *dec,
                            size_t dec_stride, const uint8_t *cb_ok, const uint8_t *init_done,
                            const uint32_t *noi, const uint32_t *crc_a, hipStream_t st,
                            const DermCall &dc = DermCall{}, uint32_t *late = nullptr,
                            const FzSrc &fz = FzSrc{}, bool inline_rows = false);
// crc_a: x^(d+24) mod CRC24A for d < tbs; crc_b: the same for CRC24B, d < 6144
hipError_t launch_dlsch_encode(const EncItem *d_items, int n, const uint32_t *crc_a,
                               const uint32_t *crc_b, hipStream_t st);
// UL-SCH channel deinterleaver (sch.c:550-568,860-881) of one TB per blockIdx.y: g[(j cols + i) Qm
// + k] = q[(i rows + j) Qm + k] for row j < rows, column i < cols, bit k < Qm
struct UlItem {
  uint64_t q_offset;
  uint32_t rows, cols, Qm;
  // UCI on the PUSCH (srsgpu_ulsch_uci_decode_dev; uci = 0: the plain UL-SCH, q already descrambled)
  uint32_t uci;
  uint32_t O_ack, O_ri, O_cqi;
  uint32_t Q_ack, Q_ri, Q_cqi;
  uint32_t tbs;      // 0: no data (the UCI kernel writes ret / noi)
  uint64_t c_offset; // scrambling bytes of the TB (q still scrambled)
};
hipError_t launch_ulsch_deinterleave(const UlItem *d_items, int n, uint32_t max_bits, const int16_t *q,
                                     int16_t *g, hipStream_t st, const uint8_t *c = nullptr);
// UCI steps (uci_kernels.hip): HARQ-ACK / RI before the deinterleaver, g[0] and CQI after it
hipError_t launch_uci_ack_ri(const UlItem *d_items, int n, const int16_t *q, const uint8_t *c, void *res,
                             hipStream_t st);
hipError_t launch_uci_cqi(const UlItem *d_items, int n, const int16_t *q, const uint8_t *c, int16_t *g, void *res,
                          int32_t *ret, uint32_t *noi, hipStream_t st);
} // namespace srsgpu

namespace srsgpu {
// Direct de-rate-matching for the window decoders: the decoder inputs SP0 / P1 / T of groups
// [0, ng) of dg (sub-block rows, nb a multiple of 8) computed from each code block's LLRs and its
// softbuffer row (skipped when fresh) as k_derm + k_load_sbt would, without writing the row.
// c.rec is indexed by decoder position (TdGroup::cb0 numbering); one workgroup per pair.
// max_ne: the largest E among the items (sizes the LDS staging of the LLRs)
// mode 0: SP0 / P1 / T; 1: SP0 / T (P1 deferred); 2: P1 of the listed pairs only (list / cnt as
// TdEs::run_list / run_cnt; nblocks as for mode 0)
hipError_t launch_load_derm(const TdGroup *dg, int ng, int nblocks, const DermCall &c,
                            const TdArrays &a, uint32_t max_ne, hipStream_t st, int mode = 0,
                            const uint32_t *list = nullptr, const uint32_t *cnt = nullptr);
} // namespace srsgpu
#endif
