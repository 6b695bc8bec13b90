// Internal launch interface of the PDSCH receive kernels (pdsch_kernels.hip).
#ifndef SRSGPU_PDSCH_KERNELS_H
#define SRSGPU_PDSCH_KERNELS_H
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <algorithm>

namespace srsgpu {

// one codeword's scrambling sequence: len bits of c(n) for c_init = seed, packed LSB first
struct GoldItem {
  uint32_t seed, len;
  uint32_t *c;
};

// one transport block: gather + equalise + demap + descramble (+ CSI)
struct LlrItem {
  const float2 *y[2];      // received grid of each rx antenna
  const float2 *h[4][2];   // channel estimate [port][rx antenna], same layout
  const uint32_t *map;     // RE j -> grid position
  const uint32_t *c;       // packed scrambling bits
  int16_t *e;              // LLRs out (nof_re * qm)
  float *csi;              // per-RE CSI (csi_mode)
  uint32_t *csi_max;       // max CSI as float bits (csi_mode; zeroed before the launch)
  uint32_t nof_re;
  int qm, mod, nrx, csi_mode;
  int cdd, layer;          // TM3 CDD 2x2 MMSE: this TB's codeword / layer (0 or 1)
  int mux;                 // TM4 spatial multiplexing: 1 + codebook_idx (2 layers: 2x2 MMSE) or
                           // -(1 + codebook_idx) (1 layer: 2x1 MRC); 0 otherwise
  int txdiv;               // TM2 transmit diversity: 2 (SFBC over RE pairs) or 4 ports (RE
                           // quadruplets, port pairs 0/2 and 1/3); 0 otherwise; 1-2 rx
  int aligned;             // e is 4-byte aligned: LLR pairs stored as 32-bit words
  float noise, inv_scaling, scaling;
  const float *noise_dev;  // if set: chest noise [rx][port] averaged as chest_dl.c:741-750 does
  int nports;              // ports in noise_dev
  int llr8;                // llr_is_8bit: int8 demapping / scrambling / CSI, values sign-extended in e
  int ce_rows;             // h planes hold the chest's compact rows (srsgpu_pdsch_set_ce_rows): 0 = full
                           // 14-symbol planes, 4 = the CRS symbols' rows (time interpolation here),
                           // 1 = one averaged row
  uint32_t nsc;            // subcarriers per symbol (12 nof_prb)
  float inv_nsc;           // 1 / nsc (RE position -> symbol)
  int dual;                // 2-layer MMSE (TM3 / TM4) with both TBs of one modulation: 1 = this item
                           // also computes the next item's layer from the same 2x2 solve, 2 = done
                           // by the previous item (its workgroups return at once)
};

// one codeword to transmit: scramble + modulate + map
struct TxItem {
  const uint8_t *e[2];     // per codeword: nof_re * qm coded bits, one per byte
  const uint32_t *c[2];    // per codeword: packed scrambling bits
  const uint32_t *map;     // RE j -> grid position
  float2 *grid;            // port-0 grid of the subframe
  uint64_t port_stride;    // complex elements between the ports' grids
  uint32_t nof_re;
  int qm[2];
  int mimo;                // SRSGPU_MIMO_*
  int nlayers, codebook;   // spatial multiplexing
  float scaling;           // rho_a
};

hipError_t launch_gold(const GoldItem *d_items, int n, uint32_t max_len, const uint32_t *x1,
                       const uint32_t *x2b, uint32_t words, hipStream_t st);
// n_dual: pairs of items with dual = 1 / 2 (both layers of a 2-layer MMSE subframe from one solve);
// p0 = nof_rx_ant (1 / 2) when every item equalises CRS port 0 alone (no transmit diversity, CDD or
// spatial multiplexing), else 0: the kernel specialised for it, with the multi-port paths compiled
// out and the antenna count fixed (fewer registers)
hipError_t launch_pdsch_llr(const LlrItem *d_items, int n, uint32_t max_re, bool csi, hipStream_t st,
                            int n_dual = 0, int p0 = 0);
// tables: 2 BPSK + 4 QPSK + 16 16QAM + 64 64QAM constellation points (lte_tables.c order)
hipError_t launch_pdsch_tx(const TxItem *d_items, int n, uint32_t max_re, const float2 *tables,
                           hipStream_t st);
// PCFICH of one subframe (srslte_pcfich_decode_multi)
struct PcfichItem {
  uint64_t grid_off, ce_off; // this subframe's [rx] grid planes / [rx][port] estimate planes
  uint32_t sf_idx;
  float noise;
  const float *dnoise; // non-null: the noise estimate in device memory (overrides noise)
};
// idx: the 16 RE indices of symbol 0; seq[sf]: the 32 scrambling bits of subframe sf
hipError_t launch_pcfich(const PcfichItem *d_items, int n, const float2 *grid, const float2 *ce,
                         size_t ant_stride, int nof_prb, int nports, int nrx, const uint32_t *idx,
                         const uint32_t *seq, uint32_t *cfi, float *corr, hipStream_t st);
// PDCCH of one subframe (srslte_pdcch_extract_llr_multi)
struct PdcchItem {
  uint64_t grid_off, ce_off, llr_off; // [rx] grid planes / [rx][port] estimate planes / LLR out
  const uint32_t *map;                // the CFI's REG symbols (srslte_regs_pdcch_get order)
  const uint32_t *c;                  // the subframe's scrambling bits, packed LSB first
  uint32_t nof_symbols;               // 36 NOF_CCE(cfi)
  float noise;                        // the noise_estimate argument
  const float *dnoise;                // non-null: the noise estimate in device memory (overrides noise)
};
hipError_t launch_pdcch_llr(const PdcchItem *d_items, int n, uint32_t max_symbols, const float2 *grid,
                            const float2 *ce, size_t ant_stride, int nports, int nrx, float *llr,
                            hipStream_t st);
} // namespace srsgpu
#endif
