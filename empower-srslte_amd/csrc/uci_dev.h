// Positions of the UCI bits in the PUSCH channel-interleaver matrix (rows = H' / N_symb, columns =
// N_symb, Qm bits per entry; q index of entry (row j, column i, bit k) = (i rows + j) Qm + k):
// bit group g of HARQ-ACK / RI sits in row rows - 1 - g / 4 and column {2, 9, 8, 3} / {1, 10, 7, 4}
// [g mod 4] (uci.c:499-546: column set[(3 g) mod 4] of {2, 3, 8, 9} / {1, 4, 7, 10}).
#ifndef SRSGPU_UCI_DEV_H
#define SRSGPU_UCI_DEV_H
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace srsgpu {

__device__ __forceinline__ uint32_t uci_col(uint32_t u, bool ri) {
  return ri ? (u == 0 ? 1u : u == 1 ? 10u : u == 2 ? 7u : 4u) : (u == 0 ? 2u : u == 1 ? 9u : u == 2 ? 8u : 3u);
}
// q index of bit k of group g
__device__ __forceinline__ uint32_t uci_pos(uint32_t g, uint32_t k, uint32_t Qm, uint32_t rows, bool ri) {
  return (uci_col(g % 4, ri) * rows + rows - 1 - g / 4) * Qm + k;
}
// the group index at (row j, column i), or 0xFFFFFFFF when the column holds none of this kind
__device__ __forceinline__ uint32_t uci_group(uint32_t j, uint32_t i, uint32_t rows, bool ri) {
  int u = -1;
  for (uint32_t v = 0; v < 4; v++)
    if (uci_col(v, ri) == i) u = (int)v;
  return u < 0 ? 0xFFFFFFFFu : 4 * (rows - 1 - j) + (uint32_t)u;
}
// RI groups (Q_ri of them) in row-major order before entry (row j, column i): the full rows below
// row j's position fill from the bottom, rows - 1 - g / 4
__device__ __forceinline__ uint32_t uci_ri_before(uint32_t j, uint32_t i, uint32_t rows, uint32_t Q_ri) {
  const int64_t above = (int64_t)Q_ri - 4 * (int64_t)(rows - j);
  uint32_t n = above > 0 ? (uint32_t)above : 0u;
  const int64_t c = (int64_t)Q_ri - 4 * (int64_t)(rows - 1 - j);
  const uint32_t cnt = c <= 0 ? 0u : c >= 4 ? 4u : (uint32_t)c;
  for (uint32_t u = 0; u < cnt; u++) n += uci_col(u, true) < i;
  return n;
}

} // namespace srsgpu
#endif
