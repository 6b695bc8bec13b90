// Internal launch interface of the turbo-decoder kernels (tdec_kernels.hip).
#ifndef SRSGPU_TDEC_KERNELS_H
#define SRSGPU_TDEC_KERNELS_H
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace srsgpu {
// user input -> SP0 (short4), P1 plane of XP1 (short2), T (short2 x 12) per pair. XP1 holds
// two [npairs][K] short2 planes: X2 (app2) then P1 (par1).
// rows != NULL: code block c's input starts at rows[c] (device array; rows_aligned: every row
// is 4-byte aligned), else at in + c * in_stride.
hipError_t launch_load(const int16_t *in, size_t in_stride, const int16_t *const *rows,
                       int rows_aligned, int sb_input, int K, int NB, int ncb, void *SP0, void *XP1,
                       void *T, hipStream_t st);
size_t win_ck_bytes(int K, int NB, int npairs);
size_t seq_scratch_bytes(int K, int npairs);
// one half-iteration n (DEC1 for even n, DEC2 for odd n). NB > 1: windowed decoder;
// NB == 1: impl_seq 0 = SSE non-window, 1 = generic.
hipError_t launch_halfit(int n, int NB, int impl_seq, void *SP0, void *XP1, void *A, void *D,
                         const void *T,
                         const uint16_t *fwd, const uint16_t *rev, void *scratch,
                         const uint8_t *pair_done, int K, int npairs, hipStream_t st);
// hard decision after half-iteration n; with crc_bytes > 0 also CRC + early-stop bookkeeping
// dmap: natural position -> chain-major decision index after DEC2 (see tdec_engine.h)
hipError_t launch_decide(int n, int K, int NB, int ncb, const uint16_t *dmap, const void *D,
                         uint8_t *outb, size_t out_stride, uint8_t *cb_done,
                         uint8_t *cb_ok, uint32_t *noi, int crc_bytes, const uint32_t *crc_pw,
                         int max_halfits, uint8_t *pair_done, hipStream_t st);
// crc_pw[d] = x^(d + 24) mod poly (24-bit CRC), d < 6144: the checksum of a crc_bits-bit message is
// the XOR of crc_pw[crc_bits - 1 - p] over its set bits p
// pair_done[p] = both CBs of pair p done
hipError_t launch_pair_done(int ncb, const uint8_t *cb_done, uint8_t *pair_done, hipStream_t st);
} // namespace srsgpu
#endif
