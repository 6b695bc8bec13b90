// Internal launch interface of the turbo-decoder kernels (tdec_kernels.hip).
#ifndef SRSGPU_TDEC_KERNELS_H
#define SRSGPU_TDEC_KERNELS_H
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#define TD_CK_W 8 // beta checkpoint period (steps) of the windowed decoder

namespace srsgpu {
hipError_t launch_load(const int16_t *in, size_t in_stride, int sb_input, int K, int NB, int ncb,
                       void *S, void *P0, void *P1, void *T, hipStream_t st);
hipError_t launch_prep_even(int n, int K, int npairs, const uint16_t *rev, const void *S,
                            const void *P0, const void *X2, const void *E, void *A, void *XY,
                            int wrap_mode, const uint8_t *pair_done, hipStream_t st);
hipError_t launch_prep_odd(int n, int K, int npairs, const uint16_t *fwd, const void *P1,
                           const void *Ein, const void *A, void *Eout, void *XY,
                           const uint8_t *pair_done, hipStream_t st);
size_t win_ck_bytes(int K, int NB, int npairs);
size_t seq_scratch_bytes(int K, int npairs);
hipError_t launch_win_dec(int NB, const void *XY, const void *T, int tail_xoff, void *out,
                          void *ck, const uint8_t *pair_done, int K, int npairs, hipStream_t st);
hipError_t launch_sse_dec(const void *XY, const void *T, int tail_xoff, void *out, void *scratch,
                          const uint8_t *pair_done, int K, int npairs, hipStream_t st);
hipError_t launch_gen_dec(const void *XY, const void *T, int tail_xoff, void *out, void *scratch,
                          const uint8_t *pair_done, int K, int npairs, hipStream_t st);
hipError_t launch_decide(int n, int K, int NB, int ncb, const uint16_t *rev, const void *E,
                         const void *X2, uint8_t *outb, size_t out_stride, const uint8_t *cb_done,
                         hipStream_t st);
hipError_t launch_crc_check(int n, int ncb, int nbytes, uint32_t poly, const uint8_t *outb,
                            size_t out_stride, uint8_t *cb_done, uint8_t *cb_ok, uint32_t *noi,
                            int max_halfits, uint8_t *pair_done, hipStream_t st);
} // namespace srsgpu
#endif
