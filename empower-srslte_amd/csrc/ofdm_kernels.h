// Internal launch interface of the OFDM receive FFT (ofdm_kernels.hip).
#ifndef SRSGPU_OFDM_KERNELS_H
#define SRSGPU_OFDM_KERNELS_H
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace srsgpu {
// nsf subframes: in + i*in_stride (15 N samples), out + i*out_stride (14 x nre; 12 x nre with
// ext_cp); tw: N twiddles
// e^{-2 pi i k / N}; radices: 4-bit radix per stage (first stage in the low nibble)
hipError_t launch_ofdm_rx(const float2 *in, size_t in_stride, float2 *out, size_t out_stride, int nsf,
                          int N, int nre, const float2 *tw, uint32_t radices, int nstages, float scale,
                          bool ext_cp, hipStream_t st);
// transmit: nsf grids (14 x nre at in + i*in_stride) -> 15 N time samples at out + i*out_stride
hipError_t launch_ofdm_tx(const float2 *in, size_t in_stride, float2 *out, size_t out_stride, int nsf,
                          int N, int nre, const float2 *tw, uint32_t radices, int nstages, float scale,
                          bool ext_cp, hipStream_t st);
} // namespace srsgpu
#endif
