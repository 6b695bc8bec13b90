// MI355X OFDM receive FFT, srslte_ofdm_rx_sf for normal cyclic prefix
// (reference: lib/src/phy/dft/ofdm.c:47-136 plan, 401-470 run): per slot, 7 forward DFTs of
// symbol_sz points (unnormalised, e^{-2 pi i k n / N} like FFTW's forward plan) on the samples
// after each CP (first CP ceil(160 N / 2048), then ceil(144 N / 2048); phy_common.h:104-109), then
// the subcarrier gather [N - nre/2, N) ++ [1, 1 + nre/2) (DC skipped), optionally scaled by
// 1/sqrt(N) (srslte_ofdm_set_normalize).
// One workgroup per OFDM symbol: the N samples go to LDS, a mixed-radix (4/2/3) Stockham
// autosort FFT runs in LDS with exact twiddles from a per-size table, and only the nof_re used
// subcarriers are written back.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ofdm_kernels.h"

namespace srsgpu {

struct cf {
  float x, y;
};
__device__ __forceinline__ cf cadd(cf a, cf b) { return {a.x + b.x, a.y + b.y}; }
__device__ __forceinline__ cf csub(cf a, cf b) { return {a.x - b.x, a.y - b.y}; }
__device__ __forceinline__ cf cmul(cf a, cf b) { return {a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x}; }
__device__ __forceinline__ cf mul_mi(cf a) { return {a.y, -a.x}; } // a * (-i)

#define OFDM_MAXN 2048

// one Stockham radix-R pass: d1[(j/Ns) Ns R + j%Ns + r Ns] = DFT_R(tw^(r k) d0[j + r N/R])
template <int R>
__device__ __forceinline__ void stage(const cf *__restrict__ d0, cf *__restrict__ d1, int N, int Ns,
                                      const float2 *__restrict__ tw) {
  const int nb = N / R;
  for (int j = threadIdx.x; j < nb; j += blockDim.x) {
    const int k = j % Ns;
    const int tstep = k * (N / (Ns * R)); // e^{-2 pi i r k / (Ns R)} = tw[r tstep]
    cf v[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
      cf a = d0[j + r * nb];
      if (r) {
        const float2 w = tw[r * tstep];
        a = cmul(a, cf{w.x, w.y});
      }
      v[r] = a;
    }
    cf y[R];
    if constexpr (R == 4) {
      const cf s02 = cadd(v[0], v[2]), d02 = csub(v[0], v[2]);
      const cf s13 = cadd(v[1], v[3]), d13 = mul_mi(csub(v[1], v[3]));
      y[0] = cadd(s02, s13);
      y[2] = csub(s02, s13);
      y[1] = cadd(d02, d13);
      y[3] = csub(d02, d13);
    } else if constexpr (R == 2) {
      y[0] = cadd(v[0], v[1]);
      y[1] = csub(v[0], v[1]);
    } else { // R == 3, w = e^{-2 pi i / 3}
      const float c = -0.5f, sn = -0.86602540378443865f;
      const cf t = cadd(v[1], v[2]), u = csub(v[1], v[2]);
      y[0] = cadd(v[0], t);
      const cf m = {v[0].x + c * t.x, v[0].y + c * t.y};
      const cf q = {-sn * u.y, sn * u.x}; // i * sn * u
      y[1] = cadd(m, q);
      y[2] = csub(m, q);
    }
    const int o = (j / Ns) * Ns * R + k;
#pragma unroll
    for (int r = 0; r < R; r++) d1[o + r * Ns] = y[r];
  }
}

__global__ __launch_bounds__(256) void k_ofdm_rx(const float2 *__restrict__ in, size_t in_stride,
                                                 float2 *__restrict__ out, size_t out_stride, int N,
                                                 int nre, int cp0, int cp, const float2 *__restrict__ tw,
                                                 const uint32_t radices, int nstages, float scale) {
  __shared__ cf buf[2][OFDM_MAXN];
  const int sym = blockIdx.x % 14, sf = blockIdx.x / 14;
  const int slot = sym / 7, l = sym % 7;
  // symbol start: slot * 7.5 N + cp0 + l * (N + cp)   (ofdm.c:98-103 guru plan strides)
  const size_t start = (size_t)slot * (N * 15 / 2) + cp0 + (size_t)l * (N + cp);
  const cf *src = (const cf *)(in + (size_t)sf * in_stride + start);
  for (int n = threadIdx.x; n < N; n += blockDim.x) buf[0][n] = src[n];
  __syncthreads();
  int cur = 0, Ns = 1;
  for (int st = 0; st < nstages; st++) {
    const int R = (radices >> (4 * st)) & 15;
    if (R == 4)
      stage<4>(buf[cur], buf[cur ^ 1], N, Ns, tw);
    else if (R == 2)
      stage<2>(buf[cur], buf[cur ^ 1], N, Ns, tw);
    else
      stage<3>(buf[cur], buf[cur ^ 1], N, Ns, tw);
    __syncthreads();
    cur ^= 1;
    Ns *= R;
  }
  // gather: [N - nre/2, N) then [1, 1 + nre/2)
  cf *dst = (cf *)(out + (size_t)sf * out_stride + (size_t)sym * nre);
  const int h = nre / 2;
  for (int k = threadIdx.x; k < nre; k += blockDim.x) {
    const cf v = buf[cur][k < h ? N - h + k : 1 + k - h];
    dst[k] = cf{v.x * scale, v.y * scale};
  }
}

hipError_t launch_ofdm_rx(const float2 *in, size_t in_stride, float2 *out, size_t out_stride, int nsf,
                          int N, int nre, const float2 *tw, uint32_t radices, int nstages, float scale,
                          hipStream_t st) {
  if (nsf <= 0) return hipSuccess;
  const int cp0 = (int)ceilf(160.0f * N / 2048.0f), cp = (int)ceilf(144.0f * N / 2048.0f);
  hipLaunchKernelGGL(k_ofdm_rx, dim3((unsigned)nsf * 14), dim3(256), 0, st, in, in_stride, out, out_stride,
                     N, nre, cp0, cp, tw, radices, nstages, scale);
  return hipGetLastError();
}

// srslte_ofdm_tx_sf (ofdm.c:491-598), normal CP: per symbol the grid row goes to bins
// [1, 1 + nre/2) (upper half) and [N - nre/2, N) (lower half), DC and guards zero, an
// unnormalised backward DFT (FFTW backward: e^{+2 pi i k n / N}, here conj(FFT(conj(x)))), the
// optional 1/sqrt(N) scaling, and the last cp samples copied in front of the symbol.
__global__ __launch_bounds__(256) void k_ofdm_tx(const float2 *__restrict__ in, size_t in_stride,
                                                 float2 *__restrict__ out, size_t out_stride, int N,
                                                 int nre, int cp0, int cp, const float2 *__restrict__ tw,
                                                 const uint32_t radices, int nstages, float scale) {
  __shared__ cf buf[2][OFDM_MAXN];
  const int sym = blockIdx.x % 14, sf = blockIdx.x / 14;
  const int slot = sym / 7, l = sym % 7;
  const cf *src = (const cf *)(in + (size_t)sf * in_stride + (size_t)sym * nre);
  const int h = nre / 2;
  for (int n = threadIdx.x; n < N; n += blockDim.x) {
    cf v = {0.f, 0.f};
    if (n >= 1 && n < 1 + h)
      v = src[h + n - 1];
    else if (n >= N - h)
      v = src[n - (N - h)];
    buf[0][n] = cf{v.x, -v.y};
  }
  __syncthreads();
  int cur = 0, Ns = 1;
  for (int st = 0; st < nstages; st++) {
    const int R = (radices >> (4 * st)) & 15;
    if (R == 4)
      stage<4>(buf[cur], buf[cur ^ 1], N, Ns, tw);
    else if (R == 2)
      stage<2>(buf[cur], buf[cur ^ 1], N, Ns, tw);
    else
      stage<3>(buf[cur], buf[cur ^ 1], N, Ns, tw);
    __syncthreads();
    cur ^= 1;
    Ns *= R;
  }
  const int c = l == 0 ? cp0 : cp;
  const size_t start = (size_t)slot * (N * 15 / 2) + (l ? cp0 + N + (size_t)(l - 1) * (N + cp) : 0);
  cf *dst = (cf *)(out + (size_t)sf * out_stride + start);
  for (int n = threadIdx.x; n < N + c; n += blockDim.x) {
    const cf v = buf[cur][n < c ? N - c + n : n - c];
    dst[n] = cf{v.x * scale, -v.y * scale};
  }
}

hipError_t launch_ofdm_tx(const float2 *in, size_t in_stride, float2 *out, size_t out_stride, int nsf,
                          int N, int nre, const float2 *tw, uint32_t radices, int nstages, float scale,
                          hipStream_t st) {
  if (nsf <= 0) return hipSuccess;
  const int cp0 = (int)ceilf(160.0f * N / 2048.0f), cp = (int)ceilf(144.0f * N / 2048.0f);
  hipLaunchKernelGGL(k_ofdm_tx, dim3((unsigned)nsf * 14), dim3(256), 0, st, in, in_stride, out, out_stride,
                     N, nre, cp0, cp, tw, radices, nstages, scale);
  return hipGetLastError();
}

} // namespace srsgpu
