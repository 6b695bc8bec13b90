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
#include <string.h>
#include <stdint.h>
#include <stdlib.h>

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
                                                 int nre, int cp0, int cp, int ns, const float2 *__restrict__ tw,
                                                 const uint32_t radices, int nstages, float scale) {
  __shared__ cf buf[2][OFDM_MAXN];
  const int sym = blockIdx.x % (2 * ns), sf = blockIdx.x / (2 * ns);
  const int slot = sym / ns, l = sym % ns;
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

// ---- fixed-size path: the LTE symbol sizes, with the whole stage plan known at compile time ----
// Radix 8 first (then 4, 2, 3): 2048 = 8.8.8.4 is four LDS passes instead of six, and with N, R
// and Ns constants every index division is a shift or a multiply. Small symbols share a
// workgroup (256 / S threads per symbol) so every size launches full 256-thread workgroups.
// the R-point DFT of one butterfly (v in, y out)
template <int R> __device__ __forceinline__ void bfly(const cf *v, cf *y) {
  if constexpr (R == 8) {
    // two 4-point DFTs (even / odd inputs) joined with W8^k = e^{-i pi k / 4}
    const float c = 0.70710678118654752f;
    cf e[4], o[4];
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const cf a0 = v[h], a1 = v[h + 2], a2 = v[h + 4], a3 = v[h + 6];
      const cf s02 = cadd(a0, a2), d02 = csub(a0, a2);
      const cf s13 = cadd(a1, a3), d13 = mul_mi(csub(a1, a3));
      cf *z = h ? o : e;
      z[0] = cadd(s02, s13);
      z[2] = csub(s02, s13);
      z[1] = cadd(d02, d13);
      z[3] = csub(d02, d13);
    }
    const cf o1 = {c * (o[1].x + o[1].y), c * (o[1].y - o[1].x)}; // * (c - ic)
    const cf o2 = mul_mi(o[2]);                                    // * -i
    const cf o3 = {c * (o[3].y - o[3].x), -c * (o[3].x + o[3].y)}; // * (-c - ic)
    y[0] = cadd(e[0], o[0]);
    y[4] = csub(e[0], o[0]);
    y[1] = cadd(e[1], o1);
    y[5] = csub(e[1], o1);
    y[2] = cadd(e[2], o2);
    y[6] = csub(e[2], o2);
    y[3] = cadd(e[3], o3);
    y[7] = csub(e[3], o3);
  } else if constexpr (R == 4) {
    const cf s02 = cadd(v[0], v[2]), d02 = csub(v[0], v[2]);
    const cf s13 = cadd(v[1], v[3]), d13 = mul_mi(csub(v[1], v[3]));
    y[0] = cadd(s02, s13);
    y[2] = csub(s02, s13);
    y[1] = cadd(d02, d13);
    y[3] = csub(d02, d13);
  } else if constexpr (R == 2) {
    y[0] = cadd(v[0], v[1]);
    y[1] = csub(v[0], v[1]);
  } else {
    const float cc = -0.5f, sn = -0.86602540378443865f;
    const cf tt = cadd(v[1], v[2]), u = csub(v[1], v[2]);
    y[0] = cadd(v[0], tt);
    const cf m = {v[0].x + cc * tt.x, v[0].y + cc * tt.y};
    const cf q = {-sn * u.y, sn * u.x};
    y[1] = cadd(m, q);
    y[2] = csub(m, q);
  }
}

// One Stockham stage in place on a single LDS buffer: each thread reads the inputs of its
// butterflies (the first stage straight from the time-domain samples in HBM, Ns = 1: no twiddles),
// the workgroup waits until every read is done, then the outputs are written back. One 8 N-byte
// buffer per symbol instead of a ping-pong pair, so twice the workgroups fit in a CU's LDS, and no
// separate pass copies the input into LDS. `live` = the thread's symbol exists (others compute on
// zeros and only keep the barriers).
// LDS slot of element p: one pad slot after every 16 elements (128 B), so the strided butterfly
// writes of the first stages (element stride 8 and 64) spread over all banks instead of landing 8-
// and 16-fold on the same ones
__device__ __forceinline__ int lpad(int p) { return p + (p >> 4); }
template <int N> constexpr int lds_slots() { return N + N / 16; }

// TWC: twiddles from the hardware sine / cosine (v_sin_f32 / v_cos_f32 take the angle in revolutions,
// here -r k / (Ns R) exactly for the power-of-two stages) instead of loads from the table: no L2 round
// trip between a stage's LDS reads and its butterflies. Results within a few ulp of the table's.
template <int R, int N, int Ns, int TPS, bool FIRST, bool TWC = false>
__device__ __forceinline__ void stage_ip(const cf *__restrict__ src, cf *buf, const float2 *__restrict__ tw,
                                         int t, bool live) {
  constexpr int nb = N / R;
  constexpr int NPT = (nb + TPS - 1) / TPS;
  cf v[NPT][R];
#pragma unroll
  for (int q = 0; q < NPT; q++) {
    const int j = t + q * TPS;
    const int k = j % Ns;
#pragma unroll
    for (int r = 0; r < R; r++) {
      cf a = {0.f, 0.f};
      if (j < nb) {
        if (FIRST) {
          if (live) a = src[j + r * nb];
        } else {
          a = buf[lpad(j + r * nb)];
          if (Ns > 1 && r) { // e^{-2 pi i r k / (Ns R)} = tw[r k N / (Ns R)]
            if constexpr (TWC) {
              const float rev = -(float)(r * k) * (1.0f / (float)(Ns * R));
              a = cmul(a, cf{__builtin_amdgcn_cosf(rev), __builtin_amdgcn_sinf(rev)});
            } else {
              const float2 w = tw[r * k * (N / (Ns * R))];
              a = cmul(a, cf{w.x, w.y});
            }
          }
        }
      }
      v[q][r] = a;
    }
  }
  if (!FIRST) __syncthreads(); // every read of buf done before the first write
#pragma unroll
  for (int q = 0; q < NPT; q++) {
    const int j = t + q * TPS;
    if (j >= nb) break;
    const int k = j % Ns;
    cf y[R];
    bfly<R>(v[q], y);
    const int o = (j / Ns) * Ns * R + k;
#pragma unroll
    for (int r = 0; r < R; r++) buf[lpad(o + r * Ns)] = y[r];
  }
  __syncthreads();
}

// stages Ns .. N in place (radix 8 first, then 4, 2, 3); the result is left in buf
template <int N, int Ns, int TPS, bool TWC = false>
__device__ __forceinline__ void fft_ip(const cf *__restrict__ src, cf *buf, const float2 *__restrict__ tw,
                                       int t, bool live) {
  if constexpr (Ns < N) {
    constexpr int rem = N / Ns;
    constexpr int R = rem % 8 == 0 ? 8 : rem % 4 == 0 ? 4 : rem % 2 == 0 ? 2 : 3;
    stage_ip<R, N, Ns, TPS, Ns == 1, TWC>(src, buf, tw, t, live);
    fft_ip<N, Ns * R, TPS, TWC>(src, buf, tw, t, live);
  }
}

template <int N>
constexpr int syms_per_wg() {
  return N >= 1024 ? 1 : N >= 512 ? 2 : N >= 256 ? 4 : 8;
}

template <int N, bool TWC>
__global__ __launch_bounds__(256) void k_ofdm_rx_c(const float2 *__restrict__ in, size_t in_stride,
                                                   float2 *__restrict__ out, size_t out_stride, int nsym,
                                                   int nre, int cp0, int cp, int ns,
                                                   const float2 *__restrict__ tw, float scale) {
  constexpr int S = syms_per_wg<N>(), TPS = 256 / S;
  __shared__ cf buf[S][lds_slots<N>()];
  const int s = threadIdx.x / TPS, t = threadIdx.x % TPS;
  const int g = blockIdx.x * S + s; // symbol of this thread group (past nsym: idle, but at barriers)
  const bool live = g < nsym;
  const int sym = g % (2 * ns), sf = g / (2 * ns);
  const int slot = sym / ns, l = sym % ns;
  const size_t start = (size_t)slot * (N * 15 / 2) + cp0 + (size_t)l * (N + cp);
  const cf *src = (const cf *)(in + (size_t)(live ? sf : 0) * in_stride + start);
  fft_ip<N, 1, TPS, TWC>(src, buf[s], tw, t, live);
  const cf *res = buf[s];
  if (live) {
    cf *dst = (cf *)(out + (size_t)sf * out_stride + (size_t)sym * nre);
    const int h = nre / 2;
    for (int k = t; k < nre; k += TPS) {
      const cf v = res[lpad(k < h ? N - h + k : 1 + k - h)];
      dst[k] = cf{v.x * scale, v.y * scale};
    }
  }
}

// Large symbols (N >= 1024, one symbol per workgroup): a resident grid of workgroups, each taking
// symbols g, g + gridDim.x, ... The first stage's inputs of the next symbol are loaded into
// registers as soon as the current symbol's first stage is in LDS, so they are in flight while the
// remaining stages and the output of the current symbol run (one symbol per workgroup left every
// wave waiting on its 16 KB read with nothing else to do).
template <int N>
__global__ __launch_bounds__(256) void k_ofdm_rx_p(const float2 *__restrict__ in, size_t in_stride,
                                                   float2 *__restrict__ out, size_t out_stride, int nsym,
                                                   int nre, int cp0, int cp, int ns, const float2 *__restrict__ tw,
                                                   float scale) {
  constexpr int R0 = N % 8 == 0 ? 8 : N % 4 == 0 ? 4 : N % 2 == 0 ? 2 : 3;
  constexpr int nb0 = N / R0, NPT = (nb0 + 255) / 256;
  __shared__ cf buf[lds_slots<N>()];
  const int t = threadIdx.x;
  cf v[NPT][R0];
  auto load = [&](int g) {
    const int sym = g % (2 * ns), sf = g / (2 * ns);
    const int slot = sym / ns, l = sym % ns;
    const size_t start = (size_t)slot * (N * 15 / 2) + cp0 + (size_t)l * (N + cp);
    const cf *src = (const cf *)(in + (size_t)sf * in_stride + start);
#pragma unroll
    for (int q = 0; q < NPT; q++) {
      const int j = t + q * 256;
#pragma unroll
      for (int r = 0; r < R0; r++) v[q][r] = j < nb0 ? src[j + r * nb0] : cf{0.f, 0.f};
    }
  };
  int g = blockIdx.x;
  if (g < nsym) load(g);
#pragma unroll 1
  for (; g < nsym; g += gridDim.x) {
    // first stage (Ns = 1, no twiddles) from the registers into LDS
#pragma unroll
    for (int q = 0; q < NPT; q++) {
      const int j = t + q * 256;
      if (j >= nb0) break;
      cf y[R0];
      bfly<R0>(v[q], y);
#pragma unroll
      for (int r = 0; r < R0; r++) buf[lpad(j * R0 + r)] = y[r];
    }
    __syncthreads();
    if (g + (int)gridDim.x < nsym) load(g + gridDim.x); // next symbol's samples, in flight from here
    __builtin_amdgcn_sched_barrier(0);
    // opaque copies of the twiddle pointer and the thread index per symbol: left alone, the compiler
    // hoists every stage's twiddle addressing out of the symbol loop and holds it in registers
    // (130 VGPRs: a third of the occupancy)
    const float2 *twl = tw;
    int tl = t; // and of the thread index: the stages' twiddle offsets are recomputed per symbol
    asm volatile("" : "+s"(twl), "+v"(tl));
    fft_ip<N, R0, 256>(nullptr, buf, twl, tl, true);
    const int sym = g % (2 * ns), sf = g / (2 * ns);
    cf *dst = (cf *)(out + (size_t)sf * out_stride + (size_t)sym * nre);
    const int h = nre / 2;
    for (int k = t; k < nre; k += 256) {
      const cf w = buf[lpad(k < h ? N - h + k : 1 + k - h)];
      dst[k] = cf{w.x * scale, w.y * scale};
    }
    __syncthreads(); // every read of buf done before the next symbol's first stage writes it
  }
}

// resident workgroups of k_ofdm_rx_p<N> on the device (CUs x workgroups per CU by its registers
// and LDS)
template <int N> static int ofdm_resident_wgs() {
  static const int n = [] {
    int dev = 0, cus = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_ofdm_rx_p<N>, 256, 0) != hipSuccess || per <= 0)
      per = 4;
    return cus * per;
  }();
  return n;
}

// CP lengths and symbols per slot (ofdm.c:75-76): normal CP ceil(160 N / 2048) then ceil(144 N / 2048),
// 7 symbols; extended CP ceil(512 N / 2048) for all 6 symbols. Both fill 7.5 N samples per slot.
static void cp_layout(int N, bool ext, int &cp0, int &cp, int &ns) {
  if (ext) {
    cp0 = cp = (int)ceilf(512.0f * N / 2048.0f);
    ns = 6;
  } else {
    cp0 = (int)ceilf(160.0f * N / 2048.0f);
    cp = (int)ceilf(144.0f * N / 2048.0f);
    ns = 7;
  }
}

hipError_t launch_ofdm_rx(const float2 *in, size_t in_stride, float2 *out, size_t out_stride, int nsf,
                          int N, int nre, const float2 *tw, uint32_t radices, int nstages, float scale,
                          bool ext_cp, hipStream_t st) {
  if (nsf <= 0) return hipSuccess;
  int cp0, cp, ns;
  cp_layout(N, ext_cp, cp0, cp, ns);
  const int nsym = nsf * 2 * ns;
  // SRSGPU_OFDM_PERSIST=1: the resident-grid kernel with next-symbol prefetch for the large sizes.
  // Off by default: alone on the GPU it took 68 us per 512 20 MHz subframes against 59 us for one
  // symbol per workgroup (profiles/r04_s6_kb_*.json), and its fixed grid fares worse still beside
  // another stream's kernels.
  static const bool persist = [] {
    const char *e = getenv("SRSGPU_OFDM_PERSIST");
    return e && e[0] == '1';
  }();
  if (persist && (N == 2048 || N == 1536 || N == 1024)) {
    // every workgroup takes the same number of symbols (no partial last round)
#define OFDM_RX_P(n)                                                                               \
  if (N == n) {                                                                                    \
    const int res = ofdm_resident_wgs<n>(), per = (nsym + res - 1) / res;                          \
    hipLaunchKernelGGL(k_ofdm_rx_p<n>, dim3((unsigned)((nsym + per - 1) / per)), dim3(256), 0, st, in, \
                       in_stride, out, out_stride, nsym, nre, cp0, cp, ns, tw, scale);                 \
    return hipGetLastError();                                                                      \
  }
    OFDM_RX_P(2048)
    OFDM_RX_P(1536)
    OFDM_RX_P(1024)
#undef OFDM_RX_P
  }
  // twiddles computed in the kernel (see stage_ip) by default: 41 us against 58 us with the table
  // loads per 512 20 MHz subframes, alone on the GPU (profiles/r04_s13_kb_*.json);
  // SRSGPU_OFDM_TW=table restores the loads
  static const bool twc = [] {
    const char *e = getenv("SRSGPU_OFDM_TW");
    return !(e && strcmp(e, "table") == 0);
  }();
#define OFDM_RX_C(n)                                                                               \
  case n:                                                                                          \
    if (twc)                                                                                       \
      hipLaunchKernelGGL((k_ofdm_rx_c<n, true>), dim3((unsigned)((nsym + syms_per_wg<n>() - 1) / syms_per_wg<n>())), \
                         dim3(256), 0, st, in, in_stride, out, out_stride, nsym, nre, cp0, cp, ns, tw, scale); \
    else                                                                                           \
      hipLaunchKernelGGL((k_ofdm_rx_c<n, false>), dim3((unsigned)((nsym + syms_per_wg<n>() - 1) / syms_per_wg<n>())), \
                         dim3(256), 0, st, in, in_stride, out, out_stride, nsym, nre, cp0, cp, ns, tw, scale); \
    return hipGetLastError();
  switch (N) {
    OFDM_RX_C(128)
    OFDM_RX_C(256)
    OFDM_RX_C(384)
    OFDM_RX_C(512)
    OFDM_RX_C(768)
    OFDM_RX_C(1024)
    OFDM_RX_C(1536)
    OFDM_RX_C(2048)
  default:
    break;
  }
#undef OFDM_RX_C
  hipLaunchKernelGGL(k_ofdm_rx, dim3((unsigned)nsym), dim3(256), 0, st, in, in_stride, out, out_stride,
                     N, nre, cp0, cp, ns, tw, radices, nstages, scale);
  return hipGetLastError();
}

// srslte_ofdm_tx_sf (ofdm.c:491-598), normal CP: per symbol the grid row goes to bins
// [1, 1 + nre/2) (upper half) and [N - nre/2, N) (lower half), DC and guards zero, an
// unnormalised backward DFT (FFTW backward: e^{+2 pi i k n / N}, here conj(FFT(conj(x)))), the
// optional 1/sqrt(N) scaling, and the last cp samples copied in front of the symbol.
__global__ __launch_bounds__(256) void k_ofdm_tx(const float2 *__restrict__ in, size_t in_stride,
                                                 float2 *__restrict__ out, size_t out_stride, int N,
                                                 int nre, int cp0, int cp, int ns, const float2 *__restrict__ tw,
                                                 const uint32_t radices, int nstages, float scale) {
  __shared__ cf buf[2][OFDM_MAXN];
  const int sym = blockIdx.x % (2 * ns), sf = blockIdx.x / (2 * ns);
  const int slot = sym / ns, l = sym % ns;
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
                          bool ext_cp, hipStream_t st) {
  if (nsf <= 0) return hipSuccess;
  int cp0, cp, ns;
  cp_layout(N, ext_cp, cp0, cp, ns);
  hipLaunchKernelGGL(k_ofdm_tx, dim3((unsigned)nsf * 2 * ns), dim3(256), 0, st, in, in_stride, out, out_stride,
                     N, nre, cp0, cp, ns, tw, radices, nstages, scale);
  return hipGetLastError();
}

} // namespace srsgpu
