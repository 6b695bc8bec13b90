// MI355X downlink CRS channel estimation, srslte_chest_dl_estimate_port (ports 0 and 1) for the
// normal-CP, non-MBSFN, per-symbol (average_subframe off) configuration
// (reference: lib/src/phy/ch_estimation/chest_dl.c:641-694 and the helpers it calls):
//   1. least squares   pilots received at the CRS REs of symbols 0/4/7/11 (refsignal_cs_get_sf,
//                      refsignal_dl.c:404-430) times conj(CRS) (refsignal_dl.c:265-318)
//   2. noise           estimate_noise_pilots (chest_dl.c:268-329), REFS algorithm, including its
//                      reference behaviour of keeping only the last symbol's residual power
//   3. smoothing       srslte_conv_same_cf with extrapolated extremes (convolution.c:172-211),
//                      default 3-tap [w, 1-2w, w] (chest_dl.c:155-160, 464-469)
//   4. frequency       srslte_interp_linear_offset per CRS symbol (interp.c:245-272), M = 6
//   5. time            srslte_interp_linear_vector(2) between CRS symbols (chest_dl.c:392-397,
//                      interp.c:150-173): running sums of (ce_b - ce_a) / d
// One workgroup per (subframe, rx antenna, port): pilots and their smoothed copy stay in LDS, each
// thread then produces whole subcarrier columns (14 symbols) in registers and streams them out.
// Float arithmetic in the reference's operation order; the stage is checked with a tolerance
// (float stages 1e-4 relative).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "chest_kernels.h"

#pragma clang fp contract(off)

namespace srsgpu {

struct c32 {
  float x, y;
};
__device__ __forceinline__ c32 cadd(c32 a, c32 b) { return {a.x + b.x, a.y + b.y}; }
__device__ __forceinline__ c32 csub(c32 a, c32 b) { return {a.x - b.x, a.y - b.y}; }
__device__ __forceinline__ c32 cscale(c32 a, float s) { return {a.x * s, a.y * s}; }
__device__ __forceinline__ c32 cmulconj(c32 a, c32 b) { // a * conj(b)
  return {a.x * b.x + a.y * b.y, a.y * b.x - a.x * b.y};
}

#define CH_MAXP (2 * 110) // pilots per CRS symbol

__global__ __launch_bounds__(256) void k_chest(const ChestItem *__restrict__ items, int nitems,
                                               int nprb, int cell_id, const float2 *__restrict__ crs,
                                               const float *__restrict__ filt, int flen) {
  __shared__ c32 ls[4][CH_MAXP];
  __shared__ c32 sm[4][CH_MAXP];
  __shared__ float red[256];
  const int it = blockIdx.x;
  if (it >= nitems) return;
  const ChestItem t = items[it];
  const int np = 2 * nprb, nsc = 12 * nprb;
  const c32 *grid = (const c32 *)t.grid;
  const c32 *pil = (const c32 *)(crs + (size_t)t.sf_idx * 4 * np);
  const int sym[4] = {0, 4, 7, 11};
  const int port = (int)t.port;
  // 1. LS: v = 0 / 3 alternating over the CRS symbols (port 1: 3 / 0), fidx = (v + id % 6) % 6;
  //    ports 0 and 1 share the pilot sequence (csr_refs.pilots[port / 2])
  for (int e = threadIdx.x; e < 4 * np; e += blockDim.x) {
    const int l = e / np, m = e % np;
    const int f = (((l & 1) ^ port ? 3 : 0) + cell_id % 6) % 6;
    ls[l][m] = cmulconj(grid[sym[l] * nsc + f + 6 * m], pil[l * np + m]);
  }
  __syncthreads();
  // 2. noise (REFS): residual of the last CRS symbol against its 4 staggered neighbours in the
  //    symbols around it (bottom one extrapolated as 2 ls[2] - ls[0]), power / 4 * sqrt(5)
  if (t.noise) {
    const int f0 = ((port ? 3 : 0) + cell_id % 6) % 6; // srslte_refsignal_cs_fidx(cell, 0, port, 0)
    const int off = f0 < 3 ? 0 : 1; // ((fidx < 3) ^ (4 & 1)) ? 0 : 1
    float acc = 0.f;
    for (int k = threadIdx.x; k < np; k += blockDim.x) {
      c32 tmp = ls[3][k];
      for (int nb = 0; nb < 2; nb++) {
        auto row = [&](int q) -> c32 {
          return nb == 0 ? ls[2][q] : csub(cscale(ls[2][q], 2.0f), ls[0][q]);
        };
        if (k >= off) tmp = cadd(tmp, row(k - off));            // tmp[off + t] += prev[t]
        if (k < np + off - 1) tmp = cadd(tmp, row(1 - off + k)); // tmp[t] += prev[1 - off + t]
        if (off && k == 0) tmp = cadd(tmp, csub(cscale(row(0), 2.0f), row(1)));
        if (!off && k == np - 1) tmp = cadd(tmp, csub(cscale(row(np - 2), 2.0f), row(np - 1)));
      }
      tmp = cscale(tmp, 1.0f / 5.0f);
      const c32 r = csub(ls[3][k], tmp);
      acc += r.x * r.x + r.y * r.y;
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
      if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
      __syncthreads();
    }
    if (threadIdx.x == 0) *t.noise = red[0] / (float)np / 4.0f * sqrtf(5.0f);
  }
  // 3. smoothing (conv_same with extrapolated extremes); flen == 0: none
  for (int e = threadIdx.x; e < 4 * np; e += blockDim.x) {
    const int l = e / np, i = e % np;
    if (flen == 0) {
      sm[l][i] = ls[l][i];
      continue;
    }
    const int M = flen, h = M / 2;
    c32 acc = {0.f, 0.f};
    for (int k = 0; k < M; k++) {
      const int src = i - h + k;
      c32 v;
      if (src < 0) { // first[i] = (2 + h - q) in[1] - (1 + h - q) in[0], q = i + k
        const float q = (float)(i + k);
        v = csub(cscale(ls[l][1], 2.0f + h - q), cscale(ls[l][0], 1.0f + h - q));
      } else if (src >= np) { // last[q] = (2 + q - h) in[N-1] - (1 + q - h) in[N-2]
        const float q = (float)(src - (np - M + 1) + 0);
        v = csub(cscale(ls[l][np - 1], 2.0f + q - h), cscale(ls[l][np - 2], 1.0f + q - h));
      } else {
        v = ls[l][src];
      }
      acc = cadd(acc, cscale(v, filt[k]));
    }
    sm[l][i] = acc;
  }
  __syncthreads();
  // 4 + 5. per subcarrier column: frequency interpolation of the 4 CRS symbols, then time
  c32 *ce = (c32 *)t.ce;
  const float inv6 = 1.0f / 6.0f;
  for (int k = threadIdx.x; k < nsc; k += blockDim.x) {
    c32 f[4];
    for (int l = 0; l < 4; l++) {
      const int fo = (((l & 1) ^ port ? 3 : 0) + cell_id % 6) % 6;
      const c32 *in = sm[l];
      if (k < fo) { // output[fo-j-1] = in[0] - (j+1) (in[1]-in[0]) / M
        const int j = fo - 1 - k;
        const c32 v = cscale(csub(in[1], in[0]), (float)(j + 1)); // complex / (6 + 0i)
        f[l] = csub(in[0], c32{v.x / 6.0f, v.y / 6.0f});
      } else {
        const int tt = k - fo, i = tt / 6, j = tt % 6;
        if (i < np - 1)
          f[l] = cadd(in[i], cscale(cscale(csub(in[i + 1], in[i]), inv6), (float)j));
        else
        {
          const c32 v = cscale(csub(in[np - 1], in[np - 2]), (float)j);
          f[l] = cadd(in[np - 1], c32{v.x / 6.0f, v.y / 6.0f});
        }
      }
    }
    c32 col[14];
    col[0] = f[0];
    col[4] = f[1];
    col[7] = f[2];
    col[11] = f[3];
    c32 d = cscale(csub(f[1], f[0]), 0.25f); // symbols 1-3: d = 4
    col[1] = cadd(f[0], d);
    col[2] = cadd(col[1], d);
    col[3] = cadd(col[2], d);
    d = cscale(csub(f[2], f[1]), 1.0f / 3.0f); // symbols 5-6: d = 3
    col[5] = cadd(f[1], d);
    col[6] = cadd(col[5], d);
    d = cscale(csub(f[3], f[2]), 0.25f); // symbols 8-10, then 12-13 extrapolated from 11
    col[8] = cadd(f[2], d);
    col[9] = cadd(col[8], d);
    col[10] = cadd(col[9], d);
    col[12] = cadd(f[3], d);
    col[13] = cadd(col[12], d);
    for (int s = 0; s < 14; s++) ce[s * nsc + k] = col[s];
  }
}

hipError_t launch_chest(const ChestItem *d_items, int n, int nprb, int cell_id, const float2 *crs,
                        const float *filt, int flen, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_chest, dim3((unsigned)n), dim3(256), 0, st, d_items, n, nprb, cell_id, crs, filt,
                     flen);
  return hipGetLastError();
}

// srslte_refsignal_cs_put_sf (refsignal_dl.c:380-402): the CRS of a port into its grid plane at
// symbols 0/4/7/11, subcarriers fidx + 6m
__global__ __launch_bounds__(256) void k_crs_put(const ChestItem *__restrict__ items, int nitems, int nprb,
                                                 int cell_id, const float2 *__restrict__ crs) {
  const int it = blockIdx.x;
  if (it >= nitems) return;
  const ChestItem t = items[it];
  const int np = 2 * nprb, nsc = 12 * nprb, port = (int)t.port;
  const int sym[4] = {0, 4, 7, 11};
  const float2 *pil = crs + (size_t)t.sf_idx * 4 * np;
  float2 *g = t.ce; // the grid plane written
  for (int e = threadIdx.x; e < 4 * np; e += blockDim.x) {
    const int l = e / np, m = e % np;
    const int f = (((l & 1) ^ port ? 3 : 0) + cell_id % 6) % 6;
    g[sym[l] * nsc + f + 6 * m] = pil[l * np + m];
  }
}

hipError_t launch_crs_put(const ChestItem *d_items, int n, int nprb, int cell_id, const float2 *crs,
                          hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_crs_put, dim3((unsigned)n), dim3(256), 0, st, d_items, n, nprb, cell_id, crs);
  return hipGetLastError();
}

} // namespace srsgpu
