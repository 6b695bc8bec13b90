// MI355X downlink CRS channel estimation, srslte_chest_dl_estimate_port (ports 0-3) for
// normal- and extended-CP, non-MBSFN subframes, in every configuration srsUE's phch_worker sets
// (srsue/src/phy/phch_worker.cc:149,553-565; reference: lib/src/phy/ch_estimation/chest_dl.c:641-694
// and the helpers it calls):
//   1. least squares   pilots received at the CRS REs of symbols 0/4/7/11 (ports 0/1) or 1/8 (ports
//                      2/3); extended CP 0/3/6/9 or 1/7 (refsignal_cs_get_sf, refsignal_dl.c:404-430) times conj(CRS)
//                      (refsignal_dl.c:265-318)
//   2. measurements    RSRP, RSSI (chest_dl.c:500-511), RSRP correlation (:652-656), CFO (:562-587)
//   3. noise (REFS)    estimate_noise_pilots (chest_dl.c:268-329), including its reference behaviour
//                      of keeping only the last symbol's residual power
//   4. filter          fixed taps, or smooth_filter_auto's order-4 Gaussian with std dev = noise x 200
//                      (chest_dl.c:471-490, 616-618)
//   5. average/smooth  average_subframe: the 4 CRS symbols folded into one row at spacing 3
//                      (chest_dl.c:528-548); srslte_conv_same_cf with extrapolated extremes
//                      (convolution.c:172-211)
//   6. frequency       srslte_interp_linear_offset (interp.c:245-272): per CRS symbol with M = 6, or
//                      the averaged row with M = 3 and offset cell_id % 3 (chest_dl.c:393-399)
//   7. time            srslte_interp_linear_vector(2) between CRS symbols (chest_dl.c:421-442,
//                      interp.c:150-173), or the averaged row copied to all 14 (12) symbols (:410-414)
//   8. noise (PSS/EMPTY) in subframes 0 and 5 only (chest_dl.c:628-637, 332-361)
// One workgroup per (subframe, rx antenna, port): pilots and their smoothed copy stay in LDS, each
// thread then produces whole subcarrier columns (14 symbols) in registers and streams them out.
// Float arithmetic in the reference's operation order; the stage is checked with a tolerance
// (float stages 1e-4 relative).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

#include "chest_kernels.h"
#include "gmem.h"

#pragma clang fp contract(off)

namespace srsgpu {

struct c32 {
  float x, y;
};
__device__ __forceinline__ c32 cadd(c32 a, c32 b) { return {a.x + b.x, a.y + b.y}; }
__device__ __forceinline__ c32 csub(c32 a, c32 b) { return {a.x - b.x, a.y - b.y}; }
__device__ __forceinline__ c32 cscale(c32 a, float s) { return {a.x * s, a.y * s}; }
__device__ __forceinline__ c32 cmul(c32 a, c32 b) { return {a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x}; }
__device__ __forceinline__ c32 cmulconj(c32 a, c32 b) { // a * conj(b)
  return {a.x * b.x + a.y * b.y, a.y * b.x - a.x * b.y};
}
__device__ __forceinline__ float cpow(c32 a) { return a.x * a.x + a.y * a.y; }

#define CH_MAXP (2 * 110) // pilots per CRS symbol
#define CH_NRED 7

// block-wide sums of nv per-thread values (block-uniform call, 256 threads); results in red[j][0].
// The pairwise tree red[t] += red[t + s], s = 128 .. 1: the two wide levels through LDS (the upper
// half hands its values to the lower half, which adds them in registers), the six levels inside
// wave 0 with shuffles (lane t adds lane t + s, as the tree does), so the sums are the tree's, with
// 4 barriers instead of 9 and 128 LDS words per value instead of 256.
template <int nv> __device__ __forceinline__ void block_sum(float (*red)[128], const float *v) {
  const int t = threadIdx.x;
  float x[nv];
  _Pragma("unroll") for (int j = 0; j < nv; j++) x[j] = v[j];
  if (t >= 128)
    _Pragma("unroll") for (int j = 0; j < nv; j++) red[j][t - 128] = x[j];
  __syncthreads();
  if (t < 128)
    _Pragma("unroll") for (int j = 0; j < nv; j++) x[j] += red[j][t];
  __syncthreads();
  if (t >= 64 && t < 128)
    _Pragma("unroll") for (int j = 0; j < nv; j++) red[j][t - 64] = x[j];
  __syncthreads();
  if (t < 64) {
    _Pragma("unroll") for (int j = 0; j < nv; j++) {
      float y = x[j] + red[j][t];
      for (int s = 32; s > 0; s >>= 1) y += __shfl_down(y, s);
      if (t == 0) red[j][0] = y;
    }
  }
  __syncthreads();
}

// srslte_conv_same_cf output i (convolution.c:172-211), any filter length M: outputs i < M/2 read
// first[], outputs i >= N - M/2 read last[], both with extrapolated extremes
__device__ __forceinline__ c32 conv_same_at(const c32 *in, int N, int i, const float *f, int M) {
  const int h = M / 2;
  c32 acc = {0.f, 0.f};
  for (int k = 0; k < M; k++) {
    c32 v;
    if (i < h) { // first[q] = (2 + h - q) in[1] - (1 + h - q) in[0] for q < h, else in[q - h]
      const int q = i + k;
      v = q < h ? csub(cscale(in[1], (float)(2 + h - q)), cscale(in[0], (float)(1 + h - q))) : in[q - h];
    } else if (i < N - h) {
      v = in[i - h + k];
    } else { // last[q] = (2 + q - h) in[N-1] - (1 + q - h) in[N-2] for q >= M - 1, else in[N-M+q+1]
      const int q = i - (N - h) + k;
      v = q >= M - 1 ? csub(cscale(in[N - 1], (float)(2 + q - h)), cscale(in[N - 2], (float)(1 + q - h)))
                     : in[N - M + q + 1];
    }
    acc = cadd(acc, cscale(v, f[k]));
  }
  return acc;
}

// srslte_interp_linear_offset output k (interp.c:245-272): n inputs, M outputs per input, off_st
// extrapolated ahead, diff_vec = (in[i+1] - in[i]) * (1/M) times the ramp j
__device__ __forceinline__ c32 interp_at(const c32 *in, int n, int k, int off, int M, float invM) {
  if (k < off) { // output[off-j-1] = in[0] - (j+1) (in[1]-in[0]) / M
    const c32 v = cscale(csub(in[1], in[0]), (float)(off - k)); // complex / (M + 0i)
    return csub(in[0], c32{v.x / (float)M, v.y / (float)M});
  }
  const int tt = k - off, i = tt / M, j = tt % M;
  if (i < n - 1) return cadd(in[i], cscale(cscale(csub(in[i + 1], in[i]), invM), (float)j));
  const c32 v = cscale(csub(in[n - 1], in[n - 2]), (float)j);
  return cadd(in[n - 1], c32{v.x / (float)M, v.y / (float)M});
}

__global__ __launch_bounds__(256) void k_chest(const ChestItem *__restrict__ items, int nitems, ChestCfg cfg,
                                               const float2 *__restrict__ crs, const float *__restrict__ filt,
                                               const float2 *__restrict__ pss) {
  __shared__ c32 ls[4 * CH_MAXP]; // LS estimates, row l at l * np (the reference's pilot_estimates)
  __shared__ c32 sm[4 * CH_MAXP];
  __shared__ float red[CH_NRED][128];
  __shared__ float fs[64];
  __shared__ float s_noise;
  const int it = blockIdx.x;
  if (it >= nitems) return;
  ChestItem t = items[it];
  t.grid = gmem(t.grid);
  t.ce = gmem(t.ce);
  t.noise = gmem(t.noise);
  t.meas = gmem(t.meas);
  const int nprb = cfg.nprb, cell_id = cfg.cell_id, np = 2 * nprb, nsc = 12 * nprb;
  // gridDim.y workgroups share a grid: each repeats steps 1-5 (pilots only) and writes its own
  // range of subcarrier columns; part 0 writes the measurements and the noise. A subframe whose
  // PSS / EMPTY noise this call updates (read at step 4, written at step 8) stays in part 0 alone.
  const bool nz05 = t.noise && cfg.noise_alg != 0 && (t.sf_idx == 0 || t.sf_idx == 5);
  const int part = nz05 ? 0 : (int)blockIdx.y, nparts = nz05 ? 1 : (int)gridDim.y;
  if (nz05 && blockIdx.y > 0) return;
  if (part > 0) {
    t.meas = nullptr;
    t.cfo = 0;
  }
  const int kb = (nsc * part) / nparts, ke = (nsc * (part + 1)) / nparts;
  const c32 *grid = (const c32 *)t.grid;
  const int port = (int)t.port;
  // ports 0/1: CRS symbols 0, ns - 3, ns, 2 ns - 3; ports 2/3: 1 and ns + 1 (srslte_refsignal_cs_nsymbol,
  // refsignal_dl.c:112-122; ns = 7 normal, 6 extended CP), their pilots (csr_refs.pilots[port / 2])
  // after the 10 x 4 rows of ports 0/1 in the table
  const int ns = cfg.ns, nsf = 2 * ns;
  const int nsym = port < 2 ? 4 : 2;
  const c32 *pil = (const c32 *)(port < 2 ? crs + (size_t)t.sf_idx * 4 * np : crs + (size_t)(40 + 2 * t.sf_idx) * np);
  const int sym[4] = {port < 2 ? 0 : 1, port < 2 ? ns - 3 : ns + 1, ns, 2 * ns - 3};
  const int tid = threadIdx.x;
  // v = 0 / 3 alternating over the CRS symbols, ports 1 / 3 starting at 3 (refsignal_dl.c:40-74)
  auto fidx = [&](int l) { return (((l & 1) ^ (port & 1) ? 3 : 0) + cell_id % 6) % 6; };
  // 1. LS: fidx = (v + id % 6) % 6. Every load of the thread (at most 4 pilots: 4 np <= 880 <
  //    4 x 256) issued before the first product: one memory round trip instead of four in a row
  {
    constexpr int PPT = (4 * CH_MAXP + 255) / 256;
    c32 g[PPT], c[PPT];
#pragma unroll
    for (int u = 0; u < PPT; u++) {
      const int e = tid + 256 * u;
      if (e < nsym * np) {
        const int l = e / np, m = e % np;
        g[u] = grid[sym[l] * nsc + fidx(l) + 6 * m];
        c[u] = pil[e];
      }
    }
#pragma unroll
    for (int u = 0; u < PPT; u++) {
      const int e = tid + 256 * u;
      if (e < nsym * np) ls[e] = cmulconj(g[u], c[u]);
    }
  }
  // the CFO of ports 2 / 3 (chest_estimate_cfo, chest_dl.c:583-603) reads rows 2 and 3 of the
  // shared pilot buffer, which still hold port 1's estimates of symbols 7 and 11 for this rx
  // antenna (estimate_multi runs the ports in order): they are recomputed into ls rows 2-3
  if (nsym == 2 && t.cfo) {
    const c32 *pil01 = (const c32 *)(crs + (size_t)t.sf_idx * 4 * np);
    for (int e = 2 * np + tid; e < 4 * np; e += blockDim.x) {
      const int l = e / np, m = e % np;
      const int f1 = (((l & 1) ^ 1 ? 3 : 0) + cell_id % 6) % 6; // port 1
      ls[e] = cmulconj(grid[(l == 2 ? ns : 2 * ns - 3) * nsc + f1 + 6 * m], pil01[e]);
    }
  }
  __syncthreads();
  // 2 + 3. block sums: REFS residual power, RSRP, RSSI, sum of estimates, CFO correlation
  const bool refs = cfg.noise_alg == 0 && (t.noise || cfg.filt_auto);
  if (refs || t.meas) {
    float v[CH_NRED] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (refs) { // residual of the last CRS symbol against its staggered neighbours: 4 symbols,
                // ls[2] and the extrapolated 2 ls[2] - ls[0]; 2 symbols, ls[0] on both sides
                // (chest_dl.c:285-299); power / nsymbols * sqrt(5)
      const int off = fidx(0) < 3 ? 0 : 1; // ((fidx < 3) ^ (nsymbols & 1)) ? 0 : 1
      const c32 *r0 = ls, *rp = ls + (nsym - 2) * np, *rl = ls + (nsym - 1) * np;
      for (int k = tid; k < np; k += blockDim.x) {
        c32 tmp = rl[k];
        for (int nb = 0; nb < 2; nb++) {
          auto row = [&](int q) -> c32 {
            return nb == 0 || nsym == 2 ? rp[q] : csub(cscale(rp[q], 2.0f), r0[q]);
          };
          if (k >= off) tmp = cadd(tmp, row(k - off));            // tmp[off + t] += prev[t]
          if (k < np + off - 1) tmp = cadd(tmp, row(1 - off + k)); // tmp[t] += prev[1 - off + t]
          if (off && k == 0) tmp = cadd(tmp, csub(cscale(row(0), 2.0f), row(1)));
          if (!off && k == np - 1) tmp = cadd(tmp, csub(cscale(row(np - 2), 2.0f), row(np - 1)));
        }
        tmp = cscale(tmp, 1.0f / 5.0f);
        v[0] += cpow(csub(rl[k], tmp));
      }
    }
    if (t.meas) {
      for (int e = tid; e < nsym * np; e += blockDim.x) {
        const int l = e / np, m = e % np;
        v[1] += cpow(grid[sym[l] * nsc + fidx(l) + 6 * m]); // pilot_recv_signal power
        v[3] += ls[e].x;
        v[4] += ls[e].y;
      }
      for (int e = tid; e < nsym * nsc; e += blockDim.x) v[2] += cpow(grid[sym[e / nsc] * nsc + e % nsc]);
      for (int e = tid; e < 2 * np; e += blockDim.x) { // slot 0 against slot 1, per CRS symbol
        const c32 p = cmulconj(ls[e], ls[e + 2 * np]);
        v[5] += p.x;
        v[6] += p.y;
      }
    }
    block_sum<CH_NRED>(red, v);
    if (tid == 0) {
      if (refs) {
        s_noise = red[0][0] / (float)np / (float)nsym * sqrtf(5.0f);
        if (t.noise && part == 0) *t.noise = s_noise;
      }
      if (t.meas) {
        const float npil = (float)(nsym * np);
        t.meas[0] = red[1][0] / npil;
        t.meas[1] = red[2][0] / (float)nsym;
        if (cfg.rsrp_neighbour) {
          const double e = hypot((double)(red[3][0] / npil), (double)(red[4][0] / npil));
          t.meas[2] = (float)(e * e);
        }
        if (t.cfo) {
          const float a = -atan2f(red[6][0], red[5][0]) * cfg.cfo_n / ((float)ns * (cfg.cfo_n + cfg.cfo_ng)) / 2;
          t.meas[3] = (float)((double)a / M_PI);
        }
      }
    }
  }
  // 4. filter taps
  if (tid == 0) {
    if (cfg.noise_alg != 0) s_noise = t.noise ? *t.noise : 0.f;
    if (cfg.filt_auto) { // srslte_chest_dl_set_smooth_filter_gauss(q, 4, noise * 200)
      const float sd = s_noise * 200.0f;
      float norm = 0.f;
      for (int i = 0; i < 5; i++) {
        fs[i] = expf(-powf((float)(i - 2), 2) / (2.0f * powf(sd, 2)));
        norm += fs[i];
      }
      const float inv = 1.0f / norm;
      for (int i = 0; i < 5; i++) fs[i] *= inv;
    } else {
      for (int i = 0; i < cfg.flen; i++) fs[i] = filt[i];
    }
  }
  __syncthreads();
  const int fl = cfg.filt_auto ? 5 : cfg.flen;
  // 5. averaging / smoothing; rows: what the frequency interpolation reads
  const c32 *rows = ls;
  if (cfg.average) {
    if (fl) { // average_pilots: interleave the slot pairs, scale 2 / nsymbols, then smooth the 2np row
      const int a = fidx(0) < 3 ? 0 : 1, b = 1 - a;
      for (int m = tid; m < np; m += blockDim.x) {
        if (nsym == 4) {
          sm[2 * m] = cscale(cadd(ls[a * np + m], ls[(a + 2) * np + m]), 0.5f);
          sm[2 * m + 1] = cscale(cadd(ls[b * np + m], ls[(b + 2) * np + m]), 0.5f);
        } else {
          sm[2 * m] = ls[a * np + m]; // x (2 / 2)
          sm[2 * m + 1] = ls[b * np + m];
        }
      }
      __syncthreads();
      for (int i = tid; i < 2 * np; i += blockDim.x) ls[i] = conv_same_at(sm, 2 * np, i, fs, fl);
      __syncthreads();
    } // no smoothing: the raw buffer (symbols 0 and 4 back to back) is interpolated as the row
  } else if (fl) {
    for (int e = tid; e < nsym * np; e += blockDim.x) {
      const int l = e / np;
      sm[e] = conv_same_at(ls + l * np, np, e - l * np, fs, fl);
    }
    __syncthreads();
    rows = sm;
  }
  // 6 + 7. per subcarrier column: frequency interpolation, then time
  c32 *ce = (c32 *)t.ce;
  const bool pss_on = nz05 && cfg.noise_alg == 1;
  const int k0 = nsc / 2 - 31; // srslte_pss_get_slot position within symbol ns - 1
  float pacc = 0.f;
  for (int k = kb + tid; k < ke; k += blockDim.x) {
    c32 c6;
    if (cfg.average) {
      const c32 v = interp_at(rows, 2 * np, k, cell_id % 3, 3, 1.0f / 3);
      if (cfg.rows)
        ce[k] = v;
      else
        for (int s = 0; s < nsf; s++) ce[s * nsc + k] = v;
      c6 = v;
    } else if (nsym == 2 && ns == 7) { // ports 2 / 3 (chest_dl.c:428-430): symbol 0 extrapolated back from 1 with
                            // (c1 - c8) / 7; 2-7 forward from 1 with (c8 - c1) / 7; 9-13 forward from
                            // symbol 1 again (the reference's in0 for that segment), i.e. 2-6 repeated
      const c32 f0 = interp_at(rows, np, k, fidx(0), 6, 1.0f / 6), f1 = interp_at(rows + np, np, k, fidx(1), 6, 1.0f / 6);
      c32 col[14];
      col[1] = f0;
      col[8] = f1;
      col[0] = cadd(f0, cscale(csub(f0, f1), 1.0f / 7.0f));
      const c32 d = cscale(csub(f1, f0), 1.0f / 7.0f);
      col[2] = cadd(f0, d);
      for (int s = 3; s < 8; s++) col[s] = cadd(col[s - 1], d);
      for (int s = 9; s < 14; s++) col[s] = col[s - 7];
      for (int s = 0; s < 14; s++) ce[s * nsc + k] = col[s];
      c6 = col[6];
    } else if (nsym == 2) { // extended CP (chest_dl.c:439-441): 1 and 7, M = 6; 8-11 repeat 2-5
      const c32 f0 = interp_at(rows, np, k, fidx(0), 6, 1.0f / 6), f1 = interp_at(rows + np, np, k, fidx(1), 6, 1.0f / 6);
      c32 col[12];
      col[1] = f0;
      col[7] = f1;
      col[0] = cadd(f0, cscale(csub(f0, f1), 1.0f / 6.0f));
      const c32 d = cscale(csub(f1, f0), 1.0f / 6.0f);
      col[2] = cadd(f0, d);
      for (int s = 3; s < 7; s++) col[s] = cadd(col[s - 1], d);
      for (int s = 8; s < 12; s++) col[s] = col[s - 6];
      for (int s = 0; s < 12; s++) ce[s * nsc + k] = col[s];
      c6 = col[5];
    } else if (ns == 6) { // extended CP, ports 0/1 (chest_dl.c:434-437): 0 / 3 / 6 / 9, M = 3, 10-11
                          // extrapolated from 9
      c32 f[4];
      for (int l = 0; l < 4; l++) f[l] = interp_at(rows + l * np, np, k, fidx(l), 6, 1.0f / 6);
      c32 col[12];
      for (int l = 0; l < 4; l++) col[3 * l] = f[l];
      for (int l = 0; l < 4; l++) {
        const c32 d = cscale(csub(f[l < 3 ? l + 1 : 3], f[l < 3 ? l : 2]), 1.0f / 3.0f);
        col[3 * l + 1] = cadd(f[l], d);
        col[3 * l + 2] = cadd(col[3 * l + 1], d);
      }
      for (int s = 0; s < 12; s++) ce[s * nsc + k] = col[s];
      c6 = col[5];
    } else {
      c32 f[4];
      for (int l = 0; l < 4; l++) f[l] = interp_at(rows + l * np, np, k, fidx(l), 6, 1.0f / 6);
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
      if (cfg.rows) // the reader interpolates in time with these same operations (pdsch ce_at)
        for (int l = 0; l < 4; l++) ce[l * nsc + k] = f[l];
      else
        for (int s = 0; s < 14; s++) ce[s * nsc + k] = col[s];
      c6 = col[6];
    }
    if (pss_on && k >= k0 && k < k0 + 62) // estimate_noise_pss: ce * PSS - received
      pacc += cpow(csub(cmul(c6, ((const c32 *)pss)[k - k0]), grid[(ns - 1) * nsc + k]));
  }
  // 8. PSS / EMPTY noise, subframes 0 and 5 only (otherwise the value is left as it was)
  if (pss_on) {
    block_sum<1>(red, &pacc);
    if (tid == 0) *t.noise = (float)((double)((float)cfg.nof_ports * (red[0][0] / 62.0f)) / sqrt(2.0));
  } else if (nz05 && tid == 0) { // estimate_noise_empty_sc: 5 empty subcarriers either side of SSS / PSS
    float np_ = 0.f;
    for (int s = ns - 2; s <= ns - 1; s++) {
      const int kk = s * nsc + k0;
      for (int side = 0; side < 2; side++) {
        const c32 *x = grid + (side ? kk + 62 : kk - 5);
        float acc = 0.f;
        for (int i = 0; i < 5; i++) acc += cpow(x[i]);
        np_ += acc / 5.0f;
      }
    }
    *t.noise = np_;
  }
}

hipError_t launch_chest(const ChestItem *d_items, int n, const ChestCfg &cfg, const float2 *crs,
                        const float *filt, const float2 *pss, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  // columns split over up to 2 workgroups per grid (12 nprb / 256 of them), each repeating steps 1-5:
  // 19.3 us per 512 20 MHz grids against 25.4 us with 4 (profiles/r04_s16_kb_parts*.json, compact
  // rows). SRSGPU_CHEST_PARTS overrides the cap (A/B)
  static const int cap = [] {
    const char *e = getenv("SRSGPU_CHEST_PARTS");
    const int v = e ? atoi(e) : 0;
    return v >= 1 && v <= 16 ? v : 2;
  }();
  const unsigned parts = (unsigned)std::max(1, std::min(cap, std::max(1, 12 * cfg.nprb / 256)));
  hipLaunchKernelGGL(k_chest, dim3((unsigned)n, parts), dim3(256), 0, st, d_items, n, cfg, crs, filt, pss);
  return hipGetLastError();
}

// srslte_refsignal_cs_put_sf (refsignal_dl.c:338-360): the CRS of a port into its grid plane at
// symbols 0/4/7/11 (ports 0/1) or 1/8 (ports 2/3) (extended CP: 0/3/6/9 or 1/7), subcarriers fidx + 6m
__global__ __launch_bounds__(256) void k_crs_put(const ChestItem *__restrict__ items, int nitems, int nprb,
                                                 int cell_id, int ns, const float2 *__restrict__ crs) {
  const int it = blockIdx.x;
  if (it >= nitems) return;
  const ChestItem t = items[it];
  const int np = 2 * nprb, nsc = 12 * nprb, port = (int)t.port, nsym = port < 2 ? 4 : 2;
  const int sym[4] = {port < 2 ? 0 : 1, port < 2 ? ns - 3 : ns + 1, ns, 2 * ns - 3};
  const float2 *pil = port < 2 ? crs + (size_t)t.sf_idx * 4 * np : crs + (size_t)(40 + 2 * t.sf_idx) * np;
  float2 *g = t.ce; // the grid plane written
  for (int e = threadIdx.x; e < nsym * np; e += blockDim.x) {
    const int l = e / np, m = e % np;
    const int f = (((l & 1) ^ (port & 1) ? 3 : 0) + cell_id % 6) % 6;
    g[sym[l] * nsc + f + 6 * m] = pil[l * np + m];
  }
}

hipError_t launch_crs_put(const ChestItem *d_items, int n, int nprb, int cell_id, int ns, const float2 *crs,
                          hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_crs_put, dim3((unsigned)n), dim3(256), 0, st, d_items, n, nprb, cell_id, ns, crs);
  return hipGetLastError();
}

} // namespace srsgpu
