// TM3 / TM4 feedback from channel estimates (srsgpu_pdsch_feedback_dev, include/srsgpu/pdsch_batch.h):
// the condition number of srslte_precoding_cn and the PMI / SINR of srslte_precoding_pmi_select
// (reference lib/src/phy/mimo/precoding.c:2335-2930), then srslte_ue_dl_ri_select /
// srslte_ue_dl_ri_pmi_select's choice (lib/src/phy/ue/ue_dl.c:684-764).
//
// One wavefront per subframe. The reference's sums are serial float accumulations over a few hundred
// sampled estimates, so each is one lane's loop in the reference's order: lanes 0-3 the one-layer
// codebooks, lanes 4-5 the two-layer ones, lane 6 the condition number. Lane 0 then picks rank and
// PMI. The complex products restate the AVX macros with LV_HAVE_FMA (simd.h:64-91): PROD(a, b) =
// fmaddsub(a, ldup(b), swap(a) * hdup(b)), PROD_ADD / PROD_SUB with the inner fmaddsub / fmsubadd.
#include <hip/hip_runtime.h>
#include <math.h>

#include "feedback_kernels.h"

namespace srsgpu {

namespace {

struct c32 {
  float r, i;
};

__device__ __forceinline__ c32 ld(const float2 *p, uint32_t k) {
  if (!p) return {0.f, 0.f}; // an rx antenna the cell lacks: the reference's zeroed ce_m buffer
  const float2 v = p[k];
  return {v.x, v.y};
}
__device__ __forceinline__ c32 cj(c32 a) { return {a.r, -a.i}; }
__device__ __forceinline__ c32 mulj(c32 a) { return {-a.i, a.r}; } // _MM256_MULJ_PS: j * a
__device__ __forceinline__ c32 add(c32 a, c32 b) { return {__fadd_rn(a.r, b.r), __fadd_rn(a.i, b.i)}; }
__device__ __forceinline__ c32 sub(c32 a, c32 b) { return {__fsub_rn(a.r, b.r), __fsub_rn(a.i, b.i)}; }
__device__ __forceinline__ c32 scale(c32 a, float k) { return {__fmul_rn(a.r, k), __fmul_rn(a.i, k)}; }
// _MM256_PROD_PS (FMA form): re = a.r b.r - (a.i b.i), im = a.i b.r + (a.r b.i), outer op fused
__device__ __forceinline__ c32 prod(c32 a, c32 b) {
  return {fmaf(a.r, b.r, -__fmul_rn(a.i, b.i)), fmaf(a.i, b.r, __fmul_rn(a.r, b.i))};
}
// _MM256_PROD_ADD_PS: a b + c with both halves fused
__device__ __forceinline__ c32 prod_add(c32 a, c32 b, c32 c) {
  const float ur = fmaf(a.i, b.i, -c.r), ui = fmaf(a.r, b.i, c.i);
  return {fmaf(a.r, b.r, -ur), fmaf(a.i, b.r, ui)};
}
// _MM256_PROD_SUB_PS: a b - c
__device__ __forceinline__ c32 prod_sub(c32 a, c32 b, c32 c) {
  const float ur = fmaf(a.i, b.i, c.r), ui = fmaf(a.r, b.i, -c.i);
  return {fmaf(a.r, b.r, -ur), fmaf(a.i, b.r, ui)};
}

constexpr uint32_t kPrec = 24; // PMI_SEL_PRECISION (precoding.c:2145)

// srslte_precoding_pmi_select_1l_avx (precoding.c:2335-2450), codebook cb
__device__ float pmi_1l(const FbItem &t, int cb) {
  float s = 0.f;
  uint32_t count = 0;
  for (uint32_t j = 0; j < t.nof_ce - kPrec * 4 + 1; j += kPrec * 4) {
    float g[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t p = j + kPrec * k;
      const c32 h00 = ld(t.h[0][0], p), h01 = ld(t.h[1][0], p), h10 = ld(t.h[0][1], p), h11 = ld(t.h[1][1], p);
      c32 a0, a1;
      switch (cb) {
      case 0: a0 = add(cj(h00), cj(h01)); a1 = add(cj(h10), cj(h11)); break;
      case 1: a0 = sub(cj(h00), cj(h01)); a1 = sub(cj(h10), cj(h11)); break;
      case 2: a0 = sub(cj(h00), mulj(cj(h01))); a1 = sub(cj(h10), mulj(cj(h11))); break;
      default: a0 = add(cj(h00), mulj(cj(h01))); a1 = add(cj(h10), mulj(cj(h11))); break;
      }
      const c32 b0 = prod_add(a0, h00, prod(a1, h10));
      const c32 b1 = prod_add(a0, h01, prod(a1, h11));
      c32 c;
      switch (cb) {
      case 0: c = add(b0, b1); break;
      case 1: c = sub(b0, b1); break;
      case 2: c = add(b0, mulj(b1)); break;
      default: c = sub(b0, mulj(b1)); break;
      }
      g[k] = __fmul_rn(c.r, 0.5f);
    }
    s = __fadd_rn(s, __fadd_rn(__fadd_rn(__fadd_rn(g[0], g[1]), g[2]), g[3]));
    count += 4;
  }
  return __fdiv_rn(s, __fmul_rn(t.noise, (float)count));
}

// srslte_precoding_pmi_select_2l_avx (precoding.c:2699-2845), codebook cb; _mm256_rcp_ps -> exact 1 / x
__device__ float pmi_2l(const FbItem &t, int cb) {
  float s = 0.f;
  uint32_t count = 0;
  const float n0 = t.noise;
  for (uint32_t j = 0; j < t.nof_ce - kPrec * 4 + 1; j += kPrec * 4) {
    float v[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t p = j + kPrec * k;
      const c32 h00 = ld(t.h[0][0], p), h01 = ld(t.h[1][0], p), h10 = ld(t.h[0][1], p), h11 = ld(t.h[1][1], p);
      c32 a00, a01, a10, a11;
      if (cb == 0) {
        a00 = add(cj(h00), cj(h01));
        a01 = add(cj(h10), cj(h11));
        a10 = sub(cj(h00), cj(h01));
        a11 = sub(cj(h10), cj(h11));
      } else {
        a00 = sub(cj(h00), mulj(cj(h01)));
        a01 = sub(cj(h10), mulj(cj(h11)));
        a10 = add(cj(h00), mulj(cj(h01)));
        a11 = add(cj(h10), mulj(cj(h11)));
      }
      const c32 b00 = prod_add(a00, h00, prod(a01, h10)), b01 = prod_add(a00, h01, prod(a01, h11));
      const c32 b10 = prod_add(a10, h00, prod(a11, h10)), b11 = prod_add(a10, h01, prod(a11, h11));
      c32 c00, c01, c10, c11;
      if (cb == 0) {
        c00 = add(b00, b01);
        c01 = sub(b00, b01);
        c10 = add(b10, b11);
        c11 = sub(b10, b11);
      } else {
        c00 = add(b00, mulj(b01));
        c01 = sub(b00, mulj(b01));
        c10 = add(b10, mulj(b11));
        c11 = sub(b10, mulj(b11));
      }
      c00 = scale(c00, 0.25f);
      c01 = scale(c01, 0.25f);
      c10 = scale(c10, 0.25f);
      c11 = scale(c11, 0.25f);
      c00 = add(c00, {n0, 0.f}); // C += noise * I (avx_noise_estimate: noise in the real lanes)
      c11 = add(c11, {n0, 0.f});
      const c32 det = prod_sub(c00, c11, prod(c01, c10)); // srslte_mat_2x2_det_avx
      // srslte_mat_cf_recip_avx: conj(det) / |det|^2 (the movehdup + moveldup sum), then * (noise, 0)
      const float sq = __fadd_rn(__fmul_rn(det.i, det.i), __fmul_rn(det.r, det.r));
      const float rc = __frcp_rn(sq);
      const c32 inv = {__fmul_rn(n0, __fmul_rn(rc, det.r)), __fmul_rn(0.f, __fmul_rn(rc, -det.i))};
      const c32 den0 = prod(c00, inv), den1 = prod(c11, inv);
      const float g0 = __fsub_rn(__frcp_rn(den0.r), 1.f), g1 = __fsub_rn(__frcp_rn(den1.r), 1.f);
      v[k] = __fadd_rn(g0, g1);
    }
    s = __fadd_rn(s, __fadd_rn(__fadd_rn(__fadd_rn(v[0], v[1]), v[2]), v[3]));
    count += 4;
  }
  return count ? __fdiv_rn(s, (float)count) : s;
}

// srslte_precoding_2x2_cn_gen + srslte_mat_2x2_cn (precoding.c:2889-2912, mat.c:107-127)
__device__ float cn_2x2(const FbItem &t) {
  float acc = 0.f;
  uint32_t count = 0;
  for (uint32_t i = 0; i < t.nof_ce; i += kPrec) {
    const c32 h00 = ld(t.h[0][0], i), h01 = ld(t.h[1][0], i), h10 = ld(t.h[0][1], i), h11 = ld(t.h[1][1], i);
    const float a00 = __fadd_rn(__fadd_rn(__fadd_rn(__fmul_rn(h00.r, h00.r), __fmul_rn(h01.r, h01.r)),
                                          __fmul_rn(h00.i, h00.i)),
                                __fmul_rn(h01.i, h01.i));
    // C99 complex products h00 * conjf(h10) + h01 * conjf(h11), each (ac - bd) + i(ad + bc)
    const float p0r = __fsub_rn(__fmul_rn(h00.r, h10.r), __fmul_rn(h00.i, -h10.i));
    const float p0i = __fadd_rn(__fmul_rn(h00.r, -h10.i), __fmul_rn(h00.i, h10.r));
    const float p1r = __fsub_rn(__fmul_rn(h01.r, h11.r), __fmul_rn(h01.i, -h11.i));
    const float p1i = __fadd_rn(__fmul_rn(h01.r, -h11.i), __fmul_rn(h01.i, h11.r));
    const float a01r = __fadd_rn(p0r, p1r), a01i = __fadd_rn(p0i, p1i);
    const float a11 = __fadd_rn(__fadd_rn(__fadd_rn(__fmul_rn(h10.r, h10.r), __fmul_rn(h11.r, h11.r)),
                                          __fmul_rn(h10.i, h10.i)),
                                __fmul_rn(h11.i, h11.i));
    const float b = __fadd_rn(a00, a11);
    const float c = __fsub_rn(__fmul_rn(a00, a11), __fadd_rn(__fmul_rn(a01r, a01r), __fmul_rn(a01i, a01i)));
    const float sqr = sqrtf(__fsub_rn(__fmul_rn(b, b), __fmul_rn(4.0f, c)));
    const float xmax = __fadd_rn(b, sqr), xmin = __fsub_rn(b, sqr);
    acc = __fadd_rn(acc, __fmul_rn(10.f, log10f(__fdiv_rn(xmax, xmin))));
    count++;
  }
  return count ? __fdiv_rn(acc, (float)count) : acc;
}

__global__ __launch_bounds__(64) void k_feedback(const FbItem *__restrict__ items, int n) {
  const int b = blockIdx.x, l = threadIdx.x;
  if (b >= n) return;
  FbItem t = items[b];
  if (t.noise_dev) t.noise = *t.noise_dev;
  __shared__ float sinr[2][4];
  __shared__ float cn;
  const bool do_pmi = (t.flags & 2u) && t.nports == 2;
  const bool do_cn = (t.flags & 1u) && t.nports == 2 && t.nrx == 2;
  if (l < 4) sinr[0][l] = do_pmi ? pmi_1l(t, l) : 0.f;
  if (l >= 4 && l < 8) {
    const int cb = l - 4;
    // srslte_pdsch_pmi_select (pdsch.c:1014-1034): 2 layers only with 2 rx antennas, -inf above
    sinr[1][cb] = !do_pmi ? 0.f : t.nrx < 2 ? -INFINITY : cb < 2 ? pmi_2l(t, cb) : 0.f;
  }
  if (l == 8) cn = do_cn ? cn_2x2(t) : 0.f;
  __syncthreads();
  if (l != 0) return;
  FbOut o;
  o.cn = cn;
  o.ri_tm3 = do_cn ? (cn < 17.0f ? 1u : 0u) : 0u;
  o.ret_cn = do_cn ? 0 : -1;
  uint32_t pmi_l[2] = {0, 0};
  for (int L = 0; L < 2; L++) { // max_sinr = 0, strict > (precoding.c:2441-2444, :2836-2839)
    float mx = 0.f;
    for (int c = 0; c < (L ? 2 : 4); c++)
      if (sinr[L][c] > mx) {
        mx = sinr[L][c];
        pmi_l[L] = (uint32_t)c;
      }
  }
  // ue_dl.c:698-707: layers 1 .. SRSLTE_MAX_LAYERS, the ones above 2 (and above nrx) at -inf; the
  // comparisons in double as the C expression promotes them
  float best = -INFINITY;
  uint32_t best_ri = 0, best_pmi = 0;
  if (do_pmi) {
    for (uint32_t L = 1; L <= 4; L++) {
      const float s = L <= 2 ? sinr[L - 1][pmi_l[L - 1]] : -INFINITY;
      const float v = __fmul_rn(__fmul_rn(s, (float)L), (float)L);
      if ((double)v > (double)best + 0.1 || (double)v > 1.0e+3) {
        best = v;
        best_pmi = L <= 2 ? pmi_l[L - 1] : 0;
        best_ri = L - 1;
      }
    }
  }
  o.ri = best_ri;
  o.pmi = best_pmi;
  o.pmi_l[0] = pmi_l[0];
  o.pmi_l[1] = pmi_l[1];
  o.ret_pmi = do_pmi ? 0 : -1;
  for (int L = 0; L < 2; L++)
    for (int c = 0; c < 4; c++) o.sinr[L][c] = sinr[L][c];
  *t.out = o;
}

} // namespace

hipError_t launch_feedback(const FbItem *d_items, int n, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_feedback, dim3(n), dim3(64), 0, st, d_items, n);
  return hipGetLastError();
}

} // namespace srsgpu
