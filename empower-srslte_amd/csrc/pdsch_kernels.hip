// MI355X PDSCH receive kernels between the channel estimate and the DL-SCH decoder (paths
// relative to /root/reference/lib), fused into one pass per resource element (RE):
//   gather      srslte_pdsch_get (src/phy/phch/pdsch.c:95-234): RE j of the codeword reads grid
//               position map[j] of the received grid and of the channel estimate (the map is
//               built on the host for each (cell, grant, lstart, sf_idx) class)
//   equalise    SISO ZF/MMSE srslte_predecoding_single_multi (src/phy/mimo/precoding.c:154-352):
//               x = y conj(h) / (|h|^2 + n0) * (1/scaling), summed over 1-2 rx antennas, with the
//               reference's operation order and no FMA contraction, so x is the reference's float
//               (CSI mode: csi = |h|^2 + n0, x = y conj(h) (1/scaling) / csi);
//               TM3 CDD 2x2 MMSE srslte_predecoding_ccd_mmse (precoding.c:930-1097) in the
//               order of srslte_mat_2x2_mmse_csi_gen (utils/mat.c:63-98), exact reciprocals
//   demap       srslte_demod_soft_demodulate_s (src/phy/modem/demod_soft.c): the SSE/AVX2
//               integer path (round-to-nearest, saturating pack, integer offsets) for REs inside
//               the reference's SIMD blocks and its scalar C tail for the rest
//   descramble  srslte_scrambling_s_offset with the PDSCH Gold sequence (scrambling.c:48-51,
//               sequence.c:51-80): LLR negated where c(n) = 1
//   CSI         pdsch.c:676-776 csi_correction (second pass, needs the codeword's max CSI)
// The Gold sequence of each codeword is produced by k_gold from two device tables (x1 and the
// 31 x2 basis sequences of unit seeds, packed 32 bits per word): c = x1 ^ XOR_{seed bit i} x2_i,
// since x2 is linear in its seed.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "pdsch_kernels.h"
#include "srsgpu/pdsch_batch.h"
#include "gmem.h"
#include "wave_prio.h"

// The equaliser must round like the reference's separate SSE/AVX multiplies and adds: no FMA
// contraction anywhere in this file (HIP's __fmul_rn is a plain '*').
#pragma clang fp contract(off)

namespace srsgpu {

__device__ __forceinline__ int16_t sat16(int32_t v) {
  return (int16_t)(v > 32767 ? 32767 : v < -32768 ? -32768 : v);
}
__device__ __forceinline__ int16_t wrap16(int32_t v) { return (int16_t)(uint16_t)(uint32_t)v; }
// x86 cvtps_epi32 / cvttps_epi32: NaN and out-of-range give 0x80000000
__device__ __forceinline__ int32_t cvt_rn(float v) {
  if (!(v >= -2147483648.0f && v < 2147483648.0f)) return INT32_MIN;
  return (int32_t)__builtin_rintf(v);
}
__device__ __forceinline__ int32_t cvt_rz(float v) {
  if (!(v >= -2147483648.0f && v < 2147483648.0f)) return INT32_MIN;
  return (int32_t)v;
}
__device__ __forceinline__ int16_t abs16(int16_t v) { return wrap16(v < 0 ? -(int32_t)v : v); }

// ------------------------------------------------------------------ Gold sequence ----
__global__ __launch_bounds__(256) void k_gold(const GoldItem *__restrict__ items, int nitems,
                                              const uint32_t *__restrict__ x1,
                                              const uint32_t *__restrict__ x2b, uint32_t words) {
  const int it = blockIdx.y;
  if (it >= nitems) return;
  const GoldItem g = items[it];
  const uint32_t nw = (g.len + 31) / 32;
  for (uint32_t w = blockIdx.x * 256 + threadIdx.x; w < nw; w += gridDim.x * 256) {
    // bits n = 32w .. 32w+31 of c are bits 1600 + n of x1 ^ x2 (36.211 7.2)
    const uint32_t b = 1600 + 32 * w, q = b / 32, r = b % 32;
    auto word = [&](uint32_t k) {
      uint32_t v = x1[k];
      uint32_t s = g.seed;
      while (s) {
        const int i = __builtin_ctz(s);
        v ^= x2b[(size_t)i * words + k];
        s &= s - 1;
      }
      return v;
    };
    const uint32_t lo = word(q);
    const uint32_t v = r ? (lo >> r) | (word(q + 1) << (32 - r)) : lo;
    g.c[w] = v;
  }
}

// ------------------------------------------------------------------ equalise + demap ----
struct Eq {
  float xr, xi, csi;
};

// One RE's received values and estimates, loaded ahead of the arithmetic (llr_body gathers
// several REs' inputs before computing any of them): y[rx], h[port][rx]; entries the
// configuration does not use are left unset.
struct ReIn {
  float2 y[2];
  float2 h[2][2];
};
// The channel estimate at grid position pos. Compact rows (srsgpu_chest_set_ce_rows): the
// estimator's time interpolation (chest_dl.c:416-421 via srslte_interp_linear_vector, k_chest's
// column loop) redone here in the same operation order, from the frequency-interpolated rows of
// CRS symbols 0 / 4 / 7 / 11: d = (f[l+1] - f[l]) x w, then sequential additions of d (symbols
// 12-13 continue from symbol 11 with the 7-11 step); or the one averaged row. The same floats as
// the full estimate grid.
__device__ __forceinline__ float2 ce_at(const LlrItem &t, const float2 *h, uint32_t pos) {
  h = gmem(h); // descriptor pointers: global accesses, not flat (gmem.h)
  if (t.ce_rows == 0) return h[pos];
  const uint32_t s = (uint32_t)(((float)pos + 0.5f) * t.inv_nsc); // exact: pos < 2^15, >= 1/(2 nsc) from an integer
  const uint32_t k = pos - s * t.nsc;
  if (t.ce_rows == 1) return h[k];
  const uint32_t l0 = s < 4 ? 0 : s < 7 ? 1 : 2; // rows l0, l0 + 1 bracket the symbol
  const uint32_t m = s < 4 ? s : s < 7 ? s - 4 : s < 11 ? s - 7 : s - 11;
  const float w = s >= 4 && s < 7 ? 1.0f / 3.0f : 0.25f;
  const float2 a = h[l0 * t.nsc + k], b = h[(l0 + 1) * t.nsc + k];
  const float dx = __fmul_rn(__fsub_rn(b.x, a.x), w), dy = __fmul_rn(__fsub_rn(b.y, a.y), w);
  float2 c = s >= 11 ? b : a;
  for (uint32_t i = 0; i < m; i++) {
    c.x = __fadd_rn(c.x, dx);
    c.y = __fadd_rn(c.y, dy);
  }
  return c;
}

// NRX: the receive antennas when known at compile time (0: t.nrx)
template <int NRX = 0>
__device__ __forceinline__ ReIn load_re(const LlrItem &t, uint32_t pos, bool two_ports) {
  ReIn in;
#pragma unroll
  for (int a = 0; a < 2; a++) {
    if (a == 1 && (NRX ? NRX : t.nrx) < 2) break;
    in.y[a] = gmem(t.y[a])[pos];
    in.h[0][a] = ce_at(t, t.h[0][a], pos);
    if (two_ports) in.h[1][a] = ce_at(t, t.h[1][a], pos);
  }
  return in;
}

template <int NRX = 0>
__device__ __forceinline__ Eq equalise(const LlrItem &t, const ReIn &in, uint32_t j) {
  const int nrx = NRX ? NRX : t.nrx;
  Eq e;
  if (!t.csi_mode && (t.nof_re <= 32 || j >= 16 * (t.nof_re / 16))) { // AVX only above 32 (:330)
    // symbols after the last whole 16 take the reference's C path (precoding.c:231-240), whose
    // conj() is the double one: products and sums in double, rounded into float accumulators,
    // then r / ((hh + n0) * scaling)
    float hh = 0.f, rr = 0.f, ri = 0.f;
    for (int a = 0; a < 2; a++) {
      if (a == 1 && nrx < 2) break;
      const float2 y = in.y[a], h = in.h[0][a];
      const double yr = y.x, yi = y.y, hr = h.x, hi = h.y;
      rr = (float)__dadd_rn((double)rr, __dsub_rn(__dmul_rn(yr, hr), __dmul_rn(yi, -hi)));
      ri = (float)__dadd_rn((double)ri, __dadd_rn(__dmul_rn(yr, -hi), __dmul_rn(yi, hr)));
      hh = (float)__dadd_rn((double)hh, __dadd_rn(__dmul_rn(hr, hr), __dmul_rn(hi, hi)));
    }
    const float d = __fmul_rn(__fadd_rn(hh, t.noise), t.scaling);
    e.csi = d;
    e.xr = __fdiv_rn(rr, d);
    e.xi = __fdiv_rn(ri, d);
    return e;
  }
  float hh = 0.f, rr = 0.f, ri = 0.f;
  for (int a = 0; a < 2; a++) {
    if (a == 1 && nrx < 2) break;
    const float2 y = in.y[a], h = in.h[0][a];
    // |h|^2 as hadd(h*h) (precoding.c:179-187), antenna sums in order
    hh = __fadd_rn(hh, __fadd_rn(__fmul_rn(h.x, h.x), __fmul_rn(h.y, h.y)));
    // y * conj(h) as PROD_AVX (addsub of products, :150): re = yr*hr - yi*(-hi)
    rr = __fadd_rn(rr, __fsub_rn(__fmul_rn(y.x, h.x), __fmul_rn(y.y, -h.y)));
    ri = __fadd_rn(ri, __fadd_rn(__fmul_rn(y.y, h.x), __fmul_rn(y.x, -h.y)));
  }
  if (t.csi_mode) { // precoding.c:256-296
    e.csi = __fadd_rn(hh, t.noise);
    const float ir = __frcp_rn(e.csi);
    e.xr = __fmul_rn(__fmul_rn(rr, t.inv_scaling), ir);
    e.xi = __fmul_rn(__fmul_rn(ri, t.inv_scaling), ir);
  } else {
    const float d = t.noise > 0.f ? __fadd_rn(hh, t.noise) : hh;
    e.csi = d;
    e.xr = __fmul_rn(__fdiv_rn(rr, d), t.inv_scaling);
    e.xi = __fmul_rn(__fdiv_rn(ri, d), t.inv_scaling);
  }
  return e;
}
__device__ __forceinline__ Eq equalise(const LlrItem &t, uint32_t pos, uint32_t j) {
  return equalise(t, load_re(t, pos, false), j);
}

// complex float arithmetic in the order gcc evaluates the reference's cf_t expressions
struct cf {
  float r, i;
};
__device__ __forceinline__ cf c_mul(cf a, cf b) { return {a.r * b.r - a.i * b.i, a.r * b.i + a.i * b.r}; }
__device__ __forceinline__ cf c_add(cf a, cf b) { return {a.r + b.r, a.i + b.i}; }
__device__ __forceinline__ cf c_sub(cf a, cf b) { return {a.r - b.r, a.i - b.i}; }
__device__ __forceinline__ cf c_conj(cf a) { return {a.r, -a.i}; }
__device__ __forceinline__ cf c_neg(cf a) { return {-a.r, -a.i}; }
__device__ __forceinline__ cf c_ld(const float2 *p, uint32_t pos) {
  const float2 v = gmem(p)[pos];
  return {v.x, v.y};
}
__device__ __forceinline__ cf c_of(float2 v) { return {v.x, v.y}; }
__device__ __forceinline__ cf ce_ld(const LlrItem &t, const float2 *h, uint32_t pos) { return c_of(ce_at(t, h, pos)); }

// TM3 large-delay CDD, 2 ports x 2 rx antennas, 2 layers (precoding.c:930-1019): the precoder
// alternates per RE (even: H = [[h00+h10, h00-h10], [h01+h11, h01-h11]] with h[port][rx], odd: the
// columns swap); MMSE row `layer` of B = (H'H + n0 I)^-1 (2/scaling), then x = (B H') y
// (srslte_mat_2x2_mmse_csi_gen, mat.c:63-98) and csi = 1 / Re(B[layer][layer]).
// TM4 spatial multiplexing with two layers (srslte_predecoding_multiplex_2x2_mmse(_csi),
// precoding.c:1331-1542) is the same MMSE with the codebook's fixed precoder: codebook 0
// H = [[h00, h10], [h01, h11]] (norm sqrt 2 / scaling), 1 [[h00+h10, h00-h10], [h01+h11, h01-h11]],
// 2 [[h00+j h10, h00-j h10], [h01+j h11, h01-j h11]] (norm 2 / scaling), j h = (-h.i, h.r) exactly.
__device__ __forceinline__ cf c_mulj(cf a) { return {-a.i, a.r}; }
// both layers' outputs (eq[0] layer 0, eq[1] layer 1) of one RE's 2x2 MMSE: the shared terms once,
// then each row with exactly the operations of the one-layer form
__device__ __forceinline__ void equalise_cdd2(const LlrItem &t, const ReIn &in, uint32_t j, Eq eq[2]) {
  const cf p00 = c_of(in.h[0][0]), p01 = c_of(in.h[0][1]);
  const cf p10 = c_of(in.h[1][0]), p11 = c_of(in.h[1][1]);
  cf h00, h01, h10, h11;
  float norm = 2.0f / t.scaling;
  if (t.mux == 1) { // codebook 0
    h00 = p00;
    h01 = p10;
    h10 = p01;
    h11 = p11;
    norm = 1.41421354f / t.scaling; // (float) M_SQRT2 / scaling
  } else if (t.mux == 3) { // codebook 2
    h00 = c_add(p00, c_mulj(p10));
    h01 = c_sub(p00, c_mulj(p10));
    h10 = c_add(p01, c_mulj(p11));
    h11 = c_sub(p01, c_mulj(p11));
  } else if (t.mux == 2 || (j & 1) == 0) { // codebook 1, or the even CDD REs
    h00 = c_add(p00, p10);
    h10 = c_add(p01, p11);
    h01 = c_sub(p00, p10);
    h11 = c_sub(p01, p11);
  } else {
    h00 = c_sub(p00, p10);
    h10 = c_sub(p01, p11);
    h01 = c_add(p00, p10);
    h11 = c_add(p01, p11);
  }
  const cf _h00 = c_conj(h00), _h01 = c_conj(h01), _h10 = c_conj(h10), _h11 = c_conj(h11);
  cf a00 = c_add(c_mul(_h00, h00), c_mul(_h10, h10));
  a00.r = a00.r + t.noise;
  const cf a01 = c_add(c_mul(_h00, h01), c_mul(_h10, h11));
  const cf a10 = c_add(c_mul(_h01, h00), c_mul(_h11, h10));
  cf a11 = c_add(c_mul(_h01, h01), c_mul(_h11, h11));
  a11.r = a11.r + t.noise;
  const cf det = c_sub(c_mul(a00, a11), c_mul(a01, a10));
  const float m2 = det.r * det.r + det.i * det.i;
  const cf rcp = {det.r / m2, -det.i / m2};
  const cf nrm = {norm * rcp.r, norm * rcp.i};
  const cf y0 = c_of(in.y[0]), y1 = c_of(in.y[1]);
#pragma unroll
  for (int layer = 0; layer < 2; layer++) {
    cf bd, bo; // diagonal and off-diagonal entries of row `layer` of B
    if (layer == 0) {
      bd = c_mul(a11, nrm);          // b00
      bo = c_mul(c_neg(a01), nrm);   // b01
    } else {
      bo = c_mul(c_neg(a10), nrm);   // b10
      bd = c_mul(a00, nrm);          // b11
    }
    // row 0: w00 = b00 _h00 + b01 _h01, w01 = b00 _h10 + b01 _h11
    // row 1: w10 = b10 _h00 + b11 _h01, w11 = b10 _h10 + b11 _h11
    const cf b0 = layer == 0 ? bd : bo, b1 = layer == 0 ? bo : bd;
    const cf wa = c_add(c_mul(b0, _h00), c_mul(b1, _h01));
    const cf wb = c_add(c_mul(b0, _h10), c_mul(b1, _h11));
    const cf x = c_add(c_mul(y0, wa), c_mul(y1, wb));
    eq[layer].xr = x.r;
    eq[layer].xi = x.i;
    eq[layer].csi = 1.0f / bd.r;
  }
}
__device__ __forceinline__ Eq equalise_cdd(const LlrItem &t, const ReIn &in, uint32_t j) {
  Eq eq[2];
  equalise_cdd2(t, in, j, eq);
  const Eq e0 = eq[0], e1 = eq[1];
  return t.layer ? e1 : e0;
}

// TM4 spatial multiplexing with one layer: 2x1 MRC (srslte_predecoding_multiplex_2x1_mrc(_csi),
// precoding.c:1546-1713) in the order of the reference's C loop: h0 / h1 = the codebook's
// combination of the two ports at rx 0 / 1 (0: h0+h1, 1: h0-h1, 2: h0+j h1, 3: h0-j h1),
// hh = norm / (|h0|^2 + |h1|^2) summed left to right, x = (conj(h0) y0 + conj(h1) y1) hh,
// csi = (|h0|^2 + |h1|^2) / norm * (float) M_SQRT1_2, norm = (float) M_SQRT2 / scaling.
__device__ __forceinline__ Eq equalise_mrc(const LlrItem &t, const ReIn &in) {
  const int cb = -t.mux - 1;
  const cf p00 = c_of(in.h[0][0]), p01 = c_of(in.h[0][1]);
  const cf p10 = c_of(in.h[1][0]), p11 = c_of(in.h[1][1]);
  cf h0, h1;
  if (cb == 0) {
    h0 = c_add(p00, p10);
    h1 = c_add(p01, p11);
  } else if (cb == 1) {
    h0 = c_sub(p00, p10);
    h1 = c_sub(p01, p11);
  } else if (cb == 2) {
    h0 = c_add(p00, c_mulj(p10));
    h1 = c_add(p01, c_mulj(p11));
  } else {
    h0 = c_sub(p00, c_mulj(p10));
    h1 = c_sub(p01, c_mulj(p11));
  }
  const float norm = 1.41421354f / t.scaling;
  const float s = h0.r * h0.r + h0.i * h0.i + h1.r * h1.r + h1.i * h1.i;
  const float hh = norm / s;
  const cf y0 = c_of(in.y[0]), y1 = c_of(in.y[1]);
  const cf x = c_add(c_mul(c_conj(h0), y0), c_mul(c_conj(h1), y1));
  Eq e;
  e.xr = x.r * hh;
  e.xi = x.i * hh;
  e.csi = s / norm * 0.707106769f; // (float) M_SQRT1_2
  return e;
}

// TM2 transmit diversity, 2 ports (srslte_predecoding_diversity_multi, precoding.c:670-685, then
// srslte_layerdemap_diversity, layermap.c:143-151): symbol j is x0 (j even) or x1 (j odd) of RE
// pair i = j / 2. Without CSI and above 32 REs the first 4*(n/4) REs take the SSE arithmetic
// (srslte_predecoding_diversity2_sse, :438-543: PROD products, |h|^2 by hadd, x / hh *
// (sqrtf(2) / scaling)); the rest, and every pair with CSI (srslte_predecoding_diversity_csi,
// :569-602), take gcc's evaluation of the C code (:356-428): float complex products, x1's
// terms in double (the double conj()), hh = 1e-4 when 0, x / (hh * scaling) * sqrt(2) in double;
// csi = hh before scaling.
__device__ __forceinline__ Eq equalise_txdiv(const LlrItem &t, uint32_t j) {
  const uint32_t i = j >> 1, p0 = gmem(t.map)[2 * i], p1 = gmem(t.map)[2 * i + 1];
  const bool odd = j & 1;
  Eq e;
  if (!t.csi_mode && t.nof_re > 32 && i < 2 * (t.nof_re / 4)) {
    float hh = 0.f;
    cf x0 = {0.f, 0.f}, x1 = {0.f, 0.f};
    for (int a = 0; a < 2; a++) {
      if (a == 1 && t.nrx < 2) break;
      const cf h00 = ce_ld(t, t.h[0][a], p0), h01 = ce_ld(t, t.h[0][a], p1);
      const cf h10 = ce_ld(t, t.h[1][a], p0), h11 = ce_ld(t, t.h[1][a], p1);
      const cf r0 = c_ld(t.y[a], p0), r1 = c_ld(t.y[a], p1);
      const float g = __fadd_rn(__fadd_rn(__fmul_rn(h00.r, h00.r), __fmul_rn(h00.i, h00.i)),
                                __fadd_rn(__fmul_rn(h11.r, h11.r), __fmul_rn(h11.i, h11.i)));
      hh = a ? __fadd_rn(hh, g) : g;
      const cf u0 = c_add(c_mul(c_conj(h00), r0), c_mul(h11, c_conj(r1)));
      const cf u1 = c_sub(c_mul(c_conj(h01), r1), c_mul(h10, c_conj(r0)));
      x0 = a ? c_add(x0, u0) : u0;
      x1 = a ? c_add(x1, u1) : u1;
    }
    const float s2 = __fdiv_rn(1.41421354f, t.scaling); // sqrtf(2) / scaling
    const cf x = odd ? x1 : x0;
    e.xr = __fmul_rn(__fdiv_rn(x.r, hh), s2);
    e.xi = __fmul_rn(__fdiv_rn(x.i, hh), s2);
    e.csi = hh;
    return e;
  }
  float hh = 0.f;
  cf x0 = {0.f, 0.f}, x1 = {0.f, 0.f};
  for (int a = 0; a < 2; a++) {
    if (a == 1 && t.nrx < 2) break;
    const cf h00 = ce_ld(t, t.h[0][a], p0), h01 = ce_ld(t, t.h[0][a], p1);
    const cf h10 = ce_ld(t, t.h[1][a], p0), h11 = ce_ld(t, t.h[1][a], p1);
    hh = __fadd_rn(hh, __fadd_rn(__fadd_rn(__fadd_rn(__fmul_rn(h00.r, h00.r), __fmul_rn(h00.i, h00.i)),
                                           __fmul_rn(h11.r, h11.r)),
                                 __fmul_rn(h11.i, h11.i)));
    const cf r0 = c_ld(t.y[a], p0), r1 = c_ld(t.y[a], p1);
    if (hh == 0.f) hh = 1e-4f;
    const cf u0 = c_add(c_mul(c_conj(h00), r0), c_mul(h11, c_conj(r1)));
    x0 = c_add(x0, u0);
    // -h10 * conj(r0) + conj(h01) * r1 in double complex
    const double nr = -(double)h10.r, ni = -(double)h10.i, cr = r0.r, ci = -(double)r0.i;
    const double pr = __dsub_rn(__dmul_rn(nr, cr), __dmul_rn(ni, ci));
    const double pi = __dadd_rn(__dmul_rn(nr, ci), __dmul_rn(ni, cr));
    const double gr = h01.r, gi = -(double)h01.i, sr = r1.r, si = r1.i;
    const double qr = __dsub_rn(__dmul_rn(gr, sr), __dmul_rn(gi, si));
    const double qi = __dadd_rn(__dmul_rn(gr, si), __dmul_rn(gi, sr));
    x1.r = (float)__dadd_rn((double)x1.r, __dadd_rn(pr, qr));
    x1.i = (float)__dadd_rn((double)x1.i, __dadd_rn(pi, qi));
  }
  e.csi = hh;
  const float hs = __fmul_rn(hh, t.scaling);
  const cf x = odd ? x1 : x0;
  e.xr = (float)__dmul_rn((double)__fdiv_rn(x.r, hs), 1.4142135623730951);
  e.xi = (float)__dmul_rn((double)__fdiv_rn(x.i, hs), 1.4142135623730951);
  return e;
}

// TM2 transmit diversity, 4 ports (srslte_predecoding_diversity_multi with nof_ports == 4,
// precoding.c:388-423 / 604-662, then srslte_layerdemap_diversity over 4 layers): symbol j is x_k
// (k = j mod 4) of RE quadruplet i = j / 4; x0 / x1 come from ports 0 and 2 on REs 4i, 4i+1 and
// x2 / x3 from ports 1 and 3 on REs 4i+2, 4i+3. Without CSI (the generic C form, no SSE variant
// for 4 ports): the pair's channels read at its first RE, gains summed over rx antennas with no
// zero guard, float complex products, x / (hh scaling) * sqrt(2) in double. With CSI: per-symbol
// gains (x0: h[p][4i] and h[p+2][4i+1]; x1: h[p][4i+1] and h[p+2][4i]), csi = a scaling / nof_rx,
// x / (a scaling) * sqrtf(2) in float. The host refuses nof_re % 4 != 0 (the reference leaves
// those symbols to whatever its buffer held).
__device__ __forceinline__ Eq equalise_txdiv4(const LlrItem &t, uint32_t j) {
  const uint32_t k = j & 3, q = k >> 1, b = (j & ~3u) + 2 * q;
  const uint32_t p0 = gmem(t.map)[b], p1 = gmem(t.map)[b + 1];
  const bool odd = k & 1;
  cf x = {0.f, 0.f};
  float g = 0.f;
  Eq e;
#pragma unroll
  for (int a = 0; a < 2; a++) { // unrolled: a run-time a would index the descriptor in scratch
    if (a == 1 && t.nrx < 2) break;
    const cf r0 = c_ld(t.y[a], p0), r1 = c_ld(t.y[a], p1);
    // the pair's planes by select, not by a run-time index into the descriptor (which would put the
    // whole item in scratch memory)
    const float2 *hq = q ? t.h[1][a] : t.h[0][a], *hq2 = q ? t.h[3][a] : t.h[2][a];
    const cf hA = ce_ld(t, hq, p0), hB = ce_ld(t, hq2, t.csi_mode && !odd ? p1 : p0);
    cf u;
    if (!t.csi_mode) { // hA = h[q][4i+2q], hB = h[q+2][4i+2q]
      g = __fadd_rn(g, __fadd_rn(__fadd_rn(__fadd_rn(__fmul_rn(hA.r, hA.r), __fmul_rn(hA.i, hA.i)),
                                           __fmul_rn(hB.r, hB.r)),
                                 __fmul_rn(hB.i, hB.i)));
      u = odd ? c_add(c_mul(c_neg(hB), c_conj(r0)), c_mul(c_conj(hA), r1))
              : c_add(c_mul(c_conj(hA), r0), c_mul(hB, c_conj(r1)));
    } else if (!odd) { // h00 = h[q][b] (hA), h11 = h[q+2][b+1] (hB)
      g = __fadd_rn(g, __fadd_rn(__fadd_rn(__fadd_rn(__fmul_rn(hA.r, hA.r), __fmul_rn(hA.i, hA.i)),
                                           __fmul_rn(hB.r, hB.r)),
                                 __fmul_rn(hB.i, hB.i)));
      u = c_add(c_mul(c_conj(hA), r0), c_mul(hB, c_conj(r1)));
    } else { // h10 = h[q][b+1], h01 = h[q+2][b] (hB)
      const cf h10 = ce_ld(t, hq, p1);
      g = __fadd_rn(g, __fadd_rn(__fadd_rn(__fadd_rn(__fmul_rn(h10.r, h10.r), __fmul_rn(h10.i, h10.i)),
                                           __fmul_rn(hB.r, hB.r)),
                                 __fmul_rn(hB.i, hB.i)));
      u = c_add(c_mul(c_neg(hB), c_conj(r0)), c_mul(c_conj(h10), r1));
    }
    x = c_add(x, u);
  }
  const float gs = __fmul_rn(g, t.scaling);
  if (t.csi_mode) {
    e.csi = __fdiv_rn(gs, (float)t.nrx);
    e.xr = __fmul_rn(__fdiv_rn(x.r, gs), 1.41421354f);
    e.xi = __fmul_rn(__fdiv_rn(x.i, gs), 1.41421354f);
  } else {
    e.csi = g;
    e.xr = (float)__dmul_rn((double)__fdiv_rn(x.r, gs), 1.4142135623730951);
    e.xi = (float)__dmul_rn((double)__fdiv_rn(x.i, gs), 1.4142135623730951);
  }
  return e;
}

// LLRs of symbol j (q per symbol) into out[0..q)
__device__ __forceinline__ void demap(int mod, uint32_t j, uint32_t n, float xr, float xi,
                                      int16_t *o) {
  switch (mod) {
  case 0: // BPSK demod_bpsk_lte_s (demod_soft.c:56-60)
    o[0] = (int16_t)(int32_t)((double)(-100.0f * (xr + xi)) / 1.4142135623730951);
    break;
  case 1: { // QPSK srslte_vec_convert_fi(-100 sqrt 2): 16-float SIMD blocks, C tail
    const float sc = -141.42135623730951f;
    const bool simd = 2 * j + 1 < 16 * ((2 * n) / 16);
    const float a = __fmul_rn(xr, sc), b = __fmul_rn(xi, sc);
    o[0] = simd ? sat16(cvt_rz(a)) : wrap16(cvt_rz(a));
    o[1] = simd ? sat16(cvt_rz(b)) : wrap16(cvt_rz(b));
    break;
  }
  case 2: { // 16QAM demod_16qam_lte_s_sse (:96-155)
    if (j < 4 * (n / 4)) {
      const int16_t re = sat16(cvt_rn(__fmul_rn(xr, -400.f)));
      const int16_t im = sat16(cvt_rn(__fmul_rn(xi, -400.f)));
      o[0] = re;
      o[1] = im;
      o[2] = wrap16(abs16(re) - 252);
      o[3] = wrap16(abs16(im) - 252);
    } else {
      const int16_t yre = wrap16(cvt_rz(__fmul_rn(400.f, xr)));
      const int16_t yim = wrap16(cvt_rz(__fmul_rn(400.f, xi)));
      o[0] = wrap16(-(int32_t)yre);
      o[1] = wrap16(-(int32_t)yim);
      o[2] = wrap16((int32_t)((double)abs(yre) - 252.98221281347036));
      o[3] = wrap16((int32_t)((double)abs(yim) - 252.98221281347036));
    }
    break;
  }
  default: { // 64QAM demod_64qam_lte_s_sse (:242-304)
    if (j < 4 * (n / 4)) {
      const int16_t re = sat16(cvt_rn(__fmul_rn(xr, -700.f)));
      const int16_t im = sat16(cvt_rn(__fmul_rn(xi, -700.f)));
      const int16_t a1r = wrap16(abs16(re) - 432), a1i = wrap16(abs16(im) - 432);
      o[0] = re;
      o[1] = im;
      o[2] = a1r;
      o[3] = a1i;
      o[4] = wrap16(abs16(a1r) - 216);
      o[5] = wrap16(abs16(a1i) - 216);
    } else {
      const float yre = (float)wrap16(cvt_rz(__fmul_rn(700.f, xr)));
      const float yim = (float)wrap16(cvt_rz(__fmul_rn(700.f, xi)));
      o[0] = wrap16((int32_t)-yre);
      o[1] = wrap16((int32_t)-yim);
      o[2] = wrap16((int32_t)((double)abs((int)yre) - 432.04937989385187));
      o[3] = wrap16((int32_t)((double)abs((int)yim) - 432.04937989385187));
      o[4] = wrap16((int32_t)((double)abs((int)o[2]) - 216.02468994692594));
      o[5] = wrap16((int32_t)((double)abs((int)o[3]) - 216.02468994692594));
    }
  }
  }
}

// int8 LLRs of symbol j: srslte_demod_soft_demodulate_b (demod_soft.c:458-477). SIMD blocks of 8
// symbols: QPSK srslte_vec_convert_fb (vector_simd.c:433-462: cvttps, packs_epi32, packs_epi16 =
// truncate and saturate), 16/64QAM demod_*_lte_b_sse (:138-191, :306-372: cvtps nearest-even, both
// packs, abs_epi8 and sub_epi8 wrapping with the int8 offsets 18 / 24, 12); C tails: (int8_t)
// conversions (truncate, low byte) and the offsets subtracted in double.
__device__ __forceinline__ int16_t sat8(int32_t v) { return (int16_t)(v > 127 ? 127 : v < -128 ? -128 : v); }
__device__ __forceinline__ int16_t wrap8(int32_t v) { return (int16_t)(int8_t)(uint8_t)(uint32_t)v; }
__device__ __forceinline__ int16_t abs8(int16_t v) { return wrap8(v < 0 ? -(int32_t)v : v); }
__device__ __forceinline__ void demap8(int mod, uint32_t j, uint32_t n, float xr, float xi,
                                       int16_t *o) {
  switch (mod) {
  case 0: // BPSK demod_bpsk_lte_b (:49-53)
    o[0] = wrap8((int32_t)((double)(-20.0f * (xr + xi)) / 1.4142135623730951));
    break;
  case 1: { // QPSK srslte_vec_convert_fb(-20 sqrt 2): 16-float SIMD blocks, C tail
    const float sc = -28.284271247461902f;
    const bool simd = 2 * j + 1 < 16 * ((2 * n) / 16);
    const float a = __fmul_rn(xr, sc), b = __fmul_rn(xi, sc);
    o[0] = simd ? sat8(sat16(cvt_rz(a))) : wrap8(cvt_rz(a));
    o[1] = simd ? sat8(sat16(cvt_rz(b))) : wrap8(cvt_rz(b));
    break;
  }
  case 2: { // 16QAM
    if (j < 8 * (n / 8)) {
      const int16_t re = sat8(sat16(cvt_rn(__fmul_rn(xr, -30.f))));
      const int16_t im = sat8(sat16(cvt_rn(__fmul_rn(xi, -30.f))));
      o[0] = re;
      o[1] = im;
      o[2] = wrap8(abs8(re) - 18);
      o[3] = wrap8(abs8(im) - 18);
    } else {
      const int16_t yre = wrap8(cvt_rz(__fmul_rn(30.f, xr)));
      const int16_t yim = wrap8(cvt_rz(__fmul_rn(30.f, xi)));
      o[0] = wrap8(-(int32_t)yre);
      o[1] = wrap8(-(int32_t)yim);
      o[2] = wrap8((int32_t)((double)abs(yre) - 18.973665961010276));
      o[3] = wrap8((int32_t)((double)abs(yim) - 18.973665961010276));
    }
    break;
  }
  default: { // 64QAM
    if (j < 8 * (n / 8)) {
      const int16_t re = sat8(sat16(cvt_rn(__fmul_rn(xr, -40.f))));
      const int16_t im = sat8(sat16(cvt_rn(__fmul_rn(xi, -40.f))));
      const int16_t a1r = wrap8(abs8(re) - 24), a1i = wrap8(abs8(im) - 24);
      o[0] = re;
      o[1] = im;
      o[2] = a1r;
      o[3] = a1i;
      o[4] = wrap8(abs8(a1r) - 12);
      o[5] = wrap8(abs8(a1i) - 12);
    } else {
      const float yre = (float)wrap8(cvt_rz(__fmul_rn(40.f, xr)));
      const float yim = (float)wrap8(cvt_rz(__fmul_rn(40.f, xi)));
      o[0] = wrap8((int32_t)-yre);
      o[1] = wrap8((int32_t)-yim);
      o[2] = wrap8((int32_t)((double)abs((int)yre) - 24.688535993934706));
      o[3] = wrap8((int32_t)((double)abs((int)yim) - 24.688535993934706));
      o[4] = wrap8((int32_t)((double)abs((int)o[2]) - 12.344267996967353));
      o[5] = wrap8((int32_t)((double)abs((int)o[3]) - 12.344267996967353));
    }
  }
  }
}

// demap, descramble and store the LLRs of RE j (and its CSI)
template <int MOD>
__device__ __forceinline__ void llr_out(const LlrItem &t, uint32_t j, const Eq &e, uint32_t c0, uint32_t c1) {
  constexpr int Q = MOD == 0 ? 1 : MOD == 1 ? 2 : MOD == 2 ? 4 : 6;
  int16_t o[Q];
  if (t.llr8)
    demap8(MOD, j, t.nof_re, e.xr, e.xi, o);
  else
    demap(MOD, j, t.nof_re, e.xr, e.xi, o);
  // scrambling bits b0 .. b0+Q-1 (may straddle the two words c0, c1)
  const uint32_t b0 = j * Q, sh = b0 & 31;
  const uint32_t cb = (uint32_t)((((uint64_t)c1 << 32) | c0) >> sh);
#pragma unroll
  for (int k = 0; k < Q; k++)
    if ((cb >> k) & 1) // _mm256_sign_epi16 / _epi8 (scrambling_sb_offset) by c = 1 - 2c
      o[k] = t.llr8 ? wrap8(-(int32_t)o[k]) : wrap16(-(int32_t)o[k]);
  if (Q % 2 == 0 && t.aligned) {
    uint32_t *dst = reinterpret_cast<uint32_t *>(gmem(t.e) + b0);
#pragma unroll
    for (int k = 0; k < Q; k += 2) dst[k / 2] = (uint16_t)o[k] | ((uint32_t)(uint16_t)o[k + 1] << 16);
  } else {
#pragma unroll
    for (int k = 0; k < Q; k++) gmem(t.e)[b0 + k] = o[k];
  }
  if (t.csi_mode) {
    gmem(t.csi)[j] = e.csi;
    atomicMax(gmem(t.csi_max), __float_as_uint(e.csi)); // csi >= 0: uint order == float order
  }
}

// LLR_RES REs per thread (stride gridDim.x * 256): every RE's map entry, then its grid / estimate
// values and scrambling words are loaded before the first one is computed, so a thread waits for
// two round trips per LLR_RES REs instead of per RE (one RE per thread left the kernel at ~1.5 TB/s,
// bound by the dependent map -> grid load chain). TM2 pairs REs across the map and keeps the
// one-RE loop.
// P0: the call's items all equalise port 0 alone (k_pdsch_llr_p0): the other equalisers are not
// compiled in, so the kernel's register budget is the single-port one.
#define LLR_RES 4
// part / nparts: this workgroup's share of the item's REs (the RE loop strides over nparts x 256)
template <int MOD, bool P0 = false, int NRX = 0>
__device__ __forceinline__ void llr_body(const LlrItem &t, uint32_t part, uint32_t nparts) {
  constexpr int Q = MOD == 0 ? 1 : MOD == 1 ? 2 : MOD == 2 ? 4 : 6;
  const uint32_t stride = nparts * 256;
  if (!P0 && t.txdiv) {
    for (uint32_t j = part * 256 + threadIdx.x; j < t.nof_re; j += stride) {
      const uint32_t w = (j * Q) >> 5;
      llr_out<MOD>(t, j, t.txdiv == 4 ? equalise_txdiv4(t, j) : equalise_txdiv(t, j), gmem(t.c)[w],
                   gmem(t.c)[w + 1]);
    }
    return;
  }
  const bool two_ports = !P0 && (t.cdd || t.mux != 0);
  for (uint32_t j0 = part * 256 + threadIdx.x; j0 < t.nof_re; j0 += stride * LLR_RES) {
    uint32_t pos[LLR_RES];
#pragma unroll
    for (int r = 0; r < LLR_RES; r++) {
      const uint32_t j = j0 + r * stride;
      pos[r] = gmem(t.map)[j < t.nof_re ? j : j0];
    }
    ReIn in[LLR_RES];
    uint32_t c0[LLR_RES], c1[LLR_RES];
#pragma unroll
    for (int r = 0; r < LLR_RES; r++) {
      const uint32_t j = j0 + r * stride;
      const uint32_t w = ((j < t.nof_re ? j : j0) * Q) >> 5;
      in[r] = load_re<NRX>(t, pos[r], two_ports);
      c0[r] = gmem(t.c)[w];
      c1[r] = gmem(t.c)[w + 1];
    }
#pragma unroll
    for (int r = 0; r < LLR_RES; r++) {
      const uint32_t j = j0 + r * stride;
      if (j >= t.nof_re) break;
      const Eq e = P0                   ? equalise<NRX>(t, in[r], j)
                   : (t.cdd || t.mux > 0) ? equalise_cdd(t, in[r], j)
                   : t.mux < 0          ? equalise_mrc(t, in[r])
                                        : equalise(t, in[r], j);
      llr_out<MOD>(t, j, e, c0[r], c1[r]);
    }
  }
}

// both layers of a 2-layer MMSE from one solve per RE: t and t2 are the two TBs' items (t2 by
// reference, so it stays in registers)
template <int MOD>
__device__ __forceinline__ void llr_body_dual(const LlrItem &t, const LlrItem &t2) {
  constexpr int Q = MOD == 0 ? 1 : MOD == 1 ? 2 : MOD == 2 ? 4 : 6;
  const uint32_t stride = gridDim.x * 256;
  for (uint32_t j0 = blockIdx.x * 256 + threadIdx.x; j0 < t.nof_re; j0 += stride * LLR_RES) {
    uint32_t pos[LLR_RES];
#pragma unroll
    for (int r = 0; r < LLR_RES; r++) {
      const uint32_t j = j0 + r * stride;
      pos[r] = gmem(t.map)[j < t.nof_re ? j : j0];
    }
    ReIn in[LLR_RES];
    uint32_t c0[LLR_RES], c1[LLR_RES], d0[LLR_RES], d1[LLR_RES];
#pragma unroll
    for (int r = 0; r < LLR_RES; r++) {
      const uint32_t j = j0 + r * stride;
      const uint32_t w = ((j < t.nof_re ? j : j0) * Q) >> 5;
      in[r] = load_re(t, pos[r], true);
      c0[r] = gmem(t.c)[w];
      c1[r] = gmem(t.c)[w + 1];
      d0[r] = gmem(t2.c)[w];
      d1[r] = gmem(t2.c)[w + 1];
    }
#pragma unroll
    for (int r = 0; r < LLR_RES; r++) {
      const uint32_t j = j0 + r * stride;
      if (j >= t.nof_re) break;
      Eq eq[2];
      equalise_cdd2(t, in[r], j, eq);
      const Eq e0 = eq[0], e1 = eq[1];
      llr_out<MOD>(t, j, t.layer ? e1 : e0, c0[r], c1[r]);
      llr_out<MOD>(t2, j, t2.layer ? e1 : e0, d0[r], d1[r]);
    }
  }
}

// the item's device pointers as global, and the noise from the estimator when it is on the device
__device__ __forceinline__ void llr_item_fix(LlrItem &u) {
#pragma unroll
  for (int a = 0; a < 2; a++) {
    u.y[a] = gmem(u.y[a]);
#pragma unroll
    for (int p = 0; p < 4; p++) u.h[p][a] = gmem(u.h[p][a]);
  }
  u.map = gmem(u.map);
  u.c = gmem(u.c);
  u.e = gmem(u.e);
  u.csi = gmem(u.csi);
  u.csi_max = gmem(u.csi_max);
  u.noise_dev = gmem(u.noise_dev);
  if (u.noise_dev) { // srslte_chest_dl_get_noise_estimate (chest_dl.c:741-750): per rx antenna
                     // the mean over ports, then the mean over antennas
    float n = 0.f;
    for (int a = 0; a < u.nrx; a++) {
      float acc = 0.f;
      for (int p = 0; p < u.nports; p++) acc += u.noise_dev[a * u.nports + p];
      n += acc / (float)u.nports;
    }
    u.noise = n / (float)u.nrx;
  }
}

// one item per TB (the dual items are k_pdsch_llr2's)
__global__ __launch_bounds__(256) void k_pdsch_llr(const LlrItem *__restrict__ items, int nitems) {
  const int it = blockIdx.y;
  if (it >= nitems) return;
  LlrItem t = items[it];
  if (t.dual) return;
  llr_item_fix(t);
  switch (t.mod) {
  case 0: llr_body<0>(t, blockIdx.x, gridDim.x); break;
  case 1: llr_body<1>(t, blockIdx.x, gridDim.x); break;
  case 2: llr_body<2>(t, blockIdx.x, gridDim.x); break;
  default: llr_body<3>(t, blockIdx.x, gridDim.x); break;
  }
}

// the same for calls whose items all equalise port 0 alone (SISO / receive diversity on port 0),
// NRX receive antennas
// XCD-aware: a 1-D grid in which an item's nparts workgroups all fall on one XCD (workgroups are dealt
// round-robin over the 8 XCDs, so b and b + 8 share one, MI355X_MICROARCH.md "Workgroup dispatch"):
// workgroup b serves item (b % 8) + 8 ((b / 8) / nparts), part (b / 8) % nparts. The item's estimate
// rows, which every part re-reads for each OFDM symbol, then come from one XCD's L2 instead of up to
// eight.
template <int NRX>
// (xcd = 0: item b / nparts, part b % nparts, for the A/B)
__global__ __launch_bounds__(256) void k_pdsch_llr_p0(const LlrItem *__restrict__ items, int nitems, int nparts,
                                                      int xcd) {
  const uint32_t b = blockIdx.x, idx = xcd ? b >> 3 : b;
  const uint32_t per = idx / (uint32_t)nparts;
  const int it = (int)(xcd ? (b & 7) + 8 * per : per);
  if (it >= nitems) return;
  const uint32_t part = idx - per * (uint32_t)nparts;
  LlrItem t = items[it];
  llr_item_fix(t);
  switch (t.mod) {
  case 0: llr_body<0, true, NRX>(t, part, nparts); break;
  case 1: llr_body<1, true, NRX>(t, part, nparts); break;
  case 2: llr_body<2, true, NRX>(t, part, nparts); break;
  default: llr_body<3, true, NRX>(t, part, nparts); break;
  }
}

// both TBs of a 2-layer MMSE subframe (item it with dual = 1 and item it + 1) from one solve per
// RE; a kernel of its own, so the single-TB kernel keeps its smaller register budget
__global__ __launch_bounds__(256) void k_pdsch_llr2(const LlrItem *__restrict__ items, int nitems) {
  const int it = blockIdx.y;
  if (it + 1 >= nitems) return;
  LlrItem t = items[it];
  if (t.dual != 1) return;
  LlrItem t2 = items[it + 1];
  llr_item_fix(t);
  llr_item_fix(t2);
  switch (t.mod) {
  case 0: llr_body_dual<0>(t, t2); break;
  case 1: llr_body_dual<1>(t, t2); break;
  case 2: llr_body_dual<2>(t, t2); break;
  default: llr_body_dual<3>(t, t2); break;
  }
}

// pdsch.c:676-776 (16-bit path): SIMD part mulhi by cvtps(csi * 32767/csi_max) with the
// reference's lane-to-symbol assignment (QPSK and 64QAM blend the neighbouring symbol's CSI into
// half of each 4-LLR group), scalar tail (int16)(e * (csi / csi_max)).
__global__ __launch_bounds__(256) void k_csi_correct(const LlrItem *__restrict__ items, int nitems) {
  const int it = blockIdx.y;
  if (it >= nitems) return;
  LlrItem t = items[it];
  t.e = gmem(t.e);
  t.csi = gmem(t.csi);
  t.csi_max = gmem(t.csi_max);
  const uint32_t nbits = t.nof_re * t.qm;
  const float cmax = __uint_as_float(*t.csi_max);
  const float scale = __fdiv_rn(32767.f, cmax);
  uint32_t simd_bits = 0; // bits covered by the SIMD loop
  if (t.mod == 1 || t.mod == 2)
    simd_bits = nbits >= 4 ? ((nbits - 4) / 4 + 1) * 4 : 0;
  else if (t.mod == 3)
    simd_bits = nbits >= 12 ? ((nbits - 12) / 12 + 1) * 12 : 0;
  for (uint32_t n = blockIdx.x * 256 + threadIdx.x; n < nbits; n += gridDim.x * 256) {
    int16_t v = t.e[n];
    if (t.llr8) { // pdsch.c:707-713: (int8_t)((float)e * (csi / csi_max)), no SIMD part
      const float c = __fdiv_rn(t.csi[n / t.qm], cmax);
      t.e[n] = wrap8(cvt_rz(__fmul_rn((float)v, c)));
      continue;
    }
    if (n < simd_bits) {
      uint32_t sym;
      if (t.mod == 1) { // 4 LLRs = symbols 2g, 2g+1; lanes 0,1 take csi[2g+1], lanes 2,3 csi[2g]
        const uint32_t g = n / 4, l = n % 4;
        sym = 2 * g + (l < 2 ? 1 : 0);
      } else if (t.mod == 2) {
        sym = n / 4;
      } else { // 12 LLRs = symbols 2g, 2g+1: e0 <- csi[2g], e1 lanes 0,1 <- csi[2g+1], lanes 2,3
               // <- csi[2g], e2 <- csi[2g+1]
        const uint32_t g = n / 12, l = n % 12;
        sym = l < 4 ? 2 * g : l < 6 ? 2 * g + 1 : l < 8 ? 2 * g : 2 * g + 1;
      }
      const int16_t s = sat16(cvt_rn(__fmul_rn(t.csi[sym], scale)));
      v = (int16_t)(((int32_t)v * (int32_t)s) >> 16);
    } else {
      const float c = __fdiv_rn(t.csi[n / t.qm], cmax);
      v = wrap16(cvt_rz(__fmul_rn((float)v, c)));
    }
    t.e[n] = v;
  }
}

static inline unsigned cdiv(size_t n, unsigned b) { return (unsigned)((n + b - 1) / b); }

hipError_t launch_gold(const GoldItem *d_items, int n, uint32_t max_len, const uint32_t *x1,
                       const uint32_t *x2b, uint32_t words, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const unsigned gx = std::min(cdiv(cdiv(max_len, 32), 256), 16u);
  hipLaunchKernelGGL(k_gold, dim3(gx ? gx : 1, (unsigned)n), dim3(256), 0, st, d_items, n, x1, x2b,
                     words);
  return hipGetLastError();
}

hipError_t launch_pdsch_llr(const LlrItem *d_items, int n, uint32_t max_re, bool csi, hipStream_t st,
                            int n_dual, int p0) {
  if (n <= 0) return hipSuccess;
  const unsigned gx = std::min(cdiv(max_re, 256 * LLR_RES), 64u);
  const bool generic = knobs().llr_generic; // A/B: the general kernel only
  if (p0 && !n_dual && !generic) {
    const int xcd = knobs().llr_noxcd ? 0 : 1; // A/B: the plain item-major mapping
    const unsigned parts = gx ? gx : 1, nb = parts * ((unsigned)(n + 7) / 8) * 8; // items rounded up to 8
    if (p0 == 1)
      hipLaunchKernelGGL(k_pdsch_llr_p0<1>, dim3(nb), dim3(256), 0, st, d_items, n, (int)parts, xcd);
    else
      hipLaunchKernelGGL(k_pdsch_llr_p0<2>, dim3(nb), dim3(256), 0, st, d_items, n, (int)parts, xcd);
  } else if (n > 2 * n_dual)
    hipLaunchKernelGGL(k_pdsch_llr, dim3(gx ? gx : 1, (unsigned)n), dim3(256), 0, st, d_items, n);
  if (n_dual > 0)
    hipLaunchKernelGGL(k_pdsch_llr2, dim3(gx ? gx : 1, (unsigned)n), dim3(256), 0, st, d_items, n);
  if (csi) {
    const unsigned gb = std::min(cdiv((size_t)max_re * 6, 256), 256u);
    hipLaunchKernelGGL(k_csi_correct, dim3(gb ? gb : 1, (unsigned)n), dim3(256), 0, st, d_items, n);
  }
  return hipGetLastError();
}

// ------------------------------------------------------------------ transmit ----
// srslte_pdsch_encode (pdsch.c:1048-1131) after the DL-SCH encoding: per codeword scrambling
// (srslte_scrambling_bytes, the codeword's own sequence) and modulation (srslte_mod_modulate_bytes with
// the LTE tables of modem/lte_tables.c: index = bits MSB first), layer mapping and precoding
// (srslte_layermap_type / srslte_precoding_type, mimo/layermap.c:43-130, mimo/precoding.c:1849-2143),
// rho_a scaling and the RE mapping of every port (srslte_pdsch_put). One thread per RE j: it builds the
// codeword symbols it needs and writes port p's value at grid + p * port_stride + map[j].
__device__ __forceinline__ float2 tx_symbol(const TxItem &t, int cw, uint32_t j, const float2 *tables) {
  const int qm = t.qm[cw];
  const float2 *tab = tables + (qm == 1 ? 0 : qm == 2 ? 2 : qm == 4 ? 6 : 22);
  const uint32_t b0 = j * (uint32_t)qm, w = b0 >> 5, sh = b0 & 31;
  const uint64_t cw64 = (uint64_t)t.c[cw][w] | ((uint64_t)t.c[cw][w + 1] << 32);
  const uint32_t cb = (uint32_t)(cw64 >> sh);
  uint32_t idx = 0;
  for (int k = 0; k < qm; k++) idx = (idx << 1) | ((t.e[cw][b0 + k] ^ (cb >> k)) & 1u);
  return tab[idx];
}
__device__ __forceinline__ float2 cscale(float2 v, float k) { return make_float2(__fmul_rn(v.x, k), __fmul_rn(v.y, k)); }
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(__fadd_rn(a.x, b.x), __fadd_rn(a.y, b.y)); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(__fsub_rn(a.x, b.x), __fsub_rn(a.y, b.y)); }

__global__ __launch_bounds__(256) void k_pdsch_tx(const TxItem *__restrict__ items, int nitems,
                                                  const float2 *__restrict__ tables) {
  const int it = blockIdx.y;
  if (it >= nitems) return;
  const TxItem t = items[it];
  for (uint32_t j = blockIdx.x * 256 + threadIdx.x; j < t.nof_re; j += gridDim.x * 256) {
    float2 y0, y1 = make_float2(0.f, 0.f);
    bool two = true;
    switch (t.mimo) {
    case SRSGPU_MIMO_TX_DIVERSITY: { // layermap_diversity + 2-port SFBC, scaled by rho_a / sqrt 2
      if (t.nlayers == 4) { // 4 ports (precoding.c:1863-1889): RE 4i+2q+r on ports q and q+2,
                            // the other two ports 0; 4 floor(n / 4) symbols per port
        const uint32_t j0 = j & ~3u, q = (j >> 1) & 1;
        if (j0 + 3 >= t.nof_re) continue;
        const float2 a = tx_symbol(t, 0, j0 + 2 * q, tables), b = tx_symbol(t, 0, j0 + 2 * q + 1, tables);
        const float k = t.scaling; // scaling / sqrtf(2) on the host
        const float2 ya = (j & 1) ? cscale(b, k) : cscale(a, k);
        const float2 yb = (j & 1) ? cscale(make_float2(a.x, -a.y), k) : cscale(make_float2(-b.x, b.y), k);
        const uint32_t m = t.map[j];
        for (uint32_t p = 0; p < 4; p++)
          t.grid[p * t.port_stride + m] = p == q ? ya : p == q + 2 ? yb : make_float2(0.f, 0.f);
        continue;
      }
      const uint32_t j0 = j & ~1u;
      if (j0 + 1 >= t.nof_re) continue; // 2 floor(n / 2) symbols per port (precoding.c:1853-1862)
      const float2 a = tx_symbol(t, 0, j0, tables), b = tx_symbol(t, 0, j0 + 1, tables);
      const float k = t.scaling; // scaling / sqrtf(2) on the host
      if (j == j0) {
        y0 = cscale(a, k);
        y1 = cscale(make_float2(-b.x, b.y), k); // -conj(x1)
      } else {
        y0 = cscale(b, k);
        y1 = cscale(make_float2(a.x, -a.y), k); // conj(x0)
      }
      break;
    }
    case SRSGPU_MIMO_CDD: { // precoding_cdd_2x2 (precoding.c:1898-1958), layers = codewords
      const float2 x0 = tx_symbol(t, 0, j, tables), x1 = tx_symbol(t, 1, j, tables);
      const float k = t.scaling; // 0.5 scaling
      y0 = cscale(cadd(x0, x1), k);
      y1 = cscale((j & 1) ? csub(x1, x0) : csub(x0, x1), k);
      break;
    }
    case SRSGPU_MIMO_SPATIAL_MULTIPLEX: { // precoding_multiplex 2 ports (precoding.c:1985-2100)
      const float k = t.scaling; // scaling / sqrt 2 (one layer, codebook 0 of two), scaling / 2 otherwise
      const float2 x0 = tx_symbol(t, 0, j, tables);
      if (t.nlayers == 1) {
        y0 = cscale(x0, k);
        y1 = t.codebook == 0 ? y0 : t.codebook == 1 ? cscale(x0, -k)
             : t.codebook == 2 ? make_float2(-__fmul_rn(x0.y, k), __fmul_rn(x0.x, k))   // x (j k)
                               : make_float2(__fmul_rn(x0.y, k), -__fmul_rn(x0.x, k)); // x (-j k)
      } else {
        const float2 x1 = tx_symbol(t, 1, j, tables);
        if (t.codebook == 0) {
          y0 = cscale(x0, k);
          y1 = cscale(x1, k);
        } else {
          y0 = cscale(cadd(x0, x1), k);
          const float2 d = csub(x0, x1);
          y1 = t.codebook == 1 ? cscale(d, k) : cscale(make_float2(-d.y, d.x), k); // j (x0 - x1)
        }
      }
      break;
    }
    default: // single antenna port
      y0 = tx_symbol(t, 0, j, tables);
      if (t.scaling != 1.0f) y0 = cscale(y0, t.scaling);
      two = false;
    }
    const uint32_t m = t.map[j];
    t.grid[m] = y0;
    if (two) t.grid[t.port_stride + m] = y1;
  }
}

hipError_t launch_pdsch_tx(const TxItem *d_items, int n, uint32_t max_re, const float2 *tables,
                           hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const unsigned gx = std::min(cdiv(max_re, 256), 64u);
  hipLaunchKernelGGL(k_pdsch_tx, dim3(gx ? gx : 1, (unsigned)n), dim3(256), 0, st, d_items, n, tables);
  return hipGetLastError();
}

// ------------------------------------------------------------------ PCFICH ----
// srslte_pcfich_decode_multi (pcfich.c:178-241) per subframe, one wavefront: lane j < 16
// equalises RE j of the 16 PCFICH REs (regs.c:477-512 + :622-665: four REGs of symbol 0) with the
// PDSCH equalisers above on the reference's paths for 16 <= 32 symbols (SISO: the C path with the
// noise estimate, scaling 1; 2 / 4 ports: generic transmit diversity + layer demapping), demaps QPSK
// (x times (float) -sqrt 2, demod_soft.c:71-73) and descrambles (+-1, sequences.c:42-44); lane 0
// correlates with the three CFI codewords as +-1 in order (pcfich.c:129-147, vector.c:359-366).
__device__ __forceinline__ int cfi_bit(int c, int i) { // 36.212 Table 5.3.4-1: 011 / 101 / 110 repeated
  const int r = i % 3;
  return c == 0 ? (r != 0) : c == 1 ? (r != 1) : (r != 2);
}
__global__ __launch_bounds__(64) void k_pcfich(const PcfichItem *__restrict__ items, int n,
                                               const float2 *__restrict__ grid,
                                               const float2 *__restrict__ ce, size_t ant_stride,
                                               int nof_prb, int nports, int nrx,
                                               const uint32_t *__restrict__ idx,
                                               const uint32_t *__restrict__ seq,
                                               uint32_t *__restrict__ cfi, float *__restrict__ corr) {
  __shared__ float l[32];
  const int s = blockIdx.x, j = threadIdx.x;
  if (s >= n) return;
  const PcfichItem it = items[s];
  LlrItem t;
  memset(&t, 0, sizeof(t));
#pragma unroll
  for (int a = 0; a < 2; a++) { // constant indices only: the descriptor stays in registers
    if (a >= nrx) break;
    t.y[a] = grid + it.grid_off + (size_t)a * ant_stride;
#pragma unroll
    for (int p = 0; p < 4; p++)
      if (p < nports) t.h[p][a] = ce + it.ce_off + (size_t)(a * nports + p) * ant_stride;
  }
  t.map = idx;
  t.nof_re = 16;
  t.nrx = nrx;
  t.noise = it.dnoise ? *it.dnoise : it.noise;
  t.scaling = 1.0f;
  t.inv_scaling = 1.0f;
  if (j < 16) {
    const Eq e = nports == 4   ? equalise_txdiv4(t, (uint32_t)j)
                 : nports == 2 ? equalise_txdiv(t, (uint32_t)j)
                               : equalise(t, idx[j], (uint32_t)j);
    const float s2 = -1.41421354f; // (float) -sqrt(2)
    const uint32_t c = seq[it.sf_idx];
    float a0 = __fmul_rn(e.xr, s2), a1 = __fmul_rn(e.xi, s2);
    if ((c >> (2 * j)) & 1u) a0 = -a0;
    if ((c >> (2 * j + 1)) & 1u) a1 = -a1;
    l[2 * j] = a0;
    l[2 * j + 1] = a1;
  }
  __syncthreads();
  if (j == 0) {
    float mx = 0.f;
    int index = 0;
    for (int k = 0; k < 3; k++) {
      float r = 0.f;
      for (int i = 0; i < 32; i++) r = __fadd_rn(r, cfi_bit(k, i) ? l[i] : -l[i]);
      if (r > mx) {
        mx = r;
        index = k;
      }
    }
    cfi[s] = (uint32_t)index + 1;
    corr[s] = mx;
  }
}

hipError_t launch_pcfich(const PcfichItem *d_items, int n, const float2 *grid, const float2 *ce,
                         size_t ant_stride, int nof_prb, int nports, int nrx, const uint32_t *idx,
                         const uint32_t *seq, uint32_t *cfi, float *corr, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_pcfich, dim3(n), dim3(64), 0, st, d_items, n, grid, ce, ant_stride, nof_prb,
                     nports, nrx, idx, seq, cfi, corr);
  return hipGetLastError();
}

// ------------------------------------------------------------------ PDCCH LLRs ----
// srslte_pdcch_extract_llr_multi (pdcch.c:424-506) for many subframes, one thread per PDCCH
// symbol j (blockIdx.y = subframe): the symbol is gathered at map[j] from every rx antenna's grid
// and estimate (srslte_regs_pdcch_get), equalised on the reference's path for nof_symbols symbols
// (1 port: srslte_predecoding_single_multi with noise_estimate / 2 and scaling 1; 2 or 4 ports:
// srslte_predecoding_diversity_multi + srslte_layerdemap_diversity), QPSK soft-demapped as float
// (demod_qpsk_lte: x (float) -sqrt(2), demod_soft.c:75-77) and descrambled
// (srslte_scrambling_f_offset: a product with +-1, scrambling.c:39-42).
__global__ __launch_bounds__(256) void k_pdcch_llr(const PdcchItem *__restrict__ items, int n,
                                                   const float2 *__restrict__ grid,
                                                   const float2 *__restrict__ ce, size_t ant_stride,
                                                   int nports, int nrx, float *__restrict__ llr) {
  const int s = blockIdx.y;
  if (s >= n) return;
  const PdcchItem it = items[s];
  const uint32_t j = blockIdx.x * 256 + threadIdx.x;
  if (j >= it.nof_symbols) return;
  LlrItem t;
  memset(&t, 0, sizeof(t));
#pragma unroll
  for (int a = 0; a < 2; a++) { // constant indices only: the descriptor stays in registers
    if (a >= nrx) break;
    t.y[a] = grid + it.grid_off + (size_t)a * ant_stride;
#pragma unroll
    for (int p = 0; p < 4; p++)
      if (p < nports) t.h[p][a] = ce + it.ce_off + (size_t)(a * nports + p) * ant_stride;
  }
  t.map = it.map;
  t.nof_re = it.nof_symbols;
  t.nrx = nrx;
  t.noise = nports >= 2 ? 0.f : (it.dnoise ? *it.dnoise : it.noise) / 2;
  t.scaling = 1.0f;
  t.inv_scaling = 1.0f;
  const Eq e = nports == 4 ? equalise_txdiv4(t, j) : nports == 2 ? equalise_txdiv(t, j) : equalise(t, it.map[j], j);
  const float s2 = -1.41421354f; // (float) -sqrt(2)
  float a0 = __fmul_rn(e.xr, s2), a1 = __fmul_rn(e.xi, s2);
  const uint32_t b = 2 * j, w = it.c[b >> 5] >> (b & 31);
  if (w & 1u) a0 = -a0;
  if (w & 2u) a1 = -a1;
  float2 *o = reinterpret_cast<float2 *>(llr + it.llr_off);
  o[j] = make_float2(a0, a1);
}

hipError_t launch_pdcch_llr(const PdcchItem *d_items, int n, uint32_t max_symbols, const float2 *grid,
                            const float2 *ce, size_t ant_stride, int nports, int nrx, float *llr,
                            hipStream_t st) {
  if (n <= 0 || max_symbols == 0) return hipSuccess;
  hipLaunchKernelGGL(k_pdcch_llr, dim3((max_symbols + 255) / 256, n), dim3(256), 0, st, d_items, n, grid,
                     ce, ant_stride, nports, nrx, llr);
  return hipGetLastError();
}

} // namespace srsgpu
