// UCI multiplexed on the PUSCH (srsgpu_ulsch_uci_decode_dev, include/srsgpu/ulsch_batch.h): the
// steps of srslte_pusch_decode around the UL-SCH data (reference: lib/src/phy/phch/pusch.c:626-657,
// sch.c:892-985, uci.c:270-790), one workgroup per transport block.
//   k_uci_ack_ri  HARQ-ACK and RI from the still scrambled q bits (srslte_uci_decode_ack_ri,
//                 uci.c:746-790): 1 bit, the sum of -(q0 + q1) over the Q' groups with both values
//                 signed by c at the group's first position (decode_ri_ack_1bit, uci.c:609-618, in
//                 uint32 arithmetic); 2 bits, the groups taken in threes, each triple added when the
//                 loop reaches the next multiple of 3 (decode_ri_ack_2bits, :620-642; a last triple
//                 is never added); bit = sum > 0. Sums are wrap-around integer sums, so any order.
//   (k_ulsch_deinterleave in dlsch_kernels.hip: descrambling, RI entries out, ACK entries zero)
//   k_uci_cqi     g[0] as the reference's lut leaves it (the RI entry with the largest q index
//                 writes last, sch.c:550-568 + vector.c:119-123), then the CQI
//                 (srslte_uci_decode_cqi_pusch, uci.c:428-464): up to 11 bits the (32, O) block
//                 code by ML (decode_cqi_short, :312-351: copies of 32 summed into g[0..32) with
//                 int16 wrap, correlation as srslte_vec_dot_prod_sss computes it on AVX2 -- 16
//                 int16 lanes of mullo + add, summed, then an int tail -- first maximum wins);
//                 above, srslte_rm_conv_rx_s, srslte_viterbi_decode_s (viterbi_dev.h) and CRC8 0x19B
//                 (decode_cqi_long, :391-425).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dlsch_kernels.h"
#include "gmem.h"
#include "srsgpu/uci_tables.h"
#include "srsgpu/ulsch_batch.h"
#include "uci_dev.h"
#include "viterbi_dev.h"

namespace srsgpu {

// 1- or 2-bit HARQ-ACK / RI of one TB; 256 threads; bits into out[0..1]
__device__ __forceinline__ void uci_bits(const int16_t *q, const uint8_t *c, uint32_t Qp, uint32_t O, uint32_t Qm,
                                         uint32_t rows, bool ri, uint32_t (*red)[256], uint8_t *out) {
  uint32_t s0 = 0, s1 = 0;
  const int t = threadIdx.x;
  if (O == 1) {
    for (uint32_t g = t; g < Qp; g += 256) {
      const uint32_t p0 = uci_pos(g, 0, Qm, rows, ri), p1 = uci_pos(g, 1, Qm, rows, ri);
      const bool cs = c[p0] != 0; // decode_ri_ack_1bit reads c at p0 for both values
      const uint32_t q0 = (uint32_t)(cs ? (int32_t)q[p0] : -(int32_t)q[p0]);
      const uint32_t q1 = (uint32_t)(cs ? (int32_t)q[p1] : -(int32_t)q[p1]);
      s0 += 0u - (q0 + q1);
    }
  } else if (O == 2) {
    const uint32_t ntri = Qp > 0 ? (Qp - 1) / 3 : 0; // triples added at i = 3, 6, .. <= Qp - 1
    for (uint32_t tr = t; tr < ntri; tr += 256) {
      int32_t v[6];
      for (int g = 0; g < 3; g++)
        for (int k = 0; k < 2; k++) {
          const uint32_t p = uci_pos(3 * tr + g, k, Qm, rows, ri);
          v[2 * g + k] = c[p] ? (int32_t)q[p] : -(int32_t)q[p];
        }
      s0 -= (uint32_t)(v[0] + v[3]);
      s1 -= (uint32_t)(v[1] + v[4]);
    }
  }
  red[0][t] = s0;
  red[1][t] = s1;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w) {
      red[0][t] += red[0][t + w];
      red[1][t] += red[1][t + w];
    }
    __syncthreads();
  }
  if (t == 0) {
    out[0] = (int32_t)red[0][0] > 0;
    out[1] = O == 2 ? (uint8_t)((int32_t)red[1][0] > 0) : 0;
  }
  __syncthreads();
}

__global__ __launch_bounds__(256) void k_uci_ack_ri(const UlItem *__restrict__ items, int n,
                                                    const int16_t *__restrict__ q_base,
                                                    const uint8_t *__restrict__ c_base,
                                                    srsgpu_uci_result_t *__restrict__ res) {
  __shared__ uint32_t red[2][256];
  __shared__ uint8_t bits[2];
  const int b = blockIdx.x;
  if (b >= n) return;
  const UlItem it = items[b];
  if (!it.uci) return;
  const int16_t *q = gmem(q_base + it.q_offset);
  const uint8_t *c = gmem(c_base + it.c_offset);
  srsgpu_uci_result_t *r = gmem(res) + b;
  if (threadIdx.x == 0) {
    r->ack[0] = r->ack[1] = r->ri = r->cqi_ack = 0;
    r->Q_ack = it.Q_ack;
    r->Q_ri = it.Q_ri;
    r->Q_cqi = it.Q_cqi;
  }
  if (it.O_ack) {
    uci_bits(q, c, it.Q_ack, it.O_ack, it.Qm, it.rows, false, red, bits);
    if (threadIdx.x == 0) {
      r->ack[0] = bits[0];
      r->ack[1] = bits[1];
    }
  }
  if (it.O_ri) { // with 2 RI bits the reference keeps the first (uci_ri is one byte)
    uci_bits(q, c, it.Q_ri, it.O_ri, it.Qm, it.rows, true, red, bits);
    if (threadIdx.x == 0) r->ri = bits[0];
  }
}

#define UCI_FMAX (SRSGPU_UCI_MAX_CQI_BITS + 8)
__global__ __launch_bounds__(64) void k_uci_cqi(const UlItem *__restrict__ items, int n,
                                                const int16_t *__restrict__ q_base,
                                                const uint8_t *__restrict__ c_base, int16_t *__restrict__ g_base,
                                                srsgpu_uci_result_t *__restrict__ res, int32_t *__restrict__ ret,
                                                uint32_t *__restrict__ noi) {
  __shared__ int16_t tmp[3 * 32 * ((UCI_FMAX - 1) / 32 + 1)];
  __shared__ int16_t rm[3 * UCI_FMAX];
  __shared__ uint16_t qv[3 * UCI_FMAX];
  __shared__ uint64_t dec[3 * UCI_FMAX + 8];
  __shared__ uint8_t bits[UCI_FMAX];
  __shared__ int16_t acc[32];
  const int b = blockIdx.x, lane = threadIdx.x;
  if (b >= n) return;
  const UlItem it = items[b];
  if (!it.uci) return;
  int16_t *g = gmem(g_base + it.q_offset);
  srsgpu_uci_result_t *r = gmem(res) + b;
  if (lane == 0 && it.Q_ri) { // the last write to g[0]: the RI entry with the largest q index
    uint32_t xr = 0;        // (row rows - 1, the largest of the first min(4, Q'_ri) columns, bit Qm - 1)
    for (uint32_t u = 0; u < 4 && u < it.Q_ri; u++) xr = max(xr, uci_pos(u, it.Qm - 1, it.Qm, it.rows, true));
    const int16_t v = gmem(q_base + it.q_offset)[xr];
    g[0] = gmem(c_base + it.c_offset)[xr] ? (int16_t)(-(int32_t)v) : v;
  }
  if (!it.tbs && lane == 0) {
    gmem(ret)[b] = 0;
    gmem(noi)[b] = 0;
  }
  __syncthreads();
  const uint32_t O = it.O_cqi, Q = it.Q_cqi * it.Qm;
  if (!O) return;
  if (O <= 11) {
    if (lane < 32) { // decode_cqi_short: copies of 32 summed into g[0..32) (int16 wrap)
      int16_t a = Q > (uint32_t)lane ? g[lane] : 0;
      if (Q > 32) {
        uint32_t i = 1;
        for (; i < Q / 32; i++) a = (int16_t)(a + g[i * 32 + lane]);
        if ((uint32_t)lane < Q % 32) a = (int16_t)(a + g[i * 32 + lane]);
        g[lane] = a;
      }
      acc[lane] = a;
    }
    __syncthreads();
    const uint32_t len = Q < 32 ? Q : 32, steps = len / 16;
    uint32_t mrow[32]; // row i of the basis as an O-bit mask, bit O - 1 - n for data bit n
    for (int i = 0; i < 32; i++) {
      uint32_t m = 0;
      for (uint32_t nb = 0; nb < O; nb++) m |= (uint32_t)SRSGPU_CQI_BASIS[i][nb] << (O - 1 - nb);
      mrow[i] = m;
    }
    int32_t best = INT32_MIN;
    uint32_t bw = 0;
    for (uint32_t w = lane; w < (1u << O); w += 64) {
      int16_t lanes16[16];
      for (int k = 0; k < 16; k++) lanes16[k] = 0;
      for (uint32_t s = 0; s < steps; s++)
        for (int k = 0; k < 16; k++) {
          const int i = 16 * s + k;
          const int16_t cw = (__popc(w & mrow[i]) & 1) ? 1 : -1;
          lanes16[k] = (int16_t)(lanes16[k] + (int16_t)(cw * acc[i]));
        }
      int32_t corr = 0;
      for (int k = 0; k < 16; k++) corr += lanes16[k];
      for (uint32_t i = 16 * steps; i < len; i++) corr += ((__popc(w & mrow[i]) & 1) ? 1 : -1) * acc[i];
      if (corr > best) { // words ascend per lane: strict > keeps the first
        best = corr;
        bw = w;
      }
    }
    for (int o = 32; o > 0; o >>= 1) { // the maximum, the lowest word among equals
      const int32_t ob = __shfl_xor(best, o);
      const uint32_t ow = (uint32_t)__shfl_xor((int)bw, o);
      if (ob > best || (ob == best && ow < bw)) {
        best = ob;
        bw = ow;
      }
    }
    for (uint32_t nb = lane; nb < O; nb += 64) r->cqi[nb] = (uint8_t)((bw >> (O - 1 - nb)) & 1u);
    return;
  }
  // decode_cqi_long: srslte_rm_conv_rx_s to 3 (O + 8) soft bits (int16 soft combining in input order,
  // 10000 = empty), srslte_viterbi_decode_s, CRC8
  const int F = (int)O + 8, out_len = 3 * F;
  const int nrows = (out_len / 3 - 1) / 32 + 1, K_p = nrows * 32;
  const int ndummy = max(K_p - out_len / 3, 0);
  for (int i = lane; i < 3 * K_p; i += 64) tmp[i] = 10000;
  __syncthreads();
  // input k lands on the valid position of rank k mod V (V = out_len valid positions per pass), as
  // in k_dci_decode: position j of rank r combines inputs r, r + V, ... in that order
  int base = 0;
  for (int c0 = 0; c0 < 3 * K_p; c0 += 64) {
    const int j = c0 + lane;
    bool valid = false;
    if (j < 3 * K_p) {
      const int d_i = (j % K_p) / nrows, d_j = (j % K_p) % nrows;
      valid = d_j * 32 + kPermCC[d_i] >= ndummy;
    }
    const uint64_t mask = __ballot(valid);
    const int rk = base + __popcll(mask & ((1ull << lane) - 1ull));
    base += __popcll(mask);
    if (valid) {
      int16_t a = 10000;
      for (uint32_t k = rk; k < Q; k += out_len) {
        const int16_t x = g[k];
        if (a == 10000)
          a = x;
        else if (x != 10000)
          a = (int16_t)(a + x);
      }
      tmp[j] = a;
    }
  }
  __syncthreads();
  for (int i = lane; i < out_len / 3; i += 64) {
    const int d_i = (i + ndummy) / 32, d_j = (i + ndummy) % 32;
    for (int s = 0; s < 3; s++) {
      const int16_t o = tmp[K_p * s + kPermCCInv[d_j] * nrows + d_i];
      rm[i * 3 + s] = o != 10000 ? o : 0;
    }
  }
  __syncthreads();
  vit_frame_s(rm, F, bits, qv, dec);
  if (lane == 0) {
    uint32_t crc = 0;
    for (int i = 0; i < F; i++) {
      const uint32_t fb = ((crc >> 7) & 1u) ^ (bits[i] & 1u);
      crc = (crc << 1) & 0xFFu;
      if (fb) crc ^= 0x9Bu;
    }
    r->cqi_ack = crc == 0;
    for (uint32_t i = 0; i < O; i++) r->cqi[i] = crc == 0 ? bits[i] : 0;
  }
}

hipError_t launch_uci_ack_ri(const UlItem *d_items, int n, const int16_t *q, const uint8_t *c, void *res,
                             hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_uci_ack_ri, dim3((unsigned)n), dim3(256), 0, st, d_items, n, q, c,
                     (srsgpu_uci_result_t *)res);
  return hipGetLastError();
}

hipError_t launch_uci_cqi(const UlItem *d_items, int n, const int16_t *q, const uint8_t *c, int16_t *g, void *res,
                          int32_t *ret, uint32_t *noi, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_uci_cqi, dim3((unsigned)n), dim3(64), 0, st, d_items, n, q, c, g,
                     (srsgpu_uci_result_t *)res, ret, noi);
  return hipGetLastError();
}

} // namespace srsgpu
