// Device side of the tail-biting K=7 r=1/3 Viterbi decoder (srsLTE's PDCCH / PUSCH CQI decoder:
// viterbi.c with VITERBI_16 -> decode37_avx2_16bit over viterbi37_avx2_16bit.c), one wavefront per
// frame, lane s = trellis state s. Shared by viterbi.hip (DCI) and uci_kernels.hip (CQI on PUSCH).
#ifndef SRSGPU_VITERBI_DEV_H
#define SRSGPU_VITERBI_DEV_H
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace srsgpu {

static __constant__ uint8_t kPermCC[32] = {1, 17, 9, 25, 5, 21, 13, 29, 3, 19, 11, 27, 7, 23, 15, 31,
                                           0, 16, 8, 24, 4, 20, 12, 28, 2, 18, 10, 26, 6, 22, 14, 30};
static __constant__ uint8_t kPermCCInv[32] = {16, 0, 24, 8, 20, 4, 28, 12, 18, 2, 26, 10, 22, 6, 30, 14,
                                              17, 1, 25, 9, 21, 5, 29, 13, 19, 3, 27, 11, 23, 7, 31, 15};

__device__ __forceinline__ int vparity(int x) { return __popc((unsigned)x) & 1; }

// One tail-biting frame of F bits on one wavefront: the trellis of decode37_avx2_16bit on quantised
// symbols q (3F uint16 in LDS), decoded bits (the middle copy) into bits[0..F) in LDS; dec is LDS
// scratch.
__device__ __forceinline__ void vit_trellis(int F, uint8_t *bits, const uint16_t *q, uint64_t *dec) {
  const int lane = threadIdx.x, nb = 3 * F;
  for (int i = lane; i < 8; i += 64) dec[nb + i] = 0; // chainback reads up to 6 past the end
  __syncthreads();
  const int b = lane >> 1, h = lane & 1;
  const uint32_t B0 = vparity((2 * b) & 0x6D) ? 65535u : 0u;
  const uint32_t B1 = vparity((2 * b) & 0x4F) ? 65535u : 0u;
  const uint32_t B2 = vparity((2 * b) & 0x57) ? 65535u : 0u;
  uint32_t m = 63; // this lane's state metric (uint16 held in 32 bits)
  int k = 0;       // t mod F
  for (int t = 0; t < nb; t++) {
    const uint32_t s0 = q[3 * k], s1 = q[3 * k + 1], s2 = q[3 * k + 2];
    if (++k == F) k = 0;
    const uint32_t m0a = ((B0 ^ s0) + (B1 ^ s1) + 1) >> 1;
    const uint32_t metric = (((B2 ^ s2) + m0a + 1) >> 1) >> 3;
    const uint32_t mm = (8191u - metric) & 0xFFFFu;
    const uint32_t ob = (uint32_t)__shfl((int)m, b), ob32 = (uint32_t)__shfl((int)m, b + 32);
    // h = 0: m0 = ob + metric vs m1 = ob32 + mm; h = 1: m2 = ob + mm vs m3 = ob32 + metric
    const uint32_t a = (ob + (h ? mm : metric)) & 0xFFFFu;
    const uint32_t c = (ob32 + (h ? metric : mm)) & 0xFFFFu;
    const bool d = (int16_t)(uint16_t)(a - c) > 0;
    m = d ? c : a;
    const uint64_t w = __ballot(d);
    if (lane == 0) dec[t] = w;
  }
  // best end state: the last index holding the minimum metric
  uint32_t mn = m;
  for (int o = 32; o > 0; o >>= 1) mn = min(mn, (uint32_t)__shfl_xor((int)mn, o));
  int best = m == mn ? lane : -1;
  for (int o = 32; o > 0; o >>= 1) best = max(best, __shfl_xor(best, o));
  __syncthreads();
  if (lane == 0) {
    uint32_t es = (uint32_t)best << 2;
    for (int t = nb - 1; t >= 0; t--) {
      const uint32_t bit = (uint32_t)((dec[t + 6] >> (es >> 2)) & 1u);
      es = (es >> 1) | (bit << 7);
      if (t >= F && t < 2 * F) bits[t - F] = (uint8_t)bit;
    }
  }
  __syncthreads();
}

// srslte_viterbi_decode_f: quantisation q = clamp((long)(32767.5f + (1000 / max|x|) x), 0, 65535)
// (viterbi.c:531-546, vector.c:408-420), then the trellis
__device__ __forceinline__ void vit_frame(const float *sym, int F, uint8_t *bits, uint16_t *q,
                                          uint64_t *dec) {
  const int lane = threadIdx.x, len = 3 * F;
  // max |x| (viterbi.c:531-536: float max starting at -9e9, fabs compared in double)
  float mx = -9e9f;
  for (int i = lane; i < len; i += 64) mx = fmaxf(mx, fabsf(sym[i]));
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
  const float gain = __fdiv_rn(1000.0f, mx);
  for (int i = lane; i < len; i += 64) {
    const float v = __fadd_rn(32767.5f, __fmul_rn(gain, sym[i]));
    long t = (v == v && v >= -9.2e18f && v < 9.2e18f) ? (long)v : (long)INT64_MIN; // cvttss2si
    t = t < 0 ? 0 : t > 65535 ? 65535 : t;
    q[i] = (uint16_t)t;
  }
  vit_trellis(F, bits, q, dec);
}

// srslte_viterbi_decode_s (viterbi.c:558-584 with VITERBI_16): srslte_vec_quant_sus with gain 1 and
// offset 32767 (vector.c:450-460), tmp = (int16_t)(32767 + (float)x) as cvttss2si truncated to 16
// bits, 0 where negative: x <= 0 gives 32767 + x (0 at -32768), x > 0 wraps negative and gives 0
__device__ __forceinline__ void vit_frame_s(const int16_t *sym, int F, uint8_t *bits, uint16_t *q,
                                            uint64_t *dec) {
  for (int i = threadIdx.x; i < 3 * F; i += 64) {
    const int16_t t = (int16_t)(int32_t)__fadd_rn(32767.0f, (float)sym[i]);
    q[i] = (uint16_t)(t < 0 ? 0 : t);
  }
  __syncthreads();
  vit_trellis(F, bits, q, dec);
}

} // namespace srsgpu
#endif
