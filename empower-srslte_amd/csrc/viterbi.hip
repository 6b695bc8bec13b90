// Batched tail-biting Viterbi decoder (include/srsgpu/viterbi_batch.h): one wavefront per frame,
// lane s = trellis state s. The reference's srslte_viterbi_decode_f on an AVX2 build
// (lib/src/phy/fec/viterbi.c:520-546 with VITERBI_16 -> decode37_avx2_16bit :133-160 ->
// viterbi37_avx2_16bit.c), restated per state:
//   quantisation  q = clamp((long)(32767.5f + (1000 / max|x|) * x), 0, 65535) (vector.c:408-420)
//   per bit t     (the frame repeated 3 times) butterfly b = s >> 1 joins old states b and b + 32;
//                 metric = avg(B2 ^ q2, avg(B0 ^ q0, B1 ^ q1)) >> 3 with B = 0 / 65535 from the
//                 polynomial parities, complement 8191 - metric; uint16 wrapping sums; decision =
//                 signed 16-bit difference > 0 ("modulo" compare); no normalisation (the
//                 reference's is a no-op: its in-lane byte shift by 16 zeroes the minimum)
//   end           best state = the last index of the minimum metric; chainback from it reading
//                 the decisions 6 positions past the bit it decides (zero beyond the frame); the
//                 middle copy of the frame is the output.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "gmem.h"
#include "srsgpu/viterbi_batch.h"

namespace srsgpu {

__device__ __forceinline__ int vparity(int x) { return __popc((unsigned)x) & 1; }

// One tail-biting frame of F bits on one wavefront: symbols at sym (3F floats, global or LDS),
// decoded bits (the middle copy) into bits[0..F) in LDS. q / dec are LDS scratch.
__device__ __forceinline__ void vit_frame(const float *sym, int F, uint8_t *bits, uint16_t *q,
                                          uint64_t *dec) {
  const int lane = threadIdx.x, len = 3 * F, nb = 3 * F;
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

__global__ __launch_bounds__(64) void k_viterbi37_tb(const srsgpu_viterbi_frame_t *__restrict__ frames,
                                                     int nframes, const float *__restrict__ sym_base,
                                                     uint8_t *__restrict__ out_base) {
  __shared__ uint16_t q[3 * SRSGPU_VITERBI_MAX_FRAME];
  __shared__ uint64_t dec[3 * SRSGPU_VITERBI_MAX_FRAME + 8];
  __shared__ uint8_t bits[SRSGPU_VITERBI_MAX_FRAME];
  const int f = blockIdx.x;
  if (f >= nframes) return;
  const srsgpu_viterbi_frame_t fr = frames[f];
  const int F = (int)fr.frame_length;
  if (F < 1 || F > SRSGPU_VITERBI_MAX_FRAME) return;
  vit_frame(gmem(sym_base + fr.sym_offset), F, bits, q, dec);
  uint8_t *out = gmem(out_base + fr.out_offset);
  for (int i = threadIdx.x; i < F; i += 64) out[i] = bits[i];
}

// DCI candidates (srslte_pdcch_decode_msg, pdcch.c:380-396 + srslte_pdcch_dci_decode :322-360):
// mean |llr| check (double, in order), srslte_rm_conv_rx (rm_conv.c:99-157), the Viterbi frame
// of nof_bits + 16, CRC16 remainder. One wavefront per candidate; the sequential parts (the mean,
// the bit collection whose soft combining adds in input order) on lane 0.
__constant__ uint8_t kPermCC[32] = {1, 17, 9, 25, 5, 21, 13, 29, 3, 19, 11, 27, 7, 23, 15, 31,
                                    0, 16, 8, 24, 4, 20, 12, 28, 2, 18, 10, 26, 6, 22, 14, 30};
__constant__ uint8_t kPermCCInv[32] = {16, 0, 24, 8, 20, 4, 28, 12, 18, 2, 26, 10, 22, 6, 30, 14,
                                       17, 1, 25, 9, 21, 5, 29, 13, 19, 3, 27, 11, 23, 7, 31, 15};

__global__ __launch_bounds__(64) void k_dci_decode(const srsgpu_dci_cand_t *__restrict__ cands, int n,
                                                   const float *__restrict__ llr_base,
                                                   uint8_t *__restrict__ out_base,
                                                   uint16_t *__restrict__ crc_rem,
                                                   uint8_t *__restrict__ decoded) {
  constexpr int FMAX = SRSGPU_DCI_MAX_BITS + 16;
  __shared__ float tmp[3 * 32 * ((FMAX - 1) / 32 + 1)];
  __shared__ float rm[3 * FMAX];
  __shared__ uint16_t q[3 * FMAX];
  __shared__ uint64_t dec[3 * FMAX + 8];
  __shared__ uint8_t bits[FMAX];
  __shared__ int go;
  const int ci = blockIdx.x;
  if (ci >= n) return;
  const srsgpu_dci_cand_t c = cands[ci];
  const int E = (int)c.E, nbits = (int)c.nof_bits, lane = threadIdx.x;
  if (E < 1 || E > SRSGPU_DCI_MAX_E || nbits < 1 || nbits > SRSGPU_DCI_MAX_BITS) return;
  const float *e = gmem(llr_base + c.llr_offset);
  const int F = nbits + 16, out_len = 3 * F;
  const int nrows = (out_len / 3 - 1) / 32 + 1, K_p = nrows * 32;
  const int ndummy = max(K_p - out_len / 3, 0);
  __shared__ float es[SRSGPU_DCI_MAX_E];
  for (int i = lane; i < E; i += 64) es[i] = e[i];
  for (int i = lane; i < 3 * K_p; i += 64) tmp[i] = 10000.0f;
  __syncthreads();
  if (lane == 0) { // the mean in the reference's order (double sum, pdcch.c:386-390)
    double mean = 0;
    for (int i = 0; i < E; i++) mean = __dadd_rn(mean, (double)fabsf(es[i]));
    mean = __ddiv_rn(mean, (double)E);
    go = mean > 0.5;
  }
  __syncthreads();
  if (go) {
    // bit collection (rm_conv_rx.c:124-143) in parallel: input k lands on the valid position of
    // rank k mod V (V = out_len valid positions per pass), so position j of rank r receives
    // inputs r, r + V, r + 2V, ... in that order, which is the reference's soft-combining order
    const int V = out_len;
    int base = 0;
    for (int c0 = 0; c0 < 3 * K_p; c0 += 64) {
      const int j = c0 + lane;
      bool valid = false;
      if (j < 3 * K_p) {
        const int d_i = (j % K_p) / nrows, d_j = (j % K_p) % nrows;
        valid = d_j * 32 + kPermCC[d_i] >= ndummy;
      }
      const uint64_t mask = __ballot(valid);
      const int r = base + __popcll(mask & ((1ull << lane) - 1ull));
      base += __popcll(mask);
      if (valid) {
        float acc = 10000.0f;
        for (int k = r; k < E; k += V) {
          const float x = es[k];
          if (acc == 10000.0f)
            acc = x;
          else if (x != 10000.0f)
            acc = __fadd_rn(acc, x);
        }
        tmp[j] = acc;
      }
    }
  }
  __syncthreads();
  if (!go) {
    if (lane == 0) decoded[ci] = 0;
    return;
  }
  for (int i = lane; i < out_len / 3; i += 64) {
    const int d_i = (i + ndummy) / 32, d_j = (i + ndummy) % 32;
    for (int s = 0; s < 3; s++) {
      const float o = tmp[K_p * s + kPermCCInv[d_j] * nrows + d_i];
      rm[i * 3 + s] = o != 10000.0f ? o : 0.0f;
    }
  }
  __syncthreads();
  vit_frame(rm, F, bits, q, dec);
  uint8_t *out = gmem(out_base + c.out_offset);
  for (int i = lane; i < F; i += 64) out[i] = bits[i];
  if (lane == 0) {
    uint32_t crc = 0;
    for (int i = 0; i < nbits; i++) {
      const uint32_t fb = ((crc >> 15) & 1u) ^ (bits[i] & 1u);
      crc = (crc << 1) & 0xFFFFu;
      if (fb) crc ^= 0x1021u;
    }
    uint32_t p = 0;
    for (int i = 0; i < 16; i++) p = (p << 1) | (bits[nbits + i] & 1u);
    crc_rem[ci] = (uint16_t)(p ^ crc);
    decoded[ci] = 1;
  }
}

} // namespace srsgpu

extern "C" int srsgpu_dci_decode_dev(const srsgpu_dci_cand_t *d_cands, uint32_t nof_cands,
                                     const float *d_llr, uint8_t *d_data, uint16_t *d_crc_rem,
                                     uint8_t *d_decoded, void *hip_stream) {
  if (!d_cands || !d_llr || !d_data || !d_crc_rem || !d_decoded) return -1;
  if (!nof_cands) return 0;
  hipLaunchKernelGGL(srsgpu::k_dci_decode, dim3(nof_cands), dim3(64), 0, (hipStream_t)hip_stream,
                     d_cands, (int)nof_cands, d_llr, d_data, d_crc_rem, d_decoded);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int srsgpu_viterbi37_tb_decode_f_dev(const srsgpu_viterbi_frame_t *d_frames,
                                                uint32_t nof_frames, const float *d_sym,
                                                uint8_t *d_out, void *hip_stream) {
  if (!d_frames || !d_sym || !d_out) return -1;
  if (!nof_frames) return 0;
  hipLaunchKernelGGL(srsgpu::k_viterbi37_tb, dim3(nof_frames), dim3(64), 0, (hipStream_t)hip_stream,
                     d_frames, (int)nof_frames, d_sym, d_out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
