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
#include "viterbi_dev.h"

namespace srsgpu {

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
