// Internal launch interface of the TM3 / TM4 feedback kernel (feedback_kernels.hip).
#ifndef SRSGPU_FEEDBACK_KERNELS_H
#define SRSGPU_FEEDBACK_KERNELS_H
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "srsgpu/pdsch_batch.h"

namespace srsgpu {

typedef srsgpu_feedback_t FbOut;

// one subframe: its estimate planes as the reference indexes them, h[port][rx antenna] (a missing
// rx antenna: null, read as zeros)
struct FbItem {
  const float2 *h[2][2];
  float noise;
  const float *noise_dev; // if set: the noise estimate is *noise_dev
  uint32_t flags, nof_ce; // SRSGPU_FEEDBACK_*; estimates per plane (SRSLTE_SF_LEN_RE)
  int nrx, nports;
  FbOut *out;
};

hipError_t launch_feedback(const FbItem *d_items, int n, hipStream_t st);

} // namespace srsgpu
#endif
