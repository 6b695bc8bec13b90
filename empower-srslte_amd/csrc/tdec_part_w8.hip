// Part 2 of the turbo-decoder kernels (tdec_kernels.hip): the 16-bit SSE16 window decoders (8 sub-blocks) and the sequential SSE / generic decoders,
// per-half-iteration and fused launchers. A translation unit of its own so the library builds
// in parallel.
#define TD_PART 2
#include "tdec_kernels.hip"
