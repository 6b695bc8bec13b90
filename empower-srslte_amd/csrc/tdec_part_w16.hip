// Part 1 of the turbo-decoder kernels (tdec_kernels.hip): the 16-bit AVX16 window decoders (16 sub-blocks),
// per-half-iteration and fused launchers. A translation unit of its own so the library builds
// in parallel.
#define TD_PART 1
#include "tdec_kernels.hip"
