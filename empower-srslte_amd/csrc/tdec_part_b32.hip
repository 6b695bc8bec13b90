// Part 4 of the turbo-decoder kernels (tdec_kernels.hip): the int8 AVX8 window decoders (32 sub-blocks),
// per-half-iteration and fused launchers. A translation unit of its own so the library builds
// in parallel.
#define TD_PART 4
#include "tdec_kernels.hip"
