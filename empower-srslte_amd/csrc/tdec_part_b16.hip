// Part 3 of the turbo-decoder kernels (tdec_kernels.hip): the int8 SSE8 window decoders (16 sub-blocks),
// per-half-iteration and fused launchers. A translation unit of its own so the library builds
// in parallel.
#define TD_PART 3
#include "tdec_kernels.hip"
