// Microbenchmark: issue rate of the decoder's packed int16 VALU ops on gfx950 at
// 1, 2 and 4 waves per SIMD, 8 independent dependency chains per wave, via inline asm so nothing
// folds. Build: hipcc -O3 --offload-arch=gfx950 vrate.hip -o vrate (tools/dbg/, not shipped).
#include <hip/hip_runtime.h>
#include <cstdio>
template <int OP>
__global__ __launch_bounds__(256) void kv(int *out, int iters, int seed) {
  int a[8];
  for (int i = 0; i < 8; i++) a[i] = seed + threadIdx.x * 7 + i;
  const int b = seed * 3;
  long long t0 = clock64();
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int r = 0; r < 16; r++)
#pragma unroll
      for (int i = 0; i < 8; i++) {
        if (OP == 0) asm volatile("v_pk_add_i16 %0, %0, %1 clamp" : "+v"(a[i]) : "v"(b));
        if (OP == 1) asm volatile("v_pk_max_i16 %0, %0, %1" : "+v"(a[i]) : "v"(b));
        if (OP == 2) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[i]) : "v"(b));
        if (OP == 3) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
        if (OP == 4) asm volatile("v_pk_add_i16 %0, %0, %1 op_sel:[0,1] op_sel_hi:[1,0] clamp" : "+v"(a[i]) : "v"(b));
      }
  }
  long long t1 = clock64();
  int acc = 0;
  for (int i = 0; i < 8; i++) acc ^= a[i];
  if (acc == 12345) out[0] = 1;
  if (threadIdx.x == 0) out[1 + blockIdx.x] = (int)(t1 - t0);
}
template <int OP> void run(int *d, const char *name) {
  const int iters = 400;
  for (int wps : {1, 2, 4}) {
    const int blocks = 256 * wps; // 256 CUs x 4 SIMDs x wps waves, 4 waves per block
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float ms = 0;
    for (int rep = 0; rep < 2; rep++) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(kv<OP>, dim3(blocks), dim3(256), 0, 0, d, iters, 1);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      hipEventElapsedTime(&ms, e0, e1);
    }
    int cyc;
    hipMemcpy(&cyc, d + 1, 4, hipMemcpyDeviceToHost);
    const double per_wave = (double)iters * 16 * 8;
    printf("%-28s waves/SIMD %d: %.2f ns per instr per SIMD, %.2f clock64 cycles per instr per wave\n",
           name, wps, ms * 1e6 / (per_wave * wps), cyc / per_wave);
  }
}
int main() {
  int *d;
  hipMalloc(&d, 4 * 4096);
  run<0>(d, "v_pk_add_i16 clamp");
  run<1>(d, "v_pk_max_i16");
  run<2>(d, "v_pk_add_u16");
  run<3>(d, "v_add_u32");
  run<4>(d, "v_pk_add_i16 clamp op_sel");
  return 0;
}
