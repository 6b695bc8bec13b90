// Microbenchmark: issue interval of packed int16 VALU ops at one wave per SIMD as a function of
// the dependency distance (ILP = number of independent chains interleaved), plus a few other
// instructions the decoder issues. Build: hipcc -O3 --offload-arch=gfx950 vdep.hip -o vdep
#include <hip/hip_runtime.h>
#include <cstdio>
template <int ILP, int OP>
__global__ __launch_bounds__(256) void kd(int *out, int iters, int seed) {
  int a[ILP];
  for (int i = 0; i < ILP; i++) a[i] = seed + threadIdx.x * 7 + i;
  const int b = seed * 3;
  long long t0 = clock64();
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int r = 0; r < 64 / ILP; r++)
#pragma unroll
      for (int i = 0; i < ILP; i++) {
        if (OP == 0) asm volatile("v_pk_add_i16 %0, %0, %1 clamp" : "+v"(a[i]) : "v"(b));
        if (OP == 1) asm volatile("v_pk_max_i16 %0, %0, %1" : "+v"(a[i]) : "v"(b));
        if (OP == 2) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
        if (OP == 3) asm volatile("v_mov_b32 %0, %1" : "=v"(a[i]) : "v"(a[(i + 1) % ILP]));
        if (OP == 4) asm volatile("s_nop 0\n v_pk_add_i16 %0, %0, %1 clamp" : "+v"(a[i]) : "v"(b));
        if (OP == 5) asm volatile("v_pk_max_i16 %0, %0, %1\n v_pk_add_i16 %0, %0, %1 clamp" : "+v"(a[i]) : "v"(b));
      }
  }
  long long t1 = clock64();
  int acc = 0;
  for (int i = 0; i < ILP; i++) acc ^= a[i];
  if (acc == 12345) out[0] = 1;
  if (threadIdx.x == 0) out[1 + blockIdx.x] = (int)(t1 - t0);
}
template <int ILP, int OP> void run(int *d, const char *name, int per_iter_instr) {
  const int iters = 200;
  const int blocks = 256; // 256 CUs x 4 SIMDs x 1 wave
  float ms = 0;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 2; rep++) {
    hipEventRecord(e0);
    hipLaunchKernelGGL((kd<ILP, OP>), dim3(blocks), dim3(256), 0, 0, d, iters, 1);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
  }
  int cyc;
  hipMemcpy(&cyc, d + 1, 4, hipMemcpyDeviceToHost);
  const double n = (double)iters * per_iter_instr;
  printf("%-34s ILP %d: %.2f ns per instr, %.2f cycles per instr (1 wave/SIMD)\n", name, ILP,
         ms * 1e6 / n, cyc / n);
}
int main() {
  int *d;
  hipMalloc(&d, 4 * 4096);
  run<1, 0>(d, "v_pk_add_i16 clamp", 64);
  run<2, 0>(d, "v_pk_add_i16 clamp", 64);
  run<3, 0>(d, "v_pk_add_i16 clamp", 63);
  run<4, 0>(d, "v_pk_add_i16 clamp", 64);
  run<8, 0>(d, "v_pk_add_i16 clamp", 64);
  run<1, 1>(d, "v_pk_max_i16", 64);
  run<2, 1>(d, "v_pk_max_i16", 64);
  run<4, 1>(d, "v_pk_max_i16", 64);
  run<1, 2>(d, "v_add_u32", 64);
  run<2, 2>(d, "v_add_u32", 64);
  run<8, 2>(d, "v_add_u32", 64);
  run<8, 3>(d, "v_mov_b32", 64);
  run<8, 4>(d, "s_nop 0 + v_pk_add (per pair)", 64);
  run<1, 5>(d, "pk_max->pk_add alternating dep", 128);
  run<4, 5>(d, "pk_max->pk_add alternating", 128);
  return 0;
}
