// Microbenchmark: issue rate of unpacked 16-bit VOP3 ops (v_add_i16 clamp, v_max_i16, v_max3_i16,
// op_sel high-half forms) vs packed ones at 1 / 2 / 4 waves per SIMD and ILP 1 / 2 / 4 / 8.
// Build: hipcc -O3 --offload-arch=gfx950 vrate16.hip -o vrate16 (tools/dbg/, not shipped).
#include <hip/hip_runtime.h>
#include <cstdio>
template <int ILP, int OP>
__global__ __launch_bounds__(256) void kd(int *out, int iters, int seed) {
  int a[ILP];
  for (int i = 0; i < ILP; i++) a[i] = seed + threadIdx.x * 7 + i;
  const int b = seed * 3, c = seed * 5;
  long long t0 = clock64();
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int r = 0; r < 64 / ILP; r++)
#pragma unroll
      for (int i = 0; i < ILP; i++) {
        if (OP == 0) asm volatile("v_pk_add_i16 %0, %0, %1 clamp" : "+v"(a[i]) : "v"(b));
        if (OP == 1) asm volatile("v_add_i16 %0, %0, %1 clamp" : "+v"(a[i]) : "v"(b));
        if (OP == 2) asm volatile("v_max_i16_e64 %0, %0, %1" : "+v"(a[i]) : "v"(b));
        if (OP == 3) asm volatile("v_max3_i16 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
        if (OP == 4) asm volatile("v_add_i16 %0, %0, %1 op_sel:[1,0,1] clamp" : "+v"(a[i]) : "v"(b));
        if (OP == 5) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
        if (OP == 6) asm volatile("v_max_i32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
        if (OP == 7) asm volatile("v_pk_max_i16 %0, %0, %1" : "+v"(a[i]) : "v"(b));
      }
  }
  long long t1 = clock64();
  int acc = 0;
  for (int i = 0; i < ILP; i++) acc ^= a[i];
  if (acc == 12345) out[0] = 1;
  if (threadIdx.x == 0) out[1 + blockIdx.x] = (int)(t1 - t0);
}
template <int ILP, int OP> void run(int *d, const char *name) {
  const int iters = 200;
  for (int wps : {1, 2, 4}) {
    const int blocks = 256 * wps;
    float ms = 0;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int rep = 0; rep < 2; rep++) {
      (void)hipEventRecord(e0);
      hipLaunchKernelGGL((kd<ILP, OP>), dim3(blocks), dim3(256), 0, 0, d, iters, 1);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      (void)hipEventElapsedTime(&ms, e0, e1);
    }
    const double n = (double)iters * (64 / ILP) * ILP;
    printf("%-26s ILP %d waves/SIMD %d: %.2f ns per instr per SIMD\n", name, ILP, wps, ms * 1e6 / (n * wps));
  }
}
#define ALL(OP, name)                                                                              \
  run<1, OP>(d, name);                                                                             \
  run<2, OP>(d, name);                                                                             \
  run<4, OP>(d, name);                                                                             \
  run<8, OP>(d, name);
int main() {
  int *d;
  (void)hipMalloc(&d, 4 * 4096);
  ALL(0, "v_pk_add_i16 clamp")
  ALL(7, "v_pk_max_i16")
  ALL(1, "v_add_i16 clamp")
  ALL(2, "v_max_i16")
  ALL(3, "v_max3_i16")
  ALL(4, "v_add_i16 op_sel hi clamp")
  ALL(5, "v_add_u32")
  ALL(6, "v_max_i32")
  return 0;
}
