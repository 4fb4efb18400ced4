// Dev tool: one-wave instruction latency / issue microbenchmark (s_memtime ticks) used for
// the per-stage cost estimates in DESIGN.md section 6.  hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <cstdio>
__device__ __forceinline__ long long mt() { long long t; asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t)); return t; }
__global__ void k(double* out, long long* cyc, double seed, int nw) {
  const int l = threadIdx.x;
  double a = seed + l, c = 1.0000001, d = 0.9999999;
  double a1 = a + 1, a2 = a + 2, a3 = a + 3, a4 = a + 4, a5 = a + 5, a6 = a + 6, a7 = a + 7;
  long long t0, t1;
  t0 = mt();
#pragma unroll
  for (int i = 0; i < 128; ++i) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a) : "v"(c), "v"(d));
  asm volatile("s_nop 0" :: "v"(a));
  t1 = mt();
  if (l == 0) cyc[0 + 16 * blockIdx.x] = t1 - t0;
  t0 = mt();
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a1) : "v"(c), "v"(d));
    asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a2) : "v"(c), "v"(d));
    asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a3) : "v"(c), "v"(d));
    asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a4) : "v"(c), "v"(d));
    asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a5) : "v"(c), "v"(d));
    asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a6) : "v"(c), "v"(d));
    asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a7) : "v"(c), "v"(d));
    asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a) : "v"(c), "v"(d));
  }
  t1 = mt();
  if (l == 0) cyc[1 + 16 * blockIdx.x] = t1 - t0;
  float f0 = a, f1 = a1, f2 = a2, f3 = a3;
  const float fc = 1.0000001f, fd = 0.99f;
  t0 = mt();
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(f0) : "v"(fc), "v"(fd));
    asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(f1) : "v"(fc), "v"(fd));
    asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(f2) : "v"(fc), "v"(fd));
    asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(f3) : "v"(fc), "v"(fd));
  }
  t1 = mt();
  if (l == 0) cyc[2 + 16 * blockIdx.x] = t1 - t0;
  double r = a + 3.0;
  t0 = mt();
#pragma unroll
  for (int i = 0; i < 64; ++i) asm volatile("v_rsq_f64 %0, %0" : "+v"(r));
  asm volatile("s_nop 0" :: "v"(r));
  t1 = mt();
  if (l == 0) cyc[3 + 16 * blockIdx.x] = t1 - t0;
  double e = a2;
  t0 = mt();
#pragma unroll
  for (int i = 0; i < 128; ++i) asm volatile("v_add_f64 %0, %0, %1" : "+v"(e) : "v"(d));
  asm volatile("s_nop 0" :: "v"(e));
  t1 = mt();
  if (l == 0) cyc[4 + 16 * blockIdx.x] = t1 - t0;
  int s0 = l, s1 = l + 1;
  t0 = mt();
#pragma unroll
  for (int i = 0; i < 128; ++i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(s0) : "v"(s1));
  asm volatile("s_nop 0" :: "v"(s0));
  t1 = mt();
  if (l == 0) cyc[5 + 16 * blockIdx.x] = t1 - t0;
  out[l + 64 * blockIdx.x] = a + a1 + a2 + a3 + a4 + a5 + a6 + a7 + r + e + f0 + f1 + f2 + f3 + s0;
}
int main() {
  double* out;
  long long* cyc;
  (void)hipMalloc(&out, 64 * 4096 * 8);
  (void)hipMalloc(&cyc, 16 * 4096 * 8);
  for (int nwv : {1, 1024, 2048}) {
    for (int rep = 0; rep < 3; ++rep) {
      hipLaunchKernelGGL(k, dim3(nwv), dim3(64), 0, 0, out, cyc, 1.5, nwv);
      (void)hipDeviceSynchronize();
    }
    long long h[16];
    (void)hipMemcpy(h, cyc, 6 * 8, hipMemcpyDeviceToHost);
    printf("waves=%d: dep fma64 %.2f | indep fma64 %.2f | indep fma32 %.2f | dep rsq64 %.2f | dep add64 %.2f | dep add_u32 %.2f cyc/op\n",
           nwv, h[0] / 128.0, h[1] / 128.0, h[2] / 128.0, h[3] / 64.0, h[4] / 128.0, h[5] / 128.0);
  }
  return 0;
}
