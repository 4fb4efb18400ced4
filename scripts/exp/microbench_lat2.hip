// Dev tool: one-wave latencies of the operations on the Riccati stage's critical path
// (s_memtime ticks, one wave alone on the chip).  hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <cstdio>
__device__ __forceinline__ long long mt() { long long t; asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t)); return t; }
__global__ void k(double* out, long long* cyc, double seed) {
  __shared__ double lds[256];
  __shared__ int ldi[256];
  const int l = threadIdx.x;
  lds[l] = seed + l; lds[l + 64] = 1.0; ldi[l] = (l + 1) & 63; ldi[l + 64] = l;
  __syncthreads();
  long long t0, t1;
  // (0) dependent LDS load chain (pointer chasing through ints)
  int p = l;
  t0 = mt();
#pragma unroll
  for (int i = 0; i < 32; ++i) p = ldi[p];
  asm volatile("s_nop 0" :: "v"(p));
  t1 = mt();
  if (l == 0) cyc[0] = t1 - t0;
  // (1) LDS store -> load round trip of a double with a dependent fma
  double a = seed + l;
  t0 = mt();
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    lds[(l + i) & 127] = a;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    a = lds[(l + i + 1) & 127] * 1.0000001 + 0.5;
  }
  asm volatile("s_nop 0" :: "v"(a));
  t1 = mt();
  if (l == 0) cyc[1] = t1 - t0;
  // (2) readlane of a double + dependent fma
  double b = seed * l;
  t0 = mt();
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(b), i & 63);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(b), i & 63);
    b = fma(__hiloint2double(hi, lo), 1.0000001, b);
  }
  asm volatile("s_nop 0" :: "v"(b));
  t1 = mt();
  if (l == 0) cyc[2] = t1 - t0;
  // (3) dependent v_rcp_f64
  double r = seed + 3.0 + l;
  t0 = mt();
#pragma unroll
  for (int i = 0; i < 64; ++i) asm volatile("v_rcp_f64 %0, %0" : "+v"(r));
  asm volatile("s_nop 0" :: "v"(r));
  t1 = mt();
  if (l == 0) cyc[3] = t1 - t0;
  // (4) dependent DPP row_half_mirror move of a double + add (one butterfly step)
  double c = seed + l;
  t0 = mt();
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(c), 0x141, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(c), 0x141, 0xF, 0xF, false);
    c = c + __hiloint2double(hi, lo);
  }
  asm volatile("s_nop 0" :: "v"(c));
  t1 = mt();
  if (l == 0) cyc[4] = t1 - t0;
  // (5) dependent permlane32_swap step of a double + add
  double e = seed + l;
  t0 = mt();
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    const auto lo = __builtin_amdgcn_permlane32_swap(__double2loint(e), __double2loint(e), false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap(__double2hiint(e), __double2hiint(e), false, false);
    e = __hiloint2double(hi[0], lo[0]) + __hiloint2double(hi[1], lo[1]);
  }
  asm volatile("s_nop 0" :: "v"(e));
  t1 = mt();
  if (l == 0) cyc[5] = t1 - t0;
  // (6) LDS broadcast read of 8 doubles (independent) after a store, then use
  double g = seed;
  t0 = mt();
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    lds[l] = g;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    double s8 = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) s8 += lds[(q * 7 + i) & 63];
    g = s8 * 0.125;
  }
  asm volatile("s_nop 0" :: "v"(g));
  t1 = mt();
  if (l == 0) cyc[6] = t1 - t0;
  // (7) dependent v_sqrt_f64
  double q = seed + 5.0 + l;
  t0 = mt();
#pragma unroll
  for (int i = 0; i < 64; ++i) asm volatile("v_sqrt_f64 %0, %0" : "+v"(q));
  asm volatile("s_nop 0" :: "v"(q));
  t1 = mt();
  if (l == 0) cyc[7] = t1 - t0;
  // (8) dependent v_mul_f64
  double m = seed + l;
  t0 = mt();
#pragma unroll
  for (int i = 0; i < 128; ++i) asm volatile("v_mul_f64 %0, %0, %0" : "+v"(m));
  asm volatile("s_nop 0" :: "v"(m));
  t1 = mt();
  if (l == 0) cyc[8] = t1 - t0;
  out[l] = a + b + r + c + e + g + p + q + m;
}
int main() {
  double* out;
  long long* cyc;
  (void)hipMalloc(&out, 64 * 8);
  (void)hipMalloc(&cyc, 16 * 8);
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, out, cyc, 1.5);
    (void)hipDeviceSynchronize();
  }
  long long h[16];
  (void)hipMemcpy(h, cyc, 9 * 8, hipMemcpyDeviceToHost);
  printf("lds dep load %.1f | lds st->ld->fma %.1f | readlane64+fma %.1f | rcp64 %.1f | dpp64+add %.1f | "
         "permlane32 64+add %.1f | st+8 ld+sum %.1f | sqrt64 %.1f | mul64 %.1f cyc/op\n",
         h[0] / 32.0, h[1] / 32.0, h[2] / 32.0, h[3] / 64.0, h[4] / 32.0, h[5] / 32.0, h[6] / 16.0, h[7] / 64.0,
         h[8] / 128.0);
  return 0;
}
