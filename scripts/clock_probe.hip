// Dev: effective shader clock with 1 busy wave vs all CUs busy: each wave runs a
// dependent FMA chain for a fixed number of iterations and records (s_memtime delta,
// s_memrealtime delta); core MHz = 100 * dtime / dreal.  Vector stores only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
__global__ void probe(double* out, long long iters, double seed) {
  double a = seed + threadIdx.x, b = 1.0000001;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (long long i = 0; i < iters; ++i) a = fma(a, b, 1e-9);
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    out[blockIdx.x * 3 + 0] = (double)(t1 - t0);
    out[blockIdx.x * 3 + 1] = (double)(r1 - r0);
    out[blockIdx.x * 3 + 2] = a;
  }
}
int main(int argc, char** argv) {
  long long iters = argc > 1 ? atoll(argv[1]) : 20000000;
  int grids[] = {1, 8, 256, 1024};
  double* d;
  hipMalloc(&d, 1024 * 3 * sizeof(double));
  double h[1024 * 3];
  for (int gi = 0; gi < 4; ++gi) {
    const int g = grids[gi];
    hipLaunchKernelGGL(probe, dim3(g), dim3(64), 0, 0, d, iters / 10, 1.0);  // warm
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(probe, dim3(g), dim3(64), 0, 0, d, iters, 1.0);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0; hipEventElapsedTime(&ms, e0, e1);
    hipMemcpy(h, d, g * 3 * sizeof(double), hipMemcpyDeviceToHost);
    printf("grid %5d: kernel %.2f ms, wave0 memtime %.0f realtime %.0f -> %.0f MHz (x100MHz ratio)\n", g, ms, h[0],
           h[1], 100.0 * h[0] / h[1]);
  }
  return 0;
}
