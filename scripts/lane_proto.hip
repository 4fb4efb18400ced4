// Dev prototype: lane utilisation of the stage-parallel passes.  The
// product runs one scenario per wave, so the stage-parallel phases (rollout, stage costs,
// rows; lane k = stage k, N + 1 = 21 of 64 lanes busy) leave 2/3 of every wave idle.
// This measures those two phases -- the rollout (prefix sums + sin/cos, as
// Solver::rollout) and the stage cost + obstacle rows (as Solver::eval_fg) -- with SPW = 1
// or 2 scenarios per wave (lanes 0..31 / 32..63), each wave repeating them ITERS times,
// at the product's occupancy (40 KB of LDS per wave: one wave per SIMD).  Reported: the
// wave's latency per repetition and the throughput in scenario-repetitions per second.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
constexpr int N = 20, NOBS = 10, NB = 5, M = NB + NOBS;
constexpr int LDS_DOUBLES = 5120;  // 40 KB per wave, as the LDS-row class
__device__ __forceinline__ void wsync() { __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); __builtin_amdgcn_wave_barrier(); __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront"); }
template <int SPW>
__global__ __launch_bounds__(64, 1) void proto(const double* __restrict__ U, const double* __restrict__ P, double* out,
                                               int B, int iters, double T) {
  extern __shared__ double sm[];
  const int lane = threadIdx.x;
  const int half = SPW == 2 ? lane >> 5 : 0;
  const int k = SPW == 2 ? lane & 31 : lane;  // stage
  const int b = blockIdx.x * SPW + half;
  if (b >= B) return;
  double* inc = sm + half * 512;           // 8 * (N + 1)
  double* X = sm + half * 512 + 256;       // 8 * (N + 1)
  const double* Ub = U + (long long)b * 6 * N;
  const double* Pb = P + (long long)b * 32;
  double acc = 0.0;
  for (int it = 0; it < iters; ++it) {
    const double a_shift = 1e-9 * it;
    // ---- rollout (Solver::rollout): angle increments, per-lane in-order prefix sums
    if (k < N) {
#pragma unroll
      for (int c = 0; c < 5; ++c) inc[k * 8 + c] = T * (Ub[k * 6 + 1 + c] + a_shift);
    }
    wsync();
    double a[5];
    double v = k < N ? Ub[k * 6] : 0.0;
    if (k <= N) {
#pragma unroll
      for (int c = 0; c < 5; ++c) a[c] = Pb[3 + c];
#pragma unroll
      for (int j = 0; j < N; ++j)
        if (j < k) {
#pragma unroll
          for (int c = 0; c < 5; ++c) a[c] = a[c] + inc[j * 8 + c];
        }
      if (k < N) {
        const double ct = cos(a[0]), st = sin(a[0]), cp = cos(a[1]), sp = sin(a[1]);
        inc[k * 8 + 5] = T * (v * cp * ct);
        inc[k * 8 + 6] = T * (v * sp * ct);
        inc[k * 8 + 7] = T * (v * st);
      }
    }
    wsync();
    if (k <= N) {
      double c0 = Pb[0], c1 = Pb[1], c2 = Pb[2];
#pragma unroll
      for (int j = 0; j < N; ++j)
        if (j < k) { c0 = c0 + inc[j * 8 + 5]; c1 = c1 + inc[j * 8 + 6]; c2 = c2 + inc[j * 8 + 7]; }
      double* xk = X + k * 8;
      xk[0] = c0; xk[1] = c1; xk[2] = c2;
#pragma unroll
      for (int c = 0; c < 5; ++c) xk[3 + c] = a[c];
    }
    wsync();
    // ---- stage cost and rows (Solver::stage_cost / row_value)
    if (k <= N) {
      const double* x = X + k * 8;
      const double hv = 0.3, hh = 0.4, z = x[2];
      if (k < N) {
        const double aa = (z * tan(x[6] + hv) - z * tan(x[6] - hv)) / 2;
        const double bb = (z * tan(x[5] + hh) - z * tan(x[5] - hh)) / 2;
        const double c7 = cos(x[7]), s7 = sin(x[7]);
        const double a2 = aa * aa, b2 = bb * bb;
        const double A = (c7 * c7) / a2 + (s7 * s7) / b2;
        const double Bq = 2 * c7 * s7 * ((1 / a2) - (1 / b2));
        const double C = (s7 * s7) / a2 + (c7 * c7) / b2;
        const double XE = x[0] + aa + z * tan(x[6] - hv), YE = x[1] + bb + z * tan(x[5] - hh);
        const double ex = Pb[8] - XE, ey = Pb[9] - YE, dx = x[0] - Pb[8], dy = x[1] - Pb[9];
        acc += sqrt(dx * dx + dy * dy) + ((A * (ex * ex) + Bq * ey * ex + C * (ey * ey)) - 1);
      }
#pragma unroll
      for (int o = 0; o < NOBS; ++o) {
        const double ddx = x[0] - Pb[12 + o], ddy = x[1] - Pb[22 + o];
        acc += -sqrt(ddx * ddx + ddy * ddy) + 5.0;
      }
    }
    wsync();
  }
  if (k <= N) out[(long long)b * 32 + k] = acc;
}
template <int SPW>
static void run(int B, int iters, const double* dU, const double* dP, double* dO, int ncu) {
  const int waves = (B + SPW - 1) / SPW;
  hipFuncSetAttribute((const void*)proto<SPW>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_DOUBLES * 8);
  hipLaunchKernelGGL(proto<SPW>, dim3(waves), dim3(64), LDS_DOUBLES * 8, 0, dU, dP, dO, B, 2, 0.2);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(proto<SPW>, dim3(waves), dim3(64), LDS_DOUBLES * 8, 0, dU, dP, dO, B, iters, 0.2);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0; hipEventElapsedTime(&ms, e0, e1);
  const double rounds = (double)waves / (4.0 * ncu) < 1 ? 1 : (double)waves / (4.0 * ncu);
  printf("SPW %d  B %6d  waves %6d  kernel %8.2f ms  wave latency per repetition %7.2f us  "
         "throughput %8.3f M scenario-repetitions/s\n", SPW, B, waves, ms, 1e3 * ms / iters / rounds,
         (double)B * iters / (ms * 1e-3) / 1e6);
}
int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 200;
  hipDeviceProp_t prop; hipGetDeviceProperties(&prop, 0);
  const int ncu = prop.multiProcessorCount;
  const int Bmax = 8192;
  std::vector<double> U((size_t)Bmax * 6 * N), P((size_t)Bmax * 32);
  for (size_t i = 0; i < U.size(); ++i) U[i] = 0.01 * ((i * 7919) % 13) - 0.05 + (i % 6 == 0 ? 12.0 : 0.0);
  for (int b = 0; b < Bmax; ++b) {
    double* p = &P[(size_t)b * 32];
    p[0] = 90 + b % 7; p[1] = 150; p[2] = 80; for (int c = 3; c < 8; ++c) p[c] = 0.01 * c;
    p[8] = 100; p[9] = 150; for (int o = 0; o < NOBS; ++o) { p[12 + o] = 200 + 30 * o; p[22 + o] = 100 + 10 * o; }
  }
  double *dU, *dP, *dO;
  hipMalloc(&dU, U.size() * 8); hipMalloc(&dP, P.size() * 8); hipMalloc(&dO, (size_t)Bmax * 32 * 8);
  hipMemcpy(dU, U.data(), U.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(dP, P.data(), P.size() * 8, hipMemcpyHostToDevice);
  for (int B : {1024, 2048, 4096, 8192}) { run<1>(B, iters, dU, dP, dO, ncu); run<2>(B, iters, dU, dP, dO, ncu); }
  return 0;
}
