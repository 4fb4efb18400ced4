// Dev: does qd(a, b) (the fdiv sequence without v_div_scale / v_div_fmas / v_div_fixup,
// nmpc_solve.hip) return a / b bit for bit?  Random operands over wide exponent ranges,
// plus the kernel's typical shapes (mu / slack, tau * slack / step).  Vector stores only.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
__device__ __forceinline__ double qd(double a, double b) {
  double r = __builtin_amdgcn_rcp(b);
  double e = fma(-b, r, 1.0);
  r = fma(r, e, r);
  e = fma(-b, r, 1.0);
  r = fma(r, e, r);
  const double q = a * r;
  return fma(fma(-b, q, a), r, q);
}
__global__ void cmp(const double* a, const double* b, unsigned long long* bad, double* ex, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double x = a[i] / b[i], y = qd(a[i], b[i]);
  unsigned long long ux, uy;
  memcpy(&ux, &x, 8); memcpy(&uy, &y, 8);
  if (ux != uy) {
    const unsigned long long k = atomicAdd(bad, 1ull);
    if (k < 8) { ex[4 * k] = a[i]; ex[4 * k + 1] = b[i]; ex[4 * k + 2] = x; ex[4 * k + 3] = y; }
  }
}
int main() {
  const int n = 1 << 22;
  double *ha = (double*)malloc(n * 8), *hb = (double*)malloc(n * 8);
  srand(3);
  for (int t = 0; t < 3; ++t) {
    for (int i = 0; i < n; ++i) {
      const double u = (double)rand() / RAND_MAX, v = (double)rand() / RAND_MAX;
      if (t == 0) { ha[i] = std::ldexp(1.0 + u, rand() % 120 - 60) * (rand() & 1 ? 1 : -1);
                    hb[i] = std::ldexp(1.0 + v, rand() % 120 - 60) * (rand() & 1 ? 1 : -1); }
      if (t == 1) { ha[i] = 1.0; hb[i] = std::ldexp(1.0 + v, rand() % 80 - 40); }
      if (t == 2) { ha[i] = -0.99 * std::ldexp(1.0 + u, rand() % 40 - 30); hb[i] = -std::ldexp(1.0 + v, rand() % 40 - 30); }
    }
    double *da, *db, *dex; unsigned long long* dbad;
    hipMalloc(&da, n * 8); hipMalloc(&db, n * 8); hipMalloc(&dex, 32 * 8); hipMalloc(&dbad, 8);
    hipMemcpy(da, ha, n * 8, hipMemcpyHostToDevice); hipMemcpy(db, hb, n * 8, hipMemcpyHostToDevice);
    hipMemset(dbad, 0, 8);
    hipLaunchKernelGGL(cmp, dim3(n / 256), dim3(256), 0, 0, da, db, dbad, dex, n);
    unsigned long long bad = 0; double ex[32];
    hipMemcpy(&bad, dbad, 8, hipMemcpyDeviceToHost); hipMemcpy(ex, dex, 32 * 8, hipMemcpyDeviceToHost);
    printf("set %d: %llu of %d quotients differ from a / b\n", t, bad, n);
    for (int k = 0; k < (bad < 8 ? (int)bad : 8); ++k)
      printf("  a %.17g b %.17g  a/b %.17g  qd %.17g\n", ex[4 * k], ex[4 * k + 1], ex[4 * k + 2], ex[4 * k + 3]);
  }
  return 0;
}
