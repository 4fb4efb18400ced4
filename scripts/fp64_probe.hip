// Dev: fp64 latencies and hardware-estimate accuracy on one wave (gfx950), the inputs of
// the Riccati / forward-sweep restructure:
//   * dependent-chain cycles per fp64 FMA, v_rsq_f64, v_rcp_f64, v_frexp_mant_f64
//   * v_rsq_f64 / v_rcp_f64 raw estimates vs the correctly rounded value (ulp), and after
//     one and two Newton steps
//   * a readlane round trip (VALU -> SGPR -> VALU) and an LDS write -> wave barrier -> read
// Vector stores only.  usage: fp64_probe [iters]
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

template <int OP>
__global__ void chain(double* out, int iters, double seed) {
  __shared__ double sh[128];
  double a = seed + threadIdx.x * 1e-3;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    if constexpr (OP == 0) a = fma(a, 1.0000001, 1e-9);
    if constexpr (OP == 1) a = __builtin_amdgcn_rsq(a) + 0.5;
    if constexpr (OP == 2) a = __builtin_amdgcn_rcp(a) + 0.75;
    if constexpr (OP == 3) a = __builtin_amdgcn_frexp_mant(a * 1.7) + 0.25;
    if constexpr (OP == 4) {
      const int lo = __builtin_amdgcn_readlane(__double2loint(a), 3);
      const int hi = __builtin_amdgcn_readlane(__double2hiint(a), 3);
      a = __hiloint2double(hi, lo) * 1.0000001 + 1e-9;
    }
    if constexpr (OP == 5) {
      sh[threadIdx.x] = a;
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      a = sh[(threadIdx.x + 1) & 63] * 1.0000001 + 1e-9;
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
    if constexpr (OP == 6) a = a * 1.0000001;  // v_mul_f64
    if constexpr (OP == 7) a = a + 1e-9;        // v_add_f64
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[0] = (double)(t1 - t0) / iters; out[1] = a; }
}

__global__ void accuracy(const double* x, double* rs, double* rc, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  rs[i] = __builtin_amdgcn_rsq(x[i]);
  rc[i] = __builtin_amdgcn_rcp(x[i]);
}

static double ulp_err(double got, long double exact) {
  const double e = (double)exact;
  const double u = std::nextafter(std::fabs(e), INFINITY) - std::fabs(e);
  return (double)(std::fabs((long double)got - exact) / u);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 200000;
  double* d;
  hipMalloc(&d, 16 * sizeof(double));
  const char* names[] = {"fma_f64", "rsq_f64 (+add)", "rcp_f64 (+add)", "frexp_mant(mul) (+add)",
                         "readlane pair (+fma)", "ds_write/barrier/ds_read (+fma)", "mul_f64", "add_f64"};
  double h[2];
  auto run = [&](auto kern, int k) {
    hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, d, iters / 10, 1.3);
    hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, d, iters, 1.3);
    hipMemcpy(h, d, 2 * sizeof(double), hipMemcpyDeviceToHost);
    printf("%-36s %8.2f cycles per dependent step\n", names[k], h[0]);
  };
  run(chain<0>, 0); run(chain<1>, 1); run(chain<2>, 2); run(chain<3>, 3);
  run(chain<4>, 4); run(chain<5>, 5); run(chain<6>, 6); run(chain<7>, 7);
  const int n = 1 << 20;
  double *hx = (double*)malloc(n * 8), *hs = (double*)malloc(n * 8), *hc = (double*)malloc(n * 8);
  srand(7);
  for (int i = 0; i < n; ++i) hx[i] = std::ldexp(1.0 + (double)rand() / RAND_MAX, (rand() % 80) - 40);
  double *dx, *ds, *dc;
  hipMalloc(&dx, n * 8); hipMalloc(&ds, n * 8); hipMalloc(&dc, n * 8);
  hipMemcpy(dx, hx, n * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(accuracy, dim3(n / 256), dim3(256), 0, 0, dx, ds, dc, n);
  hipMemcpy(hs, ds, n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(hc, dc, n * 8, hipMemcpyDeviceToHost);
  double ms = 0, mc = 0, ms1 = 0, mc1 = 0, ms2 = 0, mc2 = 0;
  for (int i = 0; i < n; ++i) {
    const long double x = hx[i];
    const long double es = 1.0L / sqrtl(x), ec = 1.0L / x;
    ms = fmax(ms, ulp_err(hs[i], es));
    mc = fmax(mc, ulp_err(hc[i], ec));
    // one / two Newton steps as the kernel's rsq() / rcp() form them
    double y = hs[i], hh = 0.5 * hx[i];
    double r = fma(-hh * y, y, 0.5); y = fma(y, r, y);
    ms1 = fmax(ms1, ulp_err(y, es));
    r = fma(-hh * y, y, 0.5); y = fma(y, r, y);
    ms2 = fmax(ms2, ulp_err(y, es));
    double z = hc[i], e = fma(-hx[i], z, 1.0); z = fma(z, e, z);
    mc1 = fmax(mc1, ulp_err(z, ec));
    e = fma(-hx[i], z, 1.0); z = fma(z, e, z);
    mc2 = fmax(mc2, ulp_err(z, ec));
  }
  printf("v_rsq_f64 raw max %.3g ulp; one Newton step %.3g; two %.3g\n", ms, ms1, ms2);
  printf("v_rcp_f64 raw max %.3g ulp; one Newton step %.3g; two %.3g\n", mc, mc1, mc2);
  return 0;
}
