// FETCH_SIZE / WRITE_SIZE calibration for the access widths the solver kernels issue
// (MI355X_MICROARCH.md, HBM section: the counters are calibrated only for 16 B/lane
// streaming reads; other widths must be calibrated on a known byte count).
// Each kernel streams a 1 GiB buffer (past the 256 MiB Infinity Cache) once, with
// 4, 8 or 16 B per lane, and writes a 256 MiB buffer with 8 B per lane.  Run under
//   rocprofv3 --pmc FETCH_SIZE -- ./fetch_calib      (and a WRITE_SIZE pass)
// and divide the counter (KB) by the bytes each kernel moved (printed).
#include <hip/hip_runtime.h>
#include <cstdio>

template <class T>
__global__ void rd(const T* __restrict__ a, size_t n, double* out) {
  T acc{};
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const T v = a[i];
    if constexpr (sizeof(T) == 16) acc.x += v.x; else acc += v;
  }
  double s;
  if constexpr (sizeof(T) == 16) s = (double)acc.x; else s = (double)acc;
  if (s != 0.0) out[0] = s;  // keep the loads (the buffer is zero)
}
__global__ void wr8(double* a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    a[i] = (double)i;
}

int main() {
  const size_t bytes = 1ull << 30, wbytes = 1ull << 28;
  void* buf;
  double* out;
  double* w;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 8) != hipSuccess ||
      hipMalloc(&w, wbytes) != hipSuccess) return 1;
  if (hipMemset(buf, 0, bytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return 1;
  const dim3 g(4096), b(256);
  rd<float><<<g, b>>>((const float*)buf, bytes / 4, out);
  rd<double><<<g, b>>>((const double*)buf, bytes / 8, out);
  rd<double2><<<g, b>>>((const double2*)buf, bytes / 16, out);
  wr8<<<g, b>>>(w, wbytes / 8);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("read kernels rd<float|double|double2>: %zu bytes each; write kernel wr8: %zu bytes\n", bytes, wbytes);
  return 0;
}
