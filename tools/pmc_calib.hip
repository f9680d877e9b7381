// pmc_calib.hip -- calibrate rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for the access
// widths the sweep kernel uses (MI355X_MICROARCH.md §HBM: "other access widths are
// uncalibrated: calibrate on a known byte count in your own access pattern").
// Streams a 1 GiB buffer (far beyond the 256 MiB Infinity Cache) once with 8-B/lane and
// once with 16-B/lane loads, and writes 1 GiB with 8-B/lane stores.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void read8(const double* __restrict__ a, size_t n, double* out) {
  double s = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += a[i];
  if (s == 12345.678) out[0] = s;  // keep the loads alive
}
__global__ void read16(const double2* __restrict__ a, size_t n, double* out) {
  double s = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    double2 v = a[i];
    s += v.x + v.y;
  }
  if (s == 12345.678) out[0] = s;
}
__global__ void write8(double* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) a[i] = (double)i;
}

int main() {
  const size_t bytes = 1ull << 30, n = bytes / 8;
  double *a, *b, *o;
  if (hipMalloc(&a, bytes) || hipMalloc(&b, bytes) || hipMalloc(&o, 8)) return 1;
  (void)hipMemset(a, 0, bytes);
  for (int r = 0; r < 3; ++r) {
    hipLaunchKernelGGL(read8, dim3(8192), dim3(256), 0, 0, a, n, o);
    hipLaunchKernelGGL(read16, dim3(8192), dim3(256), 0, 0, (const double2*)a, n / 2, o);
    hipLaunchKernelGGL(write8, dim3(8192), dim3(256), 0, 0, b, n);
  }
  (void)hipDeviceSynchronize();
  printf("bytes per launch: %zu\n", bytes);
  return 0;
}
