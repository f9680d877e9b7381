// bcast_check.hip -- test harness for collectives.h matvec_bcast (the config-5 suffix scan's
// mat-vec by row-broadcast FMAs): per 64-lane wave, a block-uniform NX x NX matrix M spread over
// each 16-lane row as the scan holds it (lane r: M[r], M[16 + r]) applied to each lane's own
// vector, beside the plain fma loop over M read from memory.  Built into
// tests/hip/libbcast_check.so (tests/hip/Makefile); used by tests/test_gpu_bcast.py only.
#include "kernels.h"

namespace mpcx {

template <int NX>
__global__ __launch_bounds__(64) void bcast_check_kernel(const double* M, const double* w, const double* acc0,
                                                         double* out_bcast, double* out_plain) {
  const int t = (int)threadIdx.x;
  const double* Mb = M + (size_t)blockIdx.x * NX * NX;  // this wave's matrix
  const long base = ((long)blockIdx.x * 64 + t) * NX;
  double wl[NX], a[NX], p[NX];
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    wl[i] = w[base + i];
    a[i] = acc0[base + i];
    p[i] = a[i];
  }
  const int r = t & 15;
  const double mA = Mb[r];
  const double mB = NX * NX > 16 ? Mb[16 + min(r, NX * NX - 17)] : 0.0;
  matvec_bcast<NX>(a, wl, mA, mB);
#pragma unroll
  for (int i = 0; i < NX; ++i)
#pragma unroll
    for (int j = 0; j < NX; ++j) p[i] = fma(Mb[i * NX + j], wl[j], p[i]);
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    out_bcast[base + i] = a[i];
    out_plain[base + i] = p[i];
  }
}

}  // namespace mpcx

extern "C" int bcast_check(int nx, int waves, const double* M, const double* w, const double* acc0, double* out_bcast,
                           double* out_plain) {
  if (waves <= 0) return 1;
  if (nx == 4)
    hipLaunchKernelGGL((mpcx::bcast_check_kernel<4>), dim3(waves), dim3(64), 0, 0, M, w, acc0, out_bcast, out_plain);
  else if (nx == 5)
    hipLaunchKernelGGL((mpcx::bcast_check_kernel<5>), dim3(waves), dim3(64), 0, 0, M, w, acc0, out_bcast, out_plain);
  else
    return 2;
  return hipDeviceSynchronize() == hipSuccess ? 0 : 3;
}
