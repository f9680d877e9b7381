// filter_check.hip -- test harness for the solve kernel's filter (mpc-verde_amd/csrc/kernels.h
// FilterLds): each lane group runs a sequence of (membership test, add) operations on its own
// filter, exactly as the solve loop calls them, and lane 0 records the outcomes.  Built into
// tests/hip/libfilter_check.so (tests/hip/Makefile); used by tests/test_gpu_filter.py only.
#include "kernels.h"

namespace mpcx {

template <int G>
__global__ __launch_bounds__(G > 64 ? G : 64) void filter_check_kernel(int groups, int n_ops, const double* th,
                                                                       const double* ph, const double* qth,
                                                                       const double* qph, int* covered, int* ovf) {
  __shared__ double xch[2 * XWave<G>::W * kXchStride];
  __shared__ double fbuf[FilterLds<G>::kDoubles];
  XWave<G> xw{xch, 0};
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int k = (int)(gid & (G - 1));
  const long g = gid / G;
  const long gs = g < groups ? g : groups - 1;  // surplus lanes of the last block repeat a group
  FilterLds<G> f;
  f.init(fbuf + threadIdx.x);
  for (int i = 0; i < n_ops; ++i) {
    const long o = gs * n_ops + i;
    const bool c = f.contains(qth[o], qph[o], xw);
    const bool v = f.add(th[o], ph[o], k, xw);
    if (k == 0 && g < groups) {
      covered[o] = c;
      ovf[o] = v;
    }
  }
}

template <int G>
static int launch(int groups, int n_ops, const double* th, const double* ph, const double* qth, const double* qph,
                  int* covered, int* ovf) {
  const int bs = G > 64 ? G : 64;
  const long threads = (long)groups * G;
  const int blocks = (int)((threads + bs - 1) / bs);
  hipLaunchKernelGGL((filter_check_kernel<G>), dim3(blocks), dim3(bs), 0, 0, groups, n_ops, th, ph, qth, qph, covered,
                     ovf);
  if (hipGetLastError() != hipSuccess) return -1;
  return hipDeviceSynchronize() == hipSuccess ? 0 : -2;
}

}  // namespace mpcx

// device pointers; returns 0 on success.  Slots per instance: filter_check_capacity(G).
extern "C" int filter_check_capacity(int G) {
  switch (G) {
    case 16: return mpcx::FilterLds<16>::kCap;
    case 32: return mpcx::FilterLds<32>::kCap;
    case 64: return mpcx::FilterLds<64>::kCap;
    case 128: return mpcx::FilterLds<128>::kCap;
    case 256: return mpcx::FilterLds<256>::kCap;
  }
  return -1;
}

extern "C" int filter_check(int G, int groups, int n_ops, const double* th, const double* ph, const double* qth,
                            const double* qph, int* covered, int* ovf) {
  if (groups <= 0 || n_ops <= 0) return -3;
  switch (G) {
    case 16: return mpcx::launch<16>(groups, n_ops, th, ph, qth, qph, covered, ovf);
    case 32: return mpcx::launch<32>(groups, n_ops, th, ph, qth, qph, covered, ovf);
    case 64: return mpcx::launch<64>(groups, n_ops, th, ph, qth, qph, covered, ovf);
    case 128: return mpcx::launch<128>(groups, n_ops, th, ph, qth, qph, covered, ovf);
    case 256: return mpcx::launch<256>(groups, n_ops, th, ph, qth, qph, covered, ovf);
  }
  return -3;
}
