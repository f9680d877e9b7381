// stage_check.hip -- test harness for the unicycle stage derivatives of the solve kernel
// (mpc-verde_amd/csrc/unicycle.h): one thread per interval evaluates uni_derivs_moments (the
// weighted-moment assembly the solve kernel uses) and uni_derivs<true> (the per-point formula)
// at the same (x, u, x_ref, u_ref, lam, fs).  Built into tests/hip/libstage_check.so; used by
// tests/test_gpu_stage.py only.
#include "unicycle.h"

namespace mpcx {

// out per interval: xf 3, q 1, A 9, B 6, g 5, H 15 (39 doubles), moments first, then per-point
__global__ void stage_check_kernel(int n, StageParams sp, const double* X, const double* U, const double* XR,
                                   const double* UR, const double* L, double fs, double* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double x[3], u[2], xr[3], ur[2], lam[3];
  for (int j = 0; j < 3; ++j) {
    x[j] = X[3 * i + j];
    xr[j] = XR[3 * i + j];
    lam[j] = L[3 * i + j];
  }
  for (int j = 0; j < 2; ++j) {
    u[j] = U[2 * i + j];
    ur[j] = UR[2 * i + j];
  }
  for (int variant = 0; variant < 2; ++variant) {
    double xf[3], q, A[9], Bm[6], g[5], H[15];
    if (variant == 0)
      uni_derivs_moments(sp, x, u, xr, ur, lam, fs, xf, q, A, Bm, g, H);
    else
      uni_derivs<true>(sp, x, u, xr, ur, lam, fs, xf, q, A, Bm, g, H);
    double* o = out + ((size_t)variant * n + i) * 39;
    for (int j = 0; j < 3; ++j) o[j] = xf[j];
    o[3] = q;
    for (int j = 0; j < 9; ++j) o[4 + j] = A[j];
    for (int j = 0; j < 6; ++j) o[13 + j] = Bm[j];
    for (int j = 0; j < 5; ++j) o[19 + j] = g[j];
    for (int j = 0; j < 15; ++j) o[24 + j] = H[j];
  }
}

}  // namespace mpcx

// device pointers; returns 0 on success.  out: 2 x n x 39 doubles.
extern "C" int stage_check(int n, double T, int M, int cost, const double* Q, const double* R, const double* X,
                           const double* U, const double* XR, const double* UR, const double* L, double fs,
                           double* out) {
  if (n <= 0 || M < 1) return -3;
  mpcx::StageParams sp;
  sp.T = T;
  sp.M = M;
  sp.h = T / M;
  sp.cost = cost;
  for (int j = 0; j < 3; ++j) sp.Q[j] = Q[j];
  for (int j = 0; j < 2; ++j) sp.R[j] = R[j];
  hipLaunchKernelGGL(mpcx::stage_check_kernel, dim3((n + 63) / 64), dim3(64), 0, 0, n, sp, X, U, XR, UR, L, fs, out);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return -1000 - (int)e;
  const hipError_t s = hipDeviceSynchronize();
  return s == hipSuccess ? 0 : -2000 - (int)s;
}
