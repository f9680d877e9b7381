// stage_check.hip -- test harness for the unicycle stage derivatives of the solve kernel
// (mpc-verde_amd/csrc/unicycle.h): one thread per interval evaluates uni_derivs_moments (the
// weighted-moment assembly the solve kernel uses) and uni_derivs<true> (the per-point formula)
// at the same (x, u, x_ref, u_ref, lam, fs).  Built into tests/hip/libstage_check.so; used by
// tests/test_gpu_stage.py only.
#include "fastmath.h"
#include "models.h"
#include "riccati.h"
#include "unicycle.h"

namespace mpcx {

// out per interval: xf 3, q 1, A 9, B 6, g 5, H 15 (39 doubles), moments first, then per-point
__global__ void stage_check_kernel(int n, StageParams sp, const double* X, const double* U, const double* XR,
                                   const double* UR, const double* L, double fs, double* out, int which) {
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
    if (which != 0 && which != variant + 1) continue;  // 0: both; 1: moments only; 2: per-point only
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

// one backward Riccati step of the unicycle's chain per thread (the solve kernel's riccati_step
// with UnicycleModel's masks and unit entries).  in per thread: Hd 15, gp 5, A 9, B 6, c 3,
// P_{k+1} 6 (packed), p_{k+1} 3 (47 doubles); out: P_k 6, p_k 3, ok, K 6, kf 2 (18 doubles)
__global__ void riccati_check_kernel(int n, const double* in, double* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double* v = in + (size_t)i * 47;
  double Hd[15], gp[5], A[9], Bm[6], c[3], P[6], p[3];
  for (int j = 0; j < 15; ++j) Hd[j] = v[j];
  for (int j = 0; j < 5; ++j) gp[j] = v[15 + j];
  for (int j = 0; j < 9; ++j) A[j] = v[20 + j];
  for (int j = 0; j < 6; ++j) Bm[j] = v[29 + j];
  for (int j = 0; j < 3; ++j) c[j] = v[35 + j];
  for (int j = 0; j < 6; ++j) P[j] = v[38 + j];
  for (int j = 0; j < 3; ++j) p[j] = v[44 + j];
  // the structural entries the model's masks declare (A = I + a02 e0 e2^T + a12 e1 e2^T, B[2][0] = 0)
  A[0] = A[4] = A[8] = 1.0;
  A[1] = A[3] = A[6] = A[7] = 0.0;
  Bm[4] = 0.0;
  double Pn[6], pn[3], K[6], kf[2];
  Fac<3, 2> fac = {};
  const bool ok = riccati_step<3, 2, UnicycleModel::AMASK, UnicycleModel::BMASK, false, false, UnicycleModel::AONE>(
      Hd, gp, A, Bm, c, P, p, Pn, pn, fac);
  riccati_gains<3, 2>(fac, K, kf);
  double* o = out + (size_t)i * 18;
  for (int j = 0; j < 6; ++j) o[j] = Pn[j];
  for (int j = 0; j < 3; ++j) o[6 + j] = pn[j];
  o[9] = (ok && fac_ok<3, 2>(fac)) ? 1.0 : (ok || fac_ok<3, 2>(fac) ? 0.5 : 0.0);
  for (int j = 0; j < 6; ++j) o[10 + j] = K[j];
  for (int j = 0; j < 2; ++j) o[16 + j] = kf[j];
}

// the kernel's fp64 log and exp (fastmath.h): out[2 i] = log_fd(x_i), out[2 i + 1] = exp_fd(y_i)
__global__ void fastmath_check_kernel(int n, const double* x, const double* y, double* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[2 * i] = log_fd(x[i]);
  out[2 * i + 1] = exp_fd(y[i]);
}

}  // namespace mpcx

extern "C" int fastmath_check(int n, const double* x, const double* y, double* out) {
  if (n <= 0) return -3;
  hipLaunchKernelGGL(mpcx::fastmath_check_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, n, x, y, out);
  return hipDeviceSynchronize() == hipSuccess ? 0 : -2;
}

extern "C" int riccati_check(int n, const double* in, double* out) {
  if (n <= 0) return -3;
  hipLaunchKernelGGL(mpcx::riccati_check_kernel, dim3((n + 63) / 64), dim3(64), 0, 0, n, in, out);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return -1000 - (int)e;
  const hipError_t s = hipDeviceSynchronize();
  return s == hipSuccess ? 0 : -2000 - (int)s;
}

// device pointers; returns 0 on success.  out: 2 x n x 39 doubles.
extern "C" int stage_check_which(int n, double T, int M, int cost, const double* Q, const double* R, const double* X,
                                 const double* U, const double* XR, const double* UR, const double* L, double fs,
                                 double* out, int which) {
  if (n <= 0 || M < 1) return -3;
  mpcx::StageParams sp;
  sp.T = T;
  sp.M = M;
  sp.h = T / M;
  sp.cost = cost;
  for (int j = 0; j < 3; ++j) sp.Q[j] = Q[j];
  for (int j = 0; j < 2; ++j) sp.R[j] = R[j];
  hipLaunchKernelGGL(mpcx::stage_check_kernel, dim3((n + 63) / 64), dim3(64), 0, 0, n, sp, X, U, XR, UR, L, fs, out,
                     which);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return -1000 - (int)e;
  const hipError_t s = hipDeviceSynchronize();
  return s == hipSuccess ? 0 : -2000 - (int)s;
}

extern "C" int stage_check(int n, double T, int M, int cost, const double* Q, const double* R, const double* X,
                           const double* U, const double* XR, const double* UR, const double* L, double fs,
                           double* out) {
  return stage_check_which(n, T, M, cost, Q, R, X, U, XR, UR, L, fs, out, 0);
}
