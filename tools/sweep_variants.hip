// sweep_variants.hip -- timing of rk4_sens_kernel store/occupancy variants (tools/, not product).
//   v8     : 24 nontemporal 8-B stores per stage (one field per lane per instruction)
//   v16    : 12 nontemporal 16-B stores per stage (field pairs), compiler's register choice
//   v16w4  : as v16 with amdgpu_waves_per_eu(4) (<= 128 VGPRs)
// B = 2^19 instances, N = 20, M = 4, T = 0.2; results are cross-checked (v16 == v8 bitwise).
// hipcc --offload-arch=gfx950 -O3 -I mpc-verde_amd/csrc tools/sweep_variants.hip -o tools/sweep_variants
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "unicycle.h"
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
using namespace mpcx;
typedef double v2d __attribute__((ext_vector_type(2)));
__device__ __forceinline__ size_t tix(int stage, int F, int i, long b, long T) {
  return (((size_t)stage * T + (b >> 6)) * F + i) * 64 + (b & 63);
}
template <bool PAIRS>
__device__ __forceinline__ void body(int B, int N, const StageParams& sp, const double* __restrict__ X,
                                     const double* __restrict__ U, const double* __restrict__ XR, double* __restrict__ J) {
  const long b = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const long T = ((long)B + 63) / 64;
  double x[3], xr[3];
  const double ur[2] = {0.0, 0.0};
  const double lz[3] = {0, 0, 0};
  for (int i = 0; i < 3; ++i) { x[i] = X[tix(0, 3, i, b, T)]; xr[i] = XR[tix(0, 3, i, b, T)]; }
  for (int k = 0; k < N; ++k) {
    double u[2], xn[3];
    for (int i = 0; i < 3; ++i) xn[i] = X[tix(k + 1, 3, i, b, T)];
    for (int i = 0; i < 2; ++i) u[i] = U[tix(k, 2, i, b, T)];
    double xf[3], q, A[9], Bm[6], g[5], H[15];
    uni_derivs<false>(sp, x, u, xr, ur, lz, 1.0, xf, q, A, Bm, g, H);
    double r[24];
    for (int i = 0; i < 3; ++i) r[i] = xf[i] - xn[i];
    r[3] = q;
    for (int i = 0; i < 9; ++i) r[4 + i] = A[i];
    for (int i = 0; i < 6; ++i) r[13 + i] = Bm[i];
    for (int i = 0; i < 5; ++i) r[19 + i] = g[i];
    if (PAIRS) {
      v2d* J2 = reinterpret_cast<v2d*>(J);
#pragma unroll
      for (int j = 0; j < 12; ++j) {
        const v2d v = {r[2 * j], r[2 * j + 1]};
        __builtin_nontemporal_store(v, &J2[tix(k, 12, j, b, T)]);
      }
    } else {
#pragma unroll
      for (int f = 0; f < 24; ++f) __builtin_nontemporal_store(r[f], &J[tix(k, 24, f, b, T)]);
    }
    for (int i = 0; i < 3; ++i) x[i] = xn[i];
  }
}
// the previous production form: fields stored straight from uni_derivs' outputs
__global__ __launch_bounds__(256) void v8o(int B, int N, StageParams sp, const double* __restrict__ X,
                                           const double* __restrict__ U, const double* __restrict__ XR,
                                           double* __restrict__ J) {
  const long b = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const long T = ((long)B + 63) / 64;
  double x[3], xr[3];
  const double ur[2] = {0.0, 0.0};
  const double lz[3] = {0, 0, 0};
#pragma unroll
  for (int i = 0; i < 3; ++i) { x[i] = X[tix(0, 3, i, b, T)]; xr[i] = XR[tix(0, 3, i, b, T)]; }
  for (int k = 0; k < N; ++k) {
    double u[2], xn[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) xn[i] = X[tix(k + 1, 3, i, b, T)];
#pragma unroll
    for (int i = 0; i < 2; ++i) u[i] = U[tix(k, 2, i, b, T)];
    double xf[3], q, A[9], Bm[6], g[5], H[15];
    uni_derivs<false>(sp, x, u, xr, ur, lz, 1.0, xf, q, A, Bm, g, H);
#pragma unroll
    for (int i = 0; i < 3; ++i) __builtin_nontemporal_store(xf[i] - xn[i], &J[tix(k, 24, i, b, T)]);
    __builtin_nontemporal_store(q, &J[tix(k, 24, 3, b, T)]);
#pragma unroll
    for (int i = 0; i < 9; ++i) __builtin_nontemporal_store(A[i], &J[tix(k, 24, 4 + i, b, T)]);
#pragma unroll
    for (int i = 0; i < 6; ++i) __builtin_nontemporal_store(Bm[i], &J[tix(k, 24, 13 + i, b, T)]);
#pragma unroll
    for (int i = 0; i < 5; ++i) __builtin_nontemporal_store(g[i], &J[tix(k, 24, 19 + i, b, T)]);
#pragma unroll
    for (int i = 0; i < 3; ++i) x[i] = xn[i];
  }
}
__global__ __launch_bounds__(256) void v8(int B, int N, StageParams sp, const double* X, const double* U,
                                          const double* XR, double* J) { body<false>(B, N, sp, X, U, XR, J); }
__global__ __launch_bounds__(256) void v16(int B, int N, StageParams sp, const double* X, const double* U,
                                           const double* XR, double* J) { body<true>(B, N, sp, X, U, XR, J); }
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void v16w4(
    int B, int N, StageParams sp, const double* X, const double* U, const double* XR, double* J) {
  body<true>(B, N, sp, X, U, XR, J);
}
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void v8w4(
    int B, int N, StageParams sp, const double* X, const double* U, const double* XR, double* J) {
  body<false>(B, N, sp, X, U, XR, J);
}

int main() {
  const int B = 1 << 19, N = 20;
  const long T = B / 64;
  StageParams sp{};
  sp.T = 0.2; sp.M = 4; sp.h = sp.T / sp.M; sp.cost = 0;
  sp.Q[0] = 1; sp.Q[1] = 5; sp.Q[2] = 0.1; sp.R[0] = 0.5; sp.R[1] = 0.05;
  const size_t nX = (size_t)(N + 1) * 3 * B, nU = (size_t)N * 2 * B, nR = 3 * (size_t)B, nJ = (size_t)N * 24 * B;
  std::vector<double> hX(nX), hU(nU), hR(nR);
  srand(7);
  auto rnd = [](double lo, double hi) { return lo + (hi - lo) * (rand() / (double)RAND_MAX); };
  for (auto& v : hX) v = rnd(-3, 3);
  for (auto& v : hU) v = rnd(-0.78, 0.78);
  for (auto& v : hR) v = rnd(-10, 10);
  double *X, *U, *R, *J;
  CK(hipMalloc(&X, nX * 8)); CK(hipMalloc(&U, nU * 8)); CK(hipMalloc(&R, nR * 8)); CK(hipMalloc(&J, nJ * 8));
  CK(hipMemcpy(X, hX.data(), nX * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(U, hU.data(), nU * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(R, hR.data(), nR * 8, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const double alg = (double)B * (256.0 * N + 48);
  std::vector<double> ref(nJ), out(nJ);
  auto run = [&](auto kern, const char* name, bool pairs) {
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(kern, dim3(B / 256), dim3(256), 0, 0, B, N, sp, X, U, R, J);
    CK(hipDeviceSynchronize());
    float ms;
    CK(hipEventRecord(e0));
    for (int r = 0; r < 20; ++r) hipLaunchKernelGGL(kern, dim3(B / 256), dim3(256), 0, 0, B, N, sp, X, U, R, J);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= 20;
    CK(hipMemcpy(out.data(), J, nJ * 8, hipMemcpyDeviceToHost));
    long bad = 0;
    if (!pairs) { if (ref[0] == 0 && ref[1] == 0) ref = out; else bad = memcmp(ref.data(), out.data(), nJ * 8) != 0; }
    else
      for (int k = 0; k < N; ++k)
        for (long t = 0; t < T; ++t)
          for (int f = 0; f < 24; ++f)
            for (int l = 0; l < 64; ++l)
              bad += ref[((k * T + t) * 24 + f) * 64 + l] != out[(((k * T + t) * 12 + f / 2) * 64 + l) * 2 + f % 2];
    printf("{\"variant\": \"%s\", \"ms\": %.4f, \"alg_GBps\": %.1f, \"frac\": %.4f, \"mismatch\": %ld}\n", name, ms,
           alg / (ms * 1e-3) / 1e9, alg / (ms * 1e-3) / 8e12, bad);
  };
  std::fill(ref.begin(), ref.end(), 0.0);
  run(v8o, "v8o (previous production kernel)", false);
  run(v8, "v8 (8-B nt stores)", false);
  run(v16, "v16 (16-B nt field pairs)", true);
  run(v16w4, "v16w4 (16-B pairs, waves_per_eu 4)", true);
  run(v8w4, "v8w4 (8-B, waves_per_eu 4)", false);
  run(v8, "v8 again", false);
  run(v16, "v16 again", true);
  return 0;
}
