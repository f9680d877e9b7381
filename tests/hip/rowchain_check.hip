// rowchain_check.hip -- test harness for rowchain.h (the unicycle's Riccati recursion spread over
// 16-lane rows): for random stages (the unicycle's Jacobian structure, random symmetric stage
// Hessians -- indefinite ones included -- and random terminal value functions) it runs the row
// chain exactly as the solve kernel does (node records in LDS, every row running its instance's
// chain) beside the sequential recursion the kernel ran before it (riccati_step on node lane j,
// the value function moved lane to lane by DPP), and writes both results per node: P_k (6), p_k
// (3) and the factors (r0, t, r1, h0[3], h1[3], g0, g1) -- for the row chain the factors and P_k come
// from each node's own step redone on the chain's value functions, as in the solve kernel.  Built into tests/hip/librowchain_check.so
// (tests/hip/Makefile); used by tests/test_gpu_rowchain.py only.
#include "kernels.h"
#include "rowchain6.h"

namespace mpcx {

constexpr int kOut = 6 + 3 + 13;  // P, p, fac

__device__ void put_out(double* o, const double* P, const double* p, const Fac<3, 2>& f) {
  for (int i = 0; i < 6; ++i) o[i] = P[i];
  for (int i = 0; i < 3; ++i) o[6 + i] = p[i];
  o[9] = f.r0;
  o[10] = f.t;
  o[11] = f.r1;
  for (int i = 0; i < 3; ++i) {
    o[12 + i] = f.h0[i];
    o[15 + i] = f.h1[i];
  }
  o[18] = f.g0;
  o[19] = f.g1;
  o[20] = f.r1 > 0.0 ? 1.0 : 0.0;  // (spare)
  o[21] = 0.0;
}

// in, per node of each instance (G nodes): Hd 15, gp 5, A 9, B 6, c 3, P 6, p 3 = 47 doubles (P, p
// used at node N only)
constexpr int kIn = 47;

__device__ __forceinline__ unsigned long long clk() {
  unsigned long long t;
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

template <int G, int R>
__global__ __launch_bounds__(64) void rowchain_check_kernel(int N, int B, const double* in, double* out_seq,
                                                            double* out_row, unsigned long long* cyc) {
  __shared__ double rcbuf[(64 / (G * R)) * G * rowchain::kRec];
  const long gid = (long)blockIdx.x * 64 + threadIdx.x;
  const int k = (int)(gid & (G - 1));
  const int inst = (int)(gid / (G * R));
  const int rho = R > 1 ? (int)((threadIdx.x / G) % R) : 0;
  const bool valid = inst < B;
  const bool hasU = valid && k < N, hasX = valid && k <= N;
  double Hd[15] = {}, gp[5] = {}, A[9] = {}, Bm[6] = {}, c[3] = {}, PN[6] = {}, pN[3] = {};
  if (valid) {
    const double* r = in + ((long)inst * G + k) * kIn;
    for (int i = 0; i < 15; ++i) Hd[i] = r[i];
    for (int i = 0; i < 5; ++i) gp[i] = r[15 + i];
    for (int i = 0; i < 9; ++i) A[i] = r[20 + i];
    for (int i = 0; i < 6; ++i) Bm[i] = r[29 + i];
    for (int i = 0; i < 3; ++i) c[i] = r[35 + i];
    for (int i = 0; i < 6; ++i) PN[i] = r[38 + i];
    for (int i = 0; i < 3; ++i) pN[i] = r[44 + i];
  }
  using M = UnicycleModel;
  // ---- the sequential recursion (the kernel's chain before the row chain)
  double P[6], p[3];
  for (int i = 0; i < 6; ++i) P[i] = k == N ? PN[i] : 0.0;
  for (int i = 0; i < 3; ++i) p[i] = k == N ? pN[i] : 0.0;
  Fac<3, 2> fac = {};
  const unsigned long long t0 = clk();
  for (int j = N - 1; j >= 0; --j) {
    double Pin_[6], pin_[3];
    for (int i = 0; i < 6; ++i) Pin_[i] = from_next(P[i]);
    for (int i = 0; i < 3; ++i) pin_[i] = from_next(p[i]);
    if (k == j) (void)riccati_step<3, 2, M::AMASK, M::BMASK, false, false, M::AONE>(Hd, gp, A, Bm, c, Pin_, pin_, P, p, fac);
  }
  const unsigned long long t1 = clk();
  if (hasX && rho == 0) put_out(out_seq + ((long)inst * G + k) * kOut, P, p, fac);
  // ---- the row chain
  double P2[6], p2[3];
  for (int i = 0; i < 6; ++i) P2[i] = k == N ? PN[i] : 0.0;
  for (int i = 0; i < 3; ++i) p2[i] = k == N ? pN[i] : 0.0;
  Fac<3, 2> fac2 = {};
  double* rinst = rcbuf + (int)((threadIdx.x & 63) / (G * R)) * G * rowchain::kRec;
  if (R == 1 || rho == 0) {
    if (hasU) rowchain::store_stage(rinst + k * rowchain::kRec, Hd, gp, A, Bm, c);
    else if (hasX && k == N) rowchain::store_terminal(rinst + k * rowchain::kRec, P2, p2);
  }
  __syncthreads();
  const unsigned long long t2 = clk();
  rowchain::run<G * R>(rinst, N);
  const unsigned long long t3 = clk();
  __syncthreads();
  if (hasU) {  // as the solve kernel: node k redoes its step from node k+1's value function
    double Pin_[6], pin_[3];
    rowchain::load_next(rinst + (k + 1) * rowchain::kRec, Pin_, pin_);
    (void)riccati_step<3, 2, M::AMASK, M::BMASK, false, false, M::AONE>(Hd, gp, A, Bm, c, Pin_, pin_, P2, p2, fac2);
  }
  if (hasX && rho == 0) put_out(out_row + ((long)inst * G + k) * kOut, P2, p2, fac2);
  if (cyc && threadIdx.x == 0) {  // cycles of the two chains (this wave)
    cyc[2 * blockIdx.x] = t1 - t0;
    cyc[2 * blockIdx.x + 1] = t3 - t2;
  }
}

// ---- the 6-state chain (rowchain6.h): one instance per 64-lane wave, window by window
// in, per node (64 per instance): Hs 36 (packed upper, 8x8), Sigma 8, A 36, B 12, gp 8, c 6
constexpr int kIn6 = 106, kOut6 = 21 + 6 + 17;

__device__ void put_out6(double* o, const double* P, const double* p, const Fac<6, 2>& f) {
  for (int i = 0; i < 21; ++i) o[i] = P[i];
  for (int i = 0; i < 6; ++i) o[21 + i] = p[i];
  o[27] = f.r0;
  o[28] = f.t;
  o[29] = f.r1;
  for (int i = 0; i < 6; ++i) {
    o[30 + i] = f.h0[i];
    o[36 + i] = f.h1[i];
  }
  o[42] = f.g0;
  o[43] = f.g1;
}

__global__ __launch_bounds__(64) void rowchain6_check_kernel(int N, double delta, const double* in, double* ws,
                                                             double* out_seq, double* out_row, unsigned long long* cyc,
                                                             int* early_out) {
  namespace rc = rowchain6;
  constexpr unsigned long long AM = rc::amask6(), BM = (1ull << 12) - 1;
  __shared__ double ring[rc::kRing];
  const int k = (int)threadIdx.x;
  const long inst = blockIdx.x;
  double Hs[36] = {}, sig[8] = {}, A[36] = {}, Bm[12] = {}, gp[8] = {}, c[6] = {};
  if (k <= N) {
    const double* r = in + (inst * 64 + k) * kIn6;
    for (int i = 0; i < 36; ++i) Hs[i] = r[i];
    for (int i = 0; i < 8; ++i) sig[i] = r[36 + i];
    for (int i = 0; i < 36; ++i) A[i] = r[44 + i];
    for (int i = 0; i < 12; ++i) Bm[i] = r[80 + i];
    for (int i = 0; i < 8; ++i) gp[i] = r[92 + i];
    for (int i = 0; i < 6; ++i) c[i] = r[100 + i];
  }
  double Hd[36];
  for (int i = 0; i < 36; ++i) Hd[i] = Hs[i];
  for (int i = 0; i < 8; ++i) Hd[symix(i, i, 8)] += sig[i] + delta;  // the solve kernel's order
  // ---- the sequential recursion (node lane j runs step j)
  double P[21], p[6];
  for (int i = 0; i < 6; ++i) {
    for (int j = i; j < 6; ++j) P[symix(i, j, 6)] = (k == N && i == j) ? sig[i] + delta : 0.0;
    p[i] = k == N ? gp[i] : 0.0;
  }
  Fac<6, 2> fac = {};
  const unsigned long long t0 = clk();
  for (int j = N - 1; j >= 0; --j) {
    double Pin_[21], pin_[6];
    for (int i = 0; i < 21; ++i) Pin_[i] = from_next(P[i]);
    for (int i = 0; i < 6; ++i) pin_[i] = from_next(p[i]);
    if (k == j) (void)riccati_step<6, 2, AM, BM, false, false, 0>(Hd, gp, A, Bm, c, Pin_, pin_, P, p, fac);
  }
  const unsigned long long t1 = clk();
  if (k <= N) put_out6(out_seq + (inst * 64 + k) * kOut6, P, p, fac);
  // ---- the row chain, then every node's own step from the chain's value functions
  auto fill = [&](int lo, int hi, bool top) __attribute__((always_inline)) {
    if (k >= lo && k <= hi) rc::store_node(ring + (k - lo) * rc::kRec, Hs, sig, delta, A, Bm, gp, c);
    if (top && k == N) rc::store_terminal(ring + (N - lo) * rc::kRec, sig, delta, gp);
  };
  double* out0 = ws + inst * 64 * rc::kOut;
  const unsigned long long t2 = clk();
  const bool early = rc::run(ring, out0, rc::kOut, true, N, fill);
  const unsigned long long t3 = clk();
  __syncthreads();
  double P2[21], p2[6];
  Fac<6, 2> fac2 = {};
  if (k < N) {
    double Pin_[21], pin_[6];
    rc::load_next(out0 + (k + 1) * rc::kOut, Pin_, pin_);
    (void)riccati_step<6, 2, AM, BM, false, false, 0>(Hd, gp, A, Bm, c, Pin_, pin_, P2, p2, fac2);
  } else {
    for (int i = 0; i < 6; ++i) {
      for (int j = i; j < 6; ++j) P2[symix(i, j, 6)] = (k == N && i == j) ? sig[i] + delta : 0.0;
      p2[i] = k == N ? gp[i] : 0.0;
    }
  }
  if (k <= N) put_out6(out_row + (inst * 64 + k) * kOut6, P2, p2, fac2);
  if (k == 0) early_out[inst] = early ? 1 : 0;  // the chain stopped at a step failing the inertia test
  if (cyc && k == 0) {
    cyc[2 * blockIdx.x] = t1 - t0;
    cyc[2 * blockIdx.x + 1] = t3 - t2;
  }
}

}  // namespace mpcx

// in: B * 64 * 106 doubles (node records, nodes 0..N used); ws: B * 64 * kOut scratch; outputs
// B * 64 * 44 doubles each; cyc (may be null): per wave the cycles of the two chains; early: per
// instance 1 if the chain stopped at a failed inertia test
extern "C" int rowchain6_check(int N, int B, double delta, const double* in, double* ws, double* out_seq,
                               double* out_row, unsigned long long* cyc, int* early) {
  if (B <= 0 || N < 1 || N > 63) return 1;
  hipLaunchKernelGGL(mpcx::rowchain6_check_kernel, dim3(B), dim3(64), 0, 0, N, delta, in, ws, out_seq, out_row, cyc,
                     early);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 3;
}

// G = 32 (R = 1: two instances per wave; R = 2: one, replicated) or 64; in: B * G * 47 doubles,
// outputs B * G * 22 doubles each, cyc (may be null): per wave the cycles of the sequential recursion
// and of the row chain (device pointers)
extern "C" int rowchain_check(int G, int R, int N, int B, const double* in, double* out_seq, double* out_row,
                              unsigned long long* cyc) {
  if (B <= 0 || N < 1 || N >= G) return 1;
  const long threads = (long)B * G * R;
  const int blocks = (int)((threads + 63) / 64);
  if (G == 32 && R == 1)
    hipLaunchKernelGGL((mpcx::rowchain_check_kernel<32, 1>), dim3(blocks), dim3(64), 0, 0, N, B, in, out_seq, out_row, cyc);
  else if (G == 32 && R == 2)
    hipLaunchKernelGGL((mpcx::rowchain_check_kernel<32, 2>), dim3(blocks), dim3(64), 0, 0, N, B, in, out_seq, out_row, cyc);
  else if (G == 64 && R == 1)
    hipLaunchKernelGGL((mpcx::rowchain_check_kernel<64, 1>), dim3(blocks), dim3(64), 0, 0, N, B, in, out_seq, out_row, cyc);
  else
    return 2;
  return hipDeviceSynchronize() == hipSuccess ? 0 : 3;
}
