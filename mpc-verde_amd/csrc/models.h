// models.h -- stage models of the fused solve kernel.
//
// A model supplies NX, NU, the structural masks of its Jacobians, a per-lane context
// (what node k of instance `inst` needs: references, stage matrices) and two stage
// functions: value (F, q) and derivatives (F, q, A, B, grad q, exact Hessian of
// fs*q + lam^T F).  The solver kernel (solver.hip) is written once against this.
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "riccati.h"
#include "solver.h"
#include "unicycle.h"


namespace mpcx {

// ------------------------------------------------------------------------------------
// Unicycle (Casadi/multiple_shooting_casadi.py:68-114; Trajectory_tracking.py:40-61)
// A = I + a02 e0 e2^T + a12 e1 e2^T,  B[2][0] = 0  (structural zeros as masks)
// ------------------------------------------------------------------------------------
struct UnicycleModel {
  static constexpr int NX = 3, NU = 2;
  static constexpr unsigned long long AMASK = (1ull << 0) | (1ull << 2) | (1ull << 4) | (1ull << 5) | (1ull << 8);
  static constexpr unsigned long long BMASK = (1ull << 0) | (1ull << 1) | (1ull << 2) | (1ull << 3) | (1ull << 5);
  static constexpr unsigned long long AONE = (1ull << 0) | (1ull << 4) | (1ull << 8);  // A's unit diagonal
  // the line search's first trial evaluates derivatives, not just values: accepted (the
  // usual case) it is the next iteration's evaluation, which is then skipped
  static constexpr bool kEvalInSearch = true;
  // second-order correction (IPOPT max_soc): not here -- the first trial's evaluation replaces
  // the current point's derivatives, and config-2/3 solves do not reach it
  static constexpr bool kSOC = false;
  // IPOPT's soft restoration and restoration phase (resto.h, the resume launch): a warm-started
  // closed-loop solve that sits at its optimum to rounding level can fail the filter line
  // search on noise in theta (tests/test_gpu_hard.py); IPOPT recovers it there
  static constexpr bool kResto = true;
  // variable bounds in LDS, re-read per phase (kernels.h LdsCol): removes the kernel's scratch
  // spills but measured 1-2 % slower on config 2 (LDS latency on the line search), so off
  static constexpr bool kBoundsLds = false;
  // backward Riccati recursion as a log-depth scan (pscan.h) instead of N dependent steps
  static constexpr bool kParallelRiccati = false;
  // a 32-lane group widened to a whole wave runs as two replicas that split the sequential work
  // (kernels.h R = 2): configs 1-2 (N <= 30) at batches below two waves per SIMD
  static constexpr bool kReplicate = true;
  // the sequential Riccati recursion spread over 16-lane rows (rowchain.h; bit-identical to
  // riccati_step) in the single-wave groups of 32 and 64 lanes
  static constexpr bool kRowChain = true;
  struct Ctx {
    double xr[3], ur[2];
  };
  // Jacobian/Hessian operands of the Newton step live in the kernel's registers
  static constexpr bool kTableJac = false, kTableHess = false;
  static constexpr int kTrigSlots = 0;  // no LDS value cache
  __device__ __forceinline__ static const double* jacA(const Ctx&, const double* A) { return A; }
  __device__ __forceinline__ static const double* jacB(const Ctx&, const double* B) { return B; }
  __device__ __forceinline__ static const double* hessW(const Ctx&, const double* H) { return H; }
  __device__ __forceinline__ static void load_ctx(const ModelArgs& a, int inst, const double* P, int k, bool hasU, Ctx& c) {
    for (int i = 0; i < 3; ++i) c.xr[i] = 0.0;
    c.ur[0] = c.ur[1] = 0.0;
    if (a.p_layout == 0) {
      for (int i = 0; i < 3; ++i) c.xr[i] = P[3 + i];
    } else if (hasU) {
      for (int i = 0; i < 3; ++i) c.xr[i] = P[3 + 5 * k + i];
      for (int i = 0; i < 2; ++i) c.ur[i] = P[3 + 5 * k + 3 + i];
    }
  }
  __device__ __forceinline__ static void derivs(const ModelArgs& a, const Ctx& c, const double* z, const double* ln, double fs,
                                double* xf, double& q, double* A, double* Bm, double* g, double* H) {
    const double u2[2] = {z[3], z[4]};
    uni_derivs_moments<0>(a.sp, z, u2, c.xr, c.ur, ln, fs, xf, q, A, Bm, g, H);  // weighted moments (unicycle.h)
  }
  // the same with the moments summed in the replicated groups' two halves: the 32-lane groups,
  // which a small batch runs replicated (stage_derivs below), so that a node's bits do not depend
  // on the batch it is solved in
  __device__ __forceinline__ static void derivs_halves(const ModelArgs& a, const Ctx& c, const double* z,
                                                       const double* ln, double fs, double* xf, double& q, double* A,
                                                       double* Bm, double* g, double* H) {
    const double u2[2] = {z[3], z[4]};
    uni_derivs_moments<1>(a.sp, z, u2, c.xr, c.ur, ln, fs, xf, q, A, Bm, g, H);
  }
  // the same evaluation split between the two replicas of a replicated lane group (kernels.h R = 2;
  // every lane of the wave must call it)
  __device__ __forceinline__ static void derivs_rep(const ModelArgs& a, const Ctx& c, const double* z, const double* ln,
                                                    double fs, double* xf, double& q, double* A, double* Bm, double* g,
                                                    double* H, int rho) {
    const double u2[2] = {z[3], z[4]};
    uni_derivs_moments<2>(a.sp, z, u2, c.xr, c.ur, ln, fs, xf, q, A, Bm, g, H, rho);
  }
  __device__ __forceinline__ static void value(const ModelArgs& a, const Ctx& c, const double* z, double* xf, double& q) {
    const double u2[2] = {z[3], z[4]};
    uni_value(a.sp, z, u2, c.xr, c.ur, xf, q);
  }
};

// The same model for problems without state bounds (configs 1 and 2: X free, |v| <= 1,
// |w| <= pi/4): the launch picks it when no node has a finite state bound, and every state-bound
// term folds away at compile time (kernels.h kXB).
struct UnicycleFreeModel : UnicycleModel {
  static constexpr bool kXBounds = false;
};

// The same model with the backward Riccati recursion as a log-depth scan (pscan.h).  The scan's
// cost is ceil(log2(N+1)) combine levels whatever N is, the sequential chain's is N steps, so the
// launch picks this instantiation for longer horizons (solver.hip kUnicycleScanMinN; A/B on one
// MI355X: config 3, N = 30, +6.5 % solves/s; config 2, N = 20, -4 %).
struct UnicycleScanModel : UnicycleModel {
  static constexpr bool kParallelRiccati = true;
  static constexpr bool kReplicate = false;  // no sequential chain to split
  static constexpr bool kRowChain = false;   // the chain is the scan's rare fallback
};

// ------------------------------------------------------------------------------------
// Linear (time-varying) model with quadratic stage cost -- the mpctools LTI/LTV QPs
// (Inverted_pendulum/inverted_pendulum_single_shooting_mpctools.py:19-64,
//  Trajectory Tracking/Trajectory_tracking_dynamic_model.py:117-145):
//   x+ = A_j x + B_j u + c_j,   l = (z - zr_k)^T W_j (z - zr_k),   z = (x, u),
// with j = table index of (instance, stage) and zr_k per-stage references in P.
// ------------------------------------------------------------------------------------
template <int NX_, int NU_>
struct LinearModel {
  static constexpr int NX = NX_, NU = NU_, NZ = NX_ + NU_, NH = NZ * (NZ + 1) / 2;
  static constexpr unsigned long long AMASK = (NX * NX >= 64) ? ~0ull : ((1ull << (NX * NX)) - 1);
  static constexpr unsigned long long BMASK = (1ull << (NX * NU)) - 1;
  static constexpr bool kEvalInSearch = false;  // a value is one mat-vec: nothing to save
  static constexpr bool kSOC = false;           // linear constraints: a full step never increases theta
  struct Ctx {
    const double *A, *B, *c, *W;
    double zr[NZ];
    bool dec;  // my stage's table is decoupled (LinTables::dec_mask)
  };
  // Log-depth Riccati scan (pscan.h), and with it A, B and the stage Hessian 2 W read from the
  // stage tables (global memory, cache-resident) instead of register copies held through the
  // whole iteration, which leaves the registers to the scan (derivs then does not fill A, Bm,
  // H).  Measured (one MI355X): config 4 (NX = 4, N = 50) 9.3 M solves/s sequential, 11.9 M
  // scan with register tables, 12.6 M scan with table operands; config 5 (NX = 5, N = 100)
  // 0.91 M sequential, 0.43 M / 0.87 M with the scan (its 65-double elements still spill), so
  // NX = 5 keeps the sequential recursion and register tables.
  static constexpr bool kScan = NX_ <= 4;
  static constexpr bool kParallelRiccati = kScan, kTableJac = kScan, kTableHess = kScan;
  // Decoupled suffix (solver.hip): the sequential recursion reuses P_k on a suffix of
  // decoupled stages -- the move-blocked stages of the cart-pole QP (lti.py).  Scan models
  // keep their scan.
  static constexpr bool kDecSuffix = !kScan;
  // variable bounds in LDS (kernels.h LdsCol), re-read per phase, instead of 2 NZ doubles of
  // registers held through every phase: A/B on one MI355X, config 5 (LinearModel<5,1>, G = 128)
  // scratch 704 -> 240 B/lane, 116 -> 100 us per IPM iteration (+15 % solves/s); config 4
  // (LinearModel<4,1>, scan) +3.5 %, scratch 404 -> 0 (LinearModel<4,2>: 680 -> 84)
  static constexpr bool kBoundsLds = true;
  static constexpr int kTrigSlots = 0;
  __device__ __forceinline__ static const double* jacA(const Ctx& c, const double* A) { return kTableJac ? c.A : A; }
  __device__ __forceinline__ static const double* jacB(const Ctx& c, const double* B) { return kTableJac ? c.B : B; }
  __device__ __forceinline__ static const double* hessW(const Ctx& c, const double* H) { return kTableHess ? c.W : H; }
  __device__ __forceinline__ static void load_ctx(const ModelArgs& a, int inst, const double* P, int k, bool hasU, Ctx& c) {
    const int N = a.N;
    int j = 0;
    if (hasU) j = min(max(a.lin.tab[(a.lin.per_instance ? (size_t)inst * N : 0) + k], 0), a.lin.n_tab - 1);
    c.A = a.lin.A + (size_t)j * NX * NX;
    c.B = a.lin.B + (size_t)j * NX * NU;
    c.c = a.lin.c + (size_t)j * NX;
    c.W = a.lin.W + (size_t)j * NH;
    c.dec = hasU && j < 64 && ((a.lin.dec_mask >> j) & 1ull);
    for (int i = 0; i < NZ; ++i) c.zr[i] = hasU ? P[NX + NZ * k + i] : 0.0;
  }
  __device__ __forceinline__ static void value(const ModelArgs& a, const Ctx& c, const double* z, double* xf, double& q) {
    double dz[NZ];
#pragma unroll
    for (int i = 0; i < NZ; ++i) dz[i] = z[i] - c.zr[i];
#pragma unroll
    for (int r = 0; r < NX; ++r) {
      double acc = c.c[r];
#pragma unroll
      for (int m = 0; m < NX; ++m) acc = fma(c.A[r * NX + m], z[m], acc);
#pragma unroll
      for (int l = 0; l < NU; ++l) acc = fma(c.B[r * NU + l], z[NX + l], acc);
      xf[r] = acc;
    }
    double acc = 0.0;
#pragma unroll
    for (int i = 0; i < NZ; ++i) {
      double wi = 0.0;
#pragma unroll
      for (int j = 0; j < NZ; ++j) wi = fma(c.W[symix(i, j, NZ)], dz[j], wi);
      acc = fma(dz[i], wi, acc);
    }
    q = acc;
  }
  __device__ __forceinline__ static void derivs(const ModelArgs& a, const Ctx& c, const double* z, const double* ln, double fs,
                                double* xf, double& q, double* A, double* Bm, double* g, double* H) {
    double dz[NZ];
#pragma unroll
    for (int i = 0; i < NZ; ++i) dz[i] = z[i] - c.zr[i];
    if constexpr (!kTableJac) {
#pragma unroll
      for (int i = 0; i < NX * NX; ++i) A[i] = c.A[i];
#pragma unroll
      for (int i = 0; i < NX * NU; ++i) Bm[i] = c.B[i];
    }
    if constexpr (!kTableHess)
#pragma unroll
      for (int i = 0; i < NH; ++i) H[i] = 2.0 * fs * c.W[i];
#pragma unroll
    for (int r = 0; r < NX; ++r) {
      double acc = c.c[r];
#pragma unroll
      for (int m = 0; m < NX; ++m) acc = fma(c.A[r * NX + m], z[m], acc);
#pragma unroll
      for (int l = 0; l < NU; ++l) acc = fma(c.B[r * NU + l], z[NX + l], acc);
      xf[r] = acc;
    }
    double acc = 0.0;
#pragma unroll
    for (int i = 0; i < NZ; ++i) {
      double wi = 0.0;
#pragma unroll
      for (int j = 0; j < NZ; ++j) wi = fma(c.W[symix(i, j, NZ)], dz[j], wi);
      g[i] = 2.0 * fs * wi;
      acc = fma(dz[i], wi, acc);
    }
    q = acc;
  }
};

// Model::kReplicate if the model declares it: a 32-lane group may run replicated (kernels.h R = 2)
template <class M, class = void>
struct ReplicateOf {
  static constexpr bool value = false;
};
template <class M>
struct ReplicateOf<M, std::void_t<decltype(M::kReplicate)>> {
  static constexpr bool value = M::kReplicate;
};

// The stage evaluation of a group of G lanes, one per node (R = 1).  Where the same group may
// also run replicated -- a replicating model's 32-lane groups, widened to a wave when the batch
// leaves SIMDs idle (solve_group_size) -- the moments are summed in the replicas' two halves, so an
// instance gets the same bits whatever batch (and hence group variant) it is solved in.  Every
// 32-lane launch of such a model is a 16 <= N < 32 group: kernels.h solve_shape never widens a
// 16-lane group (N < 16, summed in one pass at 16 and 64 lanes) to 32.
template <class Model, int G, class... Args>
__device__ __forceinline__ void stage_derivs(Args&&... args) {
  if constexpr (ReplicateOf<Model>::value && G == 32)
    Model::derivs_halves(args...);
  else
    Model::derivs(args...);
}

}  // namespace mpcx
