// solver.hip -- fused batched interior-point solve of the multiple-shooting MPC NLP
// on gfx950 (MI355X), plus the RK4+Jacobian sweep, plant and shift kernels.
//
// Replaces, for B independent instances at once, the reference's
//   sol = solver(x0=w0, lbx, ubx, lbg, ubg, p)     Casadi/multiple_shooting_casadi.py:235-242
// where solver = ca.nlpsol('solver', 'ipopt', prob, opts) (:181-197) -- IPOPT's
// primal-dual barrier method (Waechter & Biegler 2006) on the NLP of :116-178.
//
// Execution model: one *lane group* of G = 16/32/64 lanes per
// instance; lane k owns shooting node k: X_k, U_k, the defect of interval k,
// its multipliers, bound duals, the stage derivative blocks (A_k, B_k, g_k,
// H_k, all in VGPRs) and the Riccati factors (K_k, P_k).  The whole solve --
// evaluation sweep, KKT Riccati factor/solve, fraction-to-boundary, filter line
// search, barrier update -- runs inside ONE launch; nothing but the inputs and
// the solution touch HBM.  Cross-node coupling moves through cross-lane
// shuffles (ds_bpermute); per-instance scalars are group reductions whose
// result is broadcast from the group's lane 0 so that every lane of an instance
// takes bit-identical control decisions.  Every loop is wave-uniform; lanes of
// finished instances are predicated off, never branched around a shuffle.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>

#include "solver.h"

// Diagnostic build only (-DMPCX_STAMPS, `make stamps`): per-phase s_memtime cycle
// accounting of the solve loop (cdna_hip_programming.md §7 "In-kernel stamps").
#ifdef MPCX_STAMPS
__device__ unsigned long long* g_mpcx_stamps = nullptr;
#define STAMP(p)                                                                          \
  do {                                                                                    \
    __builtin_amdgcn_sched_barrier(0);                                                    \
    unsigned long long t_;                                                                \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");           \
    __builtin_amdgcn_sched_barrier(0);                                                    \
    st_acc[st_ph] += t_ - st_last;                                                        \
    st_last = t_;                                                                         \
    st_ph = (p);                                                                          \
  } while (0)
#else
#define STAMP(p) \
  do {           \
  } while (0)
#endif

namespace mpcx {



// IPOPT constants (Waechter & Biegler 2006 Table 1; IPOPT defaults)
constexpr double kEps = 2.220446049250313e-16;
constexpr double kKappaEps = 10.0, kKappaMu = 0.2, kThetaMu = 1.5, kTauMin = 0.99;
constexpr double kKappaSigma = 1e10, kSmax = 100.0;
constexpr double kGammaTheta = 1e-5, kGammaPhi = 1e-8, kDeltaSw = 1.0, kSTheta = 1.1, kSPhi = 2.3;
constexpr double kEtaPhi = 1e-8, kGammaAlpha = 0.05;
constexpr double kDw0 = 1e-4, kDwMin = 1e-20, kDwMax = 1e40, kKwMinus = 1.0 / 3, kKwPlus = 8, kKwPlusBar = 100;
constexpr double kBoundPush = 1e-2, kBoundFrac = 1e-2, kInfBound = 1e19;

// ---- lane-group collectives (width G, aligned groups), all VALU ---------------
// Neighbour moves are DPP wave shifts; all-reduces are DPP within a 16-lane row
// (quad_perm xor1, quad_perm xor2, row_half_mirror, row_mirror) followed by
// v_permlane16_swap / v_permlane32_swap across rows (gfx950).  Every combine is
// symmetric (a+b on one lane, b+a on its partner), so all lanes of a group end
// with bit-identical results and take identical control decisions.
template <int CTRL>
__device__ __forceinline__ double dpp(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffLL), CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
constexpr int kQuadXor1 = 0xb1, kQuadXor2 = 0x4e, kHalfMirror = 0x141, kMirror = 0x140;
constexpr int kWaveShl1 = 0x130, kWaveShr1 = 0x138;

// other 16-lane row of a 32-lane half (xor 16) and other half of the wave (xor 32):
// the swap builtins hand back both rows; combining p[0] and p[1] in a fixed order
// keeps the result symmetric.
struct Pair {
  double a, b;
};
__device__ __forceinline__ Pair rows16(double v) {
  const long long x = __double_as_longlong(v);
  const auto lo = __builtin_amdgcn_permlane16_swap((int)(x & 0xffffffffLL), (int)(x & 0xffffffffLL), false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap((int)(x >> 32), (int)(x >> 32), false, false);
  return {__longlong_as_double(((long long)hi[0] << 32) | (unsigned int)lo[0]),
          __longlong_as_double(((long long)hi[1] << 32) | (unsigned int)lo[1])};
}
__device__ __forceinline__ Pair halves32(double v) {
  const long long x = __double_as_longlong(v);
  const auto lo = __builtin_amdgcn_permlane32_swap((int)(x & 0xffffffffLL), (int)(x & 0xffffffffLL), false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap((int)(x >> 32), (int)(x >> 32), false, false);
  return {__longlong_as_double(((long long)hi[0] << 32) | (unsigned int)lo[0]),
          __longlong_as_double(((long long)hi[1] << 32) | (unsigned int)lo[1])};
}

struct OpSum {
  __device__ static double f(double a, double b) { return a + b; }
};
struct OpMax {
  __device__ static double f(double a, double b) { return fmax(a, b); }
};
struct OpMin {
  __device__ static double f(double a, double b) { return fmin(a, b); }
};

template <int G, class Op>
__device__ __forceinline__ double greduce(double v) {
  v = Op::f(v, dpp<kQuadXor1>(v));
  v = Op::f(v, dpp<kQuadXor2>(v));
  v = Op::f(v, dpp<kHalfMirror>(v));
  v = Op::f(v, dpp<kMirror>(v));
  if (G >= 32) {
    const Pair p = rows16(v);
    v = Op::f(p.a, p.b);
  }
  if (G >= 64) {
    const Pair p = halves32(v);
    v = Op::f(p.a, p.b);
  }
  return v;
}
template <int G>
__device__ __forceinline__ double gsum(double v) {
  return greduce<G, OpSum>(v);
}
template <int G>
__device__ __forceinline__ double gmax(double v) {
  return greduce<G, OpMax>(v);
}
template <int G>
__device__ __forceinline__ double gmin(double v) {
  return greduce<G, OpMin>(v);
}
// value of lane k+1 / k-1 (whole-wave DPP shift; groups are contiguous and the
// lanes that would read across a group boundary never use the value)
__device__ __forceinline__ double from_next(double v) { return dpp<kWaveShl1>(v); }
__device__ __forceinline__ double from_prev(double v) { return dpp<kWaveShr1>(v); }

// 1/x to full fp64 accuracy: v_rcp_f64 + two Newton steps (no IEEE division sequence
// on the Riccati critical path)
__device__ __forceinline__ double rcp64(double x) {
  double r = __builtin_amdgcn_rcp(x);
  double e = fma(-x, r, 1.0);
  r = fma(r, e, r);
  e = fma(-x, r, 1.0);
  return fma(r, e, r);
}

__device__ __forceinline__ int ixw(int k, int i) { return k == 0 ? i : 3 + 5 * (k - 1) + 2 + i; }  // X_k[i] in w
__device__ __forceinline__ int iuw(int k, int i) { return 3 + 5 * k + i; }                          // U_k[i] in w

// One backward Riccati step (stage k) of the barrier KKT system.
//   in : H (15 packed, incl. Sigma + delta), gp (barrier gradient, 5), A, Bm, c (defect k)
//        P (packed sym 3x3: 00 01 02 11 12 22), p  -- value function of node k+1
//   out: Pn, pn (node k), K (2x3), kf (2); returns false if Huu' is not PD.
__device__ __forceinline__ bool riccati_step(const double H[15], const double gp[5], const double A[9],
                                             const double Bm[6], const double c[3], const double P[6],
                                             const double p[3], double Pn[6], double pn[3], double K[6],
                                             double kf[2]) {
  const double Pf[9] = {P[0], P[1], P[2], P[1], P[3], P[4], P[2], P[4], P[5]};
  double PA[9], PB[6];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
#pragma unroll
    for (int j = 0; j < 3; ++j) PA[3 * r + j] = Pf[3 * r] * A[j] + Pf[3 * r + 1] * A[3 + j] + Pf[3 * r + 2] * A[6 + j];
#pragma unroll
    for (int j = 0; j < 2; ++j)
      PB[2 * r + j] = Pf[3 * r] * Bm[j] + Pf[3 * r + 1] * Bm[2 + j] + Pf[3 * r + 2] * Bm[4 + j];
  }
  double Hxx[9], Hux[6], Huu[3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = i; j < 3; ++j)
      Hxx[3 * i + j] = H[hix(i, j)] + A[i] * PA[j] + A[3 + i] * PA[3 + j] + A[6 + i] * PA[6 + j];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      Hux[3 * i + j] = H[hix(j, 3 + i)] + Bm[i] * PA[j] + Bm[2 + i] * PA[3 + j] + Bm[4 + i] * PA[6 + j];
  Huu[0] = H[hix(3, 3)] + Bm[0] * PB[0] + Bm[2] * PB[2] + Bm[4] * PB[4];
  Huu[1] = H[hix(3, 4)] + Bm[0] * PB[1] + Bm[2] * PB[3] + Bm[4] * PB[5];
  Huu[2] = H[hix(4, 4)] + Bm[1] * PB[1] + Bm[3] * PB[3] + Bm[5] * PB[5];
  double s[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) s[i] = Pf[3 * i] * c[0] + Pf[3 * i + 1] * c[1] + Pf[3 * i + 2] * c[2] + p[i];
  double gx[3], gu[2];
#pragma unroll
  for (int i = 0; i < 3; ++i) gx[i] = gp[i] + A[i] * s[0] + A[3 + i] * s[1] + A[6 + i] * s[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) gu[i] = gp[3 + i] + Bm[i] * s[0] + Bm[2 + i] * s[1] + Bm[4 + i] * s[2];
  const double a = Huu[0], b = Huu[1], d = Huu[2];
  const double det = a * d - b * b;
  const bool ok = (a > 0.0) && (det > 0.0) && (d - b * b / a > 0.0);
  const double id = rcp64(det);
  const double i00 = d * id, i01 = -b * id, i11 = a * id;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    K[j] = -(i00 * Hux[j] + i01 * Hux[3 + j]);
    K[3 + j] = -(i01 * Hux[j] + i11 * Hux[3 + j]);
  }
  kf[0] = -(i00 * gu[0] + i01 * gu[1]);
  kf[1] = -(i01 * gu[0] + i11 * gu[1]);
  // Pn = Hxx + Hux^T K (symmetric), pn = gx + Hux^T kf
  Pn[0] = Hxx[0] + Hux[0] * K[0] + Hux[3] * K[3];
  Pn[1] = Hxx[1] + 0.5 * (Hux[0] * K[1] + Hux[3] * K[4] + Hux[1] * K[0] + Hux[4] * K[3]);
  Pn[2] = Hxx[2] + 0.5 * (Hux[0] * K[2] + Hux[3] * K[5] + Hux[2] * K[0] + Hux[5] * K[3]);
  Pn[3] = Hxx[4] + Hux[1] * K[1] + Hux[4] * K[4];
  Pn[4] = Hxx[5] + 0.5 * (Hux[1] * K[2] + Hux[4] * K[5] + Hux[2] * K[1] + Hux[5] * K[4]);
  Pn[5] = Hxx[8] + Hux[2] * K[2] + Hux[5] * K[5];
#pragma unroll
  for (int i = 0; i < 3; ++i) pn[i] = gx[i] + Hux[i] * kf[0] + Hux[3 + i] * kf[1];
  return ok;
}

template <int G>
__global__ __launch_bounds__(64) void solve_kernel(SolveArgs a) {
  const int lane = threadIdx.x & 63;
  const int k = lane & (G - 1);
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int inst = (int)(gid / G);
  const bool valid = inst < a.B;
  const int N = a.N;
  const int nw = 3 + 5 * N, ng = 3 * (N + 1);
  const bool hasX = valid && k <= N;
  const bool hasU = valid && k < N;
  const StageParams& sp = a.sp;

  // ---- per-instance parameters
  double x0[3] = {0, 0, 0}, xr[3] = {0, 0, 0}, ur[2] = {0, 0};
  if (valid) {
    const double* P = a.P + (size_t)inst * a.p_stride;
    for (int i = 0; i < 3; ++i) x0[i] = P[i];
    if (a.p_layout == 0) {
      for (int i = 0; i < 3; ++i) xr[i] = P[3 + i];
    } else if (hasU) {
      for (int i = 0; i < 3; ++i) xr[i] = P[3 + 5 * k + i];
      for (int i = 0; i < 2; ++i) ur[i] = P[3 + 5 * k + 3 + i];
    }
  }
  // ---- bounds of my variables (z = (x_k, u_k)); x_0 is free (pinned by g_0)
  double lb[5], ub[5];
  bool hL[5], hU[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    lb[i] = -1e20;
    ub[i] = 1e20;
  }
  if (hasX && k > 0)
    for (int i = 0; i < 3; ++i) {
      lb[i] = a.lbw[ixw(k, i)];
      ub[i] = a.ubw[ixw(k, i)];
    }
  if (hasU)
    for (int i = 0; i < 2; ++i) {
      lb[3 + i] = a.lbw[iuw(k, i)];
      ub[3 + i] = a.ubw[iuw(k, i)];
    }
  int nbnd_l = 0;
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const bool own = (i < 3) ? hasX : hasU;
    hL[i] = own && lb[i] > -kInfBound;
    hU[i] = own && ub[i] < kInfBound;
    nbnd_l += (int)hL[i] + (int)hU[i];
  }
  const double nbound = gsum<G>((double)nbnd_l);

  // ---- initial point
  double z[5] = {0, 0, 0, 0, 0};  // x_k (0..2), u_k (3..4)
  if (hasX) {
    if (a.w0) {
      const double* w0 = a.w0 + (size_t)inst * nw;
      for (int i = 0; i < 3; ++i) z[i] = w0[ixw(k, i)];
      if (hasU)
        for (int i = 0; i < 2; ++i) z[3 + i] = w0[iuw(k, i)];
    } else {
      for (int i = 0; i < 3; ++i) z[i] = x0[i];  // repmat(state_init), U = 0
    }
  }
  // bound push (IPOPT bound_push / bound_frac = 1e-2; warm start: warm_start_bound_push)
  const bool warm = a.warm != 0;
  const double push = warm ? a.bound_push : kBoundPush, frac = warm ? a.bound_push : kBoundFrac;
  double lx0[5] = {0, 0, 0, 0, 0};  // given bound multipliers (zU - zL) of my variables
  if (warm && a.lamx0 && hasX) {
    const double* l = a.lamx0 + (size_t)inst * nw;
    if (k > 0)
      for (int i = 0; i < 3; ++i) lx0[i] = l[ixw(k, i)];
    if (hasU)
      for (int i = 0; i < 2; ++i) lx0[3 + i] = l[iuw(k, i)];
  }
  double zL[5], zU[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    if (hL[i] && hU[i]) {
      const double pl = fmin(push * fmax(1.0, fabs(lb[i])), frac * (ub[i] - lb[i]));
      const double pu = fmin(push * fmax(1.0, fabs(ub[i])), frac * (ub[i] - lb[i]));
      z[i] = fmin(fmax(z[i], lb[i] + pl), ub[i] - pu);
    } else if (hL[i]) {
      z[i] = fmax(z[i], lb[i] + push * fmax(1.0, fabs(lb[i])));
    } else if (hU[i]) {
      z[i] = fmin(z[i], ub[i] - push * fmax(1.0, fabs(ub[i])));
    }
    zL[i] = hL[i] ? (warm ? fmax(-lx0[i], a.mult_push) : 1.0) : 0.0;
    zU[i] = hU[i] ? (warm ? fmax(lx0[i], a.mult_push) : 1.0) : 0.0;
  }
  double lam[3] = {0, 0, 0};  // lambda_k: multiplier of g_k (defines X_k)
  if (warm && a.lam0 && hasX)
    for (int i = 0; i < 3; ++i) lam[i] = a.lam0[(size_t)inst * ng + 3 * k + i];

  // ---- stage evaluation helpers (all lanes execute; hasU masks)
  double xf[3], qv, A[9], Bm[6], gq[5], Hs[15];
  double cdef[3], c0[3];  // cdef = F(X_k,U_k) - X_{k+1} (constraint k+1), c0 = x0 - X_0 (lane 0)
  double fs = 1.0;

  auto sweep = [&](bool want_h) {
    double ln[3], xn[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      ln[i] = from_next(lam[i]);
      xn[i] = from_next(z[i]);
    }
    {
      // every lane evaluates (SIMD: no extra cost); lanes without an interval mask
      // the results.  A and B keep their structural 0/1 entries as constants.
      const double u2[2] = {z[3], z[4]};
      uni_derivs<true>(sp, z, u2, xr, ur, ln, fs, xf, qv, A, Bm, gq, Hs);
      const double m = hasU ? 1.0 : 0.0;
      qv *= m;
#pragma unroll
      for (int i = 0; i < 15; ++i) Hs[i] *= m;
#pragma unroll
      for (int i = 0; i < 5; ++i) gq[i] *= m;
#pragma unroll
      for (int i = 0; i < 3; ++i) cdef[i] = hasU ? xf[i] - xn[i] : 0.0;
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) c0[i] = (valid && k == 0) ? x0[i] - z[i] : 0.0;
  };

  // objective scaling (IPOPT nlp_scaling_method = gradient-based, max_gradient = 100)
  sweep(true);
  {
    double gm = 0;
#pragma unroll
    for (int i = 0; i < 5; ++i) gm = fmax(gm, fabs(gq[i]));
    gm = gmax<G>(gm);
    fs = gm > 100.0 ? 100.0 / gm : 1.0;
    if (fs != 1.0) {  // group-uniform; given multipliers belong to the unscaled problem
#pragma unroll
      for (int i = 0; i < 3; ++i) lam[i] *= fs;
      if (warm)
#pragma unroll
        for (int i = 0; i < 5; ++i) {
          if (hL[i]) zL[i] = fmax(zL[i] * fs, a.mult_push);
          if (hU[i]) zU[i] = fmax(zU[i] * fs, a.mult_push);
        }
      sweep(true);
    }
  }

  double mu = warm ? a.mu_init : 0.1, tau = fmax(kTauMin, 1.0 - mu);
  const double mu_min = a.tol / 10.0;
  double theta0 = 0;
#pragma unroll
  for (int i = 0; i < 3; ++i) theta0 += fabs(cdef[i]) + fabs(c0[i]);
  theta0 = gsum<G>(theta0);
  const double theta_max = 1e4 * fmax(1.0, theta0), theta_min = 1e-4 * fmax(1.0, theta0);
  double dw_last = 0.0;
  double fth = 0, fph = 0;  // filter entry #k of my instance
  int nfilt = 0, fnext = 0;
  int status = valid ? 2 : 0;
  bool done = !valid;
  int it = 0;
  double dz[5], dlam[3], dzL[5], dzU[5];
  double Pk[6], pk[3], Kk[6], kfk[2];

#ifdef MPCX_STAMPS
  unsigned long long st_acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long st_last = 0;
  int st_ph = 9;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_last)::"memory");
#endif
  for (it = 0; it <= a.max_iter; ++it) {
    STAMP(0);
    // ------------------------------------------------------------ optimality error
    double ln[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) ln[i] = from_next(lam[i]);
    double Ed = 0, Ecomp0 = 0, Ec = 0, lam1 = 0, z1 = 0;
    double rd[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) rd[i] = 0;
    if (hasX) {
#pragma unroll
      for (int i = 0; i < 3; ++i) rd[i] = gq[i] - lam[i];
      if (hasU) {
#pragma unroll
        for (int j = 0; j < 3; ++j) rd[j] += A[j] * ln[0] + A[3 + j] * ln[1] + A[6 + j] * ln[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) rd[3 + j] = gq[3 + j] + Bm[j] * ln[0] + Bm[2 + j] * ln[1] + Bm[4 + j] * ln[2];
      }
#pragma unroll
      for (int i = 0; i < 3; ++i) lam1 += fabs(lam[i]);
    }
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      rd[i] += zU[i] - zL[i];
      Ed = fmax(Ed, fabs(rd[i]));
      z1 += zL[i] + zU[i];
      if (hL[i]) Ecomp0 = fmax(Ecomp0, fabs((z[i] - lb[i]) * zL[i]));
      if (hU[i]) Ecomp0 = fmax(Ecomp0, fabs((ub[i] - z[i]) * zU[i]));
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) Ec = fmax(Ec, fmax(fabs(cdef[i]), fabs(c0[i])));
    Ed = gmax<G>(Ed);
    Ec = gmax<G>(Ec);
    Ecomp0 = gmax<G>(Ecomp0);
    lam1 = gsum<G>(lam1);
    z1 = gsum<G>(z1);
    const double sd = fmax(kSmax, (lam1 + z1) / (double)(ng + nw)) / kSmax;
    const double sc = fmax(kSmax, nbound > 0 ? z1 / nbound : 0.0) / kSmax;
    const double E0 = fmax(fmax(Ed / sd, Ec), Ecomp0 / sc);
    if (!done && E0 <= a.tol) {
      done = true;
      status = 0;
    }
    if (!done && it == a.max_iter) {
      done = true;
      status = 2;
    }
    if (__all(done)) break;

    STAMP(1);
    // ------------------------------------------------------------ barrier update
    for (int rep = 0; rep < 32; ++rep) {
      double Ecm = 0;
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        if (hL[i]) Ecm = fmax(Ecm, fabs((z[i] - lb[i]) * zL[i] - mu));
        if (hU[i]) Ecm = fmax(Ecm, fabs((ub[i] - z[i]) * zU[i] - mu));
      }
      Ecm = gmax<G>(Ecm);
      const double Emu = fmax(fmax(Ed / sd, Ec), Ecm / sc);
      const bool dec = !done && Emu <= kKappaEps * mu && mu > mu_min;
      if (dec) {
        mu = fmax(mu_min, fmin(kKappaMu * mu, pow(mu, kThetaMu)));
        tau = fmax(kTauMin, 1.0 - mu);
        nfilt = 0;
        fnext = 0;
      }
      if (!__any(dec && it == 0)) break;
    }

    STAMP(2);
    // ------------------------------------------------------------ barrier gradient, Sigma
    double sig[5], gp[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      sig[i] = 0;
      gp[i] = gq[i];
      if (hL[i]) {
        const double s = z[i] - lb[i];
        sig[i] += zL[i] / s;
        gp[i] -= mu / s;
      }
      if (hU[i]) {
        const double s = ub[i] - z[i];
        sig[i] += zU[i] / s;
        gp[i] += mu / s;
      }
    }

    STAMP(3);
    // ------------------------------------------------------------ Riccati + inertia correction
    double delta = 0.0;
    bool need = !done;  // instance still needs a factorisation
    bool failed = false;
    bool first = true;
    for (int attempt = 0; attempt < 64; ++attempt) {
      if (!__any(need)) break;
      // backward sweep: node N .. 0
      double P[6], p[3];
      bool okl = true;
      {
        // node N (lane N): P_N = Sigma_x + delta, p_N = barrier gradient
        const double dl = (k == N) ? 1.0 : 0.0;
        P[0] = dl * (sig[0] + delta); P[1] = 0; P[2] = 0;
        P[3] = dl * (sig[1] + delta); P[4] = 0;
        P[5] = dl * (sig[2] + delta);
        p[0] = dl * gp[0]; p[1] = dl * gp[1]; p[2] = dl * gp[2];
      }
      for (int j = N - 1; j >= 0; --j) {
        double Pin[6], pin[3];
#pragma unroll
        for (int i = 0; i < 6; ++i) Pin[i] = from_next(P[i]);
#pragma unroll
        for (int i = 0; i < 3; ++i) pin[i] = from_next(p[i]);
        if (k == j) {
          double Hd[15];
#pragma unroll
          for (int i = 0; i < 15; ++i) Hd[i] = Hs[i];
#pragma unroll
          for (int i = 0; i < 5; ++i) Hd[hix(i, i)] += sig[i] + delta;
          okl = riccati_step(Hd, gp, A, Bm, cdef, Pin, pin, P, p, Kk, kfk);
        }
      }
#pragma unroll
      for (int i = 0; i < 6; ++i) Pk[i] = P[i];
#pragma unroll
      for (int i = 0; i < 3; ++i) pk[i] = p[i];
      const bool ok = gmin<G>(okl ? 1.0 : 0.0) > 0.5;
      // IPOPT inertia correction (Algorithm IC)
      if (need) {
        if (ok) {
          need = false;
          if (delta > 0.0) dw_last = delta;
        } else {
          if (first) delta = dw_last == 0.0 ? kDw0 : fmax(kDwMin, kKwMinus * dw_last);
          else delta *= dw_last == 0.0 ? kKwPlusBar : kKwPlus;
          first = false;
          if (delta > kDwMax) {
            need = false;
            failed = true;
          }
        }
      }
    }
    if (!done && failed) {
      done = true;
      status = 3;
    }

    STAMP(4);
    // ------------------------------------------------------------ forward sweep: dw, lambda+
    {
      double dxn[3] = {0, 0, 0};
      for (int j = 0; j <= N; ++j) {
        double dxi[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) dxi[i] = from_prev(dxn[i]);
        if (k == j) {
          if (k == 0)
#pragma unroll
            for (int i = 0; i < 3; ++i) dxi[i] = c0[i];
#pragma unroll
          for (int i = 0; i < 3; ++i) {
            dz[i] = dxi[i];
            dlam[i] = Pk[i == 0 ? 0 : (i == 1 ? 1 : 2)] * dxi[0] + Pk[i == 0 ? 1 : (i == 1 ? 3 : 4)] * dxi[1] +
                      Pk[i == 0 ? 2 : (i == 1 ? 4 : 5)] * dxi[2] + pk[i] - lam[i];
          }
          if (k < N) {
            dz[3] = Kk[0] * dxi[0] + Kk[1] * dxi[1] + Kk[2] * dxi[2] + kfk[0];
            dz[4] = Kk[3] * dxi[0] + Kk[4] * dxi[1] + Kk[5] * dxi[2] + kfk[1];
#pragma unroll
            for (int i = 0; i < 3; ++i)
              dxn[i] = A[3 * i] * dxi[0] + A[3 * i + 1] * dxi[1] + A[3 * i + 2] * dxi[2] + Bm[2 * i] * dz[3] +
                       Bm[2 * i + 1] * dz[4] + cdef[i];
          } else {
            dz[3] = dz[4] = 0.0;
          }
        }
      }
      if (!hasX) {
#pragma unroll
        for (int i = 0; i < 5; ++i) dz[i] = 0.0;
#pragma unroll
        for (int i = 0; i < 3; ++i) dlam[i] = 0.0;
      }
    }

    STAMP(5);
    // ------------------------------------------------------------ bound-dual step, fraction to boundary
    double amax_l = 1.0, az_l = 1.0, tiny_l = 0.0, gd_l = 0.0;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      dzL[i] = dzU[i] = 0.0;
      if (hL[i]) {
        const double s = z[i] - lb[i];
        dzL[i] = mu / s - zL[i] - zL[i] / s * dz[i];
        if (dz[i] < 0) amax_l = fmin(amax_l, -tau * s / dz[i]);
        if (dzL[i] < 0) az_l = fmin(az_l, -tau * zL[i] / dzL[i]);
      }
      if (hU[i]) {
        const double s = ub[i] - z[i];
        dzU[i] = mu / s - zU[i] + zU[i] / s * dz[i];
        if (dz[i] > 0) amax_l = fmin(amax_l, tau * s / dz[i]);
        if (dzU[i] < 0) az_l = fmin(az_l, -tau * zU[i] / dzU[i]);
      }
      const bool own = (i < 3) ? hasX : hasU;
      if (own) {
        tiny_l = fmax(tiny_l, fabs(dz[i]) / (1.0 + fabs(z[i])));
        gd_l += gp[i] * dz[i];
      }
    }
    const double amax = gmin<G>(amax_l), az = gmin<G>(az_l), tiny = gmax<G>(tiny_l);
    const double gd = gsum<G>(gd_l);

    STAMP(6);
    // ------------------------------------------------------------ filter line search
    double thk_l = 0, phk_l = hasU ? fs * qv : 0.0;
#pragma unroll
    for (int i = 0; i < 3; ++i) thk_l += fabs(cdef[i]) + fabs(c0[i]);
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      if (hL[i]) phk_l -= mu * log(z[i] - lb[i]);
      if (hU[i]) phk_l -= mu * log(ub[i] - z[i]);
    }
    const double thk = gsum<G>(thk_l), phk = gsum<G>(phk_l);
    const bool tinystep = tiny < 10.0 * kEps;
    double alpha = amax;
    bool searching = !done && !tinystep;
    bool accepted = !done && tinystep;
    bool ftype = tinystep;
    const double amin = gd < 0 ? kGammaAlpha * fmin(kGammaTheta, fmin(kGammaPhi * thk / (-gd),
                                                                       kDeltaSw * pow(thk, kSTheta) / pow(-gd, kSPhi)))
                               : kGammaAlpha * kGammaTheta;
    for (int ls = 0; ls < 80; ++ls) {
      if (!__any(searching)) break;
      double zt[5];
#pragma unroll
      for (int i = 0; i < 5; ++i) zt[i] = z[i] + alpha * dz[i];
      double xtn[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) xtn[i] = from_next(zt[i]);
      double tht_l = 0, pht_l = 0;
      if (hasU) {
        double xft[3], qt;
        const double u2[2] = {zt[3], zt[4]};
        uni_value(sp, zt, u2, xr, ur, xft, qt);
#pragma unroll
        for (int i = 0; i < 3; ++i) tht_l += fabs(xft[i] - xtn[i]);
        pht_l = fs * qt;
      }
      if (valid && k == 0)
#pragma unroll
        for (int i = 0; i < 3; ++i) tht_l += fabs(x0[i] - zt[i]);
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        if (hL[i]) pht_l -= mu * log(zt[i] - lb[i]);
        if (hU[i]) pht_l -= mu * log(ub[i] - zt[i]);
      }
      const double tht = gsum<G>(tht_l), pht = gsum<G>(pht_l);
      const double inF = (k < nfilt && tht >= fth && pht >= fph) ? 1.0 : 0.0;
      const bool infilter = gmax<G>(inF) > 0.5;
      if (searching) {
        bool acc = isfinite(pht) && isfinite(tht) && tht <= theta_max && !infilter;
        bool ft = false;
        if (acc) {
          const bool sw = gd < 0 && alpha * pow(-gd, kSPhi) > kDeltaSw * pow(thk, kSTheta);
          if (thk <= theta_min && sw) {
            acc = pht - phk <= kEtaPhi * alpha * gd + 10.0 * kEps * fabs(phk);
            ft = acc;
          } else {
            acc = tht <= (1.0 - kGammaTheta) * thk || pht <= phk - kGammaPhi * thk + 10.0 * kEps * fabs(phk);
          }
        }
        if (acc) {
          searching = false;
          accepted = true;
          ftype = ft;
        } else {
          alpha *= 0.5;
          if (alpha < amin) searching = false;  // would need restoration
        }
      }
    }
    if (!done && !accepted) {
      done = true;
      status = 3;
    }

    STAMP(7);
    // ------------------------------------------------------------ update iterate
    if (!done) {
      if (!ftype) {  // augment the filter (entry slot fnext lives on lane fnext)
        if (k == fnext) {
          fth = (1.0 - kGammaTheta) * thk;
          fph = phk - kGammaPhi * thk;
        }
        fnext = (fnext + 1) & (G - 1);
        nfilt = nfilt < G ? nfilt + 1 : G;
      }
#pragma unroll
      for (int i = 0; i < 5; ++i) z[i] += alpha * dz[i];
#pragma unroll
      for (int i = 0; i < 3; ++i) lam[i] += alpha * dlam[i];
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        if (hL[i]) {
          const double s = z[i] - lb[i];
          zL[i] = fmax(fmin(zL[i] + az * dzL[i], kKappaSigma * mu / s), mu / (kKappaSigma * s));
        }
        if (hU[i]) {
          const double s = ub[i] - z[i];
          zU[i] = fmax(fmin(zU[i] + az * dzU[i], kKappaSigma * mu / s), mu / (kKappaSigma * s));
        }
      }
    }
    STAMP(8);
    sweep(true);
  }
  STAMP(9);
#ifdef MPCX_STAMPS
  if (g_mpcx_stamps && (threadIdx.x & 63) == 0) {
    const long wv = gid / 64;
    for (int i = 0; i < 10; ++i) g_mpcx_stamps[wv * 10 + i] = st_acc[i];
  }
#endif

  // ---- results
  const double fsum = gsum<G>(hasU ? qv : 0.0);
  if (valid) {
    double* w = a.w_out + (size_t)inst * nw;
    if (hasX)
      for (int i = 0; i < 3; ++i) w[ixw(k, i)] = z[i];
    if (hasU)
      for (int i = 0; i < 2; ++i) w[iuw(k, i)] = z[3 + i];
    if (a.lam_out && hasX)
      for (int i = 0; i < 3; ++i) a.lam_out[(size_t)inst * ng + 3 * k + i] = lam[i] / fs;
    if (a.lamx_out) {
      double* lx = a.lamx_out + (size_t)inst * nw;
      if (hasX)
        for (int i = 0; i < 3; ++i) lx[ixw(k, i)] = (zU[i] - zL[i]) / fs;
      if (hasU)
        for (int i = 0; i < 2; ++i) lx[iuw(k, i)] = (zU[3 + i] - zL[3 + i]) / fs;
    }
    if (k == 0) {
      if (a.f_out) a.f_out[inst] = fsum;
      if (a.status) a.status[inst] = status;
      if (a.iters) a.iters[inst] = it > a.max_iter ? a.max_iter : it;
    }
  }
}

// ------------------------------------------------------------------------------
// RK4 + Jacobian sweep over B x N intervals, structure-of-arrays streams.
// One thread per instance walks its N intervals: X_{k+1} loaded for interval k
// stays in registers as interval k+1's X_k and x_ref is loaded once, so HBM sees
// exactly the compulsory bytes (reads (N+1)*3 + 2N + 3 doubles, writes 24N
// doubles per instance).  Consecutive lanes = consecutive
// instances: every load/store of a wave is one contiguous 512-B segment.
// ------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void rk4_sens_kernel(int B, int N, StageParams sp, const double* __restrict__ X,
                                                       const double* __restrict__ U, const double* __restrict__ XR,
                                                       double* __restrict__ C, double* __restrict__ Qo,
                                                       double* __restrict__ Ao, double* __restrict__ Bo,
                                                       double* __restrict__ Go) {
  const long b = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const long Bl = B;
  double x[3], xr[3];
  const double ur[2] = {0.0, 0.0};
  const double lz[3] = {0, 0, 0};
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    x[i] = X[i * Bl + b];
    xr[i] = XR[i * Bl + b];
  }
  for (int k = 0; k < N; ++k) {
    double u[2], xn[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) xn[i] = X[((long)(k + 1) * 3 + i) * Bl + b];
#pragma unroll
    for (int i = 0; i < 2; ++i) u[i] = U[((long)k * 2 + i) * Bl + b];
    double xf[3], q, A[9], Bm[6], g[5], H[15];
    uni_derivs<false>(sp, x, u, xr, ur, lz, 1.0, xf, q, A, Bm, g, H);
#pragma unroll
    for (int i = 0; i < 3; ++i) C[((long)k * 3 + i) * Bl + b] = xf[i] - xn[i];
    Qo[(long)k * Bl + b] = q;
#pragma unroll
    for (int i = 0; i < 9; ++i) Ao[((long)k * 9 + i) * Bl + b] = A[i];
#pragma unroll
    for (int i = 0; i < 6; ++i) Bo[((long)k * 6 + i) * Bl + b] = Bm[i];
#pragma unroll
    for (int i = 0; i < 5; ++i) Go[((long)k * 5 + i) * Bl + b] = g[i];
#pragma unroll
    for (int i = 0; i < 3; ++i) x[i] = xn[i];
  }
}

// Plant: x+ = F(x0, u).xf (Casadi/multiple_shooting_casadi.py:273), one thread per instance.
__global__ void plant_kernel(int B, int p_stride, int p_layout, StageParams sp, const double* __restrict__ P,
                             const double* __restrict__ U, double* __restrict__ XF, double* __restrict__ QF) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const double* p = P + (size_t)b * p_stride;
  double x[3] = {p[0], p[1], p[2]}, xr[3], ur[2] = {0, 0};
  for (int i = 0; i < 3; ++i) xr[i] = p[3 + i];
  if (p_layout == 1)
    for (int i = 0; i < 2; ++i) ur[i] = p[6 + i];
  const double u[2] = {U[2 * b], U[2 * b + 1]};
  double xf[3], q;
  uni_value(sp, x, u, xr, ur, xf, q);
  for (int i = 0; i < 3; ++i) XF[3 * b + i] = xf[i];
  if (QF) QF[b] = q;
}

// Closed-loop update (:271-287): x0 <- F(x0, u0*), w0_next = w shifted one interval;
// multipliers shifted alike when given (warm start of the next solve).
__global__ void shift_kernel(int B, int N, int p_stride, int p_layout, StageParams sp, double* __restrict__ P,
                             const double* __restrict__ W, double* __restrict__ W0, const double* __restrict__ L,
                             double* __restrict__ L0, const double* __restrict__ LX, double* __restrict__ LX0) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const int nw = 3 + 5 * N, ng = 3 * (N + 1);
  double* p = P + (size_t)b * p_stride;
  const double* w = W + (size_t)b * nw;
  double* w0 = W0 + (size_t)b * nw;
  double x[3] = {p[0], p[1], p[2]}, xr[3], ur[2] = {0, 0};
  for (int i = 0; i < 3; ++i) xr[i] = p[3 + i];
  if (p_layout == 1)
    for (int i = 0; i < 2; ++i) ur[i] = p[6 + i];
  const double u[2] = {w[3], w[4]};
  double xf[3], q;
  uni_value(sp, x, u, xr, ur, xf, q);
  for (int i = 0; i < 3; ++i) p[i] = xf[i];
  // shifted guess: X_k <- X_{k+1}, U_k <- U_{k+1}; last node/interval repeated
  for (int kk = 0; kk <= N; ++kk) {
    const int src = kk < N ? kk + 1 : N;
    for (int i = 0; i < 3; ++i) w0[ixw(kk, i)] = w[ixw(src, i)];
    if (LX && LX0)
      for (int i = 0; i < 3; ++i) LX0[(size_t)b * nw + ixw(kk, i)] = kk == 0 ? 0.0 : LX[(size_t)b * nw + ixw(src, i)];
    if (L && L0)
      for (int i = 0; i < 3; ++i) L0[(size_t)b * ng + 3 * kk + i] = L[(size_t)b * ng + 3 * src + i];
    if (kk < N) {
      const int su = kk + 1 < N ? kk + 1 : N - 1;
      for (int i = 0; i < 2; ++i) w0[iuw(kk, i)] = w[iuw(su, i)];
      if (LX && LX0)
        for (int i = 0; i < 2; ++i) LX0[(size_t)b * nw + iuw(kk, i)] = LX[(size_t)b * nw + iuw(su, i)];
    }
  }
}

#ifdef MPCX_STAMPS
extern "C" int mpcx_diag_set_stamp_buffer(void* d_buf) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_mpcx_stamps), &d_buf, sizeof(void*));
}
#endif

// ---- launch helpers (called from capi.cpp) -----------------------------------
hipError_t launch_solve(const SolveArgs& a, hipStream_t stream) {
  const int G = a.N < 16 ? 16 : (a.N < 32 ? 32 : 64);
  const long threads = (long)a.B * G;
  const int blocks = (int)((threads + 63) / 64);
  if (G == 16) hipLaunchKernelGGL(solve_kernel<16>, dim3(blocks), dim3(64), 0, stream, a);
  else if (G == 32) hipLaunchKernelGGL(solve_kernel<32>, dim3(blocks), dim3(64), 0, stream, a);
  else hipLaunchKernelGGL(solve_kernel<64>, dim3(blocks), dim3(64), 0, stream, a);
  return hipGetLastError();
}

hipError_t launch_rk4_sens(int B, int N, const StageParams& sp, const double* X, const double* U, const double* XR,
                           double* C, double* Q, double* A, double* Bm, double* G, hipStream_t stream) {
  const long blocks = ((long)B + 255) / 256;
  hipLaunchKernelGGL(rk4_sens_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, B, N, sp, X, U, XR, C, Q, A, Bm,
                     G);
  return hipGetLastError();
}

hipError_t launch_plant(int B, int p_stride, int p_layout, const StageParams& sp, const double* P, const double* U,
                        double* XF, double* QF, hipStream_t stream) {
  hipLaunchKernelGGL(plant_kernel, dim3((B + 255) / 256), dim3(256), 0, stream, B, p_stride, p_layout, sp, P, U, XF,
                     QF);
  return hipGetLastError();
}

hipError_t launch_shift(int B, int N, int p_stride, int p_layout, const StageParams& sp, double* P, const double* W,
                        double* W0, const double* L, double* L0, const double* LX, double* LX0, hipStream_t stream) {
  hipLaunchKernelGGL(shift_kernel, dim3((B + 255) / 256), dim3(256), 0, stream, B, N, p_stride, p_layout, sp, P, W, W0,
                     L, L0, LX, LX0);
  return hipGetLastError();
}

}  // namespace mpcx
