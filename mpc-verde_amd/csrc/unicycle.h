// unicycle.h -- interval map F of the unicycle MPC and its exact derivatives, on
// the device (gfx950, fp64).
//
// Reference: Casadi/multiple_shooting_casadi.py
//   f   = (v cos th, v sin th, omega), L = (s-xr)^T Q (s-xr) + u^T R u   :68-96
//   F   = M RK4 substeps of DT = T/M on (x, q), q += DT/6 (L1+2L2+2L3+L4) :98-114
// and the mpctools node-cost variant (Trajectory Tracking/Trajectory_tracking.py:51-61):
//   F   = RK4 (M=1) on x only, q = l(x_k, u_k, p_k).
//
// Structure used (exact, not an approximation): theta' = omega is constant on an
// interval, so every RK4 stage angle is th + t_j*omega with t_j = j*DT/2,
// j = 0..2M, and RK4's k2 == k3.  Hence
//   xf = x + v * sum_j a_j cos(th + t_j w),   yf = y + v * sum_j a_j sin(...)
// with Simpson weights a_j = DT/6 {1,4,2,...,4,1}, and each stage point of the
// cost quadrature is (x + v*a, y + v*b, th + tau*w) where a, b are partial sums
// of the same cos/sin values.  Derivatives w.r.t. (th, w) of such sums only need
// the t-moments sum a_j t_j^p cos_j (p = 0, 1, 2), so the exact Jacobian and the
// exact Hessian of  fs*q + lam^T xf  cost a handful of FMAs per stage point
// instead of an AD tape.  The 2M+1 angles form an arithmetic progression, so
// only sincos(th) and sincos(DT/2 * w) are evaluated; the rest follow by exact
// rotation (c' = c cd - s sd, s' = s cd + c sd), ~2 ulp per step.
#pragma once
#include <hip/hip_runtime.h>

#include "collectives.h"

namespace mpcx {

constexpr int NX = 3, NU = 2, NZ = 5, NH = 15;

// packed upper-triangular index of the symmetric 5x5 stage Hessian, z = (x, y, th, v, w)
__host__ __device__ constexpr int hix(int i, int j) {
  return i <= j ? i * NZ - i * (i - 1) / 2 + (j - i) : j * NZ - j * (j - 1) / 2 + (i - j);
}

// sincos of a small argument: the RK4 rotation angle DT/2 * w is tiny (|w| <= pi/4 inside its
// bounds, DT/2 <= 0.1), where the Taylor series to x^13 is exact to far below an ulp
// (|x| < 0.1: truncation < 1e-23) and much cheaper than the general routine's argument
// reduction; larger arguments take the library path.
__device__ __forceinline__ void sincos_small(double x, double* s, double* c) {
  if (fabs(x) < 0.1) {
    const double x2 = x * x;
    double ps = -1.0 / 39916800.0;
    ps = fma(ps, x2, 1.0 / 362880.0);
    ps = fma(ps, x2, -1.0 / 5040.0);
    ps = fma(ps, x2, 1.0 / 120.0);
    ps = fma(ps, x2, -1.0 / 6.0);
    *s = fma(x * x2, ps, x);
    double pc = 1.0 / 479001600.0;
    pc = fma(pc, x2, -1.0 / 3628800.0);
    pc = fma(pc, x2, 1.0 / 40320.0);
    pc = fma(pc, x2, -1.0 / 720.0);
    pc = fma(pc, x2, 1.0 / 24.0);
    pc = fma(pc, x2, -0.5);
    *c = fma(x2, pc, 1.0);
  } else {
    sincos(x, s, c);
  }
}

struct StageParams {
  double T, h;      // interval, substep DT = T/M
  int M;            // RK4 substeps
  int cost;         // 0 quadrature, 1 node
  double Q[3], R[2];
};

// Value of F: xf (3) and q.  Used by the line search and the plant.
__device__ __forceinline__ void uni_value(const StageParams& sp, const double x[3], const double u[2],
                                          const double xr[3], const double ur[2], double xf[3], double& q) {
  const double v = u[0], w = u[1], th = x[2];
  const double h = sp.h, hh = 0.5 * h, h6 = h / 6.0;
  double Ac = 0.0, As = 0.0;
  double s0, c0, sd, cd;
  sincos(th, &s0, &c0);
  sincos_small(hh * w, &sd, &cd);
  double t0 = 0.0;
  double qs = 0.0;
  for (int m = 0; m < sp.M; ++m) {
    const double tm = t0 + hh, te = t0 + h;
    const double c1 = c0 * cd - s0 * sd, s1 = s0 * cd + c0 * sd;
    const double c2 = c1 * cd - s1 * sd, s2 = s1 * cd + c1 * sd;
    if (sp.cost == 0) {
      // stage points of substep m: (beta, angle index) = (0,-), (hh, t0), (hh, tm), (h, tm)
      auto Lp = [&](double a, double b, double tau) {
        const double dx = x[0] + v * a - xr[0], dy = x[1] + v * b - xr[1], dt = th + tau * w - xr[2];
        return sp.Q[0] * dx * dx + sp.Q[1] * dy * dy + sp.Q[2] * dt * dt;
      };
      qs += h6 * (Lp(Ac, As, t0) + 2.0 * Lp(Ac + hh * c0, As + hh * s0, tm) +
                  2.0 * Lp(Ac + hh * c1, As + hh * s1, tm) + Lp(Ac + h * c1, As + h * s1, te));
    }
    Ac += h6 * (c0 + 4.0 * c1 + c2);
    As += h6 * (s0 + 4.0 * s1 + s2);
    c0 = c2;
    s0 = s2;
    t0 = te;
  }
  xf[0] = x[0] + v * Ac;
  xf[1] = x[1] + v * As;
  xf[2] = th + sp.T * w;
  const double dv = v - ur[0], dw = w - ur[1];
  if (sp.cost == 0) {
    q = qs + sp.T * (sp.R[0] * dv * dv + sp.R[1] * dw * dw);
  } else {
    const double dx = x[0] - xr[0], dy = x[1] - xr[1], dt = th - xr[2];
    q = sp.Q[0] * dx * dx + sp.Q[1] * dy * dy + sp.Q[2] * dt * dt + sp.R[0] * dv * dv + sp.R[1] * dw * dw;
  }
}

// Value, Jacobian and the exact Hessian of fs*q + lam^T xf, quadrature cost, by weighted moments.
//
// Every quadrature point p (weight w, angle offset tau) has Dx = xi_x + v a, Dy = xi_y + v b,
// Dt = xi_t + tau w with xi = state - reference and (a, b, a1, b1, a2, b2) the partial sums of
// the point; the derivatives of a, b w.r.t. (th, w) are -b, a / -b1, a1 (and of a1, b1 w.r.t. w:
// -b2, a2).  Substituting Dx, Dy into the per-point gradient and Hessian terms (uni_derivs below)
// leaves sums over the points of products of (a, b, a1, b1, a2, b2): 6 linear and 11 quadratic
// weighted moments, accumulated with ~21 FMAs per point, and the gradient and Hessian are
// assembled from them once per interval (the per-point formula costs ~90).  The value q keeps
// the per-point sum of the quadratic cost, so the line search's objective is the same expression.
//
// RS = 2 (replicated lane groups, kernels.h R = 2): the two replicas of a node -- lanes l and l + 32
// of the wave, rho = 0 / 1 -- split the RK4 substeps: replica 0 takes the quadrature points of
// substeps [0, M/2), replica 1 those of [M/2, M) after advancing the rotation and partial sums over
// the first half without points (the same operations, so its state there has the bits replica 0's
// would have).  The moments of the two halves are added in one fixed order (lower + upper half, so
// both replicas hold the same bits) and both take replica 1's end-of-interval partial sums.
//
// RS = 1 (one lane per node, models that also run replicated): the same two half-sums on one lane,
// so that a node's bits do not depend on whether its group was replicated.  RS = 0: one sequential
// sum (models that never run replicated: the halves would only hold more registers).
template <int RS = 1>
__device__ __forceinline__ void uni_derivs_moments(const StageParams& sp, const double x[3], const double u[2],
                                                   const double xr[3], const double ur[2], const double lam[3],
                                                   double fs, double xf[3], double& q, double A[9], double Bm[6],
                                                   double g[5], double H[15], int rho = 0) {
  static_assert(RS >= 0 && RS <= 2, "sequential, split on one lane, or two replicas");
  const double v = u[0], w = u[1], th = x[2];
  const double h = sp.h, hh = 0.5 * h, h6 = h / 6.0, h3 = h / 3.0, third = 1.0 / 3.0;
  const double xix = x[0] - xr[0], xiy = x[1] - xr[1], xit = th - xr[2];
  // partial sums of the interval so far (position increments per unit speed, t- and t^2-moments)
  double Ac = 0, As = 0, Ac1 = 0, As1 = 0, Ac2 = 0, As2 = 0;
  // weighted moments over the quadrature points
  double Sa = 0, Sb = 0, Sa1 = 0, Sb1 = 0, Sa2 = 0, Sb2 = 0;
  double Saa = 0, Sbb = 0, Sab = 0, Saa1 = 0, Sbb1 = 0, Sab1 = 0, Sba1 = 0, Sa1a1 = 0, Sb1b1 = 0, Saa2 = 0, Sbb2 = 0;
  double W0 = 0, Wt = 0, Wtt = 0;  // sum w, sum w tau, sum w tau^2
  double qs = 0.0;
  double s0, c0, sd, cd;
  sincos(th, &s0, &c0);
  sincos_small(hh * w, &sd, &cd);
  // hh-scaled cos/sin of the substep's first angle and their t, t^2 multiples
  double t0 = 0.0;
  double u0 = hh * c0, v0 = hh * s0, u0t = 0.0, v0t = 0.0, u0tt = 0.0, v0tt = 0.0;
  auto point = [&](double a, double b, double a1, double b1, double a2, double b2, double tau, double wt)
                   __attribute__((always_inline)) {
    const double Dx = fma(v, a, xix), Dy = fma(v, b, xiy), Dt = fma(tau, w, xit);
    qs = fma(wt, fma(sp.Q[0] * Dx, Dx, fma(sp.Q[1] * Dy, Dy, sp.Q[2] * Dt * Dt)), qs);
    const double aw = wt * a, bw = wt * b, a1w = wt * a1, b1w = wt * b1;
    Sa += aw;
    Sb += bw;
    Sa1 += a1w;
    Sb1 += b1w;
    Sa2 = fma(wt, a2, Sa2);
    Sb2 = fma(wt, b2, Sb2);
    Saa = fma(aw, a, Saa);
    Sbb = fma(bw, b, Sbb);
    Sab = fma(aw, b, Sab);
    Saa1 = fma(aw, a1, Saa1);
    Sbb1 = fma(bw, b1, Sbb1);
    Sab1 = fma(aw, b1, Sab1);
    Sba1 = fma(bw, a1, Sba1);
    Sa1a1 = fma(a1w, a1, Sa1a1);
    Sb1b1 = fma(b1w, b1, Sb1b1);
    Saa2 = fma(aw, a2, Saa2);
    Sbb2 = fma(bw, b2, Sbb2);
    W0 += wt;
    Wt = fma(wt, tau, Wt);
    Wtt = fma(wt * tau, tau, Wtt);
  };
  // one RK4 substep: its quadrature points (pts) and the advance of the rotation and partial sums
  auto substep = [&](bool pts) __attribute__((always_inline)) {
    const double tm = t0 + hh, te = t0 + h;
    const double c1 = c0 * cd - s0 * sd, s1 = s0 * cd + c0 * sd;
    const double c2 = c1 * cd - s1 * sd, s2 = s1 * cd + c1 * sd;
    const double u1 = hh * c1, v1 = hh * s1, u1t = tm * u1, v1t = tm * v1, u1tt = tm * u1t, v1tt = tm * v1t;
    const double u2 = hh * c2, v2 = hh * s2, u2t = te * u2, v2t = te * v2, u2tt = te * u2t, v2tt = te * v2t;
    if (pts && sp.cost == 0) {
      // RK4 stage points: (x, th_0), (x + hh f(th_0), th_1), (x + hh f(th_1), th_1), (x + h f(th_1), th_2)
      point(Ac, As, Ac1, As1, Ac2, As2, t0, h6);
      point(Ac + u0, As + v0, Ac1 + u0t, As1 + v0t, Ac2 + u0tt, As2 + v0tt, tm, h3);
      point(Ac + u1, As + v1, Ac1 + u1t, As1 + v1t, Ac2 + u1tt, As2 + v1tt, tm, h3);
      point(fma(2.0, u1, Ac), fma(2.0, v1, As), fma(2.0, u1t, Ac1), fma(2.0, v1t, As1), fma(2.0, u1tt, Ac2),
            fma(2.0, v1tt, As2), te, h6);
    }
    // Simpson: h6 (f0 + 4 f1 + f2) = (u0 + 4 u1 + u2) / 3 in hh-scaled terms
    Ac = fma(third, fma(4.0, u1, u0 + u2), Ac);
    As = fma(third, fma(4.0, v1, v0 + v2), As);
    Ac1 = fma(third, fma(4.0, u1t, u0t + u2t), Ac1);
    As1 = fma(third, fma(4.0, v1t, v0t + v2t), As1);
    Ac2 = fma(third, fma(4.0, u1tt, u0tt + u2tt), Ac2);
    As2 = fma(third, fma(4.0, v1tt, v0tt + v2tt), As2);
    c0 = c2;
    s0 = s2;
    u0 = u2;
    v0 = v2;
    u0t = u2t;
    v0t = v2t;
    u0tt = u2tt;
    v0tt = v2tt;
    t0 = te;
  };
  if constexpr (RS == 0) {
    for (int m = 0; m < sp.M; ++m) substep(true);
  } else if constexpr (RS == 1) {
    // the same two half-sums as the replicas (lower + upper), so that an instance's bits do not
    // depend on whether its batch runs replicated groups (a property of B and the SIMD count)
    const int M0 = sp.M / 2;
    for (int m = 0; m < M0; ++m) substep(true);
#define MPCX_UNI_MOMENTS(X) \
  X(qs) X(Sa) X(Sb) X(Sa1) X(Sb1) X(Sa2) X(Sb2) X(Saa) X(Sbb) X(Sab) X(Saa1) X(Sbb1) X(Sab1) X(Sba1) X(Sa1a1) \
  X(Sb1b1) X(Saa2) X(Sbb2) X(W0) X(Wt) X(Wtt)
#define MPCX_LO_TAKE(s) const double lo_##s = s; s = 0.0;
#define MPCX_LO_ADD(s) s = lo_##s + s;
    MPCX_UNI_MOMENTS(MPCX_LO_TAKE)
    for (int m = M0; m < sp.M; ++m) substep(true);
    if (sp.cost == 0) { MPCX_UNI_MOMENTS(MPCX_LO_ADD) }
#undef MPCX_LO_ADD
#undef MPCX_LO_TAKE
#undef MPCX_UNI_MOMENTS
  } else {
    const int M0 = sp.M / 2;  // replica 0: substeps [0, M0), replica 1: [M0, M)
    for (int m = 0; m < M0; ++m)
      if (rho == 1) substep(false);
    for (int m = 0; m < sp.M - M0; ++m)
      if (rho == 1 || m < M0) substep(true);
    // moments: lower + upper half on both replicas; the partial sums: replica 1's (the interval's end)
    auto sum2 = [](double& s) __attribute__((always_inline)) {
      const Pair p = halves32(s);
      s = p.a + p.b;
    };
    auto upper = [](double& s) __attribute__((always_inline)) { s = halves32(s).b; };
    if (sp.cost == 0) {
      sum2(qs);
      sum2(Sa); sum2(Sb); sum2(Sa1); sum2(Sb1); sum2(Sa2); sum2(Sb2);
      sum2(Saa); sum2(Sbb); sum2(Sab); sum2(Saa1); sum2(Sbb1); sum2(Sab1); sum2(Sba1); sum2(Sa1a1);
      sum2(Sb1b1); sum2(Saa2); sum2(Sbb2);
      sum2(W0); sum2(Wt); sum2(Wtt);
    }
    upper(Ac); upper(As); upper(Ac1); upper(As1); upper(Ac2); upper(As2);
  }
  const double T = sp.T;
  xf[0] = x[0] + v * Ac;
  xf[1] = x[1] + v * As;
  xf[2] = th + T * w;
  A[0] = 1.0; A[1] = 0.0; A[2] = -v * As;
  A[3] = 0.0; A[4] = 1.0; A[5] = v * Ac;
  A[6] = 0.0; A[7] = 0.0; A[8] = 1.0;
  Bm[0] = Ac; Bm[1] = -v * As1;
  Bm[2] = As; Bm[3] = v * Ac1;
  Bm[4] = 0.0; Bm[5] = T;
  const double dv = u[0] - ur[0], dw = u[1] - ur[1];
  const double Cx = 2.0 * fs * sp.Q[0], Cy = 2.0 * fs * sp.Q[1], Ct = 2.0 * fs * sp.Q[2];
  const double lx = lam[0], ly = lam[1];
  if (sp.cost != 0) {  // node cost (mpctools, Trajectory_tracking.py:51-61): l(x_k, u_k, p_k)
    q = sp.Q[0] * xix * xix + sp.Q[1] * xiy * xiy + sp.Q[2] * xit * xit + sp.R[0] * dv * dv + sp.R[1] * dw * dw;
    g[0] = Cx * xix;
    g[1] = Cy * xiy;
    g[2] = Ct * xit;
    g[3] = 2.0 * sp.R[0] * fs * dv;
    g[4] = 2.0 * sp.R[1] * fs * dw;
#pragma unroll
    for (int i = 0; i < 15; ++i) H[i] = 0.0;
    H[hix(0, 0)] = Cx;
    H[hix(1, 1)] = Cy;
    H[hix(2, 2)] = Ct - v * (lx * Ac + ly * As);
    H[hix(3, 3)] = 2.0 * sp.R[0] * fs;
    H[hix(4, 4)] = 2.0 * sp.R[1] * fs - v * (lx * Ac2 + ly * As2);
    H[hix(2, 3)] = ly * Ac - lx * As;
    H[hix(2, 4)] = -v * (lx * Ac1 + ly * As1);
    H[hix(3, 4)] = ly * Ac1 - lx * As1;
    return;
  }
  q = qs + T * (sp.R[0] * dv * dv + sp.R[1] * dw * dw);
  // gradient and Hessian of fs q (C = 2 fs Q) from the moments
  const double Xa = fma(v, Saa, xix * Sa), Xb = fma(v, Sab, xix * Sb);     // sum w Dx a, sum w Dx b
  const double Ya = fma(v, Sab, xiy * Sa), Yb = fma(v, Sbb, xiy * Sb);     // sum w Dy a, sum w Dy b
  const double Xa1 = fma(v, Saa1, xix * Sa1), Xb1 = fma(v, Sab1, xix * Sb1);
  const double Ya1 = fma(v, Sba1, xiy * Sa1), Yb1 = fma(v, Sbb1, xiy * Sb1);
  const double Xa2 = fma(v, Saa2, xix * Sa2), Yb2 = fma(v, Sbb2, xiy * Sb2);
  const double Tsum = fma(w, Wt, xit * W0), Ttau = fma(w, Wtt, xit * Wt);  // sum w Dt, sum w Dt tau
  const double vv = v * v;
  g[0] = Cx * fma(v, Sa, xix * W0);
  g[1] = Cy * fma(v, Sb, xiy * W0);
  g[2] = fma(v, Cy * Ya - Cx * Xb, Ct * Tsum);
  g[3] = fma(Cx, Xa, Cy * Yb);
  g[4] = fma(v, Cy * Ya1 - Cx * Xb1, Ct * Ttau);
  H[hix(0, 0)] = Cx * W0;
  H[hix(0, 1)] = 0.0;
  H[hix(0, 2)] = -v * (Cx * Sb);
  H[hix(0, 3)] = Cx * Sa;
  H[hix(0, 4)] = -v * (Cx * Sb1);
  H[hix(1, 1)] = Cy * W0;
  H[hix(1, 2)] = v * (Cy * Sa);
  H[hix(1, 3)] = Cy * Sb;
  H[hix(1, 4)] = v * (Cy * Sa1);
  H[hix(2, 2)] = fma(vv, fma(Cx, Sbb, Cy * Saa), fma(-v, fma(Cx, Xa, Cy * Yb), Ct * W0));
  H[hix(2, 3)] = fma(v * Sab, Cy - Cx, Cy * Ya - Cx * Xb);
  H[hix(2, 4)] = fma(vv, fma(Cx, Sbb1, Cy * Saa1), fma(-v, fma(Cx, Xa1, Cy * Yb1), Ct * Wt));
  H[hix(3, 3)] = fma(Cx, Saa, Cy * Sbb);
  H[hix(3, 4)] = fma(v, Cy * Sba1 - Cx * Sab1, Cy * Ya1 - Cx * Xb1);
  H[hix(4, 4)] = fma(vv, fma(Cx, Sb1b1, Cy * Sa1a1), fma(-v, fma(Cx, Xa2, Cy * Yb2), Ct * Wtt));
  g[3] += 2.0 * T * sp.R[0] * fs * dv;
  g[4] += 2.0 * T * sp.R[1] * fs * dw;
  H[hix(3, 3)] += 2.0 * T * sp.R[0] * fs;
  H[hix(4, 4)] += 2.0 * T * sp.R[1] * fs;
  H[hix(2, 2)] -= v * (lx * Ac + ly * As);
  H[hix(2, 3)] += ly * Ac - lx * As;
  H[hix(2, 4)] -= v * (lx * Ac1 + ly * As1);
  H[hix(3, 4)] += ly * Ac1 - lx * As1;
  H[hix(4, 4)] -= v * (lx * Ac2 + ly * As2);
}

// Value, Jacobian and (if WANT_H) the exact Hessian of fs*q + lam^T xf.
//   A (3x3 row-major) = dxf/dx, Bm (3x2) = dxf/du, g (5) = fs * dq/dz,
//   H (15 packed) = fs * d2q/dz2 + sum_c lam_c d2xf_c/dz2.
template <bool WANT_H>
__device__ __forceinline__ void uni_derivs(const StageParams& sp, const double x[3], const double u[2],
                                           const double xr[3], const double ur[2], const double lam[3], double fs,
                                           double xf[3], double& q, double A[9], double Bm[6], double g[5],
                                           double H[15]) {
  const double v = u[0], w = u[1], th = x[2];
  const double h = sp.h, hh = 0.5 * h, h6 = h / 6.0;
  double Ac = 0, As = 0, Ac1 = 0, As1 = 0, Ac2 = 0, As2 = 0;
#pragma unroll
  for (int i = 0; i < 5; ++i) g[i] = 0.0;
  if (WANT_H) {
#pragma unroll
    for (int i = 0; i < 15; ++i) H[i] = 0.0;
  }
  double qs = 0.0;
  double s0, c0, sd, cd;
  sincos(th, &s0, &c0);
  sincos_small(hh * w, &sd, &cd);
  double t0 = 0.0;
  const double Qx = sp.Q[0] * fs, Qy = sp.Q[1] * fs, Qt = sp.Q[2] * fs;
  for (int m = 0; m < sp.M; ++m) {
    const double tm = t0 + hh, te = t0 + h;
    const double c1 = c0 * cd - s0 * sd, s1 = s0 * cd + c0 * sd;
    const double c2 = c1 * cd - s1 * sd, s2 = s1 * cd + c1 * sd;
    if (sp.cost == 0) {
      // one quadrature point: partial sums (a,b) and their t-moments, offset tau, weight wt
      auto point = [&](double a, double b, double a1, double b1, double a2, double b2, double tau, double wt) {
        const double Dx = x[0] + v * a - xr[0], Dy = x[1] + v * b - xr[1], Dt = th + tau * w - xr[2];
        qs += wt * (sp.Q[0] * Dx * Dx + sp.Q[1] * Dy * Dy + sp.Q[2] * Dt * Dt);
        const double cx = 2.0 * wt * Qx, cy = 2.0 * wt * Qy, ct = 2.0 * wt * Qt;
        const double ex = cx * Dx, ey = cy * Dy, et = ct * Dt;
        g[0] += ex;
        g[1] += ey;
        g[2] += v * (ey * a - ex * b) + et;
        g[3] += ex * a + ey * b;
        g[4] += v * (ey * a1 - ex * b1) + et * tau;
        if (WANT_H) {
          H[hix(0, 0)] += cx;
          H[hix(1, 1)] += cy;
          H[hix(0, 2)] -= cx * v * b;
          H[hix(0, 3)] += cx * a;
          H[hix(0, 4)] -= cx * v * b1;
          H[hix(1, 2)] += cy * v * a;
          H[hix(1, 3)] += cy * b;
          H[hix(1, 4)] += cy * v * a1;
          const double vv = v * v;
          H[hix(2, 2)] += vv * (cx * b * b + cy * a * a) + ct - v * (ex * a + ey * b);
          H[hix(2, 3)] += v * a * b * (cy - cx) + ey * a - ex * b;
          H[hix(2, 4)] += vv * (cx * b * b1 + cy * a * a1) + ct * tau - v * (ex * a1 + ey * b1);
          H[hix(3, 3)] += cx * a * a + cy * b * b;
          H[hix(3, 4)] += v * (cy * b * a1 - cx * a * b1) + ey * a1 - ex * b1;
          H[hix(4, 4)] += vv * (cx * b1 * b1 + cy * a1 * a1) + ct * tau * tau - v * (ex * a2 + ey * b2);
        }
      };
      const double h3 = h / 3.0;
      point(Ac, As, Ac1, As1, Ac2, As2, t0, h6);
      point(Ac + hh * c0, As + hh * s0, Ac1 + hh * t0 * c0, As1 + hh * t0 * s0, Ac2 + hh * t0 * t0 * c0,
            As2 + hh * t0 * t0 * s0, tm, h3);
      point(Ac + hh * c1, As + hh * s1, Ac1 + hh * tm * c1, As1 + hh * tm * s1, Ac2 + hh * tm * tm * c1,
            As2 + hh * tm * tm * s1, tm, h3);
      point(Ac + h * c1, As + h * s1, Ac1 + h * tm * c1, As1 + h * tm * s1, Ac2 + h * tm * tm * c1,
            As2 + h * tm * tm * s1, te, h6);
    }
    Ac += h6 * (c0 + 4.0 * c1 + c2);
    As += h6 * (s0 + 4.0 * s1 + s2);
    Ac1 += h6 * (t0 * c0 + 4.0 * tm * c1 + te * c2);
    As1 += h6 * (t0 * s0 + 4.0 * tm * s1 + te * s2);
    if (WANT_H) {
      Ac2 += h6 * (t0 * t0 * c0 + 4.0 * tm * tm * c1 + te * te * c2);
      As2 += h6 * (t0 * t0 * s0 + 4.0 * tm * tm * s1 + te * te * s2);
    }
    c0 = c2;
    s0 = s2;
    t0 = te;
  }
  const double T = sp.T;
  xf[0] = x[0] + v * Ac;
  xf[1] = x[1] + v * As;
  xf[2] = th + T * w;
  A[0] = 1.0; A[1] = 0.0; A[2] = -v * As;
  A[3] = 0.0; A[4] = 1.0; A[5] = v * Ac;
  A[6] = 0.0; A[7] = 0.0; A[8] = 1.0;
  Bm[0] = Ac; Bm[1] = -v * As1;
  Bm[2] = As; Bm[3] = v * Ac1;
  Bm[4] = 0.0; Bm[5] = T;
  const double dv = u[0] - ur[0], dw = u[1] - ur[1];
  if (sp.cost == 0) {
    q = qs + T * (sp.R[0] * dv * dv + sp.R[1] * dw * dw);
    g[3] += 2.0 * T * sp.R[0] * fs * dv;
    g[4] += 2.0 * T * sp.R[1] * fs * dw;
    if (WANT_H) {
      H[hix(3, 3)] += 2.0 * T * sp.R[0] * fs;
      H[hix(4, 4)] += 2.0 * T * sp.R[1] * fs;
    }
  } else {
    const double dx = x[0] - xr[0], dy = x[1] - xr[1], dt = th - xr[2];
    q = sp.Q[0] * dx * dx + sp.Q[1] * dy * dy + sp.Q[2] * dt * dt + sp.R[0] * dv * dv + sp.R[1] * dw * dw;
    g[0] = 2.0 * Qx * dx;
    g[1] = 2.0 * Qy * dy;
    g[2] = 2.0 * Qt * dt;
    g[3] = 2.0 * sp.R[0] * fs * dv;
    g[4] = 2.0 * sp.R[1] * fs * dw;
    if (WANT_H) {
      H[hix(0, 0)] = 2.0 * Qx;
      H[hix(1, 1)] = 2.0 * Qy;
      H[hix(2, 2)] = 2.0 * Qt;
      H[hix(3, 3)] = 2.0 * sp.R[0] * fs;
      H[hix(4, 4)] = 2.0 * sp.R[1] * fs;
    }
  }
  if (WANT_H) {
    const double lx = lam[0], ly = lam[1];
    H[hix(2, 2)] -= v * (lx * Ac + ly * As);
    H[hix(2, 3)] += ly * Ac - lx * As;
    H[hix(2, 4)] -= v * (lx * Ac1 + ly * As1);
    H[hix(3, 4)] += ly * Ac1 - lx * As1;
    H[hix(4, 4)] -= v * (lx * Ac2 + ly * As2);
  }
}

}  // namespace mpcx
