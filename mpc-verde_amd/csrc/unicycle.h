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
