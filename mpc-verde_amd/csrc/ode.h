// ode.h -- nonlinear ODE stage models with exact derivatives (second-order forward mode, or
// forward sensitivities with stage adjoints).
//
// The BASELINE configs name three nonlinear models that the reference only has in linearised
// or renamed form.  Each is written once, templated on its scalar
// type, and integrated by the same RK4 as the unicycle (M substeps of h = T/M):
//
//   KinBicycle   x = (X, Y, psi), u = (v, delta); psi' = v tan(delta) / L
//                (the "kinematic bicycle" of config 3; Trajectory Tracking/Trajectory_tracking.py
//                tracks with a unicycle)
//   DynBicycle   x = (X, Y, psi, vx, vy, r), u = (delta, ax), linear tyres with the
//                reference's constants m, a, b, Ca, Jz (Trajectory_tracking_dynamic_model.py:36-42).
//                Its linearisation at vx = vref, small delta, is exactly the reference's LTV
//                lateral model (:119-128, A34 with the intended precedence).
//   CartPole     x = (p, p', phi, phi'), u = F; M, m, L, g, friction c.  Its linearisation at
//                phi = 0 is exactly the reference's Ac, Bc with M = m = 1, L = 0.5, c = 10
//                (Inverted_pendulum/inverted_pendulum_single_shooting_mpctools.py:19-23).
//
// Derivatives.  The 6-state bicycle: forward sensitivities and stage adjoints through RK4 with
// closed-form partials of f (OdeModel::derivs_adjoint, below).  The others, and the 6-state
// model's reference path: a hyper-dual number v + a e1 + b e2 + ab e1e2 (e1^2 = e2^2 = 0) carries the
// first derivatives along two seed directions and the mixed second derivative.  One RK4 pass
// seeded with (e_i, e_j) gives columns i and j of dF/dz and d2F/dz_i dz_j exactly (no
// truncation).  Passes run over the pairs of variables whose second derivatives through the RK4
// map can be non-zero (NLMASK) plus one pass per remaining variable; the passes share one RK4
// body (runtime loop) so code size does not grow with the pair count.  NLMASK is every variable
// f reads, not only those entering f nonlinearly: RK4 composes f with itself, so a variable
// that enters f linearly (the bicycle's ax) still couples nonlinearly through the states it
// drives (d2F/dax dvx != 0; tests/test_ode_cpu.py checks the mask against the oracle's
// Hessian).  Variables f never reads (INDEP) have unit Jacobian columns and no curvature.  The stage cost is the mpctools node cost
// l = sum Q_i (x_i - xr_i)^2 + sum R_j (u_j - ur_j)^2 (exact gradient and Hessian in closed form).
#pragma once
#include <hip/hip_runtime.h>

#include "riccati.h"
#include "solver.h"

namespace mpcx {

using ::cos;  // the double overloads stay visible next to the HD ones below
using ::sin;
using ::tan;

struct HD {
  double v, a, b, ab;
};
__device__ __forceinline__ HD operator+(HD x, HD y) { return {x.v + y.v, x.a + y.a, x.b + y.b, x.ab + y.ab}; }
__device__ __forceinline__ HD operator-(HD x, HD y) { return {x.v - y.v, x.a - y.a, x.b - y.b, x.ab - y.ab}; }
__device__ __forceinline__ HD operator-(HD x) { return {-x.v, -x.a, -x.b, -x.ab}; }
__device__ __forceinline__ HD operator+(HD x, double c) { return {x.v + c, x.a, x.b, x.ab}; }
__device__ __forceinline__ HD operator+(double c, HD x) { return {x.v + c, x.a, x.b, x.ab}; }
__device__ __forceinline__ HD operator-(HD x, double c) { return {x.v - c, x.a, x.b, x.ab}; }
__device__ __forceinline__ HD operator-(double c, HD x) { return {c - x.v, -x.a, -x.b, -x.ab}; }
__device__ __forceinline__ HD operator*(HD x, double c) { return {x.v * c, x.a * c, x.b * c, x.ab * c}; }
__device__ __forceinline__ HD operator*(double c, HD x) { return {x.v * c, x.a * c, x.b * c, x.ab * c}; }
__device__ __forceinline__ HD operator*(HD x, HD y) {
  return {x.v * y.v, fma(x.a, y.v, x.v * y.a), fma(x.b, y.v, x.v * y.b),
          fma(x.ab, y.v, fma(x.a, y.b, fma(x.b, y.a, x.v * y.ab)))};
}
__device__ __forceinline__ HD recip(HD y) {
  const double r = 1.0 / y.v, m = -r * r;  // d(1/y) = -y'/y^2, d2 = -y''/y^2 + 2 y'_a y'_b / y^3
  return {r, m * y.a, m * y.b, fma(m, y.ab, -2.0 * m * r * y.a * y.b)};
}
__device__ __forceinline__ HD operator/(HD x, HD y) { return x * recip(y); }
__device__ __forceinline__ HD operator/(double c, HD y) { return c * recip(y); }
__device__ __forceinline__ HD sin(HD x) {
  double s, c;
  sincos(x.v, &s, &c);
  return {s, c * x.a, c * x.b, fma(c, x.ab, -s * x.a * x.b)};
}
__device__ __forceinline__ HD cos(HD x) {
  double s, c;
  sincos(x.v, &s, &c);
  return {c, -s * x.a, -s * x.b, -fma(s, x.ab, c * x.a * x.b)};
}
__device__ __forceinline__ HD tan(HD x) {
  const double t = ::tan(x.v), d = fma(t, t, 1.0);  // tan' = 1 + tan^2, tan'' = 2 tan (1 + tan^2)
  return {t, d * x.a, d * x.b, fma(d, x.ab, 2.0 * t * d * x.a * x.b)};
}

// Transcendental values of f's stage evaluations.  Every hyper-dual pass runs RK4 through
// the same stage points (the passes differ only in their seed directions), so the value parts
// of sin/cos/tan/reciprocals are the same in every pass: the value pass records them in a
// per-lane LDS cache (TrigRecord), the passes read them back (TrigReplay) and only form the
// derivative parts.  TrigDirect evaluates (value(), plants, horizons past the cache).
// Arguments tagged _u depend on the inputs only (constant over the RK4 substeps): one slot.
struct TrigDirect {
  __device__ __forceinline__ void sincos_x(double x, double& s, double& c) { ::sincos(x, &s, &c); }
  __device__ __forceinline__ void sincos_u(double x, double& s, double& c) { ::sincos(x, &s, &c); }
  __device__ __forceinline__ double recip_x(double x) { return 1.0 / x; }
  __device__ __forceinline__ double div_x(double n, double d) { return n / d; }
  __device__ __forceinline__ double tan_u(double x) { return ::tan(x); }
  __device__ __forceinline__ void sincos_x(HD x, HD& s, HD& c) { s = sin(x); c = cos(x); }
  __device__ __forceinline__ void sincos_u(HD x, HD& s, HD& c) { s = sin(x); c = cos(x); }
  __device__ __forceinline__ HD recip_x(HD x) { return recip(x); }
  __device__ __forceinline__ HD div_x(HD n, HD d) { return n / d; }
  __device__ __forceinline__ HD tan_u(HD x) { return tan(x); }
  template <int NX, class S>
  __device__ __forceinline__ void substep(int, const S*) {}
};
// slots: [0, 2) input-only (sincos_u or tan_u), then per stage evaluation in call order
struct TrigRecord {
  double* buf;  // this lane's slot 0; slot i at buf[i * stride]
  int stride, idx;
  __device__ __forceinline__ void put(double v) { buf[(idx++) * stride] = v; }
  __device__ __forceinline__ void sincos_x(double x, double& s, double& c) {
    ::sincos(x, &s, &c);
    put(s);
    put(c);
  }
  __device__ __forceinline__ void sincos_u(double x, double& s, double& c) {
    ::sincos(x, &s, &c);
    buf[0] = s;
    buf[stride] = c;
  }
  __device__ __forceinline__ double recip_x(double x) {
    const double r = 1.0 / x;
    put(r);
    return r;
  }
  // n / d as an IEEE division (the value path keeps its bits); 1/d recorded for the passes
  __device__ __forceinline__ double div_x(double n, double d) {
    put(1.0 / d);
    return n / d;
  }
  __device__ __forceinline__ double tan_u(double x) {
    const double t = ::tan(x);
    buf[0] = t;
    return t;
  }
  template <int NX, class S>
  __device__ __forceinline__ void substep(int, const S*) {}
};
struct TrigReplay {
  const double* buf;
  int stride, idx;
  __device__ __forceinline__ double get() { return buf[(idx++) * stride]; }
  __device__ __forceinline__ static void sc(double sv, double cv, HD x, HD& s, HD& c) {
    s = {sv, cv * x.a, cv * x.b, fma(cv, x.ab, -sv * x.a * x.b)};
    c = {cv, -sv * x.a, -sv * x.b, -fma(sv, x.ab, cv * x.a * x.b)};
  }
  __device__ __forceinline__ void sincos_x(HD x, HD& s, HD& c) {
    const double sv = get(), cv = get();
    sc(sv, cv, x, s, c);
  }
  __device__ __forceinline__ void sincos_u(HD x, HD& s, HD& c) { sc(buf[0], buf[stride], x, s, c); }
  __device__ __forceinline__ HD recip_x(HD y) {
    const double r = get(), m = -r * r;
    return {r, m * y.a, m * y.b, fma(m, y.ab, -2.0 * m * r * y.a * y.b)};
  }
  __device__ __forceinline__ HD div_x(HD n, HD d) { return n * recip_x(d); }
  __device__ __forceinline__ HD tan_u(HD x) {
    const double t = buf[0], d = fma(t, t, 1.0);
    return {t, d * x.a, d * x.b, fma(d, x.ab, 2.0 * t * d * x.a * x.b)};
  }
  template <int NX, class S>
  __device__ __forceinline__ void substep(int, const S*) {}
};
// The adjoint derivative path's evaluations (OdeModel::derivs_adjoint): transcendental values
// computed directly, as TrigDirect (so a value pass gives value()'s bits), with sincos of the
// input-only argument taken once per interval, the last f call's sincos(x) and reciprocal kept
// for its partials, and the state at each RK4 substep start stored to this lane's LDS column
// (checkpoints of the reverse pass)
struct TrigAdj {
  double* ck;  // checkpoint slot 0 (slot i at ck[i * stride]) or nullptr
  int stride;
  double su, cu;       // sincos of the input-only argument
  double sx, cx, rx;   // the last call's sincos_x and recip_x values
  __device__ __forceinline__ void sincos_x(double x, double& s, double& c) {
    ::sincos(x, &s, &c);
    sx = s;
    cx = c;
  }
  __device__ __forceinline__ void sincos_u(double, double& s, double& c) {
    s = su;
    c = cu;
  }
  __device__ __forceinline__ double recip_x(double x) {
    rx = 1.0 / x;
    return rx;
  }
  __device__ __forceinline__ double div_x(double n, double d) { return n / d; }
  __device__ __forceinline__ double tan_u(double x) { return ::tan(x); }
  template <int NX, class S>
  __device__ __forceinline__ void substep(int s, const S* x) {
    if (ck)
#pragma unroll
      for (int i = 0; i < NX; ++i) ck[(NX * s + i) * stride] = x[i];
  }
};

// ---------------------------------------------------------------------------- dynamics
struct KinBicycle {
  static constexpr int NX = 3, NU = 2;
  static constexpr bool kSOC = false;
  static constexpr unsigned NLMASK = (1u << 2) | (1u << 3) | (1u << 4);  // psi, v, delta
  static constexpr unsigned INDEP = (1u << 0) | (1u << 1);               // f does not read X, Y
  static constexpr int kTrigPerEval = 2, kTrigInput = 1, kTrigMaxM = 1;  // sincos(psi); tan(delta)
  static constexpr bool kAdjoint = false;  // derivatives by hyper-dual passes (OdeModel::derivs)
  template <class S, class Tc>
  __device__ __forceinline__ static void f(const S* x, const S* u, const double* par, S* dx, Tc& tc) {
    S sp, cp;
    tc.sincos_x(x[2], sp, cp);
    dx[0] = u[0] * cp;
    dx[1] = u[0] * sp;
    dx[2] = u[0] * tc.tan_u(u[1]) * (1.0 / par[0]);  // par = (L)
  }
};

struct DynBicycle {
  static constexpr int NX = 6, NU = 2;
  static constexpr bool kSOC = true;
  // psi, vx, vy, r, delta and ax: ax enters f linearly but drives vx, which enters nonlinearly,
  // so F has d2F/dax dz != 0 (X and Y are not read at all)
  static constexpr unsigned NLMASK = (1u << 2) | (1u << 3) | (1u << 4) | (1u << 5) | (1u << 6) | (1u << 7);
  static constexpr unsigned INDEP = (1u << 0) | (1u << 1);
  static constexpr int kTrigPerEval = 3, kTrigInput = 2, kTrigMaxM = 4;  // sincos(psi), 1/vx; sincos(delta)
  // closed-form partials below (OdeModel::derivs_adjoint).  A/B on one MI355X (config 4 lane
  // change, N = 50, alternating builds): 459-476 -> 258-261 us per IPM iteration, 136 k -> 337 k
  // solves/s in 10-step launches, lock-step 85 k -> 125 k, against the hyper-dual passes
  static constexpr bool kAdjoint = true;
  template <class S, class Tc>
  __device__ __forceinline__ static void f(const S* x, const S* u, const double* par, S* dx, Tc& tc) {
    // par = (m, a, b, Ca, Jz): Trajectory_tracking_dynamic_model.py:36-40 (a, b = CG-axle distances)
    const double m = par[0], a = par[1], b = par[2], Ca2 = 2.0 * par[3], Jz = par[4];
    const S psi = x[2], vx = x[3], vy = x[4], r = x[5], d = u[0];
    S sp, cp, sd, cd;
    tc.sincos_x(psi, sp, cp);
    const S ivx = tc.recip_x(vx);
    tc.sincos_u(d, sd, cd);
    const S Fyf = Ca2 * (d - (vy + a * r) * ivx);  // front axle: slip angle delta - (vy + a r)/vx
    const S Fyr = -Ca2 * ((vy - b * r) * ivx);     // rear axle: -(vy - b r)/vx
    dx[0] = vx * cp - vy * sp;
    dx[1] = vx * sp + vy * cp;
    dx[2] = r;
    dx[3] = u[1] + r * vy - Fyf * sd * (1.0 / m);
    dx[4] = (Fyf * cd + Fyr) * (1.0 / m) - vx * r;
    dx[5] = (a * (Fyf * cd) - b * Fyr) * (1.0 / Jz);
  }

  // ---- closed-form partials for the adjoint derivatives (OdeModel::derivs_adjoint).  f reads
  // the states psi, vx, vy, r (x[2..5]) and both inputs; v = (psi, vx, vy, r, delta, ax) below.
  // With w = 1/vx, P1 = vy + a r, P2 = vy - b r, C = 2 Ca:
  //   Fyf = C (delta - P1 w),  Fyr = -C P2 w,
  // and for an adjoint mu of f's value, mu^T f = mu0 f0 + mu1 f1 + mu2 r + mu3 (ax + r vy)
  // - mu4 vx r + Fyf al(delta) + Fyr be, with
  //   al = -mu3 sin(delta) / m + (mu4 / m + mu5 a / Jz) cos(delta),  be = mu4 / m - mu5 b / Jz,
  // so its gradient and Hessian follow from those of Fyf and Fyr (linear in vy, r and delta,
  // rational in vx) and of the rotation f0, f1 in psi.  tests/test_ode_cpu.py checks both
  // against complex steps of f.
  static constexpr int kVOff = 2;  // v[0..3] = x[kVOff..kVOff+3]
  struct Cst {
    double im, iJ, a, b, C;
  };
  __device__ __forceinline__ static Cst cst(const double* par) {
    return {1.0 / par[0], 1.0 / par[4], par[1], par[2], 2.0 * par[3]};
  }
  struct Blk {  // one stage point: what f's Jacobian and the Hessian of mu^T f need
    double vx, vy, r, sp, cp, w, P1, P2, Fyf, f0, f1;
  };
  __device__ __forceinline__ static Blk blk(const double* x, double d, double sp, double cp, double w, const Cst& k) {
    Blk s;
    s.vx = x[3];
    s.vy = x[4];
    s.r = x[5];
    s.sp = sp;
    s.cp = cp;
    s.w = w;
    s.P1 = fma(k.a, s.r, s.vy);
    s.P2 = fma(-k.b, s.r, s.vy);
    s.Fyf = k.C * fma(-s.P1, w, d);
    s.f0 = s.vx * cp - s.vy * sp;
    s.f1 = s.vx * sp + s.vy * cp;
    return s;
  }
  struct MuQ {  // the parts of an adjoint mu that its Hessian term needs
    double m0, m1, m3, m4, al, be, alp;  // alp = d al / d delta
  };
  __device__ __forceinline__ static MuQ muq(const double* mu, double sd, double cd, const Cst& k) {
    const double gam = fma(mu[5] * k.a, k.iJ, mu[4] * k.im);
    const double m3 = mu[3] * k.im;
    return {mu[0], mu[1], mu[3], mu[4], fma(gam, cd, -m3 * sd), fma(-mu[5] * k.b, k.iJ, mu[4] * k.im), -fma(m3, cd, gam * sd)};
  }
  // g = (d f / d(psi, vx, vy, r))^T mu
  __device__ __forceinline__ static void jt(const Blk& s, const double* mu, const MuQ& q, const Cst& k, double* g) {
    const double w2 = s.w * s.w, Cw = k.C * s.w;
    g[0] = fma(mu[1], s.f0, -mu[0] * s.f1);
    g[1] = fma(mu[0], s.cp, fma(mu[1], s.sp, fma(-mu[4], s.r, k.C * w2 * fma(s.P1, q.al, s.P2 * q.be))));
    g[2] = fma(mu[1], s.cp, fma(-mu[0], s.sp, fma(mu[3], s.r, -Cw * (q.al + q.be))));
    g[3] = mu[2] + fma(mu[3], s.vy, fma(-mu[4], s.vx, -Cw * fma(k.a, q.al, -k.b * q.be)));
  }
  // d f / dv: the rows of f3, f4, f5 over (vx, vy, r, delta) (the other entries are
  // -f1, cp, -sp / f0, sp, cp in rows 0, 1, the 1 of f2 in r and of f3 in ax)
  struct Jac {
    double j3[4], j4[4], j5[4];
  };
  __device__ __forceinline__ static Jac jac(const Blk& s, double sd, double cd, const Cst& k) {
    const double w2 = s.w * s.w;
    const double fvx = k.C * s.P1 * w2, fvy = -k.C * s.w, fr = -k.C * k.a * s.w;  // d Fyf
    const double rvx = k.C * s.P2 * w2, rvy = -k.C * s.w, rr = k.C * k.b * s.w;   // d Fyr
    const double sdm = sd * k.im;
    Jac J;
    J.j3[0] = -fvx * sdm;
    J.j3[1] = fma(-fvy, sdm, s.r);
    J.j3[2] = fma(-fr, sdm, s.vy);
    J.j3[3] = -fma(k.C, sd, s.Fyf * cd) * k.im;
    J.j4[0] = fma(fma(fvx, cd, rvx), k.im, -s.r);
    J.j4[1] = fma(fvy, cd, rvy) * k.im;
    J.j4[2] = fma(fma(fr, cd, rr), k.im, -s.vx);
    J.j4[3] = fma(k.C, cd, -s.Fyf * sd) * k.im;
    J.j5[0] = fma(k.a * fvx, cd, -k.b * rvx) * k.iJ;
    J.j5[1] = fma(k.a * fvy, cd, -k.b * rvy) * k.iJ;
    J.j5[2] = fma(k.a * fr, cd, -k.b * rr) * k.iJ;
    J.j5[3] = k.a * fma(k.C, cd, -s.Fyf * sd) * k.iJ;
    return J;
  }
  // the Hessian of mu^T f over v = (psi, vx, vy, r, delta) (ax enters linearly): its 11
  // structural non-zeros pp, pvx, pvy, xx, xy, xr, xd, yr, yd, rd, dd (vy-vy, r-r, psi-r and
  // psi-delta are zero)
  struct Hes {
    double pp, pvx, pvy, xx, xy, xr, xd, yr, yd, rd, dd;
  };
  __device__ __forceinline__ static Hes hes(const Blk& s, const MuQ& q, const Cst& k) {
    const double w2 = s.w * s.w, Cw = k.C * s.w, Cw2 = k.C * w2;
    Hes W;
    W.pp = -fma(q.m0, s.f0, q.m1 * s.f1);
    W.pvx = fma(-q.m0, s.sp, q.m1 * s.cp);
    W.pvy = -fma(q.m0, s.cp, q.m1 * s.sp);
    W.xx = -2.0 * Cw2 * s.w * fma(s.P1, q.al, s.P2 * q.be);
    W.xy = Cw2 * (q.al + q.be);
    W.xr = fma(Cw2, fma(k.a, q.al, -k.b * q.be), -q.m4);
    W.xd = Cw2 * s.P1 * q.alp;
    W.yr = q.m3;
    W.yd = -Cw * q.alp;
    W.rd = -Cw * k.a * q.alp;
    W.dd = fma(2.0 * k.C, q.alp, -s.Fyf * q.al);
    return W;
  }
};

struct CartPole {
  static constexpr int NX = 4, NU = 1;
  static constexpr bool kSOC = false;
  static constexpr unsigned NLMASK = (1u << 1) | (1u << 2) | (1u << 3) | (1u << 4);  // p', phi, phi', F
  static constexpr unsigned INDEP = (1u << 0);                                        // f does not read p
  static constexpr int kTrigPerEval = 3, kTrigInput = 0, kTrigMaxM = 1;  // sincos(phi), 1/(M + m sin^2 phi)
  static constexpr bool kAdjoint = false;
  template <class S, class Tc>
  __device__ __forceinline__ static void f(const S* x, const S* u, const double* par, S* dx, Tc& tc) {
    // par = (M, m, L, g, c); phi measured so that the upright linearisation is the reference's Ac
    const double Mc = par[0], m = par[1], L = par[2], g = par[3], c = par[4];
    S s, co;
    tc.sincos_x(x[2], s, co);
    const S pdd = tc.div_x(u[0] - c * x[1] - (m * L) * (x[3] * x[3]) * s + (m * g) * (s * co), Mc + m * (s * s));
    dx[0] = x[1];
    dx[1] = pdd;
    dx[2] = x[3];
    dx[3] = (g * s + co * pdd) * (1.0 / L);
  }
};

// RK4, M substeps, one f call site (the four stages are a runtime loop)
template <class Dyn, class S, class Tc>
__device__ __forceinline__ void ode_rk4(const S* x0, const S* u, const OdeParams& op, S* xf, Tc& tc) {
  constexpr int NX = Dyn::NX;
  S x[NX];
#pragma unroll
  for (int i = 0; i < NX; ++i) x[i] = x0[i];
  const double h = op.h;
#pragma unroll 1
  for (int s = 0; s < op.M; ++s) {
    tc.template substep<NX>(s, x);
    S acc[NX], xt[NX], k[NX];
#pragma unroll
    for (int i = 0; i < NX; ++i) xt[i] = x[i];
#pragma unroll 1
    for (int st = 0; st < 4; ++st) {
      Dyn::f(xt, u, op.par, k, tc);
      const double wa = (st == 0 || st == 3) ? 1.0 : 2.0;  // k1 + 2 k2 + 2 k3 + k4
      const double cn = (st == 2) ? h : 0.5 * h;           // next stage point x + c k
#pragma unroll
      for (int i = 0; i < NX; ++i) {
        acc[i] = st == 0 ? k[i] : acc[i] + wa * k[i];
        xt[i] = x[i] + cn * k[i];
      }
    }
#pragma unroll
    for (int i = 0; i < NX; ++i) x[i] = x[i] + (h / 6.0) * acc[i];
  }
#pragma unroll
  for (int i = 0; i < NX; ++i) xf[i] = x[i];
}

template <class Dyn>
struct OdeModel {
  static constexpr int NX = Dyn::NX, NU = Dyn::NU, NZ = NX + NU, NH = NZ * (NZ + 1) / 2;
  // a column of A is the unit vector e_j when f does not read x_j (F = x + h/6 (...))
  static constexpr unsigned long long amask() {
    unsigned long long m = 0;
    for (int c = 0; c < NX; ++c)
      for (int j = 0; j < NX; ++j)
        if (!((Dyn::INDEP >> j) & 1u) || c == j) m |= 1ull << (c * NX + j);
    return m;
  }
  static constexpr unsigned long long AMASK = amask();
  static constexpr unsigned long long BMASK = (1ull << (NX * NU)) - 1;
  static constexpr bool kEvalInSearch = false;
  // IPOPT's second-order correction (solver.hip line search, max_soc = 4), per model where it
  // measured better (one MI355X, bench --model): 6-state bicycle 24 k -> 105 k solves/s (lock-step
  // 4 k -> 53 k; max iterations 651 -> 66; failed instance-steps 10 -> 2).  Not enabled: the
  // kinematic bicycle (one config-3 instance then alternates SOC steps that trade feasibility
  // for barrier objective until max_iter, 1.09 M -> 0.27 M solves/s in multi-step launches,
  // though lock-step rises 0.47 M -> 2.19 M), the cart-pole (no gain; +14 % per iteration from
  // the extra registers).
  static constexpr bool kSOC = Dyn::kSOC;
  // IPOPT's soft restoration and feasibility restoration phase (kernels.h; state in the
  // restoration workspace): the nonlinear models are the ones whose line searches fail
  static constexpr bool kResto = true;
  // stage Hessian and Sigma of the 6-state model wait in the workspace across the inertia-
  // correction loop (kernels.h kWsStash): with them out of the registers the sequential chain's
  // operands no longer go through scratch once per step
  static constexpr bool kWsStash = NX >= 6;
  // variable bounds in LDS (kernels.h LdsCol) instead of 2 NZ doubles of registers held through
  // every phase.  A/B on one MI355X: cart-pole swing-up 122 -> 117 us per IPM iteration (scratch
  // 696 -> 204 B/lane), kinematic bicycle +1 % (scratch 400 -> 0); the 6-state bicycle, whose chain operands
  // already wait in the workspace, 3 % slower -- so not there
  static constexpr bool kBoundsLds = NX < 6;
  static constexpr bool kParallelRiccati = NX <= 5;  // NX = 6: LDS buffer too large
  // the 6-state model's chain runs spread over 16-lane rows (rowchain6.h; one instance per wave)
  static constexpr bool kRowChain = NX == 6;
  struct Ctx {
    double zr[NZ];
  };
  static constexpr bool kTableJac = false, kTableHess = false;
  __device__ __forceinline__ static const double* jacA(const Ctx&, const double* A) { return A; }
  __device__ __forceinline__ static const double* jacB(const Ctx&, const double* B) { return B; }
  __device__ __forceinline__ static const double* hessW(const Ctx&, const double* H) { return H; }
  __device__ __forceinline__ static void load_ctx(const ModelArgs& a, int inst, const double* P, int k, bool hasU, Ctx& c) {
#pragma unroll
    for (int i = 0; i < NZ; ++i) c.zr[i] = 0.0;
    if (a.p_layout == 0) {
#pragma unroll
      for (int i = 0; i < NX; ++i) c.zr[i] = P[NX + i];
    } else if (hasU) {
#pragma unroll
      for (int i = 0; i < NZ; ++i) c.zr[i] = P[NX + NZ * k + i];
    }
  }
  __device__ __forceinline__ static double wgt(const ModelArgs& a, int i) { return i < NX ? a.op.Q[i] : a.op.R[i - NX]; }
  // per-lane LDS cache of the stage evaluations' transcendental values (TrigRecord/Replay),
  // for up to Dyn::kTrigMaxM RK4 substeps (each model's default M; a larger M evaluates
  // directly) -- sized so that the cache and the Riccati scan buffer fit the LDS together
  static constexpr int kTrigMaxM = Dyn::kTrigMaxM;
  static constexpr int kTrigSlots = Dyn::kTrigInput + Dyn::kTrigPerEval * 4 * kTrigMaxM;
  template <class Tc>
  __device__ __forceinline__ static void value_tc(const ModelArgs& a, const Ctx& c, const double* z, double* xf,
                                                  double& q, Tc& tc) {
    ode_rk4<Dyn, double>(z, z + NX, a.op, xf, tc);
    double acc = 0.0;
#pragma unroll
    for (int i = 0; i < NZ; ++i) {
      const double d = z[i] - c.zr[i];
      acc = fma(wgt(a, i) * d, d, acc);
    }
    q = acc;
  }
  __device__ __forceinline__ static void value(const ModelArgs& a, const Ctx& c, const double* z, double* xf, double& q) {
    TrigDirect tc;
    ode_rk4<Dyn, double>(z, z + NX, a.op, xf, tc);
    double acc = 0.0;
#pragma unroll
    for (int i = 0; i < NZ; ++i) {
      const double d = z[i] - c.zr[i];
      acc = fma(wgt(a, i) * d, d, acc);
    }
    q = acc;
  }
  // F, q and their exact derivatives at z for the adjoint ln: the adjoint path where the model
  // has closed-form partials and its checkpoints fit this lane's LDS column, else hyper-dual passes
  __device__ __forceinline__ static void derivs(const ModelArgs& a, const Ctx& c, const double* z, const double* ln, double fs,
                                                double* xf, double& q, double* A, double* Bm, double* g, double* H) {
    if constexpr (Dyn::kAdjoint) {
      if (a.tc != nullptr && 2 * NX * a.op.M <= kTrigSlots) {  // kernel-uniform
        derivs_adjoint(a, c, z, ln, fs, xf, q, A, Bm, g, H);
        return;
      }
    }
    derivs_passes(a, c, z, ln, fs, xf, q, A, Bm, g, H);
  }
  // the mpctools node cost: q, its gradient and (diagonal) Hessian, scaled by fs
  __device__ __forceinline__ static void cost_derivs(const ModelArgs& a, const Ctx& c, const double* z, double fs,
                                                     double* g, double* H) {
#pragma unroll
    for (int i = 0; i < NH; ++i) H[i] = 0.0;
#pragma unroll
    for (int i = 0; i < NZ; ++i) {
      const double w2 = 2.0 * fs * wgt(a, i);
      g[i] = w2 * (z[i] - c.zr[i]);
      H[symix(i, i, NZ)] = w2;
    }
  }
  // Exact derivatives by forward sensitivities and stage adjoints (Dyn::kAdjoint: closed-form
  // partials of f).  Everything in RK4 but f is linear, so with mu_e the adjoint of stage e's f
  // value in lam^T F and Tv_e = dv_e/dz the sensitivity of the variables f reads at stage e,
  //   d2(lam^T F)/dz2 = sum_e Tv_e^T [d2(mu_e^T f)/dv2] Tv_e        (e over the 4 M stages).
  // Three passes over the interval: (A) the value as value() computes it, storing the state at
  // each substep start to this lane's LDS column; (B) backwards, the adjoint at each substep end
  // (stored next to them); (C) forwards, per substep: its stage points again, the stage adjoints
  // from the stored lam_{s+1}, then the sensitivities (6 x 6 over v) and the Hessian terms.
  // The 6-state bicycle (M = 4): ~14 k FP64 flops per interval against 107 k for its 21
  // hyper-dual passes (tests/test_gpu_ode.py compares the two).
  __device__ static void derivs_adjoint(const ModelArgs& a, const Ctx& c, const double* z, const double* ln, double fs,
                                        double* xf, double& q, double* A, double* Bm, double* g, double* H) {
    using D = Dyn;
    constexpr int NV = 6, VO = D::kVOff;  // v = (psi, vx, vy, r, delta, ax) = z[VO .. VO + 5]
    static_assert(NX == 6 && NU == 2 && VO == 2, "adjoint path written for the 6-state bicycle");
    using Blk = typename D::Blk;
    using MuQ = typename D::MuQ;
    const int M = a.op.M;
    const double h = a.op.h;
    double* ck = a.tc;  // slots [NX s, NX s + NX): x_s; [NX (M + s), ...): lam_{s+1}
    const int cs = a.tc_stride;
    const auto K = D::cst(a.op.par);
    const double* u = z + NX;
    double sd, cd;
    ::sincos(u[0], &sd, &cd);
    {  // (A)
      TrigAdj ta{ck, cs, sd, cd, 0.0, 0.0, 0.0};
      value_tc(a, c, z, xf, q, ta);
    }
    cost_derivs(a, c, z, fs, g, H);
    // stage points of substep s, from its checkpoint
    auto stages = [&](int s, Blk* B) __attribute__((always_inline)) {
      double x[NX], xt[NX];
#pragma unroll
      for (int i = 0; i < NX; ++i) xt[i] = x[i] = ck[(NX * s + i) * cs];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        TrigAdj tc{nullptr, 0, sd, cd, 0.0, 0.0, 0.0};
        double k[NX];
        D::f(xt, u, a.op.par, k, tc);
        B[e] = D::blk(xt, u[0], tc.sx, tc.cx, tc.rx, K);
        if (e < 3) {
          const double cn = (e == 2) ? h : 0.5 * h;
#pragma unroll
          for (int i = 0; i < NX; ++i) xt[i] = x[i] + cn * k[i];
        }
      }
    };
    // stage adjoints of a substep from l = lam_{s+1}; l becomes lam_s
    auto reverse = [&](const Blk* B, double* l, MuQ* Q) __attribute__((always_inline)) {
      double gn[4] = {0.0, 0.0, 0.0, 0.0}, gs[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int e = 3; e >= 0; --e) {
        const double cl = (e == 0 || e == 3) ? h / 6.0 : h / 3.0;  // dx_{s+1}/dk_e
        const double cg = (e == 2) ? h : 0.5 * h;                  // dxt_{e+1}/dk_e
        double mu[NX];
#pragma unroll
        for (int i = 0; i < NX; ++i) {
          mu[i] = cl * l[i];
          if (e < 3 && i >= VO && i < VO + 4) mu[i] = fma(cg, gn[i - VO], mu[i]);
        }
        Q[e] = D::muq(mu, sd, cd, K);
        D::jt(B[e], mu, Q[e], K, gn);
#pragma unroll
        for (int j = 0; j < 4; ++j) gs[j] += gn[j];
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) l[VO + j] += gs[j];
    };
    {  // (B)
      double l[NX];
#pragma unroll
      for (int i = 0; i < NX; ++i) l[i] = ln[i];
#pragma unroll 1
      for (int s = M - 1; s >= 0; --s) {
#pragma unroll
        for (int i = 0; i < NX; ++i) ck[(NX * (M + s) + i) * cs] = l[i];
        if (s == 0) break;
        Blk B[4];
        MuQ Q[4];
        stages(s, B);
        reverse(B, l, Q);
      }
    }
    // (C)
    double Tx[NX][NV], Hv[NV * (NV + 1) / 2];
#pragma unroll
    for (int r = 0; r < NX; ++r)
#pragma unroll
      for (int j = 0; j < NV; ++j) Tx[r][j] = (r >= VO && r - VO == j) ? 1.0 : 0.0;
#pragma unroll
    for (int i = 0; i < NV * (NV + 1) / 2; ++i) Hv[i] = 0.0;
#pragma unroll 1
    for (int s = 0; s < M; ++s) {
      Blk B[4];
      MuQ Q[4];
      stages(s, B);
      {
        double l[NX];
#pragma unroll
        for (int i = 0; i < NX; ++i) l[i] = ck[(NX * (M + s) + i) * cs];
        reverse(B, l, Q);
      }
      double acc[NX][NV], Tt[4][NV];  // Tt: the stage point's (psi, vx, vy, r) rows
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int j = 0; j < NV; ++j) Tt[r][j] = Tx[VO + r][j];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const auto W = D::hes(B[e], Q[e], K);
        // Hv += Tv^T W Tv, Tv = (Tt; e_delta; e_ax)
#pragma unroll
        for (int j = 0; j < NV; ++j) {
          const double tp = Tt[0][j], tx = Tt[1][j], ty = Tt[2][j], tr = Tt[3][j];
          double wp = fma(W.pp, tp, fma(W.pvx, tx, W.pvy * ty));
          double wx = fma(W.pvx, tp, fma(W.xx, tx, fma(W.xy, ty, W.xr * tr)));
          double wy = fma(W.pvy, tp, fma(W.xy, tx, W.yr * tr));
          double wr = fma(W.xr, tx, W.yr * ty);
          double wd = fma(W.xd, tx, fma(W.yd, ty, W.rd * tr));
          if (j == 4) {  // the delta column of Tv is e_delta
            wx += W.xd;
            wy += W.yd;
            wr += W.rd;
            wd += W.dd;
          }
#pragma unroll
          for (int i = 0; i <= j; ++i) {
            double v = fma(Tt[0][i], wp, fma(Tt[1][i], wx, fma(Tt[2][i], wy, Tt[3][i] * wr)));
            if (i == 4) v += wd;
            Hv[symix(i, j, NV)] += v;
          }
        }
        // sensitivities: Tk = (df/dv) Tv, then the RK4 combination and the next stage point
        const auto J = D::jac(B[e], sd, cd, K);
        const double wa = (e == 0 || e == 3) ? 1.0 : 2.0;
        const double cn = (e == 2) ? h : 0.5 * h;
#pragma unroll
        for (int j = 0; j < NV; ++j) {
          const double tp = Tt[0][j], tx = Tt[1][j], ty = Tt[2][j], tr = Tt[3][j];
          double tk[NX];
          tk[0] = fma(-B[e].f1, tp, fma(B[e].cp, tx, -B[e].sp * ty));
          tk[1] = fma(B[e].f0, tp, fma(B[e].sp, tx, B[e].cp * ty));
          tk[2] = tr;
          tk[3] = fma(J.j3[0], tx, fma(J.j3[1], ty, J.j3[2] * tr));
          tk[4] = fma(J.j4[0], tx, fma(J.j4[1], ty, J.j4[2] * tr));
          tk[5] = fma(J.j5[0], tx, fma(J.j5[1], ty, J.j5[2] * tr));
          if (j == 4) {
            tk[3] += J.j3[3];
            tk[4] += J.j4[3];
            tk[5] += J.j5[3];
          }
          if (j == 5) tk[3] += 1.0;  // f3 = ax + ...
#pragma unroll
          for (int r = 0; r < NX; ++r) acc[r][j] = (e == 0) ? tk[r] : fma(wa, tk[r], acc[r][j]);
          if (e < 3)
#pragma unroll
            for (int r = 0; r < 4; ++r) Tt[r][j] = fma(cn, tk[VO + r], Tx[VO + r][j]);
        }
      }
#pragma unroll
      for (int r = 0; r < NX; ++r)
#pragma unroll
        for (int j = 0; j < NV; ++j) Tx[r][j] = fma(h / 6.0, acc[r][j], Tx[r][j]);
    }
#pragma unroll
    for (int r = 0; r < NX; ++r) {
#pragma unroll
      for (int j = 0; j < NX; ++j) A[r * NX + j] = (j < VO) ? (r == j ? 1.0 : 0.0) : Tx[r][j - VO];
#pragma unroll
      for (int l = 0; l < NU; ++l) Bm[r * NU + l] = Tx[r][NX - VO + l];
    }
#pragma unroll
    for (int i = 0; i < NV; ++i)
#pragma unroll
      for (int j = i; j < NV; ++j) H[symix(VO + i, VO + j, NZ)] += Hv[symix(i, j, NV)];
  }
  // derivatives by hyper-dual RK4 passes (every model; the 6-state bicycle's reference path)
  __device__ __forceinline__ static void derivs_passes(const ModelArgs& a, const Ctx& c, const double* z, const double* ln,
                                                       double fs, double* xf, double& q, double* A, double* Bm, double* g,
                                                       double* H) {
    const bool cached = a.tc != nullptr && a.op.M <= kTrigMaxM;  // kernel-uniform
    if (cached) {
      TrigRecord rec{a.tc, a.tc_stride, Dyn::kTrigInput};
      value_tc(a, c, z, xf, q, rec);
    } else {
      value(a, c, z, xf, q);
    }
#pragma unroll
    for (int i = 0; i < NH; ++i) H[i] = 0.0;
#pragma unroll
    for (int i = 0; i < NZ; ++i) {
      const double w2 = 2.0 * fs * wgt(a, i);
      g[i] = w2 * (z[i] - c.zr[i]);
      H[symix(i, i, NZ)] = w2;
    }
#pragma unroll
    for (int i = 0; i < NX * NX; ++i) A[i] = 0.0;
#pragma unroll
    for (int i = 0; i < NX * NU; ++i) Bm[i] = 0.0;
    // passes (m, n): every pair of nonlinear variables, and (m, m) for the others
#pragma unroll 1
    for (int m = 0; m < NZ; ++m) {
      const bool nlm = (Dyn::NLMASK >> m) & 1u;
#pragma unroll 1
      for (int n = m; n < NZ; ++n) {
        if (n != m && !(nlm && ((Dyn::NLMASK >> n) & 1u))) continue;
        if (m < NX && n == m && ((Dyn::INDEP >> m) & 1u)) {  // column e_m, no curvature
#pragma unroll
          for (int r = 0; r < NX; ++r)
#pragma unroll
            for (int j = 0; j < NX; ++j)
              if (j == m) A[r * NX + j] = r == j ? 1.0 : 0.0;
          continue;
        }
        HD zs[NZ], xs[NX];
#pragma unroll
        for (int i = 0; i < NZ; ++i) zs[i] = HD{z[i], i == m ? 1.0 : 0.0, i == n ? 1.0 : 0.0, 0.0};
        if (cached) {
          TrigReplay rp{a.tc, a.tc_stride, Dyn::kTrigInput};
          ode_rk4<Dyn, HD>(zs, zs + NX, a.op, xs, rp);
        } else {
          TrigDirect td;
          ode_rk4<Dyn, HD>(zs, zs + NX, a.op, xs, td);
        }
        double s = 0.0;
#pragma unroll
        for (int r = 0; r < NX; ++r) {
          s = fma(ln[r], xs[r].ab, s);
#pragma unroll
          for (int j = 0; j < NZ; ++j) {
            double* e = j < NX ? &A[r * NX + j] : &Bm[r * NU + (j - NX)];
            if (j == m) *e = xs[r].a;
            else if (j == n) *e = xs[r].b;
          }
        }
#pragma unroll
        for (int i = 0; i < NZ; ++i)
#pragma unroll
          for (int j = i; j < NZ; ++j)
            if (i == m && j == n) H[symix(i, j, NZ)] += s;
      }
    }
  }
};

}  // namespace mpcx
