// ipm_ref.cpp -- C++ CPU restatement of the multiple-shooting MPC NLPs and of an
// IPOPT-style primal-dual interior-point solve of them.
//
// TEST INFRASTRUCTURE ONLY.  Built by oracle/Makefile into oracle/libipm_ref.so
// and loaded (ctypes, oracle/ipm_ref.py) only by tests/, __graft_entry__.smoke()
// and bench.py's cpu_baseline leg -- as the checker and as the timed CPU baseline,
// never as the product.  Parity: pinned against tests/golden/unicycle_N10_golden.json
// (the reference's own CasADi+IPOPT outputs) and against oracle/nlp_ref.py in
// tests/test_oracle.py; the ODE models against oracle/ode_ref.py (tests/test_ode_cpu.py).
//
// What it restates (paths relative to /root/reference):
//   NLP     Casadi/multiple_shooting_casadi.py:68-114 (unicycle f, L, RK4 with
//           cost quadrature, M substeps), :116-178 (interleaved w, lifted X_0,
//           defect constraints g, J = sum qf, bounds on U), and the mpctools
//           tracking variant Trajectory Tracking/Trajectory_tracking.py:40-67
//           (node cost l(x,u,p_k), RK4 M=1, state bounds).  The same NLP shape over
//           the BASELINE's nonlinear ODE variants (kinematic bicycle, 6-state dynamic
//           bicycle, cart-pole; equations in mpc-verde_amd/mpcx/ode.py).
//   Solver  ca.nlpsol(..., 'ipopt', ...) at :181-197 with the options of :188-196
//           (max_iter, acceptable_tol, acceptable_obj_change_tol), i.e. IPOPT
//           (third-party, not vendored; version unpinned: the reference has no
//           requirements file).  Restated from its published algorithm (Waechter &
//           Biegler, Math. Prog. 106, 2006) and documented option semantics:
//           monotone Fiacco-McCormick barrier update (fast monotone decrease),
//           fraction-to-the-boundary rule, primal-dual bound multipliers, inertia
//           correction by Hessian regularisation, filter line search with switching
//           condition and Armijo rule, filter reset heuristic, kappa_Sigma safeguard,
//           tiny-step acceptance, gradient-based objective scaling; termination
//           (tol with the unscaled dual_inf_tol / constr_viol_tol / compl_inf_tol
//           tests, acceptable level after acceptable_iter iterations, acceptable
//           point at a line-search failure); soft restoration (primal-dual error
//           reduction) and the feasibility restoration phase of W&B 2006 §3.3
//           (min rho ||p + n||_1 + zeta/2 ||D_R (x - x_R)||^2 s.t. c(x) - p + n = 0).
//           Exact Hessian of the Lagrangian (IPOPT default with CasADi).
//
// Implementation choices that are deliberately DIFFERENT from the HIP product
// (so this file checks it independently):
//   * derivatives by second-order forward-mode jets (value, gradient, Hessian)
//     pushed through the RK4 chain -- the product uses first-order tangents plus
//     a second-order adjoint (unicycle) or hyper-dual pair passes (ODE models);
//   * one instance at a time, plain arrays, the restoration phase's p, n
//     eliminated per constraint row of a dense stage recursion; OpenMP over instances.

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>
#include <cstdio>
#include <cstdlib>
#ifdef _OPENMP
#include <omp.h>
#endif

namespace {

constexpr int nh(int nz) { return nz * (nz + 1) / 2; }
template <int NZ>
inline int hix(int i, int j) {  // packed upper-triangular index
  if (i > j) std::swap(i, j);
  return i * NZ - i * (i - 1) / 2 + (j - i);
}

// Second-order forward-mode jet over the NZ stage variables.
template <int NZ>
struct Jet {
  double v;
  double g[NZ];
  double h[nh(NZ)];
};
template <int NZ>
inline Jet<NZ> jconst(double c) {
  Jet<NZ> r;
  r.v = c;
  std::memset(r.g, 0, sizeof r.g);
  std::memset(r.h, 0, sizeof r.h);
  return r;
}
template <int NZ>
inline Jet<NZ> operator+(const Jet<NZ>& a, const Jet<NZ>& b) {
  Jet<NZ> r;
  r.v = a.v + b.v;
  for (int i = 0; i < NZ; ++i) r.g[i] = a.g[i] + b.g[i];
  for (int i = 0; i < nh(NZ); ++i) r.h[i] = a.h[i] + b.h[i];
  return r;
}
template <int NZ>
inline Jet<NZ> operator-(const Jet<NZ>& a, const Jet<NZ>& b) {
  Jet<NZ> r;
  r.v = a.v - b.v;
  for (int i = 0; i < NZ; ++i) r.g[i] = a.g[i] - b.g[i];
  for (int i = 0; i < nh(NZ); ++i) r.h[i] = a.h[i] - b.h[i];
  return r;
}
template <int NZ>
inline Jet<NZ> operator*(double s, const Jet<NZ>& a) {
  Jet<NZ> r;
  r.v = s * a.v;
  for (int i = 0; i < NZ; ++i) r.g[i] = s * a.g[i];
  for (int i = 0; i < nh(NZ); ++i) r.h[i] = s * a.h[i];
  return r;
}
template <int NZ>
inline Jet<NZ> operator*(const Jet<NZ>& a, double s) { return s * a; }
template <int NZ>
inline Jet<NZ> operator+(const Jet<NZ>& a, double c) {
  Jet<NZ> r = a;
  r.v = a.v + c;
  return r;
}
template <int NZ>
inline Jet<NZ> operator+(double c, const Jet<NZ>& a) { return a + c; }
template <int NZ>
inline Jet<NZ> operator-(double c, const Jet<NZ>& a) { return jconst<NZ>(c) - a; }
template <int NZ>
inline Jet<NZ> operator*(const Jet<NZ>& a, const Jet<NZ>& b) {
  Jet<NZ> r;
  r.v = a.v * b.v;
  for (int i = 0; i < NZ; ++i) r.g[i] = a.v * b.g[i] + b.v * a.g[i];
  for (int i = 0; i < NZ; ++i)
    for (int j = i; j < NZ; ++j) {
      const int k = hix<NZ>(i, j);
      r.h[k] = a.v * b.h[k] + b.v * a.h[k] + a.g[i] * b.g[j] + a.g[j] * b.g[i];
    }
  return r;
}
// scalar function with f, f', f'' at a.v
template <int NZ>
inline Jet<NZ> jfun(const Jet<NZ>& a, double f0, double f1, double f2) {
  Jet<NZ> r;
  r.v = f0;
  for (int i = 0; i < NZ; ++i) r.g[i] = f1 * a.g[i];
  for (int i = 0; i < NZ; ++i)
    for (int j = i; j < NZ; ++j) {
      const int k = hix<NZ>(i, j);
      r.h[k] = f1 * a.h[k] + f2 * a.g[i] * a.g[j];
    }
  return r;
}
template <int NZ>
inline Jet<NZ> cos(const Jet<NZ>& a) {
  const double c = std::cos(a.v), s = std::sin(a.v);
  return jfun(a, c, -s, -c);
}
template <int NZ>
inline Jet<NZ> sin(const Jet<NZ>& a) {
  const double c = std::cos(a.v), s = std::sin(a.v);
  return jfun(a, s, c, -s);
}
template <int NZ>
inline Jet<NZ> tan(const Jet<NZ>& a) {
  const double t = std::tan(a.v), d = 1.0 + t * t;
  return jfun(a, t, d, 2.0 * t * d);
}
// n / d with the value an IEEE division (as the double path computes it)
template <int NZ>
inline Jet<NZ> operator/(const Jet<NZ>& n, const Jet<NZ>& d) {
  const double r = 1.0 / d.v;
  Jet<NZ> q = n * jfun(d, r, -r * r, 2.0 * r * r * r);
  q.v = n.v / d.v;
  return q;
}
template <int NZ>
inline Jet<NZ> operator/(double c, const Jet<NZ>& d) {
  return jconst<NZ>(c) / d;
}

// ---------------------------------------------------------------------------
// Models: f(x, u) written once over the scalar type (double or Jet)
// ---------------------------------------------------------------------------
using std::cos;
using std::sin;
using std::tan;

// Casadi/multiple_shooting_casadi.py:68-72
struct Unicycle {
  static constexpr int NX = 3, NU = 2;
  template <class S>
  static void f(const double*, const S* x, const S* u, S* o) {
    o[0] = u[0] * cos(x[2]);
    o[1] = u[0] * sin(x[2]);
    o[2] = u[1];
  }
};
// kinematic bicycle, par = (L)
struct KinBicycle {
  static constexpr int NX = 3, NU = 2;
  template <class S>
  static void f(const double* par, const S* x, const S* u, S* o) {
    o[0] = u[0] * cos(x[2]);
    o[1] = u[0] * sin(x[2]);
    o[2] = u[0] * tan(u[1]) * (1.0 / par[0]);
  }
};
// 6-state dynamic bicycle on linear tyres, par = (m, a, b, Ca, Jz)
// (Trajectory_tracking_dynamic_model.py:36-40 constants)
struct DynBicycle {
  static constexpr int NX = 6, NU = 2;
  template <class S>
  static void f(const double* par, const S* x, const S* u, S* o) {
    const double m = par[0], a = par[1], b = par[2], Ca = par[3], Jz = par[4];
    const S vx = x[3], vy = x[4], r = x[5], d = u[0];
    const S alpha_f = d - (vy + a * r) / vx;
    const S alpha_r = 0.0 - (vy - b * r) / vx;
    const S Fyf = (2.0 * Ca) * alpha_f, Fyr = (2.0 * Ca) * alpha_r;
    const S sp = sin(x[2]), cp = cos(x[2]), sd = sin(d), cd = cos(d);
    o[0] = vx * cp - vy * sp;
    o[1] = vx * sp + vy * cp;
    o[2] = r;
    o[3] = u[1] + r * vy - Fyf * sd * (1.0 / m);
    o[4] = (Fyf * cd + Fyr) * (1.0 / m) - vx * r;
    o[5] = (a * Fyf * cd - b * Fyr) * (1.0 / Jz);
  }
};
// cart-pole, par = (M, m, L, g, c)
struct CartPole {
  static constexpr int NX = 4, NU = 1;
  template <class S>
  static void f(const double* par, const S* x, const S* u, S* o) {
    const double Mc = par[0], m = par[1], L = par[2], g = par[3], c = par[4];
    const S s = sin(x[2]), co = cos(x[2]);
    const S pdd = (u[0] - c * x[1] - (m * L) * (x[3] * x[3]) * s + (m * g) * (s * co)) / (Mc + m * (s * s));
    o[0] = x[1];
    o[1] = pdd;
    o[2] = x[3];
    o[3] = (g * s + co * pdd) * (1.0 / L);
  }
};

}  // namespace

extern "C" {

// Mirrors the fields of mpcx_spec (include/mpcx.h) that the unicycle entry points need.
typedef struct oracle_spec {
  int32_t N, M;
  int32_t cost;  // 0 = RK4 quadrature of L (CasADi scripts), 1 = node cost (mpctools)
  int32_t max_iter;
  double T;
  double Q[3], R[2];
  double tol;
} oracle_spec;

// Any model (oracle_solve): model 1 unicycle, 3 kinematic bicycle, 4 dynamic bicycle, 5 cart-pole
typedef struct oracle_problem {
  int32_t model, N, M, cost;
  int32_t p_layout;  // 0: P = [x0; x_ref (nx)], 1: P = [x0; (x_ref_k, u_ref_k) x N]
  int32_t pad;
  double T;
  double Q[8], R[8], par[8];
} oracle_problem;

// IPOPT options (names and defaults of IPOPT's documentation)
typedef struct oracle_opts {
  double tol;                         // 1e-8
  double dual_inf_tol;                // 1
  double constr_viol_tol;             // 1e-4
  double compl_inf_tol;               // 1e-4
  double acceptable_tol;              // 1e-6
  double acceptable_dual_inf_tol;     // 1e10
  double acceptable_constr_viol_tol;  // 1e-2
  double acceptable_compl_inf_tol;    // 1e-2
  double acceptable_obj_change_tol;   // 1e20
  int32_t max_iter;                   // 3000
  int32_t acceptable_iter;            // 15
  int32_t restoration;                // 1: soft restoration + restoration phase; 0: a failed line search ends the solve
  int32_t max_soc;                    // IPOPT max_soc (second-order corrections per line search; IPOPT 4)
} oracle_opts;

}  // extern "C"

namespace {

// IPOPT constants (Waechter & Biegler 2006, Table 1 / IPOPT defaults)
constexpr double kEps = 2.220446049250313e-16;
constexpr double kKappaEps = 10.0, kKappaMu = 0.2, kThetaMu = 1.5, kTauMin = 0.99;
constexpr double kKappaSigma = 1e10, kSmax = 100.0;
constexpr double kGammaTheta = 1e-5, kGammaPhi = 1e-8, kDelta = 1.0, kSTheta = 1.1, kSPhi = 2.3;
constexpr double kEtaPhi = 1e-8, kGammaAlpha = 0.05;
constexpr double kDw0 = 1e-4, kDwMin = 1e-20, kDwMax = 1e40, kKwMinus = 1.0 / 3, kKwPlus = 8, kKwPlusBar = 100;
constexpr double kBoundPush = 1e-2, kBoundFrac = 1e-2, kInfBound = 1e19;
// soft restoration (soft_resto_pderror_reduction_factor, max_soft_resto_iters) and the
// restoration phase (W&B 2006 §3.3: rho, kappa_resto = required_infeasibility_reduction,
// zeta = sqrt(mu_R) proximity weight; bound_mult_reset_threshold; constr_mult_reset_threshold
// = 0: constraint multipliers restart at 0)
constexpr double kSoftResto = 0.9999;
constexpr int kMaxSoftResto = 10;
constexpr double kRho = 1000.0, kKappaResto = 0.9, kBoundMultReset = 1000.0;

// ORACLE_TRACE=1 in the environment: one line per solve event (diagnostics)
inline bool tracing() {
  static const bool t = std::getenv("ORACLE_TRACE") != nullptr;
  return t;
}
#define TRACE(...)                    \
  do {                                \
    if (tracing()) printf(__VA_ARGS__); \
  } while (0)

enum Status { kConverged = 0, kAcceptable = 1, kMaxIter = 2, kRestoFailed = 3, kInfeasible = 4, kStepFailed = 5 };

inline double sqr(double a) { return a * a; }

template <class Dyn>
struct Inst {
  static constexpr int NX = Dyn::NX, NU = Dyn::NU, NZ = NX + NU, NH = nh(NX + NU);
  const oracle_problem* pb;
  int N, nw, ng;
  std::vector<double> zr;  // N x NZ stage references (x_ref_k, u_ref_k)
  double x0[NX];
  std::vector<double> lb, ub;
  std::vector<char> hasL, hasU;
  double fscale = 1.0;
  int ix(int k, int i) const { return k == 0 ? i : NX + NZ * (k - 1) + NU + i; }  // x_k[i] in w
  int iu(int k, int i) const { return NX + NZ * k + i; }                          // u_k[i] in w
};

// One interval: RK4 with M substeps; cost 0 = RK4 quadrature of L (Casadi scripts
// :98-114), 1 = node cost at (x_k, u_k) (mpctools).  S = double or Jet: the jets' .v
// follow exactly the double arithmetic.
template <class Dyn, class S>
void stage(const oracle_problem& pb, const double* zr, const S* X0, const S* U, S* xf, S& qf) {
  constexpr int NX = Dyn::NX, NU = Dyn::NU;
  auto cost_L = [&](const S* x) {
    S acc = S(X0[0]) * 0.0;
    for (int i = 0; i < NX; ++i) {
      const S d = x[i] + (-zr[i]);
      acc = acc + pb.Q[i] * (d * d);
    }
    for (int i = 0; i < NU; ++i) {
      const S d = U[i] + (-zr[NX + i]);
      acc = acc + pb.R[i] * (d * d);
    }
    return acc;
  };
  S X[NX];
  for (int i = 0; i < NX; ++i) X[i] = X0[i];
  const double DT = pb.T / pb.M;
  S q = S(X0[0]) * 0.0;
  if (pb.cost == 1) q = cost_L(X);
  for (int m = 0; m < pb.M; ++m) {
    S k1[NX], k2[NX], k3[NX], k4[NX], s[NX];
    Dyn::f(pb.par, X, U, k1);
    for (int i = 0; i < NX; ++i) s[i] = X[i] + (DT / 2) * k1[i];
    S L2 = pb.cost == 0 ? cost_L(s) : q * 0.0;
    Dyn::f(pb.par, s, U, k2);
    for (int i = 0; i < NX; ++i) s[i] = X[i] + (DT / 2) * k2[i];
    S L3 = pb.cost == 0 ? cost_L(s) : q * 0.0;
    Dyn::f(pb.par, s, U, k3);
    for (int i = 0; i < NX; ++i) s[i] = X[i] + DT * k3[i];
    S L4 = pb.cost == 0 ? cost_L(s) : q * 0.0;
    Dyn::f(pb.par, s, U, k4);
    if (pb.cost == 0) {
      S L1 = cost_L(X);
      q = q + (DT / 6) * (L1 + 2.0 * L2 + 2.0 * L3 + L4);
    }
    for (int i = 0; i < NX; ++i) X[i] = X[i] + (DT / 6) * (k1[i] + 2.0 * k2[i] + 2.0 * k3[i] + k4[i]);
  }
  for (int i = 0; i < NX; ++i) xf[i] = X[i];
  qf = q;
}

// jets seeded at (x, u)
template <class Dyn>
void stage_jet(const oracle_problem& pb, const double* zr, const double* x, const double* u,
               Jet<Dyn::NX + Dyn::NU>* xf, Jet<Dyn::NX + Dyn::NU>& qf) {
  constexpr int NX = Dyn::NX, NU = Dyn::NU, NZ = NX + NU;
  Jet<NZ> X[NX], U[NU];
  for (int i = 0; i < NX; ++i) {
    X[i] = jconst<NZ>(x[i]);
    X[i].g[i] = 1.0;
  }
  for (int i = 0; i < NU; ++i) {
    U[i] = jconst<NZ>(u[i]);
    U[i].g[NX + i] = 1.0;
  }
  stage<Dyn, Jet<NZ>>(pb, zr, X, U, xf, qf);
}

template <class Dyn>
struct Eval {
  double f;                  // fscale * sum q
  double qsum;               // sum q (unscaled objective)
  std::vector<double> grad;  // nw, gradient of fscale * sum q
  std::vector<double> c;     // ng
  std::vector<double> A, Bm; // N x NX*NX, N x NX*NU
  std::vector<double> H;     // N x NH: Hessian of fscale * q_k + lam_{k+1}^T F_k
};

template <class Dyn>
void evaluate(const Inst<Dyn>& I, const double* w, const double* lam, bool derivs, Eval<Dyn>& e) {
  constexpr int NX = Dyn::NX, NU = Dyn::NU, NZ = NX + NU, NH = nh(NZ);
  const int N = I.N;
  e.f = 0;
  e.qsum = 0;
  e.c.assign(I.ng, 0.0);
  if (derivs) {
    e.grad.assign(I.nw, 0.0);
    e.A.assign(N * NX * NX, 0.0);
    e.Bm.assign(N * NX * NU, 0.0);
    e.H.assign(N * NH, 0.0);
  }
  for (int i = 0; i < NX; ++i) e.c[i] = I.x0[i] - w[I.ix(0, i)];
  for (int k = 0; k < N; ++k) {
    // interval 0 integrates from the parameter x0 (Casadi/multiple_shooting_casadi.py:125,157:
    // Xk = P[:n_states], F(x0=vertcat(Xk, P[3:]), p=U_0)): the lifted X_0 enters only g_0, so
    // stage 0 has no derivative with respect to it (A_0 = 0, no x-gradient, no x Hessian blocks)
    double xk[NX], uk[NU], xn[NX];
    for (int i = 0; i < NX; ++i) {
      xk[i] = k == 0 ? I.x0[i] : w[I.ix(k, i)];
      xn[i] = w[I.ix(k + 1, i)];
    }
    for (int i = 0; i < NU; ++i) uk[i] = w[I.iu(k, i)];
    const double* zr = &I.zr[NZ * k];
    if (!derivs) {
      double xf[NX], qf;
      stage<Dyn, double>(*I.pb, zr, xk, uk, xf, qf);
      e.f += I.fscale * qf;
      e.qsum += qf;
      for (int i = 0; i < NX; ++i) e.c[NX * (k + 1) + i] = xf[i] - xn[i];
      continue;
    }
    Jet<NZ> xf[NX], qf;
    stage_jet<Dyn>(*I.pb, zr, xk, uk, xf, qf);
    if (k == 0) {  // x0 is a parameter of interval 0: drop the x directions of its jets
      auto drop_x = [&](Jet<NZ>& j) {
        for (int a = 0; a < NX; ++a) j.g[a] = 0.0;
        for (int a = 0; a < NX; ++a)
          for (int b = a; b < NZ; ++b) j.h[hix<NZ>(a, b)] = 0.0;
      };
      for (int r = 0; r < NX; ++r) drop_x(xf[r]);
      drop_x(qf);
    }
    e.f += I.fscale * qf.v;
    e.qsum += qf.v;
    for (int i = 0; i < NX; ++i) e.c[NX * (k + 1) + i] = xf[i].v - xn[i];
    for (int i = 0; i < NX; ++i) e.grad[I.ix(k, i)] += I.fscale * qf.g[i];
    for (int i = 0; i < NU; ++i) e.grad[I.iu(k, i)] += I.fscale * qf.g[NX + i];
    for (int r = 0; r < NX; ++r) {
      for (int j = 0; j < NX; ++j) e.A[NX * NX * k + NX * r + j] = xf[r].g[j];
      for (int j = 0; j < NU; ++j) e.Bm[NX * NU * k + NU * r + j] = xf[r].g[NX + j];
    }
    const double* l1 = &lam[NX * (k + 1)];
    for (int t = 0; t < NH; ++t) {
      double h = I.fscale * qf.h[t];
      for (int r = 0; r < NX; ++r) h = h + l1[r] * xf[r].h[t];
      e.H[NH * k + t] = h;
    }
  }
}

// Restoration-phase data of the Newton system: per constraint row r, D_r = 1/(Sigma_p + delta)
// + 1/(Sigma_n + delta) (the p, n columns eliminated) and the modified residual ct_r.  The
// system then reads  J dw + ct - D lam+ = 0  (lam+ the new multipliers).
struct RestoRows {
  const std::vector<double>* D = nullptr;
  const std::vector<double>* ct = nullptr;
};

// Cholesky of a small SPD matrix (row-major n x n); false if not positive definite
template <int n>
bool chol(const double* S, double* L) {
  for (int i = 0; i < n * n; ++i) L[i] = 0.0;
  for (int j = 0; j < n; ++j) {
    double d = S[n * j + j];
    for (int k = 0; k < j; ++k) d -= L[n * j + k] * L[n * j + k];
    if (!(d > 0)) return false;
    L[n * j + j] = std::sqrt(d);
    for (int i = j + 1; i < n; ++i) {
      double s = S[n * i + j];
      for (int k = 0; k < j; ++k) s -= L[n * i + k] * L[n * j + k];
      L[n * i + j] = s / L[n * j + j];
    }
  }
  return true;
}
template <int n>
void chol_solve(const double* L, double* b) {
  for (int i = 0; i < n; ++i) {
    double s = b[i];
    for (int k = 0; k < i; ++k) s -= L[n * i + k] * b[k];
    b[i] = s / L[n * i + i];
  }
  for (int i = n - 1; i >= 0; --i) {
    double s = b[i];
    for (int k = i + 1; k < n; ++k) s -= L[n * k + i] * b[k];
    b[i] = s / L[n * i + i];
  }
}

// Restoration: the value function (P, p) of node j seen through row block j's elimination,
// with S = D^-1 + P (must be positive definite) in the forms that stay accurate when the
// barrier terms make P huge (no P - P S^-1 P cancellation):
//   Pt = D^-1 - D^-1 S^-1 D^-1,   pt = D^-1 S^-1 p,   and later dx_j = S^-1 (D^-1 y - p).
// L receives the Cholesky factor of S.
template <int NX>
bool resto_transform(const double* D, const double* P, const double* p, double* Pt, double* pt, double* L) {
  double S[NX * NX], Di[NX];
  for (int i = 0; i < NX; ++i) Di[i] = 1.0 / D[i];
  for (int i = 0; i < NX * NX; ++i) S[i] = P[i];
  for (int i = 0; i < NX; ++i) S[NX * i + i] += Di[i];
  if (!chol<NX>(S, L)) return false;
  double X[NX][NX + 1];  // S^-1 [D^-1 | p], column by column
  for (int c = 0; c <= NX; ++c) {
    double b[NX];
    for (int i = 0; i < NX; ++i) b[i] = c < NX ? (i == c ? Di[c] : 0.0) : p[i];
    chol_solve<NX>(L, b);
    for (int i = 0; i < NX; ++i) X[i][c] = b[i];
  }
  for (int i = 0; i < NX; ++i) {
    for (int j = 0; j < NX; ++j) Pt[NX * i + j] = (i == j ? Di[i] : 0.0) - Di[i] * X[i][j];
    pt[i] = Di[i] * X[i][NX];
  }
  for (int i = 0; i < NX; ++i)
    for (int j = i + 1; j < NX; ++j) {
      const double m = 0.5 * (Pt[NX * i + j] + Pt[NX * j + i]);
      Pt[NX * i + j] = Pt[NX * j + i] = m;
    }
  return true;
}

// Riccati factor/solve of the barrier KKT system.  Returns false on a non-PD reduced Hessian
// block (wrong inertia).  Outputs the primal step dw and the new multipliers lamNew.
template <class Dyn>
bool riccati(const Inst<Dyn>& I, const Eval<Dyn>& e, const std::vector<double>& sig, const std::vector<double>& gphi,
             const std::vector<double>* hdiag, double delta, const RestoRows& rr, std::vector<double>& dw,
             std::vector<double>& lamNew) {
  constexpr int NX = Dyn::NX, NU = Dyn::NU, NZ = NX + NU, NH = nh(NZ);
  const int N = I.N;
  const bool resto = rr.D != nullptr;
  const std::vector<double>& cc = resto ? *rr.ct : e.c;
  std::vector<double> Ks(N * NU * NX), kfs(N * NU), Ps((N + 1) * NX * NX), ps((N + 1) * NX);
  std::vector<double> Pts((N + 1) * NX * NX), pts((N + 1) * NX), Ls(resto ? (N + 1) * NX * NX : 0);
  double P[NX * NX], p[NX];
  auto hd = [&](int idx) { return sig[idx] + delta + (hdiag ? (*hdiag)[idx] : 0.0); };
  for (int i = 0; i < NX * NX; ++i) P[i] = 0;
  for (int i = 0; i < NX; ++i) {
    P[(NX + 1) * i] = hd(I.ix(N, i));
    p[i] = gphi[I.ix(N, i)];
  }
  auto store = [&](int k) -> bool {
    std::memcpy(&Ps[NX * NX * k], P, sizeof P);
    std::memcpy(&ps[NX * k], p, sizeof p);
    if (!resto) {
      std::memcpy(&Pts[NX * NX * k], P, sizeof P);
      std::memcpy(&pts[NX * k], p, sizeof p);
      return true;
    }
    const bool r_ = resto_transform<NX>(&(*rr.D)[NX * k], P, p, &Pts[NX * NX * k], &pts[NX * k], &Ls[NX * NX * k]);
    if (std::getenv("ORACLE_TRACE_NODES")) {
      double a = 0, b = 0, c = 0;
      for (int i = 0; i < NX * NX; ++i) {
        a = std::max(a, std::fabs(P[i]));
        b = std::max(b, std::fabs(Pts[NX * NX * k + i]));
      }
      for (int i = 0; i < NX; ++i) c = std::max(c, std::fabs(p[i]));
      printf("    P node %d |P| %.3e |Pt| %.3e |p| %.3e\n", k, a, b, c);
    }
    return r_;
  };
  if (!store(N)) return false;
  for (int k = N - 1; k >= 0; --k) {
    const double* A = &e.A[NX * NX * k];
    const double* B = &e.Bm[NX * NU * k];
    const double* c = &cc[NX * (k + 1)];
    const double* Pn = &Pts[NX * NX * (k + 1)];
    const double* pn_ = &pts[NX * (k + 1)];
    double H[NZ][NZ];
    for (int i = 0; i < NZ; ++i)
      for (int j = 0; j < NZ; ++j) H[i][j] = e.H[NH * k + hix<NZ>(i, j)];
    for (int i = 0; i < NX; ++i) H[i][i] += hd(I.ix(k, i));
    for (int i = 0; i < NU; ++i) H[NX + i][NX + i] += hd(I.iu(k, i));
    double PA[NX * NX], PB[NX * NU];
    for (int r = 0; r < NX; ++r) {
      for (int j = 0; j < NX; ++j) {
        double acc = Pn[NX * r] * A[j];
        for (int m = 1; m < NX; ++m) acc = acc + Pn[NX * r + m] * A[NX * m + j];
        PA[NX * r + j] = acc;
      }
      for (int j = 0; j < NU; ++j) {
        double acc = Pn[NX * r] * B[j];
        for (int m = 1; m < NX; ++m) acc = acc + Pn[NX * r + m] * B[NU * m + j];
        PB[NU * r + j] = acc;
      }
    }
    double Hxx[NX * NX], Hux[NU * NX], Huu[NU * NU];
    for (int i = 0; i < NX; ++i)
      for (int j = 0; j < NX; ++j) {
        double acc = H[i][j];
        for (int m = 0; m < NX; ++m) acc = acc + A[NX * m + i] * PA[NX * m + j];
        Hxx[NX * i + j] = acc;
      }
    for (int i = 0; i < NU; ++i)
      for (int j = 0; j < NX; ++j) {
        double acc = H[NX + i][j];
        for (int m = 0; m < NX; ++m) acc = acc + B[NU * m + i] * PA[NX * m + j];
        Hux[NX * i + j] = acc;
      }
    for (int i = 0; i < NU; ++i)
      for (int j = 0; j < NU; ++j) {
        double acc = H[NX + i][NX + j];
        for (int m = 0; m < NX; ++m) acc = acc + B[NU * m + i] * PB[NU * m + j];
        Huu[NU * i + j] = acc;
      }
    double s[NX];
    for (int i = 0; i < NX; ++i) {
      double acc = Pn[NX * i] * c[0];
      for (int m = 1; m < NX; ++m) acc = acc + Pn[NX * i + m] * c[m];
      s[i] = acc + pn_[i];
    }
    double gx[NX], gu[NU];
    for (int i = 0; i < NX; ++i) {
      double acc = gphi[I.ix(k, i)];
      for (int m = 0; m < NX; ++m) acc = acc + A[NX * m + i] * s[m];
      gx[i] = acc;
    }
    for (int i = 0; i < NU; ++i) {
      double acc = gphi[I.iu(k, i)];
      for (int m = 0; m < NX; ++m) acc = acc + B[NU * m + i] * s[m];
      gu[i] = acc;
    }
    double inv[NU * NU];
    if constexpr (NU == 2) {  // Cholesky test of Huu, explicit inverse
      const double a = Huu[0], b = 0.5 * (Huu[1] + Huu[2]), d = Huu[3];
      if (!(a > 0)) return false;
      const double l11 = std::sqrt(a), l21 = b / l11, r22 = d - l21 * l21;
      if (!(r22 > 0)) return false;
      const double det = a * d - b * b;
      inv[0] = d / det;
      inv[1] = -b / det;
      inv[2] = -b / det;
      inv[3] = a / det;
    } else {
      static_assert(NU == 1, "NU in {1, 2}");
      if (!(Huu[0] > 0)) return false;
      inv[0] = 1.0 / Huu[0];
    }
    double* K = &Ks[NU * NX * k];
    double* kf = &kfs[NU * k];
    for (int i = 0; i < NU; ++i) {
      for (int j = 0; j < NX; ++j) {
        double acc = inv[NU * i] * Hux[j];
        for (int m = 1; m < NU; ++m) acc = acc + inv[NU * i + m] * Hux[NX * m + j];
        K[NX * i + j] = -acc;
      }
      double acc = inv[NU * i] * gu[0];
      for (int m = 1; m < NU; ++m) acc = acc + inv[NU * i + m] * gu[m];
      kf[i] = -acc;
    }
    double Pk[NX * NX], pk[NX];
    for (int i = 0; i < NX; ++i) {
      for (int j = 0; j < NX; ++j) {
        double acc = Hxx[NX * i + j];
        for (int m = 0; m < NU; ++m) acc = acc + Hux[NX * m + i] * K[NX * m + j];
        Pk[NX * i + j] = acc;
      }
      double acc = gx[i];
      for (int m = 0; m < NU; ++m) acc = acc + Hux[NX * m + i] * kf[m];
      pk[i] = acc;
    }
    for (int i = 0; i < NX; ++i)
      for (int j = i + 1; j < NX; ++j) {
        const double m = 0.5 * (Pk[NX * i + j] + Pk[NX * j + i]);
        Pk[NX * i + j] = Pk[NX * j + i] = m;
      }
    std::memcpy(P, Pk, sizeof P);
    std::memcpy(p, pk, sizeof p);
    if (!store(k)) return false;
  }
  dw.assign(I.nw, 0.0);
  lamNew.assign(I.ng, 0.0);
  // node j's state step from its pre-elimination value y:  dx = S^-1 (D^-1 y - p)
  auto land = [&](int j, double* y) {
    if (!resto) return;
    const double* D = &(*rr.D)[NX * j];
    for (int i = 0; i < NX; ++i) y[i] = y[i] / D[i] - ps[NX * j + i];
    chol_solve<NX>(&Ls[NX * NX * j], y);
  };
  double dx[NX];
  for (int i = 0; i < NX; ++i) dx[i] = cc[i];  // x0 - X_0 (restoration: its modified residual)
  land(0, dx);
  for (int k = 0; k <= N; ++k) {
    const double* Pk = &Ps[NX * NX * k];
    const double* pk = &ps[NX * k];
    for (int i = 0; i < NX; ++i) {
      dw[I.ix(k, i)] = dx[i];
      double acc = Pk[NX * i] * dx[0];
      for (int m = 1; m < NX; ++m) acc = acc + Pk[NX * i + m] * dx[m];
      lamNew[NX * k + i] = acc + pk[i];
    }
    if (k == N) break;
    const double* K = &Ks[NU * NX * k];
    const double* kf = &kfs[NU * k];
    double du[NU];
    for (int i = 0; i < NU; ++i) {
      double acc = K[NX * i] * dx[0];
      for (int m = 1; m < NX; ++m) acc = acc + K[NX * i + m] * dx[m];
      du[i] = acc + kf[i];
    }
    for (int i = 0; i < NU; ++i) dw[I.iu(k, i)] = du[i];
    const double* A = &e.A[NX * NX * k];
    const double* B = &e.Bm[NX * NU * k];
    const double* c = &cc[NX * (k + 1)];
    double dn[NX];
    for (int i = 0; i < NX; ++i) {
      double acc = A[NX * i] * dx[0];
      for (int m = 1; m < NX; ++m) acc = acc + A[NX * i + m] * dx[m];
      for (int m = 0; m < NU; ++m) acc = acc + B[NU * i + m] * du[m];
      dn[i] = acc + c[i];
    }
    land(k + 1, dn);
    std::memcpy(dx, dn, sizeof dx);
  }
  return true;
}

double norm1(const std::vector<double>& v) {
  double s = 0;
  for (double a : v) s += std::fabs(a);
  return s;
}
double amax(const std::vector<double>& v) {
  double s = 0;
  for (double a : v) s = std::max(s, std::fabs(a));
  return s;
}

// Warm-start options (IPOPT warm_start_init_point = yes): multipliers from a previous
// solve, smaller initial barrier and bound pushes.  warm == nullptr -> IPOPT defaults.
struct Warm {
  double mu_init, bound_push, mult_push;
  const double* lam0;   // ng
  const double* lamx0;  // nw, CasADi convention lam_x = zU - zL
};

// Solve one instance.  Returns an oracle Status.
template <class Dyn>
int solve_one(Inst<Dyn>& I, double* w, double* lam, const oracle_opts& op, int* iters_out, double* f_out,
              const Warm* warm = nullptr, double* lamx_out = nullptr) {
  constexpr int NX = Dyn::NX;
  const int nw = I.nw, ng = I.ng;
  const double tol = op.tol;
  const int max_iter = op.max_iter;
  const double push = warm ? warm->bound_push : kBoundPush, frac = warm ? warm->bound_push : kBoundFrac;
  // ---- initial point: bound push (IPOPT bound_push / bound_frac)
  for (int i = 0; i < nw; ++i) {
    if (I.hasL[i] && I.hasU[i]) {
      double pl = std::min(push * std::max(1.0, std::fabs(I.lb[i])), frac * (I.ub[i] - I.lb[i]));
      double pu = std::min(push * std::max(1.0, std::fabs(I.ub[i])), frac * (I.ub[i] - I.lb[i]));
      w[i] = std::min(std::max(w[i], I.lb[i] + pl), I.ub[i] - pu);
    } else if (I.hasL[i]) {
      w[i] = std::max(w[i], I.lb[i] + push * std::max(1.0, std::fabs(I.lb[i])));
    } else if (I.hasU[i]) {
      w[i] = std::min(w[i], I.ub[i] - push * std::max(1.0, std::fabs(I.ub[i])));
    }
  }
  std::vector<double> zL(nw, 0.0), zU(nw, 0.0);
  int nbound = 0;
  for (int i = 0; i < nw; ++i) {
    const double lx = (warm && warm->lamx0) ? warm->lamx0[i] : 0.0;
    if (I.hasL[i]) {
      zL[i] = warm ? std::max(-lx, warm->mult_push) : 1.0;
      ++nbound;
    }
    if (I.hasU[i]) {
      zU[i] = warm ? std::max(lx, warm->mult_push) : 1.0;
      ++nbound;
    }
  }
  for (int i = 0; i < ng; ++i) lam[i] = (warm && warm->lam0) ? warm->lam0[i] : 0.0;
  // ---- gradient-based objective scaling (IPOPT nlp_scaling_max_gradient = 100)
  Eval<Dyn> e;
  I.fscale = 1.0;
  evaluate(I, w, lam, true, e);
  {
    double gmax = 0;
    for (double g : e.grad) gmax = std::max(gmax, std::fabs(g));
    if (gmax > 100.0) {
      I.fscale = 100.0 / gmax;
      // multipliers given for the unscaled problem scale with the objective
      for (int i = 0; i < ng; ++i) lam[i] *= I.fscale;
      for (int i = 0; i < nw; ++i) {
        if (warm && I.hasL[i]) zL[i] = std::max(zL[i] * I.fscale, warm->mult_push);
        if (warm && I.hasU[i]) zU[i] = std::max(zU[i] * I.fscale, warm->mult_push);
      }
      evaluate(I, w, lam, true, e);
    }
  }
  const double fs = I.fscale;
  double mu = warm ? warm->mu_init : 0.1, tau = std::max(kTauMin, 1.0 - mu);
  const double mu_min = tol / 10;
  std::vector<std::pair<double, double>> filter;
  int frej = 0, nfreset = 0;  // IPOPT filter_reset_trigger / max_filter_resets (5, 5)
  double theta_max = 1e4 * std::max(1.0, norm1(e.c)), theta_min = 1e-4 * std::max(1.0, norm1(e.c));
  double dw_last = 0.0;
  bool tiny_flag = false;
  int status = kMaxIter, it = 0;
  // termination bookkeeping: acceptable iterates in a row, objective of the last iterate
  int acc_count = 0;
  double f_last = -1e50;
  // soft restoration phase
  bool soft = false;
  int soft_count = 0;

  // ---- restoration phase state (W&B 2006 §3.3); the original problem's values are kept
  bool resto = false;
  int resto_steps = 0;
  double mu_o = 0, tau_o = 0, th_R0 = 0, ph_R0 = 0, theta_max_o = 0, theta_min_o = 0, dw_last_o = 0;
  std::vector<std::pair<double, double>> filter_o;
  std::vector<double> wR, DR2, zL_R, zU_R, pp(ng), nn(ng), zp(ng), zn(ng);
  std::vector<double> Drow(ng), ct(ng), dp(ng), dn(ng), dzp(ng), dzn(ng), hprox(nw, 0.0);
  const std::vector<double> zero_ng(ng, 0.0), zero_nw(nw, 0.0);
  auto eta_of = [](double m) { return std::sqrt(m); };

  std::vector<double> sig(nw), gphi(nw), dw, lamNew, wt(nw), dzL(nw), dzU(nw), lt(ng), zLt(nw), zUt(nw);
  std::vector<double> ppt(ng), nnt(ng), zpt(ng), znt(ng);
  Eval<Dyn> et;
  // orig-problem barrier objective and restoration objective
  auto barrier_sum = [&](const double* x) {
    double s = 0;
    for (int i = 0; i < nw; ++i) {
      if (I.hasL[i]) s += std::log(x[i] - I.lb[i]);
      if (I.hasU[i]) s += std::log(I.ub[i] - x[i]);
    }
    return s;
  };
  auto resto_obj = [&](const double* x, const double* p_, const double* n_, double m) {
    double f = 0;
    for (int r = 0; r < ng; ++r) f += kRho * (p_[r] + n_[r]);
    double pr = 0;
    for (int i = 0; i < nw; ++i) pr += DR2[i] * sqr(x[i] - wR[i]);
    f += 0.5 * eta_of(m) * pr;
    double b = barrier_sum(x);
    for (int r = 0; r < ng; ++r) b += std::log(p_[r]) + std::log(n_[r]);
    return f - m * b;
  };
  auto theta_of = [&](const std::vector<double>& c, const double* p_, const double* n_) {
    double s = 0;
    for (int r = 0; r < ng; ++r) s += std::fabs(c[r] - (p_ ? p_[r] - n_[r] : 0.0));
    return s;
  };
  // dual infeasibility vector of the current problem (w part): grad f + J^T lam - zL + zU
  auto dual_res = [&](const Eval<Dyn>& ev, const double* l, const double* zl, const double* zu, std::vector<double>& r) {
    r = ev.grad;
    for (int i = 0; i < NX; ++i) r[I.ix(0, i)] -= l[i];
    for (int k = 0; k < I.N; ++k) {
      const double* A = &ev.A[NX * NX * k];
      const double* B = &ev.Bm[NX * Dyn::NU * k];
      const double* l1 = &l[NX * (k + 1)];
      for (int j = 0; j < NX; ++j) {
        double acc = 0;
        for (int m = 0; m < NX; ++m) acc += A[NX * m + j] * l1[m];
        r[I.ix(k, j)] += acc;
      }
      for (int j = 0; j < Dyn::NU; ++j) {
        double acc = 0;
        for (int m = 0; m < NX; ++m) acc += B[Dyn::NU * m + j] * l1[m];
        r[I.iu(k, j)] += acc;
      }
      for (int j = 0; j < NX; ++j) r[I.ix(k + 1, j)] -= l1[j];
    }
    for (int i = 0; i < nw; ++i) r[i] += -zl[i] + zu[i];
  };
  // restoration: the objective gradient is the proximity term's alone (f is replaced), and
  // its Hessian diagonal; both follow the barrier parameter (zeta = sqrt(mu))
  auto set_prox = [&](Eval<Dyn>& ev, const double* x, double m) {
    const double eta = eta_of(m);
    for (int i = 0; i < nw; ++i) {
      ev.grad[i] = eta * DR2[i] * (x[i] - wR[i]);
      hprox[i] = eta * DR2[i];
    }
  };
  std::vector<double> rd;

  for (it = 0; it <= max_iter; ++it) {
    // ---- optimality error of the current problem
    auto err = [&](double m, double& Ed, double& Ec, double& Ecomp) {
      dual_res(e, lam, zL.data(), zU.data(), rd);
      Ed = amax(rd);
      Ecomp = 0;
      for (int i = 0; i < nw; ++i) {
        if (I.hasL[i]) Ecomp = std::max(Ecomp, std::fabs((w[i] - I.lb[i]) * zL[i] - m));
        if (I.hasU[i]) Ecomp = std::max(Ecomp, std::fabs((I.ub[i] - w[i]) * zU[i] - m));
      }
      Ec = 0;
      if (!resto) {
        Ec = amax(e.c);
      } else {
        for (int r = 0; r < ng; ++r) {
          Ec = std::max(Ec, std::fabs(e.c[r] - pp[r] + nn[r]));
          Ed = std::max(Ed, std::max(std::fabs(kRho - lam[r] - zp[r]), std::fabs(kRho + lam[r] - zn[r])));
          Ecomp = std::max(Ecomp, std::max(std::fabs(pp[r] * zp[r] - m), std::fabs(nn[r] * zn[r] - m)));
        }
      }
    };
    double zsum = norm1(zL) + norm1(zU), lsum = 0;
    for (int i = 0; i < ng; ++i) lsum += std::fabs(lam[i]);
    int nb = nbound, nvar = nw;
    if (resto) {
      zsum += norm1(zp) + norm1(zn);
      nb += 2 * ng;
      nvar += 2 * ng;
    }
    const double sd = std::max(kSmax, (lsum + zsum) / (ng + nvar)) / kSmax;
    const double sc = std::max(kSmax, nb ? zsum / nb : 0.0) / kSmax;
    double Ed, Ec, Ecomp;
    err(0.0, Ed, Ec, Ecomp);
    const double E0 = std::max(std::max(Ed / sd, Ec), Ecomp / sc);
    const double fcur = e.f;
    if (!resto) {
      // IPOPT OptimalityErrorConvergenceCheck: tol and the unscaled tests; acceptable level
      if (E0 <= tol && Ed / fs <= op.dual_inf_tol && Ec <= op.constr_viol_tol && Ecomp / fs <= op.compl_inf_tol) {
        status = kConverged;
        break;
      }
    }
    const bool acceptable_now = !resto && E0 <= op.acceptable_tol && Ed / fs <= op.acceptable_dual_inf_tol &&
                                Ec <= op.acceptable_constr_viol_tol && Ecomp / fs <= op.acceptable_compl_inf_tol &&
                                std::fabs(fcur - f_last) / std::max(1.0, std::fabs(fcur)) <= op.acceptable_obj_change_tol;
    if (!resto) {
      f_last = fcur;
      if (op.acceptable_iter > 0 && acceptable_now) {
        if (++acc_count >= op.acceptable_iter) {
          status = kAcceptable;
          break;
        }
      } else {
        acc_count = 0;
      }
    } else {
      // restoration: progress for the original problem (RestoConvergenceCheck) -- at least
      // one restoration step; kappa_resto, the original filter and sufficient decrease
      // against the point where the restoration phase started
      if (resto_steps > 0) {
        const double th_o = norm1(e.c);
        const double ph_o = fs * e.qsum - mu_o * barrier_sum(w);
        bool ok = th_o <= kKappaResto * th_R0;
        if (ok)
          for (auto& fe : filter_o)
            if (th_o >= fe.first && ph_o >= fe.second) {
              ok = false;
              break;
            }
        if (ok) ok = th_o <= (1.0 - kGammaTheta) * th_R0 || ph_o <= ph_R0 - kGammaPhi * th_R0;
        TRACE("it=%d resto step %d th_o=%.3e (need <= %.3e) ph_o=%.6e ok=%d E0=%.3e mu=%.2e\n", it, resto_steps, th_o,
              kKappaResto * th_R0, ph_o, (int)ok, E0, mu);
        if (ok) {
          // back to the original problem: constraint multipliers restart at 0, bound
          // multipliers from a complementarity Newton step over the whole restoration
          // step (reset to 1 above bound_mult_reset_threshold)
          resto = false;
          mu = mu_o;
          tau = tau_o;
          theta_max = theta_max_o;
          theta_min = theta_min_o;
          dw_last = dw_last_o;
          filter = filter_o;
          double zmax = 0;
          for (int i = 0; i < nw; ++i) {
            auto upd = [&](double z0, double s0, double s1) {
              const double dz = mu / s0 - z0 - z0 / s0 * (s1 - s0);
              double a = 1.0;
              if (dz < 0) a = std::min(1.0, -tau * z0 / dz);
              return z0 + a * dz;
            };
            if (I.hasL[i]) zL[i] = upd(zL_R[i], wR[i] - I.lb[i], w[i] - I.lb[i]);
            else zL[i] = 0.0;
            if (I.hasU[i]) zU[i] = upd(zU_R[i], I.ub[i] - wR[i], I.ub[i] - w[i]);
            else zU[i] = 0.0;
            zmax = std::max(zmax, std::max(zL[i], zU[i]));
          }
          if (zmax > kBoundMultReset)
            for (int i = 0; i < nw; ++i) {
              zL[i] = I.hasL[i] ? 1.0 : 0.0;
              zU[i] = I.hasU[i] ? 1.0 : 0.0;
            }
          for (int i = 0; i < ng; ++i) lam[i] = 0.0;
          soft = false;
          soft_count = 0;
          acc_count = 0;
          tiny_flag = false;
          I.fscale = fs;
          evaluate(I, w, lam, true, e);
          --it;  // leaving the restoration phase takes no iteration
          continue;
        }
      }
      if (E0 <= tol) {  // the restoration problem converged: a point of local infeasibility
        status = kInfeasible;
        break;
      }
    }
    if (it == max_iter) break;
    // ---- barrier parameter update (monotone, fast decrease: repeated while the barrier test
    //      holds; a tiny step forces one decrease)
    {
      bool first_dec = true;
      for (;;) {
        double Edm, Ecm, Ecpm;
        err(mu, Edm, Ecm, Ecpm);
        const double Emu = std::max(std::max(Edm / sd, Ecm), Ecpm / sc);
        if (!((Emu <= kKappaEps * mu || (tiny_flag && first_dec)) && mu > mu_min)) break;
        first_dec = false;
        mu = std::max(mu_min, std::min(kKappaMu * mu, std::pow(mu, kThetaMu)));
        tau = std::max(kTauMin, 1.0 - mu);
        filter.clear();
#ifdef ORACLE_LEGACY_MU
        if (it > 0) break;
#endif
      }
      tiny_flag = false;
      // restoration: the proximity weight follows the barrier parameter from here on (the
      // barrier test above used the one of the iteration's start)
      if (resto) set_prox(e, w, mu);
    }
    // ---- barrier gradient and primal-dual Sigma (restoration: also the p, n columns)
    for (int i = 0; i < nw; ++i) {
      sig[i] = 0;
      gphi[i] = e.grad[i];
      if (I.hasL[i]) {
        const double s = w[i] - I.lb[i];
        sig[i] += zL[i] / s;
        gphi[i] -= mu / s;
      }
      if (I.hasU[i]) {
        const double s = I.ub[i] - w[i];
        sig[i] += zU[i] / s;
        gphi[i] += mu / s;
      }
    }
    // ---- search direction with inertia correction
    auto newton = [&](double delta) {
      RestoRows rr;
      if (resto) {
        for (int r = 0; r < ng; ++r) {
          const double sp = zp[r] / pp[r] + delta, sn = zn[r] / nn[r] + delta;
          Drow[r] = 1.0 / sp + 1.0 / sn;
          ct[r] = e.c[r] - pp[r] + nn[r] + (kRho - mu / pp[r]) / sp - (kRho - mu / nn[r]) / sn;
        }
        rr.D = &Drow;
        rr.ct = &ct;
      }
      const bool ok_ = riccati(I, e, sig, gphi, resto ? &hprox : nullptr, delta, rr, dw, lamNew);
      if (ok_ && tracing()) {  // residuals of the Newton system (diagnostics)
        const std::vector<double>& CT = resto ? ct : e.c;
        const std::vector<double>& DD = resto ? Drow : zero_ng;
        constexpr int NU = Dyn::NU, NZ = NX + NU, NH = nh(NZ);
        std::vector<double> r1(nw, 0.0), r2(ng, 0.0);
        for (int i = 0; i < nw; ++i) r1[i] = (sig[i] + delta + (resto ? hprox[i] : 0.0)) * dw[i] + gphi[i];
        for (int k = 0; k < I.N; ++k) {
          double z[NZ];
          for (int i = 0; i < NX; ++i) z[i] = dw[I.ix(k, i)];
          for (int i = 0; i < NU; ++i) z[NX + i] = dw[I.iu(k, i)];
          for (int i = 0; i < NZ; ++i) {
            double acc = 0;
            for (int j = 0; j < NZ; ++j) acc += e.H[NH * k + hix<NZ>(i, j)] * z[j];
            r1[i < NX ? I.ix(k, i) : I.iu(k, i - NX)] += acc;
          }
        }
        dual_res(e, lamNew.data(), zero_nw.data(), zero_nw.data(), rd);  // grad f + J^T lam+
        for (int i = 0; i < nw; ++i) r1[i] += rd[i] - e.grad[i];
        for (int i = 0; i < NX; ++i) r2[i] = -dw[I.ix(0, i)] + CT[i] - DD[i] * lamNew[i];
        for (int k = 0; k < I.N; ++k)
          for (int r = 0; r < NX; ++r) {
            double acc = -dw[I.ix(k + 1, r)] + CT[NX * (k + 1) + r] - DD[NX * (k + 1) + r] * lamNew[NX * (k + 1) + r];
            for (int m = 0; m < NX; ++m) acc += e.A[NX * NX * k + NX * r + m] * dw[I.ix(k, m)];
            for (int m = 0; m < NU; ++m) acc += e.Bm[NX * NU * k + NU * r + m] * dw[I.iu(k, m)];
            r2[NX * (k + 1) + r] = acc;
          }
        if (std::getenv("ORACLE_TRACE_NODES"))
          for (int k = 0; k <= I.N; ++k) {
            double a1 = 0, a2 = 0;
            for (int i = 0; i < NX; ++i) {
              a1 = std::max(a1, std::fabs(r1[I.ix(k, i)]));
              a2 = std::max(a2, std::fabs(r2[NX * k + i]));
            }
            if (k < I.N)
              for (int i = 0; i < NU; ++i) a1 = std::max(a1, std::fabs(r1[I.iu(k, i)]));
            TRACE("    node %d r_stat %.3e r_con %.3e D %.3e lam %.3e\n", k, a1, a2, DD[NX * k], lamNew[NX * k]);
          }
        TRACE("  newton check delta=%.2e |r_stat|=%.3e |r_con|=%.3e |dw|=%.3e |lam+|=%.3e\n", delta, amax(r1), amax(r2),
              amax(dw), amax(lamNew));
      }
      return ok_;
    };
    double delta = 0.0;
    bool ok = newton(0.0);
    if (!ok) {
      delta = dw_last == 0.0 ? kDw0 : std::max(kDwMin, kKwMinus * dw_last);
      for (;;) {
        ok = newton(delta);
        if (ok) break;
        delta *= dw_last == 0.0 ? kKwPlusBar : kKwPlus;
        if (delta > kDwMax) break;
      }
      if (!ok) {
        TRACE("it=%d resto=%d inertia correction failed\n", it, (int)resto);
        status = kStepFailed;
        break;
      }
      dw_last = delta;
    }
    for (int i = 0; i < nw; ++i) {
      dzL[i] = dzU[i] = 0;
      if (I.hasL[i]) {
        const double s = w[i] - I.lb[i];
        dzL[i] = mu / s - zL[i] - zL[i] / s * dw[i];
      }
      if (I.hasU[i]) {
        const double s = I.ub[i] - w[i];
        dzU[i] = mu / s - zU[i] + zU[i] / s * dw[i];
      }
    }
    if (resto)
      for (int r = 0; r < ng; ++r) {
        const double sp = zp[r] / pp[r] + delta, sn = zn[r] / nn[r] + delta;
        dp[r] = (lamNew[r] - kRho + mu / pp[r]) / sp;
        dn[r] = (-lamNew[r] - kRho + mu / nn[r]) / sn;
        dzp[r] = mu / pp[r] - zp[r] - zp[r] / pp[r] * dp[r];
        dzn[r] = mu / nn[r] - zn[r] - zn[r] / nn[r] * dn[r];
      }
    // ---- fraction to the boundary
    double amaxp = 1.0, az = 1.0;
    for (int i = 0; i < nw; ++i) {
      if (I.hasL[i] && dw[i] < 0) amaxp = std::min(amaxp, -tau * (w[i] - I.lb[i]) / dw[i]);
      if (I.hasU[i] && dw[i] > 0) amaxp = std::min(amaxp, tau * (I.ub[i] - w[i]) / dw[i]);
      if (I.hasL[i] && dzL[i] < 0) az = std::min(az, -tau * zL[i] / dzL[i]);
      if (I.hasU[i] && dzU[i] < 0) az = std::min(az, -tau * zU[i] / dzU[i]);
    }
    if (resto)
      for (int r = 0; r < ng; ++r) {
        if (dp[r] < 0) amaxp = std::min(amaxp, -tau * pp[r] / dp[r]);
        if (dn[r] < 0) amaxp = std::min(amaxp, -tau * nn[r] / dn[r]);
        if (dzp[r] < 0) az = std::min(az, -tau * zp[r] / dzp[r]);
        if (dzn[r] < 0) az = std::min(az, -tau * zn[r] / dzn[r]);
      }
    // ---- filter line search
    const double thk = resto ? theta_of(e.c, pp.data(), nn.data()) : norm1(e.c);
    const double phk = resto ? resto_obj(w, pp.data(), nn.data(), mu) : e.f - mu * barrier_sum(w);
    double gd = 0;
    for (int i = 0; i < nw; ++i) gd += gphi[i] * dw[i];
    if (resto)
      for (int r = 0; r < ng; ++r) gd += (kRho - mu / pp[r]) * dp[r] + (kRho - mu / nn[r]) * dn[r];
    double tiny = 0;
    for (int i = 0; i < nw; ++i) tiny = std::max(tiny, std::fabs(dw[i]) / (1.0 + std::fabs(w[i])));
    if (resto)
      for (int r = 0; r < ng; ++r)
        tiny = std::max(tiny, std::max(std::fabs(dp[r]) / (1.0 + pp[r]), std::fabs(dn[r]) / (1.0 + nn[r])));
    double alpha = amaxp, alpha_d = az;
    bool accepted = false, ftype = false, lastrej_f = false, augment = true;
    const double sw_rhs = kDelta * std::pow(thk, kSTheta);
    // acceptance of a trial point (theta, phi) for primal step al: sufficient decrease
    // (switching condition + Armijo, or theta / phi decrease), then the filter
    auto acceptable = [&](double tht, double pht, double al, bool& ft) {
      bool acc = std::isfinite(pht) && tht <= theta_max;
      ft = false;
      if (acc) {
        const bool sw = gd < 0 && al * std::pow(-gd, kSPhi) > sw_rhs;
        if (thk <= theta_min && sw) {
          acc = pht - phk <= kEtaPhi * al * gd + 10 * kEps * std::fabs(phk);
          ft = acc;
        } else {
          acc = tht <= (1 - kGammaTheta) * thk || pht <= phk - kGammaPhi * thk + 10 * kEps * std::fabs(phk);
        }
      }
      bool infilter = false;
      for (auto& fe : filter)
        if (tht >= fe.first && pht >= fe.second) {
          infilter = true;
          break;
        }
      if (acc && infilter) {
        acc = false;
        lastrej_f = true;
      } else if (!acc) {
        lastrej_f = false;
      }
      return acc;
    };
    auto trial = [&](double al, double& tht, double& pht) {
      for (int i = 0; i < nw; ++i) wt[i] = w[i] + al * dw[i];
      evaluate(I, wt.data(), lam, false, et);
      if (!resto) {
        tht = norm1(et.c);
        pht = et.f - mu * barrier_sum(wt.data());
      } else {
        for (int r = 0; r < ng; ++r) {
          ppt[r] = pp[r] + al * dp[r];
          nnt[r] = nn[r] + al * dn[r];
        }
        tht = theta_of(et.c, ppt.data(), nnt.data());
        pht = resto_obj(wt.data(), ppt.data(), nnt.data(), mu);
      }
    };
    // primal-dual system error of the original barrier problem at (x, lam, z), IPOPT
    // curr/trial_primal_dual_system_error (1-norms; the common normalisation cancels)
    auto pd_error = [&](const Eval<Dyn>& ev, const double* x, const double* l, const double* zl, const double* zu) {
      dual_res(ev, l, zl, zu, rd);
      double s = norm1(rd) + norm1(ev.c);
      for (int i = 0; i < nw; ++i) {
        if (I.hasL[i]) s += std::fabs((x[i] - I.lb[i]) * zl[i] - mu);
        if (I.hasU[i]) s += std::fabs((I.ub[i] - x[i]) * zu[i] - mu);
      }
      return s;
    };
    // soft restoration step (IPOPT TrySoftRestoStep): primal and dual variables take the same
    // step min(alpha_max primal, alpha_max dual); accepted by the original acceptance test
    // (leaves the soft phase) or by a reduction of the primal-dual error
    auto soft_step = [&](bool& leaves) {
      leaves = false;
      const double as = std::min(amaxp, az);
      double tht, pht;
      trial(as, tht, pht);
      bool ft;
      if (acceptable(tht, pht, as, ft)) {
        leaves = true;
        ftype = ft;
        alpha = alpha_d = as;
        return true;
      }
      for (int i = 0; i < ng; ++i) lt[i] = lam[i] + as * (lamNew[i] - lam[i]);
      for (int i = 0; i < nw; ++i) {
        zLt[i] = zL[i] + as * dzL[i];
        zUt[i] = zU[i] + as * dzU[i];
      }
      Eval<Dyn> es;
      evaluate(I, wt.data(), lt.data(), true, es);
      const double pd_t = pd_error(es, wt.data(), lt.data(), zLt.data(), zUt.data());
      const double pd_c = pd_error(e, w, lam, zL.data(), zU.data());
      if (pd_t <= kSoftResto * pd_c) {
        alpha = alpha_d = as;
        augment = false;
        return true;
      }
      return false;
    };
    bool go_resto = false;
    if (tiny < 10 * kEps) {
      accepted = true;
      ftype = true;
#ifndef ORACLE_LEGACY_MU
      tiny_flag = true;
#endif
    } else if (soft) {
      if (++soft_count > kMaxSoftResto) {
        go_resto = true;
      } else {
        bool leaves;
        accepted = soft_step(leaves);
        if (accepted && leaves) {
          soft = false;
          soft_count = 0;
        }
        if (!accepted) go_resto = true;
      }
    } else {
      const double amin = gd < 0 ? kGammaAlpha * std::min(kGammaTheta, std::min(kGammaPhi * thk / (-gd),
                                                                                sw_rhs / std::pow(-gd, kSPhi)))
                                 : kGammaAlpha * kGammaTheta;
      bool first_trial = true;
      for (;;) {
        double tht, pht;
        trial(alpha, tht, pht);
        bool ft;
        if (acceptable(tht, pht, alpha, ft)) {
          accepted = true;
          ftype = ft;
          break;
        }
        if (first_trial && !resto && op.max_soc > 0 && tht >= thk) {
          // IPOPT's second-order correction (W&B 2006 A-5.7-A-5.9): the Newton system with the
          // same matrix for the constraint residual c_soc = alpha c(x_k) + c(x_trial), stepped to
          // the boundary and tested with the first trial's alpha; accumulated while the
          // infeasibility shrinks by kappa_soc = 0.99
          Eval<Dyn> es = e;
          for (int r = 0; r < ng; ++r) es.c[r] = alpha * e.c[r] + et.c[r];
          double th_old = thk;
          std::vector<double> dws, lamS, dzLs(nw), dzUs(nw);
          for (int ps = 0; ps < op.max_soc; ++ps) {
            if (!riccati(I, es, sig, gphi, nullptr, delta, RestoRows(), dws, lamS)) break;
            double as = 1.0, azs = 1.0;
            for (int i = 0; i < nw; ++i) {
              dzLs[i] = dzUs[i] = 0;
              if (I.hasL[i]) {
                const double sl = w[i] - I.lb[i];
                dzLs[i] = mu / sl - zL[i] - zL[i] / sl * dws[i];
                if (dws[i] < 0) as = std::min(as, -tau * sl / dws[i]);
                if (dzLs[i] < 0) azs = std::min(azs, -tau * zL[i] / dzLs[i]);
              }
              if (I.hasU[i]) {
                const double su = I.ub[i] - w[i];
                dzUs[i] = mu / su - zU[i] + zU[i] / su * dws[i];
                if (dws[i] > 0) as = std::min(as, tau * su / dws[i]);
                if (dzUs[i] < 0) azs = std::min(azs, -tau * zU[i] / dzUs[i]);
              }
            }
            for (int i = 0; i < nw; ++i) wt[i] = w[i] + as * dws[i];
            evaluate(I, wt.data(), lam, false, et);
            const double ths = norm1(et.c), phs = et.f - mu * barrier_sum(wt.data());
            bool fts;
            if (acceptable(ths, phs, alpha, fts)) {
              accepted = true;
              ftype = fts;
              dw = dws;
              lamNew = lamS;
              dzL = dzLs;
              dzU = dzUs;
              alpha = as;
              alpha_d = azs;
              break;
            }
            if (ps == op.max_soc - 1 || ths > 0.99 * th_old) break;
            for (int r = 0; r < ng; ++r) es.c[r] = as * es.c[r] + et.c[r];
            th_old = ths;
          }
          if (accepted) break;
        }
        first_trial = false;
        alpha *= 0.5;
        if (alpha < amin) break;
      }
      if (!accepted) {
        TRACE("it=%d resto=%d line search failed thk=%.3e phk=%.6e gd=%.3e mu=%.2e delta=%.2e E0=%.3e\n", it, (int)resto,
              thk, phk, gd, mu, delta, E0);
        if (!resto && !op.restoration) {
          status = acceptable_now ? kAcceptable : kRestoFailed;
          break;
        }
        if (resto) {
          status = kRestoFailed;
          break;
        }
        // soft restoration first
        soft = true;
        soft_count = 0;
        bool leaves;
        accepted = soft_step(leaves);
        if (accepted && leaves) soft = false;
        if (!accepted) go_resto = true;
        TRACE("it=%d soft restoration step accepted=%d leaves=%d\n", it, (int)accepted, (int)(accepted && leaves));
      }
    }
    if (go_resto) {
      if (acceptable_now) {  // "restoration phase called at an acceptable point"
        status = kAcceptable;
        break;
      }
      if (resto || !op.restoration) {
        status = kRestoFailed;
        break;
      }
      TRACE("it=%d enter restoration thk=%.3e phk=%.6e mu=%.2e\n", it, thk, phk, mu);
      // ---- enter the restoration phase at the current point
      filter.emplace_back((1 - kGammaTheta) * thk, phk - kGammaPhi * thk);
      filter_o = filter;
      mu_o = mu;
      tau_o = tau;
      theta_max_o = theta_max;
      theta_min_o = theta_min;
      dw_last_o = dw_last;
      th_R0 = thk;
      ph_R0 = phk;
      resto = true;
      resto_steps = 0;
      soft = false;
      soft_count = 0;
      wR.assign(w, w + nw);
      zL_R = zL;
      zU_R = zU;
      DR2.assign(nw, 1.0);
      for (int i = 0; i < nw; ++i) DR2[i] = sqr(std::min(1.0, 1.0 / std::fabs(wR[i])));
      mu = std::max(mu, amax(e.c));
      tau = std::max(kTauMin, 1.0 - mu);
      for (int r = 0; r < ng; ++r) {  // W&B 2006 (33)
        const double c = e.c[r], a = (mu - kRho * c) / (2 * kRho);
        nn[r] = a + std::sqrt(a * a + mu * c / (2 * kRho));
        pp[r] = c + nn[r];
        zp[r] = mu / pp[r];
        zn[r] = mu / nn[r];
        lam[r] = 0.0;
      }
      for (int i = 0; i < nw; ++i) {
        zL[i] = std::min(kRho, zL[i]);
        zU[i] = std::min(kRho, zU[i]);
      }
      filter.clear();
      dw_last = 0.0;
      tiny_flag = false;
      I.fscale = 0.0;  // the restoration objective replaces f
      evaluate(I, w, lam, true, e);
      set_prox(e, w, mu);
      theta_max = 1e4 * std::max(1.0, theta_of(e.c, pp.data(), nn.data()));
      theta_min = 1e-4 * std::max(1.0, theta_of(e.c, pp.data(), nn.data()));
      --it;  // entering the restoration phase takes no iteration
      continue;
    }
    if (!accepted) {
      status = kRestoFailed;
      break;
    }
    // (a soft-restoration step accepted by the primal-dual error leaves the filter and its
    //  reset heuristic untouched)
    if (augment && !ftype) filter.emplace_back((1 - kGammaTheta) * thk, phk - kGammaPhi * thk);
    if (augment) {
      if (lastrej_f) {  // filter reset heuristic
        if (++frej >= 5 && nfreset < 5) {
          filter.clear();
          ++nfreset;
          frej = 0;
        }
      } else {
        frej = 0;
      }
    }
    // ---- update
    TRACE("STEP it=%d resto=%d alpha=%.17g alpha_d=%.17g ftype=%d mu=%.17g delta=%.3g thk=%.17g phk=%.17g\n", it,
          (int)resto, alpha, alpha_d, (int)ftype, mu, delta, thk, phk);
    for (int i = 0; i < nw; ++i) w[i] += alpha * dw[i];
    for (int i = 0; i < ng; ++i) lam[i] += alpha * (lamNew[i] - lam[i]);
    for (int i = 0; i < nw; ++i) {
      if (I.hasL[i]) {
        const double s = w[i] - I.lb[i];
        zL[i] += alpha_d * dzL[i];
        zL[i] = std::max(std::min(zL[i], kKappaSigma * mu / s), mu / (kKappaSigma * s));
      }
      if (I.hasU[i]) {
        const double s = I.ub[i] - w[i];
        zU[i] += alpha_d * dzU[i];
        zU[i] = std::max(std::min(zU[i], kKappaSigma * mu / s), mu / (kKappaSigma * s));
      }
    }
    if (resto) {
      for (int r = 0; r < ng; ++r) {
        pp[r] += alpha * dp[r];
        nn[r] += alpha * dn[r];
        zp[r] += alpha_d * dzp[r];
        zp[r] = std::max(std::min(zp[r], kKappaSigma * mu / pp[r]), mu / (kKappaSigma * pp[r]));
        zn[r] += alpha_d * dzn[r];
        zn[r] = std::max(std::min(zn[r], kKappaSigma * mu / nn[r]), mu / (kKappaSigma * nn[r]));
      }
      ++resto_steps;
    }
    evaluate(I, w, lam, true, e);
    if (resto) set_prox(e, w, mu);
  }
  *iters_out = it;
  I.fscale = fs;
  if (resto) {  // ended inside the restoration phase: report the original problem's values
    evaluate(I, w, lam, false, e);
  }
  *f_out = e.f / fs;
  for (int i = 0; i < ng; ++i) lam[i] /= fs;
  if (lamx_out)
    for (int i = 0; i < nw; ++i) lamx_out[i] = (zU[i] - zL[i]) / fs;
  return status;
}

template <class Dyn>
void setup_instance(Inst<Dyn>& I, const oracle_problem* pb, const double* P, int p_layout, const double* lbw,
                    const double* ubw) {
  constexpr int NX = Dyn::NX, NZ = NX + Dyn::NU;
  const int N = pb->N;
  I.pb = pb;
  I.N = N;
  I.nw = NX + NZ * N;
  I.ng = NX * (N + 1);
  I.zr.assign(NZ * N, 0.0);
  for (int i = 0; i < NX; ++i) I.x0[i] = P[i];
  for (int k = 0; k < N; ++k) {
    if (p_layout == 1) {
      for (int i = 0; i < NZ; ++i) I.zr[NZ * k + i] = P[NX + NZ * k + i];
    } else {
      for (int i = 0; i < NX; ++i) I.zr[NZ * k + i] = P[NX + i];
    }
  }
  I.lb.assign(lbw, lbw + I.nw);
  I.ub.assign(ubw, ubw + I.nw);
  I.hasL.resize(I.nw);
  I.hasU.resize(I.nw);
  for (int i = 0; i < I.nw; ++i) {
    I.hasL[i] = I.lb[i] > -kInfBound;
    I.hasU[i] = I.ub[i] < kInfBound;
  }
}

oracle_opts default_opts(int max_iter, double tol) {
  oracle_opts o;
  o.tol = tol;
  o.dual_inf_tol = 1.0;
  o.constr_viol_tol = 1e-4;
  o.compl_inf_tol = 1e-4;
  o.acceptable_tol = 1e-6;
  o.acceptable_dual_inf_tol = 1e10;
  o.acceptable_constr_viol_tol = 1e-2;
  o.acceptable_compl_inf_tol = 1e-2;
  o.acceptable_obj_change_tol = 1e20;
  o.max_iter = max_iter;
  o.acceptable_iter = 15;
  o.restoration = 1;
  o.max_soc = 0;  // the product's unicycle kernel takes no second-order correction
  return o;
}

oracle_problem unicycle_problem(const oracle_spec* sp) {
  oracle_problem pb;
  std::memset(&pb, 0, sizeof pb);
  pb.model = 1;
  pb.N = sp->N;
  pb.M = sp->M;
  pb.cost = sp->cost;
  pb.T = sp->T;
  for (int i = 0; i < 3; ++i) pb.Q[i] = sp->Q[i];
  for (int i = 0; i < 2; ++i) pb.R[i] = sp->R[i];
  return pb;
}

template <class Dyn>
int solve_batch_t(const oracle_problem* pb, const oracle_opts* op, int B, const double* P, int p_stride,
                  int p_layout, const double* w0, const double* lbw, const double* ubw, const Warm* warm_all,
                  double* w_out, double* lam_g, double* lamx_out, double* f_out, int32_t* status, int32_t* iters,
                  int nthreads) {
  constexpr int NX = Dyn::NX, NZ = NX + Dyn::NU;
  const int N = pb->N, nw = NX + NZ * N, ng = NX * (N + 1);
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
  for (int b = 0; b < B; ++b) {
    Inst<Dyn> I;
    setup_instance(I, pb, P + (size_t)b * p_stride, p_layout, lbw, ubw);
    double* w = w_out + (size_t)b * nw;
    if (w0) {
      std::memcpy(w, w0 + (size_t)b * nw, sizeof(double) * nw);
    } else {  // cold start X_k = x0, U = 0
      std::memset(w, 0, sizeof(double) * nw);
      for (int k = 0; k <= N; ++k)
        for (int i = 0; i < NX; ++i) w[I.ix(k, i)] = P[(size_t)b * p_stride + i];
    }
    std::vector<double> lam(ng);
    Warm wm;
    const Warm* wp = nullptr;
    if (warm_all) {
      wm = *warm_all;
      wm.lam0 = warm_all->lam0 ? warm_all->lam0 + (size_t)b * ng : nullptr;
      wm.lamx0 = warm_all->lamx0 ? warm_all->lamx0 + (size_t)b * nw : nullptr;
      wp = &wm;
    }
    int it = 0;
    double f = 0;
    status[b] = solve_one(I, w, lam.data(), *op, &it, &f, wp, lamx_out ? lamx_out + (size_t)b * nw : nullptr);
    iters[b] = it;
    if (f_out) f_out[b] = f;
    if (lam_g) std::memcpy(lam_g + (size_t)b * ng, lam.data(), sizeof(double) * ng);
  }
  return 0;
}

}  // namespace

extern "C" {

// Batched solve of the unicycle NLP.  P: B x 6 ([x0; xref], Casadi scripts) -- or B x 3 (x0)
// when pstage (B x N x 5 per-stage references) is given.  w0: B x nw or NULL (cold: zeros).
int oracle_solve_batch(const oracle_spec* sp, int B, const double* P, int p_stride, const double* pstage,
                       const double* w0, const double* lbw, const double* ubw, double* w_out, double* lam_g,
                       double* f_out, int32_t* status, int32_t* iters, int nthreads) {
  const oracle_problem pb = unicycle_problem(sp);
  const oracle_opts op = default_opts(sp->max_iter, sp->tol);
  const int N = sp->N, nw = 3 + 5 * N;
  // parameters in the layout-1 form [x0; (xr_k, ur_k) x N] (stage refs copied per instance)
  std::vector<double> P1((size_t)B * (3 + 5 * N));
  for (int b = 0; b < B; ++b) {
    double* q = &P1[(size_t)b * (3 + 5 * N)];
    const double* p = P + (size_t)b * p_stride;
    for (int i = 0; i < 3; ++i) q[i] = p[i];
    for (int k = 0; k < N; ++k)
      for (int i = 0; i < 5; ++i)
        q[3 + 5 * k + i] = pstage ? pstage[((size_t)b * N + k) * 5 + i] : (i < 3 ? p[3 + i] : 0.0);
  }
  std::vector<double> w0z;
  if (!w0) w0z.assign((size_t)B * nw, 0.0);  // this entry's cold start: zeros
  return solve_batch_t<Unicycle>(&pb, &op, B, P1.data(), 3 + 5 * N, 1, w0 ? w0 : w0z.data(), lbw, ubw, nullptr,
                                 w_out, lam_g, nullptr, f_out, status, iters, nthreads);
}

// Warm-started batched unicycle solve: lam0 (B x ng) and lamx0 (B x nw) may be NULL; lamx_out
// (B x nw) receives the bound multipliers (CasADi convention) if not NULL.
int oracle_solve_batch_warm(const oracle_spec* sp, int B, const double* P, int p_stride, const double* w0,
                            const double* lbw, const double* ubw, double mu_init, double bound_push,
                            double mult_push, const double* lam0, const double* lamx0, double* w_out,
                            double* lam_g, double* lamx_out, double* f_out, int32_t* status, int32_t* iters,
                            int nthreads) {
  const oracle_problem pb = unicycle_problem(sp);
  const oracle_opts op = default_opts(sp->max_iter, sp->tol);
  const Warm wm{mu_init, bound_push, mult_push, lam0, lamx0};
  return solve_batch_t<Unicycle>(&pb, &op, B, P, p_stride, 0, w0, lbw, ubw, &wm, w_out, lam_g, lamx_out, f_out,
                                 status, iters, nthreads);
}

// Any model, any options.  w0 NULL = cold start (X_k = x0, U = 0, the product's cold start);
// warm (mu_init > 0): IPOPT warm_start_init_point with lam0 / lamx0 (either may be NULL).
int oracle_solve(const oracle_problem* pb, const oracle_opts* op, int B, const double* P, int p_stride,
                 const double* w0, const double* lbw, const double* ubw, double mu_init, double bound_push,
                 double mult_push, const double* lam0, const double* lamx0, double* w_out, double* lam_g,
                 double* lamx_out, double* f_out, int32_t* status, int32_t* iters, int nthreads) {
  const Warm wm{mu_init, bound_push, mult_push, lam0, lamx0};
  const Warm* wp = mu_init > 0 ? &wm : nullptr;
  const int L = pb->p_layout;
  switch (pb->model) {
    case 1:
      return solve_batch_t<Unicycle>(pb, op, B, P, p_stride, L, w0, lbw, ubw, wp, w_out, lam_g, lamx_out, f_out, status,
                                     iters, nthreads);
    case 3:
      return solve_batch_t<KinBicycle>(pb, op, B, P, p_stride, L, w0, lbw, ubw, wp, w_out, lam_g, lamx_out, f_out,
                                       status, iters, nthreads);
    case 4:
      return solve_batch_t<DynBicycle>(pb, op, B, P, p_stride, L, w0, lbw, ubw, wp, w_out, lam_g, lamx_out, f_out,
                                       status, iters, nthreads);
    case 5:
      return solve_batch_t<CartPole>(pb, op, B, P, p_stride, L, w0, lbw, ubw, wp, w_out, lam_g, lamx_out, f_out,
                                     status, iters, nthreads);
    default:
      return -1;
  }
}

// Interval map F and its derivatives for B intervals: x (B x 3), u (B x 2),
// xr (B x 3), ur (B x 2, may be NULL), lam (B x 3, may be NULL).
// Outputs: xf (B x 3), qf (B), jac (B x 4 x 5: rows xf0..2, qf), hess (B x 15:
// Hessian of qf + lam^T xf, packed upper triangle), any may be NULL.
int oracle_stage(const oracle_spec* sp, int B, const double* x, const double* u, const double* xr, const double* ur,
                 const double* lam, double* xf, double* qf, double* jac, double* hess) {
  const oracle_problem pb = unicycle_problem(sp);
  for (int b = 0; b < B; ++b) {
    double zr[5] = {xr[3 * b], xr[3 * b + 1], xr[3 * b + 2], ur ? ur[2 * b] : 0.0, ur ? ur[2 * b + 1] : 0.0};
    Jet<5> jx[3], jq;
    stage_jet<Unicycle>(pb, zr, x + 3 * b, u + 2 * b, jx, jq);
    for (int i = 0; i < 3; ++i)
      if (xf) xf[3 * b + i] = jx[i].v;
    if (qf) qf[b] = jq.v;
    if (jac) {
      for (int r = 0; r < 3; ++r)
        for (int j = 0; j < 5; ++j) jac[20 * b + 5 * r + j] = jx[r].g[j];
      for (int j = 0; j < 5; ++j) jac[20 * b + 15 + j] = jq.g[j];
    }
    if (hess) {
      for (int t = 0; t < 15; ++t) {
        double h = jq.h[t];
        if (lam) h += lam[3 * b] * jx[0].h[t] + lam[3 * b + 1] * jx[1].h[t] + lam[3 * b + 2] * jx[2].h[t];
        hess[15 * b + t] = h;
      }
    }
  }
  return 0;
}

}  // extern "C"
