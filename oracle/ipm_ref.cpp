// ipm_ref.cpp -- C++ CPU restatement of the multiple-shooting MPC NLP and of an
// IPOPT-style primal-dual interior-point solve of it.
//
// TEST INFRASTRUCTURE ONLY.  Built by oracle/Makefile into oracle/libipm_ref.so
// and loaded (ctypes) only by tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg -- as the checker and as the timed CPU baseline, never as
// the product.  Parity: pinned against tests/golden/unicycle_N10_golden.json
// (the reference's own CasADi+IPOPT outputs) and against oracle/nlp_ref.py in
// tests/test_oracle.py.
//
// What it restates (paths relative to /root/reference):
//   NLP     Casadi/multiple_shooting_casadi.py:68-114 (unicycle f, L, RK4 with
//           cost quadrature, M substeps), :116-178 (interleaved w, lifted X_0,
//           defect constraints g, J = sum qf, bounds on U), and the mpctools
//           tracking variant Trajectory Tracking/Trajectory_tracking.py:40-67
//           (node cost l(x,u,p_k), RK4 M=1, state bounds).
//   Solver  ca.nlpsol(..., 'ipopt', ...) at :181-197, i.e. IPOPT (third-party,
//           not vendored; version unpinned: the reference has no requirements
//           file).  Restated from its published algorithm (Waechter & Biegler,
//           Math. Prog. 106, 2006): monotone Fiacco-McCormick barrier update,
//           fraction-to-the-boundary rule, primal-dual bound multipliers,
//           inertia correction by Hessian regularisation, filter line search
//           with switching condition and Armijo rule, kappa_Sigma safeguard,
//           tiny-step acceptance, gradient-based objective scaling.
//           Exact Hessian of the Lagrangian (IPOPT default with CasADi).
//
// Implementation choices that are deliberately DIFFERENT from the HIP product
// (so this file checks it independently):
//   * derivatives by second-order forward-mode jets (value, gradient, Hessian)
//     pushed through the RK4 chain -- the product uses first-order tangents plus
//     a second-order adjoint;
//   * one instance at a time, plain arrays; OpenMP over instances.

#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>
#include <algorithm>
#ifdef _OPENMP
#include <omp.h>
#endif

namespace {

constexpr int NX = 3, NU = 2, NZ = 5, NH = 15;  // unicycle: z = (x, y, th, v, w)

inline int hix(int i, int j) {  // packed upper-triangular index, i <= j
  if (i > j) std::swap(i, j);
  return i * NZ - i * (i - 1) / 2 + (j - i);
}

// Second-order forward-mode jet over the 5 stage variables.
struct Jet {
  double v;
  double g[NZ];
  double h[NH];
};

inline Jet jconst(double c) {
  Jet r;
  r.v = c;
  std::memset(r.g, 0, sizeof r.g);
  std::memset(r.h, 0, sizeof r.h);
  return r;
}
inline Jet jvar(double c, int i) {
  Jet r = jconst(c);
  r.g[i] = 1.0;
  return r;
}
inline Jet operator+(const Jet& a, const Jet& b) {
  Jet r;
  r.v = a.v + b.v;
  for (int i = 0; i < NZ; ++i) r.g[i] = a.g[i] + b.g[i];
  for (int i = 0; i < NH; ++i) r.h[i] = a.h[i] + b.h[i];
  return r;
}
inline Jet operator-(const Jet& a, const Jet& b) {
  Jet r;
  r.v = a.v - b.v;
  for (int i = 0; i < NZ; ++i) r.g[i] = a.g[i] - b.g[i];
  for (int i = 0; i < NH; ++i) r.h[i] = a.h[i] - b.h[i];
  return r;
}
inline Jet operator*(double s, const Jet& a) {
  Jet r;
  r.v = s * a.v;
  for (int i = 0; i < NZ; ++i) r.g[i] = s * a.g[i];
  for (int i = 0; i < NH; ++i) r.h[i] = s * a.h[i];
  return r;
}
inline Jet operator*(const Jet& a, const Jet& b) {
  Jet r;
  r.v = a.v * b.v;
  for (int i = 0; i < NZ; ++i) r.g[i] = a.v * b.g[i] + b.v * a.g[i];
  for (int i = 0; i < NZ; ++i)
    for (int j = i; j < NZ; ++j) {
      int k = hix(i, j);
      r.h[k] = a.v * b.h[k] + b.v * a.h[k] + a.g[i] * b.g[j] + a.g[j] * b.g[i];
    }
  return r;
}
// scalar function with f, f', f'' at a.v
inline Jet jfun(const Jet& a, double f0, double f1, double f2) {
  Jet r;
  r.v = f0;
  for (int i = 0; i < NZ; ++i) r.g[i] = f1 * a.g[i];
  for (int i = 0; i < NZ; ++i)
    for (int j = i; j < NZ; ++j) {
      int k = hix(i, j);
      r.h[k] = f1 * a.h[k] + f2 * a.g[i] * a.g[j];
    }
  return r;
}
inline Jet jcos(const Jet& a) { double c = std::cos(a.v), s = std::sin(a.v); return jfun(a, c, -s, -c); }
inline Jet jsin(const Jet& a) { double c = std::cos(a.v), s = std::sin(a.v); return jfun(a, s, c, -s); }

}  // namespace

extern "C" {

// Mirrors the fields of mpcx_spec (include/mpcx.h) that the oracle needs.
typedef struct oracle_spec {
  int32_t N, M;
  int32_t cost;        // 0 = RK4 quadrature of L (CasADi scripts), 1 = node cost (mpctools)
  int32_t max_iter;
  double T;
  double Q[3], R[2];
  double tol;
} oracle_spec;

}

namespace {

// One interval on jets: xf (3 jets), qf (1 jet).  Casadi/multiple_shooting_casadi.py:98-114.
template <class S>
inline void rhs_t(const S x[NX], const S u[NU], S out[NX]);

template <>
inline void rhs_t<Jet>(const Jet x[NX], const Jet u[NU], Jet out[NX]) {
  out[0] = u[0] * jcos(x[2]);
  out[1] = u[0] * jsin(x[2]);
  out[2] = u[1];
}

inline Jet cost_L(const oracle_spec& sp, const Jet x[NX], const Jet u[NU], const double* xr, const double* ur) {
  Jet acc = jconst(0.0);
  for (int i = 0; i < NX; ++i) {
    Jet d = x[i] - jconst(xr[i]);
    acc = acc + sp.Q[i] * (d * d);
  }
  for (int i = 0; i < NU; ++i) {
    Jet d = u[i] - jconst(ur[i]);
    acc = acc + sp.R[i] * (d * d);
  }
  return acc;
}

void stage_jet(const oracle_spec& sp, const double* x0, const double* u0, const double* xr, const double* ur,
               Jet xf[NX], Jet& qf) {
  Jet X[NX], U[NU];
  for (int i = 0; i < NX; ++i) X[i] = jvar(x0[i], i);
  for (int i = 0; i < NU; ++i) U[i] = jvar(u0[i], NX + i);
  const double DT = sp.T / sp.M;
  Jet q = jconst(0.0);
  if (sp.cost == 1) q = cost_L(sp, X, U, xr, ur);
  for (int m = 0; m < sp.M; ++m) {
    Jet k1[NX], k2[NX], k3[NX], k4[NX], s[NX];
    rhs_t<Jet>(X, U, k1);
    for (int i = 0; i < NX; ++i) s[i] = X[i] + (DT / 2) * k1[i];
    Jet L2 = sp.cost == 0 ? cost_L(sp, s, U, xr, ur) : jconst(0);
    rhs_t<Jet>(s, U, k2);
    for (int i = 0; i < NX; ++i) s[i] = X[i] + (DT / 2) * k2[i];
    Jet L3 = sp.cost == 0 ? cost_L(sp, s, U, xr, ur) : jconst(0);
    rhs_t<Jet>(s, U, k3);
    for (int i = 0; i < NX; ++i) s[i] = X[i] + DT * k3[i];
    Jet L4 = sp.cost == 0 ? cost_L(sp, s, U, xr, ur) : jconst(0);
    rhs_t<Jet>(s, U, k4);
    if (sp.cost == 0) {
      Jet L1 = cost_L(sp, X, U, xr, ur);
      q = q + (DT / 6) * (L1 + 2.0 * L2 + 2.0 * L3 + L4);
    }
    for (int i = 0; i < NX; ++i) X[i] = X[i] + (DT / 6) * (k1[i] + 2.0 * k2[i] + 2.0 * k3[i] + k4[i]);
  }
  for (int i = 0; i < NX; ++i) xf[i] = X[i];
  qf = q;
}

// Plain double evaluation (line search): same arithmetic order as the jets' .v
void stage_val(const oracle_spec& sp, const double* x0, const double* u, const double* xr, const double* ur,
               double xf[NX], double& qf) {
  auto L = [&](const double* s) {
    double a = 0;
    for (int i = 0; i < NX; ++i) { double d = s[i] - xr[i]; a += sp.Q[i] * (d * d); }
    for (int i = 0; i < NU; ++i) { double d = u[i] - ur[i]; a += sp.R[i] * (d * d); }
    return a;
  };
  auto f = [&](const double* s, double* o) {
    o[0] = u[0] * std::cos(s[2]);
    o[1] = u[0] * std::sin(s[2]);
    o[2] = u[1];
  };
  double X[NX] = {x0[0], x0[1], x0[2]};
  const double DT = sp.T / sp.M;
  double q = sp.cost == 1 ? L(X) : 0.0;
  for (int m = 0; m < sp.M; ++m) {
    double k1[NX], k2[NX], k3[NX], k4[NX], s2[NX], s3[NX], s4[NX];
    f(X, k1);
    for (int i = 0; i < NX; ++i) s2[i] = X[i] + (DT / 2) * k1[i];
    f(s2, k2);
    for (int i = 0; i < NX; ++i) s3[i] = X[i] + (DT / 2) * k2[i];
    f(s3, k3);
    for (int i = 0; i < NX; ++i) s4[i] = X[i] + DT * k3[i];
    f(s4, k4);
    if (sp.cost == 0) q = q + (DT / 6) * (L(X) + 2.0 * L(s2) + 2.0 * L(s3) + L(s4));
    for (int i = 0; i < NX; ++i) X[i] = X[i] + (DT / 6) * (k1[i] + 2.0 * k2[i] + 2.0 * k3[i] + k4[i]);
  }
  for (int i = 0; i < NX; ++i) xf[i] = X[i];
  qf = q;
}

// ---------------------------------------------------------------------------
// Small dense helpers
// ---------------------------------------------------------------------------
inline double sqr(double a) { return a * a; }

// IPOPT constants (Waechter & Biegler 2006, Table 1 / IPOPT defaults)
constexpr double kEps = 2.220446049250313e-16;
constexpr double kKappaEps = 10.0, kKappaMu = 0.2, kThetaMu = 1.5, kTauMin = 0.99;
constexpr double kKappaSigma = 1e10, kSmax = 100.0;
constexpr double kGammaTheta = 1e-5, kGammaPhi = 1e-8, kDelta = 1.0, kSTheta = 1.1, kSPhi = 2.3;
constexpr double kEtaPhi = 1e-8, kGammaAlpha = 0.05;
constexpr double kDw0 = 1e-4, kDwMin = 1e-20, kDwMax = 1e40, kKwMinus = 1.0 / 3, kKwPlus = 8, kKwPlusBar = 100;
constexpr double kBoundPush = 1e-2, kBoundFrac = 1e-2, kInfBound = 1e19;

struct Instance {
  const oracle_spec* sp;
  int N, nw;
  std::vector<double> xr, ur;       // per-stage refs (N*3, N*2)
  double x0[NX];
  std::vector<double> lb, ub;       // per w component
  std::vector<char> hasL, hasU;
  double fscale = 1.0;
};

// w layout helpers (interleaved, Casadi/multiple_shooting_casadi.py:128-170)
inline int ix(int k, int i) { return k == 0 ? i : 3 + 5 * (k - 1) + 2 + i; }  // x_k[i]
inline int iu(int k, int i) { return 3 + 5 * k + i; }                          // u_k[i]

struct Eval {
  double f;
  std::vector<double> grad;  // nw
  std::vector<double> c;     // 3(N+1)
  std::vector<double> A, Bm; // N*9, N*6
  std::vector<double> H;     // N*15  Hessian of Lagrangian stage blocks (scaled f)
};

void evaluate(const Instance& I, const double* w, const double* lam, bool derivs, Eval& e) {
  const int N = I.N;
  e.f = 0;
  e.c.assign(3 * (N + 1), 0.0);
  if (derivs) {
    e.grad.assign(I.nw, 0.0);
    e.A.assign(N * 9, 0.0);
    e.Bm.assign(N * 6, 0.0);
    e.H.assign(N * NH, 0.0);
  }
  for (int i = 0; i < NX; ++i) e.c[i] = I.x0[i] - w[ix(0, i)];
  for (int k = 0; k < N; ++k) {
    double xk[NX], uk[NU], xn[NX];
    for (int i = 0; i < NX; ++i) { xk[i] = w[ix(k, i)]; xn[i] = w[ix(k + 1, i)]; }
    for (int i = 0; i < NU; ++i) uk[i] = w[iu(k, i)];
    const double* xr = &I.xr[3 * k];
    const double* ur = &I.ur[2 * k];
    if (!derivs) {
      double xf[NX], qf;
      stage_val(*I.sp, xk, uk, xr, ur, xf, qf);
      e.f += I.fscale * qf;
      for (int i = 0; i < NX; ++i) e.c[3 * (k + 1) + i] = xf[i] - xn[i];
      continue;
    }
    Jet xf[NX], qf;
    stage_jet(*I.sp, xk, uk, xr, ur, xf, qf);
    e.f += I.fscale * qf.v;
    for (int i = 0; i < NX; ++i) e.c[3 * (k + 1) + i] = xf[i].v - xn[i];
    for (int i = 0; i < NX; ++i) e.grad[ix(k, i)] += I.fscale * qf.g[i];
    for (int i = 0; i < NU; ++i) e.grad[iu(k, i)] += I.fscale * qf.g[NX + i];
    for (int r = 0; r < NX; ++r) {
      for (int j = 0; j < NX; ++j) e.A[9 * k + 3 * r + j] = xf[r].g[j];
      for (int j = 0; j < NU; ++j) e.Bm[6 * k + 2 * r + j] = xf[r].g[NX + j];
    }
    const double* l1 = &lam[3 * (k + 1)];
    for (int t = 0; t < NH; ++t)
      e.H[NH * k + t] = I.fscale * qf.h[t] + l1[0] * xf[0].h[t] + l1[1] * xf[1].h[t] + l1[2] * xf[2].h[t];
  }
}

// Riccati factor/solve of the barrier KKT system.  Returns false on a non-PD
// reduced Hessian block (wrong inertia).
bool riccati(const Instance& I, const Eval& e, const std::vector<double>& sig, const std::vector<double>& gphi,
             const double* w, double delta, std::vector<double>& dw, std::vector<double>& lamNew) {
  const int N = I.N;
  std::vector<double> Ks(N * 6), kfs(N * 2), Ps((N + 1) * 9), ps((N + 1) * 3);
  double P[9], p[3];
  for (int i = 0; i < 9; ++i) P[i] = 0;
  for (int i = 0; i < NX; ++i) { P[4 * i] = sig[ix(N, i)] + delta; p[i] = gphi[ix(N, i)]; }
  std::memcpy(&Ps[9 * N], P, sizeof P);
  std::memcpy(&ps[3 * N], p, sizeof p);
  for (int k = N - 1; k >= 0; --k) {
    const double* A = &e.A[9 * k];
    const double* B = &e.Bm[6 * k];
    const double* c = &e.c[3 * (k + 1)];
    double H[NZ][NZ];
    for (int i = 0; i < NZ; ++i)
      for (int j = 0; j < NZ; ++j) H[i][j] = e.H[NH * k + hix(i, j)];
    for (int i = 0; i < NX; ++i) H[i][i] += sig[ix(k, i)] + delta;
    for (int i = 0; i < NU; ++i) H[NX + i][NX + i] += sig[iu(k, i)] + delta;
    // PA = P*A, PB = P*B
    double PA[9], PB[6];
    for (int r = 0; r < 3; ++r) {
      for (int j = 0; j < 3; ++j) PA[3 * r + j] = P[3 * r] * A[j] + P[3 * r + 1] * A[3 + j] + P[3 * r + 2] * A[6 + j];
      for (int j = 0; j < 2; ++j) PB[2 * r + j] = P[3 * r] * B[j] + P[3 * r + 1] * B[2 + j] + P[3 * r + 2] * B[4 + j];
    }
    double Hxx[9], Hux[6], Huu[4];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j)
        Hxx[3 * i + j] = H[i][j] + A[i] * PA[j] + A[3 + i] * PA[3 + j] + A[6 + i] * PA[6 + j];
    for (int i = 0; i < 2; ++i)
      for (int j = 0; j < 3; ++j)
        Hux[3 * i + j] = H[NX + i][j] + B[i] * PA[j] + B[2 + i] * PA[3 + j] + B[4 + i] * PA[6 + j];
    for (int i = 0; i < 2; ++i)
      for (int j = 0; j < 2; ++j)
        Huu[2 * i + j] = H[NX + i][NX + j] + B[i] * PB[j] + B[2 + i] * PB[2 + j] + B[4 + i] * PB[4 + j];
    double s[3];
    for (int i = 0; i < 3; ++i) s[i] = P[3 * i] * c[0] + P[3 * i + 1] * c[1] + P[3 * i + 2] * c[2] + p[i];
    double gx[3], gu[2];
    for (int i = 0; i < 3; ++i) gx[i] = gphi[ix(k, i)] + A[i] * s[0] + A[3 + i] * s[1] + A[6 + i] * s[2];
    for (int i = 0; i < 2; ++i) gu[i] = gphi[iu(k, i)] + B[i] * s[0] + B[2 + i] * s[1] + B[4 + i] * s[2];
    // Cholesky of Huu (2x2)
    double a = Huu[0], b = 0.5 * (Huu[1] + Huu[2]), d = Huu[3];
    if (!(a > 0)) return false;
    double l11 = std::sqrt(a), l21 = b / l11, r22 = d - l21 * l21;
    if (!(r22 > 0)) return false;
    double det = a * d - b * b;
    double inv[4] = {d / det, -b / det, -b / det, a / det};
    double* K = &Ks[6 * k];
    double* kf = &kfs[2 * k];
    for (int i = 0; i < 2; ++i) {
      for (int j = 0; j < 3; ++j) K[3 * i + j] = -(inv[2 * i] * Hux[j] + inv[2 * i + 1] * Hux[3 + j]);
      kf[i] = -(inv[2 * i] * gu[0] + inv[2 * i + 1] * gu[1]);
    }
    double Pn[9], pn[3];
    for (int i = 0; i < 3; ++i) {
      for (int j = 0; j < 3; ++j) Pn[3 * i + j] = Hxx[3 * i + j] + Hux[i] * K[j] + Hux[3 + i] * K[3 + j];
      pn[i] = gx[i] + Hux[i] * kf[0] + Hux[3 + i] * kf[1];
    }
    for (int i = 0; i < 3; ++i)
      for (int j = i + 1; j < 3; ++j) { double m = 0.5 * (Pn[3 * i + j] + Pn[3 * j + i]); Pn[3 * i + j] = Pn[3 * j + i] = m; }
    std::memcpy(P, Pn, sizeof P);
    std::memcpy(p, pn, sizeof p);
    std::memcpy(&Ps[9 * k], P, sizeof P);
    std::memcpy(&ps[3 * k], p, sizeof p);
  }
  dw.assign(I.nw, 0.0);
  lamNew.assign(3 * (N + 1), 0.0);
  double dx[3];
  for (int i = 0; i < 3; ++i) dx[i] = e.c[i];  // x0 - X_0
  for (int k = 0; k <= N; ++k) {
    const double* Pk = &Ps[9 * k];
    const double* pk = &ps[3 * k];
    for (int i = 0; i < 3; ++i) {
      dw[ix(k, i)] = dx[i];
      lamNew[3 * k + i] = Pk[3 * i] * dx[0] + Pk[3 * i + 1] * dx[1] + Pk[3 * i + 2] * dx[2] + pk[i];
    }
    if (k == N) break;
    const double* K = &Ks[6 * k];
    const double* kf = &kfs[2 * k];
    double du[2];
    for (int i = 0; i < 2; ++i) du[i] = K[3 * i] * dx[0] + K[3 * i + 1] * dx[1] + K[3 * i + 2] * dx[2] + kf[i];
    for (int i = 0; i < 2; ++i) dw[iu(k, i)] = du[i];
    const double* A = &e.A[9 * k];
    const double* B = &e.Bm[6 * k];
    const double* c = &e.c[3 * (k + 1)];
    double dn[3];
    for (int i = 0; i < 3; ++i)
      dn[i] = A[3 * i] * dx[0] + A[3 * i + 1] * dx[1] + A[3 * i + 2] * dx[2] + B[2 * i] * du[0] + B[2 * i + 1] * du[1] + c[i];
    std::memcpy(dx, dn, sizeof dx);
  }
  return true;
}

double barrier_phi(const Instance& I, const double* w, double f, double mu) {
  double phi = f;
  for (int i = 0; i < I.nw; ++i) {
    if (I.hasL[i]) phi -= mu * std::log(w[i] - I.lb[i]);
    if (I.hasU[i]) phi -= mu * std::log(I.ub[i] - w[i]);
  }
  return phi;
}

double norm1(const std::vector<double>& v) {
  double s = 0;
  for (double a : v) s += std::fabs(a);
  return s;
}

// Solve one instance.  Returns status: 0 converged, 1 acceptable, 2 max_iter, 3 failure
// Warm-start options (IPOPT warm_start_init_point = yes): multipliers from a previous
// solve, smaller initial barrier and bound pushes.  warm == nullptr -> IPOPT defaults.
struct Warm {
  double mu_init, bound_push, mult_push;
  const double* lam0;   // ng
  const double* lamx0;  // nw, CasADi convention lam_x = zU - zL
};

int solve_one(Instance& I, double* w, double* lam, int max_iter, double tol, int* iters_out, double* f_out,
              const Warm* warm = nullptr, double* lamx_out = nullptr) {
  const int N = I.N, nw = I.nw, ng = 3 * (N + 1);
  const double push = warm ? warm->bound_push : kBoundPush;
  // ---- initial point: bound push (IPOPT bound_push / bound_frac)
  for (int i = 0; i < nw; ++i) {
    if (I.hasL[i] && I.hasU[i]) {
      double pl = std::min(push * std::max(1.0, std::fabs(I.lb[i])), push * (I.ub[i] - I.lb[i]));
      double pu = std::min(push * std::max(1.0, std::fabs(I.ub[i])), push * (I.ub[i] - I.lb[i]));
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
    if (I.hasL[i]) { zL[i] = warm ? std::max(-lx, warm->mult_push) : 1.0; ++nbound; }
    if (I.hasU[i]) { zU[i] = warm ? std::max(lx, warm->mult_push) : 1.0; ++nbound; }
  }
  for (int i = 0; i < ng; ++i) lam[i] = (warm && warm->lam0) ? warm->lam0[i] : 0.0;
  // ---- gradient-based objective scaling (IPOPT nlp_scaling_max_gradient = 100)
  Eval e;
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
  double mu = warm ? warm->mu_init : 0.1, tau = std::max(kTauMin, 1.0 - mu);
  const double mu_min = tol / 10;
  std::vector<std::pair<double, double>> filter;
  int frej = 0, nfreset = 0;  // IPOPT filter_reset_trigger / max_filter_resets (5, 5)
  double theta0 = norm1(e.c);
  const double theta_max = 1e4 * std::max(1.0, theta0), theta_min = 1e-4 * std::max(1.0, theta0);
  double dw_last = 0.0;
  int status = 2, it = 0;
  std::vector<double> sig(nw), gphi(nw), dw, lamNew, wt(nw), dzL(nw), dzU(nw);
  Eval et;
  for (it = 0; it <= max_iter; ++it) {
    // ---- optimality error (scaled problem)
    auto err = [&](double m, double& Ed, double& Ec, double& Ecomp) {
      // dual infeasibility: grad f + J^T lam - zL + zU
      std::vector<double> r(e.grad);
      for (int i = 0; i < NX; ++i) r[ix(0, i)] -= lam[i];
      for (int k = 0; k < N; ++k) {
        const double* A = &e.A[9 * k];
        const double* B = &e.Bm[6 * k];
        const double* l1 = &lam[3 * (k + 1)];
        for (int j = 0; j < 3; ++j) r[ix(k, j)] += A[j] * l1[0] + A[3 + j] * l1[1] + A[6 + j] * l1[2];
        for (int j = 0; j < 2; ++j) r[iu(k, j)] += B[j] * l1[0] + B[2 + j] * l1[1] + B[4 + j] * l1[2];
        for (int j = 0; j < 3; ++j) r[ix(k + 1, j)] -= l1[j];
      }
      Ed = 0; Ecomp = 0;
      for (int i = 0; i < nw; ++i) {
        r[i] += -zL[i] + zU[i];
        Ed = std::max(Ed, std::fabs(r[i]));
        if (I.hasL[i]) Ecomp = std::max(Ecomp, std::fabs((w[i] - I.lb[i]) * zL[i] - m));
        if (I.hasU[i]) Ecomp = std::max(Ecomp, std::fabs((I.ub[i] - w[i]) * zU[i] - m));
      }
      Ec = 0;
      for (double a : e.c) Ec = std::max(Ec, std::fabs(a));
    };
    double zn = norm1(zL) + norm1(zU);
    double ln = 0;
    for (int i = 0; i < ng; ++i) ln += std::fabs(lam[i]);
    const double sd = std::max(kSmax, (ln + zn) / (ng + nw)) / kSmax;
    const double sc = std::max(kSmax, nbound ? zn / nbound : 0.0) / kSmax;
    double Ed, Ec, Ecomp;
    err(0.0, Ed, Ec, Ecomp);
    double E0 = std::max(std::max(Ed / sd, Ec), Ecomp / sc);
    if (E0 <= tol) { status = 0; break; }
    if (it == max_iter) break;
    // ---- barrier parameter update (monotone; repeated only at the first iterate)
    for (;;) {
      double Edm, Ecm, Ecpm;
      err(mu, Edm, Ecm, Ecpm);
      double Emu = std::max(std::max(Edm / sd, Ecm), Ecpm / sc);
      if (Emu > kKappaEps * mu || mu <= mu_min) break;
      mu = std::max(mu_min, std::min(kKappaMu * mu, std::pow(mu, kThetaMu)));
      tau = std::max(kTauMin, 1.0 - mu);
      filter.clear();
      if (it > 0) break;
    }
    // ---- barrier gradient and primal-dual Sigma
    for (int i = 0; i < nw; ++i) {
      sig[i] = 0;
      gphi[i] = e.grad[i];
      if (I.hasL[i]) { double s = w[i] - I.lb[i]; sig[i] += zL[i] / s; gphi[i] -= mu / s; }
      if (I.hasU[i]) { double s = I.ub[i] - w[i]; sig[i] += zU[i] / s; gphi[i] += mu / s; }
    }
    // ---- search direction with inertia correction
    double delta = 0.0;
    bool ok = riccati(I, e, sig, gphi, w, 0.0, dw, lamNew);
    if (!ok) {
      delta = dw_last == 0.0 ? kDw0 : std::max(kDwMin, kKwMinus * dw_last);
      for (;;) {
        ok = riccati(I, e, sig, gphi, w, delta, dw, lamNew);
        if (ok) break;
        delta *= dw_last == 0.0 ? kKwPlusBar : kKwPlus;
        if (delta > kDwMax) break;
      }
      if (!ok) { status = 3; break; }
      dw_last = delta;
    }
    for (int i = 0; i < nw; ++i) {
      dzL[i] = dzU[i] = 0;
      if (I.hasL[i]) { double s = w[i] - I.lb[i]; dzL[i] = mu / s - zL[i] - zL[i] / s * dw[i]; }
      if (I.hasU[i]) { double s = I.ub[i] - w[i]; dzU[i] = mu / s - zU[i] + zU[i] / s * dw[i]; }
    }
    // ---- fraction to the boundary
    double amax = 1.0, az = 1.0;
    for (int i = 0; i < nw; ++i) {
      if (I.hasL[i] && dw[i] < 0) amax = std::min(amax, -tau * (w[i] - I.lb[i]) / dw[i]);
      if (I.hasU[i] && dw[i] > 0) amax = std::min(amax, tau * (I.ub[i] - w[i]) / dw[i]);
      if (I.hasL[i] && dzL[i] < 0) az = std::min(az, -tau * zL[i] / dzL[i]);
      if (I.hasU[i] && dzU[i] < 0) az = std::min(az, -tau * zU[i] / dzU[i]);
    }
    // ---- filter line search
    const double thk = norm1(e.c);
    const double phk = barrier_phi(I, w, e.f, mu);
    double gd = 0;
    for (int i = 0; i < nw; ++i) gd += gphi[i] * dw[i];
    double tiny = 0;
    for (int i = 0; i < nw; ++i) tiny = std::max(tiny, std::fabs(dw[i]) / (1.0 + std::fabs(w[i])));
    double alpha = amax;
    bool accepted = false, ftype = false, lastrej_f = false;
    if (tiny < 10 * kEps) {
      accepted = true;
      ftype = true;
    } else {
      double amin = gd < 0 ? kGammaAlpha * std::min(kGammaTheta, std::min(kGammaPhi * thk / (-gd),
                                                                           kDelta * std::pow(thk, kSTheta) / std::pow(-gd, kSPhi)))
                           : kGammaAlpha * kGammaTheta;
      for (;;) {
        for (int i = 0; i < nw; ++i) wt[i] = w[i] + alpha * dw[i];
        evaluate(I, wt.data(), lam, false, et);
        double tht = norm1(et.c), pht = barrier_phi(I, wt.data(), et.f, mu);
        bool acc = std::isfinite(pht) && tht <= theta_max;
        if (acc) {  // sufficient decrease first, then the filter (IPOPT's order)
          const bool sw = gd < 0 && alpha * std::pow(-gd, kSPhi) > kDelta * std::pow(thk, kSTheta);
          if (thk <= theta_min && sw) {
            acc = pht - phk <= kEtaPhi * alpha * gd + 10 * kEps * std::fabs(phk);
            ftype = acc;
          } else {
            acc = tht <= (1 - kGammaTheta) * thk || pht <= phk - kGammaPhi * thk + 10 * kEps * std::fabs(phk);
            ftype = false;
          }
        }
        bool infilter = false;
        for (auto& fe : filter)
          if (tht >= fe.first && pht >= fe.second) { infilter = true; break; }
        if (acc && infilter) {
          acc = false;
          lastrej_f = true;
        } else if (!acc) {
          lastrej_f = false;
        }
        if (acc) { accepted = true; break; }
        alpha *= 0.5;
        if (alpha < amin) break;
      }
    }
    if (!accepted) { status = 3; break; }
    if (!ftype) filter.emplace_back((1 - kGammaTheta) * thk, phk - kGammaPhi * thk);
    if (lastrej_f) {  // filter reset heuristic
      if (++frej >= 5 && nfreset < 5) {
        filter.clear();
        ++nfreset;
        frej = 0;
      }
    } else {
      frej = 0;
    }
    // ---- update
    for (int i = 0; i < nw; ++i) w[i] += alpha * dw[i];
    for (int i = 0; i < ng; ++i) lam[i] += alpha * (lamNew[i] - lam[i]);
    for (int i = 0; i < nw; ++i) {
      if (I.hasL[i]) {
        double s = w[i] - I.lb[i];
        zL[i] += az * dzL[i];
        zL[i] = std::max(std::min(zL[i], kKappaSigma * mu / s), mu / (kKappaSigma * s));
      }
      if (I.hasU[i]) {
        double s = I.ub[i] - w[i];
        zU[i] += az * dzU[i];
        zU[i] = std::max(std::min(zU[i], kKappaSigma * mu / s), mu / (kKappaSigma * s));
      }
    }
    evaluate(I, w, lam, true, e);
  }
  *iters_out = it;
  // unscaled objective
  *f_out = e.f / I.fscale;
  for (int i = 0; i < ng; ++i) lam[i] /= I.fscale;
  if (lamx_out)
    for (int i = 0; i < nw; ++i) lamx_out[i] = (zU[i] - zL[i]) / I.fscale;
  return status;
}

void setup_instance(Instance& I, const oracle_spec* sp, const double* P, const double* pstage, const double* lbw,
                    const double* ubw) {
  const int N = sp->N;
  I.sp = sp;
  I.N = N;
  I.nw = 3 + 5 * N;
  I.xr.assign(3 * N, 0.0);
  I.ur.assign(2 * N, 0.0);
  for (int i = 0; i < NX; ++i) I.x0[i] = P[i];
  for (int k = 0; k < N; ++k) {
    if (pstage) {
      for (int i = 0; i < 3; ++i) I.xr[3 * k + i] = pstage[5 * k + i];
      for (int i = 0; i < 2; ++i) I.ur[2 * k + i] = pstage[5 * k + 3 + i];
    } else {
      for (int i = 0; i < 3; ++i) I.xr[3 * k + i] = P[3 + i];
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

}  // namespace

extern "C" {

// Batched solve.  P: B x 6 ([x0; xref], Casadi scripts) -- or B x 3 (x0) when
// pstage (B x N x 5 per-stage references) is given.  w0: B x nw or NULL (cold).
int oracle_solve_batch(const oracle_spec* sp, int B, const double* P, int p_stride, const double* pstage,
                       const double* w0, const double* lbw, const double* ubw, double* w_out, double* lam_g,
                       double* f_out, int32_t* status, int32_t* iters, int nthreads) {
  const int N = sp->N, nw = 3 + 5 * N, ng = 3 * (N + 1);
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
  for (int b = 0; b < B; ++b) {
    Instance I;
    setup_instance(I, sp, P + (size_t)b * p_stride, pstage ? pstage + (size_t)b * N * 5 : nullptr, lbw, ubw);
    double* w = w_out + (size_t)b * nw;
    if (w0) std::memcpy(w, w0 + (size_t)b * nw, sizeof(double) * nw);
    else std::memset(w, 0, sizeof(double) * nw);
    std::vector<double> lam(ng);
    int it = 0;
    double f = 0;
    int st = solve_one(I, w, lam.data(), sp->max_iter, sp->tol, &it, &f);
    status[b] = st;
    iters[b] = it;
    if (f_out) f_out[b] = f;
    if (lam_g) std::memcpy(lam_g + (size_t)b * ng, lam.data(), sizeof(double) * ng);
  }
  return 0;
}

// Warm-started batched solve: lam0 (B x ng) and lamx0 (B x nw) may be NULL; lamx_out
// (B x nw) receives the bound multipliers (CasADi convention) if not NULL.
int oracle_solve_batch_warm(const oracle_spec* sp, int B, const double* P, int p_stride, const double* w0,
                            const double* lbw, const double* ubw, double mu_init, double bound_push,
                            double mult_push, const double* lam0, const double* lamx0, double* w_out,
                            double* lam_g, double* lamx_out, double* f_out, int32_t* status, int32_t* iters,
                            int nthreads) {
  const int N = sp->N, nw = 3 + 5 * N, ng = 3 * (N + 1);
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
  for (int b = 0; b < B; ++b) {
    Instance I;
    setup_instance(I, sp, P + (size_t)b * p_stride, nullptr, lbw, ubw);
    double* w = w_out + (size_t)b * nw;
    std::memcpy(w, w0 + (size_t)b * nw, sizeof(double) * nw);
    Warm wm{mu_init, bound_push, mult_push, lam0 ? lam0 + (size_t)b * ng : nullptr,
            lamx0 ? lamx0 + (size_t)b * nw : nullptr};
    std::vector<double> lam(ng);
    int it = 0;
    double f = 0;
    status[b] = solve_one(I, w, lam.data(), sp->max_iter, sp->tol, &it, &f, &wm,
                          lamx_out ? lamx_out + (size_t)b * nw : nullptr);
    iters[b] = it;
    if (f_out) f_out[b] = f;
    if (lam_g) std::memcpy(lam_g + (size_t)b * ng, lam.data(), sizeof(double) * ng);
  }
  return 0;
}

// Interval map F and its derivatives for B intervals: x (B x 3), u (B x 2),
// xr (B x 3), ur (B x 2, may be NULL), lam (B x 3, may be NULL).
// Outputs: xf (B x 3), qf (B), jac (B x 4 x 5: rows xf0..2, qf), hess (B x 15:
// Hessian of qf + lam^T xf, packed upper triangle), any may be NULL.
int oracle_stage(const oracle_spec* sp, int B, const double* x, const double* u, const double* xr, const double* ur,
                 const double* lam, double* xf, double* qf, double* jac, double* hess) {
  for (int b = 0; b < B; ++b) {
    const double zero2[2] = {0, 0};
    Jet jx[NX], jq;
    stage_jet(*sp, x + 3 * b, u + 2 * b, xr + 3 * b, ur ? ur + 2 * b : zero2, jx, jq);
    for (int i = 0; i < NX; ++i) if (xf) xf[3 * b + i] = jx[i].v;
    if (qf) qf[b] = jq.v;
    if (jac) {
      for (int r = 0; r < NX; ++r)
        for (int j = 0; j < NZ; ++j) jac[20 * b + 5 * r + j] = jx[r].g[j];
      for (int j = 0; j < NZ; ++j) jac[20 * b + 15 + j] = jq.g[j];
    }
    if (hess) {
      for (int t = 0; t < NH; ++t) {
        double h = jq.h[t];
        if (lam) h += lam[3 * b] * jx[0].h[t] + lam[3 * b + 1] * jx[1].h[t] + lam[3 * b + 2] * jx[2].h[t];
        hess[NH * b + t] = h;
      }
    }
  }
  return 0;
}

}  // extern "C"
