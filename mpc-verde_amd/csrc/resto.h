// resto.h -- IPOPT's soft restoration and feasibility restoration phase for the fused solve
// kernel (kernels.h), as ONE cold, out-of-line device function.
//
// IPOPT enters these only when a filter line search fails (Waechter & Biegler 2006 §3.3; the
// reference relies on IPOPT for it: Casadi/multiple_shooting_casadi.py:188-197).  Kept out of the
// solve launch on purpose: written into its loop the restoration code (never executed on
// configs 1-5) took registers from every iteration -- the cart-pole swing-up's iteration cost
// doubled -- and as an out-of-line call it still cost 20-30 % (the call ABI takes the AGPRs the
// loop spills into).  So the solve launch only parks an instance whose line search fails: its
// iterate, Newton step and loop scalars go to the workspace (RestoWs).  A second launch of the
// same kernel (RESUME, launch_resume: a no-op for everything else) calls recover() on them and
// continues their solves, with recover() inlined there.
//
// What recover() does for a lane group whose line search failed (or that is in IPOPT's soft
// restoration phase), in IPOPT's order (the CPU restatement in the test oracle follows the same):
//  1. soft restoration step (soft_resto_pderror_reduction_factor 0.9999, max_soft_resto_iters
//     10): primal and dual variables take the same step min(alpha_max, alpha_z); accepted by the
//     original filter / sufficient decrease (leaves the soft phase) or by a reduction of the
//     primal-dual error of the barrier problem;
//  2. otherwise, at an acceptable point: "restoration phase called at an acceptable point" ->
//     Solved_To_Acceptable_Level;
//  3. otherwise the restoration phase: min rho ||p + n||_1 + zeta/2 ||D_R (x - x_R)||^2 s.t.
//     c(x) - p + n = 0 (zeta = sqrt(mu), D_R = diag(min(1, 1/|x_R|)), rho = 1000), p, n >= 0,
//     solved by the same primal-dual barrier method (own barrier parameter, own filter, same
//     inertia correction and filter line search).  p and n are eliminated row by row from the
//     Newton system: the value function of node j is seen through its row block (D_j =
//     1/(Sigma_p + delta) + 1/(Sigma_n + delta)) before the stage step, and node j lands through
//     it in the forward pass.  It ends when the iterate is acceptable to the original filter
//     with theta <= 0.9 theta_R0 (back to the original problem: constraint multipliers 0, bound
//     multipliers by a complementarity Newton step, reset to 1 above 1000), or fails (status 3),
//     or converges to a point of local infeasibility (status 4).
#pragma once
#include <hip/hip_runtime.h>

#include "collectives.h"
#include "riccati.h"
#include "solver.h"


namespace mpcx {

// soft restoration (soft_resto_pderror_reduction_factor, max_soft_resto_iters) and the
// restoration phase (rho, kappa_resto = required_infeasibility_reduction,
// bound_mult_reset_threshold; constraint multipliers restart at 0 = constr_mult_reset_threshold 0)
constexpr double kSoftResto = 0.9999, kRho = 1000.0, kKappaResto = 0.9, kBoundMultReset = 1000.0;
constexpr int kMaxSoftResto = 10;

// Model::kResto if the model declares it (the ODE models), false otherwise
template <class M, class = void>
struct RestoOf {
  static constexpr bool value = false;
};
template <class M>
struct RestoOf<M, std::void_t<decltype(M::kResto)>> {
  static constexpr bool value = M::kResto;
};

// Cholesky of a small SPD matrix S (full n x n, row-major) into L; false unless positive definite
template <int n>
__device__ __forceinline__ bool chol_small(const double* S, double* L) {
#pragma unroll
  for (int i = 0; i < n * n; ++i) L[i] = 0.0;
  bool ok = true;
#pragma unroll
  for (int j = 0; j < n; ++j) {
    double d = S[n * j + j];
#pragma unroll
    for (int q = 0; q < j; ++q) d = fma(-L[n * j + q], L[n * j + q], d);
    ok = ok && d > 0.0;
    const double l = sqrt(fmax(d, 1e-300)), rl = 1.0 / l;
    L[n * j + j] = l;
#pragma unroll
    for (int i = j + 1; i < n; ++i) {
      double t = S[n * i + j];
#pragma unroll
      for (int q = 0; q < j; ++q) t = fma(-L[n * i + q], L[n * j + q], t);
      L[n * i + j] = t * rl;
    }
  }
  return ok;
}
template <int n>
__device__ __forceinline__ void chol_solve_small(const double* L, double* b) {
#pragma unroll
  for (int i = 0; i < n; ++i) {
    double t = b[i];
#pragma unroll
    for (int q = 0; q < i; ++q) t = fma(-L[n * i + q], b[q], t);
    b[i] = t / L[n * i + i];
  }
#pragma unroll
  for (int i = n - 1; i >= 0; --i) {
    double t = b[i];
#pragma unroll
    for (int q = i + 1; q < n; ++q) t = fma(-L[n * q + i], b[q], t);
    b[i] = t / L[n * i + i];
  }
}
// S = D^-1 + P (P packed symmetric) and its Cholesky factor; false unless positive definite
template <int NX>
__device__ __forceinline__ bool resto_chol(const double* D, const double* P, double* Di, double* L) {
  double S[NX * NX];
#pragma unroll
  for (int i = 0; i < NX; ++i) Di[i] = 1.0 / D[i];
#pragma unroll
  for (int i = 0; i < NX; ++i)
#pragma unroll
    for (int j = 0; j < NX; ++j) S[NX * i + j] = P[symix(i, j, NX)] + (i == j ? Di[i] : 0.0);
  return chol_small<NX>(S, L);
}
// The value function (P packed, p) of a node seen through its row block's elimination, in the
// forms that stay accurate when barrier terms make P huge (no P - P S^-1 P cancellation):
//   P <- D^-1 - D^-1 S^-1 D^-1,  p <- D^-1 S^-1 p   (as the test oracle's resto_transform).
template <int NX>
__device__ __forceinline__ bool resto_transform(const double* D, double* P, double* p) {
  double Di[NX], L[NX * NX];
  const bool ok = resto_chol<NX>(D, P, Di, L);
  double X[NX][NX + 1];
#pragma unroll
  for (int c = 0; c <= NX; ++c) {
    double b[NX];
#pragma unroll
    for (int i = 0; i < NX; ++i) b[i] = c < NX ? (i == c ? Di[c] : 0.0) : p[i];
    chol_solve_small<NX>(L, b);
#pragma unroll
    for (int i = 0; i < NX; ++i) X[i][c] = b[i];
  }
#pragma unroll
  for (int i = 0; i < NX; ++i) {
#pragma unroll
    for (int j = i; j < NX; ++j)
      P[symix(i, j, NX)] = (i == j ? Di[i] : 0.0) - 0.5 * (Di[i] * X[i][j] + Di[j] * X[j][i]);
    p[i] = Di[i] * X[i][NX];
  }
  return ok;
}

// Scalars handed between the solve loop and recover() (group-uniform values); the filter is
// passed by reference, the arrays travel through the workspace (RestoWs).
struct RecIO {
  // in
  int it, max_iter, k, N, nw, ng;
  bool valid, hasX, hasU, acc_now;
  bool soft_tried = false;  // the solve loop already took this iteration's soft step (kSoftInline)
  double tol, mu_min, fs, nbound, thk, phk, gd, amax, az, sw_a;
  // in / out
  double mu, tau, theta_max, theta_min, dw_last;
  int frej, nfreset, soft_count, xslot, fovf;  // fovf: filter overflows (FilterLds::add)
  bool soft;
  // out
  int status;   // -1: the solve goes on from the state written back; else the final IPOPT status
  int its;      // iteration count when finished
  int it_next;  // the iteration the solve loop continues with
  bool reset_acc;
};

template <class Model, int G>
// (inlined into the resume launch, its only caller)
__device__ __forceinline__ void recover(RecIO& io, FilterLds<G>& filt, const ModelArgs ma, const typename Model::Ctx ctx,
                                        double* wsl, const long wst, const double* lbw, const double* ubw, double* xbuf) {
  constexpr int NX = Model::NX, NU = Model::NU, NZ = NX + NU, NH = NZ * (NZ + 1) / 2, NP = NX * (NX + 1) / 2;
  const int k = io.k, N = io.N, lane = threadIdx.x & 63;
  const bool valid = io.valid, hasX = io.hasX, hasU = io.hasU, has0 = valid && k == 0;
  XWave<G> xw{xbuf, io.xslot};
  auto W = [&](int i) __attribute__((always_inline)) -> double& { return wsl[(long)i * wst]; };
  auto own = [&](int i) __attribute__((always_inline)) { return (i < NX) ? hasX : hasU; };

  // ---- bounds (as the solve kernel: x_0 free, pinned by g_0)
  double lb[NZ], ub[NZ];
  bool hL[NZ], hU[NZ];
#pragma unroll
  for (int i = 0; i < NZ; ++i) {
    lb[i] = -1e20;
    ub[i] = 1e20;
  }
  if (XBoundsOf<Model>::value && hasX && k > 0)
    for (int i = 0; i < NX; ++i) {
      lb[i] = lbw[k == 0 ? i : NX + NZ * (k - 1) + NU + i];
      ub[i] = ubw[k == 0 ? i : NX + NZ * (k - 1) + NU + i];
    }
  if (hasU)
    for (int i = 0; i < NU; ++i) {
      lb[NX + i] = lbw[NX + NZ * k + i];
      ub[NX + i] = ubw[NX + NZ * k + i];
    }
#pragma unroll
  for (int i = 0; i < NZ; ++i) {
    hL[i] = (XBoundsOf<Model>::value || i >= NX) && own(i) && lb[i] > -kInfBound;
    hU[i] = (XBoundsOf<Model>::value || i >= NX) && own(i) && ub[i] < kInfBound;
  }

  // ---- the iterate and its Newton step (RestoWs)
  double z[NZ], lam[NX], zL[NZ], zU[NZ], dz[NZ], dlam[NX], dzL[NZ], dzU[NZ], x0[NX];
#pragma unroll
  for (int i = 0; i < NZ; ++i) {
    z[i] = W(RestoWs::XZ + i);
    zL[i] = W(RestoWs::XZL(NX, NZ) + i);
    zU[i] = W(RestoWs::XZU(NX, NZ) + i);
    dz[i] = W(RestoWs::XDZ(NX, NZ) + i);
    dzL[i] = W(RestoWs::XDZL(NX, NZ) + i);
    dzU[i] = W(RestoWs::XDZU(NX, NZ) + i);
  }
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    lam[i] = W(RestoWs::XL(NZ) + i);
    dlam[i] = W(RestoWs::XDL(NX, NZ) + i);
    x0[i] = W(RestoWs::XX0(NX, NZ) + i);
  }
  auto write_back = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NZ; ++i) {
      W(RestoWs::XZ + i) = z[i];
      W(RestoWs::XZL(NX, NZ) + i) = zL[i];
      W(RestoWs::XZU(NX, NZ) + i) = zU[i];
    }
#pragma unroll
    for (int i = 0; i < NX; ++i) W(RestoWs::XL(NZ) + i) = lam[i];
    io.xslot = xw.slot;
  };

  double mu = io.mu, tau = io.tau;
  const double fs = io.fs;
  io.reset_acc = false;
  io.status = -1;
  io.it_next = io.it + 1;

  // ---- evaluation at (zz, ll): derivatives (objective scaled by fse) and the defects.  As in the
  //      solve loop, interval 0 integrates from the parameter x0 (X_0 enters only g_0): lane 0
  //      evaluates at (x0, U_0), has no x-gradient, and its Newton step treats A_0 as zero
  double xf[NX], qv, A[NX * NX], Bm[NX * NU], gq[NZ], Hs[NH], cdef[NX], c0[NX], ln[NX];
  auto stage_point = [&](const double* zz, double* ze) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NX; ++i) ze[i] = (k == 0) ? x0[i] : zz[i];
#pragma unroll
    for (int i = 0; i < NU; ++i) ze[NX + i] = zz[NX + i];
  };
  auto evaluate = [&](const double* zz, const double* ll, double fse) __attribute__((always_inline)) {
    double own_[2 * NX], nxt[2 * NX], xn[NX];
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      own_[i] = ll[i];
      own_[NX + i] = zz[i];
    }
    group_next<G, 2 * NX>(own_, nxt, xw);
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      ln[i] = nxt[i];
      xn[i] = nxt[NX + i];
    }
    double ze[NZ];
    stage_point(zz, ze);
    stage_derivs<Model, G>(ma, ctx, ze, ln, fse, xf, qv, A, Bm, gq, Hs);
    const double m = hasU ? 1.0 : 0.0, mx = (hasU && k > 0) ? 1.0 : 0.0;
    qv *= m;
#pragma unroll
    for (int i = 0; i < NH; ++i) Hs[i] *= m;
#pragma unroll
    for (int i = 0; i < NZ; ++i) gq[i] *= (i < NX) ? mx : m;
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      cdef[i] = hasU ? xf[i] - xn[i] : 0.0;
      c0[i] = has0 ? x0[i] - zz[i] : 0.0;
    }
  };
  // value at zz: the defects (set 1 on lanes with an interval, set 0 on lane 0) and the stage cost
  auto value_c = [&](const double* zz, double* c1, double* cz, double& q) __attribute__((always_inline)) {
    double xn[NX], xft[NX], ze[NZ];
    group_next<G, NX>(zz, xn, xw);
    stage_point(zz, ze);
    Model::value(ma, ctx, ze, xft, q);
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      c1[i] = hasU ? xft[i] - xn[i] : 0.0;
      cz[i] = has0 ? x0[i] - zz[i] : 0.0;
    }
    q = hasU ? q : 0.0;
  };
  // dual residual of the lane's variables after evaluate(): grad + J^T lam - zL + zU
  auto dual_res = [&](const double* ll, const double* zl, const double* zu, double* r) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NZ; ++i) r[i] = 0;
    if (hasX) {
#pragma unroll
      for (int i = 0; i < NX; ++i) r[i] = gq[i] - ll[i];
      if (hasU) {
        if (k > 0)  // (X_0 enters only g_0)
#pragma unroll
          for (int j = 0; j < NX; ++j)
#pragma unroll
            for (int m = 0; m < NX; ++m)
              if (Model::AMASK & (1ull << (m * NX + j))) r[j] = fma(A[m * NX + j], ln[m], r[j]);
#pragma unroll
        for (int l = 0; l < NU; ++l) {
          double acc = gq[NX + l];
#pragma unroll
          for (int m = 0; m < NX; ++m)
            if (Model::BMASK & (1ull << (m * NU + l))) acc = fma(Bm[m * NU + l], ln[m], acc);
          r[NX + l] = acc;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < NZ; ++i) r[i] += zu[i] - zl[i];
  };
  // primal-dual system error of the original barrier problem at (zz, ll, zl, zu) (IPOPT
  // primal_dual_system_error, 1-norms; the common normalisation cancels in its ratio test)
  auto pd_error = [&](const double* zz, const double* ll, const double* zl, const double* zu) {
    evaluate(zz, ll, fs);
    double r[NZ], acc = 0;
    dual_res(ll, zl, zu, r);
#pragma unroll
    for (int i = 0; i < NZ; ++i) {
      acc += fabs(r[i]);
      if (hL[i]) acc += fabs((zz[i] - lb[i]) * zl[i] - mu);
      if (hU[i]) acc += fabs((ub[i] - zz[i]) * zu[i] - mu);
    }
#pragma unroll
    for (int i = 0; i < NX; ++i) acc += fabs(cdef[i]) + fabs(c0[i]);
    return gsum<G>(acc, xw);
  };
  // bound multipliers after a step (kappa_Sigma safeguard at mu)
  auto clamp_z = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NZ; ++i) {
      if (hL[i]) {
        const double mrs = mu * rcp64(z[i] - lb[i]);
        zL[i] = fmax(fmin(zL[i], kKappaSigma * mrs), mrs * (1.0 / kKappaSigma));
      }
      if (hU[i]) {
        const double mrs = mu * rcp64(ub[i] - z[i]);
        zU[i] = fmax(fmin(zU[i], kKappaSigma * mrs), mrs * (1.0 / kKappaSigma));
      }
    }
  };
  // the filter-reset heuristic after an accepted step
  auto filter_reset = [&](bool lastrej_f, FilterLds<G>& f) __attribute__((always_inline)) {
    if (lastrej_f) {
      if (++io.frej >= kFilterResetTrigger && io.nfreset < kMaxFilterResets) {
        f.clear();
        ++io.nfreset;
        io.frej = 0;
      }
    } else {
      io.frej = 0;
    }
  };

  // ======================================================= 1. soft restoration step
  bool try_soft = false;
  if (io.soft_tried) {
    // the solve loop took (or, past kMaxSoftResto, declined) this iteration's soft step itself
  } else if (io.soft) {
    if (++io.soft_count <= kMaxSoftResto) try_soft = true;
  } else {
    io.soft = true;
    io.soft_count = 0;
    try_soft = true;
  }
  if (try_soft) {
    const double as = fmin(io.amax, io.az);
    double zt[NZ], c1t[NX], c0t[NX], qt;
#pragma unroll
    for (int i = 0; i < NZ; ++i) zt[i] = fma(as, dz[i], z[i]);
    value_c(zt, c1t, c0t, qt);
    double tht_l = 0;
#pragma unroll
    for (int i = 0; i < NX; ++i) tht_l += fabs(c1t[i]) + fabs(c0t[i]);
    const double tht = gsum<G>(tht_l, xw);
    const double pht = gsum<G>(fs * qt - mu * barrier_logsum<NZ>(zt, lb, ub, hL, hU), xw);
    const bool infilter = filt.contains(tht, pht, xw);
    const double thk = io.thk, phk = io.phk, gd = io.gd;
    bool acc = isfinite(pht) && isfinite(tht) && tht <= io.theta_max, ft = false, lastrej_f = false;
    if (acc) {
      if (thk <= io.theta_min && gd < 0 && as > io.sw_a) {
        acc = pht - phk <= kEtaPhi * as * gd + 10.0 * kEps * fabs(phk);
        ft = acc;
      } else {
        acc = tht <= (1.0 - kGammaTheta) * thk || pht <= phk - kGammaPhi * thk + 10.0 * kEps * fabs(phk);
      }
    }
    if (acc && infilter) {
      acc = false;
      lastrej_f = true;
    }
    if (acc) {  // the original criteria hold: a regular step, and the soft phase ends
      if (!ft) io.fovf += filt.add((1.0 - kGammaTheta) * thk, phk - kGammaPhi * thk, k, xw);
      filter_reset(lastrej_f, filt);
#pragma unroll
      for (int i = 0; i < NZ; ++i) {
        z[i] = zt[i];
        zL[i] = fma(as, dzL[i], zL[i]);
        zU[i] = fma(as, dzU[i], zU[i]);
      }
#pragma unroll
      for (int i = 0; i < NX; ++i) lam[i] = fma(as, dlam[i], lam[i]);
      clamp_z();
      io.soft = false;
      io.soft_count = 0;
      write_back();
      return;
    }
    // the primal-dual error at the trial point against the current one
    double lt[NX], zLt[NZ], zUt[NZ];
#pragma unroll
    for (int i = 0; i < NX; ++i) lt[i] = fma(as, dlam[i], lam[i]);
#pragma unroll
    for (int i = 0; i < NZ; ++i) {
      zLt[i] = fma(as, dzL[i], zL[i]);
      zUt[i] = fma(as, dzU[i], zU[i]);
    }
    const double pd_t = pd_error(zt, lt, zLt, zUt);
    const double pd_c = pd_error(z, lam, zL, zU);
    if (pd_t <= kSoftResto * pd_c) {  // accepted; the filter stays as it is
#pragma unroll
      for (int i = 0; i < NZ; ++i) {
        z[i] = zt[i];
        zL[i] = zLt[i];
        zU[i] = zUt[i];
      }
#pragma unroll
      for (int i = 0; i < NX; ++i) lam[i] = lt[i];
      clamp_z();
      write_back();
      return;
    }
  }
  // ======================================================= 2. acceptable point
  if (io.acc_now) {
    io.status = 1;
    io.its = io.it;
    write_back();
    return;
  }
  // ======================================================= 3. restoration phase
  // original problem: augment its filter with the current (theta, phi) and keep it
  io.fovf += filt.add((1.0 - kGammaTheta) * io.thk, io.phk - kGammaPhi * io.thk, k, xw);
  const double th_R0 = io.thk, ph_R0 = io.phk, mu_o = mu;
  // proximity reference and scaling, bound multipliers at the start
  double zR[NZ], dr2[NZ], zLR[NZ], zUR[NZ];
#pragma unroll
  for (int i = 0; i < NZ; ++i) {
    zR[i] = z[i];
    const double d = fmin(1.0, 1.0 / fabs(z[i]));
    dr2[i] = own(i) ? d * d : 0.0;
    zLR[i] = zL[i];
    zUR[i] = zU[i];
    zL[i] = fmin(kRho, zL[i]);
    zU[i] = fmin(kRho, zU[i]);
  }
  // restoration barrier mu_R = max(mu, ||c||_inf); p, n from W&B 2006 (33); z_p = mu/p, z_n = mu/n
  double p1[NX], n1[NX], zp1[NX], zn1[NX], p0[NX], n0[NX], zp0[NX], zn0[NX];
  double r_thmax = 0, r_thmin = 0;  // the restoration problem's theta_max, theta_min
  {
    double c1[NX], cz[NX], q;
    value_c(z, c1, cz, q);
    double cm = 0;
#pragma unroll
    for (int i = 0; i < NX; ++i) cm = fmax(cm, fmax(fabs(c1[i]), fabs(cz[i])));
    mu = fmax(mu, gmax<G>(cm, xw));
    tau = fmax(kTauMin, 1.0 - mu);
    double th = 0;
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      auto init = [&](double c, double& p_, double& n_, double& zp_, double& zn_) {
        const double a_ = (mu - kRho * c) / (2.0 * kRho);
        n_ = a_ + sqrt(a_ * a_ + mu * c / (2.0 * kRho));
        p_ = c + n_;
        zp_ = mu / p_;
        zn_ = mu / n_;
        th += fabs(c - p_ + n_);
      };
      p1[i] = n1[i] = zp1[i] = zn1[i] = p0[i] = n0[i] = zp0[i] = zn0[i] = 1.0;
      if (hasU) init(c1[i], p1[i], n1[i], zp1[i], zn1[i]);
      if (has0) init(cz[i], p0[i], n0[i], zp0[i], zn0[i]);
    }
    th = gsum<G>(th, xw);
    r_thmax = 1e4 * fmax(1.0, th);
    r_thmin = 1e-4 * fmax(1.0, th);
  }
#pragma unroll
  for (int i = 0; i < NX; ++i) lam[i] = 0.0;
  __shared__ double rfbuf[FilterLds<G>::kDoubles];  // the restoration problem's filters
  FilterLds<G> rfilt;
  rfilt.init(rfbuf + threadIdx.x);
  double dw_last = 0.0;
  bool tiny_flag = false;
  int steps = 0, itr = io.it;
  const double nvar = (double)(io.nw + 2 * io.ng), nbnd = io.nbound + 2.0 * io.ng;
  // restoration objective and constraint violation at zz with p, n stepped by al (lane parts)
  double dp1[NX], dn1[NX], dzp1[NX], dzn1[NX], dp0[NX], dn0[NX], dzp0[NX], dzn0[NX];
#pragma unroll
  for (int i = 0; i < NX; ++i) dp1[i] = dn1[i] = dzp1[i] = dzn1[i] = dp0[i] = dn0[i] = dzp0[i] = dzn0[i] = 0.0;
  auto resto_theta_phi = [&](const double* zz, double al, const double* c1, const double* cz, double eta, double& th,
                             double& ph) __attribute__((always_inline)) {
    double t = 0, f = 0, lg = 0;
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      if (hasU) {
        const double p_ = fma(al, dp1[i], p1[i]), n_ = fma(al, dn1[i], n1[i]);
        t += fabs(c1[i] - p_ + n_);
        f += kRho * (p_ + n_);
        lg += log(p_) + log(n_);
      }
      if (has0) {
        const double p_ = fma(al, dp0[i], p0[i]), n_ = fma(al, dn0[i], n0[i]);
        t += fabs(cz[i] - p_ + n_);
        f += kRho * (p_ + n_);
        lg += log(p_) + log(n_);
      }
    }
    double pr = 0;
#pragma unroll
    for (int i = 0; i < NZ; ++i) {
      const double d = zz[i] - zR[i];
      pr = fma(dr2[i] * d, d, pr);
    }
    th = gsum<G>(t, xw);
    ph = gsum<G>(f + 0.5 * eta * pr - mu * (barrier_logsum<NZ>(zz, lb, ub, hL, hU) + lg), xw);
  };

  for (;;) {
    evaluate(z, lam, 0.0);  // the restoration problem has no f
    const double eta = sqrt(mu);
    // ---- progress for the original problem (at least one restoration step)
    if (steps > 0) {
      double t = 0;
#pragma unroll
      for (int i = 0; i < NX; ++i) t += fabs(cdef[i]) + fabs(c0[i]);
      const double th_o = gsum<G>(t, xw);
      const double ph_o = gsum<G>(fs * qv - mu_o * barrier_logsum<NZ>(z, lb, ub, hL, hU), xw);
      // (filt holds the original filter, augmented at the start)
      const bool infilter = filt.contains(th_o, ph_o, xw);
      if (th_o <= kKappaResto * th_R0 && !infilter &&
          (th_o <= (1.0 - kGammaTheta) * th_R0 || ph_o <= ph_R0 - kGammaPhi * th_R0))
        break;
    }
    // ---- optimality error of the restoration problem
    double rd[NZ];
    dual_res(lam, zL, zU, rd);
    double Ed = 0, Ec = 0, Ecomp = 0, lam1 = 0, z1 = 0;
#pragma unroll
    for (int i = 0; i < NZ; ++i) {
      rd[i] = fma(eta * dr2[i], z[i] - zR[i], rd[i]);
      Ed = fmax(Ed, fabs(rd[i]));
      z1 += zL[i] + zU[i];
      if (hL[i]) Ecomp = fmax(Ecomp, fabs((z[i] - lb[i]) * zL[i]));
      if (hU[i]) Ecomp = fmax(Ecomp, fabs((ub[i] - z[i]) * zU[i]));
    }
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      if (hasX) lam1 += fabs(lam[i]);
      if (hasU) {
        Ed = fmax(Ed, fmax(fabs(kRho - ln[i] - zp1[i]), fabs(kRho + ln[i] - zn1[i])));
        Ec = fmax(Ec, fabs(cdef[i] - p1[i] + n1[i]));
        Ecomp = fmax(Ecomp, fmax(fabs(p1[i] * zp1[i]), fabs(n1[i] * zn1[i])));
        z1 += zp1[i] + zn1[i];
      }
      if (has0) {
        Ed = fmax(Ed, fmax(fabs(kRho - lam[i] - zp0[i]), fabs(kRho + lam[i] - zn0[i])));
        Ec = fmax(Ec, fabs(c0[i] - p0[i] + n0[i]));
        Ecomp = fmax(Ecomp, fmax(fabs(p0[i] * zp0[i]), fabs(n0[i] * zn0[i])));
        z1 += zp0[i] + zn0[i];
      }
    }
    Ed = gmax<G>(Ed, xw);
    Ec = gmax<G>(Ec, xw);
    Ecomp = gmax<G>(Ecomp, xw);
    lam1 = gsum<G>(lam1, xw);
    z1 = gsum<G>(z1, xw);
    const double sd = fmax(kSmax, (lam1 + z1) / ((double)io.ng + nvar)) / kSmax;
    const double sc = fmax(kSmax, nbnd > 0 ? z1 / nbnd : 0.0) / kSmax;
    if (fmax(fmax(Ed / sd, Ec), Ecomp / sc) <= io.tol) {  // converged to a point of local infeasibility
      io.status = 4;
      io.its = itr;
      write_back();
      return;
    }
    if (itr >= io.max_iter) {
      io.status = 2;
      io.its = io.max_iter;
      write_back();
      return;
    }
    // ---- barrier update (monotone, fast decrease; a tiny step forces the first decrease)
    for (int rep = 0; rep < 32; ++rep) {
      double Ecm = 0;
#pragma unroll
      for (int i = 0; i < NZ; ++i) {
        if (hL[i]) Ecm = fmax(Ecm, fabs((z[i] - lb[i]) * zL[i] - mu));
        if (hU[i]) Ecm = fmax(Ecm, fabs((ub[i] - z[i]) * zU[i] - mu));
      }
#pragma unroll
      for (int i = 0; i < NX; ++i) {
        if (hasU) Ecm = fmax(Ecm, fmax(fabs(p1[i] * zp1[i] - mu), fabs(n1[i] * zn1[i] - mu)));
        if (has0) Ecm = fmax(Ecm, fmax(fabs(p0[i] * zp0[i] - mu), fabs(n0[i] * zn0[i] - mu)));
      }
      Ecm = gmax<G>(Ecm, xw);
      const double Emu = fmax(fmax(Ed / sd, Ec), Ecm / sc);
      if (!((Emu <= kKappaEps * mu || (tiny_flag && rep == 0)) && mu > io.mu_min)) break;
      mu = fmax(io.mu_min, fmin(kKappaMu * mu, mu * sqrt(mu)));
      tau = fmax(kTauMin, 1.0 - mu);
      rfilt.clear();
    }
    tiny_flag = false;
    // ---- barrier gradient, Sigma; the proximity term at the new mu
    const double eta_n = sqrt(mu);
    double sig[NZ], gp[NZ];
#pragma unroll
    for (int i = 0; i < NZ; ++i) {
      sig[i] = eta_n * dr2[i];
      gp[i] = fma(sig[i], z[i] - zR[i], gq[i]);
      if (hL[i]) {
        const double rs = rcp64(z[i] - lb[i]);
        sig[i] = fma(zL[i], rs, sig[i]);
        gp[i] = fma(-mu, rs, gp[i]);
      }
      if (hU[i]) {
        const double rs = rcp64(ub[i] - z[i]);
        sig[i] = fma(zU[i], rs, sig[i]);
        gp[i] = fma(mu, rs, gp[i]);
      }
    }
    // ---- Newton step: sequential Riccati through the row blocks, inertia correction
    double delta = 0.0, Pk[NP], pk[NX], D1[NX], ct1[NX], D0[NX], ct0[NX];
    Fac<NX, NU> fac = {};
    bool need = true, failed = false, first = true;
    auto rows = [&](double dl) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < NX; ++i) {
        const double sp1 = zp1[i] / p1[i] + dl, sn1 = zn1[i] / n1[i] + dl;
        D1[i] = 1.0 / sp1 + 1.0 / sn1;
        ct1[i] = cdef[i] - p1[i] + n1[i] + (kRho - mu / p1[i]) / sp1 - (kRho - mu / n1[i]) / sn1;
        const double sp0 = zp0[i] / p0[i] + dl, sn0 = zn0[i] / n0[i] + dl;
        D0[i] = 1.0 / sp0 + 1.0 / sn0;
        ct0[i] = c0[i] - p0[i] + n0[i] + (kRho - mu / p0[i]) / sp0 - (kRho - mu / n0[i]) / sn0;
      }
    };
    for (int attempt = 0; attempt < 64 && need; ++attempt) {
      double Hd[NH];
#pragma unroll
      for (int i = 0; i < NH; ++i) Hd[i] = Hs[i];
#pragma unroll
      for (int i = 0; i < NZ; ++i) Hd[symix(i, i, NZ)] += sig[i] + delta;
      rows(delta);
      double P[NP], p[NX];
      const double dl = (k == N) ? 1.0 : 0.0;  // P_N = Sigma_x + delta, p_N = barrier gradient
#pragma unroll
      for (int i = 0; i < NX; ++i) {
#pragma unroll
        for (int j = i; j < NX; ++j) P[symix(i, j, NX)] = (i == j) ? dl * (sig[i] + delta) : 0.0;
        p[i] = dl * gp[i];
      }
      bool okl = true;
      auto step = [&](double* Pin_, double* pin_) __attribute__((always_inline)) {
        const bool okt = resto_transform<NX>(D1, Pin_, pin_);
        okl = riccati_step<NX, NU, Model::AMASK, Model::BMASK, false, false, AOneOf<Model>::value>(Hd, gp, A, Bm, ct1, Pin_,
                                                                                                    pin_, P, p, fac) && okt;
      };
      if constexpr (G <= 64) {
        for (int j = N - 1; j >= 0; --j) {
          double Pin_[NP], pin_[NX];
#pragma unroll
          for (int i = 0; i < NP; ++i) Pin_[i] = from_next(P[i]);
#pragma unroll
          for (int i = 0; i < NX; ++i) pin_[i] = from_next(p[i]);
          if (k == j) step(Pin_, pin_);
        }
      } else {  // wave by wave, N-side first; the value function crosses waves through LDS
        const int wv = (int)(threadIdx.x >> 6);
        for (int ph = XWave<G>::W - 1; ph >= 0; --ph) {
          if (wv == ph) {
            const double* in = xw.prev();
            const int jtop = 64 * ph + 63;
            for (int j = min(N - 1, jtop); j >= 64 * ph; --j) {
              double Pin_[NP], pin_[NX];
#pragma unroll
              for (int i = 0; i < NP; ++i) Pin_[i] = from_next(P[i]);
#pragma unroll
              for (int i = 0; i < NX; ++i) pin_[i] = from_next(p[i]);
              if (j == jtop && lane == 63) {
#pragma unroll
                for (int i = 0; i < NP; ++i) Pin_[i] = in[i];
#pragma unroll
                for (int i = 0; i < NX; ++i) pin_[i] = in[NP + i];
              }
              if (k == j) step(Pin_, pin_);
            }
            if (ph > 0 && lane == 0) {
              double* out = xw.cur();
#pragma unroll
              for (int i = 0; i < NP; ++i) out[i] = P[i];
#pragma unroll
              for (int i = 0; i < NX; ++i) out[NP + i] = p[i];
            }
          }
          xw.sync();
        }
      }
      if (k == 0) {  // node 0 (A_0 = 0, no x blocks in stage 0): P_0 = Sigma_x + delta, p_0 = gp_x
#pragma unroll
        for (int i = 0; i < NX; ++i) {
#pragma unroll
          for (int j = i; j < NX; ++j) P[symix(i, j, NX)] = (i == j) ? sig[i] + delta : 0.0;
          p[i] = gp[i];
        }
      }
#pragma unroll
      for (int i = 0; i < NP; ++i) Pk[i] = P[i];
#pragma unroll
      for (int i = 0; i < NX; ++i) pk[i] = p[i];
      if (has0) {  // X_0's row block g_0: D_0^-1 + P_0 positive definite
        double Di[NX], L[NX * NX];
        okl = resto_chol<NX>(D0, Pk, Di, L) && okl;
      }
      const bool ok = gmin<G>(okl ? 1.0 : 0.0, xw) > 0.5;
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
    if (failed) {
      io.status = 5;
      io.its = itr;
      write_back();
      return;
    }
    double Kk[NU * NX], kfk[NU];
    riccati_gains<NX, NU>(fac, Kk, kfk);
    if (k == 0)  // Hux'_0 = 0 (A_0 = 0)
#pragma unroll
      for (int i = 0; i < NU * NX; ++i) Kk[i] = 0.0;
    // ---- forward pass, node by node: node j+1 lands through its row block,
    //      dx_{j+1} = S^-1 (D^-1 y - p_{j+1}), y = A dx_j + B du_j + ct, S = D^-1 + P_{j+1}
    double Pv[NP + NX], Pn1[NP + NX];
#pragma unroll
    for (int i = 0; i < NP; ++i) Pv[i] = Pk[i];
#pragma unroll
    for (int i = 0; i < NX; ++i) Pv[NP + i] = pk[i];
    group_next<G, NP + NX>(Pv, Pn1, xw);
    double dxk[NX], dxn[NX];
#pragma unroll
    for (int i = 0; i < NX; ++i) dxk[i] = dxn[i] = 0.0;
    if (has0) {
      double Di[NX], L[NX * NX];
      resto_chol<NX>(D0, Pk, Di, L);
#pragma unroll
      for (int i = 0; i < NX; ++i) dxk[i] = fma(Di[i], ct0[i], -pk[i]);
      chol_solve_small<NX>(L, dxk);
    }
    auto advance = [&]() __attribute__((always_inline)) {  // on lane j: dx_{j+1} from dx_j
      double du[NU], y[NX], Di[NX], L[NX * NX];
#pragma unroll
      for (int l = 0; l < NU; ++l) {
        double acc = kfk[l];
#pragma unroll
        for (int m = 0; m < NX; ++m) acc = fma(Kk[l * NX + m], dxk[m], acc);
        du[l] = acc;
      }
#pragma unroll
      for (int r = 0; r < NX; ++r) {
        double acc = ct1[r];
        if (k > 0)  // dx_1 does not depend on dx_0 (A_0 = 0)
#pragma unroll
          for (int m = 0; m < NX; ++m) acc = fma(A[r * NX + m], dxk[m], acc);
#pragma unroll
        for (int l = 0; l < NU; ++l) acc = fma(Bm[r * NU + l], du[l], acc);
        y[r] = acc;
      }
      resto_chol<NX>(D1, Pn1, Di, L);
#pragma unroll
      for (int i = 0; i < NX; ++i) dxn[i] = fma(Di[i], y[i], -Pn1[NP + i]);
      chol_solve_small<NX>(L, dxn);
    };
    if constexpr (G <= 64) {
      for (int j = 0; j < N; ++j) {
        if (k == j) advance();
        double t[NX];
#pragma unroll
        for (int i = 0; i < NX; ++i) t[i] = from_prev(dxn[i]);
        if (k == j + 1)
#pragma unroll
          for (int i = 0; i < NX; ++i) dxk[i] = t[i];
      }
    } else {  // wave by wave, node 0 side first; dx crosses waves through LDS
      const int wv = (int)(threadIdx.x >> 6);
      for (int ph = 0; ph < XWave<G>::W; ++ph) {
        if (wv == ph) {
          if (ph > 0 && lane == 0) {
            const double* in = xw.prev();
#pragma unroll
            for (int i = 0; i < NX; ++i) dxk[i] = in[i];
          }
          for (int j = 64 * ph; j < min(N, 64 * ph + 64); ++j) {
            if (k == j) advance();
            double t[NX];
#pragma unroll
            for (int i = 0; i < NX; ++i) t[i] = from_prev(dxn[i]);
            if (k == j + 1 && lane != 0)
#pragma unroll
              for (int i = 0; i < NX; ++i) dxk[i] = t[i];
          }
          if (lane == 63) {
            double* out = xw.cur();
#pragma unroll
            for (int i = 0; i < NX; ++i) out[i] = dxn[i];
          }
        }
        xw.sync();
      }
    }
    // ---- the step: du_k = K dx_k + k_f, lam+ = P_k dx_k + p_k; rows' p, n and multipliers
    double lp[NX], lpn[NX];
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      dz[i] = hasX ? dxk[i] : 0.0;
      double acc = pk[i];
#pragma unroll
      for (int m = 0; m < NX; ++m) acc = fma(Pk[symix(i, m, NX)], dxk[m], acc);
      lp[i] = hasX ? acc : 0.0;
      dlam[i] = lp[i] - lam[i];
    }
#pragma unroll
    for (int l = 0; l < NU; ++l) {
      double acc = kfk[l];
#pragma unroll
      for (int m = 0; m < NX; ++m) acc = fma(Kk[l * NX + m], dxk[m], acc);
      dz[NX + l] = hasU ? acc : 0.0;
    }
    group_next<G, NX>(lp, lpn, xw);
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      auto stp = [&](double l, double p_, double n_, double zp_, double zn_, double& dp_, double& dn_, double& dzp_,
                     double& dzn_) {
        dp_ = (l - kRho + mu / p_) / (zp_ / p_ + delta);
        dn_ = (-l - kRho + mu / n_) / (zn_ / n_ + delta);
        dzp_ = mu / p_ - zp_ - zp_ / p_ * dp_;
        dzn_ = mu / n_ - zn_ - zn_ / n_ * dn_;
      };
      if (hasU) stp(lpn[i], p1[i], n1[i], zp1[i], zn1[i], dp1[i], dn1[i], dzp1[i], dzn1[i]);
      if (has0) stp(lp[i], p0[i], n0[i], zp0[i], zn0[i], dp0[i], dn0[i], dzp0[i], dzn0[i]);
    }
    // ---- bound-dual steps, fraction to the boundary, tiny step, directional derivative
    double am_l = 1.0, az_l = 1.0, tiny_l = 0.0, gd_l = 0.0;
#pragma unroll
    for (int i = 0; i < NZ; ++i) {
      dzL[i] = dzU[i] = 0.0;
      if (hL[i]) {
        const double s = z[i] - lb[i], rs = rcp64(s);
        dzL[i] = fma(mu, rs, -zL[i]) - zL[i] * rs * dz[i];
        if (dz[i] < 0) am_l = fmin(am_l, -tau * s / dz[i]);
        if (dzL[i] < 0) az_l = fmin(az_l, -tau * zL[i] / dzL[i]);
      }
      if (hU[i]) {
        const double s = ub[i] - z[i], rs = rcp64(s);
        dzU[i] = fma(mu, rs, -zU[i]) + zU[i] * rs * dz[i];
        if (dz[i] > 0) am_l = fmin(am_l, tau * s / dz[i]);
        if (dzU[i] < 0) az_l = fmin(az_l, -tau * zU[i] / dzU[i]);
      }
      if (own(i)) {
        tiny_l = fmax(tiny_l, fabs(dz[i]) / (1.0 + fabs(z[i])));
        gd_l += gp[i] * dz[i];
      }
    }
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      auto rowb = [&](double p_, double n_, double zp_, double zn_, double dp_, double dn_, double dzp_, double dzn_) {
        if (dp_ < 0) am_l = fmin(am_l, -tau * p_ / dp_);
        if (dn_ < 0) am_l = fmin(am_l, -tau * n_ / dn_);
        if (dzp_ < 0) az_l = fmin(az_l, -tau * zp_ / dzp_);
        if (dzn_ < 0) az_l = fmin(az_l, -tau * zn_ / dzn_);
        tiny_l = fmax(tiny_l, fmax(fabs(dp_) / (1.0 + p_), fabs(dn_) / (1.0 + n_)));
        gd_l += (kRho - mu / p_) * dp_ + (kRho - mu / n_) * dn_;
      };
      if (hasU) rowb(p1[i], n1[i], zp1[i], zn1[i], dp1[i], dn1[i], dzp1[i], dzn1[i]);
      if (has0) rowb(p0[i], n0[i], zp0[i], zn0[i], dp0[i], dn0[i], dzp0[i], dzn0[i]);
    }
    const double amax = gmin<G>(am_l, xw), az = gmin<G>(az_l, xw), tiny = gmax<G>(tiny_l, xw);
    const double gd = gsum<G>(gd_l, xw);
    // ---- filter line search on the restoration problem
    double thk, phk;
    resto_theta_phi(z, 0.0, cdef, c0, eta_n, thk, phk);
    double alpha = amax;
    bool accepted = false, ftype = false, lastrej_f = false;
    if (tiny < 10.0 * kEps) {
      accepted = ftype = tiny_flag = true;
    } else {
      const double sw_a = gd < 0 ? exp_fd(kSTheta * log_fd(thk) - kSPhi * log_fd(-gd)) : 0.0;  // kDeltaSw = 1
      const double amin = gd < 0 ? kGammaAlpha * fmin(kGammaTheta, fmin(kGammaPhi * thk / (-gd), sw_a))
                                 : kGammaAlpha * kGammaTheta;
      for (int ls = 0; ls < 80; ++ls) {
        double zt[NZ], c1t[NX], c0t[NX], qt, tht, pht;
#pragma unroll
        for (int i = 0; i < NZ; ++i) zt[i] = fma(alpha, dz[i], z[i]);
        value_c(zt, c1t, c0t, qt);
        resto_theta_phi(zt, alpha, c1t, c0t, eta_n, tht, pht);
        const bool infilter = rfilt.contains(tht, pht, xw);
        bool acc = isfinite(pht) && isfinite(tht) && tht <= r_thmax, ft = false;
        if (acc) {
          if (thk <= r_thmin && gd < 0 && alpha > sw_a) {
            acc = pht - phk <= kEtaPhi * alpha * gd + 10.0 * kEps * fabs(phk);
            ft = acc;
          } else {
            acc = tht <= (1.0 - kGammaTheta) * thk || pht <= phk - kGammaPhi * thk + 10.0 * kEps * fabs(phk);
          }
        }
        if (acc && infilter) {
          acc = false;
          lastrej_f = true;
        } else if (!acc) {
          lastrej_f = false;
        }
        if (acc) {
          accepted = true;
          ftype = ft;
          break;
        }
        alpha *= 0.5;
        if (alpha < amin) break;
      }
    }
    if (!accepted) {  // a failed line search inside the restoration phase
      io.status = 3;
      io.its = itr;
      write_back();
      return;
    }
    // ---- update
    if (!ftype) io.fovf += rfilt.add((1.0 - kGammaTheta) * thk, phk - kGammaPhi * thk, k, xw);
    filter_reset(lastrej_f, rfilt);
#pragma unroll
    for (int i = 0; i < NZ; ++i) {
      z[i] = fma(alpha, dz[i], z[i]);
      zL[i] = fma(az, dzL[i], zL[i]);
      zU[i] = fma(az, dzU[i], zU[i]);
    }
#pragma unroll
    for (int i = 0; i < NX; ++i) lam[i] = fma(alpha, dlam[i], lam[i]);
    clamp_z();
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      auto upd = [&](double& p_, double& n_, double& zp_, double& zn_, double dp_, double dn_, double dzp_, double dzn_) {
        p_ = fma(alpha, dp_, p_);
        n_ = fma(alpha, dn_, n_);
        const double mp = mu / p_, mn = mu / n_;
        zp_ = fmax(fmin(fma(az, dzp_, zp_), kKappaSigma * mp), mp / kKappaSigma);
        zn_ = fmax(fmin(fma(az, dzn_, zn_), kKappaSigma * mn), mn / kKappaSigma);
      };
      if (hasU) upd(p1[i], n1[i], zp1[i], zn1[i], dp1[i], dn1[i], dzp1[i], dzn1[i]);
      if (has0) upd(p0[i], n0[i], zp0[i], zn0[i], dp0[i], dn0[i], dzp0[i], dzn0[i]);
    }
    ++steps;
    ++itr;
  }
  // ---- back to the original problem at iteration itr: its barrier, filter and safeguards;
  //      constraint multipliers 0; bound multipliers from a complementarity Newton step over the
  //      whole restoration step (reset to 1 above bound_mult_reset_threshold)
  mu = mu_o;
  tau = io.tau;
  double zmax = 0;
#pragma unroll
  for (int i = 0; i < NZ; ++i) {
    auto upd = [&](double z0, double s0, double s1) {
      const double d = mu / s0 - z0 - z0 / s0 * (s1 - s0);
      const double al = d < 0 ? fmin(1.0, -tau * z0 / d) : 1.0;
      return z0 + al * d;
    };
    zL[i] = hL[i] ? upd(zLR[i], zR[i] - lb[i], z[i] - lb[i]) : 0.0;
    zU[i] = hU[i] ? upd(zUR[i], ub[i] - zR[i], ub[i] - z[i]) : 0.0;
    zmax = fmax(zmax, fmax(zL[i], zU[i]));
  }
  if (gmax<G>(zmax, xw) > kBoundMultReset)
#pragma unroll
    for (int i = 0; i < NZ; ++i) {
      zL[i] = hL[i] ? 1.0 : 0.0;
      zU[i] = hU[i] ? 1.0 : 0.0;
    }
#pragma unroll
  for (int i = 0; i < NX; ++i) lam[i] = 0.0;
  io.mu = mu;  // (unchanged: the original problem's)
  io.soft = false;
  io.soft_count = 0;
  io.reset_acc = true;
  io.it_next = itr;
  write_back();
}

}  // namespace mpcx
