"""NumPy fp64 oracle for the receding-horizon MPC NLP of gabrielhaj/mpc-verde.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the
checker.  The product path (``mpc-verde_amd/``) never imports it.

Parity status: PINNED.  The functions below are checked in ``tests/test_oracle.py``
against the reference's own closed-loop outputs ``Casadi/1exemplo.xlsx`` and
``Casadi/2exemplo.xlsx`` (decoded into ``tests/golden/unicycle_N10_golden.json``):
the RK4 plant reproduces the 84 recorded state transitions to round-off, and the
solver reproduces all 84 recorded first controls u0* (CasADi+IPOPT solves) within
the golden-vs-golden spread.

What is restated (all fp64, all citations relative to /root/reference):

* unicycle right-hand side ``rhs = [v cos th, v sin th, w]``
  -- ``Casadi/multiple_shooting_casadi.py:68-72``
* stage cost ``L = (s - xr)^T Q (s - xr) + u^T R u`` -- ``:78-87``
* the RK4 integrator with cost quadrature ``F(P, U) -> (xf, qf)``, M substeps of
  DT = T/M -- ``:98-114``
* the multiple-shooting NLP: interleaved decision vector
  ``w = [X_0 | U_0 X_1 | ... | U_{N-1} X_N]``, lifted initial state
  ``g_0 = P[:3] - X_0``, defects ``g_{k+1} = F(X_k, U_k).xf - X_{k+1}``, objective
  ``J = sum_k F(X_k, U_k).qf``, bounds on U only -- ``:116-178``
* the single-shooting NLP (decision = U only) -- ``Casadi/single_shooting_v2.py:115-158``
* the closed-loop driver (plant = F, stop when ||x - x_t||_2 <= 0.1 or t >= 20 s)
  -- ``Casadi/multiple_shooting_casadi.py:224-298``
* the mpctools tracking variant (RK4 M=1 discrete model, node cost
  ``l(x_k, u_k, p_k)``, per-stage reference p_k) --
  ``Trajectory Tracking/Trajectory_tracking.py:40-61,84-97``

The reference solves the NLP with IPOPT (CasADi ``nlpsol``, not vendored).  The
solver here is deliberately a *different* algorithm so that it can check the
product's interior-point solver independently: projected Newton (Bertsekas 1982)
on the single-shooting form (bounds on U only), with exact gradients from the
complex-step method and an exact Hessian from the discrete second-order adjoint
over per-stage Hessian blocks (finite differences of complex-step gradients).
Single and multiple shooting share their optimum (the reference shows it:
``1exemplo`` vs ``2exemplo`` agree to 1.6e-7), so either form pins the other.
"""
from __future__ import annotations

import dataclasses
import math

import numpy as np

# ----------------------------------------------------------------------------
# Problem description (mirrors the module constants of the reference scripts)
# ----------------------------------------------------------------------------


@dataclasses.dataclass
class UnicycleOCP:
    """Constants of ``Casadi/multiple_shooting_casadi.py:30-45,78-84,101``.

    cost = "quadrature": J = sum_k RK4-quadrature of L over the interval
           (``:98-113``, the CasADi scripts);
    cost = "node":       J = sum_k l(x_k, u_k, p_k) (mpctools ``nmpc``,
           ``Trajectory Tracking/Trajectory_tracking.py:57-61``).
    """

    N: int = 10
    T: float = 0.2
    M: int = 4
    Q: tuple = (1.0, 5.0, 0.1)
    R: tuple = (0.5, 0.05)
    v_max: float = 1.0
    omega_max: float = math.pi / 4
    cost: str = "quadrature"
    x_lb: tuple = (-np.inf, -np.inf, -np.inf)
    x_ub: tuple = (np.inf, np.inf, np.inf)

    @property
    def nx(self):
        return 3

    @property
    def nu(self):
        return 2

    @property
    def u_lb(self):
        return np.array([-self.v_max, -self.omega_max])

    @property
    def u_ub(self):
        return np.array([self.v_max, self.omega_max])


def tracking_ocp(N=10):
    """``Trajectory Tracking/Trajectory_tracking.py:15-67``: Q=diag(1,1,.1),
    R=diag(.5,.05), Delta=0.2, RK4 M=1, state bounds x in [-20,20], y in [-2,2]."""
    return UnicycleOCP(N=N, T=0.2, M=1, Q=(1.0, 1.0, 0.1), R=(0.5, 0.05), cost="node",
                       x_lb=(-20.0, -2.0, -np.inf), x_ub=(20.0, 2.0, np.inf))


# ----------------------------------------------------------------------------
# Model and integrator (array-broadcasting; real or complex)
# ----------------------------------------------------------------------------


def rhs(x, u):
    """Unicycle ODE -- ``Casadi/multiple_shooting_casadi.py:68-72``."""
    th = x[..., 2]
    v = u[..., 0]
    w = u[..., 1]
    return np.stack([v * np.cos(th), v * np.sin(th), w + 0 * th], axis=-1)


def stage_L(x, u, xr, ur, Q, R):
    """``L = (s - xr)^T Q (s - xr) + (u - ur)^T R (u - ur)`` -- ``:87`` (ur = 0 there)
    and ``Trajectory Tracking/Trajectory_tracking.py:57-58`` (ur = p[3:5])."""
    dx = x - xr
    du = u - ur
    return (Q[0] * dx[..., 0] ** 2 + Q[1] * dx[..., 1] ** 2 + Q[2] * dx[..., 2] ** 2
            + R[0] * du[..., 0] ** 2 + R[1] * du[..., 1] ** 2)


def F(x0, u, xr, ocp: UnicycleOCP, ur=None):
    """RK4 interval map with cost quadrature -- ``:98-114``.

    Returns (xf, qf).  For cost == "node" qf is the node cost l(x0, u, p)
    (mpctools evaluates l at the shooting node, no quadrature).
    """
    if ur is None:
        ur = np.zeros_like(u)
    Q, R = ocp.Q, ocp.R
    DT = ocp.T / ocp.M
    X = x0
    q = 0.0 * x0[..., 0]
    for _ in range(ocp.M):
        k1 = rhs(X, u)
        k2 = rhs(X + DT / 2 * k1, u)
        k3 = rhs(X + DT / 2 * k2, u)
        k4 = rhs(X + DT * k3, u)
        if ocp.cost == "quadrature":
            q1 = stage_L(X, u, xr, ur, Q, R)
            q2 = stage_L(X + DT / 2 * k1, u, xr, ur, Q, R)
            q3 = stage_L(X + DT / 2 * k2, u, xr, ur, Q, R)
            q4 = stage_L(X + DT * k3, u, xr, ur, Q, R)
            q = q + DT / 6 * (q1 + 2 * q2 + 2 * q3 + q4)
        X = X + DT / 6 * (k1 + 2 * k2 + 2 * k3 + k4)
    if ocp.cost == "node":
        q = stage_L(x0, u, xr, ur, Q, R)
    return X, q


# ----------------------------------------------------------------------------
# Multiple-shooting NLP in the reference's interleaved layout
# ----------------------------------------------------------------------------


def n_w(N):
    return 3 + 5 * N


def n_g(N):
    return 3 * (N + 1)


def split_w(w, N):
    """w = [X_0 | U_0 X_1 | ...] (``:128-170``) -> X (...,N+1,3), U (...,N,2)."""
    w = np.asarray(w)
    X0 = w[..., 0:3]
    body = w[..., 3:].reshape(w.shape[:-1] + (N, 5))
    U = body[..., 0:2]
    X = np.concatenate([X0[..., None, :], body[..., 2:5]], axis=-2)
    return X, U


def join_w(X, U):
    N = U.shape[-2]
    body = np.concatenate([U, X[..., 1:, :]], axis=-1)
    return np.concatenate([X[..., 0, :], body.reshape(body.shape[:-2] + (5 * N,))], axis=-1)


def stage_refs(P, ocp: UnicycleOCP, pstage=None):
    """Per-stage references (xr_k, ur_k), shape (..., N, 3) and (..., N, 2).

    Casadi scripts: P = [x0; xref] with one xref for all stages (``:74,87``).
    Tracking: pstage[..., k, :] = (x_r, y_r, th_r, v_r, w_r) (``Trajectory_tracking.py:84-97``).
    """
    N = ocp.N
    if pstage is None:
        xr = np.broadcast_to(np.asarray(P)[..., None, 3:6], np.shape(P)[:-1] + (N, 3))
        ur = np.zeros(np.shape(P)[:-1] + (N, 2))
    else:
        xr = np.asarray(pstage)[..., 0:3]
        ur = np.asarray(pstage)[..., 3:5]
    return xr, ur


def ms_functions(w, P, ocp: UnicycleOCP, pstage=None):
    """Objective and constraints of the multiple-shooting NLP (``:141-178``).  Interval 0
    integrates from the parameter (``Xk = P[:n_states]`` at ``:125``, ``F(x0=vertcat(Xk,
    P[3:]), p=Uk)`` at ``:157``): the lifted X_0 enters only g_0."""
    N = ocp.N
    X, U = split_w(w, N)
    xr, ur = stage_refs(P, ocp, pstage)
    Xs = X[..., :-1, :].copy()
    Xs[..., 0, :] = np.asarray(P)[..., 0:3]
    xf, qf = F(Xs, U, xr, ocp, ur)
    J = qf.sum(axis=-1)
    g0 = np.asarray(P)[..., 0:3] - X[..., 0, :]
    gk = xf - X[..., 1:, :]
    g = np.concatenate([g0, gk.reshape(gk.shape[:-2] + (3 * N,))], axis=-1)
    return J, g


def ms_bounds(ocp: UnicycleOCP):
    """lbw/ubw of ``:132-168`` (X_0 free; states bounded only for tracking)."""
    N = ocp.N
    lb = np.full(n_w(N), -np.inf)
    ub = np.full(n_w(N), np.inf)
    for k in range(N):
        lb[3 + 5 * k:5 + 5 * k] = ocp.u_lb
        ub[3 + 5 * k:5 + 5 * k] = ocp.u_ub
        lb[5 + 5 * k:8 + 5 * k] = ocp.x_lb
        ub[5 + 5 * k:8 + 5 * k] = ocp.x_ub
    return lb, ub


# ----------------------------------------------------------------------------
# Per-stage derivatives by the complex-step method (exact to round-off)
# ----------------------------------------------------------------------------

_CS_H = 1e-30


def stage_jacobian(x, u, xr, ocp: UnicycleOCP, ur=None):
    """d[xf; qf]/d[x; u] for each interval: shape (..., 4, 5).  Complex step."""
    z = np.concatenate([x, u], axis=-1).astype(complex)
    zc = z[..., None, :] + 1j * _CS_H * np.eye(5)  # (..., 5 dirs, 5)
    xrc = np.asarray(xr)[..., None, :]
    urc = None if ur is None else np.asarray(ur)[..., None, :]
    xf, qf = F(zc[..., 0:3], zc[..., 3:5], xrc, ocp, urc)
    out = np.concatenate([xf, qf[..., None]], axis=-1).imag / _CS_H  # (..., dir, 4)
    return np.swapaxes(out, -1, -2)


def stage_value_jac(x, u, xr, ocp, ur=None):
    xf, qf = F(x, u, xr, ocp, ur)
    return xf, qf, stage_jacobian(x, u, xr, ocp, ur)


def stage_hessians(x, u, xr, ocp: UnicycleOCP, ur=None, delta=2e-5):
    """Hessians of [xf_0, xf_1, xf_2, qf] w.r.t. (x, u): shape (..., 4, 5, 5).

    Central differences of the exact complex-step Jacobian; error ~1e-9."""
    z = np.concatenate([x, u], axis=-1)
    Hs = []
    for b in range(5):
        e = np.zeros(5)
        e[b] = delta
        Jp = stage_jacobian((z + e)[..., 0:3], (z + e)[..., 3:5], xr, ocp, ur)
        Jm = stage_jacobian((z - e)[..., 0:3], (z - e)[..., 3:5], xr, ocp, ur)
        Hs.append((Jp - Jm) / (2 * delta))  # (..., 4, 5): d/dz_b of row gradients
    H = np.stack(Hs, axis=-1)  # (..., 4, 5 (a), 5 (b))
    return 0.5 * (H + np.swapaxes(H, -1, -2))


# ----------------------------------------------------------------------------
# Single-shooting reduced problem: value, gradient (adjoint), Hessian (2nd-order adjoint)
# ----------------------------------------------------------------------------


def ss_rollout(U, P, ocp, pstage=None):
    """X_{k+1} = F(X_k, U_k).xf from X_0 = P[:3]; J = sum qf (``single_shooting_v2.py:128-150``)."""
    N = ocp.N
    xr, ur = stage_refs(P, ocp, pstage)
    X = [np.asarray(P)[..., 0:3]]
    J = 0.0
    for k in range(N):
        xf, qf = F(X[-1], U[..., k, :], xr[..., k, :], ocp, ur[..., k, :])
        X.append(xf)
        J = J + qf
    return np.stack(X, axis=-2), J


def ss_derivatives(U, P, ocp, pstage=None, hessian=True):
    """J, dJ/dU (N,2) and d2J/dU2 (2N,2N) for one instance."""
    N = ocp.N
    xr, ur = stage_refs(P, ocp, pstage)
    X, J = ss_rollout(U, P, ocp, pstage)
    Jac = stage_jacobian(X[:-1], U, xr, ocp, ur)  # (N, 4, 5)
    A = Jac[:, 0:3, 0:3]
    Bm = Jac[:, 0:3, 3:5]
    gx = Jac[:, 3, 0:3]
    gu = Jac[:, 3, 3:5]
    lam = np.zeros((N + 1, 3))  # lam[k] = dJ_{>=k}/dx_k
    g = np.zeros((N, 2))
    for k in range(N - 1, -1, -1):
        g[k] = gu[k] + Bm[k].T @ lam[k + 1]
        lam[k] = gx[k] + A[k].T @ lam[k + 1]
    if not hessian:
        return J, g, None, X
    Hst = stage_hessians(X[:-1], U, xr, ocp, ur)  # (N, 4, 5, 5)
    H = np.zeros((2 * N, 2 * N))
    S = np.zeros((3, 2 * N))
    for k in range(N):
        Hk = Hst[k, 3] + np.einsum("c,cab->ab", lam[k + 1], Hst[k, 0:3])
        E = np.zeros((2, 2 * N))
        E[0, 2 * k] = 1.0
        E[1, 2 * k + 1] = 1.0
        D = np.vstack([S, E])
        H += D.T @ Hk @ D
        S = A[k] @ S + Bm[k] @ E
    return J, g, 0.5 * (H + H.T), X


def solve_single_shooting(P, ocp: UnicycleOCP, u0=None, pstage=None, tol=1e-11, max_iter=200):
    """Projected Newton (Bertsekas 1982) on min_U J(U) s.t. lb <= U <= ub.

    Returns (U (N,2), X (N+1,3), info dict).  Exact gradient; exact Hessian
    (up to the ~1e-9 finite-difference error of the stage blocks, which affects
    only the rate, not the fixed point).
    """
    N = ocp.N
    lb = np.tile(ocp.u_lb, N)
    ub = np.tile(ocp.u_ub, N)
    u = np.zeros(2 * N) if u0 is None else np.clip(np.asarray(u0, float).reshape(-1), lb, ub)
    info = {"iters": 0, "status": "max_iter"}
    for it in range(max_iter):
        J, g, H, X = ss_derivatives(u.reshape(N, 2), P, ocp, pstage)
        g = g.reshape(-1)
        pg = u - np.clip(u - g, lb, ub)
        info["iters"] = it
        info["pg"] = float(np.max(np.abs(pg)))
        if info["pg"] <= tol:
            info["status"] = "converged"
            break
        eps = min(1e-3, info["pg"])
        act = ((u <= lb + eps) & (g > 0)) | ((u >= ub - eps) & (g < 0))
        fr = ~act
        d = np.zeros_like(u)
        if fr.any():
            Hf = H[np.ix_(fr, fr)]
            ev, V = np.linalg.eigh(Hf)
            floor = max(1e-10, 1e-12 * np.max(np.abs(ev)))
            ev = np.maximum(np.abs(ev), floor)
            d[fr] = -(V @ ((V.T @ g[fr]) / ev))
        if act.any():
            dg = np.maximum(np.abs(np.diag(H)[act]), 1e-6)
            d[act] = -g[act] / dg
        alpha = 1.0
        accepted = False
        for _ in range(60):
            un = np.clip(u + alpha * d, lb, ub)
            _, Jn = ss_rollout(un.reshape(N, 2), P, ocp, pstage)
            dec = -alpha * np.dot(g[fr], d[fr]) + np.dot(g[act], (u - un)[act])
            if J - Jn >= 1e-4 * dec or abs(J - Jn) <= 1e-15 * max(1.0, abs(J)) and dec <= 1e-15:
                accepted = True
                break
            alpha *= 0.5
        if not accepted:
            info["status"] = "line_search_failed"
            break
        u = un
    U = u.reshape(N, 2)
    X, J = ss_rollout(U, P, ocp, pstage)
    info["J"] = float(J)
    return U, X, info


def solve_ms(P, ocp: UnicycleOCP, u0=None, pstage=None, **kw):
    """Multiple-shooting optimum w* (interleaved) obtained from the single-shooting solve."""
    U, X, info = solve_single_shooting(P, ocp, u0, pstage, **kw)
    return join_w(X, U), info


# ----------------------------------------------------------------------------
# Closed-loop driver (``Casadi/multiple_shooting_casadi.py:224-298``)
# ----------------------------------------------------------------------------


def closed_loop(ocp: UnicycleOCP, x_init=(0.0, 0.0, 0.0), x_target=(10.0, 10.0, 0.0),
                sim_time=20.0, tol=1e-11):
    """Receding-horizon loop: solve -> apply u0 -> plant = F -> shift warm start.

    Returns dict with states (iters+1, 3), controls (iters, 2), iterations.
    """
    x = np.array(x_init, float)
    xt = np.array(x_target, float)
    states = [x.copy()]
    controls = []
    U_guess = None
    it = 0
    while np.linalg.norm(x - xt) > 1e-1 and it * ocp.T < sim_time:
        P = np.concatenate([x, xt])
        U, X, info = solve_single_shooting(P, ocp, U_guess, tol=tol)
        u0 = U[0].copy()
        controls.append(u0)
        x, _ = F(x, u0, xt, ocp)
        states.append(x.copy())
        U_guess = np.vstack([U[1:], U[-1:]])
        it += 1
    return {"states": np.array(states), "controls": np.array(controls), "iterations": it}


# ----------------------------------------------------------------------------
# Golden fixture helpers
# ----------------------------------------------------------------------------


def golden_pairs(rows):
    """84 (P_j, u0*_j) pairs from the exported rows (see tests/golden/make_golden.py)."""
    rows = np.asarray(rows, float)
    n = rows.shape[0] - 1
    P = np.zeros((n, 6))
    P[:, 0:3] = rows[1:, 0:3]
    P[:, 3:6] = (10.0, 10.0, 0.0)
    U0 = rows[:n, 3:5]
    return P, U0


def kkt_residual_ms(w, lam_g, P, ocp, pstage=None):
    """inf-norm of the multiple-shooting Lagrangian gradient projected on the bounds."""
    N = ocp.N
    lb, ub = ms_bounds(ocp)
    # gradient of J + lam^T g by complex step over w (small n_w)
    n = n_w(N)
    wc = np.asarray(w, complex)[None, :] + 1j * _CS_H * np.eye(n)
    J, g = ms_functions(wc, P, ocp, pstage)
    L = J + g @ np.asarray(lam_g)
    grad = L.imag / _CS_H
    pg = w - np.clip(w - grad, lb, ub)
    _, gval = ms_functions(np.asarray(w), P, ocp, pstage)
    return float(np.max(np.abs(pg))), float(np.max(np.abs(gval)))


def box_qp(H, g0, lb, ub, tol=1e-12, max_iter=500):
    """min 1/2 u^T H u + g0^T u  s.t.  lb <= u <= ub, H symmetric positive definite.

    Primal active-set method (Nocedal & Wright 2006, Alg. 16.3) on simple bounds: finite
    termination for strictly convex QPs; the returned point is checked against the KKT
    conditions (raises if they do not hold)."""
    n = len(g0)
    lb = np.asarray(lb, float)
    ub = np.asarray(ub, float)
    u = np.clip(np.linalg.solve(H, -g0), lb, ub)
    W = {}  # index -> -1 (at lb) / +1 (at ub)
    for i in range(n):
        if u[i] <= lb[i]:
            W[i] = -1
        elif u[i] >= ub[i]:
            W[i] = 1
    full = False  # the last step was a full Newton step on the current working set
    for _ in range(max_iter):
        g = H @ u + g0
        fr = np.array([i not in W for i in range(n)])
        p = np.zeros(n)
        if fr.any() and not full:
            p[fr] = np.linalg.solve(H[np.ix_(fr, fr)], -g[fr])
        # after a full step the equality-constrained subproblem is solved (what a new step
        # would add is rounding noise, which matters on badly scaled condensed Hessians)
        if full or np.max(np.abs(p)) <= tol * max(1.0, np.max(np.abs(u))):
            full = False
            # multipliers of the working bounds: g_i >= 0 at lb, g_i <= 0 at ub
            mult = {i: (g[i] if side < 0 else -g[i]) for i, side in W.items()}
            if not mult or min(mult.values()) >= -tol * max(1.0, np.max(np.abs(g))):
                break
            W.pop(min(mult, key=mult.get))
            continue
        alpha, block = 1.0, None
        for i in np.flatnonzero(fr):
            if p[i] < 0 and lb[i] > -np.inf:
                a = (lb[i] - u[i]) / p[i]
                if a < alpha:
                    alpha, block = a, (i, -1)
            elif p[i] > 0 and ub[i] < np.inf:
                a = (ub[i] - u[i]) / p[i]
                if a < alpha:
                    alpha, block = a, (i, 1)
        u = u + alpha * p
        full = block is None
        if block is not None:
            i, side = block
            u[i] = lb[i] if side < 0 else ub[i]
            W[i] = side
    else:
        raise RuntimeError("box_qp: no convergence")
    g = H @ u + g0
    scale = max(1.0, np.max(np.abs(g0)), np.max(np.abs(H)) * max(1.0, np.max(np.abs(u))))
    kkt = np.where(u <= lb, np.minimum(g, 0.0), np.where(u >= ub, np.maximum(g, 0.0), g))
    if np.max(np.abs(kkt)) > 1e-9 * scale:
        raise RuntimeError(f"box_qp: KKT residual {np.max(np.abs(kkt)):.3e}")
    return u


# ----------------------------------------------------------------------------
# LTI cart-pole QP with move blocking (config 5 family)
# Inverted_pendulum/inverted_pendulum_single_shooting_mpctools.py:15-78
# ----------------------------------------------------------------------------


def pendulum_model(T=0.01):
    """Ac = M^T (:19-20), Bc (:22), zero-order-hold c2d (mpctools util.c2d, :24)."""
    from scipy.linalg import expm

    Ac = np.array([[0, 0, 0, 0], [1, -10, 0, -20], [0, 9.81, 0, 39.24], [0, 0, 1, 0]], float).T
    Bc = np.array([[0.0], [1.0], [0.0], [2.0]])
    Mx = np.zeros((5, 5))
    Mx[:4, :4] = Ac
    Mx[:4, 4:] = Bc
    E = expm(Mx * T)
    return E[:4, :4], E[:4, 4:]


def pendulum_qp_solve(x0, A, Bd, N=50, n_free=5, uprev=0.0, umax=200.0, xt=(10.0, 0, 0, 0), q1=1.2, q3=1.0,
                      r=0.01, tol=1e-12):
    """The per-step QP of :34-64 condensed onto the n_free free moves (u_k = u_{n_free-1}
    for k >= n_free, Du = 0 there, :32-42): min sum_{k<N} (q1(x1-xt1))^2 + (q3 x3)^2 + (r Du_k)^2
    with |u| <= umax, Du_0 = u_0 - uprev.  Exact active-set solve (convex QP).
    Returns u (n_free,)."""
    x0 = np.asarray(x0, float)
    # x_k = A^k x0 + S_k u over the free moves u; u_k = E_k u (E_k selects move min(k, n_free-1))
    nx = 4
    E = np.zeros((N, n_free))
    for k in range(N):
        E[k, min(k, n_free - 1)] = 1.0
    Sx = np.zeros((N, nx, n_free))
    fx = np.zeros((N, nx))
    x = x0.copy()
    S = np.zeros((nx, n_free))
    for k in range(N):
        fx[k] = x
        Sx[k] = S
        x = A @ x
        S = A @ S + np.outer(Bd[:, 0], E[k])
    # cost terms: rows of residual vector r(u) = R u + c
    rows, cs = [], []
    for k in range(N):
        rows.append(q1 * Sx[k, 0]); cs.append(q1 * (fx[k, 0] - xt[0]))
        rows.append(q3 * Sx[k, 2]); cs.append(q3 * fx[k, 2])
        d = E[k] - (E[k - 1] if k > 0 else 0 * E[0])
        rows.append(r * d); cs.append(-r * uprev if k == 0 else 0.0)
    Rm = np.array(rows)
    c = np.array(cs)
    H = 2 * Rm.T @ Rm
    g0 = 2 * Rm.T @ c
    return box_qp(H, g0, -umax * np.ones(n_free), umax * np.ones(n_free), tol=tol)


def pendulum_closed_loop(nsim=1000, T=0.01, N=50):
    """:66-78 -- x0 = 0; each step solve, apply u_0, x <- A x + B u (uprev stays 0 as in the script)."""
    A, Bd = pendulum_model(T)
    x = np.zeros(4)
    xs = [x.copy()]
    us = []
    for _ in range(nsim):
        u = pendulum_qp_solve(x, A, Bd, N=N)[0]
        us.append(u)
        x = A @ x + Bd[:, 0] * u
        xs.append(x.copy())
    return np.array(xs), np.array(us)


def lq_solve(x0, A, B, c, W, tab, zr, lbu, ubu, x_lb=None, x_ub=None, tol=1e-13):
    """Generic table-driven linear-quadratic OCP (the model of mpcx MPCX_MODEL_LINEAR):
    x_{k+1} = A_j x_k + B_j u_k + c_j, J = sum_k (z_k - zr_k)^T W_j (z_k - zr_k), j = tab[k],
    lbu <= u_k <= ubu, condensed onto U and solved exactly by a primal active-set method.
    State bounds are not supported here (use x_lb/x_ub = None).  Returns (X (N+1,nx), U (N,nu), J)."""
    x0 = np.asarray(x0, float)
    N = len(tab)
    nx, nu = A.shape[-1], B.shape[-1]
    nz = nx + nu
    nU = N * nu
    # x_k = fx[k] + Sx[k] U
    fx = np.zeros((N + 1, nx))
    Sx = np.zeros((N + 1, nx, nU))
    fx[0] = x0
    for k in range(N):
        j = tab[k]
        fx[k + 1] = A[j] @ fx[k] + c[j]
        Sx[k + 1] = A[j] @ Sx[k]
        Sx[k + 1][:, k * nu:(k + 1) * nu] += B[j]
    H = np.zeros((nU, nU))
    g0 = np.zeros(nU)
    const = 0.0
    for k in range(N):
        j = tab[k]
        Sz = np.zeros((nz, nU))
        Sz[:nx] = Sx[k]
        Sz[nx:, k * nu:(k + 1) * nu] = np.eye(nu)
        fz = np.concatenate([fx[k], np.zeros(nu)]) - zr[k]
        H += 2 * Sz.T @ W[j] @ Sz
        g0 += 2 * Sz.T @ W[j] @ fz
        const += fz @ W[j] @ fz
    lb = np.tile(np.asarray(lbu, float), N)
    ub = np.tile(np.asarray(ubu, float), N)
    u = box_qp(H, g0, lb, ub, tol=tol)
    X = fx + np.einsum("kij,j->ki", Sx, u)
    J = 0.5 * u @ H @ u + g0 @ u + const
    return X, u.reshape(N, nu), J


# ----------------------------------------------------------------------------
# mpctools point-to-point variant (mpctools/multiple_shooting_mpctools.py -> Casadi/3exemplo.xlsx)
# ----------------------------------------------------------------------------


def lateral_error_solve(x0, A, Bd, par_t, q=(10.0, 1.0, 0.0), r=0.01, delta_max=0.3491):
    """The per-step QP of ``Trajectory Tracking/Trajectory_tracking_le_LTI.py:17-79`` with its
    settings Ntu = 1 (one free move: u_k = u_0 for every k, :64-67) and R_du = 0 (:28): a scalar
    QP in u_0, J(u) = sum_{k<Nt} (x_k - p_k[:3])^T Q (x_k - p_k[:3]) + R (u - p_k[3])^2 with
    x_{k+1} = A x_k + B u (:48-61), minimised in closed form and clamped to |u| <= delta_max
    (:69-73).  Written independently of the augmented-state tables of mpcx.lti.  Returns
    (u_0, x_1)."""
    x0 = np.asarray(x0, float)
    Q = np.diag(np.asarray(q, float))
    b = np.asarray(Bd, float).reshape(-1)
    h2 = h1 = 0.0
    fx, sx = x0.copy(), np.zeros_like(x0)  # x_k = fx + sx u
    for k in range(len(par_t)):
        e = fx - par_t[k][:3]
        h2 += sx @ Q @ sx + r
        h1 += sx @ Q @ e - r * par_t[k][3]
        fx, sx = A @ fx, A @ sx + b
    u = float(np.clip(-h1 / h2, -delta_max, delta_max))
    return u, A @ x0 + b * u


def mpctools_point_to_point_ocp(N=10):
    """``mpctools/multiple_shooting_mpctools.py:9-70``: RK4 M=1 model (:51), node cost
    l = (x - goal)^T Q (x - goal) + u^T u (:57-58: R = I, the script's R is unused)."""
    return UnicycleOCP(N=N, T=0.2, M=1, Q=(1.0, 5.0, 0.1), R=(1.0, 1.0), cost="node")


def unicycle_flow(x, u, T):
    """Exact flow of the unicycle ODE over T with constant (v, w) -- what the script's
    plant ``mpc.DiscreteSimulator(ode, Delta)`` (:48, an ODE integrator) computes."""
    x = np.asarray(x, float)
    v, w = float(u[0]), float(u[1])
    th = x[2]
    if abs(w) < 1e-12:
        return np.array([x[0] + v * T * np.cos(th), x[1] + v * T * np.sin(th), th])
    return np.array([x[0] + v / w * (np.sin(th + w * T) - np.sin(th)),
                     x[1] - v / w * (np.cos(th + w * T) - np.cos(th)), th + w * T])


def mpctools_closed_loop(solve_u0_x1, nsim=150, T=0.2, goal=(10.0, 10.0, 0.0)):
    """``:74-104``: stop when the simulated state is within 0.1 of the goal; each solve
    starts from the model's own prediction X_1 of the previous solve (``fixvar("x", 0,
    var["x", 1])``, :94), the logged state is the plant's.  solve_u0_x1(x0) -> (u0, X1).
    Returns (x (t, 3) logged states, u (t, 2))."""
    goal = np.asarray(goal)
    x_sim = [np.zeros(3)]
    x_solver = np.zeros(3)
    us = []
    for t in range(nsim):
        if np.linalg.norm(x_sim[t] - goal) < 1e-1:
            break
        u0, x1 = solve_u0_x1(x_solver)
        us.append(u0)
        x_solver = x1
        x_sim.append(unicycle_flow(x_sim[t], u0, T))
    n = len(us)
    return np.array(x_sim[:n]), np.array(us)
