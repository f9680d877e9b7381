"""CPU oracle for the nonlinear ODE model variants (kinematic bicycle, 6-state dynamic bicycle,
cart-pole) -- TEST INFRASTRUCTURE ONLY (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).

PARITY UNPINNED: the reference holds no model or output for these variants (SURVEY.md §0, §7
item 6); they are BASELINE-named extensions.  This module restates the same NLP independently of
the kernel (numpy, written from the equations in ``mpcx/ode.py``'s docstring):

* dynamics f(x, u) per model, RK4 with M substeps (as ``Casadi/multiple_shooting_casadi.py:98-114``
  with the node cost of ``Trajectory Tracking/Trajectory_tracking.py:57-61``);
* Jacobians by complex-step differentiation (exact to rounding), Hessians of lam^T F by central
  differences of those (affect only the Newton rate, never the fixed point);
* the reduced single-shooting problem min_U J(U), lb <= U <= ub, solved by projected Newton
  (state bounds are not modelled: tests keep them inactive);
* the KKT residual of a multiple-shooting primal-dual point (CasADi sign convention
  grad f + J_g^T lam_g + lam_x = 0), for nonconvex cases where local optima may differ.
"""
from __future__ import annotations

import numpy as np

NXU = {"kin_bicycle": (3, 2), "dyn_bicycle": (6, 2), "cartpole": (4, 1)}


def f_kin_bicycle(x, u, par):
    X, Y, psi = x[..., 0], x[..., 1], x[..., 2]
    v, d = u[..., 0], u[..., 1]
    return np.stack([v * np.cos(psi), v * np.sin(psi), v * np.tan(d) / par[0]], axis=-1)


def f_dyn_bicycle(x, u, par):
    m, a, b, Ca, Jz = par[:5]
    psi, vx, vy, r = x[..., 2], x[..., 3], x[..., 4], x[..., 5]
    d, ax = u[..., 0], u[..., 1]
    alpha_f = d - (vy + a * r) / vx
    alpha_r = -(vy - b * r) / vx
    Fyf, Fyr = 2 * Ca * alpha_f, 2 * Ca * alpha_r
    return np.stack([vx * np.cos(psi) - vy * np.sin(psi),
                     vx * np.sin(psi) + vy * np.cos(psi),
                     r,
                     ax + r * vy - Fyf * np.sin(d) / m,
                     (Fyf * np.cos(d) + Fyr) / m - vx * r,
                     (a * Fyf * np.cos(d) - b * Fyr) / Jz], axis=-1)


def f_cartpole(x, u, par):
    Mc, m, L, g, c = par[:5]
    pd, phi, phid = x[..., 1], x[..., 2], x[..., 3]
    F = u[..., 0]
    s, co = np.sin(phi), np.cos(phi)
    pdd = (F - c * pd - m * L * phid ** 2 * s + m * g * s * co) / (Mc + m * s ** 2)
    return np.stack([pd, pdd, phid, (g * s + co * pdd) / L], axis=-1)


FUNCS = {"kin_bicycle": f_kin_bicycle, "dyn_bicycle": f_dyn_bicycle, "cartpole": f_cartpole}


class Problem:
    """The NLP of an ``mpcx.ode.OdeOCP`` (duck-typed: model, N, T, M, Q, R, u_lb, u_ub, par, param)."""

    def __init__(self, ocp):
        self.model = ocp.model
        self.nx, self.nu = NXU[ocp.model]
        self.nz = self.nx + self.nu
        self.N, self.T, self.M = int(ocp.N), float(ocp.T), int(ocp.M)
        self.W = np.array(list(ocp.Q) + list(ocp.R), float)
        self.u_lb, self.u_ub = np.array(ocp.u_lb, float), np.array(ocp.u_ub, float)
        self.par = np.array(ocp.par, float)
        self.param = ocp.param
        self.f = FUNCS[ocp.model]

    def refs(self, P):
        """Stage references zr (N, nz) of one parameter vector."""
        P = np.asarray(P, float)
        nx, nz, N = self.nx, self.nz, self.N
        if self.param == "x0_xref":
            zr = np.zeros((N, nz))
            zr[:, :nx] = P[nx:2 * nx]
            return zr
        return P[nx:].reshape(N, nz)

    def F(self, x, u):
        """RK4, M substeps (complex-safe)."""
        h = self.T / self.M
        for _ in range(self.M):
            k1 = self.f(x, u, self.par)
            k2 = self.f(x + 0.5 * h * k1, u, self.par)
            k3 = self.f(x + 0.5 * h * k2, u, self.par)
            k4 = self.f(x + h * k3, u, self.par)
            x = x + (h / 6.0) * (k1 + 2 * k2 + 2 * k3 + k4)
        return x

    def l(self, z, zr):
        d = z - zr
        return np.sum(self.W * d * d, axis=-1)

    def jac(self, z):
        """dF/dz (..., nx, nz) by complex step."""
        nx, nz = self.nx, self.nz
        hstep = 1e-30
        zc = z[..., None, :] + 1j * hstep * np.eye(nz)  # (..., nz dirs, nz)
        Fc = self.F(zc[..., :nx], zc[..., nx:])          # (..., nz dirs, nx)
        return np.swapaxes(Fc.imag / hstep, -1, -2)

    def hess_lam(self, z, lam, delta=1e-5):
        """d2 (lam^T F)/dz2 (..., nz, nz): central differences of complex-step gradients."""
        nz = self.nz
        H = np.zeros(z.shape[:-1] + (nz, nz))
        for i in range(nz):
            e = np.zeros(nz)
            e[i] = delta
            gp = np.einsum("...c,...cj->...j", lam, self.jac(z + e))
            gm = np.einsum("...c,...cj->...j", lam, self.jac(z - e))
            H[..., i, :] = (gp - gm) / (2 * delta)
        return 0.5 * (H + np.swapaxes(H, -1, -2))

    # ------------------------------------------------------------------ single shooting
    def rollout(self, U, x0):
        X = [np.asarray(x0, float)]
        for k in range(self.N):
            X.append(self.F(X[-1], U[k]))
        return np.array(X)

    def cost(self, U, P):
        X = self.rollout(U, P[:self.nx])
        zr = self.refs(P)
        return float(np.sum(self.l(np.concatenate([X[:-1], U], axis=1), zr))), X

    def derivatives(self, U, P):
        nx, nu, nz, N = self.nx, self.nu, self.nz, self.N
        J, X = self.cost(U, P)
        Z = np.concatenate([X[:-1], U], axis=1)
        zr = self.refs(P)
        Jac = self.jac(Z)  # (N, nx, nz)
        A, Bm = Jac[:, :, :nx], Jac[:, :, nx:]
        gl = 2 * self.W * (Z - zr)
        lam = np.zeros((N + 1, nx))
        g = np.zeros((N, nu))
        for k in range(N - 1, -1, -1):
            g[k] = gl[k, nx:] + Bm[k].T @ lam[k + 1]
            lam[k] = gl[k, :nx] + A[k].T @ lam[k + 1]
        Hs = self.hess_lam(Z, lam[1:]) + np.diag(2 * self.W)
        H = np.zeros((nu * N, nu * N))
        S = np.zeros((nx, nu * N))
        for k in range(N):
            E = np.zeros((nu, nu * N))
            E[:, nu * k:nu * (k + 1)] = np.eye(nu)
            D = np.vstack([S, E])
            H += D.T @ Hs[k] @ D
            S = A[k] @ S + Bm[k] @ E
        return J, g.reshape(-1), 0.5 * (H + H.T), X

    def solve(self, P, U0=None, tol=1e-10, max_iter=300):
        """Projected Newton on the reduced problem.  Returns (U (N,nu), X (N+1,nx), info)."""
        nu, N = self.nu, self.N
        lb, ub = np.tile(self.u_lb, N), np.tile(self.u_ub, N)
        u = np.zeros(nu * N) if U0 is None else np.clip(np.asarray(U0, float).reshape(-1), lb, ub)
        info = {"status": "max_iter"}
        for it in range(max_iter):
            J, g, H, X = self.derivatives(u.reshape(N, nu), P)
            pg = u - np.clip(u - g, lb, ub)
            info.update(iters=it, pg=float(np.max(np.abs(pg))))
            if info["pg"] <= tol:
                info["status"] = "converged"
                break
            eps = min(1e-3, info["pg"])
            act = ((u <= lb + eps) & (g > 0)) | ((u >= ub - eps) & (g < 0))
            fr = ~act
            d = np.zeros_like(u)
            if fr.any():
                ev, V = np.linalg.eigh(H[np.ix_(fr, fr)])
                ev = np.maximum(np.abs(ev), max(1e-10, 1e-12 * np.max(np.abs(ev))))
                d[fr] = -(V @ ((V.T @ g[fr]) / ev))
            if act.any():
                d[act] = -g[act] / np.maximum(np.abs(np.diag(H)[act]), 1e-6)
            alpha, ok = 1.0, False
            for _ in range(60):
                un = np.clip(u + alpha * d, lb, ub)
                Jn, _ = self.cost(un.reshape(N, nu), P)
                dec = -alpha * np.dot(g[fr], d[fr]) + np.dot(g[act], (u - un)[act])
                if J - Jn >= 1e-4 * dec or (abs(J - Jn) <= 1e-15 * max(1.0, abs(J)) and dec <= 1e-15):
                    ok = True
                    break
                alpha *= 0.5
            if not ok:
                info["status"] = "line_search_failed"
                break
            u = un
            if info["pg"] <= 1e-6 and abs(J - Jn) <= 1e-14 * max(1.0, abs(J)):
                info["status"] = "stalled"  # objective fixed to rounding; pg limited by a near-active bound
                break
        U = u.reshape(N, nu)
        info["J"], X = self.cost(U, P)
        return U, X, info

    # ------------------------------------------------------------------ multiple shooting
    def join_w(self, X, U):
        return np.concatenate([X[0]] + [np.concatenate([U[k], X[k + 1]]) for k in range(self.N)])

    def split_w(self, w):
        nx, nu, nz, N = self.nx, self.nu, self.nz, self.N
        X = np.empty((N + 1, nx))
        U = np.empty((N, nu))
        X[0] = w[:nx]
        for k in range(N):
            U[k] = w[nx + nz * k: nx + nz * k + nu]
            X[k + 1] = w[nx + nz * k + nu: nx + nz * (k + 1)]
        return X, U

    def kkt_residual(self, w, lam_g, lam_x, P):
        """max |grad f + J_g^T lam_g + lam_x| and max |g| at a multiple-shooting point.  Interval 0
        integrates from the parameter x0 (multiple_shooting_casadi.py:125,157): X_0 enters only g_0."""
        nx, nu, nz, N = self.nx, self.nu, self.nz, self.N
        X, U = self.split_w(np.asarray(w, float))
        Xs = X[:-1].copy()
        Xs[0] = np.asarray(P[:nx], float)
        Z = np.concatenate([Xs, U], axis=1)
        zr = self.refs(P)
        Jac = self.jac(Z)
        gl = 2 * self.W * (Z - zr)
        lam_g = np.asarray(lam_g, float).reshape(N + 1, nx)
        r = np.zeros(nx + nz * N)
        ix = lambda k: np.arange(nx) if k == 0 else nx + nz * (k - 1) + nu + np.arange(nx)  # noqa: E731
        r[ix(0)] -= lam_g[0]
        for k in range(N):
            l1 = lam_g[k + 1]
            if k > 0:
                r[ix(k)] += gl[k, :nx] + Jac[k, :, :nx].T @ l1
            r[nx + nz * k: nx + nz * k + nu] += gl[k, nx:] + Jac[k, :, nx:].T @ l1
            r[ix(k + 1)] -= l1
        r += np.asarray(lam_x, float)
        gres = np.concatenate([np.asarray(P[:nx], float) - X[0]] + [self.F(Xs[k], U[k]) - X[k + 1] for k in range(N)])
        return float(np.max(np.abs(r))), float(np.max(np.abs(gres)))
