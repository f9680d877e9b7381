"""CasADi-``nlpsol``-shaped façade over libmpcx (the drop-in for the hot path).

Reference boundary (``Casadi/multiple_shooting_casadi.py``):

    solver = ca.nlpsol('solver', 'ipopt', prob, opts)                       # :197
    sol = solver(x0=w0, lbx=lbw, ubx=ubw, lbg=lbg, ubg=ubg, p=P)           # :235-242
    u = sol['x'][3:5] ...                                                   # :243-256
    state_init = F(args['p'], u[:, 0])[0]                                   # :273

Here:

    solver = mpcx.nlpsol('solver', 'mi355x', ocp, opts)
    sol = solver(x0=w0, lbx=lbw, ubx=ubw, lbg=lbg, ubg=ubg, p=P)
    F = mpcx.integrator(ocp)

``sol`` holds numpy column vectors with CasADi's shapes and sign conventions:
'x' (n_w,1), 'f' (1,1), 'g' (n_g,1), 'lam_g' (n_g,1), 'lam_x' (n_w,1),
'lam_p' (n_p,1; zeros).  ``solver.stats()`` mirrors CasADi's stats dict
('return_status', 'success', 'iter_count', 't_wall_total').  Batched use:
``solver.solve_batch(P, w0)``.  Every call runs the HIP kernel on the GPU.
"""
from __future__ import annotations

import math
import time

import numpy as np

from . import _lib
from .lti import LinearOCP, state_pad
from .ocp import IPOPT_OPTIONS, OCP, to_spec
from .ode import OdeOCP


def _vec(v, n, name, fill=None):
    """CasADi-style input coercion: list / ndarray / DM-like / scalar (broadcast)."""
    if v is None:
        if fill is None:
            return None
        return np.full(n, float(fill))
    a = np.asarray(v, dtype=np.float64).reshape(-1)
    if a.size == 1 and n != 1:
        a = np.full(n, float(a[0]))
    if a.size != n:
        raise ValueError(f"{name}: expected {n} entries, got {a.size}")
    return np.ascontiguousarray(a)


class Solver:
    """Callable returned by :func:`nlpsol`."""

    _pad = None  # lti.StatePad of a linear model embedded in a larger kernel instantiation

    def __init__(self, name: str, ocp: OCP, opts: dict | None = None, device: int = 0):
        opts = dict(opts or {})
        ip = dict(opts.get("ipopt", {}))
        self.name = name
        self.ocp = ocp
        self.max_iter = int(ip.pop("max_iter", 3000))
        self.tol = float(ip.pop("tol", 1e-8))
        # output options have no effect here (no iteration log is printed)
        for k in ("print_level", "sb"):
            ip.pop(k, None)
        # termination options (acceptable_tol / acceptable_obj_change_tol at :192-193), IPOPT's
        # semantics; the rest keep IPOPT's defaults
        term = {k: ip.pop(k) for k in IPOPT_OPTIONS if k in ip}
        if ip:
            raise ValueError(f"unsupported ipopt options: {sorted(ip)}")
        # not CasADi options: lanes per instance (0 = fill idle SIMDs, 1 = narrowest group; same
        # results); restoration (False: a failed line search ends the solve, IPOPT has no such switch)
        self.group_policy = int(opts.get("group_policy", 0))
        self.restoration = bool(opts.get("restoration", True))
        # a linear model without its own kernel instantiation runs embedded in one (lti.StatePad)
        self._pad = state_pad(ocp)
        kocp = self._pad.ocp if self._pad else ocp
        self._h = _lib.Handle(to_spec(kocp, self.max_iter, self.tol, device, group_policy=self.group_policy, ipopt=term,
                                      restoration=self.restoration))
        if ocp.model == "linear":
            self._h.set_linear_model(kocp)
        self._stats = {}

    def set_linear_model(self, lin=None):
        """Re-upload stage tables (LTV: new tables or per-instance schedule for the next step)."""
        if lin is not None:
            if lin.model != "linear" or (lin.nx, lin.nu, lin.N) != (self.ocp.nx, self.ocp.nu, self.ocp.N):
                raise ValueError("set_linear_model: incompatible problem")
            self.ocp = lin
        if self._pad is not None:
            self._pad = state_pad(self.ocp)
        self._h.set_linear_model(self._pad.ocp if self._pad else self.ocp)

    # ---------------------------------------------------------------- layout
    @property
    def n_w(self):
        return self.ocp.N * self.ocp.nu if self.ocp.formulation == "single_shooting" else self._ms_nw

    @property
    def n_g(self):
        return self.ocp.N * self._ss_ng if self.ocp.formulation == "single_shooting" else self._ms_ng

    @property
    def _ms_nw(self):
        """Multiple-shooting layout sizes of the user's problem (the kernel's unless padded)."""
        return self._pad.n_w if self._pad else self._h.n_w

    @property
    def _ms_ng(self):
        return self._pad.n_g if self._pad else self._h.n_g

    @property
    def _ss_ng(self):
        """Single shooting: g entries per node k = 1..N -- (x_k, y_k) for the unicycle
        (``single_shooting_v2.py:115-158``), the whole state for the ODE models."""
        return 2 if self.ocp.model == "unicycle" else self.ocp.nx

    @property
    def n_p(self):
        return self._pad.n_p if self._pad else self._h.n_p

    def stats(self):
        return dict(self._stats)

    # ---------------------------------------------------------------- batched core
    def solve_batch(self, P, w0=None, lbw=None, ubw=None, want_lam=True, want_g=False, lam_g0=None, lam_x0=None):
        """Solve B independent NLPs (multiple-shooting layout).

        P (B, n_p); w0 (B, n_w) or None (cold start X_k = x0, U = 0);
        lam_g0 (B, n_g) / lam_x0 (B, n_w): warm-start multipliers (IPOPT
        warm_start_init_point), or None.
        Returns dict of arrays: w (B,n_w), f (B,), lam_g (B,n_g), lam_x (B,n_w), status (B,), iters (B,),
        g (B,n_g).
        """
        P = np.ascontiguousarray(np.atleast_2d(np.asarray(P, np.float64)))
        B = P.shape[0]
        if P.shape[1] != self.n_p:
            raise ValueError(f"P: expected {self.n_p} columns, got {P.shape[1]}")
        nw, ng = self._ms_nw, self._ms_ng
        w0a = None
        if w0 is not None:
            w0a = np.ascontiguousarray(np.asarray(w0, np.float64).reshape(B, nw))
        lbw = _vec(lbw, nw, "lbw")  # the library reads n_w entries of each
        ubw = _vec(ubw, nw, "ubw")
        l0 = None if lam_g0 is None else np.ascontiguousarray(np.asarray(lam_g0, np.float64).reshape(B, ng))
        lx0 = None if lam_x0 is None else np.ascontiguousarray(np.asarray(lam_x0, np.float64).reshape(B, nw))
        pd = self._pad
        if pd is not None:  # user layout -> the kernel's padded layout (pad states unbounded, 0)
            P = pd.scatter(P, pd.p_idx, pd.n_p_pad)
            w0a = pd.scatter(w0a, pd.w_idx, pd.n_w_pad)
            lbw = None if lbw is None else pd.scatter(lbw[None, :], pd.w_idx, pd.n_w_pad, -1e20)[0]
            ubw = None if ubw is None else pd.scatter(ubw[None, :], pd.w_idx, pd.n_w_pad, 1e20)[0]
            l0 = pd.scatter(l0, pd.g_idx, pd.n_g_pad)
            lx0 = pd.scatter(lx0, pd.w_idx, pd.n_w_pad)
            nw, ng = pd.n_w_pad, pd.n_g_pad
        w = np.empty((B, nw))
        f = np.empty(B)
        lam = np.empty((B, ng)) if want_lam else None
        lamx = np.empty((B, nw)) if want_lam else None
        g = np.empty((B, ng)) if want_g else None
        st = np.empty(B, np.int32)
        it = np.empty(B, np.int32)
        lib = _lib.load()
        t0 = time.perf_counter()
        _lib.check(lib.mpcx_solve_batch(self._h.ptr, B, _lib.dptr(P), _lib.dptr(w0a), _lib.dptr(l0), _lib.dptr(lx0),
                                        _lib.dptr(lbw), _lib.dptr(ubw), _lib.dptr(w), _lib.dptr(f), _lib.dptr(g),
                                        _lib.dptr(lam), _lib.dptr(lamx), _lib.iptr(st), _lib.iptr(it)))
        t = time.perf_counter() - t0
        if pd is not None:
            w, lamx = pd.gather(w, pd.w_idx), pd.gather(lamx, pd.w_idx)
            lam, g = pd.gather(lam, pd.g_idx), pd.gather(g, pd.g_idx)
        return {"w": w, "f": f, "lam_g": lam, "lam_x": lamx, "g": g, "status": st, "iters": it, "t_wall": t}

    def rk4_sens(self, w, P):
        """Per-interval defects, costs and Jacobians at w (B, n_w) -- the sweep kernel."""
        if self.ocp.model != "unicycle":
            raise ValueError("rk4_sens: the sweep kernel evaluates the unicycle model only")
        w = np.ascontiguousarray(np.atleast_2d(np.asarray(w, np.float64)))
        P = np.ascontiguousarray(np.atleast_2d(np.asarray(P, np.float64)))
        B, N = w.shape[0], self.ocp.N
        if w.shape[1] != self._h.n_w or P.shape != (B, self._h.n_p):
            raise ValueError(f"rk4_sens: w (B, {self._h.n_w}) and P (B, {self._h.n_p}) expected")
        c = np.empty((B, N, 3))
        q = np.empty((B, N))
        A = np.empty((B, N, 3, 3))
        Bm = np.empty((B, N, 3, 2))
        gq = np.empty((B, N, 5))
        _lib.check(_lib.load().mpcx_rk4_sens(self._h.ptr, B, _lib.dptr(w), _lib.dptr(P), _lib.dptr(c), _lib.dptr(q),
                                             _lib.dptr(A), _lib.dptr(Bm), _lib.dptr(gq)))
        return {"c": c, "q": q, "A": A, "B": Bm, "gq": gq}

    def lam_x_from_kkt(self, w, P, lam_g):
        """Bound multipliers reconstructed from stationarity, grad f + J^T lam_g + lam_x = 0
        (evaluated with the sweep kernel; used to cross-check the solver's own lam_x).  Interval 0
        integrates from x0 = P[:3] (multiple_shooting_casadi.py:125,157), so X_0 enters only g_0."""
        we = np.array(np.atleast_2d(w), np.float64)
        P2 = np.atleast_2d(np.asarray(P, np.float64))
        we[:, 0:3] = P2[:, 0:3]  # the sweep evaluates interval 0 at (x0, U_0)
        s = self.rk4_sens(we, P2)
        B, N = s["q"].shape
        r = np.zeros((B, self._h.n_w))
        lam_g = np.asarray(lam_g).reshape(B, -1)
        ix = lambda k: np.arange(3) if k == 0 else 3 + 5 * (k - 1) + 2 + np.arange(3)  # noqa: E731
        r[:, 0:3] -= lam_g[:, 0:3]
        for k in range(N):
            l1 = lam_g[:, 3 * (k + 1):3 * (k + 2)]
            if k > 0:
                r[:, ix(k)] += s["gq"][:, k, 0:3] + np.einsum("bij,bi->bj", s["A"][:, k], l1)
            r[:, 3 + 5 * k:5 + 5 * k] += s["gq"][:, k, 3:5] + np.einsum("bij,bi->bj", s["B"][:, k], l1)
            r[:, ix(k + 1)] -= l1
        return -r

    # ---------------------------------------------------------------- CasADi-shaped call
    def __call__(self, x0=None, lbx=None, ubx=None, lbg=None, ubg=None, p=None, lam_x0=None, lam_g0=None):
        if p is None:
            raise ValueError("p is required")
        ocp = self.ocp
        P = _vec(p, self.n_p, "p")[None, :]
        ss = ocp.formulation == "single_shooting"
        lbx = _vec(lbx, self.n_w, "lbx", -math.inf)
        ubx = _vec(ubx, self.n_w, "ubx", math.inf)
        lbg = _vec(lbg, self.n_g, "lbg", 0.0 if not ss else -math.inf)
        ubg = _vec(ubg, self.n_g, "ubg", 0.0 if not ss else math.inf)
        if ss and ocp.model == "linear":
            raise ValueError("single shooting is mapped for the unicycle and ODE models (stage-invariant dynamics)")
        if ss:
            if np.any(np.isfinite(lbg)) or np.any(np.isfinite(ubg)):
                raise ValueError("single shooting: only inactive (+-inf) bounds on g are supported")
        elif np.any(lbg != 0) or np.any(ubg != 0):
            raise ValueError("multiple shooting: g are the shooting equalities, lbg = ubg = 0 required")
        N, nx, nu = ocp.N, ocp.nx, ocp.nu
        nz = nx + nu
        l0 = lx0 = None
        if ss:  # decision = U; bounds on U map onto the U slots of the multiple-shooting w
            lbw = np.full(self._h.n_w, -1e20)
            ubw = np.full(self._h.n_w, 1e20)
            for k in range(N):
                lbw[nx + nz * k:nx + nz * k + nu] = lbx[nu * k:nu * (k + 1)]
                ubw[nx + nz * k:nx + nz * k + nu] = ubx[nu * k:nu * (k + 1)]
            w0 = None
            if x0 is not None:
                U = _vec(x0, nu * N, "x0").reshape(N, nu)
                X = self._rollout(P[0], U)
                w0 = np.concatenate([X[0]] + [np.concatenate([U[k], X[k + 1]]) for k in range(N)])[None, :]
        else:
            lbw, ubw = lbx, ubx
            w0 = None if x0 is None else _vec(x0, self.n_w, "x0")[None, :]
            l0 = None if lam_g0 is None else _vec(lam_g0, self.n_g, "lam_g0")[None, :]
            lx0 = None if lam_x0 is None else _vec(lam_x0, self.n_w, "lam_x0")[None, :]
        lbw = np.where(np.isfinite(lbw), lbw, -1e20)
        ubw = np.where(np.isfinite(ubw), ubw, 1e20)
        r = self.solve_batch(P, w0, np.ascontiguousarray(lbw), np.ascontiguousarray(ubw), want_lam=True,
                             want_g=True, lam_g0=l0, lam_x0=lx0)
        st = int(r["status"][0])
        self._stats = {"return_status": _lib.STATUS.get(st, str(st)), "success": st <= 1,
                       "iter_count": int(r["iters"][0]), "t_wall_total": r["t_wall"], "status_code": st}
        w = r["w"][0]
        lam_x = r["lam_x"][0]
        if ss:
            U = np.stack([w[nx + nz * k:nx + nz * k + nu] for k in range(N)]).reshape(-1)
            Xs = np.stack([w[nx + nz * k + nu:nx + nz * (k + 1)] for k in range(N)])
            g = Xs[:, 0:self._ss_ng].reshape(-1)
            lx = np.concatenate([lam_x[nx + nz * k:nx + nz * k + nu] for k in range(N)])
            return {"x": U[:, None], "f": np.array([[r["f"][0]]]), "g": g[:, None],
                    "lam_g": np.zeros((self.n_g, 1)), "lam_x": lx[:, None], "lam_p": np.zeros((self.n_p, 1))}
        return {"x": w[:, None], "f": np.array([[r["f"][0]]]), "g": r["g"][0][:, None],
                "lam_g": r["lam_g"][0][:, None], "lam_x": lam_x[:, None], "lam_p": np.zeros((self.n_p, 1))}

    def _rollout(self, P, U):
        """X_{k+1} = F(X_k, U_k) on the plant kernel, stage k's references in the stage-0 slot."""
        N, nx, nz = self.ocp.N, self.ocp.nx, self.ocp.nx + self.ocp.nu
        X = [np.asarray(P[0:nx], float)]
        F = Integrator(self.ocp, handle=self._h)
        for k in range(N):
            p = np.array(P, float).copy()
            p[0:nx] = X[-1]
            if self.ocp.param == "x0_stageref":
                p[nx:nx + nz] = P[nx + nz * k:nx + nz * (k + 1)]
            X.append(F(p, U[k])[0].reshape(-1))
        return np.array(X)


class Integrator:
    """``F = ca.Function('F', [P, U], [X, Q], ['x0','p'], ['xf','qf'])`` (:114).

    For a LinearOCP this is stage 0's map x+ = A_j x + B_j u + c_j, q = l_0 (the
    reference's discrete ``f``, e.g. ``inverted_pendulum...py:24-28``).

    ``F(p, u)`` -> [xf (3,1), qf (1,1)];  ``F(x0=p, p=u)`` -> {'xf', 'qf'};
    ``F.batch(P, U)`` -> (xf (B,3), qf (B,)).  Evaluated by the plant kernel.
    """

    def __init__(self, ocp: OCP, device: int = 0, handle=None):
        self.ocp = ocp
        self._pad = state_pad(ocp)
        kocp = self._pad.ocp if self._pad else ocp
        self._h = handle if handle is not None else _lib.Handle(to_spec(kocp, device=device))
        if handle is None and ocp.model == "linear":
            self._h.set_linear_model(kocp)

    @property
    def n_p(self):
        return self._pad.n_p if self._pad else self._h.n_p

    def batch(self, P, U):
        P = np.ascontiguousarray(np.atleast_2d(np.asarray(P, np.float64)))
        U = np.ascontiguousarray(np.atleast_2d(np.asarray(U, np.float64)))
        B = P.shape[0]
        nx, nu = self.ocp.nx, self.ocp.nu
        if P.shape[1] != self.n_p:
            raise ValueError(f"P must be (B, {self.n_p})")
        if U.shape != (B, nu):
            raise ValueError(f"U must be (B, {nu})")
        pd = self._pad
        if pd is not None:
            P = pd.scatter(P, pd.p_idx, pd.n_p_pad)
        xf = np.empty((B, pd.nxp if pd else nx))
        qf = np.empty(B)
        _lib.check(_lib.load().mpcx_plant_step(self._h.ptr, B, _lib.dptr(P), _lib.dptr(U), _lib.dptr(xf),
                                               _lib.dptr(qf)))
        return np.ascontiguousarray(xf[:, :nx]), qf

    def __call__(self, *args, **kw):
        if kw:
            p = kw.get("x0")
            u = kw.get("p")
            xf, qf = self.batch(_vec(p, self.n_p, "x0")[None, :], _vec(u, self.ocp.nu, "p")[None, :])
            return {"xf": xf[0][:, None], "qf": qf[:, None]}
        p, u = args
        xf, qf = self.batch(_vec(p, self.n_p, "p")[None, :], _vec(u, self.ocp.nu, "u")[None, :])
        return [xf[0][:, None], qf[:, None]]


def nlpsol(name: str, plugin: str, prob: OCP, opts: dict | None = None, device: int = 0) -> Solver:
    """Create a solver (``ca.nlpsol`` signature).  plugin must be 'mi355x'."""
    if plugin not in ("mi355x",):
        raise ValueError(f"unknown plugin {plugin!r} (available: 'mi355x')")
    if not isinstance(prob, (OCP, LinearOCP, OdeOCP)):
        raise TypeError("prob must be an mpcx.OCP, LinearOCP or OdeOCP (symbolic CasADi problems are not supported)")
    return Solver(name, prob, opts, device)


def integrator(ocp: OCP, device: int = 0) -> Integrator:
    return Integrator(ocp, device)
