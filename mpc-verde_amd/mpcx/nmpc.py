"""mpctools-shaped façade (``mpc.nmpc`` -> ControlSolver, ``mpc.callSolver``) over libmpcx.

The reference drives its tracking and cart-pole studies through mpctools' object API
(``Trajectory Tracking/Trajectory_tracking.py:72,100-126``,
``Inverted_pendulum/inverted_pendulum_single_shooting_mpctools.py:64-78``)::

    solver = mpc.nmpc(f=..., N=N, l=l, x0=x0, lb=lb, ub=ub, p=p, ...)     # :72 / :64
    for t in range(Nsim):
        for k in range(Nt): solver.par["p", k] = par[:, k, t]             # :105-106
        solver.solve()                                                      # :107
        print(solver.stats["status"])                                       # :110
        solver.saveguess()                                                  # :111
        solver.fixvar("x", 0, solver.var["x", 1])                           # :112
        u[t, :] = np.array(solver.var["u", 0, :]).flatten()                 # :114
        pred += [solver.var["x", :, :]]                                     # :117

    solver.fixvar("x", 0, x0); sol = mpc.callSolver(solver)                # pendulum :73-74
    xcl[:, k] = sol["x"][0, :]; ucl[:, k] = sol["u"][0, :]                 # :76-77

Here the model and cost are an mpcx problem (the functions the reference builds with
``mpc.getCasadiFunc`` are compiled into the HIP kernels), and the rest of the
calls keep mpctools' names and meaning:

    solver = mpcx.nmpc(mpcx.unicycle_tracking(N=10), x0=x0, p=p)
    solver = mpcx.nmpc(mpcx.inverted_pendulum_qp(N=50), x0=x0, uprev=[0.0])

* ``par["p", k]`` -- stage k's parameter row (tracking: the stage reference (x_ref, u_ref));
  ``par["uprev"]`` -- the previous input of a move-blocked QP (fixed at the constructor's
  ``uprev`` unless set, as in the pendulum script);
* ``fixvar("x", 0, val)`` -- the initial state of the next solves;
* ``solve()`` -- one solve on the GPU (the nlpsol batched path with B = 1), from the saved guess
  if there is one (primal only: CasADi hands IPOPT the guess, multipliers start at IPOPT's
  defaults);
* ``saveguess(toffset=1)`` -- the solution shifted by ``toffset`` intervals (last entries
  repeated) becomes the next guess;
* ``var["x", k]`` / ``var["u", k]`` (column vectors), ``var["x", :, :]`` (list over time),
  ``stats["status"]`` (IPOPT's return status string), ``stats["iter_count"]``;
* ``callSolver(solver)`` -> ``{"x": (N+1, nx), "u": (N, nu), "t", "status", "obj"}``.

For the move-blocked QP (``lti.inverted_pendulum_qp``: kernel state (x, u_prev), the blocked
stages' input held by the u_prev state) ``var["x", k]`` is the plant state and ``var["u", k]``
the applied input -- the decision of a free stage, the held input of a blocked one -- as
mpctools reports them for its ``Du = 0`` constraints.
"""
from __future__ import annotations

import numpy as np

from . import _lib
from .lti import LinearOCP
from .nlpsol import nlpsol


def _col(v):
    return np.asarray(v, float).reshape(-1, 1)


class _Struct:
    """Indexable view: ``s[name, t]``, ``s[name, t, :]``, ``s[name, :]``, ``s[name, :, :]``."""

    def __init__(self, get, set_=None):
        self._get, self._set = get, set_

    def __getitem__(self, key):
        if isinstance(key, str):
            key = (key,)
        name, t = key[0], (key[1] if len(key) > 1 else slice(None))
        if len(key) > 2 and key[2] != slice(None):
            raise IndexError("only the full component slice ':' is supported as the third index")
        seq = self._get(name)
        if isinstance(t, slice):
            return [_col(v) for v in seq[t]]
        return _col(seq[t])

    def __setitem__(self, key, value):
        if self._set is None:
            raise TypeError("read-only")
        if isinstance(key, str):
            key = (key,)
        self._set(key[0], key[1] if len(key) > 1 else None, value)


class ControlSolver:
    """mpctools' ``ControlSolver`` surface for an mpcx problem (see the module docstring)."""

    def __init__(self, ocp, x0=None, p=None, uprev=None, opts=None, device=0):
        self.ocp = ocp
        self._lin_blocked = isinstance(ocp, LinearOCP) and ocp.nx == 5 and ocp.nu == 1 and hasattr(ocp, "A_plant")
        if ocp.param != "x0_stageref" and not self._lin_blocked:
            raise ValueError("nmpc supports only problems with param 'x0_stageref' (per-stage parameters) or the "
                             f"move-blocked QP of lti.inverted_pendulum_qp (got param={ocp.param!r})")
        self._solver = nlpsol("nmpc", "mi355x", ocp, opts or {}, device=device)
        N = ocp.N
        self._nxu = (4, 1) if self._lin_blocked else (ocp.nx, ocp.nu)
        nx, nu = self._nxu
        self.N = {"x": nx, "u": nu, "t": N}
        self._x0 = np.zeros(nx) if x0 is None else np.asarray(x0, float).reshape(nx)
        if self._lin_blocked:
            self._uprev = 0.0 if uprev is None else float(np.asarray(uprev, float).reshape(-1)[0])
            self._p = None
        else:
            nzr = ocp.nx + ocp.nu
            self.N["p"] = nzr
            self._p = np.zeros((N, nzr)) if p is None else np.array(np.asarray(p, float).reshape(N, nzr))
        self._w = None      # last solution (the solver's multiple-shooting layout)
        self._guess = None  # primal guess of the next solve
        self._f = np.nan
        self.stats = {}
        self.par = _Struct(self._get_par, self._set_par)
        self.var = _Struct(self._get_var)

    # ---------------------------------------------------------------- parameters
    def _get_par(self, name):
        if name == "p" and self._p is not None:
            return list(self._p)
        if name == "uprev" and self._lin_blocked:
            return [np.array([self._uprev])]
        raise KeyError(name)

    def _set_par(self, name, t, value):
        if name == "p" and self._p is not None:
            if t is None or isinstance(t, slice):
                self._p[t if t is not None else slice(None)] = np.asarray(value, float).reshape(-1, self._p.shape[1])
            else:
                self._p[t] = np.asarray(value, float).reshape(-1)
        elif name == "uprev" and self._lin_blocked:
            self._uprev = float(np.asarray(value, float).reshape(-1)[0])
        else:
            raise KeyError(name)

    def fixvar(self, name, t, val, index=None):
        """Fix a variable for the next solves; the reference fixes the initial state only."""
        if name != "x" or t != 0 or index is not None:
            raise ValueError("fixvar: only fixvar('x', 0, value) (the initial state) is supported")
        self._x0 = np.asarray(val, float).reshape(self._nxu[0])

    # ---------------------------------------------------------------- solve
    def _params(self):
        if self._lin_blocked:
            from .lti import pendulum_params
            return pendulum_params(self.ocp, self._x0[None, :], self._uprev)
        return np.concatenate([self._x0, self._p.reshape(-1)])[None, :]

    def solve(self):
        r = self._solver.solve_batch(self._params(), w0=self._guess, want_lam=False)
        st = int(r["status"][0])
        self._w = r["w"][0]
        self._f = float(r["f"][0])
        self.stats = {"status": _lib.STATUS.get(st, str(st)), "success": st <= 1, "iter_count": int(r["iters"][0]),
                      "t_wall_total": r["t_wall"], "status_code": st}

    def saveguess(self, toffset=1, default=None):
        """The current solution shifted by toffset intervals (the last entries repeated) is the
        next solve's primal guess."""
        if self._w is None:
            return
        ocp = self.ocp
        nx, nu, N = ocp.nx, ocp.nu, ocp.N
        nz = nx + nu
        w = self._w
        X = np.stack([w[0:nx]] + [w[nx + nz * k + nu:nx + nz * (k + 1)] for k in range(N)])
        U = np.stack([w[nx + nz * k:nx + nz * k + nu] for k in range(N)])
        s = int(toffset)
        Xs = np.concatenate([X[s:], np.repeat(X[-1:], s, axis=0)])[:N + 1]
        Us = np.concatenate([U[s:], np.repeat(U[-1:], s, axis=0)])[:N]
        self._guess = np.concatenate([Xs[0]] + [np.concatenate([Us[k], Xs[k + 1]]) for k in range(N)])[None, :]

    # ---------------------------------------------------------------- solution
    def _traj(self):
        ocp = self.ocp
        nx, nu, N = ocp.nx, ocp.nu, ocp.N
        nz = nx + nu
        w = self._w
        X = np.stack([w[0:nx]] + [w[nx + nz * k + nu:nx + nz * (k + 1)] for k in range(N)])
        U = np.stack([w[nx + nz * k:nx + nz * k + nu] for k in range(N)])
        if self._lin_blocked:  # plant state and applied input (held by u_prev on blocked stages)
            free = np.asarray(ocp.tab).reshape(-1) == 0
            Ua = np.where(free[:, None], U, X[:N, 4:5])
            return X[:, 0:4], Ua
        return X, U

    def _get_var(self, name):
        if self._w is None:
            raise RuntimeError("no solution yet (call solve())")
        X, U = self._traj()
        if name == "x":
            return list(X)
        if name == "u":
            return list(U)
        raise KeyError(name)


def nmpc(ocp, x0=None, p=None, uprev=None, verbosity=0, isQP=False, opts=None, device=0, **unused) -> ControlSolver:
    """``mpc.nmpc`` with an mpcx problem in place of (f, l, N, lb, ub, funcargs): the dynamics, stage
    cost and bounds live in ``ocp``.  ``verbosity`` and ``isQP`` are accepted for the call's shape
    (IPOPT's log is never printed; a linear-quadratic problem is solved by the same kernel)."""
    return ControlSolver(ocp, x0=x0, p=p, uprev=uprev, opts=opts, device=device)


def callSolver(solver: ControlSolver) -> dict:
    """``mpc.callSolver``: solve and return the trajectories as arrays."""
    solver.solve()
    X, U = solver._traj()
    T = float(getattr(solver.ocp, "T", 0.0) or 0.0)
    return {"x": X, "u": U, "t": T * np.arange(X.shape[0]), "status": solver.stats["status"], "obj": solver._f}
