"""ctypes loader for the C++ CPU oracle ``oracle/libipm_ref.so``.

TEST INFRASTRUCTURE ONLY (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


class OracleSpec(ctypes.Structure):
    _fields_ = [("N", ctypes.c_int32), ("M", ctypes.c_int32), ("cost", ctypes.c_int32),
                ("max_iter", ctypes.c_int32), ("T", ctypes.c_double), ("Q", ctypes.c_double * 3),
                ("R", ctypes.c_double * 2), ("tol", ctypes.c_double)]


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _LIB
    if _LIB is None:
        # ORACLE_LIB: another build of the same oracle (the sanitizer build, tests/test_asan.py)
        path = os.environ.get("ORACLE_LIB") or os.path.join(_HERE, "libipm_ref.so")
        if not os.path.exists(path):
            build()
        _LIB = ctypes.CDLL(path)
        dp = ctypes.POINTER(ctypes.c_double)
        ip = ctypes.POINTER(ctypes.c_int32)
        _LIB.oracle_solve_batch.argtypes = [ctypes.POINTER(OracleSpec), ctypes.c_int, dp, ctypes.c_int, dp, dp, dp,
                                            dp, dp, dp, dp, ip, ip, ctypes.c_int]
        _LIB.oracle_solve_batch_warm.argtypes = [ctypes.POINTER(OracleSpec), ctypes.c_int, dp, ctypes.c_int, dp, dp,
                                                 dp, ctypes.c_double, ctypes.c_double, ctypes.c_double, dp, dp,
                                                 dp, dp, dp, dp, ip, ip, ctypes.c_int]
        _LIB.oracle_stage.argtypes = [ctypes.POINTER(OracleSpec), ctypes.c_int, dp, dp, dp, dp, dp, dp, dp, dp, dp]
        _LIB.oracle_solve.argtypes = [ctypes.POINTER(OracleProblem), ctypes.POINTER(OracleOpts), ctypes.c_int, dp,
                                      ctypes.c_int, dp, dp, dp, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                      dp, dp, dp, dp, dp, dp, ip, ip, ctypes.c_int]
    return _LIB


def _p(a):
    if a is None:
        return None
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def _spec(ocp, max_iter=200, tol=1e-8):
    s = OracleSpec()
    s.N, s.M = ocp.N, ocp.M
    s.cost = 0 if ocp.cost == "quadrature" else 1
    s.max_iter = max_iter
    s.T = ocp.T
    s.Q[:] = list(ocp.Q)
    s.R[:] = list(ocp.R)
    s.tol = tol
    return s


def solve_batch(ocp, P, w0=None, pstage=None, lbw=None, ubw=None, max_iter=200, tol=1e-8, nthreads=0):
    """Batched IPM solve on the CPU.  Returns dict(w, lam_g, f, status, iters)."""
    from . import nlp_ref
    P = np.ascontiguousarray(P, dtype=np.float64)
    B = P.shape[0]
    nw, ng = nlp_ref.n_w(ocp.N), nlp_ref.n_g(ocp.N)
    lb, ub = nlp_ref.ms_bounds(ocp)
    lb = np.ascontiguousarray(lb if lbw is None else lbw, dtype=np.float64)
    ub = np.ascontiguousarray(ub if ubw is None else ubw, dtype=np.float64)
    lb = np.where(np.isfinite(lb), lb, -1e20)
    ub = np.where(np.isfinite(ub), ub, 1e20)
    w0a = None if w0 is None else np.ascontiguousarray(w0, dtype=np.float64).reshape(B, nw)
    ps = None if pstage is None else np.ascontiguousarray(pstage, dtype=np.float64).reshape(B, ocp.N, 5)
    w = np.zeros((B, nw))
    lam = np.zeros((B, ng))
    f = np.zeros(B)
    st = np.zeros(B, np.int32)
    it = np.zeros(B, np.int32)
    spec = _spec(ocp, max_iter, tol)
    lib().oracle_solve_batch(ctypes.byref(spec), B, _p(P), P.shape[1], _p(ps), _p(w0a), _p(lb), _p(ub), _p(w),
                             _p(lam), _p(f), st.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                             it.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), nthreads)
    return {"w": w, "lam_g": lam, "f": f, "status": st, "iters": it}


def solve_batch_warm(ocp, P, w0, lam0=None, lamx0=None, mu_init=1e-3, bound_push=1e-3, mult_push=1e-3,
                     max_iter=200, tol=1e-8, nthreads=0):
    """IPOPT-style warm start (multipliers + small initial barrier).  Returns w, lam_g, lam_x, f, status, iters."""
    from . import nlp_ref
    P = np.ascontiguousarray(P, dtype=np.float64)
    B = P.shape[0]
    nw, ng = nlp_ref.n_w(ocp.N), nlp_ref.n_g(ocp.N)
    lb, ub = nlp_ref.ms_bounds(ocp)
    lb = np.ascontiguousarray(np.where(np.isfinite(lb), lb, -1e20))
    ub = np.ascontiguousarray(np.where(np.isfinite(ub), ub, 1e20))
    w0 = np.ascontiguousarray(w0, dtype=np.float64).reshape(B, nw)
    l0 = None if lam0 is None else np.ascontiguousarray(lam0, dtype=np.float64).reshape(B, ng)
    x0 = None if lamx0 is None else np.ascontiguousarray(lamx0, dtype=np.float64).reshape(B, nw)
    w = np.zeros((B, nw)); lam = np.zeros((B, ng)); lamx = np.zeros((B, nw)); f = np.zeros(B)
    st = np.zeros(B, np.int32); it = np.zeros(B, np.int32)
    spec = _spec(ocp, max_iter, tol)
    ip_ = ctypes.POINTER(ctypes.c_int32)
    lib().oracle_solve_batch_warm(ctypes.byref(spec), B, _p(P), P.shape[1], _p(w0), _p(lb), _p(ub), mu_init,
                                  bound_push, mult_push, _p(l0), _p(x0), _p(w), _p(lam), _p(lamx), _p(f),
                                  st.ctypes.data_as(ip_), it.ctypes.data_as(ip_), nthreads)
    return {"w": w, "lam_g": lam, "lam_x": lamx, "f": f, "status": st, "iters": it}


def stage(ocp, x, u, xr, ur=None, lam=None):
    """Interval map + Jacobian (B,4,5) + packed Hessian of qf + lam^T xf (B,15)."""
    x = np.ascontiguousarray(x, np.float64).reshape(-1, 3)
    B = x.shape[0]
    u = np.ascontiguousarray(u, np.float64).reshape(B, 2)
    xr = np.ascontiguousarray(np.broadcast_to(xr, (B, 3)), np.float64)
    ur = None if ur is None else np.ascontiguousarray(np.broadcast_to(ur, (B, 2)), np.float64)
    lam = None if lam is None else np.ascontiguousarray(np.broadcast_to(lam, (B, 3)), np.float64)
    xf = np.zeros((B, 3))
    qf = np.zeros(B)
    jac = np.zeros((B, 4, 5))
    hess = np.zeros((B, 15))
    spec = _spec(ocp)
    lib().oracle_stage(ctypes.byref(spec), B, _p(x), _p(u), _p(xr), _p(ur), _p(lam), _p(xf), _p(qf), _p(jac),
                       _p(hess))
    return xf, qf, jac, hess


def unpack_sym5(h):
    """packed upper-triangular (…,15) -> (…,5,5)."""
    h = np.asarray(h)
    H = np.zeros(h.shape[:-1] + (5, 5))
    t = 0
    for i in range(5):
        for j in range(i, 5):
            H[..., i, j] = h[..., t]
            H[..., j, i] = h[..., t]
            t += 1
    return H


# ---------------------------------------------------------------------------- any model
class OracleProblem(ctypes.Structure):
    _fields_ = [("model", ctypes.c_int32), ("N", ctypes.c_int32), ("M", ctypes.c_int32), ("cost", ctypes.c_int32),
                ("p_layout", ctypes.c_int32), ("pad", ctypes.c_int32), ("T", ctypes.c_double),
                ("Q", ctypes.c_double * 8), ("R", ctypes.c_double * 8), ("par", ctypes.c_double * 8)]


class OracleOpts(ctypes.Structure):
    _fields_ = [("tol", ctypes.c_double), ("dual_inf_tol", ctypes.c_double), ("constr_viol_tol", ctypes.c_double),
                ("compl_inf_tol", ctypes.c_double), ("acceptable_tol", ctypes.c_double),
                ("acceptable_dual_inf_tol", ctypes.c_double), ("acceptable_constr_viol_tol", ctypes.c_double),
                ("acceptable_compl_inf_tol", ctypes.c_double), ("acceptable_obj_change_tol", ctypes.c_double),
                ("max_iter", ctypes.c_int32), ("acceptable_iter", ctypes.c_int32), ("restoration", ctypes.c_int32),
                ("max_soc", ctypes.c_int32)]


# IPOPT defaults (its documented option values)
IPOPT_DEFAULTS = {"tol": 1e-8, "dual_inf_tol": 1.0, "constr_viol_tol": 1e-4, "compl_inf_tol": 1e-4,
                  "acceptable_tol": 1e-6, "acceptable_dual_inf_tol": 1e10, "acceptable_constr_viol_tol": 1e-2,
                  "acceptable_compl_inf_tol": 1e-2, "acceptable_obj_change_tol": 1e20, "max_iter": 3000,
                  "acceptable_iter": 15, "restoration": 1, "max_soc": None}
# the product takes IPOPT's second-order correction (max_soc 4) for the 6-state bicycle only
# (DESIGN §3.4); max_soc=None follows that per-model choice
PRODUCT_SOC = {"dyn_bicycle": 4}
MODEL_IDS = {"unicycle": 1, "kin_bicycle": 3, "dyn_bicycle": 4, "cartpole": 5}


def _problem(ocp):
    pb = OracleProblem()
    pb.model = MODEL_IDS[getattr(ocp, "model", "unicycle")]
    pb.N, pb.M = ocp.N, ocp.M
    pb.cost = 0 if ocp.cost == "quadrature" else 1
    pb.p_layout = 0 if getattr(ocp, "param", "x0_xref") == "x0_xref" else 1
    pb.T = ocp.T
    for name in ("Q", "R"):
        v = list(getattr(ocp, name))
        getattr(pb, name)[:len(v)] = v
    v = list(getattr(ocp, "par", ()))
    pb.par[:len(v)] = v
    return pb


def ms_bounds_any(ocp):
    """lbw/ubw of the multiple-shooting w (X_0 free: pinned by g_0) for any OCP with
    u_lb/u_ub/x_lb/x_ub (ODE models) or the unicycle's nlp_ref bounds."""
    if getattr(ocp, "model", "unicycle") == "unicycle":
        from . import nlp_ref
        return nlp_ref.ms_bounds(ocp)
    nx, nu, N = ocp.nx, ocp.nu, ocp.N
    lb = [np.full(nx, -np.inf)]
    ub = [np.full(nx, np.inf)]
    for _ in range(N):
        lb += [np.asarray(ocp.u_lb, float), np.asarray(ocp.x_lb, float)]
        ub += [np.asarray(ocp.u_ub, float), np.asarray(ocp.x_ub, float)]
    return np.concatenate(lb), np.concatenate(ub)


def solve(ocp, P, w0=None, lbw=None, ubw=None, lam0=None, lamx0=None, warm=None, nthreads=0, **opts):
    """Any model (unicycle OCP or mpcx OdeOCP), IPOPT options by name (defaults IPOPT's).
    w0 None = the product's cold start (X_k = x0, U = 0); warm = (mu_init, bound_push, mult_push)."""
    o = dict(IPOPT_DEFAULTS)
    for k, v in opts.items():
        if k not in o:
            raise ValueError(f"unknown option {k}")
        o[k] = v
    if o["max_soc"] is None:
        o["max_soc"] = PRODUCT_SOC.get(getattr(ocp, "model", "unicycle"), 0)
    op = OracleOpts()
    for k, v in o.items():
        setattr(op, k, v)
    pb = _problem(ocp)
    P = np.ascontiguousarray(np.atleast_2d(P), dtype=np.float64)
    B = P.shape[0]
    nx, nz, N = pb_dims(ocp)
    nw, ng = nx + nz * N, nx * (N + 1)
    lb0, ub0 = ms_bounds_any(ocp)
    lb = np.asarray(lb0 if lbw is None else lbw, float)
    ub = np.asarray(ub0 if ubw is None else ubw, float)
    lb = np.ascontiguousarray(np.where(np.isfinite(lb), lb, -1e20))
    ub = np.ascontiguousarray(np.where(np.isfinite(ub), ub, 1e20))
    w0a = None if w0 is None else np.ascontiguousarray(w0, dtype=np.float64).reshape(B, nw)
    l0 = None if lam0 is None else np.ascontiguousarray(lam0, dtype=np.float64).reshape(B, ng)
    lx0 = None if lamx0 is None else np.ascontiguousarray(lamx0, dtype=np.float64).reshape(B, nw)
    mi, bp, mp = warm if warm is not None else (0.0, 0.0, 0.0)
    w = np.zeros((B, nw)); lam = np.zeros((B, ng)); lamx = np.zeros((B, nw)); f = np.zeros(B)
    st = np.zeros(B, np.int32); it = np.zeros(B, np.int32)
    ip_ = ctypes.POINTER(ctypes.c_int32)
    L = lib()
    L.oracle_solve(ctypes.byref(pb), ctypes.byref(op), B, _p(P), P.shape[1], _p(w0a), _p(lb), _p(ub), mi, bp, mp,
                   _p(l0), _p(lx0), _p(w), _p(lam), _p(lamx), _p(f), st.ctypes.data_as(ip_), it.ctypes.data_as(ip_),
                   nthreads)
    return {"w": w, "lam_g": lam, "lam_x": lamx, "f": f, "status": st, "iters": it}


def pb_dims(ocp):
    if getattr(ocp, "model", "unicycle") == "unicycle":
        return 3, 5, ocp.N
    return ocp.nx, ocp.nz, ocp.N
