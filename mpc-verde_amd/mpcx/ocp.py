"""Problem descriptions: the NLPs the reference scripts build symbolically.

CasADi receives ``prob = {'f': J, 'x': w, 'g': g, 'p': P}`` as symbolic
expressions.  CasADi is not the product here, so a problem is described by the
few numbers that determine those expressions; :func:`to_spec` turns one into
the C ``mpcx_spec``.  Each builder cites the script whose NLP it reproduces.
"""
from __future__ import annotations

import dataclasses
import math

from . import _lib


@dataclasses.dataclass
class OCP:
    """Multiple-shooting OCP of ``Casadi/multiple_shooting_casadi.py:30-178``.

    formulation = "multiple_shooting": decision vector w = [X_0 | U_0 X_1 | ...]
                  (interleaved, :128-170), g = [P[:3]-X_0; F(X_k,U_k).xf - X_{k+1}].
    formulation = "single_shooting": decision vector = U (interleaved v, w),
                  g = (x_k, y_k) k=1..N with +-inf bounds
                  (``Casadi/single_shooting_v2.py:115-158``).
    cost = "quadrature" (RK4-integrated L, CasADi scripts) or "node" (mpctools).
    param = "x0_xref": p = [x0; x_ref] (6); "x0_stageref": p = [x0; (x_ref_k, u_ref_k)_k].
    """

    N: int = 10
    T: float = 0.2
    M: int = 4
    Q: tuple = (1.0, 5.0, 0.1)
    R: tuple = (0.5, 0.05)
    u_lb: tuple = (-1.0, -math.pi / 4)
    u_ub: tuple = (1.0, math.pi / 4)
    x_lb: tuple = (-math.inf, -math.inf, -math.inf)
    x_ub: tuple = (math.inf, math.inf, math.inf)
    cost: str = "quadrature"
    param: str = "x0_xref"
    formulation: str = "multiple_shooting"
    model: str = "unicycle"

    @property
    def nx(self):
        return 3

    @property
    def nu(self):
        return 2

    @property
    def n_w_ms(self):
        return 3 + 5 * self.N

    @property
    def n_g_ms(self):
        return 3 * (self.N + 1)

    @property
    def n_p(self):
        return 6 if self.param == "x0_xref" else 3 + 5 * self.N


def unicycle_point_to_point(N=10, T=0.2, M=4, v_max=1.0, omega_max=math.pi / 4, Q=(1.0, 5.0, 0.1), R=(0.5, 0.05),
                            formulation="multiple_shooting"):
    """``Casadi/multiple_shooting_casadi.py:30-114`` (and ``single_shooting_v2.py``)."""
    return OCP(N=N, T=T, M=M, Q=tuple(Q), R=tuple(R), u_lb=(-v_max, -omega_max), u_ub=(v_max, omega_max),
               formulation=formulation)


def unicycle_point_to_point_mpctools(N=10, T=0.2):
    """``mpctools/multiple_shooting_mpctools.py:9-70`` (writes ``Casadi/3exemplo.xlsx``): RK4
    M=1 model, node cost (x - goal)^T diag(1,5,0.1) (x - goal) + u^T u (the script's R is not
    used by its lfunc, :57-58), |v| <= 1, |w| <= pi/4; p = [x0; goal]."""
    return OCP(N=N, T=T, M=1, Q=(1.0, 5.0, 0.1), R=(1.0, 1.0), cost="node")


def unicycle_tracking(N=10, T=0.2):
    """``Trajectory Tracking/Trajectory_tracking.py:15-72``: RK4 with M=1, node cost
    l(x,u,p_k) with Q=diag(1,1,0.1), R=diag(0.5,0.05), per-stage reference
    p_k = (x_r, y_r, th_r, v_r, w_r), bounds |v|<=1, |w|<=pi/4, x in [-20,20], y in [-2,2]."""
    return OCP(N=N, T=T, M=1, Q=(1.0, 1.0, 0.1), R=(0.5, 0.05), x_lb=(-20.0, -2.0, -math.inf),
               x_ub=(20.0, 2.0, math.inf), cost="node", param="x0_stageref")


def circular_reference(tau0, t, N, Delta=0.2):
    """Per-stage references of ``Trajectory Tracking/Trajectory_tracking.py:84-97``.

    For receding-horizon step t and stage k the reference time is
    tau = tau0 + Delta*(t + k) and p_k = (cos(0.1 tau), sin(0.1 tau), pi/2 + 0.1 tau, 1, 1)
    (the script's u_ref = (1, 1) is kept as written).  tau0 (B,) offsets the phase per
    instance (tau0 = 0 is the script's single run).  Returns (B, N, 5).
    """
    import numpy as np

    tau0 = np.atleast_1d(np.asarray(tau0, dtype=np.float64))
    tau = tau0[:, None] + Delta * (t + np.arange(N))[None, :]
    one = np.ones_like(tau)
    return np.stack([np.cos(0.1 * tau), np.sin(0.1 * tau), np.pi / 2 + 0.1 * tau, one, one], axis=-1)


MODEL_IDS = {"unicycle": _lib.MODEL_UNICYCLE, "linear": _lib.MODEL_LINEAR, "kin_bicycle": _lib.MODEL_KIN_BICYCLE,
             "dyn_bicycle": _lib.MODEL_DYN_BICYCLE, "cartpole": _lib.MODEL_CARTPOLE}


# IPOPT termination / recovery options the spec carries (IPOPT's names); values left out take
# IPOPT's defaults for every model, as ca.nlpsol without options does.  The reference script
# passes acceptable_tol 1e-8 / acceptable_obj_change_tol 1e-6 itself
# (Casadi/multiple_shooting_casadi.py:188-196), and callers mirroring it pass them the same way;
# the C ABI's mpcx_default_spec, which describes that script's problem, fills them in for the
# unicycle (include/mpcx.h).
IPOPT_OPTIONS = ("dual_inf_tol", "constr_viol_tol", "compl_inf_tol", "acceptable_tol", "acceptable_dual_inf_tol",
                 "acceptable_constr_viol_tol", "acceptable_compl_inf_tol", "acceptable_obj_change_tol",
                 "acceptable_iter")
IPOPT_DEFAULTS = {"dual_inf_tol": 1.0, "constr_viol_tol": 1e-4, "compl_inf_tol": 1e-4, "acceptable_tol": 1e-6,
                  "acceptable_dual_inf_tol": 1e10, "acceptable_constr_viol_tol": 1e-2,
                  "acceptable_compl_inf_tol": 1e-2, "acceptable_obj_change_tol": 1e20, "acceptable_iter": 15}


def to_spec(ocp, max_iter=2000, tol=1e-8, device=0, warm=(1e-4, 1e-4, 1e-4), group_policy=0, ipopt=None,
            restoration=True) -> _lib.Spec:
    """mpcx_spec of an :class:`OCP` (unicycle), :class:`mpcx.lti.LinearOCP` (linear model;
    its stage tables are uploaded separately by the solver, mpcx_set_linear_model) or
    :class:`mpcx.ode.OdeOCP` (nonlinear ODE models, constants in ``par``).  ``ipopt``: IPOPT
    termination options by name (IPOPT_OPTIONS; IPOPT's defaults otherwise)."""
    if ocp.model not in MODEL_IDS:
        raise ValueError(f"unsupported model {ocp.model!r}")
    s = _lib.Spec()
    lin = ocp.model == "linear"
    s.model = MODEL_IDS[ocp.model]
    for i, v in enumerate(getattr(ocp, "par", ())):
        s.par[i] = float(v)
    s.cost = {"quadrature": _lib.COST_QUADRATURE, "node": _lib.COST_NODE}[ocp.cost]
    s.param_layout = {"x0_xref": _lib.P_X0_XREF, "x0_stageref": _lib.P_X0_STAGEREF}[ocp.param]
    s.N, s.M, s.max_iter, s.device = int(ocp.N), int(getattr(ocp, "M", 1)), int(max_iter), int(device)
    s.T, s.tol = float(ocp.T), float(tol)
    s.warm_mu_init, s.warm_bound_push, s.warm_mult_push = (float(v) for v in warm)
    s.nx, s.nu = int(ocp.nx), int(ocp.nu)
    s.group_policy = int(group_policy)
    o = dict(IPOPT_DEFAULTS)
    for k, v in (ipopt or {}).items():
        if k not in o:
            raise ValueError(f"unknown IPOPT option {k!r}")
        o[k] = v
    for k in IPOPT_OPTIONS:
        if k == "acceptable_iter":
            s.acceptable_iter = -1 if int(o[k]) == 0 else int(o[k])  # IPOPT: 0 disables the heuristic
        elif k == "acceptable_obj_change_tol" and float(o[k]) == 0.0:
            # the spec reads a 0 field as IPOPT's default (include/mpcx.h); IPOPT's literal 0
            # (|f - f_last| <= 0) is the same test as |f - f_last| <= 5e-324 max(1, |f|)
            s.acceptable_obj_change_tol = 5e-324
        else:
            setattr(s, k, float(o[k]))
    s.no_restoration = 0 if restoration else 1
    big = 1e20

    def fin(v, default):
        return default if not math.isfinite(v) else float(v)

    for i in range(ocp.nx):
        if not lin:
            s.Q[i] = float(ocp.Q[i])
        s.lbx[i] = fin(ocp.x_lb[i], -big)
        s.ubx[i] = fin(ocp.x_ub[i], big)
    for i in range(ocp.nu):
        if not lin:
            s.R[i] = float(ocp.R[i])
        s.lbu[i] = fin(ocp.u_lb[i], -big)
        s.ubu[i] = fin(ocp.u_ub[i], big)
    return s
