"""Nonlinear ODE models: the BASELINE config variants the reference has only in linearised or
renamed form (SURVEY.md §7 item 6, §8(d) config 4 "plus the 6-state extension").

Same NLP shape as the unicycle scripts (multiple shooting, interleaved w, lifted X_0, RK4 with M
substeps, mpctools node cost l = sum Q_i (x_i - xr_i)^2 + sum R_j (u_j - ur_j)^2), solved by the
same IPM kernel with exact derivatives (``csrc/ode.h``).  Parity: against the CPU oracle
(``oracle/ode_ref.py``) only -- the reference holds no outputs for these models.

* ``kin_bicycle``  x = (X, Y, psi), u = (v, delta), psi' = v tan(delta) / L.  Config 3 variant
  ("kinematic bicycle, circular ref, N=30"): the circle of ``Trajectory_tracking.py:84-97``.
* ``dyn_bicycle``  x = (X, Y, psi, vx, vy, r), u = (delta, ax), linear tyres with the reference's
  m, a, b, Ca, Jz (``Trajectory_tracking_dynamic_model.py:36-42``); linearised at vx = vref it is
  the reference's LTV model (:119-128).  Config 4 variant ("6-state dynamic bicycle,
  lane_change.csv, N=50").  lane_change.csv is driven at 0.4-0.8 m/s, where a 1200 kg car on
  linear tyres is stiff (|A44| ~ 1000 /s, RK4 would need M ~ 20); the variant drives the same
  lateral manoeuvre with x and speed scaled by ``scale`` = 10 (same 0.05 s per row, 4-8 m/s).
* ``cartpole``     x = (p, p', phi, phi'), u = F; M = m = 1, L = 0.5, g = 9.81, c = 10: linearised
  at phi = 0 it is the reference's Ac, Bc (``inverted_pendulum_single_shooting_mpctools.py:19-23``).
  Config 5 variant ("swing-up, N=100"); cost (1.2 (p - p_ref))^2 + phi^2 + (0.01 F)^2 (:33-36).
"""
from __future__ import annotations

import dataclasses
import math

import numpy as np

from . import _lib

MODELS = {"kin_bicycle": (_lib.MODEL_KIN_BICYCLE, 3, 2), "dyn_bicycle": (_lib.MODEL_DYN_BICYCLE, 6, 2),
          "cartpole": (_lib.MODEL_CARTPOLE, 4, 1)}
DYN_BICYCLE_PAR = (1200.0, 1.5, 2.0, 55000.0, 1350.0)  # m, a, b, Ca, Jz
CARTPOLE_PAR = (1.0, 1.0, 0.5, 9.81, 10.0)              # M, m, L, g, c


@dataclasses.dataclass
class OdeOCP:
    model: str = "kin_bicycle"
    N: int = 30
    T: float = 0.2
    M: int = 1
    Q: tuple = (1.0, 1.0, 0.1)
    R: tuple = (0.5, 0.05)
    u_lb: tuple = (-1.0, -math.pi / 4)
    u_ub: tuple = (1.0, math.pi / 4)
    x_lb: tuple = (-math.inf,) * 3
    x_ub: tuple = (math.inf,) * 3
    par: tuple = (0.5,)
    cost: str = "node"
    param: str = "x0_stageref"
    formulation: str = "multiple_shooting"

    def __post_init__(self):
        if self.model not in MODELS:
            raise ValueError(f"unknown ODE model {self.model!r}")
        nx, nu = self.nx, self.nu
        for name, n in (("Q", nx), ("x_lb", nx), ("x_ub", nx), ("R", nu), ("u_lb", nu), ("u_ub", nu)):
            if len(getattr(self, name)) != n:
                raise ValueError(f"{name}: expected {n} entries")
        if self.cost != "node":
            raise ValueError("ODE models use the node cost")
        if self.formulation not in ("multiple_shooting", "single_shooting"):
            raise ValueError(f"unknown formulation {self.formulation!r}")

    @property
    def nx(self):
        return MODELS[self.model][1]

    @property
    def nu(self):
        return MODELS[self.model][2]

    @property
    def nz(self):
        return self.nx + self.nu

    @property
    def n_w_ms(self):
        return self.nx + self.nz * self.N

    @property
    def n_g_ms(self):
        return self.nx * (self.N + 1)

    @property
    def n_p(self):
        return 2 * self.nx if self.param == "x0_xref" else self.nx + self.nz * self.N

    def params(self, x0, ref):
        """P rows: x0 (B, nx) with ref = x_ref (B, nx) [x0_xref] or stage refs (B, N, nz) [x0_stageref]."""
        x0 = np.atleast_2d(np.asarray(x0, np.float64))
        ref = np.asarray(ref, np.float64)
        B = x0.shape[0]
        if self.param == "x0_xref":
            ref = np.broadcast_to(ref.reshape(-1, self.nx), (B, self.nx))
        else:
            ref = np.broadcast_to(ref.reshape(-1, self.N, self.nz), (B, self.N, self.nz)).reshape(B, -1)
        return np.ascontiguousarray(np.concatenate([x0, ref], axis=1))


# ---------------------------------------------------------------------------- builders
def kinematic_bicycle_tracking(N=30, T=0.2, L=0.5):
    """Config 3 variant: kinematic bicycle on the circle of ``Trajectory_tracking.py:84-97``
    (Q = diag(1,1,0.1), R = diag(0.5,0.05) as there; |v| <= 1, |delta| <= pi/4)."""
    return OdeOCP(model="kin_bicycle", N=N, T=T, M=1, Q=(1.0, 1.0, 0.1), R=(0.5, 0.05), u_lb=(-1.0, -math.pi / 4),
                  u_ub=(1.0, math.pi / 4), x_lb=(-math.inf,) * 3, x_ub=(math.inf,) * 3, par=(float(L),))


def bicycle_circular_reference(tau0, t, N, Delta=0.2, L=0.5):
    """Stage references (B, N, 5) on the unit circle at angular rate 0.1 (the script's
    (cos .1 tau, sin .1 tau, pi/2 + .1 tau)), with the consistent inputs v = 0.1 and
    delta = atan(L) (curvature 1)."""
    tau0 = np.atleast_1d(np.asarray(tau0, dtype=np.float64))
    tau = tau0[:, None] + Delta * (t + np.arange(N))[None, :]
    one = np.ones_like(tau)
    return np.stack([np.cos(0.1 * tau), np.sin(0.1 * tau), np.pi / 2 + 0.1 * tau, 0.1 * one,
                     math.atan(L) * one], axis=-1)


def dynamic_bicycle_lane_change(N=50, T=0.05, M=4):
    """Config 4 variant: 6-state dynamic bicycle (Q = I, R = I as the LTV script's Q = I, R = 1,
    :23-31), |delta| <= 0.5 rad, |ax| <= 5 m/s^2, vx >= 2.5 m/s.  The speed bound keeps RK4 stable
    inside every interval: the tyre terms scale as 1/vx (A44 ~ -509/vx), and M = 4 substeps of
    0.0125 s need |A44| h < 2.78, i.e. vx > 2.3 (the references run at 4-8 m/s)."""
    inf = math.inf
    return OdeOCP(model="dyn_bicycle", N=N, T=T, M=M, Q=(1.0,) * 6, R=(1.0, 1.0), u_lb=(-0.5, -5.0), u_ub=(0.5, 5.0),
                  x_lb=(-inf, -inf, -inf, 2.5, -inf, -inf), x_ub=(inf,) * 6, par=DYN_BICYCLE_PAR)


def lane_change_rows(xref, yref, vref, scale=10.0):
    """lane_change.csv (x, y, uref) with x and speed scaled (see module docstring) -> (X, Y, V)."""
    return (np.asarray(xref, float) * scale, np.asarray(yref, float), np.asarray(vref, float) * scale)


def dyn_bicycle_references(X, Y, V, t, N, Delta=0.05, par=DYN_BICYCLE_PAR, w=8):
    """Stage references (N, 8) from step t of the path rows: position, heading of the path
    tangent, vx = speed, vy = 0, yaw rate, steering of the kinematic curvature
    atan((a + b) r / vx) and ax = speed rate.  Heading and rates are centred differences over +-w
    rows (w = 8: 0.4 s): the csv's one-row differences are noisy enough to ask for 3 rad of
    steering where the path turns sharpest (rows ~224-260).  Past the last row the path continues
    along its last increment at the last speed (a consistent straight-line reference)."""
    X, Y, V = (np.asarray(c, float) for c in (X, Y, V))
    ext = max(0, t + N + w + 1 - len(X))
    if ext:
        j = np.arange(1, ext + 1)
        X = np.concatenate([X, X[-1] + j * (X[-1] - X[-2])])
        Y = np.concatenate([Y, Y[-1] + j * (Y[-1] - Y[-2])])
        V = np.concatenate([V, np.full(ext, V[-1])])
    n = len(X)
    i = np.arange(n)
    a_, b_ = np.clip(i - w, 0, n - 1), np.clip(i + w, 0, n - 1)
    psi = np.unwrap(np.arctan2(Y[b_] - Y[a_], X[b_] - X[a_]))
    span = (b_ - a_) * Delta
    r = (psi[b_] - psi[a_]) / span
    ax = (V[b_] - V[a_]) / span
    a, b = par[1], par[2]
    delta = np.arctan((a + b) * r / V)
    k = np.minimum(t + np.arange(N), n - 1)
    return np.stack([X[k], Y[k], psi[k], V[k], np.zeros(N), r[k], delta[k], ax[k]], axis=-1)


def cartpole_swingup(N=100, T=0.01, M=1, u_max=200.0, formulation="multiple_shooting"):
    """Config 5 variant: nonlinear cart-pole, p = [x0; x_ref].  formulation="single_shooting" (the
    BASELINE label): decision = U (N), g = X_1..X_N with +-inf bounds; solved through the same
    multiple-shooting kernel (same optimum)."""
    inf = math.inf
    return OdeOCP(model="cartpole", N=N, T=T, M=M, Q=(1.44, 0.0, 1.0, 0.0), R=(1e-4,), u_lb=(-u_max,), u_ub=(u_max,),
                  x_lb=(-inf,) * 4, x_ub=(inf,) * 4, par=CARTPOLE_PAR, param="x0_xref", formulation=formulation)
