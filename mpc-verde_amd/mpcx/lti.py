"""Linear (LTI / LTV) MPC problems -- the mpctools QP scripts of the reference.

A linear problem is described by stage tables (``mpcx_set_linear_model``):

    x_{k+1} = A_j x_k + B_j u_k + c_j,      l_k = (z_k - zr_k)^T W_j (z_k - zr_k),
    z = (x, u),  j = tab[k] (shared) or tab[b, k] (per instance),

with per-stage references zr_k carried in P = [x0; zr_0; ...; zr_{N-1}] and box
bounds on u (and optionally x).  mpctools' ``Du`` terms and move blocking are
expressed by augmenting the state with the previous input (u_prev) and using two
tables: "free" stages (u_prev+ = u, cost on u - u_prev) and "blocked" stages
(the applied input is u_prev, the stage's own u is a dummy held at 0).

Builders:
  * :func:`inverted_pendulum_qp` -- ``Inverted_pendulum/inverted_pendulum_single_shooting_mpctools.py:15-78``
  * :func:`lateral_ltv`          -- ``Trajectory Tracking/Trajectory_tracking_dynamic_model.py:13-145``
  * :func:`lateral_error_lti`    -- ``Trajectory Tracking/Trajectory_tracking_le_LTI.py:17-79``
  * :func:`lateral_error_ltv`    -- ``Trajectory Tracking/Trjectory_tracking_le_LTV.py:27-166``
"""
from __future__ import annotations

import dataclasses
import math

import numpy as np


def c2d(Ac, Bc, T):
    """Zero-order-hold discretisation (what ``mpctools.util.c2d`` computes):
    A = e^{Ac T}, B = int_0^T e^{Ac s} ds Bc, via the exponential of [[Ac, Bc], [0, 0]] T."""
    from scipy.linalg import expm

    Ac = np.asarray(Ac, float)
    Bc = np.asarray(Bc, float).reshape(Ac.shape[0], -1)
    n, m = Bc.shape
    Mx = np.zeros((n + m, n + m))
    Mx[:n, :n] = Ac
    Mx[:n, n:] = Bc
    E = expm(Mx * T)
    return E[:n, :n].copy(), E[:n, n:].copy()


def pack_sym(W):
    """(..., n, n) symmetric -> (..., n(n+1)/2) packed upper triangle, row-major (riccati.h symix)."""
    W = np.asarray(W, float)
    n = W.shape[-1]
    iu = np.triu_indices(n)
    return np.ascontiguousarray(W[..., iu[0], iu[1]])


@dataclasses.dataclass
class LinearOCP:
    """Multiple-shooting linear-quadratic OCP (model = "linear", mpcx_spec.model = 2).

    A (n_tab, nx, nx), B (n_tab, nx, nu), c (n_tab, nx), W (n_tab, nz, nz) symmetric,
    tab (N,) shared or (B, N) per-instance table indices.  w layout is the reference's
    interleaved [X_0 | U_0 X_1 | ...]; P = [x0 (nx); zr_k (nz) for k < N].
    """

    N: int
    A: np.ndarray
    B: np.ndarray
    W: np.ndarray
    tab: np.ndarray
    c: np.ndarray | None = None
    T: float = 0.0
    u_lb: tuple = ()
    u_ub: tuple = ()
    x_lb: tuple = ()
    x_ub: tuple = ()
    name: str = "linear"
    model: str = "linear"
    cost: str = "node"
    param: str = "x0_stageref"
    formulation: str = "multiple_shooting"

    def __post_init__(self):
        self.A = np.ascontiguousarray(np.asarray(self.A, float).reshape(-1, self.nx, self.nx))
        self.B = np.ascontiguousarray(np.asarray(self.B, float).reshape(-1, self.nx, self.nu))
        if self.c is None:
            self.c = np.zeros((self.A.shape[0], self.nx))
        self.c = np.ascontiguousarray(np.asarray(self.c, float).reshape(-1, self.nx))
        self.W = np.ascontiguousarray(np.asarray(self.W, float).reshape(-1, self.nz, self.nz))
        self.tab = np.ascontiguousarray(np.asarray(self.tab, np.int32))
        if not (self.A.shape[0] == self.B.shape[0] == self.c.shape[0] == self.W.shape[0]):
            raise ValueError("A, B, c, W must have the same number of tables")
        if self.tab.shape[-1] != self.N or self.tab.ndim not in (1, 2):
            raise ValueError("tab must be (N,) or (B, N)")
        if self.tab.min() < 0 or self.tab.max() >= self.n_tab:
            raise ValueError("tab index out of range")
        if not np.allclose(self.W, np.swapaxes(self.W, -1, -2)):
            raise ValueError("W must be symmetric")
        if not self.u_lb:
            self.u_lb = (-math.inf,) * self.nu
        if not self.u_ub:
            self.u_ub = (math.inf,) * self.nu
        if not self.x_lb:
            self.x_lb = (-math.inf,) * self.nx
        if not self.x_ub:
            self.x_ub = (math.inf,) * self.nx

    @property
    def nx(self):
        return np.asarray(self.A).shape[-1]

    @property
    def nu(self):
        return np.asarray(self.B).shape[-1]

    @property
    def nz(self):
        return self.nx + self.nu

    @property
    def n_tab(self):
        return self.A.shape[0]

    @property
    def n_w_ms(self):
        return self.nx + self.nz * self.N

    @property
    def n_g_ms(self):
        return self.nx * (self.N + 1)

    @property
    def n_p(self):
        return self.nx + self.nz * self.N

    def tables(self):
        """(n_tab, A, B, c, Wpacked, tab (rows, N), rows) as passed to mpcx_set_linear_model."""
        tab = self.tab if self.tab.ndim == 2 else self.tab[None, :]
        return (self.n_tab, self.A, self.B, self.c, pack_sym(self.W), np.ascontiguousarray(tab, np.int32),
                tab.shape[0])

    def params(self, x0, zr):
        """P (B, n_p) from x0 (B, nx) and per-stage references zr (B, N, nz) or (N, nz) or (nz,)."""
        x0 = np.atleast_2d(np.asarray(x0, float))
        Bn = x0.shape[0]
        zr = np.broadcast_to(np.asarray(zr, float), (Bn, self.N, self.nz))
        return np.ascontiguousarray(np.concatenate([x0, zr.reshape(Bn, -1)], axis=1))


# (nx, nu) shapes with a kernel instantiation (csrc/solve_linear4.hip, solve_linear5.hip,
# solve_linear4x2.hip)
NATIVE_SHAPES = ((4, 1), (5, 1), (4, 2))


class StatePad:
    """A linear OCP with fewer states than a kernel instantiation, embedded in it.

    nx < 4 with nu = 1 or 2 is solved as the 4-state model of the same nu with zero pad states: A, B, c and W are
    zero-padded (pad rows and columns of A and W are 0, pad rows of B and c are 0) and the
    pad states are unbounded.  A pad state then starts at 0 (x0 and references padded with
    0), its defect is 0 at every iterate and so is every Newton step in it (its row of the
    dynamics maps everything to 0), its Riccati blocks are 0 and the inertia test sees the
    same Huu' as the unpadded problem: the solve is the same QP, with the same optimum and
    multipliers.  One IPOPT quantity sees the pad: the dual scaling s_d averages the
    multipliers over n_g + n_w entries, which include the pad's zero entries -- it differs from
    1 only when that mean exceeds s_max = 100 (Wächter & Biegler 2006 eq. 5).
    The index maps take the user's (B, n) arrays to the kernel's layout and back: w = [X_0 |
    U_k X_{k+1}]_k, P = [x0 | (x_r, u_r)_k], g = [g_k (nx)]_k.
    """

    def __init__(self, lin: LinearOCP, nxp: int = 4):
        nx, nu, N = lin.nx, lin.nu, lin.N
        if nx >= nxp:
            raise ValueError(f"StatePad: nx = {nx} needs no padding to {nxp}")
        self.lin, self.nxp = lin, nxp
        nzp = nxp + nu
        ix = np.r_[np.arange(nx), nxp + np.arange(nu)]  # z = (x, u) -> padded z = (x, pad, u)
        A = np.zeros((lin.n_tab, nxp, nxp))
        A[:, :nx, :nx] = lin.A
        Bm = np.zeros((lin.n_tab, nxp, nu))
        Bm[:, :nx] = lin.B
        c = np.zeros((lin.n_tab, nxp))
        c[:, :nx] = lin.c
        W = np.zeros((lin.n_tab, nzp, nzp))
        W[:, ix[:, None], ix[None, :]] = lin.W
        pad = (nxp - nx,)
        self.ocp = dataclasses.replace(lin, A=A, B=Bm, c=c, W=W, tab=lin.tab.copy(),
                                       x_lb=tuple(lin.x_lb) + (-math.inf,) * pad[0],
                                       x_ub=tuple(lin.x_ub) + (math.inf,) * pad[0])
        self.w_idx = np.concatenate([np.arange(nx)] + [nxp + nzp * k + np.r_[np.arange(nu), nu + np.arange(nx)]
                                                       for k in range(N)])
        self.p_idx = np.concatenate([np.arange(nx)] + [nxp + nzp * k + ix for k in range(N)])
        self.g_idx = np.concatenate([nxp * k + np.arange(nx) for k in range(N + 1)])
        self.n_w, self.n_p, self.n_g = self.w_idx.size, self.p_idx.size, self.g_idx.size
        self.n_w_pad, self.n_p_pad, self.n_g_pad = self.ocp.n_w_ms, self.ocp.n_p, self.ocp.n_g_ms

    @staticmethod
    def scatter(a, idx, n, fill=0.0):
        """(B, len(idx)) user array -> (B, n) kernel array, `fill` in the pad entries."""
        if a is None:
            return None
        a = np.atleast_2d(np.asarray(a, np.float64))
        out = np.full((a.shape[0], n), fill)
        out[:, idx] = a
        return np.ascontiguousarray(out)

    @staticmethod
    def gather(a, idx):
        """(B, n) kernel array -> (B, len(idx)) user array."""
        return None if a is None else np.ascontiguousarray(a[:, idx])


def state_pad(lin) -> StatePad | None:
    """The embedding a LinearOCP needs to run on a kernel instantiation, or None (native shape).
    Raises for shapes no instantiation covers (nu > 2, or nx > 4 unless (5, 1))."""
    if getattr(lin, "model", None) != "linear" or (lin.nx, lin.nu) in NATIVE_SHAPES:
        return None
    if lin.nu in (1, 2) and lin.nx < 4:
        return StatePad(lin, 4)
    raise ValueError(f"linear model ({lin.nx} states, {lin.nu} inputs): the kernel is instantiated for "
                     f"{NATIVE_SHAPES}; nx < 4 with one or two inputs is embedded in the 4-state model")


# ----------------------------------------------------------------------------
# Cart-pole set-point QP (config 5 family)
# ----------------------------------------------------------------------------

def pendulum_continuous():
    """``Inverted_pendulum/inverted_pendulum_single_shooting_mpctools.py:19-22``:
    Ac is written transposed in the script (``.T``); states (x, x', th, th'), input F."""
    Ac = np.array([[0, 0, 0, 0], [1, -10, 0, -20], [0, 9.81, 0, 39.24], [0, 0, 1, 0]], float).T
    Bc = np.array([[0.0], [1.0], [0.0], [2.0]])
    return Ac, Bc


def inverted_pendulum_qp(N=50, T=0.01, n_free=5, x_target=10.0, q=(1.2, 1.0), r_du=0.01, u_max=200.0,
                         dummy_weight=1.0):
    """The per-step QP of ``inverted_pendulum_single_shooting_mpctools.py:15-64``:
    l = (q0 (x1 - x_target))^2 + (q1 x3)^2 + (r_du Du)^2 (:51-55), |u| <= u_max (:44-46),
    Du free for the first n_free moves and 0 after (move blocking, :32-42), uprev fixed (:64).

    Augmented state x~ = (x1..x4, u_prev) (nx = 5, nu = 1); table 0 = free stage,
    table 1 = blocked stage.  P = lin.params(x~0, zr) with zr = pendulum_stage_ref(...).
    """
    Ac, Bc = pendulum_continuous()
    A, Bd = c2d(Ac, Bc, T)
    A0 = np.zeros((5, 5))
    A0[:4, :4] = A
    B0 = np.zeros((5, 1))
    B0[:4] = Bd
    B0[4, 0] = 1.0  # u_prev+ = u
    A1 = np.zeros((5, 5))
    A1[:4, :4] = A
    A1[:4, 4] = Bd[:, 0]  # applied input = u_prev (Du = 0)
    A1[4, 4] = 1.0
    B1 = np.zeros((5, 1))
    W0 = np.zeros((6, 6))
    W0[0, 0] = q[0] ** 2
    W0[2, 2] = q[1] ** 2
    r2 = r_du ** 2
    W0[4, 4] = W0[5, 5] = r2
    W0[4, 5] = W0[5, 4] = -r2  # (u - u_prev)^2
    W1 = np.zeros((6, 6))
    W1[0, 0] = q[0] ** 2
    W1[2, 2] = q[1] ** 2
    W1[5, 5] = dummy_weight  # the blocked stage's own u does not act; keep it at 0
    tab = np.array([0 if k < n_free else 1 for k in range(N)], np.int32)
    lin = LinearOCP(N=N, A=np.stack([A0, A1]), B=np.stack([B0, B1]), W=np.stack([W0, W1]), tab=tab, T=T,
                    u_lb=(-u_max,), u_ub=(u_max,), name="inverted_pendulum_qp")
    lin.x_target = x_target
    lin.A_plant, lin.B_plant = A, Bd
    return lin


def pendulum_params(lin: LinearOCP, x, u_prev=0.0):
    """P for plant states x (B, 4): x~0 = (x, u_prev), zr_k = (x_target, 0, 0, 0, 0, 0)."""
    x = np.atleast_2d(np.asarray(x, float))
    up = np.broadcast_to(np.asarray(u_prev, float), (x.shape[0],))[:, None]
    zr = np.zeros(6)
    zr[0] = lin.x_target
    return lin.params(np.concatenate([x, up], axis=1), zr)


# ----------------------------------------------------------------------------
# LTV lateral-dynamics tracking (config 4 family)
# ----------------------------------------------------------------------------

LATERAL = dict(m=1200.0, a=1.5, b=2.0, Ca=55000.0, Jz=1350.0)  # :37-41


def lateral_continuous(v, m=1200.0, a=1.5, b=2.0, Ca=55000.0, Jz=1350.0):
    """``Trajectory_tracking_dynamic_model.py:119-128`` at longitudinal speed v: states
    (y, phi, v_y, r), input delta.  A34 keeps the script's operator precedence (:120):
    (2 Ca (b - a) / m) * v - v."""
    A33 = -4 * Ca / (m * v)
    A34 = (2 * Ca * (b - a) / m * v) - v
    A43 = 2 * Ca * ((b - a) / (Jz * v))
    A44 = -2 * Ca * (a ** 2 + b ** 2) / (Jz * v)
    B31 = 2 * Ca / m
    B41 = 2 * Ca * a / Jz
    Ac = np.array([[0, v, 1, 0], [0, 0, 0, 1], [0, 0, A33, A34], [0, 0, A43, A44]], float)
    Bc = np.array([[0.0], [0.0], [B31], [B41]])
    return Ac, Bc


def lateral_references(xref, yref, vref, Delta=0.05, horizon=10, last=499, v_model=None):
    """Per-(t, k) stage references p = (y_ref, phi_ref, v_ref, r_ref, delta_ref) of
    ``Trajectory_tracking_dynamic_model.py:90-116`` for t = 0..len(vref)-1.

    As written, :107/:110/:115 read A33/A34/B31 before :119-123 define them (NameError).
    The fix applied here evaluates them at the stage's own speed vref[min(t+k, last)].
    Everything else is kept as written: phi_ref = atan2(y, x) of the path point, the
    clamping at ``last`` (veclim, :91-101), the three finite-difference cases for r_ref
    (:102-113, with par[.., t-1] = 0 at t = 0 as the zero-initialised array gives), and
    v_dot, which the script only assigns while t+k < 2 and then reuses.
    Returns par (Nsim, horizon, 5).
    """
    xref, yref, vref = (np.asarray(v, float) for v in (xref, yref, vref))
    Nsim = len(vref)
    par = np.zeros((Nsim, horizon, 5))
    v_dot = 0.0
    for t in range(Nsim):
        for k in range(horizon):
            j = min(t + k, last)
            p = np.zeros(5)
            p[0] = yref[j]
            p[1] = np.arctan2(yref[j], xref[j])
            p[2] = vref[j]
            v = vref[j] if v_model is None else v_model
            Ac, Bc = lateral_continuous(v)
            A33, A34, B31 = Ac[2, 2], Ac[2, 3], Bc[2, 0]
            prev_phi = par[t - 1, k, 1] if t > 0 else 0.0
            if t + k < 2:
                phi_plus = np.arctan2(yref[k + 1 + t], xref[k + 1 + t])
                v_dot = (vref[k + t + 1] - p[2]) / Delta
                p[3] = (phi_plus - p[1]) / Delta
            elif t + k > last - 2:
                p[3] = (p[1] - prev_phi) / Delta
            else:
                phi_plus = np.arctan2(yref[k + 1 + t], xref[k + 1 + t])
                p[3] = (phi_plus - prev_phi) / (2 * Delta)
            p[4] = (v_dot - A33 * p[2] - A34 * p[3]) / B31
            par[t, k] = p
    return par


def lateral_ltv(N=10, Delta=0.05, vref=None, Q=(1.0, 1.0, 1.0, 1.0), R=1.0, delta_max=20.0, per_instance_tab=None):
    """``Trajectory_tracking_dynamic_model.py:18-35,51-55,117-141``: one table per speed
    vref[j] (A_j, B_j = c2d(Ac(vref[j]), Bc, Delta), :134), W = diag(Q, R) (:51-52),
    |delta| <= delta_max (:34-35,62-66; Du bounds are +-inf since Ntu = Nt).  The script
    re-linearises at vref[t] for the whole horizon of step t, so instance b at step t uses
    tab[b, :] = t (per_instance_tab (B,) of step indices; default: one shared table 0)."""
    vref = np.atleast_1d(np.asarray(vref if vref is not None else [1.0], float))
    As, Bs = [], []
    for v in vref:
        Ac, Bc = lateral_continuous(v)
        A, Bd = c2d(Ac, Bc, Delta)
        As.append(A)
        Bs.append(Bd)
    W = np.diag(list(Q) + [R])
    Ws = np.broadcast_to(W, (len(vref), 5, 5)).copy()
    if per_instance_tab is None:
        tab = np.zeros(N, np.int32)
    else:
        tab = np.repeat(np.asarray(per_instance_tab, np.int32)[:, None], N, axis=1)
    return LinearOCP(N=N, A=np.stack(As), B=np.stack(Bs), W=Ws, tab=tab, T=Delta, u_lb=(-delta_max,),
                     u_ub=(delta_max,), name="lateral_ltv")


# ----------------------------------------------------------------------------
# Lateral-error LTI lane change (Trajectory Tracking/Trajectory_tracking_le_LTI.py)
# ----------------------------------------------------------------------------

def lateral_error_continuous(uref, ar=-23.55, br=61.99):
    """``Trajectory_tracking_le_LTI.py:37-42``: states (y, phi, r), input delta."""
    Ac = np.array([[0.0, uref, 0.0], [0.0, 0.0, 1.0], [0.0, 0.0, ar]])
    Bc = np.array([[0.0], [0.0], [br]])
    return Ac, Bc


def lateral_error_lti(uref, N=5, n_free=1, Delta=0.05, q=(10.0, 1.0, 0.0), r=0.01, r_du=0.0, delta_max=0.3491,
                      ar=-23.55, br=61.99, dummy_weight=1.0):
    """The per-step QP of ``Trajectory_tracking_le_LTI.py:17-79``: ZOH model of (y, phi, r) at the
    mean speed ``uref`` (:39-44), l = (x - p[:3])^T Q (x - p[:3]) + R (u - p[3])^2 + R_du Du^2
    (:58-61), |u| <= delta_max (:69-73), Du free for the first n_free = Ntu moves and 0 after
    (move blocking, :64-67), uprev = 0 (:79; the script never updates it).

    As for the cart-pole QP, Du and move blocking become an augmented state x~ = (y, phi, r, u_prev)
    (nx = 4, nu = 1): table 0 = free stage (u_prev+ = u, cost on u and u - u_prev), table 1 =
    blocked stage (applied input = u_prev, cost R (u_prev - p[3])^2, the stage's own u a dummy held
    at 0).  P = lateral_error_params(lin, x, u_prev, par_t).
    """
    Ac, Bc = lateral_error_continuous(uref, ar, br)
    A, Bd = c2d(Ac, Bc, Delta)
    Q = np.diag(np.asarray(q, float))
    A0 = np.zeros((4, 4))
    A0[:3, :3] = A
    B0 = np.zeros((4, 1))
    B0[:3] = Bd
    B0[3, 0] = 1.0  # u_prev+ = u
    A1 = np.zeros((4, 4))
    A1[:3, :3] = A
    A1[:3, 3] = Bd[:, 0]  # applied input = u_prev (Du = 0)
    A1[3, 3] = 1.0
    B1 = np.zeros((4, 1))
    W0 = np.zeros((5, 5))
    W0[:3, :3] = Q
    W0[4, 4] = r + r_du
    W0[3, 3] = r_du
    W0[3, 4] = W0[4, 3] = -r_du  # R (u - ur)^2 + R_du (u - u_prev)^2, u_prev's reference = ur
    W1 = np.zeros((5, 5))
    W1[:3, :3] = Q
    W1[3, 3] = r  # R (u_prev - ur)^2: the applied input of a blocked stage
    W1[4, 4] = dummy_weight
    tab = np.array([0 if k < n_free else 1 for k in range(N)], np.int32)
    lin = LinearOCP(N=N, A=np.stack([A0, A1]), B=np.stack([B0, B1]), W=np.stack([W0, W1]), tab=tab, T=Delta,
                    u_lb=(-delta_max,), u_ub=(delta_max,), name="lateral_error_lti")
    lin.A_plant, lin.B_plant = A, Bd
    lin.n_free = n_free
    return lin


def lateral_error_ltv(speed, N=5, n_free=1, Delta=0.05, **kw):
    """The step-t QP of ``Trjectory_tracking_le_LTV.py``: the same construction as
    :func:`lateral_error_lti` with the model rebuilt at the step's own speed c[t] (:130-136) and
    that script's weights Q = diag(5, 0, 0), R = 0, R_du = 0 (:27-35).  The closed loop re-uploads
    it every step (``solver.set_linear_model(lateral_error_ltv(c[t]))``) and sets
    x0 = the simulated state (:165-166)."""
    kw.setdefault("q", (5.0, 0.0, 0.0))
    kw.setdefault("r", 0.0)
    kw.setdefault("r_du", 0.0)
    lin = lateral_error_lti(float(speed), N=N, n_free=n_free, Delta=Delta, **kw)
    lin.name = "lateral_error_ltv"
    return lin


def lateral_error_references(xref, yref, N=5, Delta=0.05, ar=-23.55, br=61.99):
    """Per-(t, k) references p = (y_ref, phi_ref, r_ref, delta_ref) of
    ``Trajectory_tracking_le_LTI.py:104-128`` for t = 0..len(xref)-1, as written: phi_ref from the
    path's chord angle (0 at t + k = 0, the last chord past the end), r_ref and delta_ref by the
    three finite-difference cases, which read the previous step's phi_ref of the same stage
    (par[1, k, t-1]; the zero-initialised array at t = 0) and of stage k-1 (Python's index -1 =
    the last stage at k = 0).  Returns par (Nsim, N, 4)."""
    a, b = np.asarray(xref, float), np.asarray(yref, float)
    Nsim = len(a)
    par = np.zeros((Nsim, N, 4))
    chord = lambda j: np.arctan2(b[j + 1] - b[j], a[j + 1] - a[j])  # noqa: E731
    for t in range(Nsim):
        prev = par[t - 1] if t > 0 else np.zeros((N, 4))  # par[:, :, -1] is still 0 at t = 0
        for k in range(N):
            p = np.zeros(4)
            if t + k > Nsim - 1:
                p[0] = b[Nsim - 1]
                p[1] = chord(Nsim - 2)
            elif t + k == 0:
                p[0] = b[k + t]
                p[1] = 0.0
            else:
                p[0] = b[k + t]
                p[1] = chord(k + t - 1)
            if t + k < 2:
                phi_plus, phi_plus2 = chord(k + t), chord(k + t + 1)
                p[2] = (phi_plus - p[1]) / Delta
                p[3] = (((phi_plus2 - 2 * phi_plus + p[1]) / Delta ** 2) - ar * p[2]) / br
            elif t + k > Nsim - 3:
                p[2] = (p[1] - prev[k, 1]) / Delta
                p[3] = (((p[1] - 2 * prev[k, 1] + prev[k - 1, 1]) / Delta ** 2) - ar * p[2]) / br
            else:
                phi_plus = chord(k + t)
                p[2] = (phi_plus - prev[k, 1]) / (2 * Delta)
                p[3] = (((phi_plus - 2 * p[1] + prev[k, 1]) / Delta ** 2) - ar * p[2]) / br
            par[t, k] = p
    return par


def lateral_error_params(lin: LinearOCP, x, u_prev, par_t):
    """P (B, n_p) of lateral_error_lti from x (B, 3), u_prev (B,) and the step's references
    par_t (N, 4) or (B, N, 4): zr_k = (y_r, phi_r, r_r, delta_r, delta_r) on free stages (the
    u_prev slot carries delta_r so that the Du term stays u - u_prev), (y_r, phi_r, r_r, delta_r, 0)
    on blocked ones."""
    x = np.atleast_2d(np.asarray(x, float))
    Bn = x.shape[0]
    par_t = np.broadcast_to(np.asarray(par_t, float), (Bn, lin.N, 4))
    zr = np.zeros((Bn, lin.N, 5))
    zr[:, :, :4] = par_t
    free = lin.tab == 0 if lin.tab.ndim == 1 else lin.tab[0] == 0
    zr[:, free, 4] = par_t[:, free, 3]
    xt = np.concatenate([x, np.broadcast_to(np.asarray(u_prev, float), (Bn,))[:, None]], axis=1)
    return lin.params(xt, zr)
