"""CPU tests of the nonlinear ODE model variants (mpcx/ode.py, oracle/ode_ref.py).

PARITY UNPINNED (no reference outputs exist for these BASELINE-named variants).  What is pinned:
* the models' linearisations ARE the reference's matrices: the cart-pole at the upright is
  ``Inverted_pendulum/inverted_pendulum_single_shooting_mpctools.py:19-23`` (Ac, Bc) exactly, and
  the dynamic bicycle's lateral block at vx = v is the LTV model of
  ``Trajectory_tracking_dynamic_model.py:119-128`` (A34 with the intended precedence -- the
  script's as-written A34 differs by exactly its precedence slip);
* the oracle is self-consistent: its single-shooting optimum, lifted to the multiple-shooting
  layout with the adjoint states as lam_g, satisfies the multiple-shooting KKT conditions.
No GPU is touched.
"""
import math
import os

import numpy as np
import pytest

from conftest import ROOT


def _cjac(f, x, u, par):
    z = np.concatenate([x, u])
    h = 1e-30
    zc = z[None, :] + 1j * h * np.eye(len(z))
    return (f(zc[:, :len(x)], zc[:, len(x):], np.asarray(par)).imag / h).T


def test_cartpole_linearisation_is_reference_pendulum():
    from oracle import ode_ref
    from mpcx import ode, lti

    J = _cjac(ode_ref.f_cartpole, np.zeros(4), np.zeros(1), ode.CARTPOLE_PAR)
    Ac, Bc = lti.pendulum_continuous()
    assert np.array_equal(J[:, :4], Ac)
    assert np.array_equal(J[:, 4:], Bc.reshape(4, 1))


@pytest.mark.parametrize("v", [0.5, 4.0, 8.0])
def test_dyn_bicycle_linearisation_is_reference_ltv(v):
    from oracle import ode_ref
    from mpcx import ode, lti

    m, a, b, Ca, Jz = ode.DYN_BICYCLE_PAR
    J = _cjac(ode_ref.f_dyn_bicycle, np.array([0.0, 0.0, 0.0, v, 0.0, 0.0]), np.zeros(2), ode.DYN_BICYCLE_PAR)
    sel = [1, 2, 4, 5]  # (Y, psi, vy, r) = the LTV state (y, phi, v_y, r)
    Ac, Bc = lti.lateral_continuous(v)[:2]
    Ac = np.array(Ac, float)
    A34_written = Ac[2, 3]
    Ac[2, 3] = 2 * Ca * (b - a) / (m * v) - v  # intended precedence
    assert abs(A34_written - ((2 * Ca * (b - a) / m * v) - v)) < 1e-9  # the script's :120 as written
    assert np.allclose(J[np.ix_(sel, sel)], Ac, rtol=1e-13, atol=1e-12)
    assert np.allclose(J[sel, 6], np.asarray(Bc, float).reshape(-1), rtol=1e-13)
    assert np.allclose(J[:, 7], [0, 0, 0, 1, 0, 0])  # ax drives vx only


def _lane_change():
    import pandas as pd
    from mpcx import ode

    g = pd.read_csv(os.path.join(ROOT, "tests", "golden", "lane_change.csv"))
    return ode.lane_change_rows(g.x, g.y, g.uref)


def test_reference_builders():
    from mpcx import ode

    X, Y, V = _lane_change()
    r = ode.dyn_bicycle_references(X, Y, V, 490, 50)  # runs past the last row: extrapolated
    assert r.shape == (50, 8) and np.all(np.isfinite(r))
    assert np.all(r[:, 3] >= 4.0 - 1e-12) and np.all(r[:, 3] <= 8.0 + 1e-12)
    c = ode.bicycle_circular_reference([0.0, 5.0], 2, 30)
    assert c.shape == (2, 30, 5)
    assert np.allclose(np.tan(c[..., 4]) * c[..., 3] / 0.5, 0.1)  # psi' = v tan(delta)/L = 0.1


def test_odeocp_spec_and_params():
    from mpcx import ode
    from mpcx.ocp import to_spec

    ocp = ode.dynamic_bicycle_lane_change(N=20)
    s = to_spec(ocp)
    assert (s.model, s.nx, s.nu, s.M, s.N) == (4, 6, 2, 4, 20)
    assert list(s.par)[:5] == list(ode.DYN_BICYCLE_PAR)
    assert s.lbx[3] == 2.5 and s.lbx[0] == -1e20
    P = ocp.params(np.zeros((3, 6)), np.zeros((20, 8)))
    assert P.shape == (3, ocp.n_p) == (3, 6 + 8 * 20)
    cp = ode.cartpole_swingup(N=10)
    assert cp.params(np.zeros(4), [10.0, 0, 0, 0]).tolist() == [[0, 0, 0, 0, 10.0, 0, 0, 0]]
    with pytest.raises(ValueError):
        ode.OdeOCP(model="kin_bicycle", Q=(1.0, 1.0))


@pytest.mark.parametrize("which", ["kin_bicycle", "cartpole"])
def test_oracle_single_shooting_optimum_is_ms_kkt_point(which):
    from oracle import ode_ref
    from mpcx import ode

    if which == "kin_bicycle":
        ocp = ode.kinematic_bicycle_tracking(N=12)
        P = ocp.params([1.0, 0.3, math.pi / 2 + 0.2], ode.bicycle_circular_reference(3.0, 0, 12)[0])[0]
    else:
        ocp = ode.cartpole_swingup(N=20)
        P = ocp.params([0.2, 0.0, 0.3, -0.2], [1.0, 0.0, 0.0, 0.0])[0]
    pr = ode_ref.Problem(ocp)
    U, X, info = pr.solve(P)
    assert info["status"] == "converged"
    _, g, _, _ = pr.derivatives(U, P)
    # lam_g = adjoint states, lam_x(u) = -reduced gradient (nonzero only on active bounds); the
    # multiplier of g_0 is 0: interval 0 integrates from the parameter x0, so X_0 enters only g_0
    # (Casadi/multiple_shooting_casadi.py:125,157)
    nx, nu, nz, N = pr.nx, pr.nu, pr.nz, pr.N
    Z = np.concatenate([X[:-1], U], axis=1)
    Jac = pr.jac(Z)
    gl = 2 * pr.W * (Z - pr.refs(P))
    lam = np.zeros((N + 1, nx))
    for k in range(N - 1, 0, -1):
        lam[k] = gl[k, :nx] + Jac[k, :, :nx].T @ lam[k + 1]
    lam_x = np.zeros(nx + nz * N)
    for k in range(N):
        lam_x[nx + nz * k: nx + nz * k + nu] = -g.reshape(N, nu)[k]
    r, gres = pr.kkt_residual(pr.join_w(X, U), lam.reshape(-1), lam_x, P)
    assert r < 1e-9 and gres < 1e-12


def _kernel_masks():
    """NLMASK / INDEP of each ODE model as written in mpc-verde_amd/csrc/ode.h."""
    import re

    src = open(os.path.join(ROOT, "mpc-verde_amd", "csrc", "ode.h")).read()
    out = {}
    for name, model in (("KinBicycle", "kin_bicycle"), ("DynBicycle", "dyn_bicycle"), ("CartPole", "cartpole")):
        body = src[src.index(f"struct {name} {{"):]
        body = body[:body.index("};")]
        bits = {}
        for key in ("NLMASK", "INDEP"):
            expr = re.search(rf"{key} = ([^;]*);", body).group(1)
            bits[key] = {int(b) for b in re.findall(r"1u << (\d+)", expr)}
        out[model] = bits
    return out


@pytest.mark.parametrize("model", ["kin_bicycle", "dyn_bicycle", "cartpole"])
def test_kernel_hessian_passes_cover_the_curvature(model):
    """The kernel's exact Hessian of lam^T F (ode.h OdeModel::derivs) runs hyper-dual passes over
    the pairs of NLMASK variables and one diagonal pass per other variable f reads; it takes every
    other entry of d2(lam^T F)/dz2 as zero and the INDEP variables' Jacobian columns as unit
    vectors.  Check both against the oracle (complex-step Jacobians, central differences) at
    random points: a variable that enters f linearly but drives a state that enters nonlinearly
    (the bicycle's ax -> vx) must be in NLMASK, since RK4 composes f with itself."""
    from mpcx import ode
    from oracle import ode_ref

    masks = _kernel_masks()[model]
    ocp = {"kin_bicycle": ode.kinematic_bicycle_tracking, "dyn_bicycle": ode.dynamic_bicycle_lane_change,
           "cartpole": ode.cartpole_swingup}[model](N=5)
    pr = ode_ref.Problem(ocp)
    nx, nz = pr.nx, pr.nz
    rng = np.random.default_rng(3)
    for _ in range(4):
        z = rng.uniform(-0.5, 0.5, nz)
        if model == "dyn_bicycle":
            z[3] = rng.uniform(3.0, 8.0)  # vx away from 0 (1/vx)
        lam = rng.normal(size=nx)
        H = pr.hess_lam(z, lam)
        J = pr.jac(z)
        scale = max(1.0, np.abs(H).max())
        for i in range(nz):
            for j in range(i, nz):
                covered = (i in masks["NLMASK"] and j in masks["NLMASK"]) or (i == j and i not in masks["INDEP"])
                if not covered:
                    assert abs(H[i, j]) <= 1e-6 * scale, (model, i, j, H[i, j])
        for j in masks["INDEP"]:
            np.testing.assert_allclose(J[:, j], np.eye(nx)[:, j], atol=1e-12)
            assert np.abs(H[j]).max() <= 1e-6 * scale
