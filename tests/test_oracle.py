"""CPU: pin the oracles against the reference's own outputs (tests/golden).

Golden data = Casadi/1exemplo.xlsx (multiple shooting, CasADi+IPOPT) and
Casadi/2exemplo.xlsx (single shooting) decoded by tests/golden/make_golden.py.
"""
import numpy as np
import pytest

from oracle import ipm_ref, nlp_ref as R

REL_TOL = 1e-4


def rel_err(a, b):
    return float(np.max(np.abs(np.asarray(a) - np.asarray(b))) / max(float(np.max(np.abs(b))), 1e-3))


@pytest.fixture(scope="module")
def rows(golden):
    return np.array(golden["multiple_shooting"]["rows"])


def test_golden_fixture_shape(golden):
    for key in ("multiple_shooting", "single_shooting"):
        r = np.array(golden[key]["rows"])
        assert r.shape == (85, 6)
        assert np.all(r[0, 0:3] == 0) and np.allclose(r[0, 3:5], [1.0, np.pi / 4])


def test_golden_spread(golden):
    """The two reference formulations agree only to IPOPT's tolerance."""
    a = np.array(golden["multiple_shooting"]["rows"])
    b = np.array(golden["single_shooting"]["rows"])
    assert np.max(np.abs(a[:, 0:3] - b[:, 0:3])) < 3e-8
    assert np.max(np.abs(a[:, 3:5] - b[:, 3:5])) < 2e-7


def test_plant_replays_golden_exactly(rows):
    """RK4-M4 F (multiple_shooting_casadi.py:98-114) reproduces every recorded transition."""
    ocp = R.UnicycleOCP()
    xf, _ = R.F(rows[1:-1, 0:3], rows[:-2, 3:5], np.array([10.0, 10.0, 0.0]), ocp)
    assert np.max(np.abs(xf - rows[2:, 0:3])) < 1e-14


def test_numpy_oracle_golden_pairs(rows):
    """Projected-Newton single-shooting oracle reproduces the 84 IPOPT u0* (every 3rd pair)."""
    P, U0 = R.golden_pairs(rows)
    ocp = R.UnicycleOCP()
    for j in range(0, 84, 3):
        U, X, info = R.solve_single_shooting(P[j], ocp)
        assert info["status"] == "converged"
        assert rel_err(U[0], U0[j]) <= 1e-5


def test_numpy_oracle_closed_loop(rows):
    """Replay of the reference's closed loop: 84 iterations, states within IPOPT tolerance."""
    cl = R.closed_loop(R.UnicycleOCP())
    assert cl["iterations"] == 84
    assert np.max(np.abs(cl["states"][:84] - rows[1:, 0:3])) < 1e-7
    assert np.max(np.abs(cl["controls"] - rows[:84, 3:5])) < 1e-6


def test_complex_step_jacobian_vs_central_differences():
    ocp = R.UnicycleOCP()
    rng = np.random.default_rng(0)
    x, u, xr = rng.normal(size=3), rng.normal(size=2), rng.normal(size=3)
    J = R.stage_jacobian(x, u, xr, ocp)
    z = np.concatenate([x, u])
    Jfd = np.zeros((4, 5))
    for b in range(5):
        e = np.zeros(5)
        e[b] = 1e-6
        xp, qp = R.F((z + e)[0:3], (z + e)[3:5], xr, ocp)
        xm, qm = R.F((z - e)[0:3], (z - e)[3:5], xr, ocp)
        Jfd[:, b] = (np.append(xp, qp) - np.append(xm, qm)) / 2e-6
    assert np.max(np.abs(J - Jfd)) < 1e-7


def test_cpp_oracle_stage_derivatives():
    """Jet (second-order forward) derivatives of the C++ oracle vs complex step / FD-of-CS."""
    for cost in ("quadrature", "node"):
        ocp = R.UnicycleOCP(cost=cost, M=4 if cost == "quadrature" else 1)
        rng = np.random.default_rng(1)
        B = 12
        x, u, xr, lam = (rng.normal(size=(B, 3)), rng.normal(size=(B, 2)), rng.normal(size=(B, 3)),
                         rng.normal(size=(B, 3)))
        xf, qf, jac, hess = ipm_ref.stage(ocp, x, u, xr, lam=lam)
        xf2, qf2 = R.F(x, u, xr, ocp)
        assert np.max(np.abs(xf - xf2)) < 1e-13 and np.max(np.abs(qf - qf2)) < 1e-12 * max(1, np.abs(qf2).max())
        assert np.max(np.abs(jac - R.stage_jacobian(x, u, xr, ocp))) < 1e-12
        H = R.stage_hessians(x, u, xr, ocp)
        Hl = H[:, 3] + np.einsum("bc,bcij->bij", lam, H[:, 0:3])
        assert np.max(np.abs(ipm_ref.unpack_sym5(hess) - Hl)) < 1e-7


def test_cpp_oracle_golden_pairs(rows):
    """The C++ IPOPT-style IPM reproduces all 84 recorded IPOPT solves from a cold start."""
    P, U0 = R.golden_pairs(rows)
    out = ipm_ref.solve_batch(R.UnicycleOCP(), P, nthreads=4)
    assert np.all(out["status"] == 0)
    assert max(rel_err(out["w"][j, 3:5], U0[j]) for j in range(84)) <= 1e-5


def test_cpp_oracle_agrees_with_numpy_oracle_N20():
    """Two independent algorithms, same NLP and start -> same optimum (config 2 sizes)."""
    from mpcx import dist

    P = dist.config2_inputs(84, 84 + 24, with_golden=False)
    ocp = R.UnicycleOCP(N=20)
    X = np.repeat(P[:, None, 0:3], 21, axis=1)
    w0 = R.join_w(X, np.zeros((P.shape[0], 20, 2)))
    out = ipm_ref.solve_batch(ocp, P, w0=w0, nthreads=4)
    assert np.all(out["status"] == 0)
    agree = 0
    for b in range(0, P.shape[0], 3):
        w, info = R.solve_ms(P[b], ocp)
        assert info["status"] == "converged"
        agree += rel_err(out["w"][b], w) <= REL_TOL
    assert agree >= 7  # of 8 sampled; a different local optimum is possible (non-convex NLP)


def test_cpp_oracle_kkt():
    ocp = R.UnicycleOCP(N=10)
    P = np.array([[1.0, -2.0, 0.3, 10.0, 10.0, 0.0]])
    out = ipm_ref.solve_batch(ocp, P)
    pg, cv = R.kkt_residual_ms(out["w"][0], out["lam_g"][0], P[0], ocp)
    assert cv < 1e-9 and pg < 1e-5


def test_tracking_variant_node_cost():
    """mpctools tracking (Trajectory_tracking.py:51-61): RK4 M=1, node cost l(x_k,u_k,p_k)."""
    ocp = R.tracking_ocp(N=10)
    x = np.array([0.1, -0.2, 1.0])
    u = np.array([0.5, 0.3])
    p = np.array([1.0, 0.0, np.pi / 2, 1.0, 1.0])
    xf, q = R.F(x, u, p[0:3], ocp, p[3:5])
    d = x - p[0:3]
    du = u - p[3:5]
    assert abs(q - (d[0] ** 2 + d[1] ** 2 + 0.1 * d[2] ** 2 + 0.5 * du[0] ** 2 + 0.05 * du[1] ** 2)) < 1e-14
    # one RK4 step of the unicycle
    h = 0.2
    f = lambda s: np.array([u[0] * np.cos(s[2]), u[0] * np.sin(s[2]), u[1]])  # noqa: E731
    k1 = f(x)
    k2 = f(x + h / 2 * k1)
    k3 = f(x + h / 2 * k2)
    k4 = f(x + h * k3)
    assert np.max(np.abs(xf - (x + h / 6 * (k1 + 2 * k2 + 2 * k3 + k4)))) < 1e-15


def test_oracle_fixtures_regenerate():
    """tests/golden/*.npz (SURVEY.md §8(c) golden vectors) are what the pinned oracle computes."""
    import os
    import sys

    from conftest import ROOT

    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import make_oracle_fixtures as M

    rk = np.load(os.path.join(ROOT, "tests", "golden", "rk4_sens_random.npz"))
    new = M.rk4_sens_case()
    for k in ("P", "w", "c", "q", "A", "B", "gq"):
        np.testing.assert_allclose(new[k], rk[k], rtol=1e-13, atol=1e-13, err_msg=k)
    fx = np.load(os.path.join(ROOT, "tests", "golden", "unicycle_N20_oracle.npz"))
    np.testing.assert_array_equal(M.n20_inputs(), fx["P"])
    assert fx["converged"].all()
    idx = [0, 3, 11, 30]
    W, J, ok = M.n20_solve(fx["P"][idx])
    assert ok.all()
    np.testing.assert_allclose(W, fx["w"][idx], rtol=0, atol=1e-9)
    np.testing.assert_allclose(J, fx["J"][idx], rtol=1e-12)


def test_mpctools_variant_reproduces_3exemplo(golden):
    """Casadi/3exemplo.xlsx (mpctools/multiple_shooting_mpctools.py): the node-cost, RK4 M=1
    path that the tracking variant also uses.  The oracle's solves reproduce all recorded
    controls, the exact-flow plant all recorded states, and the loop stops where it did."""
    rows = np.array(golden["mpctools"]["rows"])
    ocp = R.mpctools_point_to_point_ocp()
    goal = np.array([10.0, 10.0, 0.0])

    def solve(x0):
        w, info = R.solve_ms(np.concatenate([x0, goal]), ocp)
        assert info["status"] == "converged"
        X, U = R.split_w(w, ocp.N)
        return U[0], X[1]

    xs, us = R.mpctools_closed_loop(solve)
    assert xs.shape == (rows.shape[0], 3)
    assert np.abs(us - rows[:, 3:5]).max() <= 5e-7 * np.abs(rows[:, 3:5]).max()
    # the script's plant is an ODE integrator (CVODES, tolerance ~1e-7 per step): every recorded
    # transition is the exact flow to 1e-6, and the whole trajectory stays within 5e-5
    steps = [np.abs(R.unicycle_flow(rows[t, 0:3], rows[t, 3:5], 0.2) - rows[t + 1, 0:3]).max()
             for t in range(rows.shape[0] - 1)]
    assert max(steps) <= 1e-6
    assert np.abs(xs - rows[:, 0:3]).max() <= 5e-5
    np.testing.assert_allclose(rows[:, 5], 0.2 * np.arange(rows.shape[0]), atol=1e-12)


def test_cpp_oracle_restoration_phase_recovers_failed_line_searches():
    """The C++ IPOPT restatement's soft restoration + restoration phase (W&B 2006 §3.3) on the
    cold-start instances of configs 4 (6-state bicycle) and 5 (swing-up) whose filter line
    search fails: without restoration each ends with status 3 at the recorded iteration; with it
    each converges (status 0) in the recorded number of iterations (the kernel takes the same
    counts on the swing-up, tests/test_gpu_resto.py) to a KKT point of the NLP."""
    import mpcx
    from mpcx import dist as mdist
    from oracle import ode_ref

    ipm_ref.lib()
    t0, x0, (X, Y, V) = mdist.config4_bicycle_inputs(0, 1024)
    ocp4 = mpcx.dynamic_bicycle_lane_change(N=50)
    idx4 = [262, 483, 10]
    refs = np.stack([mpcx.ode.dyn_bicycle_references(X, Y, V, int(t0[b]), 50).reshape(-1) for b in idx4])
    P4 = ocp4.params(x0[idx4], refs)
    ocp5 = mpcx.cartpole_swingup(N=100)
    idx5 = [313, 12, 74, 396]
    P5 = mdist.config5_swingup_inputs(0, 2048)[idx5]
    for ocp, P, fail_at, iters in ((ocp4, P4, [28, 30, 33], [54, 73, 92]), (ocp5, P5, [8, 7, 8, 16], [22, 21, 20, 35])):
        off = ipm_ref.solve(ocp, P, restoration=0, max_iter=3000)
        assert off["status"].tolist() == [3] * len(P) and off["iters"].tolist() == fail_at, (off["status"], off["iters"])
        on = ipm_ref.solve(ocp, P, max_iter=3000)
        assert on["status"].tolist() == [0] * len(P) and on["iters"].tolist() == iters, (on["status"], on["iters"])
        pr = ode_ref.Problem(ocp)
        for b in range(len(P)):
            kkt, gres = pr.kkt_residual(on["w"][b], on["lam_g"][b], on["lam_x"][b], P[b])
            assert kkt <= 1e-6 and gres <= 1e-8, (ocp.model, b, kkt, gres)
