"""CPU tests of the linear-model family.

* the pendulum oracle (oracle/nlp_ref.py pendulum_*) reproduces the reference's own
  closed loop ``Inverted_pendulum/invertpend_data_py.xlsx`` (tests/golden/pendulum_N50_golden.json);
* the product's host-side tables (mpcx/lti.py: c2d, u_prev augmentation, move blocking)
  give, through the generic LQ oracle, the same optimum as the pinned pendulum oracle;
* the LTV lateral builder's references follow the script's as-written rules.
No GPU is touched.
"""
import json
import os

import numpy as np
import pytest

from conftest import ROOT


@pytest.fixture(scope="module")
def pend_golden():
    with open(os.path.join(ROOT, "tests", "golden", "pendulum_N50_golden.json")) as f:
        return np.array(json.load(f)["rows"])


def test_pendulum_oracle_closed_loop_matches_golden(pend_golden):
    from oracle import nlp_ref as R

    xs, us = R.pendulum_closed_loop(nsim=1000)
    assert pend_golden.shape == (1001, 6)
    assert np.abs(xs - pend_golden[:, 0:4]).max() <= 1e-9
    assert np.abs(us - pend_golden[:1000, 4]).max() <= 1e-8 * np.abs(pend_golden[:, 4]).max()
    assert abs(us[0] - (-60.84425718936204)) < 1e-9


def test_pendulum_tables_match_pinned_oracle():
    from oracle import nlp_ref as R
    from mpcx import lti

    lin = lti.inverted_pendulum_qp()
    A, Bd = R.pendulum_model()
    np.testing.assert_array_equal(lin.A_plant, A)
    np.testing.assert_array_equal(lin.B_plant, Bd)
    assert lin.nx == 5 and lin.nu == 1 and lin.n_tab == 2 and list(lin.tab[:6]) == [0, 0, 0, 0, 0, 1]
    rng = np.random.default_rng(3)
    for scale in (1.0, 30.0):  # 30: bounds |u| <= 200 active
        x = scale * rng.uniform([-1, -.5, -.2, -.5], [1, .5, .2, .5])
        up = float(rng.uniform(-50, 50))
        u_ref = R.pendulum_qp_solve(x, A, Bd, uprev=up)
        P = lti.pendulum_params(lin, x, up)[0]
        X, U, _ = R.lq_solve(P[:5], lin.A, lin.B, lin.c, lin.W, lin.tab, P[5:].reshape(50, 6), [-200], [200])
        assert np.abs(U[:5, 0] - u_ref).max() <= 1e-9 * max(1.0, np.abs(u_ref).max())
        assert np.abs(U[5:, 0]).max() <= 1e-9  # blocked stages' dummy input
        assert np.abs(X[5:, 4] - u_ref[4]).max() <= 1e-9 * max(1.0, abs(u_ref[4]))  # u_prev carries u_4
        if scale > 1:
            assert np.any(np.abs(u_ref) >= 200 - 1e-9)


def test_pack_sym_matches_symix():
    from mpcx import lti

    n = 6
    W = np.arange(n * n, dtype=float).reshape(n, n)
    W = W + W.T
    p = lti.pack_sym(W)

    def symix(i, j):
        if i > j:
            i, j = j, i
        return i * n - i * (i - 1) // 2 + (j - i)

    for i in range(n):
        for j in range(n):
            assert p[symix(i, j)] == W[i, j]


def test_lateral_ltv_builder_and_refs():
    from mpcx import lti
    import csv

    with open(os.path.join(ROOT, "tests", "golden", "lane_change.csv")) as f:
        rows = [tuple(float(v) for v in r.values()) for r in csv.DictReader(f)]
    xr, yr, vr = (np.array(c) for c in zip(*rows))
    assert len(vr) == 500
    par = lti.lateral_references(xr, yr, vr, Delta=0.05, horizon=10)
    assert par.shape == (500, 10, 5) and np.all(np.isfinite(par))
    # clamp at veclim = 499 (:94-97)
    np.testing.assert_array_equal(par[495, 9, 0:3], [yr[499], np.arctan2(yr[499], xr[499]), vr[499]])
    # centred difference in the interior (:112-113)
    t, k = 10, 3
    assert par[t, k, 3] == pytest.approx((np.arctan2(yr[k + 1 + t], xr[k + 1 + t]) - par[t - 1, k, 1]) / 0.1)
    lin = lti.lateral_ltv(N=10, Delta=0.05, vref=vr[:3], per_instance_tab=[0, 1, 2, 2])
    assert lin.tab.shape == (4, 10) and lin.n_tab == 3
    Ac, Bc = lti.lateral_continuous(vr[1])
    A, Bd = lti.c2d(Ac, Bc, 0.05)
    np.testing.assert_allclose(lin.A[1], A, rtol=0, atol=0)
    # ZOH: A = expm(Ac T) satisfies the semigroup property
    A2, _ = lti.c2d(Ac, Bc, 0.1)
    np.testing.assert_allclose(A @ A, A2, rtol=1e-10, atol=1e-12)


def test_linear_to_spec():
    from mpcx import lti, ocp, _lib

    lin = lti.inverted_pendulum_qp()
    s = ocp.to_spec(lin, max_iter=100, tol=1e-9)
    assert (s.model, s.nx, s.nu, s.N, s.param_layout) == (_lib.MODEL_LINEAR, 5, 1, 50, _lib.P_X0_STAGEREF)
    assert (s.lbu[0], s.ubu[0]) == (-200.0, 200.0)
    assert s.lbx[0] == -1e20 and s.ubx[4] == 1e20
    assert lin.n_p == 5 + 6 * 50


def test_box_qp_matches_active_set_enumeration():
    """oracle.box_qp (the LQ oracles' QP solve) vs brute force over all 3^n active sets."""
    import itertools

    from oracle import nlp_ref as R

    rng = np.random.default_rng(7)
    for trial in range(20):
        n = 6
        M = rng.normal(size=(n, n))
        H = M @ M.T + 0.05 * np.eye(n)
        g0 = 3.0 * rng.normal(size=n)
        lb, ub = -np.ones(n), np.ones(n)
        u = R.box_qp(H, g0, lb, ub)
        best = None
        for sides in itertools.product((-1, 0, 1), repeat=n):
            s = np.array(sides)
            fr = s == 0
            v = np.where(s < 0, lb, np.where(s > 0, ub, 0.0))
            if fr.any():
                v[fr] = np.linalg.solve(H[np.ix_(fr, fr)], -(g0[fr] + H[np.ix_(fr, ~fr)] @ v[~fr]))
            if np.any(v < lb - 1e-12) or np.any(v > ub + 1e-12):
                continue
            f = 0.5 * v @ H @ v + g0 @ v
            if best is None or f < best[0]:
                best = (f, v)
        np.testing.assert_allclose(u, best[1], rtol=0, atol=1e-9, err_msg=str(trial))


def _random_lin(rng, nx, nu=1, n_tab=3, N=12, B=None, umax=1.0):
    from mpcx import lti

    nz = nx + nu
    As, Bs, cs, Ws = [], [], [], []
    for _ in range(n_tab):
        A = rng.normal(size=(nx, nx))
        As.append(0.95 * A / max(abs(np.linalg.eigvals(A))))
        Bs.append(rng.normal(size=(nx, nu)))
        cs.append(0.1 * rng.normal(size=nx))
        M = rng.normal(size=(nz, nz))
        Ws.append(M @ M.T / nz + 0.1 * np.eye(nz))
    tab = rng.integers(0, n_tab, size=(N,) if B is None else (B, N)).astype(np.int32)
    return lti.LinearOCP(N=N, A=np.stack(As), B=np.stack(Bs), c=np.stack(cs), W=np.stack(Ws), tab=tab,
                         u_lb=(-umax,) * nu, u_ub=(umax,) * nu)


@pytest.mark.parametrize("nx,nu", [(1, 1), (2, 1), (3, 1), (2, 2), (3, 2)])
def test_state_pad_embedding_same_optimum(nx, nu):
    """lti.StatePad (nx < 4, nu = 1 solved as the 4-state kernel model): the padded QP has the
    unpadded QP's optimum (LQ oracle on both, bounds active), the pad states stay 0, and the
    index maps round-trip every layout (w, P, g) with the pad entries where the kernel reads them."""
    from mpcx import lti
    from oracle import nlp_ref as R

    rng = np.random.default_rng(10 + nx + 7 * nu)
    lin = _random_lin(rng, nx, nu=nu, N=12)
    pd = lti.state_pad(lin)
    assert isinstance(pd, lti.StatePad) and pd.ocp.nx == 4 and pd.ocp.nu == nu
    nzp = 4 + nu
    assert (pd.n_w, pd.n_p, pd.n_g) == (lin.n_w_ms, lin.n_p, lin.n_g_ms)
    assert (pd.n_w_pad, pd.n_p_pad, pd.n_g_pad) == (4 + nzp * 12, 4 + nzp * 12, 4 * 13)
    assert np.all(np.isinf(pd.ocp.x_lb[nx:])) and np.all(np.isinf(pd.ocp.x_ub[nx:]))
    n_active = 0
    for b in range(6):
        x0 = 3.0 * rng.normal(size=nx)
        zr = rng.normal(size=(lin.N, nx + nu))
        P = lin.params(x0, zr)
        Pp = pd.scatter(P, pd.p_idx, pd.n_p_pad)
        x0p, zrp = Pp[0, :4], Pp[0, 4:].reshape(lin.N, nzp)
        assert np.all(x0p[nx:] == 0) and np.all(zrp[:, nx:4] == 0)
        lo, hi = [-1.0] * nu, [1.0] * nu
        X, U, J = R.lq_solve(x0, lin.A, lin.B, lin.c, lin.W, lin.tab, zr, lo, hi)
        Xp, Up, Jp = R.lq_solve(x0p, pd.ocp.A, pd.ocp.B, pd.ocp.c, pd.ocp.W, pd.ocp.tab, zrp, lo, hi)
        np.testing.assert_allclose(Up, U, rtol=0, atol=1e-10)
        np.testing.assert_allclose(Xp[:, :nx], X, rtol=0, atol=1e-10)
        assert np.all(Xp[:, nx:] == 0)
        assert abs(Jp - J) <= 1e-10 * max(1.0, abs(J))
        n_active += int(np.any(np.abs(U) >= 1 - 1e-9))
        # w layout: user [X_0 | U_k X_{k+1}] -> padded and back
        w = np.concatenate([X[0]] + [np.concatenate([U[k], X[k + 1]]) for k in range(lin.N)])[None, :]
        wp = pd.scatter(w, pd.w_idx, pd.n_w_pad)
        wp_ref = np.concatenate([Xp[0]] + [np.concatenate([Up[k], Xp[k + 1]]) for k in range(lin.N)])
        np.testing.assert_allclose(wp[0], wp_ref, rtol=0, atol=1e-10)
        np.testing.assert_array_equal(pd.gather(wp, pd.w_idx), w)
    assert n_active >= 2
    g = np.arange(pd.n_g, dtype=float)[None, :] + 1
    gp = pd.scatter(g, pd.g_idx, pd.n_g_pad)
    assert np.count_nonzero(gp) == pd.n_g and np.all(gp.reshape(lin.N + 1, 4)[:, nx:] == 0)


def test_state_pad_shapes():
    from mpcx import lti

    rng = np.random.default_rng(3)
    for nx, nu in ((4, 1), (5, 1), (4, 2)):
        assert lti.state_pad(_random_lin(rng, nx, nu=nu)) is None
    for nx, nu in ((5, 2), (6, 1), (2, 3)):
        with pytest.raises(ValueError, match="instantiated"):
            lti.state_pad(_random_lin(rng, nx, nu=nu))


def _lane_change():
    import csv

    with open(os.path.join(ROOT, "tests", "golden", "lane_change.csv")) as f:
        rows = list(csv.DictReader(f))
    return tuple(np.array([float(r[c]) for r in rows]) for c in ("x", "y", "uref"))


def test_lateral_error_lti_tables_match_scalar_oracle():
    """Trajectory_tracking_le_LTI.py: the augmented-state tables (Du, move blocking with Ntu = 1)
    give, through the generic LQ oracle, the same u_0 as the script's QP restated as a scalar QP
    (oracle.nlp_ref.lateral_error_solve), along the 500 closed-loop steps of lane_change.csv with the
    script's references; x_{t+1} is the solver's predicted x_1 (solver.fixvar, :145)."""
    from mpcx import lti
    from oracle import nlp_ref as R

    a, b, c = _lane_change()
    lin = lti.lateral_error_lti(c.mean())
    par = lti.lateral_error_references(a, b, N=lin.N)
    assert par.shape == (500, 5, 4) and par[0, 0, 1] == 0.0
    x = np.zeros(3)
    n_sat = 0
    for t in range(500):
        u_ref, x1 = R.lateral_error_solve(x, lin.A_plant, lin.B_plant, par[t])
        P = lti.lateral_error_params(lin, x, 0.0, par[t])[0]
        xt0, zr = P[:4], P[4:].reshape(lin.N, 5)
        X, U, _ = R.lq_solve(xt0, lin.A, lin.B, lin.c, lin.W, lin.tab, zr, [-0.3491], [0.3491])
        assert abs(U[0, 0] - u_ref) <= 1e-9 * max(1.0, abs(u_ref)), t
        np.testing.assert_allclose(X[1, :3], x1, rtol=0, atol=1e-12)
        np.testing.assert_allclose(X[1:, 3], u_ref, rtol=0, atol=1e-9)  # u_prev carries u_0 (blocked moves)
        n_sat += abs(u_ref) >= 0.3491 - 1e-12
        x = x1
    assert np.max(np.abs(par[:, :, 0])) > 1.0  # a lane change is tracked
    assert abs(x[0] - par[-1, 0, 0]) < 0.2 * par[-1, 0, 0]  # and followed (final y 2.91 vs 2.77)
