"""GPU parity tests: the HIP path (through the C ABI / ctypes façade) vs the oracles.

Oracles: oracle/nlp_ref.py (NumPy, projected Newton, complex-step derivatives)
and oracle/libipm_ref.so (C++ IPOPT-style IPM, jet derivatives); both pinned
to the reference's CasADi+IPOPT outputs (tests/golden).  Tolerances follow
SURVEY.md §4 / BASELINE.json: solution error <= 1e-4 relative to
max(||u||_inf, 1e-3) against IPOPT; kernel-level outputs <= 1e-12 relative.
"""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REL_TOL = 1e-4  # north_star: optimal (x*, u*) within 1e-4 relative of CasADi/IPOPT
# An instance whose optimum differs from the same-algorithm C++ oracle's is certified instead:
# complex-step KKT residual (projected Lagrangian gradient, defects) of the returned point
# at most KKT_CERT_TOL, objective no worse than the oracle's.  The counts of such instances
# are bounded per test and printed (run with -s).  Measured on MI355X (round 2): every bound
# below is met with 0 differing instances, so each is 0.
KKT_CERT_TOL = 1e-8
MAX_CONFIG2_MISMATCH = 0  # of 1024 config-2 instances
MAX_HORIZON_MISMATCH = {}  # N -> allowed certified mismatches in test_horizons (none)
MAX_FIXTURE_MISMATCH = 0  # of the 32 committed N=20 oracle optima (independent algorithm)
MAX_ITER_MISMATCH = 0  # iteration counts vs the C++ IPOPT restatement, of 1024, cold and warm
MAX_TRACKING_MISMATCH = 0  # of the 4096 config-3 tracking instances (round 3)


def rel_err(a, b):
    a = np.asarray(a)
    b = np.asarray(b)
    return float(np.max(np.abs(a - b)) / max(float(np.max(np.abs(b))), 1e-3))


@pytest.fixture(scope="module")
def mpcx():
    import mpcx as m

    m._lib.load()
    return m


@pytest.fixture(scope="module")
def R():
    from oracle import nlp_ref

    return nlp_ref


@pytest.fixture(scope="module")
def C():
    from oracle import ipm_ref

    ipm_ref.lib()
    return ipm_ref


def config2_batch(B=1024, seed=20261015, golden_rows=None):
    """SURVEY.md §8(d) config 2 inputs: instances 0..83 = golden P_j, rest random."""
    from oracle import nlp_ref

    rng = np.random.default_rng(seed)
    P = np.zeros((B, 6))
    P[:, 3:6] = (10.0, 10.0, 0.0)
    n0 = 0
    if golden_rows is not None:
        Pg, _ = nlp_ref.golden_pairs(golden_rows)
        n0 = min(B, Pg.shape[0])
        P[:n0] = Pg[:n0]
    P[n0:, 0:2] = rng.uniform(-5, 5, size=(B - n0, 2))
    P[n0:, 2] = rng.uniform(-np.pi / 2, np.pi / 2, size=B - n0)
    return P


# ----------------------------------------------------------------------------- kernel level
def test_rk4_sens_matches_oracle(mpcx, R):
    """Sweep kernel outputs (defect, q, A, B, grad q) vs complex-step oracle, <= 1e-12."""
    ocp = mpcx.unicycle_point_to_point(N=20)
    solver = mpcx.nlpsol("s", "mi355x", ocp)
    rng = np.random.default_rng(1)
    B = 37
    P = np.zeros((B, 6))
    P[:, 0:3] = rng.normal(size=(B, 3)) * 3
    P[:, 3:6] = rng.normal(size=(B, 3)) * 5
    w = rng.normal(size=(B, solver.n_w))
    w[:, 3::5] = rng.uniform(-1, 1, size=(B, 20))
    out = solver.rk4_sens(w, P)
    rocp = R.UnicycleOCP(N=20)
    X, U = R.split_w(w, 20)
    xr = np.broadcast_to(P[:, None, 3:6], (B, 20, 3))
    xf, qf = R.F(X[:, :-1], U, xr, rocp)
    jac = R.stage_jacobian(X[:, :-1], U, xr, rocp)
    scale = lambda a: max(1.0, float(np.max(np.abs(a))))  # noqa: E731
    assert np.max(np.abs(out["c"] - (xf - X[:, 1:]))) <= 1e-12 * scale(xf)
    assert np.max(np.abs(out["q"] - qf)) <= 1e-12 * scale(qf)
    assert np.max(np.abs(out["A"] - jac[..., 0:3, 0:3])) <= 1e-12 * scale(jac)
    assert np.max(np.abs(out["B"] - jac[..., 0:3, 3:5])) <= 1e-12 * scale(jac)
    assert np.max(np.abs(out["gq"] - jac[..., 3, :])) <= 1e-12 * scale(jac[..., 3, :])


def test_plant_replays_golden_closed_loop(mpcx, R, golden):
    """F (plant kernel) reproduces the 83 recorded state transitions of 1exemplo.xlsx."""
    rows = np.array(golden["multiple_shooting"]["rows"])
    F = mpcx.integrator(mpcx.unicycle_point_to_point(N=10))
    P = np.zeros((rows.shape[0] - 2, 6))
    P[:, 0:3] = rows[1:-1, 0:3]
    P[:, 3:6] = (10, 10, 0)
    xf, _ = F.batch(P, rows[:-2, 3:5])
    assert np.max(np.abs(xf - rows[2:, 0:3])) < 1e-12
    # CasADi call shapes
    out = F(P[0], rows[0, 3:5])
    assert out[0].shape == (3, 1) and out[1].shape == (1, 1)
    d = F(x0=P[0], p=rows[0, 3:5])
    assert set(d) == {"xf", "qf"}


# ----------------------------------------------------------------------------- golden (IPOPT) pins
def test_golden_pairs_cold_start(mpcx, R, golden):
    """All 84 recorded IPOPT solves (P_j -> u0*_j, N=10) in ONE batch, cold start."""
    rows = np.array(golden["multiple_shooting"]["rows"])
    P, U0 = R.golden_pairs(rows)
    solver = mpcx.nlpsol("s", "mi355x", mpcx.unicycle_point_to_point(N=10))
    r = solver.solve_batch(P)
    assert np.all(r["status"] == 0), np.bincount(r["status"])
    u0 = r["w"][:, 3:5]
    errs = [rel_err(u0[j], U0[j]) for j in range(len(U0))]
    assert max(errs) <= REL_TOL, max(errs)


def test_casadi_call_shapes_and_closed_loop(mpcx, R, golden):
    """The reference's driver loop (Casadi/multiple_shooting_casadi.py:224-298), with
    ca.nlpsol swapped for mpcx.nlpsol, reproduces 1exemplo.xlsx: 84 iterations."""
    rows = np.array(golden["multiple_shooting"]["rows"])
    N, T = 10, 0.2
    ocp = mpcx.unicycle_point_to_point(N=N)
    solver = mpcx.nlpsol("solver", "mi355x", ocp, {"ipopt": {"max_iter": 2000, "print_level": 0,
                                                                "acceptable_tol": 1e-8,
                                                                "acceptable_obj_change_tol": 1e-6},
                                                    "print_time": 0})
    F = mpcx.integrator(ocp)
    lbw = [-math.inf] * 3
    ubw = [math.inf] * 3
    for _ in range(N):
        lbw += [-1, -math.pi / 4, -math.inf, -math.inf, -math.inf]
        ubw += [1, math.pi / 4, math.inf, math.inf, math.inf]
    args = {"lbg": [0] * (3 * (N + 1)), "ubg": [0] * (3 * (N + 1)), "lbx": lbw, "ubx": ubw}
    state_init = np.array([0.0, 0.0, 0.0])
    state_target = np.array([10.0, 10.0, 0.0])
    w0 = [0.0] * (3 + 5 * N)
    mpc_iter = 0
    t0 = 0.0
    states, controls = [], []
    log = mpcx.ClosedLoopLog.for_ocp(ocp, state_init)  # cat_states / cat_controls / t (:210-270)
    while np.linalg.norm(state_init - state_target) > 1e-1 and mpc_iter * T < 20:
        args["p"] = np.concatenate([state_init, state_target])
        sol = solver(x0=w0, lbx=args["lbx"], ubx=args["ubx"], lbg=args["lbg"], ubg=args["ubg"], p=args["p"])
        assert sol["x"].shape == (3 + 5 * N, 1) and sol["g"].shape == (3 * (N + 1), 1)
        assert solver.stats()["success"]
        u = np.array([sol["x"][3 + 5 * k:5 + 5 * k, 0] for k in range(N)]).T  # (2, N)
        X0 = np.array([sol["x"][0:3, 0]] + [sol["x"][5 + 5 * k:8 + 5 * k, 0] for k in range(N)]).T
        states.append(state_init.copy())
        controls.append(u[:, 0].copy())
        log.record(sol["x"], t0)
        t0 += T
        state_init = F(args["p"], u[:, 0])[0].reshape(-1)
        u0 = np.hstack([u[:, 1:], u[:, -1:]])
        X0 = np.hstack([X0[:, 1:], X0[:, -1:]])
        w0 = np.concatenate([X0.T.reshape(-1), u0.T.reshape(-1)])  # the reference's stacked layout (:284-287)
        mpc_iter += 1
    assert mpc_iter == 84
    states = np.array(states)
    controls = np.array(controls)
    assert np.max(np.abs(states - rows[1:85, 0:3])) < 1e-6
    assert rel_err(controls, rows[0:84, 3:5]) <= REL_TOL
    # the loop stops exactly where the reference's did: the state fed to the last solve
    # (row 84) is still > 0.1 away from the target, the state after it is not
    assert np.linalg.norm(states[-1] - state_target) > 1e-1 >= np.linalg.norm(state_init - state_target)
    # the exported table (:316-334) equals 1exemplo.xlsx row for row
    tab = log.table()
    got = np.stack([tab[c] for c in ("x", "y", "theta", "v", "w", "t")], axis=1)
    assert log.cat_states.shape == (3, N + 1, 85)
    assert np.max(np.abs(got[:, 0:3] - rows[:, 0:3])) < 1e-6
    assert rel_err(got[:, 3:5], rows[:, 3:5]) <= REL_TOL
    np.testing.assert_allclose(got[:, 5], rows[:, 5], atol=1e-12)


# ----------------------------------------------------------------------------- oracle parity at scale
def test_config2_batch_vs_cpp_oracle(mpcx, R, C, golden):
    """Config 2 (N=20, B=1024): GPU solve vs the C++ IPM oracle on identical inputs
    and initial guess; the golden instances also vs IPOPT-pinned numpy optimum."""
    rows = np.array(golden["multiple_shooting"]["rows"])
    P = config2_batch(1024, golden_rows=rows)
    ocp = mpcx.unicycle_point_to_point(N=20)
    solver = mpcx.nlpsol("s", "mi355x", ocp)
    r = solver.solve_batch(P)
    assert np.all(r["status"] == 0), np.bincount(r["status"], minlength=4)
    rocp = R.UnicycleOCP(N=20)
    X = np.repeat(P[:, None, 0:3], 21, axis=1)
    w0 = R.join_w(X, np.zeros((1024, 20, 2)))
    ref = C.solve_batch(rocp, P, w0=w0, nthreads=0)
    assert np.all(ref["status"] == 0)
    errs = np.array([rel_err(r["w"][b], ref["w"][b]) for b in range(1024)])
    # same algorithm, same start: the same local optimum for every instance.  An instance
    # that differs is reported by count and must be certified: a KKT point of the NLP
    # (complex-step Lagrangian gradient projected on the bounds, and the defects) whose
    # objective is no worse than the oracle's.
    diff = np.flatnonzero(errs > REL_TOL)
    print(f"config 2: {diff.size} of 1024 instances differ from the C++ oracle by > {REL_TOL:g}")
    assert diff.size <= MAX_CONFIG2_MISMATCH, (diff.size, np.sort(errs)[-10:])
    for b in diff:
        pg, cv = R.kkt_residual_ms(r["w"][b], r["lam_g"][b], P[b], rocp)
        assert pg <= KKT_CERT_TOL and cv <= KKT_CERT_TOL, (b, pg, cv)
        assert r["f"][b] <= ref["f"][b] * (1 + 1e-9), (b, r["f"][b], ref["f"][b])
    # independent numpy oracle on a sample (projected Newton, single shooting)
    for b in list(range(0, 84, 12)) + list(range(84, 1024, 157)):
        wn, info = R.solve_ms(P[b], rocp)
        assert info["status"] == "converged"
        if abs(info["J"] - r["f"][b]) <= 1e-6 * max(1.0, abs(info["J"])):
            assert rel_err(r["w"][b], wn) <= REL_TOL


def test_kkt_residual_at_solution(mpcx, R):
    """First-order optimality of the returned (w, lam_g) for the NLP (complex-step check)."""
    ocp = mpcx.unicycle_point_to_point(N=20)
    solver = mpcx.nlpsol("s", "mi355x", ocp)
    P = config2_batch(8, seed=3)
    r = solver.solve_batch(P)
    rocp = R.UnicycleOCP(N=20)
    for b in range(8):
        pg, cv = R.kkt_residual_ms(r["w"][b], r["lam_g"][b], P[b], rocp)
        assert cv < 1e-9
        assert pg < 1e-5


def test_interval0_integrates_from_parameter(mpcx, R, C):
    """Interval 0 as the script formulates it: Xk = P[:3] (:125) and F(x0=vertcat(Xk, P[3:]),
    p=U_0) (:157), so the lifted X_0 enters only g_0 = P[:3] - X_0 (:128-136) and CasADi's
    lam_g[0:3] is 0.  Cold start (X_0 = P[:3]): lam_g[0:3] exactly 0.  From guesses whose X_0 is
    NOT P[:3] (X_0 moved by up to 0.5, the shifted guess of the previous step's solution): the
    same optimum, lam_g[0:3] = 0 to the dual tolerance, g = F(P[:3], U_0) - X_1 at the solution,
    and the C++ oracle (same formulation) takes the same iteration counts from the same guess."""
    N, B = 20, 256
    ocp = mpcx.unicycle_point_to_point(N=N)
    solver = mpcx.nlpsol("s", "mi355x", ocp, {"ipopt": {"max_iter": 2000, "acceptable_tol": 1e-8,
                                                        "acceptable_obj_change_tol": 1e-6}})
    P = config2_batch(B, seed=11)
    cold = solver.solve_batch(P, want_g=True)
    assert np.all(cold["status"] == 0)
    assert np.all(cold["lam_g"][:, 0:3] == 0.0), np.abs(cold["lam_g"][:, 0:3]).max()
    w0 = cold["w"].copy()
    w0[:, 0:3] += np.random.default_rng(4).uniform(-0.5, 0.5, (B, 3))
    r = solver.solve_batch(P, w0=w0, want_g=True)
    assert np.all(r["status"] <= 1)
    assert np.max(np.abs(r["lam_g"][:, 0:3])) <= 1e-8
    assert np.max(np.abs(r["g"])) <= 1e-9
    errs = np.array([rel_err(r["w"][b], cold["w"][b]) for b in range(B)])
    assert errs.max() <= 1e-5, errs.max()  # the same optimum to the solve tolerance (measured 1.2e-6)
    # the constraint values returned are g_1 = F(P[:3], U_0) - X_1 (not F(X_0, U_0) - X_1)
    xf, _ = R.F(P[:, 0:3], r["w"][:, 3:5], P[:, 3:6], R.UnicycleOCP(N=N))
    np.testing.assert_allclose(r["g"][:, 3:6], xf - r["w"][:, 5:8], atol=1e-12)
    ref = C.solve(R.UnicycleOCP(N=N), P, w0=w0, nthreads=0, max_iter=2000, acceptable_tol=1e-8,
                  acceptable_obj_change_tol=1e-6)
    n_it = int(np.sum(ref["iters"] != r["iters"]))
    print(f"interval 0 from x0: {n_it} of {B} iteration counts differ from the C++ oracle (X_0 != x0 guesses)")
    assert n_it == 0, np.flatnonzero(ref["iters"] != r["iters"])
    assert np.max(np.abs(ref["lam_g"][:, 0:3])) <= 1e-8


def _interval0_case(mpcx, name):
    """(ocp, P, nx) of one non-config-2 kernel path for the interval-0 test below."""
    from mpcx import dist as mdist
    from mpcx import lti

    if name == "c3_unicycle_scan":  # UnicycleScanModel (Riccati scan from N = 25), state bounds
        _, P = mdist.config3_inputs(0, 256, N=30)
        return mpcx.unicycle_tracking(N=30), P, 3
    if name == "kin_bicycle_scan":  # OdeModel<KinBicycle>, Riccati scan
        _, P = mdist.config3_bicycle_inputs(0, 256, N=30)
        return mpcx.kinematic_bicycle_tracking(N=30), P, 3
    if name == "swingup_two_waves":  # OdeModel<CartPole>, N = 100: two-wave groups (G = 128)
        return mpcx.cartpole_swingup(N=100), mdist.config5_swingup_inputs(0, 128), 4
    if name == "linear4_scan":  # LinearModel<4,1> (kScan: table Jacobians, Riccati scan), config 4's tables
        t0, x0, par = mdist.config4_inputs(0, 256, N=50)
        _, _, vref = mdist.lane_change()
        ocp = mpcx.lateral_ltv(N=50, Delta=0.05, vref=vref, per_instance_tab=np.minimum(t0, 499))
        return ocp, ocp.params(x0, par[np.minimum(t0, 499)]), 4
    if name == "pendulum_qp_two_waves":  # LinearModel<5,1>, G = 128, decoupled suffix
        lin = lti.inverted_pendulum_qp(N=100)
        return lin, lti.pendulum_params(lin, mdist.config5_inputs(0, 256), 0.0), 5
    raise ValueError(name)


@pytest.mark.parametrize("name", ["c3_unicycle_scan", "kin_bicycle_scan", "swingup_two_waves", "linear4_scan",
                                  "pendulum_qp_two_waves"])
def test_interval0_from_parameter_other_paths(mpcx, C, name):
    """The interval-0 formulation (X_0 enters only g_0 = x0 - X_0) on the kernel paths the
    config-2 test above does not take: the Riccati scans (unicycle N = 30, kinematic bicycle,
    LinearModel<4,1>), the two-wave groups of N = 100 (swing-up ODE, cart-pole QP with the
    decoupled suffix).  From guesses whose X_0 is moved off x0 by up to 0.5: every status <= 1,
    lam_g[0:nx] = 0 to the dual tolerance; the ODE/unicycle paths take the C++ oracle's iteration
    counts from the same guesses and reach its optima; the QPs reach the cold solve's (unique) optimum."""
    ocp, P, nx = _interval0_case(mpcx, name)
    B = P.shape[0]
    solver = mpcx.nlpsol("s", "mi355x", ocp, {"ipopt": {"max_iter": 3000}})
    cold = solver.solve_batch(P)
    assert np.all(cold["status"] <= 1), np.unique(cold["status"], return_counts=True)
    w0 = cold["w"].copy()
    w0[:, 0:nx] += np.random.default_rng(5).uniform(-0.5, 0.5, (B, nx))
    r = solver.solve_batch(P, w0=w0)
    assert np.all(r["status"] <= 1), np.unique(r["status"], return_counts=True)
    lam0 = float(np.max(np.abs(r["lam_g"][:, 0:nx])))
    print(f"{name}: max |lam_g[0:{nx}]| = {lam0:.1e}")
    assert lam0 <= 1e-8
    if name.startswith(("linear", "pendulum")):
        errs = np.array([rel_err(r["w"][b], cold["w"][b]) for b in range(B)])
        assert errs.max() <= 1e-6, errs.max()
        return
    ref = C.solve(ocp, P, w0=w0, nthreads=0, max_iter=3000)
    assert np.all(ref["status"] <= 1)
    n_it = int(np.sum(ref["iters"] != r["iters"]))
    errs = np.array([rel_err(r["w"][b], ref["w"][b]) for b in range(B)])
    print(f"{name}: {n_it} of {B} iteration counts differ from the C++ oracle (X_0 != x0 guesses), "
          f"max optimum difference {errs.max():.1e}")
    assert n_it == 0, np.flatnonzero(ref["iters"] != r["iters"])
    assert errs.max() <= 1e-6, errs.max()


# ----------------------------------------------------------------------------- edge cases
@pytest.mark.parametrize("B", [1, 2, 3, 31, 33, 65])
def test_ragged_batch_sizes(mpcx, R, B):
    ocp = mpcx.unicycle_point_to_point(N=20)
    solver = mpcx.nlpsol("s", "mi355x", ocp)
    P = config2_batch(65, seed=7)[:B]
    r = solver.solve_batch(P)
    full = solver.solve_batch(config2_batch(65, seed=7))
    assert np.array_equal(r["w"], full["w"][:B])  # instances are independent: bitwise identical


def test_empty_batch(mpcx):
    solver = mpcx.nlpsol("s", "mi355x", mpcx.unicycle_point_to_point(N=10))
    r = solver.solve_batch(np.zeros((0, 6)))
    assert r["w"].shape == (0, 53)


@pytest.mark.parametrize("N", [1, 2, 15, 16, 31, 32, 50, 63, 64, 100, 127, 128, 200, 255])
def test_horizons(mpcx, C, R, N):
    ocp = mpcx.unicycle_point_to_point(N=N)
    solver = mpcx.nlpsol("s", "mi355x", ocp)
    P = config2_batch(16, seed=N)
    r = solver.solve_batch(P)
    rocp = R.UnicycleOCP(N=N)
    X = np.repeat(P[:, None, 0:3], N + 1, axis=1)
    ref = C.solve_batch(rocp, P, w0=R.join_w(X, np.zeros((16, N, 2))))
    assert np.all(r["status"] == 0) and np.all(ref["status"] == 0)
    errs = np.array([rel_err(r["w"][b], ref["w"][b]) for b in range(16)])
    diff = np.flatnonzero(errs > REL_TOL)
    print(f"N={N}: {diff.size} of 16 instances differ from the C++ oracle by > {REL_TOL:g}")
    for b in diff:  # certified: a KKT point no worse than the oracle's
        pg, cv = R.kkt_residual_ms(r["w"][b], r["lam_g"][b], P[b], rocp)
        print(f"  instance {b}: err {errs[b]:.2e} kkt {pg:.2e} cv {cv:.2e} f {r['f'][b]:.12g} oracle {ref['f'][b]:.12g}")
        assert pg <= KKT_CERT_TOL and cv <= KKT_CERT_TOL, (b, pg, cv)
        assert r["f"][b] <= ref["f"][b] * (1 + 1e-9), (b, r["f"][b], ref["f"][b])
    assert diff.size <= MAX_HORIZON_MISMATCH.get(N, 0), diff


@pytest.mark.parametrize("N,B", [(10, 40), (20, 37), (40, 9), (100, 5)])
def test_group_policy_same_results(mpcx, N, B):
    """Lane-group widening (spec.group_policy 0, the default: up to one instance per wave while
    SIMDs would idle) and the narrowest group (policy 1: 4/2 instances per wave at N=10/20) give
    the same bits.  Widening a 16-lane group (N = 10) or running one multi-wave group adds exact
    zeros / neutral values to every reduction.  A 32-lane group widened to a wave (N = 20) runs
    replicated (kernels.h R = 2), its replicas splitting the stage evaluation's RK4 substeps; the
    narrow 32-lane group sums the quadrature moments in the same two halves (models.h
    stage_derivs), so it too gives the same bits.  Policy 1 is also how the narrow-group code
    paths stay covered at test batch sizes."""
    ocp = mpcx.unicycle_point_to_point(N=N)
    P = config2_batch(B, seed=N + 1)
    s0 = mpcx.nlpsol("s", "mi355x", ocp)
    s1 = mpcx.nlpsol("s", "mi355x", ocp, {"group_policy": 1})
    if N == 20:  # the two policies do run different kernels here
        assert s0._h.launch_shape(B)[:2] == (32, 2) and s1._h.launch_shape(B)[:2] == (32, 1)
    r0, r1 = s0.solve_batch(P), s1.solve_batch(P)
    assert np.all(r0["status"] == 0)
    for n in ("w", "f", "lam_g", "lam_x", "status", "iters"):
        np.testing.assert_array_equal(r0[n], r1[n], err_msg=n)


def test_launch_shape_names_the_kernel(mpcx):
    """mpcx_launch_shape reports the instantiation a launch runs (what bench.py looks up in the
    PMC record and rocprofv3 prints): config 2's 1024 instances on a 1024-SIMD MI355X run
    replicated 32-lane groups, one more instance tips the batch to the narrow groups."""
    import torch

    n_simd = 4 * torch.cuda.get_device_properties(0).multi_processor_count
    h = mpcx.nlpsol("s", "mi355x", mpcx.unicycle_point_to_point(N=20))._h
    Bw = n_simd  # the largest batch that still widens 32-lane groups (B * 32 * 2 <= 64 * n_simd)
    assert h.launch_shape(Bw) == (32, 2, "void mpcx::solve_kernel<mpcx::UnicycleFreeModel, 32, false, 2>"
                                        "(mpcx::SolveArgs)")
    assert h.launch_shape(Bw + 1)[:2] == (32, 1)
    h10 = mpcx.nlpsol("s", "mi355x", mpcx.unicycle_point_to_point(N=10))._h
    assert h10.launch_shape(16)[:2] == (64, 1) and h10.launch_shape(100 * n_simd)[:2] == (16, 1)
    # a 16-lane group is never widened to exactly 32 lanes (models.h stage_derivs: the 32-lane kernel
    # sums the evaluation in the replicas' halves)
    assert h10.launch_shape(n_simd)[:2] == (64, 1) and h10.launch_shape(n_simd + 1)[:2] == (16, 1)
    assert h10.launch_shape(2 * n_simd)[:2] == (16, 1)
    h30 = mpcx.nlpsol("s", "mi355x", mpcx.unicycle_point_to_point(N=30))._h  # scan model: never replicated
    assert h30.launch_shape(16) == (64, 1, "void mpcx::solve_kernel<mpcx::UnicycleScanModel, 64, false, 1>"
                                          "(mpcx::SolveArgs)")
    hp = mpcx.nlpsol("s", "mi355x", mpcx.inverted_pendulum_qp(N=100))._h
    assert hp.launch_shape(2048) == (128, 1, "void mpcx::solve_kernel<mpcx::LinearModel<5, 1>, 128, false, 1>"
                                             "(mpcx::SolveArgs)")


def test_instance_bits_do_not_depend_on_the_batch(mpcx):
    """SURVEY.md §4 item 5 at the group-variant boundary: the same config-2 instances solved in a
    batch of n_simd (1024 on MI355X: replicated 32-lane groups), inside a batch of 2 n_simd (narrow
    groups) and inside n_simd + 1 (just across the widening threshold) give identical w, f, lambda,
    statuses and iteration counts -- cold, and warm-started from the shifted solution."""
    import torch

    import bench
    from mpcx import dist

    n_simd = 4 * torch.cuda.get_device_properties(0).multi_processor_count
    N, B = 20, n_simd
    solver = mpcx.nlpsol("s", "mi355x", mpcx.unicycle_point_to_point(N=N))
    assert solver._h.launch_shape(B)[1] == 2 and solver._h.launch_shape(B + 1)[1] == 1
    P2 = dist.config2_inputs(0, 2 * B)
    r_rep = solver.solve_batch(P2[:B])
    for Bb in (2 * B, B + 1):
        r_nar = solver.solve_batch(P2[:Bb])
        for n in ("w", "f", "lam_g", "lam_x", "status", "iters"):
            np.testing.assert_array_equal(r_rep[n], r_nar[n][:B], err_msg=f"{n} (B={Bb})")
    # one warm-started closed-loop step later (IPOPT warm_start_init_point from shifted multipliers)
    rn = solver.solve_batch(P2)
    w0, l0, lx0 = bench.shift_np(rn["w"], N), bench.shift_lam_np(rn["lam_g"], N), bench.shift_lamx_np(rn["lam_x"], N)
    Pn = P2.copy()
    Pn[:, 0:3] = rn["w"][:, 3 + 2:3 + 2 + 3]  # x0 <- the predicted X_1
    wa = solver.solve_batch(Pn[:B], w0=w0[:B], lam_g0=l0[:B], lam_x0=lx0[:B])
    wb = solver.solve_batch(Pn, w0=w0, lam_g0=l0, lam_x0=lx0)
    for n in ("w", "f", "lam_g", "lam_x", "status", "iters"):
        np.testing.assert_array_equal(wa[n], wb[n][:B], err_msg=f"warm {n}")


def test_instance_bits_do_not_depend_on_the_batch_short_horizon(mpcx):
    """The same at N = 10 (16-lane groups): one instance per wave (B <= n_simd, 64 lanes), the
    batches between n_simd and 2 n_simd (which once ran an unreplicated 32-lane kernel that sums the
    evaluation in two halves) and four instances per wave give identical bits."""
    import torch

    from mpcx import dist

    n_simd = 4 * torch.cuda.get_device_properties(0).multi_processor_count
    N, B = 10, n_simd
    solver = mpcx.nlpsol("s", "mi355x", mpcx.unicycle_point_to_point(N=N))
    P2 = dist.config2_inputs(0, 3 * B)
    r_w = solver.solve_batch(P2[:B])
    for Bb in (B + 1, 2 * B, 3 * B):
        r_n = solver.solve_batch(P2[:Bb])
        for n in ("w", "f", "lam_g", "lam_x", "status", "iters"):
            np.testing.assert_array_equal(r_w[n], r_n[n][:B], err_msg=f"{n} (B={Bb})")


def test_max_iter_status(mpcx):
    ocp = mpcx.unicycle_point_to_point(N=10)
    solver = mpcx.nlpsol("s", "mi355x", ocp, {"ipopt": {"max_iter": 2}})
    r = solver.solve_batch(config2_batch(4, seed=1))
    assert np.all(r["status"] == 2) and np.all(r["iters"] == 2)


def test_invalid_arguments(mpcx):
    solver = mpcx.nlpsol("s", "mi355x", mpcx.unicycle_point_to_point(N=10))
    with pytest.raises(ValueError):
        solver(p=[0, 0, 0, 10, 10, 0], lbg=[-1] * 33, ubg=[1] * 33)
    with pytest.raises(ValueError):
        solver.solve_batch(np.zeros((2, 5)))
    with pytest.raises(ValueError):
        mpcx.nlpsol("s", "ipopt", mpcx.unicycle_point_to_point(N=10))
    for n_bad in (0, 256):
        bad = mpcx.unicycle_point_to_point(N=10)
        bad.N = n_bad
        with pytest.raises(mpcx._lib.MpcxError):
            mpcx.nlpsol("s", "mi355x", bad)
    # buffers the library would read or write past their end are rejected before the call
    P = np.zeros((2, 6))
    with pytest.raises(ValueError):
        solver.solve_batch(P, lbw=np.zeros(10))
    with pytest.raises(ValueError):
        mpcx.integrator(mpcx.unicycle_point_to_point(N=10)).batch(np.zeros((2, 5)), np.zeros((2, 2)))
    with pytest.raises(ValueError):
        solver.rk4_sens(np.zeros((2, 40)), P)
    import torch
    from mpcx.device import DeviceLoop

    loop = DeviceLoop(solver, P + [0, 0, 0, 10, 10, 0])
    with pytest.raises(ValueError):  # too short
        loop.step(status_out=torch.zeros(1, dtype=torch.int32, device=loop.device))
    with pytest.raises(TypeError):  # wrong dtype
        loop.step(iters_out=torch.zeros(2, dtype=torch.int64, device=loop.device))
    with pytest.raises(ValueError):  # host memory
        loop.run(2, Pseq=torch.zeros((2, 2, 6), dtype=torch.float64))
    with pytest.raises(ValueError):
        loop.set_stage_refs(torch.zeros((2, 2), dtype=torch.float64, device=loop.device))
    loop.step()
    torch.cuda.synchronize()
    assert np.all(loop.status.cpu().numpy() == 0)


def test_single_shooting_formulation(mpcx, R, golden):
    """Config 1 plumbing: single_shooting_v2.py's NLP (decision = U) at P=[0,0,0,10,10,0]:
    u0* = golden row 0 of 2exemplo.xlsx."""
    rows2 = np.array(golden["single_shooting"]["rows"])
    N = 10
    ocp = mpcx.unicycle_point_to_point(N=N, formulation="single_shooting")
    solver = mpcx.nlpsol("solver", "mi355x", ocp)
    lbw, ubw = [], []
    for _ in range(N):
        lbw += [-1, -math.pi / 4]
        ubw += [1, math.pi / 4]
    sol = solver(x0=[0] * (2 * N), lbx=lbw, ubx=ubw, lbg=-math.inf, ubg=math.inf, p=[0, 0, 0, 10, 10, 0])
    assert sol["x"].shape == (2 * N, 1) and sol["g"].shape == (2 * N, 1)
    assert rel_err(sol["x"][0:2, 0], rows2[0, 3:5]) <= REL_TOL


def test_single_shooting_closed_loop_2exemplo(mpcx, golden):
    """The reference's single-shooting driver loop (Casadi/single_shooting_v2.py:201-266) with
    ca.nlpsol swapped for mpcx.nlpsol(formulation='single_shooting'): the U-only warm start
    shifted each step (:245-249), the plant F (:242), the predicted rollout (:221-224); it
    reproduces 2exemplo.xlsx -- 84 solves, states < 1e-6, controls <= 1e-4 relative -- and the
    export table of :284-301 row for row."""
    rows = np.array(golden["single_shooting"]["rows"])
    N, T = 10, 0.2
    ocp = mpcx.unicycle_point_to_point(N=N, formulation="single_shooting")
    solver = mpcx.nlpsol("solver", "mi355x", ocp, {"ipopt": {"max_iter": 2000, "print_level": 0,
                                                                "acceptable_tol": 1e-8,
                                                                "acceptable_obj_change_tol": 1e-6},
                                                    "print_time": 0})
    F = mpcx.integrator(mpcx.unicycle_point_to_point(N=N))
    lbw, ubw = [], []
    for _ in range(N):
        lbw += [-1, -math.pi / 4]
        ubw += [1, math.pi / 4]
    args = {"lbg": -math.inf, "ubg": math.inf, "lbx": lbw, "ubx": ubw}
    state_init = np.array([0.0, 0.0, 0.0])
    state_target = np.array([10.0, 10.0, 0.0])
    w0 = [0.0] * (2 * N)
    log = mpcx.ClosedLoopLog.for_ocp(mpcx.unicycle_point_to_point(N=N), state_init)
    mpc_iter, t0 = 0, 0.0
    states, controls = [], []
    while np.linalg.norm(state_init - state_target) > 1e-1 and mpc_iter * T < 20:
        args["p"] = np.concatenate([state_init, state_target])
        sol = solver(x0=w0, lbx=args["lbx"], ubx=args["ubx"], lbg=args["lbg"], ubg=args["ubg"], p=args["p"])
        assert sol["x"].shape == (2 * N, 1) and solver.stats()["success"]
        u = sol["x"][:, 0].reshape(N, 2).T  # ca.reshape(sol['x'], n_controls, N)
        X1, Xs = state_init, [state_init]
        for k in range(N):  # predicted rollout X1 = F([X1; target], u[:, k])[0]
            X1 = F(np.concatenate([X1, state_target]), u[:, k])[0].reshape(-1)
            Xs.append(X1)
        w_ms = np.concatenate([Xs[0]] + [np.concatenate([u[:, k], Xs[k + 1]]) for k in range(N)])
        log.record(w_ms, t0)
        states.append(state_init.copy())
        controls.append(u[:, 0].copy())
        t0 += T
        state_init = F(args["p"], u[:, 0])[0].reshape(-1)
        w0 = np.hstack([u[:, 1:], u[:, -1:]]).T.reshape(-1)  # ca.reshape(u0, n_controls*N, 1)
        mpc_iter += 1
    assert mpc_iter == 84
    states, controls = np.array(states), np.array(controls)
    assert np.max(np.abs(states - rows[1:85, 0:3])) < 1e-6
    assert rel_err(controls, rows[0:84, 3:5]) <= REL_TOL
    tab = log.table()
    got = np.stack([tab[c] for c in ("x", "y", "theta", "v", "w", "t")], axis=1)
    assert got.shape == rows.shape
    assert np.max(np.abs(got[:, 0:3] - rows[:, 0:3])) < 1e-6
    assert rel_err(got[:, 3:5], rows[:, 3:5]) <= REL_TOL
    np.testing.assert_allclose(got[:, 5], rows[:, 5], atol=1e-12)


# ----------------------------------------------------------------------------- warm start
def test_warm_start_multipliers(mpcx, R):
    """IPOPT-style warm start (lam_g0, lam_x0): same optimum, fewer iterations; lam_x
    from the solver agrees with the stationarity reconstruction from the sweep kernel."""
    ocp = mpcx.unicycle_point_to_point(N=20)
    solver = mpcx.nlpsol("s", "mi355x", ocp)
    P = config2_batch(64, seed=11)
    cold = solver.solve_batch(P)
    assert np.all(cold["status"] == 0)
    lx = solver.lam_x_from_kkt(cold["w"], P, cold["lam_g"])
    assert np.max(np.abs(lx - cold["lam_x"])) <= 1e-6 * max(1.0, np.max(np.abs(lx)))
    warm = solver.solve_batch(P, w0=cold["w"], lam_g0=cold["lam_g"], lam_x0=cold["lam_x"])
    assert np.all(warm["status"] == 0)
    assert max(rel_err(warm["w"][b], cold["w"][b]) for b in range(64)) <= 1e-6
    assert warm["iters"].mean() < cold["iters"].mean()


def test_device_loop_warm_matches_cold(mpcx, R, C):
    """Closed loop on the device (solve + plant/shift kernels): the warm-dual loop and the
    cold-dual loop follow the same trajectory, and the C++ oracle's warm loop agrees."""
    import torch
    import bench
    from mpcx import dist
    from mpcx.device import DeviceLoop

    ocp = mpcx.unicycle_point_to_point(N=20)
    solver = mpcx.nlpsol("s", "mi355x", ocp)
    P0 = dist.config2_inputs(0, 128)
    loops = [DeviceLoop(solver, P0, warm_duals=wd) for wd in (True, False)]
    for _ in range(6):
        for lp in loops:
            lp.step()
    torch.cuda.synchronize()
    Pw, Pc = (lp.P.cpu().numpy() for lp in loops)
    assert np.max(np.abs(Pw - Pc)) < 1e-6
    assert np.all(loops[0].status.cpu().numpy() == 0)
    # oracle loop with the same warm start
    rocp = R.UnicycleOCP(N=20)
    P = P0.copy()
    w0 = bench._cold(P, 20, R)
    lam0 = lamx0 = None
    for s in range(6):
        if s == 0:
            r = C.solve_batch(rocp, P, w0=w0)
            r["lam_x"] = np.zeros_like(r["w"])
        else:
            r = C.solve_batch_warm(rocp, P, w0, lam0=lam0, lamx0=lamx0, mu_init=1e-4, bound_push=1e-4,
                                   mult_push=1e-4)
        P[:, 0:3], _ = R.F(P[:, 0:3], r["w"][:, 3:5], P[:, 3:6], rocp)
        w0, lam0, lamx0 = bench.shift_np(r["w"], 20), bench.shift_lam_np(r["lam_g"], 20), \
            bench.shift_lamx_np(r["lam_x"], 20)
    assert np.max(np.abs(P - Pw)) < 1e-6


# ----------------------------------------------------------------------------- tracking (config 3 family)
def test_tracking_vs_oracles(mpcx, R, C):
    """Trajectory_tracking.py's NLP (RK4 M=1, node cost, per-stage reference p_k, state
    bounds) on the bench's own config-3 batch (N=30, B=4096, dist.config3_inputs): GPU vs the
    C++ IPM oracle (same tol) instance by instance -- every differing optimum counted, KKT-
    certified and no worse than the oracle's -- and vs the independent numpy oracle (tight tol;
    state bounds verified inactive there)."""
    from mpcx import dist

    N, B = 30, 4096
    tau0, P = dist.config3_inputs(0, B, N=N)
    ocp = mpcx.unicycle_tracking(N=N)
    solver = mpcx.nlpsol("trk", "mi355x", ocp)
    r = solver.solve_batch(P)
    assert np.all(r["status"] == 0), np.bincount(r["status"], minlength=4)
    rocp = R.tracking_ocp(N=N)
    x0 = P[:, 0:3]
    ps = P[:, 3:].reshape(B, N, 5)
    X = np.repeat(x0[:, None], N + 1, axis=1)
    ref = C.solve_batch(rocp, x0, w0=R.join_w(X, np.zeros((B, N, 2))), pstage=ps)
    assert np.all(ref["status"] == 0)
    errs = np.array([rel_err(r["w"][b], ref["w"][b]) for b in range(B)])
    diff = np.flatnonzero(errs > REL_TOL)
    n_it = int(np.sum(r["iters"] != ref["iters"]))
    print(f"config 3 tracking: {diff.size} of {B} instances differ from the C++ oracle by > {REL_TOL:g} "
          f"(max {errs.max():.2e}); {n_it} iteration counts differ")
    assert diff.size <= MAX_TRACKING_MISMATCH, (diff, np.sort(errs)[-5:])
    for b in diff:
        pg, cv = R.kkt_residual_ms(r["w"][b], r["lam_g"][b], x0[b], rocp, pstage=ps[b])
        assert pg <= KKT_CERT_TOL and cv <= KKT_CERT_TOL, (b, pg, cv)
        assert r["f"][b] <= ref["f"][b] * (1 + 1e-9), (b, r["f"][b], ref["f"][b])
    tight = mpcx.nlpsol("trk", "mi355x", ocp, {"ipopt": {"tol": 1e-11}}).solve_batch(P[::32])
    for i, b in enumerate(range(0, B, 32)):
        U, Xs, info = R.solve_single_shooting(x0[b], rocp, pstage=ps[b])
        assert info["status"] == "converged"
        assert np.all(np.abs(Xs[:, 1]) < 2.0) and np.all(np.abs(Xs[:, 0]) < 20.0)  # state bounds inactive
        assert rel_err(tight["w"][i], R.join_w(Xs, U)) <= 1e-5


def test_tracking_state_bounds_active(mpcx, C, R):
    """Tracking with an active y-bound: a reference pulled outside y in [-2, 2]."""
    N, B = 10, 16
    ocp = mpcx.unicycle_tracking(N=N)
    rng = np.random.default_rng(5)
    x0 = np.zeros((B, 3))
    x0[:, 1] = rng.uniform(0.5, 1.5, B)
    x0[:, 2] = np.pi / 2
    ps = np.zeros((B, N, 5))
    ps[:, :, 1] = 4.0  # y_ref beyond the bound y <= 2
    ps[:, :, 2] = np.pi / 2
    ps[:, :, 3] = 1.0
    P = np.concatenate([x0, ps.reshape(B, -1)], axis=1)
    r = mpcx.nlpsol("trk", "mi355x", ocp).solve_batch(P)
    assert np.all(r["status"] == 0)
    X, U = R.split_w(r["w"], N)
    assert np.all(X[:, 1:, 1] <= 2.0 + 1e-9) and np.max(X[:, 1:, 1]) > 2.0 - 1e-4  # bound reached, honoured
    ref = C.solve_batch(R.tracking_ocp(N=N), x0, w0=R.join_w(np.repeat(x0[:, None], N + 1, 1), np.zeros((B, N, 2))),
                        pstage=ps)
    assert max(rel_err(r["w"][b], ref["w"][b]) for b in range(B)) <= REL_TOL


def test_tracking_closed_loop_facade(mpcx, C, R):
    """Trajectory_tracking.py's receding-horizon loop (per-step references, shift of the
    guess, plant) through the façade for 30 steps: follows the C++ oracle loop."""
    N, steps = 10, 30
    ocp = mpcx.unicycle_tracking(N=N)
    solver = mpcx.nlpsol("trk", "mi355x", ocp)
    F = mpcx.integrator(ocp)
    rocp = R.tracking_ocp(N=N)
    x = np.zeros(3)
    xo = np.zeros(3)
    w0 = None
    w0o = R.join_w(np.zeros((1, N + 1, 3)), np.zeros((1, N, 2)))
    for t in range(steps):
        p = mpcx.ocp.circular_reference(0.0, t, N)[0]
        sol = solver(x0=w0, p=np.concatenate([x, p.reshape(-1)]), lbx=solver_bounds(ocp)[0], ubx=solver_bounds(ocp)[1])
        w = sol["x"][:, 0]
        x = F(np.concatenate([x, p.reshape(-1)]), w[3:5])[0][:, 0]
        w0 = np.concatenate([w[5:8], np.concatenate([w[3 + 5 * k:8 + 5 * k] for k in range(1, N)]), w[-5:]])
        ro = C.solve_batch(rocp, xo[None], w0=w0o, pstage=p[None])
        xo = R.F(xo, ro["w"][0, 3:5], p[0, 0:3], rocp, p[0, 3:5])[0]
        wo = ro["w"][0]
        w0o = np.concatenate([wo[5:8], wo[8:3 + 5 * N], wo[-5:]])[None]
    assert np.max(np.abs(x - xo)) < 1e-5


def solver_bounds(ocp):
    from oracle import nlp_ref

    lb, ub = nlp_ref.ms_bounds(nlp_ref.tracking_ocp(N=ocp.N))
    return lb, ub


@pytest.mark.parametrize("N,B", [(20, 200), (100, 24)])
def test_fused_step_matches_solve_then_shift(mpcx, N, B):
    """mpcx_step_dev (solve + plant/shift fused in one kernel, updated in place) gives
    bit-identical P, warm start and multipliers to mpcx_solve_batch_dev + mpcx_shift_dev,
    over several closed-loop steps (N = 100: multi-wave groups, LDS handoff of node k+1)."""
    import torch
    from mpcx import dist
    from mpcx.device import DeviceLoop

    solver = mpcx.nlpsol("s", "mi355x", mpcx.unicycle_point_to_point(N=N))
    P0 = dist.config2_inputs(0, B)
    fused, split = DeviceLoop(solver, P0), DeviceLoop(solver, P0)
    for _ in range(4):
        fused.step()
        split.solve()
        split.shift()
        torch.cuda.synchronize()
        for name in ("P", "w", "w0", "lam", "lam0", "lamx", "lamx0", "f", "status", "iters"):
            a, b = getattr(fused, name).cpu().numpy(), getattr(split, name).cpu().numpy()
            np.testing.assert_array_equal(a, b, err_msg=name)


def test_integration_stub_runs():
    """INTEGRATION.md §5 (the raw ctypes binding a maintainer would add) runs verbatim in a
    fresh process and prints the golden u0* = (1, pi/4)."""
    import os
    import re
    import subprocess
    import sys

    from conftest import ROOT, PKG

    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = text[text.index("## 5."):]
    code = re.search(r"```python\n(.*?)```", sec, re.S).group(1)
    env = dict(os.environ, MPCX_LIB=os.path.join(PKG, "mpcx", "libmpcx.so"))
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    u = [float(v) for v in out.stdout.strip().strip("[]").split()]
    assert abs(u[0] - 1.0) < 1e-6 and abs(u[1] - math.pi / 4) < 1e-6


# ----------------------------------------------------------------------------- committed golden vectors
def test_rk4_sens_vs_committed_fixture(mpcx):
    """Sweep kernel vs tests/golden/rk4_sens_random.npz (oracle outputs), <= 1e-12."""
    import os

    from conftest import ROOT

    fx = np.load(os.path.join(ROOT, "tests", "golden", "rk4_sens_random.npz"))
    solver = mpcx.nlpsol("s", "mi355x", mpcx.unicycle_point_to_point(N=20))
    out = solver.rk4_sens(fx["w"], fx["P"])
    for k in ("c", "q", "A", "B", "gq"):
        scale = max(1.0, float(np.max(np.abs(fx[k]))))
        assert np.max(np.abs(out[k] - fx[k])) <= 1e-12 * scale, k


def test_n20_vs_committed_oracle_optima(mpcx):
    """Config-2-shaped instances (N=20) vs tests/golden/unicycle_N20_oracle.npz: the
    independent oracle's optima from the same cold start, within 1e-4 relative."""
    import os

    from conftest import ROOT

    from oracle import nlp_ref

    fx = np.load(os.path.join(ROOT, "tests", "golden", "unicycle_N20_oracle.npz"))
    solver = mpcx.nlpsol("s", "mi355x", mpcx.unicycle_point_to_point(N=20))
    r = solver.solve_batch(fx["P"])
    assert np.all(r["status"] == 0)
    B = len(fx["J"])
    errs = np.array([rel_err(r["w"][b], fx["w"][b]) for b in range(B)])
    diff = np.flatnonzero(errs > REL_TOL)
    print(f"N=20 fixture: {diff.size} of {B} instances differ from the committed oracle optima by > {REL_TOL:g}")
    rocp = nlp_ref.UnicycleOCP(N=20)
    for b in diff:  # non-convex NLP, independent algorithm: certified KKT point instead
        pg, cv = nlp_ref.kkt_residual_ms(r["w"][b], r["lam_g"][b], fx["P"][b], rocp)
        print(f"  instance {b}: err {errs[b]:.2e} kkt {pg:.2e} cv {cv:.2e} f {r['f'][b]:.12g} oracle {fx['J'][b]:.12g}")
        assert pg <= KKT_CERT_TOL and cv <= KKT_CERT_TOL, (b, pg, cv)
    assert diff.size <= MAX_FIXTURE_MISMATCH, diff


def test_rk4_sens_ragged_tiles(mpcx):
    """B not a multiple of the 64-instance tile (partial last tile) and B > 64: every
    instance's outputs equal those of the same instance solved alone (bit-identical)."""
    import os

    from conftest import ROOT

    fx = np.load(os.path.join(ROOT, "tests", "golden", "rk4_sens_random.npz"))
    solver = mpcx.nlpsol("s", "mi355x", mpcx.unicycle_point_to_point(N=20))
    w = np.concatenate([fx["w"]] * 3)  # B = 111: tiles of 64 + 47
    P = np.concatenate([fx["P"]] * 3)
    big = solver.rk4_sens(w, P)
    one = solver.rk4_sens(fx["w"][5:6], fx["P"][5:6])
    for k in ("c", "q", "A", "B", "gq"):
        for b in (5, 42, 79):
            np.testing.assert_array_equal(big[k][b], one[k][0], err_msg=k)


# ----------------------------------------------------------------------------- multi-step launches
def _state(lp):
    return {n: getattr(lp, n).cpu().numpy() for n in ("P", "w", "w0", "lam", "lam0", "lamx", "lamx0", "f")}


@pytest.mark.parametrize("N,B,K,warm_duals", [(20, 200, 6, True), (20, 64, 4, False), (100, 24, 3, True)])
def test_run_equals_lockstep_steps(mpcx, N, B, K, warm_duals):
    """mpcx_run_dev (K closed-loop steps in one launch, instances not waiting for each
    other) == K mpcx_step_dev launches, bit for bit: states, per-step status and iterations."""
    import torch
    from mpcx import dist
    from mpcx.device import DeviceLoop

    solver = mpcx.nlpsol("s", "mi355x", mpcx.unicycle_point_to_point(N=N))
    P0 = dist.config2_inputs(0, B)
    lock = DeviceLoop(solver, P0, warm_duals=warm_duals)
    run = DeviceLoop(solver, P0, warm_duals=warm_duals)
    st_l, it_l = [], []
    for _ in range(K):
        lock.step()
        torch.cuda.synchronize()
        st_l.append(lock.status.cpu().numpy().copy())
        it_l.append(lock.iters.cpu().numpy().copy())
    st_r, it_r = run.run(K)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(st_r.cpu().numpy(), np.array(st_l))
    np.testing.assert_array_equal(it_r.cpu().numpy(), np.array(it_l))
    a, b = _state(lock), _state(run)
    for n in a:
        np.testing.assert_array_equal(b[n], a[n], err_msg=n)
    # a second multi-step launch continues the same trajectory
    run.run(2)
    for _ in range(2):
        lock.step()
    torch.cuda.synchronize()
    np.testing.assert_array_equal(run.P.cpu().numpy(), lock.P.cpu().numpy())


def test_run_tracking_with_stage_reference_sequence(mpcx):
    """Config-3 tracking: per-step references through Pseq == set_stage_refs + step()."""
    import torch
    from mpcx import dist
    from mpcx.device import DeviceLoop

    N, B, K = 30, 64, 5
    tau0, P0 = dist.config3_inputs(0, B, N=N)
    solver = mpcx.nlpsol("t", "mi355x", mpcx.unicycle_tracking(N=N))
    refs = np.stack([mpcx.ocp.circular_reference(tau0, t, N).reshape(B, -1) for t in range(K)])
    Pseq = np.zeros((K, B, P0.shape[1]))
    Pseq[:, :, 3:] = refs
    lock = DeviceLoop(solver, P0)
    run = DeviceLoop(solver, P0)
    dr = torch.from_numpy(refs).cuda()
    st_l = []
    for t in range(K):
        lock.set_stage_refs(dr[t])
        lock.step()
        torch.cuda.synchronize()
        st_l.append(lock.iters.cpu().numpy().copy())
    _, it_r = run.run(K, Pseq=torch.from_numpy(Pseq).cuda())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(it_r.cpu().numpy(), np.array(st_l))
    a, b = _state(lock), _state(run)
    for n in ("w", "w0", "lam0", "lamx0", "f"):
        np.testing.assert_array_equal(b[n], a[n], err_msg=n)
    np.testing.assert_array_equal(b["P"][:, 0:3], a["P"][:, 0:3])  # x0 (run keeps step-0 refs in P)


def test_run_ragged_last_wave_with_reference_sequence(mpcx):
    """Multi-step launch whose last wave holds lanes of no instance (narrowest groups: 4 instances
    per wave at N = 10, B = 37): those lanes are done from the start and must neither write a
    status row nor read per-step references past the batch -- run == lock-step, bit for bit."""
    import torch
    from mpcx import dist
    from mpcx.device import DeviceLoop

    N, B, K = 10, 37, 4
    tau0, P0 = dist.config3_inputs(0, B, N=N)
    solver = mpcx.nlpsol("t", "mi355x", mpcx.unicycle_tracking(N=N), {"group_policy": 1})
    refs = np.stack([mpcx.ocp.circular_reference(tau0, t, N).reshape(B, -1) for t in range(K)])
    Pseq = np.zeros((K, B, P0.shape[1]))
    Pseq[:, :, 3:] = refs
    lock = DeviceLoop(solver, P0)
    run = DeviceLoop(solver, P0)
    dr = torch.from_numpy(refs).cuda()
    st_l, it_l = [], []
    for t in range(K):
        lock.set_stage_refs(dr[t])
        lock.step()
        torch.cuda.synchronize()
        st_l.append(lock.status.cpu().numpy().copy())
        it_l.append(lock.iters.cpu().numpy().copy())
    st_r, it_r = run.run(K, Pseq=torch.from_numpy(Pseq).cuda())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(st_r.cpu().numpy(), np.array(st_l))
    np.testing.assert_array_equal(it_r.cpu().numpy(), np.array(it_l))
    a, b = _state(lock), _state(run)
    for n in ("w", "w0", "lam0", "lamx0", "f"):
        np.testing.assert_array_equal(b[n], a[n], err_msg=n)


def test_run_ltv_with_schedule_sequence(mpcx):
    """Config-4 LTV: per-step references (Pseq) and schedules (tabseq) == the lock-step loop."""
    import torch
    from mpcx import dist
    from mpcx.device import DeviceLoop

    N, B, K = 20, 16, 4
    t0, x0, par = dist.config4_inputs(0, B, N=N)
    _, _, vref = dist.lane_change()
    lin = mpcx.lateral_ltv(N=N, Delta=0.05, vref=vref, per_instance_tab=t0)
    solver = mpcx.nlpsol("ltv", "mi355x", lin)
    tt = np.minimum(t0[None, :] + np.arange(K)[:, None], 499)
    refs = np.ascontiguousarray(par[tt].reshape(K, B, -1))
    tabs = np.ascontiguousarray(np.repeat(tt[:, :, None], N, axis=2).astype(np.int32))
    P0 = lin.params(x0, par[tt[0]])
    Pseq = np.zeros((K, B, P0.shape[1]))
    Pseq[:, :, 4:] = refs
    dr, dt = torch.from_numpy(refs).cuda(), torch.from_numpy(tabs).cuda()
    lock = DeviceLoop(solver, P0)
    it_l = []
    for t in range(K):
        lock.set_stage_refs(dr[t])
        lock.set_schedule(dt[t])
        lock.step()
        torch.cuda.synchronize()
        it_l.append(lock.iters.cpu().numpy().copy())
    a = _state(lock)
    run = DeviceLoop(solver, P0)
    run.set_schedule(dt[0])
    _, it_r = run.run(K, Pseq=torch.from_numpy(Pseq).cuda(), tabseq=dt)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(it_r.cpu().numpy(), np.array(it_l))
    b = _state(run)
    for n in ("w", "w0", "lam0", "lamx0", "f"):
        np.testing.assert_array_equal(b[n], a[n], err_msg=n)
    np.testing.assert_array_equal(b["P"][:, 0:4], a["P"][:, 0:4])
    run.set_schedule(None)


def test_nonfinite_instance_fails_alone(mpcx):
    """An instance with a NaN parameter ends with a failure status (IPOPT would report a failure)
    and leaves every other instance -- including its wave-mate -- bit-identical."""
    from mpcx import dist

    solver = mpcx.nlpsol("s", "mi355x", mpcx.unicycle_point_to_point(N=20))
    P = dist.config2_inputs(0, 8)
    ref = solver.solve_batch(P)
    Pn = P.copy()
    Pn[3, 1] = np.nan  # instance 3 shares a wave with instance 2 (G = 32)
    r = solver.solve_batch(Pn)
    assert r["status"][3] >= 3  # a failure code (the NaN reaches the factorisation: 5)
    others = [b for b in range(8) if b != 3]
    np.testing.assert_array_equal(r["status"][others], ref["status"][others])
    np.testing.assert_array_equal(r["w"][others], ref["w"][others])
    np.testing.assert_array_equal(r["iters"][others], ref["iters"][others])


@pytest.mark.parametrize("workload,B", [
    ([], 1024),                                       # config 2 (BASELINE metric)
    (["--config", "4"], 1024),                        # LTV lateral, N = 50: per-instance device schedules
    (["--config", "4", "--model", "dyn_bicycle"], 1024),  # 6-state bicycle, N = 50, chain stash workspace
    (["--config", "5"], 2048),                        # cart-pole QP, N = 100: two-wave groups, suffix cache
], ids=["config2", "config4_ltv", "config4_dyn_bicycle", "config5_qp"])
def test_bench_two_ranks_rehearsal(tmp_path, workload, B):
    """The multi-rank bench path end to end (torch.distributed.run, 2 ranks, weak
    scaling, stats all_gather, max-over-ranks timing), rehearsed on ONE GPU: both ranks on
    device 0 and gloo collectives (RCCL needs a GPU per rank; the 8-GPU run is the driver's).
    Sharding is exact: the all-gathered per-instance statistics of the
    2-rank run -- final states, objective, statuses, iteration counts of every closed-loop
    step -- equal, bit for bit, those of ONE rank solving the global instance ids [0, 2B).
    Every BASELINE config that is sharded over GPUs: config 2, and configs 4 (both models) and 5,
    whose per-rank state the default config lacks -- the per-instance device schedules of the LTV
    loop (bench.py tabseq), the 6-state bicycle's chain workspace, the cart-pole QP's multi-wave
    groups and its per-handle decoupled-suffix cache (one handle per rank against one handle for
    both shards; Trajectory_tracking_dynamic_model.py:117-145,
    inverted_pendulum_single_shooting_mpctools.py:16,64)."""
    import json
    import os
    import socket
    import subprocess
    import sys

    from conftest import ROOT

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, MPCX_FORCE_DEVICE="0", MPCX_DIST_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    # config 2: B per rank = the SIMD count of the MI355X (1024): each rank's launches run replicated
    # 32-lane groups, the single rank's 2B instances the narrow ones -- the weak-scaling case of the bench
    common = workload + ["--steps", "3", "--warmup", "1", "--no-cpu", "--no-roofline", "--no-reference-warm-start"]
    flags = ["--gpus", "2", "--batch", str(B)] + common
    launched = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py")] + flags
    plain = [sys.executable, os.path.join(ROOT, "bench.py")] + flags  # bench.py starts its 2 ranks itself
    single = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--batch", str(2 * B)] + common
    stats = {}
    runs = (("launched", launched), ("plain", plain), ("single", single))
    if workload:  # the torch.distributed.run launch path is the same for every workload
        runs = runs[1:]
    for name, cmd in runs:
        dump = str(tmp_path / f"{name}.npy")
        out = subprocess.run(cmd + ["--dump-stats", dump], env=env if name != "single" else dict(os.environ),
                             capture_output=True, text=True, timeout=600, cwd=ROOT)
        assert out.returncode == 0, out.stderr[-3000:]
        lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
        assert len(lines) == 1  # rank 0 prints ONE line
        d = json.loads(lines[0])
        n = 1 if name == "single" else 2
        assert d["n_gpus"] == n and d["config"]["global_batch"] == n * d["config"]["batch_per_gpu"] == 2 * B
        assert d["failed_instances"] == 0 and d["value"] > 0 and d["steps"] == 3
        stats[name] = np.load(dump)
    assert stats["single"].shape == (2 * B, 8)
    for name in stats:
        np.testing.assert_array_equal(stats[name], stats["single"], err_msg=name)


def test_mpctools_variant_closed_loop_3exemplo(mpcx, R, golden):
    """mpctools/multiple_shooting_mpctools.py on the GPU (node cost, RK4 M=1, R = I): each
    solve starts from the previous prediction X_1, the plant is the exact ODE flow; the
    recorded controls of Casadi/3exemplo.xlsx are reproduced and the loop stops at row 88."""
    rows = np.array(golden["mpctools"]["rows"])
    ocp = mpcx.unicycle_point_to_point_mpctools(N=10)
    solver = mpcx.nlpsol("s", "mi355x", ocp)
    goal = np.array([10.0, 10.0, 0.0])

    def solve(x0):
        r = solver.solve_batch(np.concatenate([x0, goal])[None])
        assert r["status"][0] == 0
        w = r["w"][0]
        return w[3:5].copy(), w[5:8].copy()

    xs, us = R.mpctools_closed_loop(solve)
    assert us.shape[0] == rows.shape[0]
    assert rel_err(us, rows[:, 3:5]) <= REL_TOL
    assert np.abs(xs - rows[:, 0:3]).max() <= 1e-4


def test_iteration_counts_match_cpp_oracle(mpcx, R, C):
    """Algorithm fidelity, not only the optimum: the kernel and the independently written C++
    IPOPT restatement take the same number of iterations on the config-2 batch, cold and
    after one warm-started closed-loop step (IPOPT warm_start_init_point)."""
    import bench
    from mpcx import dist

    B, N = 1024, 20
    solver = mpcx.nlpsol("s", "mi355x", mpcx.unicycle_point_to_point(N=N))
    P = dist.config2_inputs(0, B)
    r = solver.solve_batch(P)
    rocp = R.UnicycleOCP(N=N)
    ref = C.solve_batch(rocp, P, w0=bench._cold(P, N, R), nthreads=0)
    n1 = int(np.sum(r["iters"] != ref["iters"]))
    print(f"cold: {n1} of {B} iteration counts differ from the C++ oracle")
    assert n1 <= MAX_ITER_MISMATCH, np.flatnonzero(r["iters"] != ref["iters"])
    # one closed-loop step later, warm-started from the shifted primal-dual solution
    P2 = P.copy()
    P2[:, 0:3], _ = R.F(P[:, 0:3], r["w"][:, 3:5], P[:, 3:6], rocp)
    w0, l0, lx0 = bench.shift_np(r["w"], N), bench.shift_lam_np(r["lam_g"], N), bench.shift_lamx_np(r["lam_x"], N)
    r2 = solver.solve_batch(P2, w0=w0, lam_g0=l0, lam_x0=lx0)
    ref2 = C.solve_batch_warm(rocp, P2, w0, lam0=l0, lamx0=lx0, mu_init=1e-4, bound_push=1e-4, mult_push=1e-4,
                              nthreads=0)
    n2 = int(np.sum(r2["iters"] != ref2["iters"]))
    print(f"warm: {n2} of {B} iteration counts differ from the C++ oracle")
    assert n2 <= MAX_ITER_MISMATCH, np.flatnonzero(r2["iters"] != ref2["iters"])
