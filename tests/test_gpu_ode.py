"""GPU parity tests of the nonlinear ODE model variants (kinematic bicycle, 6-state dynamic bicycle,
cart-pole; mpcx/ode.py) through the C ABI.

PARITY UNPINNED (BASELINE-named extensions, no reference outputs): checked against the CPU oracle
oracle/ode_ref.py (complex-step derivatives, projected Newton; its linearisations are pinned to the
reference's matrices in tests/test_ode_cpu.py).  Tolerances: plant 1e-12 relative; optimal inputs
1e-6 relative to max(|u|_inf, 1) at solver tol 1e-10 (north-star bound 1e-4);
KKT residual of the GPU's primal-dual point, evaluated by the oracle, <= 1e-6.
"""
import math
import os

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

U_TOL = 1e-6


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b)) / max(float(np.max(np.abs(b))), 1.0))


@pytest.fixture(scope="module")
def mpcx():
    import mpcx as m

    m._lib.load()
    return m


def _lane_change():
    import pandas as pd
    from mpcx import ode

    g = pd.read_csv(os.path.join(ROOT, "tests", "golden", "lane_change.csv"))
    return ode.lane_change_rows(g.x, g.y, g.uref)


def cases(which, B, N, seed=0):
    """(ocp, P (B, n_p)) of a small seeded batch."""
    from mpcx import ode

    rng = np.random.default_rng(seed)
    if which == "kin_bicycle":
        ocp = ode.kinematic_bicycle_tracking(N=N)
        tau0 = rng.uniform(0, 20 * math.pi, B)
        ref = ode.bicycle_circular_reference(tau0, 0, N)
        x0 = ref[:, 0, :3] + rng.normal(0, 0.1, (B, 3))
        return ocp, ocp.params(x0, ref)
    if which == "dyn_bicycle":
        ocp = ode.dynamic_bicycle_lane_change(N=N)
        X, Y, V = _lane_change()
        t = rng.integers(0, 440, B)
        ref = np.stack([ode.dyn_bicycle_references(X, Y, V, int(ti), N) for ti in t])
        x0 = ref[:, 0, :6] + rng.normal(0, 1, (B, 6)) * np.array([0.2, 0.2, 0.05, 0.3, 0.1, 0.05])
        return ocp, ocp.params(x0, ref)
    ocp = ode.cartpole_swingup(N=N)
    x0 = rng.uniform(-1, 1, (B, 4)) * np.array([0.5, 0.3, 0.3, 0.3])
    xr = np.zeros((B, 4))
    xr[:, 0] = rng.uniform(-1, 1, B)
    return ocp, ocp.params(x0, xr)


@pytest.mark.parametrize("which", ["kin_bicycle", "dyn_bicycle", "cartpole"])
def test_ode_plant_matches_oracle(mpcx, which):
    from oracle import ode_ref

    ocp, P = cases(which, 64, 10, seed=3)
    pr = ode_ref.Problem(ocp)
    rng = np.random.default_rng(4)
    U = rng.uniform(ocp.u_lb, ocp.u_ub, (64, ocp.nu)) * 0.5
    xf, qf = mpcx.integrator(ocp).batch(P, U)
    ref = pr.F(P[:, :ocp.nx], U)
    zr0 = np.stack([pr.refs(p)[0] for p in P])  # stage-0 reference of every instance
    q = pr.l(np.concatenate([P[:, :ocp.nx], U], axis=1), zr0)
    assert rel(xf, ref) <= 1e-12
    assert rel(qf, q) <= 1e-12


@pytest.mark.parametrize("policy", [0, 1])
@pytest.mark.parametrize("which,N,B", [("kin_bicycle", 30, 6), ("dyn_bicycle", 20, 4), ("cartpole", 50, 6),
                                       ("kin_bicycle", 1, 5), ("cartpole", 15, 5), ("cartpole", 130, 3),
                                       ("dyn_bicycle", 70, 3)])
def test_ode_optimum_matches_oracle(mpcx, which, N, B, policy):
    from oracle import ode_ref

    ocp, P = cases(which, B, N)
    # tol 1e-10: at 1e-8 an interior point keeps ~1e-6 off active bounds on these less well scaled
    # problems (kinematic bicycle: steering weight 0.05), and the check is of the fixed point
    solver = mpcx.nlpsol("ode", "mi355x", ocp, {"ipopt": {"max_iter": 300, "tol": 1e-10}, "group_policy": policy})
    r = solver.solve_batch(P)
    assert np.all(r["status"] == 0), r["status"]
    pr = ode_ref.Problem(ocp)
    for b in range(B):
        if which == "dyn_bicycle" and N > 50:
            # two-wave group (sequential multi-wave Riccati, NX = 6): the oracle's single-shooting
            # Newton is ill-conditioned over 70 intervals of this model, so the point is certified
            # by the multiple-shooting KKT residual alone
            kkt, gres = pr.kkt_residual(r["w"][b], r["lam_g"][b], r["lam_x"][b], P[b])
            assert kkt <= 1e-6 and gres <= 1e-9, (b, kkt, gres)
            continue
        X, U = pr.split_w(r["w"][b])
        Uo, Xo, info = pr.solve(P[b], U0=U)  # started at the GPU point: same local optimum
        assert info["status"] in ("converged", "stalled") and info["pg"] <= 1e-6, info
        assert rel(U, Uo) <= U_TOL, (b, rel(U, Uo))
        assert rel(X, Xo) <= U_TOL
        assert abs(r["f"][b] - info["J"]) <= 1e-8 * max(1.0, abs(info["J"]))
        kkt, gres = pr.kkt_residual(r["w"][b], r["lam_g"][b], r["lam_x"][b], P[b])
        assert kkt <= 1e-6 and gres <= 1e-9, (b, kkt, gres)
    if which == "dyn_bicycle" and N <= 50:  # the vx >= 2.5 bound stays inactive (the oracle's solve does not model it)
        assert np.min(r["w"][:, 3::8]) > 2.6


def test_cartpole_swingup_is_kkt_point(mpcx):
    """Swing-up from hanging (phi = pi), N = 100: nonconvex, so the check is the oracle's KKT
    residual at the GPU's primal-dual point (any local optimum of the NLP qualifies)."""
    from oracle import ode_ref

    ocp = mpcx.cartpole_swingup(N=100)
    P = ocp.params(np.array([[0.0, 0.0, math.pi, 0.0], [0.5, 0.0, -math.pi + 0.1, 0.2]]), np.zeros(4))
    solver = mpcx.nlpsol("swing", "mi355x", ocp, {"ipopt": {"max_iter": 1000, "tol": 1e-8}})
    r = solver.solve_batch(P)
    assert np.all(r["status"] == 0), r["status"]
    pr = ode_ref.Problem(ocp)
    for b in range(2):
        kkt, gres = pr.kkt_residual(r["w"][b], r["lam_g"][b], r["lam_x"][b], P[b])
        assert kkt <= 1e-6 and gres <= 1e-9, (b, kkt, gres)
        _, U = pr.split_w(r["w"][b])
        assert np.all(U >= -200 - 1e-9) and np.all(U <= 200 + 1e-9)


def test_cartpole_single_shooting_call(mpcx):
    """BASELINE's "single-shooting" cart-pole: decision = U, g = X_1..X_N (+-inf), CasADi-shaped
    call; same optimum as the oracle's independent single-shooting solve."""
    from oracle import ode_ref

    N = 40
    ocp = mpcx.cartpole_swingup(N=N, formulation="single_shooting")
    solver = mpcx.nlpsol("ss", "mi355x", ocp, {"ipopt": {"tol": 1e-10}})
    p = [0.1, 0.0, 0.2, -0.1, 0.5, 0.0, 0.0, 0.0]
    sol = solver(x0=[0.0] * N, lbx=-200.0, ubx=200.0, lbg=-math.inf, ubg=math.inf, p=p)
    assert sol["x"].shape == (N, 1) and sol["g"].shape == (4 * N, 1) and sol["lam_x"].shape == (N, 1)
    assert solver.stats()["success"]
    pr = ode_ref.Problem(ocp)
    U, X, info = pr.solve(np.array(p))
    assert info["status"] == "converged"
    assert rel(sol["x"][:, 0], U[:, 0]) <= U_TOL
    assert rel(sol["g"][:, 0], X[1:].reshape(-1)) <= U_TOL


@pytest.mark.parametrize("which,N", [("dyn_bicycle", 20), ("cartpole", 100)])
def test_ode_run_equals_lockstep(mpcx, which, N):
    """Multi-step launches == lock-step launches, bit for bit, for the ODE models too."""
    import torch
    from mpcx.device import DeviceLoop

    ocp, P = cases(which, 32, N, seed=7)
    solver = mpcx.nlpsol("s", "mi355x", ocp)
    lock, run = DeviceLoop(solver, P), DeviceLoop(solver, P)
    st_l, it_l = [], []
    for _ in range(3):
        lock.step()
        torch.cuda.synchronize()
        st_l.append(lock.status.cpu().numpy().copy())
        it_l.append(lock.iters.cpu().numpy().copy())
    st_r, it_r = run.run(3)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(st_r.cpu().numpy(), np.array(st_l))
    np.testing.assert_array_equal(it_r.cpu().numpy(), np.array(it_l))
    assert np.all(np.array(st_l) == 0)
    for n in ("P", "w", "w0", "lam", "lamx", "f"):
        np.testing.assert_array_equal(getattr(run, n).cpu().numpy(), getattr(lock, n).cpu().numpy(), err_msg=n)


def test_dyn_bicycle_hardest_instances_are_kkt_points(mpcx):
    """Config-4 variant (6-state bicycle, bench inputs), first closed-loop step from the cold start:
    the instances that needed the most iterations -- the ones the second-order correction acts on
    (solver.hip, Dyn::kSOC) -- end at points the oracle certifies as KKT points of the NLP, and the
    iteration tail stays short (before the correction the worst cold solve took 308 iterations)."""
    from mpcx import dist as mdist
    from oracle import ode_ref

    B, N = 256, 50
    ocp = mpcx.dynamic_bicycle_lane_change(N=N)
    t0, x0, (X, Y, V) = mdist.config4_bicycle_inputs(0, B)
    refs = np.stack([mpcx.ode.dyn_bicycle_references(X, Y, V, int(t), N).reshape(-1) for t in t0])
    P = ocp.params(x0, refs)
    solver = mpcx.nlpsol("dyn", "mi355x", ocp, {"ipopt": {"max_iter": 3000}})
    r = solver.solve_batch(P)
    assert np.all(r["status"] <= 1), np.unique(r["status"], return_counts=True)
    assert r["iters"].max() < 250, r["iters"].max()
    pr = ode_ref.Problem(ocp)
    hard = [b for b in np.argsort(-r["iters"]) if r["status"][b] == 0][:6]
    for b in hard:
        kkt, gres = pr.kkt_residual(r["w"][b], r["lam_g"][b], r["lam_x"][b], P[b])
        assert kkt <= 1e-6 and gres <= 1e-9, (b, int(r["iters"][b]), kkt, gres)


def test_dyn_bicycle_adjoint_derivatives_match_passes():
    """The 6-state bicycle's stage derivatives as the solve kernel forms them (ode.h
    OdeModel::derivs_adjoint: forward sensitivities and stage adjoints through RK4, closed-form
    partials of f) against its 21 hyper-dual RK4 passes (derivs_passes), both through the device
    harness tests/hip/flop_probe.hip on 4096 random points of the model's domain: F, q and the cost
    gradient bit-identical (the same value pass), A, B and the Hessian of q + lam^T F equal to
    1e-11 relative to each point's largest entry (both exact up to rounding)."""
    import ctypes

    import torch
    from mpcx import ode

    lib = ctypes.CDLL(os.path.join(ROOT, "tests", "hip", "libflop_probe.so"))
    vp = ctypes.c_void_p
    for fn in (lib.eval_probe, lib.eval_probe_passes):
        fn.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_int, ctypes.c_int, vp, vp, vp, vp, vp, vp,
                       ctypes.c_int, vp]
    ocp = ode.dynamic_bicycle_lane_change()
    nx, nu, n = 6, 2, 4096
    nz = nx + nu
    rng = np.random.default_rng(7)
    Z = np.stack([rng.uniform(-50, 50, n), rng.uniform(-5, 5, n), rng.uniform(-math.pi, math.pi, n),
                  rng.uniform(2.5, 30.0, n), rng.uniform(-2, 2, n), rng.uniform(-1, 1, n),
                  rng.uniform(-0.5, 0.5, n), rng.uniform(-5, 5, n)], axis=1)
    P = np.concatenate([Z[:, :nx], Z[:, :nx] + rng.normal(0, 1, (n, nx))], axis=1)
    L = rng.normal(size=(n, nx)) * 10.0 ** rng.uniform(-2, 2, (n, 1))
    arr8 = lambda v: (ctypes.c_double * 8)(*(list(v) + [0.0] * (8 - len(v))))  # noqa: E731
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float64)).cuda()  # noqa: E731
    d_z, d_l, d_p = dev(Z), dev(L), dev(P)
    no = nx + 1 + nx * nx + nx * nu + nz + nz * (nz + 1) // 2
    outs = []
    for fn in (lib.eval_probe, lib.eval_probe_passes):
        out = torch.zeros(n * no, dtype=torch.float64, device="cuda")
        rc = fn(4, n, ocp.T, ocp.M, 0, arr8(ocp.Q), arr8(ocp.R), arr8(ocp.par), vp(d_z.data_ptr()), vp(d_l.data_ptr()),
                vp(d_p.data_ptr()), 2 * nx, vp(out.data_ptr()))
        assert rc == 0
        outs.append(out.cpu().numpy().reshape(n, no))
    adj, ref = outs
    assert np.isfinite(adj).all()
    o_a = nx + 1
    o_g = o_a + nx * nx + nx * nu
    o_h = o_g + nz
    np.testing.assert_array_equal(adj[:, :o_a], ref[:, :o_a])  # F, q
    np.testing.assert_array_equal(adj[:, o_g:o_h], ref[:, o_g:o_h])  # cost gradient
    for lo, hi, name in ((o_a, o_g, "A, B"), (o_h, no, "H")):
        err = np.abs(adj[:, lo:hi] - ref[:, lo:hi]).max(axis=1) / np.maximum(np.abs(ref[:, lo:hi]).max(axis=1), 1e-300)
        print(f"{name}: max relative difference {err.max():.2e}")
        assert err.max() <= 1e-11, name
