"""GPU parity tests of the linear-model family through the C ABI.

Oracles (oracle/nlp_ref.py, CPU, exact projected-Newton QP solves):
  * pendulum_qp_solve / pendulum_closed_loop -- pinned to the reference's own output
    ``Inverted_pendulum/invertpend_data_py.xlsx`` (tests/test_linear_cpu.py);
  * lq_solve -- generic table-driven LQ OCP (cross-checked against the pinned pendulum
    oracle on CPU).  The LTV lateral model (``Trajectory_tracking_dynamic_model.py``) has no
    reference output (the script raises NameError as written): parity unpinned beyond lq_solve.
Tolerance: the interior-point solve stops at tol 1e-8 (IPOPT's default); optimal inputs
must agree within 1e-6 relative to max(|u|_inf, 1) (the north-star bound is 1e-4).
"""
import csv
import json
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


@pytest.fixture(scope="module")
def R():
    from oracle import nlp_ref

    return nlp_ref


@pytest.fixture(scope="module")
def pend(mpcx):
    lin = mpcx.inverted_pendulum_qp()
    return lin, mpcx.nlpsol("pend", "mi355x", lin, {"ipopt": {"max_iter": 200, "tol": 1e-8}})


def U_of(w, nx, nu, N):
    return np.stack([w[..., nx + (nx + nu) * k: nx + (nx + nu) * k + nu] for k in range(N)], axis=-2)


def X_of(w, nx, nu, N):
    xs = [w[..., 0:nx]] + [w[..., nx + (nx + nu) * k + nu: nx + (nx + nu) * (k + 1)] for k in range(N)]
    return np.stack(xs, axis=-2)


def close(a, b):
    """max |a - b| relative to max(1, max |b|)"""
    return float(np.max(np.abs(a - b)) / max(1.0, float(np.max(np.abs(b)))))


def test_pendulum_batch_vs_oracle(mpcx, R, pend):
    lin, S = pend
    from mpcx import lti

    rng = np.random.default_rng(11)
    B = 96
    scale = np.where(np.arange(B) % 3 == 0, 30.0, 1.0)[:, None]  # every third instance saturates |u| <= 200
    x = scale * rng.uniform([-1, -.5, -.2, -.5], [1, .5, .2, .5], size=(B, 4))
    up = rng.uniform(-50, 50, size=B)
    P = lti.pendulum_params(lin, x, up)
    r = S.solve_batch(P, want_g=True)
    assert np.all(r["status"] == 0), np.unique(r["status"], return_counts=True)
    U = U_of(r["w"], 5, 1, 50)[..., 0]
    X = X_of(r["w"], 5, 1, 50)
    A, Bd = R.pendulum_model()
    nsat = 0
    for b in range(B):
        u_ref = R.pendulum_qp_solve(x[b], A, Bd, uprev=up[b])
        assert rel(U[b, :5], u_ref) <= U_TOL, (b, U[b, :5], u_ref)
        assert np.abs(X[b, 5:, 4] - U[b, 4]).max() <= 1e-6 * max(1.0, abs(U[b, 4]))
        nsat += int(np.any(np.abs(u_ref) >= 200 - 1e-9))
    assert nsat >= B // 4
    assert np.abs(r["g"]).max() <= 1e-8 * max(1.0, np.abs(r["w"]).max())  # shooting defects closed


def test_pendulum_closed_loop_matches_reference_output(mpcx, pend):
    """The reference's 1000-step closed loop (:66-78) on the GPU: x0 = 0, u_prev fixed at 0,
    plant x <- A x + B u0 (the script's ffunc).  Compared with invertpend_data_py.xlsx."""
    lin, S = pend
    from mpcx import lti

    with open(os.path.join(ROOT, "tests", "golden", "pendulum_N50_golden.json")) as f:
        gold = np.array(json.load(f)["rows"])
    x = np.zeros(4)
    us = []
    for k in range(1000):
        r = S.solve_batch(lti.pendulum_params(lin, x, 0.0), want_lam=False)
        assert r["status"][0] == 0
        u = r["w"][0, 5]
        us.append(u)
        x = lin.A_plant @ x + lin.B_plant[:, 0] * u
        if k in (0, 1, 100, 999):
            assert rel(x, gold[k + 1, 0:4]) <= 1e-6, k
    us = np.array(us)
    assert rel(us, gold[:1000, 4]) <= U_TOL


def test_linear_plant_step(mpcx, pend):
    lin, S = pend
    from mpcx import lti

    F = mpcx.integrator(lin)
    rng = np.random.default_rng(2)
    x = rng.normal(size=(7, 4))
    up = rng.normal(size=7)
    u = rng.normal(size=(7, 1)) * 10
    P = lti.pendulum_params(lin, x, up)
    xf, qf = F.batch(P, u)
    z0 = np.concatenate([x, up[:, None]], axis=1)
    ref = z0 @ lin.A[0].T + u @ lin.B[0].T
    np.testing.assert_allclose(xf, ref, rtol=1e-14, atol=1e-12)
    dz = np.concatenate([z0, u], axis=1) - P[:, 5:11]
    np.testing.assert_allclose(qf, np.einsum("bi,ij,bj->b", dz, lin.W[0], dz), rtol=1e-13, atol=1e-12)


def lane_change():
    with open(os.path.join(ROOT, "tests", "golden", "lane_change.csv")) as f:
        rows = [tuple(float(v) for v in r.values()) for r in csv.DictReader(f)]
    return tuple(np.array(c) for c in zip(*rows))


@pytest.mark.parametrize("N", [10, 50])
def test_lateral_ltv_vs_lq_oracle(mpcx, R, N):
    """Config 4 family: per-instance tables (instance b re-linearised at vref[t_b]), stage
    references from the script's rules, |delta| <= 20.  Parity unpinned beyond lq_solve."""
    from mpcx import lti

    xr, yr, vr = lane_change()
    par = lti.lateral_references(xr, yr, vr, Delta=0.05, horizon=N)
    rng = np.random.default_rng(5)
    B = 64
    t = rng.integers(0, 450, size=B)
    lin = lti.lateral_ltv(N=N, Delta=0.05, vref=vr, per_instance_tab=t)
    S = mpcx.nlpsol("ltv", "mi355x", lin, {"ipopt": {"max_iter": 300}})
    x0 = rng.normal(scale=[0.3, 0.1, 0.3, 0.1], size=(B, 4))
    zr = par[t]  # (B, N, 5)
    P = lin.params(x0, zr)
    r = S.solve_batch(P)
    assert np.all(r["status"] == 0), np.unique(r["status"], return_counts=True)
    U = U_of(r["w"], 4, 1, N)[..., 0]
    for b in range(B):
        X_ref, U_ref, J = R.lq_solve(x0[b], lin.A, lin.B, lin.c, lin.W, lin.tab[b], zr[b], [-20], [20])
        assert rel(U[b], U_ref[:, 0]) <= U_TOL, b
        assert abs(r["f"][b] - J) <= 1e-6 * max(1.0, abs(J))


def test_linear_device_loop_matches_host_loop(mpcx, R, pend):
    """DeviceLoop on a linear model: P[0:nx] <- plant(x~, u0) (u_prev <- u0), warm-started
    solves; compared with a host loop of exact oracle solves."""
    import torch
    from mpcx import lti
    from mpcx.device import DeviceLoop

    lin, S = pend
    rng = np.random.default_rng(9)
    B = 32
    x = rng.uniform([-1, -.5, -.2, -.5], [1, .5, .2, .5], size=(B, 4))
    P0 = lti.pendulum_params(lin, x, 0.0)
    loop = DeviceLoop(S, P0, device="cuda:0")
    A, Bd = R.pendulum_model()
    xs, ups = x.copy(), np.zeros(B)
    for step in range(12):
        loop.step()
        torch.cuda.synchronize()
        st = loop.status.cpu().numpy()
        assert np.all(st == 0)
        w = loop.w.cpu().numpy()
        for b in range(B):
            u_ref = R.pendulum_qp_solve(xs[b], A, Bd, uprev=ups[b])
            assert rel(w[b, 5], u_ref[0]) <= U_TOL, (step, b)
        u0 = w[:, 5]
        xs = xs @ A.T + u0[:, None] * Bd[:, 0][None, :]
        ups = u0
        Pn = loop.P.cpu().numpy()
        np.testing.assert_allclose(Pn[:, 0:4], xs, rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(Pn[:, 4], ups, rtol=0, atol=0)


def test_linear_model_argument_errors(mpcx):
    from mpcx import _lib, lti

    lin = lti.inverted_pendulum_qp()
    h = _lib.Handle(mpcx.to_spec(lin))
    S = mpcx.Solver.__new__(mpcx.Solver)  # handle without tables -> solve must refuse
    S.ocp, S._h, S.max_iter, S.tol, S._stats = lin, h, 10, 1e-8, {}
    with pytest.raises(_lib.MpcxError, match="tables not set"):
        S.solve_batch(lti.pendulum_params(lin, np.zeros(4)))
    bad = lti.inverted_pendulum_qp()
    bad.tab = np.full(50, 7, np.int32)
    with pytest.raises(_lib.MpcxError, match="out of range"):
        h.set_linear_model(bad)


@pytest.mark.parametrize("N", [100, 160])
def test_pendulum_long_horizon_multiwave(mpcx, R, N):
    """Config 5 family at N = 100 (BASELINE.json) and beyond: one instance spans 2-4
    wavefronts (128/256-lane groups, LDS handoffs in the Riccati and forward sweeps)."""
    from mpcx import lti

    lin = lti.inverted_pendulum_qp(N=N)
    S = mpcx.nlpsol("pend", "mi355x", lin, {"ipopt": {"max_iter": 200}})
    rng = np.random.default_rng(N)
    B = 24
    scale = np.where(np.arange(B) % 3 == 0, 30.0, 1.0)[:, None]
    x = scale * rng.uniform([-1, -.5, -.2, -.5], [1, .5, .2, .5], size=(B, 4))
    up = rng.uniform(-50, 50, size=B)
    r = S.solve_batch(lti.pendulum_params(lin, x, up))
    assert np.all(r["status"] == 0)
    A, Bd = R.pendulum_model()
    for b in range(B):
        u_ref = R.pendulum_qp_solve(x[b], A, Bd, N=N, uprev=up[b])
        assert rel(r["w"][b, 5:5 + 6 * 5:6], u_ref) <= U_TOL, b
    # instances are independent: a ragged sub-batch gives bit-identical results, on a fresh handle
    # and on S, whose second launch starts from the suffix cache
    S2 = mpcx.nlpsol("pend", "mi355x", lin, {"ipopt": {"max_iter": 200}})
    for h in (S2, S):
        r2 = h.solve_batch(lti.pendulum_params(lin, x[5:12], up[5:12]))
        np.testing.assert_array_equal(r2["w"], r["w"][5:12])


@pytest.mark.parametrize("N", [50, 100])
def test_pendulum_decoupled_suffix_same_bits(mpcx, R, N, monkeypatch):
    """The move-blocked stages (B = 0, no x-u cost block) reuse P_k across iterations
    (solver.hip "decoupled suffix", riccati.h DEC), and later launches start from the P_k an
    earlier one cached.  Same solution bits, multipliers and iteration counts as the full
    recursion (MPCX_DEC_SUFFIX=0), with and without the cache, and the LQ oracle's solution.
    At N = 100 (two-wave groups) the reused suffix runs as a log-depth vector scan (kernels.h,
    "reused suffix as a log-depth scan"), whose sums associate differently: there the same
    iteration counts and a solution within 1e-9 of the full recursion's -- and the same bits with
    and without the cache (a fresh factorisation is redone on the reused path)."""
    from mpcx import lti

    lin = lti.inverted_pendulum_qp(N=N)
    rng = np.random.default_rng(100 + N)
    B = 48
    scale = np.where(np.arange(B) % 3 == 0, 30.0, 1.0)[:, None]
    x = scale * rng.uniform([-1, -.5, -.2, -.5], [1, .5, .2, .5], size=(B, 4))
    up = rng.uniform(-50, 50, size=B)
    P = lti.pendulum_params(lin, x, up)
    S_fast = mpcx.nlpsol("pend", "mi355x", lin, {"ipopt": {"max_iter": 200}})
    monkeypatch.setenv("MPCX_DEC_SUFFIX", "0")
    S_full = mpcx.nlpsol("pend", "mi355x", lin, {"ipopt": {"max_iter": 200}})
    a = S_fast.solve_batch(P)
    b = S_full.solve_batch(P)
    # the second launch of the handle starts every fs = 1 instance from the suffix's P_k that
    # the first launch cached (capi SolveArgs::pcache): the same bits again
    a2 = S_fast.solve_batch(P)
    assert np.all(a["status"] == 0)
    for n in ("w", "f", "lam_g", "lam_x", "iters", "status"):  # cache state: no effect on the bits
        np.testing.assert_array_equal(a2[n], a[n], err_msg=n)
    for r in (a, a2):
        np.testing.assert_array_equal(r["iters"], b["iters"])
        if N < 64:
            np.testing.assert_array_equal(r["w"], b["w"])
            np.testing.assert_array_equal(r["lam_g"], b["lam_g"])
        else:
            assert close(r["w"], b["w"]) <= 1e-9 and close(r["lam_g"], b["lam_g"]) <= 1e-9
    A, Bd = R.pendulum_model()
    for i in range(0, B, 7):
        u_ref = R.pendulum_qp_solve(x[i], A, Bd, N=N, uprev=up[i])
        assert rel(a["w"][i, 5:5 + 6 * 5:6], u_ref) <= U_TOL, i


def test_ltv_device_loop_with_device_schedule(mpcx, R):
    """Config-4 closed loop on the device: per step the stage references and the per-instance
    schedule (model re-linearised at vref[t], mpcx_set_linear_tab_dev) advance; compared with
    a host loop of exact LQ solves using the same tables."""
    import torch
    from mpcx import dist as mdist
    from mpcx.device import DeviceLoop

    N, B, T = 20, 16, 6
    t0, x0, par = mdist.config4_inputs(0, B, N=N)
    _, _, vref = mdist.lane_change()
    lin = mpcx.lateral_ltv(N=N, Delta=0.05, vref=vref, per_instance_tab=t0)
    S = mpcx.nlpsol("ltv", "mi355x", lin, {"ipopt": {"max_iter": 300}})
    tt = np.minimum(t0[None, :] + np.arange(T)[:, None], 499)
    refs = torch.from_numpy(np.ascontiguousarray(par[tt].reshape(T, B, -1))).to("cuda:0")
    tabs = torch.from_numpy(np.repeat(tt[:, :, None], N, axis=2).astype(np.int32)).to("cuda:0")
    loop = DeviceLoop(S, lin.params(x0, par[tt[0]]), device="cuda:0")
    x = x0.copy()
    for t in range(T):
        loop.set_stage_refs(refs[t])
        loop.set_schedule(tabs[t])
        loop.step()
        torch.cuda.synchronize()
        assert np.all(loop.status.cpu().numpy() == 0)
        w = loop.w.cpu().numpy()
        u0 = np.empty(B)
        for b in range(B):
            j = tt[t, b]
            _, U_ref, _ = R.lq_solve(x[b], lin.A, lin.B, lin.c, lin.W, np.full(N, j), par[j], [-20], [20])
            assert rel(w[b, 4:4 + 5 * N:5], U_ref[:, 0]) <= U_TOL, (t, b)
            u0[b] = w[b, 4]
            x[b] = lin.A[j] @ x[b] + lin.B[j][:, 0] * u0[b]
        np.testing.assert_allclose(loop.P.cpu().numpy()[:, 0:4], x, rtol=1e-12, atol=1e-12)
    loop.set_schedule(None)


@pytest.mark.parametrize("nx,nu,seed", [(4, 1, 0), (4, 1, 1), (5, 1, 2), (5, 1, 3), (1, 1, 4), (2, 1, 5), (3, 1, 6),
                                        (4, 2, 7), (3, 2, 8), (2, 2, 9)])
def test_random_linear_problems_vs_lq_oracle(mpcx, R, nx, nu, seed):
    """Random LTV problems through the generic linear path: 3 tables of random stable A
    (spectral radius 0.95), random B, c, SPD stage weights, per-instance random schedules,
    random per-stage references, |u| <= 1 so that bounds are active; N = 1, 12, 40 and 100
    (nu = 2: the LinearModel<4, 2> instantiation; nx < 4 runs embedded in the 4-state model of
    the same nu, lti.StatePad; nx = 4 runs the log-depth Riccati scan with table operands: single-wave groups, and at
    N = 100 a two-wave group whose scan crosses waves through LDS).
    Random problems include degenerate bounds (multiplier ~ 0 at an active bound), where an
    interior-point solution at tol 1e-8 is O(sqrt(mu)) from the vertex -- as IPOPT's would be:
    inputs are held to the north-star 1e-4, the objective (first-order insensitive there) to
    1e-7 relative."""
    from mpcx import lti

    rng = np.random.default_rng(seed)
    n_tab, B = 3, 48
    nz = nx + nu
    As, Bs, cs, Ws = [], [], [], []
    for _ in range(n_tab):
        A = rng.normal(size=(nx, nx))
        As.append(0.95 * A / max(abs(np.linalg.eigvals(A))))
        Bs.append(rng.normal(size=(nx, nu)))
        cs.append(0.1 * rng.normal(size=nx))
        M = rng.normal(size=(nz, nz))
        Ws.append(M @ M.T / nz + 0.1 * np.eye(nz))
    for N in (1, 12, 40, 100):
        tab = rng.integers(0, n_tab, size=(B, N)).astype(np.int32)
        lin = lti.LinearOCP(N=N, A=np.stack(As), B=np.stack(Bs), c=np.stack(cs), W=np.stack(Ws), tab=tab,
                            u_lb=(-1.0,) * nu, u_ub=(1.0,) * nu)
        S = mpcx.nlpsol("rnd", "mi355x", lin, {"ipopt": {"max_iter": 500}})
        x0 = 3.0 * rng.normal(size=(B, nx))
        zr = rng.normal(size=(B, N, nz))
        r = S.solve_batch(lin.params(x0, zr))
        assert np.all(r["status"] == 0), np.unique(r["status"], return_counts=True)
        U = U_of(r["w"], nx, nu, N)
        n_active = 0
        for b in range(B):
            _, U_ref, J = R.lq_solve(x0[b], lin.A, lin.B, lin.c, lin.W, tab[b], zr[b], [-1.0] * nu, [1.0] * nu)
            assert rel(U[b], U_ref) <= 1e-4, (N, b)
            assert abs(r["f"][b] - J) <= 1e-7 * max(1.0, abs(J)), (N, b)
            n_active += int(np.any(np.abs(U_ref) >= 1 - 1e-9))
        if N > 1:
            assert n_active >= B // 4  # the bounds matter


def test_scan_fallback_on_indefinite_stage_weights(mpcx, R):
    """Stage control weight slightly negative (W_uu = -0.05) under a large state weight: the stage
    R = Hd_uu is indefinite wherever the barrier terms do not cover it, so the log-depth Riccati
    scan (pscan.h) cannot build its elements and the instance takes the sequential recursion
    instead, while the reduced Huu' = R + B^T P B stays positive definite (the condensed QP is
    convex).  The optimum must still match the LQ oracle.  (With the negative weight on the
    last stage too, whose x_N carries no cost, the QP is concave in u_{N-1}: the GPU then lands
    on the bound -- a minimiser -- where the oracle's active-set method stops at u = 0.)"""
    from mpcx import lti

    rng = np.random.default_rng(11)
    nx, nu, N, B = 4, 1, 20, 32
    A = np.eye(nx) + 0.05 * rng.normal(size=(nx, nx))
    Bm = rng.normal(size=(nx, nu)) + 1.0
    W = np.zeros((2, nx + nu, nx + nu))
    W[:, :nx, :nx] = 5.0 * np.eye(nx)
    W[0, nx, nx] = -0.05  # stages 0..N-2: indefinite stage R, convex through P_{k+1}
    W[1, nx, nx] = 0.5    # last stage: x_N carries no cost, so its control needs its own weight
    tab = np.zeros(N, np.int32)
    tab[-1] = 1
    lin = lti.LinearOCP(N=N, A=np.stack([A, A]), B=np.stack([Bm, Bm]), c=np.zeros((2, nx)), W=W, tab=tab,
                        u_lb=(-1.0,), u_ub=(1.0,))
    S = mpcx.nlpsol("fb", "mi355x", lin, {"ipopt": {"max_iter": 300}})
    x0 = rng.normal(size=(B, nx))
    zr = np.zeros((B, N, nx + nu))
    r = S.solve_batch(lin.params(x0, zr))
    assert np.all(r["status"] == 0), np.unique(r["status"], return_counts=True)
    U = U_of(r["w"], nx, nu, N)[..., 0]
    for b in range(B):
        _, U_ref, J = R.lq_solve(x0[b], lin.A, lin.B, lin.c, lin.W, lin.tab, zr[b], [-1.0], [1.0])
        assert rel(U[b], U_ref[:, 0]) <= 1e-5, b
        assert abs(r["f"][b] - J) <= 1e-7 * max(1.0, abs(J)), b


@pytest.mark.parametrize("dec", ["1", "0"])
def test_pendulum_run_equals_lockstep_decoupled_suffix(mpcx, dec, monkeypatch):
    """The config-5 path as benchmarked: DeviceLoop.run(K) (one multi-step launch: warm duals,
    mu_init 1e-4, kb / pcv re-derived at every step boundary, two-wave groups at N = 100) against
    K lock-step launches, with the decoupled-suffix reuse on and off (MPCX_DEC_SUFFIX=0): the same
    iterations, status and bits at every step.  With the reuse on, the lock-step launches after
    the first start from the suffix cache, the steps of the multi-step launch from their own
    fresh factorisation, which is redone on the reused path (kernels.h), so the bits agree."""
    import torch
    from mpcx import dist as mdist
    from mpcx import lti
    from mpcx.device import DeviceLoop

    monkeypatch.setenv("MPCX_DEC_SUFFIX", dec)
    lin = lti.inverted_pendulum_qp(N=100)
    S = mpcx.nlpsol("pend", "mi355x", lin, {"ipopt": {"max_iter": 200}})
    P = lti.pendulum_params(lin, mdist.config5_inputs(0, 64), 0.0)
    lock, run = DeviceLoop(S, P), DeviceLoop(S, P)
    st_l, it_l = [], []
    for _ in range(4):
        lock.step()
        torch.cuda.synchronize()
        st_l.append(lock.status.cpu().numpy().copy())
        it_l.append(lock.iters.cpu().numpy().copy())
    st_r, it_r = run.run(4)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(st_r.cpu().numpy(), np.array(st_l))
    np.testing.assert_array_equal(it_r.cpu().numpy(), np.array(it_l))
    assert np.all(np.array(st_l) == 0)
    for n in ("P", "w", "w0", "lam", "lamx", "f"):
        got, want = getattr(run, n).cpu().numpy(), getattr(lock, n).cpu().numpy()
        np.testing.assert_array_equal(got, want, err_msg=n)


def test_pendulum_suffix_cache_follows_table_changes(mpcx):
    """The decoupled suffix's P_k cached across launches (capi SolveArgs::pcache) belong to one
    table generation: after mpcx_set_linear_model with other weights (q), and after a schedule
    change that moves the free/blocked boundary (n_free), a handle that has cached the old
    suffix gives the same result as a fresh handle of the new problem, bit for bit (the fresh
    handle's first factorisation is redone on the reused path the cached handle takes; a stale
    cache would give another problem's solution)."""
    from mpcx import lti

    N, B = 100, 64
    rng = np.random.default_rng(7)
    x = rng.uniform([-1, -.5, -.2, -.5], [1, .5, .2, .5], size=(B, 4))
    lin1 = lti.inverted_pendulum_qp(N=N)
    lin2 = lti.inverted_pendulum_qp(N=N, q=(1.5, 2.0))
    lin3 = lti.inverted_pendulum_qp(N=N, n_free=8)
    S = mpcx.nlpsol("pc", "mi355x", lin1, {"ipopt": {"max_iter": 200}})
    P = lti.pendulum_params(lin1, x, 0.0)
    for _ in range(2):  # fill, then use, the cache of lin1
        r1 = S.solve_batch(P)
    ref1 = mpcx.nlpsol("pc1", "mi355x", lin1, {"ipopt": {"max_iter": 200}}).solve_batch(P)
    np.testing.assert_array_equal(r1["iters"], ref1["iters"])
    np.testing.assert_array_equal(r1["w"], ref1["w"])
    for lin in (lin2, lin3):
        S.set_linear_model(lin)
        r = S.solve_batch(P)
        r_again = S.solve_batch(P)
        ref = mpcx.nlpsol("pcf", "mi355x", lin, {"ipopt": {"max_iter": 200}}).solve_batch(P)
        assert np.all(ref["status"] == 0)
        for got in (r, r_again):
            np.testing.assert_array_equal(got["w"], ref["w"])
            np.testing.assert_array_equal(got["lam_g"], ref["lam_g"])
            np.testing.assert_array_equal(got["iters"], ref["iters"])
        assert np.max(np.abs(r["w"] - r1["w"])) > 1e-6  # the problems really differ


def test_pendulum_suffix_cache_off_with_device_schedule(mpcx):
    """A caller-owned device schedule (mpcx_set_linear_tab_dev, one row shared by the batch) may
    be rewritten on the device between launches with no call the suffix cache's generation could
    follow.  Here the rewrite keeps the suffix's first stage (kb = 5) but points the blocked
    stages at a second blocked table with other weights: the result must equal a fresh handle of
    the new schedule, bit for bit (the cross-launch cache is off for device schedules)."""
    import ctypes

    import torch

    from mpcx import lti

    N, B = 100, 64
    rng = np.random.default_rng(8)
    x = rng.uniform([-1, -.5, -.2, -.5], [1, .5, .2, .5], size=(B, 4))
    l1 = lti.inverted_pendulum_qp(N=N)
    l2 = lti.inverted_pendulum_qp(N=N, q=(1.5, 2.0))
    A = np.concatenate([l1.A, l2.A[1:]])
    Bm = np.concatenate([l1.B, l2.B[1:]])
    W = np.concatenate([l1.W, l2.W[1:]])
    sched1 = np.array([0] * 5 + [1] * (N - 5), np.int32)
    sched2 = np.array([0] * 5 + [2] * (N - 5), np.int32)
    mk = lambda tab: lti.LinearOCP(N=N, A=A, B=Bm, W=W, tab=tab, T=l1.T, u_lb=l1.u_lb, u_ub=l1.u_ub)  # noqa: E731
    lin1 = mk(sched1)
    lin1.x_target = l1.x_target
    P = lti.pendulum_params(lin1, x, 0.0)
    S = mpcx.nlpsol("dt", "mi355x", lin1, {"ipopt": {"max_iter": 200}})
    dev = torch.from_numpy(sched1.copy()).cuda()
    lib = mpcx._lib.load()
    mpcx._lib.check(lib.mpcx_set_linear_tab_dev(S._h.ptr, ctypes.c_void_p(dev.data_ptr()), 1))
    for _ in range(2):  # a cache, were it on, would be filled and then used here
        r1 = S.solve_batch(P)
    ref1 = mpcx.nlpsol("f1", "mi355x", mk(sched1), {"ipopt": {"max_iter": 200}}).solve_batch(P)
    np.testing.assert_array_equal(r1["w"], ref1["w"])
    dev.copy_(torch.from_numpy(sched2))  # in place, on the device: no library call
    torch.cuda.synchronize()
    r2 = S.solve_batch(P)
    ref2 = mpcx.nlpsol("f2", "mi355x", mk(sched2), {"ipopt": {"max_iter": 200}}).solve_batch(P)
    assert np.all(ref2["status"] == 0)
    np.testing.assert_array_equal(r2["w"], ref2["w"])
    np.testing.assert_array_equal(r2["iters"], ref2["iters"])
    assert np.max(np.abs(r2["w"] - r1["w"])) > 1e-6  # the schedules really differ
    mpcx._lib.check(lib.mpcx_set_linear_tab_dev(S._h.ptr, None, 0))


def test_pendulum_run_with_schedule_changes_equals_lockstep(mpcx):
    """Config 5 (N = 100, two-wave groups, the reused suffix as a radix-4 scan whose matrix
    powers are formed once per launch): a multi-step run() whose schedules change from one
    closed-loop step to the next (tabseq; per instance, the blocked stages alternate between
    two tables with other weights) equals lock-step launches with the same schedules, bit for
    bit -- the powers and the suffix formed for one step's tables are not reused for another's."""
    import torch

    from mpcx import lti
    from mpcx.device import DeviceLoop

    N, B, K = 100, 64, 4
    rng = np.random.default_rng(9)
    x = rng.uniform([-1, -.5, -.2, -.5], [1, .5, .2, .5], size=(B, 4))
    l1 = lti.inverted_pendulum_qp(N=N)
    l2 = lti.inverted_pendulum_qp(N=N, q=(1.5, 2.0))
    A = np.concatenate([l1.A, l2.A[1:]])
    Bm = np.concatenate([l1.B, l2.B[1:]])
    W = np.concatenate([l1.W, l2.W[1:]])
    sched = [np.array([0] * 5 + [1 + s] * (N - 5), np.int32) for s in (0, 1)]
    lin = lti.LinearOCP(N=N, A=A, B=Bm, W=W, tab=sched[0], T=l1.T, u_lb=l1.u_lb, u_ub=l1.u_ub)
    lin.x_target = l1.x_target
    P = lti.pendulum_params(lin, x, 0.0)
    S = mpcx.nlpsol("ts", "mi355x", lin, {"ipopt": {"max_iter": 200}})
    tabs = np.stack([np.stack([sched[(t + b // 8) % 2] for b in range(B)]) for t in range(K)])
    dt = torch.from_numpy(np.ascontiguousarray(tabs)).cuda()
    lock = DeviceLoop(S, P)
    st_l, it_l = [], []
    for t in range(K):
        lock.set_schedule(dt[t])
        lock.step()
        torch.cuda.synchronize()
        st_l.append(lock.status.cpu().numpy().copy())
        it_l.append(lock.iters.cpu().numpy().copy())
    lock.set_schedule(None)
    run = DeviceLoop(S, P)
    run.set_schedule(dt[0])
    st_r, it_r = run.run(K, tabseq=dt)
    torch.cuda.synchronize()
    run.set_schedule(None)
    assert np.all(np.array(st_l) == 0)
    np.testing.assert_array_equal(st_r.cpu().numpy(), np.array(st_l))
    np.testing.assert_array_equal(it_r.cpu().numpy(), np.array(it_l))
    for n in ("P", "w", "w0", "lam", "lamx", "f"):
        got, want = getattr(run, n).cpu().numpy(), getattr(lock, n).cpu().numpy()
        np.testing.assert_array_equal(got, want, err_msg=n)
    # the schedules matter: one table throughout gives other inputs
    one = DeviceLoop(S, P)
    one.set_schedule(dt[0])
    one.run(K, tabseq=dt[:1].expand(K, B, N).contiguous())
    torch.cuda.synchronize()
    one.set_schedule(None)
    assert np.max(np.abs(one.w.cpu().numpy() - run.w.cpu().numpy())) > 1e-6


def test_padded_double_integrator_closed_loop(mpcx, R):
    """A 2-state model (double integrator, no kernel instantiation of its own) through the
    CasADi-shaped call and the integrator, in the reference's closed-loop pattern
    (solve, apply u_0 through F, shift): every step's inputs match the LQ oracle, F matches
    A x + B u + c, and the returned multipliers / g have the user's (unpadded) sizes."""
    from mpcx import lti

    T, N = 0.1, 20
    A = np.array([[1.0, T], [0.0, 1.0]])
    Bm = np.array([[0.5 * T * T], [T]])
    W = np.diag([1.0, 0.1, 0.01])
    lin = lti.LinearOCP(N=N, A=A[None], B=Bm[None], W=W[None], tab=np.zeros(N, np.int32), u_lb=(-1.0,), u_ub=(1.0,))
    S = mpcx.nlpsol("dint", "mi355x", lin, {"ipopt": {"max_iter": 200}})
    F = mpcx.integrator(lin)
    assert (S.n_w, S.n_g, S.n_p) == (2 + 3 * N, 2 * (N + 1), 2 + 3 * N)
    x = np.array([5.0, 0.0])
    zr = np.zeros((N, 3))
    lbx = np.full(S.n_w, -np.inf)
    ubx = np.full(S.n_w, np.inf)
    lbx[2::3], ubx[2::3] = -1.0, 1.0  # CasADi-style: the input bounds come with the call
    w0 = None
    for t in range(60):
        p = lin.params(x, zr)[0]
        sol = S(x0=w0, p=p, lbx=lbx, ubx=ubx)
        assert S.stats()["success"], t
        assert sol["x"].shape == (S.n_w, 1) and sol["lam_g"].shape == (S.n_g, 1) and sol["g"].shape == (S.n_g, 1)
        w = sol["x"][:, 0]
        _, U_ref, _ = R.lq_solve(x, lin.A, lin.B, lin.c, lin.W, lin.tab, zr, [-1.0], [1.0])
        # bang-bang inputs leave the bound with a multiplier ~ 0 (degenerate): an interior point
        # at tol 1e-8 is O(sqrt(mu)) from the vertex there, as in the random problems above
        assert rel(w[2::3], U_ref[:, 0]) <= 1e-4, t
        assert np.max(np.abs(sol["g"])) <= 1e-8
        xf = F(p, w[2])[0][:, 0]
        np.testing.assert_allclose(xf, A @ x + Bm[:, 0] * w[2], rtol=1e-14, atol=1e-14)
        x = xf
        w0 = np.concatenate([w[0:2] * 0 + x, w[5:], w[-3:]])  # shifted guess (X_0 = new state)
    assert abs(x[0]) < 1.0  # driven towards the origin under |u| <= 1


def test_padded_model_device_loop(mpcx, R):
    """DeviceLoop on a 3-state model embedded in the 4-state kernel: P0 in the model's layout,
    device state in the kernel's (pad states 0 throughout), u_0 of every warm-started step
    equal to the LQ oracle's, the plant-updated state equal to A x + B u + c."""
    import torch
    from mpcx import lti
    from mpcx.device import DeviceLoop

    rng = np.random.default_rng(21)
    nx, N, B = 3, 15, 16
    A = rng.normal(size=(nx, nx))
    A = 0.98 * A / max(abs(np.linalg.eigvals(A)))
    Bm = rng.normal(size=(nx, 1))
    c = 0.05 * rng.normal(size=nx)
    M = rng.normal(size=(nx + 1, nx + 1))
    W = M @ M.T / 4 + 0.1 * np.eye(nx + 1)
    lin = lti.LinearOCP(N=N, A=A[None], B=Bm[None], c=c[None], W=W[None], tab=np.zeros(N, np.int32),
                        u_lb=(-0.5,), u_ub=(0.5,))
    S = mpcx.nlpsol("pad3", "mi355x", lin, {"ipopt": {"max_iter": 200}})
    pd = S._pad
    assert pd is not None and pd.nxp == 4
    x = 2.0 * rng.normal(size=(B, nx))
    zr = np.zeros((N, nx + 1))
    loop = DeviceLoop(S, lin.params(x, zr), device="cuda:0")
    for step in range(8):
        loop.step()
        torch.cuda.synchronize()
        assert np.all(loop.status.cpu().numpy() == 0), step
        wk = loop.w.cpu().numpy()
        assert np.all(wk.reshape(B, -1)[:, 3:4] == 0)  # X_0's pad entry
        w = pd.gather(wk, pd.w_idx)
        for b in range(B):
            _, U_ref, _ = R.lq_solve(x[b], lin.A, lin.B, lin.c, lin.W, lin.tab, zr, [-0.5], [0.5])
            # random bounded problem: near-degenerate bounds, held to the north-star 1e-4 (see above)
            assert rel(w[b, nx::nx + 1], U_ref[:, 0]) <= 1e-4, (step, b)
        x = x @ A.T + w[:, nx:nx + 1] * Bm[:, 0][None, :] + c
        Pk = loop.P.cpu().numpy()
        np.testing.assert_allclose(Pk[:, 0:nx], x, rtol=1e-12, atol=1e-12)
        assert np.all(Pk[:, nx:4] == 0)


def test_lateral_error_lti_closed_loop(mpcx, R):
    """``Trajectory Tracking/Trajectory_tracking_le_LTI.py`` end to end: 500 steps of lane_change.csv
    with the script's references (:104-128), one solve per step through the CasADi-shaped façade,
    x_{t+1} = the solver's predicted x_1 (solver.fixvar, :145).  Every u_0 and x_1 against the
    script's QP restated as a scalar QP (oracle.nlp_ref.lateral_error_solve).  The script keeps no
    output, so parity is to the restatement only (unpinned)."""
    import csv

    from mpcx import lti

    with open(os.path.join(ROOT, "tests", "golden", "lane_change.csv")) as f:
        rows = list(csv.DictReader(f))
    a, b, c = (np.array([float(r[k]) for r in rows]) for k in ("x", "y", "uref"))
    lin = lti.lateral_error_lti(c.mean())
    par = lti.lateral_error_references(a, b, N=lin.N)
    S = mpcx.nlpsol("le_lti", "mi355x", lin, {"ipopt": {"max_iter": 200}})
    lbx = np.full(S.n_w, -np.inf)
    ubx = np.full(S.n_w, np.inf)
    nz = 5
    lbx[4::nz], ubx[4::nz] = -0.3491, 0.3491
    x = np.zeros(3)
    x_ref = np.zeros(3)
    worst = 0.0
    for t in range(len(a)):
        sol = S(p=lti.lateral_error_params(lin, x, 0.0, par[t])[0], lbx=lbx, ubx=ubx)
        assert S.stats()["success"], t
        w = sol["x"][:, 0]
        u_ref, x1_ref = R.lateral_error_solve(x_ref, lin.A_plant, lin.B_plant, par[t])
        worst = max(worst, abs(w[4] - u_ref))
        assert abs(w[4] - u_ref) <= 1e-4, t  # north-star bound (saturated steps sit O(sqrt(mu)) inside)
        x = w[5:8]  # predicted x_1 (the script's fixvar)
        x_ref = x1_ref
        np.testing.assert_allclose(x, x_ref, rtol=0, atol=1e-3)
    print(f"lateral-error LTI: 500 steps, max |u0 - u0_oracle| = {worst:.2e}")


def test_lateral_error_ltv_closed_loop(mpcx, R):
    """``Trajectory Tracking/Trjectory_tracking_le_LTV.py``: the model rebuilt at every step's speed
    c[t] (:130-136, tables re-uploaded through set_linear_model), Q = diag(5, 0, 0), R = 0 (:27-35),
    x_{t+1} = the simulated state (:165-166; exact ZOH here).  500 steps against the scalar-QP
    restatement; unpinned (the script keeps no output)."""
    import csv

    from mpcx import lti

    with open(os.path.join(ROOT, "tests", "golden", "lane_change.csv")) as f:
        rows = list(csv.DictReader(f))
    a, b, c = (np.array([float(r[k]) for r in rows]) for k in ("x", "y", "uref"))
    lin = lti.lateral_error_ltv(c[0])
    par = lti.lateral_error_references(a, b, N=lin.N)
    S = mpcx.nlpsol("le_ltv", "mi355x", lin, {"ipopt": {"max_iter": 300}})
    lbx = np.full(S.n_w, -np.inf)
    ubx = np.full(S.n_w, np.inf)
    lbx[4::5], ubx[4::5] = -0.3491, 0.3491
    x = np.zeros(3)
    worst = 0.0
    for t in range(len(a)):
        lin_t = lti.lateral_error_ltv(c[t])
        S.set_linear_model(lin_t)
        sol = S(p=lti.lateral_error_params(lin_t, x, 0.0, par[t])[0], lbx=lbx, ubx=ubx)
        assert S.stats()["success"], t
        u0 = sol["x"][4, 0]
        u_ref, _ = R.lateral_error_solve(x, lin_t.A_plant, lin_t.B_plant, par[t], q=(5.0, 0.0, 0.0), r=0.0)
        worst = max(worst, abs(u0 - u_ref))
        assert abs(u0 - u_ref) <= 1e-4, t
        x = lin_t.A_plant @ x + lin_t.B_plant[:, 0] * u_ref  # the oracle's input drives both
    print(f"lateral-error LTV: 500 steps, max |u0 - u0_oracle| = {worst:.2e}")
