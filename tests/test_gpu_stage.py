"""The unicycle stage derivatives of the solve kernel (mpc-verde_amd/csrc/unicycle.h) through the
device harness tests/hip/stage_check.hip: the weighted-moment assembly the kernel uses
(uni_derivs_moments) against the per-point formula (uni_derivs) on the device, and both against
the C++ oracle's jets (oracle/ipm_ref.cpp oracle_stage: interval map, Jacobian, gradient of q and
the exact Hessian of q + lam^T xf), for the quadrature cost (Casadi/multiple_shooting_casadi.py:
98-114, M = 4) and the node cost (Trajectory_tracking.py:51-61, M = 1).

Tolerances: the two device formulas <= 1e-12 relative to the entry's scale (they sum the same
terms in another order); device vs oracle <= 1e-11 relative to the largest entry of its block.
"""
import ctypes
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "hip", "libstage_check.so")


@pytest.fixture(scope="module")
def harness():
    import torch  # noqa: F401  (its HIP runtime first: the harness must bind to the same one)

    if not os.path.exists(LIB):
        pytest.fail(f"{LIB} not built (make -C tests/hip)")
    lib = ctypes.CDLL(LIB)
    dp = ctypes.c_void_p
    lib.stage_check.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                ctypes.POINTER(ctypes.c_double), dp, dp, dp, dp, dp, ctypes.c_double, dp]
    return lib


def run(harness, n, T, M, cost, Q, R, X, U, XR, UR, L, fs):
    import torch

    dev = [torch.from_numpy(np.ascontiguousarray(a, np.float64)).cuda() for a in (X, U, XR, UR, L)]
    out = torch.zeros(2 * n * 39, dtype=torch.float64, device="cuda")
    q = (ctypes.c_double * 3)(*Q)
    r = (ctypes.c_double * 2)(*R)
    rc = harness.stage_check(n, T, M, cost, q, r, *[ctypes.c_void_p(t.data_ptr()) for t in dev], fs,
                             ctypes.c_void_p(out.data_ptr()))
    assert rc == 0
    o = out.cpu().numpy().reshape(2, n, 39)
    return o[0], o[1]


def blocks(o):
    return {"xf": o[:, 0:3], "q": o[:, 3:4], "A": o[:, 4:13], "B": o[:, 13:19], "g": o[:, 19:24], "H": o[:, 24:39]}


@pytest.mark.parametrize("cost,M", [(0, 4), (0, 1), (0, 7), (1, 1)])
def test_moment_assembly_equals_per_point_formula_and_oracle(harness, cost, M):
    from oracle import ipm_ref, nlp_ref

    rng = np.random.default_rng(10 + M + cost)
    n = 4096
    T = 0.2
    Q, R = (1.0, 5.0, 0.1), (0.5, 0.05)
    X = np.column_stack([rng.uniform(-10, 10, n), rng.uniform(-10, 10, n), rng.uniform(-4, 4, n)])
    U = np.column_stack([rng.uniform(-1, 1, n), rng.uniform(-np.pi / 4, np.pi / 4, n)])
    XR = np.column_stack([rng.uniform(-10, 10, n), rng.uniform(-10, 10, n), rng.uniform(-4, 4, n)])
    UR = np.column_stack([rng.uniform(-1, 1, n), rng.uniform(-1, 1, n)]) if cost == 1 else np.zeros((n, 2))
    L = rng.normal(size=(n, 3)) * 5
    # degenerate rows: standing still, at the reference, zero rotation
    X[:8] = XR[:8]
    U[:4, 0] = 0.0
    U[4:8, 1] = 0.0
    mom, pp = (blocks(o) for o in run(harness, n, T, M, cost, Q, R, X, U, XR, UR, L, 1.0))
    for name in mom:
        scale = np.maximum(np.max(np.abs(pp[name]), axis=1, keepdims=True), 1.0)
        err = np.max(np.abs(mom[name] - pp[name]) / scale)
        assert err <= 1e-12, (name, err)
    # the C++ oracle (jets): fs = 1
    ocp = nlp_ref.UnicycleOCP(N=1, M=M)
    ocp.cost = "quadrature" if cost == 0 else "node"
    xf, qf, jac, hess = ipm_ref.stage(ocp, X, U, XR, UR if cost == 1 else None, L)
    ref = {"xf": xf, "q": qf[:, None], "A": jac[:, 0:3, 0:3].reshape(n, 9), "B": jac[:, 0:3, 3:5].reshape(n, 6),
           "g": jac[:, 3, :], "H": hess}
    for name in mom:
        scale = max(1.0, float(np.max(np.abs(ref[name]))))
        err = float(np.max(np.abs(mom[name] - ref[name]))) / scale
        assert err <= 1e-11, (name, err)
    # objective scaling fs: g and H scale (the lam^T xf part of H does not)
    mom2 = blocks(run(harness, n, T, M, cost, Q, R, X, U, XR, UR, np.zeros_like(L), 0.25)[0])
    mom1 = blocks(run(harness, n, T, M, cost, Q, R, X, U, XR, UR, np.zeros_like(L), 1.0)[0])
    np.testing.assert_allclose(mom2["g"], 0.25 * mom1["g"], rtol=1e-13, atol=1e-13)
    np.testing.assert_allclose(mom2["H"], 0.25 * mom1["H"], rtol=1e-13, atol=1e-13)


def pack(M):
    n = M.shape[-1]
    return np.stack([M[..., i, j] for i in range(n) for j in range(i, n)], axis=-1)


def unpack(v, n):
    M = np.zeros(v.shape[:-1] + (n, n))
    t = 0
    for i in range(n):
        for j in range(i, n):
            M[..., i, j] = M[..., j, i] = v[..., t]
            t += 1
    return M


def test_riccati_step_vs_dense_formula(harness):
    """One backward step of the config-2 chain (riccati.h riccati_step with the unicycle's masks,
    unit entries and Hux' = A^T (P B)) against the dense formulas: H' = Hd + M^T P M, g' = gp +
    M^T (P c + p) with M = [A B]; P_k = Hxx' - Hux'^T Huu'^-1 Hux', p_k = gx' - Hux'^T Huu'^-1
    gu', K = -Huu'^-1 Hux', k_f = -Huu'^-1 gu' (<= 1e-10 relative), and the inertia verdict taken
    from the factors after the chain (fac_ok) equals the step's own test and numpy's."""
    import torch

    rng = np.random.default_rng(3)
    n = 8192
    T = 0.2
    A = np.tile(np.eye(3), (n, 1, 1))
    A[:, 0, 2], A[:, 1, 2] = rng.normal(size=n), rng.normal(size=n)
    Bm = np.zeros((n, 3, 2))
    Bm[:, 0:2, :] = rng.normal(size=(n, 2, 2)) * 0.2
    Bm[:, 2, 1] = T
    L = rng.normal(size=(n, 5, 5))
    Hd = np.einsum("bij,bkj->bik", L, L) * 0.5
    Hd[n // 2:] -= 1.5 * np.eye(5)  # half of them indefinite in places
    Lp = rng.normal(size=(n, 3, 3))
    P1 = np.einsum("bij,bkj->bik", Lp, Lp)
    gp, c, p1 = rng.normal(size=(n, 5)), rng.normal(size=(n, 3)) * 0.1, rng.normal(size=(n, 3))
    inp = np.concatenate([pack(Hd), gp, A.reshape(n, 9), Bm.reshape(n, 6), c, pack(P1), p1], axis=1)
    d_in = torch.from_numpy(np.ascontiguousarray(inp)).cuda()
    d_out = torch.zeros(n * 18, dtype=torch.float64, device="cuda")
    harness.riccati_check.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    assert harness.riccati_check(n, ctypes.c_void_p(d_in.data_ptr()), ctypes.c_void_p(d_out.data_ptr())) == 0
    o = d_out.cpu().numpy().reshape(n, 18)
    M = np.concatenate([A, Bm], axis=2)
    H = Hd + np.einsum("bki,bkl,blj->bij", M, P1, M)
    g = gp + np.einsum("bki,bk->bi", M, np.einsum("bij,bj->bi", P1, c) + p1)
    Huu, Hux, gu = H[:, 3:, 3:], H[:, 3:, :3], g[:, 3:]
    pd = np.all(np.linalg.eigvalsh(Huu) > 0, axis=1)
    assert 0.2 * n < pd.sum() < 0.95 * n
    assert not np.any(o[:, 9] == 0.5)  # fac_ok == the step's own test on every instance
    np.testing.assert_array_equal(o[:, 9] == 1.0, pd)
    iH = np.linalg.inv(Huu[pd])
    K = -iH @ Hux[pd]
    kf = -np.einsum("bij,bj->bi", iH, gu[pd])
    Pn = H[pd, :3, :3] + np.einsum("bki,bkj->bij", Hux[pd], K)
    pn = g[pd, :3] + np.einsum("bki,bk->bi", Hux[pd], kf)
    for got, ref in ((o[pd, 0:6], pack(Pn)), (o[pd, 6:9], pn), (o[pd, 10:16], K.reshape(-1, 6)), (o[pd, 16:18], kf)):
        scale = np.maximum(np.max(np.abs(ref), axis=1, keepdims=True), 1.0)
        cond = np.linalg.cond(Huu[pd])[:, None]
        err = np.abs(got - ref) / scale / np.maximum(cond, 1.0)
        assert err.max() <= 1e-12, err.max()


def test_fast_log_exp_accuracy(harness):
    """The solve kernel's fp64 log and exp (csrc/fastmath.h: the barrier log-sums and the line
    search's switching condition) against numpy's, on 10^6-scale samples over the whole normal
    range, near 1 (where log cancels) and at the special values the library path takes: <= 2 ulp
    (the algorithm measures < 1 ulp with exact division; v_rcp_f64 + two Newton steps adds at most
    an ulp)."""
    import torch

    rng = np.random.default_rng(3)
    x = np.concatenate([np.exp(rng.uniform(-708, 709, 2_000_000)), 1.0 + rng.uniform(-0.3, 0.3, 500_000),
                        rng.uniform(0.5, 1.0, 500_000),
                        [1.0, 0.5, 2.0, 1e-310, 0.0, np.inf, 2.2250738585072014e-308, -1.0, np.nan]])
    y = np.concatenate([rng.uniform(-745, 709, 2_000_000), rng.uniform(-1, 1, 1_000_000),
                        [0.0, -800.0, 800.0, -np.inf, np.inf, 1e-300, -708.5, 5.0, np.nan]])
    n = x.size
    assert y.size == n
    harness.fastmath_check.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    dx, dy = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()
    out = torch.zeros(2 * n, dtype=torch.float64, device="cuda")
    assert harness.fastmath_check(n, ctypes.c_void_p(dx.data_ptr()), ctypes.c_void_p(dy.data_ptr()),
                                  ctypes.c_void_p(out.data_ptr())) == 0
    o = out.cpu().numpy().reshape(n, 2)
    with np.errstate(divide="ignore", over="ignore", under="ignore", invalid="ignore"):
        for got, ref in ((o[:, 0], np.log(x)), (o[:, 1], np.exp(y))):
            fin = np.isfinite(ref) & (ref != 0)  # the special values: 0 -> -inf, inf, x < 0 and nan -> nan
            np.testing.assert_array_equal(got[~fin], ref[~fin])
            ulp = np.abs(got[fin] - ref[fin]) / np.spacing(np.abs(ref[fin]))
            print(f"max {ulp.max():.2f} ulp over {fin.sum()} finite values")
            assert ulp.max() <= 2.0

