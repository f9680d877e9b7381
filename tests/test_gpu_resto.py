"""GPU tests of IPOPT's recovery and termination paths in the kernel, against the C++ IPOPT
restatement (oracle/ipm_ref.cpp) from the same starting points:

* the BASELINE-named nonlinear configs as named -- config 4's 6-state dynamic bicycle at N = 50
  on the bench's 1024-instance batch (vx >= 2.5 bound included) and config 5's single-shooting
  cart-pole swing-up at N = 100 -- every instance ends at IPOPT status <= 1, at the oracle's
  optimum or at a KKT point the oracle certifies (counts printed and bounded);
* the soft restoration / restoration phase (W&B 2006 §3.3) recovers the cold-start instances whose
  line search fails, with the oracle's outcome;
* the acceptable-level termination (acceptable_tol / acceptable_iter) at the oracle's iteration.

PARITY UNPINNED for the ODE models (no reference outputs exist: BASELINE extensions); the oracle
is an independent restatement of the same algorithm.  Tolerances: inputs 1e-6 relative to
max(|u|_inf, 1); KKT residual (oracle/ode_ref.py) <= 1e-6, constraint violation <= tol = 1e-8.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

U_TOL = 1e-6


@pytest.fixture(scope="module")
def mpcx():
    import mpcx as m

    m._lib.load()
    return m


@pytest.fixture(scope="module")
def C():
    from oracle import ipm_ref

    ipm_ref.lib()
    return ipm_ref


def u_err(wa, wb, nx, nz, N):
    """max over the controls, relative to max(|u|_inf, 1), per instance."""
    iu = np.concatenate([nx + nz * k + np.arange(nz - nx) for k in range(N)])
    ua, ub = wa[:, iu], wb[:, iu]
    return np.max(np.abs(ua - ub), axis=1) / np.maximum(np.max(np.abs(ub), axis=1), 1.0)


def config4_batch(mpcx, B=1024, N=50):
    from mpcx import dist as mdist

    ocp = mpcx.dynamic_bicycle_lane_change(N=N)
    t0, x0, (X, Y, V) = mdist.config4_bicycle_inputs(0, B)
    refs = np.stack([mpcx.ode.dyn_bicycle_references(X, Y, V, int(t), N).reshape(-1) for t in t0])
    return ocp, ocp.params(x0, refs)


def certify(pr, r, P, b):
    kkt, gres = pr.kkt_residual(r["w"][b], r["lam_g"][b], r["lam_x"][b], P[b])
    return kkt <= 1e-6 and gres <= 1e-8, (kkt, gres)  # tol = 1e-8 (constraint violation)


def compare(name, ocp, P, r, ref, nx, nz, max_differ, max_iter_differ):
    """Same outcome as the oracle instance by instance; the differing ones must be KKT points."""
    from oracle import ode_ref

    N = ocp.N
    assert np.all(r["status"] <= 1), np.unique(r["status"], return_counts=True)
    assert np.all(ref["status"] <= 1), np.unique(ref["status"], return_counts=True)
    e = u_err(r["w"], ref["w"], nx, nz, N)
    differ = np.flatnonzero(e > U_TOL)
    n_it = int(np.sum(r["iters"] != ref["iters"]))
    print(f"{name}: {len(differ)} of {len(P)} instances differ from the C++ oracle by > {U_TOL} "
          f"(max {e.max():.2e}); {n_it} iteration counts differ; statuses {np.bincount(r['status'], minlength=2)}")
    assert len(differ) <= max_differ, differ
    assert n_it <= max_iter_differ
    pr = ode_ref.Problem(ocp)
    for b in differ:
        ok, res = certify(pr, r, P, b)
        assert ok, (b, res)


def test_config4_dyn_bicycle_batch_vs_ipopt_oracle(mpcx, C):
    """BASELINE config 4 as named: 6-state dynamic bicycle, lane_change.csv reference, N = 50, the
    bench's 1024 instances, cold start (X_k = x0, U = 0) in both.  100 % status <= 1 (before the
    restoration phase 3 of these ended in a failed line search).  The bounds are the measured
    counts (the kernel is deterministic): 5 optima differ, each KKT-certified, and 108 iteration
    counts, from rounding growth between the hyper-dual and jet derivatives (DESIGN §6,
    tools/divergence.py) -- any further drift fails the test."""
    ocp, P = config4_batch(mpcx)
    solver = mpcx.nlpsol("dyn", "mi355x", ocp, {"ipopt": {"max_iter": 3000}})
    r = solver.solve_batch(P)
    ref = C.solve(ocp, P, nthreads=0)
    compare("config 4 dyn bicycle N=50", ocp, P, r, ref, 6, 8, max_differ=5, max_iter_differ=108)
    assert np.min(r["w"][:, 6 + 2 + 3::8]) >= 2.5 - 1e-7  # vx >= 2.5 holds on X_1..X_N (stage k: U_k, X_k+1)


def test_config5_single_shooting_swingup_N100(mpcx, C):
    """BASELINE config 5 as named: single-shooting cart-pole swing-up, N = 100, 128 instances of the
    bench's random hanging starts.  The single-shooting start (x0 = U = 0, X the rollout) goes to
    the kernel and to the oracle alike; the CasADi-shaped single-shooting call is checked on a few
    instances for the same answer as the batched form."""
    import math

    from mpcx import dist as mdist
    from oracle import ode_ref

    N, B = 100, 128
    ocp = mpcx.cartpole_swingup(N=N, formulation="single_shooting")
    P = mdist.config5_swingup_inputs(0, B)
    pr = ode_ref.Problem(ocp)
    U0 = np.zeros((N, 1))
    w0 = np.stack([pr.join_w(pr.rollout(U0, P[b][:4]), U0) for b in range(B)])
    solver = mpcx.nlpsol("ss", "mi355x", ocp, {"ipopt": {"max_iter": 3000}})
    r = solver.solve_batch(P, w0)
    ref = C.solve(ocp, P, w0=w0, nthreads=0)
    compare("config 5 single-shooting swing-up N=100", ocp, P, r, ref, 4, 5, max_differ=0, max_iter_differ=0)
    for b in range(3):  # the CasADi-shaped call: decision U, g = X_1..X_N
        sol = solver(x0=[0.0] * N, lbx=-200.0, ubx=200.0, lbg=-math.inf, ubg=math.inf, p=P[b])
        assert solver.stats()["success"]
        np.testing.assert_allclose(sol["x"][:, 0], r["w"][b, 4::5], rtol=0, atol=1e-9)


def test_restoration_recovers_failed_line_searches(mpcx, C):
    """Cold-start instances of configs 4 and 5 whose filter line search fails: without restoration
    the solve ends there (status 3, as IPOPT would have to enter restoration); with IPOPT's soft
    restoration and restoration phase every one converges, to the oracle's optimum."""
    from mpcx import dist as mdist

    ocp4, P4 = config4_batch(mpcx)
    ocp5 = mpcx.cartpole_swingup(N=100)
    P5 = mdist.config5_swingup_inputs(0, 2048)
    for ocp, P, idx in ((ocp4, P4, [262, 483, 10]), (ocp5, P5, [313, 12, 74, 396, 1232, 1639, 1728, 1722, 1649, 1524])):
        P = P[idx]
        off = mpcx.nlpsol("off", "mi355x", ocp, {"ipopt": {"max_iter": 3000}, "restoration": False}).solve_batch(P)
        on = mpcx.nlpsol("on", "mi355x", ocp, {"ipopt": {"max_iter": 3000}}).solve_batch(P)
        ref_off = C.solve(ocp, P, restoration=0)
        ref = C.solve(ocp, P)
        assert np.all(off["status"] == 3) and np.all(ref_off["status"] == 3), (off["status"], ref_off["status"])
        print(f"{ocp.model}: failed line search at iteration kernel {off['iters'].tolist()} oracle {ref_off['iters'].tolist()}")
        assert np.all(on["status"] == 0) and np.all(ref["status"] == 0), (on["status"], ref["status"])
        e = u_err(on["w"], ref["w"], ocp.nx, ocp.nz, ocp.N)
        print(f"{ocp.model}: restoration iterations kernel {on['iters'].tolist()} oracle {ref['iters'].tolist()}, "
              f"max input difference {e.max():.2e}")
        assert e.max() <= U_TOL


def test_kin_bicycle_iteration_counts_vs_oracle(mpcx, C):
    """Config 3 variant (kinematic bicycle, N = 30): kernel and oracle take the same number of
    iterations on the cold config-3 batch (IPOPT's fast barrier decrease and tiny-step rule on both)."""
    from mpcx import dist as mdist

    ocp = mpcx.kinematic_bicycle_tracking(N=30)
    _, P = mdist.config3_bicycle_inputs(0, 1024, N=30)
    r = mpcx.nlpsol("kin", "mi355x", ocp, {"ipopt": {"max_iter": 3000}}).solve_batch(P)
    ref = C.solve(ocp, P, nthreads=0)
    compare("config 3 kinematic bicycle N=30", ocp, P, r, ref, 3, 5, max_differ=0, max_iter_differ=0)


def test_acceptable_level_termination_matches_oracle(mpcx, C):
    """IPOPT's acceptable-level termination: with acceptable_tol = 1e-4 and acceptable_iter = 3
    (tol 1e-12 out of reach of those iterations) a solve ends with status 1 at its third iterate in
    a row below 1e-4, at the oracle's iteration, instance by instance; with the reference's own
    options (acceptable_tol = tol = 1e-8, :192-193) every instance converges (status 0)."""
    from mpcx import dist
    from oracle import nlp_ref

    N, B = 20, 256
    P = dist.config2_inputs(0, B)
    ocp = mpcx.unicycle_point_to_point(N=N)
    opts = {"tol": 1e-12, "acceptable_tol": 1e-4, "acceptable_iter": 3}
    r = mpcx.nlpsol("acc", "mi355x", ocp, {"ipopt": opts}).solve_batch(P)
    # both sides restore (the kernel's default; the oracle's restoration = 1): an instance that one
    # side recovers and the other ends at a failed line search shows up as a status difference
    ref = C.solve(nlp_ref.UnicycleOCP(N=N), P, restoration=1, nthreads=0, **opts)
    n_st = int(np.sum(r["status"] != ref["status"]))
    n_it = int(np.sum(r["iters"] != ref["iters"]))
    print(f"acceptable level: statuses {np.unique(r['status'], return_counts=True)}; {n_st} statuses and {n_it} "
          f"iteration counts of {B} differ from the oracle")
    assert np.sum(r["status"] == 1) >= B // 4
    assert n_st == 0 and n_it == 0
    r2 = mpcx.nlpsol("ref", "mi355x", ocp, {"ipopt": {"max_iter": 2000, "acceptable_tol": 1e-8,
                                                       "acceptable_obj_change_tol": 1e-6}}).solve_batch(P)
    assert np.all(r2["status"] == 0)


def test_kin_bicycle_closed_loop_outliers_vs_unbounded_filter_oracle(mpcx, C):
    """The filter holds kFilterSlots x G entries in the lanes (kernels.h FilterLanes), dominated
    entries dropped as in IPOPT's Filter::AddEntry; the oracle's filter is unbounded.  The
    kinematic bicycle's 23-step closed loop (config 3 variant, 1024 instances) has the longest
    solves of any workload (up to ~160 iterations, hundreds of filter rejections): its 16
    slowest solves, re-run from their recorded warm starts, take the oracle's iterations (one
    may differ by one iteration) with the same outcome and optimum; no filter overflow occurs
    (tools/ode_diag.py filter_overflows = 0 on this loop)."""
    import torch

    from mpcx import dist as mdist
    from mpcx.device import DeviceLoop

    N, B, S = 30, 1024, 23
    ocp = mpcx.kinematic_bicycle_tracking(N=N)
    tau0, P0 = mdist.config3_bicycle_inputs(0, B, N=N)
    solver = mpcx.nlpsol("kin", "mi355x", ocp, {"ipopt": {"max_iter": 3000}})
    loop = DeviceLoop(solver, P0)
    rec = {"P": [], "w0": [], "lam0": [], "lamx0": [], "iters": []}
    for s in range(S):
        refs = mpcx.ode.bicycle_circular_reference(tau0, s, N).reshape(B, -1)
        loop.set_stage_refs(torch.from_numpy(np.ascontiguousarray(refs)).cuda())
        for k, t in (("P", loop.P), ("w0", loop.w0), ("lam0", loop.lam0), ("lamx0", loop.lamx0)):
            rec[k].append(t.cpu().numpy().copy())
        loop.step()
        torch.cuda.synchronize()
        rec["iters"].append(loop.iters.cpu().numpy().copy())
        assert np.all(loop.status.cpu().numpy() <= 1)
    its = np.array(rec["iters"])  # (S, B)
    worst = np.argsort(-its[1:].ravel())[:16] + B  # warm-started steps (step 0 is covered above)
    st, ib = worst // B, worst % B
    pick = {k: np.stack([rec[k][s][b] for s, b in zip(st, ib)]) for k in ("P", "w0", "lam0", "lamx0")}
    r = solver.solve_batch(pick["P"], pick["w0"], lam_g0=pick["lam0"], lam_x0=pick["lamx0"])
    ref = C.solve(ocp, pick["P"], w0=pick["w0"], lam0=pick["lam0"], lamx0=pick["lamx0"], warm=(1e-4, 1e-4, 1e-4))
    print(f"kin bicycle closed-loop outliers: loop {its[st, ib].tolist()}, re-run {r['iters'].tolist()}, "
          f"oracle {ref['iters'].tolist()}")
    np.testing.assert_array_equal(r["iters"], its[st, ib])
    d_it = np.abs(r["iters"] - ref["iters"])
    # measured: 15 of 16 equal, one 130 vs 131 (the same optimum; rounding after 130 iterations)
    assert np.sum(d_it > 0) <= 1 and d_it.max() <= 1, (r["iters"], ref["iters"])
    np.testing.assert_array_equal(r["status"], ref["status"])
    assert np.max(u_err(r["w"], ref["w"], 3, 5, N)) <= U_TOL
