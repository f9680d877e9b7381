"""GPU tests on the inputs the benches never draw, against the C++ IPOPT restatement
(oracle/ipm_ref.cpp) from the same starting points:

* the unicycle NLP of Casadi/multiple_shooting_casadi.py at N = 20 on non-convex instances:
  headings over the whole circle, targets behind and beside the vehicle, targets at distance
  ~0 and exactly 0, target headings a half turn away (SURVEY.md §7 hard part 3: turn left vs
  right).  Both sides run IPOPT's restoration (the kernel: the soft restoration step inline and
  the restoration phase in the resume launch, csrc/resto.h; the oracle: ipm_ref.cpp's), so an
  instance one side restores and the other does not shows up as a status or iteration
  difference.  Statuses, iteration counts and optima are compared instance by instance (counts
  printed; 0 differ);
* the same starts through the device closed loop (multi-step launch == lock-step launches);
* IPOPT's park-and-resume path (restoration in a second launch, resto.h) through DeviceLoop:
  the fused step epilogue and multi-step launches with parked instances, bit for bit against
  the unfused path.

Parity: the unicycle NLP is pinned to the reference's IPOPT outputs (tests/golden); these inputs
have no reference output, so they are held to the oracle.  Tolerance: controls 1e-4 relative to
max(|u|_inf, 1e-3) (north star).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REL_TOL = 1e-4
KKT_CERT_TOL = 1e-8
REF_OPTS = {"max_iter": 2000, "acceptable_tol": 1e-8, "acceptable_obj_change_tol": 1e-6}  # :188-196


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


def hard_unicycle_inputs(B=1024, seed=20261017):
    """P = [x0; x_target] rows: exact degenerate cases first, then random hard draws by kind
    (0 target behind, 1 beside, 2 at distance < 1e-2, 3 anywhere), headings in [-pi, pi]."""
    rows = []
    for dth in (0.0, 1e-9, 0.5, np.pi / 2, np.pi - 1e-6, np.pi, -np.pi, 2 * np.pi, 3.0):
        rows.append([0, 0, 0, 0, 0, dth])  # already at the target position
        rows.append([1, 2, np.pi, 1, 2, np.pi + dth])
    for d in (1e-6, 1e-3, 0.1, 1.0, 3.0, 10.0):
        for th in np.linspace(-np.pi, np.pi, 5):
            for rel in (np.pi, np.pi / 2, -np.pi / 2, 3 * np.pi / 4):
                rows.append([0, 0, th, d * np.cos(th + rel), d * np.sin(th + rel), th + np.pi])
    rows = np.array(rows, float)
    n = B - rows.shape[0]
    rng = np.random.default_rng(seed)
    P = np.zeros((n, 6))
    P[:, 0:2] = rng.uniform(-5, 5, (n, 2))
    P[:, 2] = rng.uniform(-np.pi, np.pi, n)
    kind = np.arange(n) % 4
    th = P[:, 2]
    side = np.where(rng.uniform(size=n) < 0.5, -1.0, 1.0)
    ang = np.where(kind == 0, th + np.pi + rng.uniform(-0.5, 0.5, n), th + side * np.pi / 2)
    d = np.where(kind == 2, rng.uniform(0, 1e-2, n), rng.uniform(0.5, 6, n))
    ang = np.where(kind == 2, rng.uniform(-np.pi, np.pi, n), ang)
    P[:, 3] = P[:, 0] + d * np.cos(ang)
    P[:, 4] = P[:, 1] + d * np.sin(ang)
    P[:, 5] = rng.uniform(-np.pi, np.pi, n)
    far = kind == 3
    P[far, 3:5] = rng.uniform(-10, 10, (int(far.sum()), 2))
    return np.concatenate([rows, P])


def rel_err_rows(a, b):
    return np.max(np.abs(a - b), axis=1) / np.maximum(np.max(np.abs(b), axis=1), 1e-3)


def test_unicycle_hard_instances_vs_oracle_with_restoration(mpcx, C):
    from oracle import nlp_ref as R

    N, B = 20, 1024
    P = hard_unicycle_inputs(B)
    ocp = mpcx.unicycle_point_to_point(N=N)
    r = mpcx.nlpsol("hard", "mi355x", ocp, {"ipopt": REF_OPTS}).solve_batch(P)
    rocp = R.UnicycleOCP(N=N)
    ref = C.solve(rocp, P, restoration=1, nthreads=0, **REF_OPTS)
    print(f"hard unicycle: kernel statuses {np.bincount(r['status'], minlength=6).tolist()}, "
          f"oracle (restoration on) {np.bincount(ref['status'], minlength=6).tolist()}; "
          f"iterations max {r['iters'].max()} / {ref['iters'].max()}")
    assert np.all(r["status"] <= 1), np.flatnonzero(r["status"] > 1)
    assert np.all(ref["status"] <= 1), np.flatnonzero(ref["status"] > 1)
    n_st = int(np.sum(r["status"] != ref["status"]))
    n_it = int(np.sum(r["iters"] != ref["iters"]))
    errs = rel_err_rows(r["w"], ref["w"])
    diff = np.flatnonzero(errs > REL_TOL)
    print(f"hard unicycle: {n_st} statuses, {n_it} iteration counts and {diff.size} optima of {B} differ "
          f"from the oracle (max error {errs.max():.2e})")
    assert n_st == 0
    for b in diff:  # a different local optimum must still be a KKT point of the NLP
        pg, cv = R.kkt_residual_ms(r["w"][b], r["lam_g"][b], P[b], rocp)
        assert pg <= KKT_CERT_TOL and cv <= KKT_CERT_TOL, (b, pg, cv)
    # measured on MI355X: 0 differing optima and iteration counts
    assert diff.size == 0 and n_it == 0, (diff, np.flatnonzero(r["iters"] != ref["iters"]))


def test_unicycle_hard_closed_loop_run_equals_lockstep(mpcx):
    """The hard starts through the device closed loop: K lock-step launches == one K-step
    launch, bit for bit, and every solve of every step ends at status <= 1."""
    import torch

    from mpcx.device import DeviceLoop

    N, B, K = 20, 512, 12
    P = hard_unicycle_inputs(B, seed=5)
    solver = mpcx.nlpsol("hard", "mi355x", mpcx.unicycle_point_to_point(N=N), {"ipopt": REF_OPTS})
    lock, run = DeviceLoop(solver, P), DeviceLoop(solver, P)
    st_l, it_l = [], []
    for _ in range(K):
        lock.step()
        torch.cuda.synchronize()
        st_l.append(lock.status.cpu().numpy().copy())
        it_l.append(lock.iters.cpu().numpy().copy())
    st_r, it_r = run.run(K)
    torch.cuda.synchronize()
    st_l, it_l = np.array(st_l), np.array(it_l)
    print(f"hard closed loop: statuses {np.bincount(st_l.ravel(), minlength=6).tolist()}, "
          f"iterations mean {it_l.mean():.2f} max {it_l.max()}")
    assert np.all(st_l <= 1)
    np.testing.assert_array_equal(st_r.cpu().numpy(), st_l)
    np.testing.assert_array_equal(it_r.cpu().numpy(), it_l)
    for n in ("P", "w", "w0", "lam", "lamx", "f"):
        np.testing.assert_array_equal(getattr(run, n).cpu().numpy(), getattr(lock, n).cpu().numpy(), err_msg=n)


def _dyn_case(mpcx, idx, K):
    from mpcx import dist as mdist

    N = 50
    ocp = mpcx.dynamic_bicycle_lane_change(N=N)
    t0, x0, (X, Y, V) = mdist.config4_bicycle_inputs(0, 1024)
    t0, x0 = t0[idx], x0[idx]
    refs = np.stack([np.stack([mpcx.ode.dyn_bicycle_references(X, Y, V, int(t) + s, N).reshape(-1) for t in t0])
                     for s in range(K)])  # (K, B, N nz)
    return ocp, ocp.params(x0, refs[0]), refs


def test_park_and_resume_through_device_loop(mpcx):
    """Instances whose cold-start line search fails (config-4 6-state bicycle 262, 483, 10; they
    end at status 3 without restoration) next to instances that never park, through the device
    loop: the fused step (solve + resume launch + in-place plant/shift epilogue) equals separate
    solve and shift launches, K-step launches (parked instances resume at their step, reload the
    step's references from Pseq and write per-step status rows while the others finished all K
    steps in the first launch) equal K lock-step launches, and the first step equals the
    restoration-on batched solve -- all bit for bit."""
    import torch

    from mpcx.device import DeviceLoop

    idx = [262, 483, 10, 0, 1, 2, 3, 4]
    K = 3
    ocp, P0, refs = _dyn_case(mpcx, idx, K)
    opts = {"ipopt": {"max_iter": 3000}}
    off = mpcx.nlpsol("off", "mi355x", ocp, {**opts, "restoration": False}).solve_batch(P0)
    assert np.all(off["status"][:3] == 3), off["status"]  # these park when restoration is on
    solver = mpcx.nlpsol("dyn", "mi355x", ocp, opts)
    first = solver.solve_batch(P0)
    dr = torch.from_numpy(np.ascontiguousarray(refs)).cuda()
    fused, split, run = DeviceLoop(solver, P0), DeviceLoop(solver, P0), DeviceLoop(solver, P0)
    st_f, it_f = [], []
    for s in range(K):
        for lp in (fused, split):
            lp.set_stage_refs(dr[s])
        fused.step()
        split.solve()
        split.shift()
        torch.cuda.synchronize()
        if s == 0:
            np.testing.assert_array_equal(fused.w.cpu().numpy(), first["w"])
            np.testing.assert_array_equal(fused.status.cpu().numpy(), first["status"])
        st_f.append(fused.status.cpu().numpy().copy())
        it_f.append(fused.iters.cpu().numpy().copy())
        for n in ("P", "w", "w0", "lam", "lam0", "lamx", "lamx0", "f", "status", "iters"):
            np.testing.assert_array_equal(getattr(split, n).cpu().numpy(), getattr(fused, n).cpu().numpy(),
                                          err_msg=f"step {s}: {n}")
    st_f, it_f = np.array(st_f), np.array(it_f)
    assert np.all(st_f <= 1), st_f
    Pseq = np.zeros((K, len(idx), P0.shape[1]))
    Pseq[:, :, 6:] = refs
    st_r, it_r = run.run(K, Pseq=torch.from_numpy(Pseq).cuda())
    torch.cuda.synchronize()
    print(f"park/resume: iterations per step {it_f.tolist()}")
    np.testing.assert_array_equal(st_r.cpu().numpy(), st_f)
    np.testing.assert_array_equal(it_r.cpu().numpy(), it_f)
    for n in ("w", "w0", "lam", "lamx", "f"):
        np.testing.assert_array_equal(getattr(run, n).cpu().numpy(), getattr(fused, n).cpu().numpy(), err_msg=n)
    np.testing.assert_array_equal(run.P.cpu().numpy()[:, 0:6], fused.P.cpu().numpy()[:, 0:6])


def test_park_slots_cleared_between_batch_sizes(mpcx):
    """A handle's restoration workspace is laid out by each launch's thread count.  A parking
    launch at B = 1024 followed by a parking launch at B = 8 on the SAME handle must give, bit for
    bit, what a fresh handle gives for the 8 instances (and what the big launch gave for them):
    the solve launch clears every thread's park slot, so the resume launch sees only the instances
    its own solve launch parked (config-4 6-state bicycle; 262, 483 and 10 park from the cold
    start)."""
    from mpcx import dist as mdist

    N = 50
    ocp = mpcx.dynamic_bicycle_lane_change(N=N)
    t0, x0, (X, Y, V) = mdist.config4_bicycle_inputs(0, 1024)
    refs = np.stack([mpcx.ode.dyn_bicycle_references(X, Y, V, int(t), N).reshape(-1) for t in t0])
    P = ocp.params(x0, refs)
    opts = {"ipopt": {"max_iter": 3000}}
    reused = mpcx.nlpsol("reused", "mi355x", ocp, opts)
    big = reused.solve_batch(P)
    assert np.all(big["status"] <= 1), np.flatnonzero(big["status"] > 1)
    idx = [0, 262, 1, 2, 3, 4, 5, 6]
    small = reused.solve_batch(P[idx])
    fresh = mpcx.nlpsol("fresh", "mi355x", ocp, opts).solve_batch(P[idx])
    for n in ("w", "f", "lam_g", "lam_x", "status", "iters"):
        np.testing.assert_array_equal(small[n], fresh[n], err_msg=n)
        np.testing.assert_array_equal(small[n], big[n][idx], err_msg=n)
