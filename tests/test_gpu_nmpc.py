"""The reference's mpctools loops, run as written through the mpctools-shaped façade
(mpc-verde_amd/mpcx/nmpc.py) with only the constructor swapped:

* ``Trajectory Tracking/Trajectory_tracking.py:100-126`` -- 500 steps of the circular tracking
  NLP (N = 10, RK4 M = 1, node cost, x in [-20, 20], y in [-2, 2]): per-stage references through
  ``solver.par["p", k]``, ``solve()``, ``saveguess()``, and the next solve's initial state pinned
  to the previous prediction X_1 by ``fixvar("x", 0, var["x", 1])`` (:112) -- not to the plant's
  state, which the script only records (``model.sim``, an exact ODE step, :121).  Checked
  against the C++ IPOPT restatement (oracle/ipm_ref.cpp) running the same loop: the same pinned
  initial state, the same shifted primal guess.  No reference output exists for this script
  (parity unpinned beyond the pinned unicycle NLP); tolerance: every step's u_0 within 1e-6
  relative to max(|u_0|, 1) of the oracle's, all statuses Solve_Succeeded.
* ``Inverted_pendulum/inverted_pendulum_single_shooting_mpctools.py:64-78`` -- the 1000-step
  cart-pole loop with ``fixvar("x", 0, x0)`` and ``mpc.callSolver`` against
  ``invertpend_data_py.xlsx`` (tests/golden): controls within 1e-4 relative (north star), states
  within 1e-6.
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def mpcx():
    import mpcx as m

    m._lib.load()
    return m


def tracking_par(Nt=10, Nsim=500, Delta=0.2, Nx=3, Nu=2):
    """The script's parameter tensor par[:, k, t] (:87-98)."""
    times = Delta * Nsim * np.linspace(0, 1, Nsim + 1)
    par = np.ones((Nx + Nu, Nt, Nsim))
    for t in range(Nsim):
        for k in range(Nt):
            tp = times[t] + times[k]
            par[:, k, t] = (np.cos(0.1 * tp), np.sin(0.1 * tp), np.pi / 2 + 0.1 * tp, 1.0, 1.0)
    return par


def shift_guess(w, N, nx=3, nu=2, s=1):
    """saveguess(toffset=1) on the multiple-shooting layout: X, U shifted, last entries repeated."""
    nz = nx + nu
    X = np.stack([w[0:nx]] + [w[nx + nz * k + nu:nx + nz * (k + 1)] for k in range(N)])
    U = np.stack([w[nx + nz * k:nx + nz * k + nu] for k in range(N)])
    Xs = np.concatenate([X[s:], np.repeat(X[-1:], s, axis=0)])
    Us = np.concatenate([U[s:], np.repeat(U[-1:], s, axis=0)])
    return np.concatenate([Xs[0]] + [np.concatenate([Us[k], Xs[k + 1]]) for k in range(N)])


def test_trajectory_tracking_script_loop_vs_oracle(mpcx):
    from oracle import ipm_ref as C
    from oracle import nlp_ref as R

    Delta, Nt, Nsim, Nx, Nu = 0.2, 10, 500, 3, 2
    par = tracking_par(Nt, Nsim, Delta)
    x0 = np.array([0, 0, 0])
    p = np.zeros((Nt, Nx + Nu))
    # solver = mpc.nmpc(f=ode_rk4_casadi, N=N, verbosity=0, l=l, x0=x0, lb=lb, ub=ub, p=p, ...)   (:72)
    solver = mpcx.nmpc(mpcx.unicycle_tracking(N=Nt, T=Delta), x0=x0, p=p, verbosity=0)
    x = np.zeros((Nsim + 1, Nx))
    x[0, :] = x0
    u = np.zeros((Nsim, Nu))
    pred, upred, status = [], [], []
    for t in range(Nsim):  # :100-126, as written
        for k in range(Nt):
            solver.par["p", k] = par[:, k, t]
        solver.solve()
        status.append(solver.stats["status"])
        solver.saveguess()
        solver.fixvar("x", 0, solver.var["x", 1])
        u[t, :] = np.array(solver.var["u", 0, :]).flatten()
        pred += [solver.var["x", :, :]]
        upred += [solver.var["u", :, :]]
        x[t + 1, :] = R.unicycle_flow(x[t, :], u[t, :], Delta)  # model.sim: the exact ODE step
    pred3 = np.array([[np.array(j) for j in i] for i in pred])[:, :, :, 0]
    assert pred3.shape == (Nsim, Nt + 1, Nx) and len(upred[0]) == Nt
    assert set(status) == {"Solve_Succeeded"}, sorted(set(status))
    # the same loop on the C++ oracle
    rocp = R.tracking_ocp(N=Nt)
    xs = np.zeros(Nx)
    guess = R.join_w(np.zeros((1, Nt + 1, Nx)), np.zeros((1, Nt, Nu)))
    uo = np.zeros((Nsim, Nu))
    for t in range(Nsim):
        r = C.solve_batch(rocp, xs[None], w0=guess, pstage=par[:, :, t].T[None])
        assert r["status"][0] == 0
        w = r["w"][0]
        uo[t] = w[3:5]
        guess = shift_guess(w, Nt)[None]
        xs = w[5:8].copy()
    err = np.max(np.abs(u - uo), axis=1) / np.maximum(np.max(np.abs(uo), axis=1), 1.0)
    print(f"tracking script loop: max |u0 - u0_oracle| relative {err.max():.2e} over {Nsim} steps; "
          f"final simulated state {x[-1]}")
    assert err.max() <= 1e-6, (int(np.argmax(err)), err.max())


def test_pendulum_script_loop_via_callSolver(mpcx):
    with open(os.path.join(ROOT, "tests", "golden", "pendulum_N50_golden.json")) as f:
        gold = np.array(json.load(f)["rows"])
    lin = mpcx.inverted_pendulum_qp(N=50)
    A, B = lin.A_plant, lin.B_plant

    def ffunc(x, u):  # the script's discrete model (:24-25)
        return A @ x + B @ np.atleast_1d(u)

    Nx, Nu, nsim = 4, 1, 1000
    x0 = np.array([0, 0, 0, 0])
    # solver = mpc.nmpc(f, l, N, x0, lb, ub, isQP=True, verbosity=0, uprev=np.array([0]), ...)   (:64)
    solver = mpcx.nmpc(lin, x0=x0, isQP=True, verbosity=0, uprev=np.array([0]))
    xcl = np.zeros((Nx, nsim + 1))
    xcl[:, 0] = x0
    ucl = np.zeros((Nu, nsim))
    for k in range(nsim):  # :72-78, as written
        solver.fixvar("x", 0, x0)
        sol = mpcx.callSolver(solver)
        assert sol["status"] == "Solve_Succeeded"
        xcl[:, k] = sol["x"][0, :]
        ucl[:, k] = sol["u"][0, :]
        x0 = ffunc(x0, ucl[:, k])
    xcl[:, nsim] = x0
    assert sol["x"].shape == (51, 4) and sol["u"].shape == (50, 1)
    assert np.allclose(sol["u"][5:, 0], sol["u"][4, 0])  # Du = 0 after the 5 free moves (:34-42)
    uerr = np.max(np.abs(ucl[0] - gold[:nsim, 4])) / np.max(np.abs(gold[:nsim, 4]))
    xerr = np.max(np.abs(xcl.T - gold[:, 0:4]))
    print(f"pendulum script loop: controls {uerr:.2e} relative, states {xerr:.2e} absolute vs invertpend_data_py.xlsx")
    assert uerr <= 1e-4 and xerr <= 1e-6
