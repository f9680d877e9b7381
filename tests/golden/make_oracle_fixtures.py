"""Generate the oracle-derived golden vectors of SURVEY.md §8(c) (committed as .npz data).

    python tests/golden/make_oracle_fixtures.py

* ``rk4_sens_random.npz``: seeded random (X, U, P) for 37 instances x 20 intervals ->
  defects c, q, A, B, grad q from oracle/nlp_ref.py (RK4 M=4 quadrature, complex-step
  Jacobian).  Pins the sweep kernel.
* ``unicycle_N20_oracle.npz``: config-2 instances (the first 4 golden P_j and 28 random,
  seed 20261015, N = 20) -> optimum w* and J* of the independent projected-Newton oracle
  from the reference's cold start.  Oracle-pinned (not IPOPT-pinned: the reference never
  ran N = 20).

The oracle itself is pinned by the reference's outputs (tests/test_oracle.py);
tests/test_oracle.py::test_oracle_fixtures_regenerate re-derives a subset to pin these files.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import nlp_ref as R  # noqa: E402


def rk4_sens_case(seed=1, B=37, N=20):
    rng = np.random.default_rng(seed)
    P = np.zeros((B, 6))
    P[:, 0:3] = rng.normal(size=(B, 3)) * 3
    P[:, 3:6] = rng.normal(size=(B, 3)) * 5
    w = rng.normal(size=(B, 3 + 5 * N))
    w[:, 3::5] = rng.uniform(-1, 1, size=(B, N))
    ocp = R.UnicycleOCP(N=N)
    X, U = R.split_w(w, N)
    xr = np.broadcast_to(P[:, None, 3:6], (B, N, 3))
    xf, qf = R.F(X[:, :-1], U, xr, ocp)
    jac = R.stage_jacobian(X[:, :-1], U, xr, ocp)
    return dict(P=P, w=w, c=xf - X[:, 1:], q=qf, A=jac[..., 0:3, 0:3], B=jac[..., 0:3, 3:5], gq=jac[..., 3, :])


def n20_inputs(n_golden=4, n_random=28, seed=20261015):
    with open(os.path.join(HERE, "unicycle_N10_golden.json")) as f:
        rows = np.array(json.load(f)["multiple_shooting"]["rows"])
    Pg, _ = R.golden_pairs(rows)
    rng = np.random.default_rng(seed)
    Pr = np.zeros((n_random, 6))
    Pr[:, 0:2] = rng.uniform(-5, 5, size=(n_random, 2))
    Pr[:, 2] = rng.uniform(-np.pi / 2, np.pi / 2, size=n_random)
    Pr[:, 3:6] = (10.0, 10.0, 0.0)
    return np.concatenate([Pg[:n_golden], Pr])


def n20_solve(P, N=20):
    ocp = R.UnicycleOCP(N=N)
    W, J, ok = [], [], []
    for p in P:
        w, info = R.solve_ms(p, ocp)
        W.append(w)
        J.append(info["J"])
        ok.append(info["status"] == "converged")
    return np.array(W), np.array(J), np.array(ok)


def main():
    np.savez(os.path.join(HERE, "rk4_sens_random.npz"), **rk4_sens_case())
    P = n20_inputs()
    W, J, ok = n20_solve(P)
    np.savez(os.path.join(HERE, "unicycle_N20_oracle.npz"), P=P, w=W, J=J, converged=ok)
    print("wrote rk4_sens_random.npz, unicycle_N20_oracle.npz; converged", int(ok.sum()), "of", len(ok))


if __name__ == "__main__":
    main()
