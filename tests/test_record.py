"""Output-format compatibility, CPU only.

ClosedLoopLog must rebuild the reference's cat_states / cat_controls / t and its exported
table with the row alignment of Casadi/multiple_shooting_casadi.py:316-334 -- checked
against the reference's own 1exemplo.xlsx (tests/golden) -- and write_xlsx must produce a
file the stdlib decoder (tests/golden/make_golden.py) reads back exactly.
"""
import io
import json
import os

import numpy as np
import pytest

from conftest import ROOT


@pytest.fixture(scope="module")
def rows(golden):
    return np.array(golden["multiple_shooting"]["rows"])


def synth_w(x0, u0, N, rng):
    """An interleaved solution vector with X_0 = x0, U_0 = u0 and arbitrary tail."""
    w = rng.normal(size=3 + 5 * N)
    w[0:3] = x0
    w[3:5] = u0
    return w


def test_split_solution_matches_reference_extraction():
    from mpcx.record import split_solution

    N = 4
    w = np.arange(3 + 5 * N, dtype=float)
    X, U = split_solution(w, 3, 2, N)
    # :243-256: u = w[3:5], then w[e], w[e+1] with e = 3 + 5k; X0 = w[0:3], then w[e:e+3], e = 5 + 5k
    np.testing.assert_array_equal(U[:, 0], w[3:5])
    np.testing.assert_array_equal(U[:, 2], w[13:15])
    np.testing.assert_array_equal(X[:, 0], w[0:3])
    np.testing.assert_array_equal(X[:, 1], w[5:8])
    np.testing.assert_array_equal(X[:, N], w[5 + 5 * (N - 1):8 + 5 * (N - 1)])


def test_log_reproduces_1exemplo_layout(rows):
    """Feeding the golden loop's solves (X_0 of solve j = state row j+1, u0 of solve j =
    control row j) through ClosedLoopLog gives back the golden table, time column included."""
    from mpcx.record import ClosedLoopLog

    N, T = 10, 0.2
    rng = np.random.default_rng(0)
    log = ClosedLoopLog(3, 2, N, T, x_init=[0, 0, 0])
    t0 = 0.0
    for j in range(84):
        log.record(synth_w(rows[j + 1, 0:3], rows[j, 3:5], N, rng), t0)
        t0 += T
    assert log.cat_states.shape == (3, N + 1, 85)
    assert log.cat_controls.shape == (170, 1) and log.t.shape == (85, 1)
    tab = log.table()
    got = np.stack([tab[c] for c in ("x", "y", "theta", "v", "w", "t")], axis=1)
    np.testing.assert_array_equal(got[:, 0:5], rows[:, 0:5])
    np.testing.assert_allclose(got[:, 5], rows[:, 5], rtol=0, atol=1e-12)


def test_xlsx_roundtrip(rows):
    import sys

    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from make_golden import read_xlsx
    from mpcx.record import write_xlsx

    table = {c: rows[:, i] for i, c in enumerate(("x", "y", "theta", "v", "w", "t"))}
    b = io.BytesIO()
    write_xlsx(b, table)
    b.seek(0)
    back = read_xlsx(b)
    assert back[0][:6] == ["x", "y", "theta", "v", "w", "t"]  # header (index column unnamed)
    vals = np.array([r[1:7] for r in back[1:]])
    idx = np.array([r[0] for r in back[1:]])
    np.testing.assert_array_equal(vals, rows)  # repr() round-trips fp64 exactly
    np.testing.assert_array_equal(idx, np.arange(85))


def test_pendulum_table_matches_invertpend(tmp_path):
    from oracle import nlp_ref as R
    from mpcx.record import pendulum_table

    with open(os.path.join(ROOT, "tests", "golden", "pendulum_N50_golden.json")) as f:
        gold = np.array(json.load(f)["rows"])
    xs, us = R.pendulum_closed_loop(nsim=1000)
    tab = pendulum_table(xs.T, us[None, :], 0.01)
    got = np.stack([tab[c] for c in ("x", "x_dot", "theta", "theta_dot", "u", "t")], axis=1)
    assert got.shape == gold.shape
    np.testing.assert_allclose(got[:, 0:5], gold[:, 0:5], rtol=0, atol=1e-8)
    np.testing.assert_allclose(got[:, 5], gold[:, 5], rtol=0, atol=1e-12)
