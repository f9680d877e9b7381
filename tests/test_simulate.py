"""The reference's own visualisation, ``simulation_code.simulate`` (/root/reference/simulation_code.py:10-94),
driven UNCHANGED on the closed-loop arrays mpcx produces ("the driver loop ...
plus simulation_code.simulate, must run unchanged on these outputs").

The arrays come from mpcx/record.py's ClosedLoopLog -- the class the GPU closed-loop test
(tests/test_gpu_parity.py::test_casadi_call_shapes_and_closed_loop) fills from mpcx.nlpsol --
here filled by the reference's driver loop (Casadi/multiple_shooting_casadi.py:224-298, its
stacked-layout warm start included) run on the C++ CPU oracle, which reproduces 1exemplo.xlsx.
CPU only; it reads /root/reference, so it runs in the build container and is skipped where the
reference is absent (the GPU box).  matplotlib runs on the Agg backend and FuncAnimation is
replaced by a driver that calls the script's init_func and animate(i) for every frame and renders
the figure after each, so every frame the animation would show is drawn.
"""
import importlib.util
import math
import os

import numpy as np
import pytest

REF_SIM = "/root/reference/simulation_code.py"

pytestmark = pytest.mark.skipif(not os.path.exists(REF_SIM), reason="reference sources absent (GPU box)")


def reference_loop_log(N=10, T=0.2):
    """The driver loop of multiple_shooting_casadi.py:224-298 on the C++ oracle, recorded by
    ClosedLoopLog as the script records cat_states / cat_controls / t / times (:210-270)."""
    from mpcx.record import ClosedLoopLog
    from oracle import ipm_ref, nlp_ref

    ocp = nlp_ref.UnicycleOCP(N=N)
    state_init = np.zeros(3)
    state_target = np.array([10.0, 10.0, 0.0])
    w0 = np.zeros(3 + 5 * N)
    log = ClosedLoopLog(3, 2, N, T, state_init)
    mpc_iter, t0 = 0, 0.0
    while np.linalg.norm(state_init - state_target) > 1e-1 and mpc_iter * T < 20:
        P = np.concatenate([state_init, state_target])[None, :]
        r = ipm_ref.solve(ocp, P, w0=w0[None, :], max_iter=2000, acceptable_tol=1e-8, acceptable_obj_change_tol=1e-6)
        assert r["status"][0] <= 1
        x = r["w"][0]
        u = np.array([x[3 + 5 * k:5 + 5 * k] for k in range(N)]).T
        X0 = np.array([x[0:3]] + [x[5 + 5 * k:8 + 5 * k] for k in range(N)]).T
        log.record(x, t0, wall_time=0.0)
        t0 += T
        state_init, _ = nlp_ref.F(P[0, 0:3], u[:, 0], state_target, ocp)
        u0 = np.hstack([u[:, 1:], u[:, -1:]])
        X0 = np.hstack([X0[:, 1:], X0[:, -1:]])
        w0 = np.concatenate([X0.T.reshape(-1), u0.T.reshape(-1)])  # the script's stacked layout (:284-287)
        mpc_iter += 1
    return log, mpc_iter


def test_reference_simulate_runs_unchanged_on_closed_loop_log(monkeypatch, golden):
    matplotlib = pytest.importorskip("matplotlib")
    matplotlib.use("Agg", force=True)
    from matplotlib import animation

    drawn = []

    class EveryFrame:
        """FuncAnimation stand-in: init, then animate(i) and a full render for each frame."""

        def __init__(self, fig=None, func=None, frames=None, init_func=None, **kw):
            if init_func is not None:
                init_func()
            n = frames if isinstance(frames, int) else len(list(frames))
            for i in range(n):
                func(i)
                fig.canvas.draw()
                drawn.append(i)

        def save(self, *a, **kw):
            raise AssertionError("simulate(save=False) must not save")

    monkeypatch.setattr(animation, "FuncAnimation", EveryFrame)
    spec = importlib.util.spec_from_file_location("simulation_code", REF_SIM)
    sim = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(sim)  # module body: imports and the function definition only

    N, T = 10, 0.2
    log, iters = reference_loop_log(N, T)
    rows = np.array(golden["multiple_shooting"]["rows"])
    assert iters == 84 and log.cat_states.shape == (3, N + 1, 85)
    # the arrays are the reference's (cat_states[:, 0, :] = its exported state rows)
    assert np.max(np.abs(log.cat_states[:, 0, :].T - rows[:, 0:3])) < 1e-6
    reference = np.array([0.0, 0.0, 0.0, 10.0, 10.0, 0.0])  # [x_init, y_init, theta_init, x_target, ...]
    # the script's own (commented) call, :312-313: simulate(cat_states, cat_controls, times, T, N, ...)
    sim.simulate(log.cat_states, log.cat_controls, log.times, T, N, reference, save=False)
    assert drawn == list(range(len(log.t))) and len(log.t) == 85
    assert math.isclose(float(log.t[-1, 0]), 83 * T)
