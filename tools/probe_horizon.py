"""Probe: solve a few instances at horizon N for each model; print status/iters/first inputs."""
import sys

import numpy as np

sys.path.insert(0, "mpc-verde_amd")
import mpcx  # noqa: E402
from mpcx import lti  # noqa: E402

for N in [int(v) for v in sys.argv[1:]]:
    lin = lti.inverted_pendulum_qp(N=N)
    S = mpcx.nlpsol("p", "mi355x", lin, {"ipopt": {"max_iter": 200}})
    r = S.solve_batch(lti.pendulum_params(lin, np.array([[0.1, 0, 0, 0], [0.5, 0, 0.1, 0]]), 0.0))
    print("pend N", N, "status", r["status"], "iters", r["iters"], "f", r["f"], "u", r["w"][:, 5:5 + 30:6], flush=True)
    S2 = mpcx.nlpsol("u", "mi355x", mpcx.unicycle_point_to_point(N=N))
    r = S2.solve_batch(np.array([[0, 0, 0, 10, 10, 0.0], [1, 2, 0.3, 10, 10, 0]]))
    print("uni N", N, "status", r["status"], "iters", r["iters"], "f", r["f"], "u0", r["w"][:, 3:5], flush=True)
