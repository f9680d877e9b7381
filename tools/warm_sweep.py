"""Iteration counts of the config-2 closed loop for several warm-start settings
(IPOPT's mu_init / warm_start_bound_push / warm_start_mult_push)."""
import json
import sys

import numpy as np

sys.path.insert(0, "mpc-verde_amd")
import torch  # noqa: E402

import mpcx  # noqa: E402
from mpcx import _lib, dist as mdist  # noqa: E402
from mpcx.device import DeviceLoop  # noqa: E402
from mpcx.ocp import to_spec  # noqa: E402

B, N, S = 1024, 20, 23
P0 = mdist.config2_inputs(0, B)
res = []
for warm in [(1e-4, 1e-4, 1e-4), (1e-5, 1e-5, 1e-5), (1e-6, 1e-6, 1e-6), (1e-5, 1e-6, 1e-6), (1e-6, 1e-8, 1e-8),
             (1e-7, 1e-8, 1e-8), (1e-3, 1e-4, 1e-4)]:
    ocp = mpcx.unicycle_point_to_point(N=N)
    solver = mpcx.nlpsol("s", "mi355x", ocp)
    solver._h = _lib.Handle(to_spec(ocp, solver.max_iter, solver.tol, 0, warm=warm))
    loop = DeviceLoop(solver, P0)
    its, st, Pf = [], [], None
    for s in range(S):
        loop.step()
        torch.cuda.synchronize()
        its.append(loop.iters.cpu().numpy().copy())
        st.append(loop.status.cpu().numpy().copy())
    its = np.array(its)[3:]
    st = np.array(st)
    res.append({"warm": warm, "max_per_step_mean": round(float(its.max(1).mean()), 2), "mean": round(float(its.mean()), 3),
                "max": int(its.max()), "failed": int((st > 1).sum()), "final_x_checksum": float(loop.P[:, 0:3].sum())})
    print(json.dumps(res[-1]), flush=True)
