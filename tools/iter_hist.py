"""Iteration-count distribution of the config-2 closed loop (which instances set the per-step max)."""
import json
import sys

import numpy as np

sys.path.insert(0, "mpc-verde_amd")
import torch  # noqa: E402

import mpcx  # noqa: E402
from mpcx import dist as mdist  # noqa: E402
from mpcx.device import DeviceLoop  # noqa: E402

B, N, S = 1024, 20, 23
solver = mpcx.nlpsol("s", "mi355x", mpcx.unicycle_point_to_point(N=N))
loop = DeviceLoop(solver, mdist.config2_inputs(0, B))
its = []
Ps = []
for s in range(S):
    Ps.append(loop.P.cpu().numpy().copy())
    loop.step()
    torch.cuda.synchronize()
    its.append(loop.iters.cpu().numpy().copy())
its = np.array(its)  # (S, B)
Ps = np.array(Ps)
out = {"per_step_max": its.max(1).tolist(), "per_step_mean": np.round(its.mean(1), 2).tolist()}
h = np.bincount(its[3:].ravel())
out["hist_steps_3_on"] = h.tolist()
# slow instances: describe their state
slow = np.argwhere(its[3:] >= 9)
rows = []
for s, b in slow[:25]:
    P = Ps[s + 3, b]
    d = np.hypot(P[0] - P[3], P[1] - P[4])
    rows.append({"step": int(s + 3), "b": int(b), "iters": int(its[s + 3, b]), "dist": round(float(d), 3),
                 "theta": round(float(P[2]), 3), "prev_iters": int(its[s + 2, b])})
out["slow"] = rows
out["n_slow_ge9"] = int((its[3:] >= 9).sum())
print(json.dumps(out))
