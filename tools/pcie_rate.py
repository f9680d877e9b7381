"""Host-buffer (PCIe-inclusive) solve rate vs device-resident rate, config-2 instances.

mpcx_solve_batch copies P / w0 / multipliers host->device and w / f / lambda device->host
around the same kernel that mpcx_solve_batch_dev launches on device-resident inputs.
"""
import json
import sys
import time

import numpy as np

sys.path.insert(0, "mpc-verde_amd")
import torch  # noqa: E402

import mpcx  # noqa: E402
from mpcx import dist as mdist  # noqa: E402
from mpcx.device import DeviceLoop  # noqa: E402

B, N, reps = 1024, 20, 20
solver = mpcx.nlpsol("s", "mi355x", mpcx.unicycle_point_to_point(N=N))
P = mdist.config2_inputs(0, B)
r = solver.solve_batch(P)  # cold, warm-up
t = []
for _ in range(reps):
    t0 = time.perf_counter()
    r = solver.solve_batch(P, w0=r["w"], lam_g0=r["lam_g"], lam_x0=r["lam_x"])
    t.append(time.perf_counter() - t0)
host_ms = float(np.median(t)) * 1e3
loop = DeviceLoop(solver, P)
loop.solve()
torch.cuda.synchronize()
loop.w0.copy_(loop.w)
loop.lam0.copy_(loop.lam)
loop.lamx0.copy_(loop.lamx)
ev = []
for _ in range(reps):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    loop.solve()
    b.record()
    ev.append((a, b))
torch.cuda.synchronize()
dev_ms = float(np.median([a.elapsed_time(b) for a, b in ev]))
print(json.dumps({"B": B, "N": N, "host_path_ms": round(host_ms, 4), "host_path_solves_per_s": round(B / host_ms * 1e3),
                  "device_ms": round(dev_ms, 4), "device_solves_per_s": round(B / dev_ms * 1e3),
                  "note": "same instances re-solved from their own optimum + multipliers (warm), median of 20"}))
