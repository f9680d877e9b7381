"""Re-run the hard-start unicycle closed loop (tests/test_gpu_hard.py) lock-step and dump the
warm starts of every solve that ended with status > 1 (diagnostics: gpurun_out/fail_cases.npz)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mpc-verde_amd"), os.path.join(ROOT, "tests")]
import mpcx  # noqa: E402
from mpcx.device import DeviceLoop  # noqa: E402
from test_gpu_hard import REF_OPTS, hard_unicycle_inputs  # noqa: E402

N, B, K = 20, int(sys.argv[1]) if len(sys.argv) > 1 else 512, int(sys.argv[2]) if len(sys.argv) > 2 else 12
seed = int(sys.argv[3]) if len(sys.argv) > 3 else 5
P = hard_unicycle_inputs(B, seed=seed)
solver = mpcx.nlpsol("hard", "mi355x", mpcx.unicycle_point_to_point(N=N), {"ipopt": REF_OPTS})
lp = DeviceLoop(solver, P)
rec = {k: [] for k in ("P", "w0", "lam0", "lamx0", "status", "iters", "step", "inst")}
for s in range(K):
    snap = {k: getattr(lp, k).cpu().numpy().copy() for k in ("P", "w0", "lam0", "lamx0")}
    lp.step()
    torch.cuda.synchronize()
    st = lp.status.cpu().numpy()
    it = lp.iters.cpu().numpy()
    for b in np.flatnonzero(st > 1):
        for k in ("P", "w0", "lam0", "lamx0"):
            rec[k].append(snap[k][b])
        rec["status"].append(st[b]); rec["iters"].append(it[b]); rec["step"].append(s); rec["inst"].append(b)
        print(f"step {s} instance {b}: status {st[b]} after {it[b]} iterations, P {snap['P'][b]}")
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", "fail_cases.npz"), **{k: np.array(v) for k, v in rec.items()})
