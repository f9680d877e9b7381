#!/usr/bin/env python3
"""Config-5 closed loop on one library (MPCX_LIB): W warm-up step() launches, then one K-step run();
saves per-step iterations/statuses and the final w to an .npz for comparing two builds.

    MPCX_LIB=... MPCX_ALLOW_STALE_LIB=1 python tools/c5_compare.py OUT.npz [K]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpc-verde_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import mpcx  # noqa: E402
from mpcx import dist as mdist  # noqa: E402
from mpcx.device import DeviceLoop  # noqa: E402

out, K = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 10
B, N = 2048, 100
lin = mpcx.inverted_pendulum_qp(N=N)
solver = mpcx.nlpsol("c5", "mi355x", lin)
loop = DeviceLoop(solver, mpcx.lti.pendulum_params(lin, mdist.config5_inputs(0, B), 0.0))
its_w = []
for _ in range(3):
    loop.step()
    torch.cuda.synchronize()
    its_w.append(loop.iters.cpu().numpy().copy())
st, it = loop.run(K)
torch.cuda.synchronize()
np.savez(out, its_w=np.array(its_w), st=st.cpu().numpy(), it=it.cpu().numpy(), w=loop.w.cpu().numpy(),
         P=loop.P.cpu().numpy())
print("saved", out, "iters sum", int(it.cpu().numpy().sum()))
