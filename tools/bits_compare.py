#!/usr/bin/env python3
"""Results of one library build for a bit-for-bit comparison with another (A/B of a kernel change
that must not change any result): a cold solve_batch of a bench workload's batch and a 3-step
device closed loop, saved to an .npz.

    MPCX_LIB=... MPCX_ALLOW_STALE_LIB=1 python tools/bits_compare.py {c2,c5,dyn} OUT.npz
    python tools/bits_compare.py --diff A.npz B.npz
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpc-verde_amd"))
import numpy as np  # noqa: E402

if sys.argv[1] == "--diff":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    bad = [k for k in a.files if not np.array_equal(a[k], b[k])]
    for k in a.files:
        print(k, "DIFFERENT" if k in bad else "identical")
    sys.exit(1 if bad else 0)

import torch  # noqa: E402

import mpcx  # noqa: E402
from mpcx import dist as mdist  # noqa: E402
from mpcx.device import DeviceLoop  # noqa: E402

work, out = sys.argv[1], sys.argv[2]
if work == "dyn":  # config 4 variant: 6-state dynamic bicycle, N = 50, B = 1024
    N, B = 50, 1024
    ocp = mpcx.dynamic_bicycle_lane_change(N=N)
    t0, x0, (X, Y, V) = mdist.config4_bicycle_inputs(0, B)
    refs = np.stack([mpcx.ode.dyn_bicycle_references(X, Y, V, int(t), N).reshape(-1) for t in t0])
    P = ocp.params(x0, refs)
elif work == "c2":  # config 2
    ocp = mpcx.unicycle_point_to_point(N=20)
    P = mdist.config2_inputs(0, 1024)
elif work == "c5":  # config 5: cart-pole QP, N = 100, B = 2048 (two-wave groups, the suffix scan)
    from mpcx import lti

    ocp = lti.inverted_pendulum_qp(N=100)
    P = lti.pendulum_params(ocp, mdist.config5_inputs(0, 2048), 0.0)
else:
    raise SystemExit(f"unknown workload {work}")
solver = mpcx.nlpsol("s", "mi355x", ocp, {"ipopt": {"max_iter": 3000}})
r = solver.solve_batch(P)
loop = DeviceLoop(solver, P)
st, it = loop.run(3)
torch.cuda.synchronize()
np.savez(out, w=r["w"], iters=r["iters"], status=r["status"], lam_g=r["lam_g"], st=st.cpu().numpy(),
         it=it.cpu().numpy(), loop_w=loop.w.cpu().numpy())
print(f"{work}: iters mean {r['iters'].mean():.2f}, statuses {np.bincount(r['status'])}")
