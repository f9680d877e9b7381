"""How often the bench closed loops reach a failed filter line search (where the kernel parks the
instance for IPOPT's restoration): the config-2/3 unicycle loops run lock-step with restoration
off, statuses counted per step (status 1 at a failed line search = "restoration phase called at an
acceptable point", 3 = failed).  Diagnostic only.

    python tools/park_count.py CONFIG [B] [STEPS]
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mpc-verde_amd")]
import mpcx  # noqa: E402
from mpcx import dist as mdist  # noqa: E402
from mpcx.device import DeviceLoop  # noqa: E402

cfg = int(sys.argv[1])
B = int(sys.argv[2]) if len(sys.argv) > 2 else (1024 if cfg == 2 else 4096)
S = int(sys.argv[3]) if len(sys.argv) > 3 else 43
for resto in (False, True):
    if cfg == 2:
        ocp = mpcx.unicycle_point_to_point(N=20)
        opts = {"ipopt": {"max_iter": 2000, "acceptable_tol": 1e-8, "acceptable_obj_change_tol": 1e-6}}
        P0 = mdist.config2_inputs(0, B)
        refs = None
    else:
        ocp = mpcx.unicycle_tracking(N=30)
        opts = {"ipopt": {"max_iter": 3000}}
        tau0, P0 = mdist.config3_inputs(0, B, N=30)
        refs = torch.from_numpy(np.stack([mpcx.ocp.circular_reference(tau0, t, 30).reshape(B, -1)
                                          for t in range(S)])).cuda()
    solver = mpcx.nlpsol("pc", "mi355x", ocp, {**opts, "restoration": resto})
    lp = DeviceLoop(solver, P0)
    st, it = [], []
    for t in range(S):
        if refs is not None:
            lp.set_stage_refs(refs[t])
        lp.step()
        torch.cuda.synchronize()
        st.append(lp.status.cpu().numpy().copy())
        it.append(lp.iters.cpu().numpy().copy())
    st, it = np.array(st), np.array(it)
    print(f"config {cfg} restoration={resto}: statuses {np.bincount(st.ravel(), minlength=6).tolist()} over {S} steps x {B}; "
          f"iters max {it.max()} mean {it.mean():.2f}; steps with status>0: {sorted(set(np.nonzero(st > 0)[0].tolist()))[:20]}")
    if not resto:
        off_st = st
    else:
        d = np.argwhere(st != off_st)
        print(f"  instance-steps whose status changed with restoration: {len(d)}; first {d[:10].tolist()}")
