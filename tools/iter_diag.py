"""Per-instance IPM event counters of the config-2 closed loop (diagnostic build).

    make -C mpc-verde_amd stamps && python tools/iter_diag.py
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["MPCX_LIB"] = os.path.join(ROOT, "mpc-verde_amd", "mpcx", "libmpcx_stamps.so")
sys.path.insert(0, os.path.join(ROOT, "mpc-verde_amd"))
import torch  # noqa: E402

import mpcx  # noqa: E402
from mpcx import dist as mdist  # noqa: E402
from mpcx.device import DeviceLoop  # noqa: E402

NAMES = ["regularised_iters", "extra_factorisations", "backtracks", "barrier_updates", "ftb_limited_steps",
         "tiny_steps", "filter_rejections", "armijo_acceptances", "scan_fallbacks", "filter_resets", "soc_eligible", "soc_accepted",
         "soft_resto_steps", "resto_phases", "filter_overflows"]
ND = len(NAMES)  # counters per instance (solver.hip kDiag)


def main():
    cfg = int(os.environ.get("DIAG_CONFIG", "2"))  # 2: unicycle point-to-point, 5: cart-pole QP
    B = 1024 if cfg == 2 else 2048
    N, S = int(os.environ.get("DIAG_N", "20" if cfg == 2 else "100")), 23
    lib = mpcx._lib.load()
    lib.mpcx_diag_set_counter_buffer.argtypes = [ctypes.c_void_p]
    buf = torch.zeros(B * ND, dtype=torch.int32, device="cuda")
    assert lib.mpcx_diag_set_counter_buffer(ctypes.c_void_p(buf.data_ptr())) == 0
    if cfg == 2:
        solver = mpcx.nlpsol("s", "mi355x", mpcx.unicycle_point_to_point(N=N))
        loop = DeviceLoop(solver, mdist.config2_inputs(0, B))
    else:
        solver = mpcx.nlpsol("s", "mi355x", mpcx.inverted_pendulum_qp(N=N))
        loop = DeviceLoop(solver, mpcx.lti.pendulum_params(solver.ocp, mdist.config5_inputs(0, B), 0.0))
    its, cnt = [], []
    for s in range(S):
        loop.step()
        torch.cuda.synchronize()
        its.append(loop.iters.cpu().numpy().copy())
        cnt.append(buf.cpu().numpy().reshape(B, ND).copy())
    its = np.array(its)[3:].ravel()
    cnt = np.array(cnt)[3:].reshape(-1, ND)
    out = {}
    for label, m in (("iters<=5", its <= 5), ("iters 6-8", (its >= 6) & (its <= 8)), ("iters>=9", its >= 9)):
        out[label] = {"n": int(m.sum()), **{NAMES[i]: round(float(cnt[m, i].mean()), 3) for i in range(ND)}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
