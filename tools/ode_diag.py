"""Per-instance IPM event counters of the nonlinear ODE variants' closed loops (diagnostic build).

    make -C mpc-verde_amd stamps && python tools/ode_diag.py kin_bicycle|dyn_bicycle|cartpole [B] [steps]

Prints iteration/status histograms with the mean event counters per class and saves the slowest
instances' parameter vectors and warm starts (gpurun_out/ode_diag_<model>.npz) for CPU study.
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
         "tiny_steps", "filter_rejections", "armijo_acceptances", "scan_fallbacks", "filter_resets", "soc_eligible", "soc_accepted", "soft_resto_steps", "resto_phases",
         "filter_overflows"]
ND = len(NAMES)  # counters per instance (solver.hip kDiag)


def main():
    model = sys.argv[1]
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    S = int(sys.argv[3]) if len(sys.argv) > 3 else 6
    lib = mpcx._lib.load()
    lib.mpcx_diag_set_counter_buffer.argtypes = [ctypes.c_void_p]
    buf = torch.zeros(B * ND, dtype=torch.int32, device="cuda")
    assert lib.mpcx_diag_set_counter_buffer(ctypes.c_void_p(buf.data_ptr())) == 0
    refs = None
    if model == "kin_bicycle":
        N = 30
        ocp = mpcx.kinematic_bicycle_tracking(N=N)
        tau0, P0 = mdist.config3_bicycle_inputs(0, B, N=N)
        refs = [mpcx.ode.bicycle_circular_reference(tau0, t, N).reshape(B, -1) for t in range(S)]
    elif model == "dyn_bicycle":
        N = 50
        ocp = mpcx.dynamic_bicycle_lane_change(N=N)
        t0, x0, (X, Y, V) = mdist.config4_bicycle_inputs(0, B)
        refs = [np.stack([mpcx.ode.dyn_bicycle_references(X, Y, V, int(ti) + t, N).reshape(-1) for ti in t0])
                for t in range(S)]
        P0 = ocp.params(x0, refs[0])
    else:
        N = 100
        ocp = mpcx.cartpole_swingup(N=N)
        P0 = mdist.config5_swingup_inputs(0, B)
    solver = mpcx.nlpsol("s", "mi355x", ocp, {"ipopt": {"max_iter": 3000}})
    loop = DeviceLoop(solver, P0)
    its, sts, cnt, Ps, W0, L0, LX0 = [], [], [], [], [], [], []
    for s in range(S):
        if refs is not None:
            loop.set_stage_refs(torch.from_numpy(np.ascontiguousarray(refs[s])).cuda())
        Ps.append(loop.P.cpu().numpy().copy())
        W0.append(loop.w0.cpu().numpy().copy())
        L0.append(loop.lam0.cpu().numpy().copy())
        LX0.append(loop.lamx0.cpu().numpy().copy())
        loop.step()
        torch.cuda.synchronize()
        its.append(loop.iters.cpu().numpy().copy())
        sts.append(loop.status.cpu().numpy().copy())
        cnt.append(buf.cpu().numpy().reshape(B, ND).copy())
    its, sts, cnt = np.array(its), np.array(sts), np.array(cnt)
    out = {"model": model, "B": B, "steps": S, "iters_per_step_mean": its.mean(axis=1).round(2).tolist(),
           "iters_per_step_max": its.max(axis=1).tolist(), "failed_per_step": (sts > 1).sum(axis=1).tolist()}
    fi, fc = its.ravel(), cnt.reshape(-1, ND)
    for label, m in (("iters<=10", fi <= 10), ("iters 11-50", (fi > 10) & (fi <= 50)), ("iters>50", fi > 50)):
        out[label] = {"n": int(m.sum()), **{NAMES[i]: round(float(fc[m, i].mean()), 2) if m.any() else None
                                            for i in range(ND)}}
    worst = np.argsort(-its.ravel())[:16]
    out["worst"] = [{"step": int(w // B), "inst": int(w % B), "iters": int(fi[w]), "status": int(sts.ravel()[w]),
                     **{NAMES[i]: int(fc[w, i]) for i in range(ND)}} for w in worst[:8]]
    print(json.dumps(out, indent=1))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez(os.path.join(ROOT, "gpurun_out", f"ode_diag_{model}.npz"),
             P=np.array([Ps[w // B][w % B] for w in worst]), w0=np.array([W0[w // B][w % B] for w in worst]),
             lam0=np.array([L0[w // B][w % B] for w in worst]), lamx0=np.array([LX0[w // B][w % B] for w in worst]),
             step=worst // B, inst=worst % B, iters=fi[worst], status=sts.ravel()[worst])


if __name__ == "__main__":
    main()
