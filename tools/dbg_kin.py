"""Replays one saved kinematic-bicycle solve (gpurun_out/ode_diag_kin_bicycle.npz, written by
tools/ode_diag.py: parameters, primal and dual warm start of the slowest instances) on the
debug build, which prints the optimality error and the second-order-correction trials of
instance 0 per iteration (make -C mpc-verde_amd debug; python tools/dbg_kin.py [max_iter]).
"""
import os, sys
import numpy as np
ROOT = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
os.environ["MPCX_LIB"] = os.path.join(ROOT, "mpc-verde_amd", "mpcx", "libmpcx_debug.so")
sys.path.insert(0, os.path.join(ROOT, "mpc-verde_amd"))
import mpcx
d = np.load(os.path.join(ROOT, "gpurun_out", "ode_diag_kin_bicycle.npz"))
ocp = mpcx.kinematic_bicycle_tracking(N=30)
s = mpcx.nlpsol("d", "mi355x", ocp, {"ipopt": {"max_iter": int(sys.argv[1]) if len(sys.argv) > 1 else 60}})
r = s.solve_batch(d["P"][:1], d["w0"][:1], lam_g0=d["lam0"][:1], lam_x0=d["lamx0"][:1])
print("status", r["status"], "iters", r["iters"])
