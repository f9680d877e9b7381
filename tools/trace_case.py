"""Per-iteration trace of one recorded solve (npz with P, w0, lam0, lamx0 rows; tools/find_fail.py): kernel
(MPCX_LIB=...libmpcx_debug.so / _stamps.so, MPCX_ALLOW_STALE_LIB=1) or oracle (ORACLE_TRACE=1).  Diagnostic only."""
import os, sys, numpy as np
ROOT = "/root/repo" if os.path.exists("/root/repo/bench.py") else os.environ["GRAFT_REPO_ROOT"]
sys.path[:0] = [ROOT, ROOT + "/mpc-verde_amd"]
d = np.load(sys.argv[2])
P, w0, l0, lx0 = d["P"], d["w0"], d["lam0"], d["lamx0"]
o = dict(max_iter=2000, acceptable_tol=1e-8, acceptable_obj_change_tol=1e-6)
import mpcx
if sys.argv[1] == "kernel":
    r = mpcx.nlpsol("d", "mi355x", mpcx.unicycle_point_to_point(N=20), {"ipopt": o}).solve_batch(P, w0, lam_g0=l0, lam_x0=lx0)
else:
    from oracle import ipm_ref as C, nlp_ref as R
    r = C.solve(R.UnicycleOCP(N=20), P, w0=w0, lam0=l0, lamx0=lx0, warm=(1e-4, 1e-4, 1e-4), restoration=0, nthreads=1, **o)
sys.stdout.flush()
print("RESULT", r["status"], r["iters"], flush=True)
