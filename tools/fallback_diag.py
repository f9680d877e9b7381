"""Counts the Riccati-scan fallbacks (diagnostic build, make -C mpc-verde_amd stamps) on the problem of
tests/test_gpu_linear.py::test_scan_fallback_on_indefinite_stage_weights, showing that the test
exercises the sequential fallback (measured: 4-5 of the 6-8 iterations of every instance).
"""
import ctypes, os, sys
import numpy as np
ROOT =os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
os.environ["MPCX_LIB"] = os.path.join(ROOT, "mpc-verde_amd", "mpcx", "libmpcx_stamps.so")
sys.path.insert(0, os.path.join(ROOT, "mpc-verde_amd"))
import torch
import mpcx
from mpcx import lti
lib = mpcx._lib.load()
lib.mpcx_diag_set_counter_buffer.argtypes = [ctypes.c_void_p]
rng = np.random.default_rng(11)
nx, nu, N, B = 4, 1, 20, 32
A = np.eye(nx) + 0.05 * rng.normal(size=(nx, nx)); Bm = rng.normal(size=(nx, nu)) + 1.0
W = np.zeros((2, nx + nu, nx + nu)); W[:, :nx, :nx] = 5.0 * np.eye(nx); W[0, nx, nx] = -0.05; W[1, nx, nx] = 0.5
tab = np.zeros(N, np.int32); tab[-1] = 1
lin = lti.LinearOCP(N=N, A=np.stack([A, A]), B=np.stack([Bm, Bm]), c=np.zeros((2, nx)), W=W, tab=tab, u_lb=(-1.0,), u_ub=(1.0,))
buf = torch.zeros(B * 15, dtype=torch.int32, device="cuda")
assert lib.mpcx_diag_set_counter_buffer(ctypes.c_void_p(buf.data_ptr())) == 0
S = mpcx.nlpsol("fb", "mi355x", lin, {"ipopt": {"max_iter": 300}})
x0 = rng.normal(size=(B, nx))
r = S.solve_batch(lin.params(x0, np.zeros((B, N, nx + nu))))
torch.cuda.synchronize()
c = buf.cpu().numpy().reshape(B, 15)
print("iters", r["iters"].tolist())
print("scan_fallbacks per instance", c[:, 8].tolist())
