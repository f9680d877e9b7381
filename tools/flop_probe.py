"""Per-unit FP64 work of the config-2 solve's two dominant pieces, for the algorithmic roofline
(DESIGN.md §6): the interval evaluation the kernel runs (unicycle.h uni_derivs_moments: F, q,
A, B, grad q and the exact Hessian of fs q + lam^T F; M = 4, quadrature cost) and one backward
Riccati step (riccati.h riccati_step + riccati_gains with the unicycle's masks), each on one
thread per unit through the device harness tests/hip/stage_check.hip.  Run under

    rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 \\
        -d gpurun_out/flops -o flops --output-format csv -- python3 tools/flop_probe.py

then tools/flop_summary.py turns the counts into flops per unit (FMA = 2, n multiple of 64 so
every lane of every wave holds a unit).
"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N_UNITS = 64 * 4096

lib = ctypes.CDLL(os.path.join(ROOT, "tests", "hip", "libstage_check.so"))
vp = ctypes.c_void_p
lib.stage_check_which.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_int, ctypes.c_int,
                                  ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double), vp, vp, vp, vp, vp,
                                  ctypes.c_double, vp, ctypes.c_int]
lib.riccati_check.argtypes = [ctypes.c_int, vp, vp]
rng = np.random.default_rng(1)
n = N_UNITS
dev = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float64)).cuda()  # noqa: E731
X = dev(np.column_stack([rng.uniform(-5, 5, n), rng.uniform(-5, 5, n), rng.uniform(-3, 3, n)]))
U = dev(np.column_stack([rng.uniform(-1, 1, n), rng.uniform(-0.7, 0.7, n)]))
XR = dev(np.tile([10.0, 10.0, 0.0], (n, 1)))
UR = dev(np.zeros((n, 2)))
L = dev(rng.normal(size=(n, 3)))
out = torch.zeros(2 * n * 39, dtype=torch.float64, device="cuda")
Q = (ctypes.c_double * 3)(1.0, 5.0, 0.1)
R = (ctypes.c_double * 2)(0.5, 0.05)
p = lambda t: vp(t.data_ptr())  # noqa: E731
# 1: the moment evaluation (the kernel's), config 2's T = 0.2, M = 4
assert lib.stage_check_which(n, 0.2, 4, 0, Q, R, p(X), p(U), p(XR), p(UR), p(L), 1.0, p(out), 1) == 0
# Riccati step inputs (47 doubles per unit): PD stage Hessians and value functions
Hd = rng.normal(size=(n, 5, 5))
Hd = np.einsum("bij,bkj->bik", Hd, Hd) + np.eye(5)
Pk = rng.normal(size=(n, 3, 3))
Pk = np.einsum("bij,bkj->bik", Pk, Pk) + np.eye(3)
iu = [(i, j) for i in range(5) for j in range(i, 5)]
i3 = [(i, j) for i in range(3) for j in range(i, 3)]
inp = np.concatenate([np.stack([Hd[:, i, j] for i, j in iu], 1), rng.normal(size=(n, 5)), rng.normal(size=(n, 9)),
                      rng.normal(size=(n, 6)) * 0.2, rng.normal(size=(n, 3)) * 0.1,
                      np.stack([Pk[:, i, j] for i, j in i3], 1), rng.normal(size=(n, 3))], axis=1)
d_in = dev(inp)
d_out = torch.zeros(n * 18, dtype=torch.float64, device="cuda")
assert lib.riccati_check(n, p(d_in), p(d_out)) == 0
torch.cuda.synchronize()
print(f"units per launch: {n}")
