#!/usr/bin/env python3
"""Why the kinematic bicycle's slowest closed-loop solves take 50-650 IPM iterations.

    python tools/kin_tail.py [gpurun_out/ode_diag_kin_bicycle.npz]

Input: the slowest instances of a config-3 kinematic-bicycle closed loop with their warm starts
(tools/ode_diag.py kin_bicycle 4096 8 on the GPU box).  Each is re-solved on the C++ oracle
(oracle/ipm_ref.cpp, the IPOPT restatement the kernel matches iteration for iteration) with its
trace on, and the regularised iterations are related to the curvature of the stage Lagrangian:
for psi' = v tan(delta) / L the (v, delta) block of lam^T d2F/du2 has the off-diagonal
lam_psi T sec^2(delta) / L and no diagonal term, so the input block R + lam^T F_uu is indefinite
as soon as |lam_psi| T sec^2(delta) / L exceeds 2 sqrt(R_v R_delta) (scaled objective: the same
with fs) -- a saddle of the bilinear v * tan(delta).  Prints per instance: iterations, the
iterations IPOPT regularised (delta_w > 0), line-search backtracks, and at the solution the
largest |lam_psi| and the number of stages whose input block is indefinite.  Diagnostic only.
"""
import os
import re
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpc-verde_amd"))
sys.path.insert(0, ROOT)

CHILD = r"""
import sys, numpy as np
sys.path.insert(0, {root!r} + "/mpc-verde_amd"); sys.path.insert(0, {root!r})
import mpcx
from oracle import ipm_ref
d = np.load({npz!r})
b = {b}
ocp = mpcx.kinematic_bicycle_tracking(N=30)
r = ipm_ref.solve(ocp, d["P"][b:b + 1], w0=d["w0"][b:b + 1], lam0=d["lam0"][b:b + 1], lamx0=d["lamx0"][b:b + 1],
                  warm=(1e-4, 1e-4, 1e-4), nthreads=1, max_iter=3000)
np.savez("/tmp/kin_tail_%d.npz" % b, w=r["w"][0], lam=r["lam_g"][0], status=r["status"], iters=r["iters"])
"""


def main():
    npz = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "ode_diag_kin_bicycle.npz")
    d = np.load(npz)
    import mpcx
    from oracle.ode_ref import Problem

    ocp = mpcx.kinematic_bicycle_tracking(N=30)
    pb = Problem(ocp)
    nx, nu, N = 3, 2, ocp.N
    nz = nx + nu
    Rv, Rd = 2 * ocp.R[0], 2 * ocp.R[1]
    rows = []
    for b in range(d["P"].shape[0]):
        env = dict(os.environ, ORACLE_TRACE="1")
        out = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT, npz=npz, b=b)], env=env,
                             capture_output=True, text=True).stdout
        steps = re.findall(r"STEP it=(\d+) resto=\d alpha=(\S+) alpha_d=\S+ ftype=\d mu=\S+ delta=(\S+)", out)
        reg = sum(float(s[2]) > 0 for s in steps)
        back = sum(float(s[1]) < 1.0 for s in steps)
        r = np.load(f"/tmp/kin_tail_{b}.npz")
        w, lam = r["w"], r["lam"]
        X = np.stack([w[0:nx]] + [w[nx + nz * k + nu:nx + nz * (k + 1)] for k in range(N)])
        U = np.stack([w[nx + nz * k:nx + nz * k + nu] for k in range(N)])
        Lk = lam.reshape(N + 1, nx)[1:]  # multipliers of the defects F(X_k, U_k) - X_{k+1}
        z = np.concatenate([X[:N], U], axis=1)
        H = pb.hess_lam(z, Lk)
        Huu = H[:, nx:, nx:] + np.diag([Rv, Rd])
        indef = int(np.sum(np.linalg.eigvalsh(Huu)[:, 0] < 0))
        rows.append((int(d["inst"][b]), int(d["step"][b]), int(r["iters"][0]), reg, back,
                     float(np.max(np.abs(Lk[:, 2]))), float(np.min(np.abs(U[:, 0]))), indef))
        print(f"inst {rows[-1][0]:5d} step {rows[-1][1]}: {rows[-1][2]:4d} iterations, {reg:4d} regularised, "
              f"{back:4d} backtracked; at the solution max|lam_psi| {rows[-1][5]:.3g}, min|v| {rows[-1][6]:.3g}, "
              f"{indef}/{N} stages with an indefinite input block", flush=True)
    a = np.array([r[2:] for r in rows], float)
    print(f"{len(rows)} slowest solves: iterations {a[:, 0].mean():.0f} mean, regularised {a[:, 1].sum() / a[:, 0].sum():.0%} "
          f"of them, backtracked {a[:, 2].sum() / a[:, 0].sum():.0%}; solutions with an indefinite input block "
          f"{int(np.sum(a[:, 5] > 0))}/{len(rows)}")


if __name__ == "__main__":
    main()
