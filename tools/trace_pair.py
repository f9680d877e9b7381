#!/usr/bin/env python3
"""Per-iteration step traces of one config-4 dynamic-bicycle instance, kernel or oracle.

    MPCX_LIB=mpc-verde_amd/mpcx/libmpcx_debug.so MPCX_ALLOW_STALE_LIB=1 python tools/trace_pair.py kernel 16 > k.txt
    ORACLE_TRACE=1 python tools/trace_pair.py oracle 16 > o.txt

Both print "STEP it=... alpha=... ftype=... mu=... thk=... phk=..." per accepted step (the
kernel's debug build for instance 0 of the batch, oracle/ipm_ref.cpp's TRACE); diff the two to
find the first decision that differs.  Diagnostic only.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpc-verde_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import mpcx  # noqa: E402
from mpcx import dist as mdist  # noqa: E402


def main():
    who, b = sys.argv[1], int(sys.argv[2])
    max_iter = int(sys.argv[3]) if len(sys.argv) > 3 else 3000
    N = 50
    ocp = mpcx.dynamic_bicycle_lane_change(N=N)
    t0, x0, (X, Y, V) = mdist.config4_bicycle_inputs(0, 1024)
    P = ocp.params(x0[b:b + 1], mpcx.ode.dyn_bicycle_references(X, Y, V, int(t0[b]), N).reshape(1, -1))
    if who == "kernel":
        r = mpcx.nlpsol("d", "mi355x", ocp, {"ipopt": {"max_iter": max_iter}}).solve_batch(P)
    else:
        from oracle import ipm_ref
        r = ipm_ref.solve(ocp, P, nthreads=1, max_iter=max_iter)
    sys.stdout.flush()
    print(f"RESULT status={int(r['status'][0])} iters={int(r['iters'][0])}", flush=True)


if __name__ == "__main__":
    main()
