#!/usr/bin/env python3
"""First IPM iteration at which the kernel and the C++ oracle part ways, per instance.

    python tools/divergence.py [model] [n_instances]      (GPU box; model: dyn_bicycle)

Solves the cold config-4 dynamic-bicycle batch with both, picks the instances whose iteration
counts differ, then re-solves each with max_iter = 1, 2, ... and reports the first m at which
the returned iterates differ by more than 1e-9 (relative to max(|w|_inf, 1)), together with
both sides' iterates at m - 1 and m.  Diagnostic only (not a test).
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpc-verde_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import mpcx  # noqa: E402
from mpcx import dist as mdist  # noqa: E402
from oracle import ipm_ref  # noqa: E402


def main():
    n_show = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    N, B = 50, 1024
    ocp = mpcx.dynamic_bicycle_lane_change(N=N)
    t0, x0, (X, Y, V) = mdist.config4_bicycle_inputs(0, B)
    refs = np.stack([mpcx.ode.dyn_bicycle_references(X, Y, V, int(t), N).reshape(-1) for t in t0])
    P = ocp.params(x0, refs)
    ipm_ref.lib()
    r = mpcx.nlpsol("d", "mi355x", ocp, {"ipopt": {"max_iter": 3000}}).solve_batch(P)
    ref = ipm_ref.solve(ocp, P, nthreads=0)
    bad = np.flatnonzero(r["iters"] != ref["iters"])
    out = {"n_differ": int(len(bad)), "cases": []}
    sel = bad[:n_show]
    Ps = P[sel]
    first = np.full(len(sel), -1)
    for m in range(1, int(min(r["iters"][sel].max(), ref["iters"][sel].max())) + 1):
        rk = mpcx.nlpsol("d", "mi355x", ocp, {"ipopt": {"max_iter": m}}).solve_batch(Ps)
        ro = ipm_ref.solve(ocp, Ps, nthreads=0, max_iter=m)
        e = np.max(np.abs(rk["w"] - ro["w"]), axis=1) / np.maximum(np.max(np.abs(ro["w"]), axis=1), 1.0)
        for j in range(len(sel)):
            if first[j] < 0 and e[j] > 1e-9:
                first[j] = m
                out["cases"].append({"inst": int(sel[j]), "iters_kernel": int(r["iters"][sel[j]]),
                                     "iters_oracle": int(ref["iters"][sel[j]]), "first_differing_max_iter": m,
                                     "rel_diff": float(e[j]), "status_kernel": int(rk["status"][j]),
                                     "status_oracle": int(ro["status"][j])})
        if np.all(first >= 0):
            break
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
