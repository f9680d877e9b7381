#!/usr/bin/env python3
"""Per-phase cycle shares of the fused solve kernel (diagnostic build, -DMPCX_STAMPS).

    make -C mpc-verde_amd stamps && python tools/stamp_profile.py [--steps S]

Runs the bench workload (config 2 closed loop) on libmpcx_stamps.so; after the
warm-up steps it records s_memtime deltas per solver phase for one solve and
prints each phase's share and cycles per IPM iteration (slowest wave basis).
Stamps perturb timing (they fence the scheduler); read shares, not totals.
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["MPCX_LIB"] = os.environ.get("MPCX_STAMPS_LIB") or os.path.join(ROOT, "mpc-verde_amd", "mpcx", "libmpcx_stamps.so")
sys.path.insert(0, os.path.join(ROOT, "mpc-verde_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import mpcx  # noqa: E402
from mpcx import dist  # noqa: E402
from mpcx.device import DeviceLoop  # noqa: E402

PHASES = ["errors", "barrier_update", "sigma", "riccati", "forward", "fraction", "linesearch", "update", "sweep",
          "exit",
          # sub-phases of a -DMPCX_STAMP_SUB build (0 otherwise): the Riccati phase's node-parallel
          # stage setup, reused-suffix scan, sequential chain and post-chain part; the errors
          # phase's group sums and its tests
          "ric_stage", "ric_scan", "ric_chain", "ric_post", "err_sums", "err_tests"]
SLOTS = 16  # kernels.h kStampSlots


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--N", type=int, default=20)
    ap.add_argument("--model", choices=("unicycle", "pend", "kin_bicycle", "dyn_bicycle", "cartpole"),
                    default="unicycle")
    ap.add_argument("--run", type=int, default=0,
                    help="stamp one K-step launch (DeviceLoop.run(K), the bench's timed path) instead of one solve; "
                         "cycles per iteration are then per iteration of the slowest wave's K solves")
    a = ap.parse_args()
    lib = mpcx._lib.load()
    lib.mpcx_diag_set_stamp_buffer.argtypes = [ctypes.c_void_p]
    if a.model == "pend":
        lin = mpcx.inverted_pendulum_qp(N=a.N)
        solver = mpcx.nlpsol("stamps", "mi355x", lin)
        loop = DeviceLoop(solver, mpcx.lti.pendulum_params(lin, dist.config5_inputs(0, a.batch), 0.0))
    elif a.model == "kin_bicycle":
        solver = mpcx.nlpsol("stamps", "mi355x", mpcx.kinematic_bicycle_tracking(N=a.N))
        loop = DeviceLoop(solver, dist.config3_bicycle_inputs(0, a.batch, N=a.N)[1])
    elif a.model == "dyn_bicycle":
        ocp = mpcx.dynamic_bicycle_lane_change(N=a.N)
        solver = mpcx.nlpsol("stamps", "mi355x", ocp)
        t0, x0, (X, Y, V) = dist.config4_bicycle_inputs(0, a.batch)
        refs = np.stack([mpcx.ode.dyn_bicycle_references(X, Y, V, int(t), a.N) for t in t0])
        loop = DeviceLoop(solver, ocp.params(x0, refs))
    elif a.model == "cartpole":
        solver = mpcx.nlpsol("stamps", "mi355x", mpcx.cartpole_swingup(N=a.N))
        loop = DeviceLoop(solver, dist.config5_swingup_inputs(0, a.batch))
    else:
        solver = mpcx.nlpsol("stamps", "mi355x", mpcx.unicycle_point_to_point(N=a.N))
        loop = DeviceLoop(solver, dist.config2_inputs(0, a.batch))
    for _ in range(a.steps):
        loop.step()
    G = 16 if a.N < 16 else 32 if a.N < 32 else 64 if a.N < 64 else 128 if a.N < 128 else 256
    n_simd = 4 * torch.cuda.get_device_properties(0).multi_processor_count
    while G < 64 and a.batch * G * 2 <= 64 * n_simd:  # launch_solve_model's widening rule
        G *= 2
    waves = (a.batch * G + 63) // 64
    buf = torch.zeros(waves * SLOTS, dtype=torch.int64, device="cuda")
    assert lib.mpcx_diag_set_stamp_buffer(ctypes.c_void_p(buf.data_ptr())) == 0
    if a.run > 0:
        _, it_k = loop.run(a.run)
        torch.cuda.synchronize()
        it_inst = it_k.cpu().numpy().sum(axis=0)
    else:
        loop.solve()
        torch.cuda.synchronize()
        it_inst = loop.iters.cpu().numpy()
    acc = buf.view(waves, SLOTS).cpu().numpy().astype(float)
    iters = np.array([it_inst[(w * 64) // G] if G >= 64 else it_inst[w * (64 // G):(w + 1) * (64 // G)].max()
                      for w in range(waves)])
    slow = int(np.argmax(acc.sum(axis=1)))
    tot = acc[slow].sum()
    out = {"iters_slowest_wave": int(iters[slow]), "cycles_slowest_wave": tot,
           "cycles_per_iter": tot / max(iters[slow], 1),
           "share": {p: round(acc[slow, i] / tot, 4) for i, p in enumerate(PHASES)},
           "share_all_waves": {p: round(acc[:, i].sum() / acc.sum(), 4) for i, p in enumerate(PHASES)}}
    if G > 64:  # multi-wave groups: each wave of the slowest wave's group, cycles per IPM iteration
        w0 = slow - slow % (G // 64)
        out["group_waves_cycles_per_iter"] = [
            {p: round(acc[w, i] / max(iters[slow], 1)) for i, p in enumerate(PHASES)} for w in range(w0, w0 + G // 64)]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
