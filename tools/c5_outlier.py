#!/usr/bin/env python3
"""Config-5 multi-step outliers (diagnostic build): after W warm-up step() launches, one K-step
launch with the stamp and event-counter buffers set; prints the slowest waves' instances with their
per-step iterations, cycles per iteration, Riccati share and IPM event counters.

    MPCX_STAMPS_LIB=mpc-verde_amd/mpcx/libmpcx_stamps.so python tools/c5_outlier.py [K]
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["MPCX_LIB"] = os.environ.get("MPCX_STAMPS_LIB") or os.path.join(ROOT, "mpc-verde_amd", "mpcx",
                                                                           "libmpcx_stamps.so")
sys.path.insert(0, os.path.join(ROOT, "mpc-verde_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import mpcx  # noqa: E402
from mpcx import dist as mdist  # noqa: E402
from mpcx.device import DeviceLoop  # noqa: E402

NAMES = ["regularised_iters", "extra_factorisations", "backtracks", "barrier_updates", "ftb_limited_steps",
         "tiny_steps", "filter_rejections", "armijo_acceptances", "scan_fallbacks", "filter_resets", "soc_eligible",
         "soc_accepted", "soft_resto_steps", "resto_phases", "filter_overflows"]
SLOTS, ND = 16, len(NAMES)


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    B, N, G = 2048, 100, 128
    lib = mpcx._lib.load()
    lib.mpcx_diag_set_stamp_buffer.argtypes = [ctypes.c_void_p]
    lib.mpcx_diag_set_counter_buffer.argtypes = [ctypes.c_void_p]
    lin = mpcx.inverted_pendulum_qp(N=N)
    solver = mpcx.nlpsol("c5", "mi355x", lin)
    loop = DeviceLoop(solver, mpcx.lti.pendulum_params(lin, mdist.config5_inputs(0, B), 0.0))
    for _ in range(3):
        loop.step()
    torch.cuda.synchronize()
    waves = B * G // 64
    st = torch.zeros(waves * SLOTS, dtype=torch.int64, device="cuda")
    cn = torch.zeros(B * ND, dtype=torch.int32, device="cuda")
    assert lib.mpcx_diag_set_stamp_buffer(ctypes.c_void_p(st.data_ptr())) == 0
    assert lib.mpcx_diag_set_counter_buffer(ctypes.c_void_p(cn.data_ptr())) == 0
    _, it = loop.run(K)
    torch.cuda.synchronize()
    acc = st.view(waves, SLOTS).cpu().numpy().astype(float)
    its = it.cpu().numpy()  # (K, B)
    cnt = cn.cpu().numpy().reshape(B, ND)
    tot = acc.sum(axis=1)
    inst_cycles = tot.reshape(B, G // 64).max(axis=1)
    order = np.argsort(-inst_cycles)
    out = {"median_cycles": float(np.median(inst_cycles)), "slowest": []}
    for b in order[:6]:
        w = int(np.argmax(acc[b * 2:b * 2 + 2].sum(axis=1))) + 2 * b
        out["slowest"].append({"instance": int(b), "cycles": float(inst_cycles[b]), "iters_per_step": its[:, b].tolist(),
                               "riccati_share": round(acc[w, 3] / tot[w], 3),
                               "counters": {n: int(v) for n, v in zip(NAMES, cnt[b]) if v}})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
