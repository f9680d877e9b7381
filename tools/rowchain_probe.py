#!/usr/bin/env python3
"""Cycles per step of the row chain's parts, from harness builds with MPCX_ROWCHAIN_PROBE switches
(tests/hip/rowchain_check.hip built with -DMPCX_ROWCHAIN_PROBE=v into /tmp or tools/; results of the
switched builds are not the recursion's, only their timing is read).

    python tools/rowchain_probe.py LIB...     (on the GPU box)
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_gpu_rowchain import K_OUT, stages  # noqa: E402

for lib_path in sys.argv[1:]:
    lib = ctypes.CDLL(lib_path)
    lib.rowchain_check.argtypes = [ctypes.c_int] * 4 + [ctypes.c_void_p] * 4
    for G, R, N in ((32, 2, 20), (32, 1, 20)):
        B = 1024
        rng = np.random.default_rng(0)
        x = stages(rng, B, G, np.ones((B, G)))
        d_in = torch.from_numpy(np.ascontiguousarray(x)).cuda()
        o1 = torch.zeros((B, G, K_OUT), dtype=torch.float64, device="cuda")
        o2 = torch.zeros_like(o1)
        waves = (B * G * R + 63) // 64
        cyc = torch.zeros(2 * waves, dtype=torch.int64, device="cuda")
        p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        for _ in range(3):
            assert lib.rowchain_check(G, R, N, B, p(d_in), p(o1), p(o2), p(cyc)) == 0
        c = cyc.cpu().numpy().reshape(waves, 2)
        print(f"{os.path.basename(lib_path)} G={G} R={R} N={N}: cycles/step sequential {c[:, 0].mean() / N:.0f}, "
              f"row chain {c[:, 1].mean() / N:.0f}")
