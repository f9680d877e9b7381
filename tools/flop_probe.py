"""Per-unit FP64 work of the solve kernel's per-node building blocks, for the algorithmic roofline
(bench.py ALGO_UNIT_FLOPS): one stage evaluation (Model::derivs: F, q, A, B, grad q
and the exact Hessian of fs q + lam^T F, as the solve kernel calls it) and one backward Riccati
step (riccati_step + riccati_gains with the model's masks), per model, each on one thread per
unit through the device harness tests/hip/flop_probe.hip.  Run under

    rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 \\
        -d gpurun_out/flops -o flops --output-format csv -- python3 tools/flop_probe.py

then tools/flop_summary.py turns the counts into flops per unit (FMA = 2, n a multiple of 64
so every lane of every wave holds a unit; the launch order below is the summary's key order).
"""
import ctypes
import os

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N_UNITS = 64 * 2048
# (key, model id, nx, nu, T, M, cost, Q, R, par): the benchmarked configurations' stage constants
EVALS = [
    ("unicycle_quadrature_M4", 1, 3, 2, 0.2, 4, 0, (1.0, 5.0, 0.1), (0.5, 0.05), ()),  # config 2
    ("unicycle_node_M1", 1, 3, 2, 0.2, 1, 1, (1.0, 1.0, 0.1), (0.5, 0.05), ()),        # config 3
    ("kin_bicycle_M1", 3, 3, 2, 0.2, 1, 1, (1.0, 1.0, 0.1), (0.5, 0.05), (0.5,)),
    ("dyn_bicycle_M4", 4, 6, 2, 0.05, 4, 1, (1.0,) * 6, (1.0, 1.0), (1200.0, 1.5, 2.0, 55000.0, 1350.0)),
    ("cartpole_M1", 5, 4, 1, 0.01, 1, 1, (1.44, 0.0, 1.0, 0.0), (1e-4,), (1.0, 1.0, 0.5, 9.81, 10.0)),
]
RICCATI = [("unicycle", 1, 3, 2), ("kin_bicycle", 3, 3, 2), ("dyn_bicycle", 4, 6, 2), ("cartpole", 5, 4, 1),
           ("linear4x1", 41, 4, 1), ("linear5x1", 51, 5, 1)]


def arr8(v):
    return (ctypes.c_double * 8)(*(list(v) + [0.0] * (8 - len(v))))


def main():
    lib = ctypes.CDLL(os.path.join(ROOT, "tests", "hip", "libflop_probe.so"))
    vp = ctypes.c_void_p
    lib.eval_probe.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_int, ctypes.c_int, vp, vp, vp,
                               vp, vp, vp, ctypes.c_int, vp]
    lib.riccati_probe.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp]
    rng = np.random.default_rng(1)
    n = N_UNITS
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float64)).cuda()  # noqa: E731
    p = lambda t: vp(t.data_ptr())  # noqa: E731
    for key, model, nx, nu, T, M, cost, Q, R, par in EVALS:
        nz = nx + nu
        Z = rng.uniform(-1.0, 1.0, size=(n, nz))
        if model == 4:  # dynamic bicycle: forward speed 4..8 m/s (the model divides by vx)
            Z[:, 3] = rng.uniform(4.0, 8.0, n)
        P = np.concatenate([Z[:, :nx], rng.uniform(-1.0, 1.0, size=(n, nx))], axis=1)
        if model == 4:
            P[:, nx + 3] = 6.0
        L = rng.normal(size=(n, nx))
        no = nx + 1 + nx * nx + nx * nu + nz + nz * (nz + 1) // 2
        d_z, d_l, d_p = dev(Z), dev(L), dev(P)
        out = torch.zeros(n * no, dtype=torch.float64, device="cuda")
        rc = lib.eval_probe(model, n, T, M, cost, arr8(Q), arr8(R), arr8(par), p(d_z), p(d_l), p(d_p), 2 * nx, p(out))
        assert rc == 0, (key, rc)
        assert torch.isfinite(out).all(), key
        print(f"eval {key}: {n} units")
    for key, model, nx, nu in RICCATI:
        nz, nh, npk = nx + nu, (nx + nu) * (nx + nu + 1) // 2, nx * (nx + 1) // 2
        Hd = rng.normal(size=(n, nz, nz))
        Hd = np.einsum("bij,bkj->bik", Hd, Hd) + np.eye(nz)
        Pk = rng.normal(size=(n, nx, nx))
        Pk = np.einsum("bij,bkj->bik", Pk, Pk) + np.eye(nx)
        iu = [(i, j) for i in range(nz) for j in range(i, nz)]
        ix = [(i, j) for i in range(nx) for j in range(i, nx)]
        inp = np.concatenate([np.stack([Hd[:, i, j] for i, j in iu], 1), rng.normal(size=(n, nz)),
                              rng.normal(size=(n, nx * nx)) * 0.3 + np.eye(nx).reshape(1, -1),
                              rng.normal(size=(n, nx * nu)) * 0.2, rng.normal(size=(n, nx)) * 0.1,
                              np.stack([Pk[:, i, j] for i, j in ix], 1), rng.normal(size=(n, nx))], axis=1)
        assert inp.shape[1] == nh + nz + nx * nx + nx * nu + nx + npk + nx
        d_in = dev(inp)
        out = torch.zeros(n * (npk + nx + nu * nx + nu), dtype=torch.float64, device="cuda")
        assert lib.riccati_probe(model, n, p(d_in), p(out)) == 0, key
        print(f"riccati {key}: {n} units")
    torch.cuda.synchronize()
    print(f"units per launch: {n}")


if __name__ == "__main__":
    main()
