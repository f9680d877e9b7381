"""One process per GPU: instance sharding and closed-loop statistics collection.

MPC instances (initial state x reference) are independent for the whole closed
loop, so the data path has NO collective: rank r owns the
contiguous block of global instance ids [r*B, (r+1)*B) (weak scaling) and
builds its own inputs from (seed, global id).  The only communication is one
``all_gather`` of per-instance statistics after the loop -- RCCL over xGMI with
the ``nccl`` backend on ROCm, ``gloo`` on CPU (tests).
"""
from __future__ import annotations

import json
import os

import numpy as np

STAT_FIELDS = ("final_error", "iters_mean", "iters_max", "status_max", "f_last", "x", "y", "theta")


def env():
    """(rank, world_size, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def device_index(local_rank: int) -> int:
    """GPU of this rank: LOCAL_RANK, or MPCX_FORCE_DEVICE (test rehearsal of the multi-rank
    path with several ranks on one GPU; never set in production runs)."""
    forced = os.environ.get("MPCX_FORCE_DEVICE")
    return int(forced) if forced is not None else local_rank


def visible_gpu_count(topology="/sys/class/kfd/kfd/topology/nodes", environ=None):
    """GPUs this process may use, counted WITHOUT touching HIP (a launcher decides how many ranks
    to start before any GPU call): the KFD topology's GPU nodes (gpu_id != 0), capped by
    ROCR_/HIP_/CUDA_VISIBLE_DEVICES when set.  None when the topology cannot be read (each rank
    then checks its own device)."""
    environ = os.environ if environ is None else environ
    try:
        nodes = os.listdir(topology)
    except OSError:
        return None
    n = 0
    for d in nodes:
        try:
            with open(os.path.join(topology, d, "gpu_id")) as f:
                n += int(f.read().strip() or "0") != 0
        except (OSError, ValueError):
            pass
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip()]))
    return n


def backend(default: str = "nccl") -> str:
    """Process-group backend: RCCL ("nccl") unless MPCX_DIST_BACKEND overrides it (gloo for
    the one-GPU rehearsal above: RCCL needs a distinct GPU per rank)."""
    return os.environ.get("MPCX_DIST_BACKEND", default)


def _coll_device(device):
    import torch.distributed as dist

    return None if dist.get_backend() == "gloo" else device


def init(backend: str, always: bool = False):
    """Create the process group from the torch.distributed.run environment: for world_size > 1, or
    at world_size 1 too when `always` (then the stats collectives below run through the backend --
    RCCL with one rank -- instead of short-circuiting).  Call before any other HIP use of the
    process (RCCL binds the rank's device)."""
    import torch.distributed as dist

    rank, world, _ = env()
    if (world > 1 or always) and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend=backend, rank=rank, world_size=world)
    return rank, world


def shard(B_per_rank: int, rank: int):
    return rank * B_per_rank, (rank + 1) * B_per_rank


def _golden_P(path=None):
    if path is None:
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        path = os.path.join(root, "tests", "golden", "unicycle_N10_golden.json")
    if not os.path.exists(path):
        return np.zeros((0, 6))
    with open(path) as f:
        rows = np.array(json.load(f)["multiple_shooting"]["rows"], float)
    n = rows.shape[0] - 1
    P = np.zeros((n, 6))
    P[:, 0:3] = rows[1:, 0:3]
    P[:, 3:6] = (10.0, 10.0, 0.0)
    return P


def config2_inputs(start: int, stop: int, seed: int = 20261015, with_golden=True):
    """global instances 0..83 are the 84 recorded golden
    P_j (Casadi/1exemplo.xlsx); the rest x, y ~ U[-5, 5], th ~ U[-pi/2, pi/2],
    target (10, 10, 0).  Instance g's draw depends only on (seed, g)."""
    n = stop - start
    P = np.zeros((n, 6))
    P[:, 3:6] = (10.0, 10.0, 0.0)
    for i, g in enumerate(range(start, stop)):
        r = np.random.default_rng([seed, g]).uniform(size=3)
        P[i, 0:2] = -5.0 + 10.0 * r[0:2]
        P[i, 2] = -np.pi / 2 + np.pi * r[2]
    if with_golden:
        Pg = _golden_P()
        lo, hi = start, min(stop, Pg.shape[0])
        if hi > lo:
            P[0:hi - lo] = Pg[lo:hi]
    return P


def config3_inputs(start: int, stop: int, N: int = 30, seed: int = 20261016):
    """phase tau0 ~ U[0, 20 pi), x0 = ref(tau0) + N(0, 0.1^2 I).
    Returns (tau0 (n,), P (n, 3 + 5N)) with P = [x0; p_0..p_{N-1}] for step t = 0."""
    from .ocp import circular_reference

    n = stop - start
    tau0 = np.zeros(n)
    x0 = np.zeros((n, 3))
    for i, g in enumerate(range(start, stop)):
        rng = np.random.default_rng([seed, g])
        tau0[i] = rng.uniform(0.0, 20.0 * np.pi)
        x0[i] = circular_reference(tau0[i:i + 1], 0, 1)[0, 0, 0:3] + rng.normal(scale=0.1, size=3)
    P = np.concatenate([x0, circular_reference(tau0, 0, N).reshape(n, 5 * N)], axis=1)
    return tau0, P


def lane_change(path=None):
    """Trajectory Tracking/lane_change.csv (x, y, uref; 500 rows), shipped as tests/golden/lane_change.csv."""
    import csv

    if path is None:
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        path = os.path.join(root, "tests", "golden", "lane_change.csv")
    with open(path) as f:
        rows = [tuple(float(v) for v in r.values()) for r in csv.DictReader(f)]
    return tuple(np.array(c) for c in zip(*rows))


def config4_inputs(start: int, stop: int, N: int = 50, seed: int = 20261017):
    """SURVEY.md §8(d) config 4 (LTV lateral model, lane_change.csv): start offset
    t0 ~ U{0..449}; x0 = (y_ref, phi_ref, v_ref, r_ref)(t0) + N(0, diag(.1, .02, .1, .02)^2).
    Returns (t0 (n,) int, x0 (n, 4), par (500, N, 5) per-time stage references)."""
    from .lti import lateral_references

    xr, yr, vr = lane_change()
    par = lateral_references(xr, yr, vr, Delta=0.05, horizon=N)
    n = stop - start
    t0 = np.zeros(n, np.int64)
    x0 = np.zeros((n, 4))
    for i, g in enumerate(range(start, stop)):
        rng = np.random.default_rng([seed, g])
        t0[i] = rng.integers(0, 450)
        x0[i] = par[t0[i], 0, 0:4] + rng.normal(scale=[0.1, 0.02, 0.1, 0.02])
    return t0, x0, par


def config5_inputs(start: int, stop: int, seed: int = 20261018):
    """SURVEY.md §8(d) config 5 (cart-pole QP): x0 ~ U([-1,1]x[-.5,.5]x[-.2,.2]x[-.5,.5]), u_prev = 0."""
    n = stop - start
    x0 = np.zeros((n, 4))
    for i, g in enumerate(range(start, stop)):
        x0[i] = np.random.default_rng([seed, g]).uniform([-1, -.5, -.2, -.5], [1, .5, .2, .5])
    return x0


def config3_bicycle_inputs(start: int, stop: int, N: int = 30, seed: int = 20261016, L: float = 0.5):
    """Config 3 variant (kinematic bicycle on the config-3 circle): tau0 ~ U[0, 20 pi),
    x0 = ref(tau0) + N(0, 0.1^2 I).  Returns (tau0 (n,), P (n, 3 + 5N))."""
    from .ode import bicycle_circular_reference

    n = stop - start
    tau0 = np.zeros(n)
    x0 = np.zeros((n, 3))
    for i, g in enumerate(range(start, stop)):
        rng = np.random.default_rng([seed, g])
        tau0[i] = rng.uniform(0.0, 20.0 * np.pi)
        x0[i] = bicycle_circular_reference(tau0[i:i + 1], 0, 1, L=L)[0, 0, 0:3] + rng.normal(scale=0.1, size=3)
    P = np.concatenate([x0, bicycle_circular_reference(tau0, 0, N, L=L).reshape(n, 5 * N)], axis=1)
    return tau0, P


def config4_bicycle_inputs(start: int, stop: int, seed: int = 20261017):
    """Config 4 variant (6-state dynamic bicycle on the scaled lane change, mpcx/ode.py): start
    offset t0 ~ U{0..449}, x0 = ref(t0) + N(0, diag(.2, .2, .05, .3, .1, .05)^2).
    Returns (t0 (n,) int, x0 (n, 6), (X, Y, V) path rows)."""
    from .ode import dyn_bicycle_references, lane_change_rows

    X, Y, V = lane_change_rows(*lane_change())
    n = stop - start
    t0 = np.zeros(n, np.int64)
    x0 = np.zeros((n, 6))
    for i, g in enumerate(range(start, stop)):
        rng = np.random.default_rng([seed, g])
        t0[i] = rng.integers(0, 450)
        x0[i] = dyn_bicycle_references(X, Y, V, int(t0[i]), 1)[0, 0:6] + \
            rng.normal(scale=[0.2, 0.2, 0.05, 0.3, 0.1, 0.05])
    return t0, x0, (X, Y, V)


def config5_swingup_inputs(start: int, stop: int, seed: int = 20261018):
    """Config 5 variant (cart-pole swing-up): x0 = (U[-1,1], U[-.5,.5], pi + U[-.2,.2], U[-.5,.5]),
    set point 0.  Returns P (n, 8) = [x0; x_ref]."""
    n = stop - start
    P = np.zeros((n, 8))
    for i, g in enumerate(range(start, stop)):
        P[i, 0:4] = np.random.default_rng([seed, g]).uniform([-1, -.5, -.2, -.5], [1, .5, .2, .5])
        P[i, 2] += np.pi
    return P


def stats_matrix(P, w, f, status, iters_hist):
    """Per-instance closed-loop statistics, (B, len(STAT_FIELDS)) float64."""
    B = P.shape[0]
    it = np.asarray(iters_hist, float).reshape(-1, B) if len(iters_hist) else np.zeros((1, B))
    S = np.zeros((B, len(STAT_FIELDS)))
    S[:, 0] = np.linalg.norm(P[:, 0:3] - P[:, 3:6], axis=1)
    S[:, 1] = it.mean(axis=0)
    S[:, 2] = it.max(axis=0)
    S[:, 3] = np.asarray(status, float)
    S[:, 4] = np.asarray(f, float)
    S[:, 5:8] = P[:, 0:3]
    return S


def all_gather_stats(S_local, device=None):
    """Gather every rank's (B, F) statistics block on every rank (RCCL/gloo)."""
    import torch
    import torch.distributed as dist

    if not dist.is_initialized():
        return np.asarray(S_local)
    t = torch.as_tensor(np.ascontiguousarray(S_local), dtype=torch.float64)
    device = _coll_device(device)
    if device is not None:
        t = t.to(device)
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return torch.cat(out).cpu().numpy()


def max_over_ranks(x: float, device=None):
    import torch
    import torch.distributed as dist

    if not dist.is_initialized():
        return float(x)
    t = torch.tensor([x], dtype=torch.float64, device=_coll_device(device))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
