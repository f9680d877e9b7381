#!/usr/bin/env python3
"""Benchmark: batched receding-horizon MPC solves on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]     (N > 1: starts its N ranks itself)
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload: the closed loop of
Casadi/multiple_shooting_casadi.py:224-298 for B = 1024 independent instances per
GPU (unicycle, multiple shooting, N = 20, RK4 M = 4, quadrature cost), inputs
from the config-2 generator (global instances 0..83 = the golden P_j).  One
step = one batched NLP solve of all B instances to IPOPT tolerance (1e-8,
warm-started from the previous step's shifted solution; the first warmup step
is cold) + the plant/shift update, all on the device.  Weak scaling: every rank
owns B instances; no collective inside the timed region.

Printed JSON (rank 0): value = total solves/s over all ranks; ms_per_step = the
max-over-ranks wall time per step; ms_per_solve_p50 = median batched solve-call
latency (HIP events).  `roofline` describes the kernel that dominates the timed
region, the fused solve_kernel: algorithmic FP64 flops per launch (the flops one
IPM iteration of one instance needs -- per-node evaluation and Riccati step
measured by tools/flop_probe.py, profiles/r04_flop_probe.json, plus the IPM's
vector work counted in ipm_vector_flops; DESIGN.md §6 -- x the launch's
instance-iterations) / the launch's HIP-event time / the FP64 vector peak, with
the issued FP64 lane-flops of profiles/r04_solve_kernel_pmc.json beside it while
that record matches the library's source hash.  `roofline_sweep` describes the
RK4 + Jacobian sweep kernel (rk4_sens, the HBM-streaming kernel of SURVEY.md
§8(d)) at B = 2^19, N = 20.  `cpu_baseline` times the C++ CPU oracle
(oracle/ipm_ref.cpp, kind "port") on every CPU the process may use, on a
bounded sample of the same workload, next to a 1-thread figure.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mpc-verde_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

METRIC = "MPC solves/sec (batched) + ms/solve p50, unicycle N=20 at 1/2/4/8 MI355X"
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
# FP64 vector (VALU) peak: AMD's MI355X spec, half the FP32 vector peak of 157.3 TF/s
# (MI355X_MICROARCH.md); the solve kernel issues scalar-per-lane FP64 FMAs, no MFMA
PEAK_FP64_TFLOPS = 78.6
SOLVE_PMC = os.path.join("profiles", "r06_solve_kernel_pmc.json")
SOLVE_TRAFFIC = "r06_solve_traffic.json"  # HBM bytes of the timed launch (tools/solve_traffic.py)
SWEEP_BYTES_PER_STAGE = 256  # read x_k,u_k,x_{k+1} (64 B) + write c,q,A,B,grad q (192 B)
SWEEP_BYTES_PER_INSTANCE = 48  # P


DATA = {
    2: "synthetic: SURVEY config-2 generator (global instances 0-83 = golden P_j of Casadi/1exemplo.xlsx)",
    3: "synthetic: SURVEY config-3 generator (phase ~ U[0,20pi), x0 = ref + N(0,0.1^2))",
    4: "lane_change.csv reference (Trajectory Tracking/), start offsets ~ U{0..449}, x0 = ref + noise",
    5: "synthetic: x0 ~ U([-1,1]x[-.5,.5]x[-.2,.2]x[-.5,.5]), u_prev = 0",
}
DYN = {2: "unicycle", 3: "unicycle", 4: "linear LTV lateral (nx=4, nu=1)", 5: "linear LTI cart-pole (nx=5, nu=1)"}
# BASELINE-named nonlinear variants (--model; mpcx/ode.py, parity unpinned: CPU oracle only)
VARIANTS = {3: "kin_bicycle", 4: "dyn_bicycle", 5: "cartpole"}
DATA_V = {
    "kin_bicycle": "synthetic: config-3 circle (phase ~ U[0,20pi), x0 = ref + N(0,0.1^2)), bicycle inputs v=0.1, "
                   "delta=atan(L)",
    "dyn_bicycle": "lane_change.csv path with x and speed x10 (4-8 m/s), start offsets ~ U{0..449}, x0 = ref + noise",
    "cartpole": "synthetic: hanging start x0 = (U[-1,1], U[-.5,.5], pi+U[-.2,.2], U[-.5,.5]), set point 0",
}
DYN_V = {"kin_bicycle": "nonlinear kinematic bicycle (nx=3, nu=2), exact 2nd-order forward-mode derivatives",
         "dyn_bicycle": "nonlinear 6-state dynamic bicycle, linear tyres (nx=6, nu=2), exact derivatives",
         "cartpole": "nonlinear cart-pole (nx=4, nu=1), exact derivatives"}


def workload_name_v(variant, N, M):
    return {
        "kin_bicycle": f"config 3 variant: closed-loop circular tracking, kinematic bicycle, multiple shooting N={N}, "
                       f"RK4 M={M} node cost, tol 1e-8",
        "dyn_bicycle": f"config 4 variant: closed-loop lane change, 6-state dynamic bicycle, multiple shooting N={N}, "
                       f"RK4 M={M} node cost, vx >= 2.5, tol 1e-8",
        "cartpole": f"config 5 variant: closed-loop cart-pole swing-up, multiple shooting N={N}, RK4 M={M} node cost, "
                    f"|F| <= 200, tol 1e-8",
    }[variant]


def workload_name(cfg, N):
    return {
        2: f"config 2: closed-loop point-to-point MPC, unicycle, multiple shooting N={N}, RK4 M=4 quadrature cost, "
           "IPOPT tol 1e-8",
        3: f"config 3: closed-loop circular trajectory tracking (Trajectory_tracking.py), unicycle, multiple "
           f"shooting N={N}, RK4 M=1 node cost, state bounds, tol 1e-8",
        4: f"config 4: closed-loop LTV lateral lane-change tracking (Trajectory_tracking_dynamic_model.py), "
           f"ZOH c2d per step at vref[t], N={N}, |delta|<=20, tol 1e-8",
        5: f"config 5: closed-loop cart-pole set-point QP (inverted_pendulum_single_shooting_mpctools.py), "
           f"ZOH c2d T=0.01, move blocking 5 free moves, N={N}, |u|<=200, tol 1e-8",
    }[cfg]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--group-policy", type=int, default=0, choices=(0, 1),
                    help="mpcx_spec.group_policy: 0 widens lane groups to fill the SIMDs, 1 keeps the smallest")
    ap.add_argument("--config", type=int, default=2, choices=(2, 3, 4, 5),
                    help="2: point-to-point N=20 B=1024 (headline); 3: circular tracking N=30 B=4096; "
                         "4: LTV lateral lane change N=50 B=1024/GPU; 5: cart-pole QP N=100 B=2048/GPU")
    ap.add_argument("--model", choices=("default",) + tuple(VARIANTS.values()), default="default",
                    help="BASELINE-named nonlinear variant of configs 3/4/5: kin_bicycle (3), dyn_bicycle (4), "
                         "cartpole swing-up (5)")
    ap.add_argument("--batch", type=int, default=None, help="instances per GPU (default per config)")
    ap.add_argument("--N", type=int, default=None)
    ap.add_argument("--seed", type=int, default=20261015)
    ap.add_argument("--mode", choices=("async", "lockstep"), default="async",
                    help="async: the K timed steps run as ONE multi-step launch (instances independent); "
                         "lockstep: one launch per step")
    ap.add_argument("--roofline-batch", type=int, default=1 << 19)
    ap.add_argument("--roofline-reps", type=int, default=20)
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--dump-stats", default=None,
                    help="rank 0 saves the all-gathered per-instance statistics (global instance order) to this .npy")
    ap.add_argument("--no-reference-warm-start", action="store_true",
                    help="skip the second timing under the reference's warm start (shifted primal only)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="minimum timed CPU-baseline solve time")
    ap.add_argument("--profile-sweep-only", action="store_true", help="only launch the sweep (for rocprofv3 --pmc)")
    ap.add_argument("--profile-solve-only", action="store_true",
                    help="only the warm-up steps and the timed K-step launch, then exit (for rocprofv3 --pmc: "
                         "tools/solve_traffic.py takes that launch's HBM bytes)")
    return ap.parse_args()


def shift_np(w, N):
    """Host copy of shift_kernel's warm start: X_k <- X_{k+1}, U_k <- U_{k+1}, last repeated."""
    w0 = np.empty_like(w)
    ix = lambda k: slice(0, 3) if k == 0 else slice(5 + 5 * (k - 1), 8 + 5 * (k - 1))  # noqa: E731
    for k in range(N + 1):
        w0[:, ix(k)] = w[:, ix(min(k + 1, N))]
        if k < N:
            su = min(k + 1, N - 1)
            w0[:, 3 + 5 * k:5 + 5 * k] = w[:, 3 + 5 * su:5 + 5 * su]
    return w0


def shift_lam_np(lam, N):
    """Multipliers of g_k shifted like the states (the shift kernel's lam_g shift)."""
    out = lam.copy()
    out[:, :3 * N] = lam[:, 3:3 * (N + 1)]
    return out


def shift_lamx_np(lamx, N):
    out = shift_np(lamx, N)
    out[:, 0:3] = 0.0  # X_0 is free
    return out


REF_IPOPT = {"max_iter": 2000, "acceptable_tol": 1e-8, "acceptable_obj_change_tol": 1e-6}  # :188-196
# warm-start policies of the closed loop (the solve after a shift):
#   "dual": shifted primal AND multipliers, IPOPT warm_start_init_point (mu0 = bound push =
#           multiplier push = 1e-4, mpcx_spec.warm_*) -- a solver option the reference does not set;
#   "reference": the reference's own -- the shifted primal guess only, IPOPT's default start
#           (mu0 = 0.1, multipliers 0 / 1): Casadi/multiple_shooting_casadi.py:233-242,274-287
#           (args['x0'] = w0, no lam_x0 / lam_g0), in the interleaved layout
POLICY = {"dual": "warm start: shifted primal + shifted multipliers, IPOPT warm_start_init_point (mu0 1e-4)",
          "reference": "warm start as the reference: shifted primal only, IPOPT default initialisation "
                       "(mu0 0.1; multiple_shooting_casadi.py:233-242,274-287)"}


def cpu_baseline(make_P, N, steps, cores, min_seconds=10.0, max_reps=64, warm=(1e-4, 1e-4, 1e-4)):
    """C++ oracle (port of the same NLP + IPOPT-style IPM, the reference's IPOPT options) on host
    cores: closed loops of `steps` steps with the GPU loop's warm-start policy (first step cold,
    then the shifted primal plus -- warm given -- the shifted multipliers as IPOPT's
    warm_start_init_point; warm=None: the shifted primal only, the reference's policy), solve
    calls timed.  Repeated on fresh instance blocks (make_P(rep) -> (B, 6)) until >= min_seconds
    of solve time (a bounded sample).  Returns (solves/s, seconds, reps, mean iterations)."""
    from oracle import ipm_ref, nlp_ref

    ipm_ref.build()
    ocp = nlp_ref.UnicycleOCP(N=N)
    t_solve = 0.0
    n = 0
    reps = 0
    its = 0
    while reps < max_reps and (reps == 0 or t_solve < min_seconds):
        P = make_P(reps).copy()
        B = P.shape[0]
        w0 = _cold(P, N, nlp_ref)
        lam0 = lamx0 = None
        for s in range(steps):
            t0 = time.perf_counter()
            if s == 0 or warm is None:
                r = ipm_ref.solve(ocp, P, w0=w0, nthreads=cores, **REF_IPOPT)
            else:
                r = ipm_ref.solve(ocp, P, w0=w0, lam0=lam0, lamx0=lamx0, warm=warm, nthreads=cores, **REF_IPOPT)
            t_solve += time.perf_counter() - t0
            n += B
            its += int(r["iters"].sum())
            xf, _ = nlp_ref.F(P[:, 0:3], r["w"][:, 3:5], P[:, 3:6], ocp)
            P[:, 0:3] = xf
            w0 = shift_np(r["w"], N)
            lam0 = shift_lam_np(r["lam_g"], N)
            lamx0 = shift_lamx_np(r["lam_x"], N)
        reps += 1
    return n / t_solve, t_solve, reps, its / max(n, 1)


def _pseq(refs, n_p, nx):
    """(K, B, n_p) full parameter rows from (K, B, n_p - nx) stage references (x0 unused)."""
    import torch

    K, B = refs.shape[0], refs.shape[1]
    out = torch.zeros((K, B, n_p), dtype=torch.float64, device=refs.device)
    out[:, :, nx:] = refs
    return out


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def _cold(P, N, nlp_ref):
    X = np.repeat(P[:, None, 0:3], N + 1, axis=1)
    return nlp_ref.join_w(X, np.zeros((P.shape[0], N, 2)))




def usable_cpus():
    """CPUs this process may run on: the affinity mask, capped by a cgroup-v2 CPU quota
    (the GPU box's share of the host); an inherited OMP_NUM_THREADS is ignored."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(float(quota) / float(period))))
    except (OSError, ValueError):
        pass
    return max(1, n)


# ---- algorithmic FP64 work of one IPM iteration of one instance
# Per node with an interval: one stage evaluation E (Model::derivs) + one backward Riccati
# step R (riccati_step + riccati_gains), both measured per unit on the device by
# tools/flop_probe.py (profiles/r04_flop_probe.json), + the IPM's vector work V below, counted
# from the sequential algorithm (the log-depth scans' extra compositions, group-uniform
# recomputation on every lane, padding lanes and the line search's further trials are not
# algorithmic work and are not counted).  Linear models' E is counted analytically (their
# Jacobians and Hessians are tables).
FLOP_PROBE = os.path.join("profiles", "r05_flop_probe.json")
ALGO_KEYS = {  # workload -> (eval key or None for a linear model, riccati key)
    2: ("unicycle_quadrature_M4", "unicycle"), 3: ("unicycle_node_M1", "unicycle"),
    4: (None, "linear4x1"), 5: (None, "linear5x1"),
    "kin_bicycle": ("kin_bicycle_M1", "kin_bicycle"), "dyn_bicycle": ("dyn_bicycle_M4", "dyn_bicycle"),
    "cartpole": ("cartpole_M1", "cartpole"),
}


def ipm_vector_flops(n, m, nbs):
    """FP64 flops per node of the IPM's vector phases (n states, m inputs, nbs finite bound
    sides), one term per phase of kernels.h's solve loop (DESIGN.md §6 lists them)."""
    nz = n + m
    err = n + 2 * n * n + 2 * n * m + 5 * nz + 3 * n + 2 * nbs + 5  # rd = grad L, |.|_inf, complementarity, sums
    mu = 3 * nbs                                                    # barrier-test complementarity
    sig = 6 * nbs + 2 * nz                                          # Sigma, barrier gradient, Hd = H + Sigma
    fwd = 2 * m * n + 2 * n * n + 2 * n * m + n + 2 * n * n + 2 * n  # du = kf + K dx, dx+, dlam = P dx + p - lam
    frac = 14 * nbs + 5 * nz                                        # bound-dual steps, fraction to boundary, tiny, gd
    ls = 2 * nz + 2 * n + 3 * n + 2 * nbs + 4                       # one trial: z + a dz, lam, theta, phi
    upd = 2 * nz + 2 * n + 8 * nbs                                  # update + kappa_sigma safeguard
    return err + mu + sig + fwd + frac + ls + upd


def linear_eval_flops(n, m):
    """Linear-quadratic stage: c = A x + B u + c0 - x+, grad q = W z + w, q."""
    nz = n + m
    return 2 * n * nz + 2 * n + 2 * nz * nz + 4 * nz


def algorithmic_flops_per_iteration(key, ocp, N):
    """Algorithmic FP64 flops of one IPM iteration of one instance, or (None, reason)."""
    path = os.path.join(ROOT, FLOP_PROBE)
    if not os.path.exists(path):
        return None, f"{FLOP_PROBE} missing"
    with open(path) as f:
        probe = json.load(f)
    ek, rk = ALGO_KEYS[key]
    n, m = ocp.nx, ocp.nu
    fin = lambda v: sum(1 for x in v if np.isfinite(x))  # noqa: E731
    nbs = fin(ocp.x_lb) + fin(ocp.x_ub) + fin(ocp.u_lb) + fin(ocp.u_ub)
    E = linear_eval_flops(n, m) if ek is None else probe["eval"][ek]["flops_per_unit"]
    R = probe["riccati"][rk]["flops_per_unit"]
    V = ipm_vector_flops(n, m, nbs)
    total = N * (E + R + V) + ipm_vector_flops(n, 0, fin(ocp.x_lb) + fin(ocp.x_ub))  # + the terminal node
    return {"per_iteration": total, "per_node": {"eval": E, "riccati": R, "ipm_vector": V},
            "eval_source": "analytic (table model)" if ek is None else f"{FLOP_PROBE}: eval {ek}",
            "riccati_source": f"{FLOP_PROBE}: riccati {rk}", "bound_sides_per_node": nbs}, None


def load_solve_pmc(kernel):
    """The solve kernel's record in the committed PMC characterisation, if it was measured on
    the library built from the sources in this tree (else (None, reason): a stale record is
    never used)."""
    from mpcx import _lib

    path = os.path.join(ROOT, SOLVE_PMC)
    if not os.path.exists(path):
        return None, f"{SOLVE_PMC} missing"
    with open(path) as f:
        d = json.load(f)
    have, want = d.get("_meta", {}).get("mpcx_source_hash"), _lib.source_hash()
    if have is None or have != want:
        return None, f"stale: {SOLVE_PMC} measured on sources {have}, this tree is {want}"
    v = d.get(kernel)
    if v and v.get("f64_lane_flops_per_group_iteration"):
        return (kernel, v), None
    return None, f"no record for {kernel} in {SOLVE_PMC}"


def solve_roofline(kernel, algo, group_iters, ms):
    """Roofline entry of the fused solve kernel: algorithmic FP64 flops of the launch's IPM
    iterations / the launch's HIP-event time / the FP64 vector peak, with the issued FP64
    lane-flops of the committed PMC characterisation beside it (when current)."""
    if algo is None or ms <= 0 or group_iters <= 0:
        return None
    fl = algo["per_iteration"] * group_iters
    ach = fl / (ms * 1e-3) / 1e12
    r = {"kernel": kernel,
         "bound": "valu", "achieved": round(ach, 4),
         "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s", "frac": round(ach / PEAK_FP64_TFLOPS, 5), "traffic": None,
         "launch_ms": round(ms, 4), "group_iterations_per_launch": int(group_iters),
         "algorithmic_flops_per_group_iteration": round(algo["per_iteration"], 1),
         "algorithmic_flops_per_node": algo["per_node"], "algorithmic_sources": [algo["eval_source"],
                                                                                 algo["riccati_source"]],
         "algorithmic_flops_per_launch": fl,
         "note": "the kernel is bound by the issue of each instance's serial chains (one wave per SIMD), "
                 "not by HBM (traffic = its inputs/outputs, see solve_kernel.hbm_frac) nor by FP64 throughput"}
    tr, why_tr = load_solve_traffic(kernel)
    if tr is not None:
        r["traffic"] = tr
    else:
        r["traffic_note"] = why_tr
    pmc, why = load_solve_pmc(kernel)
    if pmc is None:
        r["issued"] = why
    else:
        k, v = pmc
        iss = v["f64_lane_flops_per_group_iteration"]
        r["issued"] = {"kernel": k, "f64_lane_flops_per_group_iteration": round(iss, 1),
                       "tflops": round(iss * group_iters / (ms * 1e-3) / 1e12, 3),
                       "algorithmic_over_issued": round(algo["per_iteration"] / iss, 4), "source": SOLVE_PMC}
        # the bound named above: with one wave per SIMD, the share of the wave's cycles in which it
        # issues an instruction is the kernel's fraction of its issue ceiling (1.0)
        wc = v.get("wave_cycles_share") or {}
        if "issuing" in wc:
            r["issue"] = {"issuing_share_of_wave_cycles": wc["issuing"],
                          "waitcnt_or_barrier_share": wc.get("waitcnt_or_barrier"),
                          "dependency_or_pipe_stall_share": wc.get("dependency_or_pipe_stall"),
                          "valu_active_share": v.get("valu_active_share"), "source": SOLVE_PMC}
    return r


def sweep_roofline(solver, torch, B, N, reps, stream):
    """Time the rk4_sens sweep kernel at B instances (tiled SoA buffers resident in HBM)."""
    from mpcx import _lib
    import ctypes

    dev = torch.device("cuda", torch.cuda.current_device())
    g = torch.Generator(device="cpu").manual_seed(7)
    T = (B + 63) // 64  # tiled SoA (include/mpcx.h: mpcx_rk4_sens_dev): [stage][tile][field][64]
    X = torch.empty((N + 1, T, 3, 64), dtype=torch.float64)
    X[:, :, 0:2].uniform_(-10, 10, generator=g)
    X[:, :, 2].uniform_(-3.14, 3.14, generator=g)
    U = torch.empty((N, T, 2, 64), dtype=torch.float64).uniform_(-0.78, 0.78, generator=g)
    XR = torch.empty((1, T, 3, 64), dtype=torch.float64).uniform_(-10, 10, generator=g)
    X, U, XR = X.to(dev), U.to(dev), XR.to(dev)
    J = torch.empty((N, T, 12, 64, 2), dtype=torch.float64, device=dev)  # per-interval records (field pairs)
    lib = _lib.load()
    vp = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    s = ctypes.c_void_p(stream.cuda_stream)

    def launch():
        _lib.check(lib.mpcx_rk4_sens_dev(solver._h.ptr, B, vp(X), vp(U), vp(XR), vp(J), s))

    for _ in range(3):
        launch()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        launch()
    e1.record(stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    del X, U, XR, J
    torch.cuda.empty_cache()
    return ms


def load_solve_traffic(kernel):
    """HBM bytes of the timed K-step solve launch from the committed PMC passes
    (profiles/*_solve_traffic.json, tools/solve_traffic.py), when they measured the tree's
    current sources and this kernel; else (None, why)."""
    from mpcx import _lib

    path = os.path.join(ROOT, "profiles", SOLVE_TRAFFIC)
    if not os.path.exists(path):
        return None, f"no {SOLVE_TRAFFIC}"
    with open(path) as f:
        d = json.load(f)
    src = _lib.source_hash()
    if d.get("mpcx_source_hash") != src:
        return None, f"{SOLVE_TRAFFIC} measured sources {d.get('mpcx_source_hash')}, tree {src}"
    if d.get("kernel") != kernel:
        return None, f"{SOLVE_TRAFFIC} measured {d.get('kernel')}"
    return float(d["hbm_bytes_per_launch"]), None


def load_traffic(B, N):
    """HBM bytes per sweep launch from the committed rocprofv3 PMC summary, if any."""
    path = os.path.join(ROOT, "profiles", "rk4_sens_pmc.json")
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            d = json.load(f)
        if d.get("B") == B and d.get("N") == N:
            return float(d["hbm_bytes_per_launch"])
    except Exception:
        return None
    return None


def launch_plan(gpus, env=None, n_devices=None):
    """How `--gpus N` runs (decided before any GPU call).  Returns ("run", None) when this
    process is one rank of a world of N, ("spawn", argv) when a plain `python bench.py --gpus N`
    must start the N ranks itself (torch.distributed.run, one process per GPU, LOCAL_RANK ->
    cuda:LOCAL_RANK), and raises SystemExit on any mismatch -- a line whose n_gpus differs
    from --gpus is never printed."""
    env = os.environ if env is None else env
    if gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    under_launcher = "WORLD_SIZE" in env or "RANK" in env
    world = int(env.get("WORLD_SIZE", "1"))
    if under_launcher:
        if world != gpus:
            raise SystemExit(f"--gpus {gpus} but WORLD_SIZE={world}: launch one rank per GPU "
                             f"(--nproc-per-node {gpus}) or drop the launcher")
        return "run", None
    if gpus == 1:
        return "run", None
    if n_devices is not None and gpus > n_devices and env.get("MPCX_FORCE_DEVICE") is None:
        raise SystemExit(f"--gpus {gpus} but only {n_devices} visible GPU(s)")
    import socket

    with socket.socket() as so:  # a free rendezvous port on the loopback interface
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    argv = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return "spawn", argv


def main():
    args = parse()
    from mpcx import dist as mdist

    import torch

    # the launch plan is decided before any GPU call, on a device count read from the KFD
    # topology (mdist.visible_gpu_count never initialises HIP)
    plan, argv = launch_plan(args.gpus, n_devices=mdist.visible_gpu_count())
    if plan == "spawn":
        import subprocess

        # the ranks run as child processes (never an exec from this process), rank 0 prints the line
        raise SystemExit(subprocess.run(argv).returncode)
    rank, world, local = mdist.env()
    assert world == args.gpus

    local = mdist.device_index(local)
    if local >= torch.cuda.device_count():  # each rank checks its own GPU (this rank's first GPU call)
        raise SystemExit(f"rank {rank}: GPU {local} not visible ({torch.cuda.device_count()} device(s))")
    torch.cuda.set_device(local)
    mdist.init(mdist.backend("nccl"))
    import mpcx
    from mpcx import _lib
    from mpcx.device import DeviceLoop

    cfg = args.config
    variant = None if args.model == "default" else args.model
    if variant is not None and VARIANTS.get(cfg) != variant:
        raise SystemExit(f"--model {variant} is the variant of config "
                         f"{[c for c, v in VARIANTS.items() if v == variant][0]}")
    dev = f"cuda:{local}"
    N = args.N or {2: 20, 3: 30, 4: 50, 5: 100}[cfg]
    B = args.batch or {2: 1024, 3: 4096, 4: 1024, 5: 2048}[cfg]
    start, stop = mdist.shard(B, rank)
    T_all = args.warmup + 2 * args.steps  # warmup, timed multi-step run, lock-step latency run
    per_step = None  # per-step device updates (stage references / schedules), resident in HBM
    seq = lambda t0, K: (None, None)  # noqa: E731  same, as sequences for a multi-step launch
    if variant is not None:
        ocp = {"kin_bicycle": mpcx.kinematic_bicycle_tracking, "dyn_bicycle": mpcx.dynamic_bicycle_lane_change,
               "cartpole": mpcx.cartpole_swingup}[variant](N=N)
    elif cfg in (2, 3):
        ocp = mpcx.unicycle_point_to_point(N=N) if cfg == 2 else mpcx.unicycle_tracking(N=N)
    elif cfg == 4:
        t0, x0, par = mdist.config4_inputs(start, stop, N=N)
        _, _, vref = mdist.lane_change()
        ocp = mpcx.lateral_ltv(N=N, Delta=0.05, vref=vref, per_instance_tab=np.minimum(t0, 499))
    else:
        ocp = mpcx.inverted_pendulum_qp(N=N)
    # config 2 is Casadi/multiple_shooting_casadi.py: its own IPOPT options (:188-196); the
    # others run IPOPT's defaults (mpctools / no reference script)
    ipopt = ({"max_iter": 2000, "acceptable_tol": 1e-8, "acceptable_obj_change_tol": 1e-6}
             if cfg == 2 and variant is None else {"max_iter": 3000})
    solver = mpcx.nlpsol("bench", "mi355x", ocp, {"ipopt": ipopt, "group_policy": args.group_policy}, device=local)
    stream = torch.cuda.current_stream()

    if args.profile_sweep_only:
        ms = sweep_roofline(solver, torch, args.roofline_batch, N, args.roofline_reps, stream)
        if rank == 0:
            print(json.dumps({"sweep_ms": ms, "B": args.roofline_batch, "N": N}))
        return

    if variant == "kin_bicycle":  # per-step references on the config-3 circle
        tau0, P0 = mdist.config3_bicycle_inputs(start, stop, N=N)
        refs = torch.from_numpy(np.stack([mpcx.ode.bicycle_circular_reference(tau0, t, N).reshape(B, -1)
                                          for t in range(T_all)])).to(dev)
        per_step = lambda lp, t: lp.set_stage_refs(refs[t])  # noqa: E731
        seq = lambda t0, K: (_pseq(refs[t0:t0 + K], P0.shape[1], 3), None)  # noqa: E731
    elif variant == "dyn_bicycle":  # instance time t0 + t on the scaled lane change
        t0, x0, (Xp, Yp, Vp) = mdist.config4_bicycle_inputs(start, stop)
        refs = torch.from_numpy(np.stack([np.stack([mpcx.ode.dyn_bicycle_references(Xp, Yp, Vp, int(ti) + t, N)
                                                    .reshape(-1) for ti in t0]) for t in range(T_all)])).to(dev)
        P0 = ocp.params(x0, refs[0].cpu().numpy())
        per_step = lambda lp, t: lp.set_stage_refs(refs[t])  # noqa: E731
        seq = lambda t0, K: (_pseq(refs[t0:t0 + K], P0.shape[1], 6), None)  # noqa: E731
    elif variant == "cartpole":
        P0 = mdist.config5_swingup_inputs(start, stop)
    elif cfg == 2:
        P0 = mdist.config2_inputs(start, stop, args.seed)
    elif cfg == 3:  # per-step circular references (Trajectory_tracking.py:84-97)
        tau0, P0 = mdist.config3_inputs(start, stop, N=N)
        refs = torch.from_numpy(np.stack([mpcx.ocp.circular_reference(tau0, t, N).reshape(B, -1)
                                          for t in range(T_all)])).to(dev)
        per_step = lambda lp, t: lp.set_stage_refs(refs[t])  # noqa: E731
        seq = lambda t0, K: (_pseq(refs[t0:t0 + K], P0.shape[1], 3), None)  # noqa: E731
    elif cfg == 4:  # instance time t0 + t: references par[t] and the model re-linearised at vref[t] (:117-141)
        tt = np.minimum(t0[None, :] + np.arange(T_all)[:, None], 499)  # (T_all, B)
        refs = torch.from_numpy(np.ascontiguousarray(par[tt].reshape(T_all, B, -1))).to(dev)
        tabs = torch.from_numpy(np.repeat(tt[:, :, None], N, axis=2).astype(np.int32)).to(dev)
        P0 = ocp.params(x0, par[tt[0]])

        def per_step(lp, t):
            lp.set_stage_refs(refs[t])
            lp.set_schedule(tabs[t])

        seq = lambda t0, K: (_pseq(refs[t0:t0 + K], P0.shape[1], 4), tabs[t0:t0 + K].contiguous())  # noqa: E731
    else:
        P0 = mpcx.lti.pendulum_params(ocp, mdist.config5_inputs(start, stop), 0.0)
    K = args.steps

    def closed_loop(warm_duals):
        """W untimed warm-up steps, K timed steps (one multi-step launch, or K launches in
        --mode lockstep), then K lock-step launches timed with HIP events (the latency a real-time
        loop sees per step), under one warm-start policy (POLICY).  Every policy starts from the
        same P0 and the same per-step references."""
        loop = DeviceLoop(solver, P0, device=dev, stream=stream, warm_duals=warm_duals)
        warm_it = torch.zeros((max(args.warmup, 1), B), dtype=torch.int32, device=loop.P.device)
        for t in range(args.warmup):
            if per_step is not None:
                per_step(loop, t)
            loop.step(iters_out=warm_it[t])
        torch.cuda.synchronize()
        iters_hist = torch.zeros((K, B), dtype=torch.int32, device=loop.P.device)
        status_hist = torch.zeros((K, B), dtype=torch.int32, device=loop.P.device)
        t_seq = args.warmup
        if per_step is not None:
            per_step(loop, t_seq)  # current references / schedule = those of the first timed step
        Pseq, tabseq = seq(t_seq, K)
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev_run = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        if args.mode == "async":
            # K closed-loop steps in ONE launch; every instance runs its own receding-horizon loop
            # (bit-identical to K lock-step launches, tests/test_gpu_parity.py::test_run_*)
            ev_run[0].record(stream)
            loop.run(K, status_out=status_hist, iters_out=iters_hist, Pseq=Pseq, tabseq=tabseq)
            ev_run[1].record(stream)
        else:
            for i in range(K):
                if per_step is not None and i > 0:
                    per_step(loop, t_seq + i)
                loop.step(status_out=status_hist[i], iters_out=iters_hist[i])
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        if args.profile_solve_only:  # the timed launch is the last solve dispatch of this process
            print(json.dumps({"profile_solve_only": True, "run_ms": ev_run[0].elapsed_time(ev_run[1])
                              if args.mode == "async" else None, "solve_kernel": solver._h.launch_shape(B)[2],
                              "mpcx_source_hash": _lib.source_hash()}))
            sys.exit(0)
        if world > 1:
            torch.distributed.barrier()
        elapsed = mdist.max_over_ranks(t1 - t0, device=loop.P.device)

        # lock-step latency: K further steps, one launch each, HIP events on the launch stream
        # (ms_per_solve_p50 = the latency a real-time loop sees per closed-loop step)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
        lk_st = torch.zeros((K, B), dtype=torch.int32, device=loop.P.device)
        lk_it = torch.zeros((K, B), dtype=torch.int32, device=loop.P.device)
        torch.cuda.synchronize()
        tl0 = time.perf_counter()
        for i in range(K):
            if per_step is not None:
                per_step(loop, args.warmup + K + i)
            ev[i][0].record(stream)
            loop.step(status_out=lk_st[i], iters_out=lk_it[i])
            ev[i][1].record(stream)
        torch.cuda.synchronize()
        tl1 = time.perf_counter()
        lock_elapsed = mdist.max_over_ranks(tl1 - tl0, device=loop.P.device)
        solve_ms = sorted(a.elapsed_time(b) for a, b in ev)
        dv = loop.P.device
        return {"loop": loop, "warm_it": warm_it, "iters_hist": iters_hist, "status_hist": status_hist,
                "lk_st": lk_st, "lk_it": lk_it, "elapsed": elapsed, "lock_elapsed": lock_elapsed,
                "solve_ms": solve_ms, "p50": mdist.max_over_ranks(float(np.median(solve_ms)), device=dv),
                "lock_iters_max": mdist.max_over_ranks(float(lk_it.max(dim=1).values.double().mean().item()), device=dv),
                "iters_max_step": mdist.max_over_ranks(float(iters_hist.max(dim=1).values.double().mean().item()),
                                                       device=dv),
                "iters_mean": mdist.max_over_ranks(float(iters_hist.double().mean().item()), device=dv),
                "run_ms": ev_run[0].elapsed_time(ev_run[1]) if args.mode == "async" else float(np.sum(solve_ms))}

    res = closed_loop(warm_duals=True)  # the headline policy ("dual")
    ref_res = closed_loop(warm_duals=False) if not args.no_reference_warm_start else None
    loop, warm_it, iters_hist, status_hist = res["loop"], res["warm_it"], res["iters_hist"], res["status_hist"]
    lk_it, elapsed, lock_elapsed, solve_ms = res["lk_it"], res["elapsed"], res["lock_elapsed"], res["solve_ms"]
    p50, lock_iters_max = res["p50"], res["lock_iters_max"]

    # closed-loop statistics: the only collective (RCCL all_gather over xGMI), outside the timed region
    def P_fin_of(lp):
        """Final state next to its target (first three states) for the stats matrix."""
        Pf = lp.P.cpu().numpy()
        if variant is not None:  # first three states against the stage-0 reference / set point
            return np.concatenate([Pf[:, 0:3], Pf[:, ocp.nx:ocp.nx + 3]], axis=1)
        if cfg == 3:  # final error against the stage-0 reference
            return np.concatenate([Pf[:, 0:3], Pf[:, 3:6]], axis=1)
        if cfg == 4:  # (y, phi, v_y) against the stage-0 reference
            return np.concatenate([Pf[:, 0:3], Pf[:, 4:7]], axis=1)
        if cfg == 5:  # (x, x', th) against the set point (10, 0, 0)
            return np.concatenate([Pf[:, 0:3], np.tile([ocp.x_target, 0.0, 0.0], (B, 1))], axis=1)
        return Pf

    S = mdist.stats_matrix(P_fin_of(loop), None, loop.f.cpu().numpy(), status_hist.max(dim=0).values.cpu().numpy(),
                           iters_hist.cpu().numpy())
    S_all = mdist.all_gather_stats(S, device=loop.P.device)
    if rank == 0 and args.dump_stats:
        np.save(args.dump_stats, S_all)  # (global batch, STAT_FIELDS): shard-exactness tests
    iters_max_step = res["iters_max_step"]

    # group-iterations of every solve launch of this run, both policies (PMC normalisation,
    # tools/solve_pmc_summary.py)
    iters_all = sum(int(r["warm_it"][:args.warmup].sum().item() + r["iters_hist"].sum().item() +
                        r["lk_it"].sum().item()) for r in (res, ref_res) if r is not None)

    roof = None
    if rank == 0 and not args.no_roofline and cfg == 2:
        Br = args.roofline_batch
        ms = sweep_roofline(solver, torch, Br, N, args.roofline_reps, stream)
        alg = Br * (SWEEP_BYTES_PER_STAGE * N + SWEEP_BYTES_PER_INSTANCE)
        ach = alg / (ms * 1e-3) / 1e9
        traffic = load_traffic(Br, N)
        roof = {"kernel": "rk4_sens_kernel (RK4 M=4 + Jacobian sweep)", "bound": "hbm", "achieved": round(ach, 1),
                "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": round(ach / PEAK_HBM_GBS, 4), "traffic": traffic,
                "launch_ms": round(ms, 4), "units_per_launch": Br * N, "unit_of_work": "stage evaluation",
                "bytes_per_launch": alg, "config": f"B={Br}, N={N}"}
        if traffic:  # the HBM rate the launch actually moved (PMC bytes, compulsory writes included)
            roof["frac_on_traffic"] = round(traffic / (ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4)

    # the dominant kernel of the timed region: the multi-step solve launch (async mode; HIP
    # events on the launch stream) or the mean single-step launch (lock-step latency run)
    G, Rrep, kname = solver._h.launch_shape(B)  # the instantiation the library launches (mpcx_launch_shape)
    run_ms = res["run_ms"]
    run_iters = int(iters_hist.sum().item()) if args.mode == "async" else int(lk_it.sum().item())
    algo, why_not = algorithmic_flops_per_iteration(variant or cfg, ocp, N)
    roof_solve = solve_roofline(kname, algo, run_iters, run_ms) if rank == 0 else None
    if rank == 0 and roof_solve is None:
        roof_solve = {"kernel": kname, "unavailable": why_not or "no timed iterations"}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu and cfg == 2:
        cores = usable_cpus()
        steps = args.warmup + args.steps
        make_P = lambda r: mdist.config2_inputs(r * B, (r + 1) * B, args.seed)  # noqa: E731
        rate, t, reps, its = cpu_baseline(make_P, N, steps, cores, min_seconds=args.cpu_seconds)
        # the reference's own loop is one solve at a time on one core (multiple_shooting_casadi.py:226-298)
        B1 = 128
        rate1, t1, reps1, _ = cpu_baseline(lambda r: make_P(r)[:B1], N, steps, 1, min_seconds=args.cpu_seconds / 2)
        cpu = {"value": round(rate, 1), "unit": "solves/s", "cores": cores, "kind": "port",
               "policy": POLICY["dual"],
               "sample": f"{reps} x ({steps}-step closed loop of {B} config-2 instances, N={N}, the GPU loop's "
                         f"warm start and IPOPT options); {t:.1f} s of timed solve calls on {cores} OpenMP threads",
               "iters_mean": round(its, 2),
               "value_1core": round(rate1, 1),
               "sample_1core": f"{reps1} x ({steps}-step closed loop of {B1} instances), {t1:.1f} s on 1 thread",
               "host_cpus": os.cpu_count(), "usable_cpus": cores, "cpu_model": cpu_model()}
        if ref_res is not None:  # the same loops under the reference's warm start (shifted primal only)
            rate_r, t_r, reps_r, its_r = cpu_baseline(make_P, N, steps, cores, min_seconds=args.cpu_seconds,
                                                      warm=None)
            cpu["reference_warm_start"] = {
                "value": round(rate_r, 1), "unit": "solves/s", "cores": cores, "policy": POLICY["reference"],
                "iters_mean": round(its_r, 2),
                "sample": f"{reps_r} x ({steps}-step closed loop of {B} config-2 instances), {t_r:.1f} s of timed "
                          f"solve calls on {cores} OpenMP threads"}

    # the kernel that dominates the timed step: the fused solve (+ plant/shift) launch.  Its HBM
    # traffic is its inputs and outputs only, so neither HBM nor the FP64 pipes bound it: it is
    # latency-bound on the sequential Riccati/forward chains (one wave per SIMD).
    nw, ng, npar = solver._h.n_w, solver._h.n_g, solver._h.n_p
    io_bytes = B * 8 * ((npar + 2 * nw + ng) + (nw + 1 + ng + nw) + (ocp.nx + 2 * nw + ng)) + B * 8
    solve_info = {"kernel": "solve_kernel (fused IPM solve + plant/shift, one launch per step)",
                  "bound": "VALU issue of each instance's serial instruction stream (sequential Riccati/forward "
                           "chains run by the whole wave), one wave per SIMD",
                  "ms_p50": round(p50, 4), "iters_max_per_step_mean": round(float(lock_iters_max), 2),
                  "us_per_ipm_iteration": round(p50 * 1e3 / max(lock_iters_max, 1.0), 2),
                  "hbm_bytes_per_launch": io_bytes,
                  "hbm_frac": round(io_bytes / (p50 * 1e-3) / 1e9 / PEAK_HBM_GBS, 5)}
    solve_info.update({"group_size": G, "replicas": Rrep, "timed_launch_ms": round(run_ms, 4),
                       "timed_group_iterations": run_iters})
    ref_block = None
    if ref_res is not None:
        # the same K-step / lock-step timing with the reference's warm start (POLICY["reference"]);
        # value / lockstep.value / ms_per_solve_p50 / iters as for the headline policy above
        r_ = ref_res
        S_r = mdist.all_gather_stats(mdist.stats_matrix(P_fin_of(r_["loop"]), None, r_["loop"].f.cpu().numpy(),
                                                        r_["status_hist"].max(dim=0).values.cpu().numpy(),
                                                        r_["iters_hist"].cpu().numpy()), device=loop.P.device)
        ref_block = {
            "value": round(world * B * K / r_["elapsed"], 1), "unit": "solves/s",
            "ms_per_step": round(r_["elapsed"] / K * 1e3, 4),
            "lockstep": {"value": round(world * B * K / r_["lock_elapsed"], 1),
                         "ms_per_step": round(r_["lock_elapsed"] / K * 1e3, 4),
                         "iters_max_per_step_mean": round(float(r_["lock_iters_max"]), 2)},
            "ms_per_solve_p50": round(r_["p50"], 4),
            "workload": (workload_name_v(variant, N, ocp.M) if variant else workload_name(cfg, N)) + "; " +
                        POLICY["reference"],
            "warm_start_policy": "reference",
            "iters_mean": round(float(S_r[:, 1].mean()), 2), "iters_max": int(S_r[:, 2].max()),
            "iters_max_per_step_mean": round(float(r_["iters_max_step"]), 2),
            "failed_instances": int((S_r[:, 3] > 1).sum()),
            "us_per_ipm_iteration": round(r_["p50"] * 1e3 / max(r_["lock_iters_max"], 1.0), 2),
            "timed_launch_ms": round(r_["run_ms"], 4)}
    if rank == 0:
        total = world * B * K
        out = {
            "metric": METRIC, "value": round(total / elapsed, 1), "unit": "solves/s", "n_gpus": world,
            "steps": K, "warmup": args.warmup, "ms_per_step": round(elapsed / K * 1e3, 4),
            "mode": args.mode,
            "lockstep": {"value": round(world * B * K / lock_elapsed, 1),
                         "ms_per_step": round(lock_elapsed / K * 1e3, 4),
                         "iters_max_per_step_mean": round(float(lock_iters_max), 2)},
            "ms_per_solve_p50": round(p50, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f64",
            "data": DATA_V[variant] if variant else DATA[cfg],
            "config": {"workload": (workload_name_v(variant, N, ocp.M) if variant else workload_name(cfg, N)) +
                                   "; " + POLICY["dual"],
                       "warm_start_policy": "dual",
                       "dynamics": DYN_V[variant] if variant else DYN[cfg], "N": N,
                       "M": getattr(ocp, "M", None), "batch_per_gpu": B, "global_batch": B * world,
                       "parallelism": f"instance-sharded x{world} (no data-path collective)"},
            "iters_mean": round(float(S_all[:, 1].mean()), 2), "iters_max": int(S_all[:, 2].max()),
            "iters_max_per_step_mean": round(float(iters_max_step), 2),
            "failed_instances": int((S_all[:, 3] > 1).sum()),
            "iters_sum_all_steps": int(iters_all),
            "reference_warm_start": ref_block,
            "roofline": roof_solve, "roofline_sweep": roof, "cpu_baseline": cpu, "solve_kernel": solve_info,
            "mpcx_source_hash": _lib.source_hash(),
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
