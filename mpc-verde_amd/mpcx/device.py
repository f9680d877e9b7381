"""Device-resident batched receding-horizon loop (torch tensors as device memory).

PyTorch provides device allocations, streams and events only; all arithmetic is
in libmpcx's HIP kernels, reached through the ``*_dev`` C entry points.  One
closed-loop step for B instances = one fused solve launch + one shift/plant
launch (``Casadi/multiple_shooting_casadi.py:226-287``, batched), with no host
synchronisation in between.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from .nlpsol import Solver


def _ptr(t):
    return None if t is None else ctypes_void(t.data_ptr())


def ctypes_void(p):
    import ctypes

    return ctypes.c_void_p(p)


def _check(t, name, dtype, shape, device):
    """Every tensor handed to the kernels as a raw device pointer: right dtype, exact shape,
    contiguous, on the loop's device.  A wrong one would be an out-of-bounds access or a host
    pointer dereferenced by the GPU, so it is rejected here."""
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name}: expected a torch tensor")
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected dtype {dtype}, got {t.dtype}")
    if tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name}: expected shape {tuple(shape)}, got {tuple(t.shape)}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")
    if t.device != device:
        raise ValueError(f"{name}: must live on {device}, got {t.device}")
    return t


class DeviceLoop:
    """B independent MPC instances stepped on one GPU.

    P (B, n_p) float64 parameters live on the device; w holds the last solution
    and w0 the shifted warm start.  With warm_duals (default) the constraint and
    bound multipliers are shifted as well and the next solve starts as IPOPT's
    warm_start_init_point (spec.warm_*); the first solve is always cold.
    ``step()`` enqueues one fused solve + plant/shift launch on ``stream`` and
    returns immediately (``solve()`` / ``shift()`` do the two halves separately).
    A linear model embedded in a larger kernel instantiation (``lti.StatePad``) takes P0 in
    its own layout; the device tensors hold the kernel's padded layout
    (``solver._pad.w_idx`` / ``p_idx`` / ``g_idx`` select the model's entries).
    """

    def __init__(self, solver: Solver, P0, device="cuda", stream=None, cold_first=True, warm_duals=True):
        self.solver = solver
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("DeviceLoop needs a HIP device (torch 'cuda' device)")
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        P0 = np.ascontiguousarray(np.asarray(P0, np.float64))
        if P0.ndim != 2 or P0.shape[1] != solver.n_p:
            raise ValueError(f"P0: expected (B, {solver.n_p}), got {P0.shape}")
        pd = getattr(solver, "_pad", None)
        if pd is not None:
            P0 = pd.scatter(P0, pd.p_idx, pd.n_p_pad)
        self._knx = pd.nxp if pd is not None else solver.ocp.nx  # states of the kernel layout
        self.B = P0.shape[0]
        nw, ng = solver._h.n_w, solver._h.n_g
        z = lambda *s: torch.zeros(s, dtype=torch.float64, device=self.device)  # noqa: E731
        self.P = torch.from_numpy(P0).to(self.device)
        self.w, self.w0 = z(self.B, nw), z(self.B, nw)
        self.lam, self.lam0 = z(self.B, ng), z(self.B, ng)
        self.lamx, self.lamx0 = z(self.B, nw), z(self.B, nw)
        self.f = z(self.B)
        self.status = torch.zeros(self.B, dtype=torch.int32, device=self.device)
        self.iters = torch.zeros(self.B, dtype=torch.int32, device=self.device)
        self.stream = stream if stream is not None else torch.cuda.current_stream(self.device)
        self.warm_duals = warm_duals
        self._cold = cold_first

    def solve(self, status_out=None, iters_out=None):
        """Enqueue one batched solve.  status_out / iters_out: optional int32 device
        tensors (B,) that receive this step's statuses / iteration counts directly
        from the kernel (no extra launch)."""
        lib = _lib.load()
        s = ctypes_void(self.stream.cuda_stream)
        w0 = None if self._cold else _ptr(self.w0)
        warm = self.warm_duals and not self._cold
        st = self.status if status_out is None else _check(status_out, "status_out", torch.int32, (self.B,), self.device)
        it = self.iters if iters_out is None else _check(iters_out, "iters_out", torch.int32, (self.B,), self.device)
        _lib.check(lib.mpcx_solve_batch_dev(self.solver._h.ptr, self.B, _ptr(self.P), w0,
                                            _ptr(self.lam0) if warm else None, _ptr(self.lamx0) if warm else None,
                                            _ptr(self.w), _ptr(self.f), _ptr(self.lam), _ptr(self.lamx), _ptr(st),
                                            _ptr(it), s))
        self._cold = False

    def shift(self):
        lib = _lib.load()
        s = ctypes_void(self.stream.cuda_stream)
        d = self.warm_duals
        _lib.check(lib.mpcx_shift_dev(self.solver._h.ptr, self.B, _ptr(self.P), _ptr(self.w), _ptr(self.w0),
                                      _ptr(self.lam) if d else None, _ptr(self.lam0) if d else None,
                                      _ptr(self.lamx) if d else None, _ptr(self.lamx0) if d else None, s))

    def set_stage_refs(self, refs):
        """Per-step stage references (tracking, param layout x0_stageref): refs is a
        (B, N*(nx+nu)) float64 device tensor copied into P[:, nx:] on the loop's stream
        (Trajectory_tracking.py:105-106 sets solver.par["p", k] each step)."""
        nx = self._knx
        _check(refs, "refs", torch.float64, (self.B, self.P.shape[1] - nx), self.device)
        with torch.cuda.stream(self.stream):
            self.P[:, nx:].copy_(refs, non_blocking=True)

    def run(self, K, status_out=None, iters_out=None, Pseq=None, tabseq=None):
        """K closed-loop steps in ONE launch (mpcx_run_dev): each instance runs its own
        receding-horizon loop without waiting for the others between steps; the results
        equal K calls of step() bit for bit.  status_out / iters_out: int32 (K, B) device
        tensors (or None -> allocated).  Pseq (K, B, n_p) float64 and tabseq (K, B, N) int32
        device tensors give per-step stage references / linear schedules (row 0 = the
        current ones).  Returns (status, iters)."""
        lib = _lib.load()
        s = ctypes_void(self.stream.cuda_stream)
        K = int(K)
        if K < 1:
            raise ValueError("K must be >= 1")
        z = lambda: torch.zeros((K, self.B), dtype=torch.int32, device=self.device)  # noqa: E731
        st = z() if status_out is None else _check(status_out, "status_out", torch.int32, (K, self.B), self.device)
        it = z() if iters_out is None else _check(iters_out, "iters_out", torch.int32, (K, self.B), self.device)
        if Pseq is not None:
            _check(Pseq, "Pseq", torch.float64, (K, self.B, self.P.shape[1]), self.device)
        if tabseq is not None:
            _check(tabseq, "tabseq", torch.int32, (K, self.B, self.solver.ocp.N), self.device)
        flags = _lib.STEP_COLD if self._cold else 0
        if not self.warm_duals:
            flags |= _lib.STEP_PRIMAL_ONLY
        d = self.warm_duals
        _lib.check(lib.mpcx_run_dev(self.solver._h.ptr, self.B, K, _ptr(self.P), _ptr(self.w0),
                                    _ptr(self.lam0) if d else None, _ptr(self.lamx0) if d else None, flags, _ptr(Pseq),
                                    _ptr(tabseq), _ptr(self.w), _ptr(self.f), _ptr(self.lam), _ptr(self.lamx), _ptr(st),
                                    _ptr(it), s))
        self._cold = False
        return st, it

    def set_schedule(self, tab):
        """Per-step stage schedule of a linear model: tab is a (B, N) int32 device tensor
        of table indices read by the next solves/shifts (mpcx_set_linear_tab_dev; LTV
        re-linearisation per step, Trajectory_tracking_dynamic_model.py:117-141).  The
        tensor must stay alive while it is in use; None reverts to the uploaded schedule."""
        lib = _lib.load()
        if tab is None:
            _lib.check(lib.mpcx_set_linear_tab_dev(self.solver._h.ptr, None, 0))
            self._tab = None
            return
        _check(tab, "tab", torch.int32, (self.B, self.solver.ocp.N), self.device)
        self._tab = tab
        _lib.check(lib.mpcx_set_linear_tab_dev(self.solver._h.ptr, ctypes_void(tab.data_ptr()), self.B))

    def step(self, status_out=None, iters_out=None):
        """One closed-loop step = ONE kernel launch (mpcx_step_dev): the batched solve and,
        fused into its epilogue, the plant + shifted warm start (same result as
        solve() followed by shift())."""
        lib = _lib.load()
        s = ctypes_void(self.stream.cuda_stream)
        flags = _lib.STEP_COLD if self._cold else (0 if self.warm_duals else _lib.STEP_PRIMAL_ONLY)
        d = self.warm_duals
        st = self.status if status_out is None else _check(status_out, "status_out", torch.int32, (self.B,), self.device)
        it = self.iters if iters_out is None else _check(iters_out, "iters_out", torch.int32, (self.B,), self.device)
        _lib.check(lib.mpcx_step_dev(self.solver._h.ptr, self.B, _ptr(self.P), _ptr(self.w0),
                                     _ptr(self.lam0) if d else None, _ptr(self.lamx0) if d else None, flags,
                                     _ptr(self.w), _ptr(self.f), _ptr(self.lam), _ptr(self.lamx), _ptr(st), _ptr(it),
                                     s))
        self._cold = False
