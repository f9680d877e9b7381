"""ctypes binding of ``libmpcx.so`` (the C ABI declared in ``include/mpcx.h``).

The HIP library is the only compute path: if it is missing or cannot be loaded
this module raises immediately -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MPCX_LIB", os.path.join(_HERE, "libmpcx.so"))

MODEL_UNICYCLE = 1
MODEL_LINEAR = 2
MODEL_KIN_BICYCLE = 3
MODEL_DYN_BICYCLE = 4
MODEL_CARTPOLE = 5
COST_QUADRATURE = 0
COST_NODE = 1
P_X0_XREF = 0
P_X0_STAGEREF = 1

STATUS = {0: "Solve_Succeeded", 1: "Solved_To_Acceptable_Level", 2: "Maximum_Iterations_Exceeded",
          3: "Restoration_Failed", 4: "Infeasible_Problem_Detected", 5: "Error_In_Step_Computation"}

# C-ABI entry points (include/mpcx.h) -- checked by tests/test_capi_symbols.py
EXPORTS = ("mpcx_default_spec", "mpcx_create", "mpcx_destroy", "mpcx_last_error", "mpcx_dims", "mpcx_solve_batch",
           "mpcx_solve_batch_dev", "mpcx_plant_step", "mpcx_shift_dev", "mpcx_rk4_sens", "mpcx_rk4_sens_dev",
           "mpcx_set_linear_model", "mpcx_set_linear_tab_dev", "mpcx_step_dev", "mpcx_run_dev",
           "mpcx_source_hash", "mpcx_launch_shape")
STEP_COLD = 1
STEP_PRIMAL_ONLY = 2


class Spec(ctypes.Structure):
    """Mirror of ``mpcx_spec`` (include/mpcx.h)."""

    _fields_ = [("model", ctypes.c_int32), ("cost", ctypes.c_int32), ("param_layout", ctypes.c_int32),
                ("N", ctypes.c_int32), ("M", ctypes.c_int32), ("max_iter", ctypes.c_int32),
                ("device", ctypes.c_int32), ("group_policy", ctypes.c_int32), ("T", ctypes.c_double),
                ("tol", ctypes.c_double), ("Q", ctypes.c_double * 8), ("R", ctypes.c_double * 8),
                ("lbu", ctypes.c_double * 8), ("ubu", ctypes.c_double * 8), ("lbx", ctypes.c_double * 8),
                ("ubx", ctypes.c_double * 8), ("warm_mu_init", ctypes.c_double),
                ("warm_bound_push", ctypes.c_double), ("warm_mult_push", ctypes.c_double),
                ("nx", ctypes.c_int32), ("nu", ctypes.c_int32), ("par", ctypes.c_double * 8),
                ("dual_inf_tol", ctypes.c_double), ("constr_viol_tol", ctypes.c_double),
                ("compl_inf_tol", ctypes.c_double), ("acceptable_tol", ctypes.c_double),
                ("acceptable_dual_inf_tol", ctypes.c_double), ("acceptable_constr_viol_tol", ctypes.c_double),
                ("acceptable_compl_inf_tol", ctypes.c_double), ("acceptable_obj_change_tol", ctypes.c_double),
                ("acceptable_iter", ctypes.c_int32), ("no_restoration", ctypes.c_int32)]


_lib = None


class MpcxError(RuntimeError):
    pass


def _bind_single_hip_runtime():
    """Make libmpcx resolve libamdhip64.so.7 to the copy PyTorch uses, if PyTorch is installed.

    PyTorch-ROCm ships its own libamdhip64 (NEEDED as "libamdhip64.so", found via
    its RPATH) while libmpcx is linked against /opt/rocm's (NEEDED
    "libamdhip64.so.7"); both carry the soname libamdhip64.so.7.  Loaded in the
    wrong order a process ends up with two HIP runtimes, and the second one cannot
    open the GPU ("No HIP GPUs are available").  Loading PyTorch's copy first
    (without importing torch) makes every later lookup resolve to that one file.
    """
    import importlib.util

    try:
        spec = importlib.util.find_spec("torch")
    except (ImportError, ValueError):
        spec = None
    if spec is None or not spec.origin:
        return
    p = os.path.join(os.path.dirname(spec.origin), "lib", "libamdhip64.so")
    if os.path.exists(p):
        ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL)


def source_hash():
    """Hash of the library's sources in the tree, computed as mpc-verde_amd/Makefile does
    (the sorted csrc/*.hip, csrc/capi.cpp, the sorted csrc/*.h, include/mpcx.h, then the Makefile
    for its compiler flags; sha256, 16 hex digits), or None
    when the sources are not next to the package (an installed copy)."""
    import glob
    import hashlib

    pkg = os.path.dirname(_HERE)
    files = sorted(glob.glob(os.path.join(pkg, "csrc", "*.hip")))
    files.append(os.path.join(pkg, "csrc", "capi.cpp"))
    files += sorted(glob.glob(os.path.join(pkg, "csrc", "*.h")))
    files.append(os.path.join(os.path.dirname(pkg), "include", "mpcx.h"))
    files.append(os.path.join(pkg, "Makefile"))
    if not all(os.path.exists(f) for f in files):
        return None
    h = hashlib.sha256()
    for f in files:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def load():
    """Load libmpcx.so (raises if it has not been built, or was built from other sources
    than the tree's -- a stale binary must not run as the product)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise MpcxError(f"{LIB_PATH} not found: build it with `make -C mpc-verde_amd` (hipcc, gfx950)")
    _bind_single_hip_runtime()
    lib = ctypes.CDLL(LIB_PATH)
    dp = ctypes.POINTER(ctypes.c_double)
    ip = ctypes.POINTER(ctypes.c_int32)
    vp = ctypes.c_void_p
    H = ctypes.c_void_p
    lib.mpcx_default_spec.argtypes = [ctypes.POINTER(Spec), ctypes.c_int32, ctypes.c_int32]
    lib.mpcx_create.argtypes = [ctypes.POINTER(Spec), ctypes.POINTER(H)]
    lib.mpcx_destroy.argtypes = [H]
    lib.mpcx_destroy.restype = None
    lib.mpcx_last_error.restype = ctypes.c_char_p
    lib.mpcx_dims.argtypes = [H, ip, ip, ip]
    lib.mpcx_launch_shape.argtypes = [H, ctypes.c_int32, ip, ip, ctypes.c_char_p, ctypes.c_int32]
    lib.mpcx_solve_batch.argtypes = [H, ctypes.c_int32, dp, dp, dp, dp, dp, dp, dp, dp, dp, dp, dp, ip, ip]
    lib.mpcx_solve_batch_dev.argtypes = [H, ctypes.c_int32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    lib.mpcx_plant_step.argtypes = [H, ctypes.c_int32, dp, dp, dp, dp]
    lib.mpcx_shift_dev.argtypes = [H, ctypes.c_int32, vp, vp, vp, vp, vp, vp, vp, vp]
    lib.mpcx_rk4_sens.argtypes = [H, ctypes.c_int32, dp, dp, dp, dp, dp, dp, dp]
    lib.mpcx_rk4_sens_dev.argtypes = [H, ctypes.c_int32, vp, vp, vp, vp, vp]
    lib.mpcx_set_linear_model.argtypes = [H, ctypes.c_int32, dp, dp, dp, dp, ip, ctypes.c_int32]
    lib.mpcx_set_linear_tab_dev.argtypes = [H, ctypes.c_void_p, ctypes.c_int32]
    lib.mpcx_step_dev.argtypes = [H, ctypes.c_int32, vp, vp, vp, vp, ctypes.c_int32, vp, vp, vp, vp, vp, vp, vp]
    lib.mpcx_run_dev.argtypes = [H, ctypes.c_int32, ctypes.c_int32, vp, vp, vp, vp, ctypes.c_int32, vp, vp, vp, vp, vp,
                                 vp, vp, vp, vp]
    for name in EXPORTS:
        getattr(lib, name)  # AttributeError if an export is missing
    lib.mpcx_source_hash.restype = ctypes.c_char_p
    built, tree = lib.mpcx_source_hash().decode(), source_hash()
    if tree is not None and built != tree and os.environ.get("MPCX_ALLOW_STALE_LIB") != "1":
        raise MpcxError(f"{LIB_PATH} was built from other sources (hash {built}) than the tree's ({tree}): "
                        "rebuild it with `make -C mpc-verde_amd`")
    _lib = lib
    return lib


def check(rc):
    if rc != 0:
        msg = load().mpcx_last_error().decode(errors="replace")
        raise MpcxError(f"mpcx error {rc}: {msg}")


def dptr(a):
    """double* of a C-contiguous float64 ndarray (or None)."""
    if a is None:
        return None
    if not isinstance(a, np.ndarray) or a.dtype != np.float64 or not a.flags["C_CONTIGUOUS"]:
        raise TypeError("expected a C-contiguous float64 ndarray")
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def iptr(a):
    if a is None:
        return None
    if not isinstance(a, np.ndarray) or a.dtype != np.int32 or not a.flags["C_CONTIGUOUS"]:
        raise TypeError("expected a C-contiguous int32 ndarray")
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))


class Handle:
    """Owning wrapper of an ``mpcx_handle*``."""

    def __init__(self, spec: Spec):
        lib = load()
        self._spec = spec
        self._h = ctypes.c_void_p()
        check(lib.mpcx_create(ctypes.byref(spec), ctypes.byref(self._h)))
        nw, ng, npar = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        check(lib.mpcx_dims(self._h, ctypes.byref(nw), ctypes.byref(ng), ctypes.byref(npar)))
        self.n_w, self.n_g, self.n_p = nw.value, ng.value, npar.value

    @property
    def ptr(self):
        return self._h

    def set_linear_model(self, lin):
        """Upload the stage tables of a LinearOCP (mpcx_set_linear_model)."""
        n_tab, A, B, c, Wp, tab, rows = lin.tables()
        A, B, c, Wp = (np.ascontiguousarray(v, np.float64) for v in (A, B, c, Wp))
        tab = np.ascontiguousarray(tab, np.int32)
        check(load().mpcx_set_linear_model(self._h, int(n_tab), dptr(A), dptr(B), dptr(c), dptr(Wp), iptr(tab),
                                           int(rows)))
        self._lin_refs = (A, B, c, Wp, tab)

    def launch_shape(self, B):
        """(lanes per group, replicas per wave, kernel name) of a B-instance solve launch
        (mpcx_launch_shape: the instantiation rocprofv3 will name)."""
        G, R = ctypes.c_int32(), ctypes.c_int32()
        buf = ctypes.create_string_buffer(256)
        check(load().mpcx_launch_shape(self._h, int(B), ctypes.byref(G), ctypes.byref(R), buf, len(buf)))
        return G.value, R.value, buf.value.decode()

    @property
    def spec(self):
        return self._spec

    def close(self):
        if self._h:
            load().mpcx_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
