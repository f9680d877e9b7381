"""CPU: the C-ABI library loads and exports every symbol include/mpcx.h declares;
host-side logic of the façade; the product never imports the oracle."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "mpc-verde_amd", "mpcx", "libmpcx.so")
HDR = os.path.join(ROOT, "include", "mpcx.h")


def declared_symbols():
    src = open(HDR).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char\*)\s+(mpcx_\w+)\s*\(", src, re.M)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-C", os.path.join(ROOT, "mpc-verde_amd")], check=True)
    return ctypes.CDLL(LIB)


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for s in ("mpcx_create", "mpcx_solve_batch", "mpcx_solve_batch_dev", "mpcx_plant_step", "mpcx_rk4_sens",
              "mpcx_destroy", "mpcx_last_error"):
        assert s in syms


def test_library_exports_every_declared_symbol(lib):
    for s in declared_symbols():
        assert hasattr(lib, s), s
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    for s in declared_symbols():
        assert re.search(rf"\bT {s}$", out, re.M), s


def test_library_matches_tree_sources(lib, monkeypatch):
    """The built library embeds the hash of the sources it was compiled from; the loader
    refuses one whose hash differs from the tree's (a stale .so must not run as the product)."""
    from mpcx import _lib

    lib.mpcx_source_hash.restype = ctypes.c_char_p
    assert lib.mpcx_source_hash().decode() == _lib.source_hash()
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "source_hash", lambda: "0000000000000000")
    monkeypatch.setattr(_lib, "_bind_single_hip_runtime", lambda: None)
    with pytest.raises(_lib.MpcxError, match="other sources"):
        _lib.load()


def test_library_targets_gfx950():
    """The shared library embeds a gfx950 code object (HIP fat binary)."""
    data = open(LIB, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data or b"gfx950" in data


def test_python_binding_matches_header():
    import mpcx

    assert set(mpcx._lib.EXPORTS) == set(declared_symbols())
    # struct layout: 8 int32 + 2 double + 6 x double[8] + 3 double (warm start) + 2 int32 (nx, nu)
    # + double[8] (par) + 8 double (IPOPT tolerances) + 2 int32 (acceptable_iter, no_restoration)
    assert ctypes.sizeof(mpcx._lib.Spec) == 8 * 4 + 2 * 8 + 6 * 8 * 8 + 3 * 8 + 2 * 4 + 8 * 8 + 8 * 8 + 2 * 4


def test_default_spec_without_gpu(lib):
    import mpcx

    s = mpcx._lib.Spec()
    assert lib.mpcx_default_spec(ctypes.byref(s), 1, 20) == 0
    assert s.N == 20 and s.M == 4 and abs(s.T - 0.2) < 1e-15 and s.max_iter == 2000
    assert list(s.Q[:3]) == [1.0, 5.0, 0.1] and list(s.R[:2]) == [0.5, 0.05]
    # the reference's IPOPT options (Casadi/multiple_shooting_casadi.py:190-193), IPOPT's defaults otherwise
    assert (s.acceptable_tol, s.acceptable_obj_change_tol, s.acceptable_iter) == (1e-8, 1e-6, 15)
    assert (s.dual_inf_tol, s.constr_viol_tol, s.compl_inf_tol, s.no_restoration) == (1.0, 1e-4, 1e-4, 0)
    assert lib.mpcx_default_spec(ctypes.byref(s), 99, 20) < 0
    # ODE models: dimensions, node cost and constants (include/mpcx.h mpcx_model)
    for model, nx, nu, par in ((3, 3, 2, [0.5]), (4, 6, 2, [1200.0, 1.5, 2.0, 55000.0, 1350.0]),
                               (5, 4, 1, [1.0, 1.0, 0.5, 9.81, 10.0])):
        assert lib.mpcx_default_spec(ctypes.byref(s), model, 30) == 0
        assert (s.nx, s.nu, s.cost, s.N) == (nx, nu, 1, 30)
        assert list(s.par[:len(par)]) == par


def test_no_cpu_fallback_when_gpu_missing():
    """The product path fails loudly without a HIP device (no silent CPU path)."""
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    import mpcx

    with pytest.raises(mpcx._lib.MpcxError):
        mpcx.nlpsol("s", "mi355x", mpcx.unicycle_point_to_point(N=10))


def test_to_spec_mirrors_reference_constants():
    import mpcx

    s = mpcx.to_spec(mpcx.unicycle_point_to_point(N=20))
    assert (s.N, s.M, s.cost, s.param_layout) == (20, 4, 0, 0)
    assert s.lbu[0] == -1.0 and s.ubu[1] == pytest.approx(np.pi / 4)
    assert s.lbx[0] == -1e20 and s.ubx[2] == 1e20
    t = mpcx.to_spec(mpcx.unicycle_tracking(N=30))
    assert (t.N, t.M, t.cost, t.param_layout) == (30, 1, 1, 1)
    assert (t.lbx[0], t.ubx[0], t.lbx[1], t.ubx[1]) == (-20.0, 20.0, -2.0, 2.0)


def test_to_spec_ipopt_option_mappings():
    """The spec reads a 0 field as IPOPT's default (include/mpcx.h, capi.cpp solve args), so the
    Python side maps IPOPT's literal values onto the spec: acceptable_obj_change_tol = 0 (the
    objective must not change at all) -> 5e-324, acceptable_iter = 0 (heuristic off) -> -1;
    left out, every option carries IPOPT's default explicitly."""
    import mpcx
    from mpcx.ocp import IPOPT_DEFAULTS

    ocp = mpcx.unicycle_point_to_point(N=20)
    s = mpcx.to_spec(ocp)
    for k, v in IPOPT_DEFAULTS.items():
        assert getattr(s, k) == v, k
    z = mpcx.to_spec(ocp, ipopt={"acceptable_obj_change_tol": 0.0, "acceptable_iter": 0})
    assert z.acceptable_obj_change_tol == 5e-324 and z.acceptable_obj_change_tol > 0.0
    assert z.acceptable_iter == -1
    r = mpcx.to_spec(ocp, ipopt={"acceptable_tol": 1e-8, "acceptable_obj_change_tol": 1e-6})
    assert (r.acceptable_tol, r.acceptable_obj_change_tol) == (1e-8, 1e-6)
    with pytest.raises(ValueError):
        mpcx.to_spec(ocp, ipopt={"no_such_option": 1.0})


def test_vec_coercion():
    from mpcx.nlpsol import _vec

    assert np.array_equal(_vec(3.0, 4, "a"), np.full(4, 3.0))
    assert np.array_equal(_vec([[1], [2]], 2, "a"), np.array([1.0, 2.0]))
    with pytest.raises(ValueError):
        _vec([1, 2, 3], 2, "a")


def test_product_does_not_import_oracle():
    pkg = os.path.join(ROOT, "mpc-verde_amd")
    for dp, _, fs in os.walk(pkg):
        for f in fs:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                src = open(os.path.join(dp, f)).read()
                assert not re.search(r"^\s*(from|import)\s+oracle", src, re.M), f
                assert "ipm_ref" not in src and "nlp_ref" not in src, f


def test_shift_matches_reference_receding_horizon():
    """bench.shift_np == shift_kernel semantics: X_k <- X_{k+1}, U_k <- U_{k+1}, tail repeated
    (Casadi/multiple_shooting_casadi.py:274-283, interleaved layout)."""
    import bench
    from oracle import nlp_ref

    N = 4
    rng = np.random.default_rng(0)
    X = rng.normal(size=(2, N + 1, 3))
    U = rng.normal(size=(2, N, 2))
    w0 = bench.shift_np(nlp_ref.join_w(X, U), N)
    X2, U2 = nlp_ref.split_w(w0, N)
    assert np.array_equal(X2[:, :N], X[:, 1:]) and np.array_equal(X2[:, N], X[:, N])
    assert np.array_equal(U2[:, :N - 1], U[:, 1:]) and np.array_equal(U2[:, N - 1], U[:, N - 1])


def test_filter_harness_builds_and_exports():
    """tests/hip/libfilter_check.so (the filter's device harness, tests/test_gpu_filter.py) is
    built from the product's kernels.h and exports its two entry points; capacity >= 256."""
    import subprocess

    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "hip")
    subprocess.run(["make", "-C", here], check=True, capture_output=True)
    lib = ctypes.CDLL(os.path.join(here, "libfilter_check.so"))
    assert hasattr(lib, "filter_check")
    for G in (16, 32, 64, 128, 256):
        assert lib.filter_check_capacity(G) >= 256
    assert lib.filter_check_capacity(8) == -1


def test_bench_usable_cpus():
    """bench.py's CPU count for the baseline is every CPU the process may run on (affinity mask,
    capped by a cgroup quota), never OMP_NUM_THREADS.  (The solve kernel whose PMC record the
    roofline uses is named by the library itself, mpcx_launch_shape: tests/test_gpu_parity.py.)"""
    import importlib.util

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    old = os.environ.get("OMP_NUM_THREADS")
    os.environ["OMP_NUM_THREADS"] = "1"
    try:
        n = bench.usable_cpus()
    finally:
        if old is None:
            del os.environ["OMP_NUM_THREADS"]
        else:
            os.environ["OMP_NUM_THREADS"] = old
    assert 1 <= n <= len(os.sched_getaffinity(0)) <= (os.cpu_count() or 1)


def test_bench_solve_roofline_uses_only_a_current_pmc_record(tmp_path, monkeypatch):
    """bench.py's solve-kernel roofline: achieved = algorithmic flops of the launch / its time,
    frac against the FP64 vector peak; the issued PMC figures and the issue share of wave cycles
    sit beside it only when the committed record was measured on this tree's sources, and a stale
    record is named, never used."""
    import importlib.util
    import json

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod2", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    from mpcx import _lib

    kname = "void mpcx::solve_kernel<mpcx::UnicycleFreeModel, 32, false, 2>(mpcx::SolveArgs)"
    rec = {kname: {"f64_lane_flops_per_group_iteration": 400000.0,
                   "wave_cycles_share": {"issuing": 0.8, "dependency_or_pipe_stall": 0.02, "waitcnt_or_barrier": 0.18},
                   "valu_active_share": 0.7}}
    algo = {"per_iteration": 40000.0, "per_node": {}, "eval_source": "e", "riccati_source": "r"}
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    os.makedirs(tmp_path / os.path.dirname(bench.SOLVE_PMC), exist_ok=True)
    for current in (True, False):
        meta = {"mpcx_source_hash": _lib.source_hash() if current else "0000000000000000"}
        with open(tmp_path / bench.SOLVE_PMC, "w") as f:
            json.dump({"_meta": meta, **rec}, f)
        r = bench.solve_roofline(kname, algo, 100000, 2.0)  # 4e9 flops in 2 ms
        assert r["achieved"] == pytest.approx(2.0) and r["frac"] == pytest.approx(2.0 / bench.PEAK_FP64_TFLOPS, abs=1e-5)
        if current:
            assert r["issued"]["algorithmic_over_issued"] == pytest.approx(0.1)
            assert r["issue"]["issuing_share_of_wave_cycles"] == 0.8
        else:
            assert isinstance(r["issued"], str) and r["issued"].startswith("stale") and "issue" not in r
    # roofline.traffic: the counter-measured HBM bytes of the timed launch, only from a record of
    # this tree's sources and this kernel (tools/solve_traffic.py)
    for src, kern, want in ((_lib.source_hash(), kname, 7.5e6), ("0000000000000000", kname, None),
                            (_lib.source_hash(), "other", None)):
        with open(tmp_path / "profiles" / bench.SOLVE_TRAFFIC, "w") as f:
            json.dump({"kernel": kern, "hbm_bytes_per_launch": 7.5e6, "mpcx_source_hash": src}, f)
        r = bench.solve_roofline(kname, algo, 100000, 2.0)
        assert r["traffic"] == want
        assert (want is None) == ("traffic_note" in r)
