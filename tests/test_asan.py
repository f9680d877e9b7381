"""Sanitizer runs of the host code (CPU; GPU sanitizers are not available on this pool).

* libmpcx's C ABI argument checking (mpc-verde_amd/csrc/capi.cpp) built with AddressSanitizer
  and UndefinedBehaviorSanitizer on the host side (tests/asan/Makefile), driven through every
  entry point's failure paths and every invalid spec kind (tests/asan/capi_validation.cpp).
* The C++ CPU oracle (oracle/ipm_ref.cpp, the checker of every parity test and the timed
  cpu_baseline) built with the same sanitizers (tests/asan/Makefile) and loaded in place of the
  regular build (ORACLE_LIB) by the CPU test files that exercise it: the IPOPT restatement on
  every model, restoration, warm starts, the world-size-2 sharded loop, the linear/ODE checks.
Both must run clean: any sanitizer report aborts the process (-fno-sanitize-recover=all).
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _runtime(name):
    p = subprocess.run(["g++", f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()
    assert os.path.isabs(p) and os.path.exists(p), f"{name} not found"
    return p


def test_capi_validation_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "mpc-verde_amd")], check=True)
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "asan")], check=True)
    r = subprocess.run([os.path.join(ROOT, "tests", "asan", "capi_asan")], capture_output=True, text=True,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1"), timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "capi validation clean (0 failures)" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr


def test_oracle_cpu_suite_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "asan"), "libipm_ref_asan.so"], check=True)
    lib = os.path.join(ROOT, "tests", "asan", "libipm_ref_asan.so")
    env = dict(os.environ, LD_PRELOAD=f"{_runtime('libasan.so')} {_runtime('libubsan.so')}",
               ASAN_OPTIONS="detect_leaks=0", ORACLE_LIB=lib, OMP_NUM_THREADS="4")
    # the sanitized oracle is the one loaded
    probe = ("import sys; sys.path.insert(0, %r); from oracle import ipm_ref; ipm_ref.lib(); "
             "print(any('libipm_ref_asan.so' in l for l in open('/proc/self/maps')))" % ROOT)
    r = subprocess.run([sys.executable, "-c", probe], capture_output=True, text=True, env=env, cwd=ROOT, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "True", r.stdout + r.stderr
    files = ["tests/test_oracle.py", "tests/test_dist.py", "tests/test_linear_cpu.py", "tests/test_ode_cpu.py"]
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-m", "not gpu", "-p", "no:cacheprovider"] + files,
                       capture_output=True, text=True, env=env, cwd=ROOT, timeout=1500)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "AddressSanitizer" not in r.stdout + r.stderr and "runtime error" not in r.stdout + r.stderr
