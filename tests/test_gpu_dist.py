"""GPU: the collectives of the multi-GPU path through RCCL itself.

A one-GPU box cannot run two RCCL ranks (RCCL wants a device per rank; the N-rank curve is the
driver's 8-GPU run), so the backend is exercised at world size 1: the "nccl" process group on a
TCP store on loopback, created before any other HIP use, and the bench's stats all_gather and
max-over-ranks on cuda tensors (mpcx/dist.py), checked against the numpy values."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_rccl_world1_stats_collectives():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "helpers", "rccl_world1.py")],
                         capture_output=True, text=True, timeout=300, env=dict(os.environ))
    assert out.returncode == 0, out.stderr[-3000:]
    d = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
    print(d)
    assert d["backend"] == "nccl" and d["world"] == 1 and d["max_over_ranks"] == 3.25
