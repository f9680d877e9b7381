"""collectives.h matvec_bcast -- the config-5 suffix scan's mat-vec by v_fmac_f64 with a DPP
row_newbcast source (kernels.h, the reused suffix's radix-4 scan) -- against the plain fma loop
over the same matrix read from memory, through tests/hip/bcast_check.hip: bit for bit equal for
NX = 4 and 5 (the linear models that run the scan), with a different matrix per wave and a
different vector and accumulator per lane, including signed zeros, tiny and huge values."""
import ctypes
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "hip", "libbcast_check.so")


@pytest.mark.parametrize("nx", [4, 5])
def test_row_broadcast_matvec_is_the_fma_loop(nx):
    import torch

    if not os.path.exists(LIB):
        pytest.fail(f"{LIB} not built (make -C tests/hip)")
    lib = ctypes.CDLL(LIB)
    lib.bcast_check.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 5
    waves = 64
    rng = np.random.default_rng(nx)
    M = rng.standard_normal((waves, nx, nx)) * np.exp(rng.uniform(-20, 20, (waves, nx, nx)))
    M[0] = 0.0
    M[1, 0, 0] = -0.0
    w = rng.standard_normal((waves * 64, nx)) * np.exp(rng.uniform(-20, 20, (waves * 64, nx)))
    w[5] = -0.0
    acc = rng.standard_normal((waves * 64, nx))
    acc[7] = -0.0
    d = [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (M, w, acc)]
    ob = torch.zeros((waves * 64, nx), dtype=torch.float64, device="cuda")
    op = torch.zeros_like(ob)
    ptr = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    assert lib.bcast_check(nx, waves, *[ptr(t) for t in d], ptr(ob), ptr(op)) == 0
    got, want = ob.cpu().numpy(), op.cpu().numpy()
    np.testing.assert_array_equal(got.view(np.int64), want.view(np.int64))
    # and the plain loop is what numpy's fma-free product approximates (the harness really ran)
    ref = acc + np.einsum("wij,wlj->wli", M, w.reshape(waves, 64, nx)).reshape(-1, nx)
    assert np.allclose(want, ref, rtol=1e-9, atol=1e-300 + 1e-12 * np.abs(ref).max())
