"""rowchain.h -- the unicycle's backward Riccati recursion spread over 16-lane rows (the solve
kernel's chain for configs 1-2) -- against the sequential recursion it replaced (riccati_step on
node lane j, the value function moved lane to lane by DPP), through tests/hip/rowchain_check.hip:
bit for bit the same P_k, p_k and factors (r0, t, r1, h0, h1, g0, g1) at every node, for the
unicycle's Jacobian structure with random stage Hessians (indefinite reduced Huu' included),
random defects and terminal value functions, in the three lane-group shapes that run it (32-lane
groups two per wave, 32-lane groups replicated, one 64-lane group per wave), N from 1 to G - 1."""
import ctypes
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "hip", "librowchain_check.so")
K_IN, K_OUT = 47, 22


def stages(rng, B, G, scale):
    """Random unicycle stages: A = I + a02 e0 e2^T + a12 e1 e2^T, B with B[2][0] = 0, symmetric
    stage Hessians (some with an indefinite u block), barrier gradients, defects, and a terminal
    value function at every node (the kernel reads node N's only)."""
    x = np.zeros((B, G, K_IN))
    Hf = rng.standard_normal((B, G, 5, 5)) * scale[..., None, None]
    Hf = Hf @ np.swapaxes(Hf, -1, -2) + np.eye(5) * rng.uniform(0.0, 2.0, (B, G, 1, 1))
    Hf[:, ::7, 3:, 3:] -= 4.0 * np.eye(2)  # every 7th stage: an indefinite control block
    iu = [(i, j) for i in range(5) for j in range(i, 5)]
    x[..., 0:15] = np.stack([Hf[..., i, j] for i, j in iu], axis=-1)
    x[..., 15:20] = rng.standard_normal((B, G, 5)) * scale[..., None]
    A = np.broadcast_to(np.eye(3), (B, G, 3, 3)).copy()
    A[..., 0, 2], A[..., 1, 2] = rng.standard_normal((2, B, G)) * 0.2
    Bm = rng.standard_normal((B, G, 3, 2)) * 0.2
    Bm[..., 2, 0] = 0.0
    x[..., 20:29] = A.reshape(B, G, 9)
    x[..., 29:35] = Bm.reshape(B, G, 6)
    x[..., 35:38] = rng.standard_normal((B, G, 3)) * 1e-2
    Pf = rng.standard_normal((B, G, 3, 3))
    Pf = Pf @ np.swapaxes(Pf, -1, -2) + np.eye(3)
    x[..., 38:44] = np.stack([Pf[..., i, j] for i in range(3) for j in range(i, 3)], axis=-1)
    x[..., 44:47] = rng.standard_normal((B, G, 3))
    return x


@pytest.mark.parametrize("G,R,N", [(32, 1, 20), (32, 1, 1), (32, 1, 31), (32, 2, 20), (32, 2, 16),
                                   (64, 1, 10), (64, 1, 63)])
def test_row_chain_is_the_sequential_recursion(G, R, N):
    import torch

    if not os.path.exists(LIB):
        pytest.fail(f"{LIB} not built (make -C tests/hip)")
    lib = ctypes.CDLL(LIB)
    lib.rowchain_check.argtypes = [ctypes.c_int] * 4 + [ctypes.c_void_p] * 4
    B = 257 if R == 1 else 128  # an odd batch: the last wave's second 32-lane group is empty
    rng = np.random.default_rng(1000 * G + 10 * N + R)
    scale = np.exp(rng.uniform(-3, 3, (B, G)))  # magnitudes 1e-1 .. 1e1 per stage
    x = stages(rng, B, G, scale)
    d_in = torch.from_numpy(np.ascontiguousarray(x)).cuda()
    o_seq = torch.full((B, G, K_OUT), np.nan, dtype=torch.float64, device="cuda")
    o_row = torch.full_like(o_seq, np.nan)
    ptr = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    waves = (B * G * R + 63) // 64
    cyc = torch.zeros(2 * waves, dtype=torch.int64, device="cuda")
    assert lib.rowchain_check(G, R, N, B, ptr(d_in), ptr(o_seq), ptr(o_row), ptr(cyc)) == 0
    c = cyc.cpu().numpy().reshape(waves, 2)
    print(f"G={G} R={R} N={N}: cycles per step, sequential recursion {c[:, 0].mean() / N:.0f}, "
          f"row chain {c[:, 1].mean() / N:.0f}")
    a, b = o_seq.cpu().numpy()[:, :N + 1], o_row.cpu().numpy()[:, :N + 1]
    assert np.isfinite(a[:, :N, :20]).mean() > 0.5  # the recursion ran (indefinite stages may overflow)
    np.testing.assert_array_equal(b.view(np.int64), a.view(np.int64))
    # and it is a Riccati recursion: node N-1's P from the formula in numpy (rtol, not bits; node N-1
    # of N = 1 is a stage with an indefinite control block by construction)
    if (N - 1) % 7 == 0:
        return
    s = x[:, N - 1]
    Hf = np.zeros((B, 5, 5))
    for q, (i, j) in enumerate([(i, j) for i in range(5) for j in range(i, 5)]):
        Hf[:, i, j] = Hf[:, j, i] = s[:, q]
    A, Bm, c = s[:, 20:29].reshape(B, 3, 3), s[:, 29:35].reshape(B, 3, 2), s[:, 35:38]
    PN = np.zeros((B, 3, 3))
    for q, (i, j) in enumerate([(i, j) for i in range(3) for j in range(i, 3)]):
        PN[:, i, j] = PN[:, j, i] = x[:, N, 38 + q]
    W = np.concatenate([A, Bm], axis=2)
    Q = Hf + np.swapaxes(W, 1, 2) @ PN @ W
    Pk = Q[:, :3, :3] - Q[:, :3, 3:] @ np.linalg.solve(Q[:, 3:, 3:], Q[:, 3:, :3])
    got = np.stack([b[:, N - 1, q] for q in range(6)], axis=-1)
    want = np.stack([Pk[:, i, j] for i in range(3) for j in range(i, 3)], axis=-1)
    ok = np.all(np.linalg.eigvalsh(Q[:, 3:, 3:]) > 1e-6, axis=1)
    assert ok.sum() > B // 2
    np.testing.assert_allclose(got[ok], want[ok], rtol=1e-8, atol=1e-8 * np.abs(want[ok]).max())


# ---- rowchain6.h: the 6-state bicycle's chain (one instance per 64-lane wave, window by window)
K_IN6, K_OUT6, K_WS6 = 106, 44, 42
IU8 = [(i, j) for i in range(8) for j in range(i, 8)]


def stages6(rng, B, indefinite):
    """Random 6-state stages with the model's Jacobian structure (columns x0, x1 of A unit
    vectors, the rest dense; B dense), symmetric stage Hessians (with `indefinite`, every 7th stage
    from node 3 with an indefinite control block), Sigma, gradients and defects at all 64 nodes."""
    x = np.zeros((B, 64, K_IN6))
    Hf = rng.standard_normal((B, 64, 8, 8)) * 0.5
    Hf = Hf @ np.swapaxes(Hf, -1, -2) + np.eye(8) * rng.uniform(0.0, 2.0, (B, 64, 1, 1))
    if indefinite:
        Hf[:, 3::7, 6:, 6:] -= 6.0 * np.eye(2)
    x[..., 0:36] = np.stack([Hf[..., i, j] for i, j in IU8], axis=-1)
    x[..., 36:44] = rng.uniform(0.0, 1.0, (B, 64, 8))
    A = np.eye(6) + rng.standard_normal((B, 64, 6, 6)) * 0.2
    A[..., :, 0] = np.eye(6)[:, 0]
    A[..., :, 1] = np.eye(6)[:, 1]
    x[..., 44:80] = A.reshape(B, 64, 36)
    x[..., 80:92] = (rng.standard_normal((B, 64, 6, 2)) * 0.2).reshape(B, 64, 12)
    x[..., 92:100] = rng.standard_normal((B, 64, 8))
    x[..., 100:106] = rng.standard_normal((B, 64, 6)) * 1e-2
    return x


@pytest.mark.parametrize("N,delta,indef", [(50, 0.0, False), (50, 1e-4, False), (35, 0.0, False), (36, 0.0, False),
                                           (63, 0.0, False), (1, 0.0, False), (12, 3e-3, False), (50, 0.0, True),
                                           (20, 1e-4, True)])
def test_row_chain6_is_the_sequential_recursion(N, delta, indef):
    """Bit for bit the sequential recursion at every node; with indefinite stages the chain stops at
    the first step (from N - 1 down) whose factors fail the inertia test, exactly where the
    sequential recursion's verdict first fails, and nodes at and above it still match."""
    import torch

    if not os.path.exists(LIB):
        pytest.fail(f"{LIB} not built (make -C tests/hip)")
    lib = ctypes.CDLL(LIB)
    lib.rowchain6_check.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_double] + [ctypes.c_void_p] * 6
    B = 96
    rng = np.random.default_rng(7 * N + 1)
    x = stages6(rng, B, indef)
    d_in = torch.from_numpy(np.ascontiguousarray(x)).cuda()
    ws = torch.full((B, 64, K_WS6), np.nan, dtype=torch.float64, device="cuda")
    o_seq = torch.full((B, 64, K_OUT6), np.nan, dtype=torch.float64, device="cuda")
    o_row = torch.full_like(o_seq, np.nan)
    cyc = torch.zeros(2 * B, dtype=torch.int64, device="cuda")
    early = torch.full((B,), -1, dtype=torch.int32, device="cuda")
    ptr = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    assert lib.rowchain6_check(N, B, delta, ptr(d_in), ptr(ws), ptr(o_seq), ptr(o_row), ptr(cyc), ptr(early)) == 0
    c = cyc.cpu().numpy().reshape(B, 2)
    print(f"N={N}: cycles per step, sequential recursion {c[:, 0].mean() / N:.0f}, row chain {c[:, 1].mean() / N:.0f}")
    a, b = o_seq.cpu().numpy()[:, :N + 1], o_row.cpu().numpy()[:, :N + 1]
    r0, r1 = a[:, :N, 27], a[:, :N, 29]
    with np.errstate(invalid="ignore"):
        bad = ~((r0 > 0) & (r0 < np.inf) & (r1 > 0) & (r1 < np.inf))  # fac_ok false, node by node
    first = np.where(bad.any(axis=1), N - 1 - np.argmax(bad[:, ::-1], axis=1), -1)  # first failure from N - 1 down
    np.testing.assert_array_equal(early.cpu().numpy(), (first >= 0).astype(np.int32))
    if indef:
        assert (first >= 0).mean() > 0.5
    else:
        assert (first < 0).all()
    for i in range(B):  # nodes the chain reached (all of them when it ran to node 0)
        lo = max(first[i], 0)
        np.testing.assert_array_equal(b[i, lo:].view(np.int64), a[i, lo:].view(np.int64))
    # a Riccati recursion: node N-1's P_{N-1} from the formula
    if indef:
        return
    s = x[:, N - 1]
    Hf = np.zeros((B, 8, 8))
    for q, (i, j) in enumerate(IU8):
        Hf[:, i, j] = Hf[:, j, i] = s[:, q]
    Hf += np.einsum("bi,ij->bij", s[:, 36:44] + delta, np.eye(8))
    A, Bm = s[:, 44:80].reshape(B, 6, 6), s[:, 80:92].reshape(B, 6, 2)
    PN = np.einsum("bi,ij->bij", x[:, N, 36:42] + delta, np.eye(6))
    W = np.concatenate([A, Bm], axis=2)
    Q = Hf + np.swapaxes(W, 1, 2) @ PN @ W
    Pk = Q[:, :6, :6] - Q[:, :6, 6:] @ np.linalg.solve(Q[:, 6:, 6:], Q[:, 6:, :6])
    got = np.stack([b[:, N - 1, q] for q in range(21)], axis=-1)
    want = np.stack([Pk[:, i, j] for i in range(6) for j in range(i, 6)], axis=-1)
    np.testing.assert_allclose(got, want, rtol=1e-8, atol=1e-8 * np.abs(want).max())
