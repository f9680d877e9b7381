"""CPU check of the log-depth Riccati scan algebra (mpc-verde_amd/csrc/pscan.h).

The kernel replaces the sequential backward Riccati recursion of the barrier KKT system
(riccati.h) by a Hillis-Steele suffix scan over conditional value-function elements
(A, b, C, J, p).  This restates the element construction, the combination rule and the scan
order of pscan.h in numpy and checks that they reproduce the sequential recursion's value
functions (P_k, p_k) -- including stages with indefinite state Hessians, as the exact
Lagrangian Hessian of the nonlinear models produces -- for the model shapes the kernel enables
(nx, nu) = (3, 2), (4, 1) and the others it is written for.
"""
import numpy as np
import pytest


def sequential(st, PN, pN, nx):
    """riccati.h riccati_step, node N-1 .. 0."""
    P, p = PN, pN
    out = [None] * len(st) + [(PN, pN)]
    for k in range(len(st) - 1, -1, -1):
        A, B, c, H, g = st[k]
        Hxx = H[:nx, :nx] + A.T @ P @ A
        Hux = H[nx:, :nx] + B.T @ P @ A
        Huu = H[nx:, nx:] + B.T @ P @ B
        s = p + P @ c
        gx, gu = g[:nx] + A.T @ s, g[nx:] + B.T @ s
        P = Hxx - Hux.T @ np.linalg.solve(Huu, Hux)
        p = gx - Hux.T @ np.linalg.solve(Huu, gu)
        out[k] = (P, p)
    return out


def element(stage, nx):
    """pscan.h relem_stage: eliminate u from the stage."""
    F, L, c, H, g = stage
    Q, S, R, q, r = H[:nx, :nx], H[:nx, nx:], H[nx:, nx:], g[:nx], g[nx:]
    Ri = np.linalg.inv(R)
    return [F - L @ Ri @ S.T, c - L @ Ri @ r, L @ Ri @ L.T, Q - S @ Ri @ S.T, q - S @ Ri @ r]


def combine(e1, e2):
    """pscan.h relem_combine_lds: e1 (i->j) (x) e2 (j->k)."""
    A1, b1, C1, J1, p1 = e1
    A2, b2, C2, J2, p2 = e2
    Mi = np.linalg.inv(np.eye(len(b1)) + C1 @ J2)
    T1, T2 = A2 @ Mi, Mi @ A1
    return [T1 @ A1, T1 @ (b1 - C1 @ p2) + b2, T1 @ C1 @ A2.T + C2, T2.T @ J2 @ A1 + J1, T2.T @ (p2 + J2 @ b1) + p1]


def scan(st, PN, pN, nx, G):
    N = len(st)
    z = np.zeros((nx, nx))
    E = [element(s, nx) for s in st] + [[z, np.zeros(nx), z, PN, pN]]
    E += [[np.eye(nx), np.zeros(nx), z, z, np.zeros(nx)]] * (G - N - 1)  # identity past node N
    d = 1
    while d < G and d <= N:  # solver.hip: for (d = 1; d < G && d <= N; d <<= 1)
        E = [combine(E[k], E[k + d]) if k + d < G else E[k] for k in range(G)]
        d *= 2
    return [(E[k][3], E[k][4]) for k in range(N + 1)]


def problem(rng, N, nx, nu, indefinite):
    st = []
    for _ in range(N):
        M = rng.normal(size=(nx + nu, nx + nu))
        H = M @ M.T + 0.1 * np.eye(nx + nu)
        if indefinite:
            H[:nx, :nx] -= 2.0 * np.eye(nx)
        st.append((np.eye(nx) + 0.1 * rng.normal(size=(nx, nx)), rng.normal(size=(nx, nu)), rng.normal(size=nx), H,
                   rng.normal(size=nx + nu)))
    M = rng.normal(size=(nx, nx))
    return st, M @ M.T + 0.1 * np.eye(nx), rng.normal(size=nx)


@pytest.mark.parametrize("N,nx,nu,indefinite", [(20, 3, 2, False), (20, 3, 2, True), (50, 4, 1, False),
                                                (100, 4, 1, False), (100, 5, 1, False), (30, 6, 2, False),
                                                (1, 3, 2, False), (63, 4, 1, True)])
def test_scan_equals_sequential_riccati(N, nx, nu, indefinite):
    rng = np.random.default_rng(N * 10 + nx)
    st, PN, pN = problem(rng, N, nx, nu, indefinite)
    G = 1 << int(np.ceil(np.log2(N + 1)))
    ref, got = sequential(st, PN, pN, nx), scan(st, PN, pN, nx, max(G, 16))
    for k in range(N + 1):
        scale = max(1.0, np.abs(ref[k][0]).max())
        assert np.abs(got[k][0] - ref[k][0]).max() <= 1e-9 * scale, k
        assert np.abs(got[k][1] - ref[k][1]).max() <= 1e-9 * max(1.0, np.abs(ref[k][1]).max()), k
