"""The solve kernel's filter (mpc-verde_amd/csrc/kernels.h FilterLds) against IPOPT's unbounded
filter (W&B 2006 §2.4; IPOPT Filter::AddEntry drops the entries a new one dominates), through the
device harness tests/hip/filter_check.hip, which calls FilterLds exactly as the solve loop does
(membership test of a trial point, then an addition).

* Random sequences far longer than the S x G slots (so the full-filter path -- drop dominated
  entries, take the lowest free slot -- runs many times): every membership answer equals the
  unbounded filter's, and no addition overflows, for every group size.
* A sequence of mutually non-dominated entries longer than the slots: answers equal the unbounded
  filter's until the slots are exhausted; from the first surplus entry on, add() reports the
  overflow (the diagnostic build's DIAG 14) -- the only case where the two can differ.
"""
import ctypes
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "hip", "libfilter_check.so")


class RefFilter:
    """IPOPT's filter: a list of (theta, phi) corners; (t, p) is rejected if t >= th and p >= ph
    for some entry; adding drops the entries the new one dominates."""

    def __init__(self):
        self.e = []

    def contains(self, t, p):
        return any(t >= a and p >= b for a, b in self.e)

    def add(self, t, p):
        self.e = [(a, b) for a, b in self.e if not (a >= t and b >= p)]
        self.e.append((t, p))


@pytest.fixture(scope="module")
def harness():
    import torch

    if not os.path.exists(LIB):
        pytest.fail(f"{LIB} not built (make -C tests/hip)")
    lib = ctypes.CDLL(LIB)
    lib.filter_check.argtypes = [ctypes.c_int] * 3 + [ctypes.c_void_p] * 6
    return lib, torch


def run(harness, G, th, ph, qth, qph):
    lib, torch = harness
    groups, n = th.shape
    d = [torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).cuda() for a in (th, ph, qth, qph)]
    cov = torch.zeros((groups, n), dtype=torch.int32, device="cuda")
    ovf = torch.zeros((groups, n), dtype=torch.int32, device="cuda")
    ptr = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    assert lib.filter_check(G, groups, n, *[ptr(t) for t in d], ptr(cov), ptr(ovf)) == 0
    return cov.cpu().numpy().astype(bool), ovf.cpu().numpy().astype(bool)


def reference(th, ph, qth, qph):
    cov = np.zeros(th.shape, bool)
    for g in range(th.shape[0]):
        f = RefFilter()
        for i in range(th.shape[1]):
            cov[g, i] = f.contains(qth[g, i], qph[g, i])
            f.add(th[g, i], ph[g, i])
    return cov


@pytest.mark.parametrize("G", [16, 32, 64, 128, 256])
def test_filter_matches_unbounded_ipopt_filter(harness, G):
    lib, _ = harness
    cap = lib.filter_check_capacity(G)
    assert cap >= 256
    rng = np.random.default_rng(G)
    groups, n = 4, 3 * cap
    # rounds of F mutually non-dominated entries (an anti-diagonal with jitter, up to 0.6 of the
    # slots: several slot rows in use) closed by an entry that dominates them all, at a shrinking
    # scale -- a filter that grows and collapses as in a long solve; queries near the entries,
    # ties included (equal coordinates are "in the filter")
    F = int(0.6 * cap)
    th = np.empty((groups, n))
    ph = np.empty((groups, n))
    for g in range(groups):
        scale, i = 1e3, 0
        while i < n:
            m = min(F, n - i)
            u = np.sort(rng.uniform(0, 1, m))
            th[g, i:i + m] = scale * (1 + u)
            ph[g, i:i + m] = scale * (2 - u)
            i += m
            if i < n:
                th[g, i], ph[g, i] = 0.5 * scale, 0.5 * scale
                i += 1
            scale *= 0.4
    qth = th * rng.uniform(0.98, 1.02, (groups, n))
    qph = np.roll(ph, 3, axis=1) * rng.uniform(0.98, 1.02, (groups, n))
    qth[:, ::7] = th[:, ::7]
    qph[:, ::7] = ph[:, ::7]
    cov, ovf = run(harness, G, th, ph, qth, qph)
    ref = reference(th, ph, qth, qph)
    assert not ovf.any()
    assert ref.any() and (~ref).any()
    np.testing.assert_array_equal(cov, ref)


@pytest.mark.parametrize("G", [16, 64, 128])
def test_filter_overflow_only_beyond_capacity(harness, G):
    lib, _ = harness
    cap = lib.filter_check_capacity(G)
    n = cap + 16
    i = np.arange(n, dtype=np.float64)
    th = (n - i)[None, :]          # theta decreasing, phi increasing: no entry dominates another
    ph = i[None, :].copy()
    # even steps: on the previous corner's theta, above its phi (in the filter); odd steps: a
    # point better than every entry (not in the filter)
    qth = np.roll(th, 1, axis=1)
    qph = np.roll(ph, 1, axis=1) + 0.5
    qth[:, 1::2], qph[:, 1::2] = 0.1, -1.0
    cov, ovf = run(harness, G, th, ph, qth, qph)
    ref = reference(th, ph, qth, qph)
    assert not ovf[0, :cap].any() and ovf[0, cap:].all()
    assert ref[0, 2::2].all() and not ref[0, 1::2].any()
    np.testing.assert_array_equal(cov[0, :cap + 1], ref[0, :cap + 1])
