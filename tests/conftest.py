"""Shared test setup.

`-m "not gpu"` tests run here (no GPU): the oracle against fixtures, host logic, the
C ABI library's exports.  `-m gpu` tests are the parity tests proper: the HIP engine
through the C ABI against the CPU oracle, bit for bit.
"""
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "acmmp-spherical_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")
    config.addinivalue_line("markers", "slow: takes more than ~20 s")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def gpu_ctx_factory():
    from acmmp import capi
    capi.load_library()

    def make():
        return capi.Context(0)
    return make


def canon_bits(a):
    """Bit pattern with every NaN canonicalised (NaN payloads differ between x86 and gfx950)."""
    a = np.asarray(a)
    if a.dtype == np.float32:
        b = a.view(np.uint32).copy()
        b[np.isnan(a)] = 0x7FC00000
        return b
    return a


def assert_bitwise_equal(got, want, what=""):
    g, w = canon_bits(got), canon_bits(want)
    assert g.shape == w.shape, f"{what}: shape {g.shape} != {w.shape}"
    bad = np.argwhere(g != w)
    assert bad.size == 0, (f"{what}: {len(bad)} of {g.size} elements differ, first at {bad[:5].tolist()}: "
                           f"got {np.asarray(got)[tuple(bad[0])]!r} want {np.asarray(want)[tuple(bad[0])]!r}")
