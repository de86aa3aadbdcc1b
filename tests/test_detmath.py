"""Accuracy and special cases of the deterministic elementary functions.

The oracle and the kernels share these definitions (each in its own file); here the
oracle's build is checked against float64 numpy, so the definitions are known to be
accurate approximations of the reference's expf/sinf/asinf/atan2f/acosf/rsqrtf.
"""
import numpy as np
import pytest


def ulp_err(got, want64):
    got = np.asarray(got, np.float64)
    want32 = want64.astype(np.float32)
    spacing = np.spacing(np.abs(want32)).astype(np.float64)
    spacing[spacing == 0] = np.finfo(np.float32).tiny
    return np.abs(got - want64) / spacing


@pytest.mark.parametrize("fn,np_fn,lo,hi,max_ulp", [
    ("exp", np.exp, -87.0, 88.0, 2.0),
    ("sin", np.sin, -12.0, 12.0, 2.0),
    ("cos", np.cos, -12.0, 12.0, 2.0),
    ("asin", np.arcsin, -1.0, 1.0, 2.5),
    ("acos", np.arccos, -1.0, 1.0, 2.5),
])
def test_unary_accuracy(oracle_mod, fn, np_fn, lo, hi, max_ulp):
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.uniform(lo, hi, 200_000), np.linspace(lo, hi, 20_001)]).astype(np.float32)
    got = oracle_mod.detmath(fn, x)
    want = np_fn(x.astype(np.float64))
    if fn in ("sin", "cos"):
        # absolute error near zeros of sin/cos is the meaningful bound there
        err = np.abs(got - want)
        assert err.max() < 2.5e-7
    else:
        assert ulp_err(got, want).max() <= max_ulp


def test_atan2_accuracy(oracle_mod):
    rng = np.random.default_rng(1)
    y = rng.normal(size=300_000).astype(np.float32)
    x = rng.normal(size=300_000).astype(np.float32)
    got = oracle_mod.detmath("atan2", y, x)
    want = np.arctan2(y.astype(np.float64), x.astype(np.float64))
    assert ulp_err(got, want).max() <= 3.0


def test_special_cases(oracle_mod):
    d = oracle_mod.detmath
    nan = np.float32(np.nan)
    assert np.isnan(d("exp", [nan]))[0] and d("exp", [np.float32(100)])[0] == np.inf
    assert d("exp", [np.float32(-200)])[0] == 0.0 and d("exp", [np.float32(0)])[0] == 1.0
    assert np.isnan(d("asin", [np.float32(1.0000001)]))[0] and np.isnan(d("acos", [np.float32(-1.5)]))[0]
    assert d("acos", [np.float32(1.0)])[0] == 0.0
    # C99 atan2 zero / sign rules
    pz, nz = np.float32(0.0), np.float32(-0.0)
    assert d("atan2", [pz], [pz])[0] == 0.0 and not np.signbit(d("atan2", [pz], [pz])[0])
    assert np.signbit(d("atan2", [nz], [pz])[0])
    assert abs(d("atan2", [pz], [nz])[0] - np.pi) < 1e-6
    assert abs(d("atan2", [np.float32(1)], [pz])[0] - np.pi / 2) < 1e-6
    assert np.isnan(d("atan2", [nan], [np.float32(1)])[0])
    assert d("rsqrt", [np.float32(4.0)])[0] == 0.5
    # float -> int: truncation, saturation, NaN -> 0 (cvt.rzi.s32.f32 / v_cvt_i32_f32)
    f2i = d("f2i_sat", np.array([-3.7, 3.7, np.nan, 3e9, -3e9], np.float32))
    assert f2i.tolist() == [-3.0, 3.0, 0.0, 2147483648.0, -2147483648.0]
