"""Fast-math engine mode (acmmp_set_math 'fast') -- tolerance parity, SURVEY.md §8c.

The fast mode changes only the NCC's per-sample projection arithmetic (hardware rsq / sqrt / rcp,
shorter atan polynomial, the translation folded into the rotation), as the reference's own
--use_fast_math build does (CMakeLists.txt:42).  It cannot be bit-identical to the oracle, so it is
held to tolerances:

  T1  NCC queries: the same {valid, 2.0} classification as the exact mode; the fast mode's distance
      to a float64 restatement of ComputeBilateralNCC (np_reference.py) no larger than the exact
      mode's own float32 distance to it, + 1e-4, at the median and the 99th percentile.
      (|fast - exact| <= 1e-4 holds for >= 99.5% of pinhole queries and <= 1e-3 for all; SPHERE patches, whose
      bilateral weights leave few effective samples, amplify last-bit differences to ~1e-3 -- the
      same size as the exact float32 path's own distance to float64.)
  T2  winners: after RandomInitialization every plane is identical (same RNG draws) and >= 99.5% of
      costs agree within 1e-3; after one black half-sweep >= 98.5% of pixels hold the same plane.
  T3  full RunPatchMatch: >= 99% of pixels with finite depths agree within 1%, and accuracy against
      ground truth within +-0.5 percentage points of the exact mode.
"""
import numpy as np
import pytest

import np_reference as npr
from acmmp import capi, scene, types

pytestmark = pytest.mark.gpu


def params_for(sc, **kw):
    c0 = sc.cameras[0]
    return types.default_params(num_images=len(sc.images), depth_min=float(c0["depth_min"]) * 0.6,
                                depth_max=float(c0["depth_max"]) * 1.2, **kw)


@pytest.fixture(scope="module")
def ctx():
    c = capi.Context(0)
    yield c
    c.close()


RIGS = {"pinhole": lambda: scene.pinhole_scene(320, 240, n_src=4, seed=5),
        "sphere": lambda: scene.sphere_scene(640, 320, n_src=4, seed=3)}


def run(ctx, mode, sc, p, seed, n_hs=-1, post=True):
    ctx.set_math(mode)
    ctx.set_params(p)
    ctx.upload_views(sc.images, sc.cameras)
    ctx.run_patchmatch(seed, n_half_sweeps=n_hs, do_post=post)
    pl, co = ctx.download()
    ctx.set_math("exact")
    return pl, co


def test_math_mode_switch(ctx):
    assert ctx.math() == "exact"
    ctx.set_math("fast")
    assert ctx.math() == "fast"
    ctx.set_math("exact")
    with pytest.raises(capi.AcmmpError):
        ctx._check(ctx.L.acmmp_set_math(ctx.h, 7), "set_math")


@pytest.mark.parametrize("kind", ["pinhole", "sphere"])
def test_t1_ncc_queries_within_float32_noise(ctx, kind):
    sc = RIGS[kind]()
    p = params_for(sc)
    H, W = sc.images[0].shape
    rng = np.random.default_rng(1)
    n = 250
    px, py = rng.integers(6, W - 6, n).astype(np.int32), rng.integers(6, H - 6, n).astype(np.int32)
    planes = []
    for k in range(n):                         # planes near the ground-truth surface (well-matched costs)
        d = npr.pixel_to_dir(sc.cameras[0], int(px[k]), int(py[k]))
        nrm = -d + rng.normal(0, 0.2, 3)
        nrm /= np.linalg.norm(nrm)
        depth = float(sc.gt_depth[py[k], px[k]]) * rng.uniform(0.98, 1.02)
        planes.append([*nrm, -float(nrm @ (d * depth))])
    planes = np.asarray(planes, np.float32)
    ctx.set_params(p)
    ctx.upload_views(sc.images, sc.cameras)
    ctx.set_math("fast")
    fast = ctx.debug_ncc(px, py, planes)
    ctx.set_math("exact")
    exact = ctx.debug_ncc(px, py, planes)
    ref = np.array([[npr.bilateral_ncc(sc.images, sc.cameras, p, v, int(px[k]), int(py[k]), planes[k].astype(np.float64))
                     for v in range(1, 5)] for k in range(n)])
    assert np.mean((fast >= 2.0) == (exact >= 2.0)) == 1.0
    valid = (exact < 2.0) & (ref < 2.0)
    assert valid.mean() > 0.5
    ef, ee = np.abs(fast - ref)[valid], np.abs(exact - ref)[valid]
    for q in (0.5, 0.99):
        assert np.quantile(ef, q) <= np.quantile(ee, q) + 1e-4, (q, np.quantile(ef, q), np.quantile(ee, q))
    d = np.abs(fast - exact)[valid]
    if kind == "pinhole":
        assert np.mean(d <= 1e-4) >= 0.995 and np.mean(d <= 1e-3) == 1.0
    else:
        assert np.mean(d <= 1e-3) >= 0.99


@pytest.mark.parametrize("kind", ["pinhole", "sphere"])
def test_t2_same_winners(ctx, kind):
    sc = RIGS[kind]()
    p = params_for(sc)
    fp, fc = run(ctx, "fast", sc, p, 5, n_hs=0, post=False)
    ep, ec = run(ctx, "exact", sc, p, 5, n_hs=0, post=False)
    assert np.array_equal(fp, ep)                                   # init planes: RNG only
    fin = np.isfinite(ec)
    assert np.mean(np.abs(fc - ec)[fin] <= 1e-3) >= 0.995
    fp, fc = run(ctx, "fast", sc, p, 5, n_hs=1, post=False)
    ep, ec = run(ctx, "exact", sc, p, 5, n_hs=1, post=False)
    same = np.all(np.abs(fp - ep) <= 1e-4 * np.maximum(1.0, np.abs(ep)), axis=-1)
    assert same.mean() >= 0.985, same.mean()


@pytest.mark.parametrize("kind", ["pinhole", "sphere"])
def test_t3_full_run_depths_and_accuracy(ctx, kind):
    sc = RIGS[kind]()
    p = params_for(sc)
    fp, fc = run(ctx, "fast", sc, p, 9)
    ep, ec = run(ctx, "exact", sc, p, 9)
    fd, ed = fp[..., 3], ep[..., 3]
    fin = np.isfinite(fd) & np.isfinite(ed) & (ed > 0)
    assert np.mean(np.abs(fd - ed)[fin] <= 0.01 * ed[fin]) >= 0.99
    acc_f, acc_e = scene.depth_accuracy(fd, sc.gt_depth), scene.depth_accuracy(ed, sc.gt_depth)
    assert abs(acc_f - acc_e) <= 0.005, (acc_f, acc_e)


def test_fast_mode_is_deterministic(ctx):
    sc = RIGS["sphere"]()
    p = params_for(sc)
    a = run(ctx, "fast", sc, p, 21)
    b = run(ctx, "fast", sc, p, 21)
    assert np.array_equal(a[0], b[0], equal_nan=True) and np.array_equal(a[1], b[1], equal_nan=True)
