"""Oracle behaviour on whole RunPatchMatch runs (T3 of SURVEY.md §4): accuracy against
ground truth, determinism of the snapshot semantics, and reference quirks kept."""
import numpy as np
import pytest

from acmmp import scene, types
from conftest import assert_bitwise_equal


def _params(sc, **kw):
    c0 = sc.cameras[0]
    return types.default_params(num_images=len(sc.images), depth_min=float(c0["depth_min"]) * 0.6,
                                depth_max=float(c0["depth_max"]) * 1.2, **kw)


def test_pinhole_accuracy(oracle_mod):
    sc = scene.pinhole_scene(160, 120, n_src=2, seed=1)
    r = oracle_mod.run_patchmatch(oracle_mod.Problem(sc.images, sc.cameras, _params(sc)), seed=1234)
    acc = scene.depth_accuracy(r["planes"][..., 3], sc.gt_depth)
    assert acc > 0.85, acc
    assert np.isnan(r["costs"]).mean() < 0.05   # weight_norm == 0 -> 0/0 (ACMMP.cu:1243), borders only


def test_sphere_accuracy(oracle_mod):
    sc = scene.sphere_scene(240, 120, n_src=2, seed=3)
    r = oracle_mod.run_patchmatch(oracle_mod.Problem(sc.images, sc.cameras, _params(sc)), seed=99)
    acc = scene.depth_accuracy(r["planes"][..., 3], sc.gt_depth)
    assert acc > 0.6, acc


def test_thread_count_independent(oracle_mod):
    """Snapshot (Jacobi) reads make a half-sweep order-independent: 1 thread == 8 threads."""
    sc = scene.pinhole_scene(64, 48, n_src=2, seed=5)
    prob = oracle_mod.Problem(sc.images, sc.cameras, _params(sc))
    a = oracle_mod.run_patchmatch(prob, seed=3, nthreads=1)
    b = oracle_mod.run_patchmatch(prob, seed=3, nthreads=8)
    for k in ("planes", "costs", "selected_views"):
        assert_bitwise_equal(a[k], b[k], k)
    c = oracle_mod.run_patchmatch(prob, seed=4, nthreads=8)
    assert not np.array_equal(a["planes"], c["planes"])


def test_uncovered_last_row(oracle_mod):
    """ACMMP.cu:1525: with H odd and (H-1)/2 a multiple of 16 the checkerboard grid skips the
    last row, so it keeps its initial hypothesis."""
    sc = scene.pinhole_scene(40, 33, n_src=2, seed=6)
    prob = oracle_mod.Problem(sc.images, sc.cameras, _params(sc))
    init = oracle_mod.run_patchmatch(prob, seed=8, n_half_sweeps=0, do_post=False)
    full = oracle_mod.run_patchmatch(prob, seed=8, do_post=False)
    assert_bitwise_equal(full["planes"][32], init["planes"][32], "row 32")
    assert not np.array_equal(full["planes"][31], init["planes"][31])


def test_geom_and_planar_branches_run(oracle_mod):
    sc = scene.pinhole_scene(64, 48, n_src=2, seed=9)
    p0 = _params(sc)
    prob = oracle_mod.Problem(sc.images, sc.cameras, p0)
    r0 = oracle_mod.run_patchmatch(prob, seed=1)
    depths = [r0["planes"][..., 3]] * 3
    pg = _params(sc, geom_consistency=1, max_iterations=2)
    probg = oracle_mod.Problem(sc.images, sc.cameras, pg, depths=depths)
    rg = oracle_mod.run_patchmatch(probg, seed=2, planes=r0["planes"], costs=r0["costs"])
    assert scene.depth_accuracy(rg["planes"][..., 3], sc.gt_depth) > 0.7
    prior = np.zeros((48, 64, 4), np.float32)
    mask = np.zeros((48, 64), np.uint32)
    mask[10:30, 10:40] = 1
    prior[...] = np.array([0, 0, -1, 5.0], np.float32)
    pp = _params(sc, planar_prior=1)
    probp = oracle_mod.Problem(sc.images, sc.cameras, pp, prior_planes=prior, plane_masks=mask)
    rp = oracle_mod.run_patchmatch(probp, seed=3, planes=r0["planes"], costs=r0["costs"])
    assert np.isfinite(rp["planes"]).all()
