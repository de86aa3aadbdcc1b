"""The design assumption behind the fast SPHERE k_eval_nb's interpolated source coordinates:
projecting a 6x6 patch exactly at the samples of columns / rows {0, 2, 3, 5} and taking the 4-point
Lagrange interpolation for the others changes the float64 NCC (tests/np_reference.py's restatement of
ComputeBilateralNCC, ACMMP.cu:405-516) by less than the binary32 noise floor (1e-4) for near-surface and
random planes once a reference pixel spans at most 2 pi / 2000 rad, except on the rare hypotheses whose
corner nodes spread over more than 256 source pixels (patches on a source pole) -- those the kernel projects
in full (capi.cpp build_kparams' gate; kernels.hip ncc_chunk's spread test).  At 1600x800 a 256-pixel test
misses a pole case (3.7e-3 at a 65-pixel spread): the gate starts at 2000x1000.
CPU, float64; the kernel itself is queried per hypothesis in tests/test_gpu_interp.py.
"""
import numpy as np

import np_interp as ni
import np_reference as npr
from acmmp import scene, types


def _queries(sc, p, rng, n, W, H, margin=6):
    c0 = sc.cameras[0]
    for kind in ("near_surface", "random"):
        for _ in range(n):
            px, py = int(rng.integers(margin, W - margin)), int(rng.integers(margin, H - margin))
            d = npr.pixel_to_dir(c0, px, py)
            if kind == "near_surface":
                nrm = -d + rng.normal(0, 0.2, 3)
                depth = float(sc.gt_depth[py, px]) * rng.uniform(0.98, 1.02)
            else:
                nrm = rng.normal(0, 1, 3)
                nrm = -nrm if nrm @ d > 0 else nrm
                depth = 1.0 / rng.uniform(1.0 / float(p["depth_max"]), 1.0 / float(p["depth_min"]))
            nrm /= np.linalg.norm(nrm)
            yield px, py, np.array([*nrm, -float(nrm @ (d * depth))])


def test_interpolated_ncc_within_noise_floor():
    W, H = 2000, 1000
    sc = scene.sphere_scene(W, H, n_src=3, seed=2)
    c0 = sc.cameras[0]
    p = types.default_params(num_images=len(sc.images), depth_min=float(c0["depth_min"]) * 0.6,
                             depth_max=float(c0["depth_max"]) * 1.2)
    assert ni.interp_enabled(W, H, p) and not ni.interp_enabled(1600, 800, p)
    worst, n = 0.0, 0
    for px, py, plane in _queries(sc, p, np.random.default_rng(3), 40, W, H):
        for v in range(1, len(sc.images)):
            e = ni.ncc(sc.images, sc.cameras, p, v, px, py, plane, False)[0]
            f, _, fell = ni.ncc(sc.images, sc.cameras, p, v, px, py, plane, True, nodes=ni.nodes_for(p),
                                span_max=ni.SPREAD_MAX)
            assert (e >= 2.0) == (f >= 2.0)
            if e < 2.0:
                worst = max(worst, abs(f - e))
                n += 1
    assert n > 100
    assert worst < 1e-4, worst


def test_interpolation_gate_other_patch_geometries():
    """Every (patch_size, radius_increment) the gate admits with 6x6 samples is the validated angular span
    or finer: patch 21 / increment 4 (also 6x6) spans twice the angle and only interpolates from 4000x2000,
    where its radius covers the same angle as patch 11 at 2000x1000; the 4-point weights are in index space,
    so its nodes are offsets {-10, -2, 2, 10}."""
    for ps, inc in ((11, 2), (21, 4), (13, 2), (9, 2), (11, 1)):
        p = types.default_params(patch_size=ps, radius_increment=inc)
        R = ps // 2
        six = len(range(-R, R + 1, inc)) == 6
        for W, H in ((1280, 640), (1600, 800), (2000, 1000), (2000, 1500), (3200, 1600), (4096, 2048)):
            on = ni.interp_enabled(W, H, p)
            assert on == (six and 2 * np.pi * R / W <= 2 * np.pi * 5 / 2000 + 1e-12 and np.pi * R / H <= np.pi * 5 / 1000 + 1e-12)
    p = types.default_params(patch_size=21, radius_increment=4)
    assert ni.nodes_for(p) == [-10, -2, 2, 10]
    assert not ni.interp_enabled(3200, 1600, p) and ni.interp_enabled(4096, 2048, p)


def test_interpolated_ncc_near_source_poles_and_seam():
    """The stress sets of tests/test_gpu_interp.py in float64 at the coarsest interpolated resolution: patches
    landing within 10 degrees of a source pole and across a source's longitude seam, near-surface planes and
    random ones.  With the kernel's spread test every interpolated NCC stays within 1e-4 of the projected one;
    the test is what keeps the pole-adjacent tail there (it falls back on those lanes)."""
    W, H = 2000, 1000
    sc = scene.sphere_scene(W, H, n_src=3, seed=5)
    c0 = sc.cameras[0]
    p = types.default_params(num_images=len(sc.images), depth_min=float(c0["depth_min"]) * 0.6,
                             depth_max=float(c0["depth_max"]) * 1.2)
    rng = np.random.default_rng(11)
    worst, n, fell_n = 0.0, 0, 0
    for kind in ("pole", "seam"):
        px, py, src = ni.special_pixels(sc, kind, 25, seed=13)
        assert len(px) >= 10, kind
        planes = ni.near_surface_planes(sc, px, py, 2, seed=17)
        for q in range(len(px)):
            d = npr.pixel_to_dir(c0, int(px[q]), int(py[q]))
            nrm = rng.normal(0, 1, 3)
            nrm = -nrm if nrm @ d > 0 else nrm
            nrm /= np.linalg.norm(nrm)
            depth = 1.0 / rng.uniform(1.0 / float(p["depth_max"]), 1.0 / float(p["depth_min"]))
            rand = np.array([*nrm, -float(nrm @ (d * depth))])
            for plane in (planes[q, 0].astype(np.float64), planes[q, 1].astype(np.float64), rand):
                v = int(src[q])
                e = ni.ncc(sc.images, sc.cameras, p, v, int(px[q]), int(py[q]), plane, False)[0]
                f, _, fell = ni.ncc(sc.images, sc.cameras, p, v, int(px[q]), int(py[q]), plane, True,
                                    nodes=ni.NODES, span_max=ni.SPREAD_MAX)
                fell_n += fell
                assert (e >= 2.0) == (f >= 2.0)
                if e < 2.0:
                    worst = max(worst, abs(f - e))
                    n += 1
    assert n > 60 and fell_n > 0
    assert worst < 1e-4, worst
