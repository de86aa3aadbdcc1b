"""The design assumption behind the fast SPHERE k_eval_nb's interpolated source coordinates:
projecting a 6x6 patch exactly at the samples of columns / rows {0, 2, 3, 5} and taking the 4-point
Lagrange interpolation for the others changes the float64 NCC (tests/np_reference.py's restatement of
ComputeBilateralNCC, ACMMP.cu:405-516) by less than the binary32 noise floor (1e-4), for near-surface
and random planes, once a reference pixel spans at most 2 pi / 1600 rad -- the resolution from which the
engine interpolates (capi.cpp build_kparams; coarser views project every sample: at 1280x640 the tail
reaches 8.5e-3).  CPU, float64; the kernel itself is held to the fast-mode gates in test_gpu_fastmath.py.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import interp_feasibility as itf  # noqa: E402
import np_reference as npr  # noqa: E402
from acmmp import scene, types  # noqa: E402


def test_interpolated_ncc_within_noise_floor():
    W, H = 1600, 800
    sc = scene.sphere_scene(W, H, n_src=3, seed=2)
    c0 = sc.cameras[0]
    p = types.default_params(num_images=len(sc.images), depth_min=float(c0["depth_min"]) * 0.6,
                             depth_max=float(c0["depth_max"]) * 1.2)
    rng = np.random.default_rng(3)
    worst, n = 0.0, 0
    for kind in ("near_surface", "random"):
        for _ in range(40):
            px, py = int(rng.integers(6, W - 6)), int(rng.integers(6, H - 6))
            d = npr.pixel_to_dir(c0, px, py)
            if kind == "near_surface":
                nrm = -d + rng.normal(0, 0.2, 3)
                depth = float(sc.gt_depth[py, px]) * rng.uniform(0.98, 1.02)
            else:
                nrm = rng.normal(0, 1, 3)
                nrm = -nrm if nrm @ d > 0 else nrm
                depth = 1.0 / rng.uniform(1.0 / float(p["depth_max"]), 1.0 / float(p["depth_min"]))
            nrm /= np.linalg.norm(nrm)
            plane = np.array([*nrm, -float(nrm @ (d * depth))])
            for v in range(1, len(sc.images)):
                e = itf.ncc(sc.images, sc.cameras, p, v, px, py, plane, False)[0]
                f = itf.ncc(sc.images, sc.cameras, p, v, px, py, plane, True, nodes=[-5, -1, 1, 5])[0]
                assert (e >= 2.0) == (f >= 2.0)
                if e < 2.0:
                    worst = max(worst, abs(f - e))
                    n += 1
    assert n > 100
    assert worst < 1e-4, worst
