#!/usr/bin/env python3
"""Feasibility of projecting a SPHERE patch exactly at 3x3 nodes and interpolating the other samples'
source coordinates, in float64 on the CPU: the NCC with interpolated coordinates
against the NCC with every sample projected (tests/np_reference.py's ComputeBilateralNCC restatement),
for near-surface planes (T1's queries) and for random hypotheses (RandomInitialization's).

  python scripts/interp_feasibility.py [--n 300] [--width 2000 --height 1500]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "acmmp-spherical_amd"), os.path.join(REPO, "tests")]

import numpy as np  # noqa: E402

import np_reference as npr  # noqa: E402
from acmmp import scene, types  # noqa: E402


from np_interp import lagrange, ncc  # noqa: E402,F401  (the float64 restatement lives with the tests)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=300)
    ap.add_argument("--width", type=int, default=2000)
    ap.add_argument("--height", type=int, default=1500)
    ap.add_argument("--n-src", type=int, default=4)
    ap.add_argument("--span", type=float, default=30.0, help="fallback when the corner nodes span more source pixels than this")
    a = ap.parse_args()
    sc = scene.sphere_scene(a.width, a.height, n_src=a.n_src, seed=1)
    c0 = sc.cameras[0]
    p = types.default_params(num_images=len(sc.images), depth_min=float(c0["depth_min"]) * 0.6,
                             depth_max=float(c0["depth_max"]) * 1.2)
    out = {}
    variants = {"4x4": (4, None, None), "4x4+fallback": (4, a.span, None),
                "4x4 sample-aligned": (4, None, [-5, -1, 1, 5]),
                "4x4 sample-aligned+spread64 (the kernel)": (4, 64.0, [-5, -1, 1, 5])}
    for kind in ("near_surface", "random"):
        rng = np.random.default_rng(7)
        qs = []
        for _ in range(a.n):
            px = int(rng.integers(6, a.width - 6))
            py = int(rng.integers(6, a.height - 6))
            d = npr.pixel_to_dir(c0, px, py)
            if kind == "near_surface":
                nrm = -d + rng.normal(0, 0.2, 3)
                depth = float(sc.gt_depth[py, px]) * rng.uniform(0.98, 1.02)
            else:
                nrm = rng.normal(0, 1, 3)
                if nrm @ d > 0:
                    nrm = -nrm
                depth = 1.0 / rng.uniform(1.0 / float(p["depth_max"]), 1.0 / float(p["depth_min"]))
            nrm /= np.linalg.norm(nrm)
            qs.append((px, py, np.array([*nrm, -float(nrm @ (d * depth))])))
        exact = [[ncc(sc.images, sc.cameras, p, v, px, py, pl, False)[0] for v in range(1, len(sc.images))]
                 for px, py, pl in qs]
        for name, (order, span, nodes) in variants.items():
            d_all, e_all, cls, fb = [], [], [], []
            for (px, py, pl), ev in zip(qs, exact):
                for v in range(1, len(sc.images)):
                    e = ev[v - 1]
                    f, err, fell = ncc(sc.images, sc.cameras, p, v, px, py, pl, True, order, span, nodes)
                    cls.append((e >= 2.0) == (f >= 2.0))
                    fb.append(fell)
                    if e < 2.0 and f < 2.0:
                        d_all.append(abs(f - e))
                        e_all.append(err)
            d_all, e_all = np.array(d_all), np.array(e_all)
            out[f"{kind}/{name}"] = {
                "queries": len(cls), "class_agree": float(np.mean(cls)), "fallback_frac": float(np.mean(fb)),
                "frac_dcost_le_1e-4": float((d_all <= 1e-4).mean()), "frac_dcost_le_1e-3": float((d_all <= 1e-3).mean()),
                "dcost_q50_q99_max": [float(np.quantile(d_all, 0.5)), float(np.quantile(d_all, 0.99)), float(d_all.max())],
                "coord_err_px_q50_q99_max": [float(np.quantile(e_all, 0.5)), float(np.quantile(e_all, 0.99)),
                                             float(e_all.max())]}
            print(kind, name, json.dumps(out[f"{kind}/{name}"]), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
