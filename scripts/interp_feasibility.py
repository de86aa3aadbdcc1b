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


def lagrange(t, nodes):
    cols = []
    for k, a in enumerate(nodes):
        c = np.ones_like(t, dtype=np.float64)
        for m, b in enumerate(nodes):
            if m != k:
                c = c * (t - b) / (a - b)
        cols.append(c)
    return np.stack(cols, -1)


def ncc(images, cams, params, src, px, py, plane, interp, order=3, span_max=None, nodes=None):
    rc, sc = cams[0], cams[src]
    ref, simg = images[0], images[src]
    R = int(params["patch_size"]) // 2
    inc = int(params["radius_increment"])
    offs = np.arange(-R, R + 1, inc)
    ii, jj = np.meshgrid(offs, offs, indexing="ij")
    ii, jj = ii.ravel(), jj.ravel()
    W, H = sc["width"], sc["height"]

    def src_xy(di, dj):
        rx, ry = px + di, py + dj
        dn = npr.depth_from_plane(rc, plane, rx, ry)
        x, y, _ = npr.project(sc, npr.world_point(rc, rx, ry, dn))
        return np.asarray(x, np.float64), np.asarray(y, np.float64)

    fell_back = False
    if interp:
        nodes = np.linspace(-R, R, order) if nodes is None else np.asarray(nodes, np.float64)
        order = len(nodes)
        ni, nj = np.meshgrid(nodes, nodes, indexing="ij")
        X, Y = src_xy(ni.ravel(), nj.ravel())
        mid = (order * order) // 2
        X = X - np.round((X - X[mid]) / W) * W               # unwrap across the seam around the centre node
        dn = npr.depth_from_plane(rc, plane, px + ni.ravel(), py + nj.ravel())
        bad = (span_max is not None and (np.ptp(X) > span_max or np.ptp(Y) > span_max or np.any(dn <= 0)
                                         or np.any(dn >= 1e5)))
        if span_max is not None and span_max < 0:                # depth validity only
            bad = bool(np.any(dn <= 0) or np.any(dn >= 1e5))
        if bad:
            fell_back = True
            sx, sy = src_xy(ii, jj)
        else:
            L = lagrange(ii.astype(np.float64), nodes)[:, :, None] * lagrange(jj.astype(np.float64), nodes)[:, None, :]
            L = L.reshape(len(ii), order * order)
            sx, sy = L @ X, L @ Y
    else:
        sx, sy = src_xy(ii, jj)
    exact_x, exact_y = src_xy(ii, jj)
    sx = sx - np.floor(sx / W) * W
    sy = np.clip(sy, 0, H - 1)
    ex = exact_x - np.floor(exact_x / W) * W
    err = np.abs(np.where(np.abs(sx - ex) > W / 2, W - np.abs(sx - ex), sx - ex))
    err = np.maximum(err, np.abs(sy - np.clip(exact_y, 0, H - 1)))
    spix = npr.bilinear(simg, sx, sy)
    rpix = npr.texel(ref, px + ii, py + jj)
    center = npr.texel(ref, np.array(px), np.array(py))
    latc = -(py - rc["params"][2]) / rc["height"] * npr.PI_F
    scx, scy = 2 * npr.PI_F / rc["width"] * np.cos(latc), npr.PI_F / rc["height"]
    sig = float(params["sigma_spatial"]) * npr.PI_F / rc["height"]
    dx, dy = ii * scx, jj * scy
    w = np.exp(-np.sqrt(dx * dx + dy * dy) / (2 * sig * sig) - np.abs(rpix - center) / (2 * params["sigma_color"] ** 2))
    sbw = w.sum()
    if sbw < 1e-6:
        return 2.0, float(err.max()), fell_back
    mr, ms = (w * rpix).sum() / sbw, (w * spix).sum() / sbw
    vr = (w * rpix * rpix).sum() / sbw - mr * mr
    vs = (w * spix * spix).sum() / sbw - ms * ms
    if vr < 1e-5 or vs < 1e-5:
        return 2.0, float(err.max()), fell_back
    cov = (w * rpix * spix).sum() / sbw - mr * ms
    return float(np.clip(1 - cov / np.sqrt(vr * vs), 0.0, 2.0)), float(err.max()), fell_back


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=300)
    ap.add_argument("--width", type=int, default=2000)
    ap.add_argument("--height", type=int, default=1500)
    ap.add_argument("--n-src", type=int, default=4)
    ap.add_argument("--span", type=float, default=30.0, help="fallback when the nodes span more pixels than this")
    a = ap.parse_args()
    sc = scene.sphere_scene(a.width, a.height, n_src=a.n_src, seed=1)
    c0 = sc.cameras[0]
    p = types.default_params(num_images=len(sc.images), depth_min=float(c0["depth_min"]) * 0.6,
                             depth_max=float(c0["depth_max"]) * 1.2)
    out = {}
    variants = {"4x4": (4, None, None), "4x4+fallback": (4, a.span, None),
                "4x4 sample-aligned": (4, None, [-5, -1, 1, 5]), "4x4 sample-aligned+depthfb": (4, -1, [-5, -1, 1, 5]),
                "4x4 sample-aligned+span60": (4, 60.0, [-5, -1, 1, 5]),
                "4x4 sample-aligned+span100": (4, 100.0, [-5, -1, 1, 5])}
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
