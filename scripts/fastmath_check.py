#!/usr/bin/env python3
"""Fast-math engine mode against the exact mode and the CPU oracle (SURVEY.md §8c tolerances):
T1 NCC queries, T2 winners after init / one half-sweep, T3 full runs (depth agreement and
ground-truth accuracy).  Prints one JSON object.  GPU box: python scripts/fastmath_check.py"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "acmmp-spherical_amd"), os.path.join(REPO, "oracle")]

import numpy as np  # noqa: E402

import oracle  # noqa: E402
from acmmp import capi, scene, types  # noqa: E402


def params_for(sc, **kw):
    c0 = sc.cameras[0]
    return types.default_params(num_images=len(sc.images), depth_min=float(c0["depth_min"]) * 0.6,
                                depth_max=float(c0["depth_max"]) * 1.2, **kw)


def run(ctx, mode, sc, p, seed, n_hs=-1, post=True):
    ctx.set_math(mode)
    ctx.set_params(p)
    ctx.upload_views(sc.images, sc.cameras)
    ctx.run_patchmatch(seed, n_half_sweeps=n_hs, do_post=post)
    pl, co = ctx.download()
    sel, _ = ctx.download_aux()
    return pl, co, sel


def t1(ctx, sc, p, n=3000):
    H, W = sc.images[0].shape
    V = len(sc.images) - 1
    rng = np.random.default_rng(0)
    px, py = rng.integers(0, W, n).astype(np.int32), rng.integers(0, H, n).astype(np.int32)
    gt = sc.gt_depth[py, px]
    nrm = rng.normal(0, 0.3, size=(n, 3))
    nrm[:, 2] = -1
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    d = gt * rng.uniform(0.97, 1.03, n)
    # plane through the (perturbed) ground-truth point: w = -n . (ray * d)
    prob = oracle.Problem(sc.images, sc.cameras, p)
    rays = np.zeros((n, 3), np.float32)
    for k in range(n):
        oracle.lib().or_pixel_to_dir(prob.cams[0:1].ctypes.data, int(px[k]), int(py[k]), rays[k].ctypes.data)
    w = -(nrm * rays).sum(1) * d
    planes = np.concatenate([nrm, w[:, None]], 1).astype(np.float32)
    ctx.set_params(p)
    ctx.upload_views(sc.images, sc.cameras)
    ctx.set_math("fast")
    f = ctx.debug_ncc(px, py, planes)
    ctx.set_math("exact")
    e = ctx.debug_ncc(px, py, planes)
    cls_f, cls_e = f >= 2.0, e >= 2.0
    both = ~cls_f & ~cls_e
    dif = np.abs(f - e)[both]
    return {"queries": int(n * V), "class_agree": float((cls_f == cls_e).mean()),
            "valid_frac": float(both.mean()), "max_abs_dcost": float(dif.max()) if dif.size else 0.0,
            "p999_abs_dcost": float(np.quantile(dif, 0.999)) if dif.size else 0.0,
            "frac_within_1e-4": float((dif <= 1e-4).mean()) if dif.size else 1.0}


def t2(ctx, sc, p):
    out = {}
    for hs in (0, 1):
        fp, fc, fs = run(ctx, "fast", sc, p, 5, n_hs=hs, post=False)
        ep, ec, es = run(ctx, "exact", sc, p, 5, n_hs=hs, post=False)
        same_plane = np.all(np.abs(fp - ep) <= 1e-4 * np.maximum(1, np.abs(ep)), axis=-1)
        fin = np.isfinite(fc) & np.isfinite(ec)
        out[f"hs{hs}"] = {"same_winner_frac": float(same_plane.mean()),
                          "cost_within_1e-3": float((np.abs(fc - ec)[fin] <= 1e-3).mean()),
                          "same_selected_views": float((fs == es).mean())}
    return out


def t3(ctx, sc, p):
    fp, fc, _ = run(ctx, "fast", sc, p, 9)
    ep, ec, _ = run(ctx, "exact", sc, p, 9)
    fd, ed = fp[..., 3], ep[..., 3]
    fin = np.isfinite(fd) & np.isfinite(ed) & (ed > 0)
    rel = np.abs(fd - ed)[fin] / ed[fin]
    return {"depth_within_1pct": float((rel <= 0.01).mean()),
            "gt_acc_fast": scene.depth_accuracy(fd, sc.gt_depth), "gt_acc_exact": scene.depth_accuracy(ed, sc.gt_depth),
            "nan_cost_fast": float(np.isnan(fc).mean()), "nan_cost_exact": float(np.isnan(ec).mean())}


def main():
    res = {}
    with capi.Context(0) as ctx:
        for name, sc in [("sphere_640x320_v4", scene.sphere_scene(640, 320, n_src=4, seed=3)),
                         ("sphere_2000x1000_v4", scene.sphere_scene(2000, 1000, n_src=4, seed=4, n_waves=24)),
                         ("pinhole_640x480_v4", scene.pinhole_scene(640, 480, n_src=4, seed=5)),
                         ("pinhole_800x600_v10", scene.pinhole_scene(800, 600, n_src=10, seed=6, n_waves=24))]:
            p = params_for(sc)
            res[name] = {"T1": t1(ctx, sc, p), "T2": t2(ctx, sc, p), "T3": t3(ctx, sc, p)}
            print(name, json.dumps(res[name]), file=sys.stderr, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
