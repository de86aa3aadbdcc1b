#!/usr/bin/env python3
"""Fast-math mode vs exact mode vs float64 at BASELINE.json's configurations: the measurement behind
the fast-mode gates of tests/test_gpu_fastmath.py and DESIGN.md §2.4.

T1  NCC queries (planes near the surface): the exact float32 path's own distance to a float64
    restatement of ComputeBilateralNCC (tests/np_reference.py) is the noise floor of the reference's
    arithmetic in binary32; reported beside the fast mode's distance and |fast - exact|.
T2  one black half-sweep from the same initial state: same-plane fraction, and for the pixels whose
    plane differs the |cost_fast - cost_exact| of the two winners (a near tie when it is within the
    T1 noise floor).
T3  full RunPatchMatch: depth agreement, ground-truth accuracy of both modes.
Also the same for a geometric-consistency pass, a planar-prior pass and a hierarchy pass.

GPU box: python scripts/fastmath_floor.py [--quick] > out.json
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "acmmp-spherical_amd"), os.path.join(REPO, "tests")]

import numpy as np  # noqa: E402

import np_reference as npr  # noqa: E402
from acmmp import capi, scene, types  # noqa: E402

Q = (0.5, 0.9, 0.99, 0.999)


def params_for(sc, **kw):
    c0 = sc.cameras[0]
    return types.default_params(num_images=len(sc.images), depth_min=float(c0["depth_min"]) * 0.6,
                                depth_max=float(c0["depth_max"]) * 1.2, **kw)


def quant(x):
    x = np.asarray(x, np.float64)
    if x.size == 0:
        return None
    return {**{f"q{q}": float(np.quantile(x, q)) for q in Q}, "max": float(x.max()), "n": int(x.size)}


def near_surface_planes(sc, n, rng, margin=6):
    H, W = sc.images[0].shape
    px = rng.integers(margin, W - margin, n).astype(np.int32)
    py = rng.integers(margin, H - margin, n).astype(np.int32)
    planes = []
    for k in range(n):
        d = npr.pixel_to_dir(sc.cameras[0], int(px[k]), int(py[k]))
        nrm = -d + rng.normal(0, 0.2, 3)
        nrm /= np.linalg.norm(nrm)
        depth = float(sc.gt_depth[py[k], px[k]]) * rng.uniform(0.98, 1.02)
        planes.append([*nrm, -float(nrm @ (d * depth))])
    return px, py, np.asarray(planes, np.float32)


def t1(ctx, sc, p, n, seed):
    rng = np.random.default_rng(seed)
    V = len(sc.images) - 1
    px, py, planes = near_surface_planes(sc, n, rng)
    ctx.set_math("fast")
    f = ctx.debug_ncc(px, py, planes)
    ctx.set_math("exact")
    e = ctx.debug_ncc(px, py, planes)
    t0 = time.time()
    ref = np.array([[npr.bilateral_ncc(sc.images, sc.cameras, p, v, int(px[k]), int(py[k]),
                                       planes[k].astype(np.float64)) for v in range(1, V + 1)] for k in range(n)])
    valid = (e < 2.0) & (ref < 2.0) & (f < 2.0)
    ee, ef, d = np.abs(e - ref)[valid], np.abs(f - ref)[valid], np.abs(f - e)[valid]
    # per query: the fast result is no further from float64 than the exact float32 result, + 1e-4; and the
    # symmetric pair -- if neither float32 evaluation is systematically closer to float64, the fraction of
    # queries where fast is worse by > 1e-4 matches the fraction where exact is
    per_query = np.abs(f - ref)[valid] <= np.abs(e - ref)[valid] + 1e-4
    exact_worse = np.abs(e - ref)[valid] > np.abs(f - ref)[valid] + 1e-4
    return {"queries": int(n * V), "f64_seconds": round(time.time() - t0, 1),
            "class_agree_fast_exact": float(((f >= 2.0) == (e >= 2.0)).mean()),
            "class_agree_exact_f64": float(((e >= 2.0) == (ref >= 2.0)).mean()),
            "valid_frac": float(valid.mean()),
            "exact_vs_f64": quant(ee), "fast_vs_f64": quant(ef), "fast_vs_exact": quant(d),
            "frac_fast_exact_within_1e-4": float((d <= 1e-4).mean()) if d.size else None,
            "frac_exact_f64_within_1e-4": float((ee <= 1e-4).mean()) if ee.size else None,
            "frac_per_query_fast_no_worse_1e-4": float(per_query.mean()) if per_query.size else None,
            "frac_fast_worse_by_1e-4": float(1.0 - per_query.mean()) if per_query.size else None,
            "frac_exact_worse_by_1e-4": float(exact_worse.mean()) if exact_worse.size else None}


def run(ctx, mode, seed, n_hs=-1, post=True, setup=None):
    ctx.set_math(mode)
    if setup:
        setup(ctx)
    ctx.run_patchmatch(seed, n_half_sweeps=n_hs, do_post=post)
    pl, co = ctx.download()
    ctx.set_math("exact")
    return pl, co


def t2_t3(ctx, sc, seed, setup, full=True):
    out = {}
    fp, fc = run(ctx, "fast", seed, 0, False, setup)
    ep, ec = run(ctx, "exact", seed, 0, False, setup)
    fin = np.isfinite(ec) & np.isfinite(fc)
    out["init"] = {"planes_identical": bool(np.array_equal(fp.view(np.uint32), ep.view(np.uint32))),
                   "cost_absdiff": quant(np.abs(fc - ec)[fin]),
                   "frac_cost_within_1e-3": float((np.abs(fc - ec)[fin] <= 1e-3).mean())}
    fp, fc = run(ctx, "fast", seed, 1, False, setup)
    ep, ec = run(ctx, "exact", seed, 1, False, setup)
    same = np.all(np.abs(fp - ep) <= 1e-4 * np.maximum(1.0, np.abs(ep)), axis=-1)
    mis = ~same
    fin = np.isfinite(fc) & np.isfinite(ec)
    gap = np.abs(fc - ec)[mis & fin]
    out["half_sweep"] = {"same_plane_frac": float(same.mean()), "mismatch_pixels": int(mis.sum()),
                         "mismatch_cost_gap": quant(gap),
                         "mismatch_gap_le_1e-3": float((gap <= 1e-3).mean()) if gap.size else None,
                         "mismatch_gap_le_1e-2": float((gap <= 1e-2).mean()) if gap.size else None,
                         "same_plane_cost_absdiff": quant(np.abs(fc - ec)[same & fin])}
    if full:
        fp, fc = run(ctx, "fast", seed + 1, -1, True, setup)
        ep, ec = run(ctx, "exact", seed + 1, -1, True, setup)
        fd, ed = fp[..., 3], ep[..., 3]
        fin = np.isfinite(fd) & np.isfinite(ed) & (ed > 0)
        out["full_run"] = {"depth_within_1pct": float((np.abs(fd - ed)[fin] <= 0.01 * ed[fin]).mean()),
                           "gt_acc_fast": scene.depth_accuracy(fd, sc.gt_depth),
                           "gt_acc_exact": scene.depth_accuracy(ed, sc.gt_depth),
                           "nan_cost_fast": float(np.isnan(fc).mean()), "nan_cost_exact": float(np.isnan(ec).mean())}
    return out


def config_runs(quick):
    nq = 150 if quick else 1000
    cfgs = [
        ("metric_sphere_2000x1500_v4", lambda: scene.sphere_scene(2000, 1500, n_src=4, seed=1234, n_waves=24), nq, {}),
        ("c2_pinhole_1600x1200_v10", lambda: scene.pinhole_scene(1600, 1200, n_src=10, seed=1234, n_waves=12), nq, {}),
        ("c3_sphere_3200x1600_v15_chunked", lambda: scene.sphere_scene(3200, 1600, n_src=15, seed=1234, n_waves=12),
         nq // 2, {"ACMMP_NB_VIEW_CHUNK": "8"}),
        ("c5_pinhole_1920x1080_v20", lambda: scene.pinhole_scene(1920, 1080, n_src=20, seed=55, n_waves=12), nq // 2, {}),
        ("pinhole_640x480_v32", lambda: scene.pinhole_scene(640, 480, n_src=32, seed=32, n_waves=24), nq // 2, {}),
        ("sphere_640x320_v32", lambda: scene.sphere_scene(640, 320, n_src=32, seed=33, n_waves=24), nq // 2, {}),
        ("sphere_2000x1000_v4", lambda: scene.sphere_scene(2000, 1000, n_src=4, seed=4, n_waves=24), nq, {}),
    ]
    if quick:
        cfgs = [c for c in cfgs if c[0] in ("metric_sphere_2000x1500_v4", "c2_pinhole_1600x1200_v10", "pinhole_640x480_v32")]
    return cfgs


def pass_runs(ctx, res):
    """geom / planar / hierarchy passes: the same starting state in both modes."""
    for kind, mk in (("pinhole", lambda: scene.pinhole_scene(800, 600, n_src=10, seed=61, n_waves=24)),
                     ("sphere", lambda: scene.sphere_scene(1000, 500, n_src=6, seed=62, n_waves=24))):
        sc = mk()
        H, W = sc.images[0].shape
        V = len(sc.images) - 1
        p0 = params_for(sc)
        ctx.set_math("exact")
        ctx.set_params(p0)
        ctx.upload_views(sc.images, sc.cameras)
        ctx.run_patchmatch(70)
        first_p, first_c = ctx.download()
        rng = np.random.default_rng(71)
        depths = [first_p[..., 3]] + [(sc.gt_depth * rng.uniform(0.98, 1.02, (H, W))).astype(np.float32)
                                      for _ in range(V)]

        def geom_setup(c):
            c.set_params(params_for(sc, geom_consistency=1, max_iterations=2))
            c.upload_views(sc.images, sc.cameras)
            c.upload_depths(depths)
            c.set_state(first_p, first_c)
        res[f"geom_{kind}_{W}x{H}_v{V}"] = t2_t3(ctx, sc, 72, geom_setup)

        ctx.set_params(p0)
        ctx.upload_views(sc.images, sc.cameras)
        ctx.set_state(first_p, first_c)
        ctx.set_planar_prior_from_maps(first_p[..., 3], first_c, float(p0["depth_min"]), float(p0["depth_max"]))
        prior, masks = ctx.download_planar_prior()

        def planar_setup(c):
            c.set_params(params_for(sc, planar_prior=1))
            c.upload_views(sc.images, sc.cameras)
            c.set_state(first_p, first_c)
            c.set_planar_prior(prior, masks)
        res[f"planar_{kind}_{W}x{H}_v{V}"] = t2_t3(ctx, sc, 73, planar_setup)

        h, w = H // 2, W // 2
        coarse = np.zeros((h, w, 4), np.float32)
        coarse[..., :3] = first_p[::2, ::2, :3][:h, :w]
        coarse[..., 3] = first_c[::2, ::2][:h, :w]
        cur = np.zeros((H, W, 4), np.float32)
        cur[..., 3] = first_p[..., 3]
        zc = np.zeros((H, W), np.float32)

        def hier_setup(c):
            c.set_params(params_for(sc, hierarchy=1, upsample=1, scaled_cols=w, scaled_rows=h))
            c.upload_views(sc.images, sc.cameras)
            c.set_state(cur, zc)
            c.set_scaled_state(coarse)
        res[f"hierarchy_{kind}_{W}x{H}_v{V}"] = t2_t3(ctx, sc, 74, hier_setup)
        print(kind, "passes done", file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--no-passes", action="store_true")
    a = ap.parse_args()
    res = {}
    with capi.Context(0) as ctx:
        for name, mk, nq, env in config_runs(a.quick):
            t0 = time.time()
            sc = mk()
            old = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            try:
                p = params_for(sc)
                ctx.set_params(p)
                ctx.upload_views(sc.images, sc.cameras)
                r = {"T1": t1(ctx, sc, p, nq, seed=len(name))}

                def setup(c, sc=sc, p=p):
                    c.set_params(p)
                    c.upload_views(sc.images, sc.cameras)
                r.update(t2_t3(ctx, sc, 81, setup))
            finally:
                for k, v in old.items():
                    if v is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = v
            r["seconds"] = round(time.time() - t0, 1)
            res[name] = r
            print(name, json.dumps(r), file=sys.stderr, flush=True)
        if not a.no_passes:
            pass_runs(ctx, res)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
