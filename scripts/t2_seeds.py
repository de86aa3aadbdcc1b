#!/usr/bin/env python3
"""T2 of the fast mode (tests/test_gpu_fastmath.py) over several seeds, for the arithmetic variants of the fast
SPHERE path: same plane as the exact mode after one half-sweep, and the flips' median cost gap.

  per_sample     ACMMP_INTERP=0           every sample projected (the fast arithmetic the interpolation is gated against)
  product        (defaults)               interpolated coordinates, deferred per-sample fallbacks
  no_fallback    ACMMP_SPREAD_MAX=1e30    interpolated coordinates everywhere
  all_fallback   ACMMP_SPREAD_MAX=-1      every entry falls back (must equal per_sample bit for bit)

Besides the rates it splits the product's disagreements with no_fallback by whether the pixel's result also
differs from per_sample, to show where the fallbacks move decisions.  GPU box:
    python scripts/t2_seeds.py --configs metric c3 --seeds 81 82 83 84 --out gpurun_out/t2.json
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "acmmp-spherical_amd")]

import numpy as np  # noqa: E402

from acmmp import capi, scene, types  # noqa: E402

CONFIGS = {
    "metric": (lambda: scene.sphere_scene(2000, 1500, n_src=4, seed=1234, n_waves=24), {}),
    "c3": (lambda: scene.sphere_scene(3200, 1600, n_src=15, seed=1234, n_waves=12), {"ACMMP_NB_VIEW_CHUNK": "8"}),
    "sphere2000x1000v10": (lambda: scene.sphere_scene(2000, 1000, n_src=10, seed=77, n_waves=16), {}),
}
VARIANTS = {"per_sample": {"ACMMP_INTERP": "0"}, "product": {}, "no_fallback": {"ACMMP_SPREAD_MAX": "1e30"},
            "all_fallback": {"ACMMP_SPREAD_MAX": "-1"}}
KNOBS = ("ACMMP_INTERP", "ACMMP_SPREAD_MAX")


def params_for(sc):
    c0 = sc.cameras[0]
    return types.default_params(num_images=len(sc.images), depth_min=float(c0["depth_min"]) * 0.6,
                                depth_max=float(c0["depth_max"]) * 1.2)


def one(ctx, sc, p, mode, seed, n_hs):
    ctx.set_math(mode)
    ctx.set_params(p)
    ctx.upload_views(sc.images, sc.cameras)
    ctx.run_patchmatch(seed, n_half_sweeps=n_hs, do_post=False)
    return ctx.download()


def same_plane(a, b):
    return np.all(np.abs(a - b) <= 1e-4 * np.maximum(1.0, np.abs(b)), axis=-1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", nargs="+", default=["metric", "c3"])
    ap.add_argument("--seeds", nargs="+", type=int, default=[81, 82, 83, 84])
    ap.add_argument("--out", default="gpurun_out/t2_seeds.json")
    a = ap.parse_args()
    out = {}
    with capi.Context(0) as ctx:
        for name in a.configs:
            make, env = CONFIGS[name]
            t0 = time.time()
            sc = make()
            p = params_for(sc)
            for k, v in env.items():
                os.environ[k] = v
            res = {"seeds": a.seeds, "variants": {k: [] for k in VARIANTS}, "split": []}
            for seed in a.seeds:
                ep, ec = one(ctx, sc, p, "exact", seed, 1)
                runs = {}
                for vn, venv in VARIANTS.items():
                    for k in KNOBS:
                        os.environ.pop(k, None)
                    os.environ.update(venv)
                    fp, fc = one(ctx, sc, p, "fast", seed, 1)
                    runs[vn] = (fp, fc)
                    same = same_plane(fp, ep)
                    fin = np.isfinite(fc) & np.isfinite(ec) & ~same
                    gap = float(np.median(np.abs(fc - ec)[fin])) if fin.sum() else 0.0
                    res["variants"][vn].append({"seed": seed, "same_plane": float(same.mean()), "flips": int((~same).sum()),
                                                "flip_median_cost_gap": gap})
                for k in KNOBS:
                    os.environ.pop(k, None)
                ps, pr, nf = runs["per_sample"][0], runs["product"][0], runs["no_fallback"][0]
                se = same_plane(pr, ep)
                d_pr_nf = ~same_plane(pr, nf)
                d_pr_ps = ~same_plane(pr, ps)
                res["split"].append({
                    "seed": seed,
                    "all_fallback_equals_per_sample": bool(np.array_equal(runs["all_fallback"][0].view(np.uint32), ps.view(np.uint32))),
                    "product_vs_no_fallback_differs": int(d_pr_nf.sum()),
                    "of_those_product_equals_exact": int((d_pr_nf & se).sum()),
                    "of_those_no_fallback_equals_exact": int((d_pr_nf & same_plane(nf, ep)).sum()),
                    "of_those_product_equals_per_sample": int((d_pr_nf & ~d_pr_ps).sum()),
                    "product_vs_per_sample_differs": int(d_pr_ps.sum()),
                })
                print(name, seed, {k: v[-1]["same_plane"] for k, v in res["variants"].items()}, res["split"][-1], flush=True)
            for vn in VARIANTS:
                res[vn + "_mean"] = float(np.mean([r["same_plane"] for r in res["variants"][vn]]))
            res["wall_s"] = time.time() - t0
            for k in env:
                os.environ.pop(k, None)
            out[name] = res
            os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
            with open(a.out, "w") as fh:
                json.dump(out, fh, indent=1)
    print(json.dumps({n: {k: v for k, v in r.items() if k.endswith("_mean")} for n, r in out.items()}))


if __name__ == "__main__":
    main()
