"""End-to-end timing of the multi-pass pipeline (main.cpp's schedule) on a synthetic SPHERE scene.

python scripts/pipeline_bench.py [--views 6] [--width 2000] [--height 1000] [--model sphere|pinhole] [--n-src K]
Prints one JSON line: per-pass wall times, per-stage host times, total, and depth accuracy of the
final maps.  --n-src K gives every view its K nearest views (camera centres) as sources, as a
pair.txt of a large capture would; default: all other views.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "acmmp-spherical_amd"))

import numpy as np  # noqa: E402

from acmmp import io, pipeline, scene  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--views", type=int, default=6)
    ap.add_argument("--width", type=int, default=2000)
    ap.add_argument("--height", type=int, default=1000)
    ap.add_argument("--seed", type=int, default=5)
    ap.add_argument("--model", choices=["sphere", "pinhole"], default="sphere")
    ap.add_argument("--n-src", type=int, default=0, help="sources per view (nearest camera centres); 0 = all")
    ap.add_argument("--math", choices=["exact", "fast"], default="exact", help="engine arithmetic (acmmp_set_math)")
    ap.add_argument("--n-waves", type=int, default=48, help="texture waves of the synthetic scene (fewer = faster to render)")
    a = ap.parse_args()
    make = scene.sphere_scene if a.model == "sphere" else scene.pinhole_scene
    t_scene = time.perf_counter()
    sc = make(a.width, a.height, n_src=a.views - 1, seed=a.seed, n_waves=a.n_waves)
    print(f"scene: {a.views} views {a.width}x{a.height} {a.model} in {time.perf_counter() - t_scene:.1f} s", flush=True)
    centres = np.array([-(np.asarray(c["R"], np.float64).reshape(3, 3).T @ np.asarray(c["t"], np.float64))
                        for c in sc.cameras])
    images = {i: np.asarray(sc.images[i], np.float32) for i in range(a.views)}
    cams = {i: np.array(sc.cameras[i], copy=True) for i in range(a.views)}
    problems = []
    for i in range(a.views):
        p = io.Problem(i)
        others = [j for j in range(a.views) if j != i]
        if a.n_src:
            others = sorted(others, key=lambda j: (float(np.linalg.norm(centres[j] - centres[i])), j))[:a.n_src]
        p.src_image_ids = others
        problems.append(p)
    ds = pipeline.Dataset(images, cams, problems)
    times = []
    last = [time.perf_counter()]

    def log(msg):
        now = time.perf_counter()
        times.append((msg, now - last[0]))
        last[0] = now
        print(msg, flush=True)

    t0 = time.perf_counter()
    pipe = pipeline.Pipeline(ds, order="reference", log=log, math=a.math).run()
    total = time.perf_counter() - t0
    d0 = pipe.store.get("depths_geom", 0)
    acc = scene.depth_accuracy(d0, sc.gt_depth) if d0.shape == sc.gt_depth.shape else None
    print(json.dumps({"views": a.views, "size": [a.width, a.height], "model": a.model, "math": a.math,
                      "n_src": len(problems[0].src_image_ids), "passes": [p.name for p in pipe.passes],
                      "total_s": round(total, 3), "s_per_view_pass": round(total / (a.views * len(pipe.passes)), 4),
                      "pass_s": [round(t, 3) for _, t in times[1:]] + [round(time.perf_counter() - last[0], 3)],
                      "stages_s": {k: round(v, 3) for k, v in sorted(pipe.stage_s.items())},
                      "pass_compute_s": [round(p.compute_s, 3) for p in pipe.passes],
                      "pass_stages_s": [{k: round(v, 3) for k, v in sorted(p.stages.items())} for p in pipe.passes],
                      "ref_view_frac_within_1pct_gt": acc}), flush=True)


if __name__ == "__main__":
    main()
