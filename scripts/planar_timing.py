"""Host planar-prior stage timing on a real first-pass RunPatchMatch output (GPU box): support points,
Delaunay, the full host block, and the device paths (acmmp_set_planar_prior_from_maps / _from_state)."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "acmmp-spherical_amd"))
import numpy as np  # noqa: E402

from acmmp import capi, scene, types  # noqa: E402

W, H = int(sys.argv[1]), int(sys.argv[2])
model = sys.argv[3] if len(sys.argv) > 3 else "pinhole"
sc = (scene.pinhole_scene if model == "pinhole" else scene.sphere_scene)(W, H, n_src=4, seed=3, n_waves=16)
c0 = sc.cameras[0]
p = types.default_params(num_images=5, depth_min=float(c0["depth_min"]) * 0.6, depth_max=float(c0["depth_max"]) * 1.2)
ctx = capi.Context(0)
ctx.set_math("fast")
ctx.set_params(p)
ctx.upload_views(sc.images, sc.cameras)
ctx.run_patchmatch(1)
planes, costs = ctx.download()
depth = np.ascontiguousarray(planes[..., 3])
out = {"size": [W, H], "model": model}
t = time.perf_counter(); xy = capi.support_points(costs); out["support_points_ms_x2"] = (time.perf_counter() - t) * 1e3
out["n_support"] = int(len(xy))
t = time.perf_counter(); tri = capi.delaunay(xy, W, H); out["delaunay_ms"] = (time.perf_counter() - t) * 1e3
os.environ["ACMMP_DELAUNAY_INCREMENTAL"] = "1"              # the incremental form, for comparison
t = time.perf_counter(); tri_inc = capi.delaunay(xy, W, H); out["delaunay_incremental_ms"] = (time.perf_counter() - t) * 1e3
del os.environ["ACMMP_DELAUNAY_INCREMENTAL"]
out["same_triangles_as_incremental"] = bool(np.array_equal(tri, tri_inc))
out["n_tri"] = int(len(tri))
t = time.perf_counter(); capi.planar_prior_host(c0, depth, costs, float(p["depth_min"]), float(p["depth_max"]))
out["planar_prior_host_ms"] = (time.perf_counter() - t) * 1e3
p["planar_prior"] = 1
ctx.set_params(p)
ts = []
for _ in range(3):
    t = time.perf_counter(); ctx.set_planar_prior_from_maps(depth, costs, float(p["depth_min"]), float(p["depth_max"]))
    ts.append((time.perf_counter() - t) * 1e3)
out["set_planar_prior_from_maps_ms"] = ts
ts, parts = [], []
for _ in range(3):
    t = time.perf_counter(); out["n_tri_state"] = ctx.set_planar_prior_from_state(float(p["depth_min"]), float(p["depth_max"]))
    ts.append((time.perf_counter() - t) * 1e3)
    parts.append(ctx.last_planar_timing())
out["set_planar_prior_from_state_ms"] = ts
out["set_planar_prior_from_state_parts"] = parts
# the host Delaunay alone (the triangles part's bulk) by thread count
for nt in (1, 4, 8, 16):
    os.environ["ACMMP_DELAUNAY_THREADS"] = str(nt)
    best = 1e9
    for _ in range(3):
        t = time.perf_counter(); capi.delaunay(xy, W, H); best = min(best, (time.perf_counter() - t) * 1e3)
    out[f"delaunay_ms_threads{nt}"] = best
del os.environ["ACMMP_DELAUNAY_THREADS"]
print(json.dumps(out))
