"""Dump k_eval_nb's per-query costs (interpolated fast, per-sample fast, exact) on tests/test_gpu_interp.py's query
sets for one library build (ACMMP_LIB), so builds can be compared offline against the float64 restatement.
Usage (GPU box): python scripts/interp_dump.py OUT.npz [c3|metric]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "acmmp-spherical_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np  # noqa: E402

import np_interp as ni  # noqa: E402
from acmmp import capi, scene, types  # noqa: E402

CONF = {"metric": lambda: scene.sphere_scene(2000, 1500, n_src=4, seed=1234, n_waves=24),
        "c3": lambda: scene.sphere_scene(3200, 1600, n_src=15, seed=1234, n_waves=12)}
KINDS = {"random": 40, "pole": 32, "seam": 32}
out, name = sys.argv[1], sys.argv[2]
sc = CONF[name]()
c0 = sc.cameras[0]
p = types.default_params(num_images=len(sc.images), depth_min=float(c0["depth_min"]) * 0.6,
                         depth_max=float(c0["depth_max"]) * 1.2)
res = {}
with capi.Context(0) as ctx:
    ctx.set_params(p)
    ctx.upload_views(sc.images, sc.cameras)
    for kind, n in KINDS.items():
        px, py, _ = ni.special_pixels(sc, kind, n, seed=len(kind) + 17)
        planes = ni.near_surface_planes(sc, px, py, 8, seed=len(kind) + 29)
        fx, fy = np.repeat(px, 8), np.repeat(py, 8)
        ctx.set_math("fast")
        res[kind + "_nb_f"] = ctx.debug_ncc_nb(px, py, planes)
        res[kind + "_ps_f"] = ctx.debug_ncc(fx, fy, planes.reshape(-1, 4)).reshape(res[kind + "_nb_f"].shape)
        ctx.set_math("exact")
        res[kind + "_nb_e"] = ctx.debug_ncc_nb(px, py, planes)
        res[kind + "_px"], res[kind + "_py"], res[kind + "_planes"] = px, py, planes
np.savez(out, **res)
print("dumped", out)
