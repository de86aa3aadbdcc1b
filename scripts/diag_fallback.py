"""Per query (acmmp_debug_ncc_nb) at the metric view: k_eval_nb's path with every entry deferred
(ACMMP_SPREAD_MAX=-1), a small threshold, the product one and the interpolation alone, against the
per-sample fast hook (acmmp_debug_ncc) -- bitwise agreement and max |d|.  (Round 4 found the deleted inline
fallback wrong on 22% of forced random queries this way.)"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "acmmp-spherical_amd"))
import np_interp as ni  # noqa: E402
from acmmp import capi, scene, types  # noqa: E402

sc = scene.sphere_scene(2000, 1500, n_src=4, seed=1234, n_waves=24)
c0 = sc.cameras[0]
p = types.default_params(num_images=len(sc.images), depth_min=float(c0["depth_min"]) * 0.6,
                         depth_max=float(c0["depth_max"]) * 1.2)
ctx = capi.Context(0)
ctx.set_params(p)
ctx.upload_views(sc.images, sc.cameras)
ctx.set_math("fast")
for kind in ("random", "pole"):
    px, py, _ = ni.special_pixels(sc, kind, 40, seed=len(kind) + 17)
    planes = ni.near_surface_planes(sc, px, py, 8, seed=len(kind) + 29)
    res = {}
    for tag, env in (("queue-all", {"ACMMP_SPREAD_MAX": "-1"}), ("queue4", {"ACMMP_SPREAD_MAX": "4"}),
                     ("interp", {"ACMMP_SPREAD_MAX": "1e30"}), ("queue256", {})):
        os.environ.pop("ACMMP_SPREAD_MAX", None)
        os.environ.update(env)
        ctx.set_params(p)
        res[tag] = ctx.debug_ncc_nb(px, py, planes)
    ps = ctx.debug_ncc(np.repeat(px, 8), np.repeat(py, 8), planes.reshape(-1, 4)).reshape(res["interp"].shape)
    for tag, a in res.items():
        same = np.mean(a.view(np.uint32) == ps.view(np.uint32))
        print(kind, tag, "bitwise==per-sample %.4f" % same, "max|d| %.3g" % float(np.nanmax(np.abs(a - ps))),
              "==queue4 %.4f" % np.mean(a.view(np.uint32) == res["queue4"].view(np.uint32)), flush=True)
ctx.close()
