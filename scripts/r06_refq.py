import os, sys
sys.path.insert(0, "acmmp-spherical_amd"); sys.path.insert(0, "tests")
import numpy as np
from acmmp import capi, scene, types
import np_interp as ni
sc = scene.sphere_scene(640, 320, n_src=4, seed=3)
c0 = sc.cameras[0]
p = types.default_params(num_images=5, depth_min=float(c0["depth_min"]) * 0.6, depth_max=float(c0["depth_max"]) * 1.2)
rng = np.random.default_rng(1)
H, W = 320, 640
px = rng.integers(20, W - 20, 300).astype(np.int32); py = rng.integers(60, 100, 300).astype(np.int32)
planes = ni.near_surface_planes(sc, px, py, 5, seed=5)
with capi.Context(0) as ctx:
    ctx.set_math("fast"); ctx.set_params(p); ctx.upload_views(sc.images, sc.cameras)
    out = ctx.debug_ncc_ref(px, py, planes)
np.save(sys.argv[1], out)
print(out.shape, np.isnan(out).mean())
