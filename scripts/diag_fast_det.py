"""Diagnostics (GPU): fast-mode determinism of a whole-view run and band == whole for a small SPHERE scene."""
import os
import sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "acmmp-spherical_amd"), os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402
from acmmp import capi, scene, types  # noqa: E402

for (W, H, V) in [(160, 80, 3), (160, 80, 4), (320, 160, 4)]:
    sc = scene.sphere_scene(W, H, n_src=V, seed=5)
    c0 = sc.cameras[0]
    p = types.default_params(num_images=len(sc.images), depth_min=float(c0["depth_min"]) * 0.6,
                             depth_max=float(c0["depth_max"]) * 1.2)
    outs = []
    for rep in range(3):
        with capi.Context(0) as ctx:
            ctx.set_math("fast")
            ctx.set_params(p)
            ctx.upload_views(sc.images, sc.cameras)
            ctx.run_patchmatch(11)
            outs.append(ctx.download()[0])
    d01 = int((outs[0].view(np.uint32) != outs[1].view(np.uint32)).sum())
    d02 = int((outs[0].view(np.uint32) != outs[2].view(np.uint32)).sum())
    print(W, H, V, "fast repeat diffs:", d01, d02, flush=True)
