"""How often a pixel's plane equals a 4-neighbour's bit for bit after N half-sweeps (GPU box): the ceiling of
deduplicating k_eval_nb's 8 neighbour hypotheses.  python scripts/plane_dups.py"""
import sys, os, json
sys.path.insert(0, os.path.join(os.environ.get('GRAFT_REPO_ROOT', '/root/repo'), 'acmmp-spherical_amd'))
import numpy as np
from acmmp import capi, scene, types
out = {}
for name, sc in (("metric", scene.sphere_scene(2000, 1500, n_src=4, seed=1234, n_waves=24)),
                 ("c2", scene.pinhole_scene(1600, 1200, n_src=10, seed=5, n_waves=24))):
    c0 = sc.cameras[0]
    p = types.default_params(num_images=len(sc.images), depth_min=float(c0["depth_min"]) * 0.6, depth_max=float(c0["depth_max"]) * 1.2)
    with capi.Context(0) as ctx:
        ctx.set_math("fast"); ctx.set_params(p); ctx.upload_views(sc.images, sc.cameras)
        res = {}
        for hs in (1, 2, 4, 6):
            ctx.run_patchmatch(7, n_half_sweeps=hs, do_post=False)
            pl, co = ctx.download()
            b = pl.view(np.uint32)
            same = lambda a, c: np.all(a == c, axis=-1)
            # fraction of pixels whose plane equals each 4-neighbour's plane bit for bit
            eq = [same(b[1:-1, 1:-1], b[1:-1, :-2]), same(b[1:-1, 1:-1], b[1:-1, 2:]), same(b[1:-1, 1:-1], b[:-2, 1:-1]), same(b[1:-1, 1:-1], b[2:, 1:-1])]
            n_eq = sum(e.astype(np.int32) for e in eq)
            res[hs] = {"any4": float((n_eq > 0).mean()), "mean_equal_of4": float(n_eq.mean() / 4)}
        out[name] = res
        print(name, res, flush=True)
print(json.dumps(out))
