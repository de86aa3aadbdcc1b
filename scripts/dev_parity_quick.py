import sys, time, numpy as np
sys.path.insert(0, '/root/repo/acmmp-spherical_amd'); sys.path.insert(0, '/root/repo/oracle')
import oracle
from acmmp import scene, types, capi
def canon(a):
    a = np.array(a, copy=True); 
    if a.dtype == np.float32: 
        b = a.view(np.uint32).copy(); b[np.isnan(a)] = 0x7fc00000; return b
    return a
for kind in ['pinhole', 'sphere']:
    sc = scene.pinhole_scene(96, 64, n_src=2, seed=1) if kind=='pinhole' else scene.sphere_scene(128, 64, n_src=2, seed=2)
    c0 = sc.cameras[0]
    p = types.default_params(num_images=3, depth_min=c0['depth_min']*0.6, depth_max=c0['depth_max']*1.2)
    ctx = capi.Context(0)
    ctx.set_params(p); ctx.upload_views(sc.images, sc.cameras)
    prob = oracle.Problem(sc.images, sc.cameras, p)
    # debug ncc on random planes
    rng = np.random.default_rng(0)
    n = 500; px = rng.integers(0, 96 if kind=='pinhole' else 128, n); py = rng.integers(0, 64, n)
    nrm = rng.normal(size=(n,3)); nrm /= np.linalg.norm(nrm,axis=1,keepdims=True); nrm[:,2] = -np.abs(nrm[:,2])
    planes = np.concatenate([nrm, rng.uniform(3,6,(n,1))], 1).astype(np.float32)
    g = ctx.debug_ncc(px, py, planes)
    o = np.array([[oracle.ncc(prob, v+1, int(px[k]), int(py[k]), planes[k]) for v in range(2)] for k in range(n)], np.float32)
    print(kind, 'ncc bit-equal', np.mean(canon(g)==canon(o)), 'maxdiff', np.nanmax(np.abs(g-o)))
    for hs in [0, 1, 2, 6]:
        ctx.run_patchmatch(1234, n_half_sweeps=hs, do_post=(hs==6))
        pl, co = ctx.download(); sel, pre = ctx.download_aux()
        r = oracle.run_patchmatch(prob, seed=1234, n_half_sweeps=hs, do_post=(hs==6), nthreads=8)
        print(kind, 'half_sweeps', hs, 'planes eq', np.mean(canon(pl)==canon(r['planes'])), 'costs eq', np.mean(canon(co)==canon(r['costs'])), 'sel eq', np.mean(sel==r['selected_views']))
    print(ctx.last_timing())
