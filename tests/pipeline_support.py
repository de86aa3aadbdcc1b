"""Test-side helpers for the pipeline driver: a CPU engine backed by the oracle (TEST
INFRASTRUCTURE -- the product pipeline drives capi.Context only), a gloo exchange for
world_size > 1 on the CPU, and a small synthetic multi-view dataset."""
import numpy as np

import oracle
from acmmp import io, pipeline, scene, types


class OracleEngine:
    """The capi.Context surface the pipeline uses, computed by the CPU oracle.  State persists
    between runs exactly as the engine's does (planes/costs zeroed only when the reference size
    changes, pre_costs and the prior / scaled state reset by every upload)."""

    def __init__(self, nthreads: int = 8):
        self.nthreads = nthreads
        self.shape = None
        self.depths = self.scaled = self.prior = self.masks = None

    def set_params(self, p):
        self.params = np.array(p, copy=True)

    def upload_views(self, images, cams):
        self.images = [np.ascontiguousarray(im, np.float32) for im in images]
        self.cams = np.array(cams, copy=True)
        shape = self.images[0].shape
        if shape != self.shape:
            H, W = shape
            self.planes = np.zeros((H, W, 4), np.float32)
            self.costs = np.zeros((H, W), np.float32)
            self.sel = np.zeros((H, W), np.uint32)
            self.shape = shape
        self.pre = np.zeros(shape, np.float32)             # per problem, as the engine
        self.depths = self.scaled = self.prior = self.masks = None

    def upload_depths(self, depths):
        self.depths = [np.ascontiguousarray(d, np.float32) for d in depths]

    def set_state(self, planes=None, costs=None):
        if planes is not None:
            self.planes = np.ascontiguousarray(planes, np.float32).copy()
        if costs is not None:
            self.costs = np.ascontiguousarray(costs, np.float32).copy()

    def set_scaled_state(self, planes):
        self.scaled = np.ascontiguousarray(planes, np.float32).copy()

    def set_planar_prior(self, prior, masks):
        self.prior = np.ascontiguousarray(prior, np.float32).copy()
        self.masks = np.ascontiguousarray(masks, np.uint32).copy()

    def run_patchmatch(self, seed):
        prob = oracle.Problem(self.images, self.cams, self.params, depths=self.depths, scaled_planes=self.scaled,
                              prior_planes=self.prior, plane_masks=self.masks)
        r = oracle.run_patchmatch(prob, seed=seed, planes=self.planes, costs=self.costs, pre_costs=self.pre,
                                  selected=self.sel, nthreads=self.nthreads)
        self.planes, self.costs = r["planes"], r["costs"]
        self.pre, self.sel = r["pre_costs"], r["selected_views"]

    def download(self):
        return self.planes.copy(), self.costs.copy()

    def jbu(self, ref, coarse, imagescale):
        return oracle.jbu(ref, coarse, imagescale, nthreads=self.nthreads)


class GlooExchange:
    """world_size > 1 on the CPU: the pass outputs broadcast from their owners over gloo."""

    def __init__(self, dist):
        self.dist = dist
        self.world, self.rank = dist.get_world_size(), dist.get_rank()

    def share(self, key, views, owners, store):
        import torch
        for v in views:
            if owners[v] == self.rank:
                arr = store.get(key, v)
            else:
                arr = np.empty(store.shapes[(key, v)], np.float32)
            t = torch.from_numpy(np.ascontiguousarray(arr))
            self.dist.broadcast(t, src=owners[v])
            if owners[v] != self.rank:
                store.put(key, v, t.numpy().copy())

    def close(self):
        pass


def small_dataset(width=64, height=32, n_views=3, seed=7, model="sphere"):
    """n_views views of one synthetic room; every view lists all others in pair.txt order."""
    if model == "sphere":
        sc = scene.sphere_scene(width, height, n_src=n_views - 1, seed=seed)
    else:
        sc = scene.pinhole_scene(width, height, n_src=n_views - 1, seed=seed)
    images = {i: np.asarray(sc.images[i], np.float32) for i in range(n_views)}
    cams = {i: np.array(sc.cameras[i], copy=True) for i in range(n_views)}
    problems = []
    for i in range(n_views):
        p = io.Problem(i)
        p.src_image_ids = [j for j in range(n_views) if j != i]
        problems.append(p)
    return pipeline.Dataset(images, cams, problems)


def final_maps(pipe):
    """Every stored map of the rank's own views (host copies)."""
    out = {}
    for (key, v) in list(pipe.store.shapes):
        a = pipe.store.get(key, v)
        if a is not None:
            out[(key, v)] = a
    return out


class OracleFusion:
    """capi.Fusion's surface computed by the oracle (tests only)."""

    def __init__(self, cams):
        self.cams = np.array(cams, copy=True)
        n = len(self.cams)
        self.depths, self.normals, self.rgba = [None] * n, [None] * n, [None] * n

    def set_view(self, k, depth, normals, bgr):
        self.depths[k] = np.ascontiguousarray(depth, np.float32)
        self.normals[k] = np.ascontiguousarray(normals, np.float32)
        b = np.asarray(bgr, np.uint8).astype(np.float32)
        s = np.float32(1.0 / 255.0)
        rgba = np.stack([b[..., 2] * s, b[..., 1] * s, b[..., 0] * s,
                         np.full(b.shape[:2], np.float32(255.0) * s, np.float32)], -1)
        self.rgba[k] = rgba.astype(np.float32)

    def run(self, ref, srcs):
        return oracle.fuse(self.cams, self.depths, self.normals, self.rgba, ref, srcs)
