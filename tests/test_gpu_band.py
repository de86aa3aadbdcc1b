"""Row-band split of one view (acmmp_band_*, acmmp/band.py; SURVEY.md §8e latency mode): every band's rows
equal the whole-view RunPatchMatch bit for bit.

Several contexts on the one GPU play the ranks.  The halo (23 rows of the updated colour's plane / cost /
selected views after every half-sweep) is copied device to device with the row ranges the engine reports.
The RCCL transport of the same ranges (acmmp_comm_band_exchange) needs one GPU per rank and runs in the
multi-GPU bench.  Covered: pinhole and SPHERE, 2-4 bands, the reference's uncovered last row (odd H with
floor(H/2) a multiple of 16), exact and fast math, a geometric-consistency pass on reloaded state, and
the raw state without post-processing.  Tolerance: none (NaNs compared as NaN)."""
import os

import numpy as np
import pytest

from acmmp import band, capi, scene, types
from conftest import assert_bitwise_equal

pytestmark = pytest.mark.gpu


def _params(sc, **kw):
    c0 = sc.cameras[0]
    return types.default_params(num_images=len(sc.images), depth_min=float(c0["depth_min"]) * 0.6,
                                depth_max=float(c0["depth_max"]) * 1.2, **kw)


def _scene(kind, W, H, V, seed):
    if kind == "pinhole":
        return scene.pinhole_scene(W, H, n_src=V, seed=seed)
    return scene.sphere_scene(W, H, n_src=V, seed=seed)


def _setup(ctx, sc, p, math, depths=None, state=None, scaled=None, prior=None):
    ctx.set_math(math)
    ctx.set_params(p)
    ctx.upload_views(sc.images, sc.cameras)
    if depths is not None:
        ctx.upload_depths(depths)
    if state is not None:
        ctx.set_state(*state)
    if scaled is not None:
        ctx.set_scaled_state(scaled)
    if prior is not None:
        ctx.set_planar_prior(*prior)


def _outputs(ctx):
    planes, costs = ctx.download()
    sel, _ = ctx.download_aux()
    return planes, costs, sel


def _compare_bands(sc, p, math, nbands, seed, depths=None, state=None, do_post=True, scaled=None, prior=None):
    H = sc.images[0].shape[0]
    full = capi.Context(0)
    ctxs = [capi.Context(0) for _ in range(nbands)]
    try:
        _setup(full, sc, p, math, depths, state, scaled, prior)
        full.run_patchmatch(seed, do_post=do_post)
        want = _outputs(full)
        bands = band.split_rows(H, nbands)
        assert len(bands) == nbands
        for ctx in ctxs:
            _setup(ctx, sc, p, math, depths, state, scaled, prior)
        band.run_local(ctxs, seed, bands, do_post=do_post)
        for ctx, (lo, hi) in zip(ctxs, bands):
            got = _outputs(ctx)
            for g, w, name in zip(got, want, ("planes", "costs", "selected_views")):
                assert_bitwise_equal(g[lo:hi], w[lo:hi], f"{name} rows [{lo}, {hi})")
    finally:
        for c in ctxs + [full]:
            c.close()


CASES = [("sphere", 128, 96, 4, 3, "exact"), ("pinhole", 96, 97, 3, 4, "exact"), ("pinhole", 80, 65, 2, 2, "exact"),
         ("sphere", 160, 80, 3, 2, "fast"), ("pinhole", 90, 70, 4, 3, "fast")]


@pytest.mark.parametrize("kind,W,H,V,nb,math", CASES, ids=[f"{k}-{w}x{h}-v{v}-b{n}-{m}" for k, w, h, v, n, m in CASES])
def test_bands_equal_whole_view(kind, W, H, V, nb, math):
    sc = _scene(kind, W, H, V, seed=W + H + V)
    _compare_bands(sc, _params(sc), math, nb, seed=2024)


def test_bands_raw_state_without_post():
    sc = _scene("sphere", 128, 72, 3, seed=5)
    _compare_bands(sc, _params(sc), "exact", 3, seed=11, do_post=False)


@pytest.mark.parametrize("kind", ["pinhole", "sphere"])
def test_bands_geom_pass(kind):
    """A geometric-consistency pass (ACMMP.cpp:653-678) on reloaded state, split in two bands."""
    sc = _scene(kind, 96, 64, 3, seed=17)
    H, W = sc.images[0].shape
    rng = np.random.default_rng(3)
    depths = [(sc.gt_depth * rng.uniform(0.97, 1.03, (H, W))).astype(np.float32) for _ in range(4)]
    st = np.zeros((H, W, 4), np.float32)
    st[..., 2] = -1.0
    st[..., 3] = sc.gt_depth * rng.uniform(0.9, 1.1, (H, W)).astype(np.float32)
    costs0 = rng.uniform(0, 1, (H, W)).astype(np.float32)
    p = _params(sc, geom_consistency=1, max_iterations=2)
    _compare_bands(sc, p, "exact", 2, seed=7, depths=depths, state=(st, costs0))


def test_bands_hierarchy_upsample():
    """The upsample init branch (ACMMP.cu:713-779: JBU of the coarse normals around each pixel, pre_costs)
    and the hierarchy gate, split in three bands."""
    sc = _scene("sphere", 96, 72, 2, seed=51)
    H, W, h, w = 72, 96, 36, 48
    rng = np.random.default_rng(4)
    coarse = np.zeros((h, w, 4), np.float32)
    coarse[..., :3] = rng.normal(0, 0.2, (h, w, 3))
    coarse[..., 2] -= 1.0
    coarse[..., :3] /= np.linalg.norm(coarse[..., :3], axis=-1, keepdims=True)
    coarse[..., 3] = rng.uniform(0.05, 1.5, (h, w))
    cur = np.zeros((H, W, 4), np.float32)
    cur[..., 3] = (sc.gt_depth * rng.uniform(0.95, 1.05, (H, W))).astype(np.float32)
    p = _params(sc, hierarchy=1, upsample=1, scaled_cols=w, scaled_rows=h)
    _compare_bands(sc, p, "exact", 3, seed=9, state=(cur, None), scaled=coarse)


@pytest.mark.parametrize("math,geom", [("exact", 0), ("fast", 0), ("exact", 1)])
def test_bands_planar_prior(math, geom):
    """Prior-restricted propagation / refinement, with geom the planar-prior init branch too
    (ACMMP.cu:690-711), split in two bands."""
    sc = _scene("pinhole", 88, 60, 2, seed=41)
    H, W = sc.images[0].shape
    rng = np.random.default_rng(2)
    prior = np.zeros((H, W, 4), np.float32)
    prior[..., 2] = -1.0
    prior[..., 3] = (sc.gt_depth * rng.uniform(0.95, 1.05, (H, W))).astype(np.float32)
    masks = (rng.uniform(0, 1, (H, W)) < 0.6).astype(np.uint32) * rng.integers(1, 50, (H, W)).astype(np.uint32)
    st = np.zeros((H, W, 4), np.float32)
    st[..., 2] = -1.0
    st[..., 3] = sc.gt_depth
    costs0 = rng.uniform(0, 1, (H, W)).astype(np.float32)
    depths = [(sc.gt_depth * np.float32(1.01)).astype(np.float32)] * 3 if geom else None
    p = _params(sc, planar_prior=1, geom_consistency=geom, max_iterations=2 if geom else 3)
    _compare_bands(sc, p, math, 2, seed=5, depths=depths, state=(st, costs0), prior=(prior, masks))


def test_single_band_rccl_entry_equals_run():
    """acmmp_run_patchmatch_band with one band over the whole view (no communicator) is RunPatchMatch."""
    sc = _scene("sphere", 96, 48, 2, seed=9)
    p = _params(sc)
    a, b = capi.Context(0), capi.Context(0)
    try:
        _setup(a, sc, p, "exact")
        _setup(b, sc, p, "exact")
        a.run_patchmatch(31)
        b.run_patchmatch_band(31, 0, 48)
        for g, w, name in zip(_outputs(b), _outputs(a), ("planes", "costs", "selected_views")):
            assert_bitwise_equal(g, w, name)
    finally:
        a.close()
        b.close()


def test_band_api_errors():
    sc = _scene("pinhole", 64, 64, 1, seed=1)
    ctx = capi.Context(0)
    try:
        _setup(ctx, sc, _params(sc), "exact")
        with pytest.raises(capi.AcmmpError, match="band_begin"):
            ctx.band_sweep()
        with pytest.raises(capi.AcmmpError, match="ACMMP_BAND_HALO"):
            ctx.band_begin(1, 0, 20)                        # narrower than the halo
        with pytest.raises(capi.AcmmpError, match="outside"):
            ctx.band_begin(1, 40, 80)
        ctx.band_begin(1, 0, 32)
        assert ctx.band_sweeps_left() == 6
        ranges = ctx.band_halo_ranges()
        assert ranges[0] == (0, 0) and ranges[1] == (0, 0)      # no band above row 0
        assert ranges[2] == (9, 32) and ranges[3] == (32, 55)
        while ctx.band_sweeps_left():
            ctx.band_sweep()
        ctx.band_end()
        assert ctx.band_sweeps_left() == 0
    finally:
        ctx.close()


def test_bench_band_split_single_rank(monkeypatch):
    """bench.py's band-split side measurement end to end at world 1 (gloo group, single-rank RCCL
    communicator): the path the multi-GPU bench takes, minus the neighbour transfers."""
    import importlib.util
    import os
    import sys
    import torch.distributed as dist
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--width", "160", "--height", "96", "--n-src", "2"])
    spec.loader.exec_module(bench)
    args = bench.parse()
    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.setenv("MASTER_PORT", "29571")
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        out = bench.band_split(args, 0, 1, 0, dist, lambda x: x, reps=2)
    finally:
        dist.destroy_process_group()
    assert "error" not in out, out
    assert out["bit_identical_to_whole_view"] and out["bands"] == [(0, 96)] and out["ms_per_depth_map"] > 0


def _host_rank(rank, world, port, kind, W, H, V, math, out_dir):
    """One rank of a band run in its own process, both on GPU 0, the halo through host memory over gloo."""
    import os

    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        sc = _scene(kind, W, H, V, seed=W + H + V)
        p = _params(sc)
        with capi.Context(0) as ctx:
            _setup(ctx, sc, p, math)
            lo, hi = band.run_rank_host(ctx, 2025, H, rank, world, band.gloo_exchange)
            got = _outputs(ctx)
        with capi.Context(0) as full:
            _setup(full, sc, p, math)
            full.run_patchmatch(2025)
            want = _outputs(full)
        for g, w, name in zip(got, want, ("planes", "costs", "selected_views")):
            assert_bitwise_equal(g[lo:hi], w[lo:hi], f"rank {rank} {name} rows [{lo}, {hi})")
        open(os.path.join(out_dir, f"rank{rank}.ok"), "w").write(f"{lo} {hi}\n")
    finally:
        dist.destroy_process_group()


HOST_CASES = [("sphere", 160, 96, 3, 2, "fast"), ("pinhole", 96, 97, 3, 3, "exact")]


@pytest.mark.parametrize("kind,W,H,V,world,math", HOST_CASES,
                         ids=[f"{k}-{w}x{h}-v{v}-w{n}-{m}" for k, w, h, v, n, m in HOST_CASES])
def test_bands_over_processes_with_host_transport(tmp_path, kind, W, H, V, world, math):
    """The band protocol across processes: `world` ranks, each its own process with its own context on GPU 0,
    the halo rows after every half-sweep through host buffers over gloo (band.run_rank_host; the RCCL transport of
    the same ranges needs one GPU per rank).  Every rank's band equals the whole-view run bit for bit."""
    import socket

    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_host_rank, args=(world, port, kind, W, H, V, math, str(tmp_path)), nprocs=world, join=True)
    assert sorted(os.listdir(tmp_path)) == [f"rank{r}.ok" for r in range(world)]
