"""Parity of the HIP engine (through the C ABI) with the CPU oracle -- bit for bit.

Every branch of RandomInitialization (random / planar prior / hierarchy upsample /
reuse), CheckerboardPropagation with and without geometric consistency and planar prior,
PlaneHypothesisRefinement, GetDepthandNormal, the checkerboard median filter and JBU,
for pinhole and SPHERE rigs, 1..9 source views, odd sizes and the reference's uncovered
last row.  Tolerance: none -- outputs must be bit-identical (NaNs compared as NaN).
"""
import glob
import os

import numpy as np
import pytest

from acmmp import capi, scene, types
from conftest import assert_bitwise_equal

pytestmark = pytest.mark.gpu


def params_for(sc, **kw):
    c0 = sc.cameras[0]
    return types.default_params(num_images=len(sc.images), depth_min=float(c0["depth_min"]) * 0.6,
                                depth_max=float(c0["depth_max"]) * 1.2, **kw)


def gpu_run(ctx, sc, p, seed, planes=None, costs=None, depths=None, scaled=None, prior=None, mask=None,
            n_half_sweeps=-1, do_post=True, upload=True):
    ctx.set_params(p)
    if upload:
        ctx.upload_views(sc.images, sc.cameras)
    if depths is not None:
        ctx.upload_depths(depths)
    if planes is not None or costs is not None:
        ctx.set_state(planes, costs)
    if scaled is not None:
        ctx.set_scaled_state(scaled)
    if prior is not None:
        ctx.set_planar_prior(prior, mask)
    ctx.run_patchmatch(seed, n_half_sweeps=n_half_sweeps, do_post=do_post)
    pl, co = ctx.download()
    sel, pre = ctx.download_aux()
    return {"planes": pl, "costs": co, "selected_views": sel, "pre_costs": pre}


def check(g, o, keys=("planes", "costs", "selected_views")):
    for k in keys:
        assert_bitwise_equal(g[k], o[k], k)


@pytest.fixture(scope="module")
def ctx():
    c = capi.Context(0)
    yield c
    c.close()


SCENES = [
    ("pinhole", 96, 64, 1), ("pinhole", 96, 64, 2), ("pinhole", 70, 45, 4), ("pinhole", 64, 40, 5),
    ("pinhole", 48, 33, 9), ("sphere", 128, 64, 1), ("sphere", 128, 64, 2), ("sphere", 100, 50, 4),
    ("sphere", 96, 48, 6),
]


def make(kind, W, H, V, seed=0, quantize=True):
    if kind == "pinhole":
        return scene.pinhole_scene(W, H, n_src=V, seed=seed, quantize=quantize)
    return scene.sphere_scene(W, H, n_src=V, seed=seed, quantize=quantize)


@pytest.mark.parametrize("kind,W,H,V", SCENES, ids=[f"{k}-{w}x{h}-v{v}" for k, w, h, v in SCENES])
def test_full_run_bitexact(ctx, oracle_mod, kind, W, H, V):
    sc = make(kind, W, H, V, seed=W + V)
    p = params_for(sc)
    g = gpu_run(ctx, sc, p, seed=4321)
    o = oracle_mod.run_patchmatch(oracle_mod.Problem(sc.images, sc.cameras, p), seed=4321)
    check(g, o)


@pytest.mark.parametrize("kind", ["pinhole", "sphere"])
def test_upload_views_device_bitexact(ctx, oracle_mod, kind):
    """acmmp_upload_views_device (images already in HBM, the pipeline's per-scale image cache) gives
    the run acmmp_upload_views gives: both equal the oracle bit for bit."""
    sc = make(kind, 90, 48, 3, seed=31)
    p = params_for(sc)
    bufs = []
    for im in sc.images:
        b = capi.DeviceBuffer(0, im.shape)
        b.upload(im)
        bufs.append(b)
    ctx.set_params(p)
    ctx.upload_views_device(bufs, sc.cameras)
    ctx.run_patchmatch(55)
    planes, costs = ctx.download()
    g = gpu_run(ctx, sc, p, seed=55)
    for b in bufs:
        b.free()
    assert_bitwise_equal(planes, g["planes"], "planes (device upload vs host upload)")
    assert_bitwise_equal(costs, g["costs"], "costs (device upload vs host upload)")
    o = oracle_mod.run_patchmatch(oracle_mod.Problem(sc.images, sc.cameras, p), seed=55)
    check(g, o)


SPLITS = [("sphere", 100, 50, 4, "0"), ("sphere", 100, 50, 4, "1"), ("sphere", 100, 50, 4, "3"),
          ("pinhole", 70, 45, 10, "0"), ("pinhole", 70, 45, 10, "2"), ("pinhole", 70, 45, 10, "8")]


@pytest.mark.parametrize("kind,W,H,V,split", SPLITS, ids=[f"{k}-v{v}-S{s}" for k, w, h, v, s in SPLITS])
def test_refinement_split_points_bitexact(ctx, oracle_mod, monkeypatch, kind, W, H, V, split):
    """The split refinement evaluation (k_eval_ref on views [0, S), pruning, k_eval_ref_tail on the rest)
    is exact for every split point: S = 0 (one pass over all views) and fixed S other than the default
    all equal the oracle bit for bit -- a candidate dropped by its partial bound is never accepted."""
    sc = make(kind, W, H, V, seed=W + V + 1)
    if split == "0":
        monkeypatch.setenv("ACMMP_REF_SPLIT", "0")
    else:
        monkeypatch.setenv("ACMMP_REF_SPLIT_AT", split)
    p = params_for(sc)
    g = gpu_run(ctx, sc, p, seed=777)
    o = oracle_mod.run_patchmatch(oracle_mod.Problem(sc.images, sc.cameras, p), seed=777)
    check(g, o)


@pytest.mark.parametrize("kind", ["pinhole", "sphere"])
@pytest.mark.parametrize("fmt", ["f16", "fp32-forced", "fp32-unquantized"])
def test_texel_formats_bitexact(ctx, oracle_mod, monkeypatch, kind, fmt):
    """8-bit images are fetched from the binary16 copy, others (and ACMMP_TEX16=0) from fp32:
    both equal the oracle bit for bit."""
    sc = make(kind, 88, 52, 3, seed=23, quantize=(fmt != "fp32-unquantized"))
    if fmt == "fp32-forced":
        monkeypatch.setenv("ACMMP_TEX16", "0")
    p = params_for(sc)
    g = gpu_run(ctx, sc, p, seed=99)
    assert ctx.texel_bytes() == (2 if fmt == "f16" else 4)
    o = oracle_mod.run_patchmatch(oracle_mod.Problem(sc.images, sc.cameras, p), seed=99)
    check(g, o)
    monkeypatch.delenv("ACMMP_TEX16", raising=False)
    ctx.upload_views(sc.images, sc.cameras)                    # back to the default format


def test_texel_bytes_state(oracle_mod):
    with capi.Context(0) as c:
        assert c.texel_bytes() == 0
        sc = make("sphere", 64, 32, 1, seed=3)
        c.set_params(params_for(sc))
        c.upload_views(sc.images, sc.cameras)
        assert c.texel_bytes() == 2
        imgs = [im.copy() for im in sc.images]
        imgs[1][5, 7] = 70000.0                                # beyond binary16's range
        c.upload_views(imgs, sc.cameras)
        assert c.texel_bytes() == 4
        imgs[1][5, 7] = 2.0 ** -20                              # exact binary16 subnormal
        c.upload_views(imgs, sc.cameras)
        assert c.texel_bytes() == 4


@pytest.mark.parametrize("kind", ["pinhole", "sphere"])
@pytest.mark.parametrize("hs", [0, 1, 2, 3])
def test_half_sweeps_bitexact(ctx, oracle_mod, kind, hs):
    sc = make(kind, 80, 48, 3, seed=hs)
    p = params_for(sc)
    g = gpu_run(ctx, sc, p, seed=7 + hs, n_half_sweeps=hs, do_post=False)
    o = oracle_mod.run_patchmatch(oracle_mod.Problem(sc.images, sc.cameras, p), seed=7 + hs, n_half_sweeps=hs,
                                  do_post=False)
    check(g, o)


GOLDEN = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*.npz")))


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p) for p in GOLDEN])
def test_golden_fixtures(ctx, path):
    z = np.load(path, allow_pickle=False)
    sc = scene.Scene(list(z["images"]), z["cameras"], None, "golden")
    p = np.frombuffer(z["params"].tobytes(), types.PARAMS_DTYPE)[0]
    g = gpu_run(ctx, sc, p, seed=int(z["seed"]))
    assert_bitwise_equal(g["planes"], z["planes"], "planes")
    assert_bitwise_equal(g["costs"], z["costs"], "costs")
    assert_bitwise_equal(g["selected_views"], z["selected_views"], "selected_views")
    nc = ctx.debug_ncc(z["ncc_px"], z["ncc_py"], z["ncc_planes"])
    assert_bitwise_equal(nc, z["ncc_costs"], "ncc")


@pytest.mark.parametrize("kind", ["pinhole", "sphere"])
def test_ncc_and_geom_kernels_bitexact(ctx, oracle_mod, kind):
    sc = make(kind, 90, 60, 3, seed=17)
    p = params_for(sc)
    rng = np.random.default_rng(3)
    n = 400
    px, py = rng.integers(0, 90, n).astype(np.int32), rng.integers(0, 60, n).astype(np.int32)
    nrm = rng.normal(size=(n, 3))
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    planes = np.concatenate([nrm, rng.uniform(-1, 8, (n, 1))], 1).astype(np.float32)
    # extreme plane offsets: zero, tiny and (pinhole) huge |w| through the ray-plane division
    planes[::37, 3] = 0.0
    planes[5::37, 3] = 3e-25
    if kind == "pinhole":
        # (SPHERE projections beyond |t| ~ 1.8e19, where |t|^2 overflows, are outside the documented
        # range of the projection's division -- such depths never arise from [dmin, dmax])
        planes[11::37, 3] = -2e20
    depths = [np.abs(rng.normal(5, 1, im.shape)).astype(np.float32) for im in sc.images]
    depths[1][::7, ::5] = 0.0                                    # src_depth == 0 -> 3 (ACMMP.cu:658)
    ctx.set_params(p)
    ctx.upload_views(sc.images, sc.cameras)
    ctx.upload_depths(depths)
    prob = oracle_mod.Problem(sc.images, sc.cameras, p, depths=depths)
    g = ctx.debug_ncc(px, py, planes)
    o = np.array([[oracle_mod.ncc(prob, v, int(px[k]), int(py[k]), planes[k]) for v in (1, 2, 3)] for k in range(n)],
                 np.float32)
    assert_bitwise_equal(g, o, "ncc")
    g = ctx.debug_geom(px, py, planes)
    o = np.array([[oracle_mod.geom_cost(prob, v, int(px[k]), int(py[k]), planes[k]) for v in (1, 2, 3)]
                  for k in range(n)], np.float32)
    assert_bitwise_equal(g, o, "geom")


@pytest.mark.parametrize("kind", ["pinhole", "sphere"])
def test_geom_consistency_pass_bitexact(ctx, oracle_mod, kind):
    """Pass 2 of the reference schedule: geom consistency from the previous pass's depths
    (ACMMP.cpp:653-678, 726-786), max_iterations = 2 (ACMMP.cpp:551)."""
    sc = make(kind, 72, 48, 2, seed=31)
    p0 = params_for(sc)
    first = oracle_mod.run_patchmatch(oracle_mod.Problem(sc.images, sc.cameras, p0), seed=1)
    rng = np.random.default_rng(0)
    depths = [first["planes"][..., 3]] + [first["planes"][..., 3] * rng.uniform(0.97, 1.03, (48, 72)).astype(np.float32)
                                          for _ in range(2)]
    pg = params_for(sc, geom_consistency=1, max_iterations=2)
    g = gpu_run(ctx, sc, pg, seed=2, planes=first["planes"], costs=first["costs"], depths=depths)
    o = oracle_mod.run_patchmatch(oracle_mod.Problem(sc.images, sc.cameras, pg, depths=depths), seed=2,
                                  planes=first["planes"], costs=first["costs"])
    check(g, o)


@pytest.mark.parametrize("kind", ["pinhole", "sphere"])
@pytest.mark.parametrize("split", ["1", "3"])
def test_geom_pass_split_points_bitexact(ctx, oracle_mod, monkeypatch, kind, split):
    """The refinement split in a geom pass (the pruned aggregate carries w * (c + 0.1 geom) terms) at
    non-default split points, four source views: bit-exact."""
    sc = make(kind, 72, 48, 4, seed=37)
    p0 = params_for(sc)
    first = oracle_mod.run_patchmatch(oracle_mod.Problem(sc.images, sc.cameras, p0), seed=3)
    rng = np.random.default_rng(5)
    depths = [first["planes"][..., 3]] + [first["planes"][..., 3] * rng.uniform(0.97, 1.03, (48, 72)).astype(np.float32)
                                          for _ in range(4)]
    monkeypatch.setenv("ACMMP_REF_SPLIT_AT", split)
    pg = params_for(sc, geom_consistency=1, max_iterations=2)
    g = gpu_run(ctx, sc, pg, seed=4, planes=first["planes"], costs=first["costs"], depths=depths)
    o = oracle_mod.run_patchmatch(oracle_mod.Problem(sc.images, sc.cameras, pg, depths=depths), seed=4,
                                  planes=first["planes"], costs=first["costs"])
    check(g, o)


@pytest.mark.parametrize("kind", ["pinhole", "sphere"])
@pytest.mark.parametrize("geom", [0, 1])
def test_planar_prior_pass_bitexact(ctx, oracle_mod, kind, geom):
    """Second RunPatchMatch of ProcessProblem (main.cpp:113-197) on device-resident state:
    planar prior init branch (ACMMP.cu:690-711), prior-restricted propagation and refinement."""
    sc = make(kind, 80, 52, 2, seed=41)
    H, W = sc.images[0].shape
    p0 = params_for(sc, geom_consistency=geom, max_iterations=2 if geom else 3)
    depths = [sc.gt_depth * np.float32(1.01)] * 3 if geom else None
    ctx.set_params(p0)
    ctx.upload_views(sc.images, sc.cameras)
    if geom:
        ctx.upload_depths(depths)
        rng = np.random.default_rng(1)
        st = np.zeros((H, W, 4), np.float32)
        st[..., 2] = -1.0
        st[..., 3] = sc.gt_depth * rng.uniform(0.9, 1.1, (H, W)).astype(np.float32)
        costs0 = rng.uniform(0, 1, (H, W)).astype(np.float32)
        ctx.set_state(st, costs0)
    ctx.run_patchmatch(5)
    first_p, first_c = ctx.download()
    rng = np.random.default_rng(2)
    prior = np.zeros((H, W, 4), np.float32)
    prior[..., 2] = -1.0
    prior[..., 3] = rng.uniform(4.0, 6.0, (H, W)).astype(np.float32)
    prior[..., :3] += rng.normal(0, 0.1, (H, W, 3)).astype(np.float32)
    mask = (rng.uniform(size=(H, W)) < 0.6).astype(np.uint32) * rng.integers(1, 9, (H, W)).astype(np.uint32)
    pp = params_for(sc, geom_consistency=geom, planar_prior=1, max_iterations=2 if geom else 3)
    ctx.set_params(pp)
    ctx.set_planar_prior(prior, mask)
    ctx.run_patchmatch(6)
    g_p, g_c = ctx.download()
    g_s, _ = ctx.download_aux()
    o = oracle_mod.run_patchmatch(oracle_mod.Problem(sc.images, sc.cameras, pp, depths=depths, prior_planes=prior,
                                                     plane_masks=mask), seed=6, planes=first_p, costs=first_c)
    check({"planes": g_p, "costs": g_c, "selected_views": g_s}, o)


@pytest.mark.parametrize("kind", ["pinhole", "sphere"])
def test_hierarchy_upsample_bitexact(ctx, oracle_mod, kind):
    """Finer-scale pass: RunJBU'd depth + coarse (normal, cost) -> upsample init branch
    (ACMMP.cu:713-779, ACMMP.cpp:788-844), then the hierarchy gate (ACMMP.cu:1315-1320)."""
    fine = make(kind, 96, 64, 2, seed=51)
    H, W = 64, 96
    h, w = 32, 48
    rng = np.random.default_rng(4)
    coarse = np.zeros((h, w, 4), np.float32)
    coarse[..., :3] = rng.normal(0, 0.2, (h, w, 3))
    coarse[..., 2] -= 1.0
    coarse[..., :3] /= np.linalg.norm(coarse[..., :3], axis=-1, keepdims=True)
    coarse[..., 3] = rng.uniform(0.05, 1.5, (h, w))                     # .w = coarse cost (ACMMP.cpp:823-825)
    jbu_depth = (fine.gt_depth * rng.uniform(0.95, 1.05, (H, W))).astype(np.float32)
    cur = np.zeros((H, W, 4), np.float32)
    cur[..., 3] = jbu_depth                                              # xyz = 0 (ACMMP.cpp:833-840)
    p = params_for(fine, hierarchy=1, upsample=1, scaled_cols=w, scaled_rows=h)
    g = gpu_run(ctx, fine, p, seed=9, planes=cur, scaled=coarse)
    o = oracle_mod.run_patchmatch(oracle_mod.Problem(fine.images, fine.cameras, p, scaled_planes=coarse), seed=9,
                                  planes=cur)
    check(g, o, keys=("planes", "costs", "selected_views", "pre_costs"))
    # reuse branch (hierarchy at the same size, ACMMP.cu:780-793) on the SAME context right after the
    # upsampled problem: pre_costs are zero for the new problem (a fresh ACMMP object per problem in the
    # reference, main.cpp:80), never the previous problem's upsample costs
    assert np.any(g["pre_costs"] != 0)
    same = np.zeros((H, W, 4), np.float32)
    same[..., 2] = -1.0
    same[..., 3] = jbu_depth
    p2 = params_for(fine, hierarchy=1)
    g = gpu_run(ctx, fine, p2, seed=10, planes=cur, scaled=same)
    o = oracle_mod.run_patchmatch(oracle_mod.Problem(fine.images, fine.cameras, p2, scaled_planes=same), seed=10,
                                  planes=cur)
    assert not np.any(g["pre_costs"])
    check(g, o)


def test_jbu_bitexact(ctx, oracle_mod):
    rng = np.random.default_rng(6)
    ref = np.round(rng.uniform(0, 255, (61, 90))).astype(np.float32)
    coarse = rng.uniform(2, 6, (31, 45)).astype(np.float32)
    scale = max(61 // 31, 90 // 45)
    g = ctx.jbu(ref, coarse, scale)
    o = oracle_mod.jbu(ref, coarse, scale)
    assert_bitwise_equal(g, o, "jbu")


def test_deterministic_and_seeded(ctx):
    sc = make("sphere", 120, 60, 2, seed=61)
    p = params_for(sc)
    a = gpu_run(ctx, sc, p, seed=11)
    b = gpu_run(ctx, sc, p, seed=11, upload=False)
    c = gpu_run(ctx, sc, p, seed=12, upload=False)
    check(a, b)
    assert not np.array_equal(a["planes"], c["planes"])


def test_api_errors(ctx):
    fresh = capi.Context(0)
    with pytest.raises(capi.AcmmpError, match="call order"):
        fresh.run_patchmatch(1)
    sc = make("pinhole", 32, 24, 2)
    fresh.upload_views(sc.images, sc.cameras)
    with pytest.raises(capi.AcmmpError, match="set_params"):
        fresh.run_patchmatch(1)
    fresh.set_params(params_for(sc, geom_consistency=1))
    with pytest.raises(capi.AcmmpError, match="upload_depths"):
        fresh.run_patchmatch(1)
    bad = sc.cameras.copy()
    bad["model"][1] = types.SPHERE
    with pytest.raises(capi.AcmmpError, match="mixed camera models"):
        fresh.upload_views(sc.images, bad)
    # prior / scaled state belong to one problem: a new upload_views invalidates them
    H, W = sc.images[0].shape
    fresh.set_params(params_for(sc))
    fresh.upload_views(sc.images, sc.cameras)
    fresh.set_planar_prior(np.zeros((H, W, 4), np.float32), np.zeros((H, W), np.uint32))
    fresh.set_scaled_state(np.zeros((H, W, 4), np.float32))
    fresh.upload_views(sc.images, sc.cameras)
    fresh.set_params(params_for(sc, planar_prior=1))
    with pytest.raises(capi.AcmmpError, match="set_planar_prior"):
        fresh.run_patchmatch(1)
    fresh.set_params(params_for(sc, hierarchy=1))
    with pytest.raises(capi.AcmmpError, match="set_scaled_state"):
        fresh.run_patchmatch(1)
    with pytest.raises(ValueError, match="shape"):
        fresh.upload_views([im[:-1] for im in sc.images], sc.cameras)
    with pytest.raises(ValueError, match="set_planar_prior"):
        fresh.set_planar_prior(np.zeros((H + 1, W, 4), np.float32), np.zeros((H, W), np.uint32))
    fresh.close()



@pytest.mark.parametrize("kind,W,H", [("pinhole", 160, 120), ("sphere", 256, 128), ("sphere", 2000, 1500),
                                      ("pinhole", 1600, 1200)])
def test_planar_prior_device_equals_host(ctx, kind, W, H):
    """acmmp_set_planar_prior_from_maps (raster + range mask + expansion on the device) writes exactly
    the prior planes and labels acmmp_planar_prior_host computes (main.cpp:113-181), on the first
    run's real depth/cost maps -- including the full-size views with ~10^5 triangles."""
    sc = (scene.pinhole_scene(W, H, n_src=2, seed=4) if kind == "pinhole" else scene.sphere_scene(W, H, n_src=2, seed=4))
    p = params_for(sc)
    r = gpu_run(ctx, sc, p, 21)
    depths, costs = r["planes"][..., 3].copy(), r["costs"]
    prior_h, masks_h, n_h = capi.planar_prior_host(sc.cameras[0], depths, costs, float(p["depth_min"]),
                                                   float(p["depth_max"]))
    n_d = ctx.set_planar_prior_from_maps(depths, costs, float(p["depth_min"]), float(p["depth_max"]))
    prior_d, masks_d = ctx.download_planar_prior()
    assert n_d == n_h and n_h > 0
    assert np.array_equal(masks_d, masks_h)
    assert_bitwise_equal(prior_d, prior_h, "prior planes")
    assert (masks_h > 0).mean() > 0.05
    # the planar pass then runs from either state identically
    q = params_for(sc, planar_prior=1)
    ctx.set_params(q)
    ctx.run_patchmatch(22)
    a = ctx.download()
    ctx.set_planar_prior(prior_h, masks_h)
    ctx.run_patchmatch(22)
    b = ctx.download()
    assert_bitwise_equal(a[0], b[0], "planes after the planar run")
    assert_bitwise_equal(a[1], b[1], "costs after the planar run")
