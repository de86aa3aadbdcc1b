"""BASELINE.json configs[3] (C4) and configs[4] (C5) at their full single-view sizes, exact mode, bit for
bit against the CPU oracle through the C ABI.

  C4  ETH3D-style, 6000x4000 capped to 3200x2133 (main.cpp:52-53), ~20 sources, planar prior +
      multi-scale.  One 3200x2133 pinhole reference with V = 20: the random pass, then each pass kind
      the schedule (main.cpp:417-476) runs on it from real state -- the planar-prior pass
      (ACMMP.cu:690-711, 1247-1299; prior from the first pass's maps on the device, as the pipeline
      does), the hierarchy pass (upsample branch :713-779 from a 1600x1067 coarse state) and the
      geometric-consistency pass (:646-671, 20 source depth maps).
  C5  Tanks-and-Temples-style 1920x1080, 10-20 sources, full schedule: V = 10 and V = 20 references.

The oracle replays rows: init is per pixel, and one half-sweep reads at most 23 rows away
(SURVEY.md §8e), the post stage 5 more, so a band of `n` half-sweeps with a margin of
23 n + 10 rows has inputs identical to the whole-view run.  Full-size runs check whole-view
RandomInitialization bands, the first half-sweep, and (C5 V = 10) a whole RunPatchMatch band.  The
small-size V = 20 multi-scale planar pipeline equals the oracle-driven pipeline map for map.
"""
import numpy as np
import pytest

from acmmp import capi, scene, types
from conftest import assert_bitwise_equal

pytestmark = pytest.mark.gpu

REACH = 23           # rows one half-sweep reads (3 + 2 * 10, ACMMP.cu:971-979)
POST = 10            # merge + two filters (radius 5 each)


def params_for(sc, **kw):
    c0 = sc.cameras[0]
    return types.default_params(num_images=len(sc.images), depth_min=float(c0["depth_min"]) * 0.6,
                                depth_max=float(c0["depth_max"]) * 1.2, **kw)


def margin(n_half_sweeps, post):
    return REACH * n_half_sweeps + (POST if post else 0) + 4


def compare_band(ctx, oracle_mod, prob, seed, y0, y1, n_hs, post, state=None, keys=("planes", "costs")):
    """GPU run (whole view, from the context's current state) vs the oracle replaying [y0, y1) +- margin."""
    ctx.run_patchmatch(seed, n_half_sweeps=n_hs, do_post=post)
    g_p, g_c = ctx.download()
    g_s, g_pre = ctx.download_aux()
    H = g_c.shape[0]
    m = margin(n_hs if n_hs >= 0 else 6, post)
    st = state or {}
    o = oracle_mod.run_band(prob, seed, max(0, y0 - m), min(H, y1 + m), nthreads=16, n_half_sweeps=n_hs,
                            do_post=post, planes=st.get("planes"), costs=st.get("costs"))
    got = {"planes": g_p, "costs": g_c, "selected_views": g_s, "pre_costs": g_pre}
    for k in keys:
        assert_bitwise_equal(got[k][y0:y1], o[k][y0:y1], f"{k} rows [{y0}, {y1})")
    return g_p, g_c


# ---------------------------------------------------------------- C4: 3200x2133 pinhole, V = 20

@pytest.fixture(scope="module")
def c4():
    sc = scene.pinhole_scene(3200, 2133, n_src=20, seed=44, n_waves=12)
    c = capi.Context(0)
    c.set_params(params_for(sc))
    c.upload_views(sc.images, sc.cameras)
    # the random first pass of the schedule, whole view on the GPU: the state every later pass starts from
    c.run_patchmatch(4401)
    first_p, first_c = c.download()
    yield sc, c, first_p, first_c
    c.close()


@pytest.mark.slow
def test_c4_random_pass_bands(c4, oracle_mod):
    sc, c, first_p, first_c = c4
    H = sc.images[0].shape[0]
    assert np.mean(np.abs(first_p[..., 3] - sc.gt_depth) < 0.01 * sc.gt_depth) > 0.5
    prob = oracle_mod.Problem(sc.images, sc.cameras, params_for(sc))
    c.set_params(params_for(sc))
    compare_band(c, oracle_mod, prob, 4402, 40, 72, 0, False, keys=("planes", "costs", "selected_views"))
    compare_band(c, oracle_mod, prob, 4403, H - 50, H, 1, False, keys=("planes", "costs", "selected_views"))


@pytest.mark.slow
def test_c4_planar_prior_pass_bands(c4, oracle_mod):
    """ProcessProblem's second RunPatchMatch (main.cpp:113-197) at full C4 size: the prior built on the
    device from the first pass's maps (acmmp_set_planar_prior_from_maps, the pipeline's path), then the
    planar init branch and prior-restricted propagation / refinement."""
    sc, c, first_p, first_c = c4
    H = sc.images[0].shape[0]
    p0 = params_for(sc)
    c.set_params(p0)
    c.set_state(first_p, first_c)
    ntri = c.set_planar_prior_from_maps(first_p[..., 3], first_c, float(p0["depth_min"]), float(p0["depth_max"]))
    assert ntri > 1000
    prior, masks = c.download_planar_prior()
    assert (masks > 0).mean() > 0.2
    pp = params_for(sc, planar_prior=1)
    c.set_params(pp)
    prob = oracle_mod.Problem(sc.images, sc.cameras, pp, prior_planes=prior, plane_masks=masks)
    st = {"planes": first_p, "costs": first_c}
    y0 = H // 2 - 16
    compare_band(c, oracle_mod, prob, 4404, y0, y0 + 32, 0, False, state=st, keys=("planes", "costs", "selected_views"))
    c.set_state(first_p, first_c)
    compare_band(c, oracle_mod, prob, 4405, y0, y0 + 16, 1, False, state=st, keys=("planes", "costs", "selected_views"))


@pytest.mark.slow
def test_c4_hierarchy_pass_bands(c4, oracle_mod):
    """The finer-scale pass of the C4 schedule: upsample init from a 1600x1067 coarse state
    (ACMMP.cu:713-779, ACMMP.cpp:788-844) with the JBU'd depth as the current state, the hierarchy
    gate (:1315-1320) and pre_costs."""
    sc, c, first_p, first_c = c4
    H, W = sc.images[0].shape
    h, w = 1067, 1600
    rng = np.random.default_rng(12)
    coarse = np.zeros((h, w, 4), np.float32)
    coarse[..., :3] = rng.normal(0, 0.2, (h, w, 3))
    coarse[..., 2] -= 1.0
    coarse[..., :3] /= np.linalg.norm(coarse[..., :3], axis=-1, keepdims=True)
    coarse[..., 3] = rng.uniform(0.05, 1.5, (h, w))
    cur = np.zeros((H, W, 4), np.float32)
    cur[..., 3] = (sc.gt_depth * rng.uniform(0.97, 1.03, (H, W))).astype(np.float32)
    zero_c = np.zeros((H, W), np.float32)
    p = params_for(sc, hierarchy=1, upsample=1, scaled_cols=w, scaled_rows=h)
    c.set_params(p)
    c.upload_views(sc.images, sc.cameras)             # a new problem: fresh pre_costs / scaled state
    c.set_state(cur, zero_c)
    c.set_scaled_state(coarse)
    prob = oracle_mod.Problem(sc.images, sc.cameras, p, scaled_planes=coarse)
    st = {"planes": cur, "costs": zero_c}
    keys = ("planes", "costs", "selected_views", "pre_costs")
    compare_band(c, oracle_mod, prob, 4406, 100, 132, 0, False, state=st, keys=keys)
    c.set_state(cur, zero_c)
    compare_band(c, oracle_mod, prob, 4407, H // 3, H // 3 + 16, 1, False, state=st, keys=keys)


@pytest.mark.slow
def test_c4_geom_pass_bands(c4, oracle_mod):
    """Geometric-consistency pass (ACMMP.cpp:653-678, 726-786; max_iterations 2) with the 20 sources'
    depth maps, from the random pass's state."""
    sc, c, first_p, first_c = c4
    H, W = sc.images[0].shape
    rng = np.random.default_rng(13)
    depths = [first_p[..., 3]] + [(sc.gt_depth * rng.uniform(0.98, 1.02, (H, W))).astype(np.float32)
                                  for _ in range(20)]
    pg = params_for(sc, geom_consistency=1, max_iterations=2)
    c.set_params(pg)
    c.upload_views(sc.images, sc.cameras)
    c.upload_depths(depths)
    c.set_state(first_p, first_c)
    prob = oracle_mod.Problem(sc.images, sc.cameras, pg, depths=depths)
    st = {"planes": first_p, "costs": first_c}
    compare_band(c, oracle_mod, prob, 4408, 700, 732, 0, False, state=st, keys=("planes", "costs", "selected_views"))
    c.set_state(first_p, first_c)
    compare_band(c, oracle_mod, prob, 4409, 1500, 1516, 1, False, state=st, keys=("planes", "costs", "selected_views"))


# ---------------------------------------------------------------- C5: 1920x1080 pinhole, V = 10 and 20

@pytest.fixture(scope="module")
def c5_scene():
    return scene.pinhole_scene(1920, 1080, n_src=20, seed=55, n_waves=12)


def c5_views(sc, V):
    class Sub:
        pass
    s = Sub()
    s.images, s.cameras, s.gt_depth = list(sc.images[:V + 1]), sc.cameras[:V + 1], sc.gt_depth
    return s


@pytest.mark.slow
def test_c5_v10_whole_runpatchmatch_band(c5_scene, oracle_mod):
    """A whole RunPatchMatch (init, 3 iterations, post) of a 1920x1080 V = 10 reference: rows
    [520, 536) against the oracle replaying them with the full 6-half-sweep margin."""
    sc = c5_views(c5_scene, 10)
    p = params_for(sc)
    with capi.Context(0) as c:
        c.set_params(p)
        c.upload_views(sc.images, sc.cameras)
        prob = oracle_mod.Problem(sc.images, sc.cameras, p)
        g_p, _ = compare_band(c, oracle_mod, prob, 5501, 520, 536, -1, True,
                              keys=("planes", "costs", "selected_views"))
        assert np.mean(np.abs(g_p[..., 3] - sc.gt_depth) < 0.01 * sc.gt_depth) > 0.5


@pytest.mark.slow
@pytest.mark.parametrize("V", [10, 20])
def test_c5_init_and_first_halfsweep_bands(c5_scene, oracle_mod, V):
    sc = c5_views(c5_scene, V)
    p = params_for(sc)
    H = sc.images[0].shape[0]
    with capi.Context(0) as c:
        c.set_params(p)
        c.upload_views(sc.images, sc.cameras)
        prob = oracle_mod.Problem(sc.images, sc.cameras, p)
        compare_band(c, oracle_mod, prob, 5502 + V, 0, 24, 0, False, keys=("planes", "costs", "selected_views"))
        compare_band(c, oracle_mod, prob, 5503 + V, H // 2, H // 2 + 16, 1, False,
                     keys=("planes", "costs", "selected_views"))
        # full-size NCC queries over all V sources
        rng = np.random.default_rng(V)
        n = 60
        W = sc.images[0].shape[1]
        px, py = rng.integers(0, W, n).astype(np.int32), rng.integers(0, H, n).astype(np.int32)
        nrm = rng.normal(size=(n, 3))
        nrm[:, 2] = -np.abs(nrm[:, 2])
        nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
        planes = np.concatenate([nrm, rng.uniform(-6, 6, (n, 1))], 1).astype(np.float32)
        g = c.debug_ncc(px, py, planes)
        o = np.array([[oracle_mod.ncc(prob, v, int(px[k]), int(py[k]), planes[k]) for v in range(1, V + 1)]
                      for k in range(n)], np.float32)
        assert_bitwise_equal(g, o, "ncc")


# ---------------------------------------------------------------- C4/C5 schedule with V = 20, small size

def test_pinhole_v20_multiscale_planar_pipeline_equals_oracle_pipeline():
    """main.cpp's schedule (planar -> geom -> geom_multi, JBU, hierarchy planar -> geom -> geom_multi)
    over 21 pinhole views with 20 sources each: every stored map of the GPU pipeline equals the
    oracle-driven pipeline's."""
    from acmmp import pipeline
    from pipeline_support import OracleEngine, final_maps, small_dataset
    ds = small_dataset(48, 36, 21, model="pinhole", seed=20)
    gpu = pipeline.Pipeline(ds, order="reference", size_bound=26).run()
    cpu = pipeline.Pipeline(ds, engine=OracleEngine(nthreads=16), order="reference", size_bound=26).run()
    assert [q.name for q in gpu.passes] == ["planar", "geom", "geom_multi", "hier_planar", "geom", "geom_multi"]
    mg, mc = final_maps(gpu), final_maps(cpu)
    assert mg.keys() == mc.keys() and len(mg) == 84
    for k in mc:
        assert_bitwise_equal(mg[k], mc[k], str(k))
