"""Fast-math engine mode (acmmp_set_math 'fast') -- tolerance parity at BASELINE.json's
configurations, against the exact mode (bit-identical to the CPU oracle) and a float64 restatement of
ComputeBilateralNCC (np_reference.py).

The fast mode changes only the NCC's per-sample projection arithmetic (hardware rsq / sqrt / rcp, the
latitude and longitude through one packed minimax atan, the source transform in the reference frame),
as the reference's own --use_fast_math build does to the same code (CMakeLists.txt:42).  It cannot be
bit-identical, so it is held to the gates DESIGN.md §2.4 states, measured in profiles/r03_fastmath_floor.json
(scripts/fastmath_floor.py):

  T1  NCC queries near the surface.  (a) The {valid, 2.0} classification agrees with the exact mode's as
      often as the exact mode's agrees with float64's (its thresholds are discontinuities binary32 noise
      can cross: 99.5% at the metric view), and for >= 99% of queries.
      (b) Pinhole: |fast - exact| <= 1e-4 for >= 99.5% of valid queries.  SPHERE: the
      binary32 noise floor of the reference's own arithmetic is far above 1e-4 -- the exact float32
      path is within 1e-4 of float64 for only ~91% of valid queries at the metric view (91.1% in
      profiles/r03_fastmath_floor.json; few effective samples under the sigma-in-radians weights,
      E[x^2] - E[x]^2 cancellation) -- so the gate is that
      fast departs from exact by > 1e-4 no more often than exact departs from float64, + 5 points.
      (c) No systematic accuracy loss: the fraction of queries where fast is farther from float64 than
      exact by > 1e-4 is at most the converse fraction + 3 points.
  T2  After RandomInitialization every plane is identical (same RNG draws) and costs agree within 1e-3
      for >= 99.5% (pinhole) / 99% (SPHERE) of pixels; after one black half-sweep >= 99.5% (pinhole) /
      98.5% (SPHERE) of pixels hold the same plane, and the flips are near ties: their median cost gap
      is below 1e-4.  Where the fast kernels interpolate SPHERE sample coordinates (>= 2000x1000), the
      98.5% holds for the per-sample fast arithmetic (ACMMP_INTERP=0), and over four seeds the
      interpolated runs hold >= 98.5% same planes on average, at most 0.2 pt fewer than the per-sample
      runs, every seed at most 0.5 pt below its per-sample run, with every seed's flips near ties (median
      cost gap < 3e-5; the float64 study puts the
      interpolation's NCC effect below 1e-4, tests/test_interp_design.py; the flips it adds are ties the
      binary32 noise already decides).  Measured: metric 98.58% vs 98.72%, C3 98.95% vs 99.05%
      (profiles/r05_t2_seeds.json).
  T3  A full RunPatchMatch: >= 99% of finite depths within 1% of the exact mode's, ground-truth accuracy
      within +-0.5 points.  Geom, planar-prior and hierarchy passes from one shared state (pinhole, SPHERE,
      and SPHERE at the interpolation's size): T3, T2's init gates, and after one half-sweep, for each of
      four seeds, the same plane on at least the measured four-seed mean - 0.5 pt of pixels
      (profiles/r06_pass_gates.json); the geom pass's flips are near cost ties (median gap bounded as
      measured); a planar / hierarchy flip selects by restricted cost or pre-cost, so its cost gap is not
      a tie measure and is not gated.
"""
import json
import os

import numpy as np
import pytest

import np_interp as ni
import np_reference as npr
from acmmp import capi, scene, types

pytestmark = pytest.mark.gpu


def params_for(sc, **kw):
    c0 = sc.cameras[0]
    return types.default_params(num_images=len(sc.images), depth_min=float(c0["depth_min"]) * 0.6,
                                depth_max=float(c0["depth_max"]) * 1.2, **kw)


@pytest.fixture(scope="module")
def ctx():
    c = capi.Context(0)
    yield c
    c.close()


def run(ctx, mode, seed, n_hs=-1, post=True, setup=None):
    ctx.set_math(mode)
    setup(ctx)
    ctx.run_patchmatch(seed, n_half_sweeps=n_hs, do_post=post)
    pl, co = ctx.download()
    ctx.set_math("exact")
    return pl, co


def plain_setup(sc, p):
    def f(c):
        c.set_params(p)
        c.upload_views(sc.images, sc.cameras)
    return f


def near_surface_queries(sc, n, seed):
    rng = np.random.default_rng(seed)
    H, W = sc.images[0].shape
    px, py = rng.integers(6, W - 6, n).astype(np.int32), rng.integers(6, H - 6, n).astype(np.int32)
    planes = []
    for k in range(n):
        d = npr.pixel_to_dir(sc.cameras[0], int(px[k]), int(py[k]))
        nrm = -d + rng.normal(0, 0.2, 3)
        nrm /= np.linalg.norm(nrm)
        depth = float(sc.gt_depth[py[k], px[k]]) * rng.uniform(0.98, 1.02)
        planes.append([*nrm, -float(nrm @ (d * depth))])
    return px, py, np.asarray(planes, np.float32)


def check_t1(ctx, sc, p, n, seed, sphere):
    V = len(sc.images) - 1
    px, py, planes = near_surface_queries(sc, n, seed)
    ctx.set_params(p)
    ctx.upload_views(sc.images, sc.cameras)
    ctx.set_math("fast")
    f = ctx.debug_ncc(px, py, planes)
    ctx.set_math("exact")
    e = ctx.debug_ncc(px, py, planes)
    ref = np.array([[npr.bilateral_ncc(sc.images, sc.cameras, p, v, int(px[k]), int(py[k]),
                                       planes[k].astype(np.float64)) for v in range(1, V + 1)] for k in range(n)])
    # (a) a cost of 2.0 is the reference's "no match" (centre outside, weight sum < 1e-6, variance
    # < 1e-5) or a clamped NCC; its thresholds are discontinuities the binary32 noise can cross, so the
    # fast mode may flip a query's class no more often than the exact mode's own class differs from
    # float64's, and never by more than 1% of the queries
    agree_fe = np.mean((f >= 2.0) == (e >= 2.0))
    agree_ef = np.mean((e >= 2.0) == (ref >= 2.0))
    assert agree_fe >= min(agree_ef, 0.999) - 0.002 and agree_fe >= 0.99, (agree_fe, agree_ef)
    valid = (e < 2.0) & (f < 2.0) & (ref < 2.0)
    assert valid.mean() > 0.3
    df, de, dfe = np.abs(f - ref)[valid], np.abs(e - ref)[valid], np.abs(f - e)[valid]
    if sphere:                                                                        # (b)
        assert np.mean(dfe <= 1e-4) >= np.mean(de <= 1e-4) - 0.05, (np.mean(dfe <= 1e-4), np.mean(de <= 1e-4))
    else:
        assert np.mean(dfe <= 1e-4) >= 0.995, np.mean(dfe <= 1e-4)
    fast_worse, exact_worse = np.mean(df > de + 1e-4), np.mean(de > df + 1e-4)        # (c)
    assert fast_worse <= exact_worse + 0.03, (fast_worse, exact_worse)


def check_t2(ctx, setup, seed, sphere, init=True, hs_min=None, gap_max=1e-4):
    if init:
        fp, fc = run(ctx, "fast", seed, 0, False, setup)
        ep, ec = run(ctx, "exact", seed, 0, False, setup)
        assert np.array_equal(fp.view(np.uint32), ep.view(np.uint32))                # RNG only
        fin = np.isfinite(ec) & np.isfinite(fc)
        assert np.mean(np.abs(fc - ec)[fin] <= 1e-3) >= (0.99 if sphere else 0.995)
    fp, fc = run(ctx, "fast", seed, 1, False, setup)
    ep, ec = run(ctx, "exact", seed, 1, False, setup)
    same = np.all(np.abs(fp - ep) <= 1e-4 * np.maximum(1.0, np.abs(ep)), axis=-1)
    floor = hs_min if hs_min is not None else (0.985 if sphere else 0.995)
    assert same.mean() >= floor, (same.mean(), floor)
    fin = np.isfinite(fc) & np.isfinite(ec) & ~same
    gap = float(np.median(np.abs(fc - ec)[fin])) if fin.sum() else 0.0
    if gap_max is not None and fin.sum() > 20:
        assert gap < gap_max, gap
    return float(same.mean()), gap


def check_t3(ctx, setup, seed, gt):
    fp, fc = run(ctx, "fast", seed, -1, True, setup)
    ep, ec = run(ctx, "exact", seed, -1, True, setup)
    fd, ed = fp[..., 3], ep[..., 3]
    fin = np.isfinite(fd) & np.isfinite(ed) & (ed > 0)
    assert np.mean(np.abs(fd - ed)[fin] <= 0.01 * ed[fin]) >= 0.99
    acc_f, acc_e = scene.depth_accuracy(fd, gt), scene.depth_accuracy(ed, gt)
    assert abs(acc_f - acc_e) <= 0.005, (acc_f, acc_e)


def test_math_mode_switch(ctx):
    assert ctx.math() == "exact"
    ctx.set_math("fast")
    assert ctx.math() == "fast"
    ctx.set_math("exact")
    with pytest.raises(capi.AcmmpError):
        ctx._check(ctx.L.acmmp_set_math(ctx.h, 7), "set_math")


# BASELINE.json configurations: the metric view, C2, C3 (at the 3200x1600 the
# reference scheduler runs it at, k_eval_nb view-chunked), C5 with 20 sources, and V = 32 (the maximum).
CONFIGS = {
    "metric-sphere-2000x1500-v4": (lambda: scene.sphere_scene(2000, 1500, n_src=4, seed=1234, n_waves=24), 500, {}),
    "c2-pinhole-1600x1200-v10": (lambda: scene.pinhole_scene(1600, 1200, n_src=10, seed=1234, n_waves=12), 300, {}),
    "c3-sphere-3200x1600-v15": (lambda: scene.sphere_scene(3200, 1600, n_src=15, seed=1234, n_waves=12), 200,
                                {"ACMMP_NB_VIEW_CHUNK": "8"}),
    "c5-pinhole-1920x1080-v20": (lambda: scene.pinhole_scene(1920, 1080, n_src=20, seed=55, n_waves=12), 150, {}),
    "pinhole-640x480-v32": (lambda: scene.pinhole_scene(640, 480, n_src=32, seed=32, n_waves=24), 100, {}),
    "sphere-640x320-v32": (lambda: scene.sphere_scene(640, 320, n_src=32, seed=33, n_waves=24), 100, {}),
}


@pytest.fixture(scope="module", params=list(CONFIGS))
def config(request):
    make, nq, env = CONFIGS[request.param]
    sc = make()
    return request.param, sc, nq, env


@pytest.mark.slow
def test_fast_mode_tolerance_at_baseline_configs(ctx, config, monkeypatch):
    name, sc, nq, env = config
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    sphere = name.startswith(("metric", "c3", "sphere"))
    p = params_for(sc)
    check_t1(ctx, sc, p, nq, seed=len(name), sphere=sphere)
    setup = plain_setup(sc, p)
    H, W = sc.images[0].shape
    report = {}
    if sphere and ni.interp_enabled(W, H, p):
        # T2 of the per-sample fast arithmetic against its floor, then the interpolated coordinates (k_eval_nb,
        # and k_eval_ref above 4 views) over four seeds: mean same-plane >= 98.5% and within 0.2 pt of the
        # per-sample arithmetic's mean, every seed's flips near ties (median cost gap < 3e-5)
        seeds = (81, 82, 83, 84)
        per_sample, interpolated = [], []
        for k, seed in enumerate(seeds):
            monkeypatch.setenv("ACMMP_INTERP", "0")
            per_sample.append(check_t2(ctx, setup, seed, sphere, init=k == 0))
            monkeypatch.delenv("ACMMP_INTERP")
            interpolated.append(check_t2(ctx, setup, seed, sphere, init=False, hs_min=0.0, gap_max=3e-5))
        ps_mean = float(np.mean([r[0] for r in per_sample]))
        ip_mean = float(np.mean([r[0] for r in interpolated]))
        assert ip_mean >= 0.985 and ip_mean >= ps_mean - 0.002, (ip_mean, ps_mean)
        # and no seed far below its per-sample run (a mean can hide one seed's regression)
        for seed, a, b in zip(seeds, per_sample, interpolated):
            assert b[0] >= a[0] - 0.005, (seed, b[0], a[0])
        for seed, a, b in zip(seeds, per_sample, interpolated):
            report[f"per_sample_seed{seed}"] = a
            report[f"interpolated_seed{seed}"] = b
        report["per_sample_mean"] = (ps_mean, float(np.median([r[1] for r in per_sample])))
        report["interpolated_mean"] = (ip_mean, float(np.median([r[1] for r in interpolated])))
    else:
        report["per_sample"] = check_t2(ctx, setup, 81, sphere)
    check_t3(ctx, setup, 82, sc.gt_depth)
    out_dir = os.environ.get("ACMMP_TEST_REPORT_DIR")
    if out_dir:
        os.makedirs(out_dir, exist_ok=True)
        with open(os.path.join(out_dir, f"fastmath_t2_{name}.json"), "w") as fh:
            json.dump({k: {"same_plane": v[0], "flip_median_cost_gap": v[1]} for k, v in report.items()}, fh, indent=1)


PASS_RIGS = {"pinhole": lambda: scene.pinhole_scene(800, 600, n_src=10, seed=61, n_waves=24),
             "sphere": lambda: scene.sphere_scene(1000, 500, n_src=6, seed=62, n_waves=24),
             # the interpolated coordinates (k_eval_nb, and k_eval_ref above 4 views) in every pass kind
             "sphere-interp": lambda: scene.sphere_scene(2000, 1000, n_src=6, seed=63, n_waves=24)}


def make_pass_rig(ctx, name):
    """A random first pass in the exact mode: the state the geom / planar / hierarchy passes start from."""
    sc = PASS_RIGS[name]()
    H, W = sc.images[0].shape
    V = len(sc.images) - 1
    p0 = params_for(sc)
    ctx.set_math("exact")
    ctx.set_params(p0)
    ctx.upload_views(sc.images, sc.cameras)
    ctx.run_patchmatch(70)
    first_p, first_c = ctx.download()
    rng = np.random.default_rng(71)
    depths = [first_p[..., 3]] + [(sc.gt_depth * rng.uniform(0.98, 1.02, (H, W))).astype(np.float32)
                                  for _ in range(V)]
    ctx.set_state(first_p, first_c)
    ctx.set_planar_prior_from_maps(first_p[..., 3], first_c, float(p0["depth_min"]), float(p0["depth_max"]))
    prior, masks = ctx.download_planar_prior()
    return name, sc, first_p, first_c, depths, prior, masks


@pytest.fixture(scope="module", params=list(PASS_RIGS))
def pass_rig(request, ctx):
    return make_pass_rig(ctx, request.param)


# After one half-sweep of a geom / planar / hierarchy pass from the shared first-pass state, the share of pixels
# whose fast-mode plane equals the exact mode's, over seeds 72-75 (scripts/pass_gates.py,
# profiles/r06_pass_gates.json): the floor is the measured four-seed mean - 0.5 pt per (rig, pass kind), and each
# seed's share must hold it.  In the geom pass a flip is still decided by cost (the geometric term is added to it,
# ACMMP.cu:1210-1228), so its median |cost gap| is gated too; the planar (prior-restricted acceptance by restricted
# cost, :1247-1299) and hierarchy (pre-cost gate, :1315-1324) flips are not cost ties and their gap is not a tie
# measure.
PASS_SEEDS = (72, 73, 74, 75)
PASS_FLOORS = {}              # (rig, kind) -> same-plane floor; filled from profiles/r06_pass_gates.json below
GEOM_GAP_MAX = {}             # rig -> median flip cost gap bound of the geom pass


def _load_pass_gates():
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "r06_pass_gates.json")
    if not os.path.exists(path):
        return
    d = json.load(open(path))
    for rig, kinds in d["measured"].items():
        for kind, m in kinds.items():
            PASS_FLOORS[(rig, kind)] = round(m["same_plane_mean"] - 0.005, 4)
            if kind == "geom":
                GEOM_GAP_MAX[rig] = m["gap_bound"]


_load_pass_gates()


def pass_setup(kind, sc, first_p, first_c, depths, prior, masks):
    H, W = sc.images[0].shape
    if kind == "geom":
        def setup(c):
            c.set_params(params_for(sc, geom_consistency=1, max_iterations=2))
            c.upload_views(sc.images, sc.cameras)
            c.upload_depths(depths)
            c.set_state(first_p, first_c)
    elif kind == "planar":
        def setup(c):
            c.set_params(params_for(sc, planar_prior=1))
            c.upload_views(sc.images, sc.cameras)
            c.set_state(first_p, first_c)
            c.set_planar_prior(prior, masks)
    else:
        h, w = H // 2, W // 2
        coarse = np.zeros((h, w, 4), np.float32)
        coarse[..., :3] = first_p[::2, ::2, :3][:h, :w]
        coarse[..., 3] = first_c[::2, ::2][:h, :w]
        cur = np.zeros((H, W, 4), np.float32)
        cur[..., 3] = first_p[..., 3]
        zc = np.zeros((H, W), np.float32)

        def setup(c):
            c.set_params(params_for(sc, hierarchy=1, upsample=1, scaled_cols=w, scaled_rows=h))
            c.upload_views(sc.images, sc.cameras)
            c.set_state(cur, zc)
            c.set_scaled_state(coarse)
    return setup


@pytest.mark.parametrize("kind", ["geom", "planar", "hierarchy"])
def test_fast_mode_tolerance_in_geom_planar_hierarchy_passes(ctx, pass_rig, kind):
    rig, sc, first_p, first_c, depths, prior, masks = pass_rig
    setup = pass_setup(kind, sc, first_p, first_c, depths, prior, masks)
    sphere = rig.startswith("sphere")
    floor = PASS_FLOORS.get((rig, kind), 0.85)
    gap_max = GEOM_GAP_MAX.get(rig) if kind == "geom" else None
    got = []
    for k, seed in enumerate(PASS_SEEDS):
        got.append(check_t2(ctx, setup, seed, sphere, init=k == 0, hs_min=floor, gap_max=gap_max))
    check_t3(ctx, setup, 73, sc.gt_depth)
    out_dir = os.environ.get("ACMMP_TEST_REPORT_DIR")
    if out_dir:
        os.makedirs(out_dir, exist_ok=True)
        with open(os.path.join(out_dir, f"pass_t2_{rig}_{kind}.json"), "w") as fh:
            json.dump({"floor": floor, "gap_max": gap_max, "seeds": list(PASS_SEEDS),
                       "same_plane": [g[0] for g in got], "flip_median_cost_gap": [g[1] for g in got]}, fh, indent=1)


def test_fast_mode_is_deterministic(ctx):
    sc = scene.sphere_scene(640, 320, n_src=4, seed=3)
    setup = plain_setup(sc, params_for(sc))
    a = run(ctx, "fast", 21, setup=setup)
    b = run(ctx, "fast", 21, setup=setup)
    assert np.array_equal(a[0], b[0], equal_nan=True) and np.array_equal(a[1], b[1], equal_nan=True)


@pytest.mark.parametrize("shape", [(2000, 1500, 4, None, False), (2000, 1000, 4, None, False),
                                   (2000, 1000, 6, None, False), (2000, 1000, 10, "4", False),
                                   (2000, 1000, 6, None, True)])
def test_deferred_interpolation_fallbacks_are_per_sample_bit_exact(ctx, shape, monkeypatch):
    """k_eval_nb queues the (pixel, hypothesis, view) entries whose interpolation nodes spread too far
    (ncc_chunk) and k_nb_fix recomputes them with every sample projected; k_eval_ref's interpolated instance
    (V > 4) leaves its such views to k_eval_ref_tail, which recomputes them the same way and restarts the
    candidate's chain.  With ACMMP_SPREAD_MAX=-1 every entry falls back, so a full fast-mode RunPatchMatch must be
    the per-sample fast run (ACMMP_INTERP=0) bit for bit: at V = 4 (only k_eval_nb interpolates), V = 6 and 10
    (the refinement too; split at 4 / 8 views), k_eval_nb view-chunked below V (the queue emptied per chunk), and
    in a geom pass."""
    W, H, V, chunk, geom = shape
    sc = scene.sphere_scene(W, H, n_src=V, seed=71, n_waves=16)
    if chunk:
        monkeypatch.setenv("ACMMP_NB_VIEW_CHUNK", chunk)
    if geom:
        rng = np.random.default_rng(72)
        depths = [(sc.gt_depth * rng.uniform(0.98, 1.02, (H, W))).astype(np.float32) for _ in range(V + 1)]
        p0 = params_for(sc)
        ctx.set_math("exact")
        ctx.set_params(p0)
        ctx.upload_views(sc.images, sc.cameras)
        ctx.run_patchmatch(70, n_half_sweeps=2)
        first_p, first_c = ctx.download()

        def setup(c):
            c.set_params(params_for(sc, geom_consistency=1, max_iterations=2))
            c.upload_views(sc.images, sc.cameras)
            c.upload_depths(depths)
            c.set_state(first_p, first_c)
    else:
        setup = plain_setup(sc, params_for(sc))
    monkeypatch.setenv("ACMMP_SPREAD_MAX", "-1")
    a = run(ctx, "fast", 5, setup=setup)
    monkeypatch.delenv("ACMMP_SPREAD_MAX")
    monkeypatch.setenv("ACMMP_INTERP", "0")
    b = run(ctx, "fast", 5, setup=setup)
    monkeypatch.delenv("ACMMP_INTERP")
    c = run(ctx, "fast", 5, setup=setup)
    np.testing.assert_array_equal(a[0].view(np.uint32), b[0].view(np.uint32))
    np.testing.assert_array_equal(a[1].view(np.uint32), b[1].view(np.uint32))
    assert not np.array_equal(c[1].view(np.uint32), b[1].view(np.uint32))     # the product interpolates


def test_no_interpolation_without_the_fallback_queue(ctx, monkeypatch):
    """The fallback queue's key holds the colour-grid pixel in 24 bits; a larger grid (views of 8192x4096 and up)
    gets no queue, and then nothing interpolates (capi.cpp build_kparams).  ACMMP_NBFIX_MAX_PC=1 forces that
    branch at 2000x1000: the fast run must equal the per-sample fast run (ACMMP_INTERP=0) bit for bit, and
    k_eval_nb's hook the per-sample hook."""
    sc = scene.sphere_scene(2000, 1000, n_src=4, seed=73, n_waves=16)
    p = params_for(sc)
    setup = plain_setup(sc, p)
    monkeypatch.setenv("ACMMP_NBFIX_MAX_PC", "1")
    a = run(ctx, "fast", 9, n_hs=2, setup=setup)
    rng = np.random.default_rng(5)
    px = rng.integers(10, 1990, 64).astype(np.int32)
    py = rng.integers(10, 300, 64).astype(np.int32)
    planes = ni.near_surface_planes(sc, px, py, 8, seed=6)
    ctx.set_params(p)
    ctx.upload_views(sc.images, sc.cameras)
    ctx.set_math("fast")
    nb_capped = ctx.debug_ncc_nb(px, py, planes)
    ps = ctx.debug_ncc(np.repeat(px, 8), np.repeat(py, 8), planes.reshape(-1, 4)).reshape(nb_capped.shape)
    monkeypatch.delenv("ACMMP_NBFIX_MAX_PC")
    ctx.set_params(p)
    nb = ctx.debug_ncc_nb(px, py, planes)
    ctx.set_math("exact")
    monkeypatch.setenv("ACMMP_INTERP", "0")
    b = run(ctx, "fast", 9, n_hs=2, setup=setup)
    monkeypatch.delenv("ACMMP_INTERP")
    np.testing.assert_array_equal(a[0].view(np.uint32), b[0].view(np.uint32))
    np.testing.assert_array_equal(a[1].view(np.uint32), b[1].view(np.uint32))
    np.testing.assert_array_equal(nb_capped.view(np.uint32), ps.view(np.uint32))
    assert np.any(nb.view(np.uint32) != ps.view(np.uint32))              # uncapped, it interpolates
