"""Per-query parity of the headline arithmetic: the fast SPHERE k_eval_nb with interpolated source coordinates
(kernels.hip ncc_chunk's interpolated loop), queried through acmmp_debug_ncc_nb, which runs
k_eval_nb's own staging and NCC instance.  The reference projects every sample, --use_fast_math or not
(ComputeBilateralNCC, ACMMP.cu:450-476), so the interpolation is held against:

  * the float64 per-sample restatement (np_reference.bilateral_ncc) and the float64 interpolated one
    (np_interp.ncc with the kernel's nodes), under T1's gates of test_gpu_fastmath.py with the interpolated
    costs in place of the per-sample fast ones;
  * the same engine's per-sample fast and exact NCC (acmmp_debug_ncc), and k_eval_nb's exact instance,
    which must equal the per-sample exact hook bit for bit (same staging, exact mode = the oracle's bits);

on three query sets per configuration: random pixels, pixels whose surface point lands within 10 degrees of
a source camera's pole (where longitude varies fastest over a patch) and pixels landing within 6 source
pixels of a source's longitude seam (the patch straddles x = 0 = W), 8 near-surface planes each (k_eval_nb's
8 hypotheses per pixel).  Configurations: the metric view (2000x1500, V = 4) and C3 (3200x1600, V = 15).

With ACMMP_TEST_REPORT_DIR set, each configuration writes interp_queries_<name>.json there: per query set,
the worst interpolated-vs-per-sample |dcost| and the fractions the gates use.
"""
import json
import os

import numpy as np
import pytest

import np_interp as ni
import np_reference as npr
from acmmp import capi, scene, types

pytestmark = pytest.mark.gpu

CONFIGS = {
    "metric-2000x1500-v4": (lambda: scene.sphere_scene(2000, 1500, n_src=4, seed=1234, n_waves=24), 8),
    # (C3: every plane of each pixel against float64 too -- with 2 of 8 the seam set's T1 fractions moved by up to 0.015
    # between builds of the same per-query accuracy, sampling noise, profiles/r06_nodeh_queries.txt)
    "c3-3200x1600-v15": (lambda: scene.sphere_scene(3200, 1600, n_src=15, seed=1234, n_waves=12), 8),
}
KINDS = {"random": 40, "pole": 32, "seam": 32}


@pytest.fixture(scope="module")
def ctx():
    c = capi.Context(0)
    yield c
    c.close()


def _f64(sc, p, px, py, planes, n_planes, interp):
    V = len(sc.images) - 1
    out = np.full((len(px), n_planes, V), np.nan)
    for q in range(len(px)):
        for h in range(n_planes):
            pl = planes[q, h].astype(np.float64)
            for v in range(1, V + 1):
                if interp:
                    out[q, h, v - 1] = ni.ncc(sc.images, sc.cameras, p, v, int(px[q]), int(py[q]), pl, True,
                                              nodes=ni.NODES, span_max=ni.SPREAD_MAX)[0]
                else:
                    out[q, h, v - 1] = npr.bilateral_ncc(sc.images, sc.cameras, p, v, int(px[q]), int(py[q]), pl)
    return out


@pytest.mark.slow
@pytest.mark.parametrize("name", list(CONFIGS))
def test_interpolated_k_eval_nb_per_query(ctx, name):
    make, n_f64 = CONFIGS[name]
    sc = make()
    c0 = sc.cameras[0]
    p = types.default_params(num_images=len(sc.images), depth_min=float(c0["depth_min"]) * 0.6,
                             depth_max=float(c0["depth_max"]) * 1.2)
    ctx.set_params(p)
    ctx.upload_views(sc.images, sc.cameras)
    report = {}
    for kind, n in KINDS.items():
        px, py, _ = ni.special_pixels(sc, kind, n, seed=len(kind) + 17)
        assert len(px) >= n // 2, (kind, len(px))
        planes = ni.near_surface_planes(sc, px, py, 8, seed=len(kind) + 29)
        flat_x, flat_y = np.repeat(px, 8), np.repeat(py, 8)
        ctx.set_math("fast")
        nb_f = ctx.debug_ncc_nb(px, py, planes)
        ps_f = ctx.debug_ncc(flat_x, flat_y, planes.reshape(-1, 4)).reshape(nb_f.shape)
        ctx.set_math("exact")
        nb_e = ctx.debug_ncc_nb(px, py, planes)
        ps_e = ctx.debug_ncc(flat_x, flat_y, planes.reshape(-1, 4)).reshape(nb_f.shape)
        # k_eval_nb's exact instance is the per-sample exact NCC bit for bit (the oracle's arithmetic)
        np.testing.assert_array_equal(nb_e.view(np.uint32), ps_e.view(np.uint32))
        # the interpolated loop ran (it cannot equal the per-sample fast costs everywhere)
        assert np.any(nb_f != ps_f), kind
        # float64 references on the first n_f64 planes of each pixel
        f, e, pf = nb_f[:, :n_f64], nb_e[:, :n_f64], ps_f[:, :n_f64]
        ref = _f64(sc, p, px, py, planes, n_f64, False)
        refi = _f64(sc, p, px, py, planes, n_f64, True)
        # the design claim in float64: the interpolation moves the NCC by < 1e-4 (and never its class)
        both = (ref < 2.0) & (refi < 2.0)
        assert np.mean((ref >= 2.0) == (refi >= 2.0)) >= 0.995, kind
        f64_interp_max = float(np.abs(refi - ref)[both].max()) if both.any() else 0.0
        assert f64_interp_max < 1e-4, (kind, f64_interp_max)
        # T1 (test_gpu_fastmath.check_t1) with the interpolated costs as the fast ones
        agree_fe = np.mean((f >= 2.0) == (e >= 2.0))
        agree_ef = np.mean((e >= 2.0) == (ref >= 2.0))
        assert agree_fe >= min(agree_ef, 0.999) - 0.002 and agree_fe >= 0.99, (kind, agree_fe, agree_ef)
        valid = (e < 2.0) & (f < 2.0) & (ref < 2.0)
        assert valid.sum() >= 40, (kind, int(valid.sum()))
        df, de, dfe = np.abs(f - ref)[valid], np.abs(e - ref)[valid], np.abs(f - e)[valid]
        assert np.mean(dfe <= 1e-4) >= np.mean(de <= 1e-4) - 0.05, (kind, np.mean(dfe <= 1e-4), np.mean(de <= 1e-4))
        fast_worse, exact_worse = np.mean(df > de + 1e-4), np.mean(de > df + 1e-4)
        assert fast_worse <= exact_worse + 0.03, (kind, fast_worse, exact_worse)
        # against the float64 interpolated restatement: as close as the per-sample fast path is to float64
        dpf = np.abs(pf - ref)[valid]
        dfi = np.abs(f - refi)[valid]
        assert np.mean(dfi <= 1e-4) >= np.mean(dpf <= 1e-4) - 0.03, (kind, np.mean(dfi <= 1e-4), np.mean(dpf <= 1e-4))
        # interpolated vs per-sample, same engine, all 8 planes
        v_all = (nb_f < 2.0) & (ps_f < 2.0)
        d_ip = np.abs(nb_f - ps_f)[v_all]
        agree_ip = float(np.mean((nb_f >= 2.0) == (ps_f >= 2.0)))
        assert agree_ip >= 0.99, (kind, agree_ip)
        report[kind] = {
            "pixels": int(len(px)), "queries": int(nb_f.size), "f64_queries": int(f.size),
            "worst_interp_vs_per_sample_dcost": float(d_ip.max()) if d_ip.size else 0.0,
            "q99_interp_vs_per_sample_dcost": float(np.quantile(d_ip, 0.99)) if d_ip.size else 0.0,
            "frac_interp_vs_per_sample_le_1e-4": float(np.mean(d_ip <= 1e-4)) if d_ip.size else 1.0,
            "class_agree_interp_vs_per_sample": agree_ip,
            "f64_interp_vs_f64_per_sample_max": f64_interp_max,
            "frac_interp_within_1e-4_of_exact": float(np.mean(dfe <= 1e-4)),
            "frac_exact_within_1e-4_of_f64": float(np.mean(de <= 1e-4)),
            "frac_interp_within_1e-4_of_f64_interp": float(np.mean(dfi <= 1e-4)),
            "frac_per_sample_fast_within_1e-4_of_f64": float(np.mean(dpf <= 1e-4)),
            "interp_worse_than_exact_by_1e-4": float(fast_worse), "exact_worse_than_interp_by_1e-4": float(exact_worse),
            "class_agree_interp_vs_exact": float(agree_fe), "class_agree_exact_vs_f64": float(agree_ef),
        }
    out_dir = os.environ.get("ACMMP_TEST_REPORT_DIR")
    if out_dir:
        os.makedirs(out_dir, exist_ok=True)
        with open(os.path.join(out_dir, f"interp_queries_{name}.json"), "w") as fh:
            json.dump(report, fh, indent=1)


PIN_CONFIGS = {
    "c2-pinhole-1600x1200-v10": lambda: scene.pinhole_scene(1600, 1200, n_src=10, seed=1234, n_waves=12),
    "c5-pinhole-1920x1080-v20": lambda: scene.pinhole_scene(1920, 1080, n_src=20, seed=55, n_waves=12),
}


@pytest.mark.parametrize("name", list(PIN_CONFIGS))
def test_pinhole_homogeneous_k_eval_nb_per_query(ctx, name, monkeypatch):
    """The fast pinhole k_eval_nb forms each sample's source point as one homogeneous vector affine in the
    patch offsets (ncc_chunk's kHomog loop) instead of depth -> point -> projection per sample: the same
    point up to rounding.  Held per query against the same kernel with the per-sample projection
    (ACMMP_PIN_HOMOG=0) and the exact mode: class agreement with exact; |fast - exact| <= 1e-4 as often as
    the per-sample fast arithmetic's, within 0.5 pt (T1(b)'s pinhole 99.5% is the per-sample fast mode's
    gate, test_gpu_fastmath.check_t1); and no systematic loss against the float64 per-sample restatement
    (np_reference.bilateral_ncc, ACMMP.cu:405-516) beyond the exact mode's, + 3 pt (T1(c))."""
    sc = PIN_CONFIGS[name]()
    c0 = sc.cameras[0]
    p = types.default_params(num_images=len(sc.images), depth_min=float(c0["depth_min"]) * 0.6,
                             depth_max=float(c0["depth_max"]) * 1.2)
    ctx.set_params(p)
    ctx.upload_views(sc.images, sc.cameras)
    H, W = sc.images[0].shape
    rng = np.random.default_rng(91)
    n = 96
    px = rng.integers(6, W - 6, n).astype(np.int32)
    py = rng.integers(6, H - 6, n).astype(np.int32)
    planes = ni.near_surface_planes(sc, px, py, 8, seed=93)
    ctx.set_math("fast")
    f = ctx.debug_ncc_nb(px, py, planes)
    monkeypatch.setenv("ACMMP_PIN_HOMOG", "0")
    ps = ctx.debug_ncc_nb(px, py, planes)
    monkeypatch.delenv("ACMMP_PIN_HOMOG")
    ctx.set_math("exact")
    e = ctx.debug_ncc_nb(px, py, planes)
    assert np.any(f != ps)                                   # the homogeneous loop ran
    agree_fe = float(np.mean((f >= 2.0) == (e >= 2.0)))
    agree_pe = float(np.mean((ps >= 2.0) == (e >= 2.0)))
    assert agree_fe >= min(agree_pe, 0.999) - 0.002, (agree_fe, agree_pe)
    v = (f < 2.0) & (e < 2.0) & (ps < 2.0)
    assert v.mean() > 0.3
    dfe, dpe = np.abs(f - e)[v], np.abs(ps - e)[v]
    frac_f, frac_p = float(np.mean(dfe <= 1e-4)), float(np.mean(dpe <= 1e-4))
    assert frac_f >= frac_p - 0.005, (frac_f, frac_p)
    # float64 on the first 2 planes of each pixel
    V = len(sc.images) - 1
    ref = np.full((n, 2, V), np.nan)
    for q in range(n):
        for h in range(2):
            for k in range(1, V + 1):
                ref[q, h, k - 1] = npr.bilateral_ncc(sc.images, sc.cameras, p, k, int(px[q]), int(py[q]),
                                                     planes[q, h].astype(np.float64))
    f2, p2, e2 = f[:, :2], ps[:, :2], e[:, :2]
    valid = (f2 < 2.0) & (e2 < 2.0) & (p2 < 2.0) & (ref < 2.0)
    df, dp, de = np.abs(f2 - ref)[valid], np.abs(p2 - ref)[valid], np.abs(e2 - ref)[valid]
    fast_worse, exact_worse = float(np.mean(df > de + 1e-4)), float(np.mean(de > df + 1e-4))
    assert fast_worse <= exact_worse + 0.03, (fast_worse, exact_worse)
    d_fp = np.abs(f - ps)[v]
    report = {"queries": int(f.size), "class_agree_homog_exact": agree_fe, "class_agree_per_sample_exact": agree_pe,
              "frac_homog_within_1e-4_of_exact": frac_f, "frac_per_sample_within_1e-4_of_exact": frac_p,
              "worst_homog_vs_exact": float(dfe.max()), "worst_per_sample_vs_exact": float(dpe.max()),
              "worst_homog_vs_per_sample": float(d_fp.max()),
              "frac_homog_within_1e-4_of_f64": float(np.mean(df <= 1e-4)),
              "frac_per_sample_within_1e-4_of_f64": float(np.mean(dp <= 1e-4)),
              "frac_exact_within_1e-4_of_f64": float(np.mean(de <= 1e-4)),
              "homog_worse_than_exact_by_1e-4": fast_worse, "exact_worse_than_homog_by_1e-4": exact_worse}
    out_dir = os.environ.get("ACMMP_TEST_REPORT_DIR")
    if out_dir:
        os.makedirs(out_dir, exist_ok=True)
        with open(os.path.join(out_dir, f"pinhole_queries_{name}.json"), "w") as fh:
            json.dump(report, fh, indent=1)


@pytest.mark.parametrize("name", list(CONFIGS))
def test_deferred_fallbacks_are_per_sample_bit_exact(ctx, name, monkeypatch):
    """acmmp_debug_ncc_nb runs k_eval_nb's path including the deferred interpolation fallbacks (ncc_chunk
    queues a (pixel, hypothesis, view) whose nodes spread too far; k_debug_nb_fix recomputes it with k_nb_fix's
    code).  A recomputed cost is the per-sample fast NCC (acmmp_debug_ncc) bit for bit.  With the product
    threshold on the pole / seam / random sets, and with ACMMP_SPREAD_MAX=-1, where every entry falls back --
    then every cost must equal the per-sample hook's."""
    make, _ = CONFIGS[name]
    sc = make()
    c0 = sc.cameras[0]
    p = types.default_params(num_images=len(sc.images), depth_min=float(c0["depth_min"]) * 0.6,
                             depth_max=float(c0["depth_max"]) * 1.2)
    ctx.set_params(p)
    ctx.upload_views(sc.images, sc.cameras)
    ctx.set_math("fast")
    for kind, n in KINDS.items():
        px, py, _ = ni.special_pixels(sc, kind, n, seed=len(kind) + 17)
        planes = ni.near_surface_planes(sc, px, py, 8, seed=len(kind) + 29)
        planes[:, 4:] = ni.near_surface_planes(sc, px, py, 4, seed=len(kind) + 31, spread=1.5, depth_jitter=0.4)
        ps = ctx.debug_ncc(np.repeat(px, 8), np.repeat(py, 8), planes.reshape(-1, 4)).reshape(len(px), 8, -1)
        monkeypatch.setenv("ACMMP_SPREAD_MAX", "-1")
        ctx.set_params(p)
        every = ctx.debug_ncc_nb(px, py, planes)
        monkeypatch.delenv("ACMMP_SPREAD_MAX")
        ctx.set_params(p)
        product = ctx.debug_ncc_nb(px, py, planes)
        bad = np.nonzero(every.view(np.uint32) != ps.view(np.uint32))
        assert bad[0].size == 0, (kind, bad[0].size, [(int(a), int(b), int(c), float(every[a, b, c]), float(ps[a, b, c]))
                                                      for a, b, c in zip(*bad)][:5])
        # the product's costs: interpolated or, where it fell back, the per-sample ones (and the interpolation
        # does not equal the per-sample arithmetic everywhere, so the comparison above tested the queue)
        assert np.mean(product.view(np.uint32) != ps.view(np.uint32)) > 0.2, kind
    ctx.set_math("exact")


# ---- the refinement's interpolated NCC (k_eval_ref, SPHERE V > 4) ----------------------------------------

REF_CONFIGS = {
    "c3-3200x1600-v15": (lambda: scene.sphere_scene(3200, 1600, n_src=15, seed=1234, n_waves=12), 2),
    "sphere-2000x1000-v6": (lambda: scene.sphere_scene(2000, 1000, n_src=6, seed=77, n_waves=16), 3),
}


def refinement_planes(sc, px, py, seed):
    """5 planes per pixel shaped like PlaneHypothesisRefinement's candidates (ACMMP.cu:813-874): three near the
    surface (the current plane, its perturbed depth, its perturbed normal) and two random-normal / random-depth
    ones, which are the candidates whose interpolation nodes spread far (grazing planes, depth sign flips)."""
    near = ni.near_surface_planes(sc, px, py, 3, seed=seed)
    far = ni.near_surface_planes(sc, px, py, 2, seed=seed + 1, spread=1.5, depth_jitter=0.4)
    return np.concatenate([near, far], axis=1)


@pytest.mark.slow
@pytest.mark.parametrize("name", list(REF_CONFIGS))
def test_interpolated_refinement_per_query(ctx, name, monkeypatch):
    """acmmp_debug_ncc_ref runs k_eval_ref's staging and NCC instance -- which in the fast mode interpolates SPHERE
    sample coordinates above 4 source views -- and, for the views whose interpolation nodes spread too far, the
    per-sample costs of the production fallback's entry code (queued as k_eval_ref queues them, recomputed by
    k_nb_fix<1, true>'s fix_row / fix_fold).  Held per
    query on the pole / seam / random sets against: the per-sample fast hook (bit for bit where every entry falls
    back, ACMMP_SPREAD_MAX=-1), the exact mode (k_eval_ref's exact instance = the per-sample exact hook bit for
    bit) and float64 (np_reference.bilateral_ncc; T1's gates of test_gpu_fastmath.check_t1)."""
    make, n_f64 = REF_CONFIGS[name]
    sc = make()
    c0 = sc.cameras[0]
    p = types.default_params(num_images=len(sc.images), depth_min=float(c0["depth_min"]) * 0.6,
                             depth_max=float(c0["depth_max"]) * 1.2)
    H, W = sc.images[0].shape
    assert ni.interp_enabled(W, H, p) and len(sc.images) - 1 > 4
    ctx.set_params(p)
    ctx.upload_views(sc.images, sc.cameras)
    report = {}
    for kind, n in KINDS.items():
        px, py, _ = ni.special_pixels(sc, kind, n, seed=len(kind) + 41)
        assert len(px) >= n // 2, (kind, len(px))
        planes = refinement_planes(sc, px, py, seed=len(kind) + 43)
        flat_x, flat_y = np.repeat(px, 5), np.repeat(py, 5)
        ctx.set_math("fast")
        rf = ctx.debug_ncc_ref(px, py, planes)
        ps_f = ctx.debug_ncc(flat_x, flat_y, planes.reshape(-1, 4)).reshape(rf.shape)
        monkeypatch.setenv("ACMMP_SPREAD_MAX", "-1")
        ctx.set_params(p)
        every = ctx.debug_ncc_ref(px, py, planes)
        monkeypatch.delenv("ACMMP_SPREAD_MAX")
        ctx.set_params(p)
        ctx.set_math("exact")
        re_ = ctx.debug_ncc_ref(px, py, planes)
        ps_e = ctx.debug_ncc(flat_x, flat_y, planes.reshape(-1, 4)).reshape(rf.shape)
        assert not np.isnan(rf).any() and not np.isnan(every).any()
        # every entry deferred: the per-sample fast NCC bit for bit (k_nb_fix's arithmetic)
        bad = np.nonzero(every.view(np.uint32) != ps_f.view(np.uint32))
        assert bad[0].size == 0, (kind, bad[0].size)
        # k_eval_ref's exact instance is the per-sample exact NCC bit for bit (the oracle's arithmetic)
        np.testing.assert_array_equal(re_.view(np.uint32), ps_e.view(np.uint32))
        # the interpolated loop ran
        assert np.mean(rf.view(np.uint32) != ps_f.view(np.uint32)) > 0.2, kind
        # float64 on the first n_f64 planes (near-surface) and on the two random candidates
        sel = list(range(n_f64)) + [3, 4]
        f, e, pf = rf[:, sel], re_[:, sel], ps_f[:, sel]
        ref = _f64(sc, p, px, py, planes[:, sel], len(sel), False)
        agree_fe = np.mean((f >= 2.0) == (e >= 2.0))
        agree_ef = np.mean((e >= 2.0) == (ref >= 2.0))
        assert agree_fe >= min(agree_ef, 0.999) - 0.002 and agree_fe >= 0.99, (kind, agree_fe, agree_ef)
        valid = (e < 2.0) & (f < 2.0) & (ref < 2.0)
        assert valid.sum() >= 30, (kind, int(valid.sum()))
        df, de, dfe = np.abs(f - ref)[valid], np.abs(e - ref)[valid], np.abs(f - e)[valid]
        dpf = np.abs(pf - ref)[valid]
        assert np.mean(dfe <= 1e-4) >= np.mean(de <= 1e-4) - 0.05, (kind, np.mean(dfe <= 1e-4), np.mean(de <= 1e-4))
        fast_worse, exact_worse = np.mean(df > de + 1e-4), np.mean(de > df + 1e-4)
        assert fast_worse <= exact_worse + 0.03, (kind, fast_worse, exact_worse)
        # no systematic loss against the per-sample fast arithmetic either (its own distance to float64)
        assert np.mean(df <= 1e-4) >= np.mean(dpf <= 1e-4) - 0.03, (kind, np.mean(df <= 1e-4), np.mean(dpf <= 1e-4))
        v_all = (rf < 2.0) & (ps_f < 2.0)
        d_ip = np.abs(rf - ps_f)[v_all]
        agree_ip = float(np.mean((rf >= 2.0) == (ps_f >= 2.0)))
        assert agree_ip >= 0.99, (kind, agree_ip)
        report[kind] = {
            "pixels": int(len(px)), "queries": int(rf.size), "f64_queries": int(f.size),
            "fell_back_or_equal_frac": float(np.mean(rf.view(np.uint32) == ps_f.view(np.uint32))),
            "worst_interp_vs_per_sample_dcost": float(d_ip.max()) if d_ip.size else 0.0,
            "q99_interp_vs_per_sample_dcost": float(np.quantile(d_ip, 0.99)) if d_ip.size else 0.0,
            "frac_interp_vs_per_sample_le_1e-4": float(np.mean(d_ip <= 1e-4)) if d_ip.size else 1.0,
            "worst_interp_vs_f64": float(df.max()), "worst_per_sample_fast_vs_f64": float(dpf.max()),
            "worst_exact_vs_f64": float(de.max()),
            "frac_interp_within_1e-4_of_f64": float(np.mean(df <= 1e-4)),
            "frac_per_sample_fast_within_1e-4_of_f64": float(np.mean(dpf <= 1e-4)),
            "frac_exact_within_1e-4_of_f64": float(np.mean(de <= 1e-4)),
            "class_agree_interp_vs_per_sample": agree_ip, "class_agree_interp_vs_exact": float(agree_fe),
            "class_agree_exact_vs_f64": float(agree_ef),
        }
    ctx.set_math("exact")
    out_dir = os.environ.get("ACMMP_TEST_REPORT_DIR")
    if out_dir:
        os.makedirs(out_dir, exist_ok=True)
        with open(os.path.join(out_dir, f"refinement_queries_{name}.json"), "w") as fh:
            json.dump(report, fh, indent=1)
