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
    "c3-3200x1600-v15": (lambda: scene.sphere_scene(3200, 1600, n_src=15, seed=1234, n_waves=12), 2),
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
