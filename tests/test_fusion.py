"""Fusion: RunFusionCuda / SimpleFusionKernel (ACMMP.cu:1662-2105), the PLY
writer (ACMMP.cpp:481-534) and RescaleImageAndCamera's 8-bit resize (ACMMP.cpp:213-246)."""
import numpy as np
import pytest

from acmmp import io, pipeline, types
from conftest import assert_bitwise_equal
from pipeline_support import OracleEngine, OracleFusion, small_dataset


def test_ply_roundtrip_and_quirks(tmp_path):
    pts = np.array([[1, 2, 3, 0, 0, 1, 10.9, 200.2, 255.0],
                    [np.inf, 2, 3, 0, 1, 0, 0, 0, 0],
                    [1, 2, -np.float32(np.finfo(np.float32).max), 1, 0, 0, 300.0, -1.5, 128.0]], np.float32)
    path = tmp_path / "m.ply"
    io.write_ply(str(path), pts)
    head = open(path, "rb").read(400)
    assert head.startswith(b"ply\nformat binary_little_endian 1.0\nelement vertex 3\n")
    r = io.read_ply(str(path))
    assert r.shape == (3,)
    assert (r["x"][0], r["y"][0], r["z"][0]) == (1, 2, 3)
    assert (r["r"][0], r["g"][0], r["b"][0]) == (255, 200, 10)         # red = c2, blue = c0, truncated
    assert (r["x"][1], r["y"][1], r["z"][1]) == (0, 0, 0)               # non-finite -> 0
    assert r["z"][2] == -np.finfo(np.float32).max                       # z >= -FLT_MAX kept (:511)
    assert (r["r"][2], r["g"][2], r["b"][2]) == (128, 255, 300 & 255)   # (char)(int) wraps


def test_resize_u8_constant_and_identity():
    img = np.full((20, 30, 3), 77, np.uint8)
    assert np.array_equal(pipeline.resize_linear_u8(img, 15, 10), np.full((10, 15, 3), 77, np.uint8))
    ramp = (np.arange(40, dtype=np.uint8)[None, :] * 6)[..., None].repeat(3, 2).repeat(8, 0)
    half = pipeline.resize_linear_u8(ramp, 20, 4)
    exp = ((ramp[0, 0::2, 0].astype(int) + ramp[0, 1::2, 0]) + 1) // 2
    assert np.array_equal(half[0, :, 0], exp.astype(np.uint8))


def test_rescale_image_and_camera():
    cam = types.make_camera(types.PINHOLE, K=[[100, 0, 50], [0, 100, 40], [0, 0, 1]], width=100, height=80)
    img = np.zeros((80, 100, 3), np.uint8)
    out, c = pipeline.rescale_image_and_camera(img, (40, 50), cam)
    assert out.shape == (40, 50, 3) and (c["width"], c["height"]) == (50, 40)
    assert c["K"][0] == np.float32(50) and c["K"][5] == np.float32(20)
    same, c2 = pipeline.rescale_image_and_camera(img, (80, 100), cam)
    assert same.shape == img.shape and c2["K"][0] == 100


def _gt_fusion_inputs(W=256, H=128, n=3):
    from acmmp import scene
    sc = scene.sphere_scene(W, H, n_src=n - 1, seed=3)
    bgr = [np.repeat(np.asarray(im, np.uint8)[..., None], 3, 2) for im in sc.images]
    return sc, np.array(sc.cameras), sc.extra["gt_depths"], sc.extra["gt_normals"], bgr


def test_fusion_of_ground_truth_maps_keeps_the_room():
    """On exact depth/normal maps of a convex room every pixel is seen by every view; most fuse (the
    1 px / 1% tests against the rounded source pixel reject grazing and seam pixels, as in the
    reference), onto the room's walls, with the wall normals."""
    sc, cams, depths, normals, bgr = _gt_fusion_inputs()
    fu = OracleFusion(cams)
    for k in range(len(cams)):
        fu.set_view(k, depths[k], normals[k], bgr[k])
    pts = fu.run(0, [1, 2])
    H, W = depths[0].shape
    assert pts.shape[0] > 0.7 * H * W
    half = np.array([5.0, 3.0, 4.0])
    on_wall = np.min(np.abs(np.abs(pts[:, :3]) - half[None, :]), axis=1)
    assert np.percentile(on_wall, 99) < 0.02
    assert np.mean(np.abs(np.abs(pts[:, 3:6]).max(1) - 1) < 1e-3) > 0.95


def test_pipeline_fusion_with_oracle_writes_ply(tmp_path):
    ds = small_dataset(64, 32, 3)
    pipe = pipeline.Pipeline(ds, engine=OracleEngine(), order="reference", geom_iterations=1,
                             out_folder=str(tmp_path))
    pipe.run()
    pts = pipe.run_fusion(fusion_factory=OracleFusion)
    assert pts.shape[0] > 0
    ply = io.read_ply(str(tmp_path / "ACMMP" / "ACMM_model_cuda_5.ply"))
    assert ply.shape[0] == pts.shape[0]
    nrm = np.linalg.norm(pts[:, 3:6], axis=1)
    assert np.allclose(nrm, 1, atol=1e-4)
    assert np.isfinite(pts).all()


@pytest.mark.gpu
def test_gpu_fusion_ground_truth_bitexact_vs_oracle():
    from acmmp import capi
    sc, cams, depths, normals, bgr = _gt_fusion_inputs(512, 256, 4)
    gf, of = capi.Fusion(0, cams), OracleFusion(cams)
    for k in range(len(cams)):
        gf.set_view(k, depths[k], normals[k], bgr[k])
        of.set_view(k, depths[k], normals[k], bgr[k])
    for k in range(len(cams)):
        srcs = [j for j in range(len(cams)) if j != k]
        g, o = gf.run(k, srcs), of.run(k, srcs)
        assert g.shape == o.shape and g.shape[0] > 0.7 * 512 * 256
        assert_bitwise_equal(g, o, f"view {k}")
    gf.close()


@pytest.mark.gpu
def test_gpu_fusion_bitexact_vs_oracle():
    from acmmp import capi
    ds = small_dataset(64, 32, 3)
    pipe = pipeline.Pipeline(ds, order="reference", geom_iterations=1).run()
    cams, depths, normals, colours = pipeline.fusion_inputs(ds, pipe.store, pipe.problems)
    gf, of = capi.Fusion(0, cams), OracleFusion(cams)
    for k in range(len(cams)):
        gf.set_view(k, depths[k], normals[k], colours[k])
        of.set_view(k, depths[k], normals[k], colours[k])
    total = 0
    for k in range(len(cams)):
        srcs = [j for j in range(len(cams)) if j != k] + [-1]
        g, o = gf.run(k, srcs), of.run(k, srcs)
        assert g.shape == o.shape
        assert_bitwise_equal(g, o, f"view {k}")
        total += g.shape[0]
    assert total > 0
    gf.close()
