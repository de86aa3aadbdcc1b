"""The C++ host drop-in (acmmp-spherical_amd/host): the reference's `ACMMP dense_folder` executable
(main.cpp) over the C ABI, with its readers (ReadCamera, dmb, pair.txt), cv::imread restated by a
baseline JPEG decoder, and cv::resize(INTER_LINEAR).

Pins:
  * the JPEG decoder equals libjpeg-turbo (the decoder OpenCV's imread uses; here as bundled with
    PIL) bit for bit -- grey (IMREAD_GRAYSCALE: the luma plane) and colour (IMREAD_COLOR: fancy
    chroma upsampling + the fixed-point YCbCr->RGB, BGR order) over 4:4:4 / 4:2:2 / 4:2:0, odd
    sizes, restart markers;
  * the C++ resizers / ReadCamera / rounding equal the Python restatements the pipeline uses;
  * on the GPU, the C++ driver's dmb files and PLY equal the Python pipeline's (order "reference",
    same seeds) bit for bit on a dense folder.
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from acmmp import io, pipeline, scene, types

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(os.path.dirname(HERE), "acmmp-spherical_amd")


@pytest.fixture(scope="module")
def host():
    import sys
    sys.path.insert(0, PKG)
    import build
    lib, exe = build.build_host()
    return ctypes.CDLL(lib), exe


def decode(lib, path, color):
    w, h, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    err = ctypes.create_string_buffer(256)
    buf = np.zeros(8 << 20, np.uint8)
    r = lib.acmmp_host_decode_jpeg(str(path).encode(), int(color), buf.ctypes.data_as(ctypes.c_void_p),
                                   ctypes.c_longlong(buf.size), ctypes.byref(w), ctypes.byref(h), ctypes.byref(c), err, 256)
    if r != 0:
        raise ValueError(err.value.decode())
    return buf[:w.value * h.value * c.value].reshape(h.value, w.value, c.value).copy()


def pil_gray(path):
    from PIL import Image
    with Image.open(path) as im:
        im.draft("L", im.size)
        return np.asarray(im.convert("L"))


def pil_bgr(path):
    from PIL import Image
    with Image.open(path) as im:
        return np.asarray(im.convert("RGB"))[..., ::-1]


def synthetic_rgb(rng, W, H):
    x = np.linspace(0, 6, W)[None, :]
    y = np.linspace(0, 4, H)[:, None]
    base = 127 + 80 * np.sin(x * rng.uniform(0.5, 3) + y * rng.uniform(0.5, 3))
    rgb = np.stack([base + rng.normal(0, 25, (H, W)), 0.7 * base + rng.normal(0, 25, (H, W)),
                    255 - base + rng.normal(0, 25, (H, W))], -1)
    return np.clip(rgb, 0, 255).astype(np.uint8)


@pytest.mark.parametrize("mode", ["gray", "444", "422", "420"])
def test_jpeg_decoder_equals_libjpeg_turbo(host, tmp_path, mode):
    from PIL import Image
    lib, _ = host
    rng = np.random.default_rng({"gray": 1, "444": 2, "422": 3, "420": 4}[mode])
    sizes = [(1, 1), (2, 3), (3, 2), (5, 7), (17, 9), (16, 16), (33, 31), (250, 120), (119, 187)]
    for k, (W, H) in enumerate(sizes):
        rgb = synthetic_rgb(rng, W, H)
        q = int(rng.integers(20, 101))
        p = tmp_path / f"{mode}_{k}.jpg"
        kw = {"quality": q}
        if k % 3 == 1:
            kw["restart_marker_blocks"] = 2                            # DRI + RSTn markers
        if mode == "gray":
            Image.fromarray(rgb[..., 0], "L").save(p, **kw)
        else:
            Image.fromarray(rgb, "RGB").save(p, subsampling={"444": 0, "422": 1, "420": 2}[mode], **kw)
        g = decode(lib, p, 0)[..., 0]
        c = decode(lib, p, 1)
        assert np.array_equal(g, pil_gray(p)), (mode, W, H, q)
        assert np.array_equal(c, pil_bgr(p)), (mode, W, H, q)


def test_jpeg_decoder_refuses_progressive_and_garbage(host, tmp_path):
    from PIL import Image
    lib, _ = host
    p = tmp_path / "prog.jpg"
    Image.fromarray(synthetic_rgb(np.random.default_rng(0), 40, 30)).save(p, progressive=True)
    with pytest.raises(ValueError, match="progressive"):
        decode(lib, p, 0)
    bad = tmp_path / "bad.jpg"
    bad.write_bytes(b"not a jpeg")
    with pytest.raises(ValueError):
        decode(lib, bad, 0)
    with pytest.raises(ValueError):
        decode(lib, tmp_path / "missing.jpg", 0)


def test_jpeg_decoder_rejects_malformed_tables(host, tmp_path):
    """Malformed segments fail with an error instead of writing past the decoder's tables (libjpeg's
    JERR_BAD_HUFF_TABLE / truncated DQT / short DRI / non-integral sampling ratios)."""
    from PIL import Image
    lib, _ = host
    p = tmp_path / "ok.jpg"
    Image.fromarray(synthetic_rgb(np.random.default_rng(1), 48, 32), "RGB").save(p, subsampling=2, quality=80)
    good = p.read_bytes()
    assert decode(lib, p, 1).shape == (32, 48, 3)

    def with_segment(marker, payload):
        seg = bytes([0xFF, marker]) + (len(payload) + 2).to_bytes(2, "big") + payload
        return good[:2] + seg + good[2:]

    cases = {
        # DC table 0 with three 1-bit codes (only two exist): oversubscribed
        "dht_over": with_segment(0xC4, bytes([0x00, 3] + [0] * 15) + bytes([0, 1, 2])),
        # 255 one-bit codes
        "dht_255": with_segment(0xC4, bytes([0x10, 255] + [0] * 15) + bytes(range(255))),
        # a complete length-1 table uses the all-ones code, which T.81 forbids
        "dht_all_ones": with_segment(0xC4, bytes([0x00, 2] + [0] * 15) + bytes([0, 1])),
        "dqt_truncated": with_segment(0xDB, bytes([0x00]) + bytes(10)),
        "dqt16_truncated": with_segment(0xDB, bytes([0x10]) + bytes(64)),
        "dri_short": with_segment(0xDD, b""),
    }
    sof = good.index(b"\xff\xc0")
    bad_sf = bytearray(good)
    assert bad_sf[sof + 9] == 3                                  # three components
    bad_sf[sof + 11] = 0x32                                      # Y: h=3 v=2 with Cb/Cr h=1 ok, so
    bad_sf[sof + 14] = 0x21                                      # Cb: h=2 -> hmax 3 % 2 != 0
    cases["sampling"] = bytes(bad_sf)
    expect = {"dht_over": "bad DHT", "dht_255": "bad DHT", "dht_all_ones": "bad DHT", "dqt_truncated": "bad DQT",
              "dqt16_truncated": "bad DQT", "dri_short": "bad DRI", "sampling": "unsupported sampling factors"}
    for name, data in cases.items():
        q = tmp_path / f"{name}.jpg"
        q.write_bytes(data)
        with pytest.raises(ValueError, match=expect[name]):
            decode(lib, q, 1)
    # a valid table (codes 0, 10, 110) is still accepted by the parser
    ok = with_segment(0xC4, bytes([0x01, 1, 1, 1] + [0] * 13) + bytes([0, 1, 2]))
    q = tmp_path / "dht_ok.jpg"
    q.write_bytes(ok)
    assert decode(lib, q, 1).shape == (32, 48, 3)


def test_resize_and_dims_equal_python_restatement(host):
    lib, _ = host
    rng = np.random.default_rng(7)
    for (h, w, nh, nw) in [(48, 64, 24, 32), (37, 53, 19, 27), (20, 30, 41, 61), (9, 9, 9, 9), (101, 77, 50, 38)]:
        img = rng.uniform(0, 255, (h, w)).astype(np.float32)
        out = np.zeros((nh, nw), np.float32)
        lib.acmmp_host_resize_linear(img.ctypes.data_as(ctypes.c_void_p), w, h, out.ctypes.data_as(ctypes.c_void_p), nw, nh)
        assert np.array_equal(out, pipeline.resize_linear(img, nw, nh))
        bgr = rng.integers(0, 256, (h, w, 3)).astype(np.uint8)
        o8 = np.zeros((nh, nw, 3), np.uint8)
        lib.acmmp_host_resize_linear_u8(bgr.ctypes.data_as(ctypes.c_void_p), w, h, o8.ctypes.data_as(ctypes.c_void_p), nw, nh)
        assert np.array_equal(o8, pipeline.resize_linear_u8(bgr, nw, nh))
    # std::round (half away from zero) of the float32 product: 1501 * 0.5 = 750.5 -> 751
    for rows, cols, size in [(1501, 2000, 1000), (1501, 3001, 1500), (1080, 1920, 1000), (1500, 2000, 1000), (2133, 3200, 1600),
                             (4000, 6000, 3200), (1199, 1601, 800)]:
        r, c = ctypes.c_int(), ctypes.c_int()
        lib.acmmp_host_scaled_dims(rows, cols, size, ctypes.byref(r), ctypes.byref(c))
        assert (r.value, c.value) == pipeline.round_dims(rows, cols, size)
    assert pipeline.round_dims(1501, 2000, 1000) == (751, 1000)


def test_read_camera_equals_python_reader(host, tmp_path):
    lib, _ = host
    sc = scene.sphere_scene(64, 32, n_src=1, seed=3)
    pin = scene.pinhole_scene(48, 32, n_src=1, seed=3) if hasattr(scene, "pinhole_scene") else None
    cams = [sc.cameras[0], sc.cameras[1]] + ([pin.cameras[0]] if pin is not None else [])
    for k, cam in enumerate(cams):
        path = tmp_path / f"{k:08d}_cam.txt"
        interval = float(cam["depth_max"]) if int(cam["model"]) == types.PINHOLE else 0.25
        io.write_camera(str(path), cam, depth_interval=interval)
        ref = io.read_camera(str(path))
        out = np.zeros((), types.CAMERA_DTYPE)
        lib.acmmp_host_read_camera(str(path).encode(), out.ctypes.data_as(ctypes.c_void_p))
        assert out.tobytes() == ref.tobytes(), k


def test_driver_builds_and_fails_loudly_without_gpu(host, tmp_path):
    """The executable links libacmmp.so; with no HIP device it stops like CUDA_SAFE_CALL."""
    import torch
    _, exe = host
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode != 0 and "USAGE: ACMMP dense_folder" in r.stdout
    if torch.cuda.device_count() > 0:
        return
    ds = pipeline.Dataset({0: np.full((16, 24), 100.0, np.float32), 1: np.full((16, 24), 90.0, np.float32)},
                          {i: types.make_camera(types.SPHERE, params=[1, 12, 8], width=24, height=16, depth_min=1,
                                                depth_max=2) for i in range(2)},
                          [io.Problem(0, [1]), io.Problem(1, [0])])
    pipeline.write_dense_folder(str(tmp_path), ds)
    r = subprocess.run([exe, str(tmp_path)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 1 and "no HIP device" in r.stdout


def _dense_folder(tmp_path, model):
    if model == "sphere":
        sc = scene.sphere_scene(192, 96, n_src=2, seed=21)
    else:
        sc = scene.pinhole_scene(160, 120, n_src=2, seed=21)
    n = len(sc.images)
    ds = pipeline.Dataset({i: np.asarray(sc.images[i], np.float32) for i in range(n)},
                          {i: np.array(sc.cameras[i], copy=True) for i in range(n)},
                          [io.Problem(i, [j for j in range(n) if j != i]) for i in range(n)])
    pipeline.write_dense_folder(str(tmp_path), ds, quality=92)
    return n


@pytest.mark.gpu
@pytest.mark.parametrize("model", ["sphere", "pinhole"])
def test_gpu_cpp_driver_equals_python_pipeline(host, tmp_path, model):
    """`ACMMP dense_folder` (C++) and `python -m acmmp.pipeline dense_folder` on copies of the same
    folder: every dmb the schedule writes and the fused PLY are byte-identical (two scales)."""
    import shutil
    import sys
    _, exe = host
    a, b = tmp_path / "cpp", tmp_path / "py"
    n = _dense_folder(a, model)
    shutil.copytree(a, b)
    env = dict(os.environ, PYTHONPATH=PKG)
    ra = subprocess.run([exe, str(a), "--seed", "99", "--size-bound", "100"], capture_output=True, text=True,
                        timeout=300, env=env)
    assert ra.returncode == 0, ra.stdout[-3000:] + ra.stderr[-2000:]
    rb = subprocess.run([sys.executable, "-m", "acmmp.pipeline", str(b), "--seed", "99", "--size-bound", "100"],
                        capture_output=True, text=True, env=env, timeout=300)
    assert rb.returncode == 0, rb.stdout[-3000:] + rb.stderr[-2000:]
    compared = 0
    for v in range(n):
        for f in ("depths.dmb", "depths_geom.dmb", "normals.dmb", "costs.dmb"):
            fa = a / "ACMMP" / f"2333_{v:08d}" / f
            fb = b / "ACMMP" / f"2333_{v:08d}" / f
            assert fa.exists() and fb.exists(), f
            assert fa.read_bytes() == fb.read_bytes(), (v, f)
            compared += 1
    pa, pb = a / "ACMMP" / "ACMM_model_cuda_5.ply", b / "ACMMP" / "ACMM_model_cuda_5.ply"
    assert pa.read_bytes() == pb.read_bytes()
    assert io.read_ply(str(pa)).shape[0] > 0 and compared == 4 * n
