"""COLMAP -> dense-folder converter (colmap2mvsnet_acm.py).

The reference script has no tests or fixtures, so these tests pin the restatement
by its definition on synthetic sparse models written in both COLMAP encodings: text and binary
give byte-identical folders, cam files carry the pose / intrinsics / percentile depth range the
script defines, pair.txt keeps the greedy top-k neighbours by shared tracks, and the folder loads
through the pipeline's readers."""
import os

import numpy as np
import pytest

from acmmp import colmap, io, pipeline, types


def _quat_from_rot(R):
    w = np.sqrt(max(1e-12, 1 + R[0, 0] + R[1, 1] + R[2, 2])) / 2
    return np.array([w, (R[2, 1] - R[1, 2]) / (4 * w), (R[0, 2] - R[2, 0]) / (4 * w), (R[1, 0] - R[0, 1]) / (4 * w)])


def _look_at(C, target):
    z = target - C
    z /= np.linalg.norm(z)
    x = np.cross([0.0, 1.0, 0.0], z)
    x /= np.linalg.norm(x)
    y = np.cross(z, x)
    return np.stack([x, y, z])                   # world -> camera rotation rows


def synthetic_model(n_images=6, n_points=400, sphere=False, seed=0, empty_image=None, png=()):
    """Cameras on a ring around a point cloud; each point seen by the cameras it lies in front of
    (a random subset drops out so shared counts differ)."""
    rng = np.random.default_rng(seed)
    W, H = 64, 48
    if sphere:
        cams = {1: colmap.Camera(1, "SPHERE", W, H, np.array([W / (2 * np.pi), W / 2.0, H / 2.0]))}
    else:
        cams = {1: colmap.Camera(1, "SIMPLE_PINHOLE", W, H, np.array([50.0, W / 2.0, H / 2.0]))}
    P = rng.normal(scale=1.0, size=(n_points, 3))
    imgs, seen = {}, {pid: [] for pid in range(1, n_points + 1)}
    ids = list(range(3, 3 + 2 * n_images, 2))           # non-contiguous image ids
    rng.shuffle(ids)
    for k, iid in enumerate(ids):
        ang = 2 * np.pi * k / n_images
        C = np.array([6 * np.cos(ang), 0.3 * k, 6 * np.sin(ang)])
        R = _look_at(C, np.zeros(3))
        t = -R @ C
        q = _quat_from_rot(R)
        q /= np.linalg.norm(q)
        xys, pids = [], []
        if iid != empty_image:
            for pid in range(1, n_points + 1):
                Xc = R @ P[pid - 1] + t
                if Xc[2] <= 0 or rng.random() < 0.3 * (k % 3) / 2:
                    continue
                xys.append((rng.uniform(0, W), rng.uniform(0, H)))
                pids.append(pid)
                seen[pid].append((iid, len(pids) - 1))
            for _ in range(5):                            # untriangulated keypoints
                xys.append((1.0, 2.0))
                pids.append(-1)
        name = f"img_{iid}.png" if iid in png else f"img_{iid}.jpg"
        imgs[iid] = colmap.Image(iid, q, t, 1, name, np.array(xys, float).reshape(-1, 2), np.array(pids, int))
    pts = {pid: colmap.Point3D(pid, P[pid - 1], np.array([10, 20, 30]), 0.5,
                               np.array([s[0] for s in seen[pid]], int), np.array([s[1] for s in seen[pid]], int))
           for pid in range(1, n_points + 1) if seen[pid]}
    return cams, imgs, pts


def _write_folder(root, cams, imgs, pts, ext):
    from PIL import Image as PILImage
    sparse = os.path.join(root, "sparse")
    (colmap.write_model_text if ext == ".txt" else colmap.write_model_binary)(sparse, cams, imgs, pts)
    os.makedirs(os.path.join(root, "images"), exist_ok=True)
    rng = np.random.default_rng(1)
    for im in imgs.values():
        c = cams[im.camera_id]
        arr = rng.integers(0, 256, size=(c.height, c.width, 3), dtype=np.uint8)
        PILImage.fromarray(arr).save(os.path.join(root, "images", im.name),
                                     **({"quality": 95} if im.name.endswith(".jpg") else {}))


def _convert(tmp_path, model, ext, **kw):
    src = str(tmp_path / f"colmap{ext}")
    out = str(tmp_path / f"dense{ext}")
    _write_folder(src, *model, ext)
    colmap.process_scene(src, out, ext, log=lambda *a: None, **kw)
    return src, out


def _tree(folder):
    out = {}
    for dp, _, fs in os.walk(folder):
        for f in fs:
            p = os.path.join(dp, f)
            out[os.path.relpath(p, folder)] = open(p, "rb").read()
    return out


def test_qvec2rotmat_known_rotation():
    c, s = np.cos(np.pi / 4), np.sin(np.pi / 4)           # 90 degrees about z
    R = colmap.qvec2rotmat([c, 0.0, 0.0, s])
    assert np.allclose(R, [[0, -1, 0], [1, 0, 0], [0, 0, 1]], atol=1e-15)
    q = np.random.default_rng(0).normal(size=4)
    R = colmap.qvec2rotmat(q / np.linalg.norm(q))
    assert np.allclose(R @ R.T, np.eye(3), atol=1e-12) and np.isclose(np.linalg.det(R), 1.0)


@pytest.mark.parametrize("sphere", [False, True])
def test_text_and_binary_models_convert_identically(tmp_path, sphere):
    model = synthetic_model(sphere=sphere, png=(5,))
    _, out_t = _convert(tmp_path, model, ".txt", top_k=3, min_shared=5)
    _, out_b = _convert(tmp_path, model, ".bin", top_k=3, min_shared=5)
    a, b = _tree(out_t), _tree(out_b)
    assert a.keys() == b.keys() and len(a) == 6 + 6 + 1
    for k in a:
        assert a[k] == b[k], k


@pytest.mark.parametrize("sphere", [False, True])
def test_cam_files_pose_intrinsics_depth_range(tmp_path, sphere):
    cams, imgs, pts = model = synthetic_model(sphere=sphere)
    _, out = _convert(tmp_path, model, ".txt", top_k=3, min_shared=5, max_d=192)
    order = sorted(imgs)
    for k, iid in enumerate(order):
        im = imgs[iid]
        cam = io.read_camera(os.path.join(out, "cams", f"{k:08d}_cam.txt"))
        R = colmap.qvec2rotmat(im.qvec)
        assert np.allclose(np.asarray(cam["R"]).reshape(3, 3), R, atol=1e-6)
        assert np.allclose(cam["t"], im.tvec, atol=1e-5)
        X = np.stack([pts[p].xyz for p in im.point3D_ids if p >= 0])
        Xc = X @ R.T + im.tvec
        d = np.linalg.norm(Xc, axis=1) if sphere else Xc[:, 2]
        d = np.sort(d[d > 0])
        dmin, dmax = d[int(d.size * 0.2)] * 0.75, d[int(d.size * 0.8)] * 1.25
        tok = open(os.path.join(out, "cams", f"{k:08d}_cam.txt")).read().split()
        d0, dint, nd, dm = float(tok[-4]), float(tok[-3]), int(tok[-2]), float(tok[-1])
        assert np.isclose(d0, dmin, rtol=1e-12) and np.isclose(dm, dmax, rtol=1e-12) and nd == 192
        assert np.isclose(dint, (dmax - dmin) / 191, rtol=1e-12)
        if sphere:
            assert int(cam["model"]) == types.SPHERE and np.allclose(cam["params"][:3], cams[1].params, rtol=1e-6)
            assert cam["depth_min"] == np.float32(d0) and cam["depth_max"] == np.float32(dm)
        else:
            K = np.asarray(cam["K"]).reshape(3, 3)
            assert np.allclose(K, [[50, 0, 32], [0, 50, 24], [0, 0, 1]])
            # the PINHOLE reader's quirk (ACMMP.cpp:205): the 2nd depth token becomes depth_max
            assert cam["depth_min"] == np.float32(d0) and cam["depth_max"] == np.float32(dint)


def test_pair_list_greedy_top_k_by_shared_tracks(tmp_path):
    cams, imgs, pts = model = synthetic_model(n_images=8)
    top_k, min_shared = 3, 5
    _, out = _convert(tmp_path, model, ".txt", top_k=top_k, min_shared=min_shared, theta0=0.0)
    problems = io.read_pair_list(out)
    order = sorted(imgs)
    assert [p.ref_image_id for p in problems] == list(range(8))
    lines = open(os.path.join(out, "pair.txt")).read().split("\n")
    counts = {}
    for k in range(8):
        tok = lines[2 + 2 * k].split()
        n = int(tok[0])
        assert n <= top_k
        pairs = [(int(tok[1 + 2 * m]), int(tok[2 + 2 * m])) for m in range(n)]
        scores = [s for _, s in pairs]
        assert scores == sorted(scores, reverse=True)
        for j, s in pairs:
            shared = set(imgs[order[k]].point3D_ids.tolist()) & set(imgs[order[j]].point3D_ids.tolist())
            assert s == len(shared) >= min_shared       # theta0 = 0: every kept pair scores its count
            counts[k] = counts.get(k, 0) + 1
    # the graph is symmetric (score[i, j] = score[j, i]) and every image got a neighbour
    for k, p in enumerate(problems):
        for j in p.src_image_ids:
            assert k in problems[j].src_image_ids
    assert all(counts.get(k, 0) > 0 for k in range(8))


def test_triangulation_angle_filter_and_min_shared(tmp_path):
    model = synthetic_model()
    _, out = _convert(tmp_path, model, ".txt", top_k=3, min_shared=5, theta0=179.0)
    assert all(not p.src_image_ids for p in io.read_pair_list(out))   # no pair reaches 179 degrees
    _, out2 = _convert(tmp_path / "b", model, ".txt", top_k=3, min_shared=10 ** 6)
    assert all(not p.src_image_ids for p in io.read_pair_list(out2))


def test_image_without_points_and_few_images(tmp_path):
    cams, imgs, pts = model = synthetic_model(n_images=4, empty_image=5)
    _, out = _convert(tmp_path, model, ".txt", top_k=20, min_shared=5)  # top_k + 1 > images
    k_empty = sorted(imgs).index(5)
    assert not os.path.exists(os.path.join(out, "cams", f"{k_empty:08d}_cam.txt"))
    probs = io.read_pair_list(out)
    assert len(probs) == 4 and not probs[k_empty].src_image_ids
    assert all(p.src_image_ids for k, p in enumerate(probs) if k != k_empty)


def test_images_copied_or_reencoded(tmp_path):
    model = synthetic_model(png=(5,))
    src, out = _convert(tmp_path, model, ".txt", top_k=3, min_shared=5)
    order = sorted(model[1])
    for k, iid in enumerate(order):
        dst = os.path.join(out, "images", f"{k:08d}.jpg")
        name = model[1][iid].name
        if name.endswith(".jpg"):
            assert open(dst, "rb").read() == open(os.path.join(src, "images", name), "rb").read()
        else:
            assert open(dst, "rb").read(2) == b"\xff\xd8"          # JPEG
            assert pipeline.read_gray(dst).shape == (48, 64)


def test_converted_folder_loads_into_pipeline(tmp_path):
    model = synthetic_model(sphere=True)
    _, out = _convert(tmp_path, model, ".bin", top_k=3, min_shared=5)
    ds = pipeline.load_dataset(out, with_colors=True)
    assert len(ds.problems) == 6 and all(p.src_image_ids for p in ds.problems)
    for i, cam in ds.cameras.items():
        assert (int(cam["width"]), int(cam["height"])) == (64, 48)
        assert ds.images[i].shape == (48, 64) and ds.colors[i].shape == (48, 64, 3)
        assert 0 < cam["depth_min"] < cam["depth_max"]


def test_cli_main(tmp_path):
    model = synthetic_model()
    src = str(tmp_path / "c")
    _write_folder(src, *model, ".txt")
    rc = colmap.main(["--dense_folder", src, "--save_folder", str(tmp_path / "o"), "--top_k", "3",
                      "--min_shared", "5"])
    assert rc == 0 and os.path.exists(tmp_path / "o" / "pair.txt")
