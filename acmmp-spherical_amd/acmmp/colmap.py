"""COLMAP sparse model -> ACMMP dense folder, OpenCV-free.

Restates colmap2mvsnet_acm.py (the reference's data-prep script): the COLMAP text / binary readers
(:69-167), qvec2rotmat (:172-178), the per-image depth range from the triangulated points
(:183-217), neighbour selection -- k nearest camera centres, shared-track count, greedy top-k bins,
triangulation-angle score (:222-353) -- and the writers of cams/%08d_cam.txt, pair.txt and
images/%08d.jpg (:355-406).  The folder it writes is what `acmmp.pipeline` (ProcessProblem's
readers) consumes.

Kept from the reference, deliberately:
  * images are renumbered 1..N in sorted-id order; pairs and output files are 0-based;
  * untriangulated keypoints (point id -1) count as a shared "track" of two images (:226-235);
  * the SPHERE depth is the radial distance, pinhole depth the camera z (:193-196);
  * depth line `dmin interval n dmax`; the PINHOLE reader later takes its 2nd token as depth_max
    (ACMMP.cpp:205, kept in io.read_camera).
Changed, where the reference raises:
  * an image with no point in front of it gets no depth range (and no cam file) instead of an
    IndexError at :197 -- the writers already skip such images (:357);
  * fewer than top_k + 1 images: the k-d tree's missing-neighbour index (== number of images)
    is skipped instead of raising at :283.
Not pinned bit for bit: the JPEG re-encode of non-.jpg inputs (PIL instead of OpenCV's encoder,
same default quality 95); angle scores are vectorised (float64; only exact threshold ties
could differ).
"""
from __future__ import annotations

import argparse
import os
import shutil
import struct
from dataclasses import dataclass

import numpy as np

# COLMAP camera model id -> (name, number of parameters); id 11 is the fork's SPHERE (:59)
CAMERA_MODELS = {
    0: ("SIMPLE_PINHOLE", 3), 1: ("PINHOLE", 4), 2: ("SIMPLE_RADIAL", 4), 3: ("RADIAL", 5),
    4: ("OPENCV", 8), 5: ("OPENCV_FISHEYE", 8), 6: ("FULL_OPENCV", 12), 7: ("FOV", 5),
    8: ("SIMPLE_RADIAL_FISHEYE", 4), 9: ("RADIAL_FISHEYE", 5), 10: ("THIN_PRISM_FISHEYE", 12),
    11: ("SPHERE", 3),
}
CAMERA_MODEL_IDS = {name: mid for mid, (name, _) in CAMERA_MODELS.items()}

# parameter names per model (:253-265); only f/fx/fy/cx/cy are used
PARAM_NAMES = {
    "SIMPLE_PINHOLE": ["f", "cx", "cy"],
    "PINHOLE": ["fx", "fy", "cx", "cy"],
    "SIMPLE_RADIAL": ["f", "cx", "cy", "k"],
    "RADIAL": ["f", "cx", "cy", "k1", "k2"],
    "OPENCV": ["fx", "fy", "cx", "cy", "k1", "k2", "p1", "p2"],
    "OPENCV_FISHEYE": ["fx", "fy", "cx", "cy", "k1", "k2", "k3", "k4"],
    "FULL_OPENCV": ["fx", "fy", "cx", "cy", "k1", "k2", "p1", "p2", "k3", "k4", "k5", "k6"],
    "FOV": ["fx", "fy", "cx", "cy", "omega"],
    "THIN_PRISM_FISHEYE": ["fx", "fy", "cx", "cy", "k1", "k2", "p1", "p2", "k3", "k4", "sx1", "sy1"],
    "SPHERE": ["f", "cx", "cy"],
}


@dataclass
class Camera:
    id: int
    model: str
    width: int
    height: int
    params: np.ndarray


@dataclass
class Image:
    id: int
    qvec: np.ndarray
    tvec: np.ndarray
    camera_id: int
    name: str
    xys: np.ndarray
    point3D_ids: np.ndarray


@dataclass
class Point3D:
    id: int
    xyz: np.ndarray
    rgb: np.ndarray
    error: float
    image_ids: np.ndarray
    point2D_idxs: np.ndarray


# ------------------------------------------------------------------ readers (:69-167)

def _lines(path):
    with open(path) as f:
        for ln in f:
            if ln.strip() and not ln.lstrip().startswith("#"):
                yield ln


def read_cameras_text(path: str) -> dict:
    cams = {}
    for ln in _lines(path):
        s = ln.split()
        cid = int(s[0])
        cams[cid] = Camera(cid, s[1], int(s[2]), int(s[3]), np.array([float(v) for v in s[4:]]))
    return cams


def read_cameras_binary(path: str) -> dict:
    cams = {}
    with open(path, "rb") as f:
        (n,) = struct.unpack("<Q", f.read(8))
        for _ in range(n):
            cid, mid, w, h = struct.unpack("<iiQQ", f.read(24))
            name, npar = CAMERA_MODELS[mid]
            params = np.array(struct.unpack("<" + "d" * npar, f.read(8 * npar)))
            cams[cid] = Camera(cid, name, w, h, params)
    return cams


def read_images_text(path: str) -> dict:
    """Two lines per image (the second: x y point3D_id triples; may be empty)."""
    imgs = {}
    with open(path) as f:
        while True:
            ln = f.readline()
            if not ln:
                break
            if ln.lstrip().startswith("#") or not ln.strip():
                continue
            s = ln.split()
            iid = int(s[0])
            track = f.readline().split()
            xys = np.column_stack([np.array([float(v) for v in track[0::3]]),
                                   np.array([float(v) for v in track[1::3]])])
            pids = np.array([int(v) for v in track[2::3]], dtype=int)
            imgs[iid] = Image(iid, np.array([float(v) for v in s[1:5]]), np.array([float(v) for v in s[5:8]]),
                              int(s[8]), s[9], xys, pids)
    return imgs


def read_images_binary(path: str) -> dict:
    imgs = {}
    with open(path, "rb") as f:
        (n,) = struct.unpack("<Q", f.read(8))
        for _ in range(n):
            vals = struct.unpack("<idddddddi", f.read(64))
            name = bytearray()
            while True:
                c = f.read(1)
                if c == b"\x00" or not c:
                    break
                name += c
            (npts,) = struct.unpack("<Q", f.read(8))
            data = struct.unpack("<" + "ddq" * npts, f.read(24 * npts))
            xys = np.column_stack([np.array(data[0::3]), np.array(data[1::3])])
            imgs[vals[0]] = Image(vals[0], np.array(vals[1:5]), np.array(vals[5:8]), vals[8], name.decode(),
                                  xys, np.array(data[2::3], dtype=int))
    return imgs


def read_points3d_text(path: str) -> dict:
    pts = {}
    for ln in _lines(path):
        s = ln.split()
        pid = int(s[0])
        pts[pid] = Point3D(pid, np.array([float(v) for v in s[1:4]]), np.array([int(v) for v in s[4:7]]),
                           float(s[7]), np.array([int(v) for v in s[8::2]], dtype=int),
                           np.array([int(v) for v in s[9::2]], dtype=int))
    return pts


def read_points3d_binary(path: str) -> dict:
    pts = {}
    with open(path, "rb") as f:
        (n,) = struct.unpack("<Q", f.read(8))
        for _ in range(n):
            pid, x, y, z, r, g, b, err = struct.unpack("<QdddBBBd", f.read(43))
            (length,) = struct.unpack("<Q", f.read(8))
            track = struct.unpack("<" + "ii" * length, f.read(8 * length))
            pts[pid] = Point3D(pid, np.array([x, y, z]), np.array([r, g, b]), err,
                               np.array(track[0::2], dtype=int), np.array(track[1::2], dtype=int))
    return pts


def read_model(sparse_dir: str, ext: str):
    """read_model (:156-165): cameras, images, points3D with extension .txt or .bin."""
    j = lambda name: os.path.join(sparse_dir, name + ext)  # noqa: E731
    if ext == ".txt":
        return read_cameras_text(j("cameras")), read_images_text(j("images")), read_points3d_text(j("points3D"))
    return read_cameras_binary(j("cameras")), read_images_binary(j("images")), read_points3d_binary(j("points3D"))


# ------------------------------------------------------------------ writers (tests, synthetic models)

def write_model_text(sparse_dir: str, cams: dict, imgs: dict, pts: dict) -> None:
    os.makedirs(sparse_dir, exist_ok=True)
    with open(os.path.join(sparse_dir, "cameras.txt"), "w") as f:
        f.write("# Camera list\n")
        for c in cams.values():
            f.write(f"{c.id} {c.model} {c.width} {c.height} " + " ".join(repr(float(p)) for p in c.params) + "\n")
    with open(os.path.join(sparse_dir, "images.txt"), "w") as f:
        f.write("# Image list\n")
        for im in imgs.values():
            f.write(" ".join([str(im.id), *(repr(float(v)) for v in im.qvec), *(repr(float(v)) for v in im.tvec),
                              str(im.camera_id), im.name]) + "\n")
            f.write(" ".join(f"{float(x)!r} {float(y)!r} {int(p)}" for (x, y), p in zip(im.xys, im.point3D_ids))
                    + "\n")
    with open(os.path.join(sparse_dir, "points3D.txt"), "w") as f:
        f.write("# 3D point list\n")
        for p in pts.values():
            f.write(" ".join([str(p.id), *(repr(float(v)) for v in p.xyz), *(str(int(v)) for v in p.rgb),
                              repr(float(p.error)),
                              *(f"{int(i)} {int(k)}" for i, k in zip(p.image_ids, p.point2D_idxs))]) + "\n")


def write_model_binary(sparse_dir: str, cams: dict, imgs: dict, pts: dict) -> None:
    os.makedirs(sparse_dir, exist_ok=True)
    with open(os.path.join(sparse_dir, "cameras.bin"), "wb") as f:
        f.write(struct.pack("<Q", len(cams)))
        for c in cams.values():
            f.write(struct.pack("<iiQQ", c.id, CAMERA_MODEL_IDS[c.model], c.width, c.height))
            f.write(struct.pack("<" + "d" * len(c.params), *map(float, c.params)))
    with open(os.path.join(sparse_dir, "images.bin"), "wb") as f:
        f.write(struct.pack("<Q", len(imgs)))
        for im in imgs.values():
            f.write(struct.pack("<idddddddi", im.id, *map(float, im.qvec), *map(float, im.tvec), im.camera_id))
            f.write(im.name.encode() + b"\x00")
            f.write(struct.pack("<Q", len(im.point3D_ids)))
            for (x, y), p in zip(im.xys, im.point3D_ids):
                f.write(struct.pack("<ddq", float(x), float(y), int(p)))
    with open(os.path.join(sparse_dir, "points3D.bin"), "wb") as f:
        f.write(struct.pack("<Q", len(pts)))
        for p in pts.values():
            f.write(struct.pack("<QdddBBBd", p.id, *map(float, p.xyz), *map(int, p.rgb), float(p.error)))
            f.write(struct.pack("<Q", len(p.image_ids)))
            for i, k in zip(p.image_ids, p.point2D_idxs):
                f.write(struct.pack("<ii", int(i), int(k)))


# ------------------------------------------------------------------ geometry (:172-217)

def qvec2rotmat(q) -> np.ndarray:
    """Unit quaternion (w, x, y, z) -> rotation matrix (:172-178)."""
    w, x, y, z = q
    return np.array([
        [1 - 2 * y * y - 2 * z * z, 2 * x * y - 2 * w * z, 2 * x * z + 2 * w * y],
        [2 * x * y + 2 * w * z, 1 - 2 * x * x - 2 * z * z, 2 * y * z - 2 * w * x],
        [2 * x * z - 2 * w * y, 2 * y * z + 2 * w * x, 1 - 2 * x * x - 2 * y * y],
    ])


def intrinsics(cams: dict) -> dict:
    """3x3 K per camera id from f / fx, fy, cx, cy (:266-276)."""
    out = {}
    for cid, cam in cams.items():
        vals = dict(zip(PARAM_NAMES[cam.model], cam.params))
        if "f" in vals:
            vals["fx"] = vals["fy"] = vals["f"]
        K = np.eye(3)
        K[0, 0], K[1, 1], K[0, 2], K[1, 2] = vals["fx"], vals["fy"], vals["cx"], vals["cy"]
        out[cid] = K
    return out


def extrinsics(imgs: dict) -> dict:
    out = {}
    for i, im in imgs.items():
        E = np.eye(4)
        E[:3, :3] = qvec2rotmat(im.qvec)
        E[:3, 3] = im.tvec
        out[i] = E
    return out


def compute_depth_ranges(images: dict, points3d: dict, extrinsic: dict, intrinsic: dict, max_d: int,
                         interval_scale: float, cams: dict) -> dict:
    """(dmin, interval, n, dmax) per image (:183-217): the 20th / 80th percentile sample of the
    depths of the image's points in front of it, times 0.75 / 1.25; n = max_d, or (max_d == 0) the
    inverse-depth step of one pixel at dmin."""
    out = {}
    for i, img in images.items():
        sphere = cams[img.camera_id].model == "SPHERE"
        E = extrinsic[i]
        zs = []
        for pid in img.point3D_ids:
            if pid < 0:
                continue
            Xc = E @ np.append(points3d[pid].xyz, 1.0)     # the reference's 4x4 product, same rounding
            d = np.linalg.norm(Xc[:3]) if sphere else Xc[2]
            if d > 0:
                zs.append(d)
        if not zs:
            continue
        zs.sort()
        dmin = zs[int(len(zs) * 0.2)] * 0.75
        dmax = zs[int(len(zs) * 0.8)] * 1.25
        if max_d == 0:
            K = intrinsic[img.camera_id]
            Kinv = np.linalg.inv(K)
            Rinv = np.linalg.inv(extrinsic[i][:3, :3])
            p1 = np.array([K[0, 2], K[1, 2], 1.0])
            P1 = Rinv @ ((Kinv @ p1) * dmin - extrinsic[i][:3, 3])
            P2 = Rinv @ ((Kinv @ (p1 + np.array([1.0, 0.0, 0.0]))) * dmin - extrinsic[i][:3, 3])
            depth_num = int((1 / dmin - 1 / dmax) / (1 / dmin - 1 / (dmin + np.linalg.norm(P2 - P1))))
        else:
            depth_num = max_d
        out[i] = (dmin, (dmax - dmin) / (depth_num - 1) / interval_scale, depth_num, dmax)
    return out


def camera_center(E: np.ndarray) -> np.ndarray:
    return -(E[:3, :3].T @ E[:3, 3])


def calc_shared(pair, images) -> int:
    """Shared point ids of two images, -1 included (:226-229)."""
    i, j = pair
    return len(set(images[i + 1].point3D_ids.tolist()) & set(images[j + 1].point3D_ids.tolist()))


def calc_score(pair, images, points3d, theta0, extrinsic):
    """(:231-244) 0 without shared ids or when the 75th percentile triangulation angle over the
    shared points is below theta0 degrees; otherwise the shared-id count."""
    i, j = pair
    shared = set(images[i + 1].point3D_ids.tolist()) & set(images[j + 1].point3D_ids.tolist())
    if not shared:
        return i, j, 0.0
    ids = [pid for pid in shared if pid != -1]
    if not ids:
        return i, j, 0.0
    ci, cj = camera_center(extrinsic[i + 1]), camera_center(extrinsic[j + 1])
    P = np.stack([points3d[pid].xyz for pid in ids])
    a, b = ci - P, cj - P
    cos = np.einsum("ij,ij->i", a, b) / (np.linalg.norm(a, axis=1) * np.linalg.norm(b, axis=1))
    angs = np.degrees(np.arccos(np.clip(cos, -1.0, 1.0)))
    if np.percentile(angs, 75) < theta0:
        return i, j, 0.0
    return i, j, float(len(shared))


def select_views(imgs: dict, pts: dict, extr: dict, depth_ranges: dict, top_k: int, min_shared: int,
                 theta0: float):
    """Neighbour lists (:278-353): k nearest camera centres -> candidate pairs; greedy by shared
    count (stop below min_shared) with at most top_k pairs per image; score by triangulation
    angle; each image keeps its top_k positively scored partners."""
    from scipy.spatial import cKDTree
    N = len(imgs)
    keys = sorted(depth_ranges.keys())
    candidate_pairs = set()
    if keys:
        centers = np.stack([camera_center(extr[i]) for i in keys])
        _, nnidx = cKDTree(centers).query(centers, k=top_k + 1)
        nnidx = np.asarray(nnidx).reshape(len(keys), -1)
        for src_idx, neighs in enumerate(nnidx):
            src = keys[src_idx] - 1
            for n in neighs:
                if n == src_idx or n >= len(keys):
                    continue
                dst = keys[n] - 1
                candidate_pairs.add((min(src, dst), max(src, dst)))
    all_pairs = list(candidate_pairs)
    shared_cnt = [calc_shared(p, imgs) for p in all_pairs]
    bins = {i - 1: 0 for i in depth_ranges}
    top_pairs = []
    for pair, s in sorted(zip(all_pairs, shared_cnt), key=lambda x: x[1], reverse=True):
        if s < min_shared:
            break
        i, j = pair
        if bins[i] < top_k and bins[j] < top_k:
            bins[i] += 1
            bins[j] += 1
            top_pairs.append(pair)
    score = np.zeros((N, N))
    for pair in top_pairs:
        i, j, s = calc_score(pair, imgs, pts, theta0, extr)
        score[i, j] = score[j, i] = s
    view_sel = []
    for i in range(N):
        top = np.argsort(score[i])[::-1]
        view_sel.append([(int(k), score[i, k]) for k in top if score[i, k] > 0][:top_k])
    return view_sel, top_pairs


def write_cam_file(path: str, E: np.ndarray, cam: Camera, K: np.ndarray, depth_range) -> None:
    """cams/%08d_cam.txt as the converter writes it (:355-388): str() of float64 values."""
    with open(path, "w") as f:
        f.write("extrinsic\n")
        for r in range(4):
            f.write(" ".join(map(str, E[r])) + "\n")
        f.write("\nintrinsic\n")
        if cam.model == "SPHERE":
            f.write("SPHERE\n")
            f.write(f"{cam.params[0]} {cam.params[1]} {cam.params[2]}\n")
        else:
            for r in range(3):
                f.write(" ".join(map(str, K[r])) + "\n")
        d0, dint, nd, dmax = depth_range
        f.write(f"\n{d0} {dint} {nd} {dmax}\n")


def process_scene(dense_folder: str, save_folder: str, model_ext: str = ".txt", max_d: int = 192,
                  interval_scale: float = 1.0, theta0: float = 1.0, top_k: int = 20, min_shared: int = 10,
                  log=print) -> dict:
    """process_scene (:246-406).  Returns a summary dict."""
    cams, imgs_raw, pts = read_model(os.path.join(dense_folder, "sparse"), model_ext)
    imgs = {i + 1: imgs_raw[k] for i, k in enumerate(sorted(imgs_raw))}
    N = len(imgs)
    Kdict = intrinsics(cams)
    extr = extrinsics(imgs)
    depth_ranges = compute_depth_ranges(imgs, pts, extr, Kdict, max_d, interval_scale, cams)
    log(f"depth_ranges[1] {depth_ranges.get(1)}")
    view_sel, top_pairs = select_views(imgs, pts, extr, depth_ranges, top_k, min_shared, theta0)
    log(f"[INFO] Kept {len(top_pairs)} pairs (<={top_k} per image, >={min_shared} shared tracks)")
    out_img = os.path.join(save_folder, "images")
    cam_dir = os.path.join(save_folder, "cams")
    os.makedirs(out_img, exist_ok=True)
    os.makedirs(cam_dir, exist_ok=True)
    for i in range(N):
        if (i + 1) not in depth_ranges:
            continue
        im = imgs[i + 1]
        cam = cams[im.camera_id]
        write_cam_file(os.path.join(cam_dir, f"{i:08d}_cam.txt"), extr[i + 1], cam, Kdict[cam.id],
                       depth_ranges[i + 1])
    with open(os.path.join(save_folder, "pair.txt"), "w") as f:
        f.write(f"{N}\n")
        for i, nbrs in enumerate(view_sel):
            f.write(f"{i}\n{len(nbrs)} ")
            for j, s in nbrs:
                f.write(f"{j} {int(s)} ")
            f.write("\n")
    for i in range(N):
        src = os.path.join(dense_folder, "images", imgs[i + 1].name)
        dst = os.path.join(out_img, f"{i:08d}.jpg")
        if src.lower().endswith(".jpg"):
            shutil.copyfile(src, dst)
        else:
            from PIL import Image as PILImage
            with PILImage.open(src) as pim:
                pim.convert("RGB").save(dst, quality=95)
    return {"images": N, "pairs": len(top_pairs), "with_depth_range": len(depth_ranges)}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="Convert a COLMAP sparse model to the ACMMP dense-folder layout.")
    ap.add_argument("--dense_folder", required=True, help="folder with sparse/ and images/")
    ap.add_argument("--save_folder", required=True)
    ap.add_argument("--model_ext", default=".txt", choices=[".txt", ".bin"])
    ap.add_argument("--max_d", type=int, default=192)
    ap.add_argument("--interval_scale", type=float, default=1.0)
    ap.add_argument("--theta0", type=float, default=1.0, help="min triangulation angle (deg)")
    ap.add_argument("--top_k", type=int, default=20, help="max neighbours kept per image")
    ap.add_argument("--min_shared", type=int, default=10, help="min shared tracks to keep a pair")
    ap.add_argument("--chunksize", type=int, default=512, help="accepted for compatibility (scoring is vectorised)")
    a = ap.parse_args(argv)
    os.makedirs(a.save_folder, exist_ok=True)
    process_scene(a.dense_folder, a.save_folder, a.model_ext, a.max_d, a.interval_scale, a.theta0, a.top_k,
                  a.min_shared)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
