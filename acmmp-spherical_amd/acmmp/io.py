"""The reference's on-disk formats, OpenCV-free.

  * ReadCamera            ACMMP.cpp:146-209  (cams/%08d_cam.txt; SPHERE and PINHOLE, quirks kept)
  * readDepthDmb/writeDepthDmb, readNormalDmb/writeNormalDmb  ACMMP.cpp:363-479
  * GenerateSampleList    main.cpp:4-33      (pair.txt; sources with score <= 0 dropped)
  * ComputeMultiScaleSettings main.cpp:35-71 (cap 3200, halve until <= 1000)
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field

import numpy as np

from .types import PINHOLE, SPHERE, make_camera


def read_camera(path: str) -> np.ndarray:
    """ReadCamera (ACMMP.cpp:146-209).

    Keeps the reference's behaviour: 'extrinsic' + 3 rows of `R|t` + the `0 0 0 1` row,
    'intrinsic' then either `SPHERE f cx cy` or a 3x3 K; then the depth line.  For SPHERE
    all four depth tokens are read as (min, interval, n, max).  For PINHOLE the reader
    stores the 2nd token as depth_max (ACMMP.cpp:205) -- with the converter's
    `d0 dint N dmax` layout (colmap2mvsnet_acm.py:387-388) that is the interval.
    A missing file returns a zeroed camera, as the reference returns its uninitialised one.
    """
    if not os.path.exists(path):
        return make_camera(PINHOLE)
    tok = open(path).read().split()
    it = iter(tok)
    next(it)                                   # "extrinsic"
    R = np.zeros(9, np.float32)
    t = np.zeros(3, np.float32)
    for i in range(3):
        R[3 * i + 0] = float(next(it)); R[3 * i + 1] = float(next(it)); R[3 * i + 2] = float(next(it))
        t[i] = float(next(it))
    for _ in range(4):
        next(it)                               # 0 0 0 1
    next(it)                                   # "intrinsic"
    head = next(it)
    if head == "SPHERE":
        f, cx, cy = float(next(it)), float(next(it)), float(next(it))
        dmin = float(next(it)); float(next(it)); int(float(next(it))); dmax = float(next(it))
        return make_camera(SPHERE, params=[f, cx, cy], R=R, t=t, depth_min=dmin, depth_max=dmax)
    K = np.zeros(9, np.float32)
    K[0] = float(head)
    for k in range(1, 9):
        K[k] = float(next(it))
    dmin, dmax = float(next(it)), float(next(it))
    return make_camera(PINHOLE, K=K, R=R, t=t, depth_min=dmin, depth_max=dmax)


def write_camera(path: str, cam: np.ndarray, depth_interval: float = 0.0, n_planes: int = 192) -> None:
    """Writer matching what colmap2mvsnet_acm.py emits (synthetic scenes; tests)."""
    R = np.asarray(cam["R"]).reshape(3, 3)
    t = np.asarray(cam["t"])
    lines = ["extrinsic"]
    for i in range(3):
        lines.append(" ".join(repr(float(v)) for v in (*R[i], t[i])))
    lines.append("0.0 0.0 0.0 1.0")
    lines.append("")
    lines.append("intrinsic")
    if int(cam["model"]) == SPHERE:
        p = cam["params"]
        lines.append(f"SPHERE {float(p[0])!r} {float(p[1])!r} {float(p[2])!r}")
    else:
        K = np.asarray(cam["K"]).reshape(3, 3)
        for i in range(3):
            lines.append(" ".join(repr(float(v)) for v in K[i]))
    lines.append("")
    lines.append(f"{float(cam['depth_min'])!r} {depth_interval!r} {n_planes} {float(cam['depth_max'])!r}")
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def read_dmb(path: str):
    """readDepthDmb / readNormalDmb (ACMMP.cpp:363-452): int32 type(=1), h, w, nb, then h*w*nb floats.

    Returns (h, w) or (h, w, nb) float32, or None where the reference returns -1."""
    try:
        with open(path, "rb") as f:
            hdr = np.fromfile(f, dtype="<i4", count=4)
            if hdr.size < 4 or hdr[0] != 1:
                return None
            _, h, w, nb = (int(v) for v in hdr)
            data = np.fromfile(f, dtype="<f4", count=h * w * nb)
    except OSError:
        return None
    out = np.zeros(h * w * nb, np.float32)
    out[:data.size] = data
    return out.reshape(h, w) if nb == 1 else out.reshape(h, w, nb)


def write_dmb(path: str, arr: np.ndarray) -> None:
    """writeDepthDmb / writeNormalDmb (ACMMP.cpp:395-479)."""
    a = np.ascontiguousarray(arr, np.float32)
    h, w = a.shape[:2]
    nb = 1 if a.ndim == 2 else a.shape[2]
    with open(path, "wb") as f:
        np.array([1, h, w, nb], "<i4").tofile(f)
        a.astype("<f4").tofile(f)


@dataclass
class Problem:
    """struct Problem, main.h:207-213."""
    ref_image_id: int
    src_image_ids: list = field(default_factory=list)
    max_image_size: int = 3200
    num_downscale: int = 0
    cur_image_size: int = 3200


def read_pair_list(dense_folder: str) -> list:
    """GenerateSampleList (main.cpp:4-33)."""
    tok = open(os.path.join(dense_folder, "pair.txt")).read().split()
    it = iter(tok)
    n = int(next(it))
    problems = []
    for _ in range(n):
        p = Problem(int(next(it)))
        m = int(next(it))
        for _ in range(m):
            vid, score = int(next(it)), float(next(it))
            if score <= 0.0:
                continue
            p.src_image_ids.append(vid)
        problems.append(p)
    return problems


def write_pair_list(dense_folder: str, pairs: list) -> None:
    """pairs: list of (ref_id, [(src_id, score), ...])."""
    lines = [str(len(pairs))]
    for ref, srcs in pairs:
        lines.append(str(ref))
        lines.append(" ".join([str(len(srcs))] + [f"{s} {sc!r}" for s, sc in srcs]))
    with open(os.path.join(dense_folder, "pair.txt"), "w") as f:
        f.write("\n".join(lines) + "\n")


def compute_multiscale_settings(problems: list, image_sizes: dict, max_image_size: int = 3200,
                                size_bound: int = 1000) -> int:
    """ComputeMultiScaleSettings (main.cpp:35-71); image_sizes[ref_id] = (rows, cols)."""
    max_num_downscale = -1
    for p in problems:
        rows, cols = image_sizes[p.ref_image_id]
        max_size = min(max(rows, cols), max_image_size)
        p.max_image_size = max_size
        k = 0
        while max_size > size_bound:
            max_size //= 2
            k += 1
        max_num_downscale = max(max_num_downscale, k)
        p.num_downscale = k
    return max_num_downscale


def scale_schedule(problems: list, max_num_downscale: int) -> list:
    """The per-scale cur_image_size sequence of main.cpp:417-425 (pure; for tests and the driver)."""
    import copy
    ps = copy.deepcopy(problems)
    out = []
    scale = max_num_downscale
    while scale >= 0:
        for p in ps:
            if p.num_downscale >= 0:
                p.cur_image_size = int(p.max_image_size / (2 ** p.num_downscale))
                p.num_downscale -= 1
        out.append([p.cur_image_size for p in ps])
        scale -= 1
    return out


def write_ply(path: str, points: np.ndarray) -> None:
    """StoreColorPlyFileBinaryPointCloud (ACMMP.cpp:481-534).  points: (n, 9) float32 rows
    x y z nx ny nz c0 c1 c2 as SimpleFusionKernel stores them (c0 = the texture's .z channel);
    the writer emits red = (char)(int)c2, green = (char)(int)c1, blue = (char)(int)c0 and zeroes
    coordinates that are not finite (the FLT_MAX tests of :508-512, including the z >= -FLT_MAX quirk)."""
    p = np.ascontiguousarray(points, np.float32).reshape(-1, 9)
    n = p.shape[0]
    X = p[:, 0:3].copy()
    fmax = np.float32(np.finfo(np.float32).max)
    bad = ~((X[:, 0] < fmax) & (X[:, 0] > -fmax)) | ~((X[:, 1] < fmax) & (X[:, 1] > -fmax)) | \
        ~((X[:, 2] < fmax) & (X[:, 2] >= -fmax))
    X[bad] = 0.0
    rec = np.zeros(n, dtype=[("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("nx", "<f4"), ("ny", "<f4"), ("nz", "<f4"),
                             ("r", "u1"), ("g", "u1"), ("b", "u1")])
    rec["x"], rec["y"], rec["z"] = X[:, 0], X[:, 1], X[:, 2]
    rec["nx"], rec["ny"], rec["nz"] = p[:, 3], p[:, 4], p[:, 5]

    def to_char(v):   # (char)(int)v: truncation toward zero, then the low byte
        with np.errstate(invalid="ignore"):
            iv = np.where(np.isfinite(v), np.trunc(v), 0).astype(np.int64)
        return (iv & 0xFF).astype(np.uint8)
    rec["r"], rec["g"], rec["b"] = to_char(p[:, 8]), to_char(p[:, 7]), to_char(p[:, 6])
    header = ("ply\nformat binary_little_endian 1.0\n"
              f"element vertex {n}\n"
              "property float x\nproperty float y\nproperty float z\n"
              "property float nx\nproperty float ny\nproperty float nz\n"
              "property uchar red\nproperty uchar green\nproperty uchar blue\nend_header\n")
    with open(path, "wb") as f:
        f.write(header.encode("ascii"))
        f.write(rec.tobytes())


def read_ply(path: str) -> np.ndarray:
    """Reader for write_ply's layout (tests): structured array x y z nx ny nz r g b."""
    with open(path, "rb") as f:
        data = f.read()
    end = data.index(b"end_header\n") + len(b"end_header\n")
    n = int([l for l in data[:end].decode().splitlines() if l.startswith("element vertex")][0].split()[2])
    dt = np.dtype([("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("nx", "<f4"), ("ny", "<f4"), ("nz", "<f4"),
                   ("r", "u1"), ("g", "u1"), ("b", "u1")])
    return np.frombuffer(data[end:end + n * dt.itemsize], dtype=dt).copy()
