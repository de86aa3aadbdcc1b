"""Synthetic multi-view scenes with known geometry (SURVEY.md §8d "Synthetic inputs").

No datasets are reachable from this environment, so every benchmark and test input is
rendered here by ray casting: a textured slanted-plane scene for pinhole cameras and
a textured box room around an equirectangular (SPHERE) camera.  Textures are
band-limited 3-D procedural noise evaluated at the world-space hit point, so the same
surface point has the same grey value in every view.  Images are quantised to integer
grey levels, as the reference's `cv::imread(IMREAD_GRAYSCALE)` + `convertTo(CV_32F)`
(ACMMP.cpp:578-580) would produce.

Camera convention is the reference's: X_cam = R X_world + t (ACMMP.cu:609-614).
Ground-truth depth is the z-depth for pinhole (what the reference's pinhole path
converges to, since Get3DPointonWorld_cu treats depth as z, ACMMP.cu:579-581) and
the radial distance for SPHERE.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from .types import PINHOLE, SPHERE, make_camera


@dataclass
class Scene:
    images: list            # list of float32 (H, W) arrays, index 0 = reference
    cameras: np.ndarray     # CAMERA_DTYPE array, len N
    gt_depth: np.ndarray    # float32 (H, W) ground truth for the reference view
    kind: str
    extra: dict = field(default_factory=dict)


def _texture(P: np.ndarray, seed: int, n_waves: int = 48, fmin: float = 2.0, fmax: float = 9.0) -> np.ndarray:
    """Band-limited procedural texture in [0, 255] at world points P (..., 3)."""
    rng = np.random.default_rng(seed)
    dirs = rng.normal(size=(n_waves, 3))
    dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
    freqs = rng.uniform(fmin, fmax, size=n_waves)
    phases = rng.uniform(0, 2 * np.pi, size=n_waves)
    amps = 1.0 / np.sqrt(freqs)
    P32 = P.astype(np.float32)
    acc = np.zeros(P.shape[:-1], np.float32)
    for k in range(n_waves):
        acc += np.float32(amps[k]) * np.sin(np.float32(freqs[k]) * (P32 @ dirs[k].astype(np.float32))
                                            + np.float32(phases[k]))
    acc /= np.float32(np.sqrt(np.sum(amps ** 2) / 2.0))
    return np.clip(127.5 + 60.0 * acc.astype(np.float64), 0.0, 255.0)


def _look_rotation(yaw: float, pitch: float) -> np.ndarray:
    cy, sy, cp, sp = np.cos(yaw), np.sin(yaw), np.cos(pitch), np.sin(pitch)
    Ry = np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]])
    Rx = np.array([[1, 0, 0], [0, cp, -sp], [0, sp, cp]])
    return Rx @ Ry


# ---------------------------------------------------------------- pinhole scenes

def _plane_hit(o: np.ndarray, d: np.ndarray, n: np.ndarray, c: float) -> np.ndarray:
    """t such that n.(o + t d) = c."""
    return (c - o @ n) / (d @ n)


def pinhole_scene(width: int = 640, height: int = 480, n_src: int = 1, seed: int = 0,
                  depth: float = 5.0, slant=(0.15, 0.08), baseline: float = 0.5,
                  quantize: bool = True, n_waves: int = 48) -> Scene:
    """Slanted textured plane z = depth + sx*x + sy*y in front of a pinhole rig."""
    f = 0.8 * width
    K = np.array([[f, 0, width / 2.0], [0, f, height / 2.0], [0, 0, 1]], np.float64)
    n = np.array([-slant[0], -slant[1], 1.0])
    c = depth
    rng = np.random.default_rng(seed + 1000)
    cams, imgs = [], []
    centers = [np.zeros(3)]
    rots = [np.eye(3)]
    for k in range(n_src):
        ang = 2 * np.pi * k / max(n_src, 1) + rng.uniform(-0.2, 0.2)
        C = baseline * np.array([np.cos(ang), 0.5 * np.sin(ang), 0.0])
        centers.append(C)
        rots.append(_look_rotation(-0.5 * C[0] / depth, 0.5 * C[1] / depth))
    ys, xs = np.mgrid[0:height, 0:width].astype(np.float64)
    rays_cam = np.stack([(xs - K[0, 2]) / K[0, 0], (ys - K[1, 2]) / K[1, 1], np.ones_like(xs)], -1)
    gt = None
    dmin, dmax = depth * 0.6, depth * 1.6
    ppu = f / depth                                   # pixels per world unit at the plane
    fmin, fmax = 2 * np.pi * ppu / 30.0, 2 * np.pi * ppu / 6.0   # wavelengths 6..30 px
    for C, R in zip(centers, rots):
        d = rays_cam @ R            # world direction = R^T ray_cam  (row-vector form)
        t = _plane_hit(C, d, n, c)
        P = C + t[..., None] * d
        img = _texture(P, seed, n_waves=n_waves, fmin=fmin, fmax=fmax)
        if quantize:
            img = np.round(img)
        imgs.append(img.astype(np.float32))
        tvec = -R @ C
        cams.append(make_camera(PINHOLE, K=K, R=R, t=tvec, width=width, height=height,
                                depth_min=dmin, depth_max=dmax))
        if gt is None:
            gt = (P @ R.T + tvec)[..., 2].astype(np.float32)
    cams_arr = np.array(cams)
    # the reference's pinhole ReadCamera stores the 2nd depth token as depth_max (ACMMP.cpp:205);
    # cameras built in memory carry the intended range directly.
    return Scene(imgs, cams_arr, gt, "pinhole", {"K": K})


# ---------------------------------------------------------------- spherical scenes

def _box_hit(o: np.ndarray, d: np.ndarray, half: np.ndarray) -> np.ndarray:
    """Exit distance from inside the axis-aligned box [-half, half]."""
    with np.errstate(divide="ignore", invalid="ignore"):
        tp = (half - o) / d
        tn = (-half - o) / d
    t = np.where(d > 0, tp, np.where(d < 0, tn, np.inf))
    return t.min(axis=-1)


def sphere_dirs(width: int, height: int, cx: float, cy: float, xs=None, ys=None) -> np.ndarray:
    """PixelToDir for the SPHERE model (ACMMP.cu:126-133), float64."""
    if xs is None:
        ys, xs = np.mgrid[0:height, 0:width].astype(np.float64)
    lon = (xs - cx) / width * 2.0 * np.pi
    lat = -(ys - cy) / height * np.pi
    return np.stack([np.cos(lat) * np.sin(lon), -np.sin(lat), np.cos(lat) * np.cos(lon)], -1)


def sphere_scene(width: int = 2000, height: int = 1000, n_src: int = 4, seed: int = 0,
                 half=(5.0, 3.0, 4.0), baseline: float = 0.35, quantize: bool = True, n_waves: int = 48) -> Scene:
    """Equirectangular rig inside a textured box room; sources displaced by ~`baseline`."""
    half = np.asarray(half, np.float64)
    cx, cy = width / 2.0, height / 2.0
    rng = np.random.default_rng(seed + 2000)
    centers = [np.zeros(3)]
    rots = [np.eye(3)]
    for k in range(n_src):
        ang = 2 * np.pi * k / max(n_src, 1) + rng.uniform(-0.3, 0.3)
        C = baseline * np.array([np.cos(ang), rng.uniform(-0.3, 0.3), np.sin(ang)])
        centers.append(C)
        rots.append(_look_rotation(rng.uniform(-0.05, 0.05), rng.uniform(-0.05, 0.05)))
    dirs_cam = sphere_dirs(width, height, cx, cy)
    dmin = 0.5 * float(np.min(half))
    dmax = 1.2 * float(np.linalg.norm(half))
    imgs, cams, gt = [], [], None
    gt_depths, gt_normals = [], []
    ppu = width / (2 * np.pi * float(np.mean(half)))   # pixels per world unit at mean distance
    fmin, fmax = 2 * np.pi * ppu / 30.0, 2 * np.pi * ppu / 6.0
    for C, R in zip(centers, rots):
        d = dirs_cam @ R
        t = _box_hit(C, d, half)
        P = C + t[..., None] * d
        img = _texture(P, seed, n_waves=n_waves, fmin=fmin, fmax=fmax)
        if quantize:
            img = np.round(img)
        imgs.append(img.astype(np.float32))
        tvec = -R @ C
        cams.append(make_camera(SPHERE, params=[width / (2 * np.pi), cx, cy], R=R, t=tvec,
                                width=width, height=height, depth_min=dmin, depth_max=dmax))
        if gt is None:
            gt = t.astype(np.float32)
        gt_depths.append(t.astype(np.float32))
        # world-frame normal of the face hit, facing the camera (the room is seen from inside)
        axis = np.argmin(np.where(d > 0, (half - C) / np.where(d == 0, 1, d),
                                  np.where(d < 0, (-half - C) / np.where(d == 0, 1, d), np.inf)), axis=-1)
        n = np.zeros(d.shape, np.float32)
        sgn = np.take_along_axis(d, axis[..., None], -1)[..., 0]
        np.put_along_axis(n, axis[..., None], (-np.sign(sgn))[..., None].astype(np.float32), -1)
        gt_normals.append(n)
    return Scene(imgs, np.array(cams), gt, "sphere", {"gt_depths": gt_depths, "gt_normals": gt_normals})


def depth_accuracy(depth: np.ndarray, gt: np.ndarray, rel: float = 0.01, mask=None) -> float:
    """Fraction of pixels with |d - gt| / gt < rel (NaN counts as wrong)."""
    ok = np.abs(depth.astype(np.float64) - gt) < rel * gt
    if mask is not None:
        return float(ok[mask].mean())
    return float(ok.mean())
