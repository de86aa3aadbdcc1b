"""Independent float64 numpy restatement of the reference's camera / cost functions.

A second, vectorised restatement of ACMMP.cu (written from the reference source, not
from the C oracle) used to cross-check the oracle's arithmetic within float tolerance.
Pins the oracle's geometry and NCC definitions where no reference outputs exist.
"""
import numpy as np

PINHOLE, SPHERE = 0, 11
PI_F = np.float64(np.float32(3.141592654))


def pixel_to_dir(cam, x, y):
    """PixelToDir, ACMMP.cu:119-134."""
    x = np.asarray(x, np.float64); y = np.asarray(y, np.float64)
    if int(cam["model"]) == PINHOLE:
        K = cam["K"].astype(np.float64)
        d = np.stack([(x - K[2]) / K[0], (y - K[5]) / K[4], np.ones_like(x)], -1)
        return d / np.linalg.norm(d, axis=-1, keepdims=True)
    lon = (x - cam["params"][1]) / cam["width"] * 2.0 * PI_F
    lat = -(y - cam["params"][2]) / cam["height"] * PI_F
    return np.stack([np.cos(lat) * np.sin(lon), -np.sin(lat), np.cos(lat) * np.cos(lon)], -1)


def world_point(cam, x, y, depth):
    """Get3DPointonWorld_cu, ACMMP.cu:565-600 (pinhole: depth is z)."""
    x = np.asarray(x, np.float64); y = np.asarray(y, np.float64); depth = np.asarray(depth, np.float64)
    if int(cam["model"]) == SPHERE:
        pc = pixel_to_dir(cam, x, y) * depth[..., None]
    else:
        K = cam["K"].astype(np.float64)
        pc = np.stack([depth * (x - K[2]) / K[0], depth * (y - K[5]) / K[4], depth], -1)
    R = cam["R"].astype(np.float64).reshape(3, 3)
    t = cam["t"].astype(np.float64)
    return pc @ R - (R.T @ t)


def project(cam, P):
    """ProjectonCamera_cu, ACMMP.cu:602-644 -> (x, y, depth)."""
    R = cam["R"].astype(np.float64).reshape(3, 3)
    tc = np.asarray(P, np.float64) @ R.T + cam["t"].astype(np.float64)
    if int(cam["model"]) == SPHERE:
        d = np.linalg.norm(tc, axis=-1)
        lat = -np.arcsin(tc[..., 1] / d)
        lon = np.arctan2(tc[..., 0], tc[..., 2])
        return (lon / (2 * np.pi) * cam["width"] + cam["params"][1],
                -lat / np.pi * cam["height"] + cam["params"][2], d)
    K = cam["K"].astype(np.float64).reshape(3, 3)
    h = tc @ K.T
    return h[..., 0] / tc[..., 2], h[..., 1] / tc[..., 2], tc[..., 2]


def depth_from_plane(cam, plane, x, y):
    d = pixel_to_dir(cam, x, y)
    den = d @ np.asarray(plane[:3], np.float64)
    return np.where(np.abs(den) < 1e-6, 1e6, -plane[3] / den)


def texel(img, ix, iy):
    H, W = img.shape
    return img[np.clip(iy, 0, H - 1), np.clip(ix, 0, W - 1)].astype(np.float64)


def bilinear(img, x, y):
    fx, fy = np.floor(x), np.floor(y)
    a, b = x - fx, y - fy
    ix, iy = fx.astype(np.int64), fy.astype(np.int64)
    t00, t10 = texel(img, ix, iy), texel(img, ix + 1, iy)
    t01, t11 = texel(img, ix, iy + 1), texel(img, ix + 1, iy + 1)
    return (1 - b) * ((1 - a) * t00 + a * t10) + b * ((1 - a) * t01 + a * t11)


def bilateral_ncc(images, cams, params, src, px, py, plane):
    """ComputeBilateralNCC, ACMMP.cu:405-516, float64."""
    rc, sc = cams[0], cams[src]
    ref, simg = images[0], images[src]
    R = int(params["patch_size"]) // 2
    inc = int(params["radius_increment"])
    dref = depth_from_plane(rc, plane, px, py)
    Pc = world_point(rc, px, py, dref)
    cx, cy, _ = project(sc, Pc)
    if int(sc["model"]) != SPHERE and (cx < 0 or cx >= sc["width"] or cy < 0 or cy >= sc["height"]):
        return 2.0
    sig = float(params["sigma_spatial"])
    scx = scy = 1.0
    if int(rc["model"]) == SPHERE:
        latc = -(py - rc["params"][2]) / rc["height"] * PI_F
        scx = 2 * PI_F / rc["width"] * np.cos(latc)
        scy = PI_F / rc["height"]
        sig = sig * PI_F / rc["height"]
    offs = np.arange(-R, R + 1, inc)
    ii, jj = np.meshgrid(offs, offs, indexing="ij")
    ii, jj = ii.ravel(), jj.ravel()
    rx, ry = px + ii, py + jj
    rpix = texel(ref, rx, ry)
    center = texel(ref, np.array(px), np.array(py))
    dn = depth_from_plane(rc, plane, rx, ry)
    P = world_point(rc, rx, ry, dn)
    sx, sy, _ = project(sc, P)
    W, H = sc["width"], sc["height"]
    if int(sc["model"]) == SPHERE:
        sx = sx - np.floor(sx / W) * W
        sy = np.clip(sy, 0, H - 1)
        ok = np.ones_like(sx, bool)
    else:
        ok = ~((sx < 0) | (sx >= W) | (sy < 0) | (sy >= H))
    spix = bilinear(simg, np.where(ok, sx, 0), np.where(ok, sy, 0))
    dx = ii * scx if int(rc["model"]) == SPHERE else ii.astype(np.float64)
    dy = jj * scy if int(rc["model"]) == SPHERE else jj.astype(np.float64)
    w = np.exp(-np.sqrt(dx * dx + dy * dy) / (2 * sig * sig) - np.abs(rpix - center) / (2 * params["sigma_color"] ** 2))
    w = np.where(ok, w, 0.0)
    sbw = w.sum()
    if sbw < 1e-6:
        return 2.0
    mr, ms = (w * rpix).sum() / sbw, (w * spix).sum() / sbw
    vr = (w * rpix * rpix).sum() / sbw - mr * mr
    vs = (w * spix * spix).sum() / sbw - ms * ms
    if vr < 1e-5 or vs < 1e-5:
        return 2.0
    cov = (w * rpix * spix).sum() / sbw - mr * ms
    return float(np.clip(1 - cov / np.sqrt(vr * vs), 0.0, 2.0))


def geom_cost(depths, cams, src, px, py, plane):
    """ComputeGeomConsistencyCost, ACMMP.cu:646-671, float64."""
    rc, sc = cams[0], cams[src]
    d = depth_from_plane(rc, plane, px, py)
    sx, sy, _ = project(sc, world_point(rc, px, py, d))
    dm = depths[src]
    sd = texel(dm, np.array(int(np.trunc(np.clip(sx, -2e9, 2e9)))), np.array(int(np.trunc(np.clip(sy, -2e9, 2e9)))))
    if sd == 0:
        return 3.0
    bx, by, _ = project(rc, world_point(sc, sx, sy, sd))
    return float(min(3.0, np.hypot(px - bx, py - by)))
