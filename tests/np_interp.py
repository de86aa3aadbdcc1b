"""Float64 restatement of the fast SPHERE k_eval_nb's interpolated source coordinates, and
the query sets that stress it.  Test infrastructure (no GPU): tests/test_interp_design.py, the GPU test
tests/test_gpu_interp.py and scripts/interp_feasibility.py import it.

`ncc(..., interp=True, nodes=[-5, -1, 1, 5])` is ComputeBilateralNCC (ACMMP.cu:405-516, restated in
np_reference.bilateral_ncc) with the source coordinates of the 36 patch samples taken from 16 exact
projections at the node offsets and the 2-D 4-point Lagrange interpolation through them -- what
`ncc_chunk`'s interpolated loop computes (kernels.hip), with x unwrapped across the seam around a node.
"""
import numpy as np

import np_reference as npr


def lagrange(t, nodes):
    cols = []
    for k, a in enumerate(nodes):
        c = np.ones_like(t, dtype=np.float64)
        for m, b in enumerate(nodes):
            if m != k:
                c = c * (t - b) / (a - b)
        cols.append(c)
    return np.stack(cols, -1)


def ncc(images, cams, params, src, px, py, plane, interp, order=3, span_max=None, nodes=None):
    """-> (cost, largest source-coordinate error of the interpolation in pixels, fell back to projection).
    span_max: the kernel's fallback -- every sample projected when the corner nodes spread over more than
    span_max source pixels (SPREAD_MAX in the kernel); None = always interpolate."""
    rc, sc = cams[0], cams[src]
    ref, simg = images[0], images[src]
    R = int(params["patch_size"]) // 2
    inc = int(params["radius_increment"])
    offs = np.arange(-R, R + 1, inc)
    ii, jj = np.meshgrid(offs, offs, indexing="ij")
    ii, jj = ii.ravel(), jj.ravel()
    W, H = sc["width"], sc["height"]

    def src_xy(di, dj):
        rx, ry = px + di, py + dj
        dn = npr.depth_from_plane(rc, plane, rx, ry)
        x, y, _ = npr.project(sc, npr.world_point(rc, rx, ry, dn))
        return np.asarray(x, np.float64), np.asarray(y, np.float64)

    fell_back = False
    if interp:
        nodes = np.linspace(-R, R, order) if nodes is None else np.asarray(nodes, np.float64)
        order = len(nodes)
        ni, nj = np.meshgrid(nodes, nodes, indexing="ij")
        X, Y = src_xy(ni.ravel(), nj.ravel())
        X = X - np.round((X - X[0]) / W) * W                  # unwrap across the seam around the first node
        # the kernel's smoothness test (ncc_chunk): the corner nodes' spread in source pixels
        k = [0, order - 1, order * (order - 1), order * order - 1]
        bad = span_max is not None and not (max(np.ptp(X[k]), np.ptp(Y[k])) <= span_max)
        if bad:
            fell_back = True
            sx, sy = src_xy(ii, jj)
        else:
            L = lagrange(ii.astype(np.float64), nodes)[:, :, None] * lagrange(jj.astype(np.float64), nodes)[:, None, :]
            L = L.reshape(len(ii), order * order)
            sx, sy = L @ X, L @ Y
    else:
        sx, sy = src_xy(ii, jj)
    exact_x, exact_y = src_xy(ii, jj)
    sx = sx - np.floor(sx / W) * W
    sy = np.clip(sy, 0, H - 1)
    ex = exact_x - np.floor(exact_x / W) * W
    err = np.abs(np.where(np.abs(sx - ex) > W / 2, W - np.abs(sx - ex), sx - ex))
    err = np.maximum(err, np.abs(sy - np.clip(exact_y, 0, H - 1)))
    spix = npr.bilinear(simg, sx, sy)
    rpix = npr.texel(ref, px + ii, py + jj)
    center = npr.texel(ref, np.array(px), np.array(py))
    latc = -(py - rc["params"][2]) / rc["height"] * npr.PI_F
    scx, scy = 2 * npr.PI_F / rc["width"] * np.cos(latc), npr.PI_F / rc["height"]
    sig = float(params["sigma_spatial"]) * npr.PI_F / rc["height"]
    dx, dy = ii * scx, jj * scy
    w = np.exp(-np.sqrt(dx * dx + dy * dy) / (2 * sig * sig) - np.abs(rpix - center) / (2 * params["sigma_color"] ** 2))
    sbw = w.sum()
    if sbw < 1e-6:
        return 2.0, float(err.max()), fell_back
    mr, ms = (w * rpix).sum() / sbw, (w * spix).sum() / sbw
    vr = (w * rpix * rpix).sum() / sbw - mr * mr
    vs = (w * spix * spix).sum() / sbw - ms * ms
    if vr < 1e-5 or vs < 1e-5:
        return 2.0, float(err.max()), fell_back
    cov = (w * rpix * spix).sum() / sbw - mr * ms
    return float(np.clip(1 - cov / np.sqrt(vr * vs), 0.0, 2.0)), float(err.max()), fell_back


NODES = [-5, -1, 1, 5]          # patch offsets of node columns / rows {0, 2, 3, 5} at patch_size 11, increment 2
SPREAD_MAX = 256.0              # kernels.hip kSpreadMax: beyond it the lane projects every sample of the view


def nodes_for(params):
    """Offsets of the node columns / rows {0, 2, 3, 5} of a 6x6 patch (the kernel interpolates in index space)."""
    R, inc = int(params["patch_size"]) // 2, int(params["radius_increment"])
    offs = np.arange(-R, R + 1, inc)
    assert len(offs) == 6, "the interpolated loop is for 6x6 patches"
    return [int(offs[k]) for k in (0, 2, 3, 5)]


def interp_enabled(W, H, params):
    """capi.cpp build_kparams' gate: 6x6 SPHERE patches whose radius spans at most 5 pixels of 2 pi / 2000."""
    R, inc = int(params["patch_size"]) // 2, int(params["radius_increment"])
    return len(range(-R, R + 1, inc)) == 6 and 2000 * R <= 5 * W and 1000 * R <= 5 * H


def surface_projections(sc, stride=2, margin=6):
    """Ground-truth surface point of every `stride`-th reference pixel projected into every source:
    (px, py, sx[V], sy[V]) in float64."""
    rc = sc.cameras[0]
    H, W = sc.images[0].shape
    ys, xs = np.mgrid[margin:H - margin:stride, margin:W - margin:stride]
    xs, ys = xs.ravel(), ys.ravel()
    P = npr.world_point(rc, xs, ys, sc.gt_depth[ys, xs].astype(np.float64))
    sxs, sys_ = [], []
    for v in range(1, len(sc.images)):
        x, y, _ = npr.project(sc.cameras[v], P)
        sxs.append(x)
        sys_.append(y)
    return xs, ys, np.stack(sxs, -1), np.stack(sys_, -1)


def special_pixels(sc, kind, n, seed, min_lat_deg=38.0):
    """Reference pixels (px, py) of one query kind, with the source index each was chosen for:
      "pole": the surface point lands within 10 degrees of a source camera's pole;
      "seam": it lands within 6 source pixels of a source's longitude seam (x = 0 = W);
      "random": anywhere.
    Only pixels at |latitude| >= min_lat_deg: nearer the equator the reference's sigma-in-radians weights put
    every cost at 2.0, so no interpolation is evaluated there."""
    rng = np.random.default_rng(seed)
    H, W = sc.images[0].shape
    xs, ys, sx, sy = surface_projections(sc)
    lat = np.abs((ys - sc.cameras[0]["params"][2]) / H * 180.0)
    keep = lat >= min_lat_deg
    Ws, Hs = float(sc.cameras[1]["width"]), float(sc.cameras[1]["height"])
    if kind == "pole":
        src_lat = np.abs(sy / Hs * 180.0 - 90.0)               # latitude in the source, degrees
        hit = src_lat >= 80.0
    elif kind == "seam":
        xw = sx - np.floor(sx / Ws) * Ws
        hit = (xw < 6.0) | (xw > Ws - 6.0)
    else:
        hit = np.ones_like(sx, bool)
    cand = np.nonzero(keep[:, None] & hit)
    if len(cand[0]) == 0:
        return np.zeros(0, np.int32), np.zeros(0, np.int32), np.zeros(0, np.int32)
    pick = rng.choice(len(cand[0]), size=min(n, len(cand[0])), replace=False)
    idx, src = cand[0][pick], cand[1][pick] + 1
    return xs[idx].astype(np.int32), ys[idx].astype(np.int32), src.astype(np.int32)


def near_surface_planes(sc, px, py, k, seed, spread=0.2, depth_jitter=0.02):
    """k planes per pixel near the ground-truth surface (T1's near-surface hypotheses): (n, k, 4) float32."""
    rng = np.random.default_rng(seed)
    out = np.zeros((len(px), k, 4), np.float64)
    for q in range(len(px)):
        d = npr.pixel_to_dir(sc.cameras[0], int(px[q]), int(py[q]))
        for h in range(k):
            nrm = -d + rng.normal(0, spread, 3)
            nrm /= np.linalg.norm(nrm)
            depth = float(sc.gt_depth[py[q], px[q]]) * rng.uniform(1 - depth_jitter, 1 + depth_jitter)
            out[q, h] = [*nrm, -float(nrm @ (d * depth))]
    return out.astype(np.float32)
