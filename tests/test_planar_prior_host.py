"""Planar-prior host side on the CPU: the C-ABI host functions against
independent numpy restatements of ACMMP.cpp:904-1011 / main.cpp:113-181, and the Delaunay
triangulation against its defining properties (cv::Subdiv2D itself is unavailable: the
triangle order and co-circular tie-breaks are parity unpinned)."""
import math

import numpy as np
import pytest

from acmmp import capi, types


def np_support_points(costs):
    """GetSupportPoints, ACMMP.cpp:904-930, literally."""
    H, W = costs.shape
    out = []
    for col in range(0, W, 5):
        for row in range(0, H, 5):
            best, pt = np.float32(2.0), None
            for c in range(col, min(W, col + 5)):
                for r in range(row, min(H, row + 5)):
                    v = costs[r, c]
                    if v < np.float32(2.0) and best > v:
                        pt, best = (c, r), v
            if best < np.float32(0.1):
                out.append(pt)
    return np.array(out, np.int32).reshape(-1, 2)


def test_support_points_match_restatement():
    rng = np.random.default_rng(3)
    costs = rng.uniform(0, 0.4, (37, 53)).astype(np.float32)
    costs[rng.random(costs.shape) < 0.3] = 2.0
    costs[5:10, 5:10] = np.nan                                  # NaN never wins (comparisons false)
    got = capi.support_points(costs)
    ref = np_support_points(costs)
    assert got.shape == ref.shape and np.array_equal(got, ref)
    assert capi.support_points(np.full((7, 7), 2.0, np.float32)).shape == (0, 2)


def _circumcircle_empty(tri, pts):
    (ax, ay), (bx, by), (cx, cy) = [tuple(map(int, v)) for v in tri]
    for (dx, dy) in pts:
        m = [[ax - dx, ay - dy, (ax - dx) ** 2 + (ay - dy) ** 2],
             [bx - dx, by - dy, (bx - dx) ** 2 + (by - dy) ** 2],
             [cx - dx, cy - dy, (cx - dx) ** 2 + (cy - dy) ** 2]]
        det = (m[0][0] * (m[1][1] * m[2][2] - m[1][2] * m[2][1]) - m[0][1] * (m[1][0] * m[2][2] - m[1][2] * m[2][0])
               + m[0][2] * (m[1][0] * m[2][1] - m[1][1] * m[2][0]))
        if det > 0:
            return False
    return True


def _hull(pts, keep_collinear):
    pts = sorted(set(map(tuple, pts)))

    def cross(o, a, b):
        return (a[0] - o[0]) * (b[1] - o[1]) - (a[1] - o[1]) * (b[0] - o[0])
    lower, upper = [], []
    for p in pts:
        while len(lower) >= 2 and (cross(lower[-2], lower[-1], p) < 0 if keep_collinear
                                   else cross(lower[-2], lower[-1], p) <= 0):
            lower.pop()
        lower.append(p)
    for p in reversed(pts):
        while len(upper) >= 2 and (cross(upper[-2], upper[-1], p) < 0 if keep_collinear
                                   else cross(upper[-2], upper[-1], p) <= 0):
            upper.pop()
        upper.append(p)
    return lower[:-1] + upper[:-1]


def _hull_size(pts):
    """points on the hull boundary, collinear ones included (Euler: #tri = 2n - 2 - h)"""
    return len(_hull(pts, True))


def _area2(poly):
    return sum(poly[i][0] * poly[(i + 1) % len(poly)][1] - poly[(i + 1) % len(poly)][0] * poly[i][1]
               for i in range(len(poly)))


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_delaunay_properties(seed):
    rng = np.random.default_rng(seed)
    W, H = 300, 200
    # one point per 5x5 tile at a random offset (the support-point layout), some tiles empty
    pts = [(c + rng.integers(0, 5), r + rng.integers(0, 5)) for c in range(0, 60, 5) for r in range(0, 40, 5)
           if rng.random() < 0.8]
    pts = np.array(pts, np.int32)
    tri = capi.delaunay(pts, W, H)
    n, h = len(pts), _hull_size(pts)
    assert len(tri) == 2 * n - 2 - h                            # Euler: a triangulation of the hull
    for t in tri:
        (ax, ay), (bx, by), (cx, cy) = t
        assert (bx - ax) * (cy - ay) - (by - ay) * (cx - ax) > 0  # counter-clockwise, non-degenerate
        assert _circumcircle_empty(t, pts)                    # Delaunay
    area2 = sum(int((t[1][0] - t[0][0]) * (t[2][1] - t[0][1]) - (t[1][1] - t[0][1]) * (t[2][0] - t[0][0]))
                for t in tri)
    assert area2 == _area2(_hull(pts, False))                  # the triangles tile the convex hull
    assert capi.delaunay(np.zeros((0, 2), np.int32), W, H).shape[0] == 0


def test_delaunay_cocircular_grid_is_a_valid_triangulation():
    xs, ys = np.meshgrid(np.arange(0, 50, 5), np.arange(0, 30, 5))
    pts = np.stack([xs.ravel(), ys.ravel()], 1).astype(np.int32)  # every cell co-circular
    tri = capi.delaunay(pts, 60, 40)
    assert len(tri) == 2 * len(pts) - 2 - _hull_size(pts)
    for t in tri:
        assert _circumcircle_empty(t, pts)


def np_point_on_ref_cam(x, y, depth, cam):
    """Get3DPointonRefCam (ACMMP.cpp:287-312) with the reference's float/double promotions."""
    f32 = np.float32
    if int(cam["model"]) == types.SPHERE:
        p = cam["params"]
        lon = f32((f32(f32(x) - p[1]) / f32(cam["width"])) * f32(2.0) * math.pi)
        lat = f32(-(f32(f32(y) - p[2]) / f32(cam["height"])) * math.pi)
        cl, sl, co, so = np.cos(lat), np.sin(lat), np.cos(lon), np.sin(lon)
        return np.array([f32(cl * so) * depth, f32(-sl) * depth, f32(cl * co) * depth], np.float32)
    K = cam["K"]
    return np.array([f32(depth * f32(f32(x) - K[2])) / K[0], f32(depth * f32(f32(y) - K[5])) / K[4], depth],
                    np.float32)


@pytest.mark.parametrize("model", [types.PINHOLE, types.SPHERE])
def test_prior_plane_recovers_a_true_plane(model):
    W, H = 120, 80
    if model == types.SPHERE:
        cam = types.make_camera(types.SPHERE, params=[W / (2 * math.pi), W / 2, H / 2], width=W, height=H)
    else:
        cam = types.make_camera(types.PINHOLE, K=[[100, 0, W / 2], [0, 100, H / 2], [0, 0, 1]], width=W, height=H)
    n = np.array([0.2, -0.3, -1.0])
    n /= np.linalg.norm(n)
    w = 4.0                                                      # plane n.X + w = 0, in front of the camera
    depths = np.zeros((H, W), np.float32)
    for y in range(H):
        for x in range(W):
            depths[y, x] = np.float32(capi.depth_from_plane_param(cam, np.array([*n, w], np.float32), x, y))
    tri = np.array([[10, 10], [90, 15], [40, 60]], np.int32)
    pl = capi.prior_plane_params(cam, depths, tri)
    assert pl[3] >= 0 and abs(np.linalg.norm(pl[:3]) - 1) < 1e-5
    assert np.allclose(pl[:3], n, atol=2e-3) and abs(pl[3] - w) < 1e-2
    # the triangle's vertices lie on the returned plane
    for x, y in tri:
        X = np_point_on_ref_cam(x, y, depths[y, x], cam)
        assert abs(float(np.dot(pl[:3], X) + pl[3])) < 1e-3
        assert abs(capi.depth_from_plane_param(cam, pl, x, y) - depths[y, x]) < 1e-3 * abs(depths[y, x])


def np_raster(tri, W, H, label, mask):
    """main.cpp:142-155: float p/q steps, float partial sums promoted to double, int truncation."""
    (x1, y1), (x2, y2), (x3, y3) = [tuple(map(int, v)) for v in tri]
    f32 = np.float32
    L = [math.sqrt((a - c) ** 2 + (b - d) ** 2) for (a, b, c, d) in
         ((x1, y1, x2, y2), (x1, y1, x3, y3), (x2, y2, x3, y3))]
    L = [f32(v) for v in L]
    step = f32(1.0 / max(L))
    p = f32(0.0)
    while p < 1.0:
        q = f32(0.0)
        while q < 1.0 - float(p):
            x = int(float(f32(f32(p * f32(x1)) + f32(q * f32(x2)))) + (1.0 - float(p) - float(q)) * x3)
            y = int(float(f32(f32(p * f32(y1)) + f32(q * f32(y2)))) + (1.0 - float(p) - float(q)) * y3)
            mask[y, x] = label
            q = f32(q + step)
        p = f32(p + step)


@pytest.mark.parametrize("model", [types.PINHOLE, types.SPHERE])
def test_planar_prior_host_pipeline_matches_restatement(model):
    # (SPHERE: the host half fits its planes with the row / column trig tables, prior_plane_params with libm per
    # vertex -- the same bits)
    W, H = 90, 60
    if model == types.SPHERE:
        cam = types.make_camera(types.SPHERE, params=[W / (2 * math.pi), W / 2, H / 2], width=W, height=H,
                                depth_min=2.0, depth_max=9.0)
    else:
        cam = types.make_camera(types.PINHOLE, K=[[80, 0, W / 2], [0, 80, H / 2], [0, 0, 1]], width=W, height=H,
                                depth_min=2.0, depth_max=9.0)
    rng = np.random.default_rng(5)
    depths = rng.uniform(3, 6, (H, W)).astype(np.float32)
    costs = rng.uniform(0, 0.3, (H, W)).astype(np.float32)
    prior, masks, ntri = capi.planar_prior_host(cam, depths, costs, 2.0 * 0.6, 9.0 * 1.2)
    # independent composition of the pieces, as main.cpp:120-181 does
    pts = capi.support_points(costs)
    tri = capi.delaunay(pts, W, H)
    assert ntri == len(tri)
    lab = np.zeros((H, W), np.float32)
    planes = []
    for k, t in enumerate(tri):
        np_raster(t, W, H, np.float32(k + 1.0), lab)
        planes.append(capi.prior_plane_params(cam, depths, t))
    for j in range(H):
        for i in range(W):
            if lab[j, i] > 0:
                d = capi.depth_from_plane_param(cam, planes[int(lab[j, i]) - 1], i, j)
                if not (d <= 9.0 * 1.2 and d >= 2.0 * 0.6):
                    lab[j, i] = 0
    assert np.array_equal(masks, lab.astype(np.uint32))
    exp = np.zeros((H, W, 4), np.float32)
    for j, i in zip(*np.nonzero(lab)):
        exp[j, i] = planes[int(lab[j, i]) - 1]
    assert np.array_equal(prior.view(np.uint32), exp.view(np.uint32))
    assert (masks > 0).mean() > 0.5


def _locally_delaunay(tri):
    """A triangulation (n, 3, 2) of integer points tiles its hull and is Delaunay iff every interior edge is
    locally Delaunay: the far vertex of the triangle across it lies on or outside the circumcircle (exact
    integer arithmetic in Python ints)."""
    edges = {}
    for k, t in enumerate(tri.tolist()):                     # Python ints: no fixed-width overflow below
        for j in range(3):
            a, b = tuple(t[(j + 1) % 3]), tuple(t[(j + 2) % 3])
            edges[(a, b)] = (k, tuple(t[j]))
    for (a, b), (k, c) in edges.items():
        other = edges.get((b, a))
        if other is None:
            continue
        d = other[1]
        # in-circle of d against the CCW triangle (a, b, c)
        adx, ady, bdx, bdy, cdx, cdy = a[0] - d[0], a[1] - d[1], b[0] - d[0], b[1] - d[1], c[0] - d[0], c[1] - d[1]
        det = ((adx * adx + ady * ady) * (bdx * cdy - bdy * cdx) - (bdx * bdx + bdy * bdy) * (adx * cdy - ady * cdx)
               + (cdx * cdx + cdy * cdy) * (adx * bdy - ady * bdx))
        if det > 0:
            return False
    return True


@pytest.mark.parametrize("layout", ["support", "grid", "general"])
@pytest.mark.parametrize("threads", ["1", "8"])
def test_divide_and_conquer_delaunay(monkeypatch, layout, threads):
    """The divide-and-conquer triangulation (Dwyer strips, parallel merges) on support-point layouts big enough
    to take its threaded path: a Delaunay triangulation of the hull (Euler count, orientation, local Delaunay
    edges, area), independent of the thread count, and -- points in general position, where the Delaunay
    triangulation is unique -- the incremental form's triangles exactly (ACMMP_DELAUNAY_INCREMENTAL)."""
    rng = np.random.default_rng(11)
    if layout == "support":
        W, H = 1000, 600
        pts = [(c + rng.integers(0, 5), r + rng.integers(0, 5)) for c in range(0, W, 5) for r in range(0, H, 5)
               if rng.random() < 0.4]
    elif layout == "grid":
        W, H = 600, 400
        pts = [(c, r) for c in range(0, W, 5) for r in range(0, H, 5)]                  # co-circular everywhere
    else:
        W, H = 16000, 16000
        pts = list({(int(x), int(y)) for x, y in rng.integers(0, W, (12000, 2))})
    pts = np.array(pts, np.int32)
    monkeypatch.setenv("ACMMP_DELAUNAY_THREADS", threads)
    tri = capi.delaunay(pts, W, H)
    monkeypatch.setenv("ACMMP_DELAUNAY_THREADS", "3")
    again = capi.delaunay(pts, W, H)
    np.testing.assert_array_equal(tri, again)                   # the thread count does not change the result
    assert len(tri) == 2 * len(pts) - 2 - _hull_size(pts)
    t = tri.astype(np.int64)
    orient = (t[:, 1, 0] - t[:, 0, 0]) * (t[:, 2, 1] - t[:, 0, 1]) - (t[:, 1, 1] - t[:, 0, 1]) * (t[:, 2, 0] - t[:, 0, 0])
    assert (orient > 0).all()
    assert int(orient.sum()) == _area2(_hull(pts, False))
    assert _locally_delaunay(tri)
    if layout == "general":
        monkeypatch.setenv("ACMMP_DELAUNAY_INCREMENTAL", "1")
        np.testing.assert_array_equal(capi.delaunay(pts, W, H), tri)


def test_concurrent_delaunay_calls_share_the_host_pool():
    """Several contexts' planar blocks triangulate at once (the pipeline's overlapped planar passes) on the one
    process-wide host worker pool (planar_prior.cpp HostPool): every concurrent call's triangles equal its serial
    result."""
    from concurrent.futures import ThreadPoolExecutor
    rng = np.random.default_rng(23)
    cases = []
    for k in range(4):
        W, H = 800 + 200 * k, 600 + 100 * k
        pts = np.array([(c + rng.integers(0, 5), r + rng.integers(0, 5)) for c in range(0, W, 5) for r in range(0, H, 5)
                        if rng.random() < 0.35 + 0.1 * k], np.int32)
        cases.append((pts, W, H))
    serial = [capi.delaunay(p, W, H) for p, W, H in cases]
    with ThreadPoolExecutor(4) as ex:
        futs = [ex.submit(capi.delaunay, p, W, H) for _ in range(3) for p, W, H in cases]
        got = [f.result() for f in futs]
    for k, g in enumerate(got):
        np.testing.assert_array_equal(g, serial[k % len(cases)])
