"""Second, independent restatement of the PatchMatch control logic -- TEST INFRASTRUCTURE.

RandomInitialization (random, planar-prior and reuse branches, ACMMP.cu:673-795),
CheckerboardPropagation (ACMMP.cu:938-1325) and PlaneHypothesisRefinement (ACMMP.cu:797-936),
written again from the reference source as scalar float32 Python -- one pixel at a time, in the
reference's own statement order -- NOT from oracle/acmmp_oracle.c.  Its purpose is to pin the
oracle's reading of the decision logic (adaptive neighbour picking, joint view selection, the
15 draws, aggregation, FindMin/MaxCostIndex, acceptance, refinement candidates and their RNG draw
order, the hierarchy gate), which nothing else pins: the reference has no tests or fixtures.

Injected primitives (each pinned on its own elsewhere):
  * ncc(v, px, py, plane) / geom(v, px, py, plane) -- the oracle's ComputeBilateralNCC /
    ComputeGeomConsistencyCost, checked against the float64 restatement in np_reference.py;
  * exp / sin / cos / acos -- the fixed binary32 definitions, checked against
    float64 numpy in test_detmath.py;
  * the RNG is restated here (Philox4x32-10 under curand_init(seed, subsequence = pixel, 0) and
    curand_uniform), checked against Random123 known answers in test_oracle_rng.py.

Arithmetic follows DESIGN.md §2.3: binary32 everywhere, a product whose only use is one operand of
a +/- fused into it (right-most product first), as nvcc's default contraction does.  `fma` below
is an exactly rounded binary32 fused multiply-add.  Semantics follow DESIGN.md §2.2: fix A at
:1301 and snapshot reads inside a half-sweep.
"""
from __future__ import annotations

import math

import numpy as np

F = np.float32
FLT_EPSILON = F(1.1920928955078125e-07)
CUDART_PI_F = F(3.141592654)
M_PI = 3.14159265358979323846
PINHOLE, SPHERE = 0, 11


# ---------------------------------------------------------------- binary32 helpers

def fma(a, b, c) -> np.float32:
    """Correctly rounded binary32 a*b + c (a*b is exact in binary64; TwoSum keeps the error of the
    binary64 sum, which decides a binary32 tie of the rounded sum)."""
    a, b, c = float(F(a)), float(F(b)), float(F(c))
    p = a * b
    s = p + c
    if not math.isfinite(s):
        return F(s)
    bp = s - p
    err = (p - (s - bp)) + (c - bp)
    r = F(s)
    if err != 0.0 and float(r) != s:
        other = np.nextafter(r, F(math.copysign(np.inf, s - float(r))))
        if abs(s - float(r)) == abs(float(other) - s):          # s is a binary32 midpoint
            hi, lo = (r, other) if r > other else (other, r)
            r = hi if err > 0 else lo
    return F(r)


def fmaxf(a, b):
    """C fmaxf: the non-NaN operand when one is NaN."""
    a, b = F(a), F(b)
    if a != a:
        return b
    if b != b:
        return a
    return a if a >= b else b


def fminf(a, b):
    a, b = F(a), F(b)
    if a != a:
        return b
    if b != b:
        return a
    return a if a <= b else b


def dot3(a0, a1, a2, b0, b1, b2):
    """a0*b0 + a1*b1 + a2*b2 under the contraction rule."""
    return fma(a2, b2, fma(a1, b1, F(a0) * F(b0)))


class Elementary:
    """exp/sin/cos/acos by the fixed definitions (injected, cached per argument)."""

    def __init__(self, detmath):
        self._dm = detmath
        self._cache = {}

    def _f(self, name, x):
        key = (name, F(x).tobytes())
        r = self._cache.get(key)
        if r is None:
            r = F(self._dm(name, np.array([x], np.float32))[0])
            self._cache[key] = r
        return r

    def exp(self, x):
        return self._f("exp", x)

    def sin(self, x):
        return self._f("sin", x)

    def cos(self, x):
        return self._f("cos", x)

    def acos(self, x):
        return self._f("acos", x)


def rsqrt(x):
    return F(1.0) / F(np.sqrt(F(x)))


# ---------------------------------------------------------------- RNG (curand Philox4_32_10 + curand_uniform)

_M0, _M1, _W0, _W1 = 0xD2511F53, 0xCD9E8D57, 0x9E3779B9, 0xBB67AE85


def philox4x32_10(ctr, key):
    c0, c1, c2, c3 = ctr
    k0, k1 = key
    for _ in range(10):
        p0, p1 = _M0 * c0, _M1 * c2
        c0, c1, c2, c3 = ((p1 >> 32) ^ c1 ^ k0) & 0xFFFFFFFF, p1 & 0xFFFFFFFF, \
                         ((p0 >> 32) ^ c3 ^ k1) & 0xFFFFFFFF, p0 & 0xFFFFFFFF
        k0, k1 = (k0 + _W0) & 0xFFFFFFFF, (k1 + _W1) & 0xFFFFFFFF
    return c0, c1, c2, c3


class PixelRng:
    """curand_init(seed, subsequence = pixel, offset = 0); uniform() = draw n of that stream."""

    def __init__(self, seed: int, pixel: int, n: int = 0):
        self.key = (seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
        self.pixel = pixel
        self.n = n
        self._blk = None

    def uniform(self):
        b = self.n >> 2
        if self._blk is None or self._blk[0] != b:
            self._blk = (b, philox4x32_10((b, 0, self.pixel & 0xFFFFFFFF, self.pixel >> 32), self.key))
        x = self._blk[1][self.n & 3]
        self.n += 1
        # _curand_uniform: x * 2^-32 + 2^-33 (contracted)
        return fma(F(x), F(2.3283064365386963e-10), F(1.1641532182693481e-10))


# ---------------------------------------------------------------- camera model (ACMMP.cu:119-193, 378-396)

class Rig:
    def __init__(self, cam, E: Elementary):
        self.c = cam
        self.E = E
        self.model = int(cam["model"])
        self.K = [F(v) for v in cam["K"]]
        self.R = [F(v) for v in cam["R"]]
        self.params = [F(v) for v in cam["params"]]
        self.W, self.H = int(cam["width"]), int(cam["height"])
        self._dir = {}

    def pixel_to_dir(self, px, py):
        """PixelToDir, ACMMP.cu:119-134."""
        key = (px, py)
        d = self._dir.get(key)
        if d is not None:
            return d
        if self.model == PINHOLE:
            x = (F(px) - self.K[2]) / self.K[0]
            y = (F(py) - self.K[5]) / self.K[4]
            z = F(1.0)
            inv = rsqrt(dot3(x, y, z, x, y, z))                      # NormalizeVec3 :110-117
            d = (x * inv, y * inv, z * inv)
        else:
            lon = (F(px) - self.params[1]) / F(self.W) * F(2.0) * CUDART_PI_F
            lat = -(F(py) - self.params[2]) / F(self.H) * CUDART_PI_F
            d = (self.E.cos(lat) * self.E.sin(lon), -self.E.sin(lat), self.E.cos(lat) * self.E.cos(lon))
        self._dir[key] = d
        return d

    def depth_from_plane(self, ph, px, py):
        """ComputeDepthfromPlaneHypothesis, ACMMP.cu:187-193."""
        d = self.pixel_to_dir(px, py)
        denom = dot3(ph[0], ph[1], ph[2], d[0], d[1], d[2])
        return F(1e6) if abs(denom) < F(1e-6) else -ph[3] / denom

    def dist_to_origin(self, px, py, depth, n):
        """GetDistance2Origin / Get3DPoint, ACMMP.cu:153-173."""
        d = self.pixel_to_dir(px, py)
        X = (d[0] * depth, d[1] * depth, d[2] * depth)
        return -dot3(n[0], n[1], n[2], X[0], X[1], X[2])

    def to_ref(self, n):
        """TransformNormal2RefCam, ACMMP.cu:388-396."""
        R = self.R
        return [dot3(R[0], R[1], R[2], n[0], n[1], n[2]), dot3(R[3], R[4], R[5], n[0], n[1], n[2]),
                dot3(R[6], R[7], R[8], n[0], n[1], n[2]), F(n[3])]


def normalize3(v):
    inv = rsqrt(dot3(v[0], v[1], v[2], v[0], v[1], v[2]))
    return [v[0] * inv, v[1] * inv, v[2] * inv] + list(v[3:])


def sample_depth_inv(rs: PixelRng, dmin, dmax):
    """SampleDepthInv, ACMMP.cu:14-22."""
    dmin = fmaxf(dmin, F(1e-6))
    dmax = fmaxf(dmax, dmin + F(1e-6))
    inv_min = F(1.0) / dmax
    inv_max = F(1.0) / dmin
    u = rs.uniform()
    inv = fma(u, inv_max - inv_min, inv_min)
    return F(1.0) / inv


def random_normal(rig: Rig, px, py, rs: PixelRng):
    """GenerateRandomNormal, ACMMP.cu:194-220 (Marsaglia)."""
    q1, q2, s = F(1.0), F(1.0), F(2.0)
    while s >= F(1.0):
        q1 = fma(F(2.0), rs.uniform(), F(-1.0))
        q2 = fma(F(2.0), rs.uniform(), F(-1.0))
        s = fma(q2, q2, q1 * q1)
    sq = F(np.sqrt(F(1.0) - s))
    n = [F(2.0) * q1 * sq, F(2.0) * q2 * sq, fma(F(-2.0), s, F(1.0)), F(0.0)]
    v = rig.pixel_to_dir(px, py)
    if dot3(n[0], n[1], n[2], v[0], v[1], v[2]) > F(0.0):
        n = [-n[0], -n[1], -n[2], n[3]]
    return normalize3(n)


def perturbed_normal(rig: Rig, px, py, n, rs: PixelRng, perturbation):
    """GeneratePerturbedNormal, ACMMP.cu:222-257."""
    E = rig.E
    v = rig.pixel_to_dir(px, py)
    a1 = (rs.uniform() - F(0.5)) * F(perturbation)
    a2 = (rs.uniform() - F(0.5)) * F(perturbation)
    a3 = (rs.uniform() - F(0.5)) * F(perturbation)
    s1, s2, s3 = E.sin(a1), E.sin(a2), E.sin(a3)
    c1, c2, c3 = E.cos(a1), E.cos(a2), E.cos(a3)
    R = [c2 * c3,
         fma(-c1, s3, c3 * s1 * s2),                  # cos_a3*sin_a1*sin_a2 - cos_a1*sin_a3
         fma(c1 * c3, s2, s1 * s3),                   # sin_a1*sin_a3 + cos_a1*cos_a3*sin_a2
         c2 * s3,
         fma(s1 * s2, s3, c1 * c3),                   # cos_a1*cos_a3 + sin_a1*sin_a2*sin_a3
         fma(-c3, s1, c1 * s2 * s3),                  # cos_a1*sin_a2*sin_a3 - cos_a3*sin_a1
         -s2, c2 * s1, c1 * c2]
    p = [dot3(R[0], R[1], R[2], n[0], n[1], n[2]), dot3(R[3], R[4], R[5], n[0], n[1], n[2]),
         dot3(R[6], R[7], R[8], n[0], n[1], n[2]), F(n[3])]
    if dot3(p[0], p[1], p[2], v[0], v[1], v[2]) >= F(0.0):
        p = [F(x) for x in n]
    return normalize3(p)


# ---------------------------------------------------------------- the restated kernels

class Restatement:
    """State layout: planes (H, W, 4) float32, costs, pre_costs (H, W) float32, selected (H, W)
    uint32, draws (H, W) = RNG draws each pixel's stream has consumed."""

    def __init__(self, images, cams, params, seed, ncc, geom, detmath, prior=None, masks=None):
        self.E = Elementary(detmath)
        self.rig = Rig(cams[0], self.E)
        self.N = len(images)
        self.V = self.N - 1
        self.H, self.W = images[0].shape
        self.p = params
        self.seed = int(seed)
        self.ncc_fn, self.geom_fn = ncc, geom
        self.prior, self.masks = prior, masks
        self._ncc = {}

    # ComputeMultiViewCostVector, ACMMP.cu:558-563 (v = 0..V-1 -> source image v+1)
    def ncc(self, v, px, py, plane):
        key = (v, px, py, np.asarray(plane, np.float32).tobytes())
        c = self._ncc.get(key)
        if c is None:
            c = F(self.ncc_fn(v + 1, px, py, np.asarray(plane, np.float32)))
            self._ncc[key] = c
        return c

    def geom(self, v, px, py, plane):
        return F(self.geom_fn(v + 1, px, py, np.asarray(plane, np.float32)))

    def rng(self, px, py, draws):
        return PixelRng(self.seed, py * self.W + px, int(draws))

    # ComputeMultiViewInitialCostandSelectedViews, ACMMP.cu:519-556
    def initial_cost(self, px, py, plane):
        cost_max = F(2.0)
        cv = [self.ncc(v, px, py, plane) for v in range(self.V)]
        num_valid = sum(1 for c in cv if c < cost_max)
        srt = list(cv)
        for i in range(1, len(srt)):                              # sort_small :36-45 (insertion)
            tmp, j = srt[i], i
            while j >= 1 and tmp < srt[j - 1]:
                srt[j] = srt[j - 1]
                j -= 1
            srt[j] = tmp
        sel = 0
        top_k = min(num_valid, int(self.p["top_k"]))
        if top_k > 0:
            cost = F(0.0)
            for i in range(top_k):
                cost = cost + srt[i]
            thr = srt[top_k - 1]
            for i in range(self.V):
                if cv[i] <= thr:
                    sel |= 1 << i
            return cost / F(top_k), sel
        return cost_max, sel

    # RandomInitialization, ACMMP.cu:673-795 (random, planar prior and reuse branches)
    def init(self, planes, costs, selected, draws, scaled=None):
        p, rig = self.p, self.rig
        geom, hier, planar = bool(p["geom_consistency"]), bool(p["hierarchy"]), bool(p["planar_prior"])
        if hier and not geom and not planar and bool(p["upsample"]):
            raise NotImplementedError("upsample branch (JBU-style) is not restated here")
        dmin, dmax = F(p["depth_min"]), F(p["depth_max"])
        for py in range(self.H):
            for px in range(self.W):
                rs = self.rng(px, py, 0)
                if not geom and not hier:
                    depth = fma(rs.uniform(), dmax - dmin, dmin)      # :259-265 (linear depth)
                    ph = random_normal(rig, px, py, rs)
                    ph[3] = rig.dist_to_origin(px, py, depth, ph)
                elif planar:
                    if self.masks[py, px] > 0 and costs[py, px] >= F(0.1):
                        perturbation = F(0.02)
                        pp = [F(v) for v in self.prior[py, px]]
                        dp = pp[3]
                        dmn = (F(1) - F(3) * perturbation) * dp
                        dmx = (F(1) + F(3) * perturbation) * dp
                        dp = fma(rs.uniform(), dmx - dmn, dmn)
                        # 3 * perturbation * M_PI: a float product promoted to double (:698)
                        ph = perturbed_normal(rig, px, py, pp, rs, F(float(F(3) * perturbation) * M_PI))
                        ph[3] = dp
                    else:
                        ph = [F(v) for v in planes[py, px]]
                        ph[3] = rig.dist_to_origin(px, py, ph[3], ph)
                else:
                    src = scaled[py, px] if hier else planes[py, px]
                    ph = rig.to_ref([F(v) for v in src])
                    ph[3] = rig.dist_to_origin(px, py, ph[3], ph)
                planes[py, px] = ph
                costs[py, px], selected[py, px] = self.initial_cost(px, py, ph)
                draws[py, px] = rs.n

    def checker_rows(self):
        return min(self.H, 32 * (((self.H // 2) + 15) // 16))     # grid of Black/RedPixelUpdate :1511-1530

    # one Black (colour 0) or Red (colour 1) PixelUpdate launch, ACMMP.cu:1327-1349
    def half_sweep(self, planes, costs, pre_costs, selected, draws, colour, it, trace=None):
        snap_planes, snap_costs, snap_sel = planes.copy(), costs.copy(), selected.copy()   # snapshot reads
        with np.errstate(all="ignore"):                      # 0/0 costs when no view is drawn (:1227, :1243)
            for py in range(self.checker_rows()):
                for px in range((py + colour) & 1, self.W, 2):
                    self.propagate(snap_planes, snap_costs, snap_sel, planes, costs, pre_costs, selected, draws,
                                   px, py, it, trace)

    # CheckerboardPropagation, ACMMP.cu:938-1325
    def propagate(self, P, Cst, S, planes, costs, pre_costs, selected, draws, px, py, it, trace):
        p, rig, V, W, H = self.p, self.rig, self.V, self.W, self.H
        rs = self.rng(px, py, draws[py, px])
        draws0 = rs.n
        geom = bool(p["geom_consistency"])
        dmin, dmax = F(p["depth_min"]), F(p["depth_max"])

        def cost_at(x, y):
            return Cst[y, x]

        # adaptive checkerboard sampling :952-1143; directions 0 up_near 1 up_far 2 down_near 3 down_far
        # 4 left_near 5 left_far 6 right_near 7 right_far; positions as (x, y)
        flag = [False] * 8
        pos = [None] * 8
        cost_array = [[F(0.0)] * 32 for _ in range(8)]
        cost_array[0][0] = F(2.0)                                   # `float cost_array[8][32] = {2.0f}`

        def scan(start, steps):
            best, bx = cost_at(*start), start
            for q in steps:
                c = cost_at(*q)
                if c < best:
                    best, bx = c, q
            return bx

        if py > 2:
            flag[1] = True
            pos[1] = scan((px, py - 3), [(px, py - 3 - 2 * i) for i in range(1, 11) if py > 2 + 2 * i])
        if py < H - 3:
            flag[3] = True
            pos[3] = scan((px, py + 3), [(px, py + 3 + 2 * i) for i in range(1, 11) if py < H - 3 - 2 * i])
        if px > 2:
            flag[5] = True
            pos[5] = scan((px - 3, py), [(px - 3 - 2 * i, py) for i in range(1, 11) if px > 2 + 2 * i])
        if px < W - 3:
            flag[7] = True
            pos[7] = scan((px + 3, py), [(px + 3 + 2 * i, py) for i in range(1, 11) if px < W - 3 - 2 * i])

        def vshape(start, cand):
            steps = []
            for i in range(3):
                for ok, q in cand(i):
                    if ok:
                        steps.append(q)
            return scan(start, steps)

        if py > 0:        # up_near - (1+i)*width -+ i
            flag[0] = True
            pos[0] = vshape((px, py - 1), lambda i: [(py > 1 + i and px > i, (px - i, py - 2 - i)),
                                                     (py > 1 + i and px < W - 1 - i, (px + i, py - 2 - i))])
        if py < H - 1:
            flag[2] = True
            pos[2] = vshape((px, py + 1), lambda i: [(py < H - 2 - i and px > i, (px - i, py + 2 + i)),
                                                     (py < H - 2 - i and px < W - 1 - i, (px + i, py + 2 + i))])
        if px > 0:
            flag[4] = True
            pos[4] = vshape((px - 1, py), lambda i: [(px > 1 + i and py > i, (px - 2 - i, py - i)),
                                                     (px > 1 + i and py < H - 1 - i, (px - 2 - i, py + i))])
        if px < W - 1:
            flag[6] = True
            pos[6] = vshape((px + 1, py), lambda i: [(px < W - 2 - i and py > i, (px + 2 + i, py - i)),
                                                     (px < W - 2 - i and py < H - 1 - i, (px + 2 + i, py + i))])
        # the reference evaluates far directions first, then near ones: same values either way
        for d in range(8):
            if flag[d]:
                nb = P[pos[d][1], pos[d][0]]
                for v in range(V):
                    cost_array[d][v] = self.ncc(v, px, py, nb)

        # joint view selection :1146-1208
        view_weights = [F(0.0)] * 32
        priors = [F(0.0)] * 32
        nbr = [(px, py - 1), (px, py + 1), (px - 1, py), (px + 1, py)]
        for i in range(4):
            if flag[2 * i]:
                sv = int(S[nbr[i][1], nbr[i][0]])
                for j in range(V):
                    priors[j] = priors[j] + (F(0.9) if (sv >> j) & 1 else F(0.1))
        probs = [F(0.0)] * 32
        cost_threshold = F(0.8 * float(self.E.exp(F(it * it) / F(-90.0))))
        for i in range(V):
            count, count_false, tmpw = F(0.0), 0, F(0.0)
            for j in range(8):
                c = cost_array[j][i]
                if c < cost_threshold:
                    tmpw = tmpw + self.E.exp(c * c / F(-0.18))
                    count = count + F(1.0)
                if c > F(1.2):
                    count_false += 1
            if count > F(2) and count_false < 3:
                probs[i] = tmpw / count
            elif count_false < 3:
                probs[i] = self.E.exp(cost_threshold * cost_threshold / F(-0.32))
            probs[i] = probs[i] * priors[i]
        prob_sum = F(0.0)                                            # TransformPDFToCDF :137-151
        for i in range(V):
            prob_sum = prob_sum + probs[i]
        inv_prob_sum = F(1.0) / prob_sum
        cum = F(0.0)
        for i in range(V):
            cum = fma(probs[i], inv_prob_sum, cum)                   # cum_prob += probs[i] * inv (contracted)
            probs[i] = cum
        for _ in range(15):
            rand_prob = rs.uniform() - FLT_EPSILON
            for image_id in range(V):
                if probs[image_id] > rand_prob:
                    view_weights[image_id] = view_weights[image_id] + F(1.0)
                    break
        temp_sel, weight_norm = 0, F(0.0)
        for i in range(V):
            if view_weights[i] > F(0):
                temp_sel |= 1 << i
                weight_norm = weight_norm + view_weights[i]

        # aggregated costs :1210-1228
        final_costs = [F(0.0)] * 8
        for i in range(8):
            fc = F(0.0)
            for j in range(V):
                if view_weights[j] > F(0):
                    if geom:
                        if flag[i]:
                            g = self.geom(j, px, py, P[pos[i][1], pos[i][0]])
                            fc = fma(view_weights[j], fma(F(0.2), g, cost_array[i][j]), fc)
                        else:
                            fc = fma(view_weights[j], cost_array[i][j] + F(0.1) * F(3.0), fc)
                    else:
                        fc = fma(view_weights[j], cost_array[i][j], fc)
            final_costs[i] = fc / weight_norm
        min_idx = 0                                                  # FindMinCostIndex :62-73
        for i in range(1, 8):
            if final_costs[i] <= final_costs[min_idx]:
                min_idx = i

        # current hypothesis :1230-1245 (every view; a zero weight times a finite cost adds +0)
        own = [F(v) for v in P[py, px]]
        cost_now = F(0.0)
        for i in range(V):
            c = self.ncc(i, px, py, own)
            if geom:
                cost_now = fma(view_weights[i], fma(F(0.2), self.geom(i, px, py, own), c), cost_now)
            else:
                cost_now = fma(view_weights[i], c, cost_now)
        cost_now = cost_now / weight_norm
        out_cost = cost_now                                          # costs[center] = cost_now (:1245)
        out_plane = own
        out_sel = int(S[py, px])
        depth_now = rig.depth_from_plane(own, px, py)
        restricted_cost = F(0.0)
        accepted, max_idx_tr = 8, -1
        center_prior = None
        if bool(p["planar_prior"]):                                   # :1247-1299
            gamma = F(0.5)
            depth_sigma = (dmax - dmin) / F(64.0)
            two_dss = F(2) * depth_sigma * depth_sigma
            angle_sigma = F(M_PI * float(F(5.0) / F(180.0)))
            two_ass = F(2) * angle_sigma * angle_sigma
            center_prior = [F(v) for v in self.prior[py, px]]
            depth_prior = rig.depth_from_plane(center_prior, px, py)
            beta = F(0.18)

            def prior_term(plane, depth):
                ddiff = depth - depth_prior
                ad = self.E.acos(dot3(center_prior[0], center_prior[1], center_prior[2], plane[0], plane[1], plane[2]))
                return fma(self.E.exp(-ddiff * ddiff / two_dss), self.E.exp(-ad * ad / two_ass), gamma)

            if self.masks[py, px] > 0:
                rfc = [F(0.0)] * 8
                for i in range(8):
                    if flag[i]:
                        nb = P[pos[i][1], pos[i][0]]
                        rfc[i] = self.E.exp(-final_costs[i] * final_costs[i] / beta) * \
                            prior_term(nb, rig.depth_from_plane(nb, px, py))
                max_idx = 0                                          # FindMaxCostIndex :75-86
                for i in range(1, 8):
                    if rfc[i] >= rfc[max_idx]:
                        max_idx = i
                max_idx_tr = max_idx
                rc_now = self.E.exp(-cost_now * cost_now / beta) * prior_term(own, rig.depth_from_plane(own, px, py))
                if flag[max_idx]:
                    nb = [F(v) for v in P[pos[max_idx][1], pos[max_idx][0]]]
                    db = rig.depth_from_plane(nb, px, py)
                    if db >= dmin and db <= dmax and rfc[max_idx] > rc_now:
                        depth_now = db
                        out_plane = nb
                        out_cost = final_costs[max_idx]
                        restricted_cost = rfc[max_idx]
                        out_sel = temp_sel
                        accepted = max_idx
            elif flag[min_idx]:
                nb = [F(v) for v in P[pos[min_idx][1], pos[min_idx][0]]]
                db = rig.depth_from_plane(nb, px, py)
                if db >= dmin and db <= dmax and final_costs[min_idx] < cost_now:
                    depth_now = db
                    out_plane = nb
                    out_cost = final_costs[min_idx]
                    accepted = min_idx

        plane_now = list(out_plane)                                  # fix A: plane_hypotheses[center] at :1301
        if not bool(p["planar_prior"]) and flag[min_idx]:           # :1302-1311
            nb = [F(v) for v in P[pos[min_idx][1], pos[min_idx][0]]]
            db = rig.depth_from_plane(nb, px, py)
            if db >= dmin and db <= dmax and final_costs[min_idx] < cost_now:
                depth_now = db
                plane_now = nb
                cost_now = final_costs[min_idx]
                out_sel = temp_sel
                accepted = min_idx
        cost_now_cur = cost_now

        st = {"plane": plane_now, "depth": depth_now, "cost": cost_now, "restricted": restricted_cost,
              "accepted": accepted}
        self.refine(st, rs, view_weights, weight_norm, px, py)
        plane_now, cost_now = st["plane"], st["cost"]

        if bool(p["hierarchy"]):                                      # :1315-1324
            if cost_now < pre_costs[py, px] - F(0.1):
                out_cost, out_plane = cost_now, plane_now
        else:
            out_cost, out_plane = cost_now, plane_now
        planes[py, px] = out_plane
        costs[py, px] = out_cost
        selected[py, px] = out_sel
        draws[py, px] = rs.n
        if trace is not None:
            t = trace[py, px]
            t["pos"] = [(q[1] * W + q[0]) if f else -1 for q, f in zip(pos, flag)]
            t["final_costs"] = final_costs
            t["cost_now"] = cost_now_cur
            t["min_idx"] = min_idx
            t["max_idx"] = max_idx_tr
            t["accepted"] = st["accepted"]
            t["temp_selected_views"] = temp_sel
            t["draws_before"] = draws0
            t["draws_after"] = rs.n
            t["view_weights"] = [int(w) for w in view_weights]

    # PlaneHypothesisRefinement, ACMMP.cu:797-936
    def refine(self, st, rs, view_weights, weight_norm, px, py):
        if weight_norm <= F(0.0):
            return
        p, rig, V = self.p, self.rig, self.V
        dmin, dmax = F(p["depth_min"]), F(p["depth_max"])
        perturbation = F(0.02)
        gamma = F(0.5)
        depth_sigma = (dmax - dmin) / F(64.0)
        two_dss = F(2) * depth_sigma * depth_sigma
        angle_sigma = CUDART_PI_F * (F(5.0) / F(180.0))
        two_ass = F(2) * angle_sigma * angle_sigma
        beta = F(0.18)
        use_prior = bool(p["planar_prior"]) and self.masks[py, px] > 0
        if use_prior:
            prior = [F(v) for v in self.prior[py, px]]
            depth_prior = rig.depth_from_plane(prior, px, py)
            depth_rand = sample_depth_inv(rs, fmaxf(depth_prior - F(3) * depth_sigma, dmin),
                                          fminf(depth_prior + F(3) * depth_sigma, dmax))
            n_rand = perturbed_normal(rig, px, py, prior, rs, angle_sigma)
        else:
            depth_rand = sample_depth_inv(rs, dmin, dmax)
            n_rand = random_normal(rig, px, py, rs)
        depth = st["depth"]
        lo = fmaxf((F(1.0) - perturbation) * depth, dmin)
        hi = fminf((F(1.0) + perturbation) * depth, dmax)
        if not (hi > lo):
            lo, hi = dmin, dmax
        depth_perturbed, ok = depth, False
        for _ in range(32):
            cand = sample_depth_inv(rs, lo, hi)
            if cand >= dmin and cand <= dmax:
                depth_perturbed, ok = cand, True
                break
        if not ok:
            depth_perturbed = fminf(fmaxf(depth, dmin), dmax)
        plane = st["plane"]
        n_pert = perturbed_normal(rig, px, py, plane, rs, perturbation * CUDART_PI_F)
        depths = [depth_rand, depth, depth_rand, depth, depth_perturbed]
        normals = [plane, n_rand, n_rand, n_pert, plane]
        for i in range(5):
            tp = [F(v) for v in normals[i]]
            tp[3] = rig.dist_to_origin(px, py, depths[i], tp)
            temp_cost = F(0.0)
            for j in range(V):
                if view_weights[j] > F(0.0):
                    c = self.ncc(j, px, py, tp)
                    if bool(p["geom_consistency"]):
                        temp_cost = fma(view_weights[j], fma(F(0.1), self.geom(j, px, py, tp), c), temp_cost)
                    else:
                        temp_cost = fma(view_weights[j], c, temp_cost)
            if weight_norm > F(0.0):
                temp_cost = temp_cost / weight_norm
            depth_before = rig.depth_from_plane(tp, px, py)
            if depth_before < dmin or depth_before > dmax or depth_before >= F(1e6):
                continue
            if use_prior:
                ddiff = depths[i] - depth_prior
                ac = dot3(prior[0], prior[1], prior[2], tp[0], tp[1], tp[2])
                ac = fminf(fmaxf(ac, F(-1.0)), F(1.0))
                ad = self.E.acos(ac)
                pr = fma(self.E.exp(-ddiff * ddiff / two_dss), self.E.exp(-ad * ad / two_ass), gamma)
                rtc = self.E.exp(-temp_cost * temp_cost / beta) * pr
                if rtc > st["restricted"]:
                    st.update(depth=depth_before, plane=tp, cost=temp_cost, restricted=rtc, accepted=9 + i)
            elif temp_cost < st["cost"]:
                st.update(depth=depth_before, plane=tp, cost=temp_cost, accepted=9 + i)
