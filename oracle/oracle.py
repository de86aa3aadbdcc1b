"""ctypes front-end of the CPU oracle -- ORACLE / TEST INFRASTRUCTURE ONLY.

Loaded only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
PARITY UNPINNED (see oracle/acmmp_oracle.h).  Builds oracle/liboracle.so on demand
with the recipe in oracle/Makefile.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

# Own copies of the ABI dtypes (the oracle does not import product code).
CAMERA_DTYPE = np.dtype([("model", "<i4"), ("params", "<f4", (4,)), ("R", "<f4", (9,)), ("t", "<f4", (3,)),
                         ("K", "<f4", (9,)), ("width", "<i4"), ("height", "<i4"),
                         ("depth_min", "<f4"), ("depth_max", "<f4")])
assert CAMERA_DTYPE.itemsize == 120
PARAMS_SIZE = 68


class _Problem(C.Structure):
    _fields_ = [("num_images", C.c_int32), ("cams", C.c_void_p), ("images", C.c_void_p),
                ("depths", C.c_void_p), ("depth_w", C.c_void_p), ("depth_h", C.c_void_p),
                ("scaled_planes", C.c_void_p), ("scaled_w", C.c_int32), ("scaled_h", C.c_int32),
                ("prior_planes", C.c_void_p), ("plane_masks", C.c_void_p)]


class _State(C.Structure):
    _fields_ = [("planes", C.c_void_p), ("costs", C.c_void_p), ("pre_costs", C.c_void_p),
                ("selected_views", C.c_void_p)]


_lib = None


def build(force: bool = False) -> str:
    srcs = ["acmmp_oracle.c", "acmmp_oracle.h", "detmath_ref.h", "philox_ref.h"]
    newest = max(os.path.getmtime(os.path.join(HERE, s)) for s in srcs)
    if force or not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < newest:
        subprocess.run(["make", "-s", "-C", HERE, "liboracle.so"], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        vp, i32, f32 = C.c_void_p, C.c_int32, C.c_float
        L.or_run_patchmatch.argtypes = [vp, vp, vp, C.c_uint64, i32, i32, i32]
        L.or_run_patchmatch.restype = C.c_int
        L.or_run_band.argtypes = [vp, vp, vp, C.c_uint64, i32, i32, i32, i32, i32]
        L.or_run_band.restype = C.c_int
        for fn in ("or_bilateral_ncc", "or_geom_cost"):
            getattr(L, fn).argtypes = [vp, vp, i32, i32, i32, vp]
            getattr(L, fn).restype = f32
        L.or_initial_cost.argtypes = [vp, vp, i32, i32, vp, vp]
        L.or_initial_cost.restype = f32
        L.or_pixel_to_dir.argtypes = [vp, i32, i32, vp]
        L.or_project.argtypes = [vp, vp, vp, vp]
        L.or_world_point.argtypes = [vp, f32, f32, f32, vp]
        L.or_jbu.argtypes = [vp, i32, i32, vp, i32, i32, i32, vp, i32]
        L.or_detmath_eval.argtypes = [i32, vp, vp, vp, C.c_int64]
        L.or_fuse.argtypes = [i32, vp, vp, vp, vp, i32, i32, vp, vp]
        L.or_fuse.restype = i32
        L.or_philox.argtypes = [vp, vp, vp]
        L.or_uniform_draw.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32]
        L.or_uniform_draw.restype = f32
        L.or_set_trace.argtypes = [vp]
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


class Problem:
    """Keeps every array the C side points at alive."""

    def __init__(self, images, cameras, params, depths=None, scaled_planes=None, prior_planes=None,
                 plane_masks=None):
        self.images = [np.ascontiguousarray(im, np.float32) for im in images]
        cams = np.frombuffer(np.ascontiguousarray(cameras).tobytes(), dtype=CAMERA_DTYPE).copy()
        self.cams = cams
        self.params = np.frombuffer(np.asarray(params).tobytes(), dtype=np.uint8).copy()
        assert self.params.size == PARAMS_SIZE
        n = len(self.images)
        self._img_ptrs = (C.c_void_p * n)(*[im.ctypes.data for im in self.images])
        self.depths = None
        self._dep_ptrs = None
        if depths is not None:
            self.depths = [np.ascontiguousarray(d, np.float32) for d in depths]
            self._dep_ptrs = (C.c_void_p * n)(*[d.ctypes.data for d in self.depths])
            self.depth_w = np.array([d.shape[1] for d in self.depths], np.int32)
            self.depth_h = np.array([d.shape[0] for d in self.depths], np.int32)
        self.scaled = None if scaled_planes is None else np.ascontiguousarray(scaled_planes, np.float32)
        self.prior = None if prior_planes is None else np.ascontiguousarray(prior_planes, np.float32)
        self.masks = None if plane_masks is None else np.ascontiguousarray(plane_masks, np.uint32)
        s = _Problem()
        s.num_images = n
        s.cams = self.cams.ctypes.data
        s.images = C.cast(self._img_ptrs, C.c_void_p)
        if self.depths is not None:
            s.depths = C.cast(self._dep_ptrs, C.c_void_p)
            s.depth_w = self.depth_w.ctypes.data
            s.depth_h = self.depth_h.ctypes.data
        if self.scaled is not None:
            s.scaled_planes = self.scaled.ctypes.data
            s.scaled_w = self.scaled.shape[1]
            s.scaled_h = self.scaled.shape[0]
        if self.prior is not None:
            s.prior_planes = self.prior.ctypes.data
        if self.masks is not None:
            s.plane_masks = self.masks.ctypes.data
        self.struct = s

    @property
    def shape(self):
        return int(self.cams[0]["height"]), int(self.cams[0]["width"])


def run_patchmatch(prob: Problem, seed: int, planes=None, costs=None, pre_costs=None, selected=None,
                   n_half_sweeps: int = -1, do_post: bool = True, nthreads: int = 0):
    """Returns dict(planes (H,W,4), costs, pre_costs, selected_views) after the run."""
    H, W = prob.shape
    planes = np.zeros((H, W, 4), np.float32) if planes is None else np.array(planes, np.float32, copy=True)
    costs = np.zeros((H, W), np.float32) if costs is None else np.array(costs, np.float32, copy=True)
    pre = np.zeros((H, W), np.float32) if pre_costs is None else np.array(pre_costs, np.float32, copy=True)
    sel = np.zeros((H, W), np.uint32) if selected is None else np.array(selected, np.uint32, copy=True)
    st = _State(planes.ctypes.data, costs.ctypes.data, pre.ctypes.data, sel.ctypes.data)
    rc = lib().or_run_patchmatch(C.byref(prob.struct), prob.params.ctypes.data, C.byref(st),
                                 C.c_uint64(seed), n_half_sweeps, int(do_post), nthreads)
    if rc != 0:
        raise RuntimeError(f"or_run_patchmatch failed ({rc})")
    return {"planes": planes, "costs": costs, "pre_costs": pre, "selected_views": sel}


TRACE_DTYPE = np.dtype([("pos", "<i4", (8,)), ("final_costs", "<f4", (8,)), ("cost_now", "<f4"),
                        ("min_idx", "<i4"), ("max_idx", "<i4"), ("accepted", "<i4"),
                        ("temp_selected_views", "<u4"), ("draws_before", "<u4"), ("draws_after", "<u4"),
                        ("view_weights", "u1", (32,))])


def run_patchmatch_traced(prob: Problem, seed: int, **kw):
    """run_patchmatch plus the per-pixel trace of each pixel's last half-sweep update (or_trace)."""
    H, W = prob.shape
    tr = np.zeros((H, W), TRACE_DTYPE)
    tr["min_idx"] = -2
    lib().or_set_trace(tr.ctypes.data)
    try:
        out = run_patchmatch(prob, seed, **kw)
    finally:
        lib().or_set_trace(None)
    out["trace"] = tr
    return out


def run_band(prob: Problem, seed: int, row0: int, row1: int, nthreads: int = 0, n_half_sweeps: int = -1,
             planes=None, costs=None, pre_costs=None, selected=None, do_post: bool = True):
    """The full per-pixel pipeline on rows [row0, row1) only (the CPU-baseline sample, and full-size
    parity bands).  `planes` / `costs` / ... are the state a geom, planar-prior or reuse pass starts
    from (as run_patchmatch); rows outside the band keep it untouched."""
    H, W = prob.shape
    planes = np.zeros((H, W, 4), np.float32) if planes is None else np.array(planes, np.float32, copy=True)
    costs = np.zeros((H, W), np.float32) if costs is None else np.array(costs, np.float32, copy=True)
    pre = np.zeros((H, W), np.float32) if pre_costs is None else np.array(pre_costs, np.float32, copy=True)
    sel = np.zeros((H, W), np.uint32) if selected is None else np.array(selected, np.uint32, copy=True)
    st = _State(planes.ctypes.data, costs.ctypes.data, pre.ctypes.data, sel.ctypes.data)
    rc = lib().or_run_band(C.byref(prob.struct), prob.params.ctypes.data, C.byref(st), C.c_uint64(seed),
                           n_half_sweeps, nthreads, row0, row1, int(do_post))
    if rc != 0:
        raise RuntimeError(f"or_run_band failed ({rc})")
    return {"planes": planes, "costs": costs, "pre_costs": pre, "selected_views": sel}


def ncc(prob: Problem, src: int, px: int, py: int, plane) -> float:
    pl = np.asarray(plane, np.float32)
    return float(lib().or_bilateral_ncc(C.byref(prob.struct), prob.params.ctypes.data, src, px, py, _ptr(pl)))


def geom_cost(prob: Problem, src: int, px: int, py: int, plane) -> float:
    pl = np.asarray(plane, np.float32)
    return float(lib().or_geom_cost(C.byref(prob.struct), prob.params.ctypes.data, src, px, py, _ptr(pl)))


def initial_cost(prob: Problem, px: int, py: int, plane):
    pl = np.asarray(plane, np.float32)
    sel = np.zeros(1, np.uint32)
    c = lib().or_initial_cost(C.byref(prob.struct), prob.params.ctypes.data, px, py, _ptr(pl), _ptr(sel))
    return float(c), int(sel[0])


def jbu(ref, coarse, imagescale: int, nthreads: int = 0):
    ref = np.ascontiguousarray(ref, np.float32)
    coarse = np.ascontiguousarray(coarse, np.float32)
    out = np.zeros_like(ref)
    lib().or_jbu(_ptr(ref), ref.shape[1], ref.shape[0], _ptr(coarse), coarse.shape[1], coarse.shape[0],
                 imagescale, _ptr(out), nthreads)
    return out


DETMATH_FN = {"exp": 0, "sin": 1, "cos": 2, "asin": 3, "acos": 4, "atan2": 5, "rsqrt": 6, "f2i_sat": 7}


def fuse(cams, depths, normals, rgba, ref: int, srcs) -> np.ndarray:
    """SimpleFusionKernel + in-order collection for one reference view -> (n, 9) float32."""
    cams = np.frombuffer(np.ascontiguousarray(cams).tobytes(), dtype=CAMERA_DTYPE).copy()
    d = [np.ascontiguousarray(a, np.float32) for a in depths]
    nm = [np.ascontiguousarray(a, np.float32) for a in normals]
    cl = [np.ascontiguousarray(a, np.float32) for a in rgba]
    n = len(d)
    pd = (C.c_void_p * n)(*[a.ctypes.data for a in d])
    pn = (C.c_void_p * n)(*[a.ctypes.data for a in nm])
    pc = (C.c_void_p * n)(*[a.ctypes.data for a in cl])
    s = np.ascontiguousarray(srcs, np.int32)
    L = lib()
    cnt = L.or_fuse(n, _ptr(cams), C.cast(pd, C.c_void_p), C.cast(pn, C.c_void_p), C.cast(pc, C.c_void_p), ref,
                    s.size, _ptr(s), None)
    out = np.zeros((max(cnt, 1), 9), np.float32)
    L.or_fuse(n, _ptr(cams), C.cast(pd, C.c_void_p), C.cast(pn, C.c_void_p), C.cast(pc, C.c_void_p), ref,
              s.size, _ptr(s), _ptr(out))
    return out[:cnt]


def detmath(fn: str, x, y=None):
    x = np.ascontiguousarray(x, np.float32)
    y = np.ascontiguousarray(np.zeros_like(x) if y is None else y, np.float32)
    out = np.empty_like(x)
    lib().or_detmath_eval(DETMATH_FN[fn], _ptr(x), _ptr(y), _ptr(out), x.size)
    return out


def philox(ctr, key):
    c = np.asarray(ctr, np.uint32)
    k = np.asarray(key, np.uint32)
    out = np.zeros(4, np.uint32)
    lib().or_philox(_ptr(c), _ptr(k), _ptr(out))
    return out


def uniform_draw(seed: int, subsequence: int, n: int) -> float:
    return float(lib().or_uniform_draw(seed, subsequence, n))
