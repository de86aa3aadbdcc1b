"""Multi-view, multi-scale pipeline driver.

Restates the reference's scheduler (main.cpp:392-482), ProcessProblem (main.cpp:73-210),
JointBilateralUpsampling (main.cpp:212-238) and the host half of InuputInitialization /
CudaSpaceInitialization (ACMMP.cpp:567-845) over the C ABI -- with the dmb round trip between
passes replaced by an in-memory depth store:

* each process drives one GPU (one `capi.Context`, reused for every ProcessProblem);
* reference views are sharded over the ranks (`owner(i) = i % world`, no data-path collective
  inside a pass);
* between passes, the depth maps a geometric-consistency pass reads are broadcast from their
  owners HBM-to-HBM (RCCL over xGMI, `RcclExchange`) and uploaded device-to-device;
* dmb files are still written (optional) so a reference user finds the usual outputs.

Pass ordering.  The reference runs each pass's views one after another, and a geom pass with
multi_geometry reads the depths_geom.dmb its predecessors in the SAME pass have just rewritten
(main.cpp:443-445 + ACMMP.cpp:653-664).  `order="reference"` reproduces that (single rank);
`order="snapshot"` lets every view of a pass read the previous pass's maps (Jacobi order), which
is what a sharded multi-GPU run does.  Everything else is identical.

Seeds.  The reference seeds from clock64(); here every RunPatchMatch gets
seed + 7919 * pass + 31 * ref_image_id + run.
"""
from __future__ import annotations

import contextlib
import copy
import math
import os
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field

import numpy as np

from . import capi, io, types


# ---------------------------------------------------------------- inputs

@dataclass
class Dataset:
    """What the reference reads from a dense folder: grey images (float32, full size), cameras
    (ReadCamera, width/height = image size) and the problems of pair.txt (indexed by image id,
    as the reference indexes problems[src_id], ACMMP.cpp:611)."""
    images: dict
    cameras: dict
    problems: list
    folder: str | None = None
    colors: dict | None = None        # optional BGR uint8 images for fusion (IMREAD_COLOR); grey otherwise


def read_gray(path: str) -> np.ndarray:
    """cv::imread(IMREAD_GRAYSCALE) + convertTo(CV_32F) (ACMMP.cpp:578-580).  PIL decodes the JPEG
    luma plane directly (draft 'L'); decoder differences vs OpenCV's libjpeg build are not pinned."""
    from PIL import Image
    with Image.open(path) as im:
        if im.format == "JPEG":
            im.draft("L", im.size)
        return np.asarray(im.convert("L"), dtype=np.float32).copy()


def read_bgr(path: str) -> np.ndarray:
    """cv::imread(IMREAD_COLOR): 8-bit BGR."""
    from PIL import Image
    with Image.open(path) as im:
        return np.asarray(im.convert("RGB"), dtype=np.uint8)[..., ::-1].copy()


def load_dataset(dense_folder: str, with_colors: bool = False) -> Dataset:
    problems = io.read_pair_list(dense_folder)
    images, cameras, colors = {}, {}, ({} if with_colors else None)
    for p in problems:
        i = p.ref_image_id
        images[i] = read_gray(os.path.join(dense_folder, "images", f"{i:08d}.jpg"))
        if with_colors:
            colors[i] = read_bgr(os.path.join(dense_folder, "images", f"{i:08d}.jpg"))
        cam = io.read_camera(os.path.join(dense_folder, "cams", f"{i:08d}_cam.txt"))
        cam["height"], cam["width"] = images[i].shape
        cameras[i] = cam
    return Dataset(images, cameras, problems, dense_folder, colors)


def resize_linear(img: np.ndarray, new_cols: int, new_rows: int) -> np.ndarray:
    """cv::resize(INTER_LINEAR) of a float32 image (resizeGeneric_: HResizeLinear then VResizeLinear
    with float coefficients; source coordinate (d + 0.5) * scale - 0.5, clamped at the borders).
    OpenCV's SIMD kernels may fuse the multiply-adds: parity with cv::resize is unpinned."""
    src = np.ascontiguousarray(img, np.float32)
    rows, cols = src.shape

    def taps(dsize, ssize):
        scale = ssize / dsize
        d = np.arange(dsize, dtype=np.float64)
        f = ((d + 0.5) * scale - 0.5).astype(np.float32)
        s = np.floor(f).astype(np.int64)
        f = (f - s.astype(np.float32)).astype(np.float32)
        lo = s < 0
        f[lo], s[lo] = 0.0, 0
        hi = s >= ssize - 1
        f[hi], s[hi] = 0.0, ssize - 1
        s1 = np.minimum(s + 1, ssize - 1)
        return s, s1, (np.float32(1.0) - f).astype(np.float32), f

    xs0, xs1, ax0, ax1 = taps(new_cols, cols)
    ys0, ys1, by0, by1 = taps(new_rows, rows)
    # the same float32 products and sums as (src[:, xs0] * ax0 + src[:, xs1] * ax1) and the vertical
    # equivalent, computed in place (no float64 promotion, fewer temporaries)
    h = np.take(src, xs0, axis=1)
    h *= ax0
    t = np.take(src, xs1, axis=1)
    t *= ax1
    h += t
    out = np.take(h, ys0, axis=0)
    out *= by0[:, None]
    t = np.take(h, ys1, axis=0)
    t *= by1[:, None]
    out += t
    return out


def resize_linear_u8(img: np.ndarray, new_cols: int, new_rows: int) -> np.ndarray:
    """cv::resize(INTER_LINEAR) of an 8-bit image (any channel count): OpenCV's fixed-point path --
    coefficients rounded to 11 bits, horizontal sums kept as ints, vertical pass
    (b0 * S0 + b1 * S1 + 2^21) >> 22.  SIMD-path details are not pinned."""
    src = np.asarray(img, np.uint8)
    if src.ndim == 2:
        return resize_linear_u8(src[..., None], new_cols, new_rows)[..., 0]
    rows, cols = src.shape[:2]

    def taps(dsize, ssize):
        scale = ssize / dsize
        d = np.arange(dsize, dtype=np.float64)
        f = ((d + 0.5) * scale - 0.5).astype(np.float32)
        s0 = np.floor(f).astype(np.int64)
        f = (f - s0.astype(np.float32)).astype(np.float32)
        lo = s0 < 0
        f[lo], s0[lo] = 0.0, 0
        hi = s0 >= ssize - 1
        f[hi], s0[hi] = 0.0, ssize - 1
        s1 = np.minimum(s0 + 1, ssize - 1)
        a0 = np.rint((np.float32(1.0) - f) * np.float32(2048.0)).astype(np.int64)
        a1 = np.rint(f * np.float32(2048.0)).astype(np.int64)
        return s0, s1, a0, a1

    xs0, xs1, ax0, ax1 = taps(new_cols, cols)
    ys0, ys1, by0, by1 = taps(new_rows, rows)
    S = src.astype(np.int64)
    h = S[:, xs0, :] * ax0[None, :, None] + S[:, xs1, :] * ax1[None, :, None]
    v = h[ys0] * by0[:, None, None] + h[ys1] * by1[:, None, None]
    return np.clip((v + (1 << 21)) >> 22, 0, 255).astype(np.uint8)


def rescale_image_and_camera(bgr: np.ndarray, depth_shape, cam: np.ndarray):
    """RescaleImageAndCamera (ACMMP.cpp:213-246): camera size := depth size; image resized to it
    (INTER_LINEAR) and (cx, cy) / K scaled when the sizes differ."""
    cam = np.array(cam, copy=True)
    rows, cols = depth_shape
    cam["width"], cam["height"] = cols, rows
    if bgr.shape[0] == rows and bgr.shape[1] == cols:
        return np.array(bgr, copy=True), cam
    sx = np.float32(cols) / np.float32(bgr.shape[1])
    sy = np.float32(rows) / np.float32(bgr.shape[0])
    out = resize_linear_u8(bgr, cols, rows)
    if int(cam["model"]) == types.SPHERE:
        cam["params"][1] = np.float32(cam["params"][1] * sx)
        cam["params"][2] = np.float32(cam["params"][2] * sy)
    else:
        K = cam["K"]
        K[0] = np.float32(K[0] * sx); K[2] = np.float32(K[2] * sx)
        K[4] = np.float32(K[4] * sy); K[5] = np.float32(K[5] * sy)
        cam["K"] = K
    return out, cam


def fusion_inputs(ds: "Dataset", store, problems):
    """RunFusionCuda's loading loop (ACMMP.cu:1833-1886): per view the final depth map
    (depths_geom), normals and the colour image rescaled to the depth size, with its camera."""
    cams, depths, normals, colours = [], [], [], []
    for p in problems:
        i = p.ref_image_id
        d = store.get("depths_geom", i)
        n = store.get("normals", i)
        bgr = ds.colors[i] if ds.colors and i in ds.colors else \
            np.repeat(np.clip(np.round(ds.images[i]), 0, 255).astype(np.uint8)[..., None], 3, axis=2)
        img, cam = rescale_image_and_camera(bgr, d.shape, ds.cameras[i])
        cams.append(cam); depths.append(d); normals.append(n); colours.append(img)
    return np.array(cams, dtype=types.CAMERA_DTYPE), depths, normals, colours


def cpp_round(x) -> int:
    """std::round of a non-negative float: half away from zero (np.round rounds half to even)."""
    return int(math.floor(float(x) + 0.5))


def round_dims(rows: int, cols: int, size: int):
    """std::round(rows * factor), std::round(cols * factor) with the float32 factor
    min(size / cols, size / rows) (ACMMP.cpp:616-621, main.cpp:227-231)."""
    factor = min(np.float32(size) / np.float32(cols), np.float32(size) / np.float32(rows))
    return cpp_round(np.float32(rows) * factor), cpp_round(np.float32(cols) * factor)


def scaled_dims(rows: int, cols: int, max_image_size: int):
    """(rows, cols) after InuputInitialization's rescale (ACMMP.cpp:607-617): float32 factor, rounded."""
    if cols <= max_image_size and rows <= max_image_size:
        return rows, cols
    return round_dims(rows, cols, max_image_size)


def scale_view(image: np.ndarray, cam: np.ndarray, max_image_size: int):
    """InuputInitialization's per-view rescale (ACMMP.cpp:607-643): only when the image exceeds
    max_image_size; SPHERE scales (cx, cy), PINHOLE scales K."""
    cam = np.array(cam, copy=True)
    rows, cols = image.shape
    if cols <= max_image_size and rows <= max_image_size:
        return image, cam
    new_rows, new_cols = scaled_dims(rows, cols, max_image_size)
    sx = np.float32(new_cols) / np.float32(cols)
    sy = np.float32(new_rows) / np.float32(rows)
    out = resize_linear(image, new_cols, new_rows)
    if int(cam["model"]) == types.SPHERE:
        cam["params"][1] = np.float32(cam["params"][1] * sx)
        cam["params"][2] = np.float32(cam["params"][2] * sy)
    else:
        K = cam["K"]
        K[0] = np.float32(K[0] * sx); K[2] = np.float32(K[2] * sx)
        K[4] = np.float32(K[4] * sy); K[5] = np.float32(K[5] * sy)
        cam["K"] = K
    cam["height"], cam["width"] = out.shape
    return out, cam


# ---------------------------------------------------------------- depth exchange between ranks

class LocalExchange:
    """Single rank: every view is local, nothing to move."""
    world, rank = 1, 0

    def share(self, key, views, owners, store):
        pass

    def close(self):
        pass


class ExchangeMismatch(RuntimeError):
    """A map some rank holds after the depth exchange differs from its owner's."""


def mismatched_maps(comm, checksums) -> list:
    """Indices of the maps whose checksum is not the same on every rank of `comm` (one allreduce-max over
    the 32-bit halves and their negations: max == min on every rank iff all ranks agree).  Each map's owner
    passes the checksum it took BEFORE the broadcast and every other rank the one of what it received, so
    agreement means every rank holds the owner's bytes (a broadcast from the wrong root overwrites the owner's
    buffer too, so post-broadcast checksums alone would agree on the wrong map).  comm: anything with
    allreduce_max(float64 array) -> array."""
    c = np.asarray(checksums, np.uint64)
    n = c.size
    if n == 0:
        return []
    hi = (c >> np.uint64(32)).astype(np.float64)
    lo = (c & np.uint64(0xFFFFFFFF)).astype(np.float64)
    m = np.asarray(comm.allreduce_max(np.concatenate([hi, lo, -hi, -lo])), np.float64)
    return [i for i in range(n) if m[i] != -m[2 * n + i] or m[n + i] != -m[3 * n + i]]


class RcclExchange:
    """Depth maps live in HBM (DeviceBuffer per (key, view)); a pass's outputs are broadcast from
    their owners with one grouped RCCL call.  verify (default on; ACMMP_VERIFY_EXCHANGE=0 turns it off):
    after the broadcast every rank checksums each map it now holds (acmmp_device_checksum, in HBM) and the
    ranks compare them (mismatched_maps), so a wrong root, buffer or ordering stops the run."""

    def __init__(self, comm: capi.Comm, device: int, verify: bool | None = None):
        self.comm, self.device = comm, device
        self.world, self.rank = comm.nranks, comm.rank
        self.verify = os.environ.get("ACMMP_VERIFY_EXCHANGE", "1") != "0" if verify is None else verify
        self.maps_verified = 0

    def share(self, key, views, owners, store):
        bufs = [store.device_map(key, v) for v in views]
        # the broadcast reads maps the engine contexts exported on their own streams: order it after them
        producers = store.take_producers()
        for ctx in producers:
            self.comm.after(ctx)
        pre = {}
        if self.verify:
            for ctx in producers:                    # the exports complete before the owner checksums them
                ctx.synchronize()
            pre = {i: bufs[i].checksum() for i, v in enumerate(views) if owners[v] == self.rank}
        self.comm.broadcast(bufs, [owners[v] for v in views])
        if self.verify:
            post = [b.checksum() for b in bufs]
            # an owner whose own buffer changed in the broadcast reports the complement of its checksum
            sums = [post[i] if i not in pre else (pre[i] if post[i] == pre[i] else pre[i] ^ ((1 << 64) - 1))
                    for i in range(len(bufs))]
            bad = mismatched_maps(self.comm, sums)
            if bad:
                raise ExchangeMismatch(f"depth exchange of {key}: views {[views[i] for i in bad]} differ "
                                       f"between ranks after the broadcast")
            self.maps_verified += len(bufs)
        for v in views:
            if owners[v] != self.rank:
                store.host.pop((key, v), None)      # re-read from HBM on demand

    def close(self):
        self.comm.close()


class ViewStore:
    """What the reference keeps in ACMMP/2333_<id>/{depths,depths_geom,normals,costs}.dmb."""

    def __init__(self, device: int | None):
        self.device = device
        self.host = {}                               # (key, view) -> np.ndarray
        self.dev = {}                                # (key, view) -> capi.DeviceBuffer
        self.shapes = {}                             # (key, view) -> (H, W)
        self.producers = []                          # contexts that exported maps since the last exchange

    def take_producers(self):
        p, self.producers = self.producers, []
        return p

    def put(self, key, view, arr, ctx=None):
        # float32 views are kept as they are (a depth or normals slice of the downloaded planes costs no
        # copy here; consumers that need contiguous memory make it when they do)
        arr = np.asarray(arr, np.float32)
        self.host[(key, view)] = arr
        self.shapes[(key, view)] = arr.shape
        if self.device is not None and key in ("depths", "depths_geom"):
            buf = self.device_map(key, view, arr.shape)
            if ctx is not None and hasattr(ctx, "export_depth"):
                ctx.export_depth(buf)                # HBM -> HBM, no host round trip
                if all(c is not ctx for c in self.producers):
                    self.producers.append(ctx)
            else:
                buf.upload(arr)

    def device_map(self, key, view, shape=None):
        b = self.dev.get((key, view))
        shape = shape or self.shapes[(key, view)]
        if b is None or b.shape != tuple(shape):
            if b is not None:
                b.free()
            b = capi.DeviceBuffer(self.device, shape)
            self.dev[(key, view)] = b
            self.shapes[(key, view)] = tuple(shape)
        return b

    def get(self, key, view):
        a = self.host.get((key, view))
        if a is None and (key, view) in self.dev:
            a = self.dev[(key, view)].download()
            self.host[(key, view)] = a
        return a

    def has(self, key, view):
        return (key, view) in self.host or (key, view) in self.dev


# ---------------------------------------------------------------- the driver

@dataclass
class PassLog:
    name: str
    views: list = field(default_factory=list)
    compute_s: float = 0.0            # this rank's ProcessProblem calls of the pass (host wall clock)
    exchange_s: float = 0.0           # the depth-map exchange after it (world > 1)
    exchange_bytes: int = 0           # depth-map bytes every rank holds after the exchange
    stages: dict = field(default_factory=dict)   # host seconds per stage within the pass (Pipeline.stage_s)


class Pipeline:
    """main.cpp's main loop over a Dataset, sharded over `exchange.world` ranks."""

    def __init__(self, ds: Dataset, engine=None, exchange=None, device: int = 0, seed: int = 1234,
                 order: str = "reference", geom_iterations: int = 2, out_folder: str | None = None,
                 use_device_store: bool | None = None, size_bound: int = 1000, max_image_size: int = 3200,
                 log=None, reuse_planes: bool = True, math: str | None = None, overlap: bool = True):
        self.ds = ds
        # a geom pass restarts from the previous pass's depth + normals of its view, which is that
        # pass's downloaded plane array: keep it instead of re-joining the two stored maps
        self.reuse_planes = reuse_planes
        self._last_planes = {}                              # view -> (H, W, 4) planes of its last pass
        self._dev_state = {}                                # view -> [planes, costs DeviceBuffers, (H, W) held]
        self.exchange = exchange or LocalExchange()
        self.world, self.rank = self.exchange.world, self.exchange.rank
        if self.world > 1 and order == "reference":
            raise ValueError("order='reference' is sequential over views; sharded runs use order='snapshot'")
        if order not in ("reference", "snapshot"):
            raise ValueError(order)
        self.order = order
        self.device = device
        self.engine = engine if engine is not None else capi.Context(device)
        gpu = isinstance(self.engine, capi.Context)
        if math is not None and gpu:
            self.engine.set_math(math)                      # 'exact' (bit-identical) or 'fast' 
        self.store = ViewStore(device if (gpu if use_device_store is None else use_device_store) else None)
        self.seed = seed
        self.geom_iterations = geom_iterations
        self.size_bound, self.max_image_size = size_bound, max_image_size
        self.out_folder = out_folder
        self.log = log or (lambda *a: None)
        self.problems = copy.deepcopy(ds.problems)
        self.pass_index = 0
        self._scaled = {}                                   # (view, size) -> scaled image, camera
        self._scaled_dev = {}                               # (view, size) -> its DeviceBuffer (GPU engine)
        self.passes = []
        self._pending = []
        self.stage_s = {}                                   # host wall seconds per stage (profiling)
        self._stage_lock = threading.Lock()
        # planar passes: overlap views' host planar-prior blocks with later views' first RunPatchMatch
        # (`overlap` engine contexts on the same GPU, as many worker threads; _pass_overlapped).
        # overlap=True means ACMMP_PIPELINE_SLOTS (default 3) contexts; False / 1 = the sequential loop.
        slots = int(os.environ.get("ACMMP_PIPELINE_SLOTS", "3")) if overlap is True else int(overlap or 1)
        self.overlap = slots if (gpu and slots > 1) else 0
        self.geom_overlap = os.environ.get("ACMMP_PIPELINE_GEOM_OVERLAP", "1") != "0"   # (A/B knob)
        self._extra_engines = []
        self._math = math
        # prepared (padded + binary16) images of every (view, scale), shared by this pipeline's contexts:
        # each is prepared once, not once per problem that reads it
        budget = os.environ.get("ACMMP_IMAGE_CACHE_BYTES")
        budget = int(budget) if budget is not None else self._default_cache_budget(ds, max(slots, 1))
        self.image_cache = capi.ImageCache(device, budget) if gpu else None
        if gpu:
            self.log(f"engine math: {self.engine.math()}")

    @staticmethod
    def _default_cache_budget(ds, contexts):
        """Soft byte budget of the prepared-image cache: every (view, scale) of a dataset up to 32 GiB stays
        in HBM for the whole run (no re-preparation between passes); beyond that, 4x the largest problem's
        full-scale working set per context (the views a problem pins plus room for the next problem's),
        least recently used entries evicted first.  One prepared view = padded fp32 + binary16 copy."""
        def view_bytes(v):
            im = ds.images[v]
            h, w = im.shape[:2]
            return 6 * (w + 2) * (h + 2)
        views = list(ds.images)
        total = sum(view_bytes(v) for v in views) * 4 // 3           # + the coarser scales
        if total <= 32 << 30:
            return 0
        largest = max((view_bytes(p.ref_image_id) + sum(view_bytes(s) for s in p.src_image_ids)
                       for p in ds.problems if p.ref_image_id in ds.images), default=0)
        return max(32 << 30, 4 * contexts * largest)

    @contextlib.contextmanager
    def _timed(self, stage):
        t0 = time.perf_counter()
        try:
            yield
        finally:
            dt = time.perf_counter() - t0
            with self._stage_lock:
                self.stage_s[stage] = self.stage_s.get(stage, 0.0) + dt

    @property
    def _engine2(self):
        return self._extra_engines[0] if self._extra_engines else None

    def close(self):
        """Release the engine context(s) this pipeline created or was given, and its image cache."""
        for e in self._extra_engines + [self.engine]:
            if e is not None and hasattr(e, "close"):
                e.close()
        self._extra_engines = []
        if self.image_cache is not None:
            self.image_cache.close()
            self.image_cache = None
        for dev in self._dev_state.values():
            for b in dev[:2]:
                b.free()
        self._dev_state = {}

    # -- sharding
    def owner(self, i: int) -> int:
        return i % self.world

    def my_problems(self):
        return [i for i in range(len(self.problems)) if self.owner(i) == self.rank]

    # -- the schedule (main.cpp:392-482); fusion is run_fusion()
    def run(self):
        sizes = {p.ref_image_id: self.ds.images[p.ref_image_id].shape for p in self.problems}
        max_num_downscale = io.compute_multiscale_settings(self.problems, sizes, self.max_image_size,
                                                           self.size_bound)
        flag = 0
        while max_num_downscale >= 0:
            for p in self.problems:
                if p.num_downscale >= 0:
                    p.cur_image_size = int(p.max_image_size / (2 ** p.num_downscale))
                    p.num_downscale -= 1
            self._evict_scaled()
            if flag == 0:
                flag = 1
                self._pass(geom=False, planar=True, hier=False, multi=False)
            else:
                for i in self.my_problems():
                    self.joint_bilateral_upsampling(i, self.problems[i].cur_image_size)
                self._pass(geom=False, planar=True, hier=True, multi=False)
            for g in range(self.geom_iterations):
                self._pass(geom=True, planar=False, hier=False, multi=g > 0)
            max_num_downscale -= 1
        return self

    def _pass(self, geom, planar, hier, multi):
        name = ("geom" + ("_multi" if multi else "")) if geom else ("hier_planar" if hier else "planar")
        self.log(f"[rank {self.rank}] pass {self.pass_index}: {name}")
        log = PassLog(name)
        t0 = time.perf_counter()
        # a planar pass's views are independent; so are a geom pass's when it reads only the previous
        # pass's depth maps (not multi-geometry, or snapshot order)
        independent = (planar and not geom) or (geom and self.geom_overlap and (not multi or self.order == "snapshot"))
        before = dict(self.stage_s)
        if independent and self.overlap and len(self.my_problems()) > 1:
            self._pass_overlapped(geom, planar, hier, multi, log)
        else:
            for i in self.my_problems():
                self.process_problem(i, geom, planar, hier, multi)
                log.views.append(self.problems[i].ref_image_id)
        self._commit_pending()
        log.compute_s = time.perf_counter() - t0
        log.stages = {k: v - before.get(k, 0.0) for k, v in self.stage_s.items() if v - before.get(k, 0.0) > 0}
        key = "depths_geom" if geom else "depths"
        if self.world > 1:
            views = [p.ref_image_id for p in self.problems]
            owners = {self.problems[i].ref_image_id: self.owner(i) for i in range(len(self.problems))}
            for v in views:
                if owners[v] != self.rank:
                    self.store.shapes[(key, v)] = self._pass_shape(v)
            t1 = time.perf_counter()
            with self._timed("exchange"):
                self.exchange.share(key, views, owners, self.store)
            log.exchange_s = time.perf_counter() - t1
            log.exchange_bytes = sum(4 * int(np.prod(self.store.shapes[(key, v)])) for v in views)
        self.passes.append(log)
        self.pass_index += 1

    def _pass_shape(self, view_id):
        rows, cols = self.ds.images[view_id].shape[:2]
        return scaled_dims(rows, cols, self.problems[view_id].cur_image_size)

    def _evict_scaled(self):
        """Drop the rescaled images (host and HBM) of sizes no view uses any more."""
        for key in [k for k in self._scaled if k[1] != self.problems[k[0]].cur_image_size]:
            del self._scaled[key]
        for key in [k for k in self._scaled_dev if k[1] != self.problems[k[0]].cur_image_size]:
            self._scaled_dev.pop(key).free()
        capi._POOL.release()                 # idle download mappings are sized for the previous scale

    def _commit_pending(self):
        for key, view, arr, ctx in self._pending:
            self.store.put(key, view, arr)
        self._pending = []

    def _save(self, key, view, arr, export_ctx=None):
        if self.order == "snapshot" and key in ("depths", "depths_geom"):
            self._pending.append((key, view, arr, None))
        else:
            self.store.put(key, view, arr, export_ctx)

    # -- InuputInitialization (ACMMP.cpp:567-679)
    def _inputs(self, idx):
        prob = self.problems[idx]
        ids = [prob.ref_image_id] + list(prob.src_image_ids)
        images, cams, keys = [], [], []
        for k, vid in enumerate(ids):
            size = prob.cur_image_size if k == 0 else self.problems[vid].cur_image_size
            key = (vid, size)
            if key not in self._scaled:                     # each view is rescaled once per scale
                self._scaled[key] = scale_view(self.ds.images[vid], self.ds.cameras[vid], size)
            img, cam = self._scaled[key]
            images.append(img)
            cams.append(cam)
            keys.append(key)
        self._keys = keys
        return ids, images, np.array(cams, dtype=types.CAMERA_DTYPE)

    def _upload_views(self, e, images, cams):
        """The problem's images: with a GPU engine and device store, each view's image of one scale is
        copied to HBM once and every problem reading it uploads it device to device."""
        if self.store.device is None or not hasattr(e, "upload_views_device"):
            e.upload_views(images, cams)
            return
        bufs = []
        for key, img in zip(self._keys, images):
            b = self._scaled_dev.get(key)
            if b is None:
                b = capi.DeviceBuffer(self.store.device, img.shape)
                b.upload(img)
                self._scaled_dev[key] = b
            bufs.append(b)
        if self.image_cache is not None and isinstance(e, capi.Context):
            keys = [((vid + 1) << 24) | size for vid, size in self._keys]
            e.upload_views_device(bufs, cams, cache=self.image_cache, keys=keys)
        else:
            e.upload_views_device(bufs, cams)

    def _pass_overlapped(self, geom, planar, hier, multi, log):
        """A pass over `self.overlap` engine contexts on the GPU: view k's second half runs on a worker
        thread while the main thread runs the next views' first halves on the other contexts.  In a
        planar pass the second half is the host planar prior, the second RunPatchMatch and the store
        (several views' host planar blocks -- Delaunay, on the host as in the reference -- in flight at
        once); in a geom pass it is the download of the planes and costs and the store, so the next
        view's kernels run while they copy.  Only passes whose views are independent come here (each
        reads its own view's earlier-pass state and the previous pass's depth maps), so the outputs are
        those of the sequential loop."""
        n = self.overlap
        while len(self._extra_engines) < n - 1:
            e = capi.Context(self.device)
            if self._math is not None:
                e.set_math(self._math)
            self._extra_engines.append(e)
        engines = [self.engine] + self._extra_engines[:n - 1]
        busy = [None] * n
        with ThreadPoolExecutor(n) as pool:
            for k, i in enumerate(self.my_problems()):
                slot = k % n
                if busy[slot] is not None:
                    busy[slot].result()                      # the context is free again
                head = self._problem_head(i, geom, planar, hier, multi, engines[slot], defer_download=True)
                busy[slot] = pool.submit(self._problem_tail, head)
                log.views.append(self.problems[i].ref_image_id)
            for f in busy:
                if f is not None:
                    f.result()

    # -- ProcessProblem (main.cpp:73-210)
    def process_problem(self, idx, geom, planar, hier, multi):
        return self._problem_tail(self._problem_head(idx, geom, planar, hier, multi, self.engine))

    def _problem_head(self, idx, geom, planar, hier, multi, e, defer_download=False):
        """InuputInitialization, CudaSpaceInitialization and the first RunPatchMatch of ProcessProblem."""
        prob = self.problems[idx]
        ref = prob.ref_image_id
        with self._timed("inputs"):
            ids, images, cams = self._inputs(idx)
        c0 = cams[0]
        p = types.default_params(num_images=len(images), depth_min=float(c0["depth_min"]) * 0.6,
                                 depth_max=float(c0["depth_max"]) * 1.2)
        p["depth_min"] = np.float32(c0["depth_min"] * np.float32(0.6))
        p["depth_max"] = np.float32(c0["depth_max"] * np.float32(1.2))
        if geom:                                                     # SetGeomConsistencyParams
            p["geom_consistency"] = 1
            p["max_iterations"] = 2
            p["multi_geometry"] = int(multi)
        if hier:
            p["hierarchy"] = 1
        H, W = images[0].shape
        with self._timed("upload"):
            self._upload(e, p, images, cams, ids, ref, geom, hier, H, W)
        run_seed = self.seed + 7919 * self.pass_index + 31 * ref
        with self._timed("patchmatch"):
            e.run_patchmatch(run_seed)
            # a planar pass's first run feeds only the planar block, which a GPU context takes from HBM;
            # an overlapped geom pass downloads in the second half
            skip = (planar and self._state_planar(e)) or (defer_download and not planar)
            planes, costs = (None, None) if skip else e.download()
        return dict(e=e, p=p, c0=c0, ref=ref, geom=geom, planar=planar, run_seed=run_seed, planes=planes, costs=costs)

    def _problem_tail(self, st):
        """The planar block (main.cpp:113-187) with its second RunPatchMatch, and the stores."""
        e, p, c0, ref, geom, planar, run_seed = (st[k] for k in ("e", "p", "c0", "ref", "geom", "planar", "run_seed"))
        planes, costs = st["planes"], st["costs"]
        if planes is None and not planar:
            with self._timed("download"):
                planes, costs = e.download()
        if planar:                                                   # main.cpp:113-187
            p["planar_prior"] = 1
            if self._state_planar(e):
                # support points on the device from the first run's maps in HBM, Delaunay + planes on the
                # host, raster + mask on the device (== set_planar_prior_from_maps on the downloaded maps)
                with self._timed("planar_prior"):
                    e.set_params(p)
                    e.set_planar_prior_from_state(float(p["depth_min"]), float(p["depth_max"]))
                self._planar_parts(e)
            elif hasattr(e, "set_planar_prior_from_maps"):
                # support points + Delaunay + planes on the host, raster + mask on the device
                with self._timed("planar_prior"):
                    e.set_params(p)
                    e.set_planar_prior_from_maps(planes[..., 3], costs, float(p["depth_min"]), float(p["depth_max"]))
                self._planar_parts(e)
            else:
                with self._timed("planar_prior"):
                    prior, masks, _ = capi.planar_prior_host(c0, planes[..., 3], costs, float(p["depth_min"]),
                                                             float(p["depth_max"]))
                with self._timed("upload"):
                    e.set_params(p)
                    e.set_planar_prior(prior, masks)
            with self._timed("patchmatch"):
                e.run_patchmatch(run_seed + 1)
                planes, costs = e.download()
        with self._timed("store"):
            key = "depths_geom" if geom else "depths"
            self._save(key, ref, planes[..., 3], e if isinstance(e, capi.Context) else None)
            self.store.put("normals", ref, planes[..., :3])
            self.store.put("costs", ref, costs)
            self._last_planes[ref] = planes
            if self.reuse_planes and self.store.device is not None and isinstance(e, capi.Context):
                # the same planes and costs kept in HBM too: the next geom pass restarts from them device
                # to device (set_state_device) instead of uploading them from the host again
                e.export_state(*self._state_buffers(ref, costs.shape))
            elif ref in self._dev_state:
                # no HBM copy of these planes: an older one must not pass for them in _upload
                self._dev_state[ref][2] = None
            if self.out_folder:
                d = os.path.join(self.out_folder, "ACMMP", f"2333_{ref:08d}")
                os.makedirs(d, exist_ok=True)
                io.write_dmb(os.path.join(d, key + ".dmb"), planes[..., 3])
                io.write_dmb(os.path.join(d, "normals.dmb"), planes[..., :3])
                io.write_dmb(os.path.join(d, "costs.dmb"), costs)
        return planes, costs

    def _planar_parts(self, e):
        """The planar_prior stage's split (support points / host triangles / device half), summed like it."""
        if not hasattr(e, "last_planar_timing"):
            return
        parts = e.last_planar_timing()
        with self._stage_lock:
            for k, ms in parts.items():
                key = "planar_prior." + k[:-3]
                self.stage_s[key] = self.stage_s.get(key, 0.0) + ms / 1e3

    @staticmethod
    def _state_planar(e):
        return isinstance(e, capi.Context) and hasattr(e, "set_planar_prior_from_state")

    def _state_buffers(self, ref, shape):
        """The HBM copy of view `ref`'s last planes and costs: one allocation per view, sized for its
        full-resolution image (every scale fits, so no free -- a device-wide synchronisation -- between
        scales)."""
        need = int(shape[0]) * int(shape[1])
        dev = self._dev_state.get(ref)
        if dev is None or dev[1].shape[0] < need:
            if dev is not None:
                for b in dev[:2]:
                    b.free()
            full = self.ds.images[ref].shape
            cap = max(need, int(full[0]) * int(full[1]))
            dev = [capi.DeviceBuffer(self.store.device, (cap * 4,)), capi.DeviceBuffer(self.store.device, (cap,)), None]
            self._dev_state[ref] = dev
        dev[2] = tuple(shape)
        return dev[0], dev[1]

    def _upload(self, e, p, images, cams, ids, ref, geom, hier, H, W):
        """InuputInitialization + the state reloads of ProcessProblem (ACMMP.cpp:567-679, 772-843)."""
        multi = bool(p["multi_geometry"])
        if geom:
            key = "depths_geom" if multi else "depths"
            e.set_params(p)
            self._upload_views(e, images, cams)
            if self.store.device is not None and hasattr(e, "upload_depths_device"):
                e.upload_depths_device([self.store.device_map(key, v) for v in ids])
            else:
                e.upload_depths([self.store.get(key, v) for v in ids])
            planes = self._last_planes.get(ref) if self.reuse_planes else None
            dev = self._dev_state.get(ref)
            if (planes is not None and planes.shape[:2] == (H, W) and dev is not None and dev[2] == (H, W)
                    and hasattr(e, "set_state_device")):
                e.set_state_device(dev[0], dev[1])
                return
            costs = self.store.get("costs", ref)
            if planes is None or planes.shape[:2] != (H, W):
                depth = self.store.get(key, ref)
                normals = self.store.get("normals", ref)
                planes = np.concatenate([normals, depth[..., None]], axis=-1)
            e.set_state(planes, costs)
        elif hier:
            depth = self.store.get("depths", ref)                    # JBU output, fine size
            normals = self.store.get("normals", ref)                 # previous scale
            costs = self.store.get("costs", ref)
            sh, sw = normals.shape[:2]
            if sw != W or sh != H:
                p["upsample"] = 1
                p["scaled_cols"] = np.float32(sw)
                p["scaled_rows"] = np.float32(sh)
                scaled = np.concatenate([normals, costs[..., None]], axis=-1)
            else:
                p["upsample"] = 0
                scaled = np.concatenate([normals, depth[..., None]], axis=-1)
            e.set_params(p)
            self._upload_views(e, images, cams)
            e.set_scaled_state(scaled)
            state = np.zeros((H, W, 4), np.float32)
            state[..., 3] = depth[:H, :W] if depth.shape == (H, W) else 0.0
            e.set_state(state, None)
        else:
            e.set_params(p)
            self._upload_views(e, images, cams)

    # -- RunFusionCuda (ACMMP.cu:1817-2105), after the last pass
    def run_fusion(self, fusion_factory=None, ply_path: str | None = None):
        """Fuse every view's final depth map on this rank's GPU (rank 0 when sharded: the other ranks
        broadcast their normals to it first; depths_geom were exchanged after the last pass).
        Returns the (n, 9) points and writes ACMMP/ACMM_model_cuda_5.ply when an output folder is set."""
        if self.world > 1:
            views = [p.ref_image_id for p in self.problems]
            owners = {self.problems[i].ref_image_id: self.owner(i) for i in range(len(self.problems))}
            for v in views:
                shape = (*self._pass_shape(v), 3)
                if owners[v] == self.rank and self.store.device is not None:
                    self.store.device_map("normals", v, shape).upload(self.store.get("normals", v))
                self.store.shapes[("normals", v)] = shape
            self.exchange.share("normals", views, owners, self.store)
            if self.rank != 0:
                return None
        cams, depths, normals, colours = fusion_inputs(self.ds, self.store, self.problems)
        make = fusion_factory or (lambda c: capi.Fusion(self.device, c))
        fu = make(cams)
        for k in range(len(cams)):
            fu.set_view(k, depths[k], normals[k], colours[k])
        index = {p.ref_image_id: k for k, p in enumerate(self.problems)}
        pts = []
        for k, p in enumerate(self.problems):
            srcs = [index.get(s, -1) for s in p.src_image_ids][:32]            # ACMMP.cu:2010-2023
            pts.append(fu.run(k, srcs))
        if hasattr(fu, "close"):
            fu.close()
        points = np.concatenate(pts, 0) if pts else np.zeros((0, 9), np.float32)
        path = ply_path or (os.path.join(self.out_folder, "ACMMP", "ACMM_model_cuda_5.ply") if self.out_folder else None)
        if path:
            os.makedirs(os.path.dirname(path), exist_ok=True)
            io.write_ply(path, points)
        self.fused = points
        return points

    # -- JointBilateralUpsampling (main.cpp:212-238) + RunJBU (ACMMP.cpp:1071-1122)
    def joint_bilateral_upsampling(self, idx, acmmp_size):
        ref = self.problems[idx].ref_image_id
        coarse = self.store.get("depths_geom", ref)
        img = self.ds.images[ref]
        rows, cols = img.shape
        new_rows, new_cols = round_dims(rows, cols, acmmp_size)
        scaled = resize_linear(img, new_cols, new_rows)
        imagescale = max(scaled.shape[0] // coarse.shape[0], scaled.shape[1] // coarse.shape[1])
        if imagescale == 1:                                          # ACMMP.cpp:1076-1079
            return None
        with self._timed("jbu"):
            out = self.engine.jbu(scaled, coarse, imagescale)
        self.store.put("depths", ref, out)
        if self.out_folder:
            d = os.path.join(self.out_folder, "ACMMP", f"2333_{ref:08d}")
            os.makedirs(d, exist_ok=True)
            io.write_dmb(os.path.join(d, "depths.dmb"), out)
        return out


def launcher_store():
    """The torchrun launcher's TCP key-value store (host bytes only).  Under torchrun the agent hosts
    it at MASTER_ADDR:MASTER_PORT (TORCHELASTIC_USE_AGENT_STORE); otherwise rank 0 hosts it there."""
    from torch.distributed import TCPStore
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    agent = os.environ.get("TORCHELASTIC_USE_AGENT_STORE", "").lower() == "true"
    return TCPStore(os.environ.get("MASTER_ADDR", "127.0.0.1"), int(os.environ["MASTER_PORT"]), world,
                    is_master=(rank == 0 and not agent), wait_for_workers=False)


def comm_from_env(device: int, tag: str = "acmmp"):
    """RCCL communicator of a torchrun-launched process: rank 0 makes the unique id and publishes it
    in the launcher's store; the data path is RCCL."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    store = launcher_store()
    key = f"{tag}_uid_{os.environ.get('TORCHELASTIC_RESTART_COUNT', '0')}"
    if rank == 0:
        store.set(key, capi.Comm.unique_id())
    uid = store.get(key)
    return capi.Comm(device, uid, world, rank)


def rcclexchange_from_env(device: int):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world == 1:
        return LocalExchange()
    return RcclExchange(comm_from_env(device), device)


def write_dense_folder(folder: str, ds: Dataset, pairs=None, quality: int = 95):
    """Synthetic dataset -> the reference's dense-folder layout (images/%08d.jpg, cams/%08d_cam.txt,
    pair.txt).  PINHOLE depth lines carry `dmin dmax N dmax`, so the reader quirk (ACMMP.cpp:205:
    second token -> depth_max) yields the intended range."""
    from PIL import Image
    os.makedirs(os.path.join(folder, "images"), exist_ok=True)
    os.makedirs(os.path.join(folder, "cams"), exist_ok=True)
    for i, img in ds.images.items():
        Image.fromarray(np.clip(np.round(img), 0, 255).astype(np.uint8), "L").save(
            os.path.join(folder, "images", f"{i:08d}.jpg"), quality=quality)
        cam = ds.cameras[i]
        interval = float(cam["depth_max"]) if int(cam["model"]) == types.PINHOLE else 0.0
        io.write_camera(os.path.join(folder, "cams", f"{i:08d}_cam.txt"), cam, depth_interval=interval)
    if pairs is None:
        pairs = [(p.ref_image_id, [(s, 1.0) for s in p.src_image_ids]) for p in ds.problems]
    io.write_pair_list(folder, pairs)


def main(argv=None):
    """`python -m acmmp.pipeline DENSE_FOLDER` -- the reference's `ACMMP dense_folder` (main.cpp:369-489):
    the multi-scale schedule, then RunFusionCuda into ACMMP/ACMM_model_cuda_5.ply.
    Under torchrun (WORLD_SIZE > 1) every rank drives GPU LOCAL_RANK, views are sharded and the
    depth maps are exchanged over RCCL between passes (snapshot order)."""
    import argparse
    import json
    import time
    ap = argparse.ArgumentParser()
    ap.add_argument("dense_folder")
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--order", choices=["reference", "snapshot"], default=None)
    ap.add_argument("--geom-iterations", type=int, default=2)
    ap.add_argument("--size-bound", type=int, default=1000, help="coarsest-scale bound (main.cpp:38)")
    ap.add_argument("--math", choices=["exact", "fast"], default=None,
                    help="engine arithmetic (default: exact, bit-identical to the oracle)")
    ap.add_argument("--no-dmb", action="store_true", help="keep results in memory only")
    ap.add_argument("--no-fusion", action="store_true", help="skip RunFusionCuda")
    a = ap.parse_args(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    device = int(os.environ.get("LOCAL_RANK", "0"))
    order = a.order or ("reference" if world == 1 else "snapshot")
    ds = load_dataset(a.dense_folder, with_colors=not a.no_fusion)
    exchange = rcclexchange_from_env(device)
    t0 = time.perf_counter()
    pipe = Pipeline(ds, exchange=exchange, device=device, seed=a.seed, order=order,
                    geom_iterations=a.geom_iterations, out_folder=None if a.no_dmb else a.dense_folder,
                    size_bound=a.size_bound,
                    log=lambda *m: print(*m, flush=True), math=a.math).run()
    n_points = None
    if not a.no_fusion:
        pts = pipe.run_fusion(ply_path=os.path.join(a.dense_folder, "ACMMP", "ACMM_model_cuda_5.ply"))
        n_points = None if pts is None else int(pts.shape[0])
    dt = time.perf_counter() - t0
    print(json.dumps({"rank": pipe.rank, "world": pipe.world, "views": len(pipe.my_problems()),
                      "passes": [p.name for p in pipe.passes], "fused_points": n_points,
                      "seconds": round(dt, 3)}), flush=True)
    exchange.close()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
