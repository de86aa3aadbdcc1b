"""ctypes binding of the C ABI in include/acmmp.h (libacmmp.so, built in-tree for gfx950).

This is the Python-side FFI a maintainer would add next to the reference;
tests and bench.py drive the engine only through it.  There is no fallback: if the HIP
library is missing or no GPU is visible, every call fails loudly.
"""
from __future__ import annotations

import ctypes as C
import mmap
import os
import threading
import weakref

import numpy as np

from .types import CAMERA_DTYPE, PARAMS_DTYPE

HERE = os.path.dirname(os.path.abspath(__file__))
# ACMMP_LIB selects another in-tree build of the same library (A/B experiments); default: the product build
LIB_PATH = os.environ.get("ACMMP_LIB") or os.path.join(HERE, "libacmmp.so")

class _HostPool:
    """Recycled page-aligned private mappings for large D2H destinations.  Fresh heap pages made the copy into
    them crawl (30 ms for a 800x600 view's planes + costs, 0.9 ms into a hugepage mapping,
    profiles/r05_d2h_probe.json), and a new mapping per download pays its page faults every time: a mapping
    comes back here when the last array (or view) on it is collected and the next download of that size
    reuses its resident pages.  At most `cap` bytes are kept idle (ACMMP_HOST_POOL_BYTES, default 1 GiB):
    beyond it the least recently returned mappings are dropped, so sizes a pipeline no longer requests (an
    earlier pyramid scale) do not stay held; release() drops them all."""

    def __init__(self, cap: int | None = None):
        if cap is None:
            cap = int(os.environ.get("ACMMP_HOST_POOL_BYTES", str(1 << 30)))
        self.cap, self.held = cap, 0
        self.free = {}                      # size -> [mapping]; insertion order of `order` = recency
        self.order = []                     # (size, mapping) in the order they came back, oldest first
        self.lock = threading.Lock()

    def take(self, n: int):
        with self.lock:
            lst = self.free.get(n)
            if lst:
                mm = lst.pop()
                self.order = [(k, m) for (k, m) in self.order if m is not mm]
                self.held -= n
                return mm
        mm = mmap.mmap(-1, n, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
        if hasattr(mmap, "MADV_HUGEPAGE"):
            mm.madvise(mmap.MADV_HUGEPAGE)
        return mm

    def give(self, mm, n: int):
        # (called while the array still holds its buffer export: a dropped mapping is unmapped when the last
        # reference goes, not closed here)
        if n > self.cap:
            return
        with self.lock:
            while self.held + n > self.cap and self.order:
                k, old = self.order.pop(0)              # least recently returned first
                self.free[k].remove(old)
                self.held -= k
            self.free.setdefault(n, []).append(mm)
            self.order.append((n, mm))
            self.held += n

    def release(self):
        """Drop every idle mapping (e.g. when a pipeline evicts a pyramid scale)."""
        with self.lock:
            self.free, self.order, self.held = {}, [], 0


_POOL = _HostPool()


def host_empty(shape, dtype=np.float32) -> np.ndarray:
    """An uninitialised host array for a D2H copy: arrays of 4 MiB and up live on a 2 MiB aligned private
    mapping advised MADV_HUGEPAGE from _HostPool (see there); smaller ones are plain np.empty."""
    dt = np.dtype(dtype)
    count = int(np.prod(shape))
    n = count * dt.itemsize
    if n < (4 << 20):
        return np.empty(shape, dt)
    size = (n + (2 << 20) - 1) // (2 << 20) * (2 << 20) + (2 << 20)     # whole 2 MiB pages + alignment slack
    mm = _POOL.take(size)
    base = np.frombuffer(mm, np.uint8)
    off = (-base.ctypes.data) % (2 << 20)
    del base
    flat = np.frombuffer(mm, dt, count, off)       # the base every view of the result keeps alive
    weakref.finalize(flat, _POOL.give, mm, size)
    return flat.reshape(shape)


STATUS = {0: "ok", 1: "invalid argument", 2: "HIP runtime error", 3: "out of device memory",
          4: "call order violated", 5: "unsupported configuration", 6: "no HIP device"}

# Every symbol include/acmmp.h declares (checked against the header by tests/test_capi_exports.py).
EXPORTS = [
    "acmmp_abi_version", "acmmp_device_count", "acmmp_create", "acmmp_destroy", "acmmp_status_str", "acmmp_last_error",
    "acmmp_set_params", "acmmp_upload_views", "acmmp_upload_depths", "acmmp_set_state",
    "acmmp_set_scaled_state", "acmmp_set_planar_prior", "acmmp_run_patchmatch", "acmmp_run_patchmatch_ex",
    "acmmp_download", "acmmp_download_aux", "acmmp_device_outputs", "acmmp_synchronize", "acmmp_last_timing",
    "acmmp_last_kernel_timing", "acmmp_last_work", "acmmp_last_planar_timing", "acmmp_texel_bytes", "acmmp_set_math", "acmmp_get_math", "acmmp_jbu",
    "acmmp_debug_ncc", "acmmp_debug_geom", "acmmp_debug_ncc_nb", "acmmp_debug_ncc_ref",
    "acmmp_support_points", "acmmp_delaunay", "acmmp_prior_plane_params", "acmmp_depth_from_plane_param",
    "acmmp_planar_prior_host", "acmmp_set_planar_prior_from_maps", "acmmp_set_planar_prior_from_state",
    "acmmp_download_planar_prior",
    "acmmp_upload_depths_device", "acmmp_upload_views_device", "acmmp_export_depth", "acmmp_export_state", "acmmp_set_state_device", "acmmp_device_alloc", "acmmp_device_free", "acmmp_memcpy",
    "acmmp_comm_unique_id", "acmmp_comm_create", "acmmp_comm_destroy", "acmmp_comm_broadcast", "acmmp_comm_after",
    "acmmp_comm_allreduce_max", "acmmp_comm_band_exchange", "acmmp_run_patchmatch_band",
    "acmmp_band_begin", "acmmp_band_sweep", "acmmp_band_sweeps_left", "acmmp_band_halo_ranges",
    "acmmp_band_copy_rows", "acmmp_band_get_rows", "acmmp_band_set_rows", "acmmp_band_end",
    "acmmp_fusion_create", "acmmp_fusion_set_view", "acmmp_fusion_run", "acmmp_fusion_last_error",
    "acmmp_fusion_destroy", "acmmp_image_cache_create", "acmmp_image_cache_destroy", "acmmp_image_cache_stats",
    "acmmp_upload_views_keyed", "acmmp_device_checksum", "acmmp_device_identity", "acmmp_clock_probe",
]


class AcmmpError(RuntimeError):
    pass


_lib = None


def load_library(path: str = LIB_PATH):
    """Load libacmmp.so (no GPU needed to load it)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise AcmmpError(f"{path} is missing: build it with `python acmmp-spherical_amd/build.py` "
                         "(there is no CPU fallback)")
    L = C.CDLL(path)
    vp, i32, u64 = C.c_void_p, C.c_int, C.c_uint64
    L.acmmp_abi_version.restype = i32
    L.acmmp_device_count.restype = i32
    L.acmmp_create.argtypes = [i32, C.POINTER(vp)]
    L.acmmp_destroy.argtypes = [vp]
    L.acmmp_destroy.restype = None
    L.acmmp_status_str.argtypes = [i32]
    L.acmmp_status_str.restype = C.c_char_p
    L.acmmp_last_error.argtypes = [vp]
    L.acmmp_last_error.restype = C.c_char_p
    L.acmmp_set_params.argtypes = [vp, vp]
    L.acmmp_upload_views.argtypes = [vp, i32, vp, vp, vp]
    L.acmmp_upload_depths.argtypes = [vp, i32, vp, vp, vp]
    L.acmmp_set_state.argtypes = [vp, vp, vp]
    L.acmmp_set_scaled_state.argtypes = [vp, vp, i32, i32]
    L.acmmp_set_planar_prior.argtypes = [vp, vp, vp]
    L.acmmp_run_patchmatch.argtypes = [vp, u64]
    L.acmmp_run_patchmatch_ex.argtypes = [vp, u64, i32, i32]
    L.acmmp_download.argtypes = [vp, vp, vp]
    L.acmmp_download_aux.argtypes = [vp, vp, vp]
    L.acmmp_device_outputs.argtypes = [vp, C.POINTER(vp), C.POINTER(vp)]
    L.acmmp_last_timing.argtypes = [vp, vp]
    L.acmmp_last_kernel_timing.argtypes = [vp, vp, vp]
    L.acmmp_last_work.argtypes = [vp, vp, vp]
    L.acmmp_last_planar_timing.argtypes = [vp, vp]
    L.acmmp_texel_bytes.argtypes = [vp]
    L.acmmp_set_math.argtypes = [vp, i32]
    L.acmmp_get_math.argtypes = [vp]
    L.acmmp_synchronize.argtypes = [vp]
    L.acmmp_jbu.argtypes = [vp, vp, i32, i32, vp, i32, i32, i32, vp]
    L.acmmp_debug_ncc.argtypes = [vp, i32, vp, vp, vp, vp]
    L.acmmp_debug_geom.argtypes = [vp, i32, vp, vp, vp, vp]
    L.acmmp_debug_ncc_nb.argtypes = [vp, i32, vp, vp, vp, vp]
    L.acmmp_debug_ncc_ref.argtypes = [vp, i32, vp, vp, vp, vp]
    L.acmmp_support_points.argtypes = [vp, i32, i32, vp, i32, vp]
    L.acmmp_delaunay.argtypes = [vp, i32, i32, i32, vp, i32, vp]
    L.acmmp_prior_plane_params.argtypes = [vp, vp, i32, i32, vp, vp]
    L.acmmp_depth_from_plane_param.argtypes = [vp, vp, i32, i32]
    L.acmmp_upload_depths_device.argtypes = [vp, i32, vp, vp, vp]
    L.acmmp_upload_views_device.argtypes = [vp, i32, vp, vp, vp]
    L.acmmp_export_depth.argtypes = [vp, vp]
    L.acmmp_export_state.argtypes = [vp, vp, vp]
    L.acmmp_set_state_device.argtypes = [vp, vp, vp]
    L.acmmp_device_alloc.argtypes = [i32, C.c_size_t, C.POINTER(vp)]
    L.acmmp_device_free.argtypes = [i32, vp]
    L.acmmp_memcpy.argtypes = [i32, vp, vp, C.c_size_t, i32]
    L.acmmp_comm_unique_id.argtypes = [vp]
    L.acmmp_comm_create.argtypes = [i32, vp, i32, i32, C.POINTER(vp)]
    L.acmmp_comm_destroy.argtypes = [vp]
    L.acmmp_comm_broadcast.argtypes = [vp, i32, vp, vp, vp]
    L.acmmp_comm_after.argtypes = [vp, vp]
    L.acmmp_comm_allreduce_max.argtypes = [vp, vp, i32]
    L.acmmp_comm_band_exchange.argtypes = [vp, vp, i32, i32, i32]
    L.acmmp_run_patchmatch_band.argtypes = [vp, vp, u64, i32, i32, i32, i32]
    L.acmmp_band_begin.argtypes = [vp, u64, i32, i32]
    L.acmmp_band_sweep.argtypes = [vp, C.POINTER(i32)]
    L.acmmp_band_sweeps_left.argtypes = [vp]
    L.acmmp_band_halo_ranges.argtypes = [vp, vp]
    L.acmmp_band_copy_rows.argtypes = [vp, vp, i32, i32, i32]
    L.acmmp_band_get_rows.argtypes = [vp, i32, i32, i32, vp, vp, vp]
    L.acmmp_band_set_rows.argtypes = [vp, i32, i32, i32, vp, vp, vp]
    L.acmmp_band_end.argtypes = [vp, i32]
    L.acmmp_fusion_create.argtypes = [i32, i32, vp, C.POINTER(vp)]
    L.acmmp_fusion_set_view.argtypes = [vp, i32, vp, vp, vp]
    L.acmmp_fusion_run.argtypes = [vp, i32, i32, vp, vp, i32, vp]
    L.acmmp_fusion_last_error.argtypes = [vp]
    L.acmmp_fusion_destroy.argtypes = [vp]
    L.acmmp_planar_prior_host.argtypes = [vp, vp, vp, i32, i32, C.c_float, C.c_float, vp, vp, vp]
    L.acmmp_set_planar_prior_from_maps.argtypes = [vp, vp, vp, C.c_float, C.c_float, vp]
    L.acmmp_set_planar_prior_from_state.argtypes = [vp, C.c_float, C.c_float, vp]
    L.acmmp_download_planar_prior.argtypes = [vp, vp, vp]
    L.acmmp_image_cache_create.argtypes = [i32, C.c_size_t, C.POINTER(vp)]
    L.acmmp_image_cache_destroy.argtypes = [vp]
    L.acmmp_image_cache_stats.argtypes = [vp, vp]
    L.acmmp_upload_views_keyed.argtypes = [vp, vp, i32, vp, vp, vp, vp, i32]
    L.acmmp_device_checksum.argtypes = [i32, vp, C.c_size_t, vp]
    L.acmmp_device_identity.argtypes = [i32, vp, i32, vp]
    L.acmmp_clock_probe.argtypes = [i32, C.c_float, vp]
    for name in EXPORTS:
        fn = getattr(L, name)
        if name not in ("acmmp_destroy", "acmmp_status_str", "acmmp_last_error", "acmmp_abi_version", "acmmp_device_count",
                        "acmmp_depth_from_plane_param", "acmmp_comm_destroy", "acmmp_fusion_last_error",
                        "acmmp_fusion_destroy", "acmmp_image_cache_destroy"):
            fn.restype = i32
    L.acmmp_depth_from_plane_param.restype = C.c_float
    L.acmmp_fusion_last_error.restype = C.c_char_p
    L.acmmp_image_cache_destroy.restype = None
    _lib = L
    return L


def device_count() -> int:
    """Visible HIP devices (the engine's runtime; 0 without a GPU)."""
    return int(load_library().acmmp_device_count())


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def checksum_host(arr) -> int:
    """acmmp_device_checksum on a host array (its bytes as little-endian 32-bit words): the sum mod 2^64 of
    splitmix64's finaliser of (i << 32) | w_i.  The CPU side of the exchange check and its tests."""
    w = np.frombuffer(np.ascontiguousarray(arr).tobytes(), np.uint32).astype(np.uint64)
    z = (np.arange(w.size, dtype=np.uint64) << np.uint64(32)) | w
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xbf58476d1ce4e5b9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94d049bb133111eb)
        z = z ^ (z >> np.uint64(31))
        return int(np.sum(z, dtype=np.uint64))


def device_identity(device: int) -> dict:
    """PCI bus id, UUID and (where the KFD topology lists the device) its KFD unique_id: which physical GPU a
    measurement ran on (bench.py `device`)."""
    L = load_library()
    bus = C.create_string_buffer(64)
    uuid = np.zeros(16, np.uint8)
    _host_check(L.acmmp_device_identity(device, C.cast(bus, C.c_void_p), 64, _p(uuid)), "device_identity")
    pci = bus.value.decode()
    out = {"pci_bus_id": pci, "uuid": uuid.tobytes().hex(), "kfd_unique_id": None}
    try:                                        # KFD node whose location_id is this bus:device.function
        dom, bus_, devfn = pci.split(":")
        dev_, fn = devfn.split(".")
        loc = (int(bus_, 16) << 8) | (int(dev_, 16) << 3) | int(fn, 16)
        root = "/sys/class/kfd/kfd/topology/nodes"
        for node in sorted(os.listdir(root)):
            with open(os.path.join(root, node, "properties")) as fh:
                props = dict(ln.split(None, 1) for ln in fh if len(ln.split(None, 1)) == 2)
            if (int(props.get("location_id", "-1")) == loc and
                    int(props.get("domain", "0")) == int(dom, 16)):
                out["kfd_unique_id"] = props.get("unique_id", "").strip() or None
                out["kfd_node"] = int(node)
                break
    except (OSError, ValueError):
        pass
    return out


def clock_probe(device: int, warm_ms: float = 1500.0) -> dict:
    """acmmp_clock_probe: the shader clock held under a VALU-dense load (median / min / max GHz over
    workgroups) after warm_ms of back-to-back launches."""
    out = np.zeros(4, np.float64)
    _host_check(load_library().acmmp_clock_probe(device, float(warm_ms), _p(out)), "clock_probe")
    return {"ghz": round(float(out[0]), 4), "ghz_min": round(float(out[1]), 4), "ghz_max": round(float(out[2]), 4),
            "probe_launch_ms": round(float(out[3]), 3), "warm_ms": warm_ms}


class ImageCache:
    """Prepared source images (padded fp32 + binary16) shared by the contexts of one GPU, keyed by the
    caller (acmmp_image_cache_*).  Safe to close before the contexts that used it."""

    def __init__(self, device: int = 0, budget_bytes: int = 0):
        self.L = load_library()
        h = C.c_void_p()
        rc = self.L.acmmp_image_cache_create(device, C.c_size_t(budget_bytes), C.byref(h))
        if rc != 0:
            raise AcmmpError(f"acmmp_image_cache_create: {self.L.acmmp_status_str(rc).decode()}")
        self.h, self.device = h, device

    def stats(self) -> dict:
        out = np.zeros(5, np.uint64)
        _host_check(self.L.acmmp_image_cache_stats(self.h, _p(out)), "image_cache_stats")
        return dict(zip(("hits", "misses", "bytes", "entries", "evictions"), (int(x) for x in out)))

    def close(self):
        if self.h:
            self.L.acmmp_image_cache_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:                                            # noqa: BLE001
            pass


class Context:
    """One reference-view problem on one GPU -- the device side of the reference's ACMMP object."""

    def __init__(self, device: int = 0):
        self.L = load_library()
        h = C.c_void_p()
        rc = self.L.acmmp_create(device, C.byref(h))
        if rc != 0:
            raise AcmmpError(f"acmmp_create({device}) failed: {STATUS.get(rc, rc)}")
        self.h = h
        self.device = device
        self.W = self.H = self.N = 0
        self._params = None

    def _check(self, rc, what):
        if rc != 0:
            msg = self.L.acmmp_last_error(self.h).decode()
            raise AcmmpError(f"{what}: {STATUS.get(rc, rc)}: {msg}")

    def close(self):
        if getattr(self, "h", None):
            self.L.acmmp_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # -- setup
    MATH = {"exact": 0, "fast": 1}

    def set_math(self, mode: str):
        """'exact' (bit-identical to the oracle, the default) or 'fast' (DESIGN.md §2.4)."""
        self._check(self.L.acmmp_set_math(self.h, self.MATH[mode]), "set_math")

    def math(self) -> str:
        return {0: "exact", 1: "fast"}[int(self.L.acmmp_get_math(self.h))]

    def set_params(self, params):
        p = np.frombuffer(np.asarray(params, dtype=PARAMS_DTYPE).tobytes(), np.uint8).copy()
        self._params = p
        self._check(self.L.acmmp_set_params(self.h, _p(p)), "set_params")

    @staticmethod
    def _check_view_shapes(shapes, cams):
        """The C side sizes every copy from the cameras: a mismatched array would be read past its end."""
        if len(shapes) != len(cams):
            raise ValueError(f"{len(shapes)} images for {len(cams)} cameras")
        for i, (shp, cam) in enumerate(zip(shapes, cams)):
            if tuple(shp) != (int(cam["height"]), int(cam["width"])):
                raise ValueError(f"image {i} has shape {tuple(shp)}, camera says {int(cam['height'])}x{int(cam['width'])}")

    def _check_hw(self, arr, tail, what):
        """Row-major (H, W)+tail maps, or the same elements flat: any other shape (a transposed
        (W, H) map with the right element count included) is refused, not read in the wrong layout."""
        want = (self.H, self.W) + tail
        if arr.shape != want and arr.shape != (int(np.prod(want)),):
            raise ValueError(f"{what}: shape {arr.shape}, expected {want} (or flat {int(np.prod(want))})")

    def upload_views(self, images, cameras):
        imgs = [np.ascontiguousarray(im, np.float32) for im in images]
        cams = np.frombuffer(np.ascontiguousarray(cameras, dtype=CAMERA_DTYPE).tobytes(), CAMERA_DTYPE).copy()
        self._check_view_shapes([im.shape for im in imgs], cams)
        n = len(imgs)
        ptrs = (C.c_void_p * n)(*[im.ctypes.data for im in imgs])
        self._check(self.L.acmmp_upload_views(self.h, n, C.cast(ptrs, C.c_void_p), None, _p(cams)), "upload_views")
        self.N, self.H, self.W = n, imgs[0].shape[0], imgs[0].shape[1]

    def upload_views_device(self, bufs, cameras, cache: "ImageCache | None" = None, keys=None):
        """bufs: DeviceBuffer images (index 0 = reference) on this context's GPU.  With an ImageCache and
        one nonzero content key per view (the caller's promise that equal keys mean equal pixels), views
        the cache already holds are neither copied nor converted again (acmmp_upload_views_keyed)."""
        cams = np.frombuffer(np.ascontiguousarray(cameras, dtype=CAMERA_DTYPE).tobytes(), CAMERA_DTYPE).copy()
        self._check_view_shapes([tuple(b.shape[:2]) for b in bufs], cams)
        n = len(bufs)
        ptrs = (C.c_void_p * n)(*[b.ptr for b in bufs])
        if cache is not None:
            k = np.ascontiguousarray(keys, np.uint64)
            if k.shape != (n,):
                raise ValueError(f"upload_views_device: {n} views but keys of shape {k.shape}")
            self._check(self.L.acmmp_upload_views_keyed(self.h, cache.h, n, _p(k), C.cast(ptrs, C.c_void_p), None,
                                                        _p(cams), 1), "upload_views_keyed")
        else:
            self._check(self.L.acmmp_upload_views_device(self.h, n, C.cast(ptrs, C.c_void_p), None, _p(cams)),
                        "upload_views_device")
        self.N, self.H, self.W = n, bufs[0].shape[0], bufs[0].shape[1]

    def upload_depths(self, depths):
        ds = [np.ascontiguousarray(d, np.float32) for d in depths]
        n = len(ds)
        ptrs = (C.c_void_p * n)(*[d.ctypes.data for d in ds])
        w = np.array([d.shape[1] for d in ds], np.int32)
        h = np.array([d.shape[0] for d in ds], np.int32)
        self._check(self.L.acmmp_upload_depths(self.h, n, C.cast(ptrs, C.c_void_p), _p(w), _p(h)), "upload_depths")

    def upload_depths_device(self, bufs):
        """bufs: DeviceBuffer depth maps (index 0 = reference) on this context's GPU."""
        n = len(bufs)
        ptrs = (C.c_void_p * n)(*[b.ptr for b in bufs])
        w = np.array([b.shape[1] for b in bufs], np.int32)
        h = np.array([b.shape[0] for b in bufs], np.int32)
        self._check(self.L.acmmp_upload_depths_device(self.h, n, C.cast(ptrs, C.c_void_p), _p(w), _p(h)),
                    "upload_depths_device")

    def export_depth(self, buf):
        """Copy the last run's depth map into DeviceBuffer `buf` (H x W floats)."""
        self._check(self.L.acmmp_export_depth(self.h, C.c_void_p(buf.ptr)), "export_depth")

    def set_state(self, planes=None, costs=None):
        pl = None if planes is None else np.ascontiguousarray(planes, np.float32)
        co = None if costs is None else np.ascontiguousarray(costs, np.float32)
        if pl is not None:
            self._check_hw(pl, (4,), "set_state planes")
        if co is not None:
            self._check_hw(co, (), "set_state costs")
        self._check(self.L.acmmp_set_state(self.h, _p(pl), _p(co)), "set_state")

    def _check_state_bufs(self, planes_buf, costs_buf, what):
        # (H, W, 4) / (H, W) buffers, or larger flat ones (a view's buffers sized for its finest scale)
        for b, k, name in ((planes_buf, 4, "planes"), (costs_buf, 1, "costs")):
            if b is None:
                continue
            need = 4 * k * self.H * self.W
            if b.shape != ((self.H, self.W, 4) if k == 4 else (self.H, self.W)) and (len(b.shape) != 1 or b.nbytes < need):
                raise ValueError(f"{what} {name}: buffer shape {b.shape}, expected {(self.H, self.W)}"
                                 f"{' + (4,)' if k == 4 else ''} or a flat buffer of at least {need} bytes")

    def export_state(self, planes_buf=None, costs_buf=None):
        """Copy the last run's planes into DeviceBuffer `planes_buf` (H x W x 4) and its costs into
        `costs_buf` (H x W), HBM to HBM."""
        self._check_state_bufs(planes_buf, costs_buf, "export_state")
        self._check(self.L.acmmp_export_state(self.h, C.c_void_p(planes_buf.ptr if planes_buf else None),
                                              C.c_void_p(costs_buf.ptr if costs_buf else None)), "export_state")

    def set_state_device(self, planes_buf=None, costs_buf=None):
        """set_state from DeviceBuffers of this context's GPU (shapes as export_state)."""
        self._check_state_bufs(planes_buf, costs_buf, "set_state_device")
        self._check(self.L.acmmp_set_state_device(self.h, C.c_void_p(planes_buf.ptr if planes_buf else None),
                                                  C.c_void_p(costs_buf.ptr if costs_buf else None)), "set_state_device")

    def set_scaled_state(self, planes):
        pl = np.ascontiguousarray(planes, np.float32)
        self._check(self.L.acmmp_set_scaled_state(self.h, _p(pl), pl.shape[1], pl.shape[0]), "set_scaled_state")

    def set_planar_prior(self, prior_planes, masks):
        pr = np.ascontiguousarray(prior_planes, np.float32)
        mk = np.ascontiguousarray(masks, np.uint32)
        self._check_hw(pr, (4,), "set_planar_prior planes")
        self._check_hw(mk, (), "set_planar_prior masks")
        self._check(self.L.acmmp_set_planar_prior(self.h, _p(pr), _p(mk)), "set_planar_prior")

    def set_planar_prior_from_maps(self, depths, costs, depth_min: float, depth_max: float) -> int:
        """The planar block of ProcessProblem with its per-pixel work on the device (main.cpp:113-181):
        the same prior as planar_prior_host + set_planar_prior.  Returns the triangle count."""
        d = np.ascontiguousarray(depths, np.float32)
        c = np.ascontiguousarray(costs, np.float32)
        self._check_hw(d, (), "set_planar_prior_from_maps depths")
        self._check_hw(c, (), "set_planar_prior_from_maps costs")
        n = C.c_int(0)
        self._check(self.L.acmmp_set_planar_prior_from_maps(self.h, _p(d), _p(c), float(depth_min), float(depth_max),
                                                            C.byref(n)), "set_planar_prior_from_maps")
        return n.value

    def set_planar_prior_from_state(self, depth_min: float, depth_max: float) -> int:
        """The planar block from this context's last RunPatchMatch output in HBM (support points on the
        device, Delaunay and the planes on the host, raster + mask on the device): equal to
        set_planar_prior_from_maps on the downloaded maps, without downloading them.  Returns the
        triangle count."""
        n = C.c_int(0)
        self._check(self.L.acmmp_set_planar_prior_from_state(self.h, float(depth_min), float(depth_max), C.byref(n)),
                    "set_planar_prior_from_state")
        return n.value

    def download_planar_prior(self):
        prior = host_empty((self.H, self.W, 4), np.float32)
        masks = host_empty((self.H, self.W), np.uint32)
        self._check(self.L.acmmp_download_planar_prior(self.h, _p(prior), _p(masks)), "download_planar_prior")
        return prior, masks

    # -- run
    def run_patchmatch(self, seed: int, n_half_sweeps: int = -1, do_post: bool = True):
        self._check(self.L.acmmp_run_patchmatch_ex(self.h, C.c_uint64(seed), n_half_sweeps, int(do_post)),
                    "run_patchmatch")

    def download(self):
        planes = host_empty((self.H, self.W, 4), np.float32)
        costs = host_empty((self.H, self.W), np.float32)
        self._check(self.L.acmmp_download(self.h, _p(planes), _p(costs)), "download")
        return planes, costs

    def download_into(self, planes, costs):
        """D2H into caller-owned C-contiguous float32 arrays (H, W, 4) and (H, W)."""
        for a, tail in ((planes, (4,)), (costs, ())):
            if a.dtype != np.float32 or not a.flags.c_contiguous or a.shape != (self.H, self.W) + tail:
                raise ValueError("download_into: need C-contiguous float32 (H, W, 4) planes and (H, W) costs")
        self._check(self.L.acmmp_download(self.h, _p(planes), _p(costs)), "download")

    def download_rows_into(self, planes, costs, row0: int, row1: int):
        """D2H of rows [row0, row1) of the row-major outputs into caller-owned C-contiguous float32 arrays
        (row1 - row0, W, 4) and (row1 - row0, W) -- a band's share of a split run (acmmp_band_*)."""
        n = row1 - row0
        for a, tail in ((planes, (4,)), (costs, ())):
            if a.dtype != np.float32 or not a.flags.c_contiguous or a.shape != (n, self.W) + tail:
                raise ValueError("download_rows_into: need C-contiguous float32 (rows, W, 4) and (rows, W)")
        if not (0 <= row0 < row1 <= self.H):
            raise ValueError("download_rows_into: rows outside the view")
        pp, cp = self.device_outputs()
        dev = self.device
        _host_check(self.L.acmmp_memcpy(dev, _p(planes), C.c_void_p(pp + 16 * row0 * self.W), 16 * n * self.W, 1),
                    "memcpy D2H")
        _host_check(self.L.acmmp_memcpy(dev, _p(costs), C.c_void_p(cp + 4 * row0 * self.W), 4 * n * self.W, 1),
                    "memcpy D2H")

    def download_aux(self):
        sel = host_empty((self.H, self.W), np.uint32)
        pre = host_empty((self.H, self.W), np.float32)
        self._check(self.L.acmmp_download_aux(self.h, _p(sel), _p(pre)), "download_aux")
        return sel, pre

    def device_outputs(self):
        a, b = C.c_void_p(), C.c_void_p()
        self._check(self.L.acmmp_device_outputs(self.h, C.byref(a), C.byref(b)), "device_outputs")
        return a.value, b.value

    # ---- row-band split of one view (acmmp_band_*, SURVEY.md §8e latency mode) ----
    BAND_HALO = 23

    def band_begin(self, seed: int, row0: int, row1: int):
        self._check(self.L.acmmp_band_begin(self.h, seed, row0, row1), "band_begin")

    def band_sweep(self) -> int:
        colour = C.c_int32(0)
        self._check(self.L.acmmp_band_sweep(self.h, C.byref(colour)), "band_sweep")
        return colour.value

    def band_sweeps_left(self) -> int:
        return int(self.L.acmmp_band_sweeps_left(self.h))

    def band_halo_ranges(self):
        """((send_up), (recv_up), (send_down), (recv_down)) row ranges [a, b) after a half-sweep."""
        r = np.zeros(8, np.int32)
        self._check(self.L.acmmp_band_halo_ranges(self.h, _p(r)), "band_halo_ranges")
        return tuple((int(r[2 * k]), int(r[2 * k + 1])) for k in range(4))

    def band_copy_rows_from(self, src: "Context", colour: int, row_a: int, row_b: int):
        self._check(self.L.acmmp_band_copy_rows(self.h, src.h, colour, row_a, row_b), "band_copy_rows")

    def band_get_rows(self, colour: int, row_a: int, row_b: int) -> np.ndarray:
        """Rows [row_a, row_b) of `colour`'s current band state as one host array of 6 words per colour-grid pixel
        (plane x, y, z, w, cost as float32 bits, selected-view mask) -- the host transport of the halo."""
        n = (row_b - row_a) * ((self.W + 1) // 2)
        pl = np.empty((n, 4), np.float32)
        co = np.empty(n, np.float32)
        sel = np.empty(n, np.uint32)
        self._check(self.L.acmmp_band_get_rows(self.h, colour, row_a, row_b, _p(pl), _p(co), _p(sel)), "band_get_rows")
        return np.concatenate([pl.view(np.uint32), co.view(np.uint32)[:, None], sel[:, None]], axis=1)

    def band_set_rows(self, colour: int, row_a: int, row_b: int, rows: np.ndarray):
        """Inverse of band_get_rows: write the (n, 6) words into `colour`'s current band state."""
        rows = np.asarray(rows, np.uint32).reshape(-1, 6)
        pl = np.ascontiguousarray(rows[:, :4]).view(np.float32)
        co = np.ascontiguousarray(rows[:, 4]).view(np.float32)
        sel = np.ascontiguousarray(rows[:, 5])
        self._check(self.L.acmmp_band_set_rows(self.h, colour, row_a, row_b, _p(pl), _p(co), _p(sel)), "band_set_rows")

    def band_end(self, do_post: bool = True):
        self._check(self.L.acmmp_band_end(self.h, int(do_post)), "band_end")

    def run_patchmatch_band(self, seed: int, row0: int, row1: int, comm=None, rank_up: int = -1,
                            rank_down: int = -1):
        """One band of a view split over ranks, halo exchange over RCCL (comm: a Comm, or None for a
        band covering the whole view)."""
        self._check(self.L.acmmp_run_patchmatch_band(self.h, comm.h if comm is not None else None, seed, row0, row1,
                                                     rank_up, rank_down), "run_patchmatch_band")

    def synchronize(self):
        self._check(self.L.acmmp_synchronize(self.h), "synchronize")

    def last_timing(self):
        ms = np.zeros(3, np.float32)
        self._check(self.L.acmmp_last_timing(self.h, _p(ms)), "last_timing")
        return {"init_ms": float(ms[0]), "prop_ms": float(ms[1]), "post_ms": float(ms[2])}

    KERNELS = ("k_eval_nb", "k_select", "k_eval_ref", "k_finish")

    def last_kernel_timing(self):
        """{kernel: (summed ms, launches)} for the half-sweep kernels of the last run."""
        ms = np.zeros(4, np.float32)
        n = np.zeros(4, np.int32)
        self._check(self.L.acmmp_last_kernel_timing(self.h, _p(ms), _p(n)), "last_kernel_timing")
        return {k: (float(ms[i]), int(n[i])) for i, k in enumerate(self.KERNELS)}

    def last_work(self):
        """(pixels of the last run's k_eval_nb launches whose NCCs were evaluated, all pixels)."""
        e, t = C.c_ulonglong(0), C.c_ulonglong(0)
        self._check(self.L.acmmp_last_work(self.h, C.byref(e), C.byref(t)), "last_work")
        return e.value, t.value

    def last_planar_timing(self):
        """Host wall ms of the last set_planar_prior_from_state / _from_maps: support points, Delaunay, the rest of
        the host half (triangles, plane fits, tables), device half (staging + enqueueing upload, raster, mask)."""
        ms = np.zeros(4, np.float32)
        self._check(self.L.acmmp_last_planar_timing(self.h, _p(ms)), "last_planar_timing")
        return {"support_ms": float(ms[0]), "delaunay_ms": float(ms[1]), "planes_ms": float(ms[2]),
                "device_ms": float(ms[3])}

    def texel_bytes(self) -> int:
        """Bytes per source texel the NCC fetches read (2: binary16 copy, 4: fp32, 0: no views)."""
        return int(self.L.acmmp_texel_bytes(self.h))

    def jbu(self, ref, coarse, imagescale: int):
        ref = np.ascontiguousarray(ref, np.float32)
        coarse = np.ascontiguousarray(coarse, np.float32)
        out = np.empty_like(ref)
        self._check(self.L.acmmp_jbu(self.h, _p(ref), ref.shape[1], ref.shape[0], _p(coarse), coarse.shape[1],
                                     coarse.shape[0], imagescale, _p(out)), "jbu")
        return out

    def _debug(self, fn, px, py, planes):
        px = np.ascontiguousarray(px, np.int32)
        py = np.ascontiguousarray(py, np.int32)
        pl = np.ascontiguousarray(planes, np.float32).reshape(-1, 4)
        out = np.empty((len(px), self.N - 1), np.float32)
        self._check(fn(self.h, len(px), _p(px), _p(py), _p(pl), _p(out)), "debug")
        return out

    def debug_ncc(self, px, py, planes):
        return self._debug(self.L.acmmp_debug_ncc, px, py, planes)

    def debug_geom(self, px, py, planes):
        return self._debug(self.L.acmmp_debug_geom, px, py, planes)

    def _debug_k(self, fn, k, px, py, planes, what):
        px = np.ascontiguousarray(px, np.int32)
        py = np.ascontiguousarray(py, np.int32)
        pl = np.ascontiguousarray(planes, np.float32).reshape(len(px), k, 4)
        out = np.empty((len(px), k, self.N - 1), np.float32)
        self._check(fn(self.h, len(px), _p(px), _p(py), _p(pl), _p(out)), what)
        return out

    def debug_ncc_nb(self, px, py, planes):
        """k_eval_nb's own NCC (fast SPHERE from 2000x1000 up with patch_size 11: interpolated coordinates with
        their deferred per-sample fallbacks) of planes (n, 8, 4) at pixels (px, py) -> costs (n, 8, V)."""
        return self._debug_k(self.L.acmmp_debug_ncc_nb, 8, px, py, planes, "debug_ncc_nb")

    def debug_ncc_ref(self, px, py, planes):
        """The refinement's NCC (k_eval_ref's instance; fast SPHERE with V > 4 at the interpolation's sizes:
        interpolated coordinates; where they fall back, the per-sample costs of k_nb_fix<1, true>'s entry code,
        the production fallback path) of planes (n, 5, 4) at pixels (px, py) -> costs (n, 5, V)."""
        return self._debug_k(self.L.acmmp_debug_ncc_ref, 5, px, py, planes, "debug_ncc_ref")


# ---- planar-prior host side (no GPU): ACMMP.cpp:904-1011, main.cpp:113-181 ------------------

def _host_check(rc, what):
    if rc != 0:
        raise AcmmpError(f"{what}: {load_library().acmmp_status_str(rc).decode()}")


def _cam_ptr(cam):
    cam = np.frombuffer(np.asarray(cam).tobytes(), dtype=CAMERA_DTYPE).copy()
    return cam, cam.ctypes.data


def support_points(costs) -> np.ndarray:
    """GetSupportPoints (ACMMP.cpp:904-930) -> (n, 2) int32 (x, y) in the reference's order."""
    L = load_library()
    costs = np.ascontiguousarray(costs, np.float32)
    H, W = costs.shape
    n = C.c_int(0)
    L.acmmp_support_points(_p(costs), W, H, None, 0, C.byref(n))
    xy = np.zeros((max(n.value, 1), 2), np.int32)
    _host_check(L.acmmp_support_points(_p(costs), W, H, _p(xy), n.value, C.byref(n)), "support_points")
    return xy[:n.value]


def delaunay(xy, W: int, H: int) -> np.ndarray:
    """DelaunayTriangulation (ACMMP.cpp:932-955) -> (m, 3, 2) int32 triangle vertices."""
    L = load_library()
    xy = np.ascontiguousarray(xy, np.int32).reshape(-1, 2)
    m = C.c_int(0)
    L.acmmp_delaunay(_p(xy), xy.shape[0], W, H, None, 0, C.byref(m))
    tri = np.zeros((max(m.value, 1), 3, 2), np.int32)
    _host_check(L.acmmp_delaunay(_p(xy), xy.shape[0], W, H, _p(tri), m.value, C.byref(m)), "delaunay")
    return tri[:m.value]


def prior_plane_params(cam0, depths, tri) -> np.ndarray:
    """GetPriorPlaneParams (ACMMP.cpp:957-989) for one triangle ((3, 2) ints)."""
    L = load_library()
    depths = np.ascontiguousarray(depths, np.float32)
    H, W = depths.shape
    tri = np.ascontiguousarray(tri, np.int32).reshape(6)
    out = np.zeros(4, np.float32)
    cam, cp = _cam_ptr(cam0)
    _host_check(L.acmmp_prior_plane_params(cp, _p(depths), W, H, _p(tri), _p(out)), "prior_plane_params")
    return out


def depth_from_plane_param(cam0, plane, x: int, y: int) -> float:
    """GetDepthFromPlaneParam (ACMMP.cpp:991-1011)."""
    plane = np.ascontiguousarray(plane, np.float32)
    cam, cp = _cam_ptr(cam0)
    return float(load_library().acmmp_depth_from_plane_param(cp, _p(plane), int(x), int(y)))


def planar_prior_host(cam0, depths, costs, depth_min: float, depth_max: float):
    """main.cpp:113-181 + ACMMP.cpp:851-861 -> (prior_planes (H, W, 4), masks (H, W) uint32, n_triangles)."""
    L = load_library()
    depths = np.ascontiguousarray(depths, np.float32)
    costs = np.ascontiguousarray(costs, np.float32)
    H, W = depths.shape
    prior = np.zeros((H, W, 4), np.float32)
    masks = np.zeros((H, W), np.uint32)
    n = C.c_int(0)
    cam, cp = _cam_ptr(cam0)
    _host_check(L.acmmp_planar_prior_host(cp, _p(depths), _p(costs), W, H, float(depth_min), float(depth_max),
                                          _p(prior), _p(masks), C.byref(n)), "planar_prior_host")
    return prior, masks, n.value


# ---- device buffers + RCCL communicator (multi-GPU pipeline) ---------------------

class DeviceBuffer:
    """A float32 (H, W) buffer in HBM of one GPU (pipeline depth store)."""

    def __init__(self, device: int, shape):
        self.L = load_library()
        self.device, self.shape = device, tuple(int(v) for v in shape)
        self.nbytes = 4 * int(np.prod(self.shape))
        p = C.c_void_p()
        _host_check(self.L.acmmp_device_alloc(device, self.nbytes, C.byref(p)), "device_alloc")
        self.ptr = p.value

    def upload(self, arr):
        a = np.ascontiguousarray(arr, np.float32)
        assert a.shape == self.shape
        _host_check(self.L.acmmp_memcpy(self.device, C.c_void_p(self.ptr), _p(a), self.nbytes, 0), "memcpy H2D")

    def download(self):
        a = host_empty(self.shape, np.float32)
        _host_check(self.L.acmmp_memcpy(self.device, _p(a), C.c_void_p(self.ptr), self.nbytes, 1), "memcpy D2H")
        return a

    def checksum(self) -> int:
        """acmmp_device_checksum of the buffer (equal to checksum_host of its download)."""
        out = C.c_uint64(0)
        _host_check(self.L.acmmp_device_checksum(self.device, C.c_void_p(self.ptr), self.nbytes, C.byref(out)),
                    "device_checksum")
        return int(out.value)

    def free(self):
        if self.ptr:
            self.L.acmmp_device_free(self.device, C.c_void_p(self.ptr))
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Comm:
    """RCCL communicator of this process's GPU (one rank per process)."""

    ID_BYTES = 128

    @staticmethod
    def unique_id() -> bytes:
        buf = (C.c_uint8 * Comm.ID_BYTES)()
        _host_check(load_library().acmmp_comm_unique_id(C.cast(buf, C.c_void_p)), "comm_unique_id")
        return bytes(buf)

    def __init__(self, device: int, uid: bytes, nranks: int, rank: int):
        self.L = load_library()
        assert len(uid) == self.ID_BYTES
        buf = (C.c_uint8 * self.ID_BYTES).from_buffer_copy(uid)
        h = C.c_void_p()
        _host_check(self.L.acmmp_comm_create(device, C.cast(buf, C.c_void_p), nranks, rank, C.byref(h)),
                    "comm_create")
        self.h, self.nranks, self.rank = h, nranks, rank

    def broadcast(self, bufs, roots):
        """In-place grouped broadcast of DeviceBuffers, bufs[i] from rank roots[i]."""
        n = len(bufs)
        ptrs = (C.c_void_p * n)(*[b.ptr for b in bufs])
        nb = np.array([b.nbytes for b in bufs], np.uint64)
        rt = np.array(roots, np.int32)
        _host_check(self.L.acmmp_comm_broadcast(self.h, n, C.cast(ptrs, C.c_void_p), _p(nb), _p(rt)), "broadcast")

    def after(self, ctx: "Context"):
        """Collectives queued from now on start after the work `ctx` has queued so far (device-side order)."""
        _host_check(self.L.acmmp_comm_after(self.h, ctx.h), "comm_after")

    def band_exchange(self, ctx: "Context", colour: int, rank_up: int, rank_down: int):
        _host_check(self.L.acmmp_comm_band_exchange(self.h, ctx.h, colour, rank_up, rank_down), "band_exchange")

    def allreduce_max(self, vals):
        v = np.ascontiguousarray(vals, np.float64).copy()
        _host_check(self.L.acmmp_comm_allreduce_max(self.h, _p(v), v.size), "allreduce_max")
        return v

    def close(self):
        if self.h:
            self.L.acmmp_comm_destroy(self.h)
            self.h = None


# ---- GPU fusion (RunFusionCuda / SimpleFusionKernel, ACMMP.cu:1662-2105) ---------------------------

class Fusion:
    """Depth-map fusion on one GPU.  cams: CAMERA_DTYPE array, each rescaled to its depth map."""

    def __init__(self, device: int, cams):
        self.L = load_library()
        self.cams = np.frombuffer(np.ascontiguousarray(cams, dtype=CAMERA_DTYPE).tobytes(), CAMERA_DTYPE).copy()
        h = C.c_void_p()
        _host_check(self.L.acmmp_fusion_create(device, len(self.cams), _p(self.cams), C.byref(h)), "fusion_create")
        self.h = h

    def _check(self, rc, what):
        if rc != 0:
            msg = self.L.acmmp_fusion_last_error(self.h).decode()
            raise AcmmpError(f"{what}: {self.L.acmmp_status_str(rc).decode()} ({msg})")

    def set_view(self, view: int, depth, normals, bgr):
        d = np.ascontiguousarray(depth, np.float32)
        n = np.ascontiguousarray(normals, np.float32)
        c = np.ascontiguousarray(bgr, np.uint8)
        H, W = int(self.cams[view]["height"]), int(self.cams[view]["width"])
        assert d.shape == (H, W) and n.shape == (H, W, 3) and c.shape == (H, W, 3)
        self._check(self.L.acmmp_fusion_set_view(self.h, view, _p(d), _p(n), _p(c)), "fusion_set_view")

    def run(self, ref: int, src_views) -> np.ndarray:
        """Consistent points of reference view `ref`, (n, 9) float32 in pixel order."""
        srcs = np.ascontiguousarray(src_views, np.int32)
        n = C.c_int(0)
        self.L.acmmp_fusion_run(self.h, ref, srcs.size, _p(srcs), None, 0, C.byref(n))
        out = np.zeros((max(n.value, 1), 9), np.float32)
        self._check(self.L.acmmp_fusion_run(self.h, ref, srcs.size, _p(srcs), _p(out), n.value, C.byref(n)),
                    "fusion_run")
        return out[:n.value]

    def close(self):
        if self.h:
            self.L.acmmp_fusion_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
