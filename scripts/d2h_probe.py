"""D2H rate of Context.download at two view sizes: fresh numpy arrays per call (what the pipeline does) against
arrays reused across calls.  python scripts/d2h_probe.py"""
import json
import mmap
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "acmmp-spherical_amd"))

import numpy as np  # noqa: E402

from acmmp import capi, scene, types  # noqa: E402

def huge_empty(shape, dtype=np.float32):
    """An anonymous mapping, 2 MiB aligned, advised MADV_HUGEPAGE (what capi.host_empty does)."""
    n = int(np.prod(shape)) * np.dtype(dtype).itemsize
    mm = mmap.mmap(-1, n + (2 << 20), flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
    mm.madvise(mmap.MADV_HUGEPAGE)
    addr = np.frombuffer(mm, np.uint8).ctypes.data
    off = (-addr) % (2 << 20)
    return np.frombuffer(mm, dtype, int(np.prod(shape)), off).reshape(shape)


out = {}
with capi.Context(0) as ctx:
    for (w, h) in ((800, 600), (1600, 1200), (800, 600)):
        sc = scene.pinhole_scene(w, h, n_src=2, seed=1, n_waves=8)
        c0 = sc.cameras[0]
        p = types.default_params(num_images=3, depth_min=float(c0["depth_min"]), depth_max=float(c0["depth_max"]))
        p["max_iterations"] = 1
        ctx.set_params(p)
        ctx.upload_views(sc.images, sc.cameras)
        ctx.run_patchmatch(1)
        res = {}
        for mode in ("mmap_keep", "fresh", "reused", "fresh_keep"):
            keep, ts = [], []
            pl = np.empty((h, w, 4), np.float32)
            co = np.empty((h, w), np.float32)
            for k in range(30):
                t0 = time.perf_counter()
                if mode == "reused":
                    ctx.download_into(pl, co)
                elif mode == "mmap_keep":
                    a = (huge_empty((h, w, 4)), huge_empty((h, w)))
                    ctx.download_into(*a)
                    keep.append(a)
                else:
                    a = ctx.download()
                    if mode == "fresh_keep":
                        keep.append(a)
                ts.append(time.perf_counter() - t0)
            res[mode] = {"median_ms": round(1e3 * float(np.median(ts)), 3), "max_ms": round(1e3 * max(ts), 3),
                         "GBps": round(w * h * 20 / np.median(ts) / 1e9, 2)}
        out.setdefault(f"{w}x{h}", []).append(res)
        print(w, h, res, flush=True)
print(json.dumps(out))
