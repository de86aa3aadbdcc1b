"""Host time per engine call and pass of the multi-pass pipeline (diagnosis of where a pass's wall clock goes).

Wraps every public method of capi.Context / DeviceBuffer / ImageCache with a timer (synchronous calls, so the
time includes the GPU work a call waits for), keyed by the pass running, and prints one JSON line.
    python scripts/pipe_trace.py --views 12 [pipeline_bench.py's scene options]
"""
import argparse
import collections
import json
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "acmmp-spherical_amd"))

import numpy as np  # noqa: E402

from acmmp import capi, io, pipeline, scene  # noqa: E402

CUR = ["setup"]
ACC = collections.defaultdict(lambda: collections.defaultdict(lambda: [0, 0.0]))
LOCK = threading.Lock()


def wrap(cls):
    for name in list(vars(cls)):
        f = getattr(cls, name)
        if name.startswith("_") or not callable(f) or isinstance(vars(cls)[name], (staticmethod, classmethod, property)):
            continue

        def make(f, name):
            def g(*a, **k):
                t0 = time.perf_counter()
                try:
                    return f(*a, **k)
                finally:
                    dt = time.perf_counter() - t0
                    with LOCK:
                        e = ACC[CUR[0]][f"{cls.__name__}.{name}"]
                        e[0] += 1
                        e[1] += dt
            return g
        setattr(cls, name, make(f, name))
    init = cls.__init__

    def init_t(self, *a, **k):
        t0 = time.perf_counter()
        init(self, *a, **k)
        with LOCK:
            e = ACC[CUR[0]][f"{cls.__name__}.__init__"]
            e[0] += 1
            e[1] += time.perf_counter() - t0
    cls.__init__ = init_t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--views", type=int, default=12)
    ap.add_argument("--width", type=int, default=1600)
    ap.add_argument("--height", type=int, default=1200)
    ap.add_argument("--n-src", type=int, default=10)
    ap.add_argument("--model", choices=["sphere", "pinhole"], default="pinhole")
    ap.add_argument("--math", default="fast")
    ap.add_argument("--n-waves", type=int, default=24)
    a = ap.parse_args()
    for cls in (capi.Context, capi.DeviceBuffer, capi.ImageCache):
        wrap(cls)
    make = scene.sphere_scene if a.model == "sphere" else scene.pinhole_scene
    sc = make(a.width, a.height, n_src=a.views - 1, seed=5, n_waves=a.n_waves)
    centres = np.array([-(np.asarray(c["R"], np.float64).reshape(3, 3).T @ np.asarray(c["t"], np.float64))
                        for c in sc.cameras])
    problems = []
    for i in range(a.views):
        p = io.Problem(i)
        others = sorted([j for j in range(a.views) if j != i],
                        key=lambda j: (float(np.linalg.norm(centres[j] - centres[i])), j))[:a.n_src]
        p.src_image_ids = others
        problems.append(p)
    ds = pipeline.Dataset({i: np.asarray(sc.images[i], np.float32) for i in range(a.views)},
                          {i: np.array(sc.cameras[i], copy=True) for i in range(a.views)}, problems)
    marks = []

    def log(msg):
        marks.append((msg, time.perf_counter()))
        if "pass" in msg:
            CUR[0] = msg.split(": ")[-1] + "#" + msg.split("pass ")[-1].split(":")[0]
        print(msg, flush=True)

    t0 = time.perf_counter()
    pipe = pipeline.Pipeline(ds, order="reference", log=log, math=a.math).run()
    total = time.perf_counter() - t0
    out = {"total_s": round(total, 3), "passes": [[p.name, round(p.compute_s, 3)] for p in pipe.passes], "calls": {}}
    for ps, d in ACC.items():
        out["calls"][ps] = {k: [v[0], round(v[1], 4)] for k, v in sorted(d.items(), key=lambda kv: -kv[1][1])}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
