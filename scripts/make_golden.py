"""Generate the committed golden fixtures under tests/golden/ from the CPU oracle.

PARITY UNPINNED: the reference has no fixtures and cannot be built here, so these are
the oracle's own outputs on small seeded synthetic scenes.  They pin the oracle (and the
engine, which must reproduce them bit for bit) against regressions; they are not
reference outputs.  Re-run only when the fixed semantics change on purpose:
    python scripts/make_golden.py
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "acmmp-spherical_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))

import oracle  # noqa: E402
from acmmp import scene, types  # noqa: E402

OUT = os.path.join(REPO, "tests", "golden")


def case(name, sc, seed, **pover):
    c0 = sc.cameras[0]
    p = types.default_params(num_images=len(sc.images), depth_min=float(c0["depth_min"]) * 0.6,
                             depth_max=float(c0["depth_max"]) * 1.2, **pover)
    prob = oracle.Problem(sc.images, sc.cameras, p)
    r = oracle.run_patchmatch(prob, seed=seed, nthreads=4)
    rng = np.random.default_rng(seed)
    H, W = sc.images[0].shape
    n = 64
    qx, qy = rng.integers(0, W, n).astype(np.int32), rng.integers(0, H, n).astype(np.int32)
    nrm = rng.normal(size=(n, 3))
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    nrm[:, 2] = -np.abs(nrm[:, 2])
    qp = np.concatenate([nrm, rng.uniform(float(p["depth_min"]), float(p["depth_max"]), (n, 1))], 1).astype(np.float32)
    qc = np.array([[oracle.ncc(prob, v, int(qx[k]), int(qy[k]), qp[k]) for v in range(1, len(sc.images))]
                   for k in range(n)], np.float32)
    np.savez_compressed(os.path.join(OUT, name + ".npz"), images=np.stack(sc.images), cameras=sc.cameras,
                        params=np.frombuffer(p.tobytes(), np.uint8), seed=np.uint64(seed),
                        planes=r["planes"], costs=r["costs"], selected_views=r["selected_views"],
                        ncc_px=qx, ncc_py=qy, ncc_planes=qp, ncc_costs=qc)
    print(name, "ok", os.path.getsize(os.path.join(OUT, name + ".npz")), "bytes")


if __name__ == "__main__":
    oracle.build()
    os.makedirs(OUT, exist_ok=True)
    case("pinhole_64x48_v2", scene.pinhole_scene(64, 48, n_src=2, seed=21), seed=101)
    case("sphere_80x40_v2", scene.sphere_scene(80, 40, n_src=2, seed=22), seed=102)
    case("pinhole_40x33_v5_oddrows", scene.pinhole_scene(40, 33, n_src=5, seed=23), seed=103)
