"""POD types of the drop-in boundary, as numpy dtypes.

Byte-for-byte the reference's ABI structs:
  Camera           /root/reference/main.h:40-54   (120 bytes)
  PatchMatchParams /root/reference/ACMMP.h:32-55    (68 bytes)
and the C declarations in include/acmmp.h (acmmp_camera, acmmp_params).
"""
from __future__ import annotations

import numpy as np

PINHOLE = 0
SPHERE = 11
MAX_IMAGES = 256          # main.h:181
MAX_SRC_VIEWS = 32        # cost_vector[32] / uint32 view bitmask, ACMMP.cu:522,1153

CAMERA_DTYPE = np.dtype([
    ("model", "<i4"),
    ("params", "<f4", (4,)),
    ("R", "<f4", (9,)),
    ("t", "<f4", (3,)),
    ("K", "<f4", (9,)),
    ("width", "<i4"),
    ("height", "<i4"),
    ("depth_min", "<f4"),
    ("depth_max", "<f4"),
], align=False)
assert CAMERA_DTYPE.itemsize == 120

PARAMS_DTYPE = np.dtype({
    "names": ["max_iterations", "patch_size", "num_images", "max_image_size", "radius_increment",
              "sigma_spatial", "sigma_color", "top_k", "baseline", "depth_min", "depth_max",
              "disparity_min", "disparity_max", "scaled_cols", "scaled_rows",
              "geom_consistency", "planar_prior", "multi_geometry", "hierarchy", "upsample"],
    "formats": ["<i4", "<i4", "<i4", "<i4", "<i4", "<f4", "<f4", "<i4", "<f4", "<f4", "<f4",
                "<f4", "<f4", "<f4", "<f4", "u1", "u1", "u1", "u1", "u1"],
    "offsets": [0, 4, 8, 12, 16, 20, 24, 28, 32, 36, 40, 44, 48, 52, 56, 60, 61, 62, 63, 64],
    "itemsize": 68,
})


def default_params(**overrides) -> np.ndarray:
    """PatchMatchParams with the reference's in-class defaults (ACMMP.h:33-54).

    scaled_cols/scaled_rows have no initialiser in the reference; they are zeroed here.
    """
    p = np.zeros((), dtype=PARAMS_DTYPE)
    p["max_iterations"] = 3
    p["patch_size"] = 11
    p["num_images"] = 5
    p["max_image_size"] = 3200
    p["radius_increment"] = 2
    p["sigma_spatial"] = 5.0
    p["sigma_color"] = 3.0
    p["top_k"] = 4
    p["baseline"] = 0.54
    p["depth_min"] = 0.0
    p["depth_max"] = 1.0
    p["disparity_min"] = 0.0
    p["disparity_max"] = 1.0
    for k, v in overrides.items():
        p[k] = v
    return p


def make_camera(model=PINHOLE, K=None, params=None, R=None, t=None, width=0, height=0,
                depth_min=0.0, depth_max=1.0) -> np.ndarray:
    c = np.zeros((), dtype=CAMERA_DTYPE)
    c["model"] = model
    if K is not None:
        c["K"] = np.asarray(K, np.float32).reshape(9)
    if params is not None:
        pr = np.zeros(4, np.float32)
        pr[:len(params)] = params
        c["params"] = pr
    c["R"] = np.eye(3, dtype=np.float32).reshape(9) if R is None else np.asarray(R, np.float32).reshape(9)
    c["t"] = np.zeros(3, np.float32) if t is None else np.asarray(t, np.float32).reshape(3)
    c["width"] = width
    c["height"] = height
    c["depth_min"] = depth_min
    c["depth_max"] = depth_max
    return c
