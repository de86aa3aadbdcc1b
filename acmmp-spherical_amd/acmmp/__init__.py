"""acmmp -- host side of the MI355X-native ACMMP-Spherical PatchMatch engine.

The compute path is libacmmp.so (HIP/gfx950) behind the C ABI in include/acmmp.h.
This package holds the Python mirror of the reference host API (ACMMP class +
ProcessProblem flow), the ctypes binding, synthetic scene generation and the
reference's on-disk formats.
"""
from .types import (CAMERA_DTYPE, PARAMS_DTYPE, PINHOLE, SPHERE, default_params, make_camera)  # noqa: F401

__all__ = ["CAMERA_DTYPE", "PARAMS_DTYPE", "PINHOLE", "SPHERE", "default_params", "make_camera"]
