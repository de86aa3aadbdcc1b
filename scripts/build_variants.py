"""Build experiment variants of libacmmp.so side by side (A/B on the GPU box via ACMMP_LIB).
Usage: python scripts/build_variants.py NAME=DEF1,DEF2 NAME2=DEF3 ...   (parallel, one objdir each)"""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "acmmp-spherical_amd"))
import build  # noqa: E402


def one(spec):
    name, _, defs = spec.partition("=")
    defines = [d for d in defs.split(",") if d]
    lib = os.path.join(build.HERE, "acmmp", f"libacmmp_{name}.so")
    build.build(force=True, verbose=False, lib=lib, defines=defines, objdir=os.path.join(build.HERE, f"build_exp_{name}"))
    return lib


with ThreadPoolExecutor(4) as ex:
    for lib in ex.map(one, sys.argv[1:]):
        print(lib)
