"""Build the in-tree HIP extension libacmmp.so for gfx950 (no cmake; plain hipcc).

`python acmmp-spherical_amd/build.py` or `acmmp.build.build()`; __graft_entry__.build()
calls it with force=True (every object recompiled, in parallel).  Without force, objects are rebuilt
only when a source or header is newer than them.  Every link writes `acmmp/build_info.json` (sources'
SHA-256, compiler flags, UTC time) next to the library, so a run can show which build it loaded.
"""
from __future__ import annotations

import datetime
import hashlib
import json
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
LIB = os.path.join(HERE, "acmmp", "libacmmp.so")
ARCH = os.environ.get("ACMMP_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

SOURCES = ["kernels.hip", "capi.cpp", "comm.cpp", "fusion.cpp", "planar_prior.cpp"]
HIP_CPP = {"capi.cpp", "comm.cpp", "fusion.cpp"}              # host C++ that includes HIP headers
HEADERS = ["engine.h", "detmath.h"]
COMMON = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-fno-slp-vectorize", f"--offload-arch={ARCH}",
          f"-I{INCLUDE}", f"-I{CSRC}", "-Wall", "-Wno-unused-function"]


def _newest(paths):
    return max(os.path.getmtime(p) for p in paths)


def build(force: bool = False, verbose: bool = True, lib: str = LIB, defines=(), objdir: str | None = None,
          flags=()) -> str:
    """Compile csrc/ into `lib`.  `defines` (e.g. ["ACMMP_EXPERIMENT=1"]) + a separate `objdir` give an
    experiment variant next to the product build (select it at run time with ACMMP_LIB=<path>)."""
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.join(INCLUDE, "acmmp.h")]
    if not force and os.path.exists(lib) and os.path.getmtime(lib) >= _newest(deps):
        return lib
    objdir = objdir or os.path.join(HERE, "build")
    os.makedirs(objdir, exist_ok=True)
    objs, cmds = [], []
    for src in SOURCES:
        obj = os.path.join(objdir, src + ".o")
        srcp = os.path.join(CSRC, src)
        hdrs = [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(INCLUDE, "acmmp.h")]
        if force or not os.path.exists(obj) or os.path.getmtime(obj) < _newest([srcp] + hdrs):
            lang = ["-x", "hip"] if src in HIP_CPP else []
            cmds.append([HIPCC, *COMMON, *flags, *[f"-D{d}" for d in defines], *lang, "-c", srcp, "-o", obj])
        objs.append(obj)

    def compile_one(cmd):
        if verbose:
            print("[acmmp build]", " ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)

    with ThreadPoolExecutor(max_workers=min(len(cmds), 4) or 1) as ex:
        list(ex.map(compile_one, cmds))
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib, *objs, "-L/opt/rocm/lib", "-lrccl",
           "-Wl,-rpath,/opt/rocm/lib"]
    if verbose:
        print("[acmmp build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    info = {"library": os.path.basename(lib), "built_utc": datetime.datetime.now(datetime.timezone.utc).isoformat(),
            "forced": bool(force), "arch": ARCH, "flags": COMMON + list(flags), "defines": list(defines),
            "sources_sha256": {os.path.relpath(d, os.path.dirname(HERE)): hashlib.sha256(open(d, "rb").read()).hexdigest()
                               for d in deps}}
    with open(os.path.join(os.path.dirname(lib), "build_info.json" if lib == LIB else
                           os.path.basename(lib) + ".build_info.json"), "w") as f:
        json.dump(info, f, indent=1)
    return lib


if __name__ == "__main__":
    build(force="--force" in sys.argv)
