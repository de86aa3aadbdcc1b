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
KERNEL_TUS = 5            # kernels.hip is compiled once per ACMMP_TU value in parallel (see its header)
HIP_CPP = {"capi.cpp", "comm.cpp", "fusion.cpp", "planar_prior.cpp"}              # host C++ that includes HIP headers
HEADERS = ["engine.h", "detmath.h", "planar.h"]
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
    units = [(src, None) for src in SOURCES if src != "kernels.hip"]
    units = [("kernels.hip", tu) for tu in range(KERNEL_TUS)] + units
    for src, tu in units:
        obj = os.path.join(objdir, src + (f".tu{tu}" if tu is not None else "") + ".o")
        srcp = os.path.join(CSRC, src)
        hdrs = [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(INCLUDE, "acmmp.h")]
        if force or not os.path.exists(obj) or os.path.getmtime(obj) < _newest([srcp] + hdrs):
            lang = ["-x", "hip"] if src in HIP_CPP else []
            tud = [f"-DACMMP_TU={tu}"] if tu is not None else []
            cmds.append([HIPCC, *COMMON, *flags, *[f"-D{d}" for d in defines], *tud, *lang, "-c", srcp, "-o", obj])
        objs.append(obj)

    def compile_one(cmd):
        if verbose:
            print("[acmmp build]", " ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)

    with ThreadPoolExecutor(max_workers=min(len(cmds), max(1, min(8, os.cpu_count() or 1)))) as ex:
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


HOST = os.path.join(HERE, "host")
HOST_LIB = os.path.join(HERE, "acmmp", "libacmmp_host.so")
HOST_EXE = os.path.join(HERE, "acmmp", "ACMMP")
HOST_SOURCES = ["formats.cpp", "jpeg.cpp"]
HOST_HEADERS = ["formats.hpp", "jpeg.hpp", "ACMMP.hpp"]
HOST_FLAGS = ["-O2", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-Wall", "-Wextra", "-Werror", f"-I{INCLUDE}"]


def build_host(force: bool = False, verbose: bool = True, engine_lib: str = LIB):
    """The C++ host side (plain g++, no GPU code): libacmmp_host.so (formats + JPEG decoder + their
    test entry points) and the drop-in driver executable `ACMMP` (host/acmmp_main.cpp, the reference's
    main.cpp) linked against libacmmp.so."""
    deps = [os.path.join(HOST, f) for f in HOST_SOURCES + HOST_HEADERS + ["host_capi.cpp", "acmmp_main.cpp"]] + \
        [os.path.join(INCLUDE, "acmmp.h")]
    outs = [HOST_LIB, HOST_EXE]
    if not force and all(os.path.exists(o) for o in outs) and min(os.path.getmtime(o) for o in outs) >= _newest(deps):
        return HOST_LIB, HOST_EXE
    srcs = [os.path.join(HOST, f) for f in HOST_SOURCES]
    libdir = os.path.dirname(engine_lib)
    cmds = [["g++", *HOST_FLAGS, "-shared", "-fPIC", "-o", HOST_LIB, *srcs, os.path.join(HOST, "host_capi.cpp")],
            ["g++", *HOST_FLAGS, "-o", HOST_EXE, os.path.join(HOST, "acmmp_main.cpp"), *srcs,
             f"-L{libdir}", "-l:" + os.path.basename(engine_lib), f"-Wl,-rpath,{libdir}"]]
    for cmd in cmds:
        if verbose:
            print("[acmmp build]", " ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    return HOST_LIB, HOST_EXE


if __name__ == "__main__":
    build(force="--force" in sys.argv)
    build_host(force="--force" in sys.argv)
