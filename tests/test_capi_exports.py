"""The C-ABI library loads without a GPU and exports every entry point include/acmmp.h declares;
the POD layouts match the reference's Camera / PatchMatchParams and the numpy dtypes."""
import os
import re
import subprocess

import numpy as np

from acmmp import capi, types

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "acmmp.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(acmmp_[a-z_0-9]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    L = capi.load_library()
    decl = declared_functions()
    assert len(decl) >= 20
    missing = [f for f in decl if not hasattr(L, f)]
    assert not missing, missing
    assert sorted(capi.EXPORTS) == decl
    out = subprocess.run(["nm", "-D", "--defined-only", capi.LIB_PATH], capture_output=True, text=True).stdout
    for f in decl:
        assert re.search(rf"\bT {f}$", out, re.M), f


def test_abi_version_and_status_strings():
    L = capi.load_library()
    assert L.acmmp_abi_version() == 1
    assert L.acmmp_status_str(0) == b"ok"
    assert L.acmmp_status_str(5) == b"unsupported configuration"


def test_struct_layouts_match_header(tmp_path):
    prog = tmp_path / "layout.c"
    prog.write_text(f'''#include <stdio.h>
#include <stddef.h>
#include "{HEADER}"
int main(void) {{
  printf("%zu %zu %zu %zu %zu %zu %zu %zu\\n", sizeof(acmmp_camera), sizeof(acmmp_params),
         offsetof(acmmp_camera, R), offsetof(acmmp_camera, width), offsetof(acmmp_camera, depth_max),
         offsetof(acmmp_params, scaled_cols), offsetof(acmmp_params, geom_consistency),
         offsetof(acmmp_params, upsample));
  return 0;
}}''')
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c99", "-o", str(exe), str(prog)], check=True)
    vals = [int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True).stdout.split()]
    cam, par = types.CAMERA_DTYPE, types.PARAMS_DTYPE
    assert vals == [cam.itemsize, par.itemsize, cam.fields["R"][1], cam.fields["width"][1],
                    cam.fields["depth_max"][1], par.fields["scaled_cols"][1],
                    par.fields["geom_consistency"][1], par.fields["upsample"][1]]
    assert vals[:2] == [120, 68]          # main.h:40-54, ACMMP.h:32-55


def test_no_device_fails_loudly():
    """Without a GPU the engine refuses to run (there is no CPU fallback)."""
    import pytest
    if os.path.exists("/dev/kfd"):
        pytest.skip("a GPU is visible")
    with pytest.raises(capi.AcmmpError):
        capi.Context(0)


def test_default_params_match_reference():
    p = types.default_params()
    assert (int(p["max_iterations"]), int(p["patch_size"]), int(p["radius_increment"]), int(p["top_k"])) == (3, 11, 2, 4)
    assert float(p["sigma_spatial"]) == 5.0 and float(p["sigma_color"]) == 3.0
    assert np.float32(p["baseline"]) == np.float32(0.54)


def test_host_empty_download_arrays():
    """capi.host_empty: large download arrays on 2 MiB aligned private mappings that outlive every view of them
    and return to the pool only then; small ones plain numpy."""
    import gc
    small = capi.host_empty((100, 100), np.float32)
    assert small.base is None and small.shape == (100, 100)
    held0 = capi._POOL.held
    a = capi.host_empty((800, 600, 4), np.float32)
    assert a.ctypes.data % (2 << 20) == 0 and a.flags.writeable and a.flags.c_contiguous and a.dtype == np.float32
    a[...] = 7.0
    depth, normals = a[..., 3], a[..., :3]              # the pipeline keeps slices like these
    ptr = a.ctypes.data
    del a
    gc.collect()
    assert capi._POOL.held == held0                     # still referenced through the slices
    assert float(depth.sum()) == 7.0 * 800 * 600 and normals.shape == (800, 600, 3)
    del depth, normals
    gc.collect()
    assert capi._POOL.held > held0                      # back in the pool ...
    b = capi.host_empty((800, 600, 4), np.float32)
    assert b.ctypes.data == ptr                         # ... and reused by the next array of that size
    assert capi.host_empty((600, 800), np.uint32).dtype == np.uint32


def test_host_pool_cap_evicts_least_recent():
    """_HostPool keeps at most `cap` idle bytes, dropping the least recently returned mappings first, and
    release() drops them all (sizes of earlier pyramid scales must not stay held)."""
    pool = capi._HostPool(cap=3 << 20)
    a, b, c = pool.take(1 << 20), pool.take(2 << 20), pool.take(1 << 20)
    pool.give(a, 1 << 20)
    pool.give(b, 2 << 20)
    assert pool.held == 3 << 20
    pool.give(c, 1 << 20)                     # over the cap: a (oldest) goes
    assert pool.held == 3 << 20 and pool.take(1 << 20) is c
    assert pool.take(2 << 20) is b and pool.held == 0
    pool.give(pool.take(8 << 20), 8 << 20)    # larger than the cap: never kept
    assert pool.held == 0
    pool.give(a, 1 << 20)
    pool.release()
    assert pool.held == 0 and pool.take(1 << 20) is not a
