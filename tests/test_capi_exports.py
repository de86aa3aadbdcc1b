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
