"""The built library's gfx950 device code: no VALU transcendental whose result is read by the very next
instruction (scripts/hazard_scan.py).  gfx950 wants a wait state there; the compiler inserts it for its own
instructions but not in front of inline asm, and round 6 found an inline-asm v_max_f32 right after a v_sqrt
reading a half-written register (kernels.hip, max_abs_h).  No GPU needed: the code objects are unbundled and
disassembled with the image's llvm-objdump."""
import os
import sys

import pytest

from acmmp import capi

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "scripts"))
import hazard_scan  # noqa: E402


@pytest.mark.skipif(not os.path.exists(hazard_scan.OBJDUMP), reason="llvm-objdump not in this image")
def test_no_transcendental_result_read_without_a_wait_state():
    assert os.path.exists(capi.LIB_PATH), "build the library first (__graft_entry__.build())"
    hits = hazard_scan.scan_so(capi.LIB_PATH)
    assert not hits, [(h[2][:80], h[3], h[4]) for h in hits[:5]]


def test_scan_flags_the_pattern():
    text = "\n".join([
        "_ZN5acmmp4k_okEv:",
        "\tv_sqrt_f32_e32 v3, v2",
        "\ts_nop 0",
        "\tv_max_f32_e64 v4, |v3|, |v5|",
        "_ZN5acmmp5k_badEv:",
        "\tv_rcp_f32_e32 v7, v6",
        "\t;;#ASMSTART",
        "\tv_cvt_flr_i32_f32 v8, v7",
        "\t;;#ASMEND",
        "\tv_sqrt_f32_e32 v9, v2",
        "\tv_add_f32_e32 v10, v1, v2",
    ])
    hits = hazard_scan.scan("t.s", text)
    assert [(h[2], h[5]) for h in hits] == [("_ZN5acmmp5k_badEv", True)]
