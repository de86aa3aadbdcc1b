"""The oracle reproduces the committed golden fixtures bit for bit (tests/golden, made by
scripts/make_golden.py).  PARITY UNPINNED: these are oracle outputs, not reference outputs
(the reference ships none and cannot be built here)."""
import glob
import os

import numpy as np
import pytest

from conftest import assert_bitwise_equal

GOLDEN = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*.npz")))


def load(path):
    z = np.load(path, allow_pickle=False)
    return {k: z[k] for k in z.files}


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p) for p in GOLDEN])
def test_oracle_reproduces_golden(oracle_mod, path):
    g = load(path)
    prob = oracle_mod.Problem(list(g["images"]), g["cameras"], g["params"].view(np.uint8))
    r = oracle_mod.run_patchmatch(prob, seed=int(g["seed"]), nthreads=4)
    assert_bitwise_equal(r["planes"], g["planes"], "planes")
    assert_bitwise_equal(r["costs"], g["costs"], "costs")
    assert_bitwise_equal(r["selected_views"], g["selected_views"], "selected_views")
    for k in range(len(g["ncc_px"])):
        for v in range(g["ncc_costs"].shape[1]):
            c = oracle_mod.ncc(prob, v + 1, int(g["ncc_px"][k]), int(g["ncc_py"][k]), g["ncc_planes"][k])
            assert np.float32(c).view(np.uint32) == g["ncc_costs"][k, v].view(np.uint32)


def test_golden_fixture_count():
    assert len(GOLDEN) >= 3
