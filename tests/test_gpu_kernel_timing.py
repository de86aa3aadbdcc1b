"""acmmp_last_kernel_timing's two levels: by default only the k_eval_nb bucket is timed (every event record in
the stream idles the GPU a few microseconds; profiles/r06_ab9_events_ab.txt), and with ACMMP_KERNEL_TIMING=all
in the environment all four buckets are.  Neither changes a bit of the run's result."""
import numpy as np
import pytest

from acmmp import capi, scene, types
from conftest import assert_bitwise_equal

pytestmark = pytest.mark.gpu


def test_kernel_timing_levels_leave_results_unchanged(monkeypatch):
    sc = scene.sphere_scene(160, 80, n_src=4, seed=5)
    c0 = sc.cameras[0]
    p = types.default_params(num_images=len(sc.images), depth_min=float(c0["depth_min"]) * 0.6,
                             depth_max=float(c0["depth_max"]) * 1.2)
    n = 2 * int(p["max_iterations"])
    with capi.Context(0) as ctx:
        ctx.set_math("fast")
        ctx.set_params(p)
        ctx.upload_views(sc.images, sc.cameras)
        monkeypatch.delenv("ACMMP_KERNEL_TIMING", raising=False)
        ctx.run_patchmatch(11)
        a, ka = ctx.download(), ctx.last_kernel_timing()
        monkeypatch.setenv("ACMMP_KERNEL_TIMING", "all")
        ctx.run_patchmatch(11)
        b, kb = ctx.download(), ctx.last_kernel_timing()
    assert ka["k_eval_nb"][1] == n and ka["k_eval_nb"][0] > 0.0
    for k in ("k_select", "k_eval_ref", "k_finish"):
        assert ka[k] == (0.0, 0), (k, ka[k])
    for k, (ms, launches) in kb.items():
        assert launches == n and ms > 0.0, (k, ms, launches)
    assert_bitwise_equal(a[0], b[0], "planes")
    assert_bitwise_equal(a[1], b[1], "costs")
    assert np.isfinite(a[1]).any()
