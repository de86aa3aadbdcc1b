"""acmmp_set_planar_prior_from_state: the planar block of ProcessProblem (main.cpp:113-181) from the context's
own last RunPatchMatch output in HBM -- GetSupportPoints (ACMMP.cpp:904-929) on the device, only the support
points to the host -- must equal acmmp_set_planar_prior_from_maps on the downloaded maps bit for bit (the same
support points in the same order, the same triangles, planes, raster and mask)."""
import numpy as np
import pytest

from acmmp import capi, scene, types

pytestmark = pytest.mark.gpu

SCENES = {
    "pinhole-640x480-v4": lambda: scene.pinhole_scene(640, 480, n_src=4, seed=21, n_waves=24),
    "sphere-1000x500-v4": lambda: scene.sphere_scene(1000, 500, n_src=4, seed=22, n_waves=24),
    "pinhole-1603x1201-v2": lambda: scene.pinhole_scene(1603, 1201, n_src=2, seed=23, n_waves=12),
}


@pytest.fixture(scope="module")
def ctx():
    c = capi.Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("name", list(SCENES))
@pytest.mark.parametrize("math", ["exact", "fast"])
def test_planar_prior_from_state_equals_from_maps(ctx, name, math):
    sc = SCENES[name]()
    c0 = sc.cameras[0]
    p = types.default_params(num_images=len(sc.images), depth_min=float(c0["depth_min"]) * 0.6,
                             depth_max=float(c0["depth_max"]) * 1.2)
    ctx.set_math(math)
    ctx.set_params(p)
    ctx.upload_views(sc.images, sc.cameras)
    ctx.run_patchmatch(5)
    planes, costs = ctx.download()
    dmin, dmax = float(p["depth_min"]), float(p["depth_max"])
    n_maps = ctx.set_planar_prior_from_maps(planes[..., 3], costs, dmin, dmax)
    prior_m, masks_m = ctx.download_planar_prior()
    n_state = ctx.set_planar_prior_from_state(dmin, dmax)
    prior_s, masks_s = ctx.download_planar_prior()
    ctx.set_math("exact")
    assert n_maps > 100 and n_state == n_maps
    np.testing.assert_array_equal(masks_s, masks_m)
    np.testing.assert_array_equal(prior_s.view(np.uint32), prior_m.view(np.uint32))
    # the state is the run's: a second run overwrites it, and the prior follows
    ctx.set_math(math)
    ctx.run_patchmatch(6)
    planes2, costs2 = ctx.download()
    ctx.set_math("exact")
    n2 = ctx.set_planar_prior_from_state(dmin, dmax)
    prior2, masks2 = ctx.download_planar_prior()
    assert n2 == ctx.set_planar_prior_from_maps(planes2[..., 3], costs2, dmin, dmax)
    prior2m, masks2m = ctx.download_planar_prior()
    np.testing.assert_array_equal(masks2, masks2m)
    np.testing.assert_array_equal(prior2.view(np.uint32), prior2m.view(np.uint32))


def test_planar_prior_from_state_needs_this_problems_maps(ctx):
    """After upload_views the context's planes / costs belong to the previous problem: set_planar_prior_from_state
    refuses (ACMMP_ERR_STATE) until a run or set_state of both maps (capi.cpp has_result)."""
    sc = scene.sphere_scene(200, 100, n_src=2, seed=29)
    c0 = sc.cameras[0]
    p = types.default_params(num_images=len(sc.images), depth_min=float(c0["depth_min"]) * 0.6,
                             depth_max=float(c0["depth_max"]) * 1.2)
    dmin, dmax = float(p["depth_min"]), float(p["depth_max"])
    ctx.set_params(p)
    ctx.upload_views(sc.images, sc.cameras)
    ctx.run_patchmatch(3)
    planes, costs = ctx.download()
    ctx.upload_views(sc.images, sc.cameras)
    with pytest.raises(capi.AcmmpError):
        ctx.set_planar_prior_from_state(dmin, dmax)
    ctx.set_state(planes, costs)
    ctx.set_planar_prior_from_state(dmin, dmax)
    ctx.upload_views(sc.images, sc.cameras)
    ctx.run_patchmatch(3)
    ctx.set_planar_prior_from_state(dmin, dmax)
