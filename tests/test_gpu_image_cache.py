"""The shared image cache (acmmp_image_cache_*, acmmp_upload_views_keyed): prepared source images are
reused across problems and contexts without changing a bit of any result.

The reference prepares every image of every problem again (InuputInitialization ACMMP.cpp:567-643 +
CudaSpaceInitialization :685-712); a keyed upload must give exactly the RunPatchMatch output of a plain
upload, for hits, misses, mixed keyed / unkeyed views, images that are not binary16-exact, entries
evicted under a budget, and a cache closed while a context still uses its entries.
"""
import numpy as np
import pytest

from acmmp import capi, scene, types
from conftest import assert_bitwise_equal

pytestmark = pytest.mark.gpu


def params_for(sc, **kw):
    c0 = sc.cameras[0]
    return types.default_params(num_images=len(sc.images), depth_min=float(c0["depth_min"]) * 0.6,
                                depth_max=float(c0["depth_max"]) * 1.2, **kw)


def dev_bufs(images):
    out = []
    for im in images:
        b = capi.DeviceBuffer(0, im.shape)
        b.upload(np.ascontiguousarray(im, np.float32))
        out.append(b)
    return out


def run_plain(ctx, sc, p, seed):
    ctx.set_params(p)
    ctx.upload_views(sc.images, sc.cameras)
    ctx.run_patchmatch(seed)
    return ctx.download()


def run_keyed(ctx, cache, bufs, cams, keys, p, seed):
    ctx.set_params(p)
    ctx.upload_views_device(bufs, cams, cache=cache, keys=keys)
    ctx.run_patchmatch(seed)
    return ctx.download()


@pytest.mark.parametrize("kind", ["pinhole", "sphere"])
def test_keyed_uploads_equal_plain_uploads(kind):
    sc = (scene.pinhole_scene(96, 64, n_src=5, seed=3) if kind == "pinhole"
          else scene.sphere_scene(128, 64, n_src=5, seed=3))
    n = len(sc.images)
    bufs = dev_bufs(sc.images)
    cache = capi.ImageCache(0)
    with capi.Context(0) as plain, capi.Context(0) as a, capi.Context(0) as b:
        # problem k: reference k, sources = the other views (as a pipeline pass does)
        for k in range(3):
            order = [k] + [j for j in range(n) if j != k]
            sub = type("S", (), {})()
            sub.images = [sc.images[j] for j in order]
            sub.cameras = np.asarray(sc.cameras)[order]
            p = params_for(sub)
            want = run_plain(plain, sub, p, 100 + k)
            keys = [j + 1 for j in order]
            got_a = run_keyed(a, cache, [bufs[j] for j in order], sub.cameras, keys, p, 100 + k)
            got_b = run_keyed(b, cache, [bufs[j] for j in order], sub.cameras, keys, p, 100 + k)
            for got in (got_a, got_b):
                assert_bitwise_equal(got[0], want[0], f"planes, problem {k}")
                assert_bitwise_equal(got[1], want[1], f"costs, problem {k}")
            assert a.texel_bytes() == plain.texel_bytes() == 2
        st = cache.stats()
        assert st["entries"] == n and st["misses"] == n and st["hits"] == 6 * n - n
        # unkeyed views (key 0) are prepared privately and do not enter the cache
        keys = [1, 0, 3, 0, 5, 6]
        got = run_keyed(a, cache, bufs, np.asarray(sc.cameras), keys, params_for(sc), 7)
        want = run_plain(plain, sc, params_for(sc), 7)
        assert_bitwise_equal(got[0], want[0], "planes, mixed keys")
        assert cache.stats()["entries"] == n
    cache.close()
    for bb in bufs:
        bb.free()


def test_inexact_images_fall_back_to_fp32_and_budget_evicts():
    sc = scene.pinhole_scene(80, 48, n_src=3, seed=9, quantize=False)   # not 8-bit: no exact binary16
    bufs = dev_bufs(sc.images)
    cams = np.asarray(sc.cameras)
    p = params_for(sc)
    entry = 4 * 82 * 50                                              # one padded fp32 image
    cache = capi.ImageCache(0, budget_bytes=2 * entry)
    with capi.Context(0) as plain, capi.Context(0) as a:
        want = run_plain(plain, sc, p, 11)
        assert plain.texel_bytes() == 4
        got = run_keyed(a, cache, bufs, cams, [11, 12, 13, 14], p, 11)
        assert a.texel_bytes() == 4
        assert_bitwise_equal(got[0], want[0], "planes")
        assert_bitwise_equal(got[1], want[1], "costs")
        # all four are pinned by a's problem: the soft budget cannot evict them yet
        assert cache.stats()["entries"] == 4
        sc2 = scene.pinhole_scene(80, 48, n_src=3, seed=10, quantize=False)
        bufs2 = dev_bufs(sc2.images)
        got2 = run_keyed(a, cache, bufs2, np.asarray(sc2.cameras), [21, 22, 23, 24], params_for(sc2), 12)
        want2 = run_plain(plain, sc2, params_for(sc2), 12)
        assert_bitwise_equal(got2[0], want2[0], "planes after eviction")
        st = cache.stats()
        assert st["evictions"] == 4 and st["entries"] == 4
        for bb in bufs2:
            bb.free()
    cache.close()
    for bb in bufs:
        bb.free()


def test_cache_closed_while_a_context_still_uses_it():
    sc = scene.sphere_scene(96, 48, n_src=2, seed=4)
    bufs = dev_bufs(sc.images)
    cams = np.asarray(sc.cameras)
    p = params_for(sc)
    cache = capi.ImageCache(0)
    with capi.Context(0) as plain, capi.Context(0) as a:
        want = run_plain(plain, sc, p, 5)
        run_keyed(a, cache, bufs, cams, [1, 2, 3], p, 5)
        cache.close()                                                # a still pins the entries
        a.run_patchmatch(5)
        got = a.download()
        assert_bitwise_equal(got[0], want[0], "planes after the cache was closed")
        a.upload_views(sc.images, sc.cameras)                        # releases the last reference
        a.run_patchmatch(5)
        assert_bitwise_equal(a.download()[0], want[0], "planes, plain upload on the same context")
    for bb in bufs:
        bb.free()


def test_keyed_upload_argument_errors():
    sc = scene.pinhole_scene(40, 32, n_src=1, seed=1)
    bufs = dev_bufs(sc.images)
    cache = capi.ImageCache(0)
    with capi.Context(0) as a:
        with pytest.raises(ValueError, match="keys"):
            a.upload_views_device(bufs, np.asarray(sc.cameras), cache=cache, keys=[1])
    cache.close()
    for bb in bufs:
        bb.free()
