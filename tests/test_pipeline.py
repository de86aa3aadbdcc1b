"""Multi-pass pipeline driver: the reference's schedule
(main.cpp:392-482), ProcessProblem's pass wiring (geom state reload, hierarchy scaled state,
planar second run, JBU between scales), view sharding over ranks with the depth exchange
between passes, and -- on the GPU -- the engine-driven pipeline bit-identical to the same
pipeline driven by the CPU oracle."""
import os
import socket

import numpy as np
import pytest

from acmmp import io, pipeline, types
from conftest import assert_bitwise_equal
from pipeline_support import GlooExchange, OracleEngine, final_maps, small_dataset

SCHEDULE_2_SCALES = ["planar", "geom", "geom_multi", "hier_planar", "geom", "geom_multi"]


def test_resize_linear_matches_closed_form():
    img = np.arange(12 * 8, dtype=np.float32).reshape(8, 12)        # linear ramp: exact under bilinear
    out = pipeline.resize_linear(img, 6, 4)
    # (d + 0.5) * 2 - 0.5 = 2d + 0.5 -> mean of source columns 2d, 2d+1 (and rows)
    exp = np.array([[(img[2 * r, 2 * c] + img[2 * r, 2 * c + 1] + img[2 * r + 1, 2 * c] + img[2 * r + 1, 2 * c + 1]) / 4
                     for c in range(6)] for r in range(4)], np.float32)
    assert np.array_equal(out, exp)
    up = pipeline.resize_linear(img, 24, 16)
    assert up[0, 0] == img[0, 0] and up[-1, -1] == img[-1, -1]       # clamped borders


def test_scale_view_scales_cameras():
    ds = small_dataset(64, 32, 2, model="sphere")
    img, cam = pipeline.scale_view(ds.images[0], ds.cameras[0], 32)
    assert img.shape == (16, 32) and (cam["width"], cam["height"]) == (32, 16)
    assert cam["params"][1] == np.float32(ds.cameras[0]["params"][1] * np.float32(0.5))
    same, cam2 = pipeline.scale_view(ds.images[0], ds.cameras[0], 64)
    assert same is ds.images[0] and cam2["width"] == 64


def test_pipeline_schedule_single_rank():
    ds = small_dataset(64, 32, 3)
    pipe = pipeline.Pipeline(ds, engine=OracleEngine(), order="reference", size_bound=40).run()
    assert [p.name for p in pipe.passes] == SCHEDULE_2_SCALES
    assert all(p.views == [0, 1, 2] for p in pipe.passes)
    for v in range(3):
        d = pipe.store.get("depths_geom", v)
        assert d.shape == (32, 64)
        assert np.isfinite(d).mean() > 0.9
        assert pipe.store.get("normals", v).shape == (32, 64, 3)
        assert pipe.store.get("depths", v).shape == (32, 64)         # JBU output / hier-planar pass


@pytest.mark.parametrize("order", ["reference", "snapshot"])
def test_geom_pass_state_reuse_equals_rejoined_maps(order):
    """A geom pass restarts from its view's previous-pass planes: reusing that pass's downloaded plane
    array gives exactly the run that re-joins the stored depth and normal maps (ProcessProblem's
    reload, main.cpp:87-97), over the two-scale schedule."""
    a = pipeline.Pipeline(small_dataset(64, 32, 3), engine=OracleEngine(), order=order, size_bound=40,
                          reuse_planes=True).run()
    b = pipeline.Pipeline(small_dataset(64, 32, 3), engine=OracleEngine(), order=order, size_bound=40,
                          reuse_planes=False).run()
    for key in ("depths", "depths_geom", "normals", "costs"):
        for v in range(3):
            assert_bitwise_equal(a.store.get(key, v), b.store.get(key, v), f"{key} view {v}")


def test_pipeline_writes_reference_layout(tmp_path):
    ds = small_dataset(48, 24, 2)
    pipeline.Pipeline(ds, engine=OracleEngine(), order="reference", geom_iterations=1,
                      out_folder=str(tmp_path)).run()
    for v in range(2):
        d = tmp_path / "ACMMP" / f"2333_{v:08d}"
        for f in ("depths.dmb", "depths_geom.dmb", "normals.dmb", "costs.dmb"):
            assert (d / f).exists()
        assert io.read_dmb(str(d / "normals.dmb")).shape == (24, 48, 3)


def test_reference_order_differs_from_snapshot_only_in_multi_geometry():
    """Views of a multi_geometry pass read predecessors' fresh depths_geom in reference order."""
    ds = small_dataset(48, 24, 3)
    a = pipeline.Pipeline(ds, engine=OracleEngine(), order="reference", geom_iterations=1).run()
    b = pipeline.Pipeline(ds, engine=OracleEngine(), order="snapshot", geom_iterations=1).run()
    ma, mb = final_maps(a), final_maps(b)
    assert ma.keys() == mb.keys()
    for k in ma:                                               # one geom pass, no multi_geometry
        assert_bitwise_equal(ma[k], mb[k], str(k))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_main(rank, world, port, outdir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ds = small_dataset(64, 32, 3)
    pipe = pipeline.Pipeline(ds, engine=OracleEngine(nthreads=2), exchange=GlooExchange(dist), order="snapshot",
                             size_bound=40).run()
    maps = final_maps(pipe)
    np.savez(os.path.join(outdir, f"rank{rank}.npz"),
             **{f"{k}__{v}": a for (k, v), a in maps.items()})
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_snapshot_pipeline_equals_single_rank(tmp_path):
    """world_size 2 over gloo: views sharded 2 + 1, depth maps exchanged after every pass; the
    result equals the single-rank snapshot run bit for bit (every view, every stored map)."""
    import torch.multiprocessing as mp
    mp.spawn(_rank_main, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    single = final_maps(pipeline.Pipeline(small_dataset(64, 32, 3), engine=OracleEngine(), order="snapshot",
                                          size_bound=40).run())
    seen = set()
    for r in range(2):
        z = np.load(tmp_path / f"rank{r}.npz")
        for name in z.files:
            key, v = name.split("__")
            v = int(v)
            owner = v % 2
            if key in ("normals", "costs") and owner != r:
                continue
            assert_bitwise_equal(z[name], single[(key, v)], f"rank {r} {key} view {v}")
            seen.add((key, v))
    assert {(k, v) for (k, v) in single} <= seen


@pytest.mark.gpu
def test_gpu_pipeline_bitexact_vs_oracle_pipeline():
    ds = small_dataset(64, 32, 3)
    gpu = pipeline.Pipeline(ds, order="reference", size_bound=40).run()
    cpu = pipeline.Pipeline(ds, engine=OracleEngine(), order="reference", size_bound=40).run()
    mg, mc = final_maps(gpu), final_maps(cpu)
    assert mg.keys() == mc.keys() and len(mg) >= 12
    for k in mc:
        assert_bitwise_equal(mg[k], mc[k], str(k))


@pytest.mark.gpu
@pytest.mark.parametrize("math,slots", [("exact", True), ("fast", True), ("exact", 2), ("fast", 4)])
def test_gpu_pipeline_overlapped_planar_passes_equal_sequential(math, slots):
    """Planar passes on several engine contexts, views' planar blocks overlapping later views' first
    RunPatchMatch (Pipeline(overlap=True), the default: 3 contexts) store exactly what the sequential
    loop stores."""
    ds = small_dataset(64, 32, 5)
    a = pipeline.Pipeline(ds, order="reference", size_bound=40, math=math, overlap=slots).run()
    b = pipeline.Pipeline(ds, order="reference", size_bound=40, math=math, overlap=False).run()
    assert a._engine2 is not None and b._engine2 is None
    ma, mb = final_maps(a), final_maps(b)
    assert ma.keys() == mb.keys() and len(ma) >= 20
    for k in mb:
        assert_bitwise_equal(ma[k], mb[k], str(k))
    a.close()
    b.close()


@pytest.mark.gpu
@pytest.mark.parametrize("math", ["exact", "fast"])
def test_gpu_pipeline_snapshot_geom_overlap_equals_sequential(math):
    """Snapshot order (what sharded runs use) with geom_iterations 2: the geom passes, multi-geometry ones
    included, run overlapped on several contexts (the default) and store exactly what the sequential loop
    stores (the overlap-vs-sequential test covered only the reference order)."""
    ds = small_dataset(64, 32, 5)
    a = pipeline.Pipeline(ds, order="snapshot", size_bound=40, math=math, geom_iterations=2).run()
    b = pipeline.Pipeline(ds, order="snapshot", size_bound=40, math=math, geom_iterations=2, overlap=False).run()
    assert a._engine2 is not None and b._engine2 is None
    assert any(p.name.startswith("geom") for p in a.passes)
    ma, mb = final_maps(a), final_maps(b)
    assert ma.keys() == mb.keys() and len(ma) >= 20
    for k in mb:
        assert_bitwise_equal(ma[k], mb[k], str(k))
    a.close()
    b.close()


@pytest.mark.gpu
def test_rccl_single_rank_comm_and_device_store():
    """The RCCL communicator and device buffers of the exchange path on one rank (multi-rank runs
    need one GPU per rank: RCCL refuses two ranks on one device)."""
    from acmmp import capi
    comm = capi.Comm(0, capi.Comm.unique_id(), 1, 0)
    a = np.random.default_rng(0).normal(size=(17, 33)).astype(np.float32)
    buf = capi.DeviceBuffer(0, a.shape)
    buf.upload(a)
    comm.broadcast([buf], [0])
    assert np.array_equal(buf.download(), a)
    assert np.array_equal(comm.allreduce_max([1.5, -2.0]), [1.5, -2.0])
    # the exchange step's order: an export queued on the engine stream, then the broadcast behind an event
    # recorded there (acmmp_comm_after), as pipeline.RcclExchange and bench.depth_exchange do
    ds = small_dataset(48, 24, 2)
    with capi.Context(0) as ctx:
        p = types.default_params(num_images=2, depth_min=float(ds.cameras[0]["depth_min"]) * 0.6,
                                 depth_max=float(ds.cameras[0]["depth_max"]) * 1.2)
        ctx.set_params(p)
        ctx.upload_views([ds.images[0], ds.images[1]], np.array([ds.cameras[0], ds.cameras[1]]))
        ctx.run_patchmatch(5)
        planes, _ = ctx.download()
        dbuf = capi.DeviceBuffer(0, planes.shape[:2])
        ctx.export_depth(dbuf)
        comm.after(ctx)
        comm.broadcast([dbuf], [0])
        assert_bitwise_equal(dbuf.download(), planes[..., 3], "exported depth after the broadcast")
        dbuf.free()
        # RcclExchange.share with its payload check (device checksums before / after, compared over the comm)
        store = pipeline.ViewStore(0)
        store.put("depths", 0, planes[..., 3], ctx=ctx)
        ex = pipeline.RcclExchange(comm, 0, verify=True)
        ex.share("depths", [0], {0: 0}, store)
        assert ex.maps_verified == 1
        assert store.dev[("depths", 0)].checksum() == capi.checksum_host(np.ascontiguousarray(planes[..., 3]))
        for b in store.dev.values():
            b.free()
    comm.close()
    buf.free()


@pytest.mark.gpu
def test_gpu_export_and_device_depth_upload_roundtrip():
    from acmmp import capi
    ds = small_dataset(48, 24, 2)
    pipe = pipeline.Pipeline(ds, order="reference", geom_iterations=1)
    assert pipe.store.device is not None
    pipe.run()
    for v in range(2):
        host = pipe.store.get("depths_geom", v)
        dev = pipe.store.dev[("depths_geom", v)].download()
        assert_bitwise_equal(dev, host, f"view {v}")
    assert isinstance(pipe.engine, capi.Context)


@pytest.mark.gpu
def test_gpu_device_state_restart_equals_host_upload():
    """A geom pass restarted from the state kept in HBM (export_state -> set_state_device) equals the same
    pass restarted from host planes / costs (set_state), bit for bit, in both math modes."""
    from acmmp import capi
    ds = small_dataset(64, 32, 3)
    for math in ("exact", "fast"):
        with capi.Context(0) as e:
            e.set_math(math)
            ids = [0, 1, 2]
            p = types.default_params(num_images=3, depth_min=float(ds.cameras[0]["depth_min"]) * 0.6,
                                     depth_max=float(ds.cameras[0]["depth_max"]) * 1.2)
            e.set_params(p)
            e.upload_views([ds.images[i] for i in ids], np.array([ds.cameras[i] for i in ids]))
            e.run_patchmatch(5)
            planes, costs = e.download()
            bp, bc = capi.DeviceBuffer(0, (32, 64, 4)), capi.DeviceBuffer(0, (32, 64))
            e.export_state(bp, bc)
            assert_bitwise_equal(bp.download(), planes, "exported planes")
            assert_bitwise_equal(bc.download(), costs, "exported costs")
            dep = capi.DeviceBuffer(0, (32, 64))
            e.export_depth(dep)
            g = p.copy()
            g["geom_consistency"] = 1
            g["max_iterations"] = 2
            outs = []
            for via_device in (False, True):
                e.set_params(g)
                e.upload_views([ds.images[i] for i in ids], np.array([ds.cameras[i] for i in ids]))
                e.upload_depths_device([dep, dep, dep])
                if via_device:
                    e.set_state_device(bp, bc)
                else:
                    e.set_state(planes, costs)
                e.run_patchmatch(6)
                outs.append(e.download())
            assert_bitwise_equal(outs[1][0], outs[0][0], f"{math} planes")
            assert_bitwise_equal(outs[1][1], outs[0][1], f"{math} costs")
            for b in (bp, bc, dep):
                b.free()


def test_dense_folder_roundtrip(tmp_path):
    """write_dense_folder -> load_dataset: the reference's on-disk layout, pinhole reader quirk
    handled by the writer, JPEG luma decoded back within quantisation."""
    ds = small_dataset(48, 32, 3, model="pinhole")
    pipeline.write_dense_folder(str(tmp_path), ds, quality=100)
    back = pipeline.load_dataset(str(tmp_path))
    assert [p.ref_image_id for p in back.problems] == [0, 1, 2]
    assert back.problems[1].src_image_ids == [0, 2]
    for i in range(3):
        assert back.images[i].shape == ds.images[i].shape
        assert np.abs(back.images[i] - np.round(ds.images[i])).max() <= 3
        c, d = back.cameras[i], ds.cameras[i]
        assert np.allclose(c["K"], d["K"]) and np.allclose(c["R"], d["R"]) and np.allclose(c["t"], d["t"])
        assert c["depth_min"] == d["depth_min"] and c["depth_max"] == d["depth_max"]
        assert (c["width"], c["height"]) == (48, 32)


@pytest.mark.gpu
def test_gpu_cli_end_to_end_on_dense_folder(tmp_path):
    """`python -m acmmp.pipeline DENSE_FOLDER` on a written folder: the reference's outputs
    (per-view dmb files and the fused PLY) appear, depths close to ground truth."""
    import json
    import subprocess
    import sys
    from acmmp import scene
    sc = scene.sphere_scene(256, 128, n_src=2, seed=11)
    ds = pipeline.Dataset({i: np.asarray(sc.images[i], np.float32) for i in range(3)},
                          {i: np.array(sc.cameras[i], copy=True) for i in range(3)},
                          [io.Problem(i, [j for j in range(3) if j != i]) for i in range(3)])
    pipeline.write_dense_folder(str(tmp_path), ds, quality=100)
    env = dict(os.environ, PYTHONPATH=os.path.join(os.path.dirname(os.path.dirname(__file__)), "acmmp-spherical_amd"))
    r = subprocess.run([sys.executable, "-m", "acmmp.pipeline", str(tmp_path)], capture_output=True, text=True,
                       env=env, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    summary = json.loads(r.stdout.strip().splitlines()[-1])
    assert summary["fused_points"] > 0
    for v in range(3):
        d = io.read_dmb(str(tmp_path / "ACMMP" / f"2333_{v:08d}" / "depths_geom.dmb"))
        assert d.shape == (128, 256)
        ok = np.abs(d - sc.extra["gt_depths"][v]) < 0.02 * sc.extra["gt_depths"][v]
        assert ok.mean() > 0.5                                   # oracle pipeline: 0.64-0.80 here
    ply = io.read_ply(str(tmp_path / "ACMMP" / "ACMM_model_cuda_5.ply"))
    assert ply.shape[0] == summary["fused_points"]
