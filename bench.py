#!/usr/bin/env python3
"""bench.py -- headline benchmark of the MI355X-native ACMMP-Spherical PatchMatch path.

Metric (BASELINE.json): "Mpixels/sec PatchMatch propagation + ms/depth-map, 2000x1500,
1/2/4/8 GPU".  Workload (SURVEY.md §8d "metric"): one synthetic 2000x1500
equirectangular (SPHERE) reference view with 4 source views, the reference's
RunPatchMatch schedule (random init, 3 x black/red propagation, depth+normal, two
median filters), seed-fixed.  One "step" = one full RunPatchMatch of one reference
view with inputs already resident in HBM; value = pixel-iterations of all ranks /
wall time of the timed region (max over ranks), in Mpixel-iterations/s.

N GPUs = N processes, one per GPU (torch.distributed.run); every rank owns its own
reference view (weak scaling, no data-path collective -- DESIGN.md §7).  Rank
coordination (barrier, max-over-ranks) uses torch.distributed's gloo backend on the
host: the engine's HIP runtime is /opt/rocm's, and initialising torch's bundled HIP
runtime in the same process as well would put two HIP/HSA runtimes in one process.

Extra JSON fields: `roofline` (FP32 compute roof of the propagation kernel, measured
with HIP events on the kernel's stream; HBM traffic from the committed rocprofv3 PMC
pass when one exists for this config) and `cpu_baseline` (the CPU oracle on a bounded
row-band sample of the same view, rank 0, N = 1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "acmmp-spherical_amd"))

import numpy as np  # noqa: E402

from acmmp import capi, scene, types  # noqa: E402

# MI355X peaks (/opt/skills/guides/MI355X_MICROARCH.md, chip-level parameters)
PEAK_FP32_TFLOPS = 157.3        # FP32 vector (= f32-input MFMA) dense peak
PEAK_HBM_GBS = 8000.0

# Algorithmic FLOP per pixel-iteration of CheckerboardPropagation:
# 14 hypotheses x 36 samples x V views x F_HVS + 8.7k shared per-pixel work.
F_HVS = {"sphere": 100.0, "pinhole": 46.0}
F_SHARED = 8700.0


def algorithmic_flop_per_pixel(model: str, V: int, samples: int = 36) -> float:
    return 14 * samples * V * F_HVS[model] + F_SHARED


# k_eval_nb -- the dominant kernel: per pixel of a half-sweep it evaluates the 8 adaptive-neighbour
# hypotheses (ACMMP.cu:964-1144) against every source view (the current plane's costs come from the
# cost cache): 8 x 36 x (V x F_HVS + 15 shared ray-plane/world-point FLOP) + 36 x 30 bilateral weights.
def eval_nb_flop_per_pixel(model: str, V: int, samples: int = 36) -> float:
    return 8 * samples * (V * F_HVS[model] + 15.0) + samples * 30.0


# What the fast SPHERE k_eval_nb executes per hypothesis and view when it interpolates (DESIGN.md §2.4,
# capi.cpp build_kparams' gate): 16 node samples projected in full (ray-plane depth and camera point 15 +
# F_HVS 100 each), the 20 other samples' bilinear fetch + accumulation (19 of F_HVS: SURVEY.md §8d's pinhole
# breakdown) on interpolated coordinates, and the interpolation itself: node unwrap 15 x 5, the 8 Lagrange
# samples of the node columns 8 x 14, columns 1 / 4 at the node rows 16 x 8, their 4 other samples 4 x 14,
# and the 20 samples' seam wrap and clamp 20 x 6 -- 491 FLOP.  Per pixel the 8 hypotheses plus the 36 shared
# bilateral weights.
F_INTERP_VIEW = 16 * (100.0 + 15.0) + 20 * 19.0 + 491.0


def eval_nb_executed_flop_per_pixel(V: int) -> float:
    return 8 * V * F_INTERP_VIEW + 36 * 30.0


# What the fast pinhole k_eval_nb executes per hypothesis-view-sample with the centre-relative homogeneous
# sample points: the point 8 FMA + the perspective reciprocal (16 + 3, in place of SURVEY.md
# §8d's 24 + 3), the row step 1, bilinear 13, accumulation 6 -- 39 of F_HVS's 46; per sample the ray-plane
# dot and the scale step 6 (in place of 15); per hypothesis-view the binary64 centre point and the relative
# rows, ~60.
F_HOMOG_HVS, F_HOMOG_SAMPLE, F_HOMOG_VIEW = 39.0, 6.0, 60.0


def eval_nb_executed_flop_per_pixel_pinhole(V: int, samples: int = 36) -> float:
    return 8 * (samples * (V * F_HOMOG_HVS + F_HOMOG_SAMPLE) + V * F_HOMOG_VIEW) + samples * 30.0


def interp_enabled(width: int, height: int, patch_size: int = 11, radius_increment: int = 2) -> bool:
    """capi.cpp build_kparams' gate (tests/np_interp.interp_enabled)."""
    R = patch_size // 2
    return len(range(-R, R + 1, radius_increment)) == 6 and 2000 * R <= 5 * width and 1000 * R <= 5 * height


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--mode", choices=["patchmatch", "pipeline"], default="patchmatch",
                    help="patchmatch: the headline RunPatchMatch metric; pipeline: the sharded multi-pass schedule")
    ap.add_argument("--views", type=int, default=24, help="pipeline mode: views in the capture")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--width", type=int, default=None, help="default 2000 (pipeline mode: 3200)")
    ap.add_argument("--height", type=int, default=None, help="default 1500 (pipeline mode: 2133)")
    ap.add_argument("--n-src", type=int, default=None, help="default 4 (pipeline mode: 20)")
    ap.add_argument("--model", choices=["sphere", "pinhole"], default=None, help="default sphere (pipeline: pinhole)")
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--math", choices=["exact", "fast"], default="fast",
                    help="engine arithmetic (acmmp_set_math): fast = the reference's --use_fast_math arithmetic "
                         "(tolerance parity, tests/test_gpu_fastmath.py); exact = bit-identical to the oracle")
    ap.add_argument("--no-other-mode", action="store_true", help="skip timing the other math mode beside `value`")
    ap.add_argument("--cpu-seconds", type=float, default=25.0,
                    help="target length of the CPU-baseline sample (the probe rows sit at the equator, the "
                         "slowest rows of the metric view: the sample takes about 55%% of this)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0 -> every host core this process may use (affinity and cgroup quota)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-variant", action="store_true", help="skip the non-degenerate 2000x1000 side measurement")
    ap.add_argument("--no-pipeline", action="store_true", help="skip the end-to-end ProcessProblem schedule timing")
    ap.add_argument("--pmc", default=os.path.join(REPO, "profiles", "pmc_propagate.json"),
                    help="rocprofv3 PMC summary giving HBM bytes per propagation launch")
    ap.add_argument("--timed-only", action="store_true",
                    help="profiling: nothing runs on the GPU after the timed steps (no other math mode, latency, "
                         "PCIe, variant, end-to-end or CPU legs), so a kernel trace's last launches are the timed ones")
    ap.add_argument("--no-clock", action="store_true", help="skip the clock probe after the timed region")
    ap.add_argument("--clock-warm-ms", type=float, default=1500.0,
                    help="clock probe: ms of back-to-back VALU-dense launches before the stamped one")
    ap.add_argument("--allow-shared-gpus", action="store_true",
                    help="rehearsal only: let more ranks than GPUs share devices round-robin (never a scaling point)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch/rendezvous check: ranks join the gloo group, agree on the world and exit without "
                         "touching a GPU (the CPU test of `--gpus N`)")
    a = ap.parse_args()
    if a.timed_only:
        a.no_other_mode = a.no_cpu_baseline = a.no_variant = a.no_pipeline = True
    if a.gpus < 1:
        ap.error("--gpus must be >= 1")
    pipe = a.mode == "pipeline"        # BASELINE.json configs[3] shape vs the headline metric's
    for k, head, pl in (("width", 2000, 3200), ("height", 1500, 2133), ("n_src", 4, 20), ("model", "sphere", "pinhole")):
        if getattr(a, k) is None:
            setattr(a, k, pl if pipe else head)
    return a


def make_scene(args, rank: int):
    if args.model == "sphere":
        return scene.sphere_scene(args.width, args.height, n_src=args.n_src, seed=args.seed + 7919 * rank)
    return scene.pinhole_scene(args.width, args.height, n_src=args.n_src, seed=args.seed + 7919 * rank)


def end_to_end(args, sc, device):
    """main.cpp's whole per-view schedule (multi-scale planar -> geom x2 -> JBU -> hierarchy planar ->
    geom x2) over the bench scene's views, each view a reference in turn, through the host API a
    drop-in caller uses (host images in, depth maps out between passes as the reference does).
    Reported beside `value` as the end-to-end per-view depth-map latency; never `value`."""
    from acmmp import io, pipeline
    n = len(sc.images)
    images = {i: np.asarray(sc.images[i], np.float32) for i in range(n)}
    cams = {i: np.array(sc.cameras[i], copy=True) for i in range(n)}
    problems = []
    for i in range(n):
        pr = io.Problem(i)
        pr.src_image_ids = [j for j in range(n) if j != i]
        problems.append(pr)
    pipe = pipeline.Pipeline(pipeline.Dataset(images, cams, problems), device=device, order="reference",
                             math=args.math)
    t0 = time.perf_counter()
    pipe.run()
    total = time.perf_counter() - t0
    pipe.close()
    d0 = pipe.store.get("depths_geom", 0)
    acc = scene.depth_accuracy(d0, sc.gt_depth) if d0.shape == sc.gt_depth.shape else None
    return {"views": n, "passes": [p.name for p in pipe.passes], "total_s": round(total, 3),
            "ms_per_view": round(total / n * 1e3, 1),
            "ms_per_view_pass": round(total / (n * len(pipe.passes)) * 1e3, 1),
            "math": args.math,
            "stages_s": {k: round(v, 3) for k, v in sorted(pipe.stage_s.items())},
            "frac_within_1pct_gt": None if acc is None else round(float(acc), 4),
            "note": "host wall clock, one GPU; every view's final depth map after all passes"}


def nondegenerate_variant(args, ctx, width=2000, height=1000, steps=3):
    """the metric's 2000x1500 SPHERE view puts ~40% of its pixels in the reference's
    sigma-in-radians band (every cost 2.0, short-circuited here); report the 2:1 equirectangular
    2000x1000 view beside it, where every pixel does NCC work.  Reported, never `value`."""
    sc = scene.sphere_scene(width, height, n_src=args.n_src, seed=args.seed + 1)
    c0 = sc.cameras[0]
    p = types.default_params(num_images=args.n_src + 1, max_iterations=args.iters,
                             depth_min=float(c0["depth_min"]) * 0.6, depth_max=float(c0["depth_max"]) * 1.2)
    ctx.set_params(p)
    ctx.upload_views(sc.images, sc.cameras)
    ctx.run_patchmatch(args.seed + 999)
    ctx.synchronize()
    t0 = time.perf_counter()
    nb_ms = 0.0
    for k in range(steps):
        ctx.run_patchmatch(args.seed + k)
        nb_ms += ctx.last_kernel_timing()["k_eval_nb"][0]
    ctx.synchronize()
    dt = (time.perf_counter() - t0) / steps
    ev, tot = ctx.last_work()
    planes, _ = ctx.download()
    return {"config": f"RunPatchMatch {width}x{height} sphere, 1 ref + {args.n_src} src, {args.iters} iterations",
            "value": round(width * height * args.iters / dt / 1e6, 3), "unit": "Mpixel-iterations/s",
            "ms_per_depth_map": round(dt * 1e3, 3), "k_eval_nb_ms": round(nb_ms / steps / (2 * args.iters), 4),
            "short_circuited_pixel_frac": round(1.0 - ev / max(tot, 1), 4),
            "frac_within_1pct_gt": round(scene.depth_accuracy(planes[..., 3], sc.gt_depth), 4)}


def host_cores():
    """Host cores this process may run on: the affinity mask, capped by a cgroup v2 CPU quota (a GPU
    box shares its machine: os.cpu_count() there is the whole machine, the job's share is smaller)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(-(-int(quota) // int(period)))))
    except (OSError, ValueError):
        pass
    return n


def cpu_baseline(args, sc, params, gpu_rate_check=None):
    """Time the CPU oracle (oracle/, kind "port") on a bounded sample of the same view."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle  # test/baseline infrastructure only

    oracle.build()
    threads = args.cpu_threads or host_cores()
    prob = oracle.Problem(sc.images, sc.cameras, params)
    H = args.height
    # probe: 4 rows to estimate the rate, then bands spread over the image for ~cpu_seconds
    t0 = time.perf_counter()
    oracle.run_band(prob, args.seed, H // 2, H // 2 + 4, nthreads=threads)
    probe = time.perf_counter() - t0
    per_row = probe / 4.0
    total_rows = int(max(8, min(H, args.cpu_seconds / max(per_row, 1e-6))))
    nb = 6
    rows_per_band = max(2, total_rows // nb)
    t_sum, rows_done, bands = 0.0, 0, []
    for b in range(nb):
        if b:
            # the 4-row probe carries a band's fixed halo cost, so it overestimates the per-row time:
            # resize the remaining bands from the rate measured so far to fill the time budget
            left = max(0.0, args.cpu_seconds - t_sum)
            rows_per_band = int(max(2, min(H // nb, left / (nb - b) / (t_sum / rows_done))))
        y0 = int((b + 0.5) * H / nb) - rows_per_band // 2
        y0 = max(0, min(H - rows_per_band, y0))
        t0 = time.perf_counter()
        oracle.run_band(prob, args.seed, y0, y0 + rows_per_band, nthreads=threads)
        t_sum += time.perf_counter() - t0
        rows_done += rows_per_band
        bands.append(rows_per_band)
    pix_iter = rows_done * args.width * args.iters
    rate = pix_iter / t_sum                                  # pixel-iterations per second
    return {
        "value": round(rate / 1e6, 5),
        "unit": "Mpixel-iterations/s",
        # the same rate as time per depth map of the whole view (H x W pixels x iterations), beside the GPU's
        # ms_per_depth_map; the reference itself cannot be built here (nvcc, OpenCV: DESIGN.md §3), so this is
        # its restatement's rate on the box's cores
        "ms_per_depth_map": round(args.width * args.height * args.iters / rate * 1e3, 1),
        "cores": threads,
        "kind": "port",
        "sample": f"{nb} bands of {'/'.join(map(str, bands))} rows of the same {args.width}x{args.height} {args.model} view "
                  f"(V={args.n_src}), full init + {args.iters} iterations + post on those rows, "
                  f"{t_sum:.1f} s CPU wall",
        "seconds": round(t_sum, 2),
        "host": {"nproc": os.cpu_count(), "usable_cores": host_cores(),
                 "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS")},
    }


def guarded(fn, seconds, *a):
    """Run one of the multi-rank extras (first runs of the RCCL paths on a multi-GPU node) with a deadline:
    its failure or hang must not cost the headline line.  Returns (result, abandoned); abandoned = a
    worker thread may still be blocked in a collective, so the process must exit without tearing down."""
    import threading
    box = {}

    def run():
        try:
            box["r"] = fn(*a)
        except Exception as e:                               # noqa: BLE001 -- reported in the line
            box["r"] = {"error": f"{type(e).__name__}: {e}"}
    t = threading.Thread(target=run, daemon=True)
    t.start()
    t.join(seconds)
    if t.is_alive():
        return {"error": f"no result within {seconds} s (abandoned)"}, True
    return box["r"], False


EXIT_ABANDONED = 3


def leave_abandoned():
    """A multi-rank extra was abandoned at its deadline and a worker thread may still be blocked inside a
    collective: leave without tearing down the process group or the context it uses, and with a non-zero
    status, so a hung first RCCL run never reads as success (the headline line is already out; every rank
    reaches this at the same deadline)."""
    sys.stdout.flush()
    sys.stderr.flush()
    os._exit(EXIT_ABANDONED)


def depth_exchange(args, ctx, rank, world, device, dist, allmax, reps=5):
    """Every rank broadcasts its last depth map (W x H float32, acmmp_export_depth: HBM to HBM) to all
    ranks in one grouped RCCL call -- what pipeline.RcclExchange does between two passes.  The RCCL
    unique id travels over the bench's gloo group.  Returns timing and bandwidth (max over ranks), or
    the error text: this side measurement never fails the bench."""
    try:
        uid = [capi.Comm.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        comm = capi.Comm(device, uid[0], world, rank)
        bufs = [capi.DeviceBuffer(device, (args.height, args.width)) for _ in range(world)]
        ctx.export_depth(bufs[rank])
        ctx.synchronize()
        own = bufs[rank].checksum()                                  # the owner's map before the broadcast
        comm.after(ctx)                                              # the broadcast waits for the export
        comm.broadcast(bufs, list(range(world)))                     # warm-up
        ok = all(np.isfinite(b.download()).mean() > 0.5 for b in bufs)
        # every received map bit for bit against its owner's: each rank's checksum of every buffer after the
        # broadcast (acmmp_device_checksum) and each owner's from before it, gathered over the gloo group
        # (a wrong root / buffer / order in the grouped broadcast shows here, a wrong root included: it
        # overwrites the owner's buffer as well)
        got = [None] * world
        dist.all_gather_object(got, {"own": own, "after": [b.checksum() for b in bufs]})
        identical = all(g["after"][r] == got[r]["own"] for g in got for r in range(world))
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            comm.broadcast(bufs, list(range(world)))
        dt = allmax((time.perf_counter() - t0) / reps)
        comm.close()
        for b in bufs:
            b.free()
        nbytes = 4 * args.width * args.height
        return {"ms_per_exchange": round(dt * 1e3, 3), "maps": world, "MB_per_map": round(nbytes / 1e6, 2),
                "received_GBps_per_rank": round(nbytes * (world - 1) / dt / 1e9, 2), "maps_finite": bool(ok),
                "maps_bit_identical": bool(identical), "map_checksums": [f"{g['own']:016x}" for g in got],
                "transport": "RCCL grouped ncclBroadcast over xGMI (acmmp_comm_broadcast)"}
    except Exception as e:                                           # noqa: BLE001
        return {"error": f"{type(e).__name__}: {e}"}


def band_split(args, rank, world, device, dist, allmax, reps=5):
    """SURVEY.md §8e latency mode: the metric view (rank 0's scene on every rank) split into `world` row
    bands, one per GPU, RunPatchMatch on each band with the 23-row halo swapped over RCCL after every
    half-sweep (acmmp/band.py, acmmp_run_patchmatch_band).  Reports ms per depth map (band run + D2H of
    the band's rows, max over ranks) against the same view on one GPU, and whether every band's rows
    equal that whole-view run bit for bit.  A side measurement: never fails the bench."""
    from acmmp import band
    ctx = comm = None
    try:
        sc = make_scene(args, 0)
        c0 = sc.cameras[0]
        params = types.default_params(num_images=args.n_src + 1, max_iterations=args.iters,
                                      depth_min=float(c0["depth_min"]) * 0.6, depth_max=float(c0["depth_max"]) * 1.2)
        ctx = capi.Context(device)
        ctx.set_math(args.math)
        ctx.set_params(params)
        ctx.upload_views(sc.images, sc.cameras)
        uid = [capi.Comm.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        comm = capi.Comm(device, uid[0], world, rank)
        seed = args.seed + 900
        ctx.run_patchmatch(seed)                                     # whole view on this GPU (reference)
        whole_p, whole_c = ctx.download()
        t1 = []
        for _ in range(reps):
            t0 = time.perf_counter()
            ctx.run_patchmatch(seed)
            ctx.download_into(whole_p, whole_c)
            t1.append(time.perf_counter() - t0)
        one_gpu_ms = allmax(float(np.median(t1))) * 1e3
        lo, hi = band.run_rank(ctx, comm, seed, args.height, rank, world)     # warm-up + check
        bp = np.empty((hi - lo, args.width, 4), np.float32)
        bc = np.empty((hi - lo, args.width), np.float32)
        ctx.download_rows_into(bp, bc, lo, hi)
        same = (np.array_equal(bp.view(np.uint32), whole_p[lo:hi].view(np.uint32)) and
                np.array_equal(bc.view(np.uint32), whole_c[lo:hi].view(np.uint32)))
        same_all = allmax(0.0 if same else 1.0) == 0.0
        tb = []
        for _ in range(reps):
            dist.barrier()
            t0 = time.perf_counter()
            band.run_rank(ctx, comm, seed, args.height, rank, world)
            ctx.download_rows_into(bp, bc, lo, hi)
            tb.append(allmax(time.perf_counter() - t0))
        ms = float(np.median(tb)) * 1e3
        return {"ranks": world, "bands": band.split_rows(args.height, world), "halo_rows": band.HALO,
                "ms_per_depth_map": round(ms, 3), "one_gpu_ms_per_depth_map": round(one_gpu_ms, 3),
                "speedup": round(one_gpu_ms / ms, 3), "bit_identical_to_whole_view": bool(same_all),
                "exchanges_per_map": 2 * args.iters,
                "transport": "RCCL grouped ncclSend/ncclRecv on the engine stream (acmmp_comm_band_exchange)",
                "note": "one view split by rows over the GPUs; each rank downloads its own rows"}
    except Exception as e:                                           # noqa: BLE001
        return {"error": f"{type(e).__name__}: {e}"}
    finally:
        if comm is not None:
            comm.close()
        if ctx is not None:
            ctx.close()


def pipeline_mode(args, rank, world, local_rank, barrier, allmax):
    """`--mode pipeline`: main.cpp's multi-scale ProcessProblem schedule (planar -> geom -> geom-multi,
    JBU, hierarchy planar -> geom -> geom-multi) over a synthetic multi-view capture in the ETH3D-style
    shape of BASELINE.json configs[3] (pinhole, ~20 sources per view, planar prior + multi-scale),
    reference views sharded over the ranks (one GPU each), the depth maps of every pass exchanged
    HBM-to-HBM over RCCL (pipeline.RcclExchange) before the next.  One JSON line: views/s of the
    whole job, per-pass compute and exchange wall time (max over ranks), host stage totals."""
    from acmmp import io, pipeline
    ndev = capi.device_count()
    if world > 1 and ndev and world > ndev:
        raise SystemExit(f"bench --mode pipeline: {world} ranks on {ndev} GPU(s); RCCL needs one GPU per rank")
    device = local_rank % ndev if ndev else local_rank
    make = scene.pinhole_scene if args.model == "pinhole" else scene.sphere_scene
    t_scene = time.perf_counter()
    sc = make(args.width, args.height, n_src=args.views - 1, seed=args.seed)
    scene_s = time.perf_counter() - t_scene
    centres = np.array([-(np.asarray(c["R"], np.float64).reshape(3, 3).T @ np.asarray(c["t"], np.float64))
                        for c in sc.cameras])
    problems = []
    for i in range(args.views):
        pr = io.Problem(i)
        others = sorted((j for j in range(args.views) if j != i),
                        key=lambda j: (float(np.linalg.norm(centres[j] - centres[i])), j))
        pr.src_image_ids = others[:args.n_src]
        problems.append(pr)
    ds = pipeline.Dataset({i: np.asarray(sc.images[i], np.float32) for i in range(args.views)},
                          {i: np.array(sc.cameras[i], copy=True) for i in range(args.views)}, problems)
    exchange = pipeline.rcclexchange_from_env(device) if world > 1 else pipeline.LocalExchange()
    pipe = pipeline.Pipeline(ds, exchange=exchange, device=device, seed=args.seed,
                             order="snapshot" if world > 1 else "reference", math=args.math)
    barrier()
    t0 = time.perf_counter()
    pipe.run()
    pipe.engine.synchronize()
    elapsed = time.perf_counter() - t0
    t_max = allmax(elapsed)
    passes = [{"name": p.name, "compute_ms": round(allmax(p.compute_s) * 1e3, 1),
               "exchange_ms": round(allmax(p.exchange_s) * 1e3, 2),
               "exchange_MB": round(p.exchange_bytes / 1e6, 1)} for p in pipe.passes]
    acc = [scene.depth_accuracy(pipe.store.get("depths_geom", v), sc.gt_depth)
           for v in [0] if pipe.owner(0) == rank]
    stages = {k: round(allmax(v), 3) for k, v in sorted(pipe.stage_s.items())}
    n_gpus = min(world, ndev) if ndev else world
    line = {
        "metric": "ProcessProblem schedule throughput (views/s), sharded views + RCCL depth exchange",
        "value": round(args.views / t_max, 4), "unit": "views/s", "n_gpus": n_gpus, "ranks": world,
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32", "math": args.math,
        "data": f"synthetic ({args.model.upper()} ring rig, ray-cast textured scene; no dataset reachable)",
        "config": {"workload": f"{args.views} views {args.width}x{args.height} {args.model}, {args.n_src} sources "
                               f"each (nearest centres), planar prior + multi-scale (main.cpp schedule)",
                   "views": args.views, "width": args.width, "height": args.height, "n_src": args.n_src,
                   "model": args.model, "parallelism": f"views-sharded x{world}, RCCL depth exchange"},
        "total_s": round(t_max, 3), "ms_per_view": round(t_max / args.views * 1e3, 1),
        "passes": passes, "stages_s": stages,
        "exchange": "pipeline.RcclExchange (grouped ncclBroadcast, HBM to HBM)" if world > 1 else
                    "none: one rank holds every view (no scaling curve from this run)",
        "maps_verified": getattr(exchange, "maps_verified", None),
        "scene_s": round(scene_s, 1),
        "quality": {"view0_frac_within_1pct_gt": round(float(acc[0]), 4) if acc else None},
    }
    exchange.close()
    pipe.close()
    return line


def visible_gpus() -> int:
    """GPUs this process could use, counted without any HIP call: the KFD topology's GPU nodes (a node
    with a non-zero gfx_target_version; CPU nodes report 0), limited by the visibility variables the HIP
    runtime honours.  The launcher parent must stay free of HIP state, since it starts the ranks."""
    root = "/sys/class/kfd/kfd/topology/nodes"
    n = 0
    try:
        for node in sorted(os.listdir(root)):
            try:
                with open(os.path.join(root, node, "properties")) as fh:
                    props = dict(ln.split(None, 1) for ln in fh if len(ln.split(None, 1)) == 2)
            except OSError:
                continue
            if int(props.get("gfx_target_version", "0").strip() or 0) != 0:
                n += 1
    except OSError:
        return 0
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([t for t in v.split(",") if t.strip() != ""]))
    return n


def launch_ranks(args) -> int:
    """`bench.py --gpus N` run directly (WORLD_SIZE unset, N > 1): start N ranks, one per GPU, as a
    torch.distributed.run child process with the same arguments (rendezvous on 127.0.0.1, a free port),
    wait for it and return its exit code.  Rank 0's JSON line reaches our stdout unchanged.  The parent
    initialises nothing on a GPU and never execs."""
    import socket
    import subprocess
    if not args.dry_run and not args.allow_shared_gpus:
        ndev = visible_gpus()
        if ndev < args.gpus:
            print(f"bench: --gpus {args.gpus} but {ndev} GPU(s) visible; refusing to put several ranks on one "
                  f"GPU (--allow-shared-gpus for a rehearsal)", file=sys.stderr)
            return 2
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", str(max(1, host_cores() // args.gpus)))
    return subprocess.run(cmd, env=env).returncode


def dist_setup(args):
    """(rank, world, local_rank, dist) of this process; checks the launcher agrees with --gpus."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if "WORLD_SIZE" in os.environ and args.gpus not in (1, world):
        raise SystemExit(f"bench: --gpus {args.gpus} but the launcher started {world} rank(s)")
    dist = None
    if world > 1:
        import torch.distributed as dist  # noqa: F811
        dist.init_process_group("gloo")
    return rank, world, local_rank, dist


def dry_run(args, rank, world, dist):
    """--dry-run: every rank reports in over the gloo group; rank 0 prints who came."""
    ranks = [rank]
    if dist is not None:
        got = [None] * world
        dist.all_gather_object(got, {"rank": rank, "pid": os.getpid(),
                                     "local_rank": int(os.environ.get("LOCAL_RANK", "0"))})
        ranks = sorted(g["rank"] for g in got)
        pids = sorted({g["pid"] for g in got})
    else:
        pids = [os.getpid()]
    # ACMMP_BENCH_SELFTEST_ABANDON=1: a guarded extra that hangs past its deadline, left through the same
    # exit path as main()'s (tests/test_bench_launch.py)
    selftest = os.environ.get("ACMMP_BENCH_SELFTEST_ABANDON") == "1"
    extra, abandoned = guarded(time.sleep, 0.5, 30) if selftest else (None, False)
    if rank == 0:
        print(json.dumps({"dry_run": True, "ranks": world, "rank_ids": ranks, "processes": len(pids),
                          "backend": dist.get_backend() if dist is not None else None, "gpus": args.gpus,
                          "extra": extra}), flush=True)
    if abandoned:
        leave_abandoned()
    if dist is not None:
        dist.destroy_process_group()


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    if args.mode == "pipeline":
        return main_pipeline(args)
    rank, world, local_rank, dist = dist_setup(args)
    if args.dry_run:
        return dry_run(args, rank, world, dist)

    def barrier():
        if dist is not None:
            dist.barrier()

    def allmax(x: float) -> float:
        if dist is None:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    sc = make_scene(args, rank)
    c0 = sc.cameras[0]
    params = types.default_params(num_images=args.n_src + 1, max_iterations=args.iters,
                                  depth_min=float(c0["depth_min"]) * 0.6, depth_max=float(c0["depth_max"]) * 1.2)
    # one GPU per rank; more ranks than GPUs only as an explicit rehearsal (--allow-shared-gpus)
    ndev = capi.device_count()
    if world > max(ndev, 1) and not args.allow_shared_gpus:
        raise SystemExit(f"bench: {world} ranks but {ndev} GPU(s) visible; one GPU per rank "
                         f"(--allow-shared-gpus for a rehearsal)")
    ctx = capi.Context(local_rank % ndev if ndev else local_rank)
    ctx.set_math(args.math)
    ctx.set_params(params)
    ctx.upload_views(sc.images, sc.cameras)

    for w in range(args.warmup):
        ctx.run_patchmatch(args.seed + 100 + w)
    ctx.synchronize()
    barrier()
    ctx.synchronize()
    t0 = time.perf_counter()
    stage = np.zeros(3)
    kern = {k: [0.0, 0] for k in capi.Context.KERNELS}
    work = [0, 0]                        # k_eval_nb pixels evaluated / processed (SPHERE short-circuit)
    for k in range(args.steps):
        ctx.run_patchmatch(args.seed + k)
        tm = ctx.last_timing()
        stage += [tm["init_ms"], tm["prop_ms"], tm["post_ms"]]
        for name, (ms, n) in ctx.last_kernel_timing().items():
            kern[name][0] += ms
            kern[name][1] += n
        ev, tot = ctx.last_work()
        work[0] += ev
        work[1] += tot
    ctx.synchronize()
    barrier()
    ctx.synchronize()
    elapsed = time.perf_counter() - t0
    t_max = allmax(elapsed)

    # which GPU, and the clock it holds under a VALU-dense load right after the timed region (the chip's DVFS
    # give-back differs from device to device, MI355X_MICROARCH.md; k_eval_nb's time follows that clock):
    # reported so two records of the same build on different boxes can be put side by side per GHz
    dev = local_rank % ndev if ndev else local_rank
    ident = clk = None
    try:
        ident = capi.device_identity(dev)
    except capi.AcmmpError as e:
        ident = {"error": str(e)}
    if not args.no_clock:
        try:
            clk = capi.clock_probe(dev, warm_ms=args.clock_warm_ms)
        except capi.AcmmpError as e:
            clk = {"error": str(e)}
    if dist is not None:
        got = [None] * world
        dist.all_gather_object(got, {"rank": rank, "device": ident, "clock": clk})
        ranks_hw = got
    else:
        ranks_hw = None

    # the other math mode on the same resident inputs (reported beside `value`, never `value`)
    other = None
    if not args.no_other_mode:
        om = "exact" if args.math == "fast" else "fast"
        ctx.set_math(om)
        ctx.run_patchmatch(args.seed + 500)
        ctx.synchronize()
        barrier()
        t_o = time.perf_counter()
        o_nb = [0.0, 0, 0]
        for k in range(args.steps):
            ctx.run_patchmatch(args.seed + k)
            ms, n = ctx.last_kernel_timing()["k_eval_nb"]
            o_nb[0] += ms
            o_nb[1] += n
            o_nb[2] += ctx.last_work()[0]
        ctx.synchronize()
        barrier()
        el_o = allmax(time.perf_counter() - t_o)
        o_launch = o_nb[0] / max(o_nb[1], 1)
        o_flop = eval_nb_flop_per_pixel(args.model, args.n_src) * o_nb[2] / max(o_nb[1], 1)
        o_tf = o_flop / (o_launch * 1e-3) / 1e12
        other = {"math": om, "value": round(args.width * args.height * args.iters * args.steps * world / el_o / 1e6, 3),
                 "ms_per_step": round(el_o / args.steps * 1e3, 3),
                 "roofline": {"kernel": "k_eval_nb", "bound": "valu", "launch_ms": round(o_launch, 4),
                              "launches": o_nb[1], "flop_per_launch": o_flop, "achieved": round(o_tf, 3),
                              "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s", "frac": round(o_tf / PEAK_FP32_TFLOPS, 4),
                              "note": "every sample projected in this mode: algorithmic = executed"},
                 "note": "exact = bit-identical to the CPU oracle; fast = tolerance parity (DESIGN.md §2.4)"}
        ctx.set_math(args.math)

    planes, costs = ctx.download()
    d2h_ms = pcie_ms = None
    if not args.timed_only:
        # per-map latency as the reference's RunPatchMatch ends (ACMMP.cu:1553-1554): run + D2H of planes
        # and costs into caller-owned host buffers (inputs resident, as for `value`)
        lat = []
        for k in range(3):
            t1 = time.perf_counter()
            ctx.run_patchmatch(args.seed + k)
            ctx.download_into(planes, costs)
            lat.append(time.perf_counter() - t1)
        d2h_ms = float(np.median(lat)) * 1e3
        # PCIe-inclusive rate (not `value`): host images in, RunPatchMatch, planes + costs back to the host --
        # what a caller that hands over host buffers sees per depth map
        t1 = time.perf_counter()
        ctx.upload_views(sc.images, sc.cameras)
        ctx.run_patchmatch(args.seed)
        planes, costs = ctx.download()
        pcie_ms = (time.perf_counter() - t1) * 1e3
    nan_frac = float(np.isnan(costs).mean())
    acc = scene.depth_accuracy(planes[..., 3], sc.gt_depth)

    P = args.width * args.height
    units = P * args.iters * args.steps * world
    # distinct GPUs (ranks beyond the device count share GPUs on a rehearsal box: flagged, never counted)
    n_gpus = min(world, ndev) if ndev else world
    if world > n_gpus and rank == 0:
        print(f"bench: {world} ranks on {n_gpus} GPU(s) -- a rehearsal, not a scaling point", file=sys.stderr)
    value = units / t_max / 1e6
    ms_per_step = t_max / args.steps * 1e3

    # roofline of the dominant kernel (k_eval_nb): mean launch duration from the HIP events the engine
    # records around every half-sweep kernel on its own stream
    nb_ms, nb_n = kern["k_eval_nb"]
    launch_ms = nb_ms / max(nb_n, 1)
    rows = min(args.height, 32 * (((args.height // 2) + 15) // 16))
    # algorithmic work = pixels whose NCCs are evaluated; SPHERE pixels whose patch weight sum is
    # < 1e-6 have every cost = 2.0 without evaluating a sample (ACMMP.cu:501-503) and are not counted
    pix_per_launch = work[0] / max(nb_n, 1)
    flop_launch = eval_nb_flop_per_pixel(args.model, args.n_src) * pix_per_launch
    achieved = flop_launch / (launch_ms * 1e-3) / 1e12
    traffic = None
    hbm = None
    if os.path.exists(args.pmc):
        try:
            pm = json.load(open(args.pmc))
            if pm.get("config") == {"width": args.width, "height": args.height, "n_src": args.n_src,
                                    "model": args.model, "math": args.math}:
                traffic = pm.get("kernels", {}).get("k_eval_nb", {}).get("hbm_bytes_per_launch")
                if traffic:
                    gbs = traffic / (launch_ms * 1e-3) / 1e9
                    hbm = {"achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                           "frac": round(gbs / PEAK_HBM_GBS, 4), "source": os.path.relpath(args.pmc, REPO)}
        except (OSError, ValueError, AttributeError):
            pass
    # the fast SPHERE instance projects 16 of the 36 samples per hypothesis and view and interpolates the
    # rest: `frac` prices the algorithmic work it replaces, `executed` what it performs
    executed = None
    if args.math == "fast" and args.model == "sphere" and interp_enabled(args.width, args.height):
        ex_flop = eval_nb_executed_flop_per_pixel(args.n_src) * pix_per_launch
        ex_tf = ex_flop / (launch_ms * 1e-3) / 1e12
        executed = {"flop_per_launch": ex_flop, "achieved": round(ex_tf, 3), "frac": round(ex_tf / PEAK_FP32_TFLOPS, 4),
                    "note": "16 projected + 20 interpolated samples per hypothesis-view (bench.F_INTERP_VIEW)"}
    elif args.math == "fast" and args.model == "pinhole" and os.environ.get("ACMMP_PIN_HOMOG", "1") != "0":
        ex_flop = eval_nb_executed_flop_per_pixel_pinhole(args.n_src) * pix_per_launch
        ex_tf = ex_flop / (launch_ms * 1e-3) / 1e12
        executed = {"flop_per_launch": ex_flop, "achieved": round(ex_tf, 3), "frac": round(ex_tf / PEAK_FP32_TFLOPS, 4),
                    "note": "centre-relative homogeneous sample points (bench.F_HOMOG_*)"}
    roofline = {
        "bound": "valu",
        "achieved": round(achieved, 3),
        "peak": PEAK_FP32_TFLOPS,
        "unit": "TFLOP/s",
        "frac": round(achieved / PEAK_FP32_TFLOPS, 4),
        "traffic": traffic,
        "kernel": "k_eval_nb (the 8 neighbour hypotheses of a CheckerboardPropagation half-sweep)",
        "launch_ms": round(launch_ms, 4),
        # launch time in cycles of the probed clock: comparable across boxes whose clocks differ
        "launch_mcycles_at_probe_clock": (round(launch_ms * clk["ghz"], 4) if clk and clk.get("ghz") else None),
        "launches": nb_n,
        "flop_per_launch": flop_launch,
        "evaluated_pixels_per_launch": round(pix_per_launch),
        "short_circuited_pixel_frac": round(1.0 - work[0] / max(work[1], 1), 4),
        "hbm": hbm,
        "executed": executed,
        "half_sweep_kernels_ms": {k: round(v[0] / v[1], 4) for k, v in kern.items() if v[1]},  # k_eval_nb; all four
        # with ACMMP_KERNEL_TIMING=all
        "half_sweep_reference_flop_tflops": round(algorithmic_flop_per_pixel(args.model, args.n_src) *
                                                  pix_per_launch / (stage[1] / max(nb_n, 1) * 1e-3) / 1e12, 3),
        "note": "FP32 vector peak (equal to the f32 MFMA dense peak); the path has no GEMM-shaped work",
    }

    # the pipeline's one exchange step: after a pass every rank's depth map reaches every
    # other rank -- a grouped RCCL broadcast of each rank's map, HBM to HBM, outside the timed region
    # (each under a deadline: a failed or hung first run of an RCCL path reports itself in the line)
    exch = None
    abandoned = False
    deadline = float(os.environ.get("ACMMP_BENCH_EXTRA_S", "180"))
    if world > 1 and ndev and world <= ndev and not args.timed_only and os.environ.get("ACMMP_BENCH_EXCHANGE", "1") != "0":
        exch, abandoned = guarded(depth_exchange, deadline, args, ctx, rank, world, local_rank % ndev, dist, allmax)
    # the single-view latency mode: one view's rows split over the GPUs
    bsplit = None
    if (world > 1 and ndev and world <= ndev and not args.timed_only and not abandoned
            and os.environ.get("ACMMP_BENCH_BAND", "1") != "0"):
        bsplit, abandoned = guarded(band_split, deadline, args, rank, world, local_rank % ndev, dist, allmax)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, sc, params)
    variant = None
    if rank == 0 and world == 1 and args.model == "sphere" and not args.no_variant:
        variant = nondegenerate_variant(args, ctx)

    e2e = None
    if rank == 0 and world == 1 and not args.no_pipeline:
        e2e = end_to_end(args, sc, local_rank % ndev if ndev else local_rank)

    if rank == 0:
        line = {
            "metric": "Mpixels/sec PatchMatch propagation + ms/depth-map, 2000x1500, 1/2/4/8 GPU",
            "value": round(value, 3),
            "unit": "Mpixel-iterations/s",
            "n_gpus": n_gpus,
            "ranks": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "ms_per_depth_map": None if d2h_ms is None else round(d2h_ms, 3),
            "ms_per_depth_map_note": "one RunPatchMatch incl. the D2H of planes + costs (ACMMP.cu:1553-1554), "
                                     "inputs resident; ms_per_step is the same without the D2H",
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "math": args.math,
            "other_math_mode": other,
            "data": f"synthetic (ray-cast textured box room, {args.model.upper()} cameras; no dataset reachable)",
            "config": {"workload": f"RunPatchMatch {args.width}x{args.height} {args.model}, 1 ref + {args.n_src} src, "
                                   f"{args.iters} iterations, random init, per-GPU reference view",
                       "width": args.width, "height": args.height, "n_src": args.n_src, "model": args.model,
                       "iterations": args.iters, "parallelism": f"views-sharded x{world}"},
            "stages_ms": {"init": round(stage[0] / args.steps, 3), "propagation": round(stage[1] / args.steps, 3),
                          "post": round(stage[2] / args.steps, 3)},
            "prop_only_mpix_per_s": round(P * args.iters * world / (stage[1] / args.steps * 1e-3) / 1e6, 3),
            "pcie_inclusive": None if pcie_ms is None else {
                "ms_per_depth_map": round(pcie_ms, 3), "mpix_iter_per_s": round(P * args.iters / (pcie_ms * 1e-3) / 1e6, 3),
                "note": "one rank: upload_views + run_patchmatch + download, host wall clock"},
            "quality": {"frac_within_1pct_gt": round(acc, 4), "nan_cost_frac": round(nan_frac, 4)},
            "roofline": roofline,
            "device": ident,
            "clock": None if clk is None else dict(clk, note=(
                "acmmp_clock_probe right after the timed region: median over workgroups of shader cycles / 100 MHz "
                "ticks around a VALU-dense loop on random operands, after warm_ms of such launches")),
            "value_per_ghz": (round(value / clk["ghz"], 3) if clk and clk.get("ghz") and ranks_hw is None else
                              (round(value / float(np.mean([r["clock"]["ghz"] for r in ranks_hw])), 3)
                               if ranks_hw and all(r["clock"] and r["clock"].get("ghz") for r in ranks_hw) else None)),
            "ranks_hw": ranks_hw,
            "cpu_baseline": cpu,
            "nondegenerate_variant": variant,
            "end_to_end": e2e,
            "depth_exchange": exch,
            "band_split": bsplit,
        }
        print(json.dumps(line), flush=True)
    if abandoned:
        leave_abandoned()
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


def main_pipeline(args):
    rank, world, local_rank, dist = dist_setup(args)
    if args.dry_run:
        return dry_run(args, rank, world, dist)

    def barrier():
        if dist is not None:
            dist.barrier()

    def allmax(x: float) -> float:
        if dist is None:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    line = pipeline_mode(args, rank, world, local_rank, barrier, allmax)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
