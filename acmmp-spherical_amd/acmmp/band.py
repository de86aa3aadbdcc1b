"""Row-band split of one reference view over several GPUs (the optional latency mode).

The reference computes a depth map on one GPU (`RunPatchMatch`, ACMMP.cu:1506-1556).  Here one view's rows are
split into bands, one per context / GPU.  Each band runs the whole `RunPatchMatch` schedule on its rows.  After
every half-sweep it swaps the just-updated colour's plane / cost / selected-view rows within
`Context.BAND_HALO` (23) of its edges with the neighbouring bands.  That is the far reach of the adaptive
neighbour scan, 3 + 2 * 10 rows (ACMMP.cu:971-979).  Every other per-pixel input (initialisation, RNG stream,
images, priors, post-processing) is computed locally on the band plus halo.  So each band's rows equal the
whole-view run's bit for bit.

`run_local` drives several contexts in one process and copies the halos device to device.  `run_rank` is one
rank of a multi-GPU run, with the halo exchange as grouped ncclSend / ncclRecv queued on the engine's stream
(acmmp_comm_band_exchange).  `run_rank_host` is the same rank with the halos through host memory and any
point-to-point transport (`gloo_exchange`: torch.distributed's gloo backend) -- ranks that share a GPU, or have no
device-to-device path.  All use the engine's own halo row ranges (acmmp_band_halo_ranges).
"""
from __future__ import annotations

import numpy as np

HALO = 23


def split_rows(height: int, n: int, halo: int = HALO):
    """n contiguous row bands [lo, hi) covering [0, height), as equal as possible; every band spans at least
    `halo` rows (the exchange reaches one neighbour band only), so n is capped at height // halo."""
    if height <= 0 or n <= 0:
        raise ValueError("height and n must be positive")
    n = max(1, min(n, height // halo)) if height >= halo else 1
    base, extra = divmod(height, n)
    bands, lo = [], 0
    for k in range(n):
        hi = lo + base + (1 if k < extra else 0)
        bands.append((lo, hi))
        lo = hi
    return bands


def run_local(ctxs, seed: int, bands, do_post: bool = True):
    """In-process band run: ctxs[k] (same uploaded problem and params) computes bands[k]; halos are copied
    between neighbouring contexts after every half-sweep.  Afterwards rows bands[k] of ctxs[k]'s outputs are
    final."""
    if len(ctxs) != len(bands):
        raise ValueError("one context per band")
    for ctx, (lo, hi) in zip(ctxs, bands):
        ctx.band_begin(seed, lo, hi)
    while ctxs[0].band_sweeps_left() > 0:
        colours = {ctx.band_sweep() for ctx in ctxs}
        assert len(colours) == 1
        colour = colours.pop()
        ranges = [ctx.band_halo_ranges() for ctx in ctxs]
        for k, ctx in enumerate(ctxs):
            (_, _), (ua, ub), (_, _), (da, db) = ranges[k]
            if ub > ua:
                ctx.band_copy_rows_from(ctxs[k - 1], colour, ua, ub)
            if db > da:
                ctx.band_copy_rows_from(ctxs[k + 1], colour, da, db)
    for ctx in ctxs:
        ctx.band_end(do_post)


def run_rank(ctx, comm, seed: int, height: int, rank: int, world: int):
    """This rank's band of a view split over `world` ranks (one GPU each), RCCL halo exchange.  Returns
    the band (lo, hi) whose rows of ctx's outputs are final."""
    bands = split_rows(height, world)
    if len(bands) != world:
        raise ValueError(f"{height} rows cannot be split into {world} bands of >= {HALO} rows")
    lo, hi = bands[rank]
    ctx.run_patchmatch_band(seed, lo, hi, comm if world > 1 else None,
                            rank - 1 if rank > 0 else -1, rank + 1 if rank < world - 1 else -1)
    return lo, hi


def run_rank_host(ctx, seed: int, height: int, rank: int, world: int, exchange, do_post: bool = True):
    """This rank's band of a view split over `world` ranks, the halo through host buffers: after every half-sweep
    the updated colour's rows within HALO of the band's edges go to the neighbouring ranks
    (acmmp_band_get_rows) and theirs come back (acmmp_band_set_rows).  `exchange(sends, recvs)` moves them:
    sends = [(peer, rows)], recvs = [(peer, n_pixels)] -> the received rows in recvs' order (gloo_exchange).
    Returns the band (lo, hi) whose rows of ctx's outputs are final."""
    bands = split_rows(height, world)
    if len(bands) != world:
        raise ValueError(f"{height} rows cannot be split into {world} bands of >= {HALO} rows")
    lo, hi = bands[rank]
    wh = (ctx.W + 1) // 2
    ctx.band_begin(seed, lo, hi)
    while ctx.band_sweeps_left() > 0:
        colour = ctx.band_sweep()
        (sua, sub), (rua, rub), (sda, sdb), (rda, rdb) = ctx.band_halo_ranges()
        sends, recvs, into = [], [], []
        if rank > 0:
            sends.append((rank - 1, ctx.band_get_rows(colour, sua, sub)))
            recvs.append((rank - 1, (rub - rua) * wh))
            into.append((rua, rub))
        if rank < world - 1:
            sends.append((rank + 1, ctx.band_get_rows(colour, sda, sdb)))
            recvs.append((rank + 1, (rdb - rda) * wh))
            into.append((rda, rdb))
        for (a, b), rows in zip(into, exchange(sends, recvs)):
            ctx.band_set_rows(colour, a, b, rows)
    ctx.band_end(do_post)
    return lo, hi


def gloo_exchange(sends, recvs):
    """`run_rank_host`'s transport over torch.distributed point-to-point (the gloo backend: host tensors only)."""
    import torch
    import torch.distributed as dist
    reqs, bufs = [], []
    for peer, rows in sends:
        reqs.append(dist.isend(torch.from_numpy(np.ascontiguousarray(rows).view(np.int32)), peer))
    for peer, n in recvs:
        t = torch.empty((n, 6), dtype=torch.int32)
        bufs.append(t)
        reqs.append(dist.irecv(t, peer))
    for r in reqs:
        r.wait()
    return [b.numpy().view(np.uint32) for b in bufs]
