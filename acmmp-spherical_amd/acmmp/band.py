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
(acmmp_comm_band_exchange).  Both use the engine's own halo row ranges (acmmp_band_halo_ranges).
"""
from __future__ import annotations

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
