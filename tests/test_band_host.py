"""The host transport of the row-band split (acmmp/band.py run_rank_host + gloo_exchange), on the CPU: world-2 and
world-3 gloo runs of a stand-in context whose half-sweep reads its neighbours' rows within the halo the way
CheckerboardPropagation does (ACMMP.cu:971-979: up to 23 rows away), against the same stand-in over the whole
view.  Covers the exchange's ranges, order and pairing; the engine's own bands are tests/test_gpu_band.py."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from acmmp import band

H, W, SWEEPS = 97, 30, 6


class FakeBandCtx:
    """acmmp_band_* semantics on a toy state: colour c's rows hold 6 words per colour-grid pixel; a half-sweep of
    colour c rewrites the band's rows of c from both colours' rows within HALO (wrapping sums mod 2^32), so any
    stale halo row changes the result."""

    def __init__(self):
        self.W = W
        wh = (W + 1) // 2
        rng = np.random.default_rng(7)
        self.init = rng.integers(0, 2**32, (2, H, wh, 6), dtype=np.uint64).astype(np.uint32)

    def band_begin(self, seed, lo, hi):
        self.lo, self.hi, self.sw = lo, hi, 0
        self.state = self.init.copy()

    def band_sweeps_left(self):
        return SWEEPS - self.sw

    def band_sweep(self):
        colour = self.sw & 1
        old = self.state.astype(np.uint64)
        for r in range(self.lo, self.hi):
            a, b = max(0, r - band.HALO), min(H, r + band.HALO + 1)
            acc = (old[colour, a:b].sum(0) * 3 + old[1 - colour, a:b].sum(0) + r + self.sw) % (1 << 32)
            self.state[colour, r] = acc.astype(np.uint32)
        self.sw += 1
        return colour

    def band_halo_ranges(self):
        h, lo, hi = band.HALO, self.lo, self.hi
        up = ((lo, min(lo + h, hi)), (max(0, lo - h), lo)) if lo > 0 else ((0, 0), (0, 0))
        dn = ((max(lo, hi - h), hi), (hi, min(hi + h, H))) if hi < H else ((0, 0), (0, 0))
        return up[0], up[1], dn[0], dn[1]

    def band_get_rows(self, colour, a, b):
        return self.state[colour, a:b].reshape(-1, 6).copy()

    def band_set_rows(self, colour, a, b, rows):
        self.state[colour, a:b] = np.asarray(rows, np.uint32).reshape(b - a, -1, 6)

    def band_end(self, do_post):
        pass


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, out_dir):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        ctx = FakeBandCtx()
        lo, hi = band.run_rank_host(ctx, 0, H, rank, world, band.gloo_exchange)
        np.save(os.path.join(out_dir, f"rank{rank}.npy"), ctx.state[:, lo:hi])
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_host_band_exchange_equals_whole_view(tmp_path, world):
    whole = FakeBandCtx()
    whole.band_begin(0, 0, H)
    while whole.band_sweeps_left():
        whole.band_sweep()
    mp.spawn(_rank, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for rank, (lo, hi) in enumerate(band.split_rows(H, world)):
        got = np.load(tmp_path / f"rank{rank}.npy")
        np.testing.assert_array_equal(got, whole.state[:, lo:hi])
