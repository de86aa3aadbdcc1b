"""The depth exchange's payload check (pipeline.RcclExchange, bench.depth_exchange): every rank checksums each
map it holds after the grouped broadcast and the ranks compare the checksums, so a wrong root, buffer or
ordering fails the pass.  CPU: the checksum restated in pure Python, and RcclExchange.share driven through a
fake two-rank communicator (threads) that routes one map from the wrong root.  GPU: the device checksum equals
the host one; the diagnostics the bench line carries (device identity, clock probe)."""
import threading

import numpy as np
import pytest

from acmmp import capi, pipeline

MASK = (1 << 64) - 1


def checksum_py(words) -> int:
    """acmmp_device_checksum restated word by word (splitmix64's finaliser of (i << 32) | w_i, summed mod 2^64)."""
    acc = 0
    for i, w in enumerate(words):
        z = ((i << 32) | int(w)) & MASK
        z = ((z ^ (z >> 30)) * 0xbf58476d1ce4e5b9) & MASK
        z = ((z ^ (z >> 27)) * 0x94d049bb133111eb) & MASK
        acc = (acc + (z ^ (z >> 31))) & MASK
    return acc


def test_checksum_host_matches_restatement():
    rng = np.random.default_rng(3)
    for n in (0, 1, 7, 1000):
        a = rng.random(n, dtype=np.float32) * 100
        assert capi.checksum_host(a) == checksum_py(a.view(np.uint32))
    assert capi.checksum_host(np.zeros(0, np.float32)) == 0


def test_checksum_sees_position_and_value():
    a = np.arange(64, dtype=np.float32).reshape(8, 8)
    c = capi.checksum_host(a)
    b = a.copy()
    b[0, 1], b[0, 2] = a[0, 2], a[0, 1]                 # two words swapped
    assert capi.checksum_host(b) != c
    b = a.copy()
    b.view(np.uint32)[5, 5] ^= 1                          # one bit
    assert capi.checksum_host(b) != c
    assert capi.checksum_host(a.copy()) == c


class FakeWorld:
    """In-process stand-in for RCCL: `world` ranks as threads; broadcast copies root buffers, allreduce_max takes
    the element-wise max.  wrong_root = (map index, root to read instead) routes one map wrongly."""

    def __init__(self, world, wrong_root=None):
        self.world, self.wrong_root = world, wrong_root
        self.barrier = threading.Barrier(world)
        self.slots = [None] * world

    def exchange(self, rank, item):
        self.slots[rank] = item
        self.barrier.wait()
        got = list(self.slots)
        self.barrier.wait()
        return got


class FakeComm:
    def __init__(self, w: FakeWorld, rank: int):
        self.w, self.rank, self.nranks = w, rank, w.world

    def after(self, ctx):
        pass

    def broadcast(self, bufs, roots):
        everyone = self.w.exchange(self.rank, [b.data.copy() for b in bufs])
        for i, (b, r) in enumerate(zip(bufs, roots)):
            if self.w.wrong_root is not None and self.w.wrong_root[0] == i:
                r = self.w.wrong_root[1]
            if r != self.rank:
                b.data[...] = everyone[r][i]

    def allreduce_max(self, vals):
        return np.max(np.stack(self.w.exchange(self.rank, np.asarray(vals, np.float64))), axis=0)

    def close(self):
        pass


class FakeBuffer:
    def __init__(self, data):
        self.data = data

    def checksum(self):
        return capi.checksum_host(self.data)


class FakeStore:
    """ViewStore's surface that RcclExchange.share uses: device maps per (key, view), producers, host copies."""

    def __init__(self, rank, owners, shape=(6, 10)):
        self.host, self.dev = {}, {}
        for v, o in owners.items():
            # an owner's map holds its values; every other rank holds garbage until the broadcast
            val = np.full(shape, 100.0 * v + 1, np.float32) if o == rank else np.full(shape, -1.0, np.float32)
            self.dev[("depths", v)] = FakeBuffer(val)
            self.host[("depths", v)] = val.copy()

    def device_map(self, key, v):
        return self.dev[(key, v)]

    def take_producers(self):
        return []


def run_exchange(world, owners, wrong_root=None):
    w = FakeWorld(world, wrong_root)
    out = [None] * world

    def rank_main(r):
        store = FakeStore(r, owners)
        ex = pipeline.RcclExchange(FakeComm(w, r), device=0, verify=True)
        try:
            ex.share("depths", sorted(owners), owners, store)
            out[r] = ("ok", ex.maps_verified, {v: store.dev[("depths", v)].data.copy() for v in owners})
        except pipeline.ExchangeMismatch as e:
            out[r] = ("mismatch", str(e), None)

    ts = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(30)
    assert all(not t.is_alive() for t in ts)
    return out


def test_exchange_verified_when_routed_right():
    owners = {0: 0, 1: 1, 2: 0, 3: 1, 4: 0}
    out = run_exchange(2, owners)
    for status, n, maps in out:
        assert status == "ok" and n == len(owners)
        for v in owners:
            assert np.all(maps[v] == 100.0 * v + 1)


def test_exchange_wrong_root_is_caught():
    owners = {0: 0, 1: 1, 2: 0, 3: 1}
    out = run_exchange(2, owners, wrong_root=(2, 1))     # map index 2 (view 2, owner 0) read from rank 1
    assert all(o[0] == "mismatch" for o in out)
    assert all("views [2]" in o[1] for o in out)


def test_exchange_wrong_root_three_ranks():
    owners = {0: 0, 1: 1, 2: 2, 3: 0, 4: 1, 5: 2}
    assert all(o[0] == "ok" for o in run_exchange(3, owners))
    out = run_exchange(3, owners, wrong_root=(4, 2))
    assert all(o[0] == "mismatch" and "views [4]" in o[1] for o in out)


def test_mismatched_maps_halves():
    """Checksums that agree in one 32-bit half and differ in the other are still caught."""
    class Two:
        def __init__(self, vals):
            self.vals = vals

        def allreduce_max(self, v):
            return np.max(np.stack(self.vals), axis=0)

    a = np.array([0x0000000100000002, 7], np.uint64)
    b = np.array([0x0000000100000003, 7], np.uint64)

    def packed(c):
        hi = (c >> np.uint64(32)).astype(np.float64)
        lo = (c & np.uint64(0xFFFFFFFF)).astype(np.float64)
        return np.concatenate([hi, lo, -hi, -lo])
    comm = Two([packed(a), packed(b)])
    assert pipeline.mismatched_maps(comm, a) == [0]
    assert pipeline.mismatched_maps(Two([packed(a), packed(a)]), a) == []


@pytest.mark.gpu
def test_gpu_device_checksum_and_diagnostics():
    rng = np.random.default_rng(11)
    a = rng.random((123, 457), dtype=np.float32)
    b = capi.DeviceBuffer(0, a.shape)
    try:
        b.upload(a)
        assert b.checksum() == capi.checksum_host(a)
    finally:
        b.free()
    ident = capi.device_identity(0)
    assert len(ident["pci_bus_id"]) >= 7 and len(ident["uuid"]) == 32
    clk = capi.clock_probe(0, warm_ms=200.0)
    assert 0.3 < clk["ghz_min"] <= clk["ghz"] <= clk["ghz_max"] < 3.5, clk
