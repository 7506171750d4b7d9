"""Multi-process DM sharding on CPU (gloo, world_size 2-4, uneven shards and ranks with no
trials): the shard split, the filterbank
broadcast and the statistics all-gather reproduce the single-process search exactly.
The per-shard compute is the oracle here (no GPU on this host); on GPUs it is the HIP search."""
import os
import socket
import subprocess
import sys
import textwrap

import numpy as np
import pytest

from conftest import PKG_DIR, REPO
from pulsarutils.parallel import shard_bounds


@pytest.mark.parametrize("ndm,world", [(1000, 8), (5000, 8), (7, 2), (3, 4), (1, 2)])
def test_shard_bounds_cover(ndm, world):
    spans = [shard_bounds(ndm, world, r) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == ndm
    for (a, b), (c, d) in zip(spans, spans[1:]):
        assert b == c
    sizes = [b - a for a, b in spans]
    assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


WORKER = textwrap.dedent("""
    import os, sys
    sys.path[:0] = [{pkg!r}, {repo!r}]
    import numpy as np, torch, torch.distributed as dist
    import oracle
    from pulsarutils import simulate
    from pulsarutils.parallel import sharded_search
    dist.init_process_group("gloo")
    rank = dist.get_rank()
    np.random.seed(0)
    arr, h = simulate.simulate_test_data(150)
    data = torch.from_numpy(arr.copy()) if rank == 0 else torch.zeros(arr.shape, dtype=torch.float64)
    dms = np.linspace(100, 200, {ndm})
    def compute(d, t):
        return oracle.search(d.numpy(), t, h["fbottom"], h["bandwidth"], h["tsamp"], nthreads=1)
    mx, sd, snr, win = sharded_search(data, dms, arr.shape[0], h["fbottom"], h["bandwidth"], h["tsamp"],
                                      compute=compute, collective={collective!r})
    ref = oracle.search(arr, dms, h["fbottom"], h["bandwidth"], h["tsamp"], nthreads=1)
    assert np.array_equal(data.numpy(), arr)
    for a, b in zip((mx, sd, snr, win), ref):
        assert np.array_equal(a, b), (a[:4], b[:4])
    assert win.dtype == np.int32
    dist.barrier()
    dist.destroy_process_group()
    print("rank", rank, "ok")
""")


@pytest.mark.parametrize("world,ndm,collective", [(2, 37, "broadcast"), (2, 3, "scatter_allgather"),
                                                   (3, 37, "scatter_allgather"), (3, 2, "broadcast"),
                                                   (4, 38, "scatter_allgather"), (4, 3, "broadcast")])
def test_sharded_search_gloo(tmp_path, world, ndm, collective):
    """Both filterbank exchanges (broadcast; scatter + all-gather, with a tail padded to a
    multiple of world at world 3) give every rank the source's data and the single-process
    result."""
    script = tmp_path / "worker.py"
    script.write_text(WORKER.format(pkg=PKG_DIR, repo=REPO, ndm=ndm, collective=collective))
    port = _free_port()
    procs = []
    for rank in range(world):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                   LOCAL_RANK=str(rank), OMP_NUM_THREADS="1")
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            p.kill()
            out, _ = p.communicate()
        outs.append(out)
    for p, out in zip(procs, outs):
        assert p.returncode == 0, out
        assert "ok" in out


class _FakePlan:
    """The attributes ready_tiles reads (a pu_plan's time tiling + shift extent)."""

    def __init__(self, nsamples, tt_len, shift_min, shift_max, max_spread):
        self.nsamples = nsamples
        self.info = {"time_tile": tt_len, "time_tiles": -(-nsamples // tt_len), "max_spread": max_spread}
        self.shift_min, self.shift_max = shift_min, shift_max

    def tile_window(self, tt):
        from pulsarutils._hip import Plan
        return Plan.tile_window(self, tt)


@pytest.mark.parametrize("n,chunks", [(1 << 22, 8), (1 << 20, 3), (12345, 4), (1000, 8)])
def test_column_chunks_rank_independent(n, chunks):
    """The chunked broadcast's column ranges depend on the shape only (every rank issues
    the same collectives whatever its plan), cover [0, n) and are whole quanta."""
    from pulsarutils.parallel import column_chunks
    b = column_chunks(n, chunks)
    assert b[0][0] == 0 and b[-1][1] == n
    assert all(c1 == d0 for (_, c1), (d0, _) in zip(b, b[1:]))
    assert all((c1 - c0) % 1024 == 0 for c0, c1 in b[:-1])
    assert len(b) <= max(1, chunks)


@pytest.mark.parametrize("shift_min,shift_max", [(-2084, 2914), (0, 582), (-843, 1931)])
def test_ready_tiles_halo(shift_min, shift_max):
    """A time tile is searched only once its whole read window (shift halo + LDS-DMA
    rounding) has landed; tiles whose window wraps modulo N wait for the last chunk;
    every tile is ready at the end."""
    from pulsarutils.parallel import column_chunks, ready_tiles
    n, tt_len = 1 << 20, 512
    plan = _FakePlan(n, tt_len, shift_min, shift_max, 74)
    seen = np.zeros(plan.info["time_tiles"], dtype=bool)
    for _, c1 in column_chunks(n, 8):
        r = ready_tiles(plan, c1)
        assert not (seen & ~r).any()  # monotone in the landed prefix
        for tt in np.flatnonzero(r & ~seen):
            a, b = plan.tile_window(tt)
            assert c1 >= n or (a >= 0 and b <= c1)
            # the kernel's own reads: [t0 + smin, t0 + TT + smax + spread + 1 + DMA rounding)
            assert a <= tt * tt_len + shift_min and b >= (tt + 1) * tt_len + shift_max + 74 + 1 + 256
        seen |= r
    assert seen.all()
    if shift_min < 0:
        assert not ready_tiles(plan, n - 1)[0]  # tile 0 wraps to the end of the array


PIPE_WORKER = textwrap.dedent("""
    import sys
    sys.path[:0] = [{pkg!r}, {repo!r}]
    import numpy as np, torch, torch.distributed as dist
    from pulsarutils._hip import Plan
    from pulsarutils.parallel import pipelined_broadcast_search, ready_tiles
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    nchan, n, tt_len = 6, {n}, 512
    full = (np.random.default_rng(3).random((nchan, n)) * 100).astype({dtype!r})
    data = torch.from_numpy(full.copy()) if rank == {src} else torch.zeros((nchan, n), dtype=torch.from_numpy(full).dtype)

    class FakePlan:
        nsamples = n
        info = {{"time_tile": tt_len, "time_tiles": -(-n // tt_len), "max_spread": 74}}
        shift_min, shift_max = {smin}, {smax}
        def tile_window(self, tt):
            return Plan.tile_window(self, tt)

    class CheckSearcher:
        # every searched tile's read window must already hold the source's columns
        def __init__(self):
            self.plan = FakePlan()
            self.ntiles = self.plan.info["time_tiles"]
            self.count = np.zeros(self.ntiles, dtype=int)
        def ready(self, landed):
            return ready_tiles(self.plan, landed)
        def tiles(self, d, b, e, stream=None):
            assert stream is None
            for tt in range(b, e):
                a0, b0 = self.plan.tile_window(tt)
                cols = np.arange(a0, b0) % n
                assert np.array_equal(d[:, cols].numpy(), full[:, cols]), (rank, tt)
                self.count[tt] += 1
        def finalize(self, d, stream=None):
            assert (self.count == 1).all(), self.count
            return "finalized"

    s = CheckSearcher()
    assert pipelined_broadcast_search(data, None, src={src}, chunks={chunks}, searcher=s,
                                      collective={collective!r}) == "finalized"
    assert np.array_equal(data.numpy(), full)
    dist.barrier()
    dist.destroy_process_group()
    print("rank", rank, "ok")
""")


@pytest.mark.parametrize("collective", ["broadcast", "scatter_allgather"])
@pytest.mark.parametrize("world,src,n,chunks,smin,smax,dtype", [
    (2, 0, 50000, 5, -2084, 2914, "float32"),
    (3, 1, 1 << 16, 8, 0, 582, "uint8"),
    (4, 3, 40962, 3, -843, 1931, "float64"),
    (2, 1, 9000, 8, 100, 700, "uint8"),
])
def test_pipelined_broadcast_gloo(tmp_path, world, src, n, chunks, smin, smax, dtype, collective):
    """The multi-rank branch of parallel.pipelined_broadcast_search (staging pack on the
    source, chunk broadcast, unpack on the others, ready-tile launches) on CPU under gloo
    at world 2-4 with any source rank: every time tile is searched exactly once, only
    after every column of its read window holds the source's data, and the landed data
    equals the source on every rank at the end."""
    script = tmp_path / "pipe_worker.py"
    script.write_text(PIPE_WORKER.format(pkg=PKG_DIR, repo=REPO, n=n, src=src, chunks=chunks, smin=smin, smax=smax,
                                         dtype=dtype, collective=collective))
    port = _free_port()
    procs = []
    for rank in range(world):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                   LOCAL_RANK=str(rank), OMP_NUM_THREADS="1")
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            p.kill()
            out, _ = p.communicate()
        outs.append(out)
    for p, out in zip(procs, outs):
        assert p.returncode == 0, out
        assert "ok" in out


@pytest.mark.parametrize("n,tt,ntiles,world,chunks", [(1 << 20, 256, 4096, 8, 8), (1000, 256, 4, 3, 2),
                                                       (50000, 512, 98, 4, 5), (9000, 256, 36, 2, 8)])
def test_interleaved_chunks_cover(n, tt, ntiles, world, chunks):
    """The time-tile sharded exchange's chunks: disjoint tile-aligned column ranges that
    cover [0, n) once; chunk k holds the k-th piece of every rank's slice (so each slice
    lands at the same pace), and the ranges depend on the shape only."""
    from pulsarutils.parallel import interleaved_chunks
    ch = interleaved_chunks(n, tt, ntiles, world, chunks)
    assert len(ch) <= chunks
    cover = np.zeros(n, dtype=int)
    for ranges in ch:
        for c0, c1 in ranges:
            assert c0 % tt == 0 and (c1 % tt == 0 or c1 == n) and c1 > c0
            cover[c0:c1] += 1
    assert (cover == 1).all()
    for q in range(world):
        t0, t1 = shard_bounds(ntiles, world, q)
        got = [(c0, c1) for ranges in ch for c0, c1 in ranges if t0 * tt <= c0 < max(t1 * tt, t0 * tt + 1)]
        assert sum(c1 - c0 for c0, c1 in got) == min(n, t1 * tt) - min(n, t0 * tt)


def test_ready_by_blocks_matches_columns():
    """ready_by_blocks (block prefix sums, windows wrapping modulo n) equals the brute-force
    check of every column of every window."""
    from pulsarutils.parallel import ready_by_blocks
    rng = np.random.default_rng(5)
    for n, tt, wa, wb in [(10000, 256, -300, 900), (4096, 256, 0, 256 + 700), (5000, 512, -10, 5200),
                          (3000, 256, 17, 400)]:
        nb = -(-n // tt)
        ntt = nb
        starts = np.arange(ntt, dtype=np.int64) * tt
        for _ in range(20):
            landed = rng.random(nb) < 0.7
            got = ready_by_blocks(landed, tt, n, starts, wa, wb)
            col = np.repeat(landed, tt)[:n]
            want = np.array([col[np.arange(s + wa, s + wb) % n].all() for s in starts])
            assert np.array_equal(got, want), (n, tt, wa, wb)


TILE_WORKER = textwrap.dedent("""
    import sys
    sys.path[:0] = [{pkg!r}, {repo!r}]
    import numpy as np, torch, torch.distributed as dist
    from pulsarutils.parallel import shard_bounds, slice_regions, tile_sharded_search
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    nchan, n, tt, ndm = 5, {n}, 256, {ndm}
    rng = np.random.default_rng(11)
    full = rng.random((nchan, n))
    if {nan}:
        full[2, n // 2 + 3] = np.nan
    shifts = rng.integers({smin}, {smax} + 1, size=(ndm, nchan))

    def stats(s):
        return [s.max(), s.std(), s.sum(), int(np.argmax(s))]

    class NumpySearcher:
        # per-(trial, time tile) records (sum, sum of squares, max) of the circular
        # shift-and-sum; finalize combines them in tile order (the same bits whatever rank
        # computed a tile); trials d % 3 == 1 and trials with a non-finite record are
        # "flagged" and settled from their whole series (exact_series + series_stats)
        def __init__(self):
            self.ntiles, self.tt_len, self.ndm = -(-n // tt), tt, ndm
            self.rec = torch.full((ndm, self.ntiles, 3), float("nan"), dtype=torch.float64)
            self.count = np.zeros(self.ntiles, dtype=int)
        def tile_window(self, i):
            return (i * tt + int(shifts.min()), i * tt + tt + int(shifts.max()))
        def tiles(self, d, b, e, stream=None):
            x = d.numpy()
            for i in range(b, e):
                t = np.arange(i * tt, min(n, (i + 1) * tt))
                for dd in range(ndm):
                    s = sum(x[c, (t + shifts[dd, c]) % n] for c in range(nchan))
                    self.rec[dd, i] = torch.tensor([s.sum(), (s * s).sum(), s.max()])
                self.count[i] += 1
        def records(self):
            return self.rec
        def _fast(self, lo, hi):
            out = [torch.zeros(ndm, dtype=torch.float64) for _ in range(3)] + [torch.zeros(ndm, dtype=torch.int32)]
            flagged, nnf = [], 0
            for dd in range(lo, hi):
                r = self.rec[dd].numpy()
                s1 = s2 = 0.0
                for i in range(self.ntiles):
                    s1 += r[i, 0]
                    s2 += r[i, 1]
                out[0][dd], out[1][dd], out[2][dd], out[3][dd] = r[:, 2].max(), s1, s2, dd
                if not np.isfinite(r).all():
                    flagged.append(dd)
                    nnf += 1
                elif dd % 3 == 1:
                    flagged.append(dd)
            return out, np.array(flagged, dtype=np.int32), nnf
        def finalize_range(self, d, lo, hi, stream=None):
            out, flagged, nnf = self._fast(lo, hi)
            if nnf and not np.isfinite(d.numpy()).all():
                for k, v in enumerate((float("nan"), float("nan"), 0.0, 0)):
                    out[k][lo:hi] = v
                return out
            if len(flagged):
                st = self.series_stats(self.exact_series(d, flagged))
                for k in range(4):
                    out[k][torch.as_tensor(flagged.astype(np.int64))] = st[k]
            return out
        def finalize_range_flagged(self, lo, hi, stream=None):
            return self._fast(lo, hi)
        def exact_series(self, d, trials, t_begin=0, t_end=n, stream=None):
            x = d.numpy()
            t = np.arange(t_begin, t_end)
            return torch.from_numpy(np.stack([sum(x[c, (t + shifts[dd, c]) % n] for c in range(nchan))
                                              for dd in trials]))
        def series_stats(self, ser, stream=None):
            st = [stats(r) for r in ser.numpy()]
            return [torch.tensor([s[k] for s in st], dtype=torch.float64) for k in range(3)] + \
                [torch.tensor([s[3] for s in st], dtype=torch.int32)]
        def nonfinite(self, x, stream=None):
            return torch.tensor(int(not torch.isfinite(x).all()), dtype=torch.int32)

    ref = NumpySearcher()
    ref.tiles(torch.from_numpy(full), 0, ref.ntiles)
    want = ref.finalize_range(torch.from_numpy(full), 0, ndm)
    data = torch.from_numpy(full.copy()) if rank == {src} else torch.full((nchan, n), float("nan"), dtype=torch.float64)
    s = NumpySearcher()
    res, (lo, hi) = tile_sharded_search(data, None, src={src}, chunks={chunks}, searcher=s, collective={collective!r},
                                        full_copy={full_copy})
    t0, t1 = shard_bounds(s.ntiles, world, rank)
    assert s.count.sum() == s.count[t0:t1].sum() and (s.count[t0:t1] == 1).all(), s.count
    for k in range(4):
        assert np.array_equal(res[k][lo:hi].numpy(), want[k][lo:hi].numpy(), equal_nan=True), (rank, k)
    if {full_copy}:
        assert np.array_equal(data.numpy(), full, equal_nan=True)
    else:
        a, ln = slice_regions(n, tt, s.ntiles, world, *s.tile_window(0))[rank]
        cols = np.arange(a, a + ln) % n
        assert np.array_equal(data.numpy()[:, cols], full[:, cols], equal_nan=True)
    dist.barrier()
    dist.destroy_process_group()
    print("rank", rank, "ok", lo, hi)
""")


@pytest.mark.parametrize("full_copy", [False, True])
@pytest.mark.parametrize("world,src,n,ndm,chunks,smin,smax,collective,nan", [
    (2, 0, 6000, 7, 3, 0, 700, "broadcast", False),
    (3, 2, 5000, 2, 4, 0, 1300, "scatter_allgather", False),
    (4, 1, 4099, 9, 2, 40, 300, "scatter_allgather", False),
    (3, 0, 3000, 5, 3, 0, 900, "broadcast", True),
    (2, 1, 700, 4, 2, 0, 650, "scatter_allgather", False),
])
def test_tile_sharded_search_gloo(tmp_path, world, src, n, ndm, chunks, smin, smax, collective, nan, full_copy):
    """parallel.tile_sharded_search on CPU under gloo, world 2-4, any source rank, receivers
    starting from NaN: every rank searches exactly its own time tiles and only once their
    windows (wrapping modulo n) landed; the records all_to_all brings every trial's records
    to its owner, whose finalize equals the single-process one bit for bit (ranks with no
    trials included).  full_copy: every rank ends with the source's filterbank; otherwise
    (the scatter of each rank's region) with its region, the flagged trials settled from the
    all-gathered series pieces and a NaN anywhere giving every trial the NaN rule."""
    script = tmp_path / "tile_worker.py"
    script.write_text(TILE_WORKER.format(pkg=PKG_DIR, repo=REPO, n=n, ndm=ndm, src=src, chunks=chunks, smin=smin,
                                         smax=smax, collective=collective, nan=nan, full_copy=full_copy))
    port = _free_port()
    procs = []
    for rank in range(world):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                   LOCAL_RANK=str(rank), OMP_NUM_THREADS="1")
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            p.kill()
            out, _ = p.communicate()
        outs.append(out)
    for p, out in zip(procs, outs):
        assert p.returncode == 0, out
        assert "ok" in out
