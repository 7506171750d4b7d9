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
                                      compute=compute)
    ref = oracle.search(arr, dms, h["fbottom"], h["bandwidth"], h["tsamp"], nthreads=1)
    assert np.array_equal(data.numpy(), arr)
    for a, b in zip((mx, sd, snr, win), ref):
        assert np.array_equal(a, b), (a[:4], b[:4])
    assert win.dtype == np.int32
    dist.barrier()
    dist.destroy_process_group()
    print("rank", rank, "ok")
""")


@pytest.mark.parametrize("world,ndm", [(2, 37), (2, 3), (3, 37), (3, 2), (4, 38), (4, 3)])
def test_sharded_search_gloo(tmp_path, world, ndm):
    script = tmp_path / "worker.py"
    script.write_text(WORKER.format(pkg=PKG_DIR, repo=REPO, ndm=ndm))
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
