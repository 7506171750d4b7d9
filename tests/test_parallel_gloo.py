"""Multi-process DM sharding on CPU (gloo, world_size 2): the shard split, the filterbank
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


@pytest.mark.parametrize("ndm", [37, 3])
def test_sharded_search_gloo_world2(tmp_path, ndm):
    script = tmp_path / "worker.py"
    script.write_text(WORKER.format(pkg=PKG_DIR, repo=REPO, ndm=ndm))
    port = _free_port()
    procs = []
    for rank in range(2):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2",
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
