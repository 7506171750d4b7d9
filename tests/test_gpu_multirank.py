"""the multi-rank HIP path on the one leased GPU, before any 8-GPU run
depends on it.  2 and 3 ranks (processes) share cuda:0 over a ``gloo`` process group
(RCCL refuses two ranks per device) and run the product path's world > 1 branch for
real: chunked broadcast from a non-zero source on the communication stream, staging
pack / unpack, event-gated time-tile launches (pu_plan_search_tiles) on the compute
stream, pu_plan_finalize, and sharded_search's all_gather - each rank's outputs equal
the single-rank search bit for bit (tests/mr_worker.py).  The reference's parallelism
is the prange over trials (dedispersion.py:174-181)."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,case,collective", [
    (2, "C5", "broadcast"), (3, "C5", "broadcast"), (2, "C3s", "broadcast"), (3, "C3s", "broadcast"),
    (2, "C5m", "broadcast"),
    # round 5: the mesh exchange (scatter 1/world of each chunk, then all-gather)
    (2, "C5", "scatter_allgather"), (3, "C3s", "scatter_allgather"), (3, "C5m", "scatter_allgather")])
def test_multirank_pipelined_and_sharded_on_one_gpu(gpu, world, case, collective):
    _run_ranks(world, case, collective, "dm")


@pytest.mark.parametrize("world,case,collective", [
    (2, "C5", "scatter_allgather"), (3, "C5", "broadcast"), (2, "C3s", "scatter_allgather"),
    (3, "C3s", "scatter_allgather"), (3, "C3z", "scatter_allgather"), (2, "C5n", "broadcast")])
def test_multirank_tile_sharded_on_one_gpu(gpu, world, case, collective):
    """Round 6: time-tile sharding (parallel.tile_sharded_search) - each rank searches its
    time tiles of the whole grid's plan while the interleaved chunks land, the records go
    to the trial owners (all_to_all), each owner finalizes its trials
    (pu_plan_finalize_range): bit-equal to the one-GPU search of the grid - with the whole
    filterbank sent to every rank and with each rank's region only (flagged trials settled
    from the all-gathered series pieces: C3z all-zero 8-bit data flags every trial; C5n
    one NaN gives every trial the NaN rule)."""
    _run_ranks(world, case, collective, "time")


def _run_ranks(world, case, collective, decomposition):
    port = _free_port()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="4")
    procs = [subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "mr_worker.py"), str(r), str(world), str(port),
                               case, collective, decomposition], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                              env=env)
             for r in range(world)]
    outs = []
    try:
        for p in procs:
            o, e = p.communicate(timeout=240)
            outs.append((p.returncode, o.decode(errors="replace"), e.decode(errors="replace")))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    for r, (rc, o, e) in enumerate(outs):
        assert rc == 0 and f"RANK {r} OK" in o, f"rank {r} rc {rc}\n{o}\n{e[-4000:]}"
    print("\n".join(o.strip() for _, o, _ in outs))


@pytest.mark.parametrize("case,collective,decomposition", [("C5", "broadcast", "dm"), ("C3s", "scatter_allgather", "dm"),
                                                          ("C3s", "scatter_allgather", "time")])
def test_rccl_process_group_one_rank(gpu, case, collective, decomposition):
    """The product path's collectives on an RCCL ("nccl") process group: one rank on the one
    GPU (RCCL takes one rank per device), so the same worker's broadcast / all_gather /
    barrier run through RCCL itself, bit-equal to the single-process search."""
    port = _free_port()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="4", MR_BACKEND="nccl")
    p = subprocess.run([sys.executable, "-u", os.path.join(HERE, "mr_worker.py"), "0", "1", str(port), case,
                        collective, decomposition], capture_output=True, timeout=240, env=env)
    o, e = p.stdout.decode(errors="replace"), p.stderr.decode(errors="replace")
    assert p.returncode == 0 and "RANK 0 OK" in o and " nccl " in o, f"rc {p.returncode}\n{o}\n{e[-4000:]}"
