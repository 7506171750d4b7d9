"""One GPU standing in for one rank of the 8-way C3 time-tile split (parallel.tile_sharded_search,
sliced exchange): every step the rank runs on its own GPU, without the wire.

    python scripts/tsplit_rank_sim.py [world] [chunks]        (default 8 8)

* src (rank 0): its tile search (one pu_plan_search_tiles launch: it holds every column) on the
  compute stream while the communication stream packs piece k of every other rank's region
  into the scatter buffer (the copies tile_sharded_search issues), k = 0 .. chunks - 1;
* a receiver (rank world / 2): per chunk, the unpack of its piece (scatter buffer -> its data
  columns) on the communication stream, then - gated by that chunk's event, as in
  tile_sharded_search - the launch of its tiles whose windows have landed;
* each alone: the tile search, the packs, the unpacks.
HIP events; median of 3.  Prints one JSON line per measurement."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "radio-pulsar-utils_amd"), REPO]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from pulsarutils import _hip, synth  # noqa: E402
from pulsarutils.configs import CONFIGS  # noqa: E402
from pulsarutils.dedispersion import dedispersion_plan  # noqa: E402
from pulsarutils.parallel import _cols, shard_bounds, slice_regions  # noqa: E402

world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
K = int(sys.argv[2]) if len(sys.argv) > 2 else 8
cfg = CONFIGS["C3"]
x = synth.pulsar_filterbank_device(cfg)
dev = x.device
nchan, n = x.shape
dms = dedispersion_plan(cfg.nchan, cfg.dmmin, cfg.dmmax, cfg.start_freq, cfg.bandwidth, cfg.tsamp)
sh = _hip.shift_table(cfg.nchan, dms, cfg.start_freq, cfg.bandwidth, cfg.tsamp)
plan = _hip.Plan(_hip.dtype_code(x.dtype), _hip.PU_ACC_NATIVE, cfg.nchan, cfg.nsamples, sh)
ws = torch.empty(plan.workspace_bytes, dtype=torch.uint8, device=dev)
ntt, tt = plan.info["time_tiles"], plan.info["time_tile"]
wa, wb = plan.tile_window(0)
regions = slice_regions(n, tt, ntt, world, wa, wb)
pieces = [[None if rg is None else (rg[0] + shard_bounds(rg[1], K, k)[0], rg[0] + shard_bounds(rg[1], K, k)[1])
           for rg in regions] for k in range(K)]
widths = [max(b - a for a, b in pk if True) for pk in pieces]
width = max(widths)
staging = torch.empty(world * nchan * width, dtype=x.dtype, device=dev)
comm, comp = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)


def pack(k, skip=0):
    m = nchan * widths[k]
    for q, pc in enumerate(pieces[k]):
        if q == skip or pc is None:
            continue
        blk = staging[q * m:q * m + nchan * (pc[1] - pc[0])].view(nchan, pc[1] - pc[0])
        o = 0
        for c0, c1 in _cols(pc[0], pc[1], n):
            blk[:, o:o + c1 - c0].copy_(x[:, c0:c1])
            o += c1 - c0


def unpack(k, r):
    m = nchan * widths[k]
    pc = pieces[k][r]
    blk = staging[r * m:r * m + nchan * (pc[1] - pc[0])].view(nchan, pc[1] - pc[0])
    o = 0
    for c0, c1 in _cols(pc[0], pc[1], n):
        x[:, c0:c1].copy_(blk[:, o:o + c1 - c0])  # the same bytes back: x is unchanged
        o += c1 - c0


def timed(fn, reps=3):
    out = []
    for _ in range(reps):
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        comm.wait_stream(torch.cuda.current_stream())
        comp.wait_stream(torch.cuda.current_stream())
        fn()
        torch.cuda.current_stream().wait_stream(comm)
        torch.cuda.current_stream().wait_stream(comp)
        b.record()
        torch.cuda.synchronize()
        out.append(a.elapsed_time(b))
    return round(float(np.median(out)), 3)


starts = np.arange(ntt, dtype=np.int64) * tt
res = {"config": "C3", "world": world, "chunks": K, "scatter_piece_bytes": [nchan * w for w in widths],
       "region_bytes_per_rank": int(regions[1][1]) * nchan if regions[1] else None}
# src
t0, t1 = shard_bounds(ntt, world, 0)
res["src_search_alone_ms"] = timed(lambda: plan.search_tiles(x, t0, t1, ws, stream=comp))


def src_packs():
    with torch.cuda.stream(comm):
        for k in range(K):
            pack(k)


res["src_packs_alone_ms"] = timed(src_packs)


def src_step():
    plan.search_tiles(x, t0, t1, ws, stream=comp)
    src_packs()


res["src_search_with_packs_ms"] = timed(src_step)
# a receiver
r = world // 2
t0, t1 = shard_bounds(ntt, world, r)
with torch.cuda.stream(comm):
    for k in range(K):
        pack(k, skip=-1)  # staging holds every rank's pieces (untimed)
torch.cuda.synchronize()
res["recv_rank"] = r
res["recv_search_alone_ms"] = timed(lambda: plan.search_tiles(x, t0, t1, ws, stream=comp))


def recv_unpacks():
    with torch.cuda.stream(comm):
        for k in range(K):
            unpack(k, r)


res["recv_unpacks_alone_ms"] = timed(recv_unpacks)


def recv_step():
    a, ln = regions[r]
    done = np.zeros(ntt, dtype=bool)
    mine = np.zeros(ntt, dtype=bool)
    mine[t0:t1] = True
    for k in range(K):
        with torch.cuda.stream(comm):
            unpack(k, r)
            ev = torch.cuda.Event()
            ev.record(comm)
        comp.wait_event(ev)
        ready = (starts + wb - starts[0] <= pieces[k][r][1]) & mine & ~done
        idx = np.flatnonzero(ready)
        for run in np.split(idx, np.flatnonzero(np.diff(idx) != 1) + 1) if idx.size else []:
            plan.search_tiles(x, int(run[0]), int(run[-1]) + 1, ws, stream=comp)
        done |= ready
    assert done[t0:t1].all()


res["recv_unpack_and_gated_search_ms"] = timed(recv_step)
print(json.dumps(res), flush=True)
