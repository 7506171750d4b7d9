"""DM-trial sharding across GPUs (one process per GPU, torch.distributed over RCCL/xGMI).

The reference's only parallelism is numba ``prange`` over independent DM trials
(``dedispersion.py:174,181``).  Here the same trial axis is split across ranks:

1. the filterbank is distributed from ``src`` (RCCL over xGMI; the data path of the
   search itself has no other exchange).  :func:`pipelined_broadcast_search` cuts the
   transfer into time chunks and starts the search of each time tile as soon as the
   columns it reads (its window plus the shift halo) have landed, so the transfer of
   later chunks overlaps the search of earlier ones.  Two exchanges per chunk
   (``collective``): ``"broadcast"`` (one RCCL broadcast from ``src``) or
   ``"scatter_allgather"`` (``src`` scatters 1/world of the chunk to every rank, then all
   ranks all-gather it: the second step's traffic runs over every xGMI link of the mesh
   instead of leaving ``src``'s links alone).  The default
   everywhere (``DEFAULT_COLLECTIVE``) is ``"scatter_allgather"``;
2. each rank searches its contiguous slice of the trial grid on its own GPU,
3. the per-trial statistics (max, std, snr, rebin) are all-gathered, so every rank
   ends with the reference's full-length result arrays.

``compute`` is injectable: the product path uses the HIP search; the CPU gloo tests
pass the oracle to exercise the sharding / gather plumbing without a GPU.
"""
import numpy as np


def shard_bounds(ndm, world, rank):
    """Contiguous split of ``ndm`` trials: the first ``ndm % world`` ranks get one more."""
    base, rem = divmod(int(ndm), int(world))
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def _hip_compute(data, dms, nchan, start_freq, bandwidth, sample_time, acc):
    from .dedispersion import search_device
    (mx, sd, snr, win), _ = search_device(data, dms, nchan, start_freq, bandwidth, sample_time, acc=acc)
    return mx, sd, snr, win.to(mx.dtype)


DEFAULT_COLLECTIVE = "scatter_allgather"


def broadcast_filterbank(data, src=0, group=None, collective=DEFAULT_COLLECTIVE):
    """Give every rank ``src``'s (nchan, N) filterbank tensor, in place (contiguous data:
    the whole tensor is one :func:`exchange_chunk`; a padded tail goes through a staging
    copy when ``scatter_allgather`` needs a multiple of world elements)."""
    import torch
    import torch.distributed as dist
    if collective == "broadcast":
        dist.broadcast(data, src=src, group=group)
        return data
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    flat = data.reshape(-1) if data.is_contiguous() else None
    blen = -(-data.numel() // world) * world
    if flat is None or blen != data.numel():
        staging = torch.empty(blen, dtype=data.dtype, device=data.device)
        if rank == src:
            staging[:data.numel()].copy_(data.reshape(-1))
        exchange_chunk(staging, torch.empty(blen // world, dtype=data.dtype, device=data.device), rank, src,
                       world, group, collective)
        if rank != src:
            data.copy_(staging[:data.numel()].view(data.shape))
        return data
    exchange_chunk(flat, torch.empty(blen // world, dtype=data.dtype, device=data.device), rank, src, world,
                   group, collective)
    return data


def column_chunks(nsamples, chunks, quantum=1024):
    """Split [0, nsamples) into about ``chunks`` column ranges (multiples of ``quantum``
    samples).  Depends on the shape only, so every rank issues the same collectives
    whatever its plan (plans of different DM slices may use different time tiles)."""
    n = int(nsamples)
    width = max(quantum, -(-(-(-n // max(1, int(chunks)))) // quantum) * quantum)
    return [(c0, min(n, c0 + width)) for c0 in range(0, n, width)]


COLLECTIVES = ("broadcast", "scatter_allgather")


def exchange_chunk(buf, piece, rank, src, world, group=None, collective=DEFAULT_COLLECTIVE):
    """Make every rank's ``buf`` (1-D, contiguous) equal ``src``'s.

    ``"broadcast"``: one broadcast from ``src``.  ``"scatter_allgather"``: ``buf``'s length
    is a multiple of ``world``; ``src`` scatters piece r of it to rank r (into ``piece``, a
    separate buffer of len(buf) / world elements) and every rank all-gathers the pieces
    into ``buf``.  On ``src`` the all-gather rewrites ``buf`` with its own bytes."""
    import torch.distributed as dist
    if collective == "broadcast" or world == 1:
        dist.broadcast(buf, src=src, group=group)
        return buf
    if collective != "scatter_allgather":
        raise ValueError(f"collective must be one of {COLLECTIVES}, got {collective!r}")
    m = buf.numel() // world
    if m * world != buf.numel() or piece.numel() != m:
        raise ValueError(f"scatter_allgather: buffer of {buf.numel()} elements is not {world} pieces of "
                         f"{piece.numel()}")
    dist.scatter(piece, list(buf.split(m)) if rank == src else None, src=src, group=group)
    dist.all_gather_into_tensor(buf, piece, group=group)
    return buf


def ready_tiles(plan, landed):
    """Time tiles whose whole read window lies in the landed column prefix [0, landed)
    (windows that wrap modulo nsamples wait for the whole array)."""
    n = plan.nsamples
    ntt = plan.info["time_tiles"]
    if landed >= n:
        return np.ones(ntt, dtype=bool)
    a0, b0 = plan.tile_window(0)
    starts = np.arange(ntt, dtype=np.int64) * plan.info["time_tile"]
    return (starts + a0 >= 0) & (starts + b0 <= landed)


class PlanSearcher:
    """The per-rank work of :func:`pipelined_broadcast_search` on a HIP plan: time-tile
    range searches as columns land (pu_plan_search_tiles), then pu_plan_finalize."""

    def __init__(self, plan, out=None, workspace=None, device=None):
        self.plan = plan
        self.out, self.workspace = plan._outs_ws(device, out, workspace)
        self.ntiles = plan.info["time_tiles"]

    def ready(self, landed):
        return ready_tiles(self.plan, landed)

    def tiles(self, data, begin, end, stream=None):
        self.plan.search_tiles(data, begin, end, self.workspace, stream=stream)

    def finalize(self, data, stream=None):
        return self.plan.finalize(self.workspace, data, out=self.out, stream=stream)

    def streams_done(self, stream):
        self.workspace.record_stream(stream)
        for o in self.out:
            o.record_stream(stream)


class PhaseEvents:
    """HIP events around the phases of one pipelined step (``pipelined_broadcast_search``'s
    ``phases``): ``exchange`` and ``unpack`` per chunk on the communication stream,
    ``search`` per chunk (the tile-range launches) on the compute stream, ``finalize``.
    :meth:`times_ms` (after a synchronize) gives each phase's per-chunk durations and, as
    ``exposed_tail_ms``, the time from the last chunk's unpack end to the finalize end -
    the part of the search the exchange could not hide."""

    def __init__(self):
        self.ev = {}

    def mark(self, name, stream, end=False):
        import torch
        e = torch.cuda.Event(enable_timing=True)
        e.record(stream)
        self.ev.setdefault(name, []).append((e, end))

    def _spans(self, name):
        evs = self.ev.get(name, [])
        return [(evs[i][0], evs[i + 1][0]) for i in range(0, len(evs) - 1, 2)]

    def times_ms(self):
        out = {name: [round(a.elapsed_time(b), 4) for a, b in self._spans(name)] for name in self.ev}
        res = {f"{k}_ms": v for k, v in out.items()}
        for k, v in out.items():
            res[f"{k}_total_ms"] = round(float(sum(v)), 4)
        ex, fin = self._spans("exchange"), self._spans("finalize")
        last = self._spans("unpack")[-1][1] if self._spans("unpack") else (ex[-1][1] if ex else None)
        if ex and fin:
            res["step_span_ms"] = round(ex[0][0].elapsed_time(fin[-1][1]), 4)
            res["exposed_tail_ms"] = round(last.elapsed_time(fin[-1][1]), 4)
        return res


_MASKED = {}  # (device index, reserved CUs) -> MaskedStream, kept for the process


def _masked_stream(reserve, dev):
    """The CU-masked compute stream for ``reserve`` CUs on ``dev``, created once and kept
    alive for the process: tensors record_stream'ed onto it (the searcher's workspace and
    outputs) are freed later by the caching allocator, which then records an event on
    this stream - so it must outlive them."""
    from ._hip import MaskedStream
    key = (dev.index, int(reserve))
    if key not in _MASKED:
        _MASKED[key] = MaskedStream(reserve, dev)
    return _MASKED[key]


def pipelined_broadcast_search(data, plan, out=None, workspace=None, src=0, chunks=8, group=None, searcher=None,
                               reserve_cus=0, collective=DEFAULT_COLLECTIVE, phases=None):
    """Distribute ``data`` from ``src`` in time chunks while searching it with ``plan``.

    Chunk k (a range of whole time tiles, all channels) is packed into a contiguous
    staging buffer on ``src``, exchanged (RCCL on a communication stream; ``collective``:
    :func:`exchange_chunk`'s broadcast or scatter + all-gather) and unpacked
    into ``data`` on the other ranks; every time tile whose read window has landed is
    searched (on a compute stream) as soon as its chunk's event fires
    (pu_plan_search_tiles), and the per-trial outputs are finalised when all tiles ran
    (pu_plan_finalize).  Returns the (max, std, snr, rebin) device tensors; the caller's
    current stream is ordered after all of it.  ``plan=None`` (a rank with no trials)
    only takes part in the broadcasts.

    ``reserve_cus`` > 0: while chunks are still to come, the tile searches go to a
    CU-masked stream that leaves that many CUs to the broadcast's kernels
    (pu_stream_create_cu_masked); the tiles that wait for the last chunk and the
    finalize run unmasked.  Off by default: on one MI355X the proxy
    (scripts/overlap_probe.py, profiles/r03/overlap_probe_r3b.json) shows copy kernels on
    a second stream getting 2.2 TB/s beside the unmasked search, and an 8-CU mask slowing
    the search alone by 15 % (15.6 -> 18.0 ms) without speeding the copies.

    ``phases`` (device data only): a :class:`PhaseEvents` that records HIP events around each
    chunk's exchange and unpack (communication stream), each chunk's tile searches (compute
    stream) and the finalize; :meth:`PhaseEvents.times_ms` reads them after a synchronize.

    Receiving ranks copy each landed chunk from the contiguous staging buffer into the
    strided column range ``data[:, c0:c1]`` (the ``unpack`` phase): RCCL moves contiguous
    buffers only, and the kernels read rows of ``data`` at its row stride, so a column chunk
    cannot land in place.  The copy runs on the communication stream, overlapped with the
    search of the chunks already landed; ``phases`` measures it.

    ``searcher`` replaces the HIP work (an object with ``ntiles``, ``ready(landed)``,
    ``tiles(data, begin, end, stream)`` and ``finalize(data, stream)``): with a CPU
    ``data`` tensor the same chunk / staging / unpack / ready-tile sequence runs
    synchronously, which is how the gloo tests drive the multi-rank branch on CPU.
    """
    import contextlib

    import torch
    import torch.distributed as dist
    cuda = data.is_cuda
    dev = data.device
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    if cuda and data.element_size() == 1 and data.shape[1] % 4 == 0 and (data.data_ptr() % 4 or data.stride(0) % 4):
        # 8-bit LDS-DMA plans need dword-aligned rows; data is the receive buffer
        raise ValueError("pipelined search of 8-bit data needs rows starting on 4-byte boundaries")
    nchan, n = data.shape
    bounds = column_chunks(n, chunks)
    if searcher is None and plan is not None:
        searcher = PlanSearcher(plan, out, workspace, dev)
    masked = None
    if cuda:
        cur = torch.cuda.current_stream(dev)
        comm = torch.cuda.Stream(device=dev)
        comp = torch.cuda.Stream(device=dev)
        comm.wait_stream(cur)
        comp.wait_stream(cur)
        if world > 1 and reserve_cus > 0 and searcher is not None and len(bounds) > 1:
            masked = _masked_stream(reserve_cus, dev)
            masked.stream.wait_stream(cur)
    else:
        cur = comm = comp = None
    on_comm = (lambda: torch.cuda.stream(comm)) if cuda else contextlib.nullcontext
    done = np.zeros(searcher.ntiles, dtype=bool) if searcher is not None else None
    if collective not in COLLECTIVES:
        raise ValueError(f"collective must be one of {COLLECTIVES}, got {collective!r}")
    width = max(c1 - c0 for c0, c1 in bounds)
    # staging holds whole chunks padded to a multiple of world elements (scatter pieces)
    slen = -(-nchan * width // world) * world
    staging = torch.empty(slen, dtype=data.dtype, device=dev) if world > 1 else None
    piece = (torch.empty(slen // world, dtype=data.dtype, device=dev)
             if world > 1 and collective == "scatter_allgather" else None)
    for k, (c0, c1) in enumerate(bounds):
        # tiles launched while later chunks are in flight use the masked stream
        tstream = masked.stream if masked is not None and k + 1 < len(bounds) else comp
        with on_comm():
            if world > 1:
                blen = -(-nchan * (c1 - c0) // world) * world
                flat = staging[:blen]
                buf = flat[:nchan * (c1 - c0)].view(nchan, c1 - c0)  # contiguous
                if phases is not None:
                    phases.mark("exchange", comm)
                if rank == src:
                    buf.copy_(data[:, c0:c1])
                exchange_chunk(flat, piece[:blen // world] if piece is not None else None, rank, src, world,
                               group=group, collective=collective)
                if phases is not None:
                    phases.mark("exchange", comm, end=True)
                    phases.mark("unpack", comm)
                if rank != src:
                    data[:, c0:c1].copy_(buf)
                if phases is not None:
                    phases.mark("unpack", comm, end=True)
            ev = None
            if cuda:
                ev = torch.cuda.Event()
                ev.record(comm)
        if searcher is None:
            continue
        if cuda:
            tstream.wait_event(ev)
        ready = searcher.ready(c1) & ~done
        idx = np.flatnonzero(ready)
        # contiguous runs of ready tiles, one launch each
        if phases is not None:
            phases.mark("search", tstream)
        for run in np.split(idx, np.flatnonzero(np.diff(idx) != 1) + 1) if idx.size else []:
            searcher.tiles(data, int(run[0]), int(run[-1]) + 1, stream=tstream)
        if phases is not None:
            phases.mark("search", tstream, end=True)
        done |= ready
        if masked is not None and k + 2 == len(bounds):
            comp.wait_stream(masked.stream)  # the unmasked stream takes over for the last chunk
    if cuda:
        if staging is not None:
            staging.record_stream(comm)
        if piece is not None:
            piece.record_stream(comm)
        cur.wait_stream(comm)
    if searcher is None:
        return None
    if not done.all():
        raise RuntimeError("pipelined search: time tiles left unsearched")
    if phases is not None:
        phases.mark("finalize", comp)
    res = searcher.finalize(data, stream=comp)
    if phases is not None:
        phases.mark("finalize", comp, end=True)
    if cuda:
        if hasattr(searcher, "streams_done"):
            searcher.streams_done(comp)
            if masked is not None:
                searcher.streams_done(masked.stream)
        cur.wait_stream(comp)
    return res


def sharded_search(data, trial_DMs, nchan, start_freq, bandwidth, sample_time, group=None, acc=None,
                   compute=None, broadcast=True, src=0, pipelined=False, chunks=8, collective=DEFAULT_COLLECTIVE):
    """Distributed ``_dedispersion_search``: returns (max, std, snr, rebin[int32]) numpy arrays
    covering ALL trials, on every rank.

    ``data`` must be a tensor of the right shape/dtype on every rank (only ``src``'s
    content matters when ``broadcast``).  ``pipelined`` (HIP compute only) overlaps the
    transfer with the search (:func:`pipelined_broadcast_search`); ``collective`` picks
    the transfer (:func:`exchange_chunk`: ``"broadcast"`` or ``"scatter_allgather"``).
    """
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dms = np.asarray(trial_DMs, dtype=np.float64)
    lo, hi = shard_bounds(dms.size, world, rank)
    dev = data.device
    chunk = -(-dms.size // world)  # ceil: equal-size gather buffers
    local = torch.zeros((4, chunk), dtype=torch.float64, device=dev)
    if pipelined and compute is None:
        from . import _hip
        from .dedispersion import _acc_code, _plan_for, _prepare_data
        if not (data.is_cuda and data.is_contiguous()):
            raise ValueError("pipelined sharded_search needs a contiguous device tensor (it is written in place)")
        x = _prepare_data(data)
        plan = None
        if hi > lo:
            sub = np.ascontiguousarray(dms[lo:hi])
            plan = _plan_for(x, lambda: _hip.shift_table(nchan, sub, start_freq, bandwidth, sample_time),
                             _acc_code(acc), ("dm-shard", sub.tobytes(), float(start_freq), float(bandwidth),
                                              float(sample_time)))
        if broadcast and world > 1:
            res = pipelined_broadcast_search(x, plan, src=src, chunks=chunks, group=group, collective=collective)
        else:
            res = plan.search(x) if plan is not None else None
        if res is not None:
            for k in range(4):
                local[k, :hi - lo] = res[k].to(torch.float64)
    else:
        if broadcast and world > 1:
            broadcast_filterbank(data, src=src, group=group, collective=collective)
        fn = compute or (lambda d, t: _hip_compute(d, t, nchan, start_freq, bandwidth, sample_time, acc))
        if hi > lo:
            res = fn(data, dms[lo:hi])
            for k in range(4):
                local[k, :hi - lo] = torch.as_tensor(res[k], dtype=torch.float64, device=dev)
    parts = [torch.empty_like(local) for _ in range(world)]
    dist.all_gather(parts, local, group=group)
    out = []
    for k in range(4):
        cols = [parts[r][k, :shard_bounds(dms.size, world, r)[1] - shard_bounds(dms.size, world, r)[0]]
                for r in range(world)]
        out.append(torch.cat(cols).cpu().numpy())
    return out[0], out[1], out[2], out[3].astype(np.int32)
