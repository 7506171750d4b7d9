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
    range searches as columns land (pu_plan_search_tiles), then pu_plan_finalize.  For
    :func:`tile_sharded_search` also the per-(trial, time tile) records and the finalize
    of a trial range (pu_plan_finalize_range)."""

    def __init__(self, plan, out=None, workspace=None, device=None):
        self.plan = plan
        self.out, self.workspace = plan._outs_ws(device, out, workspace)
        self.ntiles = plan.info["time_tiles"]
        self.tt_len = plan.info["time_tile"]
        self.ndm = plan.ndm

    def tile_window(self, tt):
        return self.plan.tile_window(tt)

    def records(self):
        return self.plan.records(self.workspace)

    def finalize_range(self, data, lo, hi, stream=None):
        return self.plan.finalize_range(self.workspace, data, lo, hi, out=self.out, stream=stream)

    def finalize_range_flagged(self, lo, hi, stream=None):
        return self.plan.finalize_range_flagged(self.workspace, lo, hi, out=self.out, stream=stream)

    def exact_series(self, data, trials, t_begin, t_end, stream=None):
        return self.plan.exact_series(data, trials, stream=stream, t_begin=t_begin, t_end=t_end)

    def series_stats(self, series, stream=None):
        from ._hip import series_stats
        return series_stats(series, stream=stream)

    def nonfinite(self, x, stream=None):
        import torch

        from ._hip import nonfinite_any
        flag = torch.zeros(1, dtype=torch.int32, device=x.device)
        return nonfinite_any(x, flag, stream=stream)

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


def interleaved_chunks(nsamples, tt_len, ntiles, world, chunks):
    """Column ranges of :func:`tile_sharded_search`'s exchange: rank q owns time tiles
    ``shard_bounds(ntiles, world, q)`` (columns [t0 tt_len, min(n, t1 tt_len))); chunk k is
    the k-th of ``chunks`` tile-aligned pieces of EVERY rank's slice, so each rank's slice
    lands at the same pace (1 / chunks of it per exchange).  Depends on the shape only (every
    rank issues the same collectives).  Returns the non-empty chunks, each a list of
    (c0, c1)."""
    n, tt = int(nsamples), int(tt_len)
    out = [[] for _ in range(max(1, int(chunks)))]
    for q in range(int(world)):
        t0, t1 = shard_bounds(ntiles, world, q)
        for k in range(len(out)):
            a, b = shard_bounds(t1 - t0, len(out), k)
            c0, c1 = min(n, (t0 + a) * tt), min(n, (t0 + b) * tt)
            if c1 > c0:
                out[k].append((c0, c1))
    return [c for c in out if c]


def ready_by_blocks(landed, tt_len, nsamples, starts, wa, wb):
    """Tiles (first samples ``starts``) whose read window [start + wa, start + wb) - reduced
    modulo nsamples, so a window may wrap - lies in landed column blocks; ``landed[j]``:
    columns [j tt_len, (j + 1) tt_len) have landed."""
    n, tt = int(nsamples), int(tt_len)
    P = np.concatenate([[0], np.cumsum(landed.astype(np.int64))])
    nb = landed.size

    def full(c0, c1):  # columns [c0, c1) within [0, n): every block they touch landed
        b0, b1 = c0 // tt, np.minimum(nb, -(-c1 // tt))
        return (c1 <= c0) | (P[b1] - P[b0] == b1 - b0)

    a = starts + wa
    ln = (starts + wb) - a
    a = np.mod(a, n)
    e = a + ln
    one = full(a, np.minimum(e, n)) & full(np.zeros_like(a), np.maximum(e - n, 0))
    return np.where(ln >= n, bool(landed.all()), one)


def slice_regions(nsamples, tt_len, ntiles, world, wa, wb):
    """Per rank the columns its time tiles read: (A, L) = the union of the windows
    [t tt_len + wa, t tt_len + wb) of its tiles t in shard_bounds(ntiles, world, rank), as an
    unwrapped start A (columns are taken modulo nsamples) and a length L (None: no tiles;
    L = nsamples and A = 0 when the union covers the whole array)."""
    n, tt = int(nsamples), int(tt_len)
    out = []
    for q in range(int(world)):
        t0, t1 = shard_bounds(ntiles, world, q)
        if t1 <= t0:
            out.append(None)
            continue
        a, b = t0 * tt + int(wa), (t1 - 1) * tt + int(wb)
        out.append((0, n) if b - a >= n else (a, b - a))
    return out


def _cols(c0, c1, n):
    """Unwrapped columns [c0, c1) (c1 - c0 <= n) as 1-2 ranges within [0, n)."""
    a = c0 % n
    e = a + (c1 - c0)
    return [(a, e)] if e <= n else [(a, n), (0, e - n)]


def tile_sharded_search(data, plan, out=None, workspace=None, src=0, chunks=8, group=None, searcher=None,
                        collective=DEFAULT_COLLECTIVE, phases=None, full_copy=False):
    """Time-tile sharding: every rank holds the plan of the WHOLE trial grid and searches a
    contiguous range of its time tiles (``shard_bounds(time_tiles, world, rank)``) while the
    filterbank is distributed from ``src`` (None: ``data`` is already complete on every
    rank); the per-(trial, time tile) records then move to the rank that owns each trial
    (``shard_bounds(ndm, world, rank)``, one all_to_all), and each rank finalizes its own
    trials - bit for bit the single-GPU search's result, since every record comes from the
    same kernel and tables and the finalize combines them in the same order.  Returns
    ((max, std, snr, rebin) indexed by plan trial, only [lo, hi) written; (lo, hi)).

    Why: a DM tile's cost is mostly fixed (slot build, DMA, stage skeleton do
    not shrink with its trial count), so splitting the DM grid into world slices adds DM
    tiles (C3: 20 -> 24 at 8 ranks, slowest shard 126 ms against 857 / 8 = 107); splitting
    the time tiles keeps the whole grid's 20 DM tiles, and each rank does 1 / world of them.

    The exchange (``full_copy`` False, default): ``src`` scatters to every rank only the
    columns its tiles read (:func:`slice_regions`: its 1 / world of the samples plus the
    shift halo), in ``chunks`` pieces (:func:`exchange_chunk`'s scatter; ``collective`` is
    not used), each rank's tiles launched as their windows land; ``data`` then holds only
    that region on the receivers.  Trials certification flags are recomputed exactly in
    pieces: every rank computes the float64 channel-order series of the flagged trials at
    its own samples (pu_plan_exact_series), the pieces are all-gathered and each owner takes
    pu_series_stats of its trials' whole series (a non-finite input anywhere - every rank
    scans its own samples - gives every trial the NaN rule, as the one-GPU search).
    ``full_copy`` True: the whole filterbank goes to every rank (:func:`interleaved_chunks`
    by ``collective``: each rank's slice advances by 1 / chunks per exchange) and the
    owner's finalize rechecks from it.
    ``searcher`` (tests): ``ntiles``, ``tt_len``, ``ndm``, ``tile_window(tt)``,
    ``tiles(data, b, e, stream)``, ``records()`` ((ndm, ntiles, R) tensor),
    ``finalize_range(data, lo, hi, stream)`` and, for ``full_copy`` False,
    ``finalize_range_flagged(lo, hi, stream)``, ``exact_series(data, trials, t_begin, t_end, stream)``,
    ``series_stats(series, stream)``, ``nonfinite(x, stream)`` (0-d int tensor)."""
    import contextlib

    import torch
    import torch.distributed as dist
    cuda = data.is_cuda
    dev = data.device
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    if cuda and data.element_size() == 1 and data.shape[1] % 4 == 0 and (data.data_ptr() % 4 or data.stride(0) % 4):
        raise ValueError("tile-sharded search of 8-bit data needs rows starting on 4-byte boundaries")
    if collective not in COLLECTIVES:
        raise ValueError(f"collective must be one of {COLLECTIVES}, got {collective!r}")
    nchan, n = data.shape
    if searcher is None:
        searcher = PlanSearcher(plan, out, workspace, dev)
    ntt, tt = int(searcher.ntiles), int(searcher.tt_len)
    my_t0, my_t1 = shard_bounds(ntt, world, rank)
    my_lo, my_hi = shard_bounds(searcher.ndm, world, rank)
    exchange = world > 1 and src is not None  # src None: data is already on every rank
    sliced = exchange and not full_copy
    if cuda:
        cur = torch.cuda.current_stream(dev)
        comm = torch.cuda.Stream(device=dev)
        comp = torch.cuda.Stream(device=dev)
        comm.wait_stream(cur)
        comp.wait_stream(cur)
    else:
        cur = comm = comp = None
    on_comm = (lambda: torch.cuda.stream(comm)) if cuda else contextlib.nullcontext
    on_comp = (lambda: torch.cuda.stream(comp)) if cuda else contextlib.nullcontext
    wa, wb = searcher.tile_window(0)
    starts = np.arange(ntt, dtype=np.int64) * tt
    mine = np.zeros(ntt, dtype=bool)
    mine[my_t0:my_t1] = True
    done = np.zeros(ntt, dtype=bool)
    if sliced:
        regions = slice_regions(n, tt, ntt, world, wa, wb)
        K = max(1, int(chunks))
        # chunk k: piece k of every rank's region, padded to the widest
        chunk_list = []
        for k in range(K):
            pieces = [None if rg is None else (rg[0] + shard_bounds(rg[1], K, k)[0], rg[0] + shard_bounds(rg[1], K, k)[1])
                      for rg in regions]
            w = max((b - a for pc in pieces if pc is not None for a, b in [pc]), default=0)
            if w > 0:
                chunk_list.append((pieces, w))
        width = max((w for _, w in chunk_list), default=1)
        staging = torch.empty(world * nchan * width, dtype=data.dtype, device=dev) if rank == src else None
        piece = torch.empty(nchan * width, dtype=data.dtype, device=dev)
    else:
        chunk_list = interleaved_chunks(n, tt, ntt, world, chunks if exchange else 1)
        landed = np.zeros(-(-n // tt), dtype=bool)
        width = max(sum(c1 - c0 for c0, c1 in ranges) for ranges in chunk_list)
        slen = -(-nchan * width // world) * world
        staging = torch.empty(slen, dtype=data.dtype, device=dev) if exchange else None
        piece = (torch.empty(slen // world, dtype=data.dtype, device=dev)
                 if exchange and collective == "scatter_allgather" else None)
    for item in chunk_list:
        with on_comm():
            if phases is not None and exchange:
                phases.mark("exchange", comm)
            if sliced:
                pieces, w = item
                m = nchan * w
                if rank == src:
                    for q, pc in enumerate(pieces):
                        if q == src or pc is None:
                            continue  # src keeps its own columns
                        blk = staging[q * m:q * m + nchan * (pc[1] - pc[0])].view(nchan, pc[1] - pc[0])
                        o = 0
                        for c0, c1 in _cols(pc[0], pc[1], n):
                            blk[:, o:o + c1 - c0].copy_(data[:, c0:c1])
                            o += c1 - c0
                dist.scatter(piece[:m], list(staging[:world * m].split(m)) if rank == src else None, src=src,
                             group=group)
                if phases is not None:
                    phases.mark("exchange", comm, end=True)
                    phases.mark("unpack", comm)
                pc = pieces[rank]
                if rank != src and pc is not None:
                    blk = piece[:nchan * (pc[1] - pc[0])].view(nchan, pc[1] - pc[0])
                    o = 0
                    for c0, c1 in _cols(pc[0], pc[1], n):
                        data[:, c0:c1].copy_(blk[:, o:o + c1 - c0])
                        o += c1 - c0
                if phases is not None:
                    phases.mark("unpack", comm, end=True)
            elif exchange:
                ranges = item
                tot = nchan * sum(c1 - c0 for c0, c1 in ranges)
                blen = -(-tot // world) * world
                flat = staging[:blen]
                views, off = [], 0
                for c0, c1 in ranges:
                    views.append((flat[off:off + nchan * (c1 - c0)].view(nchan, c1 - c0), c0, c1))
                    off += nchan * (c1 - c0)
                if rank == src:
                    for v, c0, c1 in views:
                        v.copy_(data[:, c0:c1])
                exchange_chunk(flat, piece[:blen // world] if piece is not None else None, rank, src, world,
                               group=group, collective=collective)
                if phases is not None:
                    phases.mark("exchange", comm, end=True)
                    phases.mark("unpack", comm)
                if rank != src:
                    for v, c0, c1 in views:
                        data[:, c0:c1].copy_(v)
                if phases is not None:
                    phases.mark("unpack", comm, end=True)
            ev = None
            if cuda:
                ev = torch.cuda.Event()
                ev.record(comm)
        if sliced:
            pc, rg = item[0][rank], regions[rank]
            if rank == src:
                ready = np.ones(ntt, dtype=bool)  # the source holds every column from the start
            elif rg is None:
                ready = np.zeros(ntt, dtype=bool)
            elif rg[1] >= n:
                ready = np.full(ntt, pc is not None and pc[1] >= rg[0] + rg[1])
            else:
                top = pc[1] if pc is not None else rg[0]
                ready = starts + wb - starts[0] <= top
        else:
            for c0, c1 in item:
                landed[c0 // tt:-(-c1 // tt)] = True
            ready = ready_by_blocks(landed, tt, n, starts, wa - starts[0], wb - starts[0])
        if cuda:
            comp.wait_event(ev)
        ready = ready & mine & ~done
        idx = np.flatnonzero(ready)
        if phases is not None:
            phases.mark("search", comp)
        for run in np.split(idx, np.flatnonzero(np.diff(idx) != 1) + 1) if idx.size else []:
            searcher.tiles(data, int(run[0]), int(run[-1]) + 1, stream=comp)
        if phases is not None:
            phases.mark("search", comp, end=True)
        done |= ready
    if not done[my_t0:my_t1].all():
        raise RuntimeError("tile-sharded search: time tiles left unsearched")
    if cuda:
        for b in (staging, piece):
            if b is not None:
                b.record_stream(comm)
        comp.wait_stream(comm)
    with on_comp():
        if world > 1:
            # every trial's records of my tiles to the trial's owner; mine from every rank
            if phases is not None:
                phases.mark("records", comp)
            rec = searcher.records()
            R = rec.shape[2]
            tb = [shard_bounds(ntt, world, q) for q in range(world)]
            db = [shard_bounds(searcher.ndm, world, q) for q in range(world)]
            send_parts = [rec[a:b, my_t0:my_t1].reshape(-1) if q != rank else rec.new_empty(0)
                          for q, (a, b) in enumerate(db)]
            in_splits = [p.numel() for p in send_parts]
            out_splits = [0 if q == rank else (my_hi - my_lo) * (t1 - t0) * R for q, (t0, t1) in enumerate(tb)]
            send = torch.cat(send_parts)
            recv = rec.new_empty(sum(out_splits))
            dist.all_to_all_single(recv, send, out_splits, in_splits, group=group)
            off = 0
            for q, (t0, t1) in enumerate(tb):
                if out_splits[q]:
                    rec[my_lo:my_hi, t0:t1].copy_(recv[off:off + out_splits[q]].view(my_hi - my_lo, t1 - t0, R))
                off += out_splits[q]
            if cuda:
                send.record_stream(comp)
                recv.record_stream(comp)
            if phases is not None:
                phases.mark("records", comp, end=True)
        if phases is not None:
            phases.mark("finalize", comp)
        if sliced:
            res = _finalize_sliced(searcher, data, my_lo, my_hi, world, rank, ntt, tt, n, group, comp)
        else:
            res = searcher.finalize_range(data, my_lo, my_hi, stream=comp)
        if phases is not None:
            phases.mark("finalize", comp, end=True)
    if cuda:
        if hasattr(searcher, "streams_done"):
            searcher.streams_done(comp)
        cur.wait_stream(comm)
        cur.wait_stream(comp)
    return res, (my_lo, my_hi)


def _finalize_sliced(searcher, data, lo, hi, world, rank, ntt, tt, n, group, stream):
    """The owner's finalize when each rank holds only its time slice: the fast statistics
    and the flagged trials (pu_plan_finalize_range_flagged), then - collectively, in the
    same order on every rank - the NaN rule or the exact recomputation of every rank's
    flagged trials from the ranks' series pieces (pu_plan_exact_series of the own samples
    [t0 tt, t1 tt) only, all_gather, pu_series_stats by the owner).  Matches resolve_flagged's
    decisions (csrc/dedisperse.hip) bit for bit."""
    import torch
    import torch.distributed as dist
    dev = data.device
    out, flagged, nnf = searcher.finalize_range_flagged(lo, hi, stream=stream)
    cnt = torch.tensor([len(flagged), nnf], dtype=torch.int64, device=dev)
    allc = torch.empty(world * 2, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(allc, cnt, group=group)
    allc = allc.view(world, 2).cpu().numpy()
    if allc[:, 0].sum() == 0:
        return out
    s0, s1 = (min(n, b * tt) for b in shard_bounds(ntt, world, rank))
    if allc[:, 1].sum() > 0:
        # a non-finite partial somewhere: does the input hold NaN / inf (each rank its samples)?
        flag = searcher.nonfinite(data[:, s0:s1], stream=stream).to(torch.int64).reshape(1)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
        if int(flag.item()):
            # every trial holds every sample: max = std = NaN, snr = 0, rebin = 0 (as nan_rule)
            out[0][lo:hi] = float("nan")
            out[1][lo:hi] = float("nan")
            out[2][lo:hi] = 0.0
            out[3][lo:hi] = 0
            return out
    mf = int(allc[:, 0].max())
    mine = torch.full((mf,), -1, dtype=torch.int64, device=dev)
    if len(flagged):
        mine[:len(flagged)] = torch.as_tensor(flagged.astype(np.int64), device=dev)
    allf = torch.empty(world * mf, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(allf, mine, group=group)
    allf = allf.cpu().numpy()
    G = allf[allf >= 0].astype(np.int32)  # owners in rank order, each ascending
    spans = [tuple(min(n, b * tt) for b in shard_bounds(ntt, world, q)) for q in range(world)]
    wmax = max(b - a for a, b in spans)
    B = max(1, (1 << 28) // (8 * max(n, wmax * world)))
    for b0 in range(0, G.size, B):
        trials = G[b0:b0 + B]
        m = trials.size
        pc = torch.zeros((m, wmax), dtype=torch.float64, device=dev)
        if s1 > s0:
            pc[:, :s1 - s0] = searcher.exact_series(data, trials, s0, s1, stream=stream)  # my samples [s0, s1)
        allp = torch.empty((world * m, wmax), dtype=torch.float64, device=dev)
        dist.all_gather_into_tensor(allp, pc, group=group)
        allp = allp.view(world, m, wmax)
        own = np.flatnonzero((trials >= lo) & (trials < hi))
        if own.size == 0:
            continue
        full = torch.empty((own.size, n), dtype=torch.float64, device=dev)
        sel = torch.as_tensor(own, device=dev)
        for q, (a, b) in enumerate(spans):
            if b > a:
                full[:, a:b] = allp[q].index_select(0, sel)[:, :b - a]
        st = searcher.series_stats(full, stream=stream)
        for k in range(4):
            out[k][torch.as_tensor(trials[own].astype(np.int64), device=dev)] = st[k]
    return out


DECOMPOSITIONS = ("dm", "time")


def sharded_search(data, trial_DMs, nchan, start_freq, bandwidth, sample_time, group=None, acc=None,
                   compute=None, broadcast=True, src=0, pipelined=False, chunks=8, collective=DEFAULT_COLLECTIVE,
                   decomposition="dm"):
    """Distributed ``_dedispersion_search``: returns (max, std, snr, rebin[int32]) numpy arrays
    covering ALL trials, on every rank.

    ``data`` must be a tensor of the right shape/dtype on every rank (only ``src``'s
    content matters when ``broadcast``).  ``pipelined`` (HIP compute only) overlaps the
    transfer with the search (:func:`pipelined_broadcast_search`); ``collective`` picks
    the transfer (:func:`exchange_chunk`: ``"broadcast"`` or ``"scatter_allgather"``).
    ``decomposition`` (with ``pipelined``): ``"dm"`` - each rank plans and searches its
    contiguous trial slice; ``"time"`` - every rank plans the whole grid, searches a slice of
    its time tiles and finalizes its trial slice (:func:`tile_sharded_search`).  Both
    return the same bits.
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
    if decomposition not in DECOMPOSITIONS:
        raise ValueError(f"decomposition must be one of {DECOMPOSITIONS}, got {decomposition!r}")
    if decomposition == "time" and not (pipelined and compute is None):
        raise ValueError("decomposition='time' needs the pipelined HIP search (pipelined=True, compute=None)")
    if decomposition == "time":
        from . import _hip
        from .dedispersion import _acc_code, _plan_for, _prepare_data
        if not (data.is_cuda and data.is_contiguous()):
            raise ValueError("pipelined sharded_search needs a contiguous device tensor (it is written in place)")
        x = _prepare_data(data)
        plan = _plan_for(x, lambda: _hip.shift_table(nchan, dms, start_freq, bandwidth, sample_time),
                         _acc_code(acc), ("dm-grid", dms.tobytes(), float(start_freq), float(bandwidth),
                                          float(sample_time)))
        res, (a, b) = tile_sharded_search(x, plan, src=src if broadcast else None, chunks=chunks, group=group,
                                          collective=collective)
        for k in range(4):
            local[k, :hi - lo] = res[k][lo:hi].to(torch.float64)
    elif pipelined and compute is None:
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
