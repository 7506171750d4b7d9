"""DM-trial sharding across GPUs (one process per GPU, torch.distributed over RCCL/xGMI).

The reference's only parallelism is numba ``prange`` over independent DM trials
(``dedispersion.py:174,181``).  Here the same trial axis is split across ranks:

1. the filterbank is broadcast from ``src`` (RCCL over xGMI; one collective, the
   data path of the search itself has no other exchange),
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


def broadcast_filterbank(data, src=0, group=None):
    """Broadcast the (nchan, N) filterbank tensor from ``src`` to every rank, in place."""
    import torch.distributed as dist
    dist.broadcast(data, src=src, group=group)
    return data


def sharded_search(data, trial_DMs, nchan, start_freq, bandwidth, sample_time, group=None, acc=None,
                   compute=None, broadcast=True, src=0):
    """Distributed ``_dedispersion_search``: returns (max, std, snr, rebin[int32]) numpy arrays
    covering ALL trials, on every rank.

    ``data`` must be a tensor of the right shape/dtype on every rank (only ``src``'s
    content matters when ``broadcast``).
    """
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if broadcast and world > 1:
        broadcast_filterbank(data, src=src, group=group)
    dms = np.asarray(trial_DMs, dtype=np.float64)
    lo, hi = shard_bounds(dms.size, world, rank)
    fn = compute or (lambda d, t: _hip_compute(d, t, nchan, start_freq, bandwidth, sample_time, acc))
    dev = data.device
    chunk = -(-dms.size // world)  # ceil: equal-size gather buffers
    local = torch.zeros((4, chunk), dtype=torch.float64, device=dev)
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
