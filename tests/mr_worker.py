"""One rank of tests/test_gpu_multirank.py (not collected by pytest: no ``test_`` prefix).

    python tests/mr_worker.py RANK WORLD PORT CASE [COLLECTIVE [DECOMPOSITION]]

Every rank runs on cuda:0 of the one leased GPU with a ``gloo`` process group (RCCL
refuses two ranks on one device; gloo's CUDA broadcast / all_gather stage device
tensors through host memory on the calling stream).  The multi-rank branch of the
product path then runs for real on the GPU: the chunked broadcast on the communication
stream, the staging pack / unpack, the events that gate the time-tile launches on the
compute stream, pu_plan_search_tiles + pu_plan_finalize on the real HIP plan, and the
all_gather of sharded_search.  ``src`` is the LAST rank (not 0); the other ranks start
from garbage.  Checks (bit for bit):
  * pipelined_broadcast_search on every rank == plan.search of the full grid on the
    full data, and the received filterbank == the source's;
  * sharded_search(pipelined=True) == the concatenation of the single-rank
    _dedispersion_search of each rank's trial slice (the same plans);
  * CASE C5m: the same with reserve_cus=8 (the CU-masked compute stream), outputs freed
    afterwards (the masked stream must outlive the tensors recorded on it).
MR_BACKEND=nccl (environment): an RCCL process group instead (WORLD 1 on the one GPU: the
RCCL calls of the product path - broadcast on the communication stream, all_gather,
barrier - with a single rank).
COLLECTIVE (default broadcast): the chunk exchange of parallel.exchange_chunk -
``broadcast`` or ``scatter_allgather`` (the mesh variant, round 5).
DECOMPOSITION (default dm): ``time`` checks parallel.tile_sharded_search instead (each rank
its time tiles of the whole grid's plan, the records all_to_all, pu_plan_finalize_range):
every rank's trial slice == the one-GPU search of the grid, and sharded_search(decomposition
="time") == that search on every rank.
Prints ``RANK r OK`` and exits 0, or raises (non-zero exit, traceback on stderr).
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path[:0] = [os.path.join(REPO, "radio-pulsar-utils_amd"), REPO]


def main():
    rank, world, port, case = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    collective = sys.argv[5] if len(sys.argv) > 5 else "broadcast"
    decomposition = sys.argv[6] if len(sys.argv) > 6 else "dm"
    from dataclasses import replace

    import numpy as np
    import torch
    import torch.distributed as dist

    from pulsarutils import _hip, parallel, synth
    from pulsarutils import dedispersion as D
    from pulsarutils.configs import CONFIGS

    torch.cuda.set_device(0)
    backend = os.environ.get("MR_BACKEND", "gloo")  # nccl (RCCL): one rank per GPU only
    if backend == "nccl":
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                                device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    src = world - 1
    c, ntrials, chunks, reserve = {
        "C5": (CONFIGS["C5"], 500, 5, 0),
        "C5m": (CONFIGS["C5"], 500, 4, 8),
        "C3s": (replace(CONFIGS["C3"], nchan=512, nsamples=1 << 18), 625, 3, 0),
        # degenerate inputs (time decomposition): all-zero 8-bit data (every trial flagged:
        # std 0) and float32 data with one NaN (the NaN rule for every trial)
        "C3z": (replace(CONFIGS["C3"], nchan=512, nsamples=1 << 18), 100, 3, 0),
        "C5n": (CONFIGS["C5"], 500, 5, 0),
    }[case]
    x_ref = synth.pulsar_filterbank_device(c)  # deterministic: the same bytes on every rank
    if case == "C3z":
        x_ref.zero_()
    elif case == "C5n":
        x_ref[7, c.nsamples // 3 + 5] = float("nan")
    full = D.dedispersion_plan(c.nchan, c.dmmin, c.dmmax, c.start_freq, c.bandwidth, c.tsamp)
    dms = full[:ntrials]
    garbage = 255 if x_ref.dtype == torch.uint8 else float("nan")

    def same(a, b):  # bit-equal tensors, NaN == NaN
        if a.is_floating_point():
            return bool(((a == b) | (a.isnan() & b.isnan())).all())
        return torch.equal(a, b)

    def received():
        return x_ref.clone() if rank == src else torch.full_like(x_ref, garbage)

    # ---- pipelined broadcast + search of the full grid on every rank
    sh = _hip.shift_table(c.nchan, dms, c.start_freq, c.bandwidth, c.tsamp)
    plan = _hip.Plan(_hip.dtype_code(x_ref.dtype), _hip.PU_ACC_NATIVE, c.nchan, c.nsamples, sh)
    ref = [o.cpu().numpy() for o in plan.search(x_ref)]
    if decomposition == "time":
        # ---- time-tile sharding: each rank its time tiles of the whole grid, records to the
        # trial owners, finalize of the own trials == the one-GPU search of the grid; with the
        # whole filterbank sent to every rank (full_copy) and with each rank's region only
        # (flagged trials settled from the ranks' series pieces)
        rechecked = plan.cert_info()["rechecked"]
        for full_copy in (True, False):
            x = received()
            res, (lo, hi) = parallel.tile_sharded_search(x, plan, src=src, chunks=chunks, collective=collective,
                                                         full_copy=full_copy)
            torch.cuda.synchronize()
            if full_copy:
                assert same(x, x_ref), f"rank {rank}: received filterbank differs (time)"
            else:
                a, ln = parallel.slice_regions(c.nsamples, plan.info["time_tile"], plan.info["time_tiles"], world,
                                               *plan.tile_window(0))[rank]
                cols = torch.as_tensor(np.arange(a, a + ln) % c.nsamples, device=x.device)
                assert same(x[:, cols], x_ref[:, cols]), f"rank {rank}: region differs (time, sliced)"
            assert (lo, hi) == parallel.shard_bounds(dms.size, world, rank)
            for k, (a_, b_) in enumerate(zip(ref, res)):
                np.testing.assert_array_equal(a_[lo:hi], b_[lo:hi].cpu().numpy(),
                                              err_msg=f"rank {rank} time output {k} full_copy {full_copy}")
            del res, x
        x2 = received()
        mx, sd, snr, win = parallel.sharded_search(x2, dms, c.nchan, c.start_freq, c.bandwidth, c.tsamp,
                                                   pipelined=True, src=src, chunks=chunks, collective=collective,
                                                   decomposition="time")
        torch.cuda.synchronize()
        for k, got_k in enumerate((mx, sd, snr, win)):
            np.testing.assert_array_equal(got_k, ref[k], err_msg=f"rank {rank} sharded time output {k}")
        print(f"rank {rank}: one-GPU search rechecked {rechecked} trials", flush=True)
        best = int(np.argmax(snr))
        dist.barrier()
        dist.destroy_process_group()
        print(f"RANK {rank} OK case {case} world {world} {backend} {collective} time best DM {dms[best]:.3f} "
              f"snr {snr[best]:.3f}", flush=True)
        return
    x = received()
    res = parallel.pipelined_broadcast_search(x, plan, src=src, chunks=chunks, reserve_cus=reserve,
                                              collective=collective)
    got = [o.cpu().numpy() for o in res]
    torch.cuda.synchronize()
    assert torch.equal(x, x_ref), f"rank {rank}: received filterbank differs"
    for k, (a, b) in enumerate(zip(ref, got)):
        np.testing.assert_array_equal(a, b, err_msg=f"rank {rank} pipelined output {k}")
    del res, got, x
    torch.cuda.synchronize()
    torch.cuda.empty_cache()  # frees the tensors recorded on the (kept) masked stream

    # ---- sharded search (each rank its trial slice, all_gather of the statistics)
    x2 = received()
    mx, sd, snr, win = parallel.sharded_search(x2, dms, c.nchan, c.start_freq, c.bandwidth, c.tsamp,
                                               pipelined=True, src=src, chunks=chunks, collective=collective)
    torch.cuda.synchronize()
    assert torch.equal(x2, x_ref), f"rank {rank}: received filterbank differs (sharded)"
    parts = []
    for r in range(world):
        lo, hi = parallel.shard_bounds(dms.size, world, r)
        if hi > lo:
            parts.append(D._dedispersion_search(x_ref, dms[lo:hi], c.nchan, c.start_freq, c.bandwidth, c.tsamp))
    for k, got_k in enumerate((mx, sd, snr, win)):
        np.testing.assert_array_equal(got_k, np.concatenate([p[k] for p in parts]),
                                      err_msg=f"rank {rank} sharded output {k}")
    assert win.dtype == np.int32
    best = int(np.argmax(snr))
    assert ntrials < full.size or abs(dms[best] - c.pulse_dm) < 1.0, (dms[best], c.pulse_dm)
    dist.barrier()
    dist.destroy_process_group()
    print(f"RANK {rank} OK case {case} world {world} {backend} {collective} best DM {dms[best]:.3f} snr {snr[best]:.3f}", flush=True)


if __name__ == "__main__":
    main()
