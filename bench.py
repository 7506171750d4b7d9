"""Benchmark: dedispersed DM-trial samples/s on the C2 config (BASELINE.json configs[1]).

One "step" = one fused DM-trial search (pu_plan_search: shift-and-sum over all
channels for every trial + the S/N epilogue + the per-trial finalize) over a
1024-channel x 2^20-sample float32 filterbank resident in HBM, 1000 trials per GPU.

Scaling (one process per GPU, torchrun; DM trials are independent: the one exchange on
the data path is the filterbank's distribution from rank 0 - DESIGN.md §5):
* N = 1 (default): C2, 1000 trials, the filterbank resident in HBM.
* N > 1 (default): BASELINE.json configs[2] as stated - C3 (4096 chan x 2^22 uint8,
  17.2 GB) held by rank 0, its 5000 trials searched by the N ranks together
  (``--scaling strong``).  ``--decomposition time`` (default, round 6): every rank searches
  its 1/N of the time tiles for all 5000 trials (the whole grid's 20 DM tiles, where N DM
  slices would add DM tiles whose fixed cost does not shrink with their trial count,
  DESIGN.md §5), the per-(trial, tile) records go to the trial owners (one all_to_all) and
  each rank finalizes its 5000 / N trials; ``dm``: each rank searches its contiguous DM
  slice (625 trials at N = 8).  One timed step is the whole job: the filterbank
  distributed from rank 0 in time chunks (``--collective``, default scatter + all-gather
  over the xGMI mesh) with each rank's search of its tiles whose rows have landed
  overlapping the later chunks, the finalize, and the all_gather of the per-trial
  (max, std, snr, rebin).  ``value`` = 5000 x 2^22 / step.
* ``--scaling weak``: the DM grid is N x ``ntrials`` trials of ``--config`` (C2), rank r
  owns trials [r ntrials, (r+1) ntrials); the filterbank is distributed before timing.
``multi_gpu`` (N > 1) reports the whole-filterbank exchange alone and one pipelined
step per collective (``broadcast`` and ``scatter_allgather``).

Prints ONE JSON line (rank 0) with the driver's contract fields plus ``roofline``
(dominant kernel, HIP events on its launch stream; HBM counter traffic from the PMC
summary committed under profiles/), ``clean`` (the C4 cleaning pass, configs[3]) and
``cpu_baseline`` (the C oracle = a port of the reference's numba search, OpenMP over
trials, timed on a bounded trial sample on the host's cores).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(REPO, "radio-pulsar-utils_amd"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from pulsarutils import _hip, synth  # noqa: E402
from pulsarutils.configs import CONFIGS  # noqa: E402
from pulsarutils.dedispersion import dedispersion_plan  # noqa: E402
from pulsarutils.parallel import pipelined_broadcast_search, shard_bounds, tile_sharded_search  # noqa: E402

# MI355X peaks (/opt/skills/guides/MI355X_MICROARCH.md, chip-level parameters)
HBM_PEAK_GBS = 8000.0
# float32 vector peak is 157.3 TFLOP/s counting an FMA as 2 FLOP; an add is one FLOP
# per lane-op, so the add-only ceiling is half of it: 256 CU x 128 lanes/clk x 2.4 GHz
VALU_ADD_PEAK_TFLOPS = 78.6
# float64 vector peak 78.6 TFLOP/s (FMA = 2 FLOP) -> 39.3 T float64 adds/s
VALU_F64_ADD_PEAK_TFLOPS = 39.3
# LDS: 256 B/clk/CU for ds_read_b64 (MI355X_MICROARCH.md §LDS) x 256 CUs x 2.4 GHz
LDS_PEAK_TBPS = 157.3


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_threads():
    """Threads for the CPU baseline: every CPU this process may run on (its affinity
    mask), capped by OMP_NUM_THREADS when the host sets it (the GPU box allots a
    CPU share per GPU and exports OMP_NUM_THREADS for it)."""
    avail = len(os.sched_getaffinity(0))
    env = os.environ.get("BENCH_CPU_THREADS") or os.environ.get("OMP_NUM_THREADS")
    return max(1, min(avail, int(env))) if env else avail


def cpu_baseline(x_host, dms, cfg, ntrials, threads, reps=3):
    """The C oracle (a port of the reference's numba prange search: float64, OpenMP over
    trials) on ``ntrials`` evenly spaced trials of the same filterbank, ``reps`` times;
    the median run is the value, the spread is reported beside it."""
    # OpenMP placement must be in the environment before libgomp initialises
    os.environ.setdefault("OMP_PROC_BIND", "close")
    os.environ.setdefault("OMP_PLACES", "cores")
    import oracle
    ntrials = min(ntrials, dms.size)
    sel = dms[np.linspace(0, dms.size - 1, ntrials).astype(int)]
    oracle.search(x_host[:, :4096], sel[:2], cfg.start_freq, cfg.bandwidth, cfg.tsamp, nthreads=threads)
    runs = []
    for _ in range(max(1, reps)):
        t0 = time.perf_counter()
        oracle.search(x_host, sel, cfg.start_freq, cfg.bandwidth, cfg.tsamp, nthreads=threads)
        runs.append(ntrials * cfg.nsamples / (time.perf_counter() - t0))
    med = float(np.median(runs))
    return {"value": med, "unit": "DM-trial samples/s", "cores": threads,
            "kind": "port", "cpu_model": cpu_model(), "host_cpus": os.cpu_count(),
            "runs": [round(r, 1) for r in runs], "spread": round((max(runs) - min(runs)) / med, 4),
            "omp": {"OMP_PROC_BIND": os.environ.get("OMP_PROC_BIND"), "OMP_PLACES": os.environ.get("OMP_PLACES")},
            "sample": f"{ntrials} of the {dms.size} {cfg.name} trials (evenly spaced), full "
                      f"{cfg.nchan}x2^{int(np.log2(cfg.nsamples))} {cfg.dtype} filterbank, float64 "
                      f"oracle/dedisp_oracle.c (numba prange -> OpenMP over trials), median of {len(runs)} runs "
                      f"of {ntrials * cfg.nsamples / med:.1f} s"}


def load_pmc(tag):
    """Per-launch HBM bytes of the dominant kernel from the committed PMC summary
    ``profiles/pmc_<tag>.json``, and whether it was collected from the kernel source this
    library was built from (the summary records the SHA-256 of csrc/dedisperse.hip)."""
    path = os.path.join(REPO, "profiles", f"pmc_{tag}.json")
    if not os.path.exists(path):
        return None, False
    try:
        pmc = json.load(open(path))
    except (OSError, ValueError):
        return None, False
    same = pmc.get("dedisperse_hip_sha256") == _hip.source_hashes().get("csrc/dedisperse.hip")
    return pmc, same


def load_sq(tag, srcfile="csrc/dedisperse.hip"):
    """The dominant kernel's SQ counter summary ``profiles/sq_<tag>.json`` (scripts/sq_json.py:
    LDS-array cycles / CU cycles etc.) if it was collected from the kernel source this library
    was built from, else None."""
    path = os.path.join(REPO, "profiles", f"sq_{tag}.json")
    try:
        sq = json.load(open(path))
    except (OSError, ValueError):
        return None
    return sq if sq.get("source_sha256") == _hip.source_hashes().get(srcfile) else None


def sq_fields(sq, tag):
    if not sq:
        return {"lds_cycle_frac": None,
                "lds_cycle_note": f"profiles/sq_{tag}.json absent or collected from another kernel source"}
    return {"lds_cycle_frac": sq["lds_cycle_frac"], "lds_bank_conflict_frac": sq.get("lds_bank_conflict_frac"),
            "insts_per_cu_cycle": sq.get("per_cu_cycle"),
            "lds_cycle_source": f"profiles/sq_{tag}.json (SQ_LDS_IDX_ACTIVE / (256 CUs x GRBM_GUI_ACTIVE/8), "
                                f"kernel {sq.get('kernel_ms_at_collection')} ms at collection)"}


def knob_env():
    """Every PU_* / PULSARUTILS_* variable: tuning knobs that reshape the kernels or the
    library loaded (a bench line is only valid with none set)."""
    return {k: v for k, v in sorted(os.environ.items()) if k.startswith(("PU_", "PULSARUTILS_"))}


def clean_bench(dev, steps):
    """The C4 cleaning pass (configs[3], clean.py:58-133) on device-resident data: the
    channel masks and renormalize_data(cut_outliers=True) per input dtype."""
    from pulsarutils import clean
    cfg = CONFIGS["C4"]
    res = {"workload": f"C4: {cfg.nchan} chan x 2^{int(np.log2(cfg.nsamples))} RFI filterbank, "
                       "get_noisier_channels + measure_channel_variability + "
                       "renormalize_data(cut_outliers=True)", "steps": steps}
    for dt in ("f32", "u8"):
        xd = torch.from_numpy(synth.rfi_filterbank_np(cfg, dtype=dt)).to(dev)
        b_in = xd.element_size()
        out = torch.empty(xd.shape, dtype=torch.float64, device=dev)

        def masks():
            # every step from scratch: the channel-means cache (kept per tensor version so
            # that measure_channel_variability reuses get_noisier_channels' pass) would
            # otherwise skip the mean pass of every step after the first
            clean.invalidate_channel_means()
            bad = clean.get_noisier_channels(xd)
            return clean.measure_channel_variability(xd, badchans_mask=bad), bad

        def renorm(bad):
            return clean.renormalize_device(xd, badchans_mask=bad, cut_outliers=True, out=out)

        var, bad = masks()
        renorm(bad)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            masks()
        torch.cuda.synchronize()
        t_mask = (time.perf_counter() - t0) / steps * 1e3
        t0 = time.perf_counter()
        for _ in range(steps):
            _, bins = renorm(bad)
        torch.cuda.synchronize()
        t_ren = (time.perf_counter() - t0) / steps * 1e3
        n_el = float(cfg.nchan) * cfg.nsamples
        # algorithmic bytes of renormalize(cut_outliers): the zero-DM column pass, the
        # per-channel mean of x*f and the apply pass each read x once; the apply pass
        # writes the float64 plane (1-D vectors and the zeroed columns are negligible)
        alg = n_el * (3 * b_in + 8)
        # one read pass: the means and the shifted moments come from the same pass and the
        # std decisions are certified from them (a second, exact pass only when one is
        # within its rounding bound: not at C4)
        mask_bytes = n_el * b_in
        res[dt] = {"masks_ms": round(t_mask, 4), "renormalize_ms": round(t_ren, 4),
                   "renormalize_alg_bytes": alg,
                   "renormalize_GBps": round(alg / t_ren / 1e6, 1),
                   "renormalize_hbm_frac": round(alg / t_ren / 1e6 / HBM_PEAK_GBS, 4),
                   "masks_alg_bytes": mask_bytes,
                   "masks_hbm_frac": round(mask_bytes / t_mask / 1e6 / HBM_PEAK_GBS, 4),
                   "bad_channels": int(bad.sum()), "variable_channels": int(var.sum()),
                   "bad_bins": int(bins.sum().item())}
        del xd, out
        torch.cuda.empty_cache()
    res["roofline"] = {"bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s",
                       "achieved": res["f32"]["renormalize_GBps"], "frac": res["f32"]["renormalize_hbm_frac"],
                       "what": "f32 renormalize_data(cut_outliers=True) end to end (host steps included)"}
    return res


def acc_f64_bench(x, dms, cfg, steps):
    """The reference-precision search on the headline workload: the same C2 filterbank and
    trials with float64 accumulation in channel order (dedisp_kernel; the series of every
    trial is the reference's dedisperse() bit for bit, dedispersion.py:86-98), as the
    drop-in's dedisperse / show=True / search_by_chunks defaults run it.  Roofline: the
    float64 vector-add peak, and the LDS array (window reads + staged rows)."""
    sh = _hip.shift_table(cfg.nchan, dms, cfg.start_freq, cfg.bandwidth, cfg.tsamp)
    plan = _hip.Plan(_hip.dtype_code(x.dtype), _hip.PU_ACC_F64, cfg.nchan, cfg.nsamples, sh)
    ws = torch.empty(plan.workspace_bytes, dtype=torch.uint8, device=x.device)
    outs = plan._outs_ws(x.device, None, ws)[0]
    plan.search(x, out=outs, workspace=ws)  # warm-up
    torch.cuda.synchronize()
    plan.enable_timing(steps)
    t0 = time.perf_counter()
    for _ in range(steps):
        plan.search(x, out=outs, workspace=ws)
    torch.cuda.synchronize()
    step_ms = (time.perf_counter() - t0) / steps * 1e3
    kms = float(np.mean(plan.kernel_times_ms(steps)))
    adds = float(cfg.nchan) * cfg.nsamples * dms.size
    info = plan.info
    lds = info["lds_traffic"] / (kms / 1e3) / 1e12
    res = {"workload": f"{cfg.name} ({dms.size} trials), float64 accumulation in channel order (acc='f64')",
           "kernel": _hip.KERNEL_NAMES[info["kernel"]], "steps": steps, "ms_per_step": round(step_ms, 4), "kernel_ms": round(kms, 4),
           "value": dms.size * cfg.nsamples / (step_ms / 1e3), "unit": "DM-trial samples/s",
           "roofline": {"bound": "valu", "achieved": round(adds / (kms / 1e3) / 1e12, 3),
                        "peak": VALU_F64_ADD_PEAK_TFLOPS, "unit": "TFLOP/s (f64 adds)",
                        "frac": round(adds / (kms / 1e3) / 1e12 / VALU_F64_ADD_PEAK_TFLOPS, 4),
                        "lds_bytes_per_launch": info["lds_traffic"], "lds_achieved_TBps": round(lds, 2),
                        "lds_peak_TBps": LDS_PEAK_TBPS, "lds_frac": round(lds / LDS_PEAK_TBPS, 4),
                        **sq_fields(load_sq("C2_f64", "csrc/dedisp_f64.hip"), "C2_f64")},
           "plan": {k: info[k] for k in ("dm_tiles", "time_tiles", "trials_per_tile", "time_tile", "chans_per_step",
                                         "lds_bytes")},
           "best_dm": float(dms[int(torch.argmax(outs[2]).item())]), "certify": plan.cert_info()}
    del plan, ws, outs
    torch.cuda.empty_cache()
    return res


def c3_strong(dev, world, rank, steps, chunks):
    """configs[2] as BASELINE states it: the C3 filterbank (4096 chan x 2^22 uint8, 17.2 GB)
    with its 5000 DM trials split contiguously over the N ranks (strong scaling).
    ``compute_ms``: one search of every rank's slice on resident data (barrier + sync on
    both sides, max over ranks); with N > 1 also the plain RCCL broadcast of the
    filterbank and the chunked broadcast pipelined with the search (``end_to_end_ms``)."""
    from pulsarutils.parallel import pipelined_broadcast_search
    cfg = CONFIGS["C3"]
    dms_all = dedispersion_plan(cfg.nchan, cfg.dmmin, cfg.dmmax, cfg.start_freq, cfg.bandwidth, cfg.tsamp)
    lo, hi = shard_bounds(dms_all.size, world, rank)
    dms = dms_all[lo:hi]
    if rank == 0:
        x = synth.pulsar_filterbank_device(cfg, device=dev)
    else:
        x = torch.empty((cfg.nchan, cfg.nsamples), dtype=torch.uint8, device=dev)
    sh = _hip.shift_table(cfg.nchan, dms, cfg.start_freq, cfg.bandwidth, cfg.tsamp)
    plan = _hip.Plan(_hip.PU_U8, _hip.PU_ACC_NATIVE, cfg.nchan, cfg.nsamples, sh)
    ws = torch.empty(plan.workspace_bytes, dtype=torch.uint8, device=dev)
    outs = plan._outs_ws(dev, None, ws)[0]
    torch.cuda.synchronize()

    def timed(fn):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        ms = torch.tensor([(time.perf_counter() - t0) * 1e3], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(ms, op=dist.ReduceOp.MAX)
        return float(ms.item())

    res = {"workload": f"C3: {cfg.nchan} chan x 2^22 u8 samples, {dms_all.size} DM trials split over {world} GPU(s)",
           "scaling": "strong", "trials_per_gpu": int(hi - lo), "group": plan.info["group"], "steps": steps}
    if world > 1:
        res["broadcast_ms"] = timed(lambda: dist.broadcast(x, src=0))
        res["end_to_end_ms"] = timed(lambda: pipelined_broadcast_search(x, plan, outs, ws, src=0, chunks=chunks))
        res["end_to_end_samples_per_s"] = dms_all.size * cfg.nsamples / (res["end_to_end_ms"] / 1e3)
        res["bcast_chunks"] = chunks
    plan.search(x, out=outs, workspace=ws)  # warm-up
    plan.enable_timing(steps)

    def search_steps():
        for _ in range(steps):
            plan.search(x, out=outs, workspace=ws)

    res["compute_ms"] = timed(search_steps) / steps
    kms = plan.kernel_times_ms(steps)
    res["kernel_ms_rank0"] = float(np.mean(kms)) if len(kms) else None
    res["value"] = dms_all.size * cfg.nsamples / (res["compute_ms"] / 1e3)
    res["unit"] = "DM-trial samples/s"
    snr = outs[2].clone()
    if world > 1:
        chunk = -(-dms_all.size // world)
        loc = torch.full((chunk,), -1.0, dtype=torch.float64, device=dev)
        loc[:hi - lo] = snr
        allv = torch.empty(world * chunk, dtype=torch.float64, device=dev)
        dist.all_gather_into_tensor(allv, loc)
        allv = allv.view(world, chunk)
        snr = torch.cat([allv[r, :shard_bounds(dms_all.size, world, r)[1] - shard_bounds(dms_all.size, world, r)[0]]
                         for r in range(world)])
    res["best_dm"] = float(dms_all[int(torch.argmax(snr).item())])
    res["certify"] = plan.cert_info()
    del x, ws, outs, plan
    torch.cuda.empty_cache()
    return res


def exchange_bench(x, plan, outs, ws, dev, chunks, decomposition="dm"):
    """N > 1: the whole filterbank distributed from rank 0 by each collective alone
    (``*_ms``, ``*_GBps`` = bytes / time), then one pipelined step per collective (chunked
    exchange + the search of each time tile as soon as its rows and halo landed +
    finalize: ``end_to_end_ms``).  Barrier + sync on both sides, max over ranks."""
    from pulsarutils.parallel import COLLECTIVES, broadcast_filterbank, pipelined_broadcast_search

    def timed(fn):
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        dist.barrier()
        ms = torch.tensor([(time.perf_counter() - t0) * 1e3], dtype=torch.float64, device=dev)
        dist.all_reduce(ms, op=dist.ReduceOp.MAX)
        return round(float(ms.item()), 3)

    nbytes = x.numel() * x.element_size()
    res = {"bytes": nbytes, "bcast_chunks": chunks, "end_to_end_ms": {},
           "what": "<collective>_ms: the whole filterbank from rank 0 by that exchange alone; end_to_end_ms: one "
                   "chunked exchange pipelined with the search (each time tile launched once its rows and halo "
                   "landed) and the finalize - per collective with the whole filterbank to every rank, and "
                   "(time split) 'sliced': each rank receives only the columns its time tiles read"}
    for c in COLLECTIVES:
        timed(lambda: broadcast_filterbank(x, src=0, collective=c))  # warm-up (communicator setup)
        ms = timed(lambda: broadcast_filterbank(x, src=0, collective=c))
        res[f"{c}_ms"] = ms
        res[f"{c}_GBps"] = round(nbytes / ms / 1e6, 1)
    for c in COLLECTIVES:
        if decomposition == "time":
            fn = (lambda: tile_sharded_search(x, plan, outs, ws, src=0, chunks=chunks, collective=c, full_copy=True))
        else:
            fn = (lambda: pipelined_broadcast_search(x, plan, outs, ws, src=0, chunks=chunks, collective=c))
        res["end_to_end_ms"][c] = timed(fn)
    if decomposition == "time":
        # the default time split: each rank receives only the columns its tiles read
        res["end_to_end_ms"]["sliced"] = timed(lambda: tile_sharded_search(x, plan, outs, ws, src=0, chunks=chunks))
    if decomposition == "time":
        t0, t1 = shard_bounds(plan.info["time_tiles"], dist.get_world_size(), dist.get_rank())
        res["search_only_ms"] = timed(lambda: plan.search_tiles(x, t0, t1, ws))
        res["search_only_what"] = "each rank's time tiles of the whole grid (pu_plan_search_tiles), resident data"
    else:
        res["search_only_ms"] = timed(lambda: plan.search(x, out=outs, workspace=ws))
    res["decomposition"] = decomposition
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default=None, help="default: C2 on one GPU, C3 (configs[2]) on N > 1")
    ap.add_argument("--acc", default="native", choices=["native", "f32", "f64"])
    ap.add_argument("--scaling", default=None, choices=["weak", "strong"],
                    help="default: weak (one GPU: the single-GPU workload), strong on N > 1")
    ap.add_argument("--collective", default="scatter_allgather", choices=["broadcast", "scatter_allgather"],
                    help="N > 1: the chunk exchange inside the timed strong-scaling step")
    ap.add_argument("--decomposition", default="time", choices=["time", "dm"],
                    help="N > 1 strong split: time - every rank searches its slice of the time tiles for the "
                         "whole grid, the per-tile records go to the trial owners (parallel.tile_sharded_search); "
                         "dm - every rank plans and searches its contiguous DM slice")
    ap.add_argument("--full-copy", action="store_true",
                    help="time split: send the whole filterbank to every rank (--collective) instead of scattering "
                         "to each rank the columns its time tiles read")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: rehearse the N > 1 path with every rank on the visible GPU(s), round robin "
                         "(RCCL refuses two ranks on one device); timings are then not the product's")
    ap.add_argument("--shard", type=int, default=0,
                    help="with --scaling strong on one GPU: search only rank 0's slice of an N-way split "
                         "(e.g. --config C3 --scaling strong --shard 8: the 625-trial shard of the 8-GPU run)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ref", action="store_true",
                    help="N > 1 strong split: skip the one-GPU run of the same workload on rank 0")
    ap.add_argument("--ref-steps", type=int, default=1)
    ap.add_argument("--cpu-trials", type=int, default=400)
    ap.add_argument("--no-clean", action="store_true")
    ap.add_argument("--clean-steps", type=int, default=20)
    ap.add_argument("--bcast-chunks", type=int, default=8)
    ap.add_argument("--cpu-reps", type=int, default=3)
    ap.add_argument("--no-c3-strong", action="store_true",
                    help="skip the configs[2] sub-benchmark (C3: 5000 trials split over the N GPUs)")
    ap.add_argument("--c3-steps", type=int, default=2)
    ap.add_argument("--no-acc-f64", action="store_true",
                    help="skip the float64-accumulation (reference precision) sub-benchmark")
    ap.add_argument("--acc-f64-steps", type=int, default=3)
    ap.add_argument("--allow-knobs", action="store_true",
                    help="time even with PU_* / PULSARUTILS_* tuning variables set (sweeps only: the line "
                         "is marked invalid)")
    args = ap.parse_args()
    knobs = knob_env()
    if knobs and not args.allow_knobs:
        sys.exit(f"bench.py: refusing to time with tuning variables set {knobs} (they reshape the kernels or "
                 "swap the library; unset them, or pass --allow-knobs for a sweep)")

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.scaling is None:
        args.scaling = "strong" if world > 1 else "weak"
    if args.config is None:
        args.config = "C3" if world > 1 and args.scaling == "strong" else "C2"
    if args.gpus != world and world != 1:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}")
    if args.dist_backend == "gloo":
        local = local % torch.cuda.device_count()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)

    cfg = CONFIGS[args.config]
    if args.scaling == "weak":
        # extend the plan to world * ntrials trials (1-sample steps, dedispersion.py:149-171)
        perdm = 4149.0 * (cfg.start_freq ** -2 - (cfg.start_freq + cfg.bandwidth) ** -2) / cfg.tsamp
        min_n = cfg.dmmin * perdm
        dmmax = (min_n + world * cfg.ntrials - 1.5) / perdm
        dms_all = dedispersion_plan(cfg.nchan, cfg.dmmin, dmmax, cfg.start_freq, cfg.bandwidth, cfg.tsamp)
        if dms_all.size != world * cfg.ntrials:
            raise RuntimeError(f"weak-scaling grid has {dms_all.size} trials, expected {world * cfg.ntrials}")
    else:
        dms_all = dedispersion_plan(cfg.nchan, cfg.dmmin, cfg.dmmax, cfg.start_freq, cfg.bandwidth, cfg.tsamp)
    lo, hi = shard_bounds(dms_all.size, world, rank)
    if args.shard > 1 and world == 1 and args.scaling == "strong":
        lo, hi = shard_bounds(dms_all.size, args.shard, 0)
        dms_all = dms_all[lo:hi]
    dms = dms_all[lo:hi]
    per_rank = dms.size
    chunk = -(-dms_all.size // world)  # equal gather slots
    pipelined = world > 1 and args.scaling == "strong"
    tsplit = pipelined and args.decomposition == "time"

    # ---- input: generated on rank 0 in HBM, RCCL-broadcast to the others
    t0 = time.perf_counter()
    if rank == 0:
        x = synth.pulsar_filterbank_device(cfg, device=dev)
    else:
        x = torch.empty((cfg.nchan, cfg.nsamples), dtype={"f32": torch.float32, "u8": torch.uint8,
                                                          "f64": torch.float64}[cfg.dtype], device=dev)
    torch.cuda.synchronize()
    log(f"rank {rank}: input ready {time.perf_counter() - t0:.1f}s")

    acc = {"native": _hip.PU_ACC_NATIVE, "f32": _hip.PU_ACC_F32, "f64": _hip.PU_ACC_F64}[args.acc]
    # time split: every rank plans the whole grid (and searches its slice of the time tiles)
    sh = _hip.shift_table(cfg.nchan, dms_all if tsplit else dms, cfg.start_freq, cfg.bandwidth, cfg.tsamp)
    plan = _hip.Plan(_hip.dtype_code(x.dtype), acc, cfg.nchan, cfg.nsamples, sh)
    log(f"rank {rank}: plan {plan.info}")
    ws = torch.empty(plan.workspace_bytes, dtype=torch.uint8, device=dev)
    nout = plan.ndm
    outs = (torch.empty(nout, dtype=torch.float64, device=dev),
            torch.empty(nout, dtype=torch.float64, device=dev),
            torch.empty(nout, dtype=torch.float64, device=dev),
            torch.empty(nout, dtype=torch.int32, device=dev))
    o_lo, o_hi = (lo, hi) if tsplit else (0, per_rank)  # this rank's trials in outs
    tt0, tt1 = (shard_bounds(plan.info["time_tiles"], world, rank) if tsplit else (0, plan.info["time_tiles"]))
    local_stats = torch.zeros((4, chunk), dtype=torch.float64, device=dev)
    gathered = torch.empty((world * 4, chunk), dtype=torch.float64, device=dev)  # rank-major (4, chunk) blocks

    bcast = None
    if world > 1:
        bcast = exchange_bench(x, plan, outs, ws, dev, args.bcast_chunks, args.decomposition if pipelined else "dm")
        if rank == 0:
            log(f"exchange {bcast}")

    def step(phases=None):
        if tsplit:
            # the whole job: rank 0's filterbank distributed in interleaved time chunks, every
            # rank searching its time tiles of the whole grid as they land, the records to the
            # trial owners, each owner's finalize
            tile_sharded_search(x, plan, outs, ws, src=0, chunks=args.bcast_chunks, collective=args.collective,
                                phases=phases, full_copy=args.full_copy)
        elif pipelined:
            # the whole job: rank 0's filterbank distributed in time chunks, every rank
            # searching the tiles whose rows have landed, then the finalize
            pipelined_broadcast_search(x, plan, outs, ws, src=0, chunks=args.bcast_chunks,
                                       collective=args.collective, phases=phases)
        else:
            plan.search(x, out=outs, workspace=ws)
        if world > 1:
            if phases is not None:
                phases.mark("gather", torch.cuda.current_stream(dev))
            local_stats[:, :per_rank].copy_(torch.stack([outs[0][o_lo:o_hi], outs[1][o_lo:o_hi], outs[2][o_lo:o_hi],
                                                         outs[3][o_lo:o_hi].to(torch.float64)]))
            dist.all_gather_into_tensor(gathered, local_stats)
            if phases is not None:
                phases.mark("gather", torch.cuda.current_stream(dev), end=True)

    for i in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # a pipelined step launches the search once per run of landed time tiles
    nslots = args.steps * (4 * args.bcast_chunks + 4 if pipelined else 1)
    plan.enable_timing(nslots)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kms = plan.kernel_times_ms(nslots)
    cert = plan.cert_info()
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    ms_per_step = elapsed / args.steps * 1e3

    # N > 1, pipelined: one more (untimed) step with HIP events around its phases - the
    # exchange, unpack and tile searches per chunk, the finalize, the gather - so a scaling
    # run explains itself; per phase the max over ranks
    phase_ms = None
    if pipelined:
        from pulsarutils.parallel import PhaseEvents
        pe = PhaseEvents()
        dist.barrier()
        step(pe)
        torch.cuda.synchronize()
        mine = pe.times_ms()
        keys = sorted(k for k, v in mine.items() if not isinstance(v, list))
        vals = torch.tensor([float(mine[k]) for k in keys], dtype=torch.float64, device=dev)
        allv = torch.empty(world * len(keys), dtype=torch.float64, device=dev)
        dist.all_gather_into_tensor(allv, vals)
        allv = allv.view(world, len(keys)).cpu().numpy()
        phase_ms = {"what": "one extra untimed step with HIP events: per-chunk exchange (scatter + all-gather "
                            "or broadcast) and unpack (staging -> strided column chunk, receivers) on the "
                            "communication stream, tile searches per chunk, records all_to_all (time split), "
                            "finalize, gather; exposed_tail = "
                            "last chunk landed -> finalize done",
                    "rank0": mine, "max_over_ranks": {k: round(float(allv[:, i].max()), 4) for i, k in enumerate(keys)}}

    # spot check: best trial of the whole grid (rank 0's view of the gathered S/N)
    if world > 1:
        snr_all = np.concatenate([gathered.view(world, 4, chunk)[r, 2, :shard_bounds(dms_all.size, world, r)[1]
                                           - shard_bounds(dms_all.size, world, r)[0]].cpu().numpy()
                                  for r in range(world)])
    else:
        snr_all = outs[2].cpu().numpy()
    best_dm = float(dms_all[np.argmax(snr_all)])

    total_samples = dms_all.size * cfg.nsamples
    value = total_samples / (ms_per_step / 1e3)
    # kernel time per step (pipelined: the sum of the step's tile-range launches)
    kernel_ms = float(np.sum(kms)) / args.steps if len(kms) else None
    # per rank: its trials x every sample, or (time split) every trial x its time tiles
    adds = (float(cfg.nchan) * min(cfg.nsamples, tt1 * plan.info["time_tile"]) - float(cfg.nchan) * tt0
            * plan.info["time_tile"]) * plan.ndm
    esz = {"f32": 4, "u8": 1, "f64": 8}[cfg.dtype]
    alg_bytes = float(cfg.nchan) * cfg.nsamples * esz  # compulsory input read per launch (stats mode)
    roof = None
    if kernel_ms:
        info = plan.info
        acc64 = bool(info["acc_is_f64"])
        peak = VALU_F64_ADD_PEAK_TFLOPS if acc64 else VALU_ADD_PEAK_TFLOPS
        achieved = adds / (kernel_ms / 1e3) / 1e12
        pmc_tag = args.config if per_rank == cfg.ntrials else f"{args.config}_{per_rank}"
        if tsplit:
            pmc_tag = f"{args.config}_time{world}"  # no committed counters for a rank's time slice
        pmc, pmc_same = load_pmc(pmc_tag)
        # counter traffic only when it was collected from this kernel source
        traffic = pmc.get("hbm_bytes_per_launch") if pmc and pmc_same else None
        roof = {"bound": "valu", "achieved": round(achieved, 3), "peak": peak,
                "unit": "TFLOP/s" + (" (f64 adds)" if acc64 else " (f32 adds)"),
                "frac": round(achieved / peak, 4), "traffic": traffic,
                "kernel": _hip.KERNEL_NAMES[info["kernel"]],
                "kernel_ms": round(kernel_ms, 4),
                "algorithmic_flop_per_launch": adds, "algorithmic_bytes_per_launch": alg_bytes,
                "time_tiles": info["time_tiles"],
                "hbm_compulsory_gbs": round(alg_bytes / (kernel_ms / 1e3) / 1e9, 1),
                "hbm_compulsory_frac": round(alg_bytes / (kernel_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4)}
        if traffic:
            roof.update({"hbm_counter_GBps": round(traffic / (kernel_ms / 1e3) / 1e9, 1),
                         "hbm_counter_frac": round(traffic / (kernel_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                         "traffic_source": f"profiles/pmc_{pmc_tag}.json ({pmc.get('source')})",
                         "traffic_kernel_ms_at_collection": pmc.get("kernel_ms_at_collection"),
                         "traffic_source_sha256_matches_build": True})
        elif pmc:
            roof["traffic_note"] = (f"profiles/pmc_{pmc_tag}.json was collected from another dedisperse.hip "
                                    "(SHA-256 differs): not reported")
        if info["group"] > 1:
            # executed work of the exact subband decomposition: G x fewer
            # adds than the algorithm's; the LDS array (256 B/clk/CU) is its binding unit
            lds = info["lds_traffic"] / (kernel_ms / 1e3) / 1e12
            roof.update({"executed_flop_per_launch": info["exec_adds"],
                         "executed_tflops": round(info["exec_adds"] / (kernel_ms / 1e3) / 1e12, 3),
                         "lds_bytes_per_launch": info["lds_traffic"], "lds_achieved_TBps": round(lds, 2),
                         "lds_peak_TBps": LDS_PEAK_TBPS, "lds_frac": round(lds / LDS_PEAK_TBPS, 4),
                         **sq_fields(load_sq(pmc_tag), pmc_tag),
                         "group": info["group"], "binding": "lds",
                         "binding_note": "frac is SURVEY 8(d)'s brute-force-equivalent adds / the f32 VALU-add "
                                         "peak; the subband decomposition executes group x fewer adds, and the "
                                         "unit that binds it is the LDS array: lds_cycle_frac (counters: LDS-array "
                                         "cycles / CU cycles), lds_frac (the planner's byte model)"})

    # N > 1, strong split: the same whole workload on rank 0's GPU alone (untimed by the
    # step; the other ranks wait), so the line carries its own one-GPU reference - the N = 1
    # headline is C2 (configs[1]), a different workload
    ref1 = None
    if pipelined and not args.no_ref:
        if rank == 0:
            log("one-GPU reference (the whole grid on rank 0) ...")
            sh_all = _hip.shift_table(cfg.nchan, dms_all, cfg.start_freq, cfg.bandwidth, cfg.tsamp)
            plan1 = _hip.Plan(_hip.dtype_code(x.dtype), acc, cfg.nchan, cfg.nsamples, sh_all)
            ws1 = torch.empty(plan1.workspace_bytes, dtype=torch.uint8, device=dev)
            plan1.search(x, workspace=ws1)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for _ in range(args.ref_steps):
                plan1.search(x, workspace=ws1)
            torch.cuda.synchronize()
            ms1 = (time.perf_counter() - t1) / args.ref_steps * 1e3
            ref1 = {"what": "the same workload (all trials, the resident filterbank, no exchange) searched on "
                            "rank 0's GPU alone, after the timed steps", "ms_per_step": ms1,
                    "value": total_samples / (ms1 / 1e3), "steps": args.ref_steps,
                    "speedup": (total_samples / (ms_per_step / 1e3)) / (total_samples / (ms1 / 1e3)),
                    "efficiency": ms1 / ms_per_step / world}
            del plan1, ws1
            torch.cuda.empty_cache()
        dist.barrier()

    f64 = None
    if rank == 0 and world == 1 and not args.no_acc_f64 and args.acc == "native" and cfg.dtype != "f64":
        log("acc_f64 ...")
        f64 = acc_f64_bench(x, dms, cfg, args.acc_f64_steps)
        log(f"acc_f64 kernel {f64['kernel_ms']:.3f} ms, step {f64['ms_per_step']:.3f} ms")

    clean = None
    if rank == 0 and world == 1 and not args.no_clean:
        log("clean (C4) ...")
        clean = clean_bench(dev, args.clean_steps)
        log(f"clean {clean['f32']['renormalize_ms']:.3f} ms f32, {clean['u8']['renormalize_ms']:.3f} ms u8")

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("cpu baseline ...")
        xh = x.cpu().numpy()
        threads = cpu_threads()
        cpu = cpu_baseline(xh, dms, cfg, args.cpu_trials, threads, reps=args.cpu_reps)
        del xh
        log(f"cpu baseline {cpu['value']:.3e} samples/s on {threads} threads ({cpu['cpu_model']})")

    c3 = None
    if not args.no_c3_strong and args.config != "C3" and world == 1:
        del x, ws, outs, plan
        torch.cuda.empty_cache()
        log("c3_strong ...")
        c3 = c3_strong(dev, world, rank, args.c3_steps, args.bcast_chunks)
        if rank == 0:
            log(f"c3_strong compute {c3['compute_ms']:.1f} ms, end-to-end {c3.get('end_to_end_ms')}")

    if rank == 0:
        line = {"metric": "dedispersed DM-trial samples/sec (whole node)", "value": value,
                "unit": "DM-trial samples/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": args.scaling,
                "vs_baseline": None,
                "dtype": {"f32": "f32", "u8": "u8", "f64": "f64"}[cfg.dtype] + ("" if args.acc == "native"
                                                                                 else f"(acc {args.acc})"),
                "data": "synthetic (noise + unit pulse at DM %g, generated in HBM%s)" % (
                    cfg.pulse_dm, " of rank 0 and distributed inside every timed step" if pipelined else ""),
                "config": {"workload": f"{cfg.name}: {cfg.nchan} chan x 2^{int(np.log2(cfg.nsamples))} "
                                      f"{cfg.dtype} samples, {dms_all.size} DM trials "
                                      f"({'per GPU' if args.scaling == 'weak' else 'in all'})",
                           "nchan": cfg.nchan, "nsamples": cfg.nsamples, "trials_per_gpu": per_rank,
                           "total_trials": int(dms_all.size),
                           "parallelism": f"time-shard{world}" if tsplit else f"dm-shard{world}",
                           "best_dm": best_dm},
                "step": ("%s pipelined with each rank's search of its time tiles for every trial, all_to_all of "
                         "the per-tile records to the trial owners, finalize of each rank's trials, all_gather of "
                         "(max, std, snr, rebin)" % ("interleaved chunked filterbank exchange from rank 0 (%s)"
                                                     % args.collective if args.full_copy else
                                                     "chunked scatter from rank 0 of the columns each rank's time "
                                                     "tiles read")
                         if tsplit else
                         "chunked filterbank exchange from rank 0 (%s) pipelined with each rank's search of its "
                         "DM slice, finalize, all_gather of (max, std, snr, rebin)" % args.collective
                         if pipelined else "pu_plan_search of the resident filterbank" +
                         (" + all_gather of (max, std, snr, rebin)" if world > 1 else "")),
                "roofline": roof, "clean": clean, "cpu_baseline": cpu,
                "certify": dict(cert, what="trials of the last timed step whose fast statistics could not be "
                                           "certified and were recomputed exactly (DESIGN.md §4.5)"),
                "env": knobs, "valid": not knobs and args.dist_backend == "nccl"}
        if f64 is not None:
            line["acc_f64"] = f64
        if c3 is not None:
            line["c3_strong"] = c3
        if bcast is not None:
            line["multi_gpu"] = bcast
        if ref1 is not None:
            line["single_gpu_same_workload"] = ref1
        if phase_ms is not None:
            line["phases"] = phase_ms
        line["build"] = _hip.build_info()  # was the library built from the sources shipped with it
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
