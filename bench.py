"""Benchmark: dedispersed DM-trial samples/s on the C2 config (BASELINE.json configs[1]).

One "step" = one fused DM-trial search (pu_plan_search: shift-and-sum over all
channels for every trial + the S/N epilogue + the per-trial finalize) over a
1024-channel x 2^20-sample float32 filterbank resident in HBM, 1000 trials per GPU.

N GPUs (one process each, torchrun): weak scaling.  The DM grid is N x 1000 trials,
sharded contiguously (rank r owns trials [1000 r, 1000 (r+1))); the filterbank is
generated on rank 0 and RCCL-broadcast over xGMI before timing (reported separately
as broadcast_ms); each step ends with an all_gather of the per-trial statistics.

Prints ONE JSON line (rank 0) with the driver's contract fields plus ``roofline``
(dominant kernel, HIP events on its launch stream) and ``cpu_baseline`` (the C
oracle = a port of the reference's numba search, timed on a bounded trial sample).
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

# MI355X peaks (/opt/skills/guides/MI355X_MICROARCH.md, chip-level parameters)
HBM_PEAK_GBS = 8000.0
# float32 vector peak is 157.3 TFLOP/s counting an FMA as 2 FLOP; an add is one FLOP
# per lane-op, so the add-only ceiling is half of it: 256 CU x 128 lanes/clk x 2.4 GHz
VALU_ADD_PEAK_TFLOPS = 78.6
# LDS: 256 B/clk/CU for ds_read_b64 (MI355X_MICROARCH.md §LDS) x 256 CUs x 2.4 GHz
LDS_PEAK_TBPS = 157.3


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def cpu_baseline(x_host, dms, cfg, ntrials, threads):
    import oracle
    ntrials = min(ntrials, dms.size)
    sel = dms[np.linspace(0, dms.size - 1, ntrials).astype(int)]
    oracle.search(x_host[:, :4096], sel[:2], cfg.start_freq, cfg.bandwidth, cfg.tsamp, nthreads=threads)
    t0 = time.perf_counter()
    oracle.search(x_host, sel, cfg.start_freq, cfg.bandwidth, cfg.tsamp, nthreads=threads)
    dt = time.perf_counter() - t0
    return {"value": ntrials * cfg.nsamples / dt, "unit": "DM-trial samples/s", "cores": threads,
            "kind": "port",
            "sample": f"{ntrials} of the {dms.size} {cfg.name} trials (evenly spaced), full "
                      f"{cfg.nchan}x2^{int(np.log2(cfg.nsamples))} {cfg.dtype} filterbank, float64 oracle/dedisp_oracle.c (numba prange -> OpenMP), {dt:.1f} s"}


def load_pmc(workload):
    path = os.path.join(REPO, "profiles", f"pmc_{workload}.json")
    if os.path.exists(path):
        try:
            return json.load(open(path)).get("hbm_bytes_per_launch")
        except Exception:
            return None
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="C2")
    ap.add_argument("--acc", default="native", choices=["native", "f32", "f64"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-trials", type=int, default=400)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world != 1:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)

    cfg = CONFIGS[args.config]
    per_rank = cfg.ntrials
    # weak scaling: extend the plan to world * ntrials trials, 1-sample steps
    perdm = 4149.0 * (cfg.start_freq ** -2 - (cfg.start_freq + cfg.bandwidth) ** -2) / cfg.tsamp
    min_n = cfg.dmmin * perdm
    dmmax = (min_n + world * per_rank - 1.5) / perdm
    dms_all = dedispersion_plan(cfg.nchan, cfg.dmmin, dmmax, cfg.start_freq, cfg.bandwidth, cfg.tsamp)
    assert dms_all.size == world * per_rank, dms_all.size
    dms = dms_all[rank * per_rank:(rank + 1) * per_rank]

    # ---- input: generated on rank 0 in HBM, RCCL-broadcast to the others
    t0 = time.perf_counter()
    if rank == 0:
        x = synth.pulsar_filterbank_device(cfg, device=dev)
    else:
        x = torch.empty((cfg.nchan, cfg.nsamples), dtype={"f32": torch.float32, "u8": torch.uint8,
                                                          "f64": torch.float64}[cfg.dtype], device=dev)
    torch.cuda.synchronize()
    log(f"rank {rank}: input ready {time.perf_counter() - t0:.1f}s")
    bcast_ms = None
    if world > 1:
        dist.barrier()
        torch.cuda.synchronize()
        tb = time.perf_counter()
        dist.broadcast(x, src=0)
        torch.cuda.synchronize()
        bcast_ms = (time.perf_counter() - tb) * 1e3

    acc = {"native": _hip.PU_ACC_NATIVE, "f32": _hip.PU_ACC_F32, "f64": _hip.PU_ACC_F64}[args.acc]
    sh = _hip.shift_table(cfg.nchan, dms, cfg.start_freq, cfg.bandwidth, cfg.tsamp)
    plan = _hip.Plan(_hip.dtype_code(x.dtype), acc, cfg.nchan, cfg.nsamples, sh)
    log(f"rank {rank}: plan {plan.info}")
    ws = torch.empty(plan.workspace_bytes, dtype=torch.uint8, device=dev)
    outs = (torch.empty(per_rank, dtype=torch.float64, device=dev),
            torch.empty(per_rank, dtype=torch.float64, device=dev),
            torch.empty(per_rank, dtype=torch.float64, device=dev),
            torch.empty(per_rank, dtype=torch.int32, device=dev))
    gathered = [torch.empty(world * per_rank, dtype=torch.float64, device=dev) for _ in range(3)]

    def step():
        plan.search(x, out=outs, workspace=ws)
        if world > 1:
            for g, o in zip(gathered, outs[:3]):
                dist.all_gather_into_tensor(g, o)

    for i in range(args.warmup):
        step()
    torch.cuda.synchronize()
    plan.enable_timing(args.steps)
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
    kms = plan.kernel_times_ms(args.steps)
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    ms_per_step = elapsed / args.steps * 1e3

    # parity spot check on rank 0's best trial (pulse DM)
    snr = outs[2].cpu().numpy()
    best_dm = float(dms[np.argmax(snr)])

    total_samples = world * per_rank * cfg.nsamples
    value = total_samples / (ms_per_step / 1e3)
    kernel_ms = float(np.mean(kms)) if len(kms) else None
    adds = float(cfg.nchan) * cfg.nsamples * per_rank
    esz = {"f32": 4, "u8": 1, "f64": 8}[cfg.dtype]
    alg_bytes = float(cfg.nchan) * cfg.nsamples * esz  # compulsory input read per launch (stats mode)
    roof = None
    if kernel_ms:
        info = plan.info
        achieved = adds / (kernel_ms / 1e3) / 1e12
        roof = {"bound": "valu", "achieved": round(achieved, 3), "peak": VALU_ADD_PEAK_TFLOPS,
                "unit": "TFLOP/s", "frac": round(achieved / VALU_ADD_PEAK_TFLOPS, 4),
                "traffic": load_pmc(args.config),
                "kernel": "dedisp_sub_kernel" if info["group"] > 1 else "dedisp_kernel",
                "kernel_ms": round(kernel_ms, 4),
                "algorithmic_flop_per_launch": adds, "algorithmic_bytes_per_launch": alg_bytes,
                "hbm_compulsory_gbs": round(alg_bytes / (kernel_ms / 1e3) / 1e9, 1),
                "hbm_compulsory_frac": round(alg_bytes / (kernel_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4)}
        if info["group"] > 1:
            # executed work of the exact subband decomposition: G x fewer
            # adds than the algorithm's; the LDS array (256 B/clk/CU) is its binding unit
            lds = info["lds_traffic"] / (kernel_ms / 1e3) / 1e12
            roof.update({"executed_flop_per_launch": info["exec_adds"],
                         "executed_tflops": round(info["exec_adds"] / (kernel_ms / 1e3) / 1e12, 3),
                         "lds_bytes_per_launch": info["lds_traffic"], "lds_achieved_TBps": round(lds, 2),
                         "lds_peak_TBps": LDS_PEAK_TBPS, "lds_frac": round(lds / LDS_PEAK_TBPS, 4),
                         "group": info["group"]})

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("cpu baseline ...")
        xh = x.cpu().numpy()
        import oracle
        threads = int(os.environ.get("BENCH_CPU_THREADS", min(16, os.cpu_count() or 1)))
        cpu = cpu_baseline(xh, dms, cfg, args.cpu_trials, threads)
        del xh
        log(f"cpu baseline {cpu['value']:.3e} samples/s on {threads} threads")

    if rank == 0:
        line = {"metric": "dedispersed DM-trial samples/sec (whole node)", "value": value,
                "unit": "DM-trial samples/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
                "dtype": {"f32": "f32", "u8": "u8", "f64": "f64"}[cfg.dtype] + ("" if args.acc == "native"
                                                                                 else f"(acc {args.acc})"),
                "data": "synthetic (|N(0,0.5)| + unit pulse at DM %g, generated in HBM)" % cfg.pulse_dm,
                "config": {"workload": f"{cfg.name}: {cfg.nchan} chan x 2^{int(np.log2(cfg.nsamples))} "
                                      f"{cfg.dtype} samples, {per_rank} DM trials per GPU",
                           "nchan": cfg.nchan, "nsamples": cfg.nsamples, "trials_per_gpu": per_rank,
                           "total_trials": world * per_rank, "parallelism": f"dm-shard{world}",
                           "best_dm_rank0": best_dm},
                "roofline": roof, "cpu_baseline": cpu}
        if bcast_ms is not None:
            line["broadcast_ms"] = bcast_ms
            line["broadcast_GBps"] = x.numel() * x.element_size() / bcast_ms / 1e6
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
