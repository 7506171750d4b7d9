"""Per-rank search time of each shard of an N-GPU DM-trial split, on ONE GPU.

Usage: python scripts/shard_times.py [config] [world] [dm|time]     (default C3 8 dm)

``time``: the time-tile split instead (parallel.tile_sharded_search): every rank holds the
whole grid's plan and searches time tiles shard_bounds(time_tiles, world, rank)
(pu_plan_search_tiles), then packs its records for the other ranks' trials and unpacks
theirs (the two copies around the records all_to_all) and finalizes its trial slice
(pu_plan_finalize_range) - each timed per rank with HIP events.

Each rank of ``bench.py --gpus N`` searches a contiguous block of trials
(``parallel.shard_bounds``); the N-GPU step time is the max over ranks, so the slowest
shard - not the first - sets it.  This times every shard's default plan (3 rounds of 3
searches, median of the kernel's HIP-event times) and prints its plan (group, kernel,
stages) - the input of DESIGN.md §5's per-rank prediction.
"""
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
from pulsarutils.parallel import shard_bounds  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C3"
world = int(sys.argv[2]) if len(sys.argv) > 2 else 8
mode = sys.argv[3] if len(sys.argv) > 3 else "dm"
cfg = CONFIGS[name]
x = synth.pulsar_filterbank_device(cfg)
dms = dedispersion_plan(cfg.nchan, cfg.dmmin, cfg.dmmax, cfg.start_freq, cfg.bandwidth, cfg.tsamp)


def ev_ms(fn, reps=3):
    out = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        out.append(a.elapsed_time(b))
    return float(np.median(out))


if mode == "time":
    sh = _hip.shift_table(cfg.nchan, dms, cfg.start_freq, cfg.bandwidth, cfg.tsamp)
    plan = _hip.Plan(_hip.dtype_code(x.dtype), _hip.PU_ACC_NATIVE, cfg.nchan, cfg.nsamples, sh)
    ws = torch.empty(plan.workspace_bytes, dtype=torch.uint8, device=x.device)
    outs = plan._outs_ws(x.device, None, ws)[0]
    ntt = plan.info["time_tiles"]
    full = ev_ms(lambda: plan.search(x, out=outs, workspace=ws))
    print(json.dumps({"config": name, "mode": "time", "whole_grid_search_ms": round(full, 3), "plan": plan.info}),
          flush=True)
    ref = [o.clone() for o in outs]
    rec = plan.records(ws)
    R = rec.shape[2]
    rows = []
    for r in range(world):
        t0, t1 = shard_bounds(ntt, world, r)
        lo, hi = shard_bounds(dms.size, world, r)
        ms = []
        for rnd in range(3):
            plan.enable_timing(3)
            for _ in range(3):
                plan.search_tiles(x, t0, t1, ws)
            torch.cuda.synchronize()
            ms.append(float(np.median(plan.kernel_times_ms(3))))
        tb = [shard_bounds(ntt, world, q) for q in range(world)]
        db = [shard_bounds(dms.size, world, q) for q in range(world)]
        pack = ev_ms(lambda: torch.cat([rec[a:b, t0:t1].reshape(-1) for q, (a, b) in enumerate(db) if q != r]))
        recv = torch.empty((hi - lo) * (ntt - (t1 - t0)) * R, dtype=rec.dtype, device=x.device)

        def unpack():
            off = 0
            for q, (u0, u1) in enumerate(tb):
                if q == r:
                    continue
                m = (hi - lo) * (u1 - u0) * R
                rec[lo:hi, u0:u1].copy_(recv[off:off + m].view(hi - lo, u1 - u0, R))
                off += m
        # the unpack writes garbage records: re-search the whole grid before the finalize
        unp = ev_ms(unpack)
        plan.search(x, out=outs, workspace=ws)
        fin = ev_ms(lambda: plan.finalize_range(ws, x, lo, hi, out=outs))
        for k in range(4):
            assert torch.equal(outs[k][lo:hi], ref[k][lo:hi]), (r, k)
        send_b = sum((b - a) for q, (a, b) in enumerate(db) if q != r) * (t1 - t0) * R * rec.element_size()
        rows.append({"rank": r, "tiles": [t0, t1], "trials": [lo, hi], "search_ms": round(float(np.median(ms)), 3),
                     "pack_ms": round(pack, 3), "unpack_ms": round(unp, 3), "finalize_range_ms": round(fin, 3),
                     "records_sent_bytes": int(send_b), "records_recv_bytes": int(recv.numel() * rec.element_size())})
        print(json.dumps(rows[-1]), flush=True)
    ms = [row["search_ms"] for row in rows]
    print(json.dumps({"config": name, "world": world, "mode": "time", "max_search_ms": max(ms),
                      "mean_search_ms": round(float(np.mean(ms)), 3), "sum_search_ms": round(float(np.sum(ms)), 3),
                      "whole_grid_search_ms": round(full, 3),
                      "max_rank_local_ms": max(r_["search_ms"] + r_["pack_ms"] + r_["unpack_ms"] + r_["finalize_range_ms"]
                                               for r_ in rows)}), flush=True)
    sys.exit(0)
plans = []
for r in range(world):
    a, b = shard_bounds(dms.size, world, r)
    sh = _hip.shift_table(cfg.nchan, dms[a:b], cfg.start_freq, cfg.bandwidth, cfg.tsamp)
    plans.append((r, a, b, _hip.Plan(_hip.dtype_code(x.dtype), _hip.PU_ACC_NATIVE, cfg.nchan, cfg.nsamples, sh)))
ws = torch.empty(max(p.workspace_bytes for *_, p in plans), dtype=torch.uint8, device=x.device)
times = {r: [] for r, *_ in plans}
for rnd in range(3):
    for r, a, b, p in plans:
        p.enable_timing(3)
        for _ in range(3):
            p.search(x, workspace=ws)
        torch.cuda.synchronize()
        times[r].append(float(np.median(p.kernel_times_ms(3))))
        print(f"round {rnd} rank {r} trials {a}:{b}: {times[r][-1]:.3f} ms", flush=True)
rows = []
for r, a, b, p in plans:
    i = p.info
    rows.append({"rank": r, "trials": [a, b], "dm": [float(dms[a]), float(dms[b - 1])],
                 "ms": round(float(np.median(times[r])), 3), "group": i["group"], "kernel": _hip.KERNEL_NAMES[i["kernel"]],
                 "stages": i["stages"], "slots": i["slots"], "max_spread": i["max_spread"],
                 "lds_traffic": i["lds_traffic"]})
    print(json.dumps(rows[-1]), flush=True)
ms = [row["ms"] for row in rows]
print(json.dumps({"config": name, "world": world, "max_ms": max(ms), "mean_ms": round(float(np.mean(ms)), 3),
                  "sum_ms": round(float(np.sum(ms)), 3), "slowest_rank": int(np.argmax(ms))}), flush=True)
