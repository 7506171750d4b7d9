"""Per-rank search time of each shard of an N-GPU DM-trial split, on ONE GPU.

Usage: python scripts/shard_times.py [config] [world]     (default C3 8)

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
cfg = CONFIGS[name]
x = synth.pulsar_filterbank_device(cfg)
dms = dedispersion_plan(cfg.nchan, cfg.dmmin, cfg.dmmax, cfg.start_freq, cfg.bandwidth, cfg.tsamp)
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
