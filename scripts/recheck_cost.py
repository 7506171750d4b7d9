"""Cost of certifying one flagged trial at C3 (4096 x 2^22 uint8), on one GPU, HIP events:
pu_plan_exact_series of one trial over the whole series and over 1/8 of it (a time-split
rank's share), pu_series_stats of the 2^22-sample series, and pu_plan_finalize_range over
625 trials with and without a flagged trial."""
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

cfg = CONFIGS["C3"]
x = synth.pulsar_filterbank_device(cfg)
dms = dedispersion_plan(cfg.nchan, cfg.dmmin, cfg.dmmax, cfg.start_freq, cfg.bandwidth, cfg.tsamp)[:625]
sh = _hip.shift_table(cfg.nchan, dms, cfg.start_freq, cfg.bandwidth, cfg.tsamp)
plan = _hip.Plan(_hip.dtype_code(x.dtype), _hip.PU_ACC_NATIVE, cfg.nchan, cfg.nsamples, sh)
ws = torch.empty(plan.workspace_bytes, dtype=torch.uint8, device=x.device)
outs = plan._outs_ws(x.device, None, ws)[0]


def ev(fn, reps=5):
    out = []
    for _ in range(reps):
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        out.append(a.elapsed_time(b))
    return round(float(np.median(out)), 3)


import time  # noqa: E402


def wall(fn, reps=5):
    out = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        out.append((time.perf_counter() - t0) * 1e3)
    return round(float(np.median(out)), 3)


plan.search(x, out=outs, workspace=ws)
res = {"cert": plan.cert_info()}
ser = torch.empty((1, cfg.nsamples), dtype=torch.float64, device=x.device)
res["exact_series_1_trial_ms"] = wall(lambda: plan.exact_series(x, [3], out=ser))
n8 = cfg.nsamples // 8
res["exact_series_1_trial_eighth_ms"] = wall(lambda: plan.exact_series(x, [3], t_begin=3 * n8, t_end=4 * n8))
ser8 = torch.empty((8, cfg.nsamples), dtype=torch.float64, device=x.device)
res["exact_series_8_trials_ms"] = wall(lambda: plan.exact_series(x, list(range(8)), out=ser8))
res["series_stats_1_ms"] = ev(lambda: _hip.series_stats(ser))
res["series_stats_1_wall_ms"] = wall(lambda: _hip.series_stats(ser))
plan.search_tiles(x, 0, plan.info["time_tiles"], ws)
res["finalize_range_ms"] = wall(lambda: plan.finalize_range(ws, x, 0, dms.size, out=outs))
res["finalize_range_rechecked"] = plan.cert_info()["rechecked"]
res["finalize_range_flagged_ms"] = wall(lambda: plan.finalize_range_flagged(ws, 0, dms.size, out=outs))
print(json.dumps(res), flush=True)
