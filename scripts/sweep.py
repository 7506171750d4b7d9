"""Interleaved A/B of dedispersion plan variants in ONE process (guide §5.4 rule 24).

Usage: python scripts/sweep.py [config] ; env PU_SWEEP="lds=32,48,64" selects LDS budgets.
Prints one line per (variant, round) and a median summary.
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "radio-pulsar-utils_amd"), REPO]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from pulsarutils import _hip, synth  # noqa: E402
from pulsarutils.configs import CONFIGS  # noqa: E402
from pulsarutils.dedispersion import dedispersion_plan  # noqa: E402

cfg = CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "C2"]
budgets = [int(v) for v in os.environ.get("PU_SWEEP", "48").split(",")]
rounds = int(os.environ.get("PU_ROUNDS", "3"))
x = synth.pulsar_filterbank_device(cfg)
dms = dedispersion_plan(cfg.nchan, cfg.dmmin, cfg.dmmax, cfg.start_freq, cfg.bandwidth, cfg.tsamp)
sh = _hip.shift_table(cfg.nchan, dms, cfg.start_freq, cfg.bandwidth, cfg.tsamp)
plans = {}
for b in budgets:
    os.environ["PU_LDS_BUDGET_KB"] = str(b)
    plans[b] = _hip.Plan(_hip.dtype_code(x.dtype), _hip.PU_ACC_NATIVE, cfg.nchan, cfg.nsamples, sh)
    print("budget", b, plans[b].info, flush=True)
ws = torch.empty(max(p.workspace_bytes for p in plans.values()), dtype=torch.uint8, device=x.device)
res = {b: [] for b in budgets}
ref = None
for r in range(rounds):
    for b, p in plans.items():
        p.enable_timing(3)
        out = p.search(x, workspace=ws)
        out = p.search(x, workspace=ws)
        out = p.search(x, workspace=ws)
        torch.cuda.synchronize()
        ms = p.kernel_times_ms(3)
        res[b].append(float(np.median(ms)))
        snr = out[2].cpu().numpy()
        if ref is None:
            ref = snr
        ok = np.allclose(snr, ref, rtol=1e-5)
        print(f"round {r} budget {b}KB: {np.median(ms):.3f} ms  ncc={p.info['chans_per_step']} same={ok}", flush=True)
adds = cfg.nchan * cfg.nsamples * dms.size
for b in budgets:
    m = float(np.median(res[b]))
    print(f"SUMMARY budget {b}KB median {m:.3f} ms  {adds / m / 1e9:.2f} Tadd/s  frac {adds / m / 1e9 / 78.6:.3f}")
