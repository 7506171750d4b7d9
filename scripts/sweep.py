"""Interleaved A/B of dedispersion plan variants in ONE process (guide §5.4 rule 24).

Usage: python scripts/sweep.py [config]
  env PU_SWEEP="G:KB[:shape],..." selects (channel-group size, LDS budget KB, subband
  workgroup shape 0 wide / 1 pair / 2 tall[, slot16 0/1]) variants, e.g.
  "1:64,4:160:0,4:80:1" (group 1 = channel mode), "8:160:2:1,8:160:2:0" (8-bit C3: 16-bit vs
  float32 slots).  PU_ROUNDS rounds, PU_TRIALS the first trials of the grid (from trial
  PU_TRIAL0, default 0: e.g. PU_TRIAL0=1875 PU_TRIALS=625 is rank 3's shard of 8 at C3).
Prints one line per (variant, round) and a median summary; the S/N of every trial
is compared with the first variant's (float32 tolerance).
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "radio-pulsar-utils_amd"), REPO]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from pulsarutils import _hip, synth  # noqa: E402
from pulsarutils.configs import CONFIGS  # noqa: E402
from pulsarutils.dedispersion import dedispersion_plan  # noqa: E402

cfg = CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "C2"]
variants = [tuple(int(u) for u in v.split(":")) for v in os.environ.get("PU_SWEEP", "1:64,4:64").split(",")]
rounds = int(os.environ.get("PU_ROUNDS", "3"))
ntrials = int(os.environ.get("PU_TRIALS", "0"))
x = synth.pulsar_filterbank_device(cfg)
dms = dedispersion_plan(cfg.nchan, cfg.dmmin, cfg.dmmax, cfg.start_freq, cfg.bandwidth, cfg.tsamp)
trial0 = int(os.environ.get("PU_TRIAL0", "0"))
if ntrials or trial0:
    dms = dms[trial0:trial0 + ntrials] if ntrials else dms[trial0:]
sh = _hip.shift_table(cfg.nchan, dms, cfg.start_freq, cfg.bandwidth, cfg.tsamp)
plans = {}
for v in variants:
    plans[v] = _hip.Plan(_hip.dtype_code(x.dtype), _hip.PU_ACC_NATIVE, cfg.nchan, cfg.nsamples, sh, group=v[0],
                         lds_budget_kb=v[1], shape=v[2] if len(v) > 2 else 0,
                         slot16=bool(v[3]) if len(v) > 3 else None)
    print("variant", v, plans[v].info, flush=True)
ws = torch.empty(max(p.workspace_bytes for p in plans.values()), dtype=torch.uint8, device=x.device)
res = {v: [] for v in plans}
ref = None
for r in range(rounds):
    for v, p in plans.items():
        p.enable_timing(3)
        for _ in range(3):
            out = p.search(x, workspace=ws)
        torch.cuda.synchronize()
        ms = p.kernel_times_ms(3)
        res[v].append(float(np.median(ms)))
        snr = out[2].cpu().numpy()
        if ref is None:
            ref = snr
        ok = np.allclose(snr, ref, rtol=1e-5)
        print(f"round {r} variant {v}: {np.median(ms):.3f} ms same={ok}", flush=True)
samples = cfg.nsamples * dms.size
for v in plans:
    m = float(np.median(res[v]))
    print(f"SUMMARY variant {v} median {m:.3f} ms  {samples / m * 1e3:.3e} samples/s  "
          f"brute-force-equivalent {cfg.nchan * samples / m / 1e9:.2f} Tadd/s")
