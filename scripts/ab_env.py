"""Interleaved A/B of planner / kernel variants selected by environment variables, in one
process (the plans are built under each variant's variables, then timed round-robin).

    PU_AB="PU_F32_DMA=1;PU_F32_DMA=0" python scripts/ab_env.py [config] [rounds]

A variant is a comma-separated list of NAME=VALUE; variants are separated by ';'.
Prints per-round kernel times (HIP events), a median summary, and whether each
variant's S/N column matches the first variant's within the float32 tolerance.
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

cfg = CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "C2"]
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
variants = [v.strip() for v in os.environ.get("PU_AB", "PU_F32_DMA=1;PU_F32_DMA=0").split(";") if v.strip()]
ntr = int(os.environ.get("PU_TRIALS", "0"))
x = synth.pulsar_filterbank_device(cfg)
dms = dedispersion_plan(cfg.nchan, cfg.dmmin, cfg.dmmax, cfg.start_freq, cfg.bandwidth, cfg.tsamp)
if ntr:
    dms = dms[:ntr]
sh = _hip.shift_table(cfg.nchan, dms, cfg.start_freq, cfg.bandwidth, cfg.tsamp)
plans = {}
for v in variants:
    kv = dict(a.split("=", 1) for a in v.split(",") if a)
    saved = {k: os.environ.get(k) for k in kv}
    os.environ.update(kv)
    acc = {"native": _hip.PU_ACC_NATIVE, "f32": _hip.PU_ACC_F32, "f64": _hip.PU_ACC_F64}[os.environ.get("AB_ACC", "native")]
    plans[v] = _hip.Plan(_hip.dtype_code(x.dtype), acc, cfg.nchan, cfg.nsamples, sh,
                         group=int(os.environ.get("AB_GROUP", "0")),  # AB_GROUP / AB_SHAPE: pin the plan
                         shape=int(os.environ["AB_SHAPE"]) if "AB_SHAPE" in os.environ else None)
    for k, val in saved.items():
        if val is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = val
    print("variant", v, json.dumps({k: plans[v].info[k] for k in ("group", "stages", "dm_tiles", "time_tiles", "lds_traffic", "lds_bytes",
                                                                    "slot_bytes", "raw_stride")}), flush=True)
ws = torch.empty(max(p.workspace_bytes for p in plans.values()), dtype=torch.uint8, device=x.device)
res = {v: [] for v in plans}
ref = None
for r in range(rounds):
    for v, p in plans.items():
        # the kernel-shaping variables are read at launch too (diagnostic knobs): set them
        kv = dict(a.split("=", 1) for a in v.split(",") if a)
        saved = {k: os.environ.get(k) for k in kv}
        os.environ.update(kv)
        p.enable_timing(3)
        for _ in range(3):
            out = p.search(x, workspace=ws)
        torch.cuda.synchronize()
        ms = p.kernel_times_ms(3)
        for k, val in saved.items():
            if val is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = val
        res[v].append(float(np.median(ms)))
        snr = out[2].cpu().numpy()
        if ref is None:
            ref = snr
        print(f"round {r} [{v}] {np.median(ms):.3f} ms same={np.allclose(snr, ref, rtol=1e-5)} "
              f"cert={p.cert_info()['rechecked']}", flush=True)
for v in plans:
    print(f"SUMMARY [{v}] median {float(np.median(res[v])):.3f} ms", flush=True)
