"""One-GPU proxy for the search / RCCL overlap of the chunked broadcast.

RCCL's broadcast runs as kernels that need CUs while dedisp_sub_kernel holds one
160 KiB-LDS workgroup on every CU.  The proxy: device-to-device copies (blit kernels,
which also need CUs) on a second stream while the search runs, with the search on an
unmasked stream and on CU-masked streams that leave ``reserve`` CUs free
(pu_stream_create_cu_masked).  Reports the search's kernel time and the copies'
throughput alone and together.

    python scripts/overlap_probe.py [--config C2] [--copy-mb 1024] [--copies 24]
"""
import argparse
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

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="C2")
ap.add_argument("--copy-mb", type=int, default=1024)
ap.add_argument("--copies", type=int, default=24)
ap.add_argument("--reserve", default="0,8,16,32")
args = ap.parse_args()

dev = torch.device("cuda", 0)
cfg = CONFIGS[args.config]
x = synth.pulsar_filterbank_device(cfg, device=dev)
dms = dedispersion_plan(cfg.nchan, cfg.dmmin, cfg.dmmax, cfg.start_freq, cfg.bandwidth, cfg.tsamp)
plan = _hip.Plan(_hip.dtype_code(x.dtype), _hip.PU_ACC_NATIVE, cfg.nchan, cfg.nsamples,
                 _hip.shift_table(cfg.nchan, dms, cfg.start_freq, cfg.bandwidth, cfg.tsamp))
ws = torch.empty(plan.workspace_bytes, dtype=torch.uint8, device=dev)
outs = plan._outs_ws(dev, None, ws)[0]
a = torch.empty(args.copy_mb << 20, dtype=torch.uint8, device=dev)
b = torch.empty_like(a)
cstream = torch.cuda.Stream(device=dev)


def copies():
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(cstream):
        e0.record(cstream)
        for _ in range(args.copies):
            b.copy_(a)
        e1.record(cstream)
    return e0, e1


def search(stream):
    plan.enable_timing(1)
    plan.search(x, out=outs, workspace=ws, stream=stream)
    return float(plan.kernel_times_ms(1)[0])


def copy_gbps(e0, e1):
    e1.synchronize()
    return 2 * args.copies * a.numel() / (e0.elapsed_time(e1) / 1e3) / 1e9


res = {"config": cfg.name, "copy_mb": args.copy_mb, "copies": args.copies}
for _ in range(2):
    search(torch.cuda.current_stream(dev))
res["search_alone_ms"] = float(np.median([search(torch.cuda.current_stream(dev)) for _ in range(3)]))
e0, e1 = copies()
res["copy_alone_GBps"] = copy_gbps(e0, e1)
torch.cuda.synchronize()
for r in [int(v) for v in args.reserve.split(",")]:
    ms = _hip.MaskedStream(r, dev) if r > 0 else None
    s = ms.stream if ms else torch.cuda.Stream(device=dev)
    search(s)  # warm
    torch.cuda.synchronize()
    e0, e1 = copies()
    t = search(s)
    res[f"reserve{r}"] = {"search_ms_with_copies": t, "copy_GBps_with_search": copy_gbps(e0, e1),
                          "copy_window_ms": e0.elapsed_time(e1)}
    torch.cuda.synchronize()
    res[f"reserve{r}"]["search_alone_ms"] = search(s)
    del ms
print(json.dumps(res), flush=True)
