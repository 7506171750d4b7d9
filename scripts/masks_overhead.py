"""Host-side cost of the channel-masks step (get_noisier_channels +
measure_channel_variability) on the C4 f32 filterbank: wall time of each call, the Python
time before the first kernel is queued, the read-back, and the helpers they use.

Usage: python scripts/masks_overhead.py [--dtype f32|u8] [--iters N]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "radio-pulsar-utils_amd"), REPO]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from pulsarutils import _hip, clean as C, synth  # noqa: E402
from pulsarutils.configs import CONFIGS  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--dtype", default="f32")
ap.add_argument("--iters", type=int, default=50)
args = ap.parse_args()
x = _hip.to_device(synth.rfi_filterbank_np(CONFIGS["C4"], dtype=args.dtype))
for _ in range(5):
    C.invalidate_channel_means()
    C.measure_channel_variability(x, badchans_mask=C.get_noisier_channels(x))
torch.cuda.synchronize()
pc = time.perf_counter


def avg(fn, n=args.iters, sync=True):
    ts = []
    for _ in range(n):
        if sync:
            torch.cuda.synchronize()
        t = pc()
        fn()
        ts.append(pc() - t)
    torch.cuda.synchronize()
    return round(float(np.median(ts)) * 1e6, 1)


out = {}
# whole step and its two calls
def step():
    C.invalidate_channel_means()
    bad = C.get_noisier_channels(x)
    return C.measure_channel_variability(x, badchans_mask=bad)
out["step_us"] = avg(step)
bad = C.get_noisier_channels(x)
out["measure_channel_variability_cached_us"] = avg(lambda: C.measure_channel_variability(x, badchans_mask=bad))
# the means pass: Python until its kernels are queued (GPU idle at the start)
out["means_pass_launch_us"] = avg(lambda: (C.invalidate_channel_means(), C._cached_stats(x)))
# helpers
out["to_device_us"] = avg(lambda: _hip.to_device(x), sync=False)
out["stream_ptr_us"] = avg(lambda: _hip.stream_ptr(), sync=False)
out["torch_empty_us"] = avg(lambda: torch.empty(1024, dtype=torch.float32, device=x.device), sync=False)
res = torch.zeros(2 * 1028, dtype=torch.uint8, device=x.device)
out["readback_cpu_numpy_us"] = avg(lambda: res.cpu().numpy())
pin = torch.empty(res.numel(), dtype=torch.uint8, pin_memory=True)
out["readback_pinned_sync_us"] = avg(lambda: (pin.copy_(res, non_blocking=True),
                                              torch.cuda.current_stream().synchronize(), pin.numpy()))
print(json.dumps(out), flush=True)
