"""Cleaning-pass timing on the C4 shape (BASELINE configs[3]).

Usage: python scripts/bench_clean.py [--dtype f32|u8] [--steps K]
Times, with torch events on torch's current stream (the one the C-ABI calls are
given), each device step of the reference's cleaning pass on a resident
1024 x 2^18 RFI-heavy filterbank:
  means     channel_means_device      (clean.py:58-67 spectrum)
  var       channel_variances_device  (clean.py:114-133 np.std)
  masks     get_noisier_channels + measure_channel_variability (clean.py:58-67, 114-133)
  renorm    renormalize_device(cut_outliers=True) (clean.py:70-111; includes the
            host median / threshold round trips the reference formula needs)
and prints one JSON line per step with algorithmic HBM bytes and GB/s vs the
8 TB/s HBM peak.  Run it under `rocprofv3 --kernel-trace --stats` and feed the
stats CSV to scripts/clean_roofline.py for per-kernel numbers.
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "radio-pulsar-utils_amd"), REPO]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from pulsarutils import _hip, clean, synth  # noqa: E402
from pulsarutils.configs import CONFIGS  # noqa: E402

HBM_PEAK_GBPS = 8000.0

ap = argparse.ArgumentParser()
ap.add_argument("--dtype", default="f32")
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--warmup", type=int, default=3)
args = ap.parse_args()

cfg = CONFIGS["C4"]
host = synth.rfi_filterbank_np(cfg, dtype=args.dtype)
x = _hip.to_device(host)
nchan, n = x.shape
b_in = x.element_size()
bad = clean.measure_channel_variability(x) | clean.get_noisier_channels(x)
out = torch.empty((nchan, n), dtype=torch.float64, device=x.device)
means = clean.channel_means_device(x)

plane = nchan * n * b_in
steps = {
    # algorithmic bytes: one read of the filterbank (+ its per-row outputs)
    # invalidate first: the channel-means cache would return the previous step's means
    "means": (lambda: (clean.invalidate_channel_means(), clean.channel_means_device(x))[1], plane),
    "var": (lambda: clean.channel_variances_device(x, means), plane),
    # col means (1 read) + factor-weighted row sums (1 read + factor) + apply
    # (1 read + float64 write + column means); small 1-D passes counted too
    # both channel masks from scratch (bench.py's masks step): one read pass + decisions
    "masks": (lambda: (clean.invalidate_channel_means(),
                       clean.measure_channel_variability(x, badchans_mask=clean.get_noisier_channels(x)))[1], plane),
    "renorm": (lambda: clean.renormalize_device(x, bad, cut_outliers=True, out=out),
               3 * plane + nchan * n * 8 + 6 * n * 8),
}
for name, (fn, nbytes) in steps.items():
    for _ in range(args.warmup):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.steps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.steps
    gbps = nbytes / (ms * 1e-3) / 1e9
    print(json.dumps({"step": name, "dtype": args.dtype, "shape": [nchan, n], "ms": round(ms, 4),
                      "alg_bytes": nbytes, "GBps": round(gbps, 1), "hbm_frac": round(gbps / HBM_PEAK_GBPS, 3)}),
          flush=True)
print("bad channels", int(np.count_nonzero(bad)), flush=True)
