"""Timing + bit check of renormalize_data's light-curve chain (pu_lc_factor) on the C4 length.

  factor = median(gaussian_filter(lc, sigma)) / gaussian_filter(lc, sigma)   (clean.py:77-82)

Checks every repetition's factor bit for bit against scipy's gaussian_filter + np.median on
the host (a new random light curve each time, every fifth with many ties), then times --steps back-to-back calls with HIP events.  (Round 5 A/B of a
one-launch form with grid barriers: profiles/r05/experiments/lc_factor_fused.log.)

usage: python scripts/bench_lc.py [--n 262144] [--sigma 101] [--checks 20] [--steps 200]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "radio-pulsar-utils_amd"), REPO]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from scipy.ndimage import gaussian_filter  # noqa: E402
from pulsarutils import _hip, clean  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=1 << 18)
ap.add_argument("--sigma", type=int, default=101)
ap.add_argument("--checks", type=int, default=20)
ap.add_argument("--steps", type=int, default=200)
args = ap.parse_args()

dev = torch.device("cuda:0")
w, radius = clean._gaussian_weights_device(args.sigma, dev)
rng = np.random.default_rng(5)
bad = 0
for i in range(args.checks):
    lc = 100.0 + np.cumsum(rng.standard_normal(args.n)) * 0.01 + rng.standard_normal(args.n)
    if i % 5 == 4:
        lc = np.round(lc, 1)  # many ties
    d = torch.from_numpy(lc).to(dev)
    med = torch.empty(1, dtype=torch.float64, device=dev)
    f = clean.light_curve_factor(d, w, radius, median_out=med).cpu().numpy()
    sm = gaussian_filter(lc, args.sigma)
    ref = np.median(sm) / sm
    if not np.array_equal(f, ref) or med.item() != np.median(sm):
        bad += 1
        print(f"check {i}: MISMATCH {np.count_nonzero(f != ref)} elements, median {med.item()!r} vs "
              f"{np.median(sm)!r}", flush=True)
d = torch.from_numpy(lc).to(dev)
for _ in range(5):
    clean.light_curve_factor(d, w, radius)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(args.steps):
    clean.light_curve_factor(d, w, radius)
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) * 1e3 / args.steps
print(json.dumps({"step": "lc_factor", "n": args.n, "sigma": args.sigma, "us": round(us, 2),
                  "checks": args.checks, "mismatches": bad}))
sys.exit(1 if bad else 0)
