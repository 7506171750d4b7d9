"""Probe: does running the factor-weighted row sums and the apply pass strip by strip of
rows (so the apply re-reads x while the strip is still in the MALL) beat the two full
passes?  Timing only (the column-mean accumulator is left out), C4 f32 and u8.

    python scripts/strip_probe.py [reps]
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "radio-pulsar-utils_amd"), REPO]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from pulsarutils import _hip, clean, synth  # noqa: E402
from pulsarutils.configs import CONFIGS  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
cfg = CONFIGS["C4"]
lib = _hip.lib()
for dt in ("f32", "u8"):
    x = synth.pulsar_filterbank_device(cfg, dtype=dt)
    nchan, n = x.shape
    code = _hip.dtype_code(x.dtype)
    factor = torch.ones(n, dtype=torch.float64, device=x.device)
    out = torch.empty((nchan, n), dtype=torch.float64, device=x.device)
    s = _hip.stream_ptr()

    def run(S):
        for r0 in range(0, nchan, S):
            xs = x[r0:r0 + S]
            spec = clean._row_sums(xs, 2, scale=factor, divisor=n)
            _hip.check(lib.pu_renorm_apply(_hip.ptr(xs), code, xs.shape[0], n, x.stride(0), _hip.ptr(factor),
                                           _hip.ptr(spec), None, _hip.ptr(out[r0:]), out.stride(0), None, s),
                       "apply")

    res = {}
    for S in (nchan, 512, 256, 128, 64, 32):
        for _ in range(2):
            run(S)
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            run(S)
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        res[S] = float(np.median(ts))
        print(json.dumps({"dtype": dt, "strip_rows": S, "ms": round(res[S], 4)}), flush=True)
