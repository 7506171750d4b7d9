"""HBM ceilings of the cleaning pass's traffic shapes on one MI355X (torch's own kernels).

    python scripts/hbm_ceiling.py   -> one JSON line per shape

C4's plane (1024 x 2^18): f64 fill (write only), f32 -> f64 and u8 -> f64 converting
copies (the apply pass's read:write mix, 1:2 and 1:8 bytes), f32 sum (read only).  Median
of 20 launches timed with HIP events on torch's current stream.
"""
import json

import torch

nchan, n = 1024, 1 << 18
dev = torch.device("cuda:0")
x32 = torch.rand((nchan, n), device=dev, dtype=torch.float32)
x8 = (x32 * 255).to(torch.uint8)
y = torch.empty((nchan, n), device=dev, dtype=torch.float64)


def timed(fn, nbytes, name):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(20):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    ms = ts[len(ts) // 2]
    print(json.dumps({"shape": name, "us": round(ms * 1e3, 1), "bytes": nbytes,
                      "TBps": round(nbytes / ms / 1e9, 3)}), flush=True)


timed(lambda: y.fill_(1.0), y.numel() * 8, "fill f64")
timed(lambda: y.copy_(x32), x32.numel() * 12, "copy f32->f64")
timed(lambda: y.copy_(x8), x8.numel() * 9, "copy u8->f64")
timed(lambda: x32.sum(dtype=torch.float32), x32.numel() * 4, "sum f32 (read)")
timed(lambda: x32.sum(dim=0), x32.numel() * 4, "column sums f32 (read, axis 0)")
timed(lambda: x32.sum(dim=1), x32.numel() * 4, "row sums f32 (read, axis 1)")
