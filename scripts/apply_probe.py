"""Time pu_renorm_apply alone (the apply pass of renormalize_data, clean.py:81-94) on the C4
shape with HIP events, per input dtype: median of 20 launches (col-mean output on, as with
cut_outliers).  PULSARUTILS_HIP_LIB picks the library (A/B of kernel variants)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "radio-pulsar-utils_amd"), REPO]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from pulsarutils import _hip, synth  # noqa: E402
from pulsarutils.configs import CONFIGS  # noqa: E402

cfg = CONFIGS["C4"]
lib = _hip.lib()
res = {"lib": os.environ.get("PULSARUTILS_HIP_LIB", "in-tree")}
for dt in ("u8", "f32"):
    x = _hip.to_device(synth.rfi_filterbank_np(cfg, dtype=dt))
    nchan, n = x.shape
    dev = x.device
    f = torch.rand(n, dtype=torch.float64, device=dev) + 0.5
    spec = torch.rand(nchan, dtype=torch.float64, device=dev) * 50 + 1.0
    bad = torch.zeros(nchan, dtype=torch.uint8, device=dev)
    bad[::37] = 1
    out = torch.empty((nchan, n), dtype=torch.float64, device=dev)
    col = torch.empty(n, dtype=torch.float64, device=dev)
    s = _hip.stream_ptr()

    def run():
        _hip.check(lib.pu_renorm_apply(_hip.ptr(x), _hip.dtype_code(x.dtype), nchan, n, x.stride(0), _hip.ptr(f),
                                       _hip.ptr(spec), _hip.ptr(bad), _hip.ptr(out), out.stride(0), _hip.ptr(col), s),
                   "pu_renorm_apply")
    run()
    torch.cuda.synchronize()
    ms = []
    for _ in range(20):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        run()
        b.record()
        torch.cuda.synchronize()
        ms.append(a.elapsed_time(b))
    # reference: numpy's (x*f - mu)/mu of a few rows, bit for bit
    xs = x[:8].cpu().numpy().astype(np.float64)
    want = (xs * f.cpu().numpy() - spec[:8, None].cpu().numpy()) / spec[:8, None].cpu().numpy()
    want[bad[:8].cpu().numpy().astype(bool)] = 0.0
    exact = bool(np.array_equal(out[:8].cpu().numpy(), want))
    nb = x.numel() * x.element_size() + out.numel() * 8
    med = float(np.median(ms))
    res[dt] = {"apply_ms": round(med, 4), "GBps": round(nb / med / 1e6, 1), "rows_bit_exact": exact}
    del x, out
print(json.dumps(res), flush=True)
