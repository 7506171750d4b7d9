"""Time pu_gaussian_filter1d (C4 light curve: n = 2^18, radius 404) in this process's
PU_GAUSS_FORM and check it bit for bit against the pair form's output saved by the first
run (gpurun_out/gauss_ref.npy).  One JSON line."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "radio-pulsar-utils_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from pulsarutils import _hip, clean  # noqa: E402

n = 1 << 18
g = torch.Generator().manual_seed(5)
x = (torch.randn(n, generator=g, dtype=torch.float64) * 3 + 100).cuda()
out = torch.empty_like(x)
w, r = clean._gaussian_weights(101.0)  # the C4 baseline window (radius 404)
wt = torch.from_numpy(w).cuda()
lib = _hip.lib()
run = lambda: lib.pu_gaussian_filter1d(_hip.ptr(x), n, _hip.ptr(wt), r, _hip.ptr(out), _hip.stream_ptr())
for _ in range(3):
    run()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(50):
    run()
e1.record()
torch.cuda.synchronize()
res = out.cpu().numpy()
ref = os.path.join(REPO, "gpurun_out", "gauss_ref.npy")
if not os.path.exists(ref):
    np.save(ref, res)
same = bool(np.array_equal(np.load(ref).view(np.int64), res.view(np.int64)))
print(json.dumps({"form": os.environ.get("PU_GAUSS_FORM", "0"), "us": round(e0.elapsed_time(e1) / 50 * 1e3, 2),
                  "bit_equal_first_run": same}))
