"""PCIe-inclusive rate of the numpy drop-in (`_dedispersion_search` with a host array).

The bench's `value` keeps inputs resident in HBM (the metric); this times what a user of
the reference's numpy API sees: host filterbank -> H2D copy -> plan -> search -> numpy out.
Usage: python scripts/pcie_rate.py [config]   (prints one JSON line)
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "radio-pulsar-utils_amd"), REPO]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from pulsarutils import dedispersion as D, synth  # noqa: E402
from pulsarutils.configs import CONFIGS  # noqa: E402

cfg = CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "C2"]
x = synth.pulsar_filterbank_device(cfg).cpu().numpy()
dms = D.dedispersion_plan(cfg.nchan, cfg.dmmin, cfg.dmmax, cfg.start_freq, cfg.bandwidth, cfg.tsamp)
D._dedispersion_search(x[:, :8192], dms[:4], cfg.nchan, cfg.start_freq, cfg.bandwidth, cfg.tsamp)
res = {}
for rep in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    xd = torch.from_numpy(x).cuda()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    out = D._dedispersion_search(x, dms, cfg.nchan, cfg.start_freq, cfg.bandwidth, cfg.tsamp)
    t2 = time.perf_counter()
    del xd
    res.setdefault("h2d_s", []).append(t1 - t0)
    res.setdefault("numpy_api_s", []).append(t2 - t1)
h2d = float(np.median(res["h2d_s"]))
cold = res["numpy_api_s"][0]  # first call builds the plan on the host
api = float(np.median(res["numpy_api_s"][1:]))  # later calls hit the plan cache
print(json.dumps({"config": cfg.name, "bytes": int(x.nbytes), "h2d_s": h2d, "h2d_GBps": x.nbytes / h2d / 1e9,
                  "numpy_api_cold_s": cold, "numpy_api_cold_samples_per_s": dms.size * cfg.nsamples / cold,
                  "numpy_api_s": api, "numpy_api_samples_per_s": dms.size * cfg.nsamples / api,
                  "best_dm": float(dms[np.argmax(out[2])])}))
