"""Where a search step's time goes besides the kernel (C5 / C1 / C2 on one GPU).

Per config: the mean wall time per step of
* ``search``      plan.search (sub kernel + finalize + certification read-back + sync)
* ``tiles``       plan.search_tiles over all tiles (the kernel alone, no sync per step)
* ``finalize``    plan.finalize alone (finalize kernel + certification read-back + sync)
* ``ctypes``      the Python validation + ctypes path of search_tiles on an empty range
and the kernel's own HIP-event time.  Prints one JSON line per config.
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "radio-pulsar-utils_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from pulsarutils import _hip, synth  # noqa: E402
from pulsarutils.configs import CONFIGS  # noqa: E402
from pulsarutils.dedispersion import dedispersion_plan  # noqa: E402


def timed(fn, k):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / k * 1e3


def main():
    names = sys.argv[1:] or ["C5", "C1", "C2"]
    dev = torch.device("cuda:0")
    for name in names:
        cfg = CONFIGS[name]
        x = synth.pulsar_filterbank_device(cfg, device=dev)
        dms = dedispersion_plan(cfg.nchan, cfg.dmmin, cfg.dmmax, cfg.start_freq, cfg.bandwidth, cfg.tsamp)
        sh = _hip.shift_table(cfg.nchan, dms, cfg.start_freq, cfg.bandwidth, cfg.tsamp)
        plan = _hip.Plan(_hip.dtype_code(x.dtype), _hip.PU_ACC_NATIVE, cfg.nchan, cfg.nsamples, sh)
        ws = torch.empty(plan.workspace_bytes, dtype=torch.uint8, device=dev)
        outs = (torch.empty(dms.size, dtype=torch.float64, device=dev),
                torch.empty(dms.size, dtype=torch.float64, device=dev),
                torch.empty(dms.size, dtype=torch.float64, device=dev),
                torch.empty(dms.size, dtype=torch.int32, device=dev))
        ntt = plan.info["time_tiles"]
        k = 200 if cfg.nchan * cfg.nsamples * dms.size < 2e11 else 10
        res = {"config": name, "steps": k, "ndm": int(dms.size)}
        for _ in range(3):
            plan.search(x, out=outs, workspace=ws)
        plan.enable_timing(k)
        res["search_ms"] = timed(lambda: plan.search(x, out=outs, workspace=ws), k)
        res["kernel_ms"] = float(np.mean(plan.kernel_times_ms(k)))
        res["tiles_ms"] = timed(lambda: plan.search_tiles(x, 0, ntt, ws), k)
        res["ctypes_empty_ms"] = timed(lambda: plan.search_tiles(x, 0, 0, ws), k)
        res["finalize_ms"] = timed(lambda: plan.finalize(ws, x, out=outs), k)
        print(json.dumps(res), flush=True)
        del x, ws, outs, plan
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
