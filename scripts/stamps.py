"""Phase breakdown of the subband kernel from in-kernel shader-clock stamps.

Loads the diagnostic library (make -C radio-pulsar-utils_amd/csrc stamps; PU_STAMPS),
runs the C2 search a few times and prints each phase's share of the summed wave
cycles (stamps drain the LDS queue at every phase boundary: read the SHARES, not the
run time - cdna_hip_programming.md §7).

    python scripts/stamps.py [config] [launches]
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("PULSARUTILS_HIP_LIB", os.path.join(REPO, "radio-pulsar-utils_amd", "pulsarutils", "_lib",
                                                          "libpulsarutils_hip_stamps.so"))
sys.path[:0] = [os.path.join(REPO, "radio-pulsar-utils_amd"), REPO]
import ctypes  # noqa: E402
import numpy as np  # noqa: E402
import torch  # noqa: E402
from pulsarutils import _hip, synth  # noqa: E402
from pulsarutils.configs import CONFIGS  # noqa: E402
from pulsarutils.dedispersion import dedispersion_plan  # noqa: E402

PHASES = ("metadata", "barrier_A_wait", "build", "barrier_B_wait", "dma_issue", "sum", "epilogue", "dma_wait")


def main():
    cfg = CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "C2"]
    launches = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    x = synth.pulsar_filterbank_device(cfg)
    dms = dedispersion_plan(cfg.nchan, cfg.dmmin, cfg.dmmax, cfg.start_freq, cfg.bandwidth, cfg.tsamp)
    ntr = int(os.environ.get("PU_TRIALS", "0"))
    if ntr:
        dms = dms[:ntr]
    sh = _hip.shift_table(cfg.nchan, dms, cfg.start_freq, cfg.bandwidth, cfg.tsamp)
    plan = _hip.Plan(_hip.dtype_code(x.dtype), _hip.PU_ACC_NATIVE, cfg.nchan, cfg.nsamples, sh)
    out = np.zeros(8, np.int64)
    buf = out.ctypes.data_as(ctypes.c_void_p)
    ws = torch.empty(plan.workspace_bytes, dtype=torch.uint8, device=x.device)
    plan.search(x, workspace=ws)
    _hip.lib().pu_plan_stamps(plan._h, buf, 8)  # arm
    for _ in range(launches):
        plan.search(x, workspace=ws)
    m = _hip.lib().pu_plan_stamps(plan._h, buf, 8)
    if m <= 0:
        print("not a stamps build", file=sys.stderr)
        return
    tot = float(out[:8].sum())
    rec = {"config": cfg.name, "plan": {k: plan.info[k] for k in ("group", "stages", "dm_tiles", "time_tiles")},
           "env": {k: os.environ.get(k) for k in ("PU_SUB_SHAPE", "PU_GROUP") if os.environ.get(k)},
           "share": {p: round(float(out[i]) / tot, 4) for i, p in enumerate(PHASES)},
           "wave_cycles_per_launch": tot / launches}
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
