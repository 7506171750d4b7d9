"""Select build vs direct build of 8-bit slots: where the dedispersed planes differ.

    PULSARUTILS_HIP_LIB=ab/lib_<x>.so python scripts/sel_diag.py

C3's channelisation, 1024 channels x 2^15 samples, DM 0-12 (every group eligible).  Prints
the plan info, the number of differing samples per trial and, for the first differing
trial, the first differing sample indices with the two values and the oracle's.
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "radio-pulsar-utils_amd"), REPO]
import numpy as np  # noqa: E402
from pulsarutils import _hip  # noqa: E402
from pulsarutils.configs import CONFIGS  # noqa: E402

c = CONFIGS["C3"]
nchan, n = 1024, 1 << 15
rng = np.random.default_rng(3)
x = (rng.random((nchan, n)) * 255).astype(np.uint8)
dms = np.linspace(0.0, 12.0, 300)
sh = _hip.shift_table(nchan, dms, c.start_freq, c.bandwidth, c.tsamp)
xd = _hip.to_device(x)
for group, shape in ((8, 2), (4, 2), (8, 0)):
    sel = _hip.Plan(_hip.PU_U8, _hip.PU_ACC_NATIVE, nchan, n, sh, group=group, shape=shape, select_build=True)
    direct = _hip.Plan(_hip.PU_U8, _hip.PU_ACC_NATIVE, nchan, n, sh, group=group, shape=shape, select_build=False)
    print("G", group, "shape", shape, "sel info", sel.info.get("select_build"), flush=True)
    a, b = sel.dedisperse(xd).cpu().numpy(), direct.dedisperse(xd).cpu().numpy()
    bad = (a != b).sum(axis=1)
    print("  trials differing", int((bad > 0).sum()), "of", a.shape[0], "samples differing", int(bad.sum()), flush=True)
    if bad.any():
        k = int(np.argmax(bad > 0))
        idx = np.nonzero(a[k] != b[k])[0]
        ref = np.zeros(n)
        for ch in range(nchan):
            ref += np.roll(x[ch].astype(np.float64), -int(sh[k, ch]))
        print("  first trial", k, "dm", dms[k], "count", idx.size, "first idx", idx[:16].tolist(), flush=True)
        print("  idx mod 64", np.bincount(idx % 64, minlength=64).tolist(), flush=True)
        for i in idx[:6]:
            print(f"   t {i}: sel {a[k, i]} direct {b[k, i]} oracle {ref[i]}", flush=True)
        print("  direct == oracle at trial k:", bool(np.array_equal(b[k].astype(np.float64), ref)), flush=True)
