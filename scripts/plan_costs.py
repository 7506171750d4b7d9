"""Plan tables of the tall 16-bit-slot C3 plans (G = 4 and 8) at 625 and 5000 trials: the
planner's cost-model inputs (LDS bytes, stages, 16-bit windows) per plan, for refitting its
terms against measured times."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "radio-pulsar-utils_amd"), REPO]
import numpy as np  # noqa: E402
from pulsarutils import _hip  # noqa: E402
from pulsarutils.configs import CONFIGS  # noqa: E402
from pulsarutils.dedispersion import dedispersion_plan  # noqa: E402

c = CONFIGS["C3"]
dms_all = dedispersion_plan(c.nchan, c.dmmin, c.dmmax, c.start_freq, c.bandwidth, c.tsamp)
for ntr in (625, 5000):
    sh = _hip.shift_table(c.nchan, dms_all[:ntr], c.start_freq, c.bandwidth, c.tsamp)
    for g in (0, 4, 8):
        p = _hip.Plan(_hip.PU_U8, _hip.PU_ACC_NATIVE, c.nchan, c.nsamples, sh, group=g, shape=None if g == 0 else 2)
        i = p.info
        first, count = p.dm_tiles()
        ngroups = -(-c.nchan // i["group"])
        win = int(sum(-(-int(k) // 16) * 16 for k in count)) * ngroups * i["time_tiles"]
        print(json.dumps({"trials": ntr, "group_req": g, "group": i["group"], "stages": i["stages"],
                          "lds_traffic": i["lds_traffic"], "windows16": win, "time_tiles": i["time_tiles"],
                          "slots": i["slots"], "kernel": i["kernel"]}), flush=True)
