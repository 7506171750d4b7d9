"""Plan statistics for the subband mode (no GPU): distinct relative-shift vectors
("slots") per (DM tile, group) and distinct windows per (wave, group) for a config."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "radio-pulsar-utils_amd"), REPO]
import numpy as np  # noqa: E402
from pulsarutils import _hip  # noqa: E402
from pulsarutils.configs import CONFIGS  # noqa: E402
from pulsarutils.dedispersion import dedispersion_plan  # noqa: E402

cfg = CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "C2"]
dms = dedispersion_plan(cfg.nchan, cfg.dmmin, cfg.dmmax, cfg.start_freq, cfg.bandwidth, cfg.tsamp)
sh = _hip.shift_table(cfg.nchan, dms, cfg.start_freq, cfg.bandwidth, cfg.tsamp)
ndm = sh.shape[0]
for G in (2, 4, 8):
    ng = cfg.nchan // G
    g = sh[:, :ng * G].reshape(ndm, ng, G)
    vec = g - g[:, :, :1]
    for T in (64, 128, 256):
        slots = []
        for t0 in range(0, ndm, T):
            v = vec[t0:t0 + T]
            for j in range(ng):
                slots.append(len({tuple(r) for r in v[:, j, 1:]}))
        # distinct (vector, b) windows per 8-trial wave
        win = []
        for t0 in range(0, ndm, 8):
            v = vec[t0:t0 + 8]
            b = g[t0:t0 + 8, :, 0]
            for j in range(0, ng, 7):
                win.append(len({tuple(r) + (bb,) for r, bb in zip(v[:, j, 1:], b[:, j])}))
        slot = np.mean(slots)
        print(f"G={G} T={T}: slots/group/tile {slot:.2f}  build-reads/channel/trial "
              f"{slot * G / T / G:.3f}  distinct windows per 8 trials {np.mean(win):.2f}")
