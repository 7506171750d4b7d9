"""Synthetic SIGPROC files for the file-statistics tests (shared with make_golden.py)."""
import os

import numpy as np


def stats_file_data(dt):
    """Time-major (25000, 64) block with hot / noisy channels (seeds 88 / 89)."""
    rng = np.random.default_rng(88 if dt == "u8" else 89)
    nch, ns = 64, 25000
    lvl = 40 + 10 * np.sin(np.arange(nch) / 9.0)
    lvl[[5, 17, 40]] *= 2.5
    sig = np.full(nch, 6.0)
    sig[[22, 50]] *= 3
    x = rng.standard_normal((ns, nch)).astype(np.float32) * sig + lvl
    return np.clip(np.rint(x), 0, 255).astype(np.uint8) if dt == "u8" else x.astype(np.float32)


def write_stats_file(dirname, dt):
    from pulsarutils import sigproc
    x = stats_file_data(dt)
    fname = os.path.join(dirname, f"syn_{dt}.fil")
    sigproc.write_filterbank(fname, x, fch1=1500.0, foff=-300.0 / x.shape[1], tsamp=64e-6)
    return fname, x
