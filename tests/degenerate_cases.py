"""Degenerate search inputs (VERDICT r2 "what's missing" 1): all-zero, constant,
NaN/inf-carrying and S/N-tie filterbanks, regenerated from code + seeds.

Shared by ``tests/golden/make_golden.py`` (which runs the REFERENCE's
``_dedispersion_search`` on them and stores only the resulting tables and the input
SHA-256) and by the tests (which rebuild the inputs and compare).  The reference's
rules these pin (``pulsarutils/dedispersion.py:186-201``):

* ``best_snr = 0, best_win = 0`` and only a strictly greater S/N replaces them
  (``snr > best_snr``), so NaN S/N values never win and exact ties keep the
  smaller window;
* ``np.max`` / ``np.std`` propagate NaN;
* ``max(reb) / std(reb)`` with ``std == 0`` gives +-inf or NaN.

Shapes: "small" (32 x 4096, every trial of a 23-trial grid starting at DM 0), "c1"
(C1's 64 x 2^16 with 8 trials) and "c2" (C2's 1024 x 2^20 with 3 trials).
"""
import numpy as np

# (nchan, nsamples, start_freq, bandwidth, tsamp)
SHAPES = {
    "small": (32, 4096, 1200.0, 200.0, 5e-4),
    "c1": (64, 1 << 16, 1200.0, 200.0, 5e-4),
    "c2": (1024, 1 << 20, 1200.0, 300.0, 64e-6),
}


def trial_dms(shape):
    """The trial list of a case: the small grid is the reference's own plan for
    DM 0..15 (23 trials); the large shapes use a few DMs including 0 (all shifts 0)."""
    if shape == "small":
        return None  # dedispersion_plan(32, 0, 15.0, ...) - computed by the caller
    if shape == "c1":
        return np.array([0.0, 0.65, 1.3, 20.0, 100.0, 130.0, 131.0, 164.4285])
    return np.array([0.0, 7.5, 40.0])


SMALL_DM_RANGE = (0.0, 15.0)


def _block(rng, nchan, n, b, hi):
    """Integer values constant over blocks of ``b`` samples: at DM 0 (all shifts 0) the
    dedispersed series is block-constant too, so its 2-, 4- and 8-sample rebinned
    series are exact multiples of the 1-sample one and their S/N tie exactly."""
    v = rng.integers(0, hi, (nchan, -(-n // b)))
    return np.repeat(v, b, axis=1)[:, :n]


def make(case):
    """(shape, data) of a named case."""
    shape, kind, dt = case.split(":")
    nchan, n = SHAPES[shape][:2]
    npdt = {"u8": np.uint8, "f32": np.float32, "f64": np.float64}[dt]
    rng = np.random.default_rng(_seed(case))
    if kind == "zero":
        x = np.zeros((nchan, n), npdt)
    elif kind == "const":
        x = np.full((nchan, n), 7 if dt == "u8" else 0.1, npdt)
    elif kind == "rowconst":
        x = (np.arange(nchan)[:, None] * 0.1 + 0.3 + np.zeros((1, n))).astype(npdt)
    elif kind == "nearconst":
        x = (1000.0 + 1e-3 * rng.standard_normal((nchan, n))).astype(npdt)
    elif kind == "nanchan":
        x = rng.standard_normal((nchan, n)).astype(npdt)
        x[nchan // 3] = np.nan
    elif kind == "nansamp":
        x = rng.standard_normal((nchan, n)).astype(npdt)
        for c, t in zip(rng.integers(0, nchan, 3), rng.integers(0, n, 3)):
            x[c, t] = np.nan
    elif kind == "posinf":
        x = rng.standard_normal((nchan, n)).astype(npdt)
        x[nchan - 1, n // 2] = np.inf
    elif kind == "infs":
        x = rng.standard_normal((nchan, n)).astype(npdt)
        x[1, 5] = np.inf
        x[2, n - 7] = -np.inf
    elif kind == "block8":
        x = _block(rng, nchan, n, 8, 50).astype(npdt)
    else:
        raise KeyError(case)
    return x


def _seed(case):
    import zlib
    return zlib.crc32(case.encode())


def band(case):
    """(nchan, start_freq, bandwidth, tsamp) of a case."""
    nchan, _, f0, bw, ts = SHAPES[case.split(":")[0]]
    return nchan, f0, bw, ts


CASES = [
    "small:zero:u8", "small:zero:f32", "small:zero:f64",
    "small:const:u8", "small:const:f32", "small:const:f64", "small:rowconst:f64", "small:rowconst:f32",
    "small:nearconst:f32",
    "small:nanchan:f32", "small:nansamp:f64", "small:posinf:f32", "small:infs:f64",
    "small:block8:u8", "small:block8:f64", "small:block8:f32",
    "c1:zero:f32", "c1:const:f32", "c1:nanchan:f32", "c1:block8:u8", "c1:const:f64",
    "c2:zero:f32", "c2:const:f32", "c2:nansamp:f32", "c2:block8:f32",
]


def key(case):
    return "deg_" + case.replace(":", "_")
