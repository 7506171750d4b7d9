"""Host-side float64 dedispersion planner (reference formula, CPython scalar semantics).

These are the non-hot-path pieces of ``pulsarutils/dedispersion.py`` that the north
star keeps on the host: per-channel integer delays and the DM-trial grid.

Bit-exactness notes (verified against golden vectors from the reference):

* ``x ** (-2)`` is evaluated with libm ``pow`` on scalars, exactly like the
  reference's interpreted loop (``dedispersion.py:130,136``).  numpy's vectorised
  ``np.power`` uses SVML on AVX-512 hosts and differs in the last ulp for ~5 % of
  inputs, so it is NOT used for shifts.
* ``//`` is Python/numpy floor division (fmod-based ``divmod``, snapped quotient).
* The bulk shift table for a whole trial grid is built by the C++ twin
  ``pu_shift_table`` in the HIP library (same libm ``pow``, same ``divmod``);
  ``tests/test_planner.py`` checks both against the goldens and each other.
"""
import math

import numpy as np


def delta_delay(dm, start_freq, stop_freq):
    """``dedispersion.py:142-146``: ``4149*dm*(f1**-2 - f2**-2)`` seconds."""
    delay1 = 4149. * dm * start_freq ** (-2)
    delay2 = 4149. * dm * stop_freq ** (-2)
    return delay1 - delay2


def dedispersion_plan(nchan, dmmin, dmmax, start_freq, bandwidth, sample_time):
    """``dedispersion.py:149-171``: DM grid with a 1-sample whole-band delay step.

    ``np.float`` (removed in numpy>=1.24) is replaced by ``float``; arithmetic order
    is the reference's, so the grid is bit-identical (golden ``plan_C*``).
    """
    stop_freq = start_freq + bandwidth
    f0 = float(start_freq)
    f1 = float(stop_freq)
    max_N = delta_delay(float(dmmax), f0, f1) / sample_time
    min_N = delta_delay(float(dmmin), f0, f1) / sample_time
    trial_N = np.arange(min_N, max_N + 1)
    trial_DM = trial_N * sample_time / 4149. * (f0 ** (-2) - f1 ** (-2)) ** (-1)
    return trial_DM


def _py_floordiv(a, b):
    """CPython ``float.__floordiv__`` / numpy ``npy_floor_divide`` for doubles."""
    return a // b


def dedispersion_shifts(nchan, dm, start_freq, bandwidth, sample_time):
    """``dedispersion.py:125-139``: per-channel integer delays, float64 array.

    Channel ``i`` sits at ``start_freq + i*dfreq`` (lower edge; channel 0 is the
    lowest frequency); delays are relative to the band centre; positive = later.
    """
    nchan = int(nchan)
    dm = float(dm)
    start_freq = float(start_freq)
    bandwidth = float(bandwidth)
    sample_time = float(sample_time)
    dfreq = bandwidth / nchan
    stop_freq = start_freq + bandwidth
    center_freq = (stop_freq + start_freq) / 2
    ref_delay = 4149 * dm * center_freq ** (-2)
    k = 4149 * dm
    shifts = np.zeros(nchan)
    for i in range(nchan):
        chan_freq = start_freq + i * dfreq
        delay = k * chan_freq ** (-2) - ref_delay
        q = delay // sample_time
        shifts[i] = int(round_half_even(q))
    return shifts


def round_half_even(x):
    """``np.rint`` on a Python float."""
    if math.isinf(x) or math.isnan(x):
        raise ValueError("cannot convert non-finite delay to an integer shift")
    return float(np.rint(x))


def normalize_shifts(shifts, N):
    """``dedispersion.py:101-122``: ``rint(shift) mod N`` into ``[0, N)`` as int32.

    The reference's ``while`` loops compute the Python modulo; this is the closed form.
    """
    s = np.rint(np.asarray(shifts, dtype=np.float64).ravel())
    out = np.mod(s, N)
    return out.astype(np.int32)
