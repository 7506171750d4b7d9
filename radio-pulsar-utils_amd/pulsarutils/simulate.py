"""Drop-in ``pulsarutils.simulate`` (reference: pulsarutils/simulate.py:6-28).

Host-side test-input generator: an impulse at ``nsamples // 2`` in every channel,
``|normal(array, noise)|`` from numpy's GLOBAL legacy RandomState (so
``np.random.seed(s)`` reproduces the reference's arrays bit for bit; the inputs'
SHA-256 are pinned in tests/golden), then channel i rolled by ``+shift_i``.
"""
import numpy as np

from ._planner import dedispersion_shifts


def simulate_test_data(dm=150, tsamp=0.0005, nsamples=1024, nchan=128, start_freq=1200., bandwidth=200.,
                       signal=1., noise=0.5):
    array = np.zeros((nchan, nsamples))
    array[:, nsamples // 2] = signal
    array = np.abs(np.random.normal(array, noise))
    nchan = array.shape[0]
    shifts = dedispersion_shifts(nchan, dm, start_freq, bandwidth, tsamp)
    for i in range(nchan):
        array[i, :] = np.roll(array[i, :], int(shifts[i]))
    header = {"bandwidth": bandwidth, "fbottom": start_freq, "foff": bandwidth / nchan, "nchans": nchan,
              "nsamples": nsamples, "tsamp": tsamp}
    return array, header
