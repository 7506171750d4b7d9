"""Drop-in ``pulsarutils.stats`` (reference: pulsarutils/stats.py).

``ref_mad`` / ``mad`` act on 1-D spectra (nchan values) and stay on the host, with
statsmodels 0.12.2's ``robust.mad`` restated (the reference imports statsmodels
without declaring it, ``stats.py:4``; statsmodels is not in this image).  The 2-D
reductions that feed them run on the GPU: ``get_spectral_stats`` streams a SIGPROC
file through HBM in the reference's 10000-sample chunks and sums each chunk with the
numpy-order HIP row reduction (``pu_row_sums`` modes 3/4), so the per-channel mean /
std spectra, the bad-channel mask and the ``.badchans`` cache are bit-identical to
the reference's.
"""
import logging
import os

import numpy as np
from scipy.signal import medfilt
from scipy.stats import norm

log = logging.getLogger("pulsarutils")

# statsmodels.robust.scale.mad default normalisation: Gaussian.ppf(3/4.)
MAD_C = norm.ppf(3 / 4.)


def mad(a, c=MAD_C, axis=0, center=np.median):
    """statsmodels 0.12.2 ``robust.mad``: ``median(|a - center(a)| / c)`` along ``axis``.

    The input is converted to float64 first, as statsmodels' ``array_like(a, "a",
    ndim=None)`` does (its default ``dtype=np.double``, robust/scale.py:49), so a float32
    input's median and deviations are float64."""
    a = np.asarray(a, dtype=np.double)
    if callable(center) and a.size:
        center = np.apply_over_axes(center, a, axis)
    else:
        center = 0.0
    return np.median((np.abs(a - center)) / c, axis=axis)


def ref_mad(array, window=1):
    """stats.py:11-32: MAD of the first difference divided by sqrt(2).

    ``window`` is accepted and ignored, as in the reference.
    """
    return mad(np.diff(array)) / np.sqrt(2)


def _chunk_row_sums(block, mode):
    """float64 per-channel sum (mode 3) or sum of squares (mode 4) of a device block."""
    from . import _hip
    t = _hip.torch()
    nrows, n = block.shape
    out = t.empty(nrows, dtype=t.float64, device=block.device)
    ws = t.empty(max(16, _hip.lib().pu_row_sums_workspace_bytes(nrows, n)), dtype=t.uint8, device=block.device)
    _hip.check(_hip.lib().pu_row_sums(_hip.ptr(block), _hip.dtype_code(block.dtype), nrows, n, block.stride(0), mode,
                                      None, None, 0.0, _hip.ptr(out), _hip.ptr(ws), ws.numel(), _hip.stream_ptr()),
               "pu_row_sums")
    return out


def get_spectral_stats(fname, chunksize=10000, show=False):
    """stats.py:35-60: per-channel mean and std over the whole file, chunk by chunk.

    ``spectrum = 0. + sum_k astype(float).sum(1)`` accumulated in chunk order on the
    host from the exact per-chunk GPU sums; ``std = sqrt(E[x^2] - E[x]^2)``.
    """
    from . import _hip
    from .sigproc import FilReader
    log.info("Getting spectral statistics...")
    fil = FilReader(fname) if isinstance(fname, (str, os.PathLike)) else fname
    nsamples = fil.header["nsamples"]
    spectrum = 0.
    spectrsq = 0.
    for istart in range(0, nsamples, chunksize):
        size = min(chunksize, nsamples - istart)
        block = fil.read_block_device(istart, size)
        if _hip.dtype_code(block.dtype) is None:
            block = block.to(_hip.torch().float64)
        local_spec = _chunk_row_sums(block, 3).cpu().numpy()
        local_sq = _chunk_row_sums(block, 4).cpu().numpy()
        spectrum += local_spec
        spectrsq += local_sq
    mean_spec = spectrum / nsamples
    mean_spectrsq = spectrsq / nsamples
    std_spec = np.sqrt(mean_spectrsq - mean_spec ** 2)
    return mean_spec, std_spec


def get_bad_chans(fname, show=False, cache=None):
    """stats.py:63-90: channels above medfilt(11) + 4 ref_mad in the mean or std spectrum.

    Cached as one text row in ``fname + '.badchans'`` (``np.savetxt(fmt='%g')``), reused
    when present, as in the reference.
    """
    if cache is None:
        cache = fname + ".badchans"
    if os.path.exists(cache):
        return np.loadtxt(cache).astype(bool)
    mean_spec, mean_std = get_spectral_stats(fname, show=show)
    badchans = np.zeros(mean_spec.size, dtype=bool)
    chans = np.arange(mean_spec.size)
    for spec in (mean_spec, mean_std):
        smooth_spec = medfilt(spec, 11)
        spec_mad = ref_mad(spec)
        threshold = smooth_spec + 4 * spec_mad
        badchans = badchans | (spec > threshold)
    print(f"Bad chans: {chans[badchans]}")
    np.savetxt(cache, [badchans], fmt="%g")
    return badchans
