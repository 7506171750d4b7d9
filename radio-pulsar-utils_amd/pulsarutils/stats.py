"""Drop-in ``pulsarutils.stats`` (reference: pulsarutils/stats.py).

``ref_mad`` / ``mad`` act on 1-D spectra (nchan values) and stay on the host, with
statsmodels 0.12.2's ``robust.mad`` restated (the reference imports statsmodels
without declaring it, ``stats.py:4``; statsmodels is not in this image).  The
2-D reductions that feed them run on the GPU (``clean.py``).
"""
import numpy as np
from scipy.stats import norm

# statsmodels.robust.scale.mad default normalisation: Gaussian.ppf(3/4.)
MAD_C = norm.ppf(3 / 4.)


def mad(a, c=MAD_C, axis=0, center=np.median):
    """statsmodels 0.12.2 ``robust.mad``: ``median(|a - center(a)| / c)`` along ``axis``."""
    a = np.asarray(a)
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
