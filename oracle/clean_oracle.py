"""ORACLE - test infrastructure only.  numpy restatement of the reference cleaning path.

Each function cites the reference source it restates.  They are the bit-exact
CHECKERS for the HIP cleaning kernels (channel masks, time-bin masks and the
renormalised data itself); they are pinned against tests/golden (run of the
reference's own code).  Third-party pieces the reference calls are used as the
reference calls them (scipy.signal.medfilt, scipy.ndimage.gaussian_filter /
uniform_filter1d) or restated (statsmodels.robust.mad 0.12.2, cross-checked
against the real package by tests/golden/make_golden.py).
"""
import numpy as np
from scipy.ndimage import gaussian_filter, uniform_filter1d
from scipy.signal import medfilt
from scipy.stats import norm

# statsmodels 0.12.2 robust.mad normalisation constant (Gaussian.ppf(3/4.))
MAD_C = norm.ppf(3 / 4.)


def mad(a, c=MAD_C):
    """statsmodels 0.12.2 ``robust.scale.mad`` for 1-D input: median(|a - median(a)| / c),
    computed in float64 (``array_like(a, "a", ndim=None)``: default dtype np.double,
    robust/scale.py:49)."""
    a = np.asarray(a, dtype=np.double)
    center = np.apply_over_axes(np.median, a, 0) if a.size else 0.0
    return np.median(np.abs(a - center) / c, axis=0)


def ref_mad(array):
    """stats.py:11-32: MAD of the first difference, / sqrt(2)."""
    return mad(np.diff(array)) / np.sqrt(2)


def noisier_channels(array):
    """clean.py:58-67: mean spectrum above medfilt(7) + 5 ref_mad."""
    spec = np.asarray(array).mean(1)
    return spec > medfilt(spec, 7) + 5 * ref_mad(spec)


def channel_variability(array, badchans_mask=None):
    """clean.py:114-133: per-channel std outside [q2-2(q2-q1), q2+2(q3-q2)].

    Quartile indices come from the UNMASKED channel count (reference quirk).
    """
    spec = np.std(np.asarray(array), axis=1)
    if badchans_mask is None:
        badchans_mask = np.zeros(spec.size, dtype=bool)
    good = np.sort(spec[~badchans_mask])
    q1, q2, q3 = good[spec.size // 4], good[spec.size // 2], good[spec.size // 4 * 3]
    lo = q2 - 2 * (q2 - q1)
    hi = q2 + 2 * (q3 - q2)
    return (spec < lo) | (spec > hi) | badchans_mask


def renormalize(array, badchans_mask=None, baseline_window=101, cut_outliers=False,
                return_badbins=False, zero_dm=False):
    """clean.py:70-111.

    float64 copy; zero-DM series over good channels; gaussian-smoothed
    multiplicative normalisation; per-channel (x - mu)/mu; bad channels zeroed;
    optional zero-DM time-bin cut where only the last window (16) survives.

    ``zero_dm`` (NOT in the reference - parity unpinned, restated from the build's
    documented contract, include/pulsarutils_hip.h pu_renorm_apply_zero_dm): subtract
    S[t]/ngood from the good channels, S = the in-order sum over channels of the
    normalised data; the outlier cut then uses S/nchan (the pre-subtraction mean).
    """
    x = np.asarray(array).astype(float)
    nchan = x.shape[0]
    if badchans_mask is None:
        badchans_mask = np.zeros(nchan, dtype=bool)
    lc = x[~badchans_mask, :].mean(0)
    sigma = min(baseline_window, lc.size // 100 * 2 + 1)
    smooth = gaussian_filter(lc, sigma)
    factor = np.median(smooth) / smooth
    x *= factor[None, :]
    spec = x.mean(1)
    x -= spec[:, None]
    x /= spec[:, None]
    x[badchans_mask, :] = 0
    lc_pre = None
    if zero_dm:
        s = x.sum(0)
        lc_pre = s / nchan
        ngood = nchan - int(np.count_nonzero(badchans_mask))
        if ngood:
            x[~badchans_mask, :] -= (s / ngood)[None, :]
    bad_bins = None
    if cut_outliers:
        lc = x.mean(0) if lc_pre is None else lc_pre
        window = 16
        lc_rebin = uniform_filter1d(lc, window)
        sd = np.std(lc_rebin[::window])
        bad_bins = (lc_rebin > 5 * sd) | (lc_rebin < -3 * sd)
        x[:, bad_bins] = 0
    if return_badbins:
        return x, bad_bins
    return x


def quick_resample(counts, rebin):
    """dedispersion.py:38-57: sum ``rebin`` consecutive samples, truncate, float64."""
    counts = np.asarray(counts)
    nchan, nbin = counts.shape
    n = nbin // rebin
    r = counts[:, :n * rebin].reshape(nchan, n, rebin)
    out = np.zeros((nchan, n))
    for i in range(rebin):
        out += r[:, :, i]
    return out


def quick_chan_rebin(counts, rebin):
    """dedispersion.py:15-35: sum groups of ``rebin`` channels (input dtype rules)."""
    counts = np.asarray(counts)
    n = counts.shape[0] // rebin
    return counts[:n * rebin].reshape(n, rebin, counts.shape[1]).sum(axis=1)


def apply_dm_shifts(data, shifts):
    """dedispersion.py:254-258: roll channel i by -rint(shift_i)."""
    data = np.asarray(data)
    out = np.empty_like(data)
    for i in range(data.shape[0]):
        out[i] = np.roll(data[i], -int(np.rint(shifts[i])))
    return out


def uniform_filter1d_running(lc, size=16):
    """scipy.ndimage.uniform_filter1d(lc, size) (mode 'reflect', origin 0) restated as
    scipy's running sum (ni_filters.c NI_UniformFilter1D): the first window summed from
    0.0 and divided by size, then tmp += (x[i + size - 1 - size//2] - x[i - 1 - size//2])
    / size over the reflected line.  The order csrc/clean.hip outlier_exact_kernel
    follows."""
    lc = np.asarray(lc, dtype=np.float64)
    n = lc.size
    s1 = size // 2

    def ext(k):
        i = k - s1
        if i < 0:
            i = -i - 1
        if i >= n:
            i = 2 * n - 1 - i
        return lc[i]

    out = np.empty(n)
    tmp = 0.0
    for j in range(size):
        tmp += ext(j)
    tmp /= size
    out[0] = tmp
    for i in range(1, n):
        tmp += (ext(i + size - 1) - ext(i - 1)) / size
        out[i] = tmp
    return out


def std_numpy_order(v):
    """np.std(v) restated: numpy add.reduce order (oracle/numpy_order.py) for the mean
    and for the squared deviations, true divides, sqrt."""
    from .numpy_order import reduce_sum
    v = np.ascontiguousarray(v, dtype=np.float64)
    m = v.size
    mean = reduce_sum(v) / m
    d = v - mean
    return np.sqrt(reduce_sum(d * d) / m)
