"""Drop-in ``pulsarutils.clean`` (reference: pulsarutils/clean.py) - the RFI-cleaning pass.

The 2-D passes (per-channel means / standard deviations, the zero-DM light curve,
the renormalisation and its column means) run in HIP kernels that reproduce numpy's
exact reduction order, so the channel masks, the time-bin mask and the renormalised
data are bit-identical to the reference (tests/test_gpu_clean.py).  The 1-D steps on
nchan- or N-length vectors (medfilt, MAD, median, uniform_filter1d, quartiles) are
host logic on the exact vectors the kernels return.

``*_device`` variants take and return device tensors (no PCIe round trip of the
2-D data) and are what the multi-GPU pipeline and the benchmark use.
"""
from dataclasses import dataclass

import numpy as np
from scipy.ndimage import uniform_filter1d
from scipy.signal import medfilt

from . import _hip
from .dedispersion import (dedispersion_plan, dedispersion_shifts,  # noqa: F401
                           apply_dm_shifts_to_data, quick_resample, quick_chan_rebin)
from .dedispersion import dedispersion_search as fast_dedispersion_search  # noqa: F401
from .stats import MAD_C, mad, ref_mad
from .table import make_table


@dataclass
class PulseInfo():
    """clean.py:27-55 container (no annotations: plain class attributes, as in the reference)."""
    nbin = 0
    nchan = 0
    ph0 = None
    amp = None
    width = None
    noise_level = None
    dm = None
    pulse_freq = None
    start_freq = None
    bandwidth = None
    dedisp_profile = None
    allprofs = None
    disp_profile = None

    disp_z2 = None
    disp_z6 = None
    disp_z12 = None
    disp_z20 = None
    disp_H = None
    disp_M = None

    dedisp_z2 = None
    dedisp_z6 = None
    dedisp_z12 = None
    dedisp_z20 = None
    dedisp_H = None
    dedisp_M = None


# ---------------------------------------------------------------- device reductions

def _row_sums(x, mode, center=None, scale=None, divisor=0.0):
    t = _hip.torch()
    code = _hip.dtype_code(x.dtype)
    acc_f32 = code == _hip.PU_F32 and mode in (0, 1)
    nrows, n = x.shape
    out = t.empty(nrows, dtype=t.float32 if acc_f32 else t.float64, device=x.device)
    ws = _workspace(x.device, _hip.lib().pu_row_sums_workspace_bytes(nrows, n))
    _hip.check(_hip.lib().pu_row_sums(_hip.ptr(x), code, nrows, n, x.stride(0), mode, _hip.ptr(center),
                                      _hip.ptr(scale), float(divisor), _hip.ptr(out), _hip.ptr(ws), ws.numel(),
                                      _hip.stream_ptr()), "pu_row_sums")
    return out


_MEANS = [None]  # (weakref to the tensor, its version counter, the means, the shifted moments)
_VAR = [None]    # (weakref to the tensor, its version counter, the bad mask, the variability mask)


_WS = {}  # device -> scratch of pu_row_moments (stream-ordered: one stream per device here)


def _workspace(dev, nbytes):
    """A scratch buffer of at least ``nbytes`` on ``dev``, kept between calls: its users are
    queued on torch's current stream, which orders every reuse after the previous one."""
    t = _hip.torch()
    key = (str(dev), _hip.stream_ptr().value)
    buf = _WS.get(key)
    if buf is None or buf.numel() < nbytes:
        buf = t.empty(max(nbytes, 16), dtype=t.uint8, device=dev)
        _WS[key] = buf
    return buf


def _row_moments(x):
    """pu_row_moments: numpy's x.mean(1) (f32 for f32 input, else f64) and, from the same
    read pass, per row (c, sum(x - c), sum((x - c)^2)) in float64 with c = x[r, 0]."""
    t = _hip.torch()
    nrows, n = x.shape
    acc_f32 = _hip.dtype_code(x.dtype) == _hip.PU_F32
    means = t.empty(nrows, dtype=t.float32 if acc_f32 else t.float64, device=x.device)
    mom = t.empty((nrows, 3), dtype=t.float64, device=x.device)
    ws = _workspace(x.device, _hip.lib().pu_row_moments_workspace_bytes(nrows, n))
    _hip.check(_hip.lib().pu_row_moments(_hip.ptr(x), _hip.dtype_code(x.dtype), nrows, n, x.stride(0),
                                         _hip.ptr(means), _hip.ptr(mom), _hip.ptr(ws), ws.numel(),
                                         _hip.stream_ptr()), "pu_row_moments")
    return means, mom


def _cached_stats(x):
    """(means, moments) of ``x`` from the cache, or one pu_row_moments pass (cached)."""
    import weakref
    c = _MEANS[0]
    if not (c is not None and c[0]() is x and c[1] == (x._version, x.data_ptr())):
        m, mom = _row_moments(x)
        c = (weakref.ref(x), (x._version, x.data_ptr()), m, mom)
        _MEANS[0] = c
    return c[2], c[3]


def _variability_args(means, n):
    """pu_variability_cert's error factors (as _certified_variability)."""
    u = 2.0 ** -24 if means.dtype == _hip.torch().float32 else 2.0 ** -53
    return moment_error_factor(n), (35 + -(-int(n) // 8192) + 4) * u, u


def _launch_variability(x, bad_dev, out_mask, out_flag):
    """Queue the device variability decision of ``x`` with the uint8 device mask ``bad_dev``."""
    means, mom = _cached_stats(x)
    nrows, n = x.shape
    mef, gam, u = _variability_args(means, n)
    _hip.check(_hip.lib().pu_variability_cert(_hip.ptr(means), _hip.dtype_code(means.dtype), _hip.ptr(mom), nrows, n,
                                              mef, gam, u, _hip.ptr(bad_dev), out_mask, out_flag,
                                              _hip.stream_ptr()), "pu_variability_cert")


def channel_means_device(x):
    """``x.mean(1)`` with numpy's dtype and summation order (float32 stays float32).

    The pass that computes them also sums each row's shifted moments (pu_row_moments),
    from which measure_channel_variability certifies its std decisions without a
    second pass.  The last result is kept for the same tensor object while it is
    unmodified (its version counter and storage pointer unchanged): get_noisier_channels
    and measure_channel_variability both start from the statistics of one block, and the
    second call then skips the pass.  A weak reference, so the cache never keeps a
    block alive; callers get a copy, so changing a result never changes the cache.
    Writes that bypass torch's version counter (raw-pointer kernels, DLPack aliases)
    are not seen: call :func:`invalidate_channel_means` after such a write (numpy inputs
    are copied to a fresh tensor per call and never hit the cache)."""
    return _cached_stats(x)[0].clone()


def invalidate_channel_means():
    """Forget the cached channel means (see :func:`channel_means_device`)."""
    _MEANS[0] = None
    _VAR[0] = None


def channel_variances_device(x, means=None):
    """``np.var(x, axis=1)`` (ddof 0) in numpy's order; ``np.std`` = host ``np.sqrt`` of it."""
    if means is None:
        means = channel_means_device(x)
    return _row_sums(x, 1, center=means, divisor=x.shape[1])


def median_device(x):
    """``np.median`` of a 1-D float64 device tensor, as a 1-element device tensor
    (radix select on the GPU; no host round trip)."""
    t = _hip.torch()
    lib = _hip.lib()
    out = t.empty(1, dtype=t.float64, device=x.device)
    ws = t.empty(lib.pu_median_workspace_bytes(), dtype=t.uint8, device=x.device)
    _hip.check(lib.pu_median(_hip.ptr(x), x.numel(), _hip.ptr(out), _hip.ptr(ws), ws.numel(), _hip.stream_ptr()),
               "pu_median")
    return out


def _host(t):
    return t.detach().cpu().numpy()


_NOISY_MAX = 4096  # pu_noisy_channels: one workgroup
_MASKS_MAX = 1024  # pu_channel_masks: one thread per channel


def get_noisier_channels(array):
    """clean.py:58-67: channels whose mean exceeds medfilt(spec, 7) + 5 ref_mad.

    The decision runs on the device (pu_noisy_channels: medfilt, ref_mad and the
    comparison in numpy's dtypes and order) and only the mask comes back; a spec with
    NaN / inf, or more than 4096 channels, is decided on the host by numpy / scipy.
    In the same read-back: measure_channel_variability's decision for this mask
    (pu_variability_cert, queued behind it; up to 1024 channels both decisions are one
    launch, pu_channel_masks), kept for the same unmodified tensor - the
    usual next call, measure_channel_variability(x, badchans_mask=<this mask>), then
    needs no GPU work and no synchronisation of its own."""
    import weakref
    x = _hip.to_device(array)
    spec_d = _cached_stats(x)[0]  # (read only here: no defensive copy)
    n = spec_d.numel()
    if 2 <= n <= _NOISY_MAX:
        t = _hip.torch()
        off = (n + 3) & ~3
        # [noisy mask | its flag | variability mask | its flag]
        res = t.empty(2 * (off + 4), dtype=t.uint8, device=spec_d.device)
        base = res.data_ptr()
        if n <= _MASKS_MAX and hasattr(_hip.lib(), "pu_channel_masks"):  # (absent: an older A/B build)
            # both decisions in one launch (pu_channel_masks)
            means, mom = _cached_stats(x)
            mef, gam, u = _variability_args(means, x.shape[1])
            _hip.check(_hip.lib().pu_channel_masks(_hip.ptr(means), _hip.dtype_code(means.dtype), _hip.ptr(mom), n,
                                                   x.shape[1], float(MAD_C), mef, gam, u, base, base + off,
                                                   base + off + 4, base + 2 * off + 4, _hip.stream_ptr()),
                       "pu_channel_masks")
        else:
            _hip.check(_hip.lib().pu_noisy_channels(_hip.ptr(spec_d), _hip.dtype_code(spec_d.dtype), n,
                                                    float(MAD_C), base, base + off, _hip.stream_ptr()),
                       "pu_noisy_channels")
            # (when the noisy flag is set the mask is unwritten: the variability result is
            # then discarded)
            _launch_variability(x, res[:n], base + off + 4, base + 2 * off + 4)
        h = _host(res)
        if not h[off:off + 4].view(np.int32)[0]:
            mask = h[:n].astype(bool)
            if not h[2 * off + 4:2 * off + 8].view(np.int32)[0]:
                _VAR[0] = (weakref.ref(x), (x._version, x.data_ptr()), mask.copy(),
                           h[off + 4:off + 4 + n].astype(bool))
            return mask
    spec = _host(spec_d)
    smooth_spec = medfilt(spec, 7)
    return spec > smooth_spec + 5 * ref_mad(spec)


def moment_error_factor(n):
    """Relative error bound of pu_row_moments' float64 sums of d and d^2 over a row of n.

    The device sums each 8192-element block in a tree (depth <= 14 + 6), the trailing
    partial block (up to 8191 elements) serially in rowsum_tail_kernel, and the block
    sums one after another in moments_combine: a summation depth of at most
    min(n, 8191) + ceil(n / 8192) + the block tree, plus the final combination
    (V = s2 - 2 (m - c) s1 + n (m - c)^2, a few roundings).  A depth-h sum of
    non-negative terms errs by <= h u of their total; the factor keeps 2^-40 as a floor
    (the round-4 constant, exact-enough for n <= 8192)."""
    depth = min(int(n), 8191) + -(-int(n) // 8192) + 64
    return max(2.0 ** -40, depth * 2.0 ** -53)


def _certified_variability(means, moments, n, acc_f32, badchans_mask):
    """measure_channel_variability's mask from one read pass, or None.

    ``moments`` rows are (c, sum(x - c), sum((x - c)^2)) in float64 (pu_row_moments), so
    V = s2 - 2 (m - c) s1 + n (m - c)^2 is the real sum of squared deviations from numpy's
    mean m up to float64 rounding.  numpy's own std (clean.py:119, np.std in the input's
    float type: squared deviations rounded, add.reduce of depth <= 35 + nblocks, the
    divide and the sqrt) lies in [s_lo, s_hi] around sqrt(V / n); the quartiles of the
    good channels (order statistics: monotone in every argument) lie in the intervals of
    the k-th smallest bounds, and the limits 2 q1 - q2 / 2 q3 - q2 (with their three
    roundings) in intervals built from those.  When every unmasked channel is clear of
    both limit intervals the decisions are the reference's; otherwise (or for non-finite
    input, or too few good channels for the reference's quartile indices) None, and the
    caller runs the exact second pass."""
    m = np.asarray(means, dtype=np.float64)
    mom = np.asarray(moments, dtype=np.float64)
    bad = np.asarray(badchans_mask, dtype=bool)
    nchan = m.size
    good = ~bad
    if not (np.isfinite(m).all() and np.isfinite(mom).all()) or nchan // 4 * 3 >= int(good.sum()):
        return None
    c, s1, s2 = mom[:, 0], mom[:, 1], mom[:, 2]
    dm = m - c
    V = s2 - 2.0 * dm * s1 + n * dm * dm
    eV = (s2 + 2.0 * np.abs(dm) * np.sqrt(n * s2) + n * dm * dm) * moment_error_factor(n) + 1e-300
    u = 2.0 ** -24 if acc_f32 else 2.0 ** -53
    gam = (35 + -(-n // 8192) + 4) * u
    s_lo = np.sqrt(np.maximum(V - eV, 0.0) * (1.0 - gam) / n * (1.0 - u)) * (1.0 - u)
    s_hi = np.sqrt((V + eV) * (1.0 + gam) / n * (1.0 + u)) * (1.0 + u)
    lo_sorted, hi_sorted = np.sort(s_lo[good]), np.sort(s_hi[good])
    a1, b1 = lo_sorted[nchan // 4], hi_sorted[nchan // 4]
    a2, b2 = lo_sorted[nchan // 2], hi_sorted[nchan // 2]
    a3, b3 = lo_sorted[nchan // 4 * 3], hi_sorted[nchan // 4 * 3]
    r = 4.0 * u * (b2 + 2.0 * (b3 - a1)) + 1e-300  # the limits' roundings (magnitudes >= 0)
    low_lo, low_hi = 2.0 * a1 - b2 - r, 2.0 * b1 - a2 + r
    hi_lo, hi_hi = 2.0 * a3 - b2 - r, 2.0 * b3 - a2 + r
    below = s_hi < low_lo
    above = s_lo > hi_hi
    sure = (below | (s_lo >= low_hi)) & (above | (s_hi <= hi_lo))
    if not sure[good].all():
        return None
    return below | above | bad


def _check_mask(badchans_mask, nrows):
    """The channel mask as a boolean vector of ``nrows``; any other shape raises numpy's own
    IndexError, as the reference's ``array[~badchans_mask]`` does (clean.py:77, :120) - the
    kernels read exactly ``nrows`` mask bytes, so a short mask must never reach them."""
    m = np.asarray(badchans_mask, dtype=bool)
    if m.shape != (nrows,):
        raise IndexError("boolean index did not match indexed array along axis 0; size of axis is %d but "
                         "size of corresponding boolean axis is %s" % (nrows, m.shape[0] if m.ndim else m.shape))
    return m


def measure_channel_variability(array, badchans_mask=None):
    """clean.py:114-133: per-channel std outside [q2 - 2(q2-q1), q2 + 2(q3-q2)].

    Quartile positions use the full channel count, as in the reference (an
    IndexError when too many channels are masked is the reference behaviour).
    The decisions are certified from the shifted moments of the means pass on the
    device (pu_variability_cert; computed ahead by get_noisier_channels for its own
    mask), no second read pass; only when one is within its rounding bound is numpy's
    std computed exactly (a second pass).  More than 4096 channels: the same
    certification on the host (_certified_variability).
    """
    if badchans_mask is None:
        badchans_mask = np.zeros(array.shape[0], dtype=bool)
    badchans_mask = _check_mask(badchans_mask, array.shape[0])
    x = _hip.to_device(array)
    t = _hip.torch()
    nrows = x.shape[0]
    v = _VAR[0]
    if (v is not None and v[0]() is x and v[1] == (x._version, x.data_ptr())
            and np.array_equal(v[2], badchans_mask)):
        return v[3].copy()
    means, mom = _cached_stats(x)
    if nrows <= _NOISY_MAX:
        off = (nrows + 3) & ~3
        bad_np = np.ascontiguousarray(badchans_mask).astype(np.uint8)
        bad = t.from_numpy(bad_np).pin_memory().to(x.device, non_blocking=True)
        res = t.empty(off + 4, dtype=t.uint8, device=x.device)
        _launch_variability(x, bad, res.data_ptr(), res.data_ptr() + off)
        h = _host(res)
        if not h[off:off + 4].view(np.int32)[0]:
            return h[:nrows].astype(bool)
    else:
        mask = _certified_variability(_host(means).astype(np.float64), _host(mom), x.shape[1],
                                      means.dtype == t.float32, badchans_mask)
        if mask is not None:
            return mask
    spec = np.sqrt(_host(channel_variances_device(x, means)))
    ordered = np.sort(spec[~badchans_mask])
    q1 = ordered[spec.size // 4]
    q2 = ordered[spec.size // 2]
    q3 = ordered[spec.size // 4 * 3]
    lowlim = q2 - 2 * (q2 - q1)
    hilim = q2 + 2 * (q3 - q2)
    return (spec < lowlim) | (spec > hilim) | badchans_mask


def _gaussian_weights(sigma):
    from scipy.ndimage._filters import _gaussian_kernel1d
    radius = int(4.0 * float(sigma) + 0.5)
    return np.ascontiguousarray(_gaussian_kernel1d(sigma, 0, radius)[::-1]), radius


_WEIGHTS = {}


def _gaussian_weights_device(sigma, dev):
    """scipy's gaussian_filter weights for ``sigma`` on ``dev``, uploaded once (cached)."""
    key = (float(sigma), str(dev))
    if key not in _WEIGHTS:
        w, radius = _gaussian_weights(sigma)
        _WEIGHTS[key] = (_hip.torch().from_numpy(w).to(dev), radius)
    return _WEIGHTS[key]


def light_curve_factor(lc, weights, radius, median_out=None):
    """clean.py:79-80 on a device light curve: factor = np.median(lc_smooth) / lc_smooth with
    lc_smooth = gaussian_filter(lc) (``weights``/``radius`` from _gaussian_weights_device),
    bit for bit as pu_gaussian_filter1d + pu_median + pu_ratio_dev (pu_lc_factor: those
    three on the current stream).  ``median_out``: optional float64 device tensor [1]."""
    t = _hip.torch()
    lib = _hip.lib()
    n = lc.numel()
    nbytes = lib.pu_lc_factor_workspace_bytes(n)
    # the caching allocator's blocks are stream-ordered and 512-byte aligned
    buf = t.empty(nbytes, dtype=t.uint8, device=lc.device)
    assert buf.data_ptr() % 256 == 0
    factor = t.empty(n, dtype=t.float64, device=lc.device)
    _hip.check(lib.pu_lc_factor(_hip.ptr(lc), n, _hip.ptr(weights), int(radius), _hip.ptr(factor),
                                _hip.ptr(median_out) if median_out is not None else None, buf.data_ptr(),
                                nbytes, _hip.stream_ptr()), "pu_lc_factor")
    return factor


_MASK = {}  # (device, stream) -> (mask bytes, the device copy): the last uploaded channel mask


def _device_mask(bad_np, dev):
    """The uint8 channel mask ``bad_np`` on ``dev``: the previous call's copy when the bytes
    are the same (read-only in the kernels; a new tensor otherwise, so a copy still in use
    by queued work is never overwritten; per stream, so the copy is ordered before every
    reader).  The upload goes through pinned memory
    asynchronously: a pageable copy would block the host until the stream drained (the
    previous call's kernels), so the next call's launches could not queue behind them."""
    key = bad_np.tobytes()
    slot = (str(dev), _hip.stream_ptr().value)
    c = _MASK.get(slot)
    if c is not None and c[0] == key:
        return c[1]
    t = _hip.torch()
    bad = t.from_numpy(bad_np).pin_memory().to(dev, non_blocking=True)
    _MASK[slot] = (key, bad)
    return bad


def renormalize_device(x, badchans_mask=None, baseline_window=101, cut_outliers=False, out=None,
                       zero_dm=False):
    """renormalize_data on a device tensor; returns (float64 device tensor, bad_bins or None),
    bad_bins a boolean device tensor (the cut_outliers time-bin mask; not copied to the
    host: renormalize_data discards it, as the reference does).

    Passes (clean.py:73-105): zero-DM light curve over good channels (column means,
    rows in order) -> gaussian_filter (scipy's order) + median (radix select) + factor in
    pu_lc_factor
    -> per-channel mean of x*factor (numpy pairwise order) -> (x*f - mu)/mu with bad
    channels zeroed [+ its column mean] -> uniform_filter1d(16) thresholds on the
    device (certified; scipy's own running sum on the device when a decision is
    ambiguous) -> zero the bad time bins.  No host synchronisation for n >= 64.

    ``zero_dm=True`` (opt-in; the reference has no counterpart, see renormalize_data)
    also subtracts, per time bin, the mean of the normalised good channels, fused into
    the apply pass (pu_renorm_apply_zero_dm).
    """
    t = _hip.torch()
    nchan, n = x.shape
    dev = x.device
    code = _hip.dtype_code(x.dtype)
    lib = _hip.lib()
    s = _hip.stream_ptr()
    if badchans_mask is None:
        badchans_mask = np.zeros(nchan, dtype=bool)
    bad_np = np.ascontiguousarray(_check_mask(badchans_mask, nchan)).astype(np.uint8)
    bad = _device_mask(bad_np, dev)
    sigma = min(baseline_window, n // 100 * 2 + 1)
    dw, radius = _gaussian_weights_device(sigma, dev)
    lc = t.empty(n, dtype=t.float64, device=dev)
    _hip.check(lib.pu_col_means(_hip.ptr(x), code, nchan, n, x.stride(0), _hip.ptr(bad), _hip.ptr(lc), s),
               "pu_col_means")
    # gaussian_filter + np.median + the factor (pu_lc_factor)
    factor = light_curve_factor(lc, dw, radius)
    spec = _row_sums(x, 2, scale=factor, divisor=n)
    if out is None:
        out = t.empty((nchan, n), dtype=t.float64, device=dev)
    col = t.empty(n, dtype=t.float64, device=dev) if cut_outliers else None
    if zero_dm:
        ngood = int(nchan - np.count_nonzero(bad_np))
        _hip.check(lib.pu_renorm_apply_zero_dm(_hip.ptr(x), code, nchan, n, x.stride(0), _hip.ptr(factor),
                                               _hip.ptr(spec), _hip.ptr(bad), ngood, _hip.ptr(out), out.stride(0),
                                               _hip.ptr(col), s), "pu_renorm_apply_zero_dm")
    else:
        _hip.check(lib.pu_renorm_apply(_hip.ptr(x), code, nchan, n, x.stride(0), _hip.ptr(factor), _hip.ptr(spec),
                                       _hip.ptr(bad), _hip.ptr(out), out.stride(0), _hip.ptr(col), s),
                   "pu_renorm_apply")
    bad_bins = None
    if cut_outliers and n >= 64:
        # device path (pu_cut_outliers): certified decisions, and the reference's own
        # arithmetic on the device for the rare ambiguous / NaN case - no host round trip
        ws = t.empty(lib.pu_cut_outliers_workspace_bytes(n), dtype=t.uint8, device=dev)
        mask = t.empty(n, dtype=t.uint8, device=dev)
        _hip.check(lib.pu_cut_outliers(_hip.ptr(col), n, _hip.ptr(out), nchan, out.stride(0), _hip.ptr(mask),
                                       _hip.ptr(ws), ws.numel(), s), "pu_cut_outliers")
        return out, mask.view(t.bool)
    if cut_outliers:
        # n < 64: scipy on the host, as the reference does
        lc2 = _host(col)
        window = 16  # only the last window of the reference loop (range(0, 5)) survives
        lc_rebin = uniform_filter1d(lc2, window)
        thresh_up = 5 * np.std(lc_rebin[::window])
        thresh_down = -3 * np.std(lc_rebin[::window])
        bad_bins = (lc_rebin > + thresh_up) | (lc_rebin < thresh_down)
        cols = np.nonzero(bad_bins)[0].astype(np.int64)
        if cols.size:
            dcols = t.from_numpy(cols).to(dev)
            _hip.check(lib.pu_zero_columns(_hip.ptr(out), nchan, out.stride(0), _hip.ptr(dcols), cols.size, s),
                       "pu_zero_columns")
        bad_bins = t.from_numpy(bad_bins).to(dev)
    return out, bad_bins


def renormalize_data(array, diagnostic_figure=None, badchans_mask=None, baseline_window=101,
                     cut_outliers=False, zero_dm=False):
    """clean.py:70-111: zero-DM normalisation + per-channel (x - mu)/mu, float64 out.

    ``zero_dm`` (default False, so the drop-in is the reference bit for bit): also
    subtract the zero-DM series - per time bin, the mean over good channels of the
    normalised data - from every good channel.  The reference only divides by the
    smoothed zero-DM series (clean.py:77-82); this opt-in subtraction is the
    north-star cleaning step and has no reference counterpart (parity unpinned; tested
    against a numpy restatement).  ``cut_outliers`` then uses the column mean of the
    data before the subtraction.
    """
    x = _hip.to_device(array)
    out, _ = renormalize_device(x, badchans_mask=badchans_mask, baseline_window=baseline_window,
                                cut_outliers=cut_outliers, zero_dm=zero_dm)
    return _host(out)


def dedispersion_search(info, dmmin, dmmax):
    """clean.py:136-180: plane search of a PulseInfo -> (plane, Table).

    sample_time = 1 / pulse_freq / nbin.  The plane is float64 (ndm, N) in memory
    (the reference writes it to ``dummy.npy`` in the CWD; not reproduced).  The
    rebin column is int64 as in the reference.
    """
    from .dedispersion import dedispersion_search as dsearch
    data = info.allprofs
    sample_time = 1 / info.pulse_freq / info.nbin
    table, plane = dsearch(data, dmmin, dmmax, info.start_freq, info.bandwidth, sample_time, show=True)
    return plane, table


def digitize(data):
    """clean.py:183-189 (diagnostics): MAD-scaled, clipped, rounded integers."""
    if isinstance(data, (int, np.integer)):
        return data
    std = mad(data)
    data = (data - np.median(data)) / std * 3
    data[data < 0] = 0
    return np.rint(data).astype(int)


def dm_broadening(dm, freq, df):
    """clean.py:272-273: intra-channel DM smearing (s)."""
    return 8300 * dm * df / freq**3


def search_by_chunks(fname, chunk_length=None, new_sample_time=None, tmin=0, dmmin=200, dmmax=800, surelybad=[],
                     save_candidates=True, snr_threshold=6, acc=None, search_dtype="f64", profile=None,
                     zero_dm=False):
    """clean.py:276-351: stream a SIGPROC file through clean + DM search, chunk by chunk.

    Same chunking as the reference: ``step = max(int(chunk_length / tsamp) * 2, 128)``
    samples (``chunk_length`` defaults to the whole-band delay at ``dmmax``), hop
    ``step // 2`` (50 % overlap), chunks shorter than ``step // 2`` and chunks before
    ``tmin`` skipped; channel mask from ``get_bad_chans`` (+ ``surelybad``);
    ``renormalize_data``; band flipped when ``foff < 0``; resampled by
    ``N = rint(new_sample_time / tsamp)`` when >= 2; ``dedispersion_search``.  All array
    work stays in HBM (read_block_device -> renormalize_device -> HIP rebin -> search).

    ``search_dtype``: the renormalised chunk is float64 (clean.py:73); ``"f64"``
    (default, the reference's behaviour, clean.py:346) searches it with float64
    accumulation in channel order (bit-exact series; certified statistics), ``"f32"``
    casts it to float32 on the device and searches with the float32 subband kernel (the
    north star's float32 summation-order tolerance; ~3x faster per chunk, but the file
    pipeline is bound by the host read + PCIe copy either way).  ``zero_dm`` is renormalize_data's opt-in subtraction.
    ``profile``: a list that receives one dict of synchronised per-step timings (ms:
    h2d, transpose, clean, cast, rebin, search) per chunk.

    Returns the list of candidate chunks (max S/N > ``snr_threshold``): dicts with
    istart, iend, t0, best DM, S/N, rebin and the full table.  With ``save_candidates``
    each candidate's PulseInfo is pickled to ``{root}_{istart}-{iend}.pkl`` like the
    reference; the diagnostic plots (``plot_diagnostics``, matplotlib + hendrics H-test)
    are out of scope and not drawn.
    """
    import os
    import pickle
    import time
    from .dedispersion import _rebin_time_device, delta_delay, search_device
    from .sigproc import FilReader, transpose_device
    from .stats import get_bad_chans
    if search_dtype not in ("f32", "f64"):
        raise ValueError(f"search_dtype must be 'f32' or 'f64', got {search_dtype!r}")
    t = _hip.require_gpu()
    fname_root = os.path.basename(fname).split('.')[0]
    mask = get_bad_chans(fname)
    for bad_chan in surelybad:
        mask[bad_chan] = True
    fil = FilReader(fname)
    header = fil.header
    nsamples = header['nsamples']
    sample_time = header['tsamp']
    start_freq = header['fbottom']
    stop_freq = header['ftop']
    bandwidth = header['bandwidth']
    nchan = header['nchans']
    foff = header['foff']
    date = header.get('tstart')
    delta = delta_delay(dmmax, start_freq, stop_freq)
    if chunk_length is None:
        chunk_length = delta
    step = max(int(chunk_length / sample_time) * 2, 128)
    dm_dt = dm_broadening(dmmin, start_freq, np.abs(foff))
    if new_sample_time is None:
        new_sample_time = max(dm_dt / 10, sample_time)
    sampl_ratio = new_sample_time / sample_time
    N = 1
    if sampl_ratio >= 2:
        N = int(np.rint(sampl_ratio))
        new_sample_time = N * sample_time
    trial_DMs = None
    plan = None
    candidates = []
    chunks = []
    for istart in range(0, nsamples, step // 2):
        chunk_size = min(step, nsamples - istart)
        if istart * sample_time < tmin or chunk_size < step // 2:
            continue
        chunks.append((istart, chunk_size))
    dev = t.device("cuda", t.cuda.current_device())
    # Chunk k+1 is copied from the memory-mapped file to the device by a loader thread
    # (a pageable H2D on a copy stream: the runtime's own staging, no extra host copy)
    # while chunk k is cleaned and searched on the current stream.  With ``profile``
    # every step is synchronised instead.
    overlap = profile is None and len(chunks) > 1
    copy_stream = t.cuda.Stream(device=dev) if overlap else None

    def load(k):
        istart, size = chunks[k]
        tc = np.ascontiguousarray(fil._block_tc(istart, size))
        with t.cuda.device(dev), t.cuda.stream(copy_stream):
            dst = t.from_numpy(tc).to(dev)
            ev = t.cuda.Event()
            ev.record(copy_stream)
        return dst, ev

    pool = None
    if overlap:
        from concurrent.futures import ThreadPoolExecutor
        pool = ThreadPoolExecutor(max_workers=1)
        pending = pool.submit(load, 0)
    for k, (istart, chunk_size) in enumerate(chunks):
        t0 = istart * sample_time
        iend = istart + chunk_size
        marks = []

        def mark(name):
            if profile is not None:
                t.cuda.synchronize()
                marks.append((name, time.perf_counter()))

        mark("start")
        if overlap:
            src, ev = pending.result()
            if k + 1 < len(chunks):
                pending = pool.submit(load, k + 1)
            t.cuda.current_stream(dev).wait_event(ev)
            src.record_stream(t.cuda.current_stream(dev))
        else:
            tc = np.ascontiguousarray(fil._block_tc(istart, chunk_size))
            src = t.from_numpy(tc).to(dev)
        mark("h2d")
        block = transpose_device(src)
        del src
        mark("transpose")
        if _hip.dtype_code(block.dtype) is None:
            block = block.to(t.float64)
        array, _ = renormalize_device(block, badchans_mask=mask, zero_dm=zero_dm)
        del block
        if foff < 0:
            array = t.flip(array, dims=(0,)).contiguous()
        mark("clean")
        if N > 1:
            array = _rebin_time_device(array, N)  # quick_resample of the float64 plane (clean.py:335-336)
        mark("rebin")
        array64 = array  # the candidate pickles hold the float64 plane, as in the reference
        if search_dtype == "f32":
            array = array.to(t.float32)
        mark("cast")
        nbin = array.shape[1]
        if trial_DMs is None or plan is None or plan.nsamples != nbin:
            trial_DMs = dedispersion_plan(nchan, dmmin, dmmax, start_freq, bandwidth, new_sample_time)
            plan = None
        (mx, sd, snr, win), plan = search_device(array, trial_DMs, nchan, start_freq, bandwidth, new_sample_time,
                                                 acc=acc, plan=plan)
        mark("search")
        if profile is not None:
            rec = {"istart": istart, "nsamples": chunk_size, "ndm": int(trial_DMs.size)}
            rec.update({name: (tt - marks[i][1]) * 1e3 for i, (name, tt) in enumerate(marks[1:])})
            profile.append(rec)
        snr = _host(snr)
        table = make_table({'DM': trial_DMs, 'max': _host(mx), 'std': _host(sd), 'snr': snr, 'rebin': _host(win)})
        if np.any(snr > snr_threshold):
            best = int(np.argmax(snr))
            cand = {'istart': istart, 'iend': iend, 't0': t0, 'dm': float(trial_DMs[best]),
                    'snr': float(snr[best]), 'rebin': int(table['rebin'][best]), 'table': table}
            candidates.append(cand)
            if save_candidates:
                info = PulseInfo()
                info.allprofs = _host(array64)
                info.start_freq = start_freq
                info.bandwidth = bandwidth
                info.nbin = nbin
                info.nchan = array.shape[0]
                info.date = date
                info.pulse_freq = 1 / (info.nbin * new_sample_time)
                with open(f'{fname_root}_{istart}-{iend}.pkl', 'wb') as fh:
                    pickle.dump(info, fh)
        del array, array64
    if pool is not None:
        pool.shutdown(wait=True)
    return candidates


__all__ = ["search_by_chunks", "PulseInfo", "get_noisier_channels", "renormalize_data", "measure_channel_variability",
           "dedispersion_search", "digitize", "dm_broadening", "renormalize_device",
           "channel_means_device", "channel_variances_device", "make_table"]
