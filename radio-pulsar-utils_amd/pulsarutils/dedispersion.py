"""Drop-in ``pulsarutils.dedispersion`` (reference: pulsarutils/dedispersion.py).

Same names, arguments, defaults and return types as the reference; numpy in, numpy
out.  The float64 planner stays on the host (``_planner.py``); every array pass runs
in a hand-written HIP kernel through ``_hip`` (no CPU fallback).

Device-resident use (no PCIe copies): pass a CUDA ``torch.Tensor`` as ``data`` to
``_dedispersion_search`` / ``dedispersion_search`` / ``dedisperse``, or use
:func:`search_device` which returns device tensors.

Accumulation: ``acc='native'`` (default) sums uint8 exactly in
float32, float32 in float32 (stated tolerance) and float64 in float64 (bit-exact);
``acc='f64'`` sums everything in float64 in channel order, bit-identical to the
reference's dedispersed series.  Nothing here or in the library is configured by the
environment (:func:`planner_options` scopes explicit planner options).
"""
import collections
import contextlib
import hashlib
import os
import threading

import numpy as np

from . import _hip
from ._planner import (delta_delay, dedispersion_plan, dedispersion_shifts,  # noqa: F401
                       normalize_shifts)
from .table import make_table

_ACC = {"native": _hip.PU_ACC_NATIVE, "f32": _hip.PU_ACC_F32, "f64": _hip.PU_ACC_F64}


def _acc_code(acc):
    acc = acc or "native"
    try:
        return _ACC[acc]
    except KeyError:
        raise ValueError(f"acc must be one of {sorted(_ACC)}, got {acc!r}") from None


def _numpy_out(t):
    return t.detach().cpu().numpy()


def quick_chan_rebin(counts, current_rebin):
    """dedispersion.py:15-35: sum groups of ``current_rebin`` channels, channel order.

    Output dtype follows ``np.sum``: float32->float32, float64->float64,
    unsigned ints->uint64, signed ints/bool->int64 (integer sums are exact).
    """
    t = _hip.require_gpu()
    out_np_dtype = None
    if not isinstance(counts, t.Tensor):
        counts = np.asarray(counts)
        k = counts.dtype.kind
        if k in "iub":
            out_np_dtype = np.uint64 if k == "u" else np.int64
            if counts.dtype != np.uint8:
                counts = counts.astype(np.int64)
        elif counts.dtype not in (np.float32, np.float64):
            counts = counts.astype(np.float64)
    x = _hip.to_device(counts, allowed=(_hip.PU_U8, _hip.PU_F32, _hip.PU_F64, _hip.PU_I64))
    nchan, nbin = x.shape
    r = int(current_rebin)
    n = nchan // r
    code = _hip.dtype_code(x.dtype)
    # uint8 sums come back as uint64 bits: allocate int64 storage and view
    out_dt = {_hip.PU_U8: t.int64, _hip.PU_F32: t.float32, _hip.PU_F64: t.float64, _hip.PU_I64: t.int64}[code]
    out = t.empty((n, nbin), dtype=out_dt, device=x.device)
    if n:
        _hip.check(_hip.lib().pu_rebin_chan(_hip.ptr(x), code, nchan, nbin, x.stride(0), r, _hip.ptr(out),
                                            _hip.stream_ptr()), "quick_chan_rebin")
    res = _numpy_out(out)
    if out_np_dtype is not None:
        res = res.view(np.uint64) if code == _hip.PU_U8 else res.astype(out_np_dtype, copy=False)
    return res


def _rebin_time_device(x, w):
    t = _hip.torch()
    nchan, nbin = x.shape
    n = nbin // int(w)
    out = t.empty((nchan, n), dtype=t.float64, device=x.device)
    if n:
        _hip.check(_hip.lib().pu_rebin_time(_hip.ptr(x), _hip.dtype_code(x.dtype), nchan, nbin, x.stride(0), int(w),
                                            _hip.ptr(out), _hip.stream_ptr()), "quick_resample")
    return out


def quick_resample(counts, current_rebin):
    """dedispersion.py:38-57: sum ``current_rebin`` consecutive samples (float64 out)."""
    x = _hip.to_device(counts, allowed=(_hip.PU_U8, _hip.PU_F32, _hip.PU_F64, _hip.PU_I64))
    if x.dim() != 2:
        raise IndexError("quick_resample expects a 2-D (nchan, nbin) array")
    return _numpy_out(_rebin_time_device(x, current_rebin))


def roll_and_sum(array, sum_array, N):
    """dedispersion.py:60-83: ``sum_array += np.roll(array, N)`` in place; returns sum_array."""
    t = _hip.require_gpu()
    a = np.asarray(array) if not isinstance(array, t.Tensor) else array
    size = a.shape[-1]
    N = int(N)
    if a.ndim != 1 or len(sum_array) != size:
        raise ValueError("roll_and_sum expects 1-D arrays of equal length")
    if N < 0 or N > size:
        raise IndexError(f"roll amount {N} outside [0, {size}]")
    x = _hip.to_device(a, allowed=(_hip.PU_U8, _hip.PU_F32, _hip.PU_F64, _hip.PU_I64))
    acc = _hip.to_device(np.asarray(sum_array, dtype=np.float64), allowed=(_hip.PU_F64,))
    if size:
        _hip.check(_hip.lib().pu_roll_and_sum(_hip.ptr(x), _hip.dtype_code(x.dtype), size, N % size, _hip.ptr(acc),
                                              _hip.stream_ptr()), "roll_and_sum")
    sum_array[...] = _numpy_out(acc)
    return sum_array


def _prepare_data(data):
    x = _hip.to_device(data)
    if x.dim() != 2:
        raise ValueError("data must be a 2-D (nchan, nsamples) array")
    return x


# Plans (tiling + device metadata) of recent calls, so repeated numpy-API calls on the same
# shape and trial grid skip the host planner (~35 ms at C2).  Sharing one across threads
# is safe: workspace and outputs are per call, and the library holds a per-plan lock
# across each launch + finalize + certification (pu_plan's mutable state: timing events,
# the certification read-back).  The key holds the planner options in force
# (:func:`planner_options`).
_PLAN_CACHE = collections.OrderedDict()
_PLAN_CACHE_SIZE = 4
_PLAN_LOCK = threading.Lock()
_PLAN_OPTS = threading.local()


@contextlib.contextmanager
def planner_options(**opts):
    """Planner options for the plans the drop-in functions build in this thread (the
    keyword arguments of :class:`pulsarutils._hip.Plan`: ``group``, ``shape``,
    ``lds_budget_kb``, ``u8_dma``, ``dt_major``, ``slot16``).  The reference has no such knob; the
    defaults are the library's automatic choices.  Explicit and scoped: nothing is read
    from the environment."""
    old = getattr(_PLAN_OPTS, "opts", {})
    _PLAN_OPTS.opts = {**old, **opts}
    try:
        yield
    finally:
        _PLAN_OPTS.opts = old


def _plan_for(x, shifts, acc, ident=None):
    """Cached plan for ``x``'s shape/dtype.  ``shifts`` is the int64 shift table or a
    callable producing it; ``ident`` (hashable) names the table cheaply (the trial grid
    and band), so a cache hit never builds or hashes the table."""
    if ident is None:
        shifts = np.ascontiguousarray(shifts, dtype=np.int64)
        ident = (hashlib.sha1(shifts.tobytes()).hexdigest(), shifts.shape)
    opts = dict(getattr(_PLAN_OPTS, "opts", {}))
    key = (_hip.dtype_code(x.dtype), acc, x.shape[0], x.shape[1], x.device.index, ident,
           tuple(sorted(opts.items())))
    with _PLAN_LOCK:
        plan = _PLAN_CACHE.get(key)
        if plan is not None:
            _PLAN_CACHE.move_to_end(key)
            return plan
    sh = shifts() if callable(shifts) else shifts
    plan = _hip.Plan(key[0], acc, x.shape[0], x.shape[1], sh, **opts)
    with _PLAN_LOCK:
        _PLAN_CACHE[key] = plan
        while len(_PLAN_CACHE) > _PLAN_CACHE_SIZE:
            _PLAN_CACHE.popitem(last=False)
    return plan


def dedisperse(data, shifts, acc="f64"):
    """dedispersion.py:93-98: circular shift-and-sum over channels, float64[N].

    ``out[t] = sum_c data[c, (t + rint(shifts[c])) mod N]``, summed in channel order
    in float64 by default (bit-identical to the reference).
    """
    x = _prepare_data(data)
    sh = np.rint(np.asarray(shifts, dtype=np.float64).reshape(1, -1)).astype(np.int64)
    if sh.shape[1] != x.shape[0]:
        raise ValueError("one shift per channel required")
    plan = _plan_for(x, sh, _acc_code(acc))
    plane = plan.dedisperse(x)
    return _numpy_out(plane[0]).astype(np.float64, copy=False)


def search_device(data, trial_DMs, nchan, start_freq, bandwidth, sample_time, acc=None, plan=None):
    """Device-resident ``_dedispersion_search``: returns (max, std, snr, rebin) tensors + plan."""
    x = _prepare_data(data)
    if int(nchan) != x.shape[0]:
        raise ValueError("nchan does not match data.shape[0]")
    if x.shape[1] < 8:
        # the reference's 8-sample quick_resample is empty and np.max of it raises
        # (dedispersion.py:192-193)
        raise ValueError("zero-size array to reduction operation maximum which has no identity "
                         f"(nsamples {x.shape[1]} < 8)")
    if plan is None:
        dms = np.ascontiguousarray(np.atleast_1d(np.asarray(trial_DMs, dtype=np.float64)))
        ident = ("dm", hashlib.sha1(dms.tobytes()).hexdigest(), dms.size, float(start_freq),
                 float(bandwidth), float(sample_time))
        plan = _plan_for(x, lambda: _hip.shift_table(nchan, dms, start_freq, bandwidth, sample_time),
                         _acc_code(acc), ident)
    return plan.search(x), plan


def _dedispersion_search(data, trial_DMs, nchan, start_freq, bandwidth, sample_time, acc=None):
    """dedispersion.py:174-202: per trial (max, std, snr, rebin[int32]) numpy arrays."""
    trial_DMs = np.asarray(trial_DMs, dtype=np.float64)
    if trial_DMs.size == 0:
        z = np.zeros(0)
        return z, z.copy(), z.copy(), np.zeros(0, np.int32)
    (mx, sd, snr, win), _ = search_device(data, trial_DMs, nchan, start_freq, bandwidth, sample_time, acc=acc)
    return _numpy_out(mx), _numpy_out(sd), _numpy_out(snr), _numpy_out(win)


def dedispersion_search(data, dmmin, dmmax, start_freq, bandwidth, sample_time, show=False, acc=None):
    """dedispersion.py:205-251: DM-trial search -> Table (and the plane if ``show``).

    ``show=True`` also returns the dedispersed plane (float64, shape (ndm, N)) and an
    int64 ``rebin`` column, like the reference's serial path; the plane lives in
    memory instead of an mkdtemp() memmap.
    """
    nchan = data.shape[0]
    trial_DMs = dedispersion_plan(nchan, dmmin, dmmax, start_freq, bandwidth, sample_time)
    if not show:
        mx, sd, snr, win = _dedispersion_search(data, trial_DMs, nchan, start_freq, bandwidth, sample_time,
                                                acc=acc)
        return make_table({"DM": trial_DMs, "max": mx, "std": sd, "snr": snr, "rebin": win})
    x = _prepare_data(data)
    if x.shape[1] < 8:
        raise ValueError("zero-size array to reduction operation maximum which has no identity "
                         f"(nsamples {x.shape[1]} < 8)")
    sh = _hip.shift_table(nchan, trial_DMs, start_freq, bandwidth, sample_time)
    plan = _plan_for(x, sh, _acc_code(acc or "f64"))
    plane = plan.dedisperse(x)
    if plane.dtype == _hip.torch().float64:
        # the reference's serial path computes each row's statistics from the plane
        # (dedispersion.py:223-243): pu_series_stats does that in numpy's order, so the
        # table is bit-identical to the reference's with the (default) float64 plane
        mx, sd, snr, win = _hip.series_stats(plane)
    else:
        mx, sd, snr, win = plan.search(x)
    table = make_table({"DM": trial_DMs, "max": _numpy_out(mx), "std": _numpy_out(sd), "snr": _numpy_out(snr),
                        "rebin": _numpy_out(win).astype(np.int64)})
    return table, _numpy_out(plane).astype(np.float64, copy=False)


def apply_dm_shifts_to_data(data, shifts):
    """dedispersion.py:254-258: roll channel i by ``-rint(shifts[i])`` (input dtype kept).

    The roll is a pure element move, done on the raw bits of 1/4/8-byte elements.
    """
    t = _hip.require_gpu()
    view_back = None
    if not isinstance(data, t.Tensor):
        data = np.ascontiguousarray(data)
        size_code = {1: np.uint8, 4: np.float32, 8: np.float64}
        if data.dtype.itemsize in size_code:
            view_back = data.dtype
            data = data.view(size_code[data.dtype.itemsize])
        else:
            view_back = data.dtype
            data = data.astype(np.float64)
    x = _hip.to_device(data, allowed=(_hip.PU_U8, _hip.PU_F32, _hip.PU_F64, _hip.PU_I64))
    nchan, n = x.shape
    sh = np.rint(np.asarray(shifts, dtype=np.float64)).astype(np.int64)
    if sh.size != nchan:
        raise ValueError("one shift per channel required")
    dsh = t.from_numpy(sh).to(x.device)
    out = t.empty_like(x)
    _hip.check(_hip.lib().pu_roll_rows(_hip.ptr(x), _hip.dtype_code(x.dtype), nchan, n, x.stride(0), _hip.ptr(dsh),
                                       _hip.ptr(out), _hip.stream_ptr()), "apply_dm_shifts_to_data")
    res = _numpy_out(out)
    if view_back is not None:
        res = res.view(view_back) if res.dtype.itemsize == np.dtype(view_back).itemsize else res.astype(view_back)
    return res
