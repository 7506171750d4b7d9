"""ORACLE - test infrastructure only (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).

CPU restatement of the reference's dedispersion + cleaning hot path, used as the
parity CHECKER of the HIP path and as the timed CPU baseline.  The product package
(``radio-pulsar-utils_amd/pulsarutils``) never imports this.

* ``liboracle.so`` (``dedisp_oracle.c``): float64 dedispersion search, bit-exact with
  the interpreted reference (pinned by tests/golden, see tests/test_oracle.py).
* :mod:`oracle.clean_oracle`: numpy restatement of ``clean.py`` / ``stats.py``.
* :mod:`oracle.numpy_order`: the numpy reduction order the bit-exact masks rely on.

Parity is PINNED: every function here is checked against golden vectors generated
by executing the reference's own source (tests/golden/make_golden.py).
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

_DT = {np.dtype(np.uint8): 0, np.dtype(np.float32): 1, np.dtype(np.float64): 2}


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        i64, f64, vp = ctypes.c_int64, ctypes.c_double, ctypes.c_void_p
        L.or_shifts.argtypes = [i64, f64, f64, f64, f64, vp]
        L.or_dedisperse.argtypes = [vp, ctypes.c_int, i64, i64, i64, vp, vp]
        L.or_dedisperse.restype = None
        L.or_search.argtypes = [vp, ctypes.c_int, i64, i64, i64, vp, i64, f64, f64, f64,
                                vp, vp, vp, vp, vp, ctypes.c_int]
        L.or_search_w.argtypes = [vp, ctypes.c_int, i64, i64, i64, vp, i64, f64, f64, f64,
                                  vp, vp, vp, vp, vp, vp, ctypes.c_int]
        L.or_np_sum.argtypes = [vp, i64]
        L.or_np_sum.restype = f64
        L.or_np_std.argtypes = [vp, i64, vp]
        L.or_np_std.restype = f64
        L.or_trial_stats.argtypes = [vp, i64, vp, vp, vp, vp, vp]
        L.or_trial_stats.restype = None
        L.or_max_threads.restype = ctypes.c_int
        _LIB = L
    return _LIB


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def shifts(nchan, dm, start_freq, bandwidth, sample_time):
    out = np.empty(int(nchan), np.int64)
    lib().or_shifts(int(nchan), float(dm), float(start_freq), float(bandwidth), float(sample_time), _p(out))
    return out


def dedisperse(data, shifts_):
    data = np.ascontiguousarray(data)
    if data.dtype not in _DT:
        data = data.astype(np.float64)
    sh = np.ascontiguousarray(np.asarray(shifts_), dtype=np.int64)
    nchan, n = data.shape
    out = np.empty(n, np.float64)
    lib().or_dedisperse(_p(data), _DT[data.dtype], nchan, n, n, _p(sh), _p(out))
    return out


def search(data, trial_dms, start_freq, bandwidth, sample_time, nthreads=0, return_dedisp=False,
           return_width_snr=False):
    """``_dedispersion_search`` restated: returns (max, std, snr, rebin[int32]), then the
    dedispersed series ``[ndm, n]`` if ``return_dedisp``, then (test-side only) the S/N of
    each rebin width 1/2/4/8 ``[ndm, 4]`` if ``return_width_snr`` (the candidates of the
    reference's first-strict-best choice, ``dedispersion.py:189-201``; NaN for widths longer
    than the series)."""
    data =np.ascontiguousarray(data)
    if data.dtype not in _DT:
        data = data.astype(np.float64)
    dms = np.ascontiguousarray(trial_dms, dtype=np.float64)
    nchan, n = data.shape
    nd = dms.size
    mx, sd, snr = (np.empty(nd) for _ in range(3))
    win = np.empty(nd, np.int64)
    dd = np.empty((nd, n)) if return_dedisp else None
    sw = np.full((nd, 4), np.nan) if return_width_snr else None
    rc = lib().or_search_w(_p(data), _DT[data.dtype], nchan, n, n, _p(dms), nd, float(start_freq),
                           float(bandwidth), float(sample_time), _p(mx), _p(sd), _p(snr), _p(win),
                           _p(dd) if dd is not None else None, _p(sw) if sw is not None else None,
                           int(nthreads))
    if rc:
        raise MemoryError("oracle search failed")
    out = (mx, sd, snr, win.astype(np.int32))
    if return_dedisp:
        out = out + (dd,)
    if return_width_snr:
        out = out + (sw,)
    return out


def trial_stats(dedisp):
    """Per-trial statistics of one dedispersed float64 series (dedispersion.py:186-201)."""
    dd = np.ascontiguousarray(dedisp, dtype=np.float64)
    n = dd.size
    work = np.empty(2 * n)
    o = [np.zeros(1) for _ in range(3)] + [np.zeros(1, np.int64)]
    lib().or_trial_stats(_p(dd), n, _p(work), *[_p(v) for v in o])
    return float(o[0][0]), float(o[1][0]), float(o[2][0]), int(o[3][0])


def np_sum(a):
    a = np.ascontiguousarray(a, dtype=np.float64)
    return lib().or_np_sum(_p(a), a.size)


def max_threads():
    return lib().or_max_threads()
