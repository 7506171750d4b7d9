"""Load the reference ``pulsarutils`` modules from /root/reference by file path.

Golden-vector generation only (this container; /root/reference does not exist on
the GPU box).  Nothing here is imported by the product, the GPU tests or bench.

Recipe: the reference's undeclared / broken third-party imports are
replaced by stub modules *before* its files are executed, so the reference's own
Python source runs with interpreted numpy semantics:

* ``numba``: ``njit`` is the identity decorator, ``prange`` is ``range``.
* ``astropy``: ``log`` is a stdlib logger, ``table.Table`` a dict of columns.
* ``sigpyproc.Readers.FilReader`` / ``hendrics.efsearch.h_test``: raise if called
  (file I/O and the H-test are out of scope).
* ``statsmodels.robust.mad``: statsmodels 0.12.2's definition restated
  (``median(abs(a - median(a)) / c)``, ``c = norm.ppf(0.75)``); cross-checked
  against the real statsmodels 0.12.2 in /opt/conda/bin/python3.9 by
  ``make_golden.py``.
* ``np.float`` / ``np.int`` / ``np.bool`` aliases restored (removed in numpy>=1.24).

The reference files are executed from where they lie; no source is copied.
"""
import importlib.util
import logging
import os
import sys
import types

import numpy as np

REF_PKG = "/root/reference/pulsarutils"
_NAME = "_refpu"


def _stub_modules():
    numba = types.ModuleType("numba")

    def njit(*args, **kwargs):
        if args and callable(args[0]) and not kwargs:
            return args[0]
        return lambda f: f

    numba.njit = njit
    numba.prange = range
    numba.int8 = np.int8
    numba.int32 = np.int32
    sys.modules["numba"] = numba

    astropy = types.ModuleType("astropy")
    astropy.log = logging.getLogger("astropy-stub")
    table = types.ModuleType("astropy.table")

    class Table(dict):
        def __init__(self, cols):
            super().__init__({k: np.asarray(v) for k, v in cols.items()})

    table.Table = Table
    astropy.table = table
    sys.modules["astropy"] = astropy
    sys.modules["astropy.table"] = table

    def _raise(*a, **k):
        raise RuntimeError("stubbed out for golden generation")

    sig = types.ModuleType("sigpyproc")
    readers = types.ModuleType("sigpyproc.Readers")
    readers.FilReader = _raise
    sig.Readers = readers
    sys.modules["sigpyproc"] = sig
    sys.modules["sigpyproc.Readers"] = readers

    hen = types.ModuleType("hendrics")
    efs = types.ModuleType("hendrics.efsearch")
    efs.h_test = _raise
    hen.efsearch = efs
    sys.modules["hendrics"] = hen
    sys.modules["hendrics.efsearch"] = efs

    from scipy.stats import norm
    sm = types.ModuleType("statsmodels")
    robust = types.ModuleType("statsmodels.robust")

    def mad(a, c=norm.ppf(3 / 4.), axis=0, center=np.median):
        a = np.asarray(a, dtype=np.double)  # array_like(a, "a", ndim=None): dtype=np.double
        if callable(center) and a.size:
            center = np.apply_over_axes(center, a, axis)
        else:
            center = 0.0
        return np.median((np.abs(a - center)) / c, axis=axis)

    robust.mad = mad
    sm.robust = robust
    sys.modules["statsmodels"] = sm
    sys.modules["statsmodels.robust"] = robust

    np.float = float
    np.int = int
    np.bool = bool


def load_reference():
    """Return a namespace with the reference modules (dedispersion, simulate, stats, clean)."""
    if _NAME in sys.modules:
        return sys.modules[_NAME]
    sys.dont_write_bytecode = True
    os.environ.setdefault("MPLBACKEND", "Agg")
    _stub_modules()
    pkg = types.ModuleType(_NAME)
    pkg.__path__ = [REF_PKG]
    sys.modules[_NAME] = pkg
    for mod in ("dedispersion", "simulate", "stats", "clean"):
        full = f"{_NAME}.{mod}"
        spec = importlib.util.spec_from_file_location(full, os.path.join(REF_PKG, mod + ".py"))
        m = importlib.util.module_from_spec(spec)
        sys.modules[full] = m
        # simulate.py imports ``pulsarutils.dedispersion`` absolutely: point that name at
        # the reference module while it executes, then restore whatever was there.
        saved = {}
        if mod == "simulate":
            for k in ("pulsarutils", "pulsarutils.dedispersion"):
                saved[k] = sys.modules.get(k)
            sys.modules["pulsarutils"] = pkg
            sys.modules["pulsarutils.dedispersion"] = sys.modules[f"{_NAME}.dedispersion"]
        try:
            spec.loader.exec_module(m)
        finally:
            for k, v in saved.items():
                if v is None:
                    sys.modules.pop(k, None)
                else:
                    sys.modules[k] = v
        setattr(pkg, mod, m)
    return pkg
