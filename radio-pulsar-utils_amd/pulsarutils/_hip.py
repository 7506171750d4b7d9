"""ctypes binding of libpulsarutils_hip.so (the C-ABI in include/pulsarutils_hip.h).

PyTorch-ROCm is plumbing here: device memory, the current HIP stream, host<->device
copies.  Every compute step of the hot path is a call into the HIP library; there is
no CPU fallback - without the library or a GPU the calls raise.
"""
import ctypes
import os
import threading

import numpy as np

PU_U8, PU_F32, PU_F64, PU_I64 = 0, 1, 2, 3
PU_ACC_NATIVE, PU_ACC_F32, PU_ACC_F64 = 0, 1, 2
_EINVAL, _EHIP, _ENOMEM, _EUNSUPPORTED = -1, -2, -3, -4

_LIB_PATH = os.environ.get(
    "PULSARUTILS_HIP_LIB",
    os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libpulsarutils_hip.so"))

_lib = None
_lock = threading.Lock()

# name -> (restype, argtypes)
_i64, _i32, _f64, _vp, _sz = ctypes.c_int64, ctypes.c_int, ctypes.c_double, ctypes.c_void_p, ctypes.c_size_t
SIGNATURES = {
    "pu_version": (ctypes.c_char_p, []),
    "pu_last_error": (ctypes.c_char_p, []),
    "pu_shift_table": (_i32, [_i64, _vp, _i64, _f64, _f64, _f64, _vp]),
    "pu_plan_create": (_i32, [ctypes.POINTER(_vp), _i32, _i32, _i64, _i64, _vp, _i64]),
    "pu_plan_create_grouped": (_i32, [ctypes.POINTER(_vp), _i32, _i32, _i64, _i64, _vp, _i64, _i32]),
    "pu_plan_create_ex": (_i32, [ctypes.POINTER(_vp), _i32, _i32, _i64, _i64, _vp, _i64, _vp]),
    "pu_plan_destroy": (None, [_vp]),
    "pu_plan_workspace_bytes": (_sz, [_vp]),
    "pu_plan_search": (_i32, [_vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _sz, _vp]),
    "pu_plan_dedisperse": (_i32, [_vp, _vp, _i64, _vp, _i64, _vp]),
    "pu_plan_dm_tiles": (_i32, [_vp, _vp, _vp, _i32]),
    "pu_plan_dedisperse_dm_tile": (_i32, [_vp, _vp, _i64, _i64, _vp, _i64, _vp]),
    "pu_plan_search_tiles": (_i32, [_vp, _vp, _i64, _i64, _i64, _vp, _sz, _vp]),
    "pu_plan_finalize": (_i32, [_vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _sz, _vp]),
    "pu_plan_finalize_range": (_i32, [_vp, _vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _sz, _vp]),
    "pu_plan_finalize_range_flagged": (_i32, [_vp, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _sz, _vp, _i64, _vp, _vp]),
    "pu_plan_exact_series": (_i32, [_vp, _vp, _i64, _vp, _i64, _i64, _i64, _vp, _vp]),
    "pu_nonfinite_any": (_i32, [_vp, _i32, _i64, _i64, _i64, _vp, _vp]),
    "pu_series_stats_workspace_bytes": (_sz, [_i64, _i64]),
    "pu_series_stats": (_i32, [_vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _sz, _vp]),
    "pu_plan_info": (_i32, [_vp, _vp, _i32]),
    "pu_plan_enable_timing": (_i32, [_vp, _i32]),
    "pu_plan_kernel_times": (_i32, [_vp, _vp, _i32]),
    "pu_plan_stamps": (_i32, [_vp, _vp, _i32]),
    "pu_row_sums": (_i32, [_vp, _i32, _i64, _i64, _i64, _i32, _vp, _vp, _f64, _vp, _vp, _sz, _vp]),
    "pu_row_sums_workspace_bytes": (_sz, [_i64, _i64]),
    "pu_row_moments": (_i32, [_vp, _i32, _i64, _i64, _i64, _vp, _vp, _vp, _sz, _vp]),
    "pu_row_moments_workspace_bytes": (_sz, [_i64, _i64]),
    "pu_col_means": (_i32, [_vp, _i32, _i64, _i64, _i64, _vp, _vp, _vp]),
    "pu_gaussian_filter1d": (_i32, [_vp, _i64, _vp, _i64, _vp, _vp]),
    "pu_ratio": (_i32, [_f64, _vp, _i64, _vp, _vp]),
    "pu_median_workspace_bytes": (_sz, []),
    "pu_median": (_i32, [_vp, _i64, _vp, _vp, _sz, _vp]),
    "pu_noisy_channels": (_i32, [_vp, _i32, _i64, _f64, _vp, _vp, _vp]),
    "pu_variability_cert": (_i32, [_vp, _i32, _vp, _i64, _i64, _f64, _f64, _f64, _vp, _vp, _vp, _vp]),
    "pu_channel_masks": (_i32, [_vp, _i32, _vp, _i64, _i64, _f64, _f64, _f64, _f64, _vp, _vp, _vp, _vp, _vp]),
    "pu_ratio_dev": (_i32, [_vp, _vp, _i64, _vp, _vp]),
    "pu_lc_factor_workspace_bytes": (_sz, [_i64]),
    "pu_lc_factor": (_i32, [_vp, _i64, _vp, _i64, _vp, _vp, _vp, _sz, _vp]),
    "pu_renorm_apply": (_i32, [_vp, _i32, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _i64, _vp, _vp]),
    "pu_renorm_apply_zero_dm": (_i32, [_vp, _i32, _i64, _i64, _i64, _vp, _vp, _vp, _i64, _vp, _i64, _vp, _vp]),
    "pu_zero_columns": (_i32, [_vp, _i64, _i64, _vp, _i64, _vp]),
    "pu_cut_outliers_workspace_bytes": (_sz, [_i64]),
    "pu_cut_outliers": (_i32, [_vp, _i64, _vp, _i64, _i64, _vp, _vp, _sz, _vp]),
    "pu_cut_outliers_exact": (_i32, [_vp, _i64, _vp, _i64, _i64, _vp, _vp, _sz, _vp]),
    "pu_rebin_time": (_i32, [_vp, _i32, _i64, _i64, _i64, _i64, _vp, _vp]),
    "pu_rebin_chan": (_i32, [_vp, _i32, _i64, _i64, _i64, _i64, _vp, _vp]),
    "pu_roll_rows": (_i32, [_vp, _i32, _i64, _i64, _i64, _vp, _vp, _vp]),
    "pu_roll_and_sum": (_i32, [_vp, _i32, _i64, _i64, _vp, _vp]),
    "pu_transpose": (_i32, [_vp, _i32, _i64, _i64, _i64, _vp, _i64, _vp]),
    "pu_stream_create_cu_masked": (_i32, [_i32, ctypes.POINTER(_vp)]),
    "pu_stream_destroy": (_i32, [_vp]),
}

INFO_FIELDS = ("ndm", "dm_tiles", "time_tiles", "trials_per_tile", "time_tile", "chans_per_step",
               "row_stride", "lds_bytes", "acc_is_f64", "max_spread", "group", "slots", "stages",
               "slot_bytes", "raw_stride", "exec_adds", "lds_traffic", "cert_rechecked", "cert_nan", "cert_std", "cert_sign",
               "cert_tie", "cert_us", "kernel", "rec_elem_bytes", "rec_stride")
KERNEL_NAMES = ("dedisp_kernel", "dedisp_f64_kernel", "dedisp_sub_kernel", "dedisp_sub_kernel (u16 slots)")


class HipBackendError(RuntimeError):
    pass


class PlanOpts(ctypes.Structure):
    """``pu_plan_opts`` (include/pulsarutils_hip.h): the planner's explicit options."""
    _fields_ = [("group", ctypes.c_int32), ("shape", ctypes.c_int32), ("lds_budget_kb", ctypes.c_int32),
                ("u8_dma", ctypes.c_int32), ("dt_major", ctypes.c_int32), ("slot16", ctypes.c_int32),
                ("reserved", ctypes.c_int32 * 2)]


SHAPES = {"wide": 0, "pair": 1, "tall": 2}


_SRC_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc")
_INC_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "include")


def source_hashes():
    """SHA-256 of every source the library is built from (csrc/*.hip|cpp|h, include/*.h)."""
    import hashlib
    out = {}
    for d, exts in ((_SRC_DIR, (".hip", ".cpp", ".h")), (_INC_DIR, (".h",))):
        if not os.path.isdir(d):
            continue
        for name in sorted(os.listdir(d)):
            if name.endswith(exts):
                with open(os.path.join(d, name), "rb") as f:
                    out[os.path.basename(d) + "/" + name] = hashlib.sha256(f.read()).hexdigest()
    return out


def build_info():
    """Provenance of the library file: what ``__graft_entry__.build()`` recorded next to it
    (source hashes, hipcc version, time) and whether the sources on disk still match -
    False means the .so was built from other sources than the ones shipped beside it."""
    import json
    path = os.path.join(os.path.dirname(_LIB_PATH), "BUILD_INFO.json")
    if not os.path.exists(path):
        return {"recorded": False}
    with open(path) as f:
        rec = json.load(f)
    return {"recorded": True, "built": rec.get("built"), "hipcc": rec.get("hipcc"),
            "sources_match": rec.get("sources") == source_hashes()}


def lib():
    """Load the HIP library (raises if it is missing: no silent fallback)."""
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(_LIB_PATH):
                    raise HipBackendError(
                        f"pulsarutils: HIP library not found at {_LIB_PATH}; build it with "
                        "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950)")
                # PyTorch first: its wheel bundles its own libamdhip64.so.7 / HSA runtime.
                # Loaded after ours (RUNPATH /opt/rocm), the process would hold TWO HIP and
                # HSA runtimes, and the second to open the GPU finds "no ROCm-capable
                # device" (seen on the MI355X box when the first call was shift_table).
                # With torch loaded, our DT_NEEDED libamdhip64.so.7 resolves to its copy.
                torch()
                L = ctypes.CDLL(_LIB_PATH)
                for name, (res, args) in SIGNATURES.items():
                    if "PULSARUTILS_HIP_LIB" in os.environ and not hasattr(L, name):
                        continue  # an older build loaded for an A/B run (scripts/ab_lib.sh)
                    fn = getattr(L, name)
                    fn.restype = res
                    fn.argtypes = args
                _lib = L
    return _lib


def check(rc, what=""):
    if rc == 0:
        return
    msg = lib().pu_last_error().decode(errors="replace")
    if rc in (_EINVAL, _EUNSUPPORTED):
        raise ValueError(f"{what}: {msg}")
    if rc == _ENOMEM:
        raise MemoryError(f"{what}: {msg}")
    raise HipBackendError(f"{what}: {msg}")


def torch():
    import torch as _t
    return _t


_GPU_OK = [False]


def require_gpu():
    t = torch()
    if not _GPU_OK[0]:  # (checked once: is_available() costs a few microseconds per call)
        if not t.cuda.is_available():
            raise HipBackendError("pulsarutils: the dedispersion/cleaning path runs on a ROCm GPU "
                                  "(MI355X / gfx950); torch.cuda.is_available() is False")
        lib()
        _GPU_OK[0] = True
    return t


def stream_ptr(stream=None):
    """The hipStream_t of ``stream``, or of torch's current stream on the current device -
    read raw (no Stream object: torch.cuda.current_stream() costs ~3 us per call)."""
    if stream is not None:
        return ctypes.c_void_p(stream.cuda_stream)
    t = torch()
    return ctypes.c_void_p(t._C._cuda_getCurrentRawStream(t.cuda.current_device()))


def ptr(tensor):
    return ctypes.c_void_p(tensor.data_ptr()) if tensor is not None else None


_DTYPE_CODES = {}


def dtype_code(tdtype):
    t = torch()
    if not _DTYPE_CODES:
        _DTYPE_CODES.update({t.uint8: PU_U8, t.float32: PU_F32, t.float64: PU_F64, t.int64: PU_I64})
    return _DTYPE_CODES.get(tdtype)


def to_device(a, allowed=(PU_U8, PU_F32, PU_F64), device=None):
    """numpy array or torch tensor -> contiguous device tensor of a supported dtype.

    Unsupported element types are converted ON THE DEVICE to float64 (exact for
    every integer below 2**53), i.e. the same promotion the reference's float64
    accumulators apply.
    """
    t = require_gpu()
    dev = device if device is not None else t.device("cuda", t.cuda.current_device())
    if isinstance(a, t.Tensor):
        x = a.to(dev)
    else:
        arr = np.asarray(a)
        if arr.dtype == np.bool_:
            arr = arr.astype(np.uint8)
        if arr.dtype.byteorder not in ("=", "|"):
            arr = arr.astype(arr.dtype.newbyteorder("="))
        x = t.from_numpy(np.ascontiguousarray(arr)).to(dev, non_blocking=False)
    if dtype_code(x.dtype) not in allowed:
        x = x.to(t.float64)
    return x.contiguous()


class Plan:
    """Owning wrapper of a ``pu_plan`` (dedispersion tiling + device metadata)."""

    def __init__(self, dtype_code_, acc, nchan, nsamples, shifts, group=0, shape=None, lds_budget_kb=0,
                 u8_dma=None, dt_major=None, slot16=None):
        """``group``: channels summed per group row (0 = library default, 1 = channel
        mode, 2/4/8); float64 accumulation always uses channel mode.  ``shape``: subband
        workgroup shape ("wide", "pair", "tall" or 0/1/2; None = the cost model's choice);
        ``lds_budget_kb``: LDS per workgroup (0 = default); ``u8_dma``: False builds 8-bit
        slots from global memory instead of LDS-DMA'd rows; ``dt_major``: work-item order
        (None = automatic); ``slot16``: 16-bit integer slots for 8-bit DMA rows in 256-sample
        tiles - None / True: at every group size, False: never (float32
        slots).  These are the planner's only inputs (pu_plan_create_ex): the
        library reads no environment."""
        require_gpu()
        sh = np.ascontiguousarray(shifts, dtype=np.int64)
        if sh.ndim != 2 or sh.shape[1] != int(nchan):
            raise ValueError(f"shift table must be (ndm, {nchan}) int64, got shape {sh.shape}")
        ndm = sh.shape[0]
        opts = PlanOpts(group=int(group), shape=-1 if shape is None else int(SHAPES.get(shape, shape)),
                        lds_budget_kb=int(lds_budget_kb), u8_dma=-1 if u8_dma is None else int(bool(u8_dma)),
                        dt_major=-1 if dt_major is None else int(bool(dt_major)),
                        slot16=-1 if slot16 is None else int(bool(slot16)))
        h = ctypes.c_void_p()
        check(lib().pu_plan_create_ex(ctypes.byref(h), dtype_code_, acc, nchan, nsamples,
                                      sh.ctypes.data_as(ctypes.c_void_p), ndm, ctypes.byref(opts)),
              "pu_plan_create")
        self._h = h
        self.dtype_code = dtype_code_
        self.nchan, self.nsamples, self.ndm = nchan, nsamples, ndm
        # shift extent of the grid: a time tile [t0, t0 + TT) reads samples
        # [t0 + shift_min, t0 + TT + shift_max] (mod nsamples) of some channel
        self.shift_min = int(sh.min()) if sh.size else 0
        self.shift_max = int(sh.max()) if sh.size else 0
        info = np.zeros(len(INFO_FIELDS), np.int64)
        lib().pu_plan_info(h, info.ctypes.data_as(ctypes.c_void_p), len(INFO_FIELDS))
        self.info = dict(zip(INFO_FIELDS, info.tolist()))
        self.workspace_bytes = lib().pu_plan_workspace_bytes(h)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and _lib is not None:
            _lib.pu_plan_destroy(h)
            self._h = None

    @property
    def acc_is_f64(self):
        return bool(self.info["acc_is_f64"])

    def _check_data(self, data):
        """Validate before any launch (raises, never asserts: under ``python -O`` an
        assert would vanish and a wrong-shaped tensor would be read out of bounds)."""
        t = torch()
        if not isinstance(data, t.Tensor) or not data.is_cuda:
            raise ValueError("plan data must be a CUDA (HIP) torch.Tensor")
        if data.dim() != 2 or data.stride(1) != 1:
            raise ValueError(f"plan data must be a 2-D row-major tensor, got shape {tuple(data.shape)} "
                             f"strides {tuple(data.stride())}")
        if tuple(data.shape) != (self.nchan, self.nsamples):
            raise ValueError(f"data shape {tuple(data.shape)} does not match the plan "
                             f"({self.nchan}, {self.nsamples})")
        if data.stride(0) < self.nsamples:
            raise ValueError(f"row stride {data.stride(0)} < nsamples {self.nsamples}")
        if dtype_code(data.dtype) != self.dtype_code:
            raise ValueError(f"data dtype {data.dtype} does not match the plan's dtype code {self.dtype_code}")

    @staticmethod
    def _rows_aligned(data, stream=None):
        """8-bit rows are staged by LDS-DMA in whole dwords: a view whose rows do not start
        on 4-byte boundaries is copied once into a fresh (aligned, contiguous) tensor.  The
        copy is made ON the launch stream (so it is ordered after whatever that stream
        waits for, and the caching allocator only reuses its memory after that stream's
        later work, i.e. after the kernel that reads it)."""
        # only 8-bit plans with N % 4 == 0 stage rows by LDS-DMA (the others read global
        # memory at any alignment)
        if (data.element_size() == 1 and data.shape[1] % 4 == 0
                and (data.data_ptr() % 4 or data.stride(0) % 4)):
            t = torch()
            with t.cuda.stream(stream if stream is not None else t.cuda.current_stream(data.device)):
                return data.clone(memory_format=t.contiguous_format)
        return data

    def _outs_ws(self, dev, out, workspace):
        """Output tensors and workspace of a search / finalize: allocated when None,
        validated otherwise (dtype, length, contiguity, device, size) before any launch
        writes them."""
        t = torch()
        want = (t.float64, t.float64, t.float64, t.int32)
        if out is None:
            out = tuple(t.empty(self.ndm, dtype=w, device=dev) for w in want)
        elif len(out) != 4 or any(not isinstance(o, t.Tensor) or o.dtype != w or o.numel() < self.ndm
                                  or not o.is_contiguous() or o.device != dev for o, w in zip(out, want)):
            raise ValueError(f"out must be 3 float64 + 1 int32 contiguous tensors of >= {self.ndm} "
                             f"elements on {dev}")
        if workspace is None:
            workspace = t.empty(max(self.workspace_bytes, 16), dtype=t.uint8, device=dev)
        elif (not isinstance(workspace, t.Tensor) or workspace.device != dev or not workspace.is_contiguous()
              or workspace.numel() * workspace.element_size() < self.workspace_bytes
              or workspace.data_ptr() % 8):
            raise ValueError(f"workspace must be a contiguous, 8-byte aligned tensor of >= "
                             f"{self.workspace_bytes} bytes on {dev}")
        return out, workspace

    def search(self, data, out=None, workspace=None, stream=None):
        """Launch the fused search (+ certification); returns (max, std,
        snr, rebin) device tensors, final when this returns."""
        self._check_data(data)
        data = self._rows_aligned(data, stream)
        out, workspace = self._outs_ws(data.device, out, workspace)
        check(lib().pu_plan_search(self._h, ptr(data), data.stride(0), ptr(out[0]), ptr(out[1]), ptr(out[2]),
                                   ptr(out[3]), ptr(workspace), workspace.numel() * workspace.element_size(),
                                   stream_ptr(stream)),
              "pu_plan_search")
        return out

    def search_tiles(self, data, tt_begin, tt_end, workspace, stream=None):
        """Shift-and-sum + per-tile statistics of time tiles [tt_begin, tt_end) only
        (pu_plan_search_tiles); ``finalize`` after every tile has run."""
        self._check_data(data)
        data = self._rows_aligned(data, stream)
        _, workspace = self._outs_ws(data.device, None, workspace)
        check(lib().pu_plan_search_tiles(self._h, ptr(data), data.stride(0), int(tt_begin), int(tt_end),
                                         ptr(workspace), workspace.numel() * workspace.element_size(),
                                         stream_ptr(stream)),
              "pu_plan_search_tiles")

    def finalize(self, workspace, data, out=None, stream=None):
        """Per-trial (max, std, snr, rebin) from the per-tile records (pu_plan_finalize);
        ``data`` is the searched filterbank (trials the fast statistics cannot certify
        are recomputed from it exactly)."""
        self._check_data(data)
        data = self._rows_aligned(data, stream)
        out, workspace = self._outs_ws(data.device, out, workspace)
        check(lib().pu_plan_finalize(self._h, ptr(data), data.stride(0), ptr(out[0]), ptr(out[1]), ptr(out[2]),
                                     ptr(out[3]), ptr(workspace), workspace.numel() * workspace.element_size(),
                                     stream_ptr(stream)), "pu_plan_finalize")
        return out

    def finalize_range(self, workspace, data, trial_begin, trial_end, out=None, stream=None):
        """``finalize`` of trials [trial_begin, trial_end) only (pu_plan_finalize_range): the
        outputs are indexed by plan trial (length ndm), only the range is written; the
        range's records in ``workspace`` must be complete (every time tile)."""
        self._check_data(data)
        data = self._rows_aligned(data, stream)
        out, workspace = self._outs_ws(data.device, out, workspace)
        check(lib().pu_plan_finalize_range(self._h, ptr(data), data.stride(0), int(trial_begin), int(trial_end),
                                           ptr(out[0]), ptr(out[1]), ptr(out[2]), ptr(out[3]), ptr(workspace),
                                           workspace.numel() * workspace.element_size(), stream_ptr(stream)),
              "pu_plan_finalize_range")
        return out

    def finalize_range_flagged(self, workspace, trial_begin, trial_end, out=None, device=None, stream=None):
        """pu_plan_finalize_range_flagged: the fast statistics of trials [begin, end) and the
        trials certification would recompute, not recomputed: returns (out, flagged int32
        numpy array of plan trials, count with a non-finite partial)."""
        t = torch()
        dev = device if device is not None else workspace.device
        out, workspace = self._outs_ws(dev, out, workspace)
        cap = max(0, int(trial_end) - int(trial_begin))
        flagged = np.zeros(max(1, cap), np.int32)
        counts = np.zeros(2, np.int64)
        check(lib().pu_plan_finalize_range_flagged(self._h, int(trial_begin), int(trial_end), ptr(out[0]), ptr(out[1]),
                                                   ptr(out[2]), ptr(out[3]), ptr(workspace),
                                                   workspace.numel() * workspace.element_size(),
                                                   flagged.ctypes.data_as(ctypes.c_void_p), cap,
                                                   counts.ctypes.data_as(ctypes.c_void_p), stream_ptr(stream)),
              "pu_plan_finalize_range_flagged")
        del t
        return out, flagged[:min(cap, int(counts[0]))].copy(), int(counts[1])

    def exact_series(self, data, trials, out=None, stream=None, t_begin=0, t_end=None):
        """pu_plan_exact_series: float64 channel-order series (len(trials), t_end - t_begin) of
        the given plan trials at samples [t_begin, t_end) (default: all), exact where the
        columns they read are in ``data``."""
        t = torch()
        self._check_data(data)
        data = self._rows_aligned(data, stream)
        tr = np.ascontiguousarray(trials, dtype=np.int32)
        t_end = self.nsamples if t_end is None else int(t_end)
        w = t_end - int(t_begin)
        if out is None:
            out = t.empty((tr.size, max(0, w)), dtype=t.float64, device=data.device)
        elif (out.dtype != t.float64 or not out.is_contiguous() or out.numel() < tr.size * w
              or out.device != data.device):
            raise ValueError("out must be a contiguous float64 tensor of >= len(trials) x (t_end - t_begin) on the "
                             "data device")
        check(lib().pu_plan_exact_series(self._h, ptr(data), data.stride(0), tr.ctypes.data_as(ctypes.c_void_p),
                                         tr.size, int(t_begin), t_end, ptr(out), stream_ptr(stream)),
              "pu_plan_exact_series")
        return out

    def records(self, workspace):
        """The per-(trial, time tile) partial records at the start of ``workspace``, as a
        (ndm, time_tiles, rec_stride) float32 / float64 view (pu_plan_finalize_range)."""
        t = torch()
        eb, rs = self.info["rec_elem_bytes"], self.info["rec_stride"]
        nel = self.ndm * self.info["time_tiles"] * rs
        dt = {4: t.float32, 8: t.float64}[eb]
        if workspace.numel() * workspace.element_size() < nel * eb:
            raise ValueError("workspace smaller than the plan's records")
        return workspace.view(t.uint8)[:nel * eb].view(dt).view(self.ndm, self.info["time_tiles"], rs)

    def cert_info(self):
        """Certification outcome of the last search / finalize: trials recomputed exactly
        and whether the input's NaN / inf rule applied."""
        info = np.zeros(len(INFO_FIELDS), np.int64)
        lib().pu_plan_info(self._h, info.ctypes.data_as(ctypes.c_void_p), len(INFO_FIELDS))
        d = dict(zip(INFO_FIELDS, info.tolist()))
        return {"rechecked": d["cert_rechecked"], "nan_rule": bool(d["cert_nan"]),
                "flagged_by": {"std": d["cert_std"], "sign": d["cert_sign"], "tie": d["cert_tie"]},
                "settle_ms": d["cert_us"] / 1e3}

    def tile_window(self, tt):
        """Half-open sample range [a, b) (NOT reduced mod nsamples) time tile ``tt``
        may read: a staged row starts at the tile's smallest shift of its channel
        (rounded down to a dword for 8-bit rows) and spans TT + the tile's largest shift
        spread + 1 samples, rounded up to whole 256-byte LDS-DMA pieces."""
        tt_len = self.info["time_tile"]
        t0 = int(tt) * tt_len
        return (t0 + self.shift_min - 8,
                t0 + tt_len + self.shift_max + self.info["max_spread"] + 1 + 256 + 8)

    def enable_timing(self, nslots):
        check(lib().pu_plan_enable_timing(self._h, int(nslots)), "pu_plan_enable_timing")

    def kernel_times_ms(self, n):
        out = np.zeros(int(n), np.float32)
        m = lib().pu_plan_kernel_times(self._h, out.ctypes.data_as(ctypes.c_void_p), int(n))
        if m < 0:
            check(m, "pu_plan_kernel_times")
        return out[:m]

    def dedisperse(self, data, plane=None, stream=None):
        """Dedispersed plane (ndm, nsamples) in the accumulation dtype."""
        t = torch()
        self._check_data(data)
        data = self._rows_aligned(data, stream)
        pdt = t.float64 if self.acc_is_f64 else t.float32
        if plane is None:
            plane = t.empty((self.ndm, self.nsamples), dtype=pdt, device=data.device)
        elif (plane.dtype != pdt or plane.dim() != 2 or plane.shape[0] < self.ndm or plane.shape[1] < self.nsamples
              or plane.stride(1) != 1 or plane.device != data.device):
            raise ValueError(f"plane must be a row-major ({self.ndm}, {self.nsamples}) {pdt} tensor on {data.device}")
        check(lib().pu_plan_dedisperse(self._h, ptr(data), data.stride(0), ptr(plane), plane.stride(0),
                                       stream_ptr(stream)), "pu_plan_dedisperse")
        return plane

    def dm_tiles(self):
        """The plan's DM tiles in launch order: int32 arrays (first trial, trial count)."""
        nt = int(self.info["dm_tiles"])
        first, count = np.zeros(nt, np.int32), np.zeros(nt, np.int32)
        lib().pu_plan_dm_tiles(self._h, first.ctypes.data_as(ctypes.c_void_p), count.ctypes.data_as(ctypes.c_void_p),
                               nt)
        return first, count

    def dedisperse_dm_tile(self, data, dt, stream=None):
        """Rows of DM tile ``dt``'s trials (``dm_tiles()[0][dt]`` onwards), shape (count,
        nsamples), computed by the same kernel, tables and tiling as a full launch."""
        t = torch()
        self._check_data(data)
        data = self._rows_aligned(data, stream)
        first, count = self.dm_tiles()
        if not 0 <= int(dt) < first.size:
            raise ValueError(f"DM tile {dt} outside [0, {first.size})")
        pdt = t.float64 if self.acc_is_f64 else t.float32
        plane = t.empty((int(count[dt]), self.nsamples), dtype=pdt, device=data.device)
        check(lib().pu_plan_dedisperse_dm_tile(self._h, ptr(data), data.stride(0), int(dt), ptr(plane),
                                               plane.stride(0), stream_ptr(stream)), "pu_plan_dedisperse_dm_tile")
        return plane


def nonfinite_any(x, flag, stream=None):
    """pu_nonfinite_any: flag (device int32, 1 element) = 1 if the 2-D float tensor x (row
    stride x.stride(0)) holds NaN / inf, else 0; asynchronous on ``stream``."""
    require_gpu()
    code = dtype_code(x.dtype)
    if x.dim() != 2 or x.stride(1) != 1 or code is None:
        raise ValueError("nonfinite_any: a 2-D row-major uint8 / float32 / float64 CUDA tensor")
    check(lib().pu_nonfinite_any(ptr(x), code, x.shape[0], x.shape[1], x.stride(0), ptr(flag), stream_ptr(stream)),
          "pu_nonfinite_any")
    return flag


def shift_table(nchan, trial_dms, start_freq, bandwidth, sample_time):
    """pu_shift_table: the reference shifts for every trial, int64 [ndm, nchan] (host)."""
    dms = np.ascontiguousarray(np.atleast_1d(np.asarray(trial_dms, dtype=np.float64)))
    out = np.empty((dms.size, int(nchan)), np.int64)
    check(lib().pu_shift_table(int(nchan), dms.ctypes.data_as(ctypes.c_void_p), dms.size, float(start_freq),
                               float(bandwidth), float(sample_time), out.ctypes.data_as(ctypes.c_void_p)),
          "pu_shift_table")
    return out


def series_stats(series, stream=None):
    """pu_series_stats: the reference's per-trial (max, std, snr, rebin) of float64
    dedispersed series (rows of a 2-D CUDA tensor), in numpy's exact order."""
    t = require_gpu()
    if not (isinstance(series, t.Tensor) and series.is_cuda and series.dtype == t.float64 and series.dim() == 2
            and series.stride(1) == 1):
        raise ValueError("series must be a 2-D row-major float64 CUDA tensor")
    rows, n = series.shape
    dev = series.device
    out = (t.empty(rows, dtype=t.float64, device=dev), t.empty(rows, dtype=t.float64, device=dev),
           t.empty(rows, dtype=t.float64, device=dev), t.empty(rows, dtype=t.int32, device=dev))
    if rows == 0:
        return out
    per = max(1, min(rows, (1 << 30) // max(1, 12 * n)))
    wsb = lib().pu_series_stats_workspace_bytes(per, n)
    ws = t.empty(wsb + 256, dtype=t.uint8, device=dev)
    off = (-ws.data_ptr()) % 256
    check(lib().pu_series_stats(ptr(series), rows, n, series.stride(0), None, ptr(out[0]), ptr(out[1]), ptr(out[2]),
                                ptr(out[3]), ctypes.c_void_p(ws.data_ptr() + off), wsb, stream_ptr(stream)),
          "pu_series_stats")
    return out


class MaskedStream:
    """A torch view of a CU-masked HIP stream (pu_stream_create_cu_masked) that leaves
    ``reserve`` CUs free for kernels of other streams (RCCL during the chunked
    broadcast).  Destroyed with the object."""

    def __init__(self, reserve, device=None):
        t = require_gpu()
        h = ctypes.c_void_p()
        with t.cuda.device(device if device is not None else t.cuda.current_device()):
            check(lib().pu_stream_create_cu_masked(int(reserve), ctypes.byref(h)), "pu_stream_create_cu_masked")
            self.stream = t.cuda.ExternalStream(h.value)
        self._h = h
        self.reserve = int(reserve)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and _lib is not None:
            _lib.pu_stream_destroy(h)
            self._h = None
