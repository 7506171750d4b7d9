"""Tuning sweep of the C4 cleaning kernels (column mean, scaled row sums, apply).

Times each C-ABI call with torch events (the calls run on torch's current stream)
under every setting of the kernels' tuning variables (PU_CLEAN_VMAX, PU_CLEAN_BATCH,
PU_CLEAN_SCALE_ROWS, PU_CLEAN_NT, PU_MEDIAN_GRID; read per call), plus renormalize_device end to end.
One JSON line per (dtype, kernel, setting).

    python scripts/sweep_clean.py [--dtype f32,u8] [--steps 20]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "radio-pulsar-utils_amd"), REPO]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from pulsarutils import _hip, clean, synth  # noqa: E402
from pulsarutils.configs import CONFIGS  # noqa: E402

HBM = 8000.0


def timed(fn, steps, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps


def setenv(**kv):
    for k, v in kv.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = str(v)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="f32,u8")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--kernels", default="col_means,row_sums_scaled,apply,median,renormalize_device")
    args = ap.parse_args()
    want = set(args.kernels.split(","))
    lib = _hip.lib()
    cfg = CONFIGS["C4"]
    for dt in args.dtype.split(","):
        x = _hip.to_device(synth.rfi_filterbank_np(cfg, dtype=dt))
        nchan, n = x.shape
        b_in = x.element_size()
        code = _hip.dtype_code(x.dtype)
        bad_np = clean.get_noisier_channels(x)
        bad = torch.from_numpy(bad_np.astype(np.uint8)).to(x.device)
        lc = torch.empty(n, dtype=torch.float64, device=x.device)
        factor = torch.rand(n, dtype=torch.float64, device=x.device) + 0.5
        spec = torch.rand(nchan, dtype=torch.float64, device=x.device) + 60.0
        out = torch.empty((nchan, n), dtype=torch.float64, device=x.device)
        col = torch.empty(n, dtype=torch.float64, device=x.device)
        plane = nchan * n * b_in
        s = _hip.stream_ptr()

        def rec(kernel, setting, ms, nbytes):
            print(json.dumps({"dtype": dt, "kernel": kernel, "setting": setting, "us": round(ms * 1e3, 1),
                              "GBps": round(nbytes / ms / 1e6, 1), "hbm_frac": round(nbytes / ms / 1e6 / HBM, 3)}),
                  flush=True)

        for vmax in ((1, 2, 4) if "col_means" in want else ()):
            for batch in (128, 256, 512):
                setenv(PU_CLEAN_VMAX=vmax, PU_CLEAN_BATCH=batch)
                ms = timed(lambda: lib.pu_col_means(_hip.ptr(x), code, nchan, n, x.stride(0), _hip.ptr(bad),
                                                    _hip.ptr(lc), s), args.steps)
                rec("col_means", {"vmax": vmax, "batch": batch}, ms, plane)
        setenv(PU_CLEAN_VMAX=None, PU_CLEAN_BATCH=None)
        for rows in ((4, 8, 16) if "row_sums_scaled" in want else ()):
            setenv(PU_CLEAN_SCALE_ROWS=rows)
            ms = timed(lambda: clean._row_sums(x, 2, scale=factor, divisor=n), args.steps)
            rec("row_sums_scaled", {"rows": rows}, ms, plane)
        setenv(PU_CLEAN_SCALE_ROWS=None)
        for vmax in ((1, 2, 4) if "apply" in want else ()):
            for nt in (0, 1):
                for batch in (128, 256, 512):
                    setenv(PU_CLEAN_VMAX=vmax, PU_CLEAN_NT=nt, PU_APPLY_BATCH=batch)
                    ms = timed(lambda: lib.pu_renorm_apply(_hip.ptr(x), code, nchan, n, x.stride(0),
                                                           _hip.ptr(factor), _hip.ptr(spec), _hip.ptr(bad),
                                                           _hip.ptr(out), out.stride(0), _hip.ptr(col), s), args.steps)
                    rec("apply", {"vmax": vmax, "nt": nt, "batch": batch}, ms, plane + nchan * n * 8)
        setenv(PU_CLEAN_VMAX=None, PU_CLEAN_NT=None, PU_APPLY_BATCH=None)
        if "ceiling" in want:
            spec_f = torch.empty(nchan, dtype=torch.float32 if code == _hip.PU_F32 else torch.float64, device=x.device)
            ws_rs = torch.empty(max(16, lib.pu_row_sums_workspace_bytes(nchan, n)), dtype=torch.uint8, device=x.device)
            # the same traffic (read the plane, write it as float64) by torch's own
            # elementwise cast kernel: the achievable rate for this read/write mix
            ms = timed(lambda: out.copy_(x), args.steps)
            rec("ceiling_cast_copy", {}, ms, plane + nchan * n * 8)
            y = torch.empty_like(out)
            ms = timed(lambda: y.copy_(out), args.steps)
            rec("ceiling_f64_copy", {}, ms, 2 * nchan * n * 8)
            del y
            # write-only and read-only streams of the same plane sizes
            ms = timed(lambda: out.fill_(1.0), args.steps)
            rec("ceiling_f64_fill", {}, ms, nchan * n * 8)
            ms = timed(lambda: lib.pu_row_sums(_hip.ptr(x), code, nchan, n, x.stride(0), 0, None, None, float(n),
                                               _hip.ptr(spec_f), _hip.ptr(ws_rs), ws_rs.numel(), s), args.steps)
            rec("ceiling_read_rowsum", {}, ms, plane)
        if "median" in want:
            # the real light curve (column means over good channels), not uninitialised memory
            lib.pu_col_means(_hip.ptr(x), code, nchan, n, x.stride(0), _hip.ptr(bad), _hip.ptr(lc), s)
            for g in (256, 128, 64, 32):
                setenv(PU_MEDIAN_GRID=g)
                ms = timed(lambda: clean.median_device(lc), args.steps)
                rec("median", {"grid": g}, ms, n * 8)
            setenv(PU_MEDIAN_GRID=None)
        for cut in ((False, True) if "renormalize_device" in want else ()):
            ms = timed(lambda: clean.renormalize_device(x, badchans_mask=bad_np, cut_outliers=cut, out=out),
                       args.steps)
            rec("renormalize_device", {"cut_outliers": cut}, ms, 3 * plane + nchan * n * 8)
        del x, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
