"""Time the file pipeline (search_by_chunks, clean.py:276-351) on a C4-sized SIGPROC file.

Writes a time-major SIGPROC file of 1024 channels (C4 band, RFI recipe of
synth.rfi_filterbank_np), 2^18-sample chunks with 50 % overlap, then runs
``get_bad_chans`` and ``search_by_chunks`` with per-chunk synchronised timings (H2D of
the block, GPU transpose, cleaning, rebin, cast, search).  One JSON line per
(dtype, search_dtype) on stdout.

    python scripts/bench_pipeline.py [--dtype u8|f32] [--chunks 4]
"""
import argparse
import json
import os
import sys
import tempfile
import time
from dataclasses import replace

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "radio-pulsar-utils_amd"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="u8", choices=["u8", "f32"])
    ap.add_argument("--chunks", type=int, default=4, help="full 2^18-sample chunks in the file")
    ap.add_argument("--search", default="f32,f64")
    args = ap.parse_args()
    import torch
    from pulsarutils import clean, sigproc, stats, synth
    from pulsarutils.configs import CONFIGS
    c4 = CONFIGS["C4"]
    half = c4.nsamples // 2
    ns = half * (args.chunks + 1)
    cfg = replace(c4, nsamples=ns)
    t0 = time.perf_counter()
    x = synth.rfi_filterbank_np(cfg, dtype=args.dtype)
    tmpd = tempfile.mkdtemp(dir=os.environ.get("TMPDIR", "/tmp"))
    fname = os.path.join(tmpd, f"c4_{args.dtype}.fil")
    # channel 0 = lowest frequency in the array; SIGPROC files usually run high -> low
    # (foff < 0): write the band reversed so search_by_chunks flips it back
    foff = -c4.bandwidth / c4.nchan
    fch1 = c4.start_freq + c4.bandwidth + 0.5 * foff
    sigproc.write_filterbank(fname, np.ascontiguousarray(x[::-1].T), fch1=fch1, foff=foff, tsamp=c4.tsamp)
    del x
    print(f"[pipe] wrote {fname} ({os.path.getsize(fname) / 1e9:.2f} GB) in {time.perf_counter() - t0:.1f}s",
          file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    tb = time.perf_counter()
    stats.get_bad_chans(fname)
    torch.cuda.synchronize()
    badchans_ms = (time.perf_counter() - tb) * 1e3
    chunk_length = (half + 0.5) * c4.tsamp
    for sd in args.search.split(","):
        for rep in range(2):  # the first pass builds the plan (host planner) and warms up
            prof = []
            torch.cuda.synchronize()
            ta = time.perf_counter()
            cands = clean.search_by_chunks(fname, chunk_length=chunk_length, dmmin=c4.dmmin, dmmax=c4.dmmax,
                                           save_candidates=False, snr_threshold=6, search_dtype=sd,
                                           profile=prof)
            torch.cuda.synchronize()
            total = (time.perf_counter() - ta) * 1e3
        # the production mode: no per-step synchronisation, chunk k+1 read + copied while
        # chunk k is cleaned and searched
        for rep in range(2):  # the first call warms the loader thread and the allocator
            torch.cuda.synchronize()
            ta = time.perf_counter()
            clean.search_by_chunks(fname, chunk_length=chunk_length, dmmin=c4.dmmin, dmmax=c4.dmmax,
                                   save_candidates=False, snr_threshold=6, search_dtype=sd)
            torch.cuda.synchronize()
            overlapped = (time.perf_counter() - ta) * 1e3
        keys = ("h2d", "transpose", "clean", "rebin", "cast", "search")
        full = [p for p in prof if p["nsamples"] == 2 * half]
        mean = {k: float(np.mean([p[k] for p in full])) for k in keys}
        rec = {"what": "search_by_chunks C4-sized SIGPROC file", "dtype": args.dtype, "search_dtype": sd,
               "nchan": c4.nchan, "chunk_samples": 2 * half, "file_samples": ns, "chunks": len(prof),
               "ndm": prof[0]["ndm"], "get_bad_chans_ms": round(badchans_ms, 2),
               "total_ms_synchronised": round(total, 2), "total_ms_overlapped": round(overlapped, 2),
               "file_GBps_overlapped": round(os.path.getsize(fname) / overlapped / 1e6, 2),
               "per_full_chunk_ms": {k: round(v, 3) for k, v in mean.items()},
               "per_full_chunk_total_ms": round(sum(mean.values()), 3),
               "best": max(((cd["snr"], cd["dm"]) for cd in cands), default=None),
               "note": "timings synchronised per step (no overlap between steps)"}
        print(json.dumps(rec), flush=True)
    os.remove(fname)


if __name__ == "__main__":
    main()
