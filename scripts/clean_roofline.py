"""Per-kernel HBM roofline of the cleaning pass from a rocprofv3 kernel-stats CSV.

Usage: python scripts/clean_roofline.py <kernel_stats.csv> <f32|u8> [nchan n]
Algorithmic bytes per launch (C4 shape by default, 1024 x 2^18):
  rowsum_chunk_kernel  nchan*n*b_in           (one read of the plane)
  colmean_kernel       nchan*n*b_in + 8n      (plane read, column means written)
  apply_kernel         nchan*n*(b_in+8) + 24n (plane read, float64 plane written,
                                               factor read, column means written)
Other kernels are O(n) or O(nchan) and are listed by time only.
"""
import csv
import json
import sys

HBM_PEAK_GBPS = 8000.0

path, dt = sys.argv[1], sys.argv[2]
nchan, n = (int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else (1024, 1 << 18)
b_in = {"u8": 1, "f32": 4, "f64": 8}[dt]
plane = nchan * n * b_in
alg = {
    "rowsum_chunk_kernel": plane,
    "colmean_kernel": plane + 8 * n,
    "apply_kernel": nchan * n * (b_in + 8) + 24 * n,
}
with open(path) as f:
    rows = list(csv.DictReader(f))
for r in rows:
    name = r["Name"]
    base = name.replace("void ", "").replace("(anonymous namespace)::", "").split("<")[0].split("(")[0].strip()
    avg_ns = float(r["AverageNs"])
    rec = {"kernel": name[:80], "calls": int(r["Calls"]), "avg_us": round(avg_ns / 1e3, 2)}
    if base in alg:
        gbps = alg[base] / avg_ns
        rec.update(alg_bytes=alg[base], GBps=round(gbps, 1), hbm_frac=round(gbps / HBM_PEAK_GBPS, 3))
    print(json.dumps(rec))
