"""Average PMC counters per kernel from a pmc_sweep.sh / pmc.sh output directory.

Usage: python scripts/pmc_summary.py gpurun_out/<tag> [kernel-substring]
"""
import collections
import csv
import glob
import sys

root = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "dedisp"
vals = collections.defaultdict(list)
for f in sorted(glob.glob(f"{root}/p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in vals.items():
    print(f"{k:24s} {sum(v) / len(v):.4e}  (n={len(v)})")
