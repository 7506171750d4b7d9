"""Per-kernel duration statistics from a rocprofv3 kernel trace, cold launches excluded.

    python scripts/warm_stats.py <dir with *_kernel_trace.csv> [--skip K] > warm_stats.csv

rocprofv3 --stats averages every launch, the first (cold: code object load, caches and
TLB empty) included.  This drops the first K launches of each kernel (default 1: the
bench's warm-up runs every kernel at least once before the timed steps) and prints
Name, Calls, AverageNs, MedianNs, MinNs, MaxNs, StdDevNs, SkippedCalls, ColdFirstNs (the median
beside the mean: one slow launch on a shared box moves the mean, not the median).
"""
import csv
import glob
import math
import os
import sys


def main():
    args = sys.argv[1:]
    skip = 1
    if "--skip" in args:
        i = args.index("--skip")
        skip = int(args[i + 1])
        del args[i:i + 2]
    paths = glob.glob(os.path.join(args[0], "**", "*kernel_trace.csv"), recursive=True)
    if not paths:
        sys.exit(f"no *kernel_trace.csv under {args[0]}")
    launches = {}
    for path in paths:
        with open(path, newline="") as f:
            for r in csv.DictReader(f):
                name = r.get("Kernel_Name") or r.get("KernelName") or r["Name"]
                t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
                launches.setdefault(name, []).append((t0, t1 - t0))
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "AverageNs", "MedianNs", "MinNs", "MaxNs", "StdDevNs", "SkippedCalls", "ColdFirstNs"])
    rows = []
    for name, ls in launches.items():
        ls.sort()
        warm = [d for _, d in ls[skip:]] or [d for _, d in ls]
        avg = sum(warm) / len(warm)
        sd = math.sqrt(sum((d - avg) ** 2 for d in warm) / len(warm))
        srt = sorted(warm)
        m = len(srt) // 2
        med = srt[m] if len(srt) % 2 else (srt[m - 1] + srt[m]) / 2
        rows.append((sum(warm), [name, len(warm), f"{avg:.1f}", f"{med:.1f}", min(warm), max(warm), f"{sd:.1f}",
                                 len(ls) - len(warm), ls[0][1]]))
    for _, row in sorted(rows, key=lambda x: -x[0]):
        w.writerow(row)


if __name__ == "__main__":
    main()
