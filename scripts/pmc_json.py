"""Per-launch HBM bytes of the dominant kernel -> <pmc dir>/pmc_<tag>.json, committed as
profiles/pmc_<tag>.json (bench.py reads it).

Usage: python scripts/pmc_json.py <pmc dir> <tag> <bench json> [kernel substring]

<pmc dir> holds the two rocprofv3 passes of one bench command: p1 (--pmc FETCH_SIZE)
and p2 (--pmc WRITE_SIZE), as scripts/r03_refresh.sh collects them.  The average over
the kernel's dispatches is corrected as /opt/skills/guides/MI355X_MICROARCH.md §HBM
prescribes for gfx950 (FETCH_SIZE x 2 for 16-B/lane streaming reads - the LDS-DMA
dwordx4 row loads here; WRITE_SIZE as is; KB = 1024 B).  The summary records the
SHA-256 of csrc/dedisperse.hip the library was built from, so bench.py only reports
the traffic against the same kernel source, and the kernel time of the bench line of
the same call (HIP events) for context.
"""
import csv
import glob
import hashlib
import json
import os
import sys

d, tag, bench = sys.argv[1], sys.argv[2], sys.argv[3]
pat = sys.argv[4] if len(sys.argv) > 4 else "dedisp_sub_kernel"
repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def avg(pass_dir, counter):
    vals, name = [], None
    for f in glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if pat in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals.append(float(r["Counter_Value"]))
                name = r["Kernel_Name"]
    if not vals:
        raise SystemExit(f"no {counter} rows for {pat} under {pass_dir}")
    return sum(vals) / len(vals), len(vals), name


fetch, nf, kname = avg(os.path.join(d, "p1"), "FETCH_SIZE")
write, nw, _ = avg(os.path.join(d, "p2"), "WRITE_SIZE")
line = json.loads(open(bench).read().strip().splitlines()[-1])
roof = line.get("roofline") or {}
src = hashlib.sha256(open(os.path.join(repo, "radio-pulsar-utils_amd", "csrc", "dedisperse.hip"), "rb").read()).hexdigest()
built = json.load(open(os.path.join(repo, "radio-pulsar-utils_amd", "pulsarutils", "_lib", "BUILD_INFO.json")))
assert built["sources"]["csrc/dedisperse.hip"] == src, "library not built from this dedisperse.hip"
out = {
    "kernel": kname,
    "config": line["config"]["workload"],
    "source": f"{d} (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, one pass each, {nf}/{nw} dispatches)",
    "fetch_size_kb_per_launch": fetch,
    "write_size_kb_per_launch": write,
    "correction": "MI355X_MICROARCH.md HBM: on gfx950 FETCH_SIZE reports half the bytes of 16-B/lane streaming "
                  "reads (LDS-DMA dwordx4 here) -> x2; WRITE_SIZE exact; KB = 1024 B",
    "hbm_bytes_per_launch": int(round(fetch * 2 * 1024 + write * 1024)),
    "compulsory_bytes_per_launch": int(roof.get("algorithmic_bytes_per_launch", 0)
                                       + 16 * 8 * line["config"]["trials_per_gpu"] * roof.get("time_tiles", 0)),
    "kernel_ms_at_collection": roof.get("kernel_ms"),
    "kernel_ms_source": f"{bench} roofline.kernel_ms (same build, HIP events)",
    "dedisperse_hip_sha256": src,
}
out["traffic_over_compulsory"] = round(out["hbm_bytes_per_launch"] / max(1, out["compulsory_bytes_per_launch"]), 3)
json.dump(out, open(os.path.join(d, f"pmc_{tag}.json"), "w"), indent=1)  # copied into profiles/ after the call
print(json.dumps(out, indent=1))
