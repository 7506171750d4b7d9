"""SQ / GRBM counters of the dominant kernel per dispatch -> <dir>/sq_<tag>.json, committed as
profiles/sq_<tag>.json (bench.py reads it for roofline.lds_cycle_frac).

Usage: python scripts/sq_json.py <pmc dir> <tag> <bench json> [kernel substring] [source file]

<pmc dir> holds one rocprofv3 pass (--pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS
SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE) of one bench command.
Per dispatch (the average over the kernel's dispatches): cycles = GRBM_GUI_ACTIVE / 8 (the
counter sums the 8 XCDs, MI355X_MICROARCH.md DVFS note); lds_cycle_frac = SQ_LDS_IDX_ACTIVE
(LDS-array cycles, MI355X_MICROARCH.md §LDS) / (256 CUs x cycles); the instruction rates per CU
and cycle; bank-conflict cycles / LDS-array cycles.  The summary records the SHA-256 of the
kernel's source file, so bench.py reports it only against the same source.
"""
import csv
import glob
import hashlib
import json
import os
import sys

d, tag, bench = sys.argv[1], sys.argv[2], sys.argv[3]
pat = sys.argv[4] if len(sys.argv) > 4 else "dedisp_sub_kernel"
srcfile = sys.argv[5] if len(sys.argv) > 5 else "csrc/dedisperse.hip"
repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CUS = 256

vals, name = {}, None
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
            name = r["Kernel_Name"]
if not vals:
    raise SystemExit(f"no counter rows for {pat} under {d}")
avg = {k: sum(v) / len(v) for k, v in vals.items()}
ndisp = min(len(v) for v in vals.values())
line = json.loads(open(bench).read().strip().splitlines()[-1])
src = hashlib.sha256(open(os.path.join(repo, "radio-pulsar-utils_amd", srcfile), "rb").read()).hexdigest()
built = json.load(open(os.path.join(repo, "radio-pulsar-utils_amd", "pulsarutils", "_lib", "BUILD_INFO.json")))
assert built["sources"][srcfile] == src, f"library not built from this {srcfile}"
cyc = avg["GRBM_GUI_ACTIVE"] / 8.0
cu_cyc = CUS * cyc
out = {"kernel": name, "config": line["config"]["workload"],
       "source": f"{d} (rocprofv3 --pmc, one pass, {ndisp} dispatches)",
       "counters_per_dispatch": {k: round(v, 1) for k, v in sorted(avg.items())},
       "cycles_per_dispatch": round(cyc, 1),
       "lds_cycle_frac": round(avg["SQ_LDS_IDX_ACTIVE"] / cu_cyc, 4) if "SQ_LDS_IDX_ACTIVE" in avg else None,
       "lds_bank_conflict_frac": (round(avg["SQ_LDS_BANK_CONFLICT"] / max(1.0, avg["SQ_LDS_IDX_ACTIVE"]), 4)
                                  if "SQ_LDS_BANK_CONFLICT" in avg and "SQ_LDS_IDX_ACTIVE" in avg else None),
       "per_cu_cycle": {k: round(avg[k] / cu_cyc, 4) for k in ("SQ_INSTS_LDS", "SQ_INSTS_VALU", "SQ_INSTS_SALU")
                        if k in avg},
       "what": "lds_cycle_frac = SQ_LDS_IDX_ACTIVE / (256 CUs x GRBM_GUI_ACTIVE / 8): the share of the LDS "
               "arrays' cycles the kernel kept busy (MI355X_MICROARCH.md §LDS: SQ_LDS_IDX_ACTIVE = all "
               "LDS-array cycles); per_cu_cycle = wave-instructions per CU and cycle",
       "kernel_ms_at_collection": (line.get("roofline") or {}).get("kernel_ms"),
       "source_file": srcfile, "source_sha256": src}
json.dump(out, open(os.path.join(d, f"sq_{tag}.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
