#!/bin/bash
# Diagnostics of the tall plans at HEAD (diagnostic build only): phase stamps for C2 / C5
# and the C2 ablation (phases skipped: results invalid, times only).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03_diag
mkdir -p $OUT
timeout -k 10 200 python -u scripts/stamps.py C2 5 > $OUT/stamps_c2.txt 2>&1 || exit $?
timeout -k 10 200 python -u scripts/stamps.py C5 20 > $OUT/stamps_c5.txt 2>&1 || exit $?
PU_SWEEP=4:160:2 CFG=C2 SKIPS="0 1 2 4 8 15" timeout -k 10 900 bash scripts/ablate.sh > $OUT/ablate_c2_tall.log 2>&1 || exit $?
echo done > $OUT/status.txt
