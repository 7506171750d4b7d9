#!/bin/bash
# Step-overhead probe (C5 / C1 / C2) and the column-mean batch sweep (C4).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03u
mkdir -p $OUT
timeout -k 10 300 python -u scripts/step_overhead.py C5 C1 C2 > $OUT/step_overhead.jsonl 2> $OUT/step_overhead.err || exit $?
timeout -k 10 300 python -u scripts/sweep_clean.py --kernels col_means,median --steps 20 > $OUT/sweep_colmean.jsonl 2> $OUT/sweep_colmean.err || exit $?
echo done > $OUT/status.txt
