#!/bin/bash
# Run-to-run spread of the headline bench line on one box (three separate processes).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03_spread
mkdir -p $OUT
for r in 1 2 3; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-c3-strong > $OUT/bench_$r.json 2> $OUT/bench_$r.err || exit $?
done
echo done > $OUT/status.txt
