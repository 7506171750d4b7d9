#!/bin/bash
# Round 4: three bench processes back to back at HEAD (run-to-run spread; masks now
# recompute the channel means every step).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r04m
mkdir -p $OUT
timeout -k 10 500 python -u bench.py > $OUT/bench_1.json 2> $OUT/bench_1.err || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-c3-strong > $OUT/bench_2.json 2> $OUT/bench_2.err || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-c3-strong > $OUT/bench_3.json 2> $OUT/bench_3.err || exit $?
echo done > $OUT/status.txt
