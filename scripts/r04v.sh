#!/bin/bash
# Round 4: C5 step timeline (kernel trace of bench.py --config C5) to see where the
# 0.06 ms between the kernel and the step goes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r04v
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_c5 -o run -- python3 bench.py --config C5 --steps 20 --warmup 3 --no-cpu-baseline --no-clean --no-c3-strong --no-acc-f64 > $OUT/bench_c5.json 2> $OUT/bench_c5.err || exit $?
echo done > $OUT/status.txt
