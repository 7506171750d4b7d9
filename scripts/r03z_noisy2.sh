#!/bin/bash
# Rank-selection medians in the noisy-channel kernel: cleaning GPU tests, bench, rocprof of the bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r03z}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_clean.py tests/test_gpu_files.py -v -m gpu -x --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_clean.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-c3-strong > $OUT/bench.json 2> $OUT/bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-c3-strong > $OUT/prof.log 2>&1 || exit $?
echo done > $OUT/status.txt
