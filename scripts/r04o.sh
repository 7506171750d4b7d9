#!/bin/bash
# Round 4: masks with the host copy of [means | moments] prefetched: cleaning tests + bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r04o
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_clean.py -v -m gpu -x --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_clean.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-c3-strong --no-acc-f64 > $OUT/bench.json 2> $OUT/bench.err || exit $?
echo done > $OUT/status.txt
