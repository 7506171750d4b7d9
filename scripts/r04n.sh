#!/bin/bash
# Round 4: one-pass channel statistics (pu_row_moments + certified variability): cleaning
# parity tests, the whole GPU suite, and a bench line (masks now one read pass).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r04n
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_clean.py -v -m gpu -x --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_clean.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-c3-strong > $OUT/bench.json 2> $OUT/bench.err || exit $?
echo done > $OUT/status.txt
