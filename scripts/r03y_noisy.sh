#!/bin/bash
# Device noisy-channel decision: cleaning GPU tests (goldens + the new parity tests), then the bench's clean section.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03y
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_clean.py tests/test_gpu_files.py -v -m gpu -x --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_clean.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-c3-strong > $OUT/bench.json 2> $OUT/bench.err || exit $?
echo done > $OUT/status.txt
