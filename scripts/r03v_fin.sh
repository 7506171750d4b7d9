#!/bin/bash
# Finalize without memset / read-back copy: dedispersion GPU tests, step-overhead probe, bench lines C2/C5/C1.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03v
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/step_overhead.py C5 C1 C2 > $OUT/step_overhead.jsonl 2> $OUT/step_overhead.err || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-c3-strong > $OUT/bench.json 2> $OUT/bench.err || exit $?
timeout -k 10 200 python -u bench.py --config C5 --steps 50 --warmup 3 --no-cpu-baseline --no-clean --no-c3-strong > $OUT/c5.json 2> $OUT/c5.err || exit $?
timeout -k 10 200 python -u bench.py --config C1 --steps 50 --warmup 3 --no-cpu-baseline --no-clean --no-c3-strong > $OUT/c1.json 2> $OUT/c1.err || exit $?
echo done > $OUT/status.txt
