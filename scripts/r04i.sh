#!/bin/bash
# Round 4: 8-bit slot build summing bytes as integers (v_add3_u32, one convert) vs HEAD's
# convert-and-add per byte: u8 parity tests, then A/B at C3 (625 / 5000 trials) and C4's
# 100-trial u8 search (interleaved processes, one box).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r04i
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_dedisperse.py tests/test_gpu_degenerate.py -v -m gpu -x --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_dedisp.log 2>&1 || exit $?
LIBS="base new pairs" CFG=C3 TRIALS=625 ROUNDS=2 timeout -k 10 600 bash scripts/ab_lib.sh > $OUT/ab_c3_625.log 2>&1 || exit $?
LIBS="base new pairs" CFG=C3 TRIALS=0 ROUNDS=1 timeout -k 10 400 bash scripts/ab_lib.sh > $OUT/ab_c3_5000.log 2>&1 || exit $?
echo done > $OUT/status.txt
