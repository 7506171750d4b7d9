#!/bin/bash
# Round 4: 8-bit slot build with four positions per lane (ds_read2_b32 + v_alignbyte_b32,
# packed 16-bit sums, 16-byte stores) vs the byte-per-lane integer build: u8 parity tests,
# then A/B at C3 (625 / 5000 trials).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r04q
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_dedisperse.py tests/test_gpu_degenerate.py tests/test_gpu_parallel.py -v -m gpu -x --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_dedisp.log 2>&1 || exit $?
LIBS="base x4" CFG=C3 TRIALS=625 ROUNDS=2 timeout -k 10 600 bash scripts/ab_lib.sh > $OUT/ab_c3_625.log 2>&1 || exit $?
LIBS="base x4" CFG=C3 TRIALS=0 ROUNDS=1 timeout -k 10 400 bash scripts/ab_lib.sh > $OUT/ab_c3_5000.log 2>&1 || exit $?
echo done > $OUT/status.txt
