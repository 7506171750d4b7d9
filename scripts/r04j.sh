#!/bin/bash
# Round 4: paired 8-bit row DMA with each half-wave predicated to its row's own cover (the
# per-row path's bytes, half the instructions) vs HEAD: u8 parity tests, A/B at C3.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r04j
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_dedisperse.py tests/test_gpu_degenerate.py -v -m gpu -x --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_dedisp.log 2>&1 || exit $?
LIBS="base pairs2" CFG=C3 TRIALS=625 ROUNDS=2 timeout -k 10 600 bash scripts/ab_lib.sh > $OUT/ab_c3_625.log 2>&1 || exit $?
LIBS="base pairs2" CFG=C3 TRIALS=0 ROUNDS=1 timeout -k 10 400 bash scripts/ab_lib.sh > $OUT/ab_c3_5000.log 2>&1 || exit $?
echo done > $OUT/status.txt
