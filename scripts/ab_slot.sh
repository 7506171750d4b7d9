#!/bin/bash
# A/B of per-slot float32 copies rounded to whole build passes (ab/lib_slot.so) against the
# previous library (ab/lib_head.so) on C5, C2 and C4's search, then the subband GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/slot6
mkdir -p $OUT
A=head B=slot CFG=C5 TRIALS=0 ROUNDS=3 timeout -k 10 300 bash scripts/ab_lib.sh > $OUT/ab_C5.log 2>&1 || exit $?
A=head B=slot CFG=C2 TRIALS=0 ROUNDS=2 timeout -k 10 300 bash scripts/ab_lib.sh > $OUT/ab_C2.log 2>&1 || exit $?
A=head B=slot CFG=C4 TRIALS=0 ROUNDS=2 timeout -k 10 300 bash scripts/ab_lib.sh > $OUT/ab_C4.log 2>&1 || exit $?
timeout -k 10 700 python -u -m pytest tests/test_gpu_dedisperse.py -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || exit $?
echo done
