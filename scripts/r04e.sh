#!/bin/bash
# Round 4: select build of 8-bit slots.  The new parity tests first, then the whole GPU
# suite, then A/B against the round-3 library at the C3 625-trial shard and 5000 trials.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r04e
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_dedisperse.py -k "select_build or u8_dma or c3_full" -v -m gpu -x --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_sel.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1 || exit $?
A=head B=new CFG=C3 TRIALS=625 ROUNDS=2 timeout -k 10 400 bash scripts/ab_lib.sh > $OUT/ab_c3_625.log 2>&1 || exit $?
A=head B=new CFG=C3 TRIALS=0 ROUNDS=1 timeout -k 10 400 bash scripts/ab_lib.sh > $OUT/ab_c3_5000.log 2>&1 || exit $?
echo done > $OUT/status.txt
A=new B=tail CFG=C2 TRIALS=1000 ROUNDS=2 timeout -k 10 300 bash scripts/ab_lib.sh > $OUT/ab_c2_tail.log 2>&1 || exit $?
A=new B=tail CFG=C5 TRIALS=0 ROUNDS=2 timeout -k 10 300 bash scripts/ab_lib.sh > $OUT/ab_c5_tail.log 2>&1 || exit $?
echo done2 > $OUT/status2.txt
