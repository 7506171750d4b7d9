#!/bin/bash
# Round 4: channel mode (convert-once windows, float64 permlane epilogue, balanced DM
# tiles), packed width-4/8 float32 epilogue, certified float32 column means.  GPU suite,
# then A/B against the round-3 library (ab/lib_head.so) on one box: C1, C2 acc=f64, C5,
# C2, C3 625-trial shard; the bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r04c
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1 || exit $?
A=head B=new CFG=C1 TRIALS=0 ROUNDS=2 timeout -k 10 300 bash scripts/ab_lib.sh > $OUT/ab_c1.log 2>&1 || exit $?
A=head B=new CFG=C2 TRIALS=1000 ROUNDS=1 ACC=f64 timeout -k 10 400 bash scripts/ab_lib.sh > $OUT/ab_c2_f64.log 2>&1 || exit $?
A=head B=new CFG=C5 TRIALS=0 ROUNDS=2 timeout -k 10 300 bash scripts/ab_lib.sh > $OUT/ab_c5.log 2>&1 || exit $?
A=head B=new CFG=C2 TRIALS=1000 ROUNDS=2 timeout -k 10 300 bash scripts/ab_lib.sh > $OUT/ab_c2.log 2>&1 || exit $?
A=head B=new CFG=C3 TRIALS=625 ROUNDS=1 timeout -k 10 400 bash scripts/ab_lib.sh > $OUT/ab_c3_625.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py --steps 20 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err || exit $?
echo done > $OUT/status.txt
