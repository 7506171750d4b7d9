#!/bin/bash
# Per-slot alignment-copy sizes for 16-bit slots + the refitted stage term (ab/lib_slot.so)
# against the previous library (ab/lib_head.so): the default plans at C3 625 / 5000 trials
# and the plans chosen at C2 / C5 / C3 (scripts/plan_costs.py), then the subband GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/slot5
mkdir -p $OUT
timeout -k 10 300 python3 -u scripts/plan_costs.py > $OUT/plans.jsonl 2> $OUT/plans.err || exit $?
A=head B=slot CFG=C3 TRIALS=625 ROUNDS=2 timeout -k 10 400 bash scripts/ab_lib.sh > $OUT/ab_C3_625.log 2>&1 || exit $?
A=head B=slot CFG=C3 TRIALS=0 ROUNDS=2 timeout -k 10 500 bash scripts/ab_lib.sh > $OUT/ab_C3_5000.log 2>&1 || exit $?
timeout -k 10 700 python -u -m pytest tests/test_gpu_dedisperse.py -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || exit $?
echo done
