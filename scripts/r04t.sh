#!/bin/bash
# Round 4: planner choices re-checked at HEAD (group size x workgroup shape), one process per
# config: C2 and the C3 625-trial shard.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r04t
mkdir -p $OUT
PU_SWEEP="4:0:2,4:0:0,8:0:2" PU_ROUNDS=2 timeout -k 10 300 python -u scripts/sweep.py C2 > $OUT/sweep_c2.log 2>&1 || exit $?
PU_SWEEP="8:0:2,8:0:0,4:0:2" PU_ROUNDS=2 PU_TRIALS=625 timeout -k 10 400 python -u scripts/sweep.py C3 > $OUT/sweep_c3_625.log 2>&1 || exit $?
echo done > $OUT/status.txt
