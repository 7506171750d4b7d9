#!/bin/bash
# Round 5: the pair shape (8 waves x 16 trials, two workgroups per CU) against the planner's
# choices at C5, C3 625 and C2 (scripts/sweep.py, one process per config).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r05u}
mkdir -p $O
export TMPDIR=/tmp
PU_ROUNDS=3 PU_SWEEP="4:160:2,4:160:0,4:80:1,2:80:1,8:80:1" timeout -k 10 300 python -u scripts/sweep.py C5 > $O/sweep_c5.log 2>&1 || exit $?
PU_ROUNDS=2 PU_TRIALS=625 PU_SWEEP="8:160:2,8:80:1,4:80:1" timeout -k 10 400 python -u scripts/sweep.py C3 > $O/sweep_c3_625.log 2>&1 || exit $?
PU_ROUNDS=2 PU_SWEEP="4:160:2,4:80:1,2:80:1" timeout -k 10 300 python -u scripts/sweep.py C2 > $O/sweep_c2.log 2>&1 || exit $?
exit 0
