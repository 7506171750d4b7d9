#!/bin/bash
# Round 4: C1 channel-mode LDS budget (channels per step) sweep, one process.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r04k
mkdir -p $OUT
PU_SWEEP="1:64,1:80,1:48,1:32" PU_ROUNDS=3 timeout -k 10 200 python -u scripts/sweep.py C1 > $OUT/sweep_c1_budget.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
echo done > $OUT/status.txt
