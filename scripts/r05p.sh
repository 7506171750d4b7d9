#!/bin/bash
# Round 5: sum-loop window reads issued after each trial's adds (sumr) vs c3a.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05p
mkdir -p $O
export TMPDIR=/tmp
LIBS="c3a sumr" CFG=C2 TRIALS=1000 ROUNDS=2 bash scripts/ab_lib.sh > $O/ab_c2.log 2>&1 || exit $?
LIBS="c3a sumr" CFG=C3 TRIALS=625 ROUNDS=2 bash scripts/ab_lib.sh > $O/ab_c3_625.log 2>&1 || exit $?
LIBS="c3a sumr" CFG=C5 TRIALS=500 ROUNDS=2 bash scripts/ab_lib.sh > $O/ab_c5.log 2>&1 || exit $?
exit 0
