#!/bin/bash
# Round 4 final: the refresh (tests, bench, warm rocprof, PMC C2), then a C5 shape check.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
PMC="C2" TAG=r04_final bash scripts/r04_refresh.sh || exit $?
PU_SWEEP="4:0:2,4:0:0" PU_ROUNDS=3 timeout -k 10 200 python -u scripts/sweep.py C5 > gpurun_out/r04_final/sweep_c5_shape.log 2>&1 || exit $?
