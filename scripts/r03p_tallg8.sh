#!/bin/bash
# Tall shape with G = 8: C2 (f32) and C3 625 / 5000 (u8) against the defaults.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r03p}; mkdir -p $O
PU_AB="PU_DUMMY=0;PU_SUB_SHAPE=2,PU_GROUP=8" timeout -k 10 300 python -u scripts/ab_env.py C2 3 > $O/ab_c2.log 2>&1 || exit $?
PU_TRIALS=625 PU_AB="PU_DUMMY=0;PU_SUB_SHAPE=2,PU_GROUP=8" timeout -k 10 300 python -u scripts/ab_env.py C3 2 > $O/ab_c3_625.log 2>&1 || exit $?
PU_AB="PU_DUMMY=0;PU_SUB_SHAPE=2,PU_GROUP=8" timeout -k 10 300 python -u scripts/ab_env.py C3 1 > $O/ab_c3_5000.log 2>&1 || exit $?
