#!/bin/bash
# Workgroup shape wide vs tall at C2 / C3 625 / C3 5000 / C5 / C1-like, with the plans' cost-model inputs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r03n}; mkdir -p $O
PU_AB="PU_SUB_SHAPE=0;PU_SUB_SHAPE=2" timeout -k 10 300 python -u scripts/ab_env.py C2 3 > $O/ab_c2.log 2>&1 || exit $?
PU_AB="PU_SUB_SHAPE=0;PU_SUB_SHAPE=2" timeout -k 10 300 python -u scripts/ab_env.py C5 4 > $O/ab_c5.log 2>&1 || exit $?
PU_TRIALS=625 PU_AB="PU_SUB_SHAPE=0;PU_SUB_SHAPE=2" timeout -k 10 300 python -u scripts/ab_env.py C3 2 > $O/ab_c3_625.log 2>&1 || exit $?
PU_AB="PU_SUB_SHAPE=0;PU_SUB_SHAPE=2" timeout -k 10 300 python -u scripts/ab_env.py C4 4 > $O/ab_c4.log 2>&1 || exit $?
