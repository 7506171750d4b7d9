#!/bin/bash
# C5 workgroup shape at HEAD (wide vs tall, both item orders) + cleaning ceilings.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r03m}; mkdir -p $O
PU_AB="PU_SUB_SHAPE=0;PU_SUB_SHAPE=2;PU_SUB_SHAPE=2,PU_DT_MAJOR=0;PU_SUB_SHAPE=0,PU_DT_MAJOR=0" timeout -k 10 300 python -u scripts/ab_env.py C5 4 > $O/ab_c5_shape.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/sweep_clean.py --kernels ceiling --dtype f32 > $O/ceiling.jsonl 2> $O/ceiling.err || exit $?
