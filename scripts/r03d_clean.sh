#!/bin/bash
# Cleaning: GPU tests of the cleaning path + median / renormalize timings; C5 group-size A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r03d}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_clean.py tests/test_gpu_files.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/sweep_clean.py --kernels median,renormalize_device > $O/sweep.jsonl 2> $O/sweep.err || exit $?
PU_MEDIAN_COOP=0 timeout -k 10 300 python -u scripts/sweep_clean.py --kernels median > $O/sweep_nocoop.jsonl 2>> $O/sweep.err || exit $?
PU_AB="PU_GROUP=4;PU_GROUP=2;PU_GROUP=8" timeout -k 10 300 python -u scripts/ab_env.py C5 3 > $O/ab_c5_group.log 2>&1 || exit $?
