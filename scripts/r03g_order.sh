#!/bin/bash
# Item order (DM-tile major, longest first) A/B + dedispersion parity tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r03g}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dedisperse.py tests/test_gpu_parallel.py tests/test_gpu_degenerate.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit $?
PU_AB="PU_DT_MAJOR=0;PU_DT_MAJOR=1" timeout -k 10 300 python -u scripts/ab_env.py C5 5 > $O/ab_c5.log 2>&1 || exit $?
PU_AB="PU_DT_MAJOR=0;PU_DT_MAJOR=1" timeout -k 10 300 python -u scripts/ab_env.py C2 3 > $O/ab_c2.log 2>&1 || exit $?
PU_AB="PU_DT_MAJOR=0;PU_DT_MAJOR=1" timeout -k 10 300 python -u scripts/ab_env.py C1 5 > $O/ab_c1.log 2>&1 || exit $?
