#!/bin/bash
# DM-tile sorting only for DM-tile-major launches: head (247f70e) vs new4, C3 625 / 5000 and C5; parity subset.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r03l}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dedisperse.py tests/test_gpu_degenerate.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit $?
A=head B=new4 CFG=C3 TRIALS=625 ROUNDS=2 bash scripts/ab_lib.sh > $O/ab_c3_625.log 2>&1 || exit $?
A=head B=new4 CFG=C3 TRIALS=0 ROUNDS=1 bash scripts/ab_lib.sh > $O/ab_c3_5000.log 2>&1 || exit $?
A=head B=new4 CFG=C5 TRIALS=0 ROUNDS=2 bash scripts/ab_lib.sh > $O/ab_c5.log 2>&1 || exit $?
