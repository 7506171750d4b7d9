#!/bin/bash
# Epilogue rewrite: dedispersion parity tests + library A/B (ab/lib_head.so vs ab/lib_new.so).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r03h}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dedisperse.py tests/test_gpu_parallel.py tests/test_gpu_degenerate.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit $?
A=head B=new CFG=C2 TRIALS=0 ROUNDS=2 bash scripts/ab_lib.sh > $O/ab_c2.log 2>&1 || exit $?
A=head B=new CFG=C5 TRIALS=0 ROUNDS=2 PU_DT_MAJOR=0 bash scripts/ab_lib.sh > $O/ab_c5.log 2>&1 || exit $?
A=head B=new CFG=C3 TRIALS=625 ROUNDS=2 bash scripts/ab_lib.sh > $O/ab_c3_625.log 2>&1 || exit $?
