#!/bin/bash
# Epilogue lane masks after the loop: dedispersion parity tests + A/B (lib_new vs lib_new2), median grid sweep.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r03i}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dedisperse.py tests/test_gpu_degenerate.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit $?
A=new B=new2 CFG=C2 TRIALS=0 ROUNDS=2 bash scripts/ab_lib.sh > $O/ab_c2.log 2>&1 || exit $?
A=new B=new2 CFG=C5 TRIALS=0 ROUNDS=2 bash scripts/ab_lib.sh > $O/ab_c5.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/sweep_clean.py --kernels median > $O/sweep_median.jsonl 2> $O/sweep.err || exit $?
