#!/bin/bash
# dwordx3 LDS-DMA tail piece: dedispersion parity + A/B (lib_recs = previous HEAD, lib_dx3).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r03t}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dedisperse.py tests/test_gpu_parallel.py tests/test_gpu_degenerate.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit $?
A=recs B=dx3 CFG=C2 TRIALS=0 ROUNDS=3 bash scripts/ab_lib.sh > $O/ab_c2.log 2>&1 || exit $?
A=recs B=dx3 CFG=C5 TRIALS=0 ROUNDS=2 bash scripts/ab_lib.sh > $O/ab_c5.log 2>&1 || exit $?
