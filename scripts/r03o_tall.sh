#!/bin/bash
# Tall shape by the cost model (float32): full GPU suite, default vs forced wide, bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r03o}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -v -m gpu -x --timeout 400 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || exit $?
PU_AB="PU_DUMMY=0;PU_SUB_SHAPE=0" timeout -k 10 300 python -u scripts/ab_env.py C2 3 > $O/ab_c2.log 2>&1 || exit $?
PU_AB="PU_DUMMY=0;PU_SUB_SHAPE=0" timeout -k 10 300 python -u scripts/ab_env.py C5 4 > $O/ab_c5.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py --steps 20 --warmup 2 --no-c3-strong > $O/bench.json 2> $O/bench.err || exit $?
