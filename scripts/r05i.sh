#!/bin/bash
# Round 5: float64 kernel - u16 records, channel-pair reload parity: dedispersion GPU tests
# with the production build (pair), C2 float64 A/B (625 trials) of bf / u16 / pair.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -m gpu tests/test_gpu_dedisperse.py tests/test_gpu_degenerate.py tests/test_gpu_files.py > $O/tests.log 2>&1 || exit $?
LIBS="bf u16 pair" ACC=f64 CFG=C2 ROUNDS=2 bash scripts/ab_lib.sh > $O/ab_c2_f64.log 2>&1 || exit $?
LIBS="bf pair" ACC=f64 CFG=C5 TRIALS=500 ROUNDS=2 bash scripts/ab_lib.sh > $O/ab_c5_f64.log 2>&1 || exit $?
exit 0
