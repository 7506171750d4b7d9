#!/bin/bash
# Round 5: float64 u16 records / channel-pair parity A/B + dedispersion tests (production =
# c3a: also the build's slot-record ping-pong and peeled first pass); C3 625 / C2 / C5 A/B
# pair (previous build code) vs c3a.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05j
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -m gpu tests/test_gpu_dedisperse.py tests/test_gpu_degenerate.py tests/test_gpu_files.py > $O/tests.log 2>&1 || exit $?
LIBS="bf u16 pair" ACC=f64 CFG=C2 ROUNDS=2 bash scripts/ab_lib.sh > $O/ab_c2_f64.log 2>&1 || exit $?
LIBS="pair c3a" CFG=C3 TRIALS=625 ROUNDS=2 bash scripts/ab_lib.sh > $O/ab_c3_625.log 2>&1 || exit $?
LIBS="pair c3a" CFG=C2 TRIALS=1000 ROUNDS=2 bash scripts/ab_lib.sh > $O/ab_c2.log 2>&1 || exit $?
LIBS="pair c3a" CFG=C5 TRIALS=500 ROUNDS=2 bash scripts/ab_lib.sh > $O/ab_c5.log 2>&1 || exit $?
exit 0
