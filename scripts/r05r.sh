#!/bin/bash
# Round 5: the subband sum as a state machine over new windows - dedispersion GPU tests
# (production build: structurizer flag, sum_fsm off by default; the tests build FSM plans
# explicitly), then A/B c3a (round-5 build code, no flag) / flag (flag only) / fsm (FSM on
# by default) at C2, C3 625, C5.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05r
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -m gpu tests/test_gpu_dedisperse.py > $O/tests.log 2>&1 || exit $?
LIBS="c3a flag fsm" CFG=C2 TRIALS=1000 ROUNDS=2 bash scripts/ab_lib.sh > $O/ab_c2.log 2>&1 || exit $?
LIBS="c3a flag fsm" CFG=C3 TRIALS=625 ROUNDS=2 bash scripts/ab_lib.sh > $O/ab_c3_625.log 2>&1 || exit $?
LIBS="c3a flag fsm" CFG=C5 TRIALS=500 ROUNDS=2 bash scripts/ab_lib.sh > $O/ab_c5.log 2>&1 || exit $?
exit 0
