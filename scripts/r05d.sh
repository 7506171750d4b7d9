#!/bin/bash
# Round 5: float64 kernel with 16 waves x 4 trials (lib new2) and the one-launch light-curve
# factor - parity (dedispersion, degenerate and cleaning GPU tests), A/B of the float64 search
# at C2 / C1 against round 4 (r4) and the 8 x 8 state machine (new), the bench's clean block.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05d
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_dedisperse.py tests/test_gpu_degenerate.py tests/test_gpu_clean.py > $O/tests.log 2>&1 || exit $?
LIBS="r4 new new2" ACC=f64 CFG=C2 TRIALS=0 ROUNDS=2 bash scripts/ab_lib.sh > $O/ab_c2_f64.log 2>&1 || exit $?
LIBS="r4 new new2" ACC=f64 CFG=C1 TRIALS=0 ROUNDS=2 bash scripts/ab_lib.sh > $O/ab_c1_f64.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-c3-strong > $O/bench.json 2> $O/bench.err || exit $?
exit 0
