set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03b; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dedisperse.py tests/test_gpu_parallel.py tests/test_gpu_degenerate.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit $?
PU_AB="PU_ITEMS=1;PU_ITEMS=2;PU_ITEMS=4" timeout -k 10 300 python -u scripts/ab_env.py C2 3 > $O/ab_c2.log 2>&1 || exit $?
PU_AB="PU_ITEMS=1;PU_ITEMS=2;PU_ITEMS=4;PU_ITEMS=8" timeout -k 10 300 python -u scripts/ab_env.py C5 4 > $O/ab_c5.log 2>&1 || exit $?
PU_TRIALS=625 PU_AB="PU_ITEMS=1;PU_ITEMS=2;PU_ITEMS=4" timeout -k 10 300 python -u scripts/ab_env.py C3 2 > $O/ab_c3_625.log 2>&1 || exit $?
