set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/ex
mkdir -p $OUT
timeout -k 10 300 python3 -u scripts/recheck_cost.py > $OUT/recheck.json 2> $OUT/recheck.err || exit $?
timeout -k 10 900 python -u -m pytest tests/test_gpu_parallel.py tests/test_gpu_degenerate.py tests/test_gpu_multirank.py -v -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || exit $?
echo done
