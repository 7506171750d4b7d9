set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/k8
mkdir -p $OUT
A=head B=k8 CFG=C2 TRIALS=0 ROUNDS=2 ACC=f64 timeout -k 10 500 bash scripts/ab_lib.sh > $OUT/ab_c2_f64.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_dedisperse.py tests/test_gpu_degenerate.py -v -x -k "f64 or C1 or acc or reference or plane or degenerate or nan or tie or const" --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || exit $?
echo done
