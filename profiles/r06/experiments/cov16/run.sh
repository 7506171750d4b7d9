set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/cov16
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests/test_gpu_dedisperse.py -v -x -k "u8 or slot16 or c3" --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || exit $?
A=head B=cov16 CFG=C3 TRIALS=625 ROUNDS=2 bash scripts/ab_lib.sh > $OUT/ab_c3_625.log 2>&1 || exit $?
A=head B=cov16 CFG=C3 TRIALS=0 ROUNDS=2 bash scripts/ab_lib.sh > $OUT/ab_c3_5000.log 2>&1 || exit $?
echo done
