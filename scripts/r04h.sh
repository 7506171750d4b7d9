#!/bin/bash
# Round 4: GPU suite after removing the select build (kept as an archived diff) and with the
# device-side exact cut_outliers path; then the apply-pass store A/B (scripts/r04g.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r04h
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_clean.py -v -m gpu -x --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_clean.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1 || exit $?
bash scripts/r04g.sh || exit $?
echo done > $OUT/status.txt
