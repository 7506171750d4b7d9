#!/bin/bash
# Round 4: the C2-shaped near-constant float32 certification test.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r04n2
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_degenerate.py -k nearconst_f32_c2 -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/test.log 2>&1 || exit $?
echo done > $OUT/status.txt
