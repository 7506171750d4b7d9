#!/bin/bash
# Round 4 closing check at HEAD: every GPU test and smoke on the production library.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r04z
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.txt 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-c3-strong > $OUT/bench.json 2> $OUT/bench.err || exit $?
echo done > $OUT/status.txt
