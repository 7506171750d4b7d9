#!/bin/bash
# Round 5: device variability certification (one read-back for both channel masks) -
# cleaning GPU tests, then the default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05k
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_clean.py > $O/tests_clean.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
exit 0
