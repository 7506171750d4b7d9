#!/bin/bash
# Round 5: diagnose the r05e abort in test_clean_ragged - serialized kernels, no capture.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05f
mkdir -p $O
export TMPDIR=/tmp
AMD_SERIALIZE_KERNEL=3 timeout -k 10 240 python -u -m pytest -x -s -v --timeout 200 --timeout-method thread \
  -p no:cacheprovider tests/test_gpu_clean.py -k "ragged or light_curve" > $O/tests_ragged.log 2>&1 || exit $?
exit 0
