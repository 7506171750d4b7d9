#!/bin/bash
# Round 5: barrier-light sorts in the channel-mask kernels - cleaning tests, per-kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05m
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_clean.py > $O/tests_clean.log 2>&1 || exit $?
for dt in f32 u8; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_clean_$dt -o run -- \
    python3 scripts/bench_clean.py --dtype $dt --steps 10 --warmup 2 > $O/prof_clean_$dt.log 2>&1 || exit $?
done
exit 0
