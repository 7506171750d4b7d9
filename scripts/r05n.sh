#!/bin/bash
# Round 5: median passes select in their last workgroup - cleaning tests, light-curve chain
# timing with per-repetition bit checks, per-kernel trace of the cleaning steps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05n
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_clean.py > $O/tests_clean.log 2>&1 || exit $?
timeout -k 10 300 python3 -u scripts/bench_lc.py --checks 30 > $O/lc.log 2>&1 || exit $?
for dt in f32 u8; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_clean_$dt -o run -- \
    python3 scripts/bench_clean.py --dtype $dt --steps 10 --warmup 2 > $O/prof_clean_$dt.log 2>&1 || exit $?
done
exit 0
