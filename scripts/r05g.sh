#!/bin/bash
# Round 5: light-curve chain variants (atomics-only grid barrier, fenced barrier, split
# launches) with a bit check per repetition; cleaning tests; cleaning bench after the
# apply-kernel revert.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05g
mkdir -p $O
export TMPDIR=/tmp
STAMPLIB=radio-pulsar-utils_amd/pulsarutils/_lib/libpulsarutils_hip_stamps.so
timeout -k 10 300 python3 -u scripts/bench_lc.py --checks 30 > $O/lc_default.log 2>&1 || exit $?
PULSARUTILS_HIP_LIB=$STAMPLIB PU_LC_FENCED=1 timeout -k 10 300 python3 -u scripts/bench_lc.py --checks 5 > $O/lc_fenced.log 2>&1 || exit $?
PULSARUTILS_HIP_LIB=$STAMPLIB PU_LC_SPLIT=1 timeout -k 10 300 python3 -u scripts/bench_lc.py --checks 5 > $O/lc_split.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_clean.py > $O/tests_clean.log 2>&1 || exit $?
for dt in f32 u8; do
  timeout -k 10 300 python3 scripts/bench_clean.py --dtype $dt --steps 20 --warmup 3 >> $O/bench_clean.log 2>&1 || exit $?
done
for dt in f32 u8; do
  PULSARUTILS_HIP_LIB=$STAMPLIB PU_LC_SPLIT=1 timeout -k 10 300 python3 scripts/bench_clean.py --dtype $dt --steps 20 --warmup 3 >> $O/bench_clean_split.log 2>&1 || exit $?
done
exit 0
