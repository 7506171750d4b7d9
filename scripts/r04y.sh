#!/bin/bash
# Round 4: quad Gaussian workgroup size A/B (64 / 128 / 256 threads, 4 outputs each) on the
# diagnostic library: the Gaussian tests, then warm kernel stats of the f32 cleaning bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r04y
mkdir -p $OUT
export PULSARUTILS_HIP_LIB=$PWD/radio-pulsar-utils_amd/pulsarutils/_lib/libpulsarutils_hip_stamps.so
for T in 256 128; do
  PU_GAUSS_THREADS=$T timeout -k 10 200 python -u -m pytest tests/test_gpu_clean.py -k gaussian -q -m gpu -x --timeout 100 --timeout-method thread -p no:cacheprovider > $OUT/tests_$T.log 2>&1 || exit $?
  PU_GAUSS_THREADS=$T timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$T -o run -- python3 scripts/bench_clean.py --dtype f32 --steps 10 > $OUT/bench_$T.log 2>&1 || exit $?
  python3 scripts/warm_stats.py $OUT/prof_$T --skip 1 > $OUT/warm_$T.csv || exit $?
done
echo done > $OUT/status.txt
