#!/bin/bash
# Round 4: cleaning-pass kernels (certified float32 column means, 3-launch median,
# 16-byte non-temporal stores in the 8-bit apply pass).  Cleaning GPU tests, then per-kernel
# rocprofv3 stats of the C4 cleaning bench with the round-3 library and with the new one.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r04d
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_clean.py tests/test_gpu_files.py -v -m gpu -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_clean.log 2>&1 || exit $?
for lib in head new; do
  for dt in f32 u8; do
    PULSARUTILS_HIP_LIB=ab/lib_$lib.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_${lib}_$dt -o run -- python3 scripts/bench_clean.py --dtype $dt --steps 10 > $OUT/clean_${lib}_$dt.log 2>&1 || exit $?
  done
done
for rep in 1 2; do
  for lib in head new; do
    for dt in f32 u8; do
      PULSARUTILS_HIP_LIB=ab/lib_$lib.so timeout -k 10 300 python3 scripts/bench_clean.py --dtype $dt --steps 20 > $OUT/time_${lib}_${dt}_$rep.log 2>&1 || exit $?
    done
  done
done
echo done > $OUT/status.txt
