#!/bin/bash
# A/B of the finalize path (HEAD: memset + read-back copy; mapped counters; mapped +
# unrolled loop) and of the Gaussian filter forms; the cleaning GPU tests at the new default.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03w
mkdir -p $OUT
rm -f gpurun_out/gauss_ref.npy
for f in 2 0 1 0 2; do
  PU_GAUSS_FORM=$f timeout -k 10 120 python -u scripts/gauss_ab.py >> $OUT/gauss_ab.jsonl 2>> $OUT/gauss_ab.err || exit $?
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_clean.py tests/test_gpu_files.py -v -m gpu -x --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_clean.log 2>&1 || exit $?
for r in 1 2; do
  for v in head nounroll unroll; do
    PULSARUTILS_HIP_LIB=ab/lib_$v.so timeout -k 10 200 python -u scripts/step_overhead.py C5 C1 C2 > $OUT/so_${v}_$r.jsonl 2> $OUT/so_${v}_$r.err || exit $?
  done
done
echo done > $OUT/status.txt
