#!/bin/bash
# Round 4: renormalize's factor-weighted row sums walked last row group first (Infinity
# Cache hand-over between the three read passes) vs first-to-last: cleaning parity tests,
# then end-to-end renormalize A/B (interleaved processes, f32 and u8).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r04l
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_clean.py -v -m gpu -x --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_clean.log 2>&1 || exit $?
for r in 1 2 3; do
  for dt in f32 u8; do
    for v in fwd rev; do
      echo "== round $r dtype $dt lib $v" >> $OUT/ab_rowsum_order.log
      PULSARUTILS_HIP_LIB=ab/lib_$v.so timeout -k 10 200 python -u scripts/bench_clean.py --dtype $dt --steps 20 >> $OUT/ab_rowsum_order.log 2>&1 || exit $?
    done
  done
done
for r in 1 2; do
  for v in fwd rev; do
    PULSARUTILS_HIP_LIB=ab/lib_$v.so timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-c3-strong --no-acc-f64 > $OUT/bench_${v}_$r.json 2> $OUT/bench_${v}_$r.err || exit $?
  done
done
echo done > $OUT/status.txt
