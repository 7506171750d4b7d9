#!/bin/bash
# Round 4: row-major outlier zeroing from a compact bad-bin list: cleaning tests, then the
# cleaning kernels' warm rocprof stats and a bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r04u
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_clean.py -v -m gpu -x --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_clean.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_f32 -o run -- python3 scripts/bench_clean.py --dtype f32 --steps 10 > $OUT/bench_clean_f32.log 2>&1 || exit $?
python3 scripts/warm_stats.py $OUT/prof_f32 --skip 1 > $OUT/warm_stats_f32.csv || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-c3-strong --no-acc-f64 > $OUT/bench.json 2> $OUT/bench.err || exit $?
echo done > $OUT/status.txt
