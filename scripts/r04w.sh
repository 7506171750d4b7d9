#!/bin/bash
# Round 4: quad-output Gaussian kernel: the Gaussian / median / clean tests, then the
# cleaning kernels' warm rocprof stats (f32 and u8) and the C5 step timeline.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r04w
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_clean.py -v -m gpu -x --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_clean.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_f32 -o run -- python3 scripts/bench_clean.py --dtype f32 --steps 10 > $OUT/bench_clean_f32.log 2>&1 || exit $?
python3 scripts/warm_stats.py $OUT/prof_f32 --skip 1 > $OUT/warm_stats_f32.csv || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_u8 -o run -- python3 scripts/bench_clean.py --dtype u8 --steps 10 > $OUT/bench_clean_u8.log 2>&1 || exit $?
python3 scripts/warm_stats.py $OUT/prof_u8 --skip 1 > $OUT/warm_stats_u8.csv || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_c5 -o run -- python3 bench.py --config C5 --steps 20 --warmup 3 --no-cpu-baseline --no-clean --no-c3-strong --no-acc-f64 > $OUT/bench_c5.json 2> $OUT/bench_c5.err || exit $?
echo done > $OUT/status.txt
