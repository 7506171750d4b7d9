#!/bin/bash
# Round 4: vector record loads in pu_finalize_kernel: every GPU test, then the C2 and C5
# lines and warm kernel stats of a C5 run (finalize time).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r04fin
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.txt 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-c3-strong > $OUT/bench.json 2> $OUT/bench.err || exit $?
timeout -k 10 300 python -u bench.py --config C5 --steps 20 --no-cpu-baseline --no-clean --no-c3-strong --no-acc-f64 > $OUT/cfg_C5.json 2> $OUT/cfg_C5.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 10 --no-cpu-baseline --no-clean --no-c3-strong --no-acc-f64 > $OUT/bench_prof.json 2> $OUT/bench_prof.err || exit $?
python3 scripts/warm_stats.py $OUT/prof --skip 1 > $OUT/rocprof_warm_stats.csv || exit $?
echo done > $OUT/status.txt
