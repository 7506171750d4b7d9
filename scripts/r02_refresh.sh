#!/bin/bash
# One GPU call that refreshes every judged artefact at the current tree: the GPU parity
# suite, the bench line (C2 + clean + cpu baseline), the rocprofv3 kernel stats of the
# same bench command, the C2 HBM PMC passes (FETCH_SIZE, WRITE_SIZE: one rocprofv3 --pmc
# run each) and bench lines for C1/C3/C5.  Each GPU step has its own time limit; the
# script stops at the first step that fails.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-refresh}
OUT=gpurun_out/${TAG}
mkdir -p $OUT
if [ -z "$NOTEST" ]; then
  timeout -k 10 1000 python -u -m pytest tests -v -m gpu -x --timeout 400 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1 || exit $?
fi
timeout -k 10 400 python -u bench.py --steps 20 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/prof.log 2>&1 || exit $?
i=0
for set in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $set --output-format csv -d $OUT/pmc_p$i -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-clean > $OUT/pmc_p$i.log 2>&1 || exit $?
done
if [ -n "$CFGS" ]; then
  timeout -k 10 300 python -u bench.py --config C3 --steps 3 --warmup 1 --cpu-trials 8 > $OUT/c3_bench.json 2> $OUT/c3_bench.err || exit $?
  timeout -k 10 200 python -u bench.py --config C5 --steps 20 --warmup 2 --cpu-trials 100 > $OUT/c5_bench.json 2> $OUT/c5_bench.err || exit $?
  timeout -k 10 200 python -u bench.py --config C1 --steps 20 --warmup 2 > $OUT/c1_bench.json 2> $OUT/c1_bench.err || exit $?
fi
echo done > $OUT/status.txt
exit 0
