#!/bin/bash
# One GPU call: bench lines for the non-headline configs (C1, C3, C5) and FETCH_SIZE /
# WRITE_SIZE PMC passes (one rocprofv3 --pmc run each) for C3 and C5.  Stops at the
# first step that fails or times out.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-cfg}
OUT=gpurun_out/${TAG}
mkdir -p $OUT
timeout -k 10 300 python -u bench.py --config C3 --steps 5 --warmup 1 --cpu-trials 8 > $OUT/c3_bench.json 2> $OUT/c3_bench.err || exit $?
timeout -k 10 200 python -u bench.py --config C5 --steps 20 --warmup 2 --cpu-trials 100 > $OUT/c5_bench.json 2> $OUT/c5_bench.err || exit $?
timeout -k 10 200 python -u bench.py --config C1 --steps 20 --warmup 2 > $OUT/c1_bench.json 2> $OUT/c1_bench.err || exit $?
for cfg in C3 C5; do
  i=0
  for set in "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $OUT/${cfg}_p$i -o run -- python3 bench.py --config $cfg --steps 1 --warmup 1 --no-cpu-baseline > $OUT/${cfg}_p$i.log 2>&1 || exit $?
  done
done
exit 0
