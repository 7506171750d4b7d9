#!/bin/bash
# Round 5: HBM PMC passes (FETCH_SIZE, WRITE_SIZE; one rocprofv3 --pmc run each) of the
# cleaning steps (bench_clean.py f32 and u8) at the shipped clean.hip.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r05ao}
mkdir -p $O
export TMPDIR=/tmp
for d in f32 u8; do
  i=0
  for c in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $O/pmc_$d/p$i -o run -- python3 scripts/bench_clean.py --dtype $d --steps 3 --warmup 1 > $O/pmc_${d}_p$i.log 2>&1 || exit $?
  done
done
exit 0
