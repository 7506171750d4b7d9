#!/bin/bash
# Round 5: per-kernel trace of the cleaning steps (masks + renormalize), f32 and u8.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05l
mkdir -p $O
export TMPDIR=/tmp
for dt in f32 u8; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_clean_$dt -o run -- \
    python3 scripts/bench_clean.py --dtype $dt --steps 10 --warmup 2 > $O/prof_clean_$dt.log 2>&1 || exit $?
done
exit 0
