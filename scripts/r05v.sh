#!/bin/bash
# Round 5: rocprofv3 kernel stats of the cleaning steps (bench_clean.py) at the current
# clean.hip, f32 and u8.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r05v}
mkdir -p $O
export TMPDIR=/tmp
for d in f32 u8; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$d -o run -- python3 scripts/bench_clean.py --dtype $d --steps 10 --warmup 2 > $O/bench_clean_$d.log 2>&1 || exit $?
done
exit 0
