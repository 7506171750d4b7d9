#!/bin/bash
# Round 4: per-kernel times of the C4 cleaning pass at HEAD (rocprofv3 kernel trace of
# bench_clean.py, f32 and u8), with the warm statistics (first launch of each kernel dropped).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r04s
mkdir -p $OUT
for dt in f32 u8; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$dt -o run -- python3 scripts/bench_clean.py --dtype $dt --steps 10 > $OUT/bench_clean_$dt.log 2>&1 || exit $?
  python3 scripts/warm_stats.py $OUT/prof_$dt --skip 1 > $OUT/warm_stats_$dt.csv || exit $?
done
echo done > $OUT/status.txt
