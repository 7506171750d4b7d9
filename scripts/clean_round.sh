#!/bin/bash
# One GPU call: cleaning-pass timing (events) + rocprofv3 kernel stats, f32 and u8 (C4 shape).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-clean}
export TMPDIR=/tmp
for dt in ${DTYPES:-f32 u8}; do
  timeout -k 10 300 python -u scripts/bench_clean.py --dtype $dt > gpurun_out/${TAG}_${dt}.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof_${dt} -o run -- python3 scripts/bench_clean.py --dtype $dt --steps 5 --warmup 1 > gpurun_out/${TAG}_prof_${dt}.log 2>&1 || exit $?
  python scripts/clean_roofline.py $(find gpurun_out/${TAG}_prof_${dt} -name 'run_kernel_stats.csv' | head -1) $dt > gpurun_out/${TAG}_roofline_${dt}.jsonl || exit $?
done
exit 0
