#!/bin/bash
# Round 5: host overhead after the raw stream handle / cached GPU check - cleaning GPU tests,
# masks_overhead.py (f32, u8), the C5 and C1 bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r05x}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -m gpu tests/test_gpu_clean.py > $O/tests.log 2>&1 || exit $?
for d in f32 u8; do
  timeout -k 10 200 python -u scripts/masks_overhead.py --dtype $d > $O/overhead_$d.json 2> $O/overhead_$d.err || exit $?
done
for c in C5 C1; do
  timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 2 --no-cpu-baseline --no-clean --no-c3-strong --no-acc-f64 > $O/bench_$c.json 2> $O/bench_$c.err || exit $?
done
exit 0
