#!/bin/bash
# GPU round recipe: parity tests -> bench -> rocprofv3 kernel stats.  Each GPU step has
# its own time limit; any failure other than ordinary test failures stops the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-run}
timeout -k 10 1000 python -m pytest tests -q -m gpu --maxfail=15 -p no:cacheprovider ${PYTEST_ARGS} > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/${TAG}_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py --steps ${STEPS:-10} --warmup 2 ${BENCH_ARGS} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
if [ -n "$PROFILE" ]; then
  export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1 || exit $?
fi
exit $rc
