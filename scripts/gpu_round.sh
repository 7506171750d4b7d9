#!/bin/bash
# One GPU call: probe -> parity tests -> plan sweep -> bench.  Each GPU step has its own
# time limit; the script stops at the first step that crashes or times out.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-run}
if [ -x scripts/valu_probe ] && [ -n "$PROBE" ]; then
  timeout -k 10 60 scripts/valu_probe > gpurun_out/${TAG}_probe.log 2>&1 || exit $?
fi
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread -p no:cacheprovider ${PYTEST_ARGS} > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?
  echo "pytest rc=$rc" >> gpurun_out/${TAG}_tests.log
  [ $rc -le 1 ] || exit $rc
fi
if [ -n "$SWEEP" ]; then
  PU_SWEEP="$SWEEP" timeout -k 10 400 python -u scripts/sweep.py ${SWEEP_CFG:-C2} > gpurun_out/${TAG}_sweep.log 2>&1 || exit $?
fi
if [ -z "$NOBENCH" ]; then
  timeout -k 10 400 python -u bench.py --steps ${STEPS:-10} --warmup 2 ${BENCH_ARGS} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
fi
if [ -n "$PROFILE" ]; then
  export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/${TAG}_prof.log 2>&1 || exit $?
fi
exit 0
