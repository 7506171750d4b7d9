#!/bin/bash
# Round-2 GPU call: parity tests -> bench (C2 + clean + cpu baseline) -> pipeline timing.
# Each GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r02}
if [ -z "$NOTEST" ]; then
  timeout -k 10 1100 python -u -m pytest tests -v -m gpu -x --timeout 400 --timeout-method thread -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?
  echo "pytest rc=$rc" >> gpurun_out/${TAG}_tests.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ -z "$NOBENCH" ]; then
  timeout -k 10 400 python -u bench.py --steps ${STEPS:-10} --warmup 2 ${BENCH_ARGS} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
fi
if [ -n "$PIPE" ]; then
  timeout -k 10 400 python -u scripts/bench_pipeline.py --dtype u8 > gpurun_out/${TAG}_pipe_u8.json 2> gpurun_out/${TAG}_pipe_u8.err || exit $?
  timeout -k 10 400 python -u scripts/bench_pipeline.py --dtype f32 --search f32 > gpurun_out/${TAG}_pipe_f32.json 2> gpurun_out/${TAG}_pipe_f32.err || exit $?
fi
if [ -n "$SWEEP" ]; then
  PU_SWEEP="$SWEEP" PU_ROUNDS=${ROUNDS:-3} timeout -k 10 600 python -u scripts/sweep.py ${SWEEP_CFG:-C2} > gpurun_out/${TAG}_sweep.log 2>&1 || exit $?
fi
if [ -n "$ABLATE" ]; then
  for sk in $ABLATE; do
    echo "skip=$sk" >> gpurun_out/${TAG}_ablate.log
    PULSARUTILS_HIP_LIB=radio-pulsar-utils_amd/pulsarutils/_lib/libpulsarutils_hip_stamps.so PU_SUB_SKIP=$sk PU_ROUNDS=1 PU_SWEEP=${ABLATE_VARIANT:-4:160:0} timeout -k 10 200 python3 scripts/sweep.py C2 >> gpurun_out/${TAG}_ablate.log 2>&1 || exit $?
  done
fi
if [ -n "$CLEANSWEEP" ]; then
  timeout -k 10 400 python -u scripts/sweep_clean.py > gpurun_out/${TAG}_sweep_clean.jsonl 2>&1 || exit $?
fi
if [ -n "$STRONG" ]; then
  # per-rank kernel time of a strong-scaled run (total grid / N trials per GPU), N = 1, 2, 4, 8
  for cfg in C2 C3; do
    full=$([ $cfg = C2 ] && echo 1000 || echo 5000)
    for nr in 1 2 4 8; do
      echo "config=$cfg ranks=$nr trials=$((full / nr))" >> gpurun_out/${TAG}_strong.log
      PU_TRIALS=$((full / nr)) PU_SWEEP=$([ $cfg = C2 ] && echo 4:160:0 || echo 8:160:0) PU_ROUNDS=1 timeout -k 10 300 python3 scripts/sweep.py $cfg >> gpurun_out/${TAG}_strong.log 2>&1 || exit $?
    done
  done
fi
if [ -n "$PROFILE" ]; then
  export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/${TAG}_prof.log 2>&1 || exit $?
fi
exit 0
