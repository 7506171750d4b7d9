#!/bin/bash
# Planner candidates wide/tall x G4/G8: full GPU suite, bench line, C3 and C5 config lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r03q}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -v -m gpu -x --timeout 400 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py --steps 20 --warmup 2 > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 300 python -u bench.py --config C5 --steps 10 --warmup 2 --cpu-trials 16 --no-c3-strong --no-clean > $O/cfg_C5.json 2> $O/cfg_C5.err || exit $?
timeout -k 10 300 python -u bench.py --config C3 --scaling strong --shard 8 --steps 5 --warmup 1 --cpu-trials 16 --no-c3-strong --no-clean > $O/cfg_C3_625.json 2> $O/cfg_C3_625.err || exit $?
