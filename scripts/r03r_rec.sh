#!/bin/bash
# Float partial records: full GPU suite + bench line + rocprof of the C2 bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r03r}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -v -m gpu -x --timeout 400 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py --steps 20 --warmup 2 --no-c3-strong --no-clean > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-c3-strong --no-clean > $O/prof.log 2>&1 || exit $?
