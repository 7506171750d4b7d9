#!/bin/bash
# Round 5: the prefetching float64 kernel (dedisp_f64.hip) - parity (every dedispersion
# and degenerate-trial GPU test, smoke), then the bench's acc_f64 line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05b
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_dedisperse.py tests/test_gpu_degenerate.py > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-clean --no-cpu-baseline --no-c3-strong --acc-f64-steps 5 \
  > $O/bench.json 2> $O/bench.err || exit $?
exit 0
