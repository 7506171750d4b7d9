#!/bin/bash
# Round 4, first GPU call: the whole GPU suite at the current tree (multi-rank path,
# explicit planner options, float64 mad), then diagnostics of the C3 kernel (u8, tall
# G = 8) at the 625-trial shard and at 5000 trials: phase stamps and the ablation
# (diagnostic build only; results invalid in the ablation), C5/C2 stamps beside them,
# and the default bench line.  Each GPU step has its own limit; stop at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r04a
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1 || exit $?
PU_TRIALS=625 timeout -k 10 300 python -u scripts/stamps.py C3 4 > $OUT/stamps_c3_625.txt 2>&1 || exit $?
timeout -k 10 300 python -u scripts/stamps.py C3 2 > $OUT/stamps_c3_5000.txt 2>&1 || exit $?
timeout -k 10 200 python -u scripts/stamps.py C5 20 > $OUT/stamps_c5.txt 2>&1 || exit $?
timeout -k 10 200 python -u scripts/stamps.py C2 5 > $OUT/stamps_c2.txt 2>&1 || exit $?
PU_TRIALS=625 PU_SWEEP=8:160:2 CFG=C3 SKIPS="0 1 2 4 8 15" timeout -k 10 900 bash scripts/ablate.sh > $OUT/ablate_c3_625.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py --steps 20 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err || exit $?
echo done > $OUT/status.txt
