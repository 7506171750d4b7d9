#!/bin/bash
# Round 5: float64 kernel with LDS-carried records and even reload counts - full GPU tests,
# C2 / C1 float64 A/B against the previous build (new2), SQ counters of the new kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -m gpu tests > $O/tests.log 2>&1 || exit $?
LIBS="new2 bf" ACC=f64 CFG=C2 ROUNDS=2 bash scripts/ab_lib.sh > $O/ab_c2_f64.log 2>&1 || exit $?
LIBS="new2 bf" ACC=f64 CFG=C1 ROUNDS=2 bash scripts/ab_lib.sh > $O/ab_c1_f64.log 2>&1 || exit $?
CMD="python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-clean --no-c3-strong --no-acc-f64 --acc f64"
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" \
           "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $O/pmc_f64_p$i -o run -- $CMD > $O/pmc_f64_p$i.log 2>&1 || exit $?
done
exit 0
