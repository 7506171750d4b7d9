#!/bin/bash
# Round 5: A/B of the subband kernel (round-4 library, HEAD, C3 build change) at C2 and the
# C3 625-trial shard, and the SQ counters of the float64 kernel at C2 acc='f64'.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05c
mkdir -p $O
LIBS="r4 head new" CFG=C2 TRIALS=0 ROUNDS=2 bash scripts/ab_lib.sh > $O/ab_c2.log 2>&1 || exit $?
LIBS="head new" CFG=C3 TRIALS=625 ROUNDS=2 bash scripts/ab_lib.sh > $O/ab_c3_625.log 2>&1 || exit $?
export TMPDIR=/tmp
CMD="python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-clean --no-c3-strong --no-acc-f64 --acc f64"
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" \
           "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $O/pmc_f64_p$i -o run -- $CMD > $O/pmc_f64_p$i.log 2>&1 || exit $?
done
exit 0
