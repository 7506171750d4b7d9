#!/bin/bash
# Round 5: SQ counter passes of the C2 headline kernel at the shipped source (one rocprofv3
# --pmc run per counter set, kernel trace only).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r05am}
mkdir -p $O
export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" \
           "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $set --output-format csv -d $O/sq_c2/p$i -o run -- python3 bench.py --config C2 --steps 1 --warmup 1 --no-cpu-baseline --no-clean --no-c3-strong --no-acc-f64 > $O/sq_c2_p$i.log 2>&1 || exit $?
done
exit 0
