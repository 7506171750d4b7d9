#!/bin/bash
# PMC passes over one sweep variant (scripts/sweep.py), one rocprofv3 run per counter
# set (--pmc only).  Usage: TAG=x PU_SWEEP=4:80 bash scripts/pmc_sweep.sh [config]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
export PU_ROUNDS=1
TAG=${TAG:-pmcs}
OUT=gpurun_out/${TAG}
mkdir -p $OUT
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" \
           "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o run -- python3 scripts/sweep.py "$@" > $OUT/p$i.log 2>&1 || { echo "pass $i failed rc=$?" >> $OUT/status.txt; exit 1; }
done
echo done >> $OUT/status.txt
